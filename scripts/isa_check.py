#!/usr/bin/env python3
"""Build-time ISA invariant of vn_mlp_head_f32 (csrc/voxnav_policy_f32.hip,
``mh_layer``): the wave's LDS weight ring is guarded by hand-counted waits.

Each k-group's B operand arrives by ``global_load_lds_dwordx4`` (PER = 1 or 2
loads per k-group: one or two 32-column tiles), two k-groups in flight, and
the loop reads a ring slot after ``s_waitcnt vmcnt(PER)``, an inline-asm
wait the compiler does not check.  That count is right only if, in the
compiled loop, exactly PER vector-memory instructions -- all of them the
ring's LDS-DMA loads -- are issued between consecutive such waits (and 2 x
PER before the loop).  Any other VMEM instruction there (a spill, a hoisted
load, a store) would make the wait release a slot whose data is still in
flight: the data race behind round 5's one GPU fault.

``check(so)`` extracts the gfx950 code objects from the built library,
disassembles ``mlp_head_f32_kernel`` with llvm-objdump and asserts, for
every innermost loop that issues ring loads: no other VMEM instruction in the loop;
one nonzero vmcnt value P in the loop; exactly P ring loads between
consecutive nonzero waits around the loop's cycle; exactly 2P ring loads
between the last vmcnt(0) before the loop and its head.  Both template
instances (P = 1 and P = 2) must be found.  Raises AssertionError otherwise.

  python scripts/isa_check.py [path/to/libvoxnav.so]
"""
from __future__ import annotations

import re
import struct
import subprocess
import sys
import tempfile
from pathlib import Path

REPO = Path(__file__).resolve().parent.parent
LIB = REPO / "3d-navigation-reinforcement-learning_amd" / "voxnav" / "_lib" / "libvoxnav.so"
OBJDUMP = "/opt/rocm/llvm/bin/llvm-objdump"
KERNEL = "mlp_head_f32_kernel"
MAGIC = b"__CLANG_OFFLOAD_BUNDLE__"
RING_LOAD = "global_load_lds_dwordx4"
VMEM = re.compile(r"^(global_|buffer_|scratch_|flat_)")


def code_objects(so: Path, target: str = "gfx950"):
    """The device code objects (ELF bytes) of every offload bundle in the library."""
    data = so.read_bytes()
    out, i = [], 0
    while True:
        i = data.find(MAGIC, i)
        if i < 0:
            return out
        n = struct.unpack_from("<Q", data, i + 24)[0]
        p = i + 32
        for _ in range(n):
            off, size, tl = struct.unpack_from("<QQQ", data, p)
            p += 24
            triple = data[p:p + tl].decode(errors="replace")
            p += tl
            if target in triple and size > 0:
                out.append(data[i + off:i + off + size])
        i += len(MAGIC)


def kernel_listing(so: Path, name: str = KERNEL):
    """[(address, mnemonic, operands, branch_target or None)] of the kernel."""
    with tempfile.TemporaryDirectory() as td:
        for k, co in enumerate(code_objects(so)):
            f = Path(td) / f"co{k}.elf"
            f.write_bytes(co)
            txt = subprocess.run([OBJDUMP, "-d", "--mcpu=gfx950", str(f)], capture_output=True, text=True,
                                 check=True).stdout
            m = re.search(r"^([0-9a-f]+) <(\S*" + name + r"\S*)>:\n", txt, re.M)
            if not m:
                continue
            base, sym = int(m.group(1), 16), m.group(2)
            body = txt[m.end():]
            end = body.find("\n\n")
            ins = []
            for line in body[:end if end >= 0 else None].splitlines():
                line = line.strip()
                am = re.search(r"//\s*([0-9A-Fa-f]+):", line)
                if not line or am is None:
                    continue
                code = line.split("//")[0].strip()
                mnem, _, ops = code.partition(" ")
                tm = re.search(r"<" + re.escape(sym) + r"\+0x([0-9a-f]+)>", line)
                ins.append((int(am.group(1), 16), mnem, ops.strip(), base + int(tm.group(1), 16) if tm else None))
            return sym, ins
    raise AssertionError(f"{name} not found in the gfx950 code objects of {so}")


def vm_wait(mnem: str, ops: str):
    """vmcnt value of an s_waitcnt (None when it does not wait on vmcnt)."""
    if mnem != "s_waitcnt":
        return None
    m = re.search(r"vmcnt\((\d+)\)", ops)
    return int(m.group(1)) if m else None


def check(so: Path = LIB) -> dict:
    return check_listing(*kernel_listing(so))


def check_listing(sym: str, ins) -> dict:
    addr_ix = {a: k for k, (a, _, _, _) in enumerate(ins)}
    loops = []
    for k, (a, mnem, ops, tgt) in enumerate(ins):
        if tgt is None or not mnem.startswith("s_cbranch") or tgt > a:
            continue
        head = addr_ix.get(tgt)
        assert head is not None, f"{sym}: branch at {a:#x} into the middle of an instruction"
        body = ins[head:k + 1]
        if any(m == RING_LOAD for _, m, _, _ in body):
            loops.append((head, k))
    assert loops, f"{sym}: no loop issues {RING_LOAD}"
    # innermost only: the layer loop around a ring loop also contains its loads
    loops = [(h, t) for h, t in loops if not any((h2, t2) != (h, t) and h <= h2 and t2 <= t for h2, t2 in loops)]
    found = {}
    for head, tail in loops:
        body = ins[head:tail + 1]
        where = f"{sym} loop {ins[head][0]:#x}..{ins[tail][0]:#x}"
        other = [(a, m) for a, m, _, _ in body if VMEM.match(m) and m != RING_LOAD]
        assert not other, f"{where}: VMEM instructions besides the ring loads inside the loop: {other}"
        waits = [(j, vm_wait(m, o)) for j, (_, m, o, _) in enumerate(body) if vm_wait(m, o)]
        vals = {w for _, w in waits}
        assert len(vals) == 1, f"{where}: expected one nonzero vmcnt value, found {sorted(vals)}"
        P = vals.pop()
        assert P in (1, 2), f"{where}: vmcnt({P}) is not a ring wait"
        zeros = [j for j, (_, m, o, _) in enumerate(body) if vm_wait(m, o) == 0]
        assert not zeros, f"{where}: a vmcnt(0) inside the ring loop"
        # loads between consecutive nonzero waits, around the cycle
        pos = [j for j, _ in waits]
        for n, j in enumerate(pos):
            nxt = pos[(n + 1) % len(pos)]
            seg = body[j + 1:nxt] if nxt > j else body[j + 1:] + body[:nxt]
            cnt = sum(1 for _, m, _, _ in seg if m == RING_LOAD)
            assert cnt == P, (f"{where}: {cnt} ring loads between the waits at {body[j][0]:#x} and "
                              f"{body[nxt][0]:#x}, vmcnt({P}) needs exactly {P}")
        # the prologue: 2P ring loads (MH_D = 2 k-groups) since the last full drain
        k = head - 1
        pro = []
        while k >= 0 and vm_wait(ins[k][1], ins[k][2]) != 0:
            pro.append(ins[k])
            k -= 1
        assert k >= 0, f"{where}: no vmcnt(0) before the loop"
        bad = [(a, m) for a, m, _, _ in pro if VMEM.match(m) and m != RING_LOAD]
        assert not bad, f"{where}: VMEM instructions besides the ring loads before the loop: {bad}"
        npro = sum(1 for _, m, _, _ in pro if m == RING_LOAD)
        assert npro == 2 * P, f"{where}: {npro} ring loads before the loop, vmcnt({P}) with two slots needs {2 * P}"
        found[P] = {"loop": [hex(ins[head][0]), hex(ins[tail][0])], "waits": len(pos),
                    "ring_loads": sum(1 for _, m, _, _ in body if m == RING_LOAD), "prologue_loads": npro}
    assert set(found) == {1, 2}, f"{sym}: expected the one- and two-tile ring loops, found P = {sorted(found)}"
    return {"kernel": sym, "loops": found}


if __name__ == "__main__":
    import json
    print(json.dumps(check(Path(sys.argv[1]) if len(sys.argv) > 1 else LIB), indent=1))
