"""The C-ABI library builds for gfx950, loads, and exports include/voxnav.h."""
import ctypes
import re
import subprocess

from helpers import REPO

HEADER = REPO / "include" / "voxnav.h"


def declared_functions():
    text = HEADER.read_text()
    return sorted(set(re.findall(r"^\s*(?:const\s+)?\w+\s*\*?\s*(vn_\w+)\s*\(", text, flags=re.M)))


def test_library_loads_and_exports_header_symbols():
    from voxnav import _native
    lib = _native.load()
    decl = declared_functions()
    assert len(decl) >= 11
    for name in decl:
        assert hasattr(lib, name), name
    assert set(decl) == set(_native.EXPORTED_SYMBOLS)
    assert lib.vn_abi_version() == _native.VN_ABI_VERSION == 2
    out = subprocess.run(["nm", "-D", "--defined-only", str(_native._build.LIB)], capture_output=True, text=True)
    exported = set(re.findall(r" T (vn_\w+)", out.stdout))
    assert set(decl) <= exported


def test_code_object_targets_gfx950():
    from voxnav import _build
    blob = _build.LIB.read_bytes()
    assert b"amdgcn-amd-amdhsa--gfx950" in blob      # the offload bundle id of the device code object
    assert b"gfx942" not in blob and b"gfx90a" not in blob


def test_errors_cross_the_boundary_as_codes():
    from voxnav import _native
    lib = _native.load()
    h = ctypes.c_void_p()
    cfg = _native.VnConfig(0, 1, 1, 0, -2.0, 0.84, 0, 0)   # L = 0 is invalid
    rc = lib.vn_create(None, 4, ctypes.byref(cfg), 0, ctypes.byref(h))
    assert rc < 0 and b"NULL" in lib.vn_last_error()
    import numpy as np
    whd = np.array([4, 4, 4], np.int32)
    walls = np.zeros(64, np.uint8)
    rs = _native.VnRoomSet(1, whd.ctypes.data, walls.ctypes.data, None, None)
    rc = lib.vn_create(ctypes.byref(rs), 4, ctypes.byref(cfg), 0, ctypes.byref(h))
    assert rc == -1 and b"local_map_length" in lib.vn_last_error()
    assert lib.vn_step(None, None, None, None, None, None, None, None, None) == -1
    bad = _native.VnConfig(4, 1, 1, 7, -2.0, 0.84, 0, 0)  # unknown variant
    rc = lib.vn_create(ctypes.byref(rs), 4, ctypes.byref(bad), 0, ctypes.byref(h))
    assert rc == -1 and b"variant" in lib.vn_last_error()


def test_bindings_match_header_arity():
    """Every ctypes binding (voxnav/_native.py) takes as many arguments as
    its include/voxnav.h declaration (a stale binding passes garbage)."""
    from voxnav import _native
    text = re.sub(r"/\*.*?\*/", "", HEADER.read_text(), flags=re.S)
    for name, (_, args) in _native._SIGS.items():
        m = re.search(r"\b" + name + r"\s*\(([^)]*)\)\s*;", text)
        assert m, name
        params = [p for p in m.group(1).split(",") if p.strip() and p.strip() != "void"]
        assert len(params) == len(args), (name, len(params), len(args))


def _isa_check():
    import importlib.util
    spec = importlib.util.spec_from_file_location("isa_check", REPO / "scripts" / "isa_check.py")
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def test_mlp_head_ring_wait_counts_hold_in_the_built_code():
    """vn_mlp_head_f32's hand-counted ``s_waitcnt vmcnt(PER)`` ring waits
    (csrc/voxnav_policy_f32.hip mh_layer) are right only if the compiled
    ring loops issue exactly PER ring loads and no other VMEM instruction
    between consecutive waits, and 2 x PER before the loop: checked on the
    disassembly of the built library (scripts/isa_check.py), both template
    instances (one- and two-tile loops)."""
    from voxnav import _build
    mod = _isa_check()
    rep = mod.check(_build.LIB)
    assert set(rep["loops"]) == {1, 2}
    # the checker rejects what it guards against: an extra VMEM op in a ring
    # loop (a spill / hoisted load), or one ring load too few before the loop
    sym, ins = mod.kernel_listing(_build.LIB)
    lo, hi = (int(v, 16) for v in rep["loops"][2]["loop"])
    k = next(i for i, x in enumerate(ins) if lo < x[0] < hi and x[1] == mod.RING_LOAD)
    bad = ins[:k] + [(ins[k][0] - 2, "global_load_dword", "v1, v[2:3], off", None)] + ins[k:]
    try:
        mod.check_listing(sym, bad)
    except AssertionError as e:
        assert "besides the ring loads" in str(e)
    else:
        raise AssertionError("the checker accepted a foreign VMEM load inside the ring loop")
    first = next(i for i, x in enumerate(ins) if x[1] == mod.RING_LOAD)      # a prologue load
    short = ins[:first] + ins[first + 1:]
    try:
        mod.check_listing(sym, short)
    except AssertionError:
        pass
    else:
        raise AssertionError("the checker accepted a ring prologue one load short")
