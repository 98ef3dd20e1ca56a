"""Compile libvoxnav.so (HIP, gfx950) in-tree.

The library is the drop-in boundary (include/voxnav.h).  It is built with
plain ``hipcc`` so the product has no build-system dependency; the .so lands
in ``voxnav/_lib/`` and travels with the repo snapshot to the GPU box.
"""
from __future__ import annotations

import os
import shutil
import subprocess
from concurrent.futures import ThreadPoolExecutor
from pathlib import Path

PKG = Path(__file__).resolve().parent
PROJECT = PKG.parent
REPO = PROJECT.parent
CSRC = PROJECT / "csrc"
INCLUDE = REPO / "include"
LIBDIR = PKG / "_lib"
LIB = LIBDIR / "libvoxnav.so"
SOURCES = [CSRC / "voxnav_env.hip", CSRC / "voxnav_simple.hip", CSRC / "voxnav_collect.hip",
           CSRC / "voxnav_learn_f32.hip", CSRC / "voxnav_learn_rows.hip", CSRC / "voxnav_gemm_f32.hip",
           CSRC / "voxnav_policy_f32.hip", CSRC / "voxnav_ppo_loss.hip"]
HEADERS = [INCLUDE / "voxnav.h", CSRC / "vn_common.h", CSRC / "env_core.h"]
ARCH = os.environ.get("VOXNAV_ARCH", "gfx950")

# -ffp-contract=off: the reward (f64) and obs quotients must follow the
# reference's operation order without fused multiply-adds.
HIPCC_FLAGS = ["-O3", "-std=c++17", "-ffp-contract=off", "-fPIC", f"--offload-arch={ARCH}"]


def hipcc() -> str:
    for cand in (os.environ.get("HIPCC"), shutil.which("hipcc"), "/opt/rocm/bin/hipcc"):
        if cand and Path(cand).exists():
            return cand
    raise RuntimeError("hipcc not found (set HIPCC or install ROCm)")


def needs_build() -> bool:
    if not LIB.exists():
        return True
    t = LIB.stat().st_mtime
    return any(p.stat().st_mtime > t for p in SOURCES + HEADERS + [Path(__file__)])


def _compile_link(out: Path, defines=(), verbose: bool = False) -> Path:
    """One object per source, compiled in parallel (the CubicEnv unit dominates), then one link."""
    objdir = out.parent / (out.name + ".objs")
    objdir.mkdir(parents=True, exist_ok=True)
    base = [hipcc(), *HIPCC_FLAGS, "-I", str(INCLUDE), *[f"-D{d}" for d in defines]]
    cmds = [base + ["-c", str(src), "-o", str(objdir / (src.stem + ".o"))] for src in SOURCES]
    if verbose:
        for c in cmds:
            print(" ".join(c))
    with ThreadPoolExecutor(max_workers=len(cmds)) as ex:
        results = list(ex.map(lambda c: subprocess.run(c, capture_output=True, text=True), cmds))
    for c, r in zip(cmds, results):
        if r.returncode != 0:
            raise RuntimeError(f"hipcc failed ({r.returncode}): {' '.join(c)}\n{r.stdout}\n{r.stderr}")
    tmp = out.with_suffix(".so.tmp")
    link = [hipcc(), "-shared", "-fPIC", f"--offload-arch={ARCH}", *[str(objdir / (src.stem + ".o")) for src in SOURCES],
            "-o", str(tmp)]
    r = subprocess.run(link, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"link failed ({r.returncode}):\n{r.stdout}\n{r.stderr}")
    os.replace(tmp, out)
    shutil.rmtree(objdir, ignore_errors=True)
    return out


def build_variant(name: str, defines=(), verbose: bool = False) -> Path:
    """A differently-configured build (-D flags) under _lib/variants/ for A/B
    timing: the diagnostics build (VN_DIAG), the only one whose compile-time
    knobs may differ from the product's defaults (csrc/vn_common.h)."""
    out = LIBDIR / "variants" / f"libvoxnav_{name}.so"
    out.parent.mkdir(parents=True, exist_ok=True)
    return _compile_link(out, ("VN_DIAG", *defines), verbose)


def build(force: bool = False, verbose: bool = False) -> Path:
    if not force and not needs_build():
        return LIB
    LIBDIR.mkdir(parents=True, exist_ok=True)
    return _compile_link(LIB, (), verbose)


if __name__ == "__main__":
    print(build(force=True, verbose=True))
