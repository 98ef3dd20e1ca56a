#!/usr/bin/env python3
"""VGPRs / spills / LDS of the rollout-buffer env kernels (PH 8 and 16) for
one or more sets of extra hipcc flags:
    python scripts/kres.py "" "-DVN_PC_MIN_WAVES=3"
"""
import subprocess
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT / "3d-navigation-reinforcement-learning_amd"))
from voxnav import _build as b  # noqa: E402

flags = [f for f in b.HIPCC_FLAGS if f not in ("-shared", "-fPIC")]
src = ROOT / "3d-navigation-reinforcement-learning_amd" / "csrc" / "voxnav_env.hip"
for extra in [a.split() for a in sys.argv[1:]] or [[]]:
    cmd = [b.hipcc(), *flags, *extra, "-I", str(b.INCLUDE), "-c", str(src), "-o", "/tmp/kres.o",
           "-Rpass-analysis=kernel-resource-usage"]
    r = subprocess.run(cmd, capture_output=True, text=True)
    cur, res = None, {}
    for line in r.stderr.splitlines():
        if " error" in line:
            print(line)
        if "Function Name" in line:
            name = line.split("Function Name: ")[1].split(" ")[0]
            keep = "env_kernel" in name and ("ILi8ELb0ELb1ELb0E" in name or "ILi16ELb0ELb1ELb0E" in name)
            cur = name if keep else None
        elif cur and ("VGPRs:" in line or "VGPRs Spill" in line or "LDS Size" in line):
            res.setdefault(cur, []).append(line.split("remark: ")[-1].split(" [")[0].strip())
    for k, v in res.items():
        print(extra, k.split("env_kernel")[1][:26], v)
