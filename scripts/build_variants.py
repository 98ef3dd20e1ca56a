#!/usr/bin/env python3
"""Build A/B library variants in parallel:  build_variants.py name:DEF1,DEF2 name2:DEF ...
(outputs voxnav/_lib/variants/libvoxnav_<name>.so; diagnostics only)."""
import sys
from concurrent.futures import ThreadPoolExecutor
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parent.parent / "3d-navigation-reinforcement-learning_amd"))
from voxnav import _build  # noqa: E402


def one(spec):
    name, _, defs = spec.partition(":")
    return _build.build_variant(name, [d for d in defs.split(",") if d])


with ThreadPoolExecutor(max_workers=6) as ex:
    for p in ex.map(one, sys.argv[1:]):
        print(p)
