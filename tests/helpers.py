"""Shared helpers for the parity tests (golden fixtures, room sources)."""
from __future__ import annotations

import hashlib
import tarfile
from pathlib import Path

import numpy as np

REPO = Path(__file__).resolve().parent.parent
GOLDEN = REPO / "tests" / "golden"
ARCHIVE = REPO / "rooms" / "reference_rooms.tar.xz"

STATE13 = ("x", "y", "z", "facing", "last_action", "step_count", "visited_count", "bump_count",
           "done", "last_bump", "near_wall", "was_near_wall", "cells_insight_down")


def grid_hash(a: np.ndarray) -> int:
    h = hashlib.blake2b(np.ascontiguousarray(a, dtype=np.int64).tobytes(), digest_size=8).digest()
    return int(np.frombuffer(h, dtype=np.uint64)[0])


_ARCH_CACHE = {}


def archive_texts() -> dict:
    """{'P2_training/kitchen2.txt': text, ...} from the committed room archive."""
    if not _ARCH_CACHE:
        with tarfile.open(ARCHIVE) as tf:
            for m in tf.getmembers():
                if m.isfile():
                    rel = str(Path(m.name).relative_to("rooms"))
                    _ARCH_CACHE[rel] = tf.extractfile(m).read().decode()
    return _ARCH_CACHE


def set_members(setname: str):
    """Sorted (name, text) of a room set, the glob('*.txt') of that directory."""
    texts = archive_texts()
    out = [(Path(k).name, v) for k, v in texts.items() if Path(k).parent.name == setname and k.endswith(".txt")]
    return sorted(out, key=lambda t: t[0])


def box_text(W, D, H) -> str:
    lines = [f"Size={W},{D},{H}"]
    for z in range(H):
        lines.append(f"Layer z={z}")
        for y in range(D):
            lines.append(" ".join("2" if (x in (0, W - 1) or y in (0, D - 1) or z in (0, H - 1)) else "0"
                                  for x in range(W)))
    return "\n".join(lines) + "\n"


def source_texts(src: str):
    """room_source string of a golden file -> ([(name, text)], use_room_draw, ctor_whd)."""
    kind, arg = src.split(":", 1)
    if kind == "ctor":
        return [], False, tuple(int(v) for v in arg.split("x"))
    if kind == "box":
        W, D, H = (int(v) for v in arg.split("x"))
        return [(f"box_{arg}.txt", box_text(W, D, H))], True, None
    if kind == "file":
        return [(Path(arg).name, archive_texts()[arg])], True, None
    if kind == "set":
        return set_members(arg), True, None
    raise ValueError(src)


def oracle_env(src: str, L: int, n_agents: int = 1, crash_penalty: float = -2.0, variant: int = 0):
    from oracle.oracle import OracleEnv, parse_room_text, walled_box
    texts, draw, whd = source_texts(src)
    rooms = [walled_box(*whd)] if whd else [parse_room_text(t, n) for n, t in texts]
    return OracleEnv(rooms, n_agents=n_agents, local_map_length=L, crash_penalty=crash_penalty, use_room_draw=draw,
                     variant=variant)


def simple_golden_trajectories():
    return sorted(GOLDEN.glob("simple_*.npz"))


def product_room_set(src: str):
    from voxnav.rooms import RoomSet, ctor_box_set, parse_room
    texts, draw, whd = source_texts(src)
    if whd:
        return ctor_box_set(*whd)
    return RoomSet([parse_room(t, n) for n, t in texts], use_room_draw=draw, source=src)


def golden_trajectories():
    return sorted(GOLDEN.glob("traj_*.npz"))


def load_golden(path) -> dict:
    with np.load(path, allow_pickle=False) as z:
        return {k: z[k] for k in z.files}
