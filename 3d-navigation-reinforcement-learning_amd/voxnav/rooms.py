"""Room files: parse, synthesise, and pack for the device.

The text grammar is the reference's (README.md:9-19, parser
``GridAgent.load_room`` at envs/CubicEnv.py:402-438):

    Size=W,D,H            -> new all-free W x D x H grid
    Layer z=K             -> select layer K (numpy indexing: negative K wraps)
    <W ints>              -> row y of layer K, x = column; token 2 is a wall
    Start position=x,y,z  -> fixed start (optional)
    Goal=x,y,z            -> goal (optional; used by the simpleEnv variant)

Quirks kept on purpose: any value other than 2 (or an explicit -2) is free;
the simpleEnv variant (envs/simpleEnv.py:282, :381) keeps the raw values,
so there only 2 is a wall and a -2 token is free (``Room.walls_for``);
a row with the wrong width raises ``ValueError`` (:435-436); a row past D or
a layer index outside [-H, H) raises ``IndexError`` like the reference's
numpy assignment (:437); ``Layer z=-2`` writes layer H-2
(rooms/P3_training/kitchen2.txt).  Rooms are parsed ONCE on the host and
packed; the reference re-reads the file on every reset (:408).

A room set is ``sorted(Path(room_path).glob('*.txt'))`` by file name; the
reference's glob order (:66) is unspecified, so sorting is the build's
deterministic choice and the oracle harness sorts the same way.
"""
from __future__ import annotations

import io
import tarfile
from dataclasses import dataclass, field
from pathlib import Path
from typing import Iterable, List, Optional, Sequence, Tuple, Union

import numpy as np

REPO_ROOT = Path(__file__).resolve().parents[2]
REFERENCE_ROOM_ARCHIVE = REPO_ROOT / "rooms" / "reference_rooms.tar.xz"


VARIANT_CUBIC = 0    # envs/CubicEnv.py
VARIANT_SIMPLE = 1   # envs/simpleEnv.py


@dataclass
class Room:
    """One parsed room: walls[x, y, z] is True where the CubicEnv grid is -2
    (file value 2 or -2); ``minus2`` marks the cells written as -2, which
    are free in the simpleEnv variant."""

    name: str
    walls: np.ndarray
    start: Optional[Tuple[int, int, int]] = None
    goal: Optional[Tuple[int, int, int]] = None
    minus2: Optional[np.ndarray] = None

    def walls_for(self, variant: int = VARIANT_CUBIC) -> np.ndarray:
        if variant == VARIANT_SIMPLE and self.minus2 is not None:
            return self.walls & ~self.minus2
        return self.walls

    def total_free_cells_for(self, variant: int = VARIANT_CUBIC) -> int:
        return int((~self.walls_for(variant)[1:-1, 1:-1, 1:-1]).sum())

    @property
    def shape(self) -> Tuple[int, int, int]:
        return tuple(int(v) for v in self.walls.shape)

    def grid(self) -> np.ndarray:
        """The reference's ``self.grid`` view: int64, -2 wall, 0 free."""
        return np.where(self.walls, -2, 0).astype(np.int64)

    @property
    def total_free_cells(self) -> int:
        """Interior free cells (envs/CubicEnv.py:450-457) = max_steps (:459)."""
        return int((~self.walls[1:-1, 1:-1, 1:-1]).sum())

    def start_cells(self) -> np.ndarray:
        """Interior free cells in the reference's x -> y -> z scan order."""
        W, D, H = self.shape
        idx = np.argwhere(~self.walls[1:-1, 1:-1, 1:-1]) + 1   # argwhere is C-order = x, y, z
        return idx.astype(np.int32)


def parse_room(text: str, name: str = "<room>") -> Room:
    walls = None
    minus2 = None
    start = goal = None
    layer = None
    row = 0
    W = D = H = 0
    for raw in text.splitlines():
        line = raw.strip()
        if not line:
            continue
        if line.startswith("Start position"):
            start = tuple(int(v) for v in line.split("=")[1].split(","))
            continue
        if line.startswith("Goal"):
            goal = tuple(int(v) for v in line.split("=")[1].split(","))
            continue
        if line.startswith("Size"):
            dims = line.split("=")[1].split(",")
            W, D, H = int(dims[0]), int(dims[1]), int(dims[2])
            walls = np.zeros((W, D, H), dtype=bool)
            minus2 = np.zeros((W, D, H), dtype=bool)
            continue
        if line.startswith("Layer"):
            layer = int(line.split("=")[1])
            row = 0
            continue
        if walls is None:
            raise ValueError(f"{name}: data row before any 'Size=' line: {line!r}")
        if layer is None:
            raise ValueError(f"{name}: data row before any 'Layer' line: {line!r}")
        vals = [int(v) for v in line.split()]
        if len(vals) != W:
            raise ValueError(f"Line '{line}' has {len(vals)} values, but width is {W} for layer {layer}, row {row}.")
        if not -H <= layer < H:
            raise IndexError(f"{name}: layer index {layer} is out of bounds for height {H}")
        if row >= D:
            raise IndexError(f"{name}: row {row} is out of bounds for depth {D}")
        walls[:, row, layer % H] = [v in (2, -2) for v in vals]
        minus2[:, row, layer % H] = [v == -2 for v in vals]
        row += 1
    if walls is None:
        raise ValueError(f"{name}: no 'Size=' line")
    return Room(name=name, walls=walls, start=start, goal=goal, minus2=minus2 if minus2.any() else None)


def load_room_file(path: Union[str, Path]) -> Room:
    p = Path(path)
    return parse_room(p.read_text(), name=p.name)


def box_room(width: int, depth: int, height: int, name: Optional[str] = None) -> Room:
    """Walls on all six faces: the ctor fallback room (envs/CubicEnv.py:440-448)."""
    w = np.zeros((width, depth, height), dtype=bool)
    w[0, :, :] = w[-1, :, :] = True
    w[:, 0, :] = w[:, -1, :] = True
    w[:, :, 0] = w[:, :, -1] = True
    return Room(name=name or f"box_{width}x{depth}x{height}", walls=w)


def room_to_text(room: Room) -> str:
    """Serialise in the reference grammar (walls as 2, free as 0)."""
    W, D, H = room.shape
    out = io.StringIO()
    out.write(f"Size={W},{D},{H}\n")
    if room.start is not None:
        out.write("Start position=%d,%d,%d\n" % room.start)
    if room.goal is not None:
        out.write("Goal=%d,%d,%d\n" % room.goal)
    for z in range(H):
        out.write(f"Layer z={z}\n")
        for y in range(D):
            out.write(" ".join("2" if room.walls[x, y, z] else "0" for x in range(W)) + "\n")
        out.write("\n")
    return out.getvalue()


@dataclass
class RoomSet:
    """Rooms in random.choice order, plus whether reset draws a room.

    ``use_room_draw`` mirrors ``room_path != None`` in the reference
    (envs/CubicEnv.py:64-66, :406-407): a directory of rooms draws one per
    reset; the ctor box (room_path=None) does not consume that draw.
    """

    rooms: List[Room]
    use_room_draw: bool = True
    source: str = ""
    _packed: dict = field(default_factory=dict, repr=False)

    def __len__(self):
        return len(self.rooms)

    @property
    def max_shape(self):
        return tuple(int(max(r.shape[i] for r in self.rooms)) for i in range(3))

    def pack(self, variant: int = VARIANT_CUBIC):
        """(whd int32 [n,3], walls uint8 concat, fixed_start int32 [n,3],
        goal int32 [n,3]) for vn_create; walls of the given env variant."""
        if variant not in self._packed:
            whd = np.asarray([r.shape for r in self.rooms], dtype=np.int32)
            walls = np.concatenate([np.ascontiguousarray(r.walls_for(variant), dtype=np.uint8).reshape(-1)
                                    for r in self.rooms])
            fs = np.asarray([r.start if r.start is not None else (-1, -1, -1) for r in self.rooms], dtype=np.int32)
            gl = np.asarray([r.goal if r.goal is not None else (-1, -1, -1) for r in self.rooms], dtype=np.int32)
            self._packed[variant] = tuple(np.ascontiguousarray(a) for a in (whd, walls, fs, gl))
        return self._packed[variant]


def load_room_dir(room_path: Union[str, Path]) -> RoomSet:
    """``Path(room_path).glob('*.txt')`` sorted by file name."""
    files = sorted(Path(room_path).glob("*.txt"), key=lambda p: p.name)
    if not files:
        raise ValueError(f"no *.txt room files in {room_path}")
    return RoomSet([load_room_file(p) for p in files], use_room_draw=True, source=str(room_path))


def load_archive_set(subdir: str, archive: Union[str, Path] = REFERENCE_ROOM_ARCHIVE) -> RoomSet:
    """Rooms of one set (e.g. 'P2_training') from a tar archive of room dirs."""
    members = []
    with tarfile.open(archive) as tf:
        for m in tf.getmembers():
            p = Path(m.name)
            if m.isfile() and p.parent.name == subdir and p.suffix == ".txt":
                members.append((p.name, tf.extractfile(m).read().decode()))
    if not members:
        raise ValueError(f"no rooms for {subdir!r} in {archive}")
    members.sort(key=lambda t: t[0])
    return RoomSet([parse_room(txt, name) for name, txt in members], use_room_draw=True, source=f"{archive}:{subdir}")


def extract_archive(dest: Union[str, Path], archive: Union[str, Path] = REFERENCE_ROOM_ARCHIVE) -> Path:
    """Unpack the room archive (rooms/<set>/*.txt) under dest; returns dest/rooms."""
    dest = Path(dest)
    with tarfile.open(archive) as tf:
        tf.extractall(dest, filter="data") if hasattr(tarfile, "data_filter") else tf.extractall(dest)
    return dest / "rooms"


def ctor_box_set(width: int = 20, depth: int = 20, height: int = 12) -> RoomSet:
    """room_path=None: the walled box from the ctor dims, no room draw."""
    return RoomSet([box_room(width, depth, height)], use_room_draw=False, source="ctor")


def single_room_set(room: Room) -> RoomSet:
    """A room directory holding one file: the room draw still happens."""
    return RoomSet([room], use_room_draw=True, source=room.name)


def as_room_set(rooms=None, room_path=None, width=20, depth=20, height=12) -> RoomSet:
    if isinstance(rooms, RoomSet):
        return rooms
    if rooms is not None:
        rl = list(rooms)
        return RoomSet(rl, use_room_draw=True, source="list")
    if room_path is not None:
        return load_room_dir(room_path)
    return ctor_box_set(width, depth, height)
