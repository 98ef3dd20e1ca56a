"""Product room loader (voxnav.rooms) vs the reference's parsed rooms."""
import tempfile
from pathlib import Path

import numpy as np
import pytest

from helpers import GOLDEN, archive_texts, grid_hash, load_golden
from voxnav import rooms as R


def test_every_room_file_parses_like_the_reference():
    z = load_golden(GOLDEN / "rooms_parsed.npz")
    texts = archive_texts()
    for name, whd, tf, h in zip(z["names"], z["whd"], z["total_free"], z["grid_hash"]):
        room = R.parse_room(texts[str(name)], str(name))
        assert room.shape == tuple(int(v) for v in whd), name
        assert grid_hash(room.grid()) == int(h), name
        assert room.total_free_cells == int(tf), name
        assert len(room.start_cells()) == int(tf)


def test_start_cells_scan_order():
    room = R.box_room(5, 4, 4)
    cells = room.start_cells()
    expect = [(x, y, z) for x in range(1, 4) for y in range(1, 3) for z in range(1, 3)]
    assert [tuple(c) for c in cells] == expect


def test_room_dir_is_sorted_glob_and_ignores_non_txt():
    with tempfile.TemporaryDirectory() as d:
        root = R.extract_archive(d)
        rs = R.load_room_dir(root / "P1_train")          # holds a stray r.tcxt
        names = [r.name for r in rs.rooms]
        assert names == sorted(names) and len(names) == 5 and rs.use_room_draw
        rs2 = R.load_archive_set("P1_train")
        assert [r.name for r in rs2.rooms] == names
        for a, b in zip(rs.rooms, rs2.rooms):
            assert (a.walls == b.walls).all()


def test_negative_layer_and_errors():
    k2 = R.parse_room(archive_texts()["P3_training/kitchen2.txt"])
    assert not k2.walls[:, :, 2].any()       # 'Layer z=-2' went to layer 10
    with pytest.raises(ValueError):
        R.parse_room("Size=3,3,3\nLayer z=0\n2 2\n")
    with pytest.raises(IndexError):
        R.parse_room("Size=2,1,3\nLayer z=0\n2 2\n2 2\n")
    with pytest.raises(IndexError):
        R.parse_room("Size=2,1,3\nLayer z=3\n2 2\n")
    r = R.parse_room("Size=3,1,3\nStart position=1,0,1\nGoal=1,0,2\nLayer z=0\n2 -2 0\n")
    assert r.start == (1, 0, 1) and r.goal == (1, 0, 2)
    assert r.walls[:, 0, 0].tolist() == [True, True, False]


def test_text_round_trip_and_box():
    b = R.box_room(8, 8, 4)
    again = R.parse_room(R.room_to_text(b))
    assert (again.walls == b.walls).all() and b.total_free_cells == 6 * 6 * 2
    ctor = R.ctor_box_set(32, 32, 8)
    assert not ctor.use_room_draw and ctor.rooms[0].total_free_cells == 5400


def test_pack_layout():
    rs = R.load_archive_set("P2_training")
    whd, walls, fs, gl = rs.pack()
    assert whd.shape == (25, 3) and walls.dtype == np.uint8
    assert walls.size == int(np.prod(whd, axis=1).sum())
    off = 0
    for r, s in zip(rs.rooms, whd):
        n = int(np.prod(s))
        assert (walls[off:off + n].reshape(tuple(s)) == r.walls).all()
        off += n
    assert (fs == -1).all()


def test_simple_variant_walls_match_oracle_tokens():
    """simpleEnv keeps raw file values: only 2 is a wall, -2 is free
    (envs/simpleEnv.py:282, :381); checked on every reference room file."""
    from helpers import archive_texts
    from oracle.oracle import parse_room_text
    n_minus2 = 0
    for rel, text in archive_texts().items():
        if not rel.endswith(".txt"):
            continue
        r = R.parse_room(text, rel)
        o = parse_room_text(text, rel)
        assert (r.walls_for(R.VARIANT_SIMPLE) == o.simple_walls.astype(bool)).all(), rel
        assert (r.walls_for(R.VARIANT_CUBIC) == o.walls.astype(bool)).all(), rel
        n_minus2 += r.minus2 is not None
    assert n_minus2 >= 1     # kitchen2.txt


def test_pack_goal_and_variant_walls():
    text = R.room_to_text(R.box_room(6, 5, 4)).replace("Size=6,5,4\n", "Size=6,5,4\nGoal=2,3,1\n")
    room = R.parse_room(text)
    rs = R.RoomSet([room])
    whd, walls, fs, gl = rs.pack(R.VARIANT_SIMPLE)
    assert tuple(gl[0]) == (2, 3, 1) and (fs == -1).all()
