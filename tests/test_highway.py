"""Highway-layout output readers (mapfx.highway) against the
output file the reference ships (tests/golden/highway/vis_gmap.json, a copy of
MARL-curve-main/src/vis_export/tmp/vis_gmap.json) and round trips through the
generator's file format (highway_layout_v19.py:1538-1575)."""
import os

import numpy as np

from conftest import GOLDEN

HW_ROWS = ["@@ssss@@nn@",          # 7 x 11, non-square like the generator's maps
           "eeeeeeeeeee",
           "@@s..L@@n@@",
           "@@s..L@@n@@",
           "wwwwwwwwwww",
           "@@ssss@@nn@",
           "@@@@@@@@@@@"]


def test_vis_gmap_fixture():
    from mapfx.highway import read_vis_gmap
    grid, js = read_vis_gmap(os.path.join(GOLDEN, "highway", "vis_gmap.json"))
    assert grid.shape == (8, 8) and grid.dtype == np.uint8 and not grid.any()
    assert js["vtype_to_p_id"]["@"] == "#EDEED4"


def test_round_trip(tmp_path):
    from mapfx import highway as hw
    towns = {0: {"map": ["..L", "...", "@.."], "origin": (2, 3)},
             3: {"map": ["L@", ".."], "origin": (7, 1)}}
    locks = {35: (0, [35, 41, 18]), 18: (3, [])}
    edges = np.array([[2, 0, 1, 0, 0, 1], [8, 6, 0, 1, 1, 0]], dtype=np.int32)
    vis = {"g_map": HW_ROWS, "vtype_to_p_id": {"`": "LightSlateGray"}, "annotation": HW_ROWS}
    out = tmp_path / "results" / "m"
    hw.write_highway_outputs(str(out), HW_ROWS, towns, locks, edges.tolist(), vis, cfg={"n": 1})
    grid, rows = hw.read_highways(str(out / "highways.txt"))
    assert rows == HW_ROWS
    assert np.array_equal(grid, np.array([[c == "@" for c in r] for r in HW_ROWS], dtype=np.uint8))
    t = hw.read_towns(str(out / "towns.json"))
    assert sorted(t) == [0, 3] and t[0]["origin"] == (2, 3) and t[3]["map"] == ["L@", ".."]
    assert np.array_equal(t[0]["grid"], np.array([[0, 0, 1], [0, 0, 0], [1, 0, 0]], dtype=np.uint8))
    assert hw.read_locks(str(out / "locks.txt")) == locks
    assert np.array_equal(hw.read_rl_edges(str(out / "rl_edge.txt")), edges)
    g2, js = hw.read_vis_gmap(str(out / "vis_gmap.json"))
    assert np.array_equal(g2, grid) and js["annotation"] == HW_ROWS


def test_town_and_highway_map_text():
    from mapfx import highway as hw
    from mapfx.maps import parse_map_text
    town = {"map": ["..L", "@.."], "origin": (0, 0)}
    # MAPF-490-main/main.py:11-22: header, then the rows with lock cells as '@'
    assert hw.town_map_text(town) == "type octile\nheight 2\nwidth 3\nmap\n..@\n@..\n"
    g = parse_map_text(hw.highway_map_text(HW_ROWS))
    assert np.array_equal(g != 0, np.array([[c == "@" for c in r] for r in HW_ROWS]))


def test_reader_errors(tmp_path):
    import pytest
    from mapfx import highway as hw
    p = tmp_path / "highways.txt"
    p.write_text("height (n_rows): 2 \nwidth (n_cols): 3 \nHighway Map: \n@@@\n@@")
    with pytest.raises(ValueError):
        hw.read_highways(str(p))
    p.write_text("not a highway file")
    with pytest.raises(ValueError):
        hw.read_highways(str(p))
