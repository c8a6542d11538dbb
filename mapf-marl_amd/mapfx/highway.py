"""Readers for the highway-layout generator's output files.

The reference's generator (highway_layout_v19.py) cannot run here (it imports
modules absent from the reference tree), but its output format is fixed by
`to_file` (highway_layout_v19.py:1425-1575), and the reference's own consumers
read it back: MAPF-490-main/main.py:6-33 turns `towns.json` into MovingAI town
maps ('L' lock cells become '@').  These readers give the gridworld envs the
same maps:

  results/<map>/highways.txt   'height (n_rows): H' / 'width (n_cols): W' /
                               'Highway Map:' then H rows, '@' = obstacle,
                               any other character a free cell labelled with
                               its highway direction (:1442-1454, :1539-1543)
  results/<map>/towns.json     {town id: {'town id', 'map': rows, 'origin':
                               [min_x, min_y]}} (:1500-1531, :1546-1547)
  results/<map>/locks.txt      'lock_key town_id reach_key ...' per line,
                               key = x + y * n_cols (:1532-1537, :1550-1555)
  results/<map>/rl_edge.txt    'x y u d l r' per highway/lock node (:1556-1575)
  results/<map>/vis_gmap.json  {'g_map': rows, 'vtype_to_p_id', 'annotation'}
                               (:1455-1487)

Row 0 of every map is the generator's top row (y = n_rows - 1), i.e. the same
top-first row order as a MovingAI .map, so a grid from here feeds
MapfGridBatch / MARL_PARTIAL_ENV unchanged (non-square maps included).
Format parity is pinned by the one output file the reference ships
(MARL-curve-main/src/vis_export/tmp/vis_gmap.json, tests/golden/highway/) and by
round trips through writers that follow `to_file` line by line.
"""
from __future__ import annotations

import json

import numpy as np

OBSTACLE = "@"


def _grid(rows) -> np.ndarray:
    """Rows of characters -> uint8 [H, W] obstacle grid ('@' = 1).  Rows must be
    equally long (the generator writes rectangular maps)."""
    rows = list(rows)
    if not rows:
        raise ValueError("empty map")
    w = len(rows[0])
    for i, r in enumerate(rows):
        if len(r) != w:
            raise ValueError("row %d has %d cells, row 0 has %d" % (i, len(r), w))
    return np.array([[1 if ch == OBSTACLE else 0 for ch in r] for r in rows], dtype=np.uint8)


def read_highways(path):
    """highways.txt -> (grid uint8 [H, W] with 1 = obstacle, labels [H] of str rows)."""
    with open(path) as f:
        lines = f.read().split("\n")
    if len(lines) < 3 or not lines[0].startswith("height (n_rows):") \
            or not lines[1].startswith("width (n_cols):") or not lines[2].startswith("Highway Map:"):
        raise ValueError("%s: not a highway_layout highways.txt" % path)
    h = int(lines[0].split(":", 1)[1])
    w = int(lines[1].split(":", 1)[1])
    rows = lines[3:3 + h]
    if len(rows) != h or any(len(r) != w for r in rows):
        raise ValueError("%s: expected %d rows of %d cells" % (path, h, w))
    return _grid(rows), rows


def read_towns(path):
    """towns.json -> {town_id (int): {'map': [rows], 'origin': (x, y), 'grid': uint8
    [h, w] with '@' and lock cells 'L' as obstacles (MAPF-490-main/main.py:17-20)}}."""
    with open(path) as f:
        js = json.load(f)
    out = {}
    for key, t in js.items():
        rows = list(t["map"])
        out[int(t.get("town id", key))] = {
            "map": rows,
            "origin": (int(t["origin"][0]), int(t["origin"][1])),
            "grid": _grid([r.replace("L", OBSTACLE) for r in rows]),
        }
    return out


def town_map_text(town) -> str:
    """A town as MovingAI .map text, as MAPF-490-main/main.py:11-22 writes it."""
    rows = [r.replace("L", OBSTACLE) for r in town["map"]]
    return "type octile\nheight %d\nwidth %d\nmap\n%s\n" % (len(rows), len(rows[0]), "\n".join(rows))


def highway_map_text(rows) -> str:
    """highways.txt rows as MovingAI .map text: '@' stays an obstacle, every highway /
    town / lock cell becomes '.' (MAPF_GRID treats any other character as an obstacle,
    envs/mapf_gridworld.py:282-288)."""
    rows = ["".join(OBSTACLE if ch == OBSTACLE else "." for ch in r) for r in rows]
    return "type octile\nheight %d\nwidth %d\nmap\n%s\n" % (len(rows), len(rows[0]), "\n".join(rows))


def read_locks(path):
    """locks.txt -> {lock_key: (town_id, [reachable lock keys])}; key = x + y * n_cols."""
    out = {}
    with open(path) as f:
        for line in f:
            v = line.split()
            if not v:
                continue
            out[int(v[0])] = (int(v[1]), [int(x) for x in v[2:]])
    return out


def read_rl_edges(path):
    """rl_edge.txt -> int32 [M, 6] rows (x, y, up, down, left, right)."""
    rows = []
    with open(path) as f:
        for line in f:
            v = line.split()
            if v:
                if len(v) != 6:
                    raise ValueError("%s: bad line %r" % (path, line))
                rows.append([int(x) for x in v])
    return np.array(rows, dtype=np.int32).reshape(-1, 6)


def read_vis_gmap(path):
    """vis_gmap.json -> (grid uint8 [H, W], the json dict)."""
    with open(path) as f:
        js = json.load(f)
    return _grid(js["g_map"]), js


def write_highway_outputs(result_path, hw_rows, towns, locks, rl_edges, vis_gmap, cfg=None):
    """Write the five files in the generator's exact format (highway_layout_v19.py
    :1538-1575): the inverse of the readers, used to round-trip them."""
    import os
    os.makedirs(result_path, exist_ok=True)
    with open(os.path.join(result_path, "highways.txt"), "w") as f:
        f.write("height (n_rows): {} \n".format(len(hw_rows)))
        f.write("width (n_cols): {} \n".format(len(hw_rows[0])))
        f.write("Highway Map: \n")
        f.write("\n".join(hw_rows))
    with open(os.path.join(result_path, "map_config_used.json"), "w") as f:
        json.dump([cfg or {}], f, indent=4)
    with open(os.path.join(result_path, "towns.json"), "w") as f:
        json.dump({tid: {"town id": tid, "map": t["map"], "origin": list(t["origin"])}
                   for tid, t in towns.items()}, f, indent=4)
    with open(os.path.join(result_path, "vis_gmap.json"), "w") as f:
        json.dump(vis_gmap, f, indent=4)
    with open(os.path.join(result_path, "locks.txt"), "w") as f:
        for k, (tid, reach) in locks.items():
            f.write("{} {} ".format(k, tid))
            f.writelines(["{} ".format(i) for i in reach])
            f.write("\n")
    with open(os.path.join(result_path, "rl_edge.txt"), "w") as f:
        for x, y, u, d, l, r in rl_edges:
            f.write("{} {} {} {} {} {} ".format(x, y, u, d, l, r))
            f.write("\n")
