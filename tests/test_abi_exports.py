"""CPU-side checks of the C-ABI library: it loads, exports every symbol the
header declares, and its host-only helpers agree with the Python host code."""
import os
import re
import subprocess

import numpy as np

from conftest import REPO

HEADERS = [os.path.join(REPO, "include", h) for h in ("mapfx.h", "mapfx_partial.h", "mapfx_primal.h", "mapfx_runner.h")]


def _declared():
    out = set()
    for hdr in HEADERS:
        text = open(hdr).read()
        out |= set(re.findall(r"^\s*(?:[A-Za-z_][\w\s\*]*?)\b(mapfx_\w+)\s*\(", text, re.M))
    return sorted(out)


def test_library_exports_every_declared_symbol():
    import mapfx
    from mapfx import _abi
    declared = _declared()
    assert set(declared) == set(_abi.EXPORTS), declared
    nm = subprocess.run(["nm", "-D", "--defined-only", _abi.LIB_PATH], stdout=subprocess.PIPE,
                        text=True, check=True).stdout
    exported = set(re.findall(r"\bT (mapfx_\w+)", nm))
    missing = set(declared) - exported
    assert not missing, missing
    assert mapfx.lib.mapfx_abi_version() == 6
    bid = _abi.build_id()
    assert bid.startswith("src=") and " git=" in bid and "unknown" not in bid, bid


def test_host_helpers():
    from mapfx import lib, maps
    for h, w in ((8, 8), (32, 32), (13, 7), (128, 128), (64, 64)):
        assert lib.mapfx_map_stride(h, w) == maps.map_stride(h, w)
    assert lib.mapfx_obs_elem_size(16) == 1
    assert lib.mapfx_obs_elem_size(127) == 1
    assert lib.mapfx_obs_elem_size(128) == 2
    # an edge count is at most N - 1: exact in u8 up to N = 256, u16 above
    assert lib.mapfx_edge_elem_size(256) == 1
    assert lib.mapfx_edge_elem_size(257) == 2


def test_action_generator_host_vs_numpy():
    from mapfx import lib, rng
    seed = 0x1234ABCD5678
    envs = [0, 1, 7, 4095, 32767, 123456789]
    ts = [0, 1, 99, 2 ** 31 - 1]
    ref = rng.gen_actions(seed, envs, ts, 17)
    for ti, t in enumerate(ts):
        for ei, e in enumerate(envs):
            for a in range(17):
                assert lib.mapfx_action(seed, e, t, a) == ref[ti, ei, a]
    # uniform-ish over {0..4}
    big = rng.gen_actions(3, np.arange(512), np.arange(8), 16)
    counts = np.bincount(big.reshape(-1), minlength=5)
    assert counts.min() > 0.18 * big.size and counts.max() < 0.22 * big.size


def test_oracle_generator_matches():
    from mapfx import lib
    from oracle import corc
    for e in (0, 5, 99999):
        for t in (0, 3):
            for a in (0, 15):
                assert corc.lib().orc_action(77, e, t, a) == lib.mapfx_action(77, e, t, a)


def test_synthetic_instances_shard_invariant():
    from mapfx.maps import synthetic_instances
    full = synthetic_instances(64, 16, 16, 8, p_obstacle=0.15, seed=9)
    a = synthetic_instances(32, 16, 16, 8, p_obstacle=0.15, seed=9, env_offset=0)
    b = synthetic_instances(32, 16, 16, 8, p_obstacle=0.15, seed=9, env_offset=32)
    for k in ("grid", "bits", "init_pos", "goals"):
        assert np.array_equal(full[k], np.concatenate([a[k], b[k]]))
    g = full["grid"]
    ip = full["init_pos"]
    for e in range(64):
        cells = ip[e, :, 0] * 16 + ip[e, :, 1]
        assert len(set(cells.tolist())) == 8                       # distinct starts
        assert (g[e].reshape(-1)[cells] == 0).all()                 # on free cells
    frac = (g != 0).mean()
    assert 0.12 < frac < 0.18


def test_bits_roundtrip():
    from mapfx.maps import pack_bits, unpack_bits, warehouse_grid
    rs = np.random.RandomState(0)
    g = -(rs.random_sample((5, 13, 7)) < 0.3).astype(np.int8)
    assert np.array_equal(unpack_bits(pack_bits(g), 13, 7), g)
    w = warehouse_grid(64)
    assert w.shape == (64, 64) and (w[0] == -1).all() and 0.3 < (w != 0).mean() < 0.6


def test_create_rejects_out_of_range_configs():
    """mapfx_create validates its configuration before any HIP call (no GPU needed):
    the grid size of a launch travels in 26 bits of a preloaded kernel argument
    (MAPFX_HOT_ARGS), so n_envs is limited to 2^26 - 1 envs per handle."""
    import ctypes
    from mapfx import lib
    from mapfx._abi import Cfg

    def create(**kw):
        c = Cfg(H=8, W=8, n_agents=2, n_envs=4, env_offset=0, episode_limit=100,
                step_reward=-0.01, collide_reward=-10.0, obs_mode=0, window=5,
                primal_size=5, map_shared=0)
        for k, v in kw.items():
            setattr(c, k, v)
        h = ctypes.c_void_p()
        return lib.mapfx_create(ctypes.byref(c), ctypes.byref(h)), lib.mapfx_last_error()

    for kw, what in (({"n_envs": 1 << 26}, b"n_envs"), ({"n_envs": -1}, b"n_envs"),
                     ({"n_agents": 0}, b"n_agents"), ({"n_agents": 1025}, b"n_agents"),
                     ({"H": 0}, b"grid"), ({"W": 4097}, b"grid")):
        rc, msg = create(**kw)
        assert rc == -1 and what in msg, (kw, rc, msg)
