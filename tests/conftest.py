import glob
import os
import sys

import numpy as np
import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG_ROOT = os.path.join(REPO, "mapf-marl_amd")
for p in (REPO, PKG_ROOT):
    if p not in sys.path:
        sys.path.insert(0, p)

GOLDEN = os.path.join(REPO, "tests", "golden")

# On a CPU-only host where build() has not run yet, the GPU-only runner test cannot
# even be collected (it imports mapfx at module level). Skip collecting it there; on
# a GPU box the missing library stays a loud collection error.
_LIB = os.path.join(PKG_ROOT, "mapfx", "libmapfx.so")
collect_ignore = []
if not os.path.exists(_LIB):
    try:
        import torch
        _has_gpu = torch.cuda.device_count() > 0
    except Exception:
        _has_gpu = False
    if not _has_gpu:
        collect_ignore.append("test_gpu_runner.py")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (HIP device)")


def load_fixture(name):
    d = np.load(os.path.join(GOLDEN, name + ".npz"), allow_pickle=False)
    return {k: d[k] for k in d.files}


def step_fixtures():
    return sorted(os.path.basename(p)[:-4] for p in glob.glob(os.path.join(GOLDEN, "*.npz"))
                  if not os.path.basename(p).startswith(("primal", "mp_", "pd_", "pw_", "runner_", "big_maps")))


def partial_fixtures():
    """MARL_PARTIAL_ENV goldens (tests/golden/gen_partial_fixtures.py)."""
    return sorted(os.path.basename(p)[:-4] for p in glob.glob(os.path.join(GOLDEN, "mp_*.npz")))


def primal_fixtures():
    return sorted(os.path.basename(p)[:-4] for p in glob.glob(os.path.join(GOLDEN, "primal*.npz")))


def fixture_rewards(fx):
    """(step_reward, collide_reward) with the Python types the reference saw."""
    sr = fx["meta_step_reward"].item()
    cr = fx["meta_collide_reward"].item()
    sr = int(sr) if bool(fx["meta_step_is_int"]) else float(sr)
    cr = int(cr) if bool(fx["meta_collide_is_int"]) else float(cr)
    return sr, cr


@pytest.fixture
def fixture_loader():
    return load_fixture
