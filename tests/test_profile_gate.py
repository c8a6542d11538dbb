"""bench.py cites a PMC profile's traffic only when the profile was taken of the
running kernel code (the src= hash of mapfx_build_id: HIP sources, headers and
flags), of the kernel instance the bench launched (mapfx_last_kernel) and of the
same workload; otherwise traffic is null and the reason is reported (a
profile of a superseded build had been cited).  The git= part of the build id only
records where the library was built."""
import json
import os

import pytest

from conftest import REPO


@pytest.fixture
def bench_mod():
    import bench
    return bench


def _write(tmp_path, **kw):
    p = tmp_path / "pmc_x.json"
    p.write_text(json.dumps(kw))
    return str(p)


K = "void (anonymous namespace)::mapf_wave_kernel<5, true, true, true, 16, true, false, 8>(int*, int const*)"


def test_profile_of_this_build_and_kernel_is_cited(bench_mod, tmp_path):
    from mapfx import _abi
    p = _write(tmp_path, build_id=_abi.build_id(), kernel=K, config="c2", T=20, E=4096,
               traffic_bytes_per_launch=123, command="cmd")
    t, src = bench_mod.profile_traffic("x", kernel=K + " ", path=p, config="c2", T=20, E=4096)
    assert t == 123 and src.endswith("cmd")


def test_same_sources_built_at_another_commit_are_cited(bench_mod, tmp_path):
    from mapfx import _abi
    src_part = _abi.build_id().split()[0]
    p = _write(tmp_path, build_id=src_part + " git=0123456789ab", kernel=K, config="c2", T=20,
               E=4096, traffic_bytes_per_launch=7, command="cmd")
    t, src = bench_mod.profile_traffic("x", kernel=K, path=p, config="c2", T=20, E=4096)
    assert t == 7 and "git=0123456789ab" in src


def test_same_unit_other_units_changed_is_cited(bench_mod, tmp_path):
    """A profile stays valid when only OTHER translation units changed: the tu= hash of
    the unit that defines the kernel (mapfx.hip for mapf_wave_kernel) matches."""
    from mapfx import _abi
    bid = _abi.build_id()
    tu = [p for p in bid.split() if p.startswith("tu=")][0]
    items = dict(i.split(":") for i in tu[3:].split(","))
    items["partial"] = "0" * 12                     # another unit differs
    other = "src=ffffffffffffffff git=abc tu=" + ",".join("%s:%s" % kv for kv in items.items())
    p = _write(tmp_path, build_id=other, kernel=K, config="c2", T=20, E=4096,
               traffic_bytes_per_launch=9, command="cmd")
    t, src = bench_mod.profile_traffic("x", kernel=K, path=p, config="c2", T=20, E=4096)
    assert t == 9
    items["mapfx"] = "1" * 12                       # the kernel's own unit differs
    other = "src=ffffffffffffffff git=abc tu=" + ",".join("%s:%s" % kv for kv in items.items())
    p = _write(tmp_path, build_id=other, kernel=K, config="c2", T=20, E=4096,
               traffic_bytes_per_launch=9, command="cmd")
    t, src = bench_mod.profile_traffic("x", kernel=K, path=p, config="c2", T=20, E=4096)
    assert t is None and "taken of build" in src


def test_kernel_units():
    import bench
    assert bench.kernel_unit("void (anonymous namespace)::partial_kernel<5, 5, 16, 1, false>(a)") == "partial"
    assert bench.kernel_unit(K) == "mapfx"
    assert bench.kernel_unit("void (anonymous namespace)::primal_seq_kernel<10, false>(x)") == "primal"


@pytest.mark.parametrize("field,value,why", [
    ("build_id", "src=0000000000000000 git=deadbeef", "taken of build"),
    ("build_id", "src=unknown git=unknown", "taken of build"),
    ("kernel", K.replace("false, 8>", "false, 0>"), "profiled kernel"),
    ("T", 64, "workload keys"),
])
def test_stale_profile_is_refused(bench_mod, tmp_path, field, value, why):
    from mapfx import _abi
    d = dict(build_id=_abi.build_id(), kernel=K, config="c2", T=20, E=4096,
             traffic_bytes_per_launch=123)
    d[field] = value
    t, src = bench_mod.profile_traffic("x", kernel=K, path=_write(tmp_path, **d), config="c2", T=20, E=4096)
    assert t is None and why in src


def test_committed_profiles_name_their_instance():
    """Every committed profiles/pmc_*.json records the build and the exact kernel instance
    it measured, and its trace saw that instance."""
    import glob
    files = sorted(glob.glob(os.path.join(REPO, "profiles", "pmc_*.json")))
    assert files
    for f in files:
        d = json.load(open(f))
        assert d.get("build_id", "").startswith("src=") and "<" in d.get("kernel", ""), f
        names = [k["name"] for k in d["trace"]["kernels"]]
        assert any(n.split("(")[0] == d["kernel"].split("(")[0] or n == d["kernel"] for n in names) or \
            any(n[:n.find("(", n.find("<"))] == d["kernel"][:d["kernel"].find("(", d["kernel"].find("<"))]
                for n in names), f
