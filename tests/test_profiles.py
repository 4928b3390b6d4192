"""The committed measurement evidence agrees with itself (CPU, no GPU).

bench.py's `roofline.traffic` falls back to profiles/pmc_<config>.json (live PMC passes otherwise), and
DESIGN quotes the default command's line next to the rocprofv3 kernel
averages of the same run (profiles/rNN/final/, the newest round).  These checks keep those
files consistent: PMC traffic equals the algorithmic bytes, and every timed
config's kernel_ms in the line under the profiler matches the profiler's own
average for that kernel.
"""
import csv
import glob
import json
import os

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
# the newest round's round-final profile (profiles/rNN/final/)
# (none on the GPU box, where old rounds' profiles are not shipped: skip)
FINAL = (sorted(glob.glob(os.path.join(ROOT, "profiles", "r[0-9][0-9]", "final"))) or [os.path.join(ROOT, "profiles", "none")])[-1]


def _line(path):
    with open(path) as f:
        lines = [x for x in f if x.startswith("{")]
    assert lines, path
    return json.loads(lines[-1])


def _stats(path):
    with open(path) as f:
        return {r["Name"]: (int(r["Calls"]), float(r["AverageNs"]) / 1e6) for r in csv.DictReader(f)}


def test_pmc_traffic_equals_algorithmic_bytes():
    files = sorted(glob.glob(os.path.join(ROOT, "profiles", "pmc_*.json")))
    assert files
    for path in files:
        j = json.load(open(path))
        assert j["kernels"], path
        # read = 2 x FETCH_SIZE KiB (gfx950 halving), write = WRITE_SIZE KiB
        assert j["hbm_bytes_per_launch"] == pytest.approx(
            j["read_bytes_per_launch"] + j["write_bytes_per_launch"], rel=1e-9)
        assert j["read_bytes_per_launch"] == pytest.approx(2 * 1024 * j["FETCH_SIZE_kib_per_launch"], rel=1e-9)
        algo = j["algorithmic_read_bytes"] + j["algorithmic_write_bytes"]
        assert j["traffic_over_algorithmic"] == pytest.approx(j["hbm_bytes_per_launch"] / algo, rel=1e-9)
        assert 0.999 <= j["traffic_over_algorithmic"] <= 1.001, path


@pytest.mark.parametrize("name,kernel_of", [
    ("configs[1]", lambda d: (d["roofline"]["kernel_ms"], "gf8_kernel<10, 4, false, 1, 64")),
    ("configs[2]", lambda d: (d["decode"]["kernel_ms"], "gf8_kernel<10, 4, false, 0, 256")),
    ("configs[4] encode", lambda d: (d["other_configs"]["configs[4]"]["kernel_ms"], "bm_kernel<4, 4, false, 64, 2>")),
    ("configs[4] decode", lambda d: (d["other_configs"]["configs[4]"]["decode"]["kernel_ms"],
                                     "bm_kernel<4, 4, false, 256, 4>")),
])
def test_default_line_agrees_with_rocprof(name, kernel_of):
    line = os.path.join(FINAL, "default_cmd_under_rocprof.json")
    stats = os.path.join(FINAL, "default_cmd_kernel_stats.csv")
    if not (os.path.exists(line) and os.path.exists(stats)):
        pytest.skip("round-final profile not present")
    d = _line(line)
    ms, kernel = kernel_of(d)
    hits = [v for k, v in _stats(stats).items() if kernel in k]
    assert len(hits) == 1, (kernel, hits)
    calls, avg_ms = hits[0]
    assert calls >= 20
    assert ms == pytest.approx(avg_ms, rel=0.03), (name, ms, avg_ms)


def test_default_line_pins_parity_on_every_timed_config():
    path = os.path.join(FINAL, "default_cmd_under_rocprof.json")
    if not os.path.exists(path):
        pytest.skip("round-final profile not present")
    d = _line(path)
    assert d["parity"]["equal"] and d["decode"]["parity"]["equal"]
    for name, c in d["other_configs"].items():
        assert c["parity"]["equal"], name
        if "decode" in c:
            assert c["decode"]["parity"]["equal"], name


def test_bench_live_pmc_parser_matches_the_committed_summary():
    """bench.py measures roofline.traffic live (rocprofv3 --pmc child passes,
    bench.live_traffic); its CSV parser must give the same per-launch
    counters as tools/pmc_summary.py gave for the committed profile."""
    import sys
    sys.path.insert(0, ROOT)
    import bench
    fetch = os.path.join(ROOT, "profiles", "r04", "final", "pmc", "pmc_fetch_rs_enc.csv")
    write = os.path.join(ROOT, "profiles", "r04", "final", "pmc", "pmc_write_rs_enc.csv")
    if not (os.path.exists(fetch) and os.path.exists(write)):
        pytest.skip("round-4 PMC CSVs not present")
    j = json.load(open(os.path.join(ROOT, "profiles", "pmc_rs_enc.json")))
    f, name = bench.pmc_per_launch(fetch, "FETCH_SIZE")
    w, _ = bench.pmc_per_launch(write, "WRITE_SIZE")
    assert "gf8_kernel<10, 4, false, 1, 64" in name
    assert f == pytest.approx(j["FETCH_SIZE_kib_per_launch"], rel=1e-12)
    assert w == pytest.approx(j["WRITE_SIZE_kib_per_launch"], rel=1e-12)


def test_bench_skips_live_pmc_under_a_profiler(monkeypatch):
    import sys
    sys.path.insert(0, ROOT)
    import bench
    monkeypatch.delenv("LD_PRELOAD", raising=False)
    for k in [k for k in os.environ if k.startswith("ROCPROF")]:
        monkeypatch.delenv(k)
    assert not bench.under_profiler()
    monkeypatch.setenv("LD_PRELOAD", "/opt/rocm/lib/rocprofiler-sdk/librocprofiler-sdk-tool.so")
    assert bench.under_profiler()
