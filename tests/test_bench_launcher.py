"""bench.py's multi-rank entry (`python bench.py --gpus N` without a
launcher): the command it builds, the real spawn of N ranks (rehearsed on
CPU with --dist-check, gloo), the rank-count check, and the host-core probe
behind the CPU baseline."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402


def _env():
    env = dict(os.environ)
    for v in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(v, None)
    return env


def test_launcher_cmd_shape():
    cmd = bench.launcher_cmd(["--gpus", "8", "--config", "crs_enc", "--strong", "--stripes", "32768"], 8, 29555,
                             python="/usr/bin/python3")
    assert cmd[:3] == ["/usr/bin/python3", "-m", "torch.distributed.run"]
    assert "--nnodes=1" in cmd and "--nproc-per-node=8" in cmd
    assert "--master-addr=127.0.0.1" in cmd and "--master-port=29555" in cmd
    i = cmd.index(os.path.join(ROOT, "bench.py"))
    assert cmd[i + 1:] == ["--gpus", "8", "--config", "crs_enc", "--strong", "--stripes", "32768"]


def test_spawn_two_ranks_on_cpu():
    out = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--dist-check"],
                         env=_env(), capture_output=True, text=True, timeout=240)
    assert out.returncode == 0, out.stderr[-2000:]
    lines = [l for l in out.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, out.stdout
    rec = json.loads(lines[0])
    assert rec["n_gpus"] == 2 and rec["world_size"] == 2
    ranks = sorted(tuple(r) for r in rec["ranks"])
    assert [r[0] for r in ranks] == [0, 1] and [r[1] for r in ranks] == [0, 1]
    assert len({r[2] for r in ranks}) == 2  # two processes
    assert os.getpid() not in {r[2] for r in ranks}


def test_single_gpu_runs_in_process():
    out = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--dist-check"],
                         env=_env(), capture_output=True, text=True, timeout=240)
    assert out.returncode == 0, out.stderr[-2000:]
    rec = json.loads(out.stdout.strip().splitlines()[-1])
    assert rec["world_size"] == 1 and rec["n_gpus"] == 1


def test_rank_count_mismatch_fails_loudly():
    env = _env()
    env.update(WORLD_SIZE="2", RANK="0", LOCAL_RANK="0")
    out = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "4", "--dist-check"],
                         env=env, capture_output=True, text=True, timeout=120)
    assert out.returncode != 0
    assert "--gpus 4" in out.stderr


def test_host_cores():
    threads, info = bench.host_cores()
    assert threads >= 1
    assert info["affinity"] >= 1 and info["nproc"] >= info["affinity"]
    if info["cgroup_cpu_quota"]:
        assert threads <= max(1, int(info["cgroup_cpu_quota"] + 0.5))
    else:
        assert threads == info["affinity"]


def test_extra_configs_are_baseline_configs():
    """The default line's other_configs: configs[0]'s RS(4,2)@4 KiB shape on
    the GPU per GPU (weak, encode + timed decode {0,1}), configs[3] per GPU
    (weak) and configs[4] as BASELINE's 32768-stripe global batch sharded
    over ranks."""
    labels = {label: (name, strong) for label, name, strong in bench.EXTRA_CONFIGS}
    assert labels == {"configs[0]": ("rs42", None), "configs[3]": ("rs8_small", None),
                      "configs[4]": ("crs_enc", 32768)}
    assert bench.DECODE_TWINS == {"crs_enc": "crs_dec", "rs42": "rs42_dec"}
    fam, k, m, cs, stripes, op, _ = bench.CONFIGS["rs42"]
    assert (fam, k, m, cs, op) == ("rs", 4, 2, 4096, "encode") and bench.CONFIGS["rs42_dec"][6] == [0, 1]
    assert "stripes total" not in bench.workload_name("rs42_dec", 65536, False, 65536)
    fam, k, m, cs, stripes, op, _ = bench.CONFIGS["rs8_small"]
    assert (fam, k, m, cs, stripes, op) == ("rs", 8, 2, 4096, 65536, "encode")
    fam, k, m, cs, stripes, op, _ = bench.CONFIGS["crs_enc"]
    assert (fam, k, m, cs, op) == ("cauchy", 12, 4, 65536, "encode")
    assert bench.CONFIGS["crs_dec"][6] == [0, 1, 2, 3]
    name = bench.workload_name("crs_enc", 4096, True, 32768)
    assert "32768 stripes total, sharded over ranks" in name and "configs[4]" in name
    assert bench.workload_name("rs8_small", 65536) == bench.WORKLOAD_NAMES["rs8_small"]
