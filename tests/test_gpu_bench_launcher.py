"""`python bench.py --gpus 2` on the one-GPU box: the parent spawns two rank
processes itself (no external launcher), both share cuda:0 over gloo
(MEC_BENCH_DIST_BACKEND=gloo stands in for RCCL with fewer GPUs than
ranks), and rank 0 prints one line with n_gpus 2, the process group's
world size, and encode/decode output verified on every rank."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(*extra, gpus=2):
    env = dict(os.environ, MEC_BENCH_DIST_BACKEND="gloo")
    for v in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(v, None)
    out = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", str(gpus), "--steps", "3",
                          "--warmup", "1", "--no-ceiling", *extra],
                         env=env, capture_output=True, text=True, timeout=600)
    assert out.returncode == 0, out.stderr[-3000:]
    lines = [l for l in out.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, out.stdout
    return json.loads(lines[0])


def test_bench_gpus2_spawns_ranks_weak():
    rec = _run("--stripes", "64")
    assert rec["n_gpus"] == 2
    assert rec["dist"]["world_size"] == 2 and rec["dist"]["backend"] == "gloo"
    assert rec["config"]["global_stripes"] == 128 and rec["config"]["stripes_per_gpu"] == 64
    assert rec["decode"]["verified"] is True
    assert rec["value"] > 0 and rec["roofline"]["kernel_ms"] > 0
    # the reference CPU path beside the N = 2 line too (rank 0, after the GPU legs)
    cb = rec["cpu_baseline"]
    assert cb["kind"] == "reference" and cb["matches_gpu"] is True and cb["value"] > 0, cb
    assert rec["decode"]["cpu_baseline"]["kind"] == "reference"
    assert rec["decode"]["cpu_baseline"]["matches_gpu"] is True


@pytest.mark.timeout(500)
def test_bench_gpus2_default_line_rehearsal():
    """The driver's default 8-GPU line at N=2: configs[1]/[2] on 64 stripes
    per rank plus other_configs — configs[3] per rank and the 32768-stripe
    configs[4] batch split 16384 / 16384 — every output verified and
    parity-pinned against the reference on both ranks."""
    rec = _run("--stripes", "64", "--extra-configs")
    assert rec["n_gpus"] == 2 and rec["dist"]["world_size"] == 2
    assert rec["parity"]["equal"] is True and rec["parity"]["ranks"] == 2
    assert rec["decode"]["verified"] is True and rec["decode"]["parity"]["equal"] is True
    assert rec["decode"]["parity"]["non_codeword_stripes"] > 0
    c0 = rec["other_configs"]["configs[0]"]
    assert c0["stripes_per_gpu"] == 65536 and c0["global_stripes"] == 131072 and c0["parity"]["equal"] is True
    assert c0["decode"]["verified"] is True and c0["decode"]["parity"]["equal"] is True
    assert c0["reference_cpu"]["encode_value"] > 0 and c0["reference_cpu"]["encode_matches_oracle"] is True
    assert rec["cpu_baseline"]["kind"] == "reference" and rec["cpu_baseline"]["matches_gpu"] is True
    c3, c4 = rec["other_configs"]["configs[3]"], rec["other_configs"]["configs[4]"]
    assert c3["stripes_per_gpu"] == 65536 and c3["global_stripes"] == 131072
    assert c3["verified"] is True and c3["parity"]["equal"] is True and c3["decode_parity"]["equal"] is True
    assert c4["scaling"] == "strong" and c4["stripes_per_gpu"] == 16384 and c4["global_stripes"] == 32768
    assert c4["parity"]["equal"] is True
    assert c4["decode"]["verified"] is True and c4["decode"]["parity"]["equal"] is True


def test_bench_gpus2_strong_crs():
    rec = _run("--config", "crs_enc", "--strong", "--stripes", "96", "--no-cpu-baseline")
    assert rec["n_gpus"] == 2 and rec["scaling"] == "strong"
    assert rec["config"]["global_stripes"] == 96 and rec["config"]["stripes_per_gpu"] == 48
    assert rec["decode"]["verified"] is True


def test_bench_under_launcher_uses_rccl():
    """Under torch.distributed.run, one rank on the one-GPU box: the same
    RCCL ("nccl") process group, barriers and max-over-ranks reductions the
    driver's 2/4/8-GPU runs use, exercised on the hardware."""
    env = dict(os.environ)
    env.pop("MEC_BENCH_DIST_BACKEND", None)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    for v in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(v, None)
    sys.path.insert(0, ROOT)
    import bench
    cmd = bench.launcher_cmd(["--gpus", "1", "--steps", "3", "--warmup", "1", "--no-ceiling", "--no-cpu-baseline",
                              "--stripes", "64", "--extra-configs"], 1, bench._free_port())
    out = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=300)
    assert out.returncode == 0, out.stderr[-3000:]
    lines = [l for l in out.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, out.stdout
    rec = json.loads(lines[0])
    assert rec["n_gpus"] == 1
    assert rec["dist"]["backend"] == "nccl" and rec["dist"]["rccl"] is True and rec["dist"]["world_size"] == 1
    assert rec["decode"]["verified"] is True
    assert rec["other_configs"]["configs[3]"]["verified"] is True
    assert rec["other_configs"]["configs[4]"]["decode"]["verified"] is True


@pytest.mark.timeout(500)
def test_bench_gpus4_carries_cpu_baseline():
    """N = 4 (four gloo ranks on the one GPU): the line rank 0 prints carries
    the reference CPU baseline, checked against rank 0's GPU parity."""
    rec = _run("--stripes", "32", gpus=4)
    assert rec["n_gpus"] == 4 and rec["dist"]["world_size"] == 4
    cb = rec["cpu_baseline"]
    assert cb["kind"] == "reference" and cb["matches_gpu"] is True and cb["cores"] >= 1, cb
    assert "rank 0 of 4" in cb["when"]


@pytest.mark.timeout(900)
def test_bench_gpus8_default_line_rehearsal():
    """The driver's 8-GPU default line rehearsed with 8 gloo ranks sharing
    the one GPU: world size 8; configs[4]'s 32768
    stripes sharded 4096 per rank; every parity pin and verification true
    on all 8 ranks; configs[0]'s reference leg and the reference CPU
    baseline timed on rank 0 after the other 7 ranks left; and the line's
    memory plan — with one rank per GPU at full size (56 GiB of configs[1]
    buffers, the 128 GiB decode-twin phase, 24 GiB of mec_xor streams on
    rank 0) — fits one device, the plan agreeing with the measured peak of
    this run on every rank."""
    rec = _run("--stripes", "64", "--extra-configs", gpus=8)
    assert rec["n_gpus"] == 8 and rec["dist"]["world_size"] == 8 and len(rec["dist"]["rank_devices"]) == 8
    assert rec["config"]["global_stripes"] == 8 * 64
    assert rec["parity"]["equal"] is True and rec["parity"]["ranks"] == 8
    assert rec["decode"]["verified"] is True and rec["decode"]["parity"]["equal"] is True
    oc = rec["other_configs"]
    c0, c3, c4 = oc["configs[0]"], oc["configs[3]"], oc["configs[4]"]
    assert c0["global_stripes"] == 8 * 65536 and c0["parity"]["equal"] is True and c0["decode"]["verified"] is True
    assert c3["global_stripes"] == 8 * 65536 and c3["verified"] is True and c3["parity"]["equal"] is True
    assert c4["scaling"] == "strong" and c4["stripes_per_gpu"] == 4096 and c4["global_stripes"] == 32768
    assert c4["parity"]["equal"] is True and c4["parity"]["ranks"] == 8
    assert c4["decode"]["verified"] is True and c4["decode"]["parity"]["equal"] is True
    assert c0["reference_cpu"]["encode_matches_oracle"] is True and c0["reference_cpu"]["kind"] == "reference"
    cb = rec["cpu_baseline"]
    assert cb["kind"] == "reference" and cb["matches_gpu"] is True and "rank 0 of 8" in cb["when"], cb
    assert rec["decode"]["cpu_baseline"]["kind"] == "reference"
    mp = rec["memory_plan"]
    full = mp["full_size_one_rank_per_gpu"]
    assert full["world"] == 8 and full["stripes_per_gpu"] == 4096
    assert full["phases"]["timed"] == 56 << 30 and full["phases"]["reference_streams"] == (56 + 24) << 30
    assert full["peak_bytes"] <= mp["device_bytes"] and mp["full_size_fits"] is True, mp
    plan = mp["this_run"]["peak_bytes"]
    assert len(mp["measured_peak_bytes_per_rank"]) == 8
    for got in mp["measured_peak_bytes_per_rank"]:
        assert 0.5 * plan <= got <= 1.3 * plan + (256 << 20), (got, plan)
