"""Multi-rank GPU path (two ranks sharing cuda:0, gloo): every rank encodes
its stripe shard (memec_amd.shard.shard_range) with the HIP kernel, times
it with the bench's barrier + max-over-ranks helper, and the gathered
per-stripe parity digests equal a single-process encode of the whole batch
— the sharded bench path (bench.py, one process per GPU over RCCL at N > 1)
computes exactly what one process does."""
import hashlib
import json
import os
import socket

import pytest

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

K, M, CS, N, SEED = 10, 4, 65536, 96, 0x4D454D4543


def _digests(par):
    p = par.cpu().numpy()
    return [hashlib.sha256(p[s].tobytes()).hexdigest() for s in range(p.shape[0])]


def _worker(rank, world, port, outdir):
    import torch.distributed as dist
    from memec_amd import Codec, fill_random
    from memec_amd.shard import max_over_ranks, shard_range, timed_steps

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    s0, s1 = shard_range(N, rank, world)
    codec = Codec("rs", K, M, CS, device=0)
    data = torch.empty(s1 - s0, K, CS, dtype=torch.uint8, device="cuda:0")
    # stripe s of the global batch = words [s*K*CS/8, ...) of the seed stream
    fill_random(data, SEED, word_offset=s0 * K * CS // 8)
    par = torch.empty(s1 - s0, M, CS, dtype=torch.uint8, device="cuda:0")
    ev = (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
    wall, kern = timed_steps(lambda: codec.encode(data, par), steps=3, warmup=1,
                             sync=torch.cuda.synchronize, dist=dist, events=ev)
    gathered = [None] * world
    dist.all_gather_object(gathered, _digests(par))
    mx = max_over_ranks([float(s1 - s0)], dist)
    if rank == 0:
        with open(os.path.join(outdir, "r0.json"), "w") as f:
            json.dump({"digests": [d for part in gathered for d in part], "max": mx[0],
                       "wall": wall, "kern": kern}, f)
    dist.barrier()
    codec.close()
    dist.destroy_process_group()


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_two_ranks_share_gpu_and_match_single_process(tmp_path):
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import torch.multiprocessing as mp
    world = 2
    mp.spawn(_worker, args=(world, _free_port(), str(tmp_path)), nprocs=world, join=True)
    rec = json.load(open(tmp_path / "r0.json"))
    from memec_amd import Codec, fill_random
    torch.cuda.set_device(0)
    data = torch.empty(N, K, CS, dtype=torch.uint8, device="cuda:0")
    fill_random(data, SEED)
    par = torch.empty(N, M, CS, dtype=torch.uint8, device="cuda:0")
    Codec("rs", K, M, CS).encode(data, par)
    assert rec["digests"] == _digests(par)
    assert rec["max"] == float(N // world)
    assert rec["wall"] > 0 and rec["kern"] > 0
