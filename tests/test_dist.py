"""Multi-rank path on CPU (gloo, world_size 2): stripe sharding, barrier +
max-over-ranks timing (memec_amd.shard, the helpers bench.py uses), and a
checksum of checksums — every rank encodes only its own stripe range with
the CPU oracle and the union equals the single-process result."""
import hashlib
import json
import os
import socket

import numpy as np
import pytest

import _oracle as O
from memec_amd.shard import shard_range


def test_shard_range_partitions():
    for n in [0, 1, 7, 8, 4096, 32768, 32769]:
        for world in [1, 2, 3, 4, 8]:
            got = [shard_range(n, r, world) for r in range(world)]
            assert got[0][0] == 0 and got[-1][1] == n
            for (a, b), (c, d) in zip(got, got[1:]):
                assert b == c and a <= b
            sizes = [b - a for a, b in got]
            assert max(sizes) - min(sizes) <= 1
    with pytest.raises(ValueError):
        shard_range(8, 2, 2)


K, M, CS, N, SEED = 10, 4, 4096, 10, 77


def _stripe_digests(s0, s1):
    out = []
    for s in range(s0, s1):
        data = O.fill(K * CS, SEED, word_offset=s * K * CS // 8)
        par = O.encode("rs", K, M, [data[j * CS:(j + 1) * CS].copy() for j in range(K)], CS)
        out.append(hashlib.sha256(np.concatenate(par).tobytes()).hexdigest())
    return out


def _worker(rank, world, port, outdir):
    import torch.distributed as dist
    from memec_amd.shard import max_over_ranks, timed_steps

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    s0, s1 = shard_range(N, rank, world)
    box = {}

    def step():
        box["d"] = _stripe_digests(s0, s1)

    wall, ev = timed_steps(step, steps=2, warmup=1, dist=dist)
    gathered = [None] * world
    dist.all_gather_object(gathered, box["d"])
    mx = max_over_ranks([float(rank + 1)], dist)
    if rank == 0:
        with open(os.path.join(outdir, "r0.json"), "w") as f:
            json.dump({"digests": [d for part in gathered for d in part], "max": mx[0], "wall": wall,
                       "ev": ev}, f)
    dist.barrier()
    dist.destroy_process_group()


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_two_rank_gloo_shards_match_single_process(tmp_path):
    import torch.multiprocessing as mp
    world = 2
    mp.spawn(_worker, args=(world, _free_port(), str(tmp_path)), nprocs=world, join=True)
    rec = json.load(open(tmp_path / "r0.json"))
    assert rec["max"] == float(world)
    assert rec["wall"] > 0 and rec["ev"] is None
    assert rec["digests"] == _stripe_digests(0, N)
    # checksum of checksums
    assert hashlib.sha256("".join(rec["digests"]).encode()).hexdigest() == \
        hashlib.sha256("".join(_stripe_digests(0, N)).encode()).hexdigest()
