"""Stripe sharding and timing across ranks (one process per GPU).

Stripes are independent, so a batch is partitioned into
contiguous stripe ranges with no data-path collective; RCCL (backend "nccl")
is used only for the start/end barriers and the max-over-ranks reduction of
the timings.  The same helpers run on CPU with backend "gloo" (tests).
"""
import time


def shard_range(n_stripes, rank, world):
    """Contiguous [begin, end) slice of n_stripes owned by `rank`
    (GPU g gets stripes [g*N/G, (g+1)*N/G))."""
    if world < 1 or not 0 <= rank < world:
        raise ValueError("bad rank/world")
    return n_stripes * rank // world, n_stripes * (rank + 1) // world


def dist_env():
    import os
    return (int(os.environ.get("WORLD_SIZE", "1")), int(os.environ.get("RANK", "0")),
            int(os.environ.get("LOCAL_RANK", "0")))


def max_over_ranks(values, dist=None, device="cpu"):
    """Element-wise max of a list of floats over all ranks."""
    if dist is None or not dist.is_initialized():
        return list(values)
    import torch
    t = torch.tensor(list(values), dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return [float(x) for x in t.tolist()]


def timed_steps(step, steps, warmup, sync=None, dist=None, events=None):
    """Run `warmup` untimed steps, then time exactly `steps` steps bracketed
    by a barrier + device sync on both sides.  Returns (wall_seconds,
    event_ms_per_step or None), each the max over ranks.

    events: optional (start_event, end_event) recorded on the launch stream
    around the timed steps (device-side duration)."""
    sync = sync or (lambda: None)
    use_dist = dist is not None and dist.is_initialized()
    for _ in range(warmup):
        step()
    sync()
    if use_dist:
        dist.barrier()
    sync()
    t0 = time.perf_counter()
    if events:
        events[0].record()
    for _ in range(steps):
        step()
    if events:
        events[1].record()
    sync()
    t1 = time.perf_counter()
    if use_dist:
        dist.barrier()
    ev_ms = events[0].elapsed_time(events[1]) / steps if events else -1.0
    wall, ev_ms = max_over_ranks([t1 - t0, ev_ms], dist if use_dist else None,
                                 device=_dist_device(dist) if use_dist else "cpu")
    return wall, (ev_ms if events else None)


def _dist_device(dist):
    backend = dist.get_backend()
    if backend == "gloo":
        return "cpu"
    import torch
    return torch.device("cuda", torch.cuda.current_device())
