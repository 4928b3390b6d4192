#!/usr/bin/env python3
"""Interleaved A/B of the block-window count (MEC_WINDOWS) per bench config:
rounds x {1, 2, 4} windows, 10 launches each, HIP events; prints the median
and best kernel ms per window count.  Not product code."""
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

from bench import CONFIGS  # noqa: E402
from memec_amd import Codec, fill_random, set_knob  # noqa: E402


def run(cfg, rounds=5, wins=(1, 2, 4), var="MEC_WINDOWS"):
    fam, k, m, cs, n, op, erased = CONFIGS[cfg]
    codec = Codec(fam, k, m, cs, device=0)
    if op == "encode":
        data = torch.empty(n, k, cs, dtype=torch.uint8, device="cuda")
        fill_random(data, 1)
        par = torch.empty(n, m, cs, dtype=torch.uint8, device="cuda")
        step = lambda: codec.encode(data, par)  # noqa: E731
        nbytes = (k + m) * cs * n
    elif op == "update":
        delta = torch.empty(n, cs, dtype=torch.uint8, device="cuda")
        fill_random(delta, 1)
        par = torch.zeros(n, m, cs, dtype=torch.uint8, device="cuda")
        step = lambda: codec.encode_update(erased, delta, par)  # noqa: E731
        nbytes = (1 + 2 * m) * cs * n
    else:
        st = torch.empty(n, k + m, cs, dtype=torch.uint8, device="cuda")
        fill_random(st, 1)
        present = sum(1 << i for i in range(k + m) if i not in erased)
        step = lambda: codec.decode(st, present)  # noqa: E731
        nbytes = (k + len(erased)) * cs * n
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    res = {w: [] for w in wins}
    for _ in range(rounds):
        for w in wins:
            set_knob(var, str(w))
            step()
            ev[0].record()
            for _ in range(10):
                step()
            ev[1].record()
            ev[1].synchronize()
            res[w].append(ev[0].elapsed_time(ev[1]) / 10)
    for w in wins:
        med, best = statistics.median(res[w]), min(res[w])
        print(("%-10s " + var + "=%d  median %.4f ms (%.1f%%)  best %.4f ms (%.1f%%)") %
              (cfg, w, med, nbytes / med / 1e6 / 80, best, nbytes / best / 1e6 / 80), flush=True)
    codec.close()


if __name__ == "__main__":
    torch.cuda.set_device(0)
    var = os.environ.get("AB_VAR", "MEC_WINDOWS")
    vals = tuple(int(x) for x in os.environ.get("AB_VALUES", "1,2,4").split(","))
    for c in sys.argv[1:] or ["rs_enc", "rs_dec", "rs8_small", "crs_enc", "crs_dec", "rs42"]:
        run(c, wins=vals, var=var)
        torch.cuda.empty_cache()
