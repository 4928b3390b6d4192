#!/usr/bin/env python3
"""Interleaved A/B of mec_xor launch shapes (MEC_BLOCK x MEC_WPC) over
3 x 8 GiB, the bench's streaming-ceiling measurement.  Median ms of 5 launches
x rounds.  Not product code."""
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

from memec_amd import fill_random, xor, set_knob  # noqa: E402


def main():
    rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 5
    torch.cuda.set_device(0)
    n = 8 << 30
    a = torch.empty(n, dtype=torch.uint8, device="cuda")
    b = torch.empty_like(a)
    o = torch.empty_like(a)
    fill_random(a, 1)
    fill_random(b, 2)
    xor(o, a, b)
    torch.cuda.synchronize()
    assert torch.equal(o[:1 << 20], a[:1 << 20] ^ b[:1 << 20])
    arms = [(bt, w) for bt in ("64", "256") for w in (None, "0", "12", "16", "20", "24")]
    res = {x: [] for x in arms}
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    for _ in range(rounds):
        for bt, w in arms:
            set_knob("MEC_BLOCK", bt)
            if w is None:
                set_knob("MEC_WPC", None)
            else:
                set_knob("MEC_WPC", w)
            xor(o, a, b)
            ev[0].record()
            for _ in range(5):
                xor(o, a, b)
            ev[1].record()
            ev[1].synchronize()
            res[(bt, w)].append(ev[0].elapsed_time(ev[1]) / 5)
    for x in arms:
        med = statistics.median(res[x])
        print("block %-3s wpc %-7s %.3f ms  %.1f GB/s  %.1f %%" % (x[0], x[1] or "default", med, 3 * n / med / 1e6,
                                                                  3 * n / med / 1e6 / 80), flush=True)


if __name__ == "__main__":
    main()
