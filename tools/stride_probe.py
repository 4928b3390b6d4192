#!/usr/bin/env python3
"""RS(10,4) split-buffer encode at a fixed ~56 GiB of traffic: chunk size
64 KiB .. 4 MiB on dense [stripe][chunk][bytes] buffers, and 1 MiB chunks
with padded chunk / stripe strides (does the power-of-two spacing of the
k reads of a wave cost the 1 MiB config against the 64 KiB ones?).
Interleaved rounds, median kernel ms over 10 launches (HIP events).
Not product code.

  python3 tools/stride_probe.py [rounds=5]
"""
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

from memec_amd import Codec, fill_random  # noqa: E402

K, M = 10, 4
TOTAL = 56 << 30  # algorithmic bytes per launch, all arms


def main():
    rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 5
    torch.cuda.set_device(0)
    # (label, chunk, chunk-stride pad, stripe-stride pad)
    shapes = [("dense", 64 << 10, 0, 0), ("dense", 256 << 10, 0, 0), ("dense", 1 << 20, 0, 0),
              ("dense", 4 << 20, 0, 0), ("pad chunk +1K", 1 << 20, 1024, 0), ("pad chunk +4K", 1 << 20, 4096, 0),
              ("pad chunk +64K", 1 << 20, 65536, 0), ("pad stripe +4K", 1 << 20, 0, 4096),
              ("pad chunk 64K +1K", 64 << 10, 1024, 0)]
    pool_d = torch.empty(TOTAL * K // (K + M) * 107 // 100, dtype=torch.uint8, device="cuda")
    pool_p = torch.empty(TOTAL * M // (K + M) * 107 // 100, dtype=torch.uint8, device="cuda")
    fill_random(pool_d, 3)
    arms = []
    for label, cs, cpad, spad in shapes:
        n = TOTAL // ((K + M) * cs)
        dcs, pcs = cs + cpad, cs + cpad
        dss, pss = K * dcs + spad, M * pcs + spad
        assert n * dss <= pool_d.numel() and n * pss <= pool_p.numel()
        data = pool_d.as_strided((n, K, cs), (dss, dcs, 1))
        par = pool_p.as_strided((n, M, cs), (pss, pcs, 1))
        c = Codec("rs", K, M, cs)
        arms.append(("%-18s chunk %5d KiB, %5d stripes" % (label, cs >> 10, n),
                     (lambda c=c, d=data, p=par: c.encode(d, p)), (K + M) * cs * n, c))
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    res = [[] for _ in arms]
    for _ in range(rounds):
        for i, (_, step, _, _) in enumerate(arms):
            step()
            ev[0].record()
            for _ in range(10):
                step()
            ev[1].record()
            ev[1].synchronize()
            res[i].append(ev[0].elapsed_time(ev[1]) / 10)
    for (name, _, nbytes, _), r in zip(arms, res):
        med = statistics.median(r)
        print("%s  median %.4f ms  %.1f %% of 8 TB/s" % (name, med, nbytes / med / 1e6 / 80), flush=True)


if __name__ == "__main__":
    main()
