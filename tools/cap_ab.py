#!/usr/bin/env python3
"""Interleaved A/B of the default occupancy caps (gf8_target_waves /
bm_target_waves) against uncapped launches (MEC_WPC=0) on bench.py's own
configs, at their full BASELINE sizes.  Median kernel time of 10 launches
per sample, 5 rounds.  Not product code.

  python3 tools/cap_ab.py [config ...]   (default: every bench config)
"""
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

import bench  # noqa: E402
from memec_amd import Codec, fill_random, set_knob  # noqa: E402

ARMS = [("default", None), ("uncapped", "0")]
# CAP_ARMS="64:12,256:16,..." = MEC_BLOCK:MEC_WPC pairs ("-" leaves a knob unset)
GRID = [tuple(a.split(":")) for a in os.environ["CAP_ARMS"].split(",")] if os.environ.get("CAP_ARMS") else None


def workload(name, dev):
    fam, k, m, cs, n, op, extra = bench.CONFIGS[name]
    codec = Codec(fam, k, m, cs, device=0)
    if op == "encode":
        data = torch.empty(n, k, cs, dtype=torch.uint8, device=dev)
        fill_random(data, 1)
        par = torch.empty(n, m, cs, dtype=torch.uint8, device=dev)
        return codec, (lambda: codec.encode(data, par)), (k + m) * cs * n, [data, par]
    if op == "update":
        delta = torch.empty(n, cs, dtype=torch.uint8, device=dev)
        fill_random(delta, 2)
        par = torch.zeros(n, m, cs, dtype=torch.uint8, device=dev)
        return codec, (lambda: codec.encode_update(extra, delta, par)), (1 + 2 * m) * cs * n, [delta, par]
    st = torch.empty(n, k + m, cs, dtype=torch.uint8, device=dev)
    fill_random(st, 3)
    present = sum(1 << i for i in range(k + m) if i not in extra)
    return codec, (lambda: codec.decode(st, present)), (k + len(extra)) * cs * n, [st]


def main():
    names = sys.argv[1:] or list(bench.CONFIGS)
    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    for name in names:
        codec, step, nbytes, keep = workload(name, dev)
        arms = [("B%s/W%s" % g, g) for g in GRID] if GRID else [(a, ("-", v or "-")) for a, v in ARMS]
        res = {a: [] for a, _ in arms}
        for _ in range(5):
            for arm, (blk, wpc) in arms:
                for var, val in (("MEC_BLOCK", blk), ("MEC_WPC", wpc)):
                    if val == "-":
                        set_knob(var, None)
                    else:
                        set_knob(var, val)
                step()
                ev[0].record()
                for _ in range(10):
                    step()
                ev[1].record()
                ev[1].synchronize()
                res[arm].append(ev[0].elapsed_time(ev[1]) / 10)
        set_knob("MEC_WPC", None)
        set_knob("MEC_BLOCK", None)
        pct = {a: nbytes / (statistics.median(v) * 1e-3) / 8e12 * 100 for a, v in res.items()}
        if GRID:
            best = max(pct, key=pct.get)
            print("%-13s " % name + " ".join("%s %5.1f" % (a, pct[a]) for a, _ in arms) + "  best %s" % best,
                  flush=True)
            continue
        print("%-13s " % name + "  ".join("%s %.4f ms %5.1f %%" % (a, statistics.median(res[a]), pct[a])
                                          for a, _ in ARMS) + "   delta %+.1f" % (pct["default"] - pct["uncapped"]),
              flush=True)
        del keep, step, codec
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
