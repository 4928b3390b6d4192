#!/usr/bin/env python3
"""Interleaved A/B of libmec's launch knobs (any MEC_* environment
variables, read per launch) on bench.py's configs at their full BASELINE
sizes.  Median kernel time of 10 launches per sample, 5 rounds; % of 8 TB/s
over the algorithmic bytes.  Not product code.

  ENV_ARMS='default:;b64w1:MEC_BLOCK=64+MEC_WINDOWS=1' python3 tools/env_ab.py rs_dec crs_dec
"""
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))
import torch  # noqa: E402

import bench  # noqa: E402
from cap_ab import workload  # noqa: E402
from memec_amd import set_knob  # noqa: E402

KNOBS = ("MEC_BLOCK", "MEC_WINDOWS", "MEC_WPC", "MEC_BM_VW")


def parse_arms(text):
    arms = []
    for item in text.split(";"):
        if not item.strip():
            continue
        name, _, spec = item.partition(":")
        env = dict(kv.split("=", 1) for kv in spec.split("+") if kv)
        arms.append((name.strip(), env))
    return arms


def main():
    arms = parse_arms(os.environ.get("ENV_ARMS", "default:"))
    names = sys.argv[1:] or list(bench.CONFIGS)
    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    for name in names:
        codec, step, nbytes, keep = workload(name, dev)
        res = {a: [] for a, _ in arms}
        for _ in range(5):
            for arm, env in arms:
                for k in KNOBS:
                    set_knob(k, None)
                [set_knob(_k, _v) for _k, _v in env.items()]
                step()
                ev[0].record()
                for _ in range(10):
                    step()
                ev[1].record()
                ev[1].synchronize()
                res[arm].append(ev[0].elapsed_time(ev[1]) / 10)
        for k in KNOBS:
            set_knob(k, None)
        pct = {a: nbytes / (statistics.median(v) * 1e-3) / 8e12 * 100 for a, v in res.items()}
        best = max(pct, key=pct.get)
        print("%-13s " % name + " ".join("%s %5.1f" % (a, pct[a]) for a, _ in arms) +
              "  best %s (%+.1f)" % (best, pct[best] - pct[arms[0][0]]), flush=True)
        del keep, step, codec
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
