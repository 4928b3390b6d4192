#!/usr/bin/env python3
"""Interleaved A/B of launch knobs for device-resident pointer-array batches
(mec_encode_batch / mec_decode_batch on chunks scattered over a ChunkPool-like
slab: slot = header + chunk, slots in random order, as tools/bench_batch.py).
Median per-call time over 5 rounds x 8 calls (host grouping + table upload
included, the same for every arm); GB/s over the algorithmic bytes.
Not product code.

  GA_ARMS='default:;g64:MEC_GBLOCK=64;g64w12:MEC_GBLOCK=64+MEC_GWPC=12' python3 tools/gather_ab.py
"""
import os
import statistics
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

from memec_amd import Codec, fill_random, set_knob  # noqa: E402

KNOBS = ("MEC_GBLOCK", "MEC_GWPC", "MEC_WPC", "MEC_BLOCK")
# (family, k, m, chunk, stripes, slot header; -1 = one contiguous [stripe][k+m][chunk] buffer, op)
CASES = [("rs", 10, 4, 1 << 20, 1024, 8, "encode"), ("rs", 10, 4, 1 << 20, 1024, 256, "encode"),
         ("rs", 8, 2, 4096, 65536, 8, "encode"), ("rs", 10, 4, 65536, 4096, 8, "encode"),
         ("rs", 10, 4, 65536, 4096, 256, "encode"),
         ("rs", 10, 4, 1 << 20, 1024, 8, "decode"), ("rs", 10, 4, 1 << 20, 1024, 256, "decode"),
         ("rs", 10, 4, 65536, 4096, -1, "decode"), ("rs", 10, 4, 65536, 4096, 8, "decode"),
         ("cauchy", 12, 4, 65536, 4096, 8, "encode"), ("cauchy", 12, 4, 65536, 4096, 256, "encode"),
         ("cauchy", 12, 4, 65536, 4096, -1, "decode"), ("cauchy", 12, 4, 65536, 4096, 8, "decode"),
         # 13..: 16-byte-aligned slots that are not line-aligned (tools/align_probe.hip)
         ("rs", 10, 4, 1 << 20, 1024, 16, "encode"), ("rs", 10, 4, 65536, 4096, 16, "encode"),
         ("rs", 10, 4, 65536, 4096, 64, "decode"), ("rs", 10, 4, 1 << 20, 1024, 128, "encode")]
if os.environ.get("GA_CASES"):  # indices into CASES
    CASES = [CASES[int(i)] for i in os.environ["GA_CASES"].split(",")]


def parse_arms(text):
    arms = []
    for item in text.split(";"):
        if item.strip():
            name, _, spec = item.partition(":")
            arms.append((name.strip(), dict(kv.split("=", 1) for kv in spec.split("+") if kv)))
    return arms


def main():
    arms = parse_arms(os.environ.get("GA_ARMS", "default:;g64:MEC_GBLOCK=64"))
    torch.cuda.set_device(0)
    for fam, k, m, cs, n, hdr, op in CASES:
        c = Codec(fam, k, m, cs)
        slot = cs + max(hdr, 0)
        slab = torch.empty(n * (k + m) * slot, dtype=torch.uint8, device="cuda")
        fill_random(slab, 1)
        if hdr < 0:  # contiguous stripes, chunk pointers in order
            rows = (np.arange(n * (k + m), dtype=np.uint64) * np.uint64(cs) + np.uint64(slab.data_ptr())).reshape(n, k + m)
        else:
            perm = np.random.default_rng(0).permutation(n * (k + m))
            rows = perm.reshape(n, k + m).astype(np.uint64) * np.uint64(slot) + np.uint64(slab.data_ptr() + hdr)
        dptr = np.ascontiguousarray(rows[:, :k]).reshape(-1)
        pptr = np.ascontiguousarray(rows[:, k:]).reshape(-1)
        allp = np.ascontiguousarray(rows).reshape(-1)
        masks = np.full(n, ((1 << (k + m)) - 1) & ~0b1111, dtype=np.uint64)
        call = (lambda: c.encode_batch(dptr, pptr)) if op == "encode" else (lambda: c.decode_batch(allp, masks))
        res = {a: [] for a, _ in arms}
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
        for _ in range(5):
            for arm, env in arms:
                for kn in KNOBS:
                    set_knob(kn, None)
                [set_knob(_k, _v) for _k, _v in env.items()]
                call()
                ev[0].record()
                for _ in range(8):
                    call()
                ev[1].record()
                ev[1].synchronize()
                res[arm].append(ev[0].elapsed_time(ev[1]) / 8)
        for kn in KNOBS:
            set_knob(kn, None)
        nbytes = n * (k + m) * cs  # encode: k + m chunks; decode of 4 erasures at m = 4: k + 4
        print("%-6s %-6s k=%-2d m=%d cs=%-7d hdr=%-3d " % (op, fam, k, m, cs, hdr) +
              " ".join("%s %6.1f GB/s" % (a, nbytes / (statistics.median(v) * 1e-3) / 1e9) for a, v in res.items()),
              flush=True)
        del slab
        c.close()
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
