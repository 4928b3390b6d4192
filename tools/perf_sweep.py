#!/usr/bin/env python3
"""GPU counterpart of the reference's coding performance sweep
(scripts/test_coding.sh:5-39: chunk 2 KiB-128 KiB x k in {4,6,8,12}, m = 2,
driving test/common/coding/performance.cc).  Device-resident batches of
~2 GiB per launch: encode and decode of erasures {0,1} in place, best of 10
launches by HIP events, reported as data GiB/s (the reference's MB/s
convention, common.hh:17-22) and % of the 8 TB/s HBM peak over the
algorithmic bytes.  One JSON line per (family, k, chunk).  Not product code;
tools/perf_sweep.sh adds the single-stripe host rate (performance.cc's
Kop/s) through the C++ adapter."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

from memec_amd import Codec, fill_random  # noqa: E402

PEAK = 8000.0  # GB/s


def best_ms(fn, reps=10):
    fn()
    torch.cuda.synchronize()
    best = 1e9
    for _ in range(reps):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        fn()
        e1.record()
        e1.synchronize()
        best = min(best, e0.elapsed_time(e1))
    return best


def one(fam, k, m, cs, target=2 << 30):
    n = max(1, target // ((k + m) * cs))
    try:
        c = Codec(fam, k, m, cs, device=0)
    except Exception as e:  # e.g. no Cauchy w for this chunk size (cauchycoding.cc:191-198)
        return {"family": fam, "k": k, "m": m, "chunk": cs, "error": str(e)}
    st = torch.empty(n, k + m, cs, dtype=torch.uint8, device="cuda")
    fill_random(st, k * 131 + cs)
    enc = best_ms(lambda: c.encode(st[:, :k], st[:, k:]))
    orig = st[:, :2].clone()
    present = ((1 << (k + m)) - 1) & ~0b11
    st[:, :2].zero_()
    c.decode(st, present)
    ok = bool(torch.equal(st[:, :2], orig))
    dec = best_ms(lambda: c.decode(st, present))
    c.close()
    data = n * k * cs
    return {"family": fam, "k": k, "m": m, "chunk": cs, "stripes": n,
            "encode_ms": round(enc, 4), "encode_data_GiBps": round(data / enc / 1e-3 / 2**30, 1),
            "encode_frac": round(n * (k + m) * cs / enc / 1e6 / PEAK, 4),
            "decode_ms": round(dec, 4), "decode_data_GiBps": round(data / dec / 1e-3 / 2**30, 1),
            "decode_frac": round(n * (k + 2) * cs / dec / 1e6 / PEAK, 4), "decode_verified": ok}


def main():
    """SWEEP_FAMS=cauchy SWEEP_KS=6,8,12 SWEEP_SIZES=2048,16384 narrow the grid."""
    torch.cuda.set_device(0)
    fams = os.environ.get("SWEEP_FAMS", "rs,cauchy").split(",")
    ks = [int(x) for x in os.environ.get("SWEEP_KS", "4,6,8,12").split(",")]
    sizes = [int(x) for x in os.environ.get("SWEEP_SIZES", "2048,4096,8192,16384,32768,65536,131072").split(",")]
    for fam in fams:
        for k in ks:
            for cs in sizes:
                print(json.dumps(one(fam, k, 2, cs)), flush=True)
                torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
