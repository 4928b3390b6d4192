#!/usr/bin/env python3
"""A/B of wide codes (m > 4) between kernel arms, interleaved in one
process: "bs" the run-time compiled bit-sliced kernel (MEC_BITSLICE=2,
compiled before timing), "mg" the one-pass multi-group kernel
(gf8_mg_kernel, MEC_BITSLICE=0), "split" 4-row launches that re-read the
sources (MEC_BITSLICE=0 MEC_WIDE=0).

  python tools/wide_ab.py [--arms bs,mg] [--steps N] [--shape I]

Every launch is checked against the other arm's parity (bit-exact), and the
GPU time per step (HIP events around `steps` encodes / decodes) is printed
as JSON lines.  Under `rocprofv3 --pmc FETCH_SIZE` (or WRITE_SIZE) run one
mode only: the counter CSV then holds exactly warmup + steps coding steps
after the fill launches, and tools/wide_ab.py --summarise sums them per step.
"""
import argparse
import csv
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

SHAPES = [("rs", 16, 8, 65536, 16384, "encode"), ("isal_rs", 12, 8, 65536, 16384, "encode"),
          ("rs", 16, 8, 65536, 16384, "decode"), ("rs", 10, 6, 262144, 4096, "encode"),
          ("isal_cauchy", 12, 6, 65536, 16384, "encode"), ("rs", 8, 5, 16384, 32768, "encode"),
          ("isal_cauchy", 20, 8, 4096, 65536, "encode"), ("rs", 10, 6, 262144, 4096, "decode"),
          ("rs", 4, 12, 1 << 20, 512, "encode"), ("cauchy", 10, 6, 65536, 16384, "encode"),
          ("cauchy", 10, 6, 65536, 16384, "decode"), ("cauchy", 8, 5, 16384, 32768, "encode"),
          ("cauchy", 20, 8, 40960, 8192, "encode"), ("cauchy", 20, 8, 40960, 8192, "decode"),
          ("rs", 16, 8, 65536, 16384, "batch"), ("isal_rs", 12, 8, 65536, 16384, "batch"),
          ("cauchy", 10, 6, 65536, 16384, "batch"), ("rs", 10, 4, 1 << 20, 4096, "batch"),
          ("rs", 10, 4, 1 << 20, 4096, "encode"), ("rs", 4, 12, 1 << 20, 512, "decode"),
          ("isal_cauchy", 4, 12, 1 << 20, 512, "encode"), ("rs", 10, 6, 262144, 4096, "batch"),
          ("rs", 16, 8, 65536, 16384, "batchdec"), ("rs", 16, 8, 4096, 131072, "encode"),
          ("isal_rs", 12, 8, 4096, 131072, "encode"), ("rs", 16, 8, 4096, 131072, "batch"),
          ("rs", 8, 6, 8192, 131072, "encode"), ("rs", 16, 8, 4096, 131072, "decode"),
          ("isal_rs", 12, 8, 65536, 16384, "decode"), ("rs", 8, 5, 16384, 32768, "decode"),
          ("isal_cauchy", 12, 6, 65536, 16384, "decode"), ("rs", 10, 6, 65536, 16384, "decode"),
          ("rs", 8, 2, 4096, 65536, "encode"), ("rs", 8, 2, 4096, 65536, "batch"),
          ("rs", 8, 2, 4096, 262144, "encode"), ("rs", 8, 2, 4096, 262144, "batch"),
          # 32-bit slab offsets (mec_encode_batch32, ABI 6) over the same chunks
          ("rs", 8, 2, 4096, 65536, "batch32"), ("rs", 8, 2, 4096, 262144, "batch32"),
          ("rs", 10, 4, 1 << 20, 4096, "batch32"), ("rs", 16, 8, 65536, 16384, "batch32"),
          # one-map gathered gf8 at 4 KiB and 64 KiB (MEC_GU A/B): strided and batch of the same chunks
          ("rs", 10, 4, 4096, 65536, "encode"), ("rs", 10, 4, 4096, 65536, "batch"),
          ("rs", 4, 2, 4096, 65536, "encode"), ("rs", 4, 2, 4096, 65536, "batch"),
          ("rs", 10, 4, 65536, 16384, "encode"), ("rs", 10, 4, 65536, 16384, "batch"),
          ("rs", 8, 2, 4096, 65536, "batchdec"),
          # MEC_GU rule sweep: one-map 4 KiB batches by source and output count
          ("rs", 2, 2, 4096, 131072, "batch"), ("rs", 3, 2, 4096, 131072, "batch"), ("rs", 5, 2, 4096, 65536, "batch"),
          ("rs", 6, 2, 4096, 65536, "batch"), ("rs", 4, 1, 4096, 131072, "batch"), ("rs", 4, 3, 4096, 65536, "batch"),
          ("rs", 4, 4, 4096, 65536, "batch"), ("rs", 4, 2, 4096, 65536, "batchdec"), ("rs", 4, 2, 8192, 32768, "batch"),
          ("rs", 4, 2, 65536, 4096, "batch"),
          # Cauchy-RS bitmatrix batches against strided launches of the same chunks
          ("cauchy", 12, 4, 65536, 4096, "encode"), ("cauchy", 12, 4, 65536, 4096, "batch"),
          ("cauchy", 4, 2, 4096, 65536, "encode"), ("cauchy", 4, 2, 4096, 65536, "batch"),
          ("cauchy", 8, 2, 4096, 65536, "encode"), ("cauchy", 8, 2, 4096, 65536, "batch"),
          ("cauchy", 12, 4, 65536, 4096, "batchdec"), ("cauchy", 4, 2, 4096, 65536, "batchdec"),
          # one-map gf8 decode batches (block windows A/B)
          ("rs", 10, 4, 4096, 65536, "batchdec"), ("rs", 10, 4, 65536, 16384, "batchdec"),
          ("rs", 10, 4, 1 << 20, 1024, "batchdec"), ("isal_rs", 6, 3, 4096, 65536, "batchdec"),
          ("rs", 8, 2, 4096, 262144, "batchdec"), ("rs", 12, 4, 16384, 16384, "batchdec")]


ARMS = {"bs": {"MEC_BITSLICE": "3"}, "auto": {"MEC_BITSLICE": "2"}, "mg": {"MEC_BITSLICE": "0"},
        "bs3": {"MEC_BITSLICE": "3", "MEC_BS_WAVES": "3"}, "bs4": {"MEC_BITSLICE": "3", "MEC_BS_WAVES": "4"},
        "bs5": {"MEC_BITSLICE": "3", "MEC_BS_WAVES": "5"}, "bsp0": {"MEC_BITSLICE": "3", "MEC_BS_PREFETCH": "0"},
        "bsp2": {"MEC_BITSLICE": "3", "MEC_BS_PREFETCH": "2"}, "bsp8": {"MEC_BITSLICE": "3", "MEC_BS_PREFETCH": "8"},
        "bst4": {"MEC_BITSLICE": "3", "MEC_BS_TPB": "4"}, "bst2": {"MEC_BITSLICE": "3", "MEC_BS_TPB": "2"},
        "bst8": {"MEC_BITSLICE": "3", "MEC_BS_TPB": "8"}, "bst16": {"MEC_BITSLICE": "3", "MEC_BS_TPB": "16"},
        "bsw4": {"MEC_BITSLICE": "3", "MEC_WPC": "4"}, "bsw6": {"MEC_BITSLICE": "3", "MEC_WPC": "6"},
        "bsw8": {"MEC_BITSLICE": "3", "MEC_WPC": "8"}, "bsw10": {"MEC_BITSLICE": "3", "MEC_WPC": "10"},
        "bsnocap": {"MEC_BITSLICE": "3", "MEC_WPC": "0"}, "mgw": {"MEC_BITSLICE": "0"},
        # gathered: tiles per block x wave cap
        "t2w8": {"MEC_BITSLICE": "3", "MEC_BS_TPB": "2", "MEC_WPC": "8"},
        "t2w12": {"MEC_BITSLICE": "3", "MEC_BS_TPB": "2", "MEC_WPC": "12"},
        "t4w8": {"MEC_BITSLICE": "3", "MEC_BS_TPB": "4", "MEC_WPC": "8"},
        "t4w12": {"MEC_BITSLICE": "3", "MEC_BS_TPB": "4", "MEC_WPC": "12"},
        "t8w8": {"MEC_BITSLICE": "3", "MEC_BS_TPB": "8", "MEC_WPC": "8"},
        "t1w12": {"MEC_BITSLICE": "3", "MEC_WPC": "12"}, "t1w16": {"MEC_BITSLICE": "3", "MEC_WPC": "16"},
        "bsw5": {"MEC_BITSLICE": "3", "MEC_WPC": "5"}, "bsw7": {"MEC_BITSLICE": "3", "MEC_WPC": "7"},
        "bsw12": {"MEC_BITSLICE": "3", "MEC_WPC": "12"},
        "bsnf": {"MEC_BITSLICE": "3", "MEC_BS_FENCE": "0"}, "bsf1": {"MEC_BITSLICE": "3", "MEC_BS_FENCE": "1"}, "autonf": {"MEC_BITSLICE": "2", "MEC_BS_FENCE": "0"},
        "split": {"MEC_BITSLICE": "0", "MEC_WIDE": "0"},
        # gathered pointer rows: one vector load (default) / a scalar load per entry; XCD runs; row prefetch
        "bsrow": {"MEC_BITSLICE": "3", "MEC_BS_VROW": "1"}, "bssrow": {"MEC_BITSLICE": "3", "MEC_BS_VROW": "0"},
        "bsxcd": {"MEC_BITSLICE": "3", "MEC_BS_XCD": "1"}, "bsnx": {"MEC_BITSLICE": "3", "MEC_BS_XCD": "0"},
        "bsx5": {"MEC_BITSLICE": "3", "MEC_BS_XCD": "1", "MEC_WPC": "5"},
        "bsnxw8": {"MEC_BITSLICE": "3", "MEC_BS_XCD": "0", "MEC_WPC": "8"},
        "bsnxw10": {"MEC_BITSLICE": "3", "MEC_BS_XCD": "0", "MEC_WPC": "10"},
        "bsnxw12": {"MEC_BITSLICE": "3", "MEC_BS_XCD": "0", "MEC_WPC": "12"},
        "bsnxw0": {"MEC_BITSLICE": "3", "MEC_BS_XCD": "0", "MEC_WPC": "0"},
        "bsx6": {"MEC_BITSLICE": "3", "MEC_BS_XCD": "1", "MEC_WPC": "6"},
        "bsx7": {"MEC_BITSLICE": "3", "MEC_WPC": "7"}, "bsx8": {"MEC_BITSLICE": "3", "MEC_WPC": "8"},
        # gathered (<= 4-output) launches: wave cap per CU (MEC_GWPC; rule 16 for 128 B-aligned chunks)
        "gw8": {"MEC_GWPC": "8"}, "gw10": {"MEC_GWPC": "10"}, "gw12": {"MEC_GWPC": "12"}, "gw16": {"MEC_GWPC": "16"},
        "gw20": {"MEC_GWPC": "20"}, "gw24": {"MEC_GWPC": "24"}, "gw0": {"MEC_GWPC": "0"},
        # pointer-table copy: the launch waits on the device (tw0, rule) or on the host while its stream is busy (tw1)
        "tw0": {"MEC_TAB_WAIT": "0"}, "tw1": {"MEC_TAB_WAIT": "1"},
        # one-map gathered gf8 launches: XCD runs off / on, with caps
        "gx0": {"MEC_GXCD": "0"}, "gx1": {"MEC_GXCD": "1"}, "gx1w10": {"MEC_GXCD": "1", "MEC_GWPC": "10"},
        "gx1w12": {"MEC_GXCD": "1", "MEC_GWPC": "12"},
        # one-map gathered gf8: two 16-byte units per lane (MEC_GU=2), with caps
        "gu1": {"MEC_GU": "1"}, "gu2": {"MEC_GU": "2"}, "gu2w8": {"MEC_GU": "2", "MEC_GWPC": "8"},
        "gu2w10": {"MEC_GU": "2", "MEC_GWPC": "10"}, "gu2w12": {"MEC_GU": "2", "MEC_GWPC": "12"},
        "gu2w20": {"MEC_GU": "2", "MEC_GWPC": "20"},
        # gathered block shape (MEC_GBLOCK) with caps: bitmatrix one-map batches at 4 KiB
        "gb64": {"MEC_GBLOCK": "64"}, "gb64w16": {"MEC_GBLOCK": "64", "MEC_GWPC": "16"},
        "gb64w12": {"MEC_GBLOCK": "64", "MEC_GWPC": "12"}, "gb64w20": {"MEC_GBLOCK": "64", "MEC_GWPC": "20"},
        "vw2": {"MEC_BM_VW": "2"}, "vw4": {"MEC_BM_VW": "4"},
        "win1": {"MEC_WINDOWS": "1"}, "win2": {"MEC_WINDOWS": "2"}, "win4": {"MEC_WINDOWS": "4"},
        # arithmetic-free twins (mec_set_probe): the same launch's loads and stores, no products
        "bstwin": {"MEC_BITSLICE": "3", "PROBE": "xor"}, "bsnftwin": {"MEC_BITSLICE": "3", "MEC_BS_FENCE": "0", "PROBE": "xor"}}
KNOBS = sorted({kn for a in ARMS.values() for kn in a if kn.startswith("MEC_")})


def run(arms_list, steps, warmup, shapes):
    import torch
    import memec_amd
    from memec_amd import Codec, fill_random
    torch.cuda.set_device(0)
    out = []
    for fam, k, m, cs, n, op in shapes:
        c = Codec(fam, k, m, cs)
        data = torch.empty(n, k, cs, dtype=torch.uint8, device="cuda")
        fill_random(data, 1234)
        if op in ("encode", "batch", "batch32"):
            par = torch.empty(n, m, cs, dtype=torch.uint8, device="cuda")
            if op == "encode":
                step = lambda: c.encode(data, par)  # noqa: E731
            else:  # the pointer-array ABI (mec_encode_batch) over the same chunks
                # uint64 arrays built once (no per-step Python list conversion)
                import numpy as np
                db, pb = data.data_ptr(), par.data_ptr()
                dptr = (db + (np.arange(n, dtype=np.uint64)[:, None] * k + np.arange(k, dtype=np.uint64)) * cs).ravel()
                pptr = (pb + (np.arange(n, dtype=np.uint64)[:, None] * m + np.arange(m, dtype=np.uint64)) * cs).ravel()
                step = lambda: c.encode_batch(dptr, pptr, mem="device")  # noqa: E731
                if op == "batch32":  # offsets from the lower of the two buffers, in the smallest unit that fits
                    base = min(db, pb)
                    span = int(max(dptr.max(), pptr.max()) - base) + cs
                    sh = 3
                    while span >> sh >= 2 ** 32 - 1:
                        sh += 1
                    assert all(int(x - base) % (1 << sh) == 0 for x in (dptr[:64].tolist() + pptr[:64].tolist()))
                    doff = ((dptr - np.uint64(base)) >> np.uint64(sh)).astype(np.uint32)
                    poff = ((pptr - np.uint64(base)) >> np.uint64(sh)).astype(np.uint32)
                    step = lambda: c.encode_batch32(base, sh, doff, poff)  # noqa: E731
            alg = (k + m) * cs * n
            result = lambda: par  # noqa: E731
        else:
            st = torch.empty(n, k + m, cs, dtype=torch.uint8, device="cuda")
            st[:, :k] = data
            c.encode(st[:, :k], st[:, k:])
            erased = list(range(m))
            present = sum(1 << i for i in range(k + m) if i not in erased)
            orig = st[:, erased].clone()
            st[:, erased] = 0
            if op == "batchdec":  # the pointer-array ABI (mec_decode_batch), one pattern: one-map batch
                import numpy as np
                sb = st.data_ptr()
                cptr = (sb + (np.arange(n, dtype=np.uint64)[:, None] * (k + m) + np.arange(k + m, dtype=np.uint64)) * cs).ravel()
                masks = np.full(n, present, dtype=np.uint64)
                step = lambda: c.decode_batch(cptr, masks, mem="device", as_array=True)  # noqa: E731
            else:
                step = lambda: c.decode(st, present)  # noqa: E731
            alg = (k + m) * cs * n
            result = lambda: st[:, erased]  # noqa: E731
        arms = {}
        for arm in arms_list:
            for kn in KNOBS:  # every knob any arm sets: unset unless this arm sets it
                memec_amd.set_knob(kn, ARMS[arm].get(kn))
            c.set_probe(ARMS[arm].get("PROBE") == "xor")
            j0 = c.stats()["jit_launches"]
            for _ in range(warmup):
                step()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(steps):
                step()
            e1.record()
            e1.synchronize()
            ms = e0.elapsed_time(e1) / steps
            if arm in arms:  # a repeated arm (interleaved A/B): keep the earlier timings
                arms.setdefault(arm + "_runs", []).append(arms[arm]["frac"])
            arms[arm] = {"ms_per_step": round(ms, 4), "GBps": round(alg / (ms * 1e-3) / 1e9, 1),
                         "frac": round(alg / (ms * 1e-3) / 8e12, 4)}
            arms[arm]["digest"] = int(result().view(torch.int64).sum().item())
            arms[arm]["jit_launches"] = c.stats()["jit_launches"] - j0  # warmup + timed steps on the JIT kernel
        for kn in KNOBS:
            memec_amd.set_knob(kn, None)
        c.set_probe(False)
        rec = {"family": fam, "k": k, "m": m, "chunk": cs, "stripes": n, "op": op, "alg_bytes": alg, **arms}
        if op == "decode":
            rec["restored"] = bool(torch.equal(result(), orig))
        rec["equal"] = len({arms[a]["digest"] for a in arms_list if "PROBE" not in ARMS[a]}) == 1
        rec["jit"] = {x: c.stats()[x] for x in ("jit_kernels", "jit_launches", "jit_compile_ms", "jit_failed")}
        print(json.dumps(rec), flush=True)
        out.append(rec)
        c.close()
        torch.cuda.empty_cache()
    return out


def summarise(csv_path, counter, steps, warmup):
    """Counter total per coding step (every gf8 kernel launch after the
    fills, decodes' setup encode excluded by the caller's shape list)."""
    tot, n = 0.0, 0
    with open(csv_path) as f:
        for row in csv.DictReader(f):
            if row["Counter_Name"] != counter:
                continue
            name = row["Kernel_Name"]
            if "gf8" in name or "bm_kernel" in name or "mec_bs" in name:
                tot += float(row["Counter_Value"])
                n += 1
    return tot / (steps + warmup), n


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--arms", default="bs,mg", help="comma-separated arms of ARMS, timed in this order")
    ap.add_argument("--rounds", type=int, default=1, help="repeat the whole shape list")
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--shape", default="-1", help="comma-separated indices into SHAPES (default: all)")
    ap.add_argument("--bytewise", action="store_true", help="skip the bitmatrix (Jerasure Cauchy) shapes")
    ap.add_argument("--ops", default="", help="comma-separated ops to keep (encode, decode, batch)")
    ap.add_argument("--summarise", nargs=2, metavar=("FETCH_CSV", "WRITE_CSV"))
    a = ap.parse_args()
    idx = [int(x) for x in a.shape.split(",")]
    shapes = SHAPES if idx == [-1] else [SHAPES[i] for i in idx]
    if a.bytewise:
        shapes = [x for x in shapes if x[0] != "cauchy"]
    if a.ops:
        shapes = [x for x in shapes if x[5] in a.ops.split(",")]
    if a.summarise:
        fam, k, m, cs, n, op = shapes[0]
        fk, nf = summarise(a.summarise[0], "FETCH_SIZE", a.steps, a.warmup)
        wk, nw = summarise(a.summarise[1], "WRITE_SIZE", a.steps, a.warmup)
        rd, wr = 2 * fk * 1024, wk * 1024
        alg_r = k * cs * n
        alg_w = m * cs * n
        # per launch too: a decode shape's setup encode moves the same bytes
        # as each decode (k read, m written), so every coding launch counts
        steps = a.steps + a.warmup
        rl, wl = rd * steps / max(nf, 1), wr * steps / max(nw, 1)
        print(json.dumps({"shape": shapes[0], "arms": a.arms, "launch_rows": [nf, nw],
                          "read_bytes_per_step": rd, "write_bytes_per_step": wr,
                          "read_ratio": round(rd / alg_r, 4), "write_ratio": round(wr / alg_w, 4),
                          "traffic_ratio": round((rd + wr) / (alg_r + alg_w), 4),
                          "read_ratio_per_launch": round(rl / alg_r, 4), "write_ratio_per_launch": round(wl / alg_w, 4),
                          "traffic_ratio_per_launch": round((rl + wl) / (alg_r + alg_w), 4)}))
    else:
        for _ in range(a.rounds):
            run(a.arms.split(","), a.steps, a.warmup, shapes)
