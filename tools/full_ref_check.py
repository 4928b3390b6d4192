#!/usr/bin/env python3
"""Every byte of every BASELINE GPU config against the reference, at full
size.  For configs[0] (RS(4,2)@4 KiB x 65536), configs[1] / [2] (RS(10,4)@1
MiB x 4096), configs[3] (RS(8,2)@4 KiB x 65536) and configs[4]
(CRS(12,4)@64 KiB x 32768, the whole global batch on one GPU): one GPU
encode launch over the full batch, compared stripe by stripe with MemEC's
own Coding::encode compiled from the reference sources (oracle/_ref, the
bench's CPU baseline library), then one in-place GPU decode launch of the
config's erasures over the full batch filled with random NON-codewords
(so the survivor choice and the decoding matrix are pinned, not a round
trip), compared with the reference's Coding::decode of the same stripes.
Host copies in slabs, reference on the usable cores.  One JSON line per
config.  Not product code.

  python3 tools/full_ref_check.py [c0,c1,c3,c4]
"""
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
from memec_amd import Codec, fill_random  # noqa: E402

CASES = {  # label: (family, k, m, chunk, stripes, erased)
    "c0": ("rs", 4, 2, 4096, 65536, [0, 1]),
    "c1": ("rs", 10, 4, 1 << 20, 4096, [0, 1, 2, 3]),  # configs[1] encode + configs[2] decode
    "c3": ("rs", 8, 2, 4096, 65536, [0, 1]),
    "c4": ("cauchy", 12, 4, 65536, 32768, [0, 1, 2, 3]),
}
SLAB = 1 << 30  # host bytes per comparison slab


def main():
    labels = sys.argv[1].split(",") if len(sys.argv) > 1 else list(CASES)
    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    threads = bench.host_cores()[0]
    for lab in labels:
        fam, k, m, cs, n, erased = CASES[lab]
        t0 = time.time()
        c = Codec(fam, k, m, cs)
        per = max(1, SLAB // ((k + m) * cs))
        # encode: one launch over the full batch
        data = torch.empty(n, k, cs, dtype=torch.uint8, device=dev)
        fill_random(data, 0xF011 + n)
        par = torch.empty(n, m, cs, dtype=torch.uint8, device=dev)
        c.encode(data, par)
        torch.cuda.synchronize()
        enc_ok, vs = True, None
        for s0 in range(0, n, per):
            s1 = min(n, s0 + per)
            want, vs = bench.ref_encode(fam, k, m, cs, data[s0:s1].cpu().numpy(), threads)
            enc_ok = enc_ok and bool(np.array_equal(par[s0:s1].cpu().numpy(), want))
        print("%s: encode of %d stripes checked (%s), %.0f s" % (lab, n, enc_ok, time.time() - t0), file=sys.stderr,
              flush=True)
        del data, par
        torch.cuda.empty_cache()
        # decode: random non-codewords everywhere, one in-place launch
        st = torch.empty(n, k + m, cs, dtype=torch.uint8, device=dev)
        fill_random(st, 0xDEC0 + n)
        st0 = st.clone()  # the input, kept in HBM (288 GB: room for both)
        present = sum(1 << i for i in range(k + m) if i not in erased)
        c.decode(st, present)
        torch.cuda.synchronize()
        dec_ok = True
        for s0 in range(0, n, per):
            s1 = min(n, s0 + per)
            want, _ = bench.ref_decode(fam, k, m, cs, st0[s0:s1].cpu().numpy(), erased, threads)
            dec_ok = dec_ok and bool(np.array_equal(st[s0:s1].cpu().numpy(), want))  # survivors untouched too
        del st, st0
        torch.cuda.empty_cache()
        c.close()
        print(json.dumps({"config": lab, "family": fam, "k": k, "m": m, "chunk": cs, "stripes": n,
                          "encode_equal": enc_ok, "decode_equal": dec_ok, "erased": erased,
                          "decode_input": "random non-codewords in every stripe", "vs": vs,
                          "threads": threads, "seconds": round(time.time() - t0, 1)}), flush=True)


if __name__ == "__main__":
    main()
