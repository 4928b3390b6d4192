#!/usr/bin/env python3
"""Where does in-place RS(10,4)@1 MiB decode lose its 1-2 points to encode?
Interleaved A/B over one [4096][14][1 MiB] stripe buffer (56 GiB): in-place
decode of several erasure patterns (which chunks are written, which read,
dense or Vandermonde rows), the in-place encode (parity written into the
same buffer), and the split-buffer encode and decode for reference.
Median kernel ms over rounds x 10 launches (HIP events).  Not product code.

  python3 tools/dec_pos_ab.py [rounds=5]
"""
import statistics
import sys
import os

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

from memec_amd import Codec, fill_random, set_knob  # noqa: E402

K, M, CS, N = 10, 4, 1 << 20, 4096


def main():
    rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 5
    torch.cuda.set_device(0)
    c = Codec("rs", K, M, CS, device=0)
    st = torch.empty(N, K + M, CS, dtype=torch.uint8, device="cuda")
    fill_random(st, 7)
    arms = []
    for pat in ([0, 1, 2, 3], [6, 7, 8, 9], [10, 11, 12, 13], [0, 5, 10, 13], [9, 10, 11, 12], [0, 1]):
        present = sum(1 << i for i in range(K + M) if i not in pat)
        arms.append(("decode in place %s" % pat, (lambda p=present: c.decode(st, p)), (K + len(pat)) * CS * N))
    arms.append(("encode in place (parity 10..13)", lambda: c.encode(st[:, :K], st[:, K:]), (K + M) * CS * N))
    # split buffers: 40 GiB data + 16 GiB parity, reusing the stripe buffer's bytes as two views
    flat = st.view(-1)
    data = flat[: N * K * CS].view(N, K, CS)
    par = flat[N * K * CS:].view(N, M, CS)
    arms.append(("encode split", lambda: c.encode(data, par), (K + M) * CS * N))
    present = sum(1 << i for i in range(K + M) if i not in (0, 1, 2, 3))
    surv = flat[: N * K * CS].view(N, K, CS)  # as if chunks 4..13 had been gathered compactly
    outs = flat[N * K * CS:].view(N, M, CS)
    from memec_amd.codec import _stream, check, lib, vp

    def dec_split():  # survivors 4..13 compact: chunk t at surv + s*10*CS + (t-4)*CS
        check(lib().mec_decode_split(c._h, vp(surv.data_ptr() - 4 * CS), K * CS, CS, vp(outs.data_ptr()), M * CS, CS,
                                     N, present, _stream(None)))
    arms.append(("decode split {0,1,2,3}", dec_split, (K + M) * CS * N))
    if os.environ.get("DPA_CAPS"):  # cap sweep of the two in-place decode structures instead
        caps = os.environ["DPA_CAPS"].split(",")
        base = [a for a in arms if a[0].startswith("decode in place [0, 1, 2, 3]") or
                a[0].startswith("decode in place [10, 11, 12, 13]")]
        arms = []
        for name, step, nb in base:
            for cap in caps:
                def capped(step=step, cap=cap):
                    set_knob("MEC_WPC", cap)
                    step()
                arms.append(("%s wpc=%s" % (name, cap), capped, nb))
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    res = [[] for _ in arms]
    for _ in range(rounds):
        for i, (_, step, _) in enumerate(arms):
            step()
            ev[0].record()
            for _ in range(10):
                step()
            ev[1].record()
            ev[1].synchronize()
            res[i].append(ev[0].elapsed_time(ev[1]) / 10)
    for (name, _, nbytes), r in zip(arms, res):
        med = statistics.median(r)
        print("%-36s median %.4f ms  %.1f %% of 8 TB/s" % (name, med, nbytes / med / 1e6 / 80), flush=True)


if __name__ == "__main__":
    main()
