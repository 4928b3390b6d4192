#!/usr/bin/env python3
"""Layout probe: is the RS(10,4) decode-vs-encode gap arithmetic or layout?

Times (HIP events on the launch stream, best of N) the same 4096-stripe
1 MiB RS(10,4) work in several HBM layouts:
  enc_split      encode, data [S][10][C] and parity [S][4][C] separate
  enc_inplace    encode inside one [S][14][C] stripe buffer
  dec_inplace    decode {0,1,2,3} in place in [S][14][C]
  dec_split      decode {0,1,2,3}: survivors [S][10][C] -> outputs [S][4][C]
  dec_mixed      decode {0,5,10,13} in place
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from memec_amd import Codec, fill_random  # noqa: E402

K, M, C, S = 10, 4, 1 << 20, int(os.environ.get("STRIPES", "4096"))


def t_best(fn, reps=8):
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    fn()
    best = 1e9
    for _ in range(reps):
        ev[0].record()
        fn()
        ev[1].record()
        ev[1].synchronize()
        best = min(best, ev[0].elapsed_time(ev[1]))
    return best


def main():
    torch.cuda.set_device(0)
    codec = Codec("rs", K, M, C, device=0)
    res = {}
    stripe = torch.empty(S, K + M, C, dtype=torch.uint8, device="cuda")
    fill_random(stripe, 7)
    res["enc_inplace"] = t_best(lambda: codec.encode(stripe[:, :K], stripe[:, K:]))
    full = (1 << (K + M)) - 1
    present = full & ~0xF
    res["dec_inplace"] = t_best(lambda: codec.decode(stripe, present))
    present_m = full & ~((1 << 0) | (1 << 5) | (1 << 10) | (1 << 13))
    res["dec_mixed"] = t_best(lambda: codec.decode(stripe, present_m))
    del stripe
    torch.cuda.empty_cache()
    data = torch.empty(S, K, C, dtype=torch.uint8, device="cuda")
    fill_random(data, 7)
    par = torch.empty(S, M, C, dtype=torch.uint8, device="cuda")
    res["enc_split"] = t_best(lambda: codec.encode(data, par))
    # survivors 4..13 packed as [S][10][C] (data 4..9, parity 0..3) and
    # outputs [S][4][C]: decode_split with the survivor base shifted back by
    # 4 chunk slots, so slot c (c >= 4) of stripe s is src[s][c - 4]
    import ctypes
    from memec_amd._lib import check, lib
    src = torch.cat([data[:, 4:], par], dim=1)
    del data, par
    torch.cuda.empty_cache()
    out = torch.empty(S, 4, C, dtype=torch.uint8, device="cuda")
    vp = ctypes.c_void_p
    st = vp(torch.cuda.current_stream().cuda_stream)

    def dec_split():
        check(lib().mec_decode_split(codec._h, vp(src.data_ptr() - 4 * C), K * C, C,
                                     vp(out.data_ptr()), 4 * C, C, S, present, st))
    res["dec_split"] = t_best(dec_split)
    for name, ms in res.items():
        if ms is None:
            continue
        nbytes = 14 * C * S
        print("%-12s %8.3f ms  %7.1f GB/s  %.1f%% of 8 TB/s" % (name, ms, nbytes / ms / 1e6, nbytes / ms / 1e6 / 80))


if __name__ == "__main__":
    main()
