"""Small-chunk encode efficiency vs (k, m, chunk, layout): in-place stripes
[n, k+m, cs], padded stripe stride, and split data / parity tensors.  All at
~2.5-10 GiB of traffic per launch (mec_xor ceiling ~6.5 TB/s at any size)."""
import sys
import torch
sys.path.insert(0, "/root/repo")
from memec_amd import Codec

torch.cuda.set_device(0)


def best_ms(fn, reps=10):
    fn(); torch.cuda.synchronize()
    best = 1e9
    for _ in range(reps):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(); fn(); e1.record(); e1.synchronize(); best = min(best, e0.elapsed_time(e1))
    return best


def run(k, m, cs, n, layout, pad=0):
    c = Codec("rs", k, m, cs)
    if layout == "inplace":
        st = torch.randint(0, 256, (n, k + m + pad, cs), dtype=torch.uint8, device="cuda")
        d, p = st[:, :k], st[:, k:k + m]
    else:
        d = torch.randint(0, 256, (n, k, cs), dtype=torch.uint8, device="cuda")
        p = torch.empty((n, m, cs), dtype=torch.uint8, device="cuda")
    ms = best_ms(lambda: c.encode(d, p))
    tot = n * (k + m) * cs
    print("RS(%2d,%d)@%-6d n=%-7d %-8s pad=%d  %7.3f ms  %7.1f GB/s  %5.1f%%"
          % (k, m, cs, n, layout, pad, ms, tot / ms / 1e6, tot / ms / 1e6 / 80), flush=True)


for args in ((8, 2, 4096, 65536, "inplace"), (8, 2, 4096, 65536, "split"), (8, 2, 4096, 65536, "inplace", 1),
             (8, 2, 4096, 65536, "inplace", 2), (8, 2, 4096, 65536, "inplace", 6),
             (4, 2, 4096, 65536, "inplace"), (6, 2, 4096, 65536, "inplace"), (10, 4, 4096, 65536, "inplace"),
             (8, 2, 8192, 32768, "inplace"), (8, 2, 16384, 16384, "inplace"), (8, 2, 65536, 4096, "inplace"),
             (8, 2, 65536, 4096, "split"), (8, 2, 1 << 20, 256, "inplace"), (8, 2, 1 << 20, 256, "split"),
             (10, 4, 1 << 20, 512, "split"), (10, 4, 1 << 20, 512, "inplace")):
    run(*args)
