"""Streaming ceiling vs launch size: mec_xor over total traffic from 0.25 to
24 GiB, and RS(8,2)@4 KiB / CRS(12,4)@64 KiB encode at growing stripe
counts — separates per-launch ramp/tail cost from per-stripe kernel cost."""
import sys
import torch
sys.path.insert(0, "/root/repo")
from memec_amd import xor, Codec

torch.cuda.set_device(0)


def best_ms(fn, reps=10):
    fn(); torch.cuda.synchronize()
    best = 1e9
    for _ in range(reps):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(); fn(); e1.record(); e1.synchronize(); best = min(best, e0.elapsed_time(e1))
    return best


for gib in (0.25, 0.5, 1, 2, 4, 8):
    n = int(gib * (1 << 30)) // 3 // 4096 * 4096
    a = torch.randint(0, 256, (n,), dtype=torch.uint8, device="cuda"); b = torch.empty_like(a); o = torch.empty_like(a)
    ms = best_ms(lambda: xor(o, a, b))
    print("xor   total %6.2f GiB  %8.3f ms  %7.1f GB/s" % (3 * n / 2**30, ms, 3 * n / ms / 1e6), flush=True)
    del a, b, o

for fam, k, m, cs, counts in (("rs", 8, 2, 4096, (16384, 65536, 262144)),
                              ("cauchy", 12, 4, 65536, (1024, 4096, 16384))):
    c = Codec(fam, k, m, cs)
    for n in counts:
        st = torch.randint(0, 256, (n, k + m, cs), dtype=torch.uint8, device="cuda")
        ms = best_ms(lambda: c.encode(st[:, :k], st[:, k:]))
        tot = n * (k + m) * cs
        print("%-6s (%d,%d)@%d  stripes %6d  total %6.2f GiB  %8.3f ms  %7.1f GB/s"
              % (fam, k, m, cs, n, tot / 2**30, ms, tot / ms / 1e6), flush=True)
        del st
