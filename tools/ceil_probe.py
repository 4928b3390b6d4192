import sys, torch
sys.path.insert(0, "/root/repo")
from memec_amd import xor
torch.cuda.set_device(0)
n = 8 << 30
src = torch.empty(n, dtype=torch.uint8, device="cuda"); dst = torch.empty_like(src); b = torch.empty_like(src)
def t(fn, nbytes, name):
    fn(); torch.cuda.synchronize()
    best = 1e9
    for _ in range(5):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(); fn(); e1.record(); e1.synchronize(); best = min(best, e0.elapsed_time(e1))
    print("%-28s %8.1f GB/s" % (name, nbytes / best / 1e6), flush=True)
t(lambda: dst.copy_(src), 2 * n, "torch copy uint8")
t(lambda: dst.view(torch.int32).copy_(src.view(torch.int32)), 2 * n, "torch copy int32")
t(lambda: dst.view(torch.float32).copy_(src.view(torch.float32)), 2 * n, "torch copy float32")
t(lambda: dst.view(torch.int64).copy_(src.view(torch.int64)), 2 * n, "torch copy int64")
t(lambda: torch.bitwise_xor(src.view(torch.int64), b.view(torch.int64), out=dst.view(torch.int64)), 3 * n, "torch xor int64")
t(lambda: xor(dst, src, b), 3 * n, "mec_xor")
