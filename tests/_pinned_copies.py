"""GPU test runs: every host <-> device copy the tests make through torch goes
through pinned host memory, never through the HIP runtime's pageable-copy
path.

Why: three full GPU suites in rounds 4 and 6 stopped at
`hipErrorIllegalAddress` raised by a pageable copy — the runtime's
`hipMemcpyAsync` of a caller's pageable buffer (r06j, before the library
stopped doing such copies), torch's `.to()` of a pageable tensor (round 4)
and torch's `.cpu()` into pageable memory (r06t) — each time right after a
device-wide synchronize had succeeded, i.e. with no kernel of the library in
flight.  libmec itself no longer DMAs pageable memory on any path; this
module makes the tests' own copies take the same route (pin, then copy), so
a parity check is not lost to that path.  It changes where the test copies
bytes through, never what is compared.

Installed by tests/conftest.py when a GPU is present; a no-op otherwise."""


def install():
    import torch
    if getattr(torch.Tensor, "_mec_pinned_copies", False):
        return
    orig_to, orig_cpu, orig_cuda, orig_copy = torch.Tensor.to, torch.Tensor.cpu, torch.Tensor.cuda, torch.Tensor.copy_

    def target(args, kwargs):
        dev = kwargs.get("device")
        if dev is None and args:
            a = args[0]
            if isinstance(a, (str, torch.device)):
                dev = a
            elif isinstance(a, torch.Tensor):
                dev = a.device
        return None if dev is None else torch.device(dev)

    def d2h(src):
        out = torch.empty(src.shape, dtype=src.dtype, pin_memory=True)
        orig_copy(out, src)  # synchronous: pinned destination, non_blocking=False
        return out

    def to(self, *args, **kwargs):
        d = target(args, kwargs)
        if d is not None:
            if d.type == "cuda" and self.device.type == "cpu" and not self.is_pinned():
                self = self.pin_memory()
            elif d.type == "cpu" and self.is_cuda:
                self = d2h(self)
        return orig_to(self, *args, **kwargs)

    def cpu(self, *args, **kwargs):
        if self.is_cuda:
            return d2h(self)
        return orig_cpu(self, *args, **kwargs)

    def cuda(self, *args, **kwargs):
        if self.device.type == "cpu" and not self.is_pinned():
            self = self.pin_memory()
        return orig_cuda(self, *args, **kwargs)

    def copy_(self, src, non_blocking=False):
        if isinstance(src, torch.Tensor):
            if self.is_cuda and src.device.type == "cpu" and not src.is_pinned():
                src = src.pin_memory()
            elif self.device.type == "cpu" and src.is_cuda and not self.is_pinned():
                return orig_copy(self, d2h(src))
        return orig_copy(self, src, non_blocking=non_blocking)

    torch.Tensor.to, torch.Tensor.cpu, torch.Tensor.cuda, torch.Tensor.copy_ = to, cpu, cuda, copy_
    torch.Tensor._mec_pinned_copies = True
