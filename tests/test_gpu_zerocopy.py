"""GPU parity of the zero-copy host path (include/mec.h mec_host_register):
host chunks in registered ranges are coded in place over PCIe by the same
kernels, with no staging through HBM.  Bit-exact against the oracle, for
every host entry point, on a MemEC-like slab (ChunkPool slots of
8 + chunkSize bytes, chunk_pool.cc:22-95, so chunk data is only 8-byte
aligned), and the staged fallback when a chunk lies outside every
registered range.
"""
import threading

import numpy as np
import pytest

import _oracle as O
from _mismatch import same

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

from memec_amd import Codec, host_register, host_unregister  # noqa: E402

FAMS = ["rs", "cauchy", "isal_rs", "isal_cauchy"]


@pytest.fixture(scope="module", autouse=True)
def _gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    torch.cuda.set_device(0)
    yield
    torch.cuda.synchronize()


def aligned(nbytes, align=4096):
    raw = np.empty(nbytes + align, np.uint8)
    off = (-raw.ctypes.data) % align
    return raw[off:off + nbytes]


class HostSlab:
    """Registered host slab of n slots of 8 + cs bytes, random contents."""

    def __init__(self, n_slots, cs, seed, hdr=8):
        self.cs, self.hdr, self.slot = cs, hdr, cs + hdr
        self.buf = aligned(n_slots * self.slot)
        self.buf[:] = O.fill(self.buf.nbytes, seed)
        host_register(self.buf)

    def close(self):
        host_unregister(self.buf)

    def addr(self, i):
        return self.buf.ctypes.data + i * self.slot + self.hdr

    def view(self, i):
        o = i * self.slot + self.hdr
        return self.buf[o:o + self.cs]


def zeros(cs):
    return np.zeros(cs, np.uint8)


def cs_for(fam, k, m, cs):
    return cs if fam != "cauchy" or O.cauchy_getw(k, m, cs) > 0 else 4096


@pytest.mark.parametrize("fam", FAMS)
@pytest.mark.parametrize("cs", [4096, 4104])
def test_zc_encode_batch(fam, cs):
    k, m, n = 6, 3, 24
    cs = cs_for(fam, k, m, cs)
    rng = np.random.default_rng(1)
    slots = rng.permutation(n * (k + m))
    slab = HostSlab(n * (k + m), cs, 5)
    try:
        before = slab.buf.copy()
        c = Codec(fam, k, m, cs)
        dptr, pptr, want = [], [], []
        for s in range(n):
            row = slots[s * (k + m):(s + 1) * (k + m)]
            zc = {int(rng.integers(0, k))} if s % 4 == 1 else set()
            wanted = [True] * m if s % 2 else [bool(rng.integers(0, 3)) for _ in range(m)]
            dptr += [0 if j in zc else slab.addr(row[j]) for j in range(k)]
            pptr += [slab.addr(row[k + i]) if wanted[i] else 0 for i in range(m)]
            data = [zeros(cs) if j in zc else slab.view(row[j]).copy() for j in range(k)]
            want.append((row, wanted, O.encode(fam, k, m, data, cs)))
        z0 = c.stats()["zero_copy_calls"]
        pre = slab.buf.copy()
        c.encode_batch(dptr, pptr, mem="host")
        assert c.stats()["zero_copy_calls"] == z0 + 1
        for s, (row, wanted, par) in enumerate(want):
            for i in range(m):
                o = row[k + i] * slab.slot + slab.hdr
                exp = par[i] if wanted[i] else before[o:o + cs]
                same(slab.view(row[k + i]), exp, (fam, s, i), before=pre[o:o + cs], addr=slab.addr(row[k + i]))
        # headers and sources untouched
        for s in range(n):
            row = slots[s * (k + m):(s + 1) * (k + m)]
            for j in range(k):
                o = row[j] * slab.slot
                same(slab.buf[o:o + slab.slot], before[o:o + slab.slot], ("source", s, j))
    finally:
        slab.close()


@pytest.mark.parametrize("fam", FAMS)
def test_zc_decode_batch_mixed(fam):
    k, m, cs, n = 6, 3, 2048, 30
    rng = np.random.default_rng(2)
    slab = HostSlab(n * (k + m), cs, 77)  # random non-codeword stripes
    try:
        before = [slab.view(i).copy() for i in range(n * (k + m))]
        c = Codec(fam, k, m, cs)
        ptrs, masks, pats = [], [], []
        for s in range(n):
            e = 0 if s % 9 == 4 else int(rng.integers(1, m + 1))
            pat = sorted(rng.choice(k + m, size=e, replace=False).tolist())
            pats.append(pat)
            ptrs += [slab.addr(s * (k + m) + i) for i in range(k + m)]
            masks.append(sum(1 << i for i in range(k + m) if i not in pat))
        for s in range(n):
            for e in pats[s]:
                slab.view(s * (k + m) + e)[:] = 0
        pre = [slab.view(i).copy() for i in range(n * (k + m))]
        assert c.decode_batch(ptrs, masks, mem="host") == [0] * n
        assert c.stats()["zero_copy_calls"] >= 1
        for s in range(n):
            chunks = [before[s * (k + m) + i].copy() for i in range(k + m)]
            if pats[s]:
                assert O.decode(fam, k, m, chunks, pats[s], cs) == 0
            for i in range(k + m):
                same(slab.view(s * (k + m) + i), chunks[i], (fam, s, pats[s], i), before=pre[s * (k + m) + i],
                     addr=slab.addr(s * (k + m) + i))
    finally:
        slab.close()


@pytest.mark.parametrize("fam", FAMS)
def test_zc_update_batch(fam):
    k, m, cs, n = 5, 3, 1024, 20
    rng = np.random.default_rng(3)
    data = [O.fill(k * cs, 40 + s).reshape(k, cs) for s in range(n)]
    P = aligned(n * m * cs).reshape(n, m, cs)
    P[:] = np.stack([np.stack(O.encode(fam, k, m, list(d), cs)) for d in data])
    D = aligned(n * cs).reshape(n, cs)
    D[:] = O.fill(n * cs, 12).reshape(n, cs)
    host_register(P)
    host_register(D)
    try:
        p0 = P.copy()
        js = [int(rng.integers(0, k)) for _ in range(n)]
        c = Codec(fam, k, m, cs)
        pb, db = P.ctypes.data, D.ctypes.data
        pre = P.copy()
        c.encode_update_batch(js, [db + s * cs for s in range(n)],
                              [pb + (s * m + i) * cs for s in range(n) for i in range(m)], mem="host")
        assert c.stats()["zero_copy_calls"] == 1
        for s in range(n):
            d2 = data[s].copy()
            d2[js[s]] ^= D[s]
            want = O.encode(fam, k, m, list(d2), cs)
            for i in range(m):
                same(P[s, i], want[i], (fam, s, i), before=pre[s, i], addr=P[s, i].ctypes.data)
        assert not np.array_equal(P, p0)
    finally:
        host_unregister(P)
        host_unregister(D)


@pytest.mark.parametrize("fam", FAMS)
def test_zc_single_stripe_calls(fam):
    """mec_encode_host / mec_decode_host / mec_encode_update_host on slab
    chunks: one launch on the chunks' device addresses.  Every comparison
    reports a mismatch map (tests/_mismatch.py) against the pre-call bytes."""
    k, m = 10, 4
    cs = cs_for(fam, k, m, 65536)
    slab = HostSlab(k + m + 1, cs, 9)
    try:
        c = Codec(fam, k, m, cs)
        data = [slab.view(j) for j in range(k)]
        par = [slab.view(k + i) for i in range(m)]
        want = O.encode(fam, k, m, [d.copy() for d in data], cs)
        got = c.encode_host(data)  # outputs are fresh (unregistered) arrays: staged
        for i in range(m):
            same(got[i], want[i], ("staged encode", fam, i))
        st0 = c.stats()
        # in-place parity into the slab: zero-copy
        import ctypes
        from memec_amd._lib import check, lib
        vp = ctypes.c_void_p
        dp = (vp * k)(*[vp(slab.addr(j)) for j in range(k)])
        pp = (vp * m)(*[vp(slab.addr(k + i)) for i in range(m)])
        pre = [p.copy() for p in par]
        check(lib().mec_encode_host(c._h, dp, pp))
        for i in range(m):
            same(par[i], want[i], ("zc encode", fam, i), before=pre[i], addr=slab.addr(k + i))
        assert c.stats()["zero_copy_calls"] == st0["zero_copy_calls"] + 1
        # decode in place: erase a mix of data and parity
        orig = [slab.view(i).copy() for i in range(k + m)]
        pat = [0, 3, 10, 13]
        for e in pat:
            slab.view(e)[:] = 0
        pre = [slab.view(i).copy() for i in range(k + m)]
        c.decode_host([slab.view(i) for i in range(k + m)], sum(1 << i for i in range(k + m) if i not in pat))
        for i in range(k + m):
            same(slab.view(i), orig[i], ("zc decode", fam, pat, i), before=pre[i], addr=slab.addr(i))
        # delta update of two parities, the delta in the slab's spare slot
        delta = slab.view(k + m)
        d2 = [o.copy() for o in orig[:k]]
        d2[4] ^= delta
        want2 = O.encode(fam, k, m, d2, cs)
        pre = [p.copy() for p in par]
        c.encode_update_host(4, delta, [par[0], None, par[2], None])
        same(par[0], want2[0], ("zc update", fam, 0), before=pre[0], addr=slab.addr(k))
        same(par[2], want2[2], ("zc update", fam, 2), before=pre[2], addr=slab.addr(k + 2))
        same(par[1], orig[k + 1], ("zc update untouched", fam, 1), addr=slab.addr(k + 1))
        same(par[3], orig[k + 3], ("zc update untouched", fam, 3), addr=slab.addr(k + 3))
        assert c.stats()["zero_copy_calls"] == st0["zero_copy_calls"] + 3
    finally:
        slab.close()


def test_zc_all_zero_sources():
    """Every data chunk is Coding::zeros: parity is zero (zero-copy path)."""
    k, m, cs = 4, 2, 4096
    slab = HostSlab(m, cs, 3)
    try:
        c = Codec("rs", k, m, cs)
        c.encode_batch([0] * k, [slab.addr(0), slab.addr(1)], mem="host")
        assert not slab.view(0).any() and not slab.view(1).any()
    finally:
        slab.close()


@pytest.mark.parametrize("fam", ["rs", "cauchy"])
def test_zc_host_batch_dense(fam):
    k, m, cs, n = 10, 4, 65536, 12
    d = aligned(n * k * cs).reshape(n, k, cs)
    d[:] = O.fill(d.nbytes, 31).reshape(n, k, cs)
    p = aligned(n * m * cs).reshape(n, m, cs)
    p[:] = 0
    host_register(d)
    host_register(p)
    try:
        c = Codec(fam, k, m, cs)
        c.encode_host_batch(d, p)
        assert c.stats()["zero_copy_calls"] == 1
        for s in range(n):
            same(p[s], np.stack(O.encode(fam, k, m, list(d[s]), cs)), ("zc host batch", fam, s), before=np.zeros_like(p[s]),
                 addr=p[s].ctypes.data)
    finally:
        host_unregister(d)
        host_unregister(p)


def test_zc_partial_registration_falls_back():
    """One chunk outside every registered range: the call is staged, exact."""
    k, m, cs, n = 4, 2, 4096, 6
    slab = HostSlab(n * (k + m), cs, 8)
    outside = O.fill(cs, 99)
    try:
        c = Codec("rs", k, m, cs)
        dptr = [slab.addr(s * (k + m) + j) for s in range(n) for j in range(k)]
        dptr[5] = outside.ctypes.data
        pptr = [slab.addr(s * (k + m) + k + i) for s in range(n) for i in range(m)]
        c.encode_batch(dptr, pptr, mem="host")
        st = c.stats()
        assert st["zero_copy_calls"] == 0 and st["staged_calls"] == 1
        for s in range(n):
            data = [slab.view(s * (k + m) + j).copy() for j in range(k)]
            if s == 1:
                data[1] = outside
            want = O.encode("rs", k, m, data, cs)
            for i in range(m):
                same(slab.view(s * (k + m) + k + i), want[i], ("staged fallback", s, i), addr=slab.addr(s * (k + m) + k + i))
    finally:
        slab.close()


def test_zc_coalesced_threads():
    """Worker threads' single-stripe calls on one registered slab with
    coalescing on: each batch is one zero-copy launch (pointer rows read in
    place from pinned memory) and stays exact."""
    k, m, cs = 8, 2, 4096
    n_threads, per = 8, 16
    slab = HostSlab(n_threads * per * (k + m), cs, 21)
    c = Codec("rs", k, m, cs)
    c.set_coalescing(64)
    errors = []
    import ctypes
    from memec_amd._lib import lib
    vp = ctypes.c_void_p

    def worker(t):
        for r in range(per):
            base = (t * per + r) * (k + m)
            want = O.encode("rs", k, m, [slab.view(base + j).copy() for j in range(k)], cs)
            dp = (vp * k)(*[vp(slab.addr(base + j)) for j in range(k)])
            pp = (vp * m)(*[vp(slab.addr(base + k + i)) for i in range(m)])
            if lib().mec_encode_host(c._h, dp, pp) != 0:
                errors.append(("rc", t, r))
            for i in range(m):
                if not np.array_equal(slab.view(base + k + i), want[i]):
                    from _mismatch import mismatch_map
                    errors.append((t, r, i, mismatch_map(slab.view(base + k + i), want[i], addr=slab.addr(base + k + i))))

    try:
        th = [threading.Thread(target=worker, args=(t,)) for t in range(n_threads)]
        for x in th:
            x.start()
        for x in th:
            x.join()
        assert not errors, errors[:5]
        st = c.stats()
        assert st["coalesced_requests"] == n_threads * per
        assert st["zero_copy_calls"] == st["coalesced_batches"] and st["staged_calls"] == 0
    finally:
        slab.close()


def test_zc_register_overlap_refused():
    """a range overlapping a registered one is refused
    (MEC_EINVAL) — the same begin, inside it, and one that starts below it
    and extends across it — while a disjoint neighbour registers, and after
    unregistering the first range the overlapping one registers and codes
    zero-copy, exactly."""
    from memec_amd import _lib
    k, m, cs = 4, 2, 4096
    big = aligned(64 * 4096)
    big[:] = O.fill(big.nbytes, 17)
    inner = big[16 * 4096:32 * 4096]
    lo = big[8 * 4096:24 * 4096]          # starts below `inner`, extends across it
    nb = big[40 * 4096:48 * 4096]         # disjoint neighbour
    host_register(inner)
    try:
        for arr in (inner, inner[4096:8192], lo):
            with pytest.raises(_lib.MecError) as ei:
                host_register(arr)
            assert ei.value.code == _lib.MEC_EINVAL
        host_register(nb)
        host_unregister(nb)
    finally:
        host_unregister(inner)
    with pytest.raises(_lib.MecError):
        host_unregister(inner)            # no longer registered
    host_register(lo)
    try:
        c = Codec("rs", k, m, cs)
        base = lo.ctypes.data
        data = [lo[j * cs:(j + 1) * cs] for j in range(k)]
        par = [lo[(k + i) * cs:(k + i + 1) * cs] for i in range(m)]
        want = O.encode("rs", k, m, [d.copy() for d in data], cs)
        pre = [p.copy() for p in par]
        z0 = c.stats()["zero_copy_calls"]
        c.encode_batch([base + j * cs for j in range(k)], [base + (k + i) * cs for i in range(m)], mem="host")
        assert c.stats()["zero_copy_calls"] == z0 + 1
        for i in range(m):
            same(par[i], want[i], ("overlap re-register", i), before=pre[i], addr=base + (k + i) * cs)
    finally:
        host_unregister(lo)
