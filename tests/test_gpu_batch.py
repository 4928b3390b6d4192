"""GPU parity of the pointer-array batch ABI (mec_encode_batch,
mec_decode_batch, mec_encode_update_batch) and the request coalescer,
against the oracle.  Bit-exact.

Chunks are scattered over a slab in random slot order, as server/ holds them
(ChunkPool slots of 8 + chunkSize bytes, chunk_pool.cc:22-95, so chunk data
is only 8-byte aligned; ChunkUtil::getData, chunk_util.hh:131-133), with
Coding::zeros columns (NULL), unwanted parities (NULL) and, for decode, a
different erasure pattern per stripe including none and more than m
(recovery_worker.cc:210-296 batches stripes; worker.cc:49 decodes each).
"""
import threading

import numpy as np
import pytest

import _oracle as O

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

from memec_amd import Codec, fill_random  # noqa: E402
from memec_amd import _lib  # noqa: E402

DEV = "cuda:0"
FAMS = ["rs", "cauchy", "isal_rs", "isal_cauchy"]


@pytest.fixture(scope="module", autouse=True)
def _gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    torch.cuda.set_device(0)
    yield
    torch.cuda.synchronize()


class Slab:
    """n_slots chunk slots of `slot` bytes; chunk data at +`hdr` (8 = the
    reference's ChunkIdentifier header).  Device (torch) or host (numpy)."""

    def __init__(self, n_slots, cs, hdr, device, seed):
        self.cs, self.hdr, self.slot = cs, hdr, cs + hdr
        nbytes = n_slots * self.slot
        self.host = O.fill(nbytes, seed)
        if device:
            self.t = torch.from_numpy(self.host.copy()).to(DEV)
            self.base = self.t.data_ptr()
        else:
            self.t = None
            self.base = self.host.ctypes.data

    def addr(self, i):
        return self.base + i * self.slot + self.hdr

    def chunk(self, i):
        """Current contents of slot i's chunk (numpy copy)."""
        if self.t is not None:
            torch.cuda.synchronize()
            return self.t[i * self.slot + self.hdr: i * self.slot + self.hdr + self.cs].cpu().numpy()
        return self.host[i * self.slot + self.hdr: i * self.slot + self.hdr + self.cs].copy()

    def snapshot(self):
        if self.t is not None:
            torch.cuda.synchronize()
            return self.t.cpu().numpy()
        return self.host.copy()


def zeros(cs):
    return np.zeros(cs, np.uint8)


def chunk_of(snap, slab, i):
    o = i * slab.slot + slab.hdr
    return snap[o:o + slab.cs]


# --------------------------------------------------------------------------- encode


@pytest.mark.parametrize("mem", ["device", "host"])
@pytest.mark.parametrize("fam", FAMS)
@pytest.mark.parametrize("hdr", [8, 256])
def test_encode_batch_scattered(fam, mem, hdr):
    k, m, cs, n = 6, 3, 4096 if fam != "cauchy" else 4104, 40
    if fam == "cauchy" and O.cauchy_getw(k, m, cs) < 0:
        cs = 4096
    rng = np.random.default_rng(7)
    slots = rng.permutation(n * (k + m))
    slab = Slab(n * (k + m), cs, hdr, mem == "device", 99)
    before = slab.snapshot()
    dptr, pptr, want = [], [], []
    for s in range(n):
        row = slots[s * (k + m):(s + 1) * (k + m)]
        zero_cols = set(rng.choice(k, size=rng.integers(0, k + 1), replace=False).tolist()) if s % 3 == 0 else set()
        wanted = [bool(rng.integers(0, 4)) for _ in range(m)] if s % 2 else [True] * m
        dptr += [0 if j in zero_cols else slab.addr(row[j]) for j in range(k)]
        pptr += [slab.addr(row[k + i]) if wanted[i] else 0 for i in range(m)]
        data = [zeros(cs) if j in zero_cols else chunk_of(before, slab, row[j]).copy() for j in range(k)]
        want.append((row, wanted, O.encode(fam, k, m, data, cs)))
    c = Codec(fam, k, m, cs)
    c.encode_batch(dptr, pptr, mem=mem)
    after = slab.snapshot()
    for s, (row, wanted, par) in enumerate(want):
        for i in range(m):
            got = chunk_of(after, slab, row[k + i])
            if wanted[i]:
                assert np.array_equal(got, par[i]), (fam, mem, s, i)
            else:
                assert np.array_equal(got, chunk_of(before, slab, row[k + i])), (fam, mem, s, i, "unwanted")
        for j in range(k):  # sources untouched
            assert np.array_equal(chunk_of(after, slab, row[j]), chunk_of(before, slab, row[j]))
    # slot headers untouched
    for i in range(n * (k + m)):
        o = i * slab.slot
        assert np.array_equal(after[o:o + hdr], before[o:o + hdr])


def test_encode_batch_parity_mask_and_big_chunks_host():
    """RS(10,4)@1MiB on host memory (staged through mapped pinned buffers)."""
    k, m, cs, n = 10, 4, 1 << 20, 3
    c = Codec("rs", k, m, cs)
    data = [O.fill(cs, 500 + i) for i in range(n * k)]
    par = [np.full(cs, 0xA5, np.uint8) for _ in range(n * m)]
    c.encode_batch([a.ctypes.data for a in data], [a.ctypes.data for a in par], parity_mask=0b1011, mem="host")
    for s in range(n):
        want = O.encode("rs", k, m, data[s * k:(s + 1) * k], cs)
        for i in range(m):
            if i == 2:
                assert (par[s * m + i] == 0xA5).all()
            else:
                assert np.array_equal(par[s * m + i], want[i]), (s, i)


# --------------------------------------------------------------------------- decode


def random_patterns(rng, n, k, m):
    pats = []
    for s in range(n):
        if s % 11 == 5:
            e = m + 1  # too many: decode() == false, chunks untouched
        elif s % 7 == 3:
            e = 0
        else:
            e = int(rng.integers(1, m + 1))
        pats.append(sorted(rng.choice(k + m, size=e, replace=False).tolist()))
    return pats


@pytest.mark.parametrize("mem", ["device", "host"])
@pytest.mark.parametrize("fam", FAMS)
def test_decode_batch_mixed_patterns(fam, mem):
    k, m, cs, n = 6, 3, 2048, 48
    rng = np.random.default_rng(11)
    slots = rng.permutation(n * (k + m))
    slab = Slab(n * (k + m), cs, 8, mem == "device", 1234)  # random (non-codeword) stripes
    before = slab.snapshot()
    pats = random_patterns(rng, n, k, m)
    ptrs, masks = [], []
    for s in range(n):
        row = slots[s * (k + m):(s + 1) * (k + m)]
        ptrs += [slab.addr(i) for i in row]
        masks.append(sum(1 << i for i in range(k + m) if i not in pats[s]))
    c = Codec(fam, k, m, cs)
    res = c.decode_batch(ptrs, masks, mem=mem)
    after = slab.snapshot()
    for s in range(n):
        row = slots[s * (k + m):(s + 1) * (k + m)]
        chunks = [chunk_of(before, slab, i).copy() for i in row]
        if len(pats[s]) > m:
            assert res[s] == _lib.MEC_ETOOMANY, s
            want = chunks
        else:
            assert res[s] == 0, (s, res[s])
            if pats[s]:
                assert O.decode(fam, k, m, chunks, pats[s], cs) == 0
            want = chunks
        for i in range(k + m):
            assert np.array_equal(chunk_of(after, slab, row[i]), want[i]), (fam, mem, s, pats[s], i)
    assert c.stats()["cached_plans"] == len({tuple(p) for p in pats if 0 < len(p) <= m})


def test_decode_batch_roundtrip_baseline_shape():
    """RS(10,4)@64KiB codewords, device, every stripe a different pattern of
    4 erasures: decode restores the originals."""
    k, m, cs, n = 10, 4, 65536, 64
    c = Codec("rs", k, m, cs)
    data = torch.empty(n, k, cs, dtype=torch.uint8, device=DEV)
    fill_random(data, 4321)
    par = torch.zeros(n, m, cs, dtype=torch.uint8, device=DEV)
    c.encode(data, par)
    stripe = torch.cat([data, par], dim=1).contiguous()
    orig = stripe.clone()
    rng = np.random.default_rng(5)
    masks = []
    for s in range(n):
        pat = rng.choice(k + m, size=m, replace=False)
        stripe[s, list(pat)] = 0
        masks.append(sum(1 << i for i in range(k + m) if i not in pat))
    base = stripe.data_ptr()
    ptrs = [base + (s * (k + m) + i) * cs for s in range(n) for i in range(k + m)]
    assert c.decode_batch(ptrs, masks) == [0] * n
    torch.cuda.synchronize()
    assert torch.equal(stripe, orig)


# --------------------------------------------------------------------------- delta update


@pytest.mark.parametrize("mem", ["device", "host"])
@pytest.mark.parametrize("fam", FAMS)
def test_update_batch(fam, mem):
    """parity ^= A[:, j] * delta per stripe, mixed j: equals re-encoding the
    updated data (parity_chunk_buffer.cc:340-415)."""
    k, m, cs, n = 5, 3, 1024, 30
    rng = np.random.default_rng(3)
    data = [O.fill(k * cs, 70 + s).reshape(k, cs) for s in range(n)]
    parity0 = [np.stack(O.encode(fam, k, m, list(d), cs)) for d in data]
    deltas = [O.fill(cs, 900 + s) for s in range(n)]
    js = [int(rng.integers(0, k)) for _ in range(n)]
    wanted = [[bool(rng.integers(0, 3)) for _ in range(m)] for _ in range(n)]
    c = Codec(fam, k, m, cs)
    if mem == "device":
        P = torch.from_numpy(np.stack(parity0)).to(DEV)
        D = torch.from_numpy(np.stack(deltas)).to(DEV)
        pb, db = P.data_ptr(), D.data_ptr()
    else:
        P = np.stack(parity0).copy()
        D = np.stack(deltas)
        pb, db = P.ctypes.data, D.ctypes.data
    pptr = [pb + (s * m + i) * cs if wanted[s][i] else 0 for s in range(n) for i in range(m)]
    dptr = [db + s * cs if s % 9 != 4 else 0 for s in range(n)]  # some all-zero deltas
    c.encode_update_batch(js, dptr, pptr, mem=mem)
    got = P.cpu().numpy() if mem == "device" else P
    for s in range(n):
        d2 = data[s].copy()
        if s % 9 != 4:
            d2[js[s]] ^= deltas[s]
        want = O.encode(fam, k, m, list(d2), cs)
        for i in range(m):
            exp = want[i] if wanted[s][i] else parity0[s][i]
            assert np.array_equal(got[s, i], exp), (fam, mem, s, i)


# --------------------------------------------------------------------------- coalescer


@pytest.mark.parametrize("fam", ["rs", "cauchy"])
def test_coalesced_host_calls_from_threads(fam):
    """Concurrent single-stripe mec_*_host calls (the server's worker threads
    sharing one Coding, worker.cc:128-137) are batched and stay exact."""
    k, m, cs = 8, 2, 4096
    c = Codec(fam, k, m, cs)
    c.set_coalescing(256)
    n_threads, per = 12, 20
    errors = []

    def worker(t):
        try:
            for r in range(per):
                seed = 10000 + t * 100 + r
                data = [O.fill(cs, seed * 16 + j) for j in range(k)]
                if r % 4 == 1:
                    data[r % k] = None
                got = c.encode_host(data)
                want = O.encode(fam, k, m, [d if d is not None else zeros(cs) for d in data], cs)
                for i in range(m):
                    if not np.array_equal(got[i], want[i]):
                        errors.append(("enc", t, r, i))
                chunks = [d.copy() if d is not None else zeros(cs) for d in data] + [w.copy() for w in want]
                orig = [x.copy() for x in chunks]
                pat = [r % (k + m), (r * 3 + 1) % (k + m)] if r % 2 else [t % (k + m)]
                for e in pat:
                    chunks[e][:] = 0
                c.decode_host(chunks, sum(1 << i for i in range(k + m) if i not in pat))
                for i in range(k + m):
                    if not np.array_equal(chunks[i], orig[i]):
                        errors.append(("dec", t, r, i))
                delta = O.fill(cs, seed + 7)
                par = [w.copy() for w in want]
                c.encode_update_host(r % k, delta, par)
                d2 = [x.copy() for x in orig[:k]]
                d2[r % k] ^= delta
                want2 = O.encode(fam, k, m, d2, cs)
                for i in range(m):
                    if not np.array_equal(par[i], want2[i]):
                        errors.append(("upd", t, r, i))
        except Exception as exc:  # pragma: no cover - reported below
            errors.append(("exc", t, repr(exc)))

    th = [threading.Thread(target=worker, args=(t,)) for t in range(n_threads)]
    for x in th:
        x.start()
    for x in th:
        x.join()
    assert not errors, errors[:10]
    st = c.stats()
    assert st["coalesced_requests"] == n_threads * per * 3
    assert st["coalesced_batches"] <= st["coalesced_requests"]


def test_batch_errors():
    c = Codec("rs", 4, 2, 4096)
    with pytest.raises(Exception):
        c.encode_batch([0] * 4, [0] * 3)
    with pytest.raises(_lib.MecError):
        _lib.check(_lib.lib().mec_encode_batch(c._h, None, None, 1, 0, 0, None))
    with pytest.raises(_lib.MecError):
        _lib.check(_lib.lib().mec_encode_batch(c._h, None, None, 1, 0, 7, None))
    # decode: NULL chunk pointer in a stripe that needs decoding -> EINVAL for that stripe
    res = c.decode_batch([0] * 6, [0b111110])
    assert res == [_lib.MEC_EINVAL]


@pytest.mark.parametrize("fam", FAMS)
def test_decode_batch_single_pattern(fam):
    """Every stripe has the same erasures: the map runs from kernel
    arguments (gf8_kernel / bm_kernel gather mode) instead of descriptors."""
    k, m, cs, n = 6, 3, 4104 if fam != "rs" else 4096, 24
    if fam == "cauchy" and O.cauchy_getw(k, m, cs) < 0:
        cs = 4096
    rng = np.random.default_rng(21)
    slots = rng.permutation(n * (k + m))
    slab = Slab(n * (k + m), cs, 8, True, 777)
    before = slab.snapshot()
    for pat in ([0, 4, 7], [8], [1, 2]):
        slab.t.copy_(torch.from_numpy(before).to(DEV))
        ptrs = [slab.addr(i) for s in range(n) for i in slots[s * (k + m):(s + 1) * (k + m)]]
        mask = sum(1 << i for i in range(k + m) if i not in pat)
        c = Codec(fam, k, m, cs)
        assert c.decode_batch(ptrs, [mask] * n) == [0] * n
        after = slab.snapshot()
        for s in range(n):
            row = slots[s * (k + m):(s + 1) * (k + m)]
            chunks = [chunk_of(before, slab, i).copy() for i in row]
            assert O.decode(fam, k, m, chunks, pat, cs) == 0
            for i in range(k + m):
                assert np.array_equal(chunk_of(after, slab, row[i]), chunks[i]), (fam, pat, s, i)


@pytest.mark.parametrize("fam", ["rs", "cauchy"])
def test_update_batch_single_column(fam):
    k, m, cs, n, j = 5, 3, 2048, 16, 3
    data = [O.fill(k * cs, 170 + s).reshape(k, cs) for s in range(n)]
    parity0 = np.stack([np.stack(O.encode(fam, k, m, list(d), cs)) for d in data])
    deltas = np.stack([O.fill(cs, 1900 + s) for s in range(n)])
    P = torch.from_numpy(parity0.copy()).to(DEV)
    D = torch.from_numpy(deltas).to(DEV)
    c = Codec(fam, k, m, cs)
    c.encode_update_batch([j] * n, [D.data_ptr() + s * cs for s in range(n)],
                          [P.data_ptr() + (s * m + i) * cs for s in range(n) for i in range(m)], parity_mask=0b101)
    got = P.cpu().numpy()
    for s in range(n):
        d2 = data[s].copy()
        d2[j] ^= deltas[s]
        want = O.encode(fam, k, m, list(d2), cs)
        for i in range(m):
            assert np.array_equal(got[s, i], want[i] if i != 1 else parity0[s, i]), (fam, s, i)


@pytest.mark.parametrize("block", ["64", "256"])
def test_block_override_every_launch_kind(block, knobs):
    """MEC_BLOCK (layout experiments) forces the block size of strided
    launches and must leave results unchanged; gathered (pointer-table)
    launches ignore it (their kernels exist for 256 threads only)."""
    knobs("MEC_BLOCK", block)
    test_encode_batch_scattered("rs", "device", 8)
    test_encode_batch_scattered("cauchy", "device", 8)
    for fam in ("rs", "cauchy"):
        k, m, cs, n = 6, 3, 4096, 24
        c = Codec(fam, k, m, cs)
        base = O.fill(n * (k + m) * cs, 555).reshape(n, k + m, cs)
        for s in range(n):
            base[s, k:] = np.stack(O.encode(fam, k, m, [base[s, j].copy() for j in range(k)], cs))
        t = torch.from_numpy(base.copy()).to("cuda")
        t[:, [0, 4, 7]] = 0
        c.decode(t, sum(1 << i for i in range(k + m) if i not in (0, 4, 7)))
        torch.cuda.synchronize()
        assert np.array_equal(t.cpu().numpy(), base), (fam, block)


@pytest.mark.parametrize("fam,k,m,bitslice", [("rs", 10, 4, None), ("cauchy", 6, 3, None), ("rs", 8, 6, "0"),
                                              ("rs", 16, 8, "3"), ("isal_cauchy", 10, 6, "3")])
@pytest.mark.parametrize("cs", [512, 2560])
def test_one_map_batch_partial_wave(fam, k, m, bitslice, cs, knobs):
    """One-map pointer batches whose last wave is partial (512-byte chunks:
    32 of 64 lanes hold a unit; 2560: the bit-sliced kernel's second 2 KiB
    tile half full).  Gathered kernels fetch the pointer row one entry per
    lane (outputs in lanes 32 +) and read it back with v_readlane, so no
    lane may leave before the last read (stream_common.hpp gather_unit):
    gf8 (RS(10,4)), bitmatrix (Cauchy(6,3)), one-pass multi-group
    (RS(8,6), MEC_BITSLICE=0) and bit-sliced (MEC_BITSLICE=3) launches,
    encode then a delta update of one column, both against the oracle."""
    knobs("MEC_BITSLICE", bitslice)
    n = 5
    rng = np.random.default_rng(cs + k)
    slots = rng.permutation(n * (k + m))
    slab = Slab(n * (k + m), cs, 8, True, 77 + k)
    before = slab.snapshot()
    c = Codec(fam, k, m, cs)
    dptr, pptr = [], []
    for s in range(n):
        row = slots[s * (k + m):(s + 1) * (k + m)]
        dptr += [slab.addr(row[j]) for j in range(k)]
        pptr += [slab.addr(row[k + i]) for i in range(m)]
    c.encode_batch(dptr, pptr, mem="device")
    after = slab.snapshot()
    for s in range(n):
        row = slots[s * (k + m):(s + 1) * (k + m)]
        par = O.encode(fam, k, m, [chunk_of(before, slab, row[j]).copy() for j in range(k)], cs)
        for i in range(m):
            assert np.array_equal(chunk_of(after, slab, row[k + i]), par[i]), (fam, cs, s, i)
    # delta update of column 1 into every parity (read-modify-write gathers)
    j = 1
    deltas = torch.from_numpy(np.stack([O.fill(cs, 500 + s) for s in range(n)])).to(DEV)
    c.encode_update_batch([j] * n, [deltas.data_ptr() + s * cs for s in range(n)], pptr)
    upd = slab.snapshot()
    dh = deltas.cpu().numpy()
    for s in range(n):
        row = slots[s * (k + m):(s + 1) * (k + m)]
        dat = [np.zeros(cs, np.uint8) for _ in range(k)]
        dat[j] = dh[s]
        dp = O.encode(fam, k, m, dat, cs)
        for i in range(m):
            want = chunk_of(after, slab, row[k + i]) ^ dp[i]
            assert np.array_equal(chunk_of(upd, slab, row[k + i]), want), (fam, cs, "update", s, i)
    c.close()


def test_device_batches_from_threads_share_table_slots():
    """One-map device batches large enough for the HBM table copy (> 256
    stripes: the rows go through the context's copy stream, batch.cpp
    table_upload) from 4 threads on one context, each on its own stream and
    alternating between two buffer sets, so a table slot reused before its
    launches finished would code another call's chunks.  Every call's parity
    must equal the strided launch over the same data."""
    k, m, cs, n, calls = 6, 3, 4096, 600, 12
    c = Codec("rs", k, m, cs)
    errors = []

    def worker(t):
        try:
            st = torch.cuda.Stream()
            with torch.cuda.stream(st):
                sets = []
                for b in range(2):
                    d = torch.empty(n, k, cs, dtype=torch.uint8, device=DEV)
                    fill_random(d, 4000 + 10 * t + b)
                    sets.append((d, torch.zeros(n, m, cs, dtype=torch.uint8, device=DEV)))
                ref = []
                for d, _ in sets:
                    r = torch.empty(n, m, cs, dtype=torch.uint8, device=DEV)
                    c.encode(d, r, stream=st.cuda_stream)
                    ref.append(r)
                for i in range(calls):
                    d, p = sets[i % 2]
                    p.zero_()
                    dp = [d.data_ptr() + (s * k + j) * cs for s in range(n) for j in range(k)]
                    pp = [p.data_ptr() + (s * m + j) * cs for s in range(n) for j in range(m)]
                    c.encode_batch(dp, pp, mem="device", stream=st.cuda_stream)
                    st.synchronize()
                    if not torch.equal(p, ref[i % 2]):
                        errors.append((t, i))
        except Exception as e:  # noqa: BLE001 - reported below
            errors.append((t, repr(e)))

    th = [threading.Thread(target=worker, args=(t,)) for t in range(4)]
    for x in th:
        x.start()
    for x in th:
        x.join()
    c.close()
    assert not errors, errors


@pytest.mark.parametrize("fam", FAMS)
@pytest.mark.parametrize("cs,shift", [(4096, 3), (1032, 3), (65536, 0)])
def test_batch32_slab_offsets(fam, cs, shift):
    """mec_*_batch32 (ABI 6): the pointer batches given
    as 32-bit offsets into one device slab (ChunkPool-like slots of
    8 + chunkSize bytes in random order, chunk_pool.cc:22-55) — encode with
    Coding::zeros columns and unwanted parities (MEC_NULL_OFF), decode with a
    different pattern per stripe (none, <= m, > m), delta updates with
    skipped stripes — equal the 64-bit pointer-row calls and the oracle."""
    k, m, n = 6, 3, 40
    if fam == "cauchy" and O.cauchy_getw(k, m, cs) < 1:
        pytest.skip("no Cauchy w for this chunk size")
    NULL = _lib.NULL_OFF
    rng = np.random.default_rng(cs + shift)
    slab = Slab(n * (k + m), cs, 8, True, 9 + cs)
    twin = Slab(n * (k + m), cs, 8, True, 9 + cs)
    slots = rng.permutation(n * (k + m))
    off = lambda i: (i * slab.slot + slab.hdr) >> shift  # noqa: E731
    if shift:
        assert all((i * slab.slot + slab.hdr) % (1 << shift) == 0 for i in range(4))
    c = Codec(fam, k, m, cs)
    # encode: column 2 of every 5th stripe is Coding::zeros, parity 1 unwanted on odd stripes
    doff, poff, dptr, pptr = [], [], [], []
    for s in range(n):
        row = slots[s * (k + m):(s + 1) * (k + m)]
        for j in range(k):
            z = s % 5 == 0 and j == 2
            doff.append(NULL if z else off(row[j]))
            dptr.append(0 if z else twin.addr(row[j]))
        for i in range(m):
            u = s % 2 == 1 and i == 1
            poff.append(NULL if u else off(row[k + i]))
            pptr.append(0 if u else twin.addr(row[k + i]))
    c.encode_batch32(slab.t, shift, doff, poff)
    c.encode_batch(dptr, pptr)
    torch.cuda.synchronize()
    assert torch.equal(slab.t, twin.t)
    for s in range(0, n, 7):
        row = slots[s * (k + m):(s + 1) * (k + m)]
        data = [np.zeros(cs, np.uint8) if (s % 5 == 0 and j == 2) else slab.chunk(row[j]) for j in range(k)]
        want = O.encode(fam, k, m, data, cs)
        for i in range(m):
            if not (s % 2 == 1 and i == 1):
                assert np.array_equal(slab.chunk(row[k + i]), want[i]), (s, i)
    # decode: per-stripe patterns, every 9th has more than m missing
    masks, coff, cptr, pats = [], [], [], []
    for s in range(n):
        row = slots[s * (k + m):(s + 1) * (k + m)]
        e = m + 1 if s % 9 == 4 else int(rng.integers(0, m + 1))
        pat = sorted(rng.choice(k + m, size=e, replace=False).tolist())
        pats.append(pat)
        masks.append(sum(1 << i for i in range(k + m) if i not in pat))
        coff += [off(x) for x in row]
        cptr += [twin.addr(x) for x in row]
    before = slab.t.clone()
    r32 = c.decode_batch32(slab.t, shift, coff, masks)
    r64 = c.decode_batch(cptr, masks)
    assert r32 == r64
    assert all((r == _lib.MEC_ETOOMANY) == (s % 9 == 4) for s, r in enumerate(r32))
    torch.cuda.synchronize()
    assert torch.equal(slab.t, twin.t)
    hb = before.cpu().numpy()
    for s in range(1, n, 6):
        if len(pats[s]) > m or not pats[s]:
            continue
        row = slots[s * (k + m):(s + 1) * (k + m)]
        chunks = [hb[x * slab.slot + 8:x * slab.slot + 8 + cs].copy() for x in row]
        assert O.decode(fam, k, m, chunks, pats[s], cs) == 0
        for i in range(k + m):
            assert np.array_equal(slab.chunk(row[i]), chunks[i]), (s, pats[s], i)
    # delta updates: stripe s's delta is slot row[0]'s chunk, every 4th stripe skipped
    js = [int(rng.integers(0, k)) for _ in range(n)]
    dl32 = [NULL if s % 4 == 3 else off(slots[s * (k + m)]) for s in range(n)]
    dl64 = [0 if s % 4 == 3 else twin.addr(slots[s * (k + m)]) for s in range(n)]
    po32 = [off(slots[s * (k + m) + k + i]) for s in range(n) for i in range(m)]
    po64 = [twin.addr(slots[s * (k + m) + k + i]) for s in range(n) for i in range(m)]
    c.encode_update_batch32(slab.t, shift, js, dl32, po32, parity_mask=0b101)
    c.encode_update_batch(js, dl64, po64, parity_mask=0b101)
    torch.cuda.synchronize()
    assert torch.equal(slab.t, twin.t)
    # bad arguments
    with pytest.raises(_lib.MecError):
        c.encode_batch32(slab.t, 13, doff, poff)
    with pytest.raises(_lib.MecError):
        c.encode_batch32(0, shift, doff, poff)
