"""GPU parity of codes with more than 4 outputs per launch (m > 4): the
one-pass multi-group GF(2^8) kernel (gf8_mg_kernel: every source read once,
row groups of 3 or 4 coded from the same registers) and the bitmatrix
kernel's 5..8-output instantiations.  The reference accepts any k + m <= 32
(rscoding.cc:26-29, RS_N_MAX); every result is compared bit for bit with
the oracle (pinned on the reference, tests/test_oracle.py): Vandermonde
(row 0 / column 0 ones) and dense matrices, padded last groups (m = 5, 7,
9, 13), in-place and split layouts, accumulating delta updates, parity
subsets, and decodes of 5..8 erasures."""
import itertools

import numpy as np
import pytest

import _oracle as O

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

from memec_amd import Codec  # noqa: E402

DEV = "cuda:0"
FAMS = ["rs", "cauchy", "isal_rs", "isal_cauchy"]


@pytest.fixture(scope="module", autouse=True)
def _gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    torch.cuda.set_device(0)
    yield
    torch.cuda.synchronize()


def dev(a):
    return torch.from_numpy(np.ascontiguousarray(a)).to(DEV)


def host(t):
    torch.cuda.synchronize()
    return t.cpu().numpy()


def ok_shape(fam, k, m, cs):
    if fam == "cauchy":
        w = O.cauchy_getw(k, m, cs)
        return 1 <= w <= 8
    return cs % 8 == 0


SHAPES = [(16, 8, 65536, 3), (12, 8, 4096, 5), (10, 6, 4096, 4), (8, 5, 8192, 3), (20, 7, 2048, 3),
          (4, 9, 1024, 4), (3, 13, 512, 2), (1, 31, 256, 2), (24, 8, 1024, 2)]


@pytest.mark.parametrize("fam", FAMS)
def test_wide_encode_vs_oracle(fam):
    for k, m, cs, n in SHAPES:
        if not ok_shape(fam, k, m, cs):
            continue
        data = O.fill(n * k * cs, 700 + k * 10 + m).reshape(n, k, cs)
        c = Codec(fam, k, m, cs)
        par = torch.zeros(n, m, cs, dtype=torch.uint8, device=DEV)
        c.encode(dev(data), par)
        got = host(par)
        for s in range(n):
            want = np.stack(O.encode(fam, k, m, [data[s, j].copy() for j in range(k)], cs))
            assert np.array_equal(got[s], want), (fam, k, m, cs, s)
        c.close()


@pytest.mark.parametrize("fam", ["rs", "isal_cauchy", "cauchy"])
def test_wide_encode_in_place_and_subsets(fam):
    """Parity inside the stripe buffer (in-place layout, two windows) and
    parity subsets of 5..7 rows (row 0 missing: no all-ones row)."""
    k, m, cs, n = 10, 8, 4096, 6
    data = O.fill(n * k * cs, 4711).reshape(n, k, cs)
    want = np.stack([np.stack(O.encode(fam, k, m, [data[s, j].copy() for j in range(k)], cs)) for s in range(n)])
    c = Codec(fam, k, m, cs)
    st = torch.zeros(n, k + m, cs, dtype=torch.uint8, device=DEV)
    st[:, :k] = dev(data)
    c.encode(st[:, :k], st[:, k:])
    assert np.array_equal(host(st[:, k:]), want)
    for mask in (0b11111110, 0b01111100, 0b11011011, 0b11111):
        out = torch.full((n, m, cs), 0xA5, dtype=torch.uint8, device=DEV)
        c.encode(st[:, :k], out, mask)
        o = host(out)
        for i in range(m):
            if mask >> i & 1:
                assert np.array_equal(o[:, i], want[:, i]), (mask, i)
            else:
                assert (o[:, i] == 0xA5).all(), (mask, i)
    c.close()


@pytest.mark.parametrize("fam", FAMS)
def test_wide_decode_vs_oracle(fam):
    """5..8 erasures, data-only / parity-only / mixed, on random stripes
    (non-codewords pin the survivor choice), in place and split."""
    k, m, cs, n = 12, 8, 2048, 2
    if not ok_shape(fam, k, m, cs):
        pytest.skip("no Cauchy w")
    base = O.fill(n * (k + m) * cs, 99).reshape(n, k + m, cs)
    c = Codec(fam, k, m, cs)
    pats = [list(range(5)), list(range(8)), [0, 3, 12, 13, 14, 19], list(range(12, 20)), [1, 2, 5, 7, 11, 15, 17]]
    for pat in pats:
        t = dev(base.copy())
        t[:, pat] = 0
        present = sum(1 << i for i in range(k + m) if i not in pat)
        c.decode(t, present)
        got = host(t)
        out = torch.zeros(n, k + m, cs, dtype=torch.uint8, device=DEV)
        c.decode_split(dev(base), out, present)
        got2 = host(out)
        for s in range(n):
            chunks = [base[s, i].copy() for i in range(k + m)]
            assert O.decode(fam, k, m, chunks, pat, cs) == 0
            for i in range(k + m):
                assert np.array_equal(got[s, i], chunks[i]), (fam, pat, s, i)
            for i in pat:
                assert np.array_equal(got2[s, i], chunks[i]), (fam, pat, s, i)
    c.close()


@pytest.mark.parametrize("rows", ["3", "4", "8", None])
@pytest.mark.parametrize("fam", ["rs", "isal_cauchy"])
def test_wide_group_rows_forced(fam, rows, knobs):
    """8 outputs coded in groups of 3, 4 or 8 rows (MEC_MG_ROWS; the rule
    picks 8 for RS(16,8) and the dense ISA-L Cauchy(12,8)): same bytes,
    encode and in-place decode of 8 erasures, plus an accumulating update."""
    knobs("MEC_BITSLICE", "0")  # the one-pass kernel itself (the bit-sliced one takes these once compiled)
    knobs("MEC_MG_ROWS", rows)
    for k, m, cs, n in [(16, 8, 4096, 3), (12, 8, 2048, 3), (20, 8, 1024, 2), (24, 8, 1024, 2), (12, 16, 512, 2)]:
        data = O.fill(n * k * cs, 60 + k + m).reshape(n, k, cs)
        want = np.stack([np.stack(O.encode(fam, k, m, [data[s, j].copy() for j in range(k)], cs)) for s in range(n)])
        c = Codec(fam, k, m, cs)
        st = torch.zeros(n, k + m, cs, dtype=torch.uint8, device=DEV)
        st[:, :k] = dev(data)
        c.encode(st[:, :k], st[:, k:])
        assert np.array_equal(host(st[:, k:]), want), (fam, rows, k, m)
        pat = list(range(0, k + m, 3))[:m]
        t = st.clone()
        t[:, pat] = 0
        c.decode(t, sum(1 << i for i in range(k + m) if i not in pat))
        torch.cuda.synchronize()
        assert torch.equal(t, st), (fam, rows, k, m, pat)
        delta = O.fill(n * cs, 61 + k).reshape(n, cs)
        d2 = data.copy()
        d2[:, 1] ^= delta
        par = st[:, k:].clone()
        c.encode_update(1, dev(delta), par)
        want2 = np.stack([np.stack(O.encode(fam, k, m, [d2[s, j].copy() for j in range(k)], cs)) for s in range(n)])
        assert np.array_equal(host(par), want2), (fam, rows, k, m, "update")
        c.close()


@pytest.mark.parametrize("fam", ["rs", "isal_rs"])
def test_forced_three_row_groups_31_rows(fam, knobs):
    """RS(1,31) with MEC_MG_ROWS=3: 31 rows in groups
    of 3 would be 11 groups, 33 of the one-pass kernel's 32 output slots —
    the round-4 library read dst_off[32] past its kernel arguments.  The
    planner now keeps the forced count only where the groups fit and falls
    back to the rule (8 groups of 4) here; encode, a 30-erasure in-place
    decode and an accumulating update equal the oracle, and RS(1,30) keeps
    the forced 10 x 3 groups."""
    knobs("MEC_BITSLICE", "0")
    knobs("MEC_MG_ROWS", "3")
    for k, m in [(1, 31), (1, 30), (2, 30)]:
        cs, n = 512, 3
        data = O.fill(n * k * cs, 900 + m).reshape(n, k, cs)
        want = np.stack([np.stack(O.encode(fam, k, m, [data[s, j].copy() for j in range(k)], cs)) for s in range(n)])
        c = Codec(fam, k, m, cs)
        st = torch.zeros(n, k + m, cs, dtype=torch.uint8, device=DEV)
        st[:, :k] = dev(data)
        c.encode(st[:, :k], st[:, k:])
        assert np.array_equal(host(st[:, k:]), want), (fam, k, m)
        keep = k + m - 1  # only the last parity survives (k = 1) / two chunks (k = 2)
        pat = [i for i in range(k + m) if i != keep and (k == 1 or i != 0)]
        t = st.clone()
        t[:, pat] = 0
        c.decode(t, sum(1 << i for i in range(k + m) if i not in pat))
        torch.cuda.synchronize()
        assert torch.equal(t, st), (fam, k, m)
        delta = O.fill(n * cs, 901 + m).reshape(n, cs)
        d2 = data.copy()
        d2[:, 0] ^= delta
        par = st[:, k:].clone()
        c.encode_update(0, dev(delta), par)
        want2 = np.stack([np.stack(O.encode(fam, k, m, [d2[s, j].copy() for j in range(k)], cs)) for s in range(n)])
        assert np.array_equal(host(par), want2), (fam, k, m, "update")
        c.close()


def test_one_pass_table_cache_is_bounded(monkeypatch, knobs):
    """The one-pass kernel's permute tables are cached per matrix up to
    MEC_MG_CACHE_BYTES (the cache grew without bound, one
    device allocation per erasure pattern).  RS(16,8) decodes of 60
    distinct 5..8-erasure patterns under a 3-table cap: every stripe is
    rebuilt, the cache holds at most the cap, the patterns past it ran as
    4-row launches, and no device memory leaks past the cap."""
    k, m, cs, n = 16, 8, 1024, 2
    monkeypatch.setenv("MEC_MG_CACHE_BYTES", str(3 * 8 * 16 * 32))
    knobs("MEC_BITSLICE", "0")
    c = Codec("rs", k, m, cs)
    data = O.fill(n * k * cs, 321).reshape(n, k, cs)
    st = torch.zeros(n, k + m, cs, dtype=torch.uint8, device=DEV)
    st[:, :k] = dev(data)
    c.encode(st[:, :k], st[:, k:])
    torch.cuda.synchronize()
    free0 = torch.cuda.mem_get_info()[0]
    rng = np.random.default_rng(5)
    seen = set()
    while len(seen) < 60:
        e = int(rng.integers(5, m + 1))
        pat = tuple(sorted(rng.choice(k + m, size=e, replace=False).tolist()))
        if pat in seen:
            continue
        seen.add(pat)
        t = st.clone()
        t[:, list(pat)] = 0
        c.decode(t, sum(1 << i for i in range(k + m) if i not in pat))
        torch.cuda.synchronize()
        assert torch.equal(t, st), pat
        del t
    s = c.stats()
    assert s["mg_cache_bytes"] <= 3 * 8 * 16 * 32, s
    assert 1 <= s["mg_cache_tables"] <= 4, s
    assert s["mg_cache_uncached"] >= 50, s
    # one 4 MiB arena block at most (plus torch's own caching slack)
    assert free0 - torch.cuda.mem_get_info()[0] <= (8 << 20), (free0, torch.cuda.mem_get_info()[0])
    c.close()


@pytest.mark.parametrize("fam", ["rs", "cauchy", "isal_rs"])
def test_wide_roundtrip_every_pattern_small(fam):
    """RS(3,6)-sized code: every erasure pattern of 5 and 6 chunks."""
    k, m, cs, n = 3, 6, 96, 2
    c = Codec(fam, k, m, cs)
    data = O.fill(n * k * cs, 5).reshape(n, k, cs)
    par = torch.zeros(n, m, cs, dtype=torch.uint8, device=DEV)
    c.encode(dev(data), par)
    stripe = torch.cat([dev(data), par], dim=1)
    for e in (5, 6):
        for pat in itertools.combinations(range(k + m), e):
            t = stripe.clone()
            t[:, list(pat)] = 0
            c.decode(t, sum(1 << i for i in range(k + m) if i not in pat))
            torch.cuda.synchronize()
            assert torch.equal(t, stripe), pat
    c.close()


@pytest.mark.parametrize("fam", ["rs", "cauchy", "isal_rs"])
def test_wide_update_linearity(fam):
    """encode(D ^ delta_j) == encode(D) ^ update_j(delta) with 6..8 parities
    (the accumulate path reads and writes every parity once)."""
    for k, m, cs in [(16, 8, 8192), (6, 6, 4096)]:
        n, j = 16, 3
        data = O.fill(n * k * cs, 31 + m).reshape(n, k, cs)
        delta = O.fill(n * cs, 32 + m).reshape(n, cs)
        c = Codec(fam, k, m, cs)
        par = torch.zeros(n, m, cs, dtype=torch.uint8, device=DEV)
        c.encode(dev(data), par)
        d2 = data.copy()
        d2[:, j] ^= delta
        par2 = torch.zeros_like(par)
        c.encode(dev(d2), par2)
        c.encode_update(j, dev(delta), par)
        torch.cuda.synchronize()
        assert torch.equal(par, par2), (fam, k, m)
        c.close()


# ---- pointer batches (gathered kernels): every row group in one launch ----

from test_gpu_batch import Slab, chunk_of, random_patterns, zeros  # noqa: E402


@pytest.mark.parametrize("cs", [1024, 1032])
@pytest.mark.parametrize("mem", ["device", "host"])
@pytest.mark.parametrize("fam", FAMS)
def test_wide_encode_batch_scattered(fam, mem, cs):
    """mec_encode_batch with 7 parities (row groups of 4 + 3), scattered
    ChunkPool-like slots, Coding::zeros columns and unwanted parities;
    cs = 1032 has an 8-byte tail (the per-row-group tail
    launches of multi-map wide batches were untested)."""
    k, m, n = 10, 7, 24
    if fam == "cauchy" and not ok_shape(fam, k, m, cs):
        pytest.skip("no Cauchy w")
    rng = np.random.default_rng(17)
    slots = rng.permutation(n * (k + m))
    slab = Slab(n * (k + m), cs, 8, mem == "device", 77)
    before = slab.snapshot()
    dptr, pptr, want = [], [], []
    for s in range(n):
        row = slots[s * (k + m):(s + 1) * (k + m)]
        zero_cols = set(rng.choice(k, size=int(rng.integers(0, 4)), replace=False).tolist())
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
            ref = par[i] if wanted[i] else chunk_of(before, slab, row[k + i])
            assert np.array_equal(got, ref), (fam, mem, s, i, wanted[i])
    c.close()


@pytest.mark.parametrize("cs", [1024, 1032])
@pytest.mark.parametrize("mem", ["device", "host"])
@pytest.mark.parametrize("fam", FAMS)
def test_wide_decode_batch_mixed_patterns(fam, mem, cs):
    """mec_decode_batch, RS/CRS(8,6): every stripe its own pattern of 0..6
    erasures (and some with 7: too many), random non-codeword stripes;
    cs = 1032: the per-row-group tail launches (8-byte tail)."""
    k, m, n = 8, 6, 40
    if fam == "cauchy" and not ok_shape(fam, k, m, cs):
        pytest.skip("no Cauchy w")
    rng = np.random.default_rng(23)
    slots = rng.permutation(n * (k + m))
    slab = Slab(n * (k + m), cs, 8, mem == "device", 4242)
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
        if len(pats[s]) <= m and pats[s]:
            assert res[s] == 0
            assert O.decode(fam, k, m, chunks, pats[s], cs) == 0
        for i in range(k + m):
            assert np.array_equal(chunk_of(after, slab, row[i]), chunks[i]), (fam, mem, s, pats[s], i)
    c.close()


@pytest.mark.parametrize("mem", ["device", "host"])
@pytest.mark.parametrize("fam", ["rs", "isal_rs", "isal_cauchy", "cauchy"])
def test_wide_batch_one_map_one_pass(fam, mem):
    """Pointer batches whose stripes share one map (every parity wanted, no
    zero columns; one erasure pattern): the one-pass kernel reads the
    pointer rows itself (gathered gf8_mg_kernel: row-0 / column-0 XORs,
    groups of 8 at K = 16, of 3 + 3 at K = 6), scattered 8-byte-aligned
    slots: encode, then in-place decode of the same 6 erasures in every
    stripe.  Cauchy bitmatrix maps of up to 8 outputs run one gathered
    bm_kernel launch."""
    for k, m, cs, n in [(16, 8, 4096, 20), (6, 6, 2048, 24), (10, 6, 4096, 12)]:
        if not ok_shape(fam, k, m, cs):
            continue
        rng = np.random.default_rng(k * 31 + m)
        slots = rng.permutation(n * (k + m))
        slab = Slab(n * (k + m), cs, 8, mem == "device", 500 + k)
        before = slab.snapshot()
        c = Codec(fam, k, m, cs)
        dptr, pptr = [], []
        for s in range(n):
            row = slots[s * (k + m):(s + 1) * (k + m)]
            dptr += [slab.addr(row[j]) for j in range(k)]
            pptr += [slab.addr(row[k + i]) for i in range(m)]
        c.encode_batch(dptr, pptr, mem=mem)
        after = slab.snapshot()
        full = []
        for s in range(n):
            row = slots[s * (k + m):(s + 1) * (k + m)]
            data = [chunk_of(before, slab, row[j]).copy() for j in range(k)]
            par = O.encode(fam, k, m, data, cs)
            for i in range(m):
                assert np.array_equal(chunk_of(after, slab, row[k + i]), par[i]), (fam, mem, k, m, s, i)
            full.append(data + list(par))
        # the same 6 erasures in every stripe, rebuilt in place
        pat = [0, 2, 5, k, k + 1, k + m - 1]
        present = sum(1 << i for i in range(k + m) if i not in pat)
        ptrs = []
        for s in range(n):
            row = slots[s * (k + m):(s + 1) * (k + m)]
            ptrs += [slab.addr(i) for i in row]
            for i in pat:
                o = int(row[i]) * slab.slot + slab.hdr
                if slab.t is not None:
                    slab.t[o:o + cs] = 0
                else:
                    slab.host[o:o + cs] = 0
        res = c.decode_batch(ptrs, [present] * n, mem=mem)
        assert all(r == 0 for r in res), res
        after = slab.snapshot()
        for s in range(n):
            row = slots[s * (k + m):(s + 1) * (k + m)]
            for i in range(k + m):
                assert np.array_equal(chunk_of(after, slab, row[i]), full[s][i]), (fam, mem, k, m, s, i)
        c.close()


# ---- run-time compiled bit-sliced kernels (jit.cpp, bitslice.cpp) ----

BS_SHAPES = [(16, 8, 8192, 3), (12, 8, 4096, 3), (10, 6, 2048, 4), (8, 5, 3072, 3), (20, 7, 1040, 3),
             (1, 31, 512, 2), (24, 8, 16, 5), (3, 13, 2064, 2)]


@pytest.mark.parametrize("fam", ["rs", "isal_rs", "isal_cauchy"])
def test_bitslice_encode_decode_update_vs_oracle(fam, knobs):
    """MEC_BITSLICE=3 (compile at first use, every wide launch): every >
    4-output launch runs the matrix's own bit-sliced kernel — encode split and in place, decodes
    of 5..m erasures in place and split (random non-codeword stripes pin the
    decoding matrix), accumulating updates — on chunks that are and are not
    multiples of the 2 KiB tile (16, 1040, 2064, 3072 bytes), equal to the
    oracle; the stats show the kernels built and launched, none failed."""
    knobs("MEC_BITSLICE", "3")
    for k, m, cs, n in BS_SHAPES:
        data = O.fill(n * k * cs, 7000 + k * 10 + m).reshape(n, k, cs)
        want = np.stack([np.stack(O.encode(fam, k, m, [data[s, j].copy() for j in range(k)], cs)) for s in range(n)])
        c = Codec(fam, k, m, cs)
        par = torch.zeros(n, m, cs, dtype=torch.uint8, device=DEV)
        c.encode(dev(data), par)
        assert np.array_equal(host(par), want), (fam, k, m, cs, "split")
        st = torch.zeros(n, k + m, cs, dtype=torch.uint8, device=DEV)
        st[:, :k] = dev(data)
        c.encode(st[:, :k], st[:, k:])
        assert np.array_equal(host(st[:, k:]), want), (fam, k, m, cs, "in place")
        base = O.fill(n * (k + m) * cs, 7100 + k + m).reshape(n, k + m, cs)  # non-codewords
        rng = np.random.default_rng(k * 100 + m)
        sizes = [e for e in sorted({5, min(m, 6), m}) if e <= m]
        for e in sizes:
            pat = sorted(rng.choice(k + m, size=e, replace=False).tolist())
            present = sum(1 << i for i in range(k + m) if i not in pat)
            t = dev(base.copy())
            c.decode(t, present)
            got = host(t)
            out = torch.zeros(n, k + m, cs, dtype=torch.uint8, device=DEV)
            c.decode_split(dev(base), out, present)
            got2 = host(out)
            for s in range(n):
                chunks = [base[s, i].copy() for i in range(k + m)]
                assert O.decode(fam, k, m, chunks, pat, cs) == 0
                for i in pat:
                    assert np.array_equal(got[s, i], chunks[i]), (fam, k, m, cs, pat, s, i)
                    assert np.array_equal(got2[s, i], chunks[i]), (fam, k, m, cs, pat, s, i, "split")
        delta = O.fill(n * cs, 7200 + k).reshape(n, cs)
        j = k // 2
        d2 = data.copy()
        d2[:, j] ^= delta
        c.encode_update(j, dev(delta), par)
        want2 = np.stack([np.stack(O.encode(fam, k, m, [d2[s, jj].copy() for jj in range(k)], cs)) for s in range(n)])
        assert np.array_equal(host(par), want2), (fam, k, m, cs, "update")
        s = c.stats()
        # every launch above ran a bit-sliced kernel: the encode (split and
        # in place), each decode pattern (in place and split), the update;
        # one kernel per distinct matrix (RS(1,31)'s decodes of 31 chunks
        # reuse the encode's all-ones matrix)
        assert s["jit_failed"] == 0 and s["jit_kernels"] >= 2, (k, m, s)
        assert s["jit_launches"] >= 3 + 2 * len(sizes), (k, m, s)
        c.close()


def test_bitslice_rule(knobs):
    """MEC_BITSLICE=2: the rule (jit.cpp jit_wanted) — every byte-wise launch
    of more than 4 outputs on 16-byte-multiple chunks takes the bit-sliced
    kernel: Vandermonde encodes under 12 sources and outputs outnumbering
    the sources included (their wave caps, plan_bs), strided and through
    pointer rows; 4-output launches do not; same bytes."""
    knobs("MEC_BITSLICE", "2")
    for k, m, cs, want_enc, want_dec in [(10, 6, 2048, True, True), (12, 6, 2048, True, True),
                                         (4, 12, 2048, True, True), (10, 4, 2048, False, False)]:
        n = 2
        data = O.fill(n * k * cs, 9100 + k).reshape(n, k, cs)
        want = np.stack([np.stack(O.encode("rs", k, m, [data[s, j].copy() for j in range(k)], cs)) for s in range(n)])
        c = Codec("rs", k, m, cs)
        par = torch.zeros(n, m, cs, dtype=torch.uint8, device=DEV)
        data_t = dev(data)
        c.encode(data_t, par)
        assert np.array_equal(host(par), want)
        assert (c.stats()["jit_launches"] == 1) == want_enc, (k, m, c.stats())
        st = torch.cat([dev(data), par], dim=1)
        t = st.clone()
        pat = list(range(m))
        t[:, pat] = 0
        before = c.stats()["jit_launches"]
        c.decode(t, sum(1 << i for i in range(k + m) if i not in pat))
        torch.cuda.synchronize()
        assert torch.equal(t, st)
        assert c.stats()["jit_launches"] == before + int(want_dec), c.stats()
        # through pointer rows (a one-map batch) too
        par2 = torch.zeros_like(par)
        before = c.stats()["jit_launches"]
        c.encode_batch([data_t[s, j].data_ptr() for s in range(n) for j in range(k)],
                       [par2[s, i].data_ptr() for s in range(n) for i in range(m)], mem="device")
        torch.cuda.synchronize()
        assert torch.equal(par2, par)
        assert c.stats()["jit_launches"] == before + int(m > 4), (k, m, c.stats())
        c.close()


def test_bitslice_async_takes_over(knobs):
    """Default mode (MEC_BITSLICE unset = 1): the first call of a matrix
    runs gf8_mg_kernel while its bit-sliced kernel compiles in the
    background; once built, the next calls launch it — same bytes either
    way (RS(16,8) encode)."""
    import time
    knobs("MEC_BITSLICE", None)
    k, m, cs, n = 16, 8, 4096, 4
    data = O.fill(n * k * cs, 8123).reshape(n, k, cs)
    want = np.stack([np.stack(O.encode("rs", k, m, [data[s, j].copy() for j in range(k)], cs)) for s in range(n)])
    c = Codec("rs", k, m, cs)
    d = dev(data)
    par = torch.zeros(n, m, cs, dtype=torch.uint8, device=DEV)
    c.encode(d, par)
    assert np.array_equal(host(par), want)
    assert c.stats()["jit_launches"] == 0
    t0 = time.time()
    while c.stats()["jit_pending"] and time.time() - t0 < 60:
        time.sleep(0.05)
    s = c.stats()
    assert s["jit_pending"] == 0 and s["jit_kernels"] == 1 and s["jit_failed"] == 0, s
    par.zero_()
    c.encode(d, par)
    assert np.array_equal(host(par), want)
    assert c.stats()["jit_launches"] == 1
    c.close()


@pytest.mark.parametrize("mem", ["device", "host"])
def test_bitslice_pointer_batch_one_map(mem, knobs):
    """Pointer batches with one map and > 4 outputs through the gathered
    bit-sliced kernel (scattered 8-byte-aligned ChunkPool-like slots; one
    straight-line 2 KiB tile per block by default, and blocks looping over
    3 tiles under MEC_BS_TPB=3): RS(16,8) and ISA-L
    Cauchy(10,6) encode, then the same 6 erasures rebuilt in place in every
    stripe."""
    knobs("MEC_BITSLICE", "2")
    knobs("MEC_BS_TPB", {"device": "3", "host": None}[mem])
    for fam, k, m, cs, n in [("rs", 16, 8, 4096, 12), ("isal_cauchy", 10, 6, 2064, 10)]:
        rng = np.random.default_rng(k * 7 + m)
        slots = rng.permutation(n * (k + m))
        slab = Slab(n * (k + m), cs, 8, mem == "device", 900 + k)
        before = slab.snapshot()
        c = Codec(fam, k, m, cs)
        dptr, pptr = [], []
        for s in range(n):
            row = slots[s * (k + m):(s + 1) * (k + m)]
            dptr += [slab.addr(row[j]) for j in range(k)]
            pptr += [slab.addr(row[k + i]) for i in range(m)]
        c.encode_batch(dptr, pptr, mem=mem)
        after = slab.snapshot()
        full = []
        for s in range(n):
            row = slots[s * (k + m):(s + 1) * (k + m)]
            dat = [chunk_of(before, slab, row[j]).copy() for j in range(k)]
            par = O.encode(fam, k, m, dat, cs)
            for i in range(m):
                assert np.array_equal(chunk_of(after, slab, row[k + i]), par[i]), (fam, mem, s, i)
            full.append(dat + list(par))
        pat = [0, 2, 5, k, k + 1, k + m - 1]
        present = sum(1 << i for i in range(k + m) if i not in pat)
        ptrs = []
        for s in range(n):
            row = slots[s * (k + m):(s + 1) * (k + m)]
            ptrs += [slab.addr(i) for i in row]
            for i in pat:
                o = int(row[i]) * slab.slot + slab.hdr
                if slab.t is not None:
                    slab.t[o:o + cs] = 0
                else:
                    slab.host[o:o + cs] = 0
        res = c.decode_batch(ptrs, [present] * n, mem=mem)
        assert all(r == 0 for r in res), res
        after = slab.snapshot()
        for s in range(n):
            row = slots[s * (k + m):(s + 1) * (k + m)]
            for i in range(k + m):
                assert np.array_equal(chunk_of(after, slab, row[i]), full[s][i]), (fam, mem, s, i)
        if mem == "device":
            assert c.stats()["jit_launches"] >= 2, c.stats()
        c.close()


def test_bitslice_xor_twin_probe(knobs):
    """mec_set_probe(MEC_PROBE_XOR) on a wide launch runs the bit-sliced
    kernel's arithmetic-free twin (same loads and stores): every output is
    the XOR of the sources; off again, the code's bytes come back."""
    knobs("MEC_BITSLICE", "2")
    k, m, cs, n = 16, 8, 4096, 3
    data = O.fill(n * k * cs, 8321).reshape(n, k, cs)
    c = Codec("rs", k, m, cs)
    par = torch.zeros(n, m, cs, dtype=torch.uint8, device=DEV)
    c.set_probe(True)
    c.encode(dev(data), par)
    x = np.bitwise_xor.reduce(data, axis=1)
    got = host(par)
    for i in range(m):
        assert np.array_equal(got[:, i], x), i
    c.set_probe(False)
    c.encode(dev(data), par)
    want = np.stack([np.stack(O.encode("rs", k, m, [data[s, j].copy() for j in range(k)], cs)) for s in range(n)])
    assert np.array_equal(host(par), want)
    assert c.stats()["jit_kernels"] == 2, c.stats()
    c.close()


@pytest.mark.parametrize("m", list(range(5, 32)))
def test_bitslice_every_output_count(m, knobs):
    """The bit-sliced kernel of every output count m = 5..31 (sync compile,
    MEC_BITSLICE=2) at one, half and all of the source counts k + m <= 32
    allows: the RS encode (Vandermonde, capped split launch) and an in-place
    decode of min(m, 8) erasures over random non-codewords (dense matrix,
    capped in-place launch), on a chunk with a partial 2 KiB tile (2064 B),
    equal to the oracle."""
    knobs("MEC_BITSLICE", "2")
    cs, n = 2064, 2
    for k in sorted({1, max(1, (32 - m) // 2), 32 - m}):
        data = O.fill(n * k * cs, 7700 + 31 * m + k).reshape(n, k, cs)
        want = np.stack([np.stack(O.encode("rs", k, m, [data[s, j].copy() for j in range(k)], cs)) for s in range(n)])
        c = Codec("rs", k, m, cs)
        par = torch.zeros(n, m, cs, dtype=torch.uint8, device=DEV)
        c.encode(dev(data), par)
        assert np.array_equal(host(par), want), (k, m)
        base = O.fill(n * (k + m) * cs, 7800 + 31 * m + k).reshape(n, k + m, cs)
        rng = np.random.default_rng(31 * m + k)
        pat = sorted(rng.choice(k + m, size=min(m, 8), replace=False).tolist())
        t = dev(base.copy())
        c.decode(t, sum(1 << i for i in range(k + m) if i not in pat))
        got = host(t)
        for s in range(n):
            chunks = [base[s, i].copy() for i in range(k + m)]
            assert O.decode("rs", k, m, chunks, pat, cs) == 0
            for i in pat:
                assert np.array_equal(got[s, i], chunks[i]), (k, m, pat, s, i)
        st = c.stats()
        assert st["jit_failed"] == 0 and st["jit_launches"] >= 1 + int(len(pat) > 4), (k, m, st)
        c.close()


WIDE_ARMS = {"bitsliced": {"MEC_BITSLICE": "3"}, "one_pass": {"MEC_BITSLICE": "0"},
             "four_row": {"MEC_BITSLICE": "0", "MEC_WIDE": "0"}}


@pytest.mark.parametrize("arm", list(WIDE_ARMS))
def test_wide_fixtures_vs_reference(golden, arm, knobs):
    """every wide fixture recorded from the reference
    itself (tests/golden/make_golden.py wide_cases: Jerasure RS / Cauchy
    through MemEC's plugin, ISA-L RS / Cauchy through its USE_ISAL build) —
    m > 4 encodes, decodes of 5..8 erasures of random non-codeword stripes
    (which pin the survivor choice and the decoding matrix, not only the
    round trip), and the ISA-L RS pattern whose survivor matrix is singular —
    on each wide kernel: the run-time compiled bit-sliced kernel (forced for
    every wide launch), the one-pass kernel, and 4-row launches; strided
    in place and as a one-map device pointer batch."""
    from memec_amd import MecError, _lib
    for name, value in WIDE_ARMS[arm].items():
        knobs(name, value)
    meta, blobs = golden
    cases = [(n, c) for n, c in sorted(meta["cases"].items()) if c.get("wide") and c["kind"] != "encode_offsets_isal"]
    assert len(cases) >= 50
    jit0, bytewise_launches = {}, 0
    for name, c in cases:
        fam, k, m, cs, kind = c["family"], c["k"], c["m"], c["chunk"], c["kind"]
        codec = Codec(fam, k, m, cs)
        if kind == "encode":
            n = c["stripes"]
            data = dev(O.fill(n * k * cs, c["seed"]).reshape(n, k, cs))
            par = torch.zeros(n, m, cs, dtype=torch.uint8, device=DEV)
            codec.encode(data, par)
            assert np.array_equal(host(par).reshape(-1), blobs[name]), (arm, name)
            par2 = torch.zeros(n, m, cs, dtype=torch.uint8, device=DEV)
            codec.encode_batch([data[s, j].data_ptr() for s in range(n) for j in range(k)],
                               [par2[s, i].data_ptr() for s in range(n) for i in range(m)])
            assert np.array_equal(host(par2).reshape(-1), blobs[name]), (arm, "batch", name)
        else:
            buf = O.fill((k + m) * cs, c["seed"]).reshape(k + m, cs).copy()
            buf[c["erased"]] = 0
            present = sum(1 << i for i in range(k + m) if i not in c["erased"])
            chunks = dev(buf).view(1, k + m, cs).clone()
            chunks2 = chunks.clone()
            if kind == "decode_singular_isal":
                with pytest.raises(MecError) as ei:
                    codec.decode(chunks, present)
                assert ei.value.code == _lib.MEC_ESINGULAR, (arm, name)
                res = codec.decode_batch([chunks2[0, i].data_ptr() for i in range(k + m)], [present])
                assert res == [_lib.MEC_ESINGULAR], (arm, name, res)
                continue
            codec.decode(chunks, present)
            assert codec.decode_batch([chunks2[0, i].data_ptr() for i in range(k + m)], [present]) == [0]
            for form, t in (("strided", chunks), ("batch", chunks2)):
                got = host(t)[0]
                for i in range(k + m):
                    if i not in c["erased"]:
                        assert np.array_equal(got[i], buf[i]), (arm, form, name, "survivor", i)
                for r, e in enumerate(sorted(c["erased"])):
                    seg = slice(r * cs, (r + 1) * cs)
                    if kind == "decode_random":
                        assert np.array_equal(got[e], blobs[name][seg]), (arm, form, name, e)
                    else:  # ISA-L: the plugin's bytes for data, its own re-encode for parity
                        assert np.array_equal(got[e], blobs[name + "/fixed"][seg]), (arm, form, name, e)
                        if e < k:
                            assert np.array_equal(got[e], blobs[name][seg]), (arm, form, name, e)
        st = codec.stats()
        if fam != "cauchy" and cs % 16 == 0 and (kind == "encode" or len(c["erased"]) > 4):
            bytewise_launches += 1
            jit0[name] = st["jit_launches"]
        codec.close()
    assert bytewise_launches > 30
    if arm == "bitsliced":
        assert all(v > 0 for v in jit0.values()), [n for n, v in jit0.items() if v == 0][:5]
    else:
        assert all(v == 0 for v in jit0.values()), [n for n, v in jit0.items() if v][:5]


def test_wide_knob_off_turns_jit_off_everywhere(knobs):
    """MEC_WIDE=0 forces 4-row launches on the strided and
    zero-copy paths as on the pointer-batch path — even with the bit-sliced
    kernels forced on (MEC_BITSLICE=3), no launch runs one; results equal."""
    k, m, cs, n = 12, 8, 4096, 3
    data = O.fill(n * k * cs, 515).reshape(n, k, cs)
    want = [np.stack(O.encode("isal_rs", k, m, list(data[s]), cs)) for s in range(n)]
    knobs("MEC_BITSLICE", "3")
    knobs("MEC_WIDE", "0")
    c = Codec("isal_rs", k, m, cs)
    d = dev(data)
    par = torch.zeros(n, m, cs, dtype=torch.uint8, device=DEV)
    c.encode(d, par)
    par2 = torch.zeros(n, m, cs, dtype=torch.uint8, device=DEV)
    c.encode_batch([d[s, j].data_ptr() for s in range(n) for j in range(k)],
                   [par2[s, i].data_ptr() for s in range(n) for i in range(m)])
    got, got2 = host(par), host(par2)
    for s in range(n):
        assert np.array_equal(got[s], want[s]) and np.array_equal(got2[s], want[s]), s
    assert c.stats()["jit_launches"] == 0
    knobs("MEC_WIDE", None)
    c.encode(d, par)
    assert np.array_equal(host(par)[0], want[0])
    assert c.stats()["jit_launches"] >= 1


def test_jit_queue_bounded_and_destroy_cancels(knobs):
    """in the default async mode a decode workload that
    walks many erasure patterns queues at most MEC_JIT_MAX_QUEUED (16)
    compiles per context, every call stays exact on the one-pass kernel
    meanwhile, and mec_destroy cancels what is queued — it waits for the one
    compile already running (~1 s), not for the whole queue."""
    import itertools
    import time
    knobs("MEC_BITSLICE", None)
    k, m, cs, n = 16, 8, 4096, 2
    c = Codec("rs", k, m, cs)
    base = O.fill(n * (k + m) * cs, 616).reshape(n, k + m, cs)
    pats = list(itertools.islice(itertools.combinations(range(k + m), 6), 40))
    peak = 0
    for pat in pats[:40:4]:
        st = dev(base)
        st[:, list(pat)] = 0
        c.decode(st, sum(1 << i for i in range(k + m) if i not in pat))
        peak = max(peak, c.stats()["jit_pending"])
        if pat is pats[0]:
            got = host(st)
            for s in range(n):
                chunks = [base[s, i].copy() for i in range(k + m)]
                for e in pat:
                    chunks[e][:] = 0
                assert O.decode("rs", k, m, chunks, list(pat), cs) == 0
                assert all(np.array_equal(got[s, i], chunks[i]) for i in range(k + m))
    for pat in pats:
        st = dev(base)
        c.decode(st, sum(1 << i for i in range(k + m) if i not in pat))
        peak = max(peak, c.stats()["jit_pending"])
    assert peak <= 16, peak
    t0 = time.perf_counter()
    c.close()
    assert time.perf_counter() - t0 < 10.0
