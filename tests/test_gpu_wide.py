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
