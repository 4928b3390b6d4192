"""GPU geometry sweep: a seeded sample of (k, m, chunk size) over every code
family, k + m <= 32 (the reference's limit, rscoding.cc:26-29), each encoded
on the device and compared bit-exact with the oracle, then decoded after a
random erasure pattern of 1..m chunks (data-only, parity-only or mixed) and
compared with the oracle's decode of the same pattern.

The fixed cases in test_gpu_parity.py pin the BASELINE shapes; this sweep
covers the row-group splits of the kernels (m > 4 parities, decode of > 4
erasures, k up to 31) and chunk sizes that are not multiples of 16 B.
"""
import os
import random

import numpy as np
import pytest

import _oracle as O

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

from memec_amd import Codec, MecError, fill_random  # noqa: E402

DEV = "cuda:0"
FAMS = ["rs", "cauchy", "isal_rs", "isal_cauchy"]


@pytest.fixture(scope="module", autouse=True)
def _gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    torch.cuda.set_device(0)
    yield
    torch.cuda.synchronize()


def _shapes(fam, count, seed, max_units=96):
    rng = random.Random(seed)
    out = []
    while len(out) < count:
        n_total = rng.randint(2, 32)
        m = rng.randint(1, n_total - 1)
        k = n_total - m
        cs = 8 * rng.randint(1, max_units)  # 8 .. 768 B by default: tails below 16 B included
        if fam == "cauchy":
            w = O.cauchy_getw(k, m, cs)
            if w < 1 or w > 8:
                continue
        out.append((k, m, cs))
    return out


@pytest.mark.parametrize("fam", FAMS)
def test_geometry_sweep_vs_oracle(fam):
    _sweep(fam, _shapes(fam, 40, 0xC0DE + FAMS.index(fam)), random.Random(0x5EED + FAMS.index(fam)), 2)


@pytest.mark.parametrize("fam", FAMS)
def test_geometry_sweep_extended(fam):
    """The same check over 1000 shapes per family (MEC_SWEEP_EXTENDED=<n>
    for more; 3000 in profiles/r04/parity/sweep_extended_3000.log) with
    chunks of 8 B-64 KiB: every launch shape the rules pick (one-wave /
    4-wave blocks, 8- / 16-byte bitmatrix lanes, the tiny in-place rule,
    tails, one-pass wide codes with groups of 3, 4 and 8 rows), another
    seed.  ~15 s per family on the MI355X."""
    count = int(os.environ.get("MEC_SWEEP_EXTENDED") or 1000)
    _sweep(fam, _shapes(fam, count, 0xE77 + FAMS.index(fam), max_units=8192), random.Random(0xE5 + FAMS.index(fam)), 3)


def _sweep(fam, shapes, rng, n):
    for (k, m, cs) in shapes:
        seed = rng.getrandbits(40)
        c = Codec(fam, k, m, cs)
        data = torch.empty(n * k * cs, dtype=torch.uint8, device=DEV)
        fill_random(data, seed)
        data = data.view(n, k, cs)
        par = torch.zeros(n, m, cs, dtype=torch.uint8, device=DEV)
        c.encode(data, par)
        torch.cuda.synchronize()
        got = par.cpu().numpy()
        host = O.fill(n * k * cs, seed).reshape(n, k, cs)
        assert np.array_equal(data.cpu().numpy(), host)
        want = [np.stack(O.encode(fam, k, m, [host[s, j].copy() for j in range(k)], cs)) for s in range(n)]
        for s in range(n):
            assert np.array_equal(got[s], want[s]), (fam, k, m, cs, s)

        # decode one random pattern of 1..m erasures
        e = rng.randint(1, m)
        pat = sorted(rng.sample(range(k + m), e))
        base = np.concatenate([host, np.stack(want)], axis=1)  # [n, k+m, cs]
        ref = [[base[s, i].copy() for i in range(k + m)] for s in range(n)]
        for s in range(n):
            for i in pat:
                ref[s][i][:] = 0
        rcs = [O.decode(fam, k, m, ref[s], pat, cs) for s in range(n)]
        t = torch.from_numpy(base.copy()).to(DEV)
        t[:, pat] = 0
        present = sum(1 << i for i in range(k + m) if i not in pat)
        if any(rcs):  # singular decoding matrix (ISA-L's non-MDS RS shapes): the call must fail
            with pytest.raises(MecError):
                c.decode(t, present)
                torch.cuda.synchronize()
            continue
        c.decode(t, present)
        torch.cuda.synchronize()
        out = t.cpu().numpy()
        for s in range(n):
            for i in range(k + m):
                assert np.array_equal(out[s, i], ref[s][i]), (fam, k, m, cs, pat, s, i)
                assert np.array_equal(out[s, i], base[s, i]), (fam, k, m, cs, pat, s, i)
