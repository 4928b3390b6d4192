"""The oracle (oracle/oracle.c) against MemEC's own plugin (oracle/_ref,
compiled from the reference sources) over random code shapes — the pin that
lets the GPU sweeps (test_gpu_sweep.py) use the oracle as their checker
anywhere in the shape space, not only at the committed fixtures.

For each family, seeded random (k, m, chunk) with k + m <= 32
(rscoding.cc:26-29) and chunks that are multiples of 8 B: the oracle's
encode equals `Coding::encode` for every parity index, and its decode of a
random NON-codeword stripe (so the survivor choice and the `row_k_ones`
path show, jerasure.c:167-268) equals `Coding::decode` for a random pattern
of 1..m erasures; more than m erasures fail in both.  ISA-L: erased parity
as the plugin's own encode of the decoded data, and the
singular survivor matrices of ISA-L RS refused by both."""
import random

import numpy as np
import pytest

import _oracle as O
import _refplugin as R

pytestmark = pytest.mark.skipif(not R.available(), reason="oracle/_ref not built (make -C oracle ref)")

FAMS = ["rs", "cauchy", "isal_rs", "isal_cauchy"]


def shapes(fam, count, seed, max_units=64):
    rng = random.Random(seed)
    out = []
    while len(out) < count:
        n = rng.randint(2, 32)
        m = rng.randint(1, n - 1)
        k = n - m
        cs = 8 * rng.randint(1, max_units)
        if fam == "cauchy" and not 1 <= O.cauchy_getw(k, m, cs) <= 8:
            continue
        out.append((k, m, cs))
    return out


@pytest.mark.parametrize("fam", FAMS)
def test_random_shapes_oracle_equals_reference(fam):
    rng = random.Random(0xA11CE + FAMS.index(fam))
    singular = wide = 0
    for i, (k, m, cs) in enumerate(shapes(fam, 600, 0x5EA + FAMS.index(fam), 256)):
        seed = 1000 * FAMS.index(fam) + i
        data = O.fill(k * cs, seed).reshape(k, cs)
        want = R.encode(fam, k, m, cs, data)
        got = np.stack(O.encode(fam, k, m, [data[j].copy() for j in range(k)], cs))
        assert np.array_equal(got, want), ("encode", fam, k, m, cs)

        chunks = O.fill((k + m) * cs, seed + 7).reshape(k + m, cs)  # not a codeword
        e = rng.randint(1, m) if rng.random() < 0.9 else m + 1
        pat = sorted(rng.sample(range(k + m), min(e, k + m)))
        ok, ref = R.decode(fam, k, m, cs, chunks, pat)
        mine = [chunks[i].copy() for i in range(k + m)]
        for x in pat:
            mine[x][:] = 0
        rc = O.decode(fam, k, m, mine, pat, cs)
        if len(pat) > m:
            assert not ok and rc != 0, ("too many", fam, k, m, pat)
            continue
        if not ok:  # ISA-L RS: gf_gen_rs_matrix is not MDS for every shape
            assert fam == "isal_rs" and rc != 0, ("singular", fam, k, m, cs, pat)
            singular += 1
            continue
        assert rc == 0, ("oracle refused", fam, k, m, cs, pat)
        for x in range(k + m):
            assert np.array_equal(mine[x], ref[x]), ("decode", fam, k, m, cs, pat, x)
        wide += len(pat) > 4
    assert wide >= 100  # decodes of 5..31 erasures, where the engine runs its wide kernels
    if fam != "isal_rs":
        assert singular == 0
