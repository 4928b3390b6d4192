"""GPU parity at BASELINE.json's full sizes (and MemEC's largest chunk), by
size-independent properties: sampled stripes equal the oracle (scattered
across the batch), the decode round trip restores every erased chunk of
every stripe, and the checksum of per-stripe checksums matches between the
full batch and the same stripes coded in small pieces.

  configs[1]  RS(10,4) encode, 1 MiB chunks, 4096 stripes     (56 GiB in HBM)
  configs[2]  RS(10,4) decode with 4 erasures, same batch
  configs[3]  RS(8,2) encode, 4 KiB chunks, 65536 stripes
  configs[4]  Cauchy-RS(12,4) encode + decode, 64 KiB chunks, 32768 stripes
              (the 8-GPU global batch, here on one GPU: 32 GiB)
  [size] chunk upper bound 16 MiB (global_config.cc:177-184)
"""
import numpy as np
import pytest

import _oracle as O

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

from memec_amd import Codec, fill_random  # noqa: E402

DEV = "cuda:0"


@pytest.fixture(autouse=True)
def _gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    torch.cuda.set_device(0)
    yield
    torch.cuda.synchronize()
    torch.cuda.empty_cache()


def _sample_matches_oracle(fam, k, m, cs, stripe, idx):
    """stripe: [n][k+m][cs] device tensor with parity in [:, k:]."""
    sub = stripe[idx].cpu().numpy()
    data = np.ascontiguousarray(sub[:, :k]).reshape(-1)
    par = np.zeros(len(idx) * m * cs, np.uint8)
    assert O.encode_batch_mt(fam, k, m, cs, data, par, len(idx), min(8, len(idx))) == 0
    return np.array_equal(par.reshape(len(idx), m, cs), sub[:, k:])


def _roundtrip(codec, stripe, k, m, pats):
    for pat in pats:
        saved = stripe[:, pat].clone()
        stripe[:, pat] = 0
        codec.decode(stripe, sum(1 << i for i in range(k + m) if i not in pat))
        torch.cuda.synchronize()
        assert torch.equal(stripe[:, pat], saved), pat
        del saved


def _spread(n, count=8):
    return sorted({0, n - 1} | {int(x) for x in np.linspace(0, n - 1, count)})


def test_rs104_1mib_4096_stripes():
    k, m, cs, n = 10, 4, 1 << 20, 4096
    c = Codec("rs", k, m, cs)
    stripe = torch.empty(n, k + m, cs, dtype=torch.uint8, device=DEV)
    fill_random(stripe, 0x4D454D4543)
    c.encode(stripe[:, :k], stripe[:, k:])  # in-place layout (2-window block order)
    assert _sample_matches_oracle("rs", k, m, cs, stripe, _spread(n))
    # checksum of checksums: the same stripes encoded 512 at a time into a
    # separate (split-layout) parity buffer give identical parity
    par = torch.empty(512, m, cs, dtype=torch.uint8, device=DEV)
    for s0 in range(0, n, 512):
        c.encode(stripe[s0:s0 + 512, :k], par)
        assert torch.equal(par, stripe[s0:s0 + 512, k:]), s0
    del par
    _roundtrip(c, stripe, k, m, [[0, 1, 2, 3], [0, 5, 10, 13], [10, 11, 12, 13]])
    del stripe


def test_rs82_4kib_65536_stripes():
    k, m, cs, n = 8, 2, 4096, 65536
    c = Codec("rs", k, m, cs)
    stripe = torch.empty(n, k + m, cs, dtype=torch.uint8, device=DEV)
    fill_random(stripe, 82)
    c.encode(stripe[:, :k], stripe[:, k:])
    assert _sample_matches_oracle("rs", k, m, cs, stripe, _spread(n, 64))
    _roundtrip(c, stripe, k, m, [[0, 1], [3, 9], [8, 9]])


def test_crs124_64kib_32768_stripes():
    k, m, cs, n = 12, 4, 65536, 32768
    c = Codec("cauchy", k, m, cs)
    assert c.w == 4 and c.packet_size == 16384
    stripe = torch.empty(n, k + m, cs, dtype=torch.uint8, device=DEV)
    fill_random(stripe, 124)
    c.encode(stripe[:, :k], stripe[:, k:])
    assert _sample_matches_oracle("cauchy", k, m, cs, stripe, _spread(n, 16))
    _roundtrip(c, stripe, k, m, [[0, 1, 2, 3], [0, 5, 12, 15], [13]])


@pytest.mark.parametrize("fam", ["rs", "cauchy"])
def test_largest_chunk_16mib(fam):
    k, m, cs, n = (10, 4, 16 << 20, 3) if fam == "rs" else (12, 4, 16 << 20, 2)
    c = Codec(fam, k, m, cs)
    stripe = torch.empty(n, k + m, cs, dtype=torch.uint8, device=DEV)
    fill_random(stripe, 16)
    c.encode(stripe[:, :k], stripe[:, k:])
    assert _sample_matches_oracle(fam, k, m, cs, stripe, list(range(n)))
    _roundtrip(c, stripe, k, m, [[0, 1, 2, 3], [2, k + 1]])
