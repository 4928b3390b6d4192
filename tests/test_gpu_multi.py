"""GPU parity of multi-GPU contexts (include/mec.h mec_create_multi): one
host process spreading its host-memory calls over several devices.  The
one-GPU test box lists cuda:0 several times (a device may repeat), which
exercises the stripe-range split, the concurrent shard execution, the
per-stripe decode results and the error reporting exactly as on 8 GPUs.
Bit-exact against the oracle."""
import numpy as np
import pytest

import _oracle as O
from _mismatch import same

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

from memec_amd import Codec, host_register, host_unregister  # noqa: E402
from memec_amd import _lib  # noqa: E402


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


@pytest.mark.parametrize("registered", [False, True])
@pytest.mark.parametrize("fam", ["rs", "cauchy"])
def test_multi_encode_decode_update_batches(fam, registered):
    k, m, cs, n = 6, 3, 4096, 37  # 37 stripes over 3 shards: ranges 12 / 12 / 13
    slot = cs + 8
    slab = aligned(n * (k + m) * slot)
    slab[:] = O.fill(slab.size, 9)
    if registered:
        host_register(slab)
    try:
        c = Codec(fam, k, m, cs, devices=[0, 0, 0])
        base = slab.ctypes.data

        def addr(s, i):
            return base + (s * (k + m) + i) * slot + 8

        def view(s, i):
            o = (s * (k + m) + i) * slot + 8
            return slab[o:o + cs]

        data = [[view(s, j).copy() for j in range(k)] for s in range(n)]
        c.encode_batch([addr(s, j) for s in range(n) for j in range(k)],
                       [addr(s, k + i) for s in range(n) for i in range(m)], mem="host")
        want = [O.encode(fam, k, m, data[s], cs) for s in range(n)]
        for s in range(n):
            for i in range(m):
                same(view(s, k + i), want[s][i], (s, i))
        # decode: a different pattern per stripe, including > m in two shards
        rng = np.random.default_rng(4)
        pats, masks = [], []
        for s in range(n):
            e = m + 1 if s in (5, 30) else int(rng.integers(0, m + 1))
            pat = sorted(rng.choice(k + m, size=e, replace=False).tolist())
            pats.append(pat)
            masks.append(sum(1 << i for i in range(k + m) if i not in pat))
        orig = [[view(s, i).copy() for i in range(k + m)] for s in range(n)]
        for s in range(n):
            if len(pats[s]) <= m:
                for e in pats[s]:
                    view(s, e)[:] = 0
        res = c.decode_batch([addr(s, i) for s in range(n) for i in range(k + m)], masks, mem="host")
        for s in range(n):
            if len(pats[s]) > m:
                assert res[s] == _lib.MEC_ETOOMANY, (s, res[s])
            else:
                assert res[s] == 0, (s, res[s])
            for i in range(k + m):
                same(view(s, i), orig[s][i], (s, pats[s], i))
        # delta update, mixed columns
        js = [int(rng.integers(0, k)) for _ in range(n)]
        deltas = aligned(n * cs).reshape(n, cs)
        deltas[:] = O.fill(n * cs, 77).reshape(n, cs)
        if registered:
            host_register(deltas)
        try:
            c.encode_update_batch(js, [deltas.ctypes.data + s * cs for s in range(n)],
                                  [addr(s, k + i) for s in range(n) for i in range(m)], mem="host")
        finally:
            if registered:
                host_unregister(deltas)
        for s in range(n):
            d2 = [x.copy() for x in data[s]]
            d2[js[s]] ^= deltas[s]
            w2 = O.encode(fam, k, m, d2, cs)
            for i in range(m):
                same(view(s, k + i), w2[i], (s, i))
        st = c.stats()
        if registered:
            assert st["zero_copy_calls"] >= 9 and st["staged_calls"] == 0  # 3 calls x 3 shards
        else:
            assert st["staged_calls"] >= 9
        c.close()
    finally:
        if registered:
            host_unregister(slab)


def test_multi_dense_batch_and_single_stripe_calls():
    k, m, cs, n = 10, 4, 65536, 10
    c = Codec("rs", k, m, cs, devices=[0, 0])
    d = O.fill(n * k * cs, 3).reshape(n, k, cs)
    p = np.zeros((n, m, cs), np.uint8)
    c.encode_host_batch(d, p)
    for s in range(n):
        same(p[s], np.stack(O.encode("rs", k, m, list(d[s]), cs)), s)
    # single-stripe calls alternate between the shards
    for s in range(4):
        got = c.encode_host(list(d[s]))
        for i in range(m):
            same(got[i], p[s, i], "")
    assert c.stats()["staged_calls"] >= 2 + 4
    # device-memory calls run on devices[0]
    dd = torch.from_numpy(d.copy()).to("cuda:0")
    pp = torch.zeros(n, m, cs, dtype=torch.uint8, device="cuda:0")
    c.encode(dd, pp)
    torch.cuda.synchronize()
    same(pp.cpu().numpy(), p, "")
    c.close()


def test_multi_bad_device_list():
    with pytest.raises(_lib.MecError):
        Codec("rs", 4, 2, 4096, devices=[])
    with pytest.raises(_lib.MecError):
        Codec("rs", 4, 2, 4096, devices=[0, 99])
