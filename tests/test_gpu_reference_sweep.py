"""GPU against MemEC's own plugin (oracle/_ref, compiled from the reference
sources; tests/_refplugin.py) over random code shapes: no restatement in
between.  test_gpu_sweep.py checks the same space against the oracle, which
test_oracle_vs_reference.py pins to this plugin; here the engine's output is
compared with the plugin's directly, on random NON-codeword stripes, so the
survivor choice and the decoding matrix of every pattern show
(jerasure.c:167-268, cauchycoding.cc:87-180, rscoding.cc:155-177).

* every family, 400 seeded shapes with k + m <= 32 (rscoding.cc:26-29) and
  chunks of 8 B-16 KiB, the hand-written kernels (MEC_BITSLICE=0): encode of
  3 stripes; a delta update of one column (against the plugin's encode of
  that column alone); a strided in-place decode of one pattern; a device pointer
  batch with a different pattern per stripe (1..m erasures, data-only,
  parity-only and mixed, and one stripe with m + 1);
* the byte-wise families with the run-time compiled bit-sliced kernel forced
  for every wide launch (MEC_BITSLICE=3), 16 shapes with m > 4 each."""
import random

import numpy as np
import pytest

import _oracle as O
import _refplugin as R
from _mismatch import same

torch = pytest.importorskip("torch")
pytestmark = [pytest.mark.gpu,
              pytest.mark.skipif(not R.available(), reason="oracle/_ref not built (make -C oracle ref)")]

from memec_amd import Codec, MecError, _lib  # noqa: E402

DEV = "cuda:0"
FAMS = ["rs", "cauchy", "isal_rs", "isal_cauchy"]


@pytest.fixture(scope="module", autouse=True)
def _gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    torch.cuda.set_device(0)
    yield
    torch.cuda.synchronize()


def shapes(fam, count, seed, max_units, min_m=1, mult=8):
    rng = random.Random(seed)
    out = []
    while len(out) < count:
        n = rng.randint(max(2, min_m + 1), 32)
        m = rng.randint(min_m, n - 1)
        k = n - m
        cs = mult * rng.randint(1, max_units)
        if fam == "cauchy" and not 1 <= O.cauchy_getw(k, m, cs) <= 8:
            continue
        out.append((k, m, cs))
    return out


def host(t):
    torch.cuda.synchronize()
    return t.cpu().numpy()


def check_shape(fam, k, m, cs, seed, rng, n=3, batch=True):
    codec = Codec(fam, k, m, cs)
    # encode
    data = O.fill(n * k * cs, seed).reshape(n, k, cs)
    dd = torch.from_numpy(data.copy()).to(DEV)
    par = torch.zeros(n, m, cs, dtype=torch.uint8, device=DEV)
    codec.encode(dd, par)
    got = host(par)
    for s in range(n):
        same(got[s], R.encode(fam, k, m, cs, data[s]), ("encode", fam, k, m, cs, s))
    # strided in-place decode of one pattern, random non-codeword stripes
    stripes = O.fill(n * (k + m) * cs, seed + 1).reshape(n, k + m, cs)
    pat = sorted(rng.sample(range(k + m), rng.randint(1, m)))
    want = [R.decode(fam, k, m, cs, stripes[s], pat) for s in range(n)]
    t = torch.from_numpy(stripes.copy()).to(DEV)
    t[:, pat] = 0
    present = sum(1 << i for i in range(k + m) if i not in pat)
    if not want[0][0]:  # ISA-L RS: singular survivor matrix, the plugin's decode() is false
        assert fam == "isal_rs", (fam, k, m, cs, pat)
        with pytest.raises(MecError) as ei:
            codec.decode(t, present)
            torch.cuda.synchronize()
        assert ei.value.code == _lib.MEC_ESINGULAR
    else:
        codec.decode(t, present)
        out = host(t)
        for s in range(n):
            same(out[s], want[s][1], ("decode", fam, k, m, cs, pat, s))
    # delta update (the server's encode of one changed column, parity_chunk_buffer.cc:342-353):
    # parity ^= A[:, j] * delta, against the plugin's encode of a stripe whose only
    # non-zero column is the delta
    j = rng.randrange(k)
    delta = O.fill(n * cs, seed + 2).reshape(n, cs)
    before = O.fill(n * m * cs, seed + 3).reshape(n, m, cs)
    p = torch.from_numpy(before.copy()).to(DEV)
    codec.encode_update(j, torch.from_numpy(delta.copy()).to(DEV), p)
    after = host(p)
    for s in range(n):
        z = np.zeros((k, cs), np.uint8)
        z[j] = delta[s]
        same(after[s] ^ before[s], R.encode(fam, k, m, cs, z), ("update", fam, k, m, cs, j, s))
    if not batch:
        st = codec.stats()
        codec.close()
        return st
    # device pointer batch: a pattern per stripe, the last one beyond m
    pats = [sorted(rng.sample(range(k + m), rng.randint(1, m))) for _ in range(n - 1)]
    pats.append(sorted(rng.sample(range(k + m), m + 1)) if k + m > m + 1 else pats[-1])
    wants = [R.decode(fam, k, m, cs, stripes[s], pats[s]) for s in range(n)]
    t = torch.from_numpy(stripes.copy()).to(DEV)
    for s in range(n):
        t[s, pats[s]] = 0
    ptrs = [t[s, i].data_ptr() for s in range(n) for i in range(k + m)]
    masks = [sum(1 << i for i in range(k + m) if i not in pats[s]) for s in range(n)]
    res = codec.decode_batch(ptrs, masks, mem="device")
    out = host(t)
    for s in range(n):
        ok, w = wants[s]
        if len(pats[s]) > m:
            assert res[s] == _lib.MEC_ETOOMANY and not ok, (fam, k, m, pats[s], res[s])
        elif not ok:
            assert fam == "isal_rs" and res[s] == _lib.MEC_ESINGULAR, (fam, k, m, pats[s], res[s])
        else:
            assert res[s] == 0, (fam, k, m, cs, pats[s], res[s])
            same(out[s], w, ("batch decode", fam, k, m, cs, pats[s], s))
    st = codec.stats()
    codec.close()
    return st


@pytest.mark.parametrize("fam", FAMS)
def test_random_shapes_vs_reference_plugin(fam, knobs):
    knobs("MEC_BITSLICE", "0")
    rng = random.Random(0xBEEF + FAMS.index(fam))
    for i, (k, m, cs) in enumerate(shapes(fam, 400, 0xFACE + FAMS.index(fam), 2048)):
        assert check_shape(fam, k, m, cs, 50000 * (1 + FAMS.index(fam)) + 2 * i, rng)["jit_launches"] == 0


@pytest.mark.parametrize("fam", ["rs", "isal_rs", "isal_cauchy"])
def test_random_wide_shapes_bitsliced_vs_reference_plugin(fam, knobs):
    knobs("MEC_BITSLICE", "3")
    rng = random.Random(0xD00D + FAMS.index(fam))
    launches = 0
    for i, (k, m, cs) in enumerate(shapes(fam, 16, 0xC0FFEE + FAMS.index(fam), 384, min_m=5, mult=16)):
        st = check_shape(fam, k, m, cs, 90000 * (1 + FAMS.index(fam)) + 2 * i, rng, n=2, batch=False)
        assert st["jit_failed"] == 0, (fam, k, m, cs)
        launches += st["jit_launches"]
    assert launches >= 16  # every shape's encode at least ran on the bit-sliced kernel


# --------------------------------------------------------------------------- host memory

def _aligned(nbytes, align=4096):
    raw = np.empty(nbytes + align, np.uint8)
    off = (-raw.ctypes.data) % align
    return raw[off:off + nbytes]


HOST_ARMS = ["staged", "zerocopy", "queue"]


@pytest.mark.parametrize("arm", HOST_ARMS)
@pytest.mark.parametrize("fam", FAMS)
def test_random_shapes_host_paths_vs_reference_plugin(fam, arm):
    """The server's own calls on host chunks (include/mec.h mec_*_host, the
    host pointer batches) over a ChunkPool-like slab (slot = 8 + chunk,
    chunk_pool.cc:22-55), for 60 random shapes per family, against the
    plugin: `staged` (unregistered chunks through pinned staging), `zerocopy`
    (the slab registered, mec_host_register), `queue` (registered, the
    resident submission queue for single-stripe calls, mec_set_host_queue).
    Single-stripe encode, in-place decode of a random non-codeword stripe
    and delta update, then host pointer batches with a pattern per stripe."""
    import ctypes
    from memec_amd import host_register, host_unregister
    from memec_amd._lib import lib
    vp = ctypes.c_void_p
    queued = 0
    rng = random.Random(0xF00D + 7 * FAMS.index(fam) + HOST_ARMS.index(arm))
    for i, (k, m, cs) in enumerate(shapes(fam, 60, 0xAB + 11 * FAMS.index(fam) + HOST_ARMS.index(arm), 2048)):
        n, slot = 2, cs + 8
        slab = _aligned(n * (k + m) * slot)
        slab[:] = O.fill(slab.size, 70000 + i)
        seed = 80000 * (1 + FAMS.index(fam)) + 10 * i + HOST_ARMS.index(arm)

        def view(s, c):
            o = (s * (k + m) + c) * slot + 8
            return slab[o:o + cs]

        def addr(s, c):
            return slab.ctypes.data + (s * (k + m) + c) * slot + 8

        if arm != "staged":
            host_register(slab)
        try:
            codec = Codec(fam, k, m, cs)
            if arm == "queue":
                codec.set_host_queue(4)
            h = codec._h
            what = (arm, fam, k, m, cs)
            # single-stripe encode straight into the slab's parity slots
            data = np.stack([view(0, j).copy() for j in range(k)])
            dp = (vp * k)(*[vp(addr(0, j)) for j in range(k)])
            pp = (vp * m)(*[vp(addr(0, k + r)) for r in range(m)])
            assert lib().mec_encode_host(h, dp, pp) == 0, what
            want = R.encode(fam, k, m, cs, data)
            for r in range(m):
                same(view(0, k + r), want[r], ("encode_host",) + what + (r,))
            # in-place decode of a random non-codeword stripe
            for c in range(k + m):
                view(1, c)[:] = O.fill(cs, seed + c)
            stripe = np.stack([view(1, c).copy() for c in range(k + m)])
            pat = sorted(rng.sample(range(k + m), rng.randint(1, m)))
            ok, ref = R.decode(fam, k, m, cs, stripe, pat)
            for e in pat:
                view(1, e)[:] = 0
            cp = (vp * (k + m))(*[vp(addr(1, c)) for c in range(k + m)])
            present = sum(1 << c for c in range(k + m) if c not in pat)
            rc = lib().mec_decode_host(h, cp, ctypes.c_uint64(present))
            if not ok:
                assert fam == "isal_rs" and rc == _lib.MEC_ESINGULAR, what + (pat, rc)
            else:
                assert rc == 0, what + (pat, rc)
                for c in range(k + m):
                    same(view(1, c), ref[c], ("decode_host",) + what + (pat, c))
            # delta update of one column into stripe 0's parity slots
            j = rng.randrange(k)
            delta = _aligned(cs)
            delta[:] = O.fill(cs, seed + 99)
            if arm != "staged":
                host_register(delta)
            try:
                before = np.stack([view(0, k + r).copy() for r in range(m)])
                assert lib().mec_encode_update_host(h, j, vp(delta.ctypes.data), pp) == 0, what
            finally:
                if arm != "staged":
                    host_unregister(delta)
            z = np.zeros((k, cs), np.uint8)
            z[j] = delta
            dwant = R.encode(fam, k, m, cs, z)
            for r in range(m):
                same(view(0, k + r) ^ before[r], dwant[r], ("update_host",) + what + (j, r))
            # host pointer batches: encode both stripes, then a pattern per stripe
            for s in range(n):
                for c in range(k + m):
                    view(s, c)[:] = O.fill(cs, seed + 1000 * (s + 1) + c)
            datas = [np.stack([view(s, c).copy() for c in range(k)]) for s in range(n)]
            codec.encode_batch([addr(s, c) for s in range(n) for c in range(k)],
                               [addr(s, k + r) for s in range(n) for r in range(m)], mem="host")
            for s in range(n):
                w = R.encode(fam, k, m, cs, datas[s])
                for r in range(m):
                    same(view(s, k + r), w[r], ("encode_batch host",) + what + (s, r))
            stripes = [np.stack([view(s, c).copy() for c in range(k + m)]) ^ np.uint8(s + 1) for s in range(n)]
            pats = [sorted(rng.sample(range(k + m), rng.randint(1, m))) for _ in range(n)]
            wants = [R.decode(fam, k, m, cs, stripes[s], pats[s]) for s in range(n)]
            for s in range(n):
                for c in range(k + m):
                    view(s, c)[:] = 0 if c in pats[s] else stripes[s][c]
            res = codec.decode_batch([addr(s, c) for s in range(n) for c in range(k + m)],
                                     [sum(1 << c for c in range(k + m) if c not in pats[s]) for s in range(n)],
                                     mem="host")
            for s in range(n):
                ok, w = wants[s]
                if not ok:
                    assert fam == "isal_rs" and res[s] == _lib.MEC_ESINGULAR, what + (pats[s], res[s])
                    continue
                assert res[s] == 0, what + (pats[s], res[s])
                for c in range(k + m):
                    same(view(s, c), w[c], ("decode_batch host",) + what + (s, pats[s], c))
            st = codec.stats()
            if arm == "staged":
                assert st["zero_copy_calls"] == 0, st
            else:
                assert st["staged_calls"] == 0 and st["zero_copy_calls"] + st["queue_calls"] > 0, st
            queued += st["queue_calls"]
            codec.close()
        finally:
            if arm != "staged":
                host_unregister(slab)
    # the queue serves single-stripe calls of <= 4 outputs; wider ones launch
    assert (queued >= 20) if arm == "queue" else (queued == 0), queued
