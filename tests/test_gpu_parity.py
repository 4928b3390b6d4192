"""GPU parity: libmec's HIP path vs the reference fixtures and the oracle.

Every comparison is bit-exact (integer/byte work).  Inputs come from the
splitmix64 stream, generated on the device by mec_fill_random and on the
host by the oracle, so both sides see the same bytes.  Sizes: fixture sizes,
plus BASELINE.json's full chunk sizes with fewer stripes, checked through
size-independent properties (encode -> erase -> decode round trips) and
per-stripe comparisons against the oracle.
"""
import hashlib
import itertools

import numpy as np
import pytest

import _oracle as O

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

from memec_amd import Codec, MecError, fill_random, xor  # noqa: E402
from memec_amd import _lib  # noqa: E402

DEV = "cuda:0"


@pytest.fixture(scope="module", autouse=True)
def _gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    torch.cuda.set_device(0)
    yield
    torch.cuda.synchronize()


def dev_fill(n_bytes, seed):
    t = torch.empty(n_bytes, dtype=torch.uint8, device=DEV)
    fill_random(t, seed)
    return t


def to_np(t):
    torch.cuda.synchronize()
    return t.cpu().numpy()


def encode_dense(fam, k, m, cs, n, seed, parity_mask=0):
    c = Codec(fam, k, m, cs)
    data = dev_fill(n * k * cs, seed).view(n, k, cs)
    par = torch.zeros(n, m, cs, dtype=torch.uint8, device=DEV)
    c.encode(data, par, parity_mask)
    return c, data, par


# --------------------------------------------------------------------------- fill


def test_fill_matches_oracle():
    for n, off in [(1000003, 0), (4096, 5), (17, 123456789)]:
        t = torch.empty(n, dtype=torch.uint8, device=DEV)
        fill_random(t, 0xABC, off)
        assert np.array_equal(to_np(t), O.fill(n, 0xABC, off))


# --------------------------------------------------------------------------- encode


@pytest.mark.parametrize("fam", ["rs", "cauchy", "isal_rs", "isal_cauchy"])
def test_encode_matches_reference_fixtures(golden, fam):
    meta, blobs = golden
    cases = [(n, c) for n, c in sorted(meta["cases"].items()) if c["kind"] == "encode" and c["family"] == fam]
    assert cases
    for name, c in cases:
        _, _, par = encode_dense(fam, c["k"], c["m"], c["chunk"], c["stripes"], c["seed"])
        assert np.array_equal(to_np(par).reshape(-1), blobs[name]), name


def test_encode_full_size_digests(golden):
    """BASELINE chunk sizes: RS(10,4)@1MiB, CRS(12,4)@64KiB (w=4, 16 KiB
    packets), RS(8,2)/RS(4,2)@4KiB, and an odd CRS size (65544 B)."""
    meta, _ = golden
    cases = [(n, c) for n, c in sorted(meta["cases"].items()) if c["kind"] == "encode_digest"]
    assert len(cases) >= 5
    for name, c in cases:
        _, _, par = encode_dense(c["family"], c["k"], c["m"], c["chunk"], c["stripes"], c["seed"])
        assert hashlib.sha256(to_np(par).tobytes()).hexdigest() == c["parity_sha256"], name


@pytest.mark.parametrize("fam", ["rs", "cauchy", "isal_rs", "isal_cauchy"])
def test_encode_matches_oracle_odd_sizes(fam):
    """Tail units (chunk or packet not a multiple of 16 B) and many shapes."""
    shapes = [(4, 2, 4104, 3), (3, 3, 24, 5), (5, 3, 40, 7), (12, 4, 520, 2), (7, 5, 8, 9),
              (1, 1, 64, 4), (31, 1, 96, 2), (16, 16, 48, 2), (20, 4, 320, 2), (20, 4, 112, 2), (2, 2, 4, 3)]
    for (k, m, cs, n) in shapes:
        if fam == "rs" and cs % 8:
            continue
        if fam == "cauchy" and (O.cauchy_getw(k, m, cs) < 1 or O.cauchy_getw(k, m, cs) > 8):
            continue
        seed = 1000 + k * 100 + m * 10 + cs
        _, _, par = encode_dense(fam, k, m, cs, n, seed)
        got = to_np(par)
        buf = O.fill(n * k * cs, seed)
        for s in range(n):
            want = O.encode(fam, k, m, [buf[(s * k + j) * cs:(s * k + j + 1) * cs].copy() for j in range(k)], cs)
            assert np.array_equal(got[s], np.stack(want)), (fam, k, m, cs, s)


@pytest.mark.parametrize("fam", ["rs", "cauchy"])
def test_parity_mask_and_strided_layout(fam):
    """Parity subsets (the plugin's encode(index)) and chunks inside a
    [stripe][k+m][slot] buffer with slot > chunk (ChunkPool-like strides)."""
    k, m, cs, n, slot = 10, 4, 4096, 8, 4096 + 256
    buf = torch.zeros(n, k + m, slot, dtype=torch.uint8, device=DEV)
    src = dev_fill(n * k * cs, 77).view(n, k, cs)
    buf[:, :k, :cs] = src
    c = Codec(fam, k, m, cs)
    data_view = buf[:, :k, :cs]
    par_view = buf[:, k:, :cs]
    c.encode(data_view, par_view)
    full = to_np(par_view).copy()
    ref = torch.zeros(n, m, cs, dtype=torch.uint8, device=DEV)
    c.encode(src, ref)
    assert np.array_equal(full, to_np(ref))
    for mask in [1, 2, 4, 8, 5, 0b1010]:
        out = torch.full((n, m, cs), 0xEE, dtype=torch.uint8, device=DEV)
        c.encode(src, out, mask)
        o = to_np(out)
        for i in range(m):
            if mask >> i & 1:
                assert np.array_equal(o[:, i], full[:, i]), (mask, i)
            else:
                assert (o[:, i] == 0xEE).all(), (mask, i)
    assert (to_np(buf[:, :, cs:]) == 0).all()  # slot padding untouched


# --------------------------------------------------------------------------- decode


def test_decode_matches_reference_fixtures(golden):
    """Random (non-codeword) stripes: pins the reference's exact survivor
    choice and decoding matrices (jerasure.c:167-268, 817-945)."""
    meta, blobs = golden
    cases = [(n, c) for n, c in sorted(meta["cases"].items()) if c["kind"] == "decode_random"]
    for name, c in cases:
        k, m, cs = c["k"], c["m"], c["chunk"]
        chunks = dev_fill((k + m) * cs, c["seed"]).view(1, k + m, cs).clone()
        for e in c["erased"]:
            chunks[0, e] = 0
        present = sum(1 << i for i in range(k + m) if i not in c["erased"])
        Codec(c["family"], k, m, cs).decode(chunks, present)
        got = to_np(chunks)[0]
        assert np.array_equal(np.concatenate([got[e] for e in sorted(c["erased"])]), blobs[name]), name
        # survivors untouched
        orig = O.fill((k + m) * cs, c["seed"]).reshape(k + m, cs)
        for i in range(k + m):
            if i not in c["erased"]:
                assert np.array_equal(got[i], orig[i]), (name, i)


def test_isal_decode_matches_reference_plugin(golden):
    """USE_ISAL decode vs the reference plugin itself (rscoding.cc /
    cauchycoding.cc built -DUSE_ISAL over ISA-L ec_base.c,
    oracle/ref_isal_plugin.cc): erased data chunks equal the reference's
    output; erased parity chunks equal the reference plugin's encode of the
    decoded data (`fixed`) — the reference's own output there reads past the
    k x k inverse into uninitialised stack."""
    meta, blobs = golden
    cases = [(n, c) for n, c in sorted(meta["cases"].items()) if c["kind"] == "decode_random_isal"]
    assert len(cases) >= 60
    for name, c in cases:
        k, m, cs = c["k"], c["m"], c["chunk"]
        chunks = dev_fill((k + m) * cs, c["seed"]).view(1, k + m, cs).clone()
        for e in c["erased"]:
            chunks[0, e] = 0
        present = sum(1 << i for i in range(k + m) if i not in c["erased"])
        Codec(c["family"], k, m, cs).decode(chunks, present)
        got = to_np(chunks)[0]
        ref, fixed = blobs[name], blobs[name + "/fixed"]
        for r, e in enumerate(sorted(c["erased"])):
            assert np.array_equal(got[e], fixed[r * cs:(r + 1) * cs]), (name, e)
            if e < k:
                assert np.array_equal(got[e], ref[r * cs:(r + 1) * cs]), (name, e)
        orig = O.fill((k + m) * cs, c["seed"]).reshape(k + m, cs)
        for i in range(k + m):
            if i not in c["erased"]:
                assert np.array_equal(got[i], orig[i]), (name, i)


@pytest.mark.parametrize("fam", ["rs", "cauchy", "isal_rs", "isal_cauchy"])
def test_decode_every_pattern_vs_oracle(fam):
    """Every erasure pattern of size 1..m for (6,3), random stripes, against
    the oracle (parity-only, data-only and mixed patterns)."""
    k, m, cs, n = 6, 3, 256, 3
    c = Codec(fam, k, m, cs)
    base = O.fill(n * (k + m) * cs, 4242).reshape(n, k + m, cs)
    for e in range(1, m + 1):
        for pat in itertools.combinations(range(k + m), e):
            t = torch.from_numpy(base.copy()).to(DEV)
            t[:, list(pat)] = 0
            present = sum(1 << i for i in range(k + m) if i not in pat)
            c.decode(t, present)
            got = to_np(t)
            for s in range(n):
                chunks = [base[s, i].copy() for i in range(k + m)]
                assert O.decode(fam, k, m, chunks, list(pat), cs) == 0
                for i in range(k + m):
                    assert np.array_equal(got[s, i], chunks[i]), (fam, pat, s, i)


@pytest.mark.parametrize("fam,k,m,cs,n,pats", [
    ("rs", 10, 4, 1 << 20, 16, [[0, 1, 2, 3], [0, 5, 10, 13], [10, 11, 12, 13], [4]]),
    ("cauchy", 12, 4, 65536, 64, [[0, 1, 2, 3], [0, 5, 12, 15], [13]]),
    ("rs", 8, 2, 4096, 2048, [[0, 1], [3, 9]]),
    ("rs", 4, 2, 4096, 512, [[0, 1], [4, 5], [1]]),
])
def test_roundtrip_baseline_sizes(fam, k, m, cs, n, pats):
    c, data, par = encode_dense(fam, k, m, cs, n, 31337 + k)
    # spot-check two stripes against the oracle
    d = to_np(data)
    p = to_np(par)
    for s in (0, n - 1):
        want = O.encode(fam, k, m, [d[s, j].copy() for j in range(k)], cs)
        assert np.array_equal(p[s], np.stack(want)), s
    stripe = torch.cat([data, par], dim=1)
    for pat in pats:
        t = stripe.clone()
        t[:, pat] = 0
        present = sum(1 << i for i in range(k + m) if i not in pat)
        c.decode(t, present)
        torch.cuda.synchronize()
        assert torch.equal(t, stripe), pat


def test_decode_split_and_too_many():
    k, m, cs, n = 10, 4, 4096, 32
    c, data, par = encode_dense("rs", k, m, cs, n, 5)
    stripe = torch.cat([data, par], dim=1)
    out = torch.zeros_like(stripe)
    present = (1 << (k + m)) - 1 - 0b1111
    c.decode_split(stripe, out, present)
    torch.cuda.synchronize()
    assert torch.equal(out[:, :4], stripe[:, :4])
    assert (to_np(out[:, 4:]) == 0).all()
    with pytest.raises(MecError) as e:
        c.decode(stripe.clone(), present & ~(1 << 5))
    assert e.value.code == _lib.MEC_ETOOMANY
    c.decode(stripe, (1 << (k + m)) - 1)  # nothing missing: no-op


# --------------------------------------------------------------------------- delta / update


def test_delta_matches_reference_fixtures(golden):
    meta, blobs = golden
    for name, c in sorted(meta["cases"].items()):
        if c["kind"] != "delta":
            continue
        k, m, cs, col, idx = c["k"], c["m"], c["chunk"], c["column"], c["index"]
        data = torch.from_numpy(O.fill(k * cs, c["seed"]).reshape(1, k, cs)).to(DEV)
        codec = Codec(c["family"], k, m, cs)
        # (a) the plugin's form: every other column is Coding::zeros
        z = torch.zeros_like(data)
        z[:, col] = data[:, col]
        par = torch.zeros(1, m, cs, dtype=torch.uint8, device=DEV)
        codec.encode(z, par, 1 << (idx - 1))
        assert np.array_equal(to_np(par)[0, idx - 1], blobs[name]), name
        # (b) the batched delta kernel: parity ^= A[:,col] * delta on zero parity
        par2 = torch.zeros(1, m, cs, dtype=torch.uint8, device=DEV)
        codec.encode_update(col, data[:, col].contiguous(), par2)
        assert np.array_equal(to_np(par2)[0, idx - 1], blobs[name]), name


def test_isal_update_matches_reference_fixtures(golden):
    meta, blobs = golden
    for name, c in sorted(meta["cases"].items()):
        if c["kind"] != "update":
            continue
        k, m, cs, col = c["k"], c["m"], c["chunk"], c["column"]
        base = blobs["enc/%s/%d_%d_%d_x1" % (c["family"], k, m, cs)].reshape(1, m, cs)
        par = torch.from_numpy(base.copy()).to(DEV)
        delta = torch.from_numpy(O.fill(cs, c["delta_seed"]).reshape(1, cs)).to(DEV)
        Codec(c["family"], k, m, cs).encode_update(col, delta, par)
        assert np.array_equal(to_np(par).reshape(-1), blobs[name]), name


@pytest.mark.parametrize("fam", ["rs", "cauchy"])
def test_update_linearity_batch(fam):
    """encode(D ^ delta_j) == encode(D) ^ update_j(delta): the server's SEAL /
    UPDATE identity (parity_chunk_buffer.cc:340-415), batched."""
    k, m, cs, n, j = 8, 3, 8192, 64, 5
    c, data, par = encode_dense(fam, k, m, cs, n, 9)
    delta = dev_fill(n * cs, 10).view(n, cs)
    data2 = data.clone()
    data2[:, j] ^= delta
    par2 = torch.zeros_like(par)
    c.encode(data2, par2)
    c.encode_update(j, delta, par)
    torch.cuda.synchronize()
    assert torch.equal(par, par2)


# --------------------------------------------------------------------------- host entry points


@pytest.mark.parametrize("fam", ["rs", "cauchy", "isal_rs"])
def test_host_entry_points(fam):
    k, m, cs = 10, 4, 65536
    c = Codec(fam, k, m, cs)
    buf = O.fill(k * cs, 123)
    data = [buf[j * cs:(j + 1) * cs].copy() for j in range(k)]
    want = O.encode(fam, k, m, data, cs)
    got = c.encode_host(data)
    for i in range(m):
        assert np.array_equal(got[i], want[i]), i
    # zero sentinel columns + a single wanted parity (delta encode form)
    zdata = [None] * k
    zdata[3] = data[3]
    got = c.encode_host(zdata, want=[False, False, True, False])
    zref = O.encode(fam, k, m, [d if d is not None else np.zeros(cs, np.uint8) for d in zdata], cs)
    assert got[0] is None and np.array_equal(got[2], zref[2])
    # decode on host chunks
    chunks = data + [w.copy() for w in want]
    orig = [x.copy() for x in chunks]
    for pat in ([0, 1, 2, 3], [0, 5, 10, 13], [11]):
        for e in pat:
            chunks[e][:] = 0
        c.decode_host(chunks, sum(1 << i for i in range(k + m) if i not in pat))
        for i in range(k + m):
            assert np.array_equal(chunks[i], orig[i]), (pat, i)
    # update on host
    delta = O.fill(cs, 321)
    par = [w.copy() for w in want]
    c.encode_update_host(2, delta, par)
    data2 = [d.copy() for d in data]
    data2[2] ^= delta
    want2 = O.encode(fam, k, m, data2, cs)
    for i in range(m):
        assert np.array_equal(par[i], want2[i]), i


def test_host_batch_encode():
    k, m, cs, n = 10, 4, 1 << 20, 24
    c = Codec("rs", k, m, cs)
    data = O.fill(n * k * cs, 55).reshape(n, k, cs)
    par = np.zeros((n, m, cs), np.uint8)
    c.encode_host_batch(data, par)
    ddev = torch.from_numpy(data).to(DEV)
    pdev = torch.zeros(n, m, cs, dtype=torch.uint8, device=DEV)
    c.encode(ddev, pdev)
    assert np.array_equal(par, to_np(pdev))


def test_xor():
    # partial 16-byte units, partial one-wave tiles (1 KiB), aligned sizes
    for n in [1, 15, 16, 1023, 1025, 1040, 4097, (1 << 20) + 7, 1 << 20]:
        a, b = dev_fill(n, 1), dev_fill(n, 2)
        d = torch.empty_like(a)
        xor(d, a, b)
        assert np.array_equal(to_np(d), O.fill(n, 1) ^ O.fill(n, 2)), n
    # dst aliasing a source (parity ^= delta, Coding::bitwiseXOR's use)
    a, b = dev_fill(5000, 3), dev_fill(5000, 4)
    xor(a, a, b)
    assert np.array_equal(to_np(a), O.fill(5000, 3) ^ O.fill(5000, 4))


@pytest.mark.parametrize("k,m,cs,layout", [(10, 4, 65536, "split"), (4, 2, 4096, "inplace"), (3, 1, 4096 + 16, "split")])
def test_xor_twin_probe(k, m, cs, layout):
    """mec_set_probe(MEC_PROBE_XOR): the same launches with every product a
    plain XOR (the bench's live ceiling) — each output is the XOR of the
    launch's sources; switching it off codes again, bit-exact."""
    n = 5
    c = Codec("rs", k, m, cs)
    data = torch.empty(n, k, cs, dtype=torch.uint8, device="cuda")
    from memec_amd import fill_random
    fill_random(data, 31 + k)
    host = data.cpu().numpy()
    x = np.bitwise_xor.reduce(host, axis=1)
    if layout == "split":
        par = torch.zeros(n, m, cs, dtype=torch.uint8, device="cuda")
        c.set_probe(True)
        c.encode(data, par)
        c.set_probe(False)
        torch.cuda.synchronize()
        got = par.cpu().numpy()
        full = cs // 16 * 16  # the < 16-byte tail is always coded (tail kernel)
        for i in range(m):
            assert np.array_equal(got[:, i, :full], x[:, :full])
        c.encode(data, par)
        torch.cuda.synchronize()
        got = par.cpu().numpy()
        for s_ in (0, n - 1):
            assert np.array_equal(got[s_], np.stack(O.encode("rs", k, m, [host[s_, j].copy() for j in range(k)], cs)))
    else:
        st = torch.zeros(n, k + m, cs, dtype=torch.uint8, device="cuda")
        st[:, :k] = data
        c.encode(st[:, :k], st[:, k:])
        want = st.clone()
        st[:, [0, 1]] = 0
        present = sum(1 << i for i in range(2, k + m))
        c.set_probe(True)
        c.decode(st, present)
        torch.cuda.synchronize()
        sv = want.cpu().numpy()[:, 2:2 + k]  # the decode plan reads the first k survivors
        xs = np.bitwise_xor.reduce(sv, axis=1)
        got = st.cpu().numpy()
        assert np.array_equal(got[:, 0], xs) and np.array_equal(got[:, 1], xs)
        c.set_probe(False)
        c.decode(st, present)
        torch.cuda.synchronize()
        assert torch.equal(st, want)
    c.close()


def test_xor_twin_probe_refuses_bitmatrix():
    c = Codec("cauchy", 4, 2, 4096)
    with pytest.raises(MecError):
        c.set_probe(True)
    c.close()


def test_xor_grid_stride_past_16_gib():
    """Past 2^24 one-wave tiles (16 GiB) the launch strides its grid; the
    tail tile is partial too."""
    n = (16 << 30) + 4096 + 3
    a, b = dev_fill(n, 5), dev_fill(n, 6)
    d = torch.empty_like(a)
    xor(d, a, b)
    torch.bitwise_xor(a, b, out=a)
    assert torch.equal(d, a)
    del a, b, d
    torch.cuda.empty_cache()
