"""Pin the CPU restatement (oracle/) against the reference's own outputs.

Every expected value here was produced by the compiled reference
(tests/golden/make_golden.py over oracle/_ref/libmemec_ref.so).  These tests
run on CPU only and gate every GPU parity claim: the GPU path is checked
against this oracle and against the same fixtures.
"""
import hashlib
import os

import numpy as np
import pytest

import _oracle as O


def _data_chunks(n, k, cs, seed):
    buf = O.fill(n * k * cs, seed)
    return [[buf[(s * k + j) * cs:(s * k + j + 1) * cs].copy() for j in range(k)] for s in range(n)]


def test_gf_fields(golden):
    meta, _ = golden
    L = O.lib()
    for w in range(1, 9):
        g = meta["gf"][str(w)]
        n = 1 << w
        tab = np.array([[L.orc_gf_mul(a, b, w) for b in range(n)] for a in range(n)], np.int32)
        assert hashlib.sha256(tab.tobytes()).hexdigest() == g["mul_table_sha256_int32"], w
        assert [L.orc_gf_div(1, a, w) for a in range(1, n)] == g["inverses"], w


def test_rs_matrices(golden):
    meta, _ = golden
    for key, mat in meta["rs_matrices"].items():
        k, m = map(int, key.split(","))
        assert O.rs_matrix(k, m) == mat, key


def test_cbest_is_ones_then_value_order(golden):
    meta, _ = golden
    L = O.lib()
    for w in range(2, 9):
        derived = sorted(range(1, 1 << w), key=lambda c: (L.orc_cauchy_n_ones(c, w), c))
        assert derived == meta["cbest"][str(w)], w


def test_cauchy_matrices_bitmatrices_schedules(golden):
    meta, _ = golden
    for key, rec in meta["cauchy_matrices"].items():
        k, m, w = map(int, key.split(","))
        mat = O.cauchy_matrix(k, m, w)
        assert mat == rec["matrix"], key
        if k * m * w * w > 4096:
            continue  # keep the CPU suite quick; matrix equality implies the rest
        bm = O.bitmatrix(k, m, w, mat)
        assert sum(bm) == rec["bitmatrix_ones"], key
        ops, n = O.smart_schedule(k, m, w, bm)
        assert n == rec["schedule_ops"], key
        assert hashlib.sha256(np.array(ops, np.int32).tobytes()).hexdigest() == rec["schedule_sha256_int32"], key


def _encode_cases(meta, kind):
    return [(n, c) for n, c in sorted(meta["cases"].items()) if c["kind"] == kind]


@pytest.mark.parametrize("fam", ["rs", "cauchy", "isal_rs", "isal_cauchy"])
def test_encode_small(golden, fam):
    meta, blobs = golden
    cases = [(n, c) for n, c in _encode_cases(meta, "encode") if c["family"] == fam]
    assert cases
    for name, c in cases:
        k, m, cs, ns = c["k"], c["m"], c["chunk"], c["stripes"]
        got = []
        for stripe in _data_chunks(ns, k, cs, c["seed"]):
            got.extend(O.encode(fam, k, m, stripe, cs))
        assert np.array_equal(np.concatenate(got), blobs[name]), name


def test_encode_full_size_digests(golden):
    meta, _ = golden
    for name, c in _encode_cases(meta, "encode_digest"):
        k, m, cs, ns = c["k"], c["m"], c["chunk"], c["stripes"]
        got = []
        for stripe in _data_chunks(ns, k, cs, c["seed"]):
            got.extend(O.encode(c["family"], k, m, stripe, cs))
        assert hashlib.sha256(np.concatenate(got).tobytes()).hexdigest() == c["parity_sha256"], name


def test_decode_random_stripes(golden):
    """Decode of non-codeword stripes pins the survivor choice, the
    row_k_ones shortcut (jerasure.c:204-253) and the schedule-decode matrix
    (jerasure.c:817-945), not just uniqueness."""
    meta, blobs = golden
    cases = _encode_cases(meta, "decode_random")
    assert len(cases) > 30
    for name, c in cases:
        k, m, cs = c["k"], c["m"], c["chunk"]
        buf = O.fill((k + m) * cs, c["seed"])
        chunks = [buf[i * cs:(i + 1) * cs].copy() for i in range(k + m)]
        rc = O.decode(c["family"], k, m, chunks, c["erased"], cs)
        assert rc == 0 == c["rc"], name
        got = np.concatenate([chunks[e] for e in sorted(c["erased"])])
        assert np.array_equal(got, blobs[name]), name


def test_decode_too_many_erasures(golden):
    meta, _ = golden
    c = meta["cases"]["dec/rs/4_2_64/0-1-2"]
    assert c["rc"] == -1
    chunks = [np.zeros(64, np.uint8) for _ in range(6)]
    assert O.decode("rs", 4, 2, chunks, [0, 1, 2], 64) == -1


def test_delta_encode(golden):
    meta, blobs = golden
    for name, c in _encode_cases(meta, "delta"):
        k, m, cs = c["k"], c["m"], c["chunk"]
        data = O.fill(k * cs, c["seed"])
        chunks = [np.zeros(cs, np.uint8) for _ in range(k)]
        chunks[c["column"]] = data[c["column"] * cs:(c["column"] + 1) * cs].copy()
        par = O.encode(c["family"], k, m, chunks, cs)
        assert np.array_equal(par[c["index"] - 1], blobs[name]), name


def test_isal_matrices_and_update(golden):
    meta, blobs = golden
    for key, mat in meta["isal_matrices"].items():
        fam, km = key.split("/")
        k, m = map(int, km.split(","))
        assert O.isal_matrix(fam, k, m).tolist() == mat, key
    for name, c in _encode_cases(meta, "update"):
        k, m, cs, col = c["k"], c["m"], c["chunk"], c["column"]
        base = blobs["enc/%s/%d_%d_%d_x1" % (c["family"], k, m, cs)].copy()
        delta = O.fill(cs, c["delta_seed"])
        enc = O.isal_matrix(c["family"], k, m)
        coef = np.ascontiguousarray(enc[k * k:])
        dst = [base[i * cs:(i + 1) * cs] for i in range(m)]
        O.lib().orc_isal_encode_update(cs, k, m, col, O.ptr(coef), O.ptr(delta), O._ptrs(dst))
        assert np.array_equal(base, blobs[name]), name


def test_isal_plugin_decode_fixtures(golden):
    """USE_ISAL decode, pinned on the reference plugin itself (MemEC's
    rscoding.cc / cauchycoding.cc built -DUSE_ISAL over ISA-L's ec_base.c,
    oracle/ref_isal_plugin.cc): every erased DATA chunk equals the
    reference's output bit for bit; for an erased PARITY chunk the reference
    reads rows of the k x k inverse past k (uninitialised stack,
    rscoding.cc:173-175; its output there is undefined and the generator
    recorded it differing from `fixed` in every case), and the oracle equals
    `fixed`, the reference plugin's own encode of the decoded data."""
    meta, blobs = golden
    cases = _encode_cases(meta, "decode_random_isal")
    assert len(cases) >= 60
    n_parity = 0
    for name, c in cases:
        k, m, cs = c["k"], c["m"], c["chunk"]
        assert c["rc"] == 1, name
        buf = O.fill((k + m) * cs, c["seed"])
        chunks = [buf[i * cs:(i + 1) * cs].copy() for i in range(k + m)]
        assert O.decode(c["family"], k, m, chunks, c["erased"], cs) == 0, name
        ref, fixed = blobs[name], blobs[name + "/fixed"]
        parity_erased = [e for e in sorted(c["erased"]) if e >= k]
        assert c["reference_parity_defect"] == [True] * len(parity_erased), name
        for r, e in enumerate(sorted(c["erased"])):
            got = chunks[e]
            assert np.array_equal(got, fixed[r * cs:(r + 1) * cs]), (name, e)
            if e < k:
                assert np.array_equal(got, ref[r * cs:(r + 1) * cs]), (name, e)
            else:
                n_parity += 1
    assert n_parity > 20


def test_isal_plugin_encode_offsets_fixtures(golden):
    """encode(..., index, startOff, endOff) of the USE_ISAL plugin: RS XORs
    ec_encode_data_update over the touched columns into the caller's parity
    (rscoding.cc:82-89); Cauchy ignores the offsets (cauchycoding.cc:78-79)."""
    meta, blobs = golden
    cases = _encode_cases(meta, "encode_offsets_isal")
    assert len(cases) >= 20  # 8 with m <= 4, 12 wide (round 6)
    for name, c in cases:
        k, m, cs, idx = c["k"], c["m"], c["chunk"], c["index"]
        data = O.fill(k * cs, c["seed"])
        cols = [data[j * cs:(j + 1) * cs].copy() for j in range(k)]
        par = O.fill(cs, c["parity_seed"])
        enc = O.isal_matrix(c["family"], k, m)
        if c["family"] == "isal_rs":
            coef = np.ascontiguousarray(enc[k * k:])
            dst = [np.zeros(cs, np.uint8) for _ in range(m)]
            dst[idx - 1] = par
            for col in range(c["startOff"] // cs, (c["endOff"] - 1) // cs + 1):
                O.lib().orc_isal_encode_update(cs, k, m, col, O.ptr(coef), O.ptr(cols[col]), O._ptrs(dst))
        else:
            par = O.encode(c["family"], k, m, cols, cs)[idx - 1]
        assert np.array_equal(par, blobs[name]), name


@pytest.mark.parametrize("fam", ["rs", "cauchy", "isal_rs", "isal_cauchy"])
def test_roundtrip_every_pattern_small(fam):
    """encode -> erase -> decode restores the originals for every erasure
    pattern of size <= m (RS/CRS(4,2) and (6,3)), parity erasures included."""
    import itertools
    for k, m, cs in [(4, 2, 128), (6, 3, 96)]:
        data = _data_chunks(1, k, cs, 99 + k)[0]
        par = O.encode(fam, k, m, data, cs)
        orig = data + par
        for e in range(1, m + 1):
            for pat in itertools.combinations(range(k + m), e):
                chunks = [c.copy() for c in orig]
                assert O.decode(fam, k, m, chunks, list(pat), cs) == 0
                for i in range(k + m):
                    assert np.array_equal(chunks[i], orig[i]), (fam, k, m, pat, i)


@pytest.mark.parametrize("fam", ["rs", "cauchy"])
def test_batch_mt_paths_match_single_stripe(fam):
    """The CPU-baseline drivers (orc_encode_batch_mt / orc_decode_batch_mt,
    threads on disjoint stripes) equal the single-stripe oracle."""
    k, m, cs, n = 10, 4, 4096, 12
    data = O.fill(n * k * cs, 31)
    par = np.zeros(n * m * cs, np.uint8)
    assert O.encode_batch_mt(fam, k, m, cs, data, par, n, 3) == 0
    d3, p3 = data.reshape(n, k, cs), par.reshape(n, m, cs)
    stripes = np.concatenate([d3, p3], axis=1)
    for s in range(n):
        assert np.array_equal(p3[s], np.stack(O.encode(fam, k, m, list(d3[s]), cs))), s
    for erased in ([0, 1, 2, 3], [0, 5, 10, 13], [12]):
        buf = stripes.copy().reshape(-1)
        buf.reshape(n, k + m, cs)[:, erased] = 0
        assert O.decode_batch_mt(fam, k, m, cs, buf, n, erased, 4) == 0
        assert np.array_equal(buf.reshape(n, k + m, cs), stripes), erased
    buf = stripes.copy().reshape(-1)
    assert O.decode_batch_mt(fam, k, m, cs, buf, n, [0, 1, 2, 3, 4], 2) != 0  # > m erasures


REFI_SO = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "oracle", "_ref",
                       "libmemec_ref_isal.so")


@pytest.mark.skipif(not os.path.exists(REFI_SO), reason="oracle/_ref/libmemec_ref_isal.so not built (make -C oracle ref)")
def test_isal_fixtures_reproduce_from_reference_plugin(golden):
    """The USE_ISAL fixtures are the reference plugin's own outputs: re-run
    MemEC's RSCoding / CauchyCoding (built -DUSE_ISAL, oracle/_ref) on a
    sample of the recorded inputs and compare with the committed bytes."""
    import ctypes
    meta, blobs = golden
    L = ctypes.CDLL(REFI_SO)
    u8p = ctypes.POINTER(ctypes.c_uint8)
    L.refi_instantiate.restype = ctypes.c_void_p
    L.refi_instantiate.argtypes = [ctypes.c_int, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32]
    L.refi_destroy.argtypes = [ctypes.c_void_p]
    L.refi_encode.argtypes = [ctypes.c_void_p, u8p, ctypes.c_uint32, u8p] + [ctypes.c_uint32] * 3
    L.refi_decode.argtypes = [ctypes.c_void_p, u8p, ctypes.c_uint64]
    scheme = {"isal_rs": 4, "isal_cauchy": 7}
    n = 0
    for name, c in _encode_cases(meta, "decode_random_isal")[::3]:
        k, m, cs = c["k"], c["m"], c["chunk"]
        work = O.fill((k + m) * cs, c["seed"])
        for e in c["erased"]:
            work[e * cs:(e + 1) * cs] = 0
        h = ctypes.c_void_p(L.refi_instantiate(scheme[c["family"]], k, m, cs))
        assert L.refi_decode(h, work.ctypes.data_as(u8p), sum(1 << i for i in range(k + m) if i not in c["erased"])) == 0
        L.refi_destroy(h)
        for r, e in enumerate(sorted(c["erased"])):
            if e < k:
                assert np.array_equal(work[e * cs:(e + 1) * cs], blobs[name][r * cs:(r + 1) * cs]), (name, e)
                n += 1
    for name, c in _encode_cases(meta, "encode_offsets_isal"):
        k, m, cs = c["k"], c["m"], c["chunk"]
        data, par = O.fill(k * cs, c["seed"]), O.fill(cs, c["parity_seed"])
        h = ctypes.c_void_p(L.refi_instantiate(scheme[c["family"]], k, m, cs))
        L.refi_encode(h, data.ctypes.data_as(u8p), 0, par.ctypes.data_as(u8p), c["index"], c["startOff"], c["endOff"])
        L.refi_destroy(h)
        assert np.array_equal(par, blobs[name]), name
        n += 1
    assert n > 20


def test_wide_fixtures_present(golden):
    """Round 6: the wide codes are pinned on the reference itself — encodes
    with m > 4 for every family, decodes of 5..8 erasures of random
    non-codeword stripes through Jerasure (RS, Cauchy) and the USE_ISAL
    plugin (data-only and mixed patterns), ISA-L startOff/endOff encodes at
    m > 4, and an ISA-L RS pattern whose survivor matrix is singular."""
    meta, _ = golden
    wide = [c for c in meta["cases"].values() if c.get("wide")]
    fams = {(c["kind"], c["family"]) for c in wide}
    for fam in ("rs", "cauchy", "isal_rs", "isal_cauchy"):
        assert ("encode", fam) in fams, fam
    for fam in ("rs", "cauchy"):
        assert ("decode_random", fam) in fams
    for fam in ("isal_rs", "isal_cauchy"):
        assert ("decode_random_isal", fam) in fams
        assert ("encode_offsets_isal", fam) in fams
    assert max(len(c["erased"]) for c in wide if c["kind"].startswith("decode")) == 8
    assert all(c["m"] > 4 for c in wide)
    assert ("decode_singular_isal", "isal_rs") in fams


def test_isal_singular_pattern_refused(golden):
    """ISA-L's gf_gen_rs_matrix is not MDS at (12,8): the reference plugin's
    gf_invert_matrix fails on the recorded pattern and decode() returns false
    (rscoding.cc:166-169); the oracle refuses it too, and the same pattern
    decodes under ISA-L Cauchy (gf_gen_cauchy1_matrix is MDS)."""
    meta, _ = golden
    cases = _encode_cases(meta, "decode_singular_isal")
    assert cases
    for name, c in cases:
        k, m, cs = c["k"], c["m"], c["chunk"]
        buf = O.fill((k + m) * cs, c["seed"])
        chunks = [buf[i * cs:(i + 1) * cs].copy() for i in range(k + m)]
        assert O.decode(c["family"], k, m, chunks, c["erased"], cs) != 0, name
        twin = name.replace("isal_rs", "isal_cauchy")
        assert meta["cases"][twin]["kind"] == "decode_random_isal", twin
