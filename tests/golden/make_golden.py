#!/usr/bin/env python3
"""Generate golden fixtures from the REAL reference coding path.

Run in the build container only (needs /root/reference and
``make -C oracle ref``).  It loads oracle/_ref/libmemec_ref.so — MemEC's own
``Coding`` plugin over its vendored Jerasure 2.0 + gf_complete, plus ISA-L
2.14's ec_base.c — and records inputs/outputs as data:

* ``golden.json``  — matrices, bitmatrix/schedule statistics, GF samples,
  case metadata and SHA-256 digests at full BASELINE sizes;
* ``golden.npz``   — raw expected output bytes for the small cases.

The ISA-L family comes from oracle/_ref/libmemec_ref_isal.so: MemEC's own
``common/coding`` compiled with -DUSE_ISAL over ISA-L 2.14's ec_base.c and
ec_highlevel_func.c (oracle/ref_isal_plugin.cc has the recipe), so the
plugin's glue — the survivor rows it inverts, the columns its
startOff/endOff update touches — is the reference's own code.

Inputs are never stored: they are regenerated from the splitmix64 stream
(oracle.c ``orc_fill_splitmix`` == device ``mec_fill_random``) with the seed
recorded per case.  Load the npz with ``allow_pickle=False``.
"""
import ctypes
import hashlib
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
REF = ctypes.CDLL(os.path.join(ROOT, "oracle", "_ref", "libmemec_ref.so"))
ORC = ctypes.CDLL(os.path.join(ROOT, "oracle", "build", "liboracle.so"))

CS_RS, CS_CAUCHY = 4, 7
u8p = ctypes.POINTER(ctypes.c_uint8)
REF.ref_instantiate.restype = ctypes.c_void_p
REF.ref_instantiate.argtypes = [ctypes.c_int, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32]
REF.ref_destroy.argtypes = [ctypes.c_void_p]
REF.ref_encode.argtypes = [ctypes.c_void_p, u8p, ctypes.c_uint32, ctypes.c_uint32, u8p]
REF.ref_decode.argtypes = [ctypes.c_void_p, u8p, ctypes.c_uint64]
REF.ref_isal_gf_mul.restype = ctypes.c_uint8
REFI = ctypes.CDLL(os.path.join(ROOT, "oracle", "_ref", "libmemec_ref_isal.so"))
REFI.refi_instantiate.restype = ctypes.c_void_p
REFI.refi_instantiate.argtypes = [ctypes.c_int, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32]
REFI.refi_destroy.argtypes = [ctypes.c_void_p]
REFI.refi_encode.argtypes = [ctypes.c_void_p, u8p, ctypes.c_uint32, u8p] + [ctypes.c_uint32] * 3
REFI.refi_decode.argtypes = [ctypes.c_void_p, u8p, ctypes.c_uint64]
REFI.refi_decode_poisoned.argtypes = [ctypes.c_void_p, u8p, ctypes.c_uint64, ctypes.c_uint8]
ISAL_SCHEME = {"isal_rs": CS_RS, "isal_cauchy": CS_CAUCHY}


def refi_encode(fam, k, m, cs, data, parity, index, st=0, ed=0, zero_mask=0):
    """USE_ISAL Coding::encode(data, parity, index, startOff, endOff) on a
    parity chunk holding `parity` (modified in place)."""
    h = ctypes.c_void_p(REFI.refi_instantiate(ISAL_SCHEME[fam], k, m, cs))
    REFI.refi_encode(h, ptr(data), zero_mask, ptr(parity), index, st, ed)
    REFI.refi_destroy(h)


def fill(n, seed, word_offset=0):
    buf = np.empty(n, dtype=np.uint8)
    ORC.orc_fill_splitmix(buf.ctypes.data_as(u8p), ctypes.c_size_t(n),
                          ctypes.c_uint64(seed), ctypes.c_uint64(word_offset))
    return buf


def ptr(a):
    return a.ctypes.data_as(u8p)


def ref_getw(scheme, k, m, cs):
    fn = ORC.orc_rs_getw if scheme == CS_RS else ORC.orc_cauchy_getw
    return fn(k, m, cs)


def ref_encode_stripes(scheme, k, m, cs, n, seed):
    """Encode n stripes with the reference plugin, parity 1..m one call each
    (test/common/coding/coding.cc:150-152)."""
    h = REF.ref_instantiate(scheme, k, m, cs)
    h = ctypes.c_void_p(h)
    data = fill(n * k * cs, seed)
    par = np.zeros(n * m * cs, dtype=np.uint8)
    out = np.empty(cs, dtype=np.uint8)
    for s in range(n):
        d = data[s * k * cs:(s + 1) * k * cs]
        for i in range(m):
            REF.ref_encode(h, ptr(d), ctypes.c_uint32(0), ctypes.c_uint32(i + 1), ptr(out))
            par[(s * m + i) * cs:(s * m + i + 1) * cs] = out
    REF.ref_destroy(h)
    return data, par


def ref_decode_random(scheme, k, m, cs, seed, erased):
    """Decode a stripe of RANDOM chunks (not a codeword): pins the exact
    linear combination the reference applies, not just uniqueness."""
    h = ctypes.c_void_p(REF.ref_instantiate(scheme, k, m, cs))
    chunks = fill((k + m) * cs, seed)
    present = sum(1 << i for i in range(k + m) if i not in erased)
    work = chunks.copy()
    rc = REF.ref_decode(h, ptr(work), ctypes.c_uint64(present))
    REF.ref_destroy(h)
    out = np.concatenate([work[e * cs:(e + 1) * cs] for e in sorted(erased)]) if erased else np.zeros(0, np.uint8)
    return rc, out


def ref_delta(scheme, k, m, cs, seed, col, index):
    h = ctypes.c_void_p(REF.ref_instantiate(scheme, k, m, cs))
    data = fill(k * cs, seed)
    out = np.empty(cs, dtype=np.uint8)
    zero_mask = ((1 << k) - 1) & ~(1 << col)
    REF.ref_encode(h, ptr(data), ctypes.c_uint32(zero_mask), ctypes.c_uint32(index), ptr(out))
    REF.ref_destroy(h)
    return out


def isal_decode_case(fam, k, m, cs, pat, s):
    """The USE_ISAL plugin's decode of a random non-codeword stripe (as the
    ISA-L section of main()): (ok, out, fixed, defect).  Erased data chunks
    are the plugin's bytes; erased parity chunks are zeros in `out` (the
    plugin reads them from uninitialised stack, rscoding.cc:173-175) and the
    plugin's own encode of the decoded data in `fixed`."""
    chunks = fill((k + m) * cs, s)
    present = sum(1 << i for i in range(k + m) if i not in pat)
    outs, rcs = [], []
    for poison in (0x00, 0xA5):
        work = chunks.copy()
        for e in pat:
            work[e * cs:(e + 1) * cs] = 0
        h = ctypes.c_void_p(REFI.refi_instantiate(ISAL_SCHEME[fam], k, m, cs))
        rcs.append(REFI.refi_decode_poisoned(h, ptr(work), ctypes.c_uint64(present), poison))
        REFI.refi_destroy(h)
        outs.append(work)
    assert rcs[0] == rcs[1], (fam, k, m, pat)
    if rcs[1] != 0:
        return False, None, None, None
    work = outs[1]
    out = np.concatenate([work[e * cs:(e + 1) * cs] for e in sorted(pat)])
    for e in pat:
        if e < k:
            assert np.array_equal(outs[0][e * cs:(e + 1) * cs], work[e * cs:(e + 1) * cs]), (fam, pat)
    fixed = out.copy()
    defect = []
    for r, e in enumerate(sorted(pat)):
        if e < k:
            continue
        par = np.zeros(cs, np.uint8)
        refi_encode(fam, k, m, cs, work[:k * cs].copy(), par, e - k + 1)
        fixed[r * cs:(r + 1) * cs] = par
        defect.append(bool(not np.array_equal(out[r * cs:(r + 1) * cs], par)))
        out[r * cs:(r + 1) * cs] = 0
    return True, out, fixed, defect


def wide_cases(meta, blobs, seed):
    """Round 6: wide codes pinned on the reference itself
    — more than 4 parities, decodes of 5..8 erasures — where the engine runs
    its bit-sliced and one-pass kernels.  Jerasure RS /
    Cauchy through libmemec_ref.so (jerasure.c:167-268, cauchycoding.cc:87-180),
    ISA-L RS / Cauchy through the USE_ISAL plugin (rscoding.cc:155-177).
    Chunk sizes include ones that are not a multiple of the bit-sliced
    kernels' 2 KiB tile."""
    # Jerasure encodes, m > 4
    for idx, (fam, k, m, cs, n) in enumerate([("rs", 16, 8, 2560, 1), ("rs", 12, 8, 1024, 2), ("rs", 10, 6, 2048, 1),
                                              ("rs", 4, 12, 512, 1), ("cauchy", 10, 6, 2560, 1),
                                              ("cauchy", 16, 8, 1024, 1), ("cauchy", 8, 5, 1280, 1)]):
        scheme = CS_RS if fam == "rs" else CS_CAUCHY
        s = seed + 6000 + idx
        _, par = ref_encode_stripes(scheme, k, m, cs, n, s)
        name = "enc/%s/%d_%d_%d_x%d" % (fam, k, m, cs, n)
        assert name not in meta["cases"], name
        blobs[name] = par
        meta["cases"][name] = {"kind": "encode", "family": fam, "k": k, "m": m, "chunk": cs, "stripes": n, "seed": s,
                               "w": ref_getw(scheme, k, m, cs), "wide": True,
                               "data_layout": "[stripe][k][chunk] from one splitmix stream",
                               "parity_layout": "[stripe][m][chunk]"}
    # Jerasure decodes of random non-codeword stripes, 5..8 erasures
    jdec = [
        ("rs", 16, 8, 2560, [[0, 1, 2, 3, 4], [0, 2, 4, 6, 8, 10], [1, 3, 5, 7, 9, 11, 13], [0, 1, 2, 3, 4, 5, 6, 7],
                             [3, 7, 11, 15, 16, 18, 20, 22], [16, 17, 18, 19, 20, 21, 22, 23], [0, 5, 9, 13, 17, 21, 23],
                             [8, 9, 10, 11, 12, 16, 17, 18], [15, 16]]),
        ("rs", 12, 8, 1024, [[0, 1, 2, 3, 4, 5], [0, 12, 13, 14, 15, 16, 17, 18], [11, 12, 19], [2, 4, 6, 8, 10, 13, 15]]),
        ("cauchy", 10, 6, 2560, [[0, 1, 2, 3, 4], [0, 1, 2, 3, 4, 5], [0, 3, 6, 9, 10, 15], [10, 11, 12, 13, 14, 15],
                                 [1, 4, 7, 11, 13]]),
        ("cauchy", 16, 8, 1024, [[0, 1, 2, 3, 4, 5, 6, 7], [2, 5, 8, 11, 16, 19, 22, 23], [16, 17, 18, 19, 20]]),
    ]
    for idx, (fam, k, m, cs, pats) in enumerate(jdec):
        scheme = CS_RS if fam == "rs" else CS_CAUCHY
        for p_i, pat in enumerate(pats):
            s = seed + 8000 + 100 * idx + p_i
            rc, out = ref_decode_random(scheme, k, m, cs, s, pat)
            assert rc == 0, (fam, k, m, pat)
            name = "dec/%s/%d_%d_%d/%s" % (fam, k, m, cs, "-".join(map(str, pat)))
            blobs[name] = out
            meta["cases"][name] = {"kind": "decode_random", "family": fam, "k": k, "m": m, "chunk": cs,
                                   "seed": s, "erased": pat, "rc": rc, "w": ref_getw(scheme, k, m, cs), "wide": True,
                                   "input_layout": "[k+m][chunk] random; erased chunks cleared before decode",
                                   "output_layout": "erased chunks ascending"}
    # ISA-L encodes and offset updates, m > 4 (ec_encode_data_base through the plugin)
    for (k, m, cs) in [(12, 8, 1024), (12, 6, 2560), (4, 12, 512)]:
        for fam, gen in (("isal_rs", REF.ref_isal_gen_rs_matrix), ("isal_cauchy", REF.ref_isal_gen_cauchy1_matrix)):
            a = np.zeros((k + m) * k, dtype=np.uint8)
            gen(ptr(a), k + m, k)
            meta["isal_matrices"]["%s/%d,%d" % (fam, k, m)] = a.tolist()
            s = seed + 9000 + k * 100 + m + (0 if fam == "isal_rs" else 50)
            data = fill(k * cs, s)
            par = np.zeros(m * cs, dtype=np.uint8)
            for i in range(m):
                one = np.zeros(cs, dtype=np.uint8)
                refi_encode(fam, k, m, cs, data, one, i + 1)
                par[i * cs:(i + 1) * cs] = one
            chk = np.zeros(m * cs, dtype=np.uint8)
            src = (u8p * k)(*[ptr(data[j * cs:]) for j in range(k)])
            dst = (u8p * m)(*[ptr(chk[i * cs:]) for i in range(m)])
            REF.ref_isal_encode(cs, k, m, ptr(a[k * k:].copy()), src, dst)
            assert np.array_equal(par, chk), (fam, k, m)
            name = "enc/%s/%d_%d_%d_x1" % (fam, k, m, cs)
            blobs[name] = par
            meta["cases"][name] = {"kind": "encode", "family": fam, "k": k, "m": m, "chunk": cs, "stripes": 1,
                                   "seed": s, "wide": True, "data_layout": "[k][chunk]", "parity_layout": "[m][chunk]"}
            # the server's delta call: encode(data, parity, index, startOff, endOff)
            for j, (index, st, ed) in enumerate([(m, 1 * cs + 5, (k - 1) * cs + 1), (m - 2, (k - 1) * cs, k * cs)]):
                s2 = seed + 9500 + k * 100 + m * 4 + j + (0 if fam == "isal_rs" else 50)
                d2 = fill(k * cs, s2)
                p2 = fill(cs, s2 + 1)
                refi_encode(fam, k, m, cs, d2, p2, index, st, ed)
                name = "encoff/%s/%d_%d_%d/i%d_s%d_e%d" % (fam, k, m, cs, index, st, ed)
                blobs[name] = p2
                meta["cases"][name] = {"kind": "encode_offsets_isal", "family": fam, "k": k, "m": m, "chunk": cs,
                                       "seed": s2, "parity_seed": s2 + 1, "index": index, "startOff": st, "endOff": ed,
                                       "wide": True, "data_layout": "[k][chunk] splitmix(seed)",
                                       "parity_in": "[chunk] splitmix(parity_seed), the caller's parity chunk",
                                       "expected": "the caller's parity chunk after the reference plugin's "
                                                   "RSCoding/CauchyCoding::encode (USE_ISAL)"}
    # ISA-L decodes of random non-codeword stripes, 5..8 erasures: data-only
    # patterns (the plugin's own bytes) and mixed ones (`fixed` for parity)
    idec = [(12, 8, 1024, [[0, 1, 2, 3, 4], [0, 2, 4, 6, 8, 10], [0, 1, 2, 3, 4, 5, 6], [4, 5, 6, 7, 8, 9, 10, 11],
                           [0, 1, 2, 3, 5, 7, 9, 11], [1, 3, 5, 12, 14, 16, 18], [12, 13, 14, 15, 16, 17, 18, 19],
                           # singular for ISA-L RS (gf_gen_rs_matrix is not MDS at this size: the
                           # plugin's gf_invert_matrix fails, decode() returns false); Cauchy decodes it
                           [0, 1, 2, 4, 5, 8, 12, 15]]),
            (12, 6, 2560, [[0, 1, 2, 3, 4], [0, 1, 2, 3, 4, 5], [6, 7, 8, 9, 10, 11], [1, 3, 5, 7, 9, 11],
                           [0, 11, 12, 14, 16, 17]])]
    for fam_i, fam in enumerate(("isal_rs", "isal_cauchy")):
        for idx, (k, m, cs, pats) in enumerate(idec):
            for p_i, pat in enumerate(pats):
                s = seed + 10000 + 1000 * fam_i + 100 * idx + p_i
                ok, out, fixed, defect = isal_decode_case(fam, k, m, cs, pat, s)
                name = "dec/%s/%d_%d_%d/%s" % (fam, k, m, cs, "-".join(map(str, pat)))
                if not ok:  # the k x k survivor matrix is singular: the plugin returns false
                    meta["cases"][name] = {"kind": "decode_singular_isal", "family": fam, "k": k, "m": m,
                                           "chunk": cs, "seed": s, "erased": pat, "rc": 0, "wide": True}
                    continue
                blobs[name] = out
                blobs[name + "|fixed"] = fixed
                meta["cases"][name] = {"kind": "decode_random_isal", "family": fam, "k": k, "m": m, "chunk": cs,
                                       "seed": s, "erased": pat, "rc": 1, "reference_parity_defect": defect,
                                       "wide": True,
                                       "input_layout": "[k+m][chunk] random; erased chunks cleared before decode",
                                       "output_layout": "erased chunks ascending (reference plugin output; "
                                                        "erased parity undefined there, zeroed)",
                                       "fixed_layout": "same; erased parity = the reference plugin's encode "
                                                       "of the decoded data"}


def main():
    meta = {"generator": "tests/golden/make_golden.py",
            "reference": "mtyiu/memec common/coding over lib/jerasure + lib/gf_complete; the same plugin built USE_ISAL over ISA-L 2.14 ec_base.c + ec_highlevel_func.c",
            "prng": "splitmix64: word q = mix(seed + (q+1)*0x9E3779B97F4A7C15), little-endian bytes",
            "cases": {}}
    blobs = {}

    # --- GF samples (galois_single_multiply / divide) -----------------------
    gf = {}
    for w in range(1, 9):
        n = 1 << w
        tab = [[REF.ref_gf_mul(a, b, w) for b in range(n)] for a in range(n)]
        h = hashlib.sha256(np.array(tab, dtype=np.int32).tobytes()).hexdigest()
        inv = [REF.ref_gf_div(1, a, w) for a in range(1, n)]
        gf[str(w)] = {"mul_table_sha256_int32": h, "inverses": inv}
        if w <= 4:
            gf[str(w)]["mul_table"] = tab
    meta["gf"] = gf

    # --- matrices ------------------------------------------------------------
    rs = {}
    for k in range(1, 31):
        for m in range(1, 33 - k):
            mat = (ctypes.c_int * (k * m))()
            if REF.ref_rs_matrix(k, m, 8, mat) == 0:
                rs["%d,%d" % (k, m)] = list(mat)
    meta["rs_matrices"] = rs

    cau = {}
    for w in range(1, 9):
        for k in range(1, 33):
            for m in range(1, 33 - k):
                if k + m > (1 << w):
                    continue
                mat = (ctypes.c_int * (k * m))()
                if REF.ref_cauchy_matrix(k, m, w, mat) != 0:
                    continue
                bm = (ctypes.c_int * (k * m * w * w))()
                REF.ref_bitmatrix(k, m, w, mat, bm)
                ops = (ctypes.c_int * (5 * (k * m * w * w + 1)))()
                nops = REF.ref_smart_schedule(k, m, w, bm, ops, k * m * w * w + 1)
                cau["%d,%d,%d" % (k, m, w)] = {
                    "matrix": list(mat), "bitmatrix_ones": sum(bm),
                    "bitmatrix_sha256_int32": hashlib.sha256(bytes(bm)).hexdigest(),
                    "schedule_ops": nops,
                    "schedule_sha256_int32": hashlib.sha256(bytes(ops)[:20 * nops]).hexdigest()}
    meta["cauchy_matrices"] = cau
    cbest = {}
    for w in range(2, 9):
        k = (1 << w) - 1
        mat = (ctypes.c_int * (k * 2))()
        REF.ref_cauchy_matrix(k, 2, w, mat)
        cbest[str(w)] = list(mat)[k:]
    meta["cbest"] = cbest

    # --- Jerasure encode: raw small cases --------------------------------------
    enc_cases = [
        ("rs", 4, 2, 4096, 2), ("rs", 8, 2, 4096, 2), ("rs", 10, 4, 4096, 1),
        ("rs", 3, 3, 64, 3), ("rs", 6, 3, 1024, 1), ("rs", 12, 4, 520, 1),
        ("rs", 16, 16, 64, 1), ("rs", 28, 4, 72, 1), ("rs", 1, 1, 64, 1),
        ("cauchy", 12, 4, 256, 2), ("cauchy", 4, 2, 4096, 1), ("cauchy", 8, 2, 4096, 1),
        ("cauchy", 4, 2, 96, 2), ("cauchy", 20, 4, 320, 1), ("cauchy", 20, 4, 96, 1),
        ("cauchy", 20, 4, 112, 1), ("cauchy", 20, 4, 64, 1), ("cauchy", 10, 4, 1024, 1),
        ("cauchy", 6, 3, 48, 2), ("cauchy", 1, 1, 16, 1), ("cauchy", 3, 1, 24, 1),
    ]
    seed = 0x4D454D4543
    for idx, (fam, k, m, cs, n) in enumerate(enc_cases):
        scheme = CS_RS if fam == "rs" else CS_CAUCHY
        s = seed + idx
        _, par = ref_encode_stripes(scheme, k, m, cs, n, s)
        name = "enc/%s/%d_%d_%d_x%d" % (fam, k, m, cs, n)
        blobs[name] = par
        meta["cases"][name] = {"kind": "encode", "family": fam, "k": k, "m": m, "chunk": cs,
                               "stripes": n, "seed": s, "w": ref_getw(scheme, k, m, cs),
                               "data_layout": "[stripe][k][chunk] from one splitmix stream",
                               "parity_layout": "[stripe][m][chunk]"}

    # --- full-size digests --------------------------------------------------------
    big = [("rs", 10, 4, 1 << 20, 2), ("cauchy", 12, 4, 65536, 4), ("rs", 8, 2, 4096, 64),
           ("rs", 4, 2, 4096, 64), ("cauchy", 12, 4, 65536 + 8, 1)]
    for idx, (fam, k, m, cs, n) in enumerate(big):
        scheme = CS_RS if fam == "rs" else CS_CAUCHY
        s = seed + 1000 + idx
        _, par = ref_encode_stripes(scheme, k, m, cs, n, s)
        name = "digest/%s/%d_%d_%d_x%d" % (fam, k, m, cs, n)
        meta["cases"][name] = {"kind": "encode_digest", "family": fam, "k": k, "m": m, "chunk": cs,
                               "stripes": n, "seed": s, "w": ref_getw(scheme, k, m, cs),
                               "parity_sha256": hashlib.sha256(par.tobytes()).hexdigest(),
                               "per_chunk_sha256": [hashlib.sha256(par[i * cs:(i + 1) * cs].tobytes()).hexdigest()
                                                    for i in range(min(n * m, 8))]}

    # --- decode of random (non-codeword) stripes --------------------------------------
    dec_cases = [
        ("rs", 4, 2, 512, [[0], [1], [4], [5], [0, 1], [0, 4], [1, 5], [4, 5], [2, 3], [0, 5]]),
        ("rs", 10, 4, 256, [[0, 1, 2, 3], [0, 5, 10, 13], [10, 11, 12, 13], [3], [11], [10], [2, 7], [0, 10],
                            [1, 2, 3, 11], [9, 10, 12], [0, 1, 2, 13]]),
        ("rs", 8, 3, 256, [[1, 2, 3], [1], [1, 2], [8, 9, 10], [0, 9], [7, 8]]),
        ("rs", 8, 2, 4096, [[0, 1], [0], [8, 9], [3, 8]]),
        ("cauchy", 12, 4, 256, [[0, 1, 2, 3], [0, 5, 12, 15], [12, 13, 14, 15], [3], [13], [12], [2, 7], [0, 12]]),
        ("cauchy", 4, 2, 4096, [[0, 1], [0], [4, 5], [2, 4], [1, 5]]),
        ("cauchy", 8, 3, 256, [[1, 2, 3], [1], [8, 9, 10], [0, 9]]),
        ("cauchy", 20, 4, 320, [[0, 1, 2, 3], [19, 20], [21]]),
        ("cauchy", 20, 4, 112, [[0, 1, 2, 3], [5, 22]]),
    ]
    for idx, (fam, k, m, cs, pats) in enumerate(dec_cases):
        scheme = CS_RS if fam == "rs" else CS_CAUCHY
        for p_i, pat in enumerate(pats):
            s = seed + 2000 + 100 * idx + p_i
            rc, out = ref_decode_random(scheme, k, m, cs, s, pat)
            name = "dec/%s/%d_%d_%d/%s" % (fam, k, m, cs, "-".join(map(str, pat)))
            blobs[name] = out
            meta["cases"][name] = {"kind": "decode_random", "family": fam, "k": k, "m": m, "chunk": cs,
                                   "seed": s, "erased": pat, "rc": rc, "w": ref_getw(scheme, k, m, cs),
                                   "input_layout": "[k+m][chunk] random; erased chunks cleared before decode",
                                   "output_layout": "erased chunks ascending"}
    # too many erasures -> false
    rc, _ = ref_decode_random(CS_RS, 4, 2, 64, 7, [0, 1, 2])
    meta["cases"]["dec/rs/4_2_64/0-1-2"] = {"kind": "decode_fail", "family": "rs", "k": 4, "m": 2,
                                             "chunk": 64, "erased": [0, 1, 2], "rc": rc}

    # --- delta (single non-zero column, Coding::zeros elsewhere) ------------------------
    for idx, (fam, k, m, cs, col, index) in enumerate([("rs", 8, 2, 4096, 3, 2), ("rs", 10, 4, 512, 0, 4),
                                                      ("cauchy", 12, 4, 256, 11, 3), ("cauchy", 4, 2, 4096, 1, 1)]):
        scheme = CS_RS if fam == "rs" else CS_CAUCHY
        s = seed + 3000 + idx
        out = ref_delta(scheme, k, m, cs, s, col, index)
        name = "delta/%s/%d_%d_%d/c%d_p%d" % (fam, k, m, cs, col, index)
        blobs[name] = out
        meta["cases"][name] = {"kind": "delta", "family": fam, "k": k, "m": m, "chunk": cs, "seed": s,
                               "column": col, "index": index,
                               "data_layout": "[k][chunk] splitmix; every column but `column` is Coding::zeros"}

    # --- ISA-L base family -------------------------------------------------------------
    isal = {}
    for (k, m) in [(4, 2), (8, 2), (10, 4), (12, 4), (6, 3)]:
        for fam, gen in (("isal_rs", REF.ref_isal_gen_rs_matrix), ("isal_cauchy", REF.ref_isal_gen_cauchy1_matrix)):
            a = np.zeros((k + m) * k, dtype=np.uint8)
            gen(ptr(a), k + m, k)
            isal["%s/%d,%d" % (fam, k, m)] = a.tolist()
            cs, s = 512, seed + 4000 + k * 10 + m + (0 if fam == "isal_rs" else 500)
            data = fill(k * cs, s)
            par = np.zeros(m * cs, dtype=np.uint8)
            coef = a[k * k:].copy()
            # the plugin's encode, one call per parity index (coding.cc:150-152)
            for i in range(m):
                one = np.zeros(cs, dtype=np.uint8)
                refi_encode(fam, k, m, cs, data, one, i + 1)
                par[i * cs:(i + 1) * cs] = one
            # == ISA-L's own ec_encode_data_base over gf_vect_mul_init tables
            chk = np.zeros(m * cs, dtype=np.uint8)
            src = (u8p * k)(*[ptr(data[j * cs:]) for j in range(k)])
            dst = (u8p * m)(*[ptr(chk[i * cs:]) for i in range(m)])
            REF.ref_isal_encode(cs, k, m, ptr(coef), src, dst)
            assert np.array_equal(par, chk), (fam, k, m)
            name = "enc/%s/%d_%d_%d_x1" % (fam, k, m, cs)
            blobs[name] = par
            meta["cases"][name] = {"kind": "encode", "family": fam, "k": k, "m": m, "chunk": cs, "stripes": 1,
                                   "seed": s, "data_layout": "[k][chunk]", "parity_layout": "[m][chunk]"}
            # update: parity ^= coef[:,col] * data[col]   (ec_encode_data_update_base)
            col = k // 2
            upd = par.copy()
            dst2 = (u8p * m)(*[ptr(upd[i * cs:]) for i in range(m)])
            delta = fill(cs, s + 1)
            REF.ref_isal_encode_update(cs, k, m, col, ptr(coef), ptr(delta), dst2)
            name = "upd/%s/%d_%d_%d/c%d" % (fam, k, m, cs, col)
            blobs[name] = upd
            meta["cases"][name] = {"kind": "update", "family": fam, "k": k, "m": m, "chunk": cs, "seed": s,
                                   "delta_seed": s + 1, "column": col,
                                   "semantics": "parity (enc case) ^= coef[i][col] * delta"}
    meta["isal_matrices"] = isal

    # --- ISA-L plugin decode (USE_ISAL RSCoding/CauchyCoding::decode) ----------------
    # Random non-codeword stripes through the reference plugin itself
    # (rscoding.cc:97-187, cauchycoding.cc:87-180, libmemec_ref_isal.so).
    # Erased DATA chunks are the reference's output bit for bit.  For an
    # erased PARITY chunk the plugin reads rows past the k x k inverse, i.e.
    # uninitialised stack (rscoding.cc:173-175): its bytes are undefined, so
    # the blob holds zeros there, `fixed` holds the reference plugin's own
    # encode of the decoded data (what a correct decode writes),
    # and `reference_parity_defect` records that the plugin's output, with
    # the stack poisoned, differs from `fixed` in every such chunk.
    isal_dec = [
        (4, 2, [[0], [1, 3], [0, 1], [4], [5], [4, 5], [0, 4], [3, 5]]),
        (10, 4, [[0, 1, 2, 3], [0, 5, 9], [3], [9], [10], [13], [10, 11, 12, 13], [0, 5, 10, 13], [2, 7, 11],
                 [9, 12]]),
        (12, 4, [[0, 1, 2, 3], [11], [4, 8], [12], [15], [12, 13, 14, 15], [0, 5, 12, 15], [1, 14]]),
        (6, 3, [[0, 1, 2], [5], [6], [8], [6, 7, 8], [0, 6], [2, 4, 8], [1, 7]]),
    ]
    cs = 256
    for fam_i, fam in enumerate(("isal_rs", "isal_cauchy")):
        for idx, (k, m, pats) in enumerate(isal_dec):
            for p_i, pat in enumerate(pats):
                s = seed + 5000 + 1000 * fam_i + 100 * idx + p_i
                chunks = fill((k + m) * cs, s)
                present = sum(1 << i for i in range(k + m) if i not in pat)
                outs = []
                for poison in (0x00, 0xA5):
                    work = chunks.copy()
                    for e in pat:
                        work[e * cs:(e + 1) * cs] = 0
                    h = ctypes.c_void_p(REFI.refi_instantiate(ISAL_SCHEME[fam], k, m, cs))
                    rc = REFI.refi_decode_poisoned(h, ptr(work), ctypes.c_uint64(present), poison)
                    REFI.refi_destroy(h)
                    outs.append(work)
                work = outs[1]
                out = np.concatenate([work[e * cs:(e + 1) * cs] for e in sorted(pat)])
                # erased data chunks do not depend on the stack
                for e in pat:
                    if e < k:
                        assert np.array_equal(outs[0][e * cs:(e + 1) * cs], work[e * cs:(e + 1) * cs]), (fam, pat)
                # reference re-encode of the decoded data -> correct parity
                fixed = out.copy()
                defect = []
                for r, e in enumerate(sorted(pat)):
                    if e < k:
                        continue
                    par = np.zeros(cs, np.uint8)
                    refi_encode(fam, k, m, cs, work[:k * cs].copy(), par, e - k + 1)
                    fixed[r * cs:(r + 1) * cs] = par
                    defect.append(bool(not np.array_equal(out[r * cs:(r + 1) * cs], par)))
                    out[r * cs:(r + 1) * cs] = 0
                name = "dec/%s/%d_%d_%d/%s" % (fam, k, m, cs, "-".join(map(str, pat)))
                blobs[name] = out
                blobs[name + "|fixed"] = fixed
                meta["cases"][name] = {"kind": "decode_random_isal", "family": fam, "k": k, "m": m, "chunk": cs,
                                       "seed": s, "erased": pat, "rc": 1 if rc == 0 else 0,
                                       "reference_parity_defect": defect,
                                       "input_layout": "[k+m][chunk] random; erased chunks cleared before decode",
                                       "output_layout": "erased chunks ascending (reference plugin output; "
                                                        "erased parity undefined there, zeroed)",
                                       "fixed_layout": "same; erased parity = the reference plugin's encode "
                                                       "of the decoded data"}

    # --- ISA-L plugin encode with startOff/endOff (the server's delta call) -------------
    # RSCoding::encode's USE_ISAL update branch XORs ec_encode_data_update
    # over data columns [startOff/chunk, (endOff-1)/chunk] into the caller's
    # parity (rscoding.cc:82-89); CauchyCoding ignores the offsets and
    # overwrites it with a full ec_encode_data (cauchycoding.cc:78-79).  Both
    # run as the reference plugin's own encode here.
    for fam_i, fam in enumerate(("isal_rs", "isal_cauchy")):
        for idx, (k, m, cs, index, st, ed) in enumerate([(10, 4, 512, 2, 3 * 512 + 100, 5 * 512 + 7),
                                                        (4, 2, 4096, 1, 0, 4096), (6, 3, 256, 3, 1 * 256, 2 * 256),
                                                        (12, 4, 512, 4, 11 * 512 + 1, 12 * 512)]):
            s = seed + 7000 + 100 * fam_i + idx
            data = fill(k * cs, s)
            par = fill(cs, s + 1)
            refi_encode(fam, k, m, cs, data, par, index, st, ed)
            name = "encoff/%s/%d_%d_%d/i%d_s%d_e%d" % (fam, k, m, cs, index, st, ed)
            blobs[name] = par
            meta["cases"][name] = {"kind": "encode_offsets_isal", "family": fam, "k": k, "m": m, "chunk": cs,
                                   "seed": s, "parity_seed": s + 1, "index": index, "startOff": st, "endOff": ed,
                                   "data_layout": "[k][chunk] splitmix(seed)",
                                   "parity_in": "[chunk] splitmix(parity_seed), the caller's parity chunk",
                                   "expected": "the caller's parity chunk after the reference plugin's "
                                               "RSCoding/CauchyCoding::encode (USE_ISAL)"}

    wide_cases(meta, blobs, seed)

    np.savez_compressed(os.path.join(HERE, "golden.npz"), **{k.replace("/", "|"): v for k, v in blobs.items()})
    with open(os.path.join(HERE, "golden.json"), "w") as f:
        json.dump(meta, f, separators=(",", ":"), sort_keys=True)
    print("cases:", len(meta["cases"]), "blobs:", len(blobs),
          "npz bytes:", os.path.getsize(os.path.join(HERE, "golden.npz")),
          "json bytes:", os.path.getsize(os.path.join(HERE, "golden.json")))


if __name__ == "__main__":
    sys.exit(main())
