#!/usr/bin/env python3
"""Device-resident stripe encode/decode throughput on MI355X.

Default workload = BASELINE.json configs[1]: RS(10,4) encode, 1 MiB chunks,
4096 stripes per GPU, inputs resident in HBM.  A "step" is one batched
encode of the whole batch (one kernel launch).  Multi-GPU: one process per
GPU (torchrun), stripes sharded by rank with no data-path collective
(weak scaling: every rank encodes its own 4096-stripe batch); the barrier,
max-over-ranks time and the final reduction use RCCL ("nccl").

Prints ONE JSON line (rank 0).  value = data GiB/s (k * chunk * stripes /
2^30 / s, the reference's MB/s convention, test/common/coding/common.hh:17-22)
summed over all ranks.  roofline.achieved = algorithmic HBM bytes
((k+m) * chunk per stripe for encode, (k+e) * chunk for decode) per launch /
average launch time from HIP events on the launch stream.
"""
import argparse
import json
import os
import re
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "GiB/s device-resident RS(k,m) encode+decode; % of HBM3E roofline"
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md)

CONFIGS = {
    # name: (family, k, m, chunk, stripes per GPU, op, erased)
    "rs_enc": ("rs", 10, 4, 1 << 20, 4096, "encode", None),                # configs[1]
    "rs_dec": ("rs", 10, 4, 1 << 20, 4096, "decode", [0, 1, 2, 3]),        # configs[2]
    "rs_dec_mixed": ("rs", 10, 4, 1 << 20, 4096, "decode", [0, 5, 10, 13]),
    "rs8_small": ("rs", 8, 2, 4096, 65536, "encode", None),                # configs[3]
    "crs_enc": ("cauchy", 12, 4, 65536, 4096, "encode", None),             # configs[4] per GPU
    "crs_dec": ("cauchy", 12, 4, 65536, 4096, "decode", [0, 1, 2, 3]),
    "rs42": ("rs", 4, 2, 4096, 65536, "encode", None),                    # configs[0] shape on the GPU
    "rs42_dec": ("rs", 4, 2, 4096, 65536, "decode", [0, 1]),
    # the server's delta path (parity_chunk_buffer.cc:342-353): parity ^=
    # A[:, j] * delta for one data column j (last field = j)
    "rs8_update": ("rs", 8, 2, 4096, 65536, "update", 3),
    "rs_update": ("rs", 10, 4, 1 << 20, 4096, "update", 3),
    # wide codes (m > 4, k + m <= 32: rscoding.cc:26-29): one pass over the
    # sources for every parity (gf8_mg_kernel)
    "rs16_8": ("rs", 16, 8, 65536, 16384, "encode", None),
    "rs16_8_dec": ("rs", 16, 8, 65536, 16384, "decode", [0, 1, 2, 3, 4, 5, 6, 7]),
    "isal12_8": ("isal_rs", 12, 8, 65536, 16384, "encode", None),
}
WORKLOAD_NAMES = {
    "rs_enc": "RS(10,4) encode, 1 MiB chunks, 4096 stripes per GPU (BASELINE configs[1])",
    "rs_dec": "RS(10,4) decode 4 erasures {0,1,2,3}, 1 MiB chunks, 4096 stripes per GPU (configs[2])",
    "rs_dec_mixed": "RS(10,4) decode 4 erasures {0,5,10,13}, 1 MiB chunks, 4096 stripes per GPU",
    "rs8_small": "RS(8,2) encode, 4 KiB chunks, 65536 stripes per GPU (configs[3])",
    "crs_enc": "Cauchy-RS(12,4) encode, 64 KiB chunks, 4096 stripes per GPU (configs[4] sharded)",
    "crs_dec": "Cauchy-RS(12,4) decode {0,1,2,3}, 64 KiB chunks, 4096 stripes per GPU",
    "rs42": "RS(4,2) encode, 4 KiB chunks, 65536 stripes per GPU (configs[0] shape)",
    "rs42_dec": "RS(4,2) decode 2 erasures {0,1}, 4 KiB chunks, 65536 stripes per GPU (configs[0] shape)",
    "rs8_update": "RS(8,2) delta update of data column 3 into both parities, 4 KiB chunks, 65536 stripes per GPU",
    "rs_update": "RS(10,4) delta update of data column 3 into all 4 parities, 1 MiB chunks, 4096 stripes per GPU",
    "rs16_8": "RS(16,8) encode, 64 KiB chunks, 16384 stripes per GPU (wide code, one pass)",
    "rs16_8_dec": "RS(16,8) decode 8 erasures {0..7}, 64 KiB chunks, 16384 stripes per GPU (wide code)",
    "isal12_8": "ISA-L RS(12,8) encode, 64 KiB chunks, 16384 stripes per GPU (wide code, one pass)",
}


def workload_name(config, stripes, strong=False, global_stripes=0):
    """WORKLOAD_NAMES[config] with the stripe count actually run (--stripes /
    --strong override the BASELINE count; the name must not claim it then)."""
    name = WORKLOAD_NAMES[config]
    m = re.search(r"(\d+) stripes per GPU", name)
    if strong:
        return name[:m.start()] + "%d stripes total, sharded over ranks" % global_stripes + name[m.end():]
    if int(m.group(1)) != stripes:
        return name[:m.start()] + "%d stripes per GPU (reduced)" % stripes + name[m.end():]
    return name


def cpu_baseline(fam, k, m, cs, gpu_parity_np, seed, threads):
    """Oracle restatement (same algorithm as the reference's scalar
    Jerasure/gf_complete path) on this host, a bounded sample of the same
    workload; its output is checked against the GPU's for those stripes."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import numpy as np
    import _oracle as O

    per = k * cs
    sample = cpu_sample(k, m, cs, threads)
    p = cpu_parallelism(threads, host_cores()[0], sample)
    log("cpu_baseline encode: port, %d stripes on %d threads" % (sample, threads))
    data = O.fill(sample * per, seed)
    par = np.zeros(sample * m * cs, np.uint8)
    # 1 thread, 1 pass over `p` stripes (single-core figure)
    t0 = time.perf_counter()
    O.encode_batch_mt(fam, k, m, cs, data, par, p, 1)
    t1 = time.perf_counter()
    single = p * per / (t1 - t0) / 2**30
    passes, t_total = 0, 0.0
    t0 = time.perf_counter()
    while True:
        O.encode_batch_mt(fam, k, m, cs, data, par, sample, threads)
        passes += 1
        t_total = time.perf_counter() - t0
        if t_total * p >= CPU_WORK_S[0] or passes >= 64:
            break
    value = passes * sample * per / t_total / 2**30
    verified = None
    if gpu_parity_np is not None:
        n = min(sample, gpu_parity_np.shape[0])
        verified = bool((gpu_parity_np[:n].reshape(-1) == par[: n * m * cs]).all())
    return {"value": round(value, 4), "unit": "GiB/s", "cores": threads, "kind": "port",
            "sample": "%d stripes x %d passes of the same workload, oracle/oracle.c orc_encode_batch_mt "
                      "(scalar 256x256 table + 64-bit XOR, as MemEC's default build), %d threads, "
                      "disjoint stripes per thread" % (sample, passes, threads),
            "single_thread_value": round(single, 4), "matches_gpu": verified, "cpu_model": cpu_model()}


REF_SO = os.path.join(ROOT, "oracle", "_ref", "libmemec_ref.so")


def _ref_lib():
    """The reference's own coding path (MemEC plugin + Jerasure +
    gf_complete) compiled from its sources in the build container by
    oracle/Makefile into oracle/_ref/ (travels with the tree; absent in a
    fresh checkout -> None).  Used only for the CPU baseline."""
    import ctypes
    if not os.path.exists(REF_SO):
        return None
    L = ctypes.CDLL(REF_SO)
    vp, u32 = ctypes.c_void_p, ctypes.c_uint32
    L.ref_instantiate.restype = vp
    L.ref_instantiate.argtypes = [ctypes.c_int, u32, u32, u32]
    L.ref_destroy.argtypes = [vp]
    L.ref_encode_batch_mt.restype = ctypes.c_double
    L.ref_encode_batch_mt.argtypes = [vp, vp, vp, u32, u32, u32]
    L.ref_decode_batch_mt.restype = ctypes.c_double
    L.ref_decode_batch_mt.argtypes = [vp, vp, u32, ctypes.c_uint64, u32, u32]
    L.ref_update_batch_mt.restype = ctypes.c_double
    L.ref_update_batch_mt.argtypes = [vp, vp, vp, u32, u32, u32, u32]
    return L


def log(msg):
    """Progress on stderr (the JSON line alone goes to stdout)."""
    sys.stderr.write("bench: %s\n" % msg)
    sys.stderr.flush()


# CPU-baseline samples are sized by bytes, never by the thread count: a
# --cpu-threads far above the host's cores once asked for 256 stripes of
# 14 MiB per leg and ~512 CPU-seconds of reference work, which the GPU
# box's output watchdog killed (profiles/r02/cpu/cpu_threads_ab.log).
CPU_SAMPLE_BYTES = 768 << 20      # stripe bytes ((k + m) * chunk) per leg
CPU_SAMPLE_BYTES_MAX = 1 << 30    # ... when more stripes are needed to give every thread one
CPU_WORK_S = (10.0, 30.0)         # CPU-seconds of reference work per leg (min, max)


def cpu_sample(k, m, cs, threads):
    """Stripes in one CPU-baseline leg: ~768 MiB (1 to 64 stripes), raised
    to one stripe per thread while that stays under 1 GiB, and a multiple
    of the threads that get work."""
    sb = (k + m) * cs
    base = max(1, min(64, CPU_SAMPLE_BYTES // sb))
    hi = max(base, CPU_SAMPLE_BYTES_MAX // sb)
    n = min(max(base, threads), hi)
    t = max(1, min(threads, n))
    return n // t * t


def cpu_parallelism(threads, usable, sample):
    """Workers that actually run at once: requested threads, capped by the
    host's usable cores (cgroup quota / affinity) and the sample's stripes."""
    return max(1, min(threads, usable, sample))


def cpu_work_plan(probe_s, threads, usable, sample):
    """Passes of a timed CPU leg whose single-worker pass over the sample
    took probe_s: 10-30 CPU-seconds of work (2 s per running worker), so
    the wall time stays ~10 s at one core and ~2 s at 16 whatever the
    requested thread count.  Returns (passes, estimated wall seconds)."""
    p = cpu_parallelism(threads, usable, sample)
    cpu_s = min(CPU_WORK_S[1], max(CPU_WORK_S[0], 2.0 * p))
    passes = int(max(1, min(4096, round(cpu_s / max(probe_s, 1e-6)))))
    return passes, passes * probe_s / p


def ref_baseline(fam, k, m, cs, threads, sample, run, usable=None, label=""):
    """Time the compiled reference on `sample` stripes: a single-worker
    probe pass, then the passes of cpu_work_plan on `threads` workers.
    run(L, h, passes, n_stripes, threads) -> seconds."""
    L = _ref_lib()
    if L is None or fam not in ("rs", "cauchy"):
        return None
    h = L.ref_instantiate(4 if fam == "rs" else 7, k, m, cs)  # CS_RS / CS_CAUCHY
    if not h:
        return None
    usable = usable or host_cores()[0]
    try:
        probe = run(L, h, 1, sample, 1)  # one worker, one pass over the sample
        passes, est = cpu_work_plan(probe, threads, usable, sample)
        log("cpu_baseline %s: reference, %d stripes x %d passes on %d threads (%d usable cores), ~%.1f s"
            % (label, sample, passes, threads, usable, est))
        dt = run(L, h, passes, sample, threads)
    finally:
        L.ref_destroy(h)
    return probe, passes, dt


def cpu_baseline_reference(fam, k, m, cs, gpu_parity_np, seed, threads, op, erased=None, codewords=None):
    """kind "reference": MemEC's Coding::encode / Coding::decode themselves
    (oracle/ref_shim.cc ref_*_batch_mt: worker threads on disjoint stripes,
    chunks allocated once, as test/common/coding/batch_performance.cc runs
    them).  The outputs are checked against the GPU's."""
    import numpy as np
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import _oracle as O

    sample = cpu_sample(k, m, cs, threads)
    if op != "encode":  # the GPU-encoded codewords handed over (fewer on a small --stripes run)
        sample = min(sample, codewords.shape[0])
        codewords = codewords[:sample]
    per = k * cs
    if op == "encode":
        data = O.fill(sample * per, seed)
        par = np.zeros(sample * m * cs, np.uint8)

        def run(L, h, passes, n, t):
            return L.ref_encode_batch_mt(h, data.ctypes.data, par.ctypes.data, n, t, passes)
    else:
        present = sum(1 << i for i in range(k + m) if i not in erased)
        buf = np.ascontiguousarray(codewords).reshape(-1).copy()

        def run(L, h, passes, n, t):
            return L.ref_decode_batch_mt(h, buf.ctypes.data, n, present, t, passes)
    r = ref_baseline(fam, k, m, cs, threads, sample, run, label=op)
    if r is None:
        return None
    probe, passes, dt = r
    if dt < 0:
        return {"error": "reference decode reported failure"}
    if op == "encode":
        match = None
        if gpu_parity_np is not None:
            n = min(sample, gpu_parity_np.shape[0])
            match = bool((gpu_parity_np[:n].reshape(-1) == par[: n * m * cs]).all())
    else:
        match = bool(np.array_equal(buf.reshape(sample, k + m, cs), codewords))
    return {"value": round(passes * sample * per / dt / 2**30, 4), "unit": "GiB/s", "cores": threads,
            "kind": "reference",
            "sample": "%d stripes x %d passes of the same workload%s through MemEC's own Coding::%s "
                      "(common/coding + Jerasure + gf_complete compiled from the reference sources, "
                      "oracle/_ref), %d worker threads on disjoint stripes as batch_performance.cc"
                      % (sample, passes, "" if op == "encode" else ", erasures %s" % list(erased),
                         "encode" if op == "encode" else "decode", threads),
            "single_thread_value": round(sample * per / probe / 2**30, 4), "matches_gpu": match,
            "cpu_model": cpu_model()}


def configs0_reference(seconds=2.0):
    """BASELINE configs[0] as it is quoted: RS(4,2) encode and decode of
    erasures {0,1} at 4 KiB chunks through the reference's own CPU path
    (oracle/_ref: MemEC's Coding + Jerasure + gf_complete compiled from its
    sources), one process, one thread, as performance.cc runs it; about
    `seconds` of timed work per leg.  The decode's output is checked against
    the codewords and the encode's against the oracle."""
    L = _ref_lib()
    if L is None:
        return None
    import numpy as np
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import _oracle as O
    k, m, cs, n = 4, 2, 4096, 256
    h = L.ref_instantiate(4, k, m, cs)  # CS_RS
    if not h:
        return None
    try:
        data = O.fill(n * k * cs, 0x4D454D4543)
        par = np.zeros(n * m * cs, np.uint8)
        probe = L.ref_encode_batch_mt(h, data.ctypes.data, par.ctypes.data, n, 1, 1)
        ep = max(1, int(seconds / max(probe, 1e-6)))
        log("configs[0]: reference RS(4,2)@4 KiB encode, %d stripes x %d passes on 1 thread" % (n, ep))
        et = L.ref_encode_batch_mt(h, data.ctypes.data, par.ctypes.data, n, 1, ep)
        enc_ok = all(np.array_equal(par[s_ * m * cs:(s_ + 1) * m * cs],
                                    np.stack(O.encode("rs", k, m, [data[(s_ * k + j) * cs:(s_ * k + j + 1) * cs].copy()
                                                                   for j in range(k)], cs)).reshape(-1))
                     for s_ in (0, n - 1))
        code = np.concatenate([data.reshape(n, k, cs), par.reshape(n, m, cs)], axis=1)
        buf = code.reshape(-1).copy()
        present = 0b111100
        probe = L.ref_decode_batch_mt(h, buf.ctypes.data, n, present, 1, 1)
        dp = max(1, int(seconds / max(probe, 1e-6)))
        log("configs[0]: reference RS(4,2)@4 KiB decode {0,1}, %d stripes x %d passes on 1 thread" % (n, dp))
        dt = L.ref_decode_batch_mt(h, buf.ctypes.data, n, present, 1, dp)
        dec_ok = dt > 0 and bool(np.array_equal(buf.reshape(n, k + m, cs), code))
    finally:
        L.ref_destroy(h)
    return {"kind": "reference", "unit": "GiB/s", "cores": 1,
            "encode_value": round(ep * n * k * cs / et / 2**30, 4),
            "decode_value": round(dp * n * k * cs / dt / 2**30, 4) if dt > 0 else None,
            "sample": "%d stripes x %d / %d passes through MemEC's own Coding::encode(index 1) / Coding::decode "
                      "(erasures {0,1}), compiled from the reference sources (oracle/_ref), one thread, as "
                      "performance.cc" % (n, ep, dp),
            "encode_matches_oracle": bool(enc_ok), "decode_restores_codewords": dec_ok, "cpu_model": cpu_model()}


def cpu_baseline_reference_update(fam, k, m, cs, j, threads):
    """kind "reference" for the delta path: MemEC's own calls as each parity
    server makes them (parity_chunk_buffer.cc:342-353, 387-393) — per
    stripe and parity index i, Coding::encode over Coding::zeros except
    column j into a cleared chunk, then Coding::bitwiseXOR into parity i
    (oracle/ref_shim.cc ref_update_batch_mt).  Checked against the oracle:
    parity of (old data + delta) = old parity XOR parity delta (linearity)."""
    import numpy as np
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import _oracle as O

    sample = cpu_sample(k, m, cs, threads)
    delta = O.fill(sample * cs, 5)
    par0 = O.fill(sample * m * cs, 6)
    par = par0.copy()

    applied = np.zeros(sample, np.int64)  # delta applications per stripe, every call counted

    def run(L, h, passes, n, t):
        applied[:n] += passes
        return L.ref_update_batch_mt(h, delta.ctypes.data, par.ctypes.data, j, n, t, passes)
    r = ref_baseline(fam, k, m, cs, threads, sample, run, label="update")
    if r is None:
        return None
    probe, passes, dt = r
    # every application XORs the same parity delta: an odd count leaves
    # par0 ^ dpar, an even one par0
    dz = [np.zeros(cs, np.uint8)] * k
    ok = True
    for s_ in (0, sample - 1):
        cols = list(dz)
        cols[j] = delta[s_ * cs:(s_ + 1) * cs].copy()
        dpar = np.stack(O.encode(fam, k, m, cols, cs)).reshape(-1)
        want = par0[s_ * m * cs:(s_ + 1) * m * cs] ^ (dpar if applied[s_] % 2 else 0)
        ok = ok and bool(np.array_equal(par[s_ * m * cs:(s_ + 1) * m * cs], want))
    return {"value": round(passes * sample * cs / dt / 2**30, 4), "unit": "GiB/s (delta bytes)", "cores": threads,
            "kind": "reference",
            "sample": "%d stripes x %d passes: per stripe and parity index, MemEC's own Coding::encode over "
                      "Coding::zeros + the delta column into a cleared chunk, then Coding::bitwiseXOR into the "
                      "parity, as each parity server runs it (oracle/_ref), %d worker threads"
                      % (sample, passes, threads),
            "single_thread_value": round(sample * cs / probe / 2**30, 4), "matches_oracle": ok,
            "cpu_model": cpu_model()}


def cpu_baseline_decode(fam, k, m, cs, erased, codewords, threads):
    """Oracle decode (jerasure_matrix_decode / schedule decode restated,
    decoding matrix rebuilt per stripe as the reference does per call) on a
    bounded sample of GPU-encoded stripes with the same erasures; the
    rebuilt chunks are checked against the codewords."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import numpy as np
    import _oracle as O

    sample = codewords.shape[0]
    buf = np.ascontiguousarray(codewords).reshape(-1).copy()
    view = buf.reshape(sample, k + m, cs)
    view[:, erased] = 0
    per = k * cs
    p = cpu_parallelism(threads, host_cores()[0], sample)
    log("cpu_baseline decode: port, %d stripes on %d threads" % (sample, threads))
    t0 = time.perf_counter()
    O.decode_batch_mt(fam, k, m, cs, buf, p, erased, 1)
    single = p * per / (time.perf_counter() - t0) / 2**30
    passes = 0
    t0 = time.perf_counter()
    while True:
        rc = O.decode_batch_mt(fam, k, m, cs, buf, sample, erased, threads)
        passes += 1
        t_total = time.perf_counter() - t0
        if rc != 0 or t_total * p >= CPU_WORK_S[0] or passes >= 64:
            break
    value = passes * sample * per / t_total / 2**30
    return {"value": round(value, 4), "unit": "GiB/s", "cores": threads, "kind": "port",
            "sample": "%d stripes x %d passes, erasures %s, oracle/oracle.c orc_decode_batch_mt (decoding "
                      "matrix per stripe, scalar 256x256 table / packet XOR), %d threads, disjoint stripes"
                      % (sample, passes, erased, threads),
            "single_thread_value": round(single, 4),
            "matches_gpu": bool(rc == 0 and np.array_equal(view, codewords)), "cpu_model": cpu_model()}


def cpu_baseline_update(fam, k, m, cs, j, threads):
    """The reference's delta path on the CPU: Coding::encode over the k
    columns with Coding::zeros everywhere but column j (the plugin reads and
    multiplies the zero chunks too, rscoding.cc:51-95), then
    Coding::bitwiseXOR of the result into the parity (coding.cc:88-118,
    parity_chunk_buffer.cc:387-393); threads on disjoint stripes."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import numpy as np
    import _oracle as O

    sample = cpu_sample(k, m, cs, threads)
    p = cpu_parallelism(threads, host_cores()[0], sample)
    log("cpu_baseline update: port, %d stripes on %d threads" % (sample, threads))
    data = np.zeros((sample, k, cs), np.uint8)
    data[:, j] = O.fill(sample * cs, 5).reshape(sample, cs)
    data = data.reshape(-1)
    delta_par = np.zeros(sample * m * cs, np.uint8)
    parity = O.fill(sample * m * cs, 6)
    passes = 0
    t0 = time.perf_counter()
    while True:
        O.encode_batch_mt(fam, k, m, cs, data, delta_par, sample, threads)
        np.bitwise_xor(parity, delta_par, out=parity)
        passes += 1
        t_total = time.perf_counter() - t0
        if t_total * p >= CPU_WORK_S[0] or passes >= 64:
            break
    value = passes * sample * cs / t_total / 2**30
    return {"value": round(value, 4), "unit": "GiB/s (delta bytes)", "cores": threads, "kind": "port",
            "sample": "%d stripes x %d passes: orc_encode_batch_mt over the zero-padded delta stripe + XOR "
                      "into parity (numpy), %d threads" % (sample, passes, threads),
            "matches_gpu": None, "cpu_model": cpu_model()}


# ---- parity pins: sampled GPU outputs against the reference itself ----------
# Every config the bench times is checked here, outside the timed region, on
# stripes spread over the whole batch, against oracle/_ref (MemEC's own
# Coding::encode / Coding::decode compiled from the reference sources; the
# oracle port when that library did not travel) — the reference's checker
# re-encodes and memcmps the same way (test/common/coding/checker.cc:132-164).
# Decode batches also carry random NON-codeword stripes: their "rebuilt"
# chunks depend on exactly which survivors and which decoding matrix the
# decoder uses (jerasure.c:98-126, 167-268), so equality there pins the
# survivor choice, which a round trip of codewords cannot.
REF_VS = "oracle/_ref (MemEC Coding::%s compiled from the reference sources)"
PORT_VS = "oracle/oracle.c (restatement; oracle/_ref absent)"
# ISA-L families: the restatement of ec_encode_data_base / the plugin's
# decode steps, itself pinned to MemEC's USE_ISAL plugin (oracle/_ref/
# libmemec_ref_isal.so) by the committed fixtures (tests/test_oracle.py)
ISAL_VS = "oracle/oracle.c (ISA-L restatement, pinned to MemEC's USE_ISAL plugin by tests/golden)"
PARITY_BYTES = 192 << 20  # stripe bytes per sampled set


def parity_count(k, m, cs):
    """Stripes per sampled set: ~192 MiB of stripe bytes, 4 to 64."""
    return int(max(4, min(64, PARITY_BYTES // ((k + m) * cs))))


def spread(lo, hi, n):
    """Up to n distinct indices spread evenly over [lo, hi), both ends
    included."""
    n = max(0, min(n, hi - lo))
    if n <= 1:
        return [lo] if n == 1 else []
    return sorted({lo + (hi - 1 - lo) * i // (n - 1) for i in range(n)})


def ref_encode(fam, k, m, cs, data, threads=1):
    """data [n][k][cs] uint8 -> (the reference's parity [n][m][cs], source)."""
    import numpy as np
    data = np.ascontiguousarray(data)
    n = data.shape[0]
    par = np.zeros((n, m, cs), np.uint8)
    L = _ref_lib() if fam in ("rs", "cauchy") else None
    h = L.ref_instantiate(4 if fam == "rs" else 7, k, m, cs) if L is not None else None
    if h:
        try:
            L.ref_encode_batch_mt(h, data.ctypes.data, par.ctypes.data, n, max(1, min(threads, n)), 1)
        finally:
            L.ref_destroy(h)
        return par, REF_VS % "encode"
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import _oracle as O
    for s_ in range(n):
        par[s_] = np.stack(O.encode(fam, k, m, [data[s_, j].copy() for j in range(k)], cs))
    return par, PORT_VS if fam in ("rs", "cauchy") else ISAL_VS


def ref_decode(fam, k, m, cs, stripes, erased, threads=1):
    """stripes [n][k+m][cs] (the erased chunks' bytes are ignored: cleared
    first, as server_peer_res_worker.cc:818-828 clears them) -> (the
    reference's rebuilt stripes, source)."""
    import numpy as np
    buf = np.ascontiguousarray(stripes).copy()
    n = buf.shape[0]
    buf[:, erased] = 0
    present = sum(1 << i for i in range(k + m) if i not in erased)
    L = _ref_lib() if fam in ("rs", "cauchy") else None
    h = L.ref_instantiate(4 if fam == "rs" else 7, k, m, cs) if L is not None else None
    if h:
        try:
            rc = L.ref_decode_batch_mt(h, buf.ctypes.data, n, present, max(1, min(threads, n)), 1)
        finally:
            L.ref_destroy(h)
        if rc < 0:
            raise RuntimeError("reference decode returned false")
        return buf, REF_VS % "decode"
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import _oracle as O
    for s_ in range(n):
        chunks = [buf[s_, i].copy() for i in range(k + m)]
        if O.decode(fam, k, m, chunks, erased, cs) != 0:
            raise RuntimeError("oracle decode failed")
        buf[s_] = np.stack(chunks)
    return buf, PORT_VS if fam in ("rs", "cauchy") else ISAL_VS


def _rows(t, idx):
    """Stripes idx of a [n, ...] CUDA tensor as a numpy array."""
    import torch
    return t[torch.tensor(idx, dtype=torch.long, device=t.device)].cpu().numpy()


def check_encode(fam, k, m, cs, data, parity, threads=1):
    """Sampled stripes of a GPU encode (data [n][k][cs], parity [n][m][cs]
    CUDA tensors) against the reference's encode of the same stripes."""
    import numpy as np
    idx = spread(0, data.shape[0], parity_count(k, m, cs))
    want, vs = ref_encode(fam, k, m, cs, _rows(data, idx), threads)
    return {"vs": vs, "stripes": len(idx), "equal": bool(np.array_equal(_rows(parity, idx), want)),
            "sample": "%d stripes spread over [0, %d)" % (len(idx), data.shape[0])}


def plant_noncodewords(st, k, m, cs, seed):
    """Before a decode: overwrite stripes spread over the second half of
    `st` ([n][k+m][cs] CUDA tensor of codewords) with random bytes in every
    chunk, and keep host copies of those and of codeword stripes spread
    over the first half.  Returns the record check_decode needs."""
    import torch
    n = st.shape[0]
    cnt = parity_count(k, m, cs)
    nc = spread(n // 2, n, cnt) if n >= 2 else []
    cw = spread(0, max(1, n // 2), cnt)
    rec = {"nc": nc, "cw": cw, "cw_np": _rows(st, cw), "nc_np": None}
    if nc:
        from memec_amd import fill_random
        noise = torch.empty(len(nc), k + m, cs, dtype=torch.uint8, device=st.device)
        if st.is_cuda:
            fill_random(noise, seed)
        else:  # CPU tests of this harness (tests/test_bench_baseline.py)
            noise.copy_(torch.randint(0, 256, noise.shape, dtype=torch.uint8,
                                      generator=torch.Generator().manual_seed(seed)))
        st[torch.tensor(nc, dtype=torch.long, device=st.device)] = noise
        rec["nc_np"] = noise.cpu().numpy()
    return rec


def check_decode(fam, k, m, cs, st, erased, rec, threads=1):
    """After a GPU decode of `st` (in place): the sampled codeword and
    non-codeword stripes, whole, against the reference's decode of the
    same stripes with the same erasures."""
    import numpy as np
    eq, vs = True, None
    for idx, before in ((rec["cw"], rec["cw_np"]), (rec["nc"], rec["nc_np"])):
        if not idx:
            continue
        want, vs = ref_decode(fam, k, m, cs, before, erased, threads)
        eq = eq and bool(np.array_equal(_rows(st, idx), want))
    return {"vs": vs, "codeword_stripes": len(rec["cw"]), "non_codeword_stripes": len(rec["nc"]),
            "erased": list(erased), "equal": eq,
            "sample": "codewords spread over the first half of %d stripes, random non-codewords over the second"
                      % st.shape[0]}


def restore_noncodewords(st, saved, erased, rec):
    """`saved` holds the erased chunks of the original codewords: the
    non-codeword stripes' chunks are replaced by the GPU's own output there,
    so a whole-batch round-trip check covers every other stripe."""
    import torch
    if rec["nc"]:
        t = torch.tensor(rec["nc"], dtype=torch.long, device=st.device)
        saved[t] = st[t][:, erased]


def twin_rate(codec, step, alg_bytes, reps=5):
    """The same launch with every GF(2^8) product a plain XOR
    (mec_set_probe): best of `reps` launches, GB/s of the same algorithmic
    bytes.  The outputs are garbage afterwards.  None for Cauchy-RS."""
    import torch
    if codec.family == "cauchy":
        return None
    codec.set_probe(True)
    try:
        step()
        torch.cuda.synchronize()
        best = None
        for _ in range(reps):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            step()
            e1.record()
            e1.synchronize()
            ms = e0.elapsed_time(e1)
            best = ms if best is None else min(best, ms)
    finally:
        codec.set_probe(False)
    return alg_bytes / (best * 1e-3) / 1e9


def box_info(dev):
    """Which box this ran on, for box-to-box comparisons (the
    configs[4] decode runs in one of two modes): the device's UUID from
    torch, and clocks / firmware / VBIOS from rocm-smi run as a child
    process (None fields if it is absent or slow)."""
    import subprocess
    import torch
    p = torch.cuda.get_device_properties(dev)
    info = {"gpu_uuid": str(getattr(p, "uuid", "")), "name": p.name, "cus": p.multi_processor_count}
    # not under a profiler: its preloaded library initialises the GPU in
    # every process it starts, and rocm-smi's #!/usr/bin/env launcher then
    # re-execs (refused on the GPU boxes)
    if any(k.startswith(("ROCPROF", "ROCP_")) for k in os.environ) or "rocprof" in os.environ.get("LD_PRELOAD", ""):
        info["smi_error"] = "skipped under rocprofv3"
        return info
    try:
        out = subprocess.run(["rocm-smi", "--showclocks", "--showfwinfo", "--showvbios", "--json"],
                             capture_output=True, text=True, timeout=30)
        cards = json.loads(out.stdout)
        cards = {c: v for c, v in cards.items() if c.startswith("card")}
        info["smi_cards"] = len(cards)
        if cards:
            v = cards[sorted(cards)[0]]
            keep = ("mclk", "sclk", "fclk", "socclk", "vbios", "smc", "psp sos", "mec", "rlc", "sdma", "ta ras")
            info["smi"] = {k: x for k, x in v.items() if any(t in k.lower() for t in keep)}
    except Exception as exc:  # informational only
        info["smi_error"] = repr(exc)[:200]
    return info


def cpu_model():
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return None


def load_traffic(cfg_name, stripes):
    """PMC-measured HBM bytes per launch and where they come from: NOT
    measured in this run, but read from profiles/pmc_<cfg>.json, written by
    tools/pmc_summary.py from separate rocprofv3 FETCH_SIZE / WRITE_SIZE
    passes of this bench at the config's default stripe count (the file
    names its round).  (None, reason) for other sizes or no file."""
    path = os.path.join(ROOT, "profiles", "pmc_%s.json" % cfg_name)
    if not os.path.exists(path):
        return None, "no PMC profile for this config"
    if stripes != CONFIGS[cfg_name][4]:
        return None, "PMC profile is for %d stripes, not %d" % (CONFIGS[cfg_name][4], stripes)
    try:
        with open(path) as f:
            j = json.load(f)
    except Exception as exc:
        return None, "unreadable PMC profile: %r" % exc
    tag = j.get("round") or j.get("source", "").rpartition("tag ")[2] or "untagged"
    return j.get("hbm_bytes_per_launch"), ("profiles/pmc_%s.json (%s; rocprofv3 FETCH_SIZE + WRITE_SIZE passes, "
                                          "gfx950-corrected; not measured in this run)" % (cfg_name, tag))


def under_profiler():
    """True inside a rocprofv3 run (its tool library is preloaded), where
    the live PMC passes below would nest one profiler in another."""
    return "rocprof" in os.environ.get("LD_PRELOAD", "") or any(k.startswith("ROCPROF") for k in os.environ)


def wants_live_pmc(world, disabled):
    """Live PMC passes only for the plain single-process run (no launcher,
    no profiler around it, not turned off by --no-pmc-live or
    MEC_BENCH_PMC_LIVE=0): the child passes must start before this process
    touches the GPU, and a multi-rank job leaves the counters to N = 1."""
    return (world < 2 and "WORLD_SIZE" not in os.environ and not disabled and not under_profiler()
            and os.environ.get("MEC_BENCH_PMC_LIVE", "1") != "0")


def pmc_per_launch(path, counter):
    """Counter average per launch of the dominant coding kernel in a
    rocprofv3 --pmc CSV (the kernel launched most often; fills and the XOR
    twin excluded), as tools/pmc_summary.py."""
    import csv
    by_name = {}
    with open(path) as f:
        for row in csv.DictReader(f):
            name = row["Kernel_Name"]
            if row["Counter_Name"] != counter or re.search(r"gf8_kernel<\d+, \d+, (true|false), 2,", name):
                continue
            if "gf8_kernel" in name or "gf8_mg_kernel" in name or "bm_kernel" in name:
                by_name.setdefault(name, []).append(float(row["Counter_Value"]))
    if not by_name:
        return None, None
    name = max(by_name, key=lambda n: len(by_name[n]))
    return sum(by_name[name]) / len(by_name[name]), name


def live_traffic(cfg_name, stripes, timeout=120):
    """HBM bytes per launch of this config's coding kernel, measured in this
    run: two child processes of this script, each under `rocprofv3 --pmc`
    with one counter (FETCH_SIZE, then WRITE_SIZE; separate passes, as
    MI355X_MICROARCH.md prescribes), started before this process touches
    the GPU.  gfx950 correction: read bytes = 2 x FETCH_SIZE KiB (a wide
    streaming read is counted at half), write bytes = WRITE_SIZE KiB.
    Returns (bytes, detail) or (None, reason); never raises."""
    import shutil
    import signal
    import subprocess
    import tempfile
    exe = shutil.which("rocprofv3") or ("/opt/rocm/bin/rocprofv3" if os.path.exists("/opt/rocm/bin/rocprofv3") else None)
    if not exe:
        return None, "rocprofv3 not found"
    kib = {}
    kernel = None
    with tempfile.TemporaryDirectory(prefix="mec_pmc_") as tmp:
        for counter in ("FETCH_SIZE", "WRITE_SIZE"):
            d = os.path.join(tmp, counter)
            cmd = [exe, "--pmc", counter, "--output-format", "csv", "-d", d, "-o", "run", "--", sys.executable,
                   os.path.abspath(__file__), "--config", cfg_name, "--stripes", str(stripes), "--steps", "3",
                   "--warmup", "1", "--no-cpu-baseline", "--no-extra-configs", "--no-ceiling", "--no-secondary",
                   "--no-pmc-live"]
            try:
                with open(os.path.join(tmp, counter + ".log"), "w") as log:
                    p = subprocess.Popen(cmd, stdout=log, stderr=subprocess.STDOUT, start_new_session=True)
                    try:
                        rc = p.wait(timeout=timeout)
                    except subprocess.TimeoutExpired:
                        os.killpg(p.pid, signal.SIGKILL)
                        p.wait()
                        return None, "rocprofv3 %s pass timed out after %d s" % (counter, timeout)
            except OSError as exc:
                return None, "rocprofv3 %s pass did not start: %r" % (counter, exc)
            if rc != 0:
                return None, "rocprofv3 %s pass exited %d" % (counter, rc)
            path = os.path.join(d, "run_counter_collection.csv")
            if not os.path.exists(path):
                return None, "rocprofv3 %s pass wrote no counter CSV" % counter
            kib[counter], kernel = pmc_per_launch(path, counter)
            if kib[counter] is None:
                return None, "no coding kernel in the %s pass" % counter
    rd, wr = 2 * kib["FETCH_SIZE"] * 1024, kib["WRITE_SIZE"] * 1024
    return rd + wr, {"read_bytes": rd, "write_bytes": wr, "kernel": kernel,
                     "source": "live: two child runs of this config (%d stripes, 3 steps) under rocprofv3 --pmc "
                               "FETCH_SIZE / --pmc WRITE_SIZE, started before this process touched the GPU; read = "
                               "2 x FETCH_SIZE KiB (gfx950 wide-stream halving), write = WRITE_SIZE KiB" % stripes}


def launcher_cmd(argv, gpus, port, python=None):
    """The command that starts `gpus` rank processes of this script (one per
    GPU) when bench.py is run as `python bench.py --gpus N` without a
    launcher: torch.distributed.run on 127.0.0.1 with the same arguments.
    The parent never touches the GPU; it waits and exits with the launcher's
    status."""
    return [python or sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
            "--nproc-per-node=%d" % gpus, "--master-addr=127.0.0.1", "--master-port=%d" % port,
            os.path.abspath(__file__)] + list(argv)


def _free_port():
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def spawn_ranks(argv, gpus):
    """Run the N-rank job as a child process (no exec: the parent has not
    initialised the GPU, but a child keeps the rule simple) and return its
    exit status."""
    import subprocess
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    return subprocess.call(launcher_cmd(argv, gpus, _free_port()), env=env)


def host_cores():
    """CPU threads the CPU baseline may use on this host: the affinity mask,
    capped by a cgroup CPU quota when one is set (the GPU box hands each GPU a
    share of a larger machine, and nproc / os.cpu_count() show the whole
    machine there).  Returns (threads, details)."""
    nproc = os.cpu_count() or 1
    try:
        aff = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        aff = nproc
    quota = None
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, period = f.read().split()[:2]
        if q != "max":
            quota = int(q) / int(period)
    except (OSError, ValueError):
        pass
    threads = aff
    if quota:
        threads = max(1, min(aff, int(quota + 0.5)))
    return threads, {"nproc": nproc, "affinity": aff, "cgroup_cpu_quota": quota}


def probe_warmup(step, sync):
    """Untimed warmup steps for >= 0.3 s of work (at least 3), sized from one
    probe step after a first, cold one."""
    step()
    sync()
    t0 = time.perf_counter()
    step()
    sync()
    return int(min(2000, max(3, 0.3 / max(time.perf_counter() - t0, 1e-5))))


# BASELINE configs measured beside the default line (configs[1] encode +
# configs[2] decode), so that the driver's 1/2/4/8-GPU runs of the default
# command record every GPU config north_star asks for: configs[3] at its
# per-GPU batch (weak) and configs[4] encode + decode as the fixed global
# batch of 32768 stripes sharded over the ranks (strong), as BASELINE states.
EXTRA_CONFIGS = (("configs[0]", "rs42", None), ("configs[3]", "rs8_small", None), ("configs[4]", "crs_enc", 32768))
# encode configs whose decode twin is timed too (the others verify a decode untimed)
DECODE_TWINS = {"crs_enc": "crs_dec", "rs42": "rs42_dec"}


def measure_extra(name, strong_global, steps, rank, world, dev, dist, all_ranks_ok):
    """One BASELINE config with its own warmup, the main line's barrier +
    max-over-ranks timing, parity pins against the reference (sampled
    encode stripes; codeword and non-codeword decode stripes) and a
    verified decode: the timed twin decode for configs[4], an untimed
    decode of the first stripes for configs[3]."""
    import torch
    from memec_amd import Codec, fill_random
    from memec_amd.shard import shard_range, timed_steps

    fam, k, m, cs, stripes, op, _ = CONFIGS[name]
    if strong_global:
        s0, s1 = shard_range(strong_global, rank, world)
        stripes, global_stripes = s1 - s0, strong_global
    else:
        global_stripes = stripes * world
    codec = Codec(fam, k, m, cs, device=dev.index)
    data = torch.empty(stripes, k, cs, dtype=torch.uint8, device=dev)
    fill_random(data, 0x4D454D4543 + 17 * (rank + 1))
    parity = torch.empty(stripes, m, cs, dtype=torch.uint8, device=dev)
    d = dist if dist.is_initialized() else None

    def run(step, alg):
        warm = probe_warmup(step, torch.cuda.synchronize)
        ev = (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
        wall, kern = timed_steps(step, steps, warm, sync=torch.cuda.synchronize, dist=d, events=ev)
        return {"value": round(global_stripes * k * cs * steps / wall / 2**30, 3), "unit": "GiB/s",
                "steps": steps, "warmup": warm, "ms_per_step": round(wall / steps * 1e3, 4),
                "kernel_ms": round(kern, 4), "achieved_GBps": round(alg / (kern * 1e-3) / 1e9, 1),
                "frac": round(alg / (kern * 1e-3) / 1e9 / HBM_PEAK_GBS, 4)}

    def pin(rec):
        rec["equal"] = all_ranks_ok(rec["equal"])
        rec["ranks"] = world
        return rec

    res = {"workload": workload_name(name, stripes, bool(strong_global), global_stripes),
           "scaling": "strong" if strong_global else "weak", "stripes_per_gpu": stripes,
           "global_stripes": global_stripes}
    enc_step = lambda: codec.encode(data, parity)  # noqa: E731
    res.update(run(enc_step, (k + m) * cs * stripes))
    res["parity"] = pin(check_encode(fam, k, m, cs, data, parity))
    twin = DECODE_TWINS.get(name)
    erased = CONFIGS[twin][6] if twin else list(range(m))
    n = stripes if twin else min(stripes, 4096)
    st = torch.empty(n, k + m, cs, dtype=torch.uint8, device=dev)
    st[:, :k] = data[:n]
    st[:, k:] = parity[:n]
    saved = st[:, erased].clone()
    rec = plant_noncodewords(st, k, m, cs, 0x5EED + rank)
    st[:, erased] = 0
    present = sum(1 << i for i in range(k + m) if i not in erased)
    dec_step = lambda: codec.decode(st, present)  # noqa: E731
    if twin:
        dec = run(dec_step, (k + len(erased)) * cs * n)
        dec["workload"] = workload_name(twin, n, bool(strong_global), global_stripes)
        dec["erased"] = erased
    else:
        dec_step()
        torch.cuda.synchronize()
    dpin = pin(check_decode(fam, k, m, cs, st, erased, rec))
    restore_noncodewords(st, saved, erased, rec)
    ok = all_ranks_ok(torch.equal(st[:, erased], saved))
    if twin:
        dec["parity"] = dpin
        dec["verified"] = ok
        res["decode"] = dec
    else:
        res["decode_parity"] = dpin
        res["verified"] = ok
        res["verification"] = ("decode of erasures %s restores the first %d encoded stripes (the %d planted "
                               "non-codewords checked against the reference instead)" % (erased, n, len(rec["nc"])))
    # the same launches with the arithmetic removed (byte-wise only): what
    # this memory stream reaches without the GF(2^8) work, live on this box
    tw = twin_rate(codec, enc_step, (k + m) * cs * stripes)
    if tw:
        res["xor_twin_GBps"] = round(tw, 1)
        res["frac_of_xor_twin"] = round(res["achieved_GBps"] / tw, 4)
    del data, parity, st, saved
    codec.close()
    torch.cuda.empty_cache()
    return res


def memory_plan(config, stripes, world, rank0, extras, ceiling, strong=False):
    """Device bytes each phase of this process holds at once (torch
    tensors; libmec's own tables are KiBs), for `stripes` per rank of
    `config`: the timed launch's buffers, the decode twin's stripe copy and
    saved erasures, rank 0's live reference streams (3 x 8 GiB of mec_xor
    buffers), and each extra config beside the main buffers (which stay
    allocated).  The driver's 8-GPU line runs one rank per GPU, so its peak
    must fit one device."""
    fam, k, m, cs, _, op, erased = CONFIGS[config]
    S = stripes
    phases = {}
    if op == "encode":
        base = (k + m) * cs * S
        phases["timed"] = base
        twin = {"rs_enc": "rs_dec", "crs_enc": "crs_dec", "rs42": "rs42_dec"}.get(config)
        if twin:
            e = len(CONFIGS[twin][6])
            phases["decode_twin"] = base + (k + m) * cs * S + e * cs * S
    elif op == "update":
        base = (1 + m) * cs * S
        phases["timed"] = base + (k + m) * cs * min(S, 256)
    else:
        base = (k + m) * cs * S + len(erased) * cs * S  # stripes + saved erasures
        phases["timed"] = base + k * cs * S  # the data copy while the stripes are built
    if ceiling and rank0:
        phases["reference_streams"] = base + 3 * (8 << 30)
    if extras:
        for label, name, strong_global in EXTRA_CONFIGS:
            _, k2, m2, cs2, s2, _, _ = CONFIGS[name]
            if strong_global:
                s2 = strong_global // world + (1 if strong_global % world else 0)
            twin2 = DECODE_TWINS.get(name)
            n = s2 if twin2 else min(s2, 4096)
            e2 = len(CONFIGS[twin2][6]) if twin2 else m2
            phases[label] = base + (k2 + m2) * cs2 * s2 + (k2 + m2) * cs2 * n + e2 * cs2 * n
    return {"peak_bytes": max(phases.values()), "phases": phases}


def runs_cpu_legs(rank, world, disabled):
    """Whether this rank times the reference CPU path (cpu_baseline, the
    decode twin's baseline, configs[0]'s reference_cpu): rank 0 at every N —
    the 2/4/8-GPU lines carry the baseline as the 1-GPU line does — after
    every rank's GPU legs (main's barrier), never inside a timed region."""
    del world  # every world size
    return rank == 0 and not disabled


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=None,
                    help="untimed warmup steps (default: enough steps for >= 0.3 s of work, at least 3, "
                         "so short configs run at a settled clock)")
    ap.add_argument("--config", default="rs_enc", choices=sorted(CONFIGS))
    ap.add_argument("--stripes", type=int, default=0, help="override stripes per GPU")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-secondary", action="store_true",
                    help="encode configs: skip the decode twin measurement (configs[2] for configs[1])")
    ap.add_argument("--no-ceiling", action="store_true", help="skip the live reference streams (the XOR twin of the timed launch, mec_xor)")
    ap.add_argument("--no-extra-configs", action="store_true",
                    help="default run: skip configs[3] and configs[4] beside the configs[1]/[2] line")
    ap.add_argument("--extra-configs", action="store_true",
                    help="measure configs[3] and configs[4] even with --stripes (multi-rank rehearsals)")
    ap.add_argument("--cpu-threads", type=int, default=0)
    ap.add_argument("--e2e", action="store_true", help="also time the host-memory (PCIe) batch encode")
    ap.add_argument("--strong", action="store_true",
                    help="--stripes is the global batch, sharded over ranks (default: per-GPU batch, weak scaling)")
    ap.add_argument("--no-pmc-live", action="store_true",
                    help="read roofline.traffic from profiles/pmc_<config>.json instead of measuring it "
                         "(rocprofv3 --pmc child passes before the run; N = 1 only)")
    ap.add_argument("--dist-check", action="store_true", help=argparse.SUPPRESS)
    args = ap.parse_args()

    from memec_amd.shard import dist_env, max_over_ranks, shard_range, timed_steps

    world, rank, local = dist_env()
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        # `python bench.py --gpus N` without a launcher: start the N ranks
        # before anything touches the GPU, wait, and return their status
        sys.exit(spawn_ranks(sys.argv[1:], args.gpus))
    if world != args.gpus:
        sys.exit("bench.py: --gpus %d but the launcher started %d ranks" % (args.gpus, world))

    import torch
    import torch.distributed as dist

    if args.dist_check:  # launcher rehearsal without a GPU (tests/test_bench_launcher.py)
        if world > 1:
            dist.init_process_group("gloo")
        ranks = [None] * world
        if world > 1:
            dist.all_gather_object(ranks, (rank, local, os.getpid()))
            dist.destroy_process_group()
        else:
            ranks = [(rank, local, os.getpid())]
        if rank == 0:
            print(json.dumps({"dist_check": True, "n_gpus": args.gpus, "world_size": world, "ranks": ranks}),
                  flush=True)
        return

    from memec_amd import Codec, fill_random, set_knob

    # wide codes (more than 4 outputs): compile a matrix's bit-sliced kernel
    # at its first call, which the untimed cold step makes, instead of in
    # the background while warmup runs the one-pass kernel (the library's
    # default, MEC_BITSLICE=1), so the timed steps and the XOR twin run the
    # kernel a server runs once the compile is done
    if "MEC_BITSLICE" not in os.environ:
        set_knob("MEC_BITSLICE", "2")

    # roofline.traffic measured live: PMC passes in child processes, before
    # this process touches the GPU (N = 1, plain runs, not under a profiler)
    pmc_live = None
    if wants_live_pmc(world, args.no_pmc_live):
        pmc_live = live_traffic(args.config, args.stripes or CONFIGS[args.config][4])
        if pmc_live[0] is None:
            print("bench: live PMC traffic unavailable (%s); using the committed profile" % pmc_live[1],
                  file=sys.stderr, flush=True)

    # MEC_BENCH_DIST_BACKEND=gloo rehearses the multi-rank harness on fewer
    # GPUs than ranks (ranks share devices round-robin); the real run is
    # one rank per GPU over RCCL ("nccl").
    backend = os.environ.get("MEC_BENCH_DIST_BACKEND", "nccl")
    if backend != "nccl":
        local = local % max(1, torch.cuda.device_count())
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    dist_info = None
    # a process group whenever a launcher started the job, one rank included
    # (`torchrun --nproc-per-node 1 bench.py` runs the RCCL init, barriers
    # and max-over-ranks reductions on a one-GPU box); `python bench.py`
    # alone is the plain N=1 run
    use_pg = world > 1 or "WORLD_SIZE" in os.environ
    if use_pg:
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group(backend)
        if dist.get_world_size() != args.gpus:
            raise SystemExit("bench.py: process group has %d ranks, --gpus %d"
                             % (dist.get_world_size(), args.gpus))
        devs = [None] * world
        dist.all_gather_object(devs, local)
        dist_info = {"backend": dist.get_backend(), "world_size": dist.get_world_size(),
                     "rccl": dist.get_backend() == "nccl", "rank_devices": devs}

    def all_ranks_ok(flag):
        """A verification holds only if it held on every rank."""
        if not use_pg:
            return bool(flag)
        bad = max_over_ranks([0.0 if flag else 1.0], dist,
                             device="cpu" if dist.get_backend() == "gloo" else dev)
        return bad[0] == 0.0

    fam, k, m, cs, stripes, op, erased = CONFIGS[args.config]
    if args.stripes:
        stripes = args.stripes
    global_stripes = stripes * world
    if args.strong:  # fixed total batch, partitioned by stripe ranges
        global_stripes = stripes
        s0, s1 = shard_range(stripes, rank, world)
        stripes = s1 - s0
    codec = Codec(fam, k, m, cs, device=local)
    seed = 0x4D454D4543 + rank

    if op == "encode":
        data = torch.empty(stripes, k, cs, dtype=torch.uint8, device=dev)
        fill_random(data, seed)
        parity = torch.empty(stripes, m, cs, dtype=torch.uint8, device=dev)

        def step():
            codec.encode(data, parity)
        alg_bytes = (k + m) * cs * stripes
    elif op == "update":
        j = erased  # the updated data column
        erased = None
        delta = torch.empty(stripes, cs, dtype=torch.uint8, device=dev)
        fill_random(delta, seed + 1)
        parity = torch.zeros(stripes, m, cs, dtype=torch.uint8, device=dev)  # parity of all-zero data
        n_updates = [0]

        def step():
            codec.encode_update(j, delta, parity)
            n_updates[0] += 1
        alg_bytes = (1 + 2 * m) * cs * stripes  # read delta, read + write every parity
    else:
        stripe = torch.empty(stripes, k + m, cs, dtype=torch.uint8, device=dev)
        d = torch.empty(stripes, k, cs, dtype=torch.uint8, device=dev)
        fill_random(d, seed)
        stripe[:, :k] = d
        del d
        codec.encode(stripe[:, :k], stripe[:, k:])
        present = sum(1 << i for i in range(k + m) if i not in erased)
        orig = stripe[:, erased].clone() if stripes * len(erased) * cs <= (24 << 30) else None
        codewords_np = None  # CPU-baseline sample: GPU-encoded stripes before the erasure
        if runs_cpu_legs(rank, world, args.no_cpu_baseline):
            threads_cb = args.cpu_threads or host_cores()[0]
            codewords_np = stripe[:cpu_sample(k, m, cs, threads_cb)].cpu().numpy()
        # random non-codewords planted in the second half pin the survivor
        # choice against the reference (check_decode)
        nc_rec = plant_noncodewords(stripe, k, m, cs, 0x5EED + rank)
        stripe[:, erased] = 0

        def step():
            codec.decode(stripe, present)
        alg_bytes = (k + len(erased)) * cs * stripes

    if args.warmup is None:  # size the warmup from one probe step (after a first, cold one)
        args.warmup = probe_warmup(step, torch.cuda.synchronize)
    ev = (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
    wall, kern_ms = timed_steps(step, args.steps, args.warmup, sync=torch.cuda.synchronize,
                                dist=dist if use_pg else None, events=ev)  # one launch per step

    def pin(rec):
        rec["equal"] = all_ranks_ok(rec["equal"])
        rec["ranks"] = world
        return rec

    # parity pins of the timed launches' outputs (before anything reuses them)
    parity_pin, ok, gpu_parity_np = None, None, None
    if op == "encode":
        parity_pin = pin(check_encode(fam, k, m, cs, data, parity))
        if runs_cpu_legs(rank, world, args.no_cpu_baseline):
            gpu_parity_np = parity[:64].cpu().numpy()
    elif op == "decode":
        parity_pin = pin(check_decode(fam, k, m, cs, stripe, erased, nc_rec))
        if orig is not None:
            restore_noncodewords(stripe, orig, erased, nc_rec)
            ok = all_ranks_ok(torch.equal(stripe[:, erased], orig))
    else:
        # parity started as the parity of all-zero data and received the
        # same delta n times: it must equal the encode of (delta in column
        # j, zeros elsewhere) if n is odd, zero if n is even — checked on
        # the GPU for 256 stripes, and against the reference's encode on
        # stripes spread over the batch
        import numpy as np
        ref = torch.zeros(min(stripes, 256), m, cs, dtype=torch.uint8, device=dev)
        if n_updates[0] % 2:
            dz = torch.zeros(ref.shape[0], k, cs, dtype=torch.uint8, device=dev)
            dz[:, j] = delta[:ref.shape[0]]
            codec.encode(dz, ref)
            del dz
        ok = all_ranks_ok(torch.equal(parity[:ref.shape[0]], ref))
        del ref
        idx = spread(0, stripes, parity_count(k, m, cs))
        dz = np.zeros((len(idx), k, cs), np.uint8)
        if n_updates[0] % 2:
            dz[:, j] = _rows(delta, idx)
        want, vs = ref_encode(fam, k, m, cs, dz)
        parity_pin = pin({"vs": vs, "stripes": len(idx), "equal": bool(np.array_equal(_rows(parity, idx), want)),
                          "sample": "%d stripes spread over [0, %d): parity after %d delta updates vs the "
                                    "reference's encode of the delta stripe" % (len(idx), stripes, n_updates[0])})

    # the metric is encode+decode: an encode config also times its decode
    # twin (configs[2] for configs[1]) on the just-encoded stripes, every
    # rank, same barrier + max-over-ranks timing; reported beside `value`
    secondary = None
    twin = {"rs_enc": "rs_dec", "crs_enc": "crs_dec", "rs42": "rs42_dec"}.get(args.config)
    if op == "encode" and twin and not args.no_secondary:
        derased = CONFIGS[twin][6]
        st = torch.empty(stripes, k + m, cs, dtype=torch.uint8, device=dev)
        st[:, :k] = data
        st[:, k:] = parity
        dcodewords = None  # CPU-baseline sample of the twin: GPU-encoded codewords
        if runs_cpu_legs(rank, world, args.no_cpu_baseline):
            dcodewords = st[:cpu_sample(k, m, cs, args.cpu_threads or host_cores()[0])].cpu().numpy()
        saved = st[:, derased].clone()
        drec = plant_noncodewords(st, k, m, cs, 0x5EED + 7 * rank + 1)
        st[:, derased] = 0
        dpresent = sum(1 << i for i in range(k + m) if i not in derased)
        dstep = lambda: codec.decode(st, dpresent)  # noqa: E731
        dev_ev = (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
        dwall, dkern = timed_steps(dstep, args.steps, args.warmup,
                                   sync=torch.cuda.synchronize, dist=dist if use_pg else None, events=dev_ev)
        dalg = (k + len(derased)) * cs * stripes
        dpin = pin(check_decode(fam, k, m, cs, st, derased, drec))
        restore_noncodewords(st, saved, derased, drec)
        secondary = {"workload": workload_name(twin, stripes, args.strong, global_stripes), "erased": derased,
                     "value": round(global_stripes * k * cs * args.steps / dwall / 2**30, 3), "unit": "GiB/s",
                     "ms_per_step": round(dwall / args.steps * 1e3, 4), "kernel_ms": round(dkern, 4),
                     "achieved_GBps": round(dalg / (dkern * 1e-3) / 1e9, 1),
                     "frac": round(dalg / (dkern * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
                     "parity": dpin,
                     "verified": all_ranks_ok(torch.equal(st[:, derased], saved))}
        if not args.no_ceiling and rank == 0:
            tw = twin_rate(codec, dstep, dalg)
            if tw:
                secondary["xor_twin_GBps"] = round(tw, 1)
                secondary["frac_of_xor_twin"] = round(secondary["achieved_GBps"] / tw, 4)
        del st, saved

    # live reference streams, measured after every output above was checked: the
    # arithmetic-free twin of the timed launch (mec_set_probe: same kernel,
    # launch shape, loads and stores, every GF(2^8) product a plain XOR), and
    # libmec's region XOR (Coding::bitwiseXOR, 2 reads + 1 write per lane)
    # over 3 x 8 GiB, for reference
    twin_gbps, xor_gbps = None, None
    if rank == 0 and not args.no_ceiling:
        twin_gbps = twin_rate(codec, step, alg_bytes)
        if op == "decode":
            step()  # the outputs again (the twin overwrote them)
        from memec_amd import xor as mec_xor
        a = torch.empty(8 << 30, dtype=torch.uint8, device=dev)
        b = torch.empty_like(a)
        out = torch.empty_like(a)
        mec_xor(out, a, b)
        best = None
        for _ in range(5):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            mec_xor(out, a, b)
            e1.record()
            e1.synchronize()
            ms = e0.elapsed_time(e1)
            best = ms if best is None else min(best, ms)
        xor_gbps = 3 * a.numel() / (best * 1e-3) / 1e9
        del a, b, out
        if op == "encode":
            step()  # correct parity again for the e2e leg

    extras = None
    if args.config == "rs_enc" and not args.strong and not args.no_extra_configs and (args.extra_configs or not args.stripes):
        extras = {label: measure_extra(name, strong_global, args.steps, rank, world, dev, dist, all_ranks_ok)
                  for label, name, strong_global in EXTRA_CONFIGS}

    e2e = None
    if args.e2e and rank == 0 and op == "encode":
        import numpy as np
        n = min(stripes, max(8, (4 << 30) // ((k + m) * cs)))
        hd = np.empty((n, k, cs), np.uint8)
        hd[:] = data[:n].cpu().numpy()
        hp = np.empty((n, m, cs), np.uint8)
        from memec_amd import host_register, host_unregister
        res = {}
        for mode in ("pageable", "registered"):
            if mode == "registered":
                host_register(hd)
                host_register(hp)
            codec.encode_host_batch(hd, hp)
            t2 = time.perf_counter()
            reps = 3
            for _ in range(reps):
                codec.encode_host_batch(hd, hp)
            dt = (time.perf_counter() - t2) / reps
            res[mode] = round(n * k * cs / dt / 2**30, 3)
            if mode == "registered":
                host_unregister(hd)
                host_unregister(hp)
        e2e = {"unit": "GiB/s data, host memory in and out (PCIe-inclusive)", "stripes": n,
               "modes": {"pageable": "hipMemcpyAsync H2D -> kernel in HBM -> D2H, two streams",
                         "registered": "mec_host_register: kernel reads/writes host memory over PCIe (zero-copy)"},
               **res}

    # device memory: this run's measured peak on every rank against the plan
    # for this run and for the full-size line with one rank per GPU
    peak = int(torch.cuda.max_memory_allocated(dev))
    peaks = [peak]
    if use_pg:
        peaks = [None] * world
        dist.all_gather_object(peaks, peak)
    with_extras = extras is not None
    mem_plan = None
    if rank == 0:
        full_cfg = CONFIGS[args.config][4]
        mem_plan = {
            "device_bytes": int(torch.cuda.mem_get_info(dev)[1]),
            "measured_peak_bytes_per_rank": peaks,
            "this_run": memory_plan(args.config, stripes, world, True, with_extras, not args.no_ceiling, args.strong),
            "full_size_one_rank_per_gpu": dict(
                memory_plan(args.config, full_cfg, world, True, args.config == "rs_enc", True),
                stripes_per_gpu=full_cfg, world=world),
        }
        mem_plan["full_size_fits"] = mem_plan["full_size_one_rank_per_gpu"]["peak_bytes"] <= mem_plan["device_bytes"]

    # every rank's GPU work (timed legs, pins, verifications) ends here; the
    # CPU legs below run on rank 0 alone, outside every timed region, while
    # the other ranks leave (a rank parked in an RCCL barrier would spin a
    # host core the reference's threads need), as the reference runs its
    # batch benchmark as worker threads on one host
    # (test/common/coding/batch_performance.cc:143-154)
    if use_pg:
        dist.barrier()
    if rank == 0:
        traffic, traffic_src = load_traffic(args.config, stripes)
        traffic_committed = traffic
        traffic_detail = None
        if pmc_live and pmc_live[0] is not None:
            traffic, traffic_detail = pmc_live
            traffic_src = traffic_detail["source"]
        elif pmc_live:
            traffic_src = "%s; live PMC passes unavailable: %s" % (traffic_src, pmc_live[1])
        # data GiB/s: k data chunks per stripe (encode / decode), the one
        # delta chunk per stripe for updates
        value = global_stripes * (cs if op == "update" else k * cs) * args.steps / wall / 2**30
        achieved = alg_bytes / (kern_ms * 1e-3) / 1e9
        line = {
            "metric": METRIC,
            "value": round(value, 3),
            "unit": "GiB/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(wall / args.steps * 1e3, 4),
            "higher_is_better": True,
            "scaling": "strong" if args.strong else "weak",
            "vs_baseline": None,
            "dtype": "u8",
            "data": "synthetic (splitmix64 stripes generated in HBM)",
            "config": {"workload": workload_name(args.config, stripes, args.strong, global_stripes), "family": fam, "k": k, "m": m,
                       "chunk_bytes": cs, "stripes_per_gpu": stripes, "global_stripes": global_stripes,
                       "op": op, "erased": erased, "parallelism": "stripe-sharded x%d" % world},
            "roofline": {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": traffic,
                         "traffic_source": traffic_src,
                         "traffic_over_algorithmic": round(traffic / alg_bytes, 4) if traffic else None,
                         "traffic_read_write": [traffic_detail["read_bytes"], traffic_detail["write_bytes"]]
                         if traffic_detail else None,
                         "traffic_committed_profile": traffic_committed if traffic_detail else None,
                         "algorithmic_bytes_per_launch": alg_bytes, "kernel_ms": round(kern_ms, 4),
                         "xor_twin_GBps": round(twin_gbps, 1) if twin_gbps else None,
                         "frac_of_xor_twin": round(achieved / twin_gbps, 4) if twin_gbps else None,
                         "region_xor_2r1w_GBps": round(xor_gbps, 1) if xor_gbps else None,
                         "frac_of_region_xor": round(achieved / xor_gbps, 4) if xor_gbps else None,
                         "reference_streams": "live, best of 5 each. xor_twin = this launch with every GF(2^8) "
                                              "product a plain XOR (mec_set_probe): same loads, stores and launch "
                                              "shape, so frac_of_xor_twin ~1 says the arithmetic costs nothing; it "
                                              "is not an upper bound (the arithmetic shifts wave timing, and the "
                                              "coding kernel may run up to a few % faster). region_xor_2r1w = "
                                              "mec_xor over 3 x 8 GiB (2 reads + 1 write per lane), a second live "
                                              "read/write stream for box-to-box comparison; the coding kernel runs "
                                              "0.96-1.04x of it, so neither is a hard bound: the bound is "
                                              "peak (spec HBM3E)"},
            "parity": parity_pin,
            "cpu_baseline": None,
        }
        if ok is not None:
            line["decode_verified" if op == "decode" else "update_verified"] = ok
        if dist_info:
            line["dist"] = dist_info
        line["memory_plan"] = mem_plan
        line["box"] = box_info(dev)
        if e2e:
            line["e2e_host_memory"] = e2e
        if extras:
            line["other_configs"] = extras
            if "configs[0]" in extras and runs_cpu_legs(rank, world, args.no_cpu_baseline):
                # configs[0] is the reference's own CPU path: time it here too
                try:
                    extras["configs[0]"]["reference_cpu"] = configs0_reference()
                except Exception as exc:  # report, never fake
                    extras["configs[0]"]["reference_cpu"] = {"error": repr(exc)}
        if secondary:
            line["decode"] = secondary
        if runs_cpu_legs(rank, world, args.no_cpu_baseline):
            threads, host = host_cores()
            threads = args.cpu_threads or threads
            try:
                if op == "encode":
                    port = cpu_baseline(fam, k, m, cs, gpu_parity_np, seed, threads)
                elif op == "update":
                    port = cpu_baseline_update(fam, k, m, cs, j, threads)
                else:
                    port = cpu_baseline_decode(fam, k, m, cs, erased, codewords_np, threads)
                # the compiled reference itself, when oracle/_ref travelled
                if op == "update":
                    ref = cpu_baseline_reference_update(fam, k, m, cs, j, threads)
                else:
                    ref = cpu_baseline_reference(fam, k, m, cs, gpu_parity_np if op == "encode" else None, seed,
                                                 threads, op, erased, codewords_np if op == "decode" else None)
                if secondary is not None and dcodewords is not None:  # the decode twin's reference
                    secondary["cpu_baseline"] = cpu_baseline_reference(fam, k, m, cs, None, seed, threads, "decode",
                                                                       secondary["erased"], dcodewords)
                if ref and "error" not in ref:
                    ref["port"] = {x: port[x] for x in ("value", "single_thread_value", "sample", "matches_gpu")
                                   if x in port}
                    line["cpu_baseline"] = ref
                else:
                    line["cpu_baseline"] = port
            except Exception as exc:  # report, never fake
                line["cpu_baseline"] = {"error": repr(exc)}
            for cb in (line["cpu_baseline"], (secondary or {}).get("cpu_baseline")):
                if cb and "error" not in cb:
                    cb["host"] = dict(host, threads_used=threads)
                    cb["when"] = ("rank 0 of %d, after every rank finished its GPU legs (barrier), other ranks "
                                  "exited; sample from rank 0's stripes" % world)
        print(json.dumps(line), flush=True)
    if use_pg:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
