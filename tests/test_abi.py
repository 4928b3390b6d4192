"""CPU checks of the C ABI: libmec.so loads, exports every symbol declared in
include/mec.h, and its host-side math (matrices, getW rules, error codes)
matches the reference fixtures.  No compute call is made (no GPU here)."""
import ctypes
import os
import re

import numpy as np
import pytest

import _oracle as O
from memec_amd import Codec, MecError, _lib

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _declared_symbols():
    src = open(os.path.join(ROOT, "include", "mec.h")).read()
    return sorted(set(re.findall(r"\b(mec_[a-z_0-9]+)\s*\(", src)))


def test_exports_every_declared_symbol():
    L = _lib.lib()
    declared = _declared_symbols()
    assert len(declared) >= 19
    for name in declared:
        assert hasattr(L, name), name
    assert set(declared) == set(_lib.SYMBOLS)
    assert L.mec_abi_version() == 6


def test_coding_adapter_library_links():
    so = os.path.join(ROOT, "memec_amd", "libmemec_coding.so")
    assert os.path.exists(so)
    L = ctypes.CDLL(so)
    for sym in ("_ZN6Coding11instantiateE12CodingSchemeR12CodingParamsj", "_ZN6Coding10bitwiseXOREPcS0_S0_j"):
        assert hasattr(L, sym), sym


def test_rs_matrices_match_reference(golden):
    meta, _ = golden
    for key in ["4,2", "8,2", "10,4", "12,4", "6,3", "1,1", "16,16", "30,2", "2,30"]:
        k, m = map(int, key.split(","))
        with Codec("rs", k, m, 4096, device=-1) as c:
            assert c.matrix() == meta["rs_matrices"][key], key
            assert c.w == 8 and c.packet_size == 4096


def test_all_rs_matrices(golden):
    meta, _ = golden
    for key, mat in meta["rs_matrices"].items():
        k, m = map(int, key.split(","))
        with Codec("rs", k, m, 64, device=-1) as c:
            assert c.matrix() == mat, key


def test_cauchy_matrices_and_w(golden):
    meta, _ = golden
    for (k, m, cs) in [(12, 4, 65536), (4, 2, 4096), (8, 2, 4096), (4, 2, 96), (20, 4, 320), (20, 4, 96),
                       (20, 4, 112), (20, 4, 64), (10, 4, 1024), (6, 3, 48), (3, 1, 24), (1, 1, 16)]:
        w = O.cauchy_getw(k, m, cs)
        with Codec("cauchy", k, m, cs, device=-1) as c:
            assert c.w == w, (k, m, cs)
            assert c.packet_size == cs // w
            assert c.matrix() == meta["cauchy_matrices"]["%d,%d,%d" % (k, m, w)]["matrix"], (k, m, cs)
            bm = c.bitmatrix()
            assert sum(bm) == meta["cauchy_matrices"]["%d,%d,%d" % (k, m, w)]["bitmatrix_ones"]
            assert bm == O.bitmatrix(k, m, w, c.matrix())


def test_every_cauchy_matrix(golden):
    meta, _ = golden
    for key, rec in meta["cauchy_matrices"].items():
        k, m, w = map(int, key.split(","))
        # pick the smallest chunk size for which getW lands on this w
        cs = None
        for cand in range(w, 8 * 64 + 1, w):
            if O.cauchy_getw(k, m, cand) == w:
                cs = cand
                break
        if cs is None:
            continue
        with Codec("cauchy", k, m, cs, device=-1) as c:
            assert c.matrix() == rec["matrix"], key


def test_isal_matrices(golden):
    meta, _ = golden
    for key, mat in meta["isal_matrices"].items():
        fam, km = key.split("/")
        k, m = map(int, km.split(","))
        with Codec(fam, k, m, 512, device=-1) as c:
            assert c.matrix() == mat, key


def test_reference_parameter_errors():
    # rscoding.cc:26-29: k + m > 32 -> exit(-1); here MEC_EINVAL
    with pytest.raises(MecError) as e:
        Codec("rs", 30, 3, 4096, device=-1)
    assert e.value.code == _lib.MEC_EINVAL
    # rscoding.cc:210-213: chunkSize % w
    with pytest.raises(MecError):
        Codec("rs", 4, 2, 4100, device=-1)
    # cauchy w > 8 unsupported here (reference sizes are multiples of 8, w <= 8)
    with pytest.raises(MecError):
        Codec("cauchy", 20, 4, 9 * 11 * 13, device=-1)
    with pytest.raises(MecError):
        Codec("nope" if False else 9, 4, 2, 4096, device=-1)


def test_host_only_context_refuses_compute():
    with Codec("rs", 4, 2, 4096, device=-1) as c:
        with pytest.raises(MecError) as e:
            c.encode_host([np.zeros(4096, np.uint8)] * 4)
        assert e.value.code == _lib.MEC_ENODEV
        a = np.zeros((6, 4096), np.uint8)
        for call in (lambda: c.encode_batch([a[j].ctypes.data for j in range(4)],
                                            [a[4 + i].ctypes.data for i in range(2)], mem="host"),
                     lambda: c.encode_update_batch([0], [a[0].ctypes.data], [a[4].ctypes.data, 0], mem="host"),
                     lambda: c.decode_batch([a[i].ctypes.data for i in range(6)], [0b111101], mem="host"),
                     lambda: c.set_coalescing(8)):
            with pytest.raises(MecError) as e:
                call()
            assert e.value.code == _lib.MEC_ENODEV


def test_gf8_perm_decomposition_emulated():
    """The device multiplies by splitting each byte into bit fields 0-2, 3-5,
    6-7 and looking each up with v_perm_b32.  Emulate v_perm_b32 (select byte
    s of {S0:S1}, S1 = bytes 0-3) and check every (c, x) product."""
    def perm(s0, s1, sel):
        b = [(s1 >> (8 * i)) & 0xFF for i in range(4)] + [(s0 >> (8 * i)) & 0xFF for i in range(4)]
        return sum(b[(sel >> (8 * i)) & 0xFF] << (8 * i) for i in range(4))

    L = O.lib()
    mul = np.array([[L.orc_gf_mul(a, b, 8) for b in range(256)] for a in range(256)], np.uint32)

    def pack(c, vals):
        return int(sum(int(mul[c][v]) << (8 * i) for i, v in enumerate(vals)))

    xs = np.arange(256, dtype=np.uint32).reshape(64, 4)
    words = (xs[:, 0] | xs[:, 1] << 8 | xs[:, 2] << 16 | xs[:, 3] << 24).tolist()
    for c in range(256):
        t0, t1 = pack(c, [0, 1, 2, 3]), pack(c, [4, 5, 6, 7])
        u0, u1 = pack(c, [0, 8, 16, 24]), pack(c, [32, 40, 48, 56])
        v = pack(c, [0, 64, 128, 192])
        for wi, x in enumerate(words):
            s0, s1, s2 = x & 0x07070707, (x >> 3) & 0x07070707, (x >> 6) & 0x03030303
            got = perm(t1, t0, s0) ^ perm(u1, u0, s1) ^ perm(v, v, s2)
            want = sum(int(mul[c][(x >> (8 * i)) & 0xFF]) << (8 * i) for i in range(4))
            assert got == want, (c, x)


def test_knobs_through_the_api_not_the_environment():
    """Launch-shape knobs are read from the environment once; mec_set_knob
    changes them at run time (no getenv on a launch path) and refuses
    unknown names."""
    import memec_amd
    for name, value in (("MEC_WPC", "12"), ("MEC_SGROUP", "0"), ("MEC_SGROUP", "16:8"), ("MEC_BLOCK", "256"),
                        ("MEC_BM_VW", "2"), ("MEC_GBLOCK", "64"), ("MEC_GWPC", "0"), ("MEC_WINDOWS", "2"),
                        ("MEC_COPY_THREADS", "4"), ("MEC_WIDE", "0"), ("MEC_MG_ROWS", "8")):
        memec_amd.set_knob(name, value)
        memec_amd.set_knob(name, None)
    with pytest.raises(MecError):
        memec_amd.set_knob("MEC_NO_SUCH_KNOB", "1")
    # values outside a knob's accepted set are refused (knobs.cpp kSpecs)
    for name, value in (("MEC_MG_ROWS", "5"), ("MEC_BLOCK", "128"), ("MEC_WPC", "33"), ("MEC_WPC", "1x"),
                        ("MEC_WINDOWS", "0"), ("MEC_SGROUP", "4:7"), ("MEC_BM_VW", "3"), ("MEC_WIDE", "2")):
        with pytest.raises(MecError) as e:
            memec_amd.set_knob(name, value)
        assert "accepted" in str(e.value), (name, value)
    src = open(os.path.join(ROOT, "memec_amd", "csrc", "kernels.hip")).read()
    assert "getenv" not in src


def test_every_knob_is_read_from_the_environment():
    """knobs.cpp reads each knob's variable once at first use, from one
    table (kSpecs) that also holds its accepted values; every knob of the
    Knob enum has an entry (a static assert) and mec.h documents each
    variable (round 4: MEC_MG_ROWS was accepted by mec_set_knob but never
    read from the environment, which voided an A/B run)."""
    import re
    src = open(os.path.join(ROOT, "memec_amd", "csrc", "knobs.cpp")).read()
    table = src[src.index("kSpecs[] = {"):src.index("};", src.index("kSpecs[] = {"))]
    env = set(re.findall(r'\{"(MEC_[A-Z_]+)", kKnob', table))
    hdr_k = open(os.path.join(ROOT, "memec_amd", "csrc", "knobs.hpp")).read()
    knobs_enum = set(re.findall(r"// (MEC_[A-Z_]+)=", hdr_k))
    assert env == knobs_enum, (env ^ knobs_enum)
    hdr = open(os.path.join(ROOT, "include", "mec.h")).read()
    for name in env:
        assert name in hdr, name


def test_probe_needs_a_context():
    L = _lib.lib()
    assert L.mec_set_probe(None, 1) == _lib.MEC_EINVAL


def test_launch_planner_invariants_every_knob(tmp_path):
    """tests/cpp/launch_plan_check.cc: the launch planner
    (memec_amd/csrc/launch_plan.cpp, the only source of every launch's
    shape) under every accepted value of every MEC_* knob, ~10^8 plans of
    gf8 / one-pass / bitmatrix / gathered / XOR launches: rows per group x
    groups <= 32 (the round-4 MEC_MG_ROWS=3 overrun,
    profiles/r05/parity/launch_plan_check_before_fix.log), LDS <= 160 KiB,
    instantiated templates and block sizes only, 32-bit lane offsets,
    stripe-group runs that tile the stripe, sub-launches covering the batch,
    and no legal call refused.  Host code only (g++, UBSan)."""
    import shutil
    import subprocess
    if not shutil.which("g++"):
        pytest.skip("g++ not available")
    exe = str(tmp_path / "launch_plan_check")
    csrc = os.path.join(ROOT, "memec_amd", "csrc")
    subprocess.check_call(["g++", "-std=c++17", "-O2", "-fsanitize=undefined", "-fno-sanitize-recover=undefined",
                           "-D__HIP_PLATFORM_AMD__", "-I/opt/rocm/include", "-I" + os.path.join(ROOT, "include"),
                           "-I" + csrc, os.path.join(ROOT, "tests", "cpp", "launch_plan_check.cc"),
                           os.path.join(csrc, "launch_plan.cpp"), os.path.join(csrc, "knobs.cpp"), "-o", exe])
    env = {k: v for k, v in os.environ.items() if not k.startswith("MEC_")}
    out = subprocess.run([exe], capture_output=True, text=True, timeout=600, env=env)
    assert out.returncode == 0, out.stdout[-3000:] + out.stderr[-2000:]
    assert out.stdout.startswith("ok "), out.stdout
    assert int(out.stdout.split()[1]) > 10 ** 8


def test_bitslice_programs_equal_gf8_products(tmp_path):
    """tests/cpp/bitslice_check.cc: every bit-sliced program the JIT would
    compile (memec_amd/csrc/bitslice.cpp: 8 x 8 bit transposes and the
    four-Russians XOR schedule) for 5..31 outputs x every source count with
    k + m <= 32, random / Vandermonde-like / sparse matrices, overwrite and
    accumulate, interpreted on the CPU over random chunks equals the
    byte-wise GF(2^8) products (ASan + UBSan), and its HIP source is
    generated.  No device runs a program that has not passed this."""
    import shutil
    import subprocess
    if not shutil.which("g++"):
        pytest.skip("g++ not available")
    exe = str(tmp_path / "bitslice_check")
    csrc = os.path.join(ROOT, "memec_amd", "csrc")
    subprocess.check_call(["g++", "-std=c++17", "-O1", "-fsanitize=address,undefined", "-fno-sanitize-recover=undefined",
                           "-I" + os.path.join(ROOT, "include"), "-I" + csrc,
                           os.path.join(ROOT, "tests", "cpp", "bitslice_check.cc"),
                           os.path.join(csrc, "bitslice.cpp"), os.path.join(csrc, "gf_math.cpp"), "-o", exe])
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=1:verify_asan_link_order=0")
    out = subprocess.run([exe], capture_output=True, text=True, timeout=600, env=env)
    assert out.returncode == 0, out.stdout[-3000:] + out.stderr[-2000:]
    assert out.stdout.splitlines()[-1].startswith("ok "), out.stdout
    assert int(out.stdout.splitlines()[-1].split()[1]) > 2900


def test_bitslice_kernels_compile_for_gfx950(tmp_path):
    """The generated bit-sliced kernel (RS(16,8) encode program) compiles for
    gfx950 in each addressing form the JIT builds — strided, gathered
    straight-line (default), gathered looping over MEC_BS_TPB tiles — with
    no scratch (register spills): the forms with scheduling fences between
    sources (the gathered ones by default) within 128 VGPRs (4 waves per
    SIMD), the strided one without them within 168 (3 waves).  hipcc
    cross-compiles here; the product compiles the same source with hiprtc
    on the device's host."""
    import re
    import shutil
    import subprocess
    hipcc = "/opt/rocm/bin/hipcc"
    readelf = "/opt/rocm/lib/llvm/bin/llvm-readelf"
    if not (shutil.which("g++") and os.path.exists(hipcc) and os.path.exists(readelf)):
        pytest.skip("toolchain not available")
    exe = str(tmp_path / "bitslice_check")
    csrc = os.path.join(ROOT, "memec_amd", "csrc")
    subprocess.check_call(["g++", "-std=c++17", "-O1", "-I" + os.path.join(ROOT, "include"), "-I" + csrc,
                           os.path.join(ROOT, "tests", "cpp", "bitslice_check.cc"),
                           os.path.join(csrc, "bitslice.cpp"), os.path.join(csrc, "gf_math.cpp"), "-o", exe])
    out = subprocess.run([exe, str(tmp_path)], capture_output=True, text=True, timeout=600)
    assert out.returncode == 0, out.stdout[-2000:] + out.stderr[-2000:]
    for form in ("strided", "gather1", "gather4", "strided_fence", "gather1_srow"):
        src = str(tmp_path / f"bs_{form}.hip")
        obj = str(tmp_path / f"bs_{form}.co")
        subprocess.check_call([hipcc, "--offload-arch=gfx950", "--cuda-device-only", "--no-gpu-bundle-output", "-O3", "-std=c++17", "-include", "hip/hip_runtime.h",
                               "-x", "hip", src, "-o", obj], timeout=600)
        notes = subprocess.run([readelf, "--notes", obj], capture_output=True, text=True, check=True).stdout
        vgpr = int(re.search(r"\.vgpr_count:\s+(\d+)", notes).group(1))
        scratch = int(re.search(r"\.private_segment_fixed_size:\s+(\d+)", notes).group(1))
        assert scratch == 0, (form, scratch)
        assert vgpr <= (168 if form == "strided" else 128), (form, vgpr)


def test_registry_ranges_disjoint(tmp_path):
    """tests/cpp/registry_check.cc: the zero-copy registry
    (memec_amd/csrc/registry.hpp, hostmem.cpp) refuses a range that overlaps
    a registered one — re-registration and a range that starts below a
    registered one and extends across it included —
    unregisters by begin only, and translates an address only inside one
    range; random register / unregister / lookup sequences against a
    brute-force model (ASan + UBSan)."""
    import shutil
    import subprocess
    if not shutil.which("g++"):
        pytest.skip("g++ not available")
    exe = str(tmp_path / "registry_check")
    subprocess.check_call(["g++", "-std=c++17", "-O1", "-fsanitize=address,undefined", "-fno-sanitize-recover=undefined",
                           "-I" + os.path.join(ROOT, "memec_amd", "csrc"),
                           os.path.join(ROOT, "tests", "cpp", "registry_check.cc"), "-o", exe])
    out = subprocess.run([exe], capture_output=True, text=True, timeout=120)
    assert out.returncode == 0, out.stdout[-3000:] + out.stderr[-2000:]
    assert out.stdout.startswith("ok "), out.stdout


def test_unregister_unknown_range_is_refused():
    """mec_host_unregister of a pointer that begins no registered range is
    MEC_EINVAL before any HIP call (so it holds on a host without a GPU)."""
    import ctypes
    L = _lib.lib()
    buf = ctypes.create_string_buffer(4096)
    assert L.mec_host_unregister(ctypes.cast(buf, ctypes.c_void_p)) == _lib.MEC_EINVAL
    assert b"does not begin a registered range" in L.mec_last_error()
    assert L.mec_host_register(None, 16) == _lib.MEC_EINVAL
