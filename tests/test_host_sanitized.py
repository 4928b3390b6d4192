"""Host code under AddressSanitizer + UBSan (CPU only): libmec's matrix
construction and decode planning (memec_amd/csrc/gf_math.cpp) for every
family and every (k, m) with k + m <= 32, checked by re-deriving the erased
symbols of random codewords (tests/cpp/gf_math_check.cc)."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_decode_plans_all_codes_asan_ubsan(tmp_path):
    if not shutil.which("g++"):
        pytest.skip("g++ not available")
    exe = str(tmp_path / "gf_math_check")
    subprocess.check_call(["g++", "-std=c++17", "-O1", "-g", "-fsanitize=address,undefined",
                           "-fno-omit-frame-pointer", "-fno-sanitize-recover=undefined",
                           "-I" + os.path.join(ROOT, "include"), "-I" + os.path.join(ROOT, "memec_amd", "csrc"),
                           os.path.join(ROOT, "tests", "cpp", "gf_math_check.cc"),
                           os.path.join(ROOT, "memec_amd", "csrc", "gf_math.cpp"), "-o", exe])
    # verify_asan_link_order=0: tolerate libraries the environment preloads
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=1:verify_asan_link_order=0")
    out = subprocess.run([exe], capture_output=True, text=True, env=env, timeout=300)
    assert out.returncode == 0, out.stdout[-2000:] + out.stderr[-2000:]
    assert out.stdout.startswith("ok "), out.stdout
    assert int(out.stdout.split()[1]) > 100000
