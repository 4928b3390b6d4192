"""The C++ drop-in for MemEC's `class Coding` (memec_amd/csrc/coding/):
build it standalone like server/ would link it (CPU), then run the
coding_test program (tests/cpp/coding_test.cc, the reference's own coding
test flow) against the GPU (gpu)."""
import os
import subprocess

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CODING = os.path.join(ROOT, "memec_amd", "csrc", "coding")


def _build(tmpdir, isal):
    out = os.path.join(str(tmpdir), "coding_test_isal" if isal else "coding_test")
    srcs = [os.path.join(CODING, f) for f in sorted(os.listdir(CODING)) if f.endswith(".cc")]
    cmd = ["g++", "-std=c++11", "-O2", "-Wall", "-Werror", "-I" + CODING, "-I" + os.path.join(ROOT, "include"),
           os.path.join(ROOT, "tests", "cpp", "coding_test.cc")] + srcs + \
          ["-L" + os.path.join(ROOT, "memec_amd"), "-lmec", "-Wl,-rpath," + os.path.join(ROOT, "memec_amd"),
           "-lpthread", "-o", out]
    if isal:
        cmd.insert(1, "-DUSE_ISAL")
    subprocess.check_call(cmd)
    return out


@pytest.fixture(scope="module")
def binaries(tmp_path_factory):
    d = tmp_path_factory.mktemp("coding")
    return _build(d, False), _build(d, True)


def test_adapter_builds_standalone(binaries):
    for b in binaries:
        assert os.path.exists(b)


@pytest.mark.gpu
@pytest.mark.parametrize("args", [
    ["rs"], ["cauchy"], ["rs", "10", "4", "65536"], ["cauchy", "12", "4", "65536"],
    ["rs", "4", "2", "4096"], ["cauchy", "4", "2", "96"], ["rs", "20", "12", "1032"],
])
def test_coding_flow_on_gpu(binaries, args):
    for b in binaries:
        r = subprocess.run([b] + args, capture_output=True, text=True, timeout=120)
        assert r.returncode == 0, (b, args, r.stdout, r.stderr)
        assert ": ok" in r.stdout


@pytest.mark.gpu
@pytest.mark.parametrize("env", [{"MEMEC_GPU_DEVICES": "0,0"}, {"MEMEC_GPU_COALESCE": "64"},
                                 {"CODING_TEST_REGISTER": "1"}, {"CODING_TEST_REGISTER": "1", "MEMEC_GPU_QUEUE": "0"}])
def test_coding_flow_adapter_modes(binaries, env):
    """The same flow with the adapter driving a multi-device context
    (MEMEC_GPU_DEVICES, device repeated on a one-GPU box), with the request
    coalescer on, and on registered chunks (zero-copy; single-stripe calls
    through the resident host queue unless MEMEC_GPU_QUEUE=0)."""
    for b in binaries:
        for args in (["rs", "10", "4", "65536"], ["cauchy", "12", "4", "65536"], ["rs", "8", "3", "4096"],
                     ["rs", "6", "2", "4104"]):
            r = subprocess.run([b] + args, capture_output=True, text=True, timeout=120,
                               env=dict(os.environ, **env))
            assert r.returncode == 0, (b, args, env, r.stdout, r.stderr)
            assert ": ok" in r.stdout


@pytest.mark.gpu
def test_isal_encode_offsets_match_reference(binaries, golden, tmp_path):
    """The USE_ISAL adapter's encode(data, parity, index, startOff, endOff)
    on a parity chunk holding bytes, vs the reference plugin's steps
    (tests/golden/make_golden.py: rscoding.cc:82-89 XORs
    ec_encode_data_update_base over the touched columns; cauchycoding.cc:78-79
    overwrites with a full encode)."""
    meta, blobs = golden
    cases = [(n, c) for n, c in sorted(meta["cases"].items()) if c["kind"] == "encode_offsets_isal"]
    assert len(cases) >= 20  # 8 with m <= 4, 12 wide (round 6)
    isal_bin = binaries[1]
    for name, c in cases:
        out = tmp_path / "par.bin"
        args = [isal_bin, "encode-offsets", "rs" if c["family"] == "isal_rs" else "cauchy"] + \
            [str(c[x]) for x in ("k", "m", "chunk", "index", "startOff", "endOff", "seed", "parity_seed")] + [str(out)]
        r = subprocess.run(args, capture_output=True, text=True, timeout=120)
        assert r.returncode == 0, (name, r.stdout, r.stderr)
        assert np.array_equal(np.fromfile(str(out), dtype=np.uint8), blobs[name]), name


@pytest.mark.gpu
@pytest.mark.parametrize("fam", ["rs", "cauchy", "isal_rs", "isal_cauchy"])
def test_adapter_random_shapes_vs_reference_plugin(binaries, fam, tmp_path):
    """The drop-in class itself (Coding::instantiate / encode / decode, both
    plugin builds) on 80 random shapes against MemEC's own plugin
    (oracle/_ref, tests/_refplugin.py): encode of every parity index, the
    server's delta form (one data chunk, Coding::zeros elsewhere) and decode
    of a random NON-codeword stripe with 1..m lost chunks (and m + 1 for
    every tenth case: decode() false in both) — byte for byte, decode()'s
    return value included (ISA-L RS's singular patterns: false in both)."""
    import random
    import _oracle as O
    import _refplugin as R
    from _mismatch import same
    if not R.available():
        pytest.skip("oracle/_ref not built")
    rng = random.Random(0xADA + len(fam))
    cases, blobs = [], []
    while len(cases) < 80:
        n = rng.randint(2, 32)
        m = rng.randint(1, n - 1)
        k = n - m
        cs = 8 * rng.randint(1, 1024)
        if fam == "cauchy" and not 1 <= O.cauchy_getw(k, m, cs) <= 8:
            continue
        e = m + 1 if len(cases) % 10 == 9 else rng.randint(1, m)
        lost = sorted(rng.sample(range(k + m), e))
        present = sum(1 << i for i in range(k + m) if i not in lost)
        stripe = O.fill((k + m) * cs, 0xC0DE00 + len(cases)).reshape(k + m, cs)
        cases.append((k, m, cs, present, rng.randrange(k), lost))
        blobs.append(stripe)
    (tmp_path / "cases.txt").write_text("".join("%d %d %d %d %d\n" % c[:5] for c in cases))
    np.concatenate([b.reshape(-1) for b in blobs]).tofile(str(tmp_path / "stripes.bin"))
    b = binaries[1] if fam.startswith("isal") else binaries[0]
    r = subprocess.run([b, "sweep", "cauchy" if fam.endswith("cauchy") else "rs", str(tmp_path / "cases.txt"),
                        str(tmp_path / "stripes.bin"), str(tmp_path / "out.bin")],
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, (r.stdout, r.stderr)
    out = np.fromfile(str(tmp_path / "out.bin"), dtype=np.uint8)
    pos = 0
    for (k, m, cs, present, col, lost), stripe in zip(cases, blobs):
        what = (fam, k, m, cs, lost)
        enc = out[pos:pos + m * cs].reshape(m, cs)
        dlt = out[pos + m * cs:pos + 2 * m * cs].reshape(m, cs)
        dec = out[pos + 2 * m * cs:pos + (2 * m + k + m) * cs].reshape(k + m, cs)
        ok = bool(out[pos + (3 * m + k) * cs])
        pos += (3 * m + k) * cs + 1
        same(enc, R.encode(fam, k, m, cs, stripe[:k]), ("encode",) + what)
        z = np.zeros((k, cs), np.uint8)
        z[col] = stripe[col]
        same(dlt, R.encode(fam, k, m, cs, z), ("delta",) + what + (col,))
        rok, want = R.decode(fam, k, m, cs, stripe, lost)
        assert ok == rok, ("decode() return",) + what
        if ok:
            same(dec, want, ("decode",) + what)
    assert pos == out.size
