"""The drop-in inside a MemEC tree (VERDICT r1 "prove the in-tree drop-in").

tests/memec_tree/Makefile assembles a scratch MemEC tree from the reference
checkout with the adapter in common/coding beside the reference's XOR codes
(INTEGRATION.md §2), and builds the reference's own coding test
(test/common/coding/coding.cc, unchanged, -DTEST_DELTA as its Makefile:7)
against libmec.so, in the default and the USE_ISAL flavour.

CPU: the tree builds, and RAID5 / RDP / EVENODD — the reference's own XOR
codes, constructed by the adapter's Coding::instantiate — pass the
reference test.  GPU: rs and cauchy pass it through the MI355X engine."""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
TREE = os.path.join(ROOT, "tests", "memec_tree")
BUILD = os.path.join(TREE, "_build")
REF = "/root/reference"


def _binary(flavour):
    return os.path.join(BUILD, "coding_" + flavour)


def _run(flavour, scheme):
    r = subprocess.run([_binary(flavour), scheme], capture_output=True, text=True, timeout=120)
    return r.returncode, r.stdout + r.stderr


@pytest.mark.skipif(not os.path.isdir(os.path.join(REF, "test", "common", "coding")),
                    reason="needs the reference checkout (build container only)")
def test_tree_builds_and_xor_codes_pass():
    subprocess.check_call(["make", "-s", "-C", TREE, "-j8"])
    for flavour in ("jerasure", "isal"):
        assert os.access(_binary(flavour), os.X_OK)
        for scheme in ("raid5", "rdp", "evenodd"):
            rc, out = _run(flavour, scheme)
            assert rc == 0, (flavour, scheme, out)
            assert "FAILED" not in out and "Data recovered" in out, (flavour, scheme, out)
            if scheme != "raid5":
                assert ".. Data 2 recovered" in out, (flavour, scheme, out)


@pytest.mark.gpu
@pytest.mark.parametrize("flavour", ["jerasure", "isal"])
@pytest.mark.parametrize("scheme", ["rs", "cauchy"])
def test_reference_coding_test_on_gpu(flavour, scheme):
    """test/common/coding/coding.cc:76-286 unchanged: encode 3 parities,
    TEST_DELTA update of chunks 1..3 through encode(startOff, endOff) +
    bitwiseXOR, then 1, 2 and 3 data failures, each memcmp-checked."""
    assert os.access(_binary(flavour), os.X_OK), \
        "tests/memec_tree/_build missing: run __graft_entry__.build() in the build container"
    rc, out = _run(flavour, scheme)
    assert rc == 0, out
    assert "FAILED" not in out, out
    for line in (">> encode K: 8   M: 3", "Data recovered", ".. Data 2 recovered", ".. Data 3 recovered"):
        assert line in out, (line, out)
