"""CPU checks of bench.py's cpu_baseline legs (no GPU): the compiled
reference (oracle/_ref, kind "reference") and the oracle port produce the
same parity / reconstructions as the oracle's single-stripe functions on
the bench's own synthetic stripes, and the reported fields are the ones the
bench contract names.  Small chunk sizes so the ~10 s CPU budget per leg is
reached in few passes."""
import os

import numpy as np
import pytest

import _oracle as O

bench = pytest.importorskip("bench")

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
needs_ref = pytest.mark.skipif(not os.path.exists(bench.REF_SO), reason="oracle/_ref not built")


def _stripes(fam, k, m, cs, n, seed):
    data = O.fill(n * k * cs, seed).reshape(n, k, cs)
    par = np.stack([np.stack(O.encode(fam, k, m, [data[s, j].copy() for j in range(k)], cs)) for s in range(n)])
    return data, par


@needs_ref
@pytest.mark.parametrize("fam,k,m,cs", [("rs", 4, 2, 4096), ("cauchy", 4, 2, 4096)])
def test_reference_encode_leg(fam, k, m, cs, monkeypatch):
    monkeypatch.setattr(bench, "ref_baseline", _fast(bench.ref_baseline))
    seed = 1234
    n = bench.decode_sample(k, m, cs, 2)
    _, par = _stripes(fam, k, m, cs, n, seed)
    r = bench.cpu_baseline_reference(fam, k, m, cs, par, seed, 2, "encode")
    assert r["kind"] == "reference" and r["cores"] == 2 and r["unit"] == "GiB/s"
    assert r["matches_gpu"] is True and r["value"] > 0 and r["single_thread_value"] > 0
    bad = par.copy()
    bad[0, 0, 0] ^= 1
    assert bench.cpu_baseline_reference(fam, k, m, cs, bad, seed, 2, "encode")["matches_gpu"] is False


@needs_ref
@pytest.mark.parametrize("fam,k,m,cs,erased", [("rs", 4, 2, 4096, [0, 1]), ("cauchy", 4, 2, 4096, [1, 5])])
def test_reference_decode_leg(fam, k, m, cs, erased, monkeypatch):
    monkeypatch.setattr(bench, "ref_baseline", _fast(bench.ref_baseline))
    n = bench.decode_sample(k, m, cs, 2)
    data, par = _stripes(fam, k, m, cs, n, 99)
    cw = np.concatenate([data, par], axis=1)
    r = bench.cpu_baseline_reference(fam, k, m, cs, None, 0, 2, "decode", erased, cw)
    assert r["kind"] == "reference" and r["matches_gpu"] is True and r["value"] > 0


def test_reference_leg_absent_or_other_family():
    assert bench.cpu_baseline_reference("isal_rs", 4, 2, 4096, None, 0, 2, "encode") is None


def test_port_encode_leg():
    k, m, cs = 4, 2, 4096
    n = bench.decode_sample(k, m, cs, 2)
    _, par = _stripes("rs", k, m, cs, n, 77)
    r = bench.cpu_baseline("rs", k, m, cs, par, 77, 2)
    assert r["kind"] == "port" and r["matches_gpu"] is True and r["value"] > 0


def _fast(fn):
    """ref_baseline with a 0.2 s budget instead of ~10 s (same code path)."""
    def wrapped(fam, k, m, cs, threads, sample, run):
        def short_run(L, h, passes, n, t):
            return run(L, h, min(passes, 2), n, t)
        return fn(fam, k, m, cs, threads, sample, short_run)
    return wrapped


@needs_ref
def test_reference_update_leg(monkeypatch):
    monkeypatch.setattr(bench, "ref_baseline", _fast(bench.ref_baseline))
    r = bench.cpu_baseline_reference_update("rs", 4, 2, 4096, 1, 2)
    assert r["kind"] == "reference" and r["matches_oracle"] is True and r["value"] > 0
