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
    n = bench.cpu_sample(k, m, cs, 2)
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
    n = bench.cpu_sample(k, m, cs, 2)
    data, par = _stripes(fam, k, m, cs, n, 99)
    cw = np.concatenate([data, par], axis=1)
    r = bench.cpu_baseline_reference(fam, k, m, cs, None, 0, 2, "decode", erased, cw)
    assert r["kind"] == "reference" and r["matches_gpu"] is True and r["value"] > 0


def test_reference_leg_absent_or_other_family():
    assert bench.cpu_baseline_reference("isal_rs", 4, 2, 4096, None, 0, 2, "encode") is None


def test_port_encode_leg():
    k, m, cs = 4, 2, 4096
    n = bench.cpu_sample(k, m, cs, 2)
    _, par = _stripes("rs", k, m, cs, n, 77)
    r = bench.cpu_baseline("rs", k, m, cs, par, 77, 2)
    assert r["kind"] == "port" and r["matches_gpu"] is True and r["value"] > 0


def _fast(fn):
    """ref_baseline with a 0.2 s budget instead of ~10 s (same code path)."""
    def wrapped(fam, k, m, cs, threads, sample, run, **kw):
        def short_run(L, h, passes, n, t):
            return run(L, h, min(passes, 2), n, t)
        return fn(fam, k, m, cs, threads, sample, short_run, **kw)
    return wrapped


@needs_ref
def test_reference_update_leg(monkeypatch):
    monkeypatch.setattr(bench, "ref_baseline", _fast(bench.ref_baseline))
    r = bench.cpu_baseline_reference_update("rs", 4, 2, 4096, 1, 2)
    assert r["kind"] == "reference" and r["matches_oracle"] is True and r["value"] > 0


# ---- sample and work bounds (a 256-thread baseline once asked
# for 3.5 GiB per leg and ~512 CPU-seconds, and the box killed it) ---------

CONFIG_SHAPES = [(10, 4, 1 << 20), (8, 2, 4096), (12, 4, 65536), (4, 2, 4096), (10, 4, 16 << 20)]


@pytest.mark.parametrize("threads", [1, 2, 16, 64, 256, 1024])
@pytest.mark.parametrize("k,m,cs", CONFIG_SHAPES)
def test_cpu_sample_bounded_by_bytes(k, m, cs, threads):
    n = bench.cpu_sample(k, m, cs, threads)
    sb = (k + m) * cs
    assert n >= 1
    assert n * sb <= max(bench.CPU_SAMPLE_BYTES_MAX, sb)
    assert n % min(threads, n) == 0


@pytest.mark.parametrize("usable", [1, 16, 64])
@pytest.mark.parametrize("threads", [1, 16, 256, 1024])
@pytest.mark.parametrize("probe_s", [1e-4, 0.05, 1.0, 12.0])
def test_cpu_work_plan_bounded_on_usable_cores(probe_s, threads, usable):
    sample = 48
    passes, est = bench.cpu_work_plan(probe_s, threads, usable, sample)
    p = min(threads, usable, sample)
    assert passes >= 1 and est == pytest.approx(passes * probe_s / p)
    # <= 30 CPU-seconds of work unless a single pass alone is longer, and
    # >= 10 unless the 4096-pass cap binds
    assert passes * probe_s <= max(bench.CPU_WORK_S[1] * 1.05, probe_s * 1.5)
    assert passes * probe_s >= bench.CPU_WORK_S[0] * 0.95 or passes == 4096
    # the wall time no longer grows with the requested thread count
    assert est <= max(11.0, probe_s * 1.5)


# ---- parity pins (bench.check_encode / check_decode) ------------------------

torch = pytest.importorskip("torch")


@pytest.mark.parametrize("fam,k,m,cs", [("rs", 4, 2, 4096), ("cauchy", 4, 2, 4096), ("rs", 10, 4, 1024)])
def test_check_encode_pins_reference(fam, k, m, cs):
    n = 9
    data, par = _stripes(fam, k, m, cs, n, 4321)
    d, p = torch.from_numpy(data), torch.from_numpy(par.copy())
    r = bench.check_encode(fam, k, m, cs, d, p)
    assert r["equal"] is True and r["stripes"] == min(n, bench.parity_count(k, m, cs))
    assert ("oracle/_ref" in r["vs"]) == os.path.exists(bench.REF_SO)
    p[n - 1, m - 1, 7] ^= 0x40  # the last stripe is always sampled
    assert bench.check_encode(fam, k, m, cs, d, p)["equal"] is False


def _oracle_decode_rows(fam, k, m, cs, st, erased):
    out = st.copy()
    for s_ in range(st.shape[0]):
        chunks = [out[s_, i].copy() for i in range(k + m)]
        assert O.decode(fam, k, m, chunks, erased, cs) == 0
        out[s_] = np.stack(chunks)
    return out


@pytest.mark.parametrize("fam,k,m,cs,erased", [("rs", 4, 2, 4096, [0]), ("rs", 6, 3, 2048, [1, 4]),
                                               ("cauchy", 4, 2, 4096, [1])])
def test_check_decode_pins_survivor_choice(fam, k, m, cs, erased):
    """A decoder that rebuilds the same chunks from a different survivor set
    passes a codeword round trip but fails the planted non-codewords."""
    n = 10
    data, par = _stripes(fam, k, m, cs, n, 777)
    st = torch.from_numpy(np.concatenate([data, par], axis=1))
    rec = bench.plant_noncodewords(st, k, m, cs, 99)
    assert rec["nc"] and rec["cw"] and max(rec["cw"]) < min(rec["nc"])
    before = st.numpy().copy()
    good = _oracle_decode_rows(fam, k, m, cs, before, erased)
    r = bench.check_decode(fam, k, m, cs, torch.from_numpy(good), erased, rec)
    assert r["equal"] is True and r["non_codeword_stripes"] == len(rec["nc"])
    # wrong survivors: also treat the first surviving parity as lost, so the
    # decoder reads a different set (one more data/parity chunk is skipped)
    extra = next(i for i in range(k, k + m) if i not in erased)
    wrong = _oracle_decode_rows(fam, k, m, cs, before, sorted(erased + [extra]))
    wrong[:, extra] = before[:, extra]  # the extra chunk was never lost
    for s_ in rec["cw"]:  # codewords: identical, a round trip cannot tell
        assert np.array_equal(wrong[s_], good[s_])
    assert bench.check_decode(fam, k, m, cs, torch.from_numpy(wrong), erased, rec)["equal"] is False


def test_restore_noncodewords():
    k, m, cs, n, erased = 4, 2, 256, 8, [0, 5]
    st = torch.zeros(n, k + m, cs, dtype=torch.uint8)
    rec = bench.plant_noncodewords(st, k, m, cs, 3)
    saved = torch.zeros(n, len(erased), cs, dtype=torch.uint8)
    bench.restore_noncodewords(st, saved, erased, rec)
    assert torch.equal(st[:, erased], saved)


def test_spread_indices():
    assert bench.spread(0, 1, 5) == [0]
    assert bench.spread(3, 3, 4) == []
    assert bench.spread(0, 4096, 13)[0] == 0 and bench.spread(0, 4096, 13)[-1] == 4095
    assert len(bench.spread(0, 4096, 13)) == 13 and len(bench.spread(0, 5, 13)) == 5


def test_configs0_reference_cpu_leg():
    """BASELINE configs[0] through the reference's own CPU path
    (oracle/_ref): RS(4,2)@4 KiB encode and decode {0,1} on one thread,
    outputs checked (encode vs the oracle, decode vs the codewords)."""
    if bench._ref_lib() is None:
        pytest.skip("oracle/_ref not built here")
    r = bench.configs0_reference(seconds=0.05)
    assert r["kind"] == "reference" and r["cores"] == 1
    assert r["encode_value"] > 0 and r["decode_value"] > 0
    assert r["encode_matches_oracle"] is True and r["decode_restores_codewords"] is True


def test_cpu_legs_run_on_rank0_at_every_world_size():
    """The reference CPU baseline is in every line rank 0 prints — at N = 1,
    2, 4 and 8 — and every CPU leg (cpu_baseline, the decode twin's, configs[0]'s
    reference_cpu, the samples they take) is gated by that one rule, after
    the barrier that ends every rank's GPU legs."""
    import inspect
    for world in (1, 2, 4, 8):
        assert bench.runs_cpu_legs(0, world, False) is True
        assert bench.runs_cpu_legs(0, world, True) is False
        for r in range(1, world):
            assert bench.runs_cpu_legs(r, world, False) is False
    src = inspect.getsource(bench.main)
    assert "world == 1" not in src
    assert src.count("runs_cpu_legs(rank, world, args.no_cpu_baseline)") == 5
    assert src.index("dist.barrier()") < src.index("threads, host = host_cores()")


@needs_ref
def test_reference_decode_leg_fewer_codewords_than_sample(monkeypatch):
    """A small --stripes run hands over fewer GPU codewords than the leg's
    sample (N = 4 x 32 stripes): the leg decodes only those (it once read
    past them: heap corruption at exit)."""
    monkeypatch.setattr(bench, "ref_baseline", _fast(bench.ref_baseline))
    k, m, cs = 10, 4, 65536
    assert bench.cpu_sample(k, m, cs, 16) > 8
    data, par = _stripes("rs", k, m, cs, 8, 3)
    cw = np.concatenate([data, par], axis=1)
    r = bench.cpu_baseline_reference("rs", k, m, cs, None, 0, 16, "decode", [0, 1, 2, 3], cw)
    assert r["kind"] == "reference" and r["matches_gpu"] is True
    assert r["sample"].startswith("8 stripes")


def test_memory_plan_full_size_fits_one_mi355x():
    """bench.memory_plan: the default line (configs[1] with its decode twin,
    rank 0's 3 x 8 GiB reference streams, configs[0]/[3]/[4] beside it) at
    full size, one rank per GPU at 1..8 ranks, peaks at 128 GiB — under one
    MI355X's 288 GB; every timed config alone fits too."""
    import bench
    for world in (1, 2, 4, 8):
        p = bench.memory_plan("rs_enc", 4096, world, True, True, True)
        assert p["phases"]["timed"] == 56 << 30
        assert p["phases"]["reference_streams"] == 80 << 30
        assert p["peak_bytes"] == 128 << 30
    for name, cfg in bench.CONFIGS.items():
        assert bench.memory_plan(name, cfg[4], 1, True, False, True)["peak_bytes"] < 288e9 * 0.9, name
