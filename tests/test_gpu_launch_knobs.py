"""GPU parity under every launch shape the strided kernels can take.

The launch rules (stream_common.hpp: lane width of the bitmatrix kernel,
block size, wave caps) pick one shape per launch from the layout and the
chunk size; the experiment knobs MEC_BM_VW / MEC_BLOCK / MEC_WPC force the
others.  Whatever the shape, the bytes must equal the oracle's
(Jerasure/gf_complete restatement, pinned to the reference by
tests/golden): split and in-place encodes, in-place decodes and delta
updates, at chunk sizes whose packets are and are not multiples of the lane
slice (tails).
"""
import numpy as np
import pytest

import _oracle as O

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

from memec_amd import Codec, MecError  # noqa: E402

K, M, N = 6, 3, 20
ERASED = (0, 4, 7)


@pytest.fixture(scope="module", autouse=True)
def _gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    torch.cuda.set_device(0)
    yield
    torch.cuda.synchronize()


def _stripes(fam, cs, seed):
    base = O.fill(N * (K + M) * cs, seed).reshape(N, K + M, cs)
    for s in range(N):
        base[s, K:] = np.stack(O.encode(fam, K, M, [base[s, j].copy() for j in range(K)], cs))
    return base


def _check_all_layouts(fam, cs, seed):
    base = _stripes(fam, cs, seed)
    c = Codec(fam, K, M, cs)
    # split encode: [s][k] data -> [s][m] parity
    data = torch.from_numpy(np.ascontiguousarray(base[:, :K])).to("cuda")
    par = torch.zeros(N, M, cs, dtype=torch.uint8, device="cuda")
    c.encode(data, par)
    torch.cuda.synchronize()
    assert np.array_equal(par.cpu().numpy(), base[:, K:]), ("split encode", fam, cs)
    # in-place encode: parity written inside [s][k+m]
    st = torch.from_numpy(base.copy()).to("cuda")
    st[:, K:] = 0
    c.encode(st[:, :K], st[:, K:])
    torch.cuda.synchronize()
    assert np.array_equal(st.cpu().numpy(), base), ("in-place encode", fam, cs)
    # in-place decode of data and parity erasures
    st[:, list(ERASED)] = 0
    c.decode(st, sum(1 << i for i in range(K + M) if i not in ERASED))
    torch.cuda.synchronize()
    assert np.array_equal(st.cpu().numpy(), base), ("in-place decode", fam, cs)
    # delta update of column 2 into every parity (read-modify-write)
    delta = O.fill(N * cs, seed + 1).reshape(N, cs)
    par2 = torch.from_numpy(np.ascontiguousarray(base[:, K:])).to("cuda")
    c.encode_update(2, torch.from_numpy(delta).to("cuda"), par2)
    torch.cuda.synchronize()
    got = par2.cpu().numpy()
    for s in (0, N - 1):
        d2 = base[s, :K].copy()
        d2[2] ^= delta[s]
        assert np.array_equal(got[s], np.stack(O.encode(fam, K, M, list(d2), cs))), ("update", fam, cs, s)
    c.close()


@pytest.mark.parametrize("cs", [96, 4096, 4128, 65536])
@pytest.mark.parametrize("vw", ["2", "4", None])
def test_bitmatrix_lane_widths(vw, cs, knobs):
    """8- and 16-byte lane slices (MEC_BM_VW), and the rule's own choice:
    packets of 24 B and 1032 B leave tails for 16-byte slices only."""
    if vw is None:
        knobs("MEC_BM_VW", None)
    else:
        knobs("MEC_BM_VW", vw)
    _check_all_layouts("cauchy", cs, 900 + cs % 997)


@pytest.mark.parametrize("fam", ["rs", "cauchy", "isal_rs"])
@pytest.mark.parametrize("block,wpc", [("64", "0"), ("64", "6"), ("256", "24"), ("256", "0")])
def test_block_and_wave_cap_overrides(fam, block, wpc, knobs):
    """Forced block sizes and resident-wave caps (down to one block per CU's
    share of LDS) change timing only."""
    knobs("MEC_BLOCK", block)
    knobs("MEC_WPC", wpc)
    _check_all_layouts(fam, 8192, 1300)


@pytest.mark.parametrize("stride_chunk", [2048, 65536])
def test_power_of_two_stripe_strides(stride_chunk):
    """RS(6,2) stripes are 8 chunks: 16 KiB and 512 KiB strides, the two
    sides of the in-place block-size rule for power-of-two strides."""
    k, m, cs, n = 6, 2, stride_chunk, 16
    base = O.fill(n * (k + m) * cs, 77).reshape(n, k + m, cs)
    for s in range(n):
        base[s, k:] = np.stack(O.encode("rs", k, m, [base[s, j].copy() for j in range(k)], cs))
    c = Codec("rs", k, m, cs)
    st = torch.from_numpy(base.copy()).to("cuda")
    st[:, [0, 1]] = 0
    c.decode(st, sum(1 << i for i in range(2, k + m)))
    torch.cuda.synchronize()
    assert np.array_equal(st.cpu().numpy(), base)
    c.close()


@pytest.mark.parametrize("fam", ["rs", "cauchy", "isal_rs", "isal_cauchy"])
def test_empty_batches_and_no_erasures(fam):
    """Zero stripes is a successful no-op for every entry point, and a decode
    with every chunk present returns success without writing (the
    reference returns true for failed == 0, rscoding.cc:118-120)."""
    k, m, cs = 4, 2, 4096
    c = Codec(fam, k, m, cs)
    data = torch.empty(0, k, cs, dtype=torch.uint8, device="cuda")
    par = torch.empty(0, m, cs, dtype=torch.uint8, device="cuda")
    c.encode(data, par)
    c.decode(torch.empty(0, k + m, cs, dtype=torch.uint8, device="cuda"), (1 << (k + m)) - 1)
    c.encode_update(1, torch.empty(0, cs, dtype=torch.uint8, device="cuda"), par)
    base = _stripes_km(fam, k, m, cs, 4, 31)
    st = torch.from_numpy(base.copy()).to("cuda")
    c.decode(st, (1 << (k + m)) - 1)
    torch.cuda.synchronize()
    assert np.array_equal(st.cpu().numpy(), base)
    c.close()


def _stripes_km(fam, k, m, cs, n, seed):
    base = O.fill(n * (k + m) * cs, seed).reshape(n, k + m, cs)
    for s in range(n):
        base[s, k:] = np.stack(O.encode(fam, k, m, [base[s, j].copy() for j in range(k)], cs))
    return base


@pytest.mark.parametrize("group", ["0", "3:8", "7:16", "4:64", "64:8", "5:128"])
def test_stripe_group_overrides(group, knobs):
    """The stripe-group block map (stream_common.hpp stripe_tile) with
    forced groups and run lengths, a last group shorter than the rest
    (N = 20 stripes), and a run that does not tile the stripe (128 of 64
    tiles: the planner keeps the identity map); every layout stays
    bit-exact.  64 KiB chunks: 64 one-wave tiles.  Values outside the
    accepted set (a run of 7, a non-number) are refused at mec_set_knob."""
    for bad in ("bad:7", "4:7", "65"):
        with pytest.raises(MecError):
            knobs("MEC_SGROUP", bad)
    knobs("MEC_SGROUP", group)
    _check_all_layouts("rs", 65536, 1500)


def test_stripe_groups_default_rule_large_chunks(knobs):
    """Split-layout encodes with chunks of 2 MiB or more take the grouped
    map by default (16 stripes, runs of 8 tiles): RS(4,2) at 2 MiB over 19
    stripes (one full group and a short one) equals the identity map, and
    its first and last stripes equal the oracle."""
    k, m, cs, n = 4, 2, 2 << 20, 19
    knobs("MEC_SGROUP", None)
    c = Codec("rs", k, m, cs)
    data = torch.empty(n, k, cs, dtype=torch.uint8, device="cuda")
    from memec_amd import fill_random
    fill_random(data, 4242)
    par = torch.zeros(n, m, cs, dtype=torch.uint8, device="cuda")
    c.encode(data, par)
    knobs("MEC_SGROUP", "0")
    ref = torch.zeros_like(par)
    c.encode(data, ref)
    torch.cuda.synchronize()
    assert torch.equal(par, ref)
    host = data.cpu().numpy()
    got = par.cpu().numpy()
    for s in (0, n - 1):
        assert np.array_equal(got[s], np.stack(O.encode("rs", k, m, [host[s, j].copy() for j in range(k)], cs)))
    c.close()


@pytest.mark.parametrize("k,m,cs", [(8, 2, 2048), (12, 2, 2056), (12, 4, 1024), (4, 2, 520),  # tiny: split-layout launch
                                    (6, 2, 2048), (12, 4, 2048), (8, 2, 4096)])                # other side of the rule
def test_tiny_inplace_cauchy_rule(k, m, cs, knobs):
    """In-place Cauchy-RS launches of tiny stripes run as split layouts
    (bm_windows, kernels.hip: chunks <= 1 KiB, or <= 2 KiB with <= 2
    outputs and k >= 8 -> one window, one-wave blocks, split caps): in-place
    encode and decode of data + parity erasures on both sides of the rule,
    and with the windows forced back to 2, equal the oracle."""
    n = 40
    base = _stripes_km("cauchy", k, m, cs, n, 1700 + k + cs)
    c = Codec("cauchy", k, m, cs)
    erased = sorted({0, k - 1, k + m - 1})[:m]
    for win in (None, "2"):
        knobs("MEC_WINDOWS", win)
        st = torch.from_numpy(base.copy()).to("cuda")
        st[:, k:] = 0
        c.encode(st[:, :k], st[:, k:])
        torch.cuda.synchronize()
        assert np.array_equal(st.cpu().numpy(), base), ("in-place encode", k, m, cs, win)
        st[:, erased] = 0
        c.decode(st, sum(1 << i for i in range(k + m) if i not in erased))
        torch.cuda.synchronize()
        assert np.array_equal(st.cpu().numpy(), base), ("in-place decode", k, m, cs, win)
    c.close()


@pytest.mark.parametrize("skew", ["8", "64", "256"])
@pytest.mark.parametrize("fam", ["rs", "cauchy"])
def test_tile_skew_in_place(fam, skew, knobs):
    """MEC_TILE_SKEW (experiment: in-place launches rotate stripe s's tiles
    by s * skew): every layout still equals the oracle,
    at chunks with few tiles (skew reduced mod tiles) and many."""
    knobs("MEC_TILE_SKEW", skew)
    for cs in (4096, 65536 + 16):
        _check_all_layouts(fam, cs if fam == "rs" else cs - cs % 64, 900 + len(skew))


@pytest.mark.parametrize("wb", ["2", "4"])
@pytest.mark.parametrize("fam", ["rs", "isal_rs"])
def test_write_batched_in_place_decode(fam, wb, knobs):
    """MEC_WBATCH (A/B of VERDICT r05 item 3: gf8_wb_kernel stores T tiles'
    outputs per block in one burst): RS(10,4)@1 MiB in-place decodes — the
    configs[2] shape the form takes — of data, mixed and parity erasures on
    random non-codeword stripes equal the oracle (the survivor choice and
    decoding matrix included), and equal the default kernel's bytes."""
    k, m, cs, n = 10, 4, 1 << 20, 3
    base = O.fill(n * (k + m) * cs, 4242).reshape(n, k + m, cs)
    for pat in ([0, 1, 2, 3], [0, 5, 10, 13], [1, 11]):
        present = sum(1 << i for i in range(k + m) if i not in pat)
        outs = []
        for v in (wb, None):
            knobs("MEC_WBATCH", v)
            st = torch.from_numpy(base.copy()).to("cuda")
            st[:, pat] = 0
            Codec(fam, k, m, cs).decode(st, present)
            torch.cuda.synchronize()
            outs.append(st.cpu().numpy())
        assert np.array_equal(outs[0], outs[1]), (fam, wb, pat)
        for s in (0, n - 1):
            chunks = [base[s, i].copy() for i in range(k + m)]
            for e in pat:
                chunks[e][:] = 0
            assert O.decode(fam, k, m, chunks, pat, cs) == 0
            for i in range(k + m):
                assert np.array_equal(outs[0][s, i], chunks[i]), (fam, wb, pat, s, i)


@pytest.mark.parametrize("cs", [4096, 1040, 65536 + 16])
@pytest.mark.parametrize("fam", ["rs", "isal_cauchy"])
def test_gathered_xcd_runs(fam, cs, knobs):
    """MEC_GXCD=1 (one-map gathered gf8 launches deal each XCD a contiguous
    run of blocks): encode and one-pattern decode batches over scattered
    8-byte-header slots equal the oracle, tails included."""
    knobs("MEC_GXCD", "1")
    k, m, n = 8, 2, 37
    slot = cs + 8
    rng = np.random.default_rng(cs)
    host = O.fill(n * (k + m) * slot, 71 + cs)
    slab = torch.from_numpy(host.copy()).to("cuda")
    perm = rng.permutation(n * (k + m))
    addr = lambda i: slab.data_ptr() + int(i) * slot + 8  # noqa: E731
    c = Codec(fam, k, m, cs)
    rows = perm.reshape(n, k + m)
    c.encode_batch([addr(x) for x in rows[:, :k].reshape(-1)], [addr(x) for x in rows[:, k:].reshape(-1)])
    torch.cuda.synchronize()
    got = slab.cpu().numpy()
    view = lambda buf, i: buf[int(i) * slot + 8:int(i) * slot + 8 + cs]  # noqa: E731
    for s in (0, n // 2, n - 1):
        want = O.encode(fam, k, m, [view(host, x).copy() for x in rows[s, :k]], cs)
        for i in range(m):
            assert np.array_equal(view(got, rows[s, k + i]), want[i]), (s, i)
    pat = [1, 8]
    before = slab.cpu().numpy()
    res = c.decode_batch([addr(x) for x in rows.reshape(-1)], [sum(1 << i for i in range(k + m) if i not in pat)] * n)
    assert res == [0] * n
    got = slab.cpu().numpy()
    for s in (0, n - 1):
        chunks = [view(before, x).copy() for x in rows[s]]
        assert O.decode(fam, k, m, chunks, pat, cs) == 0
        for i in range(k + m):
            assert np.array_equal(view(got, rows[s, i]), chunks[i]), (s, i)


@pytest.mark.parametrize("cs", [4096, 2048, 6144, 65536, 3072])
@pytest.mark.parametrize("fam", ["rs", "isal_cauchy"])
def test_gathered_two_units_per_lane(fam, cs, knobs):
    """MEC_GU=2 (one-wave one-map gathered gf8 blocks code two 16-byte units
    per lane, a 2 KiB tile per pointer-row fetch; only where the tiles are
    whole, 3072 B falls back to one unit): encode, one-pattern decode and
    delta-update batches over 128-byte-aligned scattered chunks (the
    one-wave shape) equal the oracle on every stripe."""
    knobs("MEC_GU", "2")
    k, m, n = 8, 2, 67
    rng = np.random.default_rng(cs + 1)
    host = O.fill(n * (k + m) * cs, 91 + cs)
    slab = torch.from_numpy(host.copy()).to("cuda")
    perm = rng.permutation(n * (k + m))
    addr = lambda i: slab.data_ptr() + int(i) * cs  # noqa: E731
    view = lambda buf, i: buf[int(i) * cs:int(i) * cs + cs]  # noqa: E731
    c = Codec(fam, k, m, cs)
    rows = perm.reshape(n, k + m)
    c.encode_batch([addr(x) for x in rows[:, :k].reshape(-1)], [addr(x) for x in rows[:, k:].reshape(-1)])
    torch.cuda.synchronize()
    got = slab.cpu().numpy()
    for s in range(n):
        want = O.encode(fam, k, m, [view(host, x).copy() for x in rows[s, :k]], cs)
        for i in range(m):
            assert np.array_equal(view(got, rows[s, k + i]), want[i]), (s, i)
    pat = [0, 5]
    before = got.copy()
    for s in range(n):
        for e in pat:
            view(before, rows[s, e])[:] = 0
    slab.copy_(torch.from_numpy(before))
    res = c.decode_batch([addr(x) for x in rows.reshape(-1)], [sum(1 << i for i in range(k + m) if i not in pat)] * n)
    assert res == [0] * n
    after = slab.cpu().numpy()
    for s in range(n):
        for i in range(k + m):
            assert np.array_equal(view(after, rows[s, i]), view(got, rows[s, i])), (s, i)
    # delta update of column 3 into every stripe's parity (read-modify-write)
    delta = torch.from_numpy(O.fill(n * cs, 17 + cs).reshape(n, cs)).to("cuda")
    c.encode_update_batch([3] * n, [delta[s].data_ptr() for s in range(n)],
                          [addr(x) for x in rows[:, k:].reshape(-1)])
    upd = slab.cpu().numpy()
    dh = delta.cpu().numpy()
    for s in range(n):
        d2 = [view(got, x).copy() for x in rows[s, :k]]
        d2[3] ^= dh[s]
        want = O.encode(fam, k, m, d2, cs)
        for i in range(m):
            assert np.array_equal(view(upd, rows[s, k + i]), want[i]), (s, i)
