"""GPU parity of the device-side submission queue (mec_set_host_queue,
memec_amd/csrc/queue.hip): single-stripe host calls on registered chunks
posted to a resident kernel instead of launched.  Bit-exact against the
oracle for encode(index) / decode / delta update, under concurrent callers
(MemEC's workers share one Coding, worker.cc:128-137), across an idle exit
and relaunch, and with the launch path taking what the queue does not serve
(chunks above MEC_QUEUE_MAX_CHUNK, queue stopped).  Jerasure Cauchy-RS
(bitmatrix over w packets) is served too.  Unregistered (staged) chunks
reach the queue through mapped pinned lanes.  The grid-wide idle exit keeps
a caller on a quiet slot from stranding while another slot stays busy, and
a timed-out call withdraws its job and falls back to the launch path.
"""
import ctypes
import os
import threading
import time

import numpy as np
import pytest

import _oracle as O
from _mismatch import same

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

from memec_amd import Codec, host_register, host_unregister  # noqa: E402
from memec_amd._lib import check, lib  # noqa: E402

vp = ctypes.c_void_p
BYTEWISE = ["rs", "isal_rs", "isal_cauchy"]
FAMILIES = BYTEWISE + ["cauchy"]


@pytest.fixture(scope="module", autouse=True)
def _gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    torch.cuda.set_device(0)
    yield
    torch.cuda.synchronize()


def aligned(nbytes, align=4096):
    raw = np.empty(nbytes + align, np.uint8)
    off = (-raw.ctypes.data) % align
    return raw[off:off + nbytes]


class Slab:
    """Registered ChunkPool-like slab: slots of 8 + cs bytes (chunk_pool.cc:22-95)."""

    def __init__(self, n, cs, seed):
        self.cs, self.slot = cs, cs + 8
        self.buf = aligned(n * self.slot)
        self.buf[:] = O.fill(self.buf.nbytes, seed)
        host_register(self.buf)

    def close(self):
        host_unregister(self.buf)

    def addr(self, i):
        return self.buf.ctypes.data + i * self.slot + 8

    def view(self, i):
        o = i * self.slot + 8
        return self.buf[o:o + self.cs]


def encode_index(c, slab, k, dslots, pslot, index):
    """Coding::encode(data, parity, index): parity row index-1 only."""
    dp = (vp * k)(*[vp(slab.addr(s)) if s is not None else vp() for s in dslots])
    pp = (vp * c.m)(*[vp(slab.addr(pslot)) if i == index - 1 else vp() for i in range(c.m)])
    check(lib().mec_encode_host(c._h, dp, pp))


@pytest.mark.parametrize("fam", FAMILIES)
@pytest.mark.parametrize("k,m,cs", [(8, 2, 4096), (10, 4, 16384), (4, 2, 4104), (12, 4, 1024), (20, 4, 2048)])
def test_queue_encode_decode_update(fam, k, m, cs):
    """Cauchy w: 4 (packets of 1 KiB, 4 KiB, 256 B), 3 (1368 B), 8 (256 B)."""
    _encode_decode_update(fam, k, m, cs)


@pytest.mark.parametrize("devslot", ["0", "1"])
@pytest.mark.parametrize("fam", FAMILIES)
def test_queue_slot_placement(fam, devslot, qenv):
    """Slot descriptors in device memory written through the BAR (the
    default on large-BAR devices) and in host memory (MEC_QUEUE_DEVSLOT=0):
    same results, single- and multi-part slots, and the placement is
    reported."""
    qenv(MEC_QUEUE_DEVSLOT=devslot, MEC_QUEUE_MAX_CHUNK=128 << 10)
    for k, m, cs, parts in [(8, 2, 4096, 1), (10, 4, 65536, 4)]:
        _encode_decode_update(fam, k, m, cs, parts=parts)
    c = Codec(fam, 4, 2, 4096)
    try:
        c.set_host_queue(2)
        if devslot == "0":
            assert not c.stats()["queue_devslot"]
        elif not c.stats()["queue_devslot"]:
            pytest.skip("no large BAR: host-memory slots only")
    finally:
        c.close()


@pytest.mark.parametrize("k,m,cs", [(4, 2, 4100), (3, 1, 24), (12, 4, 16376), (6, 3, 4104)])
def test_queue_cauchy_packet_tails(k, m, cs):
    """Bitmatrix packets that are not whole 8-byte units: w=4 / 1025 B,
    w=2 / 12 B, w=4 / 4094 B, w=4 / 1026 B."""
    _encode_decode_update("cauchy", k, m, cs)


def auto_parts(cs):
    """queue_start's rule: one part per 16 KiB of chunk, below 64 KiB one
    per 8 KiB up to 4 (queue.hip)."""
    units = (cs + 15) // 16
    return min(64, max(1, (units + 1023) // 1024, min(4, (units + 511) // 512)))


def _encode_decode_update(fam, k, m, cs, parts=None, slots=8):
    parts = auto_parts(cs) if parts is None else parts
    slab = Slab(k + m + 1, cs, 31 + k)
    c = Codec(fam, k, m, cs)
    try:
        c.set_host_queue(8)
        st = c.stats()
        assert st["queue_parts"] == parts
        # slots=None: capped by the device (at most half its resident 1024-thread workgroups)
        assert st["queue_slots"] == slots if slots else 1 <= st["queue_slots"] * parts <= 128
        data = [slab.view(j).copy() for j in range(k)]
        want = O.encode(fam, k, m, [d.copy() for d in data], cs)
        q0 = c.stats()["queue_calls"]
        for i in range(m):  # the SEAL pattern: encode(index) for every parity
            encode_index(c, slab, k, list(range(k)), k + i, i + 1)
        for i in range(m):
            same(slab.view(k + i), want[i], (fam, i))
        assert c.stats()["queue_calls"] == q0 + m
        # Coding::zeros sources (NULL) in a single-column encode
        single = [None] * k
        single[2] = 2
        encode_index(c, slab, k, single, k + m, 1)
        z = [np.zeros(cs, np.uint8)] * k
        z = list(z)
        z[2] = data[2].copy()
        same(slab.view(k + m), O.encode(fam, k, m, z, cs)[0], "")
        # decode in place, data and parity erased
        orig = [slab.view(i).copy() for i in range(k + m)]
        pat = sorted({0, k - 1, k, k + m - 1})[:m]
        for e in pat:
            slab.view(e)[:] = 0
        c.decode_host([slab.view(i) for i in range(k + m)], sum(1 << i for i in range(k + m) if i not in pat))
        for i in range(k + m):
            same(slab.view(i), orig[i], (fam, pat, i))
        # delta update of every parity (the spare slot holds the delta)
        delta = slab.view(k + m)
        d2 = [o.copy() for o in orig[:k]]
        d2[1] ^= delta
        c.encode_update_host(1, delta, [slab.view(k + i) for i in range(m)])
        want2 = O.encode(fam, k, m, d2, cs)
        for i in range(m):
            same(slab.view(k + i), want2[i], (fam, i))
        st = c.stats()
        assert st["queue_calls"] == q0 + m + 3 and st["queue_launches"] >= 1
    finally:
        c.close()
        slab.close()


@pytest.fixture
def qenv():
    """Queue settings read at mec_set_host_queue (never on a call path)."""
    keys = []

    def set_(**kv):
        for k_, v in kv.items():
            keys.append(k_)
            os.environ[k_] = str(v)
    yield set_
    for k_ in keys:
        os.environ.pop(k_, None)


@pytest.mark.parametrize("fam", FAMILIES)
@pytest.mark.parametrize("k,m,cs", [(10, 4, 65536), (12, 4, 32768), (4, 2, 65536 + 40), (6, 3, 20480 + 24)])
def test_queue_multi_part_slots(fam, k, m, cs, qenv):
    """Chunks above 16 KiB on the queue: one call's units are spread over
    the slot's parts (workgroups on different CUs), each with its own done
    word; partial units and bitmatrix packet tails land on the right part."""
    qenv(MEC_QUEUE_MAX_CHUNK=128 << 10)
    _encode_decode_update(fam, k, m, cs)


@pytest.mark.parametrize("fam", ["rs", "cauchy"])
def test_queue_default_cut_1mib(fam):
    """The default chunk cut (1 MiB): 64 parts of 1024 threads per slot,
    and the resident grid capped at half of what the device holds (256 CUs
    x one 1024-thread workgroup -> 128 -> 2 slots of 64 parts)."""
    _encode_decode_update(fam, 6, 3, 1 << 20, parts=64, slots=None)


@pytest.mark.parametrize("pthr", [64, 256])
def test_queue_one_wave_parts(pthr, qenv):
    """Many small parts per slot (MEC_QUEUE_PART_THREADS): 64-thread parts
    build their coefficient tables in several passes (4 x 32 > 64)."""
    qenv(MEC_QUEUE_MAX_CHUNK=65536, MEC_QUEUE_PART_THREADS=pthr)
    for fam, k, m, cs in (("rs", 20, 4, 32768), ("isal_cauchy", 12, 4, 16384), ("cauchy", 10, 4, 65536)):
        _encode_decode_update(fam, k, m, cs, parts=min(64, (cs // 16 + pthr - 1) // pthr))


@pytest.mark.parametrize("parts", [2, 3, 8])
def test_queue_forced_parts(parts, qenv):
    """MEC_QUEUE_PARTS splits even small chunks (uneven shares: 3 parts of
    a 16 KiB chunk, 8 parts of a 4 KiB one leave some parts idle)."""
    qenv(MEC_QUEUE_PARTS=parts)
    for fam, k, m, cs in (("rs", 10, 4, 16384), ("cauchy", 8, 2, 4096)):
        _encode_decode_update(fam, k, m, cs, parts=parts)


def test_queue_multi_part_idle_exit_concurrent(qenv):
    """Parts follow part 0 out of the grid (the `left` epoch) and back in
    after a relaunch: 8 threads x 64 KiB calls, quiet gaps longer than the
    idle timeout between bursts, every result checked."""
    qenv(MEC_QUEUE_MAX_CHUNK=65536, MEC_QUEUE_IDLE_MS=3)
    k, m, cs, T = 10, 4, 65536, 8
    slab = Slab(T * (k + m), cs, 17)
    c = Codec("rs", k, m, cs)
    errs = []
    try:
        c.set_host_queue(8)
        assert c.stats()["queue_parts"] == 4
        wants = [O.encode("rs", k, m, [slab.view(t * (k + m) + j).copy() for j in range(k)], cs) for t in range(T)]

        def worker(t):
            try:
                base = t * (k + m)
                for n in range(12):
                    i = n % m
                    slab.view(base + k + i)[:] = 0
                    encode_index(c, slab, k, [base + j for j in range(k)], base + k + i, i + 1)
                    if not np.array_equal(slab.view(base + k + i), wants[t][i]):
                        errs.append((t, n))
            except Exception as e:  # noqa: BLE001
                errs.append(repr(e))
        for burst in range(3):
            th = [threading.Thread(target=worker, args=(t,)) for t in range(T)]
            for x in th:
                x.start()
            for x in th:
                x.join()
            time.sleep(0.05)  # the grid idles out
        assert not errs, errs[:5]
        st = c.stats()
        assert st["queue_calls"] > 0 and st["queue_launches"] >= 2 and not st["queue_broken"]
    finally:
        c.close()
        slab.close()


def test_queue_concurrent_callers():
    """16 threads share one context; every call's parity checked."""
    k, m, cs, T, per = 8, 2, 4096, 16, 40
    slab = Slab(T * (k + m), cs, 5)
    c = Codec("rs", k, m, cs)
    errs = []
    try:
        c.set_host_queue(8)  # fewer slots than callers: the rest take the launch path
        wants = [O.encode("rs", k, m, [slab.view(t * (k + m) + j).copy() for j in range(k)], cs) for t in range(T)]
        st0 = c.stats()

        def worker(t):
            try:
                base = t * (k + m)
                for n in range(per):
                    i = n % m
                    slab.view(base + k + i)[:] = 0
                    encode_index(c, slab, k, [base + j for j in range(k)], base + k + i, i + 1)
                    if not np.array_equal(slab.view(base + k + i), wants[t][i]):
                        errs.append((t, n))
            except Exception as e:  # noqa: BLE001
                errs.append(repr(e))

        th = [threading.Thread(target=worker, args=(t,)) for t in range(T)]
        for x in th:
            x.start()
        for x in th:
            x.join()
        assert not errs, errs[:5]
        st = c.stats()
        served = st["queue_calls"] - st0["queue_calls"]
        launched = st["zero_copy_calls"] - st0["zero_copy_calls"] - served
        assert served > 0 and served + launched == T * per
    finally:
        c.close()
        slab.close()


def test_queue_idle_exit_and_relaunch():
    k, m, cs = 6, 3, 8192
    os.environ["MEC_QUEUE_IDLE_MS"] = "5"
    slab = Slab(k + m, cs, 8)
    c = Codec("rs", k, m, cs)
    try:
        c.set_host_queue(4)
        want = O.encode("rs", k, m, [slab.view(j).copy() for j in range(k)], cs)
        for rnd in range(4):
            slab.view(k)[:] = 0
            encode_index(c, slab, k, list(range(k)), k, 1)
            same(slab.view(k), want[0], rnd)
            time.sleep(0.05)  # > idle: the resident kernel exits
        st = c.stats()
        assert st["queue_calls"] == 4 and st["queue_launches"] >= 2
    finally:
        os.environ.pop("MEC_QUEUE_IDLE_MS", None)
        c.close()
        slab.close()


def test_queue_quiet_slot_beside_busy_slot():
    """one caller keeps a slot busy while a second caller
    posts to another slot only every few idle periods.  The idle exit is
    grid-wide, so the quiet caller is never left waiting on a workgroup that
    has left while the rest of the grid keeps the stream busy."""
    k, m, cs = 8, 2, 4096
    os.environ["MEC_QUEUE_IDLE_MS"] = "5"
    slab = Slab(2 * (k + m), cs, 77)
    c = Codec("rs", k, m, cs)
    stop = threading.Event()
    errs, slow = [], []
    try:
        c.set_host_queue(2)
        wants = [O.encode("rs", k, m, [slab.view(b + j).copy() for j in range(k)], cs) for b in (0, k + m)]

        def busy():
            try:
                while not stop.is_set():
                    slab.view(k)[:] = 0
                    encode_index(c, slab, k, list(range(k)), k, 1)
                    if not np.array_equal(slab.view(k), wants[0][0]):
                        errs.append("busy")
            except Exception as e:  # noqa: BLE001
                errs.append(repr(e))

        th = threading.Thread(target=busy)
        th.start()
        b = k + m
        for rnd in range(12):
            time.sleep(0.02)  # 4 idle periods of the quiet slot
            slab.view(b + k + 1)[:] = 0
            t0 = time.perf_counter()
            encode_index(c, slab, k, [b + j for j in range(k)], b + k + 1, 2)
            dt = time.perf_counter() - t0
            if dt > 0.5:
                slow.append((rnd, dt))
            same(slab.view(b + k + 1), wants[1][1], rnd)
        stop.set()
        th.join()
        assert not errs, errs[:5]
        assert not slow, slow
    finally:
        stop.set()
        os.environ.pop("MEC_QUEUE_IDLE_MS", None)
        c.close()
        slab.close()


@pytest.mark.parametrize("fam", ["rs", "cauchy"])
def test_queue_timeout_withdraws_and_falls_back(fam):
    """a call that sees no completion in time withdraws
    its job, stops the queue for good and — when the job never ran — codes
    on the launch path.  MEC_QUEUE_TIMEOUT_MS=0 makes the first call time
    out at once; every result stays exact, and later calls use launches."""
    k, m, cs = 6, 3, 4096
    os.environ["MEC_QUEUE_TIMEOUT_MS"] = "0"
    slab = Slab(k + m, cs, 91)
    c = Codec(fam, k, m, cs)
    try:
        c.set_host_queue(4)
        want = O.encode(fam, k, m, [slab.view(j).copy() for j in range(k)], cs)
        for rnd in range(3):
            for i in range(m):
                slab.view(k + i)[:] = 0
                encode_index(c, slab, k, list(range(k)), k + i, i + 1)
                same(slab.view(k + i), want[i], (rnd, i))
        st = c.stats()
        assert st["queue_broken"] and st["queue_timeouts"] >= 1
        assert st["queue_calls"] <= 1  # at most the first call, if it beat the withdrawal
        assert st["zero_copy_calls"] == 3 * m
        # staged calls on the broken queue take launches too
        data = [O.fill(cs, 300 + j) for j in range(k)]
        got = c.encode_host(data)
        w2 = O.encode(fam, k, m, [d.copy() for d in data], cs)
        for i in range(m):
            same(got[i], w2[i], "")
    finally:
        os.environ.pop("MEC_QUEUE_TIMEOUT_MS", None)
        c.close()
        slab.close()


@pytest.mark.parametrize("fam", ["rs", "cauchy"])
def test_queue_timeout_multipart_all_or_nothing(fam):
    """the timeout path on a multi-part slot (64 KiB
    chunks: 4 workgroups per slot).  After the withdrawal the caller checks
    every part's done word: all -> the job ran, none -> the launch path codes
    it; so encodes and accumulating delta updates (which must not be applied
    twice) stay exact whichever way each call went."""
    k, m, cs = 6, 3, 65536
    os.environ["MEC_QUEUE_TIMEOUT_MS"] = "0"
    slab = Slab(k + m + 1, cs, 93)
    c = Codec(fam, k, m, cs)
    try:
        c.set_host_queue(4)
        assert c.stats()["queue_parts"] == 4
        data = [slab.view(j).copy() for j in range(k)]
        want = O.encode(fam, k, m, [d.copy() for d in data], cs)
        for i in range(m):
            slab.view(k + i)[:] = 0
            encode_index(c, slab, k, list(range(k)), k + i, i + 1)
            same(slab.view(k + i), want[i], i)
        # accumulate: parity ^= A[:, 2] * delta, twice -> back to `want`, and
        # once more -> the encode of data with column 2 ^= delta
        delta = slab.view(k + m)
        for rnd in range(3):
            c.encode_update_host(2, delta, [slab.view(k + i) for i in range(m)])
        d2 = [d.copy() for d in data]
        d2[2] ^= delta
        want2 = O.encode(fam, k, m, d2, cs)
        for i in range(m):
            same(slab.view(k + i), want2[i], i)
        st = c.stats()
        assert st["queue_broken"] and st["queue_timeouts"] >= 1
    finally:
        os.environ.pop("MEC_QUEUE_TIMEOUT_MS", None)
        c.close()
        slab.close()


def test_queue_fallbacks():
    """Calls the queue does not serve still code correctly through launches."""
    k, m = 4, 2
    # chunk above MEC_QUEUE_MAX_CHUNK (default 1 MiB), then the queue stopped
    cs = (1 << 20) + 4096
    slab = Slab(k + m, cs, 4)
    c = Codec("rs", k, m, cs)
    try:
        c.set_host_queue(4)
        want = O.encode("rs", k, m, [slab.view(j).copy() for j in range(k)], cs)
        encode_index(c, slab, k, list(range(k)), k + 1, 2)
        same(slab.view(k + 1), want[1], "")
        assert c.stats()["queue_calls"] == 0
        c.set_host_queue(0)
        slab.view(k + 1)[:] = 0
        encode_index(c, slab, k, list(range(k)), k + 1, 2)
        same(slab.view(k + 1), want[1], "")
    finally:
        c.close()
        slab.close()
    # unregistered chunks above the queue's chunk limit: staged + launched
    cs = (1 << 20) + 4096
    c = Codec("rs", k, m, cs)
    try:
        c.set_host_queue(4)
        data = [O.fill(cs, 70 + j) for j in range(k)]
        got = c.encode_host(data)
        want = O.encode("rs", k, m, [d.copy() for d in data], cs)
        for i in range(m):
            same(got[i], want[i], "")
        st = c.stats()
        assert st["queue_calls"] == 0 and st["staged_calls"] == 1
    finally:
        c.close()


@pytest.mark.parametrize("fam", FAMILIES)
@pytest.mark.parametrize("k,m,cs", [(8, 2, 4096), (10, 4, 16384), (4, 2, 4104), (20, 4, 2048)])
def test_queue_staged_calls(fam, k, m, cs):
    """Unregistered host chunks go through a lane's mapped pinned buffer to
    the resident kernel.  The same lanes are reused call after call with new
    contents, so stale lines from an earlier call would show up here."""
    c = Codec(fam, k, m, cs)
    try:
        c.set_host_queue(4)
        st0 = c.stats()
        for rnd in range(6):
            data = [O.fill(cs, 1000 * rnd + 10 * k + j) for j in range(k)]
            want = O.encode(fam, k, m, [d.copy() for d in data], cs)
            got = c.encode_host(data)
            for i in range(m):
                same(got[i], want[i], (rnd, i))
            chunks = [d.copy() for d in data] + [w.copy() for w in want]
            pat = sorted({rnd % k, k - 1, k + rnd % m})[:m]
            for e in pat:
                chunks[e][:] = 0
            c.decode_host(chunks, sum(1 << i for i in range(k + m) if i not in pat))
            for i in range(k + m):
                same(chunks[i], data[i] if i < k else want[i - k], (rnd, pat, i))
            delta = O.fill(cs, 7777 + rnd)
            par = [w.copy() for w in want]
            c.encode_update_host(rnd % k, delta, par)
            d2 = [d.copy() for d in data]
            d2[rnd % k] ^= delta
            want2 = O.encode(fam, k, m, d2, cs)
            for i in range(m):
                same(par[i], want2[i], (rnd, i))
        st = c.stats()
        assert st["queue_calls"] - st0["queue_calls"] == 18
        assert st["staged_calls"] - st0["staged_calls"] == 18
    finally:
        c.close()


def test_queue_staged_concurrent_callers():
    """16 threads of unregistered single-stripe encodes through 8 slots."""
    k, m, cs, T, per = 8, 2, 4096, 16, 30
    c = Codec("rs", k, m, cs)
    errs = []
    try:
        c.set_host_queue(8)
        st0 = c.stats()

        def worker(t):
            try:
                for n in range(per):
                    data = [O.fill(cs, 100000 * t + 100 * n + j) for j in range(k)]
                    want = O.encode("rs", k, m, [d.copy() for d in data], cs)
                    got = c.encode_host(data)
                    if not all(np.array_equal(got[i], want[i]) for i in range(m)):
                        errs.append((t, n))
            except Exception as e:  # noqa: BLE001
                errs.append(repr(e))

        th = [threading.Thread(target=worker, args=(t,)) for t in range(T)]
        for x in th:
            x.start()
        for x in th:
            x.join()
        assert not errs, errs[:5]
        st = c.stats()
        assert st["staged_calls"] - st0["staged_calls"] == T * per
        assert st["queue_calls"] - st0["queue_calls"] > 0
    finally:
        c.close()
