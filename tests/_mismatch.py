"""Mismatch maps for host-path parity assertions.

A bare `np.array_equal` failure says only that a chunk differs.  `same()`
raises with a map of where and how: the differing byte ranges (chunk
offsets), the 4 KiB pages and 1 KiB tiles they fall in (by absolute host
address when the chunk's address is known, so a range that follows page or
cache-line boundaries shows), and — given the chunk's contents before the
call — how many of the wrong bytes still hold those pre-call bytes (stores
that never became visible) against bytes that are neither (wrong data).
"""
import numpy as np


def _ranges(idx, limit=12):
    """[(first, last)] runs of consecutive indices, at most `limit`."""
    out = []
    if idx.size == 0:
        return out, 0
    cuts = np.nonzero(np.diff(idx) != 1)[0]
    starts = np.concatenate(([idx[0]], idx[cuts + 1]))
    ends = np.concatenate((idx[cuts], [idx[-1]]))
    for a, b in zip(starts[:limit], ends[:limit]):
        out.append((int(a), int(b)))
    return out, len(starts)


def mismatch_map(got, want, before=None, addr=None):
    got = np.asarray(got, np.uint8).reshape(-1)
    want = np.asarray(want, np.uint8).reshape(-1)
    if got.shape != want.shape:
        return "shape %s != %s" % (got.shape, want.shape)
    idx = np.nonzero(got != want)[0]
    if idx.size == 0:
        return "equal"
    runs, nruns = _ranges(idx)
    lines = ["%d of %d bytes differ in %d run(s): %s%s" % (
        idx.size, got.size, nruns, ", ".join("[%d..%d]" % r for r in runs), " ..." if nruns > len(runs) else "")]
    base = int(addr) if addr is not None else 0
    absb = idx + base
    pages = np.unique(absb // 4096)
    tiles = np.unique(idx // 1024)
    lines.append("addr %s; pages touched %d (%s); 1 KiB chunk tiles %s; first/last byte mod 128 of abs addr: %d / %d" % (
        hex(base) if addr is not None else "unknown", pages.size,
        ", ".join(hex(int(p) * 4096) for p in pages[:6]) + (" ..." if pages.size > 6 else ""),
        tiles[:16].tolist() + (["..."] if tiles.size > 16 else []), int(absb[0] % 128), int((absb[-1] + 1) % 128)))
    if before is not None:
        before = np.asarray(before, np.uint8).reshape(-1)
        stale = int((got[idx] == before[idx]).sum())
        zeros = int((got[idx] == 0).sum())
        lines.append("of the wrong bytes: %d equal the pre-call contents (stores not visible), %d are zero, %d are "
                     "neither (wrong data)" % (stale, zeros, idx.size - stale))
    lines.append("first bytes got %s want %s" % (got[idx[:8]].tolist(), want[idx[:8]].tolist()))
    return "\n".join(lines)


def same(got, want, what="", before=None, addr=None):
    """assert got == want bytewise, with a mismatch map on failure."""
    if np.array_equal(got, want):
        return
    raise AssertionError("%s: %s" % (what, mismatch_map(got, want, before, addr)))
