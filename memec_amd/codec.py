"""Python host binding of libmec for tests, bench and Python callers.

Device-resident batches are torch uint8 CUDA tensors shaped
[stripes, chunks, chunk_size] (any stripe/chunk strides, unit byte stride);
work is enqueued on torch's current stream.  Host entry points take numpy
uint8 arrays.  Every call goes through the C ABI (include/mec.h) into the
HIP kernels; there is no CPU fallback.
"""
import ctypes

import numpy as np

from . import _lib
from ._lib import check, lib

vp = ctypes.c_void_p


def _stream(stream):
    if stream is not None:
        return vp(stream)
    import torch
    return vp(torch.cuda.current_stream().cuda_stream)


def _dev3(t, name):
    if not t.is_cuda or t.dtype.itemsize != 1 or t.dim() != 3 or t.stride(2) != 1:
        raise ValueError("%s must be a uint8 CUDA tensor [stripes, chunks, bytes] with unit byte stride" % name)
    return vp(t.data_ptr()), t.stride(0), t.stride(1)


class Codec:
    """One coding context: family in {"rs", "cauchy", "isal_rs", "isal_cauchy"}.

    device=-1 makes a host-only context (matrices only; compute raises)."""

    def __init__(self, family, k, m, chunk_size, device=0, devices=None):
        """devices: list of GPU ordinals -> a multi-GPU context (host-memory
        batches split over them, include/mec.h mec_create_multi)."""
        self._h = vp()
        fam = _lib.FAMILIES[family] if isinstance(family, str) else int(family)
        if devices is not None:
            arr = (ctypes.c_int * len(devices))(*devices)
            check(lib().mec_create_multi(fam, k, m, chunk_size, arr, len(devices), ctypes.byref(self._h)))
        else:
            check(lib().mec_create(fam, k, m, chunk_size, device, ctypes.byref(self._h)))
        inf = _lib.MecInfo()
        check(lib().mec_get_info(self._h, ctypes.byref(inf)))
        self.family, self.k, self.m, self.w = family, inf.k, inf.m, inf.w
        self.chunk_size, self.packet_size, self.device = inf.chunk_size, inf.packet_size, inf.device

    def close(self):
        if self._h:
            lib().mec_destroy(self._h)
            self._h = vp()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    # ---- matrices -----------------------------------------------------------
    def matrix(self):
        cap = (self.k + self.m) * self.k
        out = (ctypes.c_int32 * cap)()
        n = check(lib().mec_get_matrix(self._h, out, cap))
        return list(out)[:n]

    def bitmatrix(self):
        cap = self.m * self.w * self.k * self.w
        out = (ctypes.c_int32 * cap)()
        n = check(lib().mec_get_bitmatrix(self._h, out, cap))
        return list(out)[:n]

    # ---- device batches -------------------------------------------------------
    def encode(self, data, parity, parity_mask=0, stream=None):
        d, dss, dcs = _dev3(data, "data")
        p, pss, pcs = _dev3(parity, "parity")
        n = data.shape[0]
        if parity.shape[0] != n or data.shape[1] < self.k or parity.shape[1] < self.m:
            raise ValueError("shape mismatch")
        if data.shape[2] != self.chunk_size or parity.shape[2] != self.chunk_size:
            raise ValueError("chunk size mismatch")
        check(lib().mec_encode(self._h, d, dss, dcs, p, pss, pcs, n, parity_mask, _stream(stream)))

    def decode(self, chunks, present_mask, stream=None):
        c, ss, cs = _dev3(chunks, "chunks")
        if chunks.shape[1] < self.k + self.m or chunks.shape[2] != self.chunk_size:
            raise ValueError("shape mismatch")
        check(lib().mec_decode(self._h, c, ss, cs, chunks.shape[0], present_mask, _stream(stream)))

    def decode_split(self, src, dst, present_mask, stream=None):
        a, ass, acs = _dev3(src, "src")
        b, bss, bcs = _dev3(dst, "dst")
        if src.shape[0] != dst.shape[0]:
            raise ValueError("shape mismatch")
        check(lib().mec_decode_split(self._h, a, ass, acs, b, bss, bcs, src.shape[0], present_mask,
                                     _stream(stream)))

    def encode_update(self, data_index, delta, parity, parity_mask=0, stream=None):
        if not delta.is_cuda or delta.dim() != 2 or delta.stride(1) != 1:
            raise ValueError("delta must be a uint8 CUDA tensor [stripes, bytes]")
        p, pss, pcs = _dev3(parity, "parity")
        check(lib().mec_encode_update(self._h, data_index, vp(delta.data_ptr()), delta.stride(0), p, pss, pcs,
                                      parity.shape[0], parity_mask, _stream(stream)))

    # ---- host, one stripe -------------------------------------------------------
    def encode_host(self, data, want=None):
        """data: k numpy uint8 arrays (None = all-zero chunk).  Returns the
        wanted parities (list; None where not wanted)."""
        cs = self.chunk_size
        want = [True] * self.m if want is None else want
        out = [np.empty(cs, np.uint8) if w else None for w in want]
        dp = (vp * self.k)(*[vp(a.ctypes.data) if a is not None else vp() for a in data])
        pp = (vp * self.m)(*[vp(a.ctypes.data) if a is not None else vp() for a in out])
        check(lib().mec_encode_host(self._h, dp, pp))
        return out

    def decode_host(self, chunks, present_mask):
        cp = (vp * (self.k + self.m))(*[vp(a.ctypes.data) for a in chunks])
        check(lib().mec_decode_host(self._h, cp, present_mask))

    def encode_update_host(self, data_index, delta, parity):
        pp = (vp * self.m)(*[vp(a.ctypes.data) if a is not None else vp() for a in parity])
        check(lib().mec_encode_update_host(self._h, data_index, vp(delta.ctypes.data), pp))

    def encode_host_batch(self, data, parity, parity_mask=0):
        """data: numpy [S, k, cs] contiguous; parity: numpy [S, m, cs] contiguous."""
        assert data.flags.c_contiguous and parity.flags.c_contiguous
        check(lib().mec_encode_host_batch(self._h, vp(data.ctypes.data), vp(parity.ctypes.data),
                                          data.shape[0], parity_mask))


    # ---- pointer-array batches (any memory kind) ----------------------------------
    # Pointers are integers (0 = NULL), one row per stripe: k data / m parity
    # for encode, k + m chunks for decode.  mem: "device" (CUDA tensor
    # addresses, enqueued on the stream) or "host" (numpy addresses,
    # synchronous; zero-copy on registered memory, else pinned staging).
    @staticmethod
    def _ptr_array(ptrs):
        """uint64 numpy array (zero-copy) or a sequence of ints -> (void**, keepalive)."""
        a = np.ascontiguousarray(np.asarray(ptrs, dtype=np.uint64))
        return ctypes.cast(a.ctypes.data, ctypes.POINTER(vp)), a

    @staticmethod
    def _mem(mem):
        return {"device": _lib.MEM_DEVICE, "host": _lib.MEM_HOST}[mem]

    def _stream_for(self, mem, stream):
        return _stream(stream) if mem == "device" else vp()

    def encode_batch(self, data_ptrs, parity_ptrs, parity_mask=0, mem="device", stream=None):
        n = len(data_ptrs) // self.k
        if len(data_ptrs) != n * self.k or len(parity_ptrs) != n * self.m:
            raise ValueError("need n*k data and n*m parity pointers")
        dp, _a = self._ptr_array(data_ptrs)
        pp, _b = self._ptr_array(parity_ptrs)
        check(lib().mec_encode_batch(self._h, dp, pp, n, parity_mask, self._mem(mem), self._stream_for(mem, stream)))

    @staticmethod
    def _results(rc, res, as_array):
        """Per-stripe statuses (numpy int32) -> list, or the array itself
        (as_array: no per-stripe Python objects, for large batches)."""
        if rc < 0 and not (res == rc).any():  # a failure not attributable to one stripe
            check(rc)
        return res if as_array else res.tolist()

    def decode_batch(self, chunk_ptrs, present_masks, mem="device", stream=None, as_array=False):
        """Returns the per-stripe status list (0 ok, MEC_ETOOMANY, ...), or
        a numpy int32 array with as_array=True."""
        n = len(present_masks)
        if len(chunk_ptrs) != n * (self.k + self.m):
            raise ValueError("need n*(k+m) chunk pointers")
        cp, _a = self._ptr_array(chunk_ptrs)
        pmv = np.ascontiguousarray(np.asarray(present_masks, dtype=np.uint64))
        pm = ctypes.cast(pmv.ctypes.data, ctypes.POINTER(_lib.u64))
        res = np.zeros(n, np.int32)
        rc = lib().mec_decode_batch(self._h, cp, pm, n, ctypes.cast(res.ctypes.data, ctypes.POINTER(ctypes.c_int32)),
                                    self._mem(mem), self._stream_for(mem, stream))
        return self._results(rc, res, as_array)

    def encode_update_batch(self, data_index, delta_ptrs, parity_ptrs, parity_mask=0, mem="device", stream=None):
        n = len(data_index)
        if len(delta_ptrs) != n or len(parity_ptrs) != n * self.m:
            raise ValueError("need n deltas and n*m parity pointers")
        div = np.ascontiguousarray(np.asarray(data_index, dtype=np.uint32))
        di = ctypes.cast(div.ctypes.data, ctypes.POINTER(_lib.u32))
        dp, _a = self._ptr_array(delta_ptrs)
        pp, _b = self._ptr_array(parity_ptrs)
        check(lib().mec_encode_update_batch(self._h, di, dp, pp, n, parity_mask, self._mem(mem),
                                            self._stream_for(mem, stream)))

    # ---- pointer batches as 32-bit slab offsets (device memory, ABI 6) -------------
    # base: device address of the slab (int or CUDA tensor); offsets in units
    # of 1 << unit_shift bytes, _lib.NULL_OFF = NULL.
    @staticmethod
    def _u32_array(vals):
        a = np.ascontiguousarray(np.asarray(vals, dtype=np.uint32))
        return ctypes.cast(a.ctypes.data, ctypes.POINTER(_lib.u32)), a

    @staticmethod
    def _base(base):
        return vp(base.data_ptr() if hasattr(base, "data_ptr") else int(base))

    def encode_batch32(self, base, unit_shift, data_off, parity_off, parity_mask=0, stream=None):
        n = len(data_off) // self.k
        if len(data_off) != n * self.k or len(parity_off) != n * self.m:
            raise ValueError("need n*k data and n*m parity offsets")
        d, _a = self._u32_array(data_off)
        p, _b = self._u32_array(parity_off)
        check(lib().mec_encode_batch32(self._h, self._base(base), unit_shift, d, p, n, parity_mask, _stream(stream)))

    def decode_batch32(self, base, unit_shift, chunk_off, present_masks, stream=None, as_array=False):
        n = len(present_masks)
        if len(chunk_off) != n * (self.k + self.m):
            raise ValueError("need n*(k+m) chunk offsets")
        o, _a = self._u32_array(chunk_off)
        pmv = np.ascontiguousarray(np.asarray(present_masks, dtype=np.uint64))
        pm = ctypes.cast(pmv.ctypes.data, ctypes.POINTER(_lib.u64))
        res = np.zeros(n, np.int32)
        rc = lib().mec_decode_batch32(self._h, self._base(base), unit_shift, o, pm, n,
                                      ctypes.cast(res.ctypes.data, ctypes.POINTER(ctypes.c_int32)), _stream(stream))
        return self._results(rc, res, as_array)

    def encode_update_batch32(self, base, unit_shift, data_index, delta_off, parity_off, parity_mask=0, stream=None):
        n = len(data_index)
        if len(delta_off) != n or len(parity_off) != n * self.m:
            raise ValueError("need n deltas and n*m parity offsets")
        di, _a = self._u32_array(data_index)
        d, _b = self._u32_array(delta_off)
        p, _c = self._u32_array(parity_off)
        check(lib().mec_encode_update_batch32(self._h, self._base(base), unit_shift, di, d, p, n, parity_mask,
                                              _stream(stream)))

    def set_coalescing(self, max_batch):
        check(lib().mec_set_coalescing(self._h, max_batch))

    def set_host_queue(self, slots):
        """Resident submission-queue kernel for single-stripe calls on
        registered host memory (mec_set_host_queue); 0 stops it."""
        check(lib().mec_set_host_queue(self._h, slots))

    def set_probe(self, on):
        """Measurement only (mec_set_probe): while on, this context's strided
        byte-wise launches run their arithmetic-free XOR twin (outputs are
        not codes)."""
        check(lib().mec_set_probe(self._h, 1 if on else 0))

    def stats(self):
        st = _lib.MecStats()
        check(lib().mec_get_stats(self._h, ctypes.byref(st)))
        return {"coalesced_batches": st.coalesced_batches, "coalesced_requests": st.coalesced_requests,
                "cached_plans": st.cached_plans, "zero_copy_calls": st.zero_copy_calls,
                "staged_calls": st.staged_calls, "queue_calls": st.queue_calls,
                "queue_launches": st.queue_launches, "queue_slots": st.queue_slots,
                "queue_parts": st.queue_parts, "queue_broken": bool(st.queue_broken), "queue_devslot": bool(st.queue_devslot),
                "queue_timeouts": st.queue_timeouts, "mg_cache_bytes": st.mg_cache_bytes,
                "mg_cache_tables": st.mg_cache_tables, "mg_cache_uncached": st.mg_cache_uncached,
                "jit_kernels": st.jit_kernels, "jit_failed": st.jit_failed, "jit_pending": st.jit_pending,
                "jit_compile_ms": st.jit_compile_ms, "jit_launches": st.jit_launches}


def fill_random(t, seed, word_offset=0, stream=None):
    """Fill a contiguous uint8 CUDA tensor with the splitmix64 stream."""
    if not t.is_cuda or not t.is_contiguous():
        raise ValueError("contiguous CUDA tensor required")
    check(lib().mec_fill_random(vp(t.data_ptr()), t.numel() * t.element_size(), seed, word_offset,
                                _stream(stream)))


def xor(dst, a, b, stream=None):
    n = dst.numel() * dst.element_size()
    check(lib().mec_xor(vp(dst.data_ptr()), vp(a.data_ptr()), vp(b.data_ptr()), n, _stream(stream)))


def host_register(arr):
    check(lib().mec_host_register(vp(arr.ctypes.data), arr.nbytes))


def host_unregister(arr):
    check(lib().mec_host_unregister(vp(arr.ctypes.data)))
