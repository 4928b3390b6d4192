// queue.hip — device-side submission queue for single-stripe host calls.
//
// MemEC's workers call Coding::encode / decode one stripe at a time from
// many threads at once (server.cc:107, worker.cc:128-137; SURVEY §8b:
// "a GPU implementation needs per-thread streams or a submission queue").
// A kernel launch per call costs ~5 us of HIP runtime on the calling
// thread, takes runtime locks shared by every caller, and completion is
// seen through hipStreamSynchronize.  This queue removes the runtime from
// the per-call path:
//   * a resident kernel runs `parts` workgroups per slot (one per 16 KiB of
//     chunk); part 0 polls its slot in GPU-mapped, coherent host memory
//     (relaxed system-scope loads, one acquire per job taken) and hands
//     each job to the other parts through device memory;
//   * a caller takes a free slot, writes the call's descriptor (device
//     addresses of registered chunks, GF(2^8) coefficients), publishes a new
//     sequence number, and spins on the slot's `done` words, which every
//     part stores (system-scope release, one L2 writeback) after its
//     outputs;
//   * each part builds the v_perm tables (gf8_kernel.hpp) from the raw
//     coefficients in LDS and codes its share of the chunk over PCIe, one
//     16-byte unit per lane.
// Exit conditions every wave reaches: the stop word (mec_set_host_queue(0),
// mec_destroy, a timed-out call) or a grid-wide idle exit.  The idle exit is
// decided for the whole grid at once: workgroup 0 (the leader) watches every
// slot's last-activity time and, when no slot has had work for
// MEC_QUEUE_IDLE_MS, sets the exit word that every workgroup polls.  So the
// grid always leaves together and the stream completes: a caller whose job
// is still pending then relaunches the kernel (queue_revive), which starts
// from each slot's `done`, so no job is lost or run twice.  (A per-workgroup
// idle timer would let one slot's workgroup leave while others keep the
// stream busy, stranding calls posted to that slot.)  Launches of the
// resident kernel go to one stream, so two instances never run at once.
//
// A call that sees no completion within MEC_QUEUE_TIMEOUT_MS (5 s) withdraws its job (its
// sequence number moves back), stops the queue for good and waits for the
// grid to leave; if its job never ran, the caller codes it on the launch
// path instead (queue_try returns false).
//
// Scope: chunks of at most MEC_QUEUE_MAX_CHUNK bytes (default 1 MiB: a
// slot runs one workgroup per 16 KiB of chunk, at most kQMaxParts, and
// measured faster than a launch from 4 KiB to 1 MiB for 1, 4 and 16
// callers, profiles/r03/host/queue_fence_ab.jsonl, queue_cut_ab.jsonl), either
// zero-copy (registered) or staged (mec.cpp lane_run), for every family:
// byte-wise GF(2^8) products (RS, ISA-L) and the Jerasure Cauchy bitmatrix
// over w packets of chunk/w bytes (cauchycoding.cc:80), whose masks the
// caller expands from the GF(2^w) coefficients.
#include <hip/hip_runtime.h>
#include <immintrin.h>

#include <chrono>
#include <cstddef>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <thread>

#include <time.h>

#include "ctx.hpp"
#include "kernels.hpp"
#include "stream_common.hpp"

namespace mec {
namespace core {
namespace {

using detail::u32x2;
using detail::u32x4;
constexpr int kQThreads = 1024;  // most threads per slot: a 16 KiB chunk in one pass
constexpr int kQBatch = 16;

__device__ __forceinline__ uint32_t tmul(const uint32_t *t, uint32_t x) {  // gf8_mul over LDS tables
    return __builtin_amdgcn_perm(t[1], t[0], x & 0x07070707u) ^ __builtin_amdgcn_perm(t[3], t[2], (x >> 3) & 0x07070707u) ^
           __builtin_amdgcn_perm(t[4], t[4], (x >> 6) & 0x03030303u);
}

// < 16 bytes, register-only (the tail of a chunk that is not a multiple of 16)
__device__ __forceinline__ u32x4 ld_part(const uint8_t *p, uint32_t n) {
    uint32_t w[4] = {0, 0, 0, 0};
#pragma unroll
    for (int i = 0; i < 16; ++i)
        if (uint32_t(i) < n) w[i / 4] |= uint32_t(p[i]) << (8 * (i % 4));
    return u32x4{w[0], w[1], w[2], w[3]};
}

__device__ __forceinline__ void st_part(uint8_t *p, const u32x4 &v, uint32_t n) {
    const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
    for (int i = 0; i < 16; ++i)
        if (uint32_t(i) < n) p[i] = uint8_t(w[i / 4] >> (8 * (i % 4)));
}

// One 16-byte unit (FULL) or the n-byte tail at byte offset off of every
// chunk: acc[r] (^)= sum_j coef[r][j] * src_j.  Source loads are issued in
// groups of kQBatch back to back, one PCIe round trip per group.
template <bool FULL>
__device__ __forceinline__ void code_unit(const uint64_t *addr, const uint32_t *tab, uint32_t ns, uint32_t nd,
                                          uint32_t acc_in, uint64_t off, uint32_t n, uint64_t *t_loaded = nullptr) {
    auto ld = [&](uint64_t p) {
        if constexpr (FULL) return *reinterpret_cast<const u32x4 *>(p);
        else return ld_part(reinterpret_cast<const uint8_t *>(p), n);
    };
    u32x4 acc[kQMaxDst];
#pragma unroll
    for (int r = 0; r < int(kQMaxDst); ++r) {
        const uint64_t d = addr[kQMaxSrc + r];
        acc[r] = (acc_in && uint32_t(r) < nd && d) ? ld(d + off) : u32x4{0, 0, 0, 0};
    }
    for (uint32_t j0 = 0; j0 < ns; j0 += kQBatch) {
        u32x4 x[kQBatch];
#pragma unroll
        for (int jj = 0; jj < kQBatch; ++jj) {
            const uint64_t a = j0 + jj < ns ? addr[j0 + jj] : 0;  // 0: Coding::zeros / past ns
            x[jj] = a ? ld(a + off) : u32x4{0, 0, 0, 0};
        }
        if (t_loaded && j0 == 0) {  // traced jobs, thread 0 only: when its first loads returned
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            *t_loaded = __builtin_amdgcn_s_memrealtime();
        }
#pragma unroll
        for (int jj = 0; jj < kQBatch; ++jj) {
#pragma unroll
            for (int r = 0; r < int(kQMaxDst); ++r) {
                if (j0 + jj < ns && uint32_t(r) < nd) {
                    const uint32_t *T = tab + (r * ns + j0 + jj) * 5;
                    acc[r] ^= u32x4{tmul(T, x[jj].x), tmul(T, x[jj].y), tmul(T, x[jj].z), tmul(T, x[jj].w)};
                }
            }
        }
    }
#pragma unroll
    for (int r = 0; r < int(kQMaxDst); ++r) {
        const uint64_t d = addr[kQMaxSrc + r];
        if (uint32_t(r) >= nd || !d) continue;
        if constexpr (FULL) *reinterpret_cast<u32x4 *>(d + off) = acc[r];
        else st_part(reinterpret_cast<uint8_t *>(d + off), acc[r], n);
    }
}

// ---- bitmatrix (Jerasure Cauchy-RS) jobs --------------------------------
// acc ^= d & m as one v_bitop3_b32 (truth table 0x6A), as bm_kernel.hpp.
__device__ __forceinline__ u32x2 bm_axor(u32x2 d, uint32_t m, u32x2 acc) {
    return u32x2{uint32_t(__builtin_amdgcn_bitop3_b32(d.x, m, acc.x, 0x6A)),
                 uint32_t(__builtin_amdgcn_bitop3_b32(d.y, m, acc.y, 0x6A))};
}

__device__ __forceinline__ u32x2 ld8(uint64_t p, uint32_t n) {
    if (n == 8) return *reinterpret_cast<const u32x2 *>(p);
    const uint8_t *b = reinterpret_cast<const uint8_t *>(p);
    uint32_t w[2] = {0, 0};
#pragma unroll
    for (int i = 0; i < 8; ++i)
        if (uint32_t(i) < n) w[i / 4] |= uint32_t(b[i]) << (8 * (i % 4));
    return u32x2{w[0], w[1]};
}

__device__ __forceinline__ void st8(uint64_t p, u32x2 v, uint32_t n) {
    if (n == 8) {
        *reinterpret_cast<u32x2 *>(p) = v;
        return;
    }
    uint8_t *b = reinterpret_cast<uint8_t *>(p);
    const uint32_t w[2] = {v.x, v.y};
#pragma unroll
    for (int i = 0; i < 8; ++i)
        if (uint32_t(i) < n) b[i] = uint8_t(w[i / 4] >> (8 * (i % 4)));
}

// The n-byte slice (n <= 8) at offset off of every packet: output packet
// (r, l) (^)= XOR over (j, x) with bit x of mk[j][r*W + l] of source packet
// (j, x) (jerasure_do_scheduled_operations' result, jerasure.c:1162-1185).
// Sources are loaded B at a time (B*W slices in flight, one PCIe round trip).
template <int W>
__device__ __forceinline__ void bm_unit(const uint64_t *addr, const uint8_t *mk, uint32_t ns, uint32_t nd,
                                        uint32_t acc_in, uint64_t off, uint32_t n, uint64_t P) {
    constexpr int B = W >= 16 ? 1 : 16 / W;
    u32x2 acc[kQMaxDst * W];
#pragma unroll
    for (int r = 0; r < int(kQMaxDst); ++r) {
        const uint64_t d = addr[kQMaxSrc + r];
#pragma unroll
        for (int l = 0; l < W; ++l)
            acc[r * W + l] = (acc_in && uint32_t(r) < nd && d) ? ld8(d + l * P + off, n) : u32x2{0, 0};
    }
    for (uint32_t j0 = 0; j0 < ns; j0 += B) {
        u32x2 x[B][W];
#pragma unroll
        for (int jj = 0; jj < B; ++jj) {
            const uint64_t a = j0 + jj < ns ? addr[j0 + jj] : 0;  // 0: Coding::zeros / past ns
#pragma unroll
            for (int xw = 0; xw < W; ++xw) x[jj][xw] = a ? ld8(a + xw * P + off, n) : u32x2{0, 0};
        }
#pragma unroll
        for (int jj = 0; jj < B; ++jj) {
            if (j0 + jj >= ns) break;
            const uint8_t *mb = mk + (j0 + jj) * kQBmRows;
#pragma unroll
            for (int r = 0; r < int(kQMaxDst); ++r) {
                if (uint32_t(r) >= nd) break;
#pragma unroll
                for (int l = 0; l < W; ++l) {
                    const uint32_t bits = mb[r * W + l];
#pragma unroll
                    for (int xw = 0; xw < W; ++xw)
                        acc[r * W + l] = bm_axor(x[jj][xw], 0u - ((bits >> xw) & 1u), acc[r * W + l]);
                }
            }
        }
    }
#pragma unroll
    for (int r = 0; r < int(kQMaxDst); ++r) {
        const uint64_t d = addr[kQMaxSrc + r];
        if (uint32_t(r) >= nd || !d) continue;
#pragma unroll
        for (int l = 0; l < W; ++l) st8(d + l * P + off, acc[r * W + l], n);
    }
}

template <int W>
__device__ __forceinline__ void bm_job(const uint64_t *addr, const uint8_t *mk, uint32_t ns, uint32_t nd,
                                       uint32_t acc_in, uint32_t P, uint32_t t, uint32_t nthr) {
    const uint32_t units = (P + 7) / 8;
    for (uint32_t u = t; u < units; u += nthr) {
        const uint32_t off = u * 8;
        bm_unit<W>(addr, mk, ns, nd, acc_in, off, P - off < 8 ? P - off : 8, P);
    }
}

template <typename T>
__device__ __forceinline__ T sys_load(const T *p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

__device__ __forceinline__ void mark_active(uint64_t *act) {
    __hip_atomic_store(act, __builtin_amdgcn_s_memrealtime(), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// descriptor words read per job: hdr, src, dst, then the tables (byte-wise)
// or the masks (bitmatrix); a job's own share is a prefix of that payload,
// but the whole of it is read in the same round trip as the rest
constexpr uint32_t kQHeadWords = 8 + 2 * (kQMaxSrc + kQMaxDst);
constexpr uint32_t kQDescWords = kQHeadWords + kQMaxDst * kQMaxSrc * 5;  // the tables outsize the masks
static_assert(kQMaxDst * kQMaxSrc * 5 >= kQMaxSrc * kQBmRows / 4, "descriptor LDS holds the masks");
static_assert(kQHeadWords % 4 == 0, "16-byte descriptor loads");
static_assert(offsetof(QDesc, tab_w) == kQHeadWords * 4, "descriptor head layout");
static_assert(offsetof(QSlot, d) % 16 == 0 && offsetof(QDevSlot, d) % 16 == 0, "16-byte descriptor loads");
static_assert(sizeof(QDevSlot) % 64 == 0, "device slots on their own cache lines");
// dwords of a job's descriptor: the head, then its tables / masks
__host__ __device__ __forceinline__ uint32_t desc_words(uint32_t ns, uint32_t nd, bool bitmatrix) {
    return kQHeadWords + (bitmatrix ? ns * (kQBmRows / 4) : nd * ns * 5);
}

// Workgroup b serves slot b / parts as part b % parts: part 0 polls the
// slot in host memory and, when it takes a job, publishes its number in
// device memory (`go`), where the slot's other parts poll; every part codes
// its share of the units (16-byte units part, part + parts, ... of each
// nthr-thread pass) and stores its own done word.  Part 0 alone watches the
// control words; when it leaves it records the launch epoch in `left`, and
// the other parts leave only after that, having run every job part 0 took
// — so a job is run by all of a slot's parts or by none (a withdrawn job
// is never taken, queue_try).
// The slot's sequence word and descriptor are at seq_base / desc_base +
// slot * dstride: inside the host-memory QSlot, or in device memory
// (QDevSlot) that the host writes through the BAR.
__global__ __launch_bounds__(kQThreads) void queue_kernel(QSlot *slots, const uint8_t *seq_base, const uint8_t *desc_base,
                                                         uint32_t dstride, uint32_t *ctl, uint64_t *act, uint64_t *link,
                                                         uint64_t epoch, uint64_t idle_ticks, uint32_t nthr,
                                                         uint32_t nslots, uint32_t parts, uint32_t bitmatrix) {
    __shared__ u32x4 desc4[kQDescWords / 4];  // the slot's descriptor: hdr, src, dst, tab_w | mask_w
    __shared__ uint32_t cmd, shape;
    uint32_t *desc = reinterpret_cast<uint32_t *>(desc4);
    const uint32_t si = blockIdx.x / parts, part = blockIdx.x - si * parts;
    QSlot *s = slots + si;
    const uint64_t *seqp = reinterpret_cast<const uint64_t *>(seq_base + size_t(si) * dstride);
    const u32x4 *sw = reinterpret_cast<const u32x4 *>(desc_base + size_t(si) * dstride);
    uint64_t *go = link + si, *left = link + nslots + si;
    const uint32_t t = threadIdx.x;
    const bool leader = blockIdx.x == 0;
    uint64_t last = 0, t0 = 0, t_take = 0, t_fence = 0, t_loaded = 0;
    if (t == 0) {
        last = sys_load(&s->done[part]);
        t0 = __builtin_amdgcn_s_memrealtime();
    }
    const uint32_t *hdr = desc;
    const uint64_t *addr = reinterpret_cast<const uint64_t *>(desc + 8);
    const uint32_t *tab = desc + kQHeadWords;
    const uint8_t *mk = reinterpret_cast<const uint8_t *>(desc + kQHeadWords);
    for (;;) {
        if (t == 0 && part != 0) {  // the other parts: part 0's jobs, from device memory
            uint32_t c = 0;
            // relaxed polls, one acquire fence per job taken (an acquire
            // load per poll invalidated caches at every poll); system scope,
            // as part 0's: this part reads the caller's chunks through its
            // own XCD's L2, which must not serve lines of an earlier job
            for (;;) {
                const uint64_t lf = __hip_atomic_load(left, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                const uint64_t q = __hip_atomic_load(go, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                if ((q >> 16) > last) {  // go = part 0's seq word (job number, shape)
                    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
                    last = q >> 16;
                    shape = uint32_t(q & 0xffffu);
                    c = 1;
                    break;
                }
                if (lf == epoch) {
                    // part 0 has left: `left` was stored (release) after its
                    // last `go`, so acquire and read `go` once more — the two
                    // relaxed loads above are not ordered, and a stale `go`
                    // seen with the new `left` would skip part 0's last job
                    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
                    const uint64_t q2 = __hip_atomic_load(go, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    if ((q2 >> 16) > last) {
                        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
                        last = q2 >> 16;
                        shape = uint32_t(q2 & 0xffffu);
                        c = 1;
                    }
                    break;
                }
                __builtin_amdgcn_s_sleep(2);
            }
            cmd = c;
        } else if (t == 0) {
            uint32_t c = 0;
            for (uint32_t n = 1;; ++n) {  // one PCIe read per poll; control words every 64th
                const uint64_t q = __hip_atomic_load(seqp, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
                if ((q >> 16) > last) {  // a withdrawn job moves seq back (queue_try)
                    t_take = __builtin_amdgcn_s_memrealtime();
                    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");  // system scope, once per job
                    t_fence = __builtin_amdgcn_s_memrealtime();
                    last = q >> 16;
                    shape = uint32_t(q & 0xffffu);
                    c = 1;
                    if (parts > 1) __hip_atomic_store(go, q, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
                    break;
                }
                if (n % 64 == 0) {
                    if ((sys_load(ctl + kQCtlStop) | sys_load(ctl + kQCtlExit)) != 0u) break;
                    if (leader) {  // grid-wide idle: no slot has worked for idle_ticks
                        uint64_t newest = t0;
                        for (uint32_t i = 0; i < nslots; ++i) {
                            const uint64_t a = __hip_atomic_load(act + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                            newest = a > newest ? a : newest;
                        }
                        if (__builtin_amdgcn_s_memrealtime() - newest > idle_ticks) {
                            __hip_atomic_store(ctl + kQCtlExit, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
                            break;
                        }
                    }
                }
                __builtin_amdgcn_s_sleep(4);
            }
            cmd = c;
            if (c) mark_active(act + si);
            else if (parts > 1) __hip_atomic_store(left, epoch, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
        }
        __syncthreads();
        if (cmd == 0) return;  // uniform: stop or grid idle
        {  // descriptor: the head, then this job's tables or masks only (its
           // size came with the seq word), 16 bytes per lane, one round trip
            const uint32_t n4 = (desc_words(shape >> 8, shape & 0xffu, bitmatrix != 0) + 3) / 4;
            for (uint32_t i = t; i < n4; i += nthr) desc4[i] = __builtin_nontemporal_load(sw + i);
        }
        __syncthreads();
        const uint32_t ns = hdr[0], nd = hdr[1], bytes = hdr[2], acc_in = hdr[3], w = hdr[4], P = hdr[5];
        MEC_DASSERT(ns <= kQMaxSrc && nd <= kQMaxDst && ns == (shape >> 8) && nd == (shape & 0xffu) && w <= 8);
        const bool traced = hdr[6] != 0u && part == 0 && t == 0;
        const uint64_t t_desc = traced ? __builtin_amdgcn_s_memrealtime() : 0;
        if (w == 0) {  // byte-wise GF(2^8): the host's v_perm tables, read in place from LDS
            // this part's units: passes of nthr units, part-th of every parts
            const uint32_t full = bytes / 16, me = part * nthr + t, step = parts * nthr;
            for (uint32_t u = me; u < full; u += step)
                code_unit<true>(addr, tab, ns, nd, acc_in, uint64_t(u) * 16, 16, traced && u == me ? &t_loaded : nullptr);
            if (bytes % 16 && me == full % step)  // the partial last unit
                code_unit<false>(addr, tab, ns, nd, acc_in, uint64_t(full) * 16, bytes % 16);
        } else {
            const uint32_t me = part * nthr + t, step = parts * nthr;
            switch (w) {  // uniform
                case 1: bm_job<1>(addr, mk, ns, nd, acc_in, P, me, step); break;
                case 2: bm_job<2>(addr, mk, ns, nd, acc_in, P, me, step); break;
                case 3: bm_job<3>(addr, mk, ns, nd, acc_in, P, me, step); break;
                case 4: bm_job<4>(addr, mk, ns, nd, acc_in, P, me, step); break;
                case 5: bm_job<5>(addr, mk, ns, nd, acc_in, P, me, step); break;
                case 6: bm_job<6>(addr, mk, ns, nd, acc_in, P, me, step); break;
                case 7: bm_job<7>(addr, mk, ns, nd, acc_in, P, me, step); break;
                case 8: bm_job<8>(addr, mk, ns, nd, acc_in, P, me, step); break;
                default: break;
            }
        }
        // Completion: every wave waits until its own output stores are
        // acknowledged, the barrier orders that before thread 0, and thread
        // 0's system-scope release store of `done` writes the L2 back once
        // for the whole workgroup.  (A __threadfence_system per lane cost
        // every wave an L2 writeback + invalidate per job, which made a
        // 64 KiB call 2.4x slower on the queue than as a launch even with the
        // launch's own geometry; profiles/r03/host/queue_pthr_ab.log.)
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        if (traced) {  // measurement only (mec_queue_trace_enable): vector stores before the release
            const uint64_t t_end = __builtin_amdgcn_s_memrealtime();
            __hip_atomic_store(&s->trace[0], t_take, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            __hip_atomic_store(&s->trace[1], t_fence, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            __hip_atomic_store(&s->trace[2], t_desc, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            __hip_atomic_store(&s->trace[3], t_loaded, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            __hip_atomic_store(&s->trace[4], t_end, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        }
        if (t == 0) {
            __hip_atomic_store(&s->done[part], last, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
            if (part == 0) mark_active(act + si);
        }
    }
}

// Gf8Coef of every GF(2^8) value, built once (gf8_coef: 20 field products)
const Gf8Coef *gf8_coef_table() {
    static const std::vector<Gf8Coef> t = [] {
        std::vector<Gf8Coef> v(256);
        for (int c = 0; c < 256; ++c) v[size_t(c)] = gf8_coef(uint8_t(c));
        return v;
    }();
    return t.data();
}

uint64_t mono_ns() {  // CLOCK_MONOTONIC, the clock mec_queue_trace reports in
    timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return uint64_t(ts.tv_sec) * 1000000000ull + uint64_t(ts.tv_nsec);
}

// The calling thread's last traced queue call (mec_queue_last_trace).
struct QTrace {
    uint64_t host_post_ns, host_seen_ns, dev_take, dev_fence, dev_desc, dev_loaded, dev_end;
    uint32_t parts, valid;
};
QTrace &last_trace() {
    static thread_local QTrace t{};
    return t;
}

uint64_t env_u64(const char *name, uint64_t dflt) {
    const char *e = std::getenv(name);
    return e && *e ? std::strtoull(e, nullptr, 10) : dflt;
}

// Launch the resident kernel (caller holds q->mu; no instance is running).
int queue_launch(mec_ctx *c, HostQueue *q) {
    DeviceGuard dg(c->device);
    __atomic_store_n(q->ctl_host + kQCtlExit, 0u, __ATOMIC_RELEASE);
    ++q->epoch;
    const uint8_t *seq_base = q->dslot ? reinterpret_cast<const uint8_t *>(&q->dslot->seq)
                                       : reinterpret_cast<const uint8_t *>(&q->dev->seq);
    const uint8_t *desc_base = q->dslot ? reinterpret_cast<const uint8_t *>(&q->dslot->d)
                                        : reinterpret_cast<const uint8_t *>(&q->dev->d);
    const uint32_t dstride = q->dslot ? uint32_t(sizeof(QDevSlot)) : uint32_t(sizeof(QSlot));
    hipLaunchKernelGGL(queue_kernel, dim3(q->slots * q->parts), dim3(q->threads), 0, q->stream, q->dev, seq_base,
                       desc_base, dstride, q->ctl_dev,
                       q->act, q->link, q->epoch, q->idle_ticks, q->threads, q->slots, q->parts,
                       c->byte_wise() ? 0u : 1u);
    HIP_TRY(hipGetLastError());
    q->launches++;
    return MEC_OK;
}

// The resident grid has exited (idle) while jobs may be pending: relaunch.
// While it is still leaving (the exit word reaches every workgroup within
// one poll interval) the stream is busy and the caller retries.
int queue_revive(mec_ctx *c, HostQueue *q) {
    std::lock_guard<std::mutex> g(q->mu);
    if (q->broken.load()) return fail(MEC_EHIP, "host queue stopped after a timed-out call");
    const hipError_t e = hipStreamQuery(q->stream);
    if (e == hipErrorNotReady) return MEC_OK;  // still running
    if (e != hipSuccess) return hip_fail(e, "queue kernel");
    return queue_launch(c, q);
}

// Wait up to `ms` for the resident grid to leave.
enum class Drain { kLeft, kFailed, kRunning };
Drain queue_drained(HostQueue *q, int ms) {
    const auto t0 = std::chrono::steady_clock::now();
    for (;;) {
        const hipError_t e = hipStreamQuery(q->stream);
        if (e == hipSuccess) return Drain::kLeft;
        if (e != hipErrorNotReady) return Drain::kFailed;  // the grid faulted: its outputs are unknown
        if (std::chrono::steady_clock::now() - t0 >= std::chrono::milliseconds(ms)) return Drain::kRunning;
        std::this_thread::sleep_for(std::chrono::microseconds(200));
    }
}

}  // namespace

bool queue_stop(mec_ctx *c) {
    HostQueue *q = c->hq;
    if (!q) return true;
    c->hq = nullptr;
    {
        DeviceGuard dg(c->device);
        __atomic_store_n(q->ctl_host + kQCtlStop, 1u, __ATOMIC_RELEASE);
        // every workgroup sees the stop word within one poll interval; a grid
        // still running after the cap (a hung job) keeps its memory: freeing
        // slots and control words under a running kernel would fault it
        if (queue_drained(q, int(std::max<uint64_t>(q->timeout_ms, 1000))) == Drain::kRunning) {
            fprintf(stderr, "libmec: host queue kernel still running at mec_destroy; its memory is leaked\n");
            return false;
        }
        (void)hipStreamDestroy(q->stream);
        (void)hipHostFree(q->host);
        (void)hipFree(q->act);
        (void)hipFree(q->link);
        if (q->dslot) (void)hipFree(q->dslot);
        if (q->push) (void)hipFree(q->push);
    }
    delete[] q->hs;
    delete q;
    return true;
}

int queue_start(mec_ctx *c, uint32_t slots) {
    if (slots > kQMaxSlots) return fail(MEC_EINVAL, "at most %u queue slots", kQMaxSlots);
    DeviceGuard dg(c->device);
    std::unique_ptr<HostQueue> q(new HostQueue);
    q->max_chunk = uint32_t(env_u64("MEC_QUEUE_MAX_CHUNK", 1 << 20));
    // a lone call on a chunk above this codes faster as a launch (many
    // workgroups over PCIe) than on one queue workgroup
    q->solo_max = uint32_t(env_u64("MEC_QUEUE_SOLO_MAX", q->max_chunk));
    q->idle_ticks = env_u64("MEC_QUEUE_IDLE_MS", 50) * 100000ull;  // s_memrealtime: 100 MHz
    q->timeout_ms = env_u64("MEC_QUEUE_TIMEOUT_MS", 5000);
    // workgroups per slot: one per 16 KiB of chunk (a kQThreads pass of
    // 16-byte units), and below 64 KiB one per 8 KiB up to 4 — a lone
    // caller's sources then stream over PCIe through more CUs: one caller's
    // RS(8,2)@16 KiB calls 68 -> 82 K/s with 2 parts (96 K with 4, but 16
    // callers lose 5 % there), while 64 KiB is fastest at 4 parts for one
    // and for 16 callers (profiles/r04/host/queue_parts_ab.jsonl,
    // queue_parts_rule_ab.jsonl: 16 KiB 68 -> 84 K/s, 16 callers equal); at most
    // kQMaxParts.  MEC_QUEUE_PART_THREADS=<n> sets one part per n units,
    // MEC_QUEUE_PARTS the count directly (A/Bs)
    const uint32_t units = (c->cs + 15) / 16;
    uint32_t auto_parts = std::max((units + kQThreads - 1) / kQThreads, std::min(4u, (units + 511) / 512));
    if (std::getenv("MEC_QUEUE_PART_THREADS")) {
        const uint32_t pthr = uint32_t(std::min<uint64_t>(kQThreads, std::max<uint64_t>(64, env_u64("MEC_QUEUE_PART_THREADS", kQThreads))));
        auto_parts = (units + pthr - 1) / pthr;
    }
    auto_parts = std::min<uint32_t>(kQMaxParts, std::max<uint32_t>(1, auto_parts));
    q->parts = std::min<uint32_t>(kQMaxParts, std::max<uint64_t>(1, env_u64("MEC_QUEUE_PARTS", auto_parts)));
    // one 16-byte unit per thread up to kQThreads (a 4 KiB chunk: 256 threads;
    // idle threads only cost barrier time), at least 128 (descriptor loads)
    const uint32_t per_part = (units + q->parts - 1) / q->parts;
    q->threads = std::min<uint32_t>(kQThreads, std::max<uint32_t>(q->parts > 1 ? 64 : 128, (per_part + 63) / 64 * 64));
    // every workgroup of every slot must be resident at once (a slot whose
    // workgroup waits for another to exit would never be served), and the
    // resident grid holds at most half of what the device can hold, so
    // launches beside it (calls beyond the slots, batches) keep CUs to run on
    {
        int per_cu = 0, cus = 0;
        HIP_TRY(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, queue_kernel, int(q->threads), 0));
        HIP_TRY(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, c->device));
        const uint32_t cap = uint32_t(std::max(1, per_cu * cus / 2)) / q->parts;
        slots = std::max<uint32_t>(1, std::min(slots, cap));
    }
    q->slots = slots;
    const size_t bytes = sizeof(QSlot) * slots + 256;
    void *h = nullptr;
    HIP_TRY(hipHostMalloc(&h, bytes, hipHostMallocMapped | hipHostMallocCoherent | hipHostMallocPortable));
    std::memset(h, 0, bytes);
    void *d = nullptr;
    hipError_t e = hipHostGetDevicePointer(&d, h, 0);
    if (e == hipSuccess) e = hipMalloc(reinterpret_cast<void **>(&q->act), sizeof(uint64_t) * slots);
    if (e == hipSuccess) e = hipMalloc(reinterpret_cast<void **>(&q->link), sizeof(uint64_t) * 2 * slots);
    if (e != hipSuccess) {
        (void)hipHostFree(h);
        if (q->act) (void)hipFree(q->act);
        if (q->link) (void)hipFree(q->link);
        return hip_fail(e, "queue memory");
    }
    q->host = static_cast<QSlot *>(h);
    q->dev = static_cast<QSlot *>(d);
    q->hs = new HostQueue::HostSlotState[slots];
    // device-memory slot halves when the host can store to device memory
    // (large BAR): uncached, so part 0's polls and descriptor reads never
    // meet a stale L2 line; MEC_QUEUE_DEVSLOT=0 keeps them in host memory
    {
        int large_bar = 0;
        if (hipDeviceGetAttribute(&large_bar, hipDeviceAttributeIsLargeBar, c->device) != hipSuccess) large_bar = 0;
        if (large_bar && env_u64("MEC_QUEUE_DEVSLOT", 1) != 0) {
            void *ds = nullptr;
            if (hipExtMallocWithFlags(&ds, sizeof(QDevSlot) * slots, hipDeviceMallocUncached) == hipSuccess) {
                // zeroed through the BAR like every later write (no device-wide
                // synchronize that would wait for the caller's own launches);
                // the kernel launch below is a later PCIe write, so it lands after
                const __m128i z = _mm_setzero_si128();
                __m128i *w = static_cast<__m128i *>(ds);
                for (size_t k = 0; k < sizeof(QDevSlot) * slots / 16; ++k) _mm_stream_si128(w + k, z);
                _mm_sfence();
                q->dslot = static_cast<QDevSlot *>(ds);
            }
            (void)hipGetLastError();  // a refused allocation leaves host-memory slots
        }
    }
    // source push area (MEC_QUEUE_PUSH, device-memory slots only): kQMaxSrc
    // chunks per slot
    q->push_max = uint32_t(env_u64("MEC_QUEUE_PUSH", 0));
    if (q->dslot && q->push_max && c->cs <= q->push_max) {
        q->push_chunk = (size_t(c->cs) + 63) & ~size_t(63);
        void *pa = nullptr;
        if (hipExtMallocWithFlags(&pa, size_t(slots) * kQMaxSrc * q->push_chunk, hipDeviceMallocUncached) == hipSuccess)
            q->push = static_cast<uint8_t *>(pa);
        (void)hipGetLastError();  // refused: sources stay in host memory
    }
    q->ctl_host = reinterpret_cast<uint32_t *>(static_cast<uint8_t *>(h) + sizeof(QSlot) * slots);
    q->ctl_dev = reinterpret_cast<uint32_t *>(static_cast<uint8_t *>(d) + sizeof(QSlot) * slots);
    e = hipStreamCreateWithFlags(&q->stream, hipStreamNonBlocking);
    // the zeroed per-slot words must be in place before the kernel reads
    // them: a hipMemset need not have finished when work on a non-blocking
    // stream starts, and a reused allocation still holds an earlier queue's
    // `go` numbers (which made a part skip a job)
    if (e == hipSuccess) e = hipMemsetAsync(q->act, 0, sizeof(uint64_t) * slots, q->stream);
    if (e == hipSuccess) e = hipMemsetAsync(q->link, 0, sizeof(uint64_t) * 2 * slots, q->stream);
    if (e == hipSuccess) e = hipStreamSynchronize(q->stream);
    if (e != hipSuccess) {
        if (q->stream) (void)hipStreamDestroy(q->stream);
        (void)hipHostFree(h);
        (void)hipFree(q->act);
        (void)hipFree(q->link);
        if (q->dslot) (void)hipFree(q->dslot);
        if (q->push) (void)hipFree(q->push);
        delete[] q->hs;
        return hip_fail(e, "queue stream");
    }
    {
        std::lock_guard<std::mutex> g(q->mu);
        int rc = queue_launch(c, q.get());
        if (rc != MEC_OK) {
            (void)hipStreamDestroy(q->stream);
            (void)hipHostFree(h);
            (void)hipFree(q->act);
            (void)hipFree(q->link);
            if (q->dslot) (void)hipFree(q->dslot);
            if (q->push) (void)hipFree(q->push);
            delete[] q->hs;
            return rc;
        }
    }
    c->hq = q.release();
    return MEC_OK;
}

// The job's sources streamed through the BAR into the slot's device area
// (16-byte streaming stores; the caller's chunk data may be only 8-byte
// aligned, ChunkPool slots), descriptor entries pointed at them.  A later
// store fence and the sequence word follow, so the GPU that sees the word
// sees the bytes (PCIe keeps posted writes in order).
void push_sources(HostQueue *q, uint32_t slot, QDesc &d, size_t ns, const uint8_t *const *hsrc, uint32_t cs) {
    uint8_t *area = q->push + size_t(slot) * kQMaxSrc * q->push_chunk;
    for (size_t j = 0; j < ns; ++j) {
        if (!d.src[j] || !hsrc[j]) continue;
        __m128i *to = reinterpret_cast<__m128i *>(area + j * q->push_chunk);
        const uint8_t *from = hsrc[j];
        const uint32_t full = cs / 16;
        for (uint32_t u = 0; u < full; ++u)
            _mm_stream_si128(to + u, _mm_loadu_si128(reinterpret_cast<const __m128i *>(from + size_t(u) * 16)));
        if (cs % 16) {
            alignas(16) uint8_t tail[16] = {};
            std::memcpy(tail, from + size_t(full) * 16, cs % 16);
            _mm_stream_si128(to + full, _mm_load_si128(reinterpret_cast<const __m128i *>(tail)));
        }
        d.src[j] = uint64_t(uintptr_t(area + j * q->push_chunk));
    }
}

bool queue_try(mec_ctx *c, const uint64_t *addrs, size_t ns, size_t nd, const Mat &coef, bool accumulate, int &rc,
               const uint8_t *const *hsrc) {
    HostQueue *q = c->hq;
    if (!q || q->broken.load(std::memory_order_relaxed) || c->cs > q->max_chunk || ns > kQMaxSrc ||
        nd > kQMaxDst || nd == 0 || (!c->byte_wise() && (c->w < 1 || c->w > 8)))
        return false;
    // the in-flight count only matters to chunks above solo_max (no RMW on a
    // shared line per call otherwise)
    const bool track = c->cs > q->solo_max;
    if (track && q->inflight.load(std::memory_order_relaxed) == 0) return false;
    // a free slot, starting from a per-thread hint so callers spread out
    static thread_local uint32_t hint = uint32_t(std::hash<std::thread::id>()(std::this_thread::get_id()));
    uint32_t i = 0;
    bool got = false;
    for (uint32_t n = 0; n < q->slots && !got; ++n) {
        i = (hint + n) % q->slots;
        bool f = false;
        got = !q->hs[i].busy.load(std::memory_order_relaxed) && q->hs[i].busy.compare_exchange_strong(f, true);
    }
    if (!got) return false;  // every slot busy: the launch path takes this call
    hint = i;
    if (track) q->inflight.fetch_add(1, std::memory_order_relaxed);
    QSlot *s = q->host + i;
    QDesc &d = s->d;  // built in host memory (the device copy follows, below)
    d.hdr[0] = uint32_t(ns);
    d.hdr[1] = uint32_t(nd);
    d.hdr[2] = c->cs;
    d.hdr[3] = accumulate ? 1u : 0u;
    d.hdr[4] = c->byte_wise() ? 0u : c->w;
    d.hdr[5] = c->byte_wise() ? c->cs : c->packet;
    const bool traced = q->trace.load(std::memory_order_relaxed);
    d.hdr[6] = traced ? 1u : 0u;
    for (size_t j = 0; j < ns; ++j) d.src[j] = addrs[j];
    for (size_t r = 0; r < nd; ++r) d.dst[r] = addrs[ns + r];
    if (c->byte_wise()) {  // the v_perm tables, [output][source] (a table per GF(2^8) value)
        for (size_t b = 0; b < nd * ns; ++b) std::memcpy(&d.tab_w[b * 5], &gf8_coef_table()[coef[b]], sizeof(Gf8Coef));
    } else {  // GF(2^w) coefficients -> bitmatrix rows (jerasure_matrix_to_bitmatrix)
        const Field &f = Field::get(int(c->w));
        uint8_t mk[kQMaxSrc][kQBmRows] = {};
        for (size_t r = 0; r < nd; ++r)
            for (size_t j = 0; j < ns; ++j) bit_block(f, coef[r * ns + j], c->w, &mk[j][r * c->w], 1);
        std::memcpy(d.mask_w, mk, sizeof(mk));
    }
    if (q->push && hsrc && c->cs <= q->push_max) push_sources(q, i, d, ns, hsrc, c->cs);
    const uint64_t seq = q->hs[i].seqno + 1;
    q->hs[i].seqno = seq;
    const uint64_t t_post = traced ? mono_ns() : 0;
    // publishes the descriptor; the word carries its shape (sources, outputs)
    const uint64_t word = seq << 16 | uint64_t(ns) << 8 | uint64_t(nd);
    if (q->dslot) {
        // through the BAR: the job's prefix of the descriptor in 16-byte
        // streaming stores, a store fence (the BAR mapping may combine and
        // reorder them), then the sequence word and another fence so it
        // leaves the write-combining buffer now; PCIe keeps posted writes in
        // order, so the GPU that sees the word sees the descriptor
        QDevSlot *ds = q->dslot + i;
        const uint32_t n16 = (desc_words(uint32_t(ns), uint32_t(nd), !c->byte_wise()) + 3) / 4;
        const __m128i *from = reinterpret_cast<const __m128i *>(&d);
        __m128i *to = reinterpret_cast<__m128i *>(&ds->d);
        for (uint32_t k = 0; k < n16; ++k) _mm_stream_si128(to + k, _mm_load_si128(from + k));
        _mm_sfence();
        _mm_stream_si64(reinterpret_cast<long long *>(&ds->seq), static_cast<long long>(word));
        _mm_sfence();
    } else {
        __atomic_store_n(&s->seq, word, __ATOMIC_RELEASE);
    }
    // wait for the workgroup; relaunch the grid if it idled out meanwhile
    rc = MEC_OK;
    bool taken = true;
    const auto t0 = std::chrono::steady_clock::now();
    uint32_t spins = 0;
    auto finished = [&] {  // every part of the slot has stored this job's number
        for (uint32_t p = 0; p < q->parts; ++p)
            if (__atomic_load_n(&s->done[p], __ATOMIC_ACQUIRE) != seq) return false;
        return true;
    };
    while (!finished()) {
        if (++spins % 2048 == 0 || q->timeout_ms == 0) {
            const auto dt = std::chrono::steady_clock::now() - t0;
            if (dt > std::chrono::milliseconds(q->timeout_ms) || q->broken.load()) {
                // Withdraw the job (seq moves back: a part 0 that has not
                // taken it never will; once taken, every part runs the
                // unchanged descriptor to the end), stop the queue for good,
                // and wait for the whole grid to leave, at most
                // kQDrainFactor x the call timeout.  Then: every part's done
                // word == seq -> the job ran, MEC_OK; none -> nothing touched
                // the chunks and the launch path codes them (taken = false);
                // some, a faulted grid, or a grid still running at the cap ->
                // MEC_EHIP with the slot left busy (its outputs are partial or
                // may still be written; an accumulate job must not be run
                // again on top of the parts that applied it).
                if (dt > std::chrono::milliseconds(q->timeout_ms)) q->timeouts++;
                q->hs[i].seqno = seq - 1;
                if (q->dslot) {
                    _mm_stream_si64(reinterpret_cast<long long *>(&q->dslot[i].seq), static_cast<long long>((seq - 1) << 16));
                    _mm_sfence();
                } else {
                    __atomic_store_n(&s->seq, (seq - 1) << 16, __ATOMIC_SEQ_CST);
                }
                q->broken.store(true);
                __atomic_store_n(q->ctl_host + kQCtlStop, 1u, __ATOMIC_RELEASE);
                const Drain dr = queue_drained(
                    q, int(std::min<uint64_t>(std::max<uint64_t>(kQDrainFactor * q->timeout_ms, 10000), 600000)));
                uint32_t ran = 0;
                for (uint32_t p = 0; p < q->parts; ++p) ran += __atomic_load_n(&s->done[p], __ATOMIC_ACQUIRE) == seq;
                if (dr == Drain::kLeft && ran == q->parts) {
                    rc = MEC_OK;
                } else if (dr == Drain::kLeft && ran == 0) {
                    rc = MEC_OK;
                    taken = false;  // never ran: the launch path takes the call
                } else {
                    rc = fail(MEC_EHIP, "host queue call timed out after %llu ms and the resident kernel %s "
                                        "(%u of %u parts finished); the outputs are undefined",
                              (unsigned long long)q->timeout_ms,
                              dr == Drain::kFailed ? "faulted" : dr == Drain::kRunning ? "did not leave" : "left",
                              ran, q->parts);
                }
                break;
            }
            if (dt > std::chrono::microseconds(200)) std::this_thread::yield();
            if (queue_revive(c, q) != MEC_OK && !q->broken.load()) {
                q->broken.store(true);  // the relaunch failed: the next pass withdraws the job
            }
        }
        __builtin_ia32_pause();
    }
    if (traced && taken && rc == MEC_OK) {
        QTrace &tr = last_trace();
        tr.host_seen_ns = mono_ns();
        tr.host_post_ns = t_post;
        tr.dev_take = s->trace[0];
        tr.dev_fence = s->trace[1];
        tr.dev_desc = s->trace[2];
        tr.dev_loaded = s->trace[3];
        tr.dev_end = s->trace[4];
        tr.parts = q->parts;
        tr.valid = 1;
    }
    if (track) q->inflight.fetch_sub(1, std::memory_order_relaxed);
    if (rc == MEC_OK && taken) {
        q->hs[i].calls.fetch_add(1, std::memory_order_relaxed);
        q->hs[i].busy.store(false, std::memory_order_release);
    }
    return taken;
}

}  // namespace core
}  // namespace mec

using namespace mec::core;

extern "C" {

int mec_queue_trace_enable(mec_ctx *c, int on) {
    CHECK_CTX(c);
    for (mec_ctx *s : c->shards) mec_queue_trace_enable(s, on);
    std::lock_guard<std::mutex> g(c->hq_mu);
    if (!c->hq) return c->shards.empty() ? fail(MEC_EINVAL, "no host queue on this context") : MEC_OK;
    c->hq->trace.store(on != 0);
    return MEC_OK;
}

int mec_queue_last_trace(mec_queue_trace *out) {
    if (!out) return fail(MEC_EINVAL, "null argument");
    QTrace &t = last_trace();
    if (!t.valid) return fail(MEC_EINVAL, "no traced queue call on this thread");
    out->host_post_ns = t.host_post_ns;
    out->host_seen_ns = t.host_seen_ns;
    out->dev_take = t.dev_take;
    out->dev_fence = t.dev_fence;
    out->dev_desc = t.dev_desc;
    out->dev_loaded = t.dev_loaded;
    out->dev_end = t.dev_end;
    out->parts = t.parts;
    t.valid = 0;
    return MEC_OK;
}

int mec_set_host_queue(mec_ctx *c, uint32_t slots) {
    CHECK_CTX(c);
    for (mec_ctx *s : c->shards) {
        int rc = mec_set_host_queue(s, slots);
        if (rc != MEC_OK) return rc;
    }
    if (!c->shards.empty()) return MEC_OK;  // a multi-device context's host calls all go to its shards
    std::lock_guard<std::mutex> g(c->hq_mu);
    if (!queue_stop(c)) return fail(MEC_EHIP, "the host queue kernel did not leave; its memory is leaked");
    return slots ? queue_start(c, slots) : MEC_OK;
}

}  // extern "C"
