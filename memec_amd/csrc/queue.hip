// queue.hip — device-side submission queue for single-stripe host calls.
//
// MemEC's workers call Coding::encode / decode one stripe at a time from
// many threads at once (server.cc:107, worker.cc:128-137; SURVEY §8b:
// "a GPU implementation needs per-thread streams or a submission queue").
// A kernel launch per call costs ~5 us of HIP runtime on the calling
// thread, takes runtime locks shared by every caller, and completion is
// seen through hipStreamSynchronize.  This queue removes the runtime from
// the per-call path:
//   * a resident kernel runs one workgroup per slot; each polls its slot in
//     GPU-mapped, coherent host memory (system-scope acquire loads);
//   * a caller takes a free slot, writes the call's descriptor (device
//     addresses of registered chunks, GF(2^8) coefficients), publishes a new
//     sequence number, and spins on the slot's `done` word, which the
//     workgroup stores (system-scope release) after its outputs;
//   * the workgroup builds the v_perm tables (gf8_kernel.hpp) from the raw
//     coefficients in LDS and codes the chunk over PCIe, one 16-byte unit
//     per lane.
// Exit conditions every wave reaches: the stop word (mec_set_host_queue(0),
// mec_destroy) or an idle timeout measured with s_memrealtime.  A caller that
// finds the kernel gone (idle exit) with its job pending relaunches it; the
// new kernel starts from each slot's `done`, so no job is lost or run twice.
// Launches of the resident kernel go to one stream, so two instances never
// run at once.
//
// Scope: byte-wise families (RS, ISA-L), chunks of at most
// MEC_QUEUE_MAX_CHUNK bytes (default 16 KiB; larger chunks want the whole
// GPU, so they keep the launch path), either zero-copy (registered) or
// staged: unregistered chunks are copied into a lane's mapped pinned buffer
// and the workgroup codes that buffer in place (mec.cpp lane_run).
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdlib>
#include <cstring>
#include <thread>

#include "ctx.hpp"
#include "kernels.hpp"
#include "stream_common.hpp"

namespace mec {
namespace core {
namespace {

using detail::u32x4;
constexpr int kQThreads = 1024;  // most threads per slot: a 16 KiB chunk in one pass
constexpr int kQBatch = 16;

__device__ __forceinline__ uint32_t gmul8(uint32_t a, uint32_t b) {  // GF(2^8), poly 0x11d
    uint32_t p = 0;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        p ^= (b & 1u) ? a : 0u;
        b >>= 1;
        a <<= 1;
        a ^= (a & 0x100u) ? 0x11du : 0u;
    }
    return p;
}

__device__ __forceinline__ uint32_t pack4(uint32_t c, uint32_t a, uint32_t b, uint32_t d, uint32_t e) {
    return gmul8(c, a) | gmul8(c, b) << 8 | gmul8(c, d) << 16 | gmul8(c, e) << 24;
}

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
                                          uint32_t acc_in, uint64_t off, uint32_t n) {
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
#pragma unroll
        for (int jj = 0; jj < kQBatch; ++jj) {
#pragma unroll
            for (int r = 0; r < int(kQMaxDst); ++r) {
                if (j0 + jj < ns && uint32_t(r) < nd) {
                    const uint32_t *T = tab + (r * kQMaxSrc + j0 + jj) * 8;
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

template <typename T>
__device__ __forceinline__ T sys_load(const T *p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

__global__ __launch_bounds__(kQThreads) void queue_kernel(QSlot *slots, const uint32_t *stop, uint64_t idle_ticks,
                                                         uint32_t nthr) {
    __shared__ uint32_t tab[kQMaxDst * kQMaxSrc * 8];
    __shared__ uint64_t addr[kQMaxSrc + kQMaxDst];
    __shared__ uint32_t hdr[4];
    __shared__ uint32_t cw[kQMaxDst * kQMaxSrc / 4];
    __shared__ uint32_t cmd;
    QSlot *s = slots + blockIdx.x;
    const uint32_t t = threadIdx.x;
    uint64_t last = 0, t0 = 0;
    if (t == 0) {
        last = sys_load(&s->done);
        t0 = __builtin_amdgcn_s_memrealtime();
    }
    for (;;) {
        if (t == 0) {
            uint32_t c = 0;
            for (uint32_t n = 1;; ++n) {  // one PCIe read per poll; stop / idle every 64th
                const uint64_t q = __hip_atomic_load(&s->seq, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM);
                if (q != last) {
                    last = q;
                    c = 1;
                    break;
                }
                if (n % 64 == 0 &&
                    (sys_load(stop) != 0u || __builtin_amdgcn_s_memrealtime() - t0 > idle_ticks))
                    break;
                __builtin_amdgcn_s_sleep(4);
            }
            cmd = c;
        }
        __syncthreads();
        if (cmd == 0) return;  // uniform: stop or idle
        if (t < 4) hdr[t] = sys_load(&s->hdr[t]);
        if (t < kQMaxSrc) addr[t] = sys_load(&s->src[t]);
        else if (t < kQMaxSrc + kQMaxDst) addr[t] = sys_load(&s->dst[t - kQMaxSrc]);
        else if (t < kQMaxSrc + kQMaxDst + kQMaxDst * kQMaxSrc / 4)
            cw[t - kQMaxSrc - kQMaxDst] = sys_load(&s->coef_w[t - kQMaxSrc - kQMaxDst]);
        __syncthreads();
        const uint32_t ns = hdr[0], nd = hdr[1], bytes = hdr[2], acc_in = hdr[3];
        if (t < nd * ns) {
            const uint32_t r = t / ns, j = t - r * ns, b = r * kQMaxSrc + j;
            const uint32_t c = (cw[b / 4] >> (8 * (b % 4))) & 0xffu;
            uint32_t *T = tab + b * 8;
            T[0] = pack4(c, 0, 1, 2, 3);
            T[1] = pack4(c, 4, 5, 6, 7);
            T[2] = pack4(c, 0, 8, 16, 24);
            T[3] = pack4(c, 32, 40, 48, 56);
            T[4] = pack4(c, 0, 64, 128, 192);
        }
        __syncthreads();
        const uint32_t full = bytes / 16;
        for (uint32_t u = t; u < full; u += nthr)
            code_unit<true>(addr, tab, ns, nd, acc_in, uint64_t(u) * 16, 16);
        if (bytes % 16 && t == full % nthr)  // the partial last unit
            code_unit<false>(addr, tab, ns, nd, acc_in, uint64_t(full) * 16, bytes % 16);
        __threadfence_system();  // this lane's outputs reach host memory ...
        __syncthreads();         // ... before the slot is marked done
        if (t == 0) {
            __hip_atomic_store(&s->done, last, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
            t0 = __builtin_amdgcn_s_memrealtime();
        }
    }
}

uint64_t env_u64(const char *name, uint64_t dflt) {
    const char *e = std::getenv(name);
    return e && *e ? std::strtoull(e, nullptr, 10) : dflt;
}

// Launch the resident kernel (caller holds q->mu).
int queue_launch(mec_ctx *c, HostQueue *q) {
    DeviceGuard dg(c->device);
    hipLaunchKernelGGL(queue_kernel, dim3(q->slots), dim3(q->threads), 0, q->stream, q->dev, q->stop_dev, q->idle_ticks,
                       q->threads);
    HIP_TRY(hipGetLastError());
    q->launches++;
    return MEC_OK;
}

// The resident kernel has exited (idle) while jobs may be pending: relaunch.
int queue_revive(mec_ctx *c, HostQueue *q) {
    std::lock_guard<std::mutex> g(q->mu);
    const hipError_t e = hipStreamQuery(q->stream);
    if (e == hipErrorNotReady) return MEC_OK;  // still running
    if (e != hipSuccess) return hip_fail(e, "queue kernel");
    return queue_launch(c, q);
}

}  // namespace

void queue_stop(mec_ctx *c) {
    HostQueue *q = c->hq;
    if (!q) return;
    c->hq = nullptr;
    {
        DeviceGuard dg(c->device);
        __atomic_store_n(q->stop_host, 1u, __ATOMIC_RELEASE);
        (void)hipStreamSynchronize(q->stream);  // every workgroup sees the stop word and returns
        (void)hipStreamDestroy(q->stream);
        (void)hipHostFree(q->host);
    }
    delete[] q->busy;
    delete q;
}

int queue_start(mec_ctx *c, uint32_t slots) {
    if (slots > kQMaxSlots) return fail(MEC_EINVAL, "at most %u queue slots", kQMaxSlots);
    DeviceGuard dg(c->device);
    std::unique_ptr<HostQueue> q(new HostQueue);
    q->slots = slots;
    q->max_chunk = uint32_t(env_u64("MEC_QUEUE_MAX_CHUNK", 16 << 10));
    // a lone call on a chunk above this codes faster as a launch (many
    // workgroups over PCIe) than on one queue workgroup
    q->solo_max = uint32_t(env_u64("MEC_QUEUE_SOLO_MAX", q->max_chunk));
    q->idle_ticks = env_u64("MEC_QUEUE_IDLE_MS", 50) * 100000ull;  // s_memrealtime: 100 MHz
    // one 16-byte unit per thread up to kQThreads (a 4 KiB chunk: 256 threads;
    // idle threads only cost barrier time), at least 128 (descriptor loads)
    q->threads = std::min<uint32_t>(kQThreads, std::max<uint32_t>(128, (c->cs / 16 + 63) / 64 * 64));
    const size_t bytes = sizeof(QSlot) * slots + 256;
    void *h = nullptr;
    HIP_TRY(hipHostMalloc(&h, bytes, hipHostMallocMapped | hipHostMallocCoherent | hipHostMallocPortable));
    std::memset(h, 0, bytes);
    void *d = nullptr;
    hipError_t e = hipHostGetDevicePointer(&d, h, 0);
    if (e != hipSuccess) {
        (void)hipHostFree(h);
        return hip_fail(e, "hipHostGetDevicePointer");
    }
    q->host = static_cast<QSlot *>(h);
    q->dev = static_cast<QSlot *>(d);
    q->stop_host = reinterpret_cast<uint32_t *>(static_cast<uint8_t *>(h) + sizeof(QSlot) * slots);
    q->stop_dev = reinterpret_cast<uint32_t *>(static_cast<uint8_t *>(d) + sizeof(QSlot) * slots);
    q->busy = new std::atomic<bool>[slots];
    for (uint32_t i = 0; i < slots; ++i) q->busy[i].store(false);
    e = hipStreamCreateWithFlags(&q->stream, hipStreamNonBlocking);
    if (e != hipSuccess) {
        (void)hipHostFree(h);
        delete[] q->busy;
        return hip_fail(e, "hipStreamCreate");
    }
    {
        std::lock_guard<std::mutex> g(q->mu);
        int rc = queue_launch(c, q.get());
        if (rc != MEC_OK) {
            (void)hipStreamDestroy(q->stream);
            (void)hipHostFree(h);
            delete[] q->busy;
            return rc;
        }
    }
    c->hq = q.release();
    return MEC_OK;
}

bool queue_try(mec_ctx *c, const uint64_t *addrs, size_t ns, size_t nd, const Mat &coef, bool accumulate, int &rc) {
    HostQueue *q = c->hq;
    if (!q || !c->byte_wise() || c->cs > q->max_chunk || ns > kQMaxSrc || nd > kQMaxDst || nd == 0)
        return false;
    if (c->cs > q->solo_max && q->inflight.load(std::memory_order_relaxed) == 0) return false;
    // a free slot, starting from a per-thread hint so callers spread out
    static thread_local uint32_t hint = uint32_t(std::hash<std::thread::id>()(std::this_thread::get_id()));
    uint32_t i = 0;
    bool got = false;
    for (uint32_t n = 0; n < q->slots && !got; ++n) {
        i = (hint + n) % q->slots;
        bool f = false;
        got = !q->busy[i].load(std::memory_order_relaxed) && q->busy[i].compare_exchange_strong(f, true);
    }
    if (!got) return false;  // every slot busy: the launch path takes this call
    hint = i;
    q->inflight.fetch_add(1, std::memory_order_relaxed);
    QSlot *s = q->host + i;
    s->hdr[0] = uint32_t(ns);
    s->hdr[1] = uint32_t(nd);
    s->hdr[2] = c->cs;
    s->hdr[3] = accumulate ? 1u : 0u;
    for (size_t j = 0; j < ns; ++j) s->src[j] = addrs[j];
    for (size_t r = 0; r < nd; ++r) s->dst[r] = addrs[ns + r];
    uint8_t cb[kQMaxDst * kQMaxSrc] = {};
    for (size_t r = 0; r < nd; ++r)
        for (size_t j = 0; j < ns; ++j) cb[r * kQMaxSrc + j] = coef[r * ns + j];
    std::memcpy(s->coef_w, cb, sizeof(cb));
    const uint64_t seq = __atomic_load_n(&s->seq, __ATOMIC_RELAXED) + 1;
    __atomic_store_n(&s->seq, seq, __ATOMIC_RELEASE);  // publishes the descriptor
    // wait for the workgroup; relaunch the kernel if it idled out meanwhile
    rc = MEC_OK;
    const auto t0 = std::chrono::steady_clock::now();
    uint32_t spins = 0;
    while (__atomic_load_n(&s->done, __ATOMIC_ACQUIRE) != seq) {
        if (++spins % 2048 == 0) {
            const auto dt = std::chrono::steady_clock::now() - t0;
            if (dt > std::chrono::seconds(5)) {
                rc = fail(MEC_EHIP, "host queue: no completion within 5 s");
                break;  // the slot stays busy: its job may still run
            }
            if (dt > std::chrono::microseconds(200)) std::this_thread::yield();
            rc = queue_revive(c, q);
            if (rc != MEC_OK) break;
        }
        __builtin_ia32_pause();
    }
    q->inflight.fetch_sub(1, std::memory_order_relaxed);
    if (rc == MEC_OK) {
        q->busy[i].store(false, std::memory_order_release);
        q->calls++;
    }
    return true;
}

}  // namespace core
}  // namespace mec

using namespace mec::core;

extern "C" {

int mec_set_host_queue(mec_ctx *c, uint32_t slots) {
    CHECK_CTX(c);
    for (mec_ctx *s : c->shards) {
        int rc = mec_set_host_queue(s, slots);
        if (rc != MEC_OK) return rc;
    }
    std::lock_guard<std::mutex> g(c->hq_mu);
    queue_stop(c);
    return slots ? queue_start(c, slots) : MEC_OK;
}

}  // extern "C"
