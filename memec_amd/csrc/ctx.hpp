// ctx.hpp — libmec internals shared by mec.cpp (lifecycle, strided entry
// points, single-stripe host staging) and batch.cpp (pointer-table batches,
// host pipeline, request coalescer).  Not part of the ABI.
#pragma once

#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <condition_variable>
#include <cstdint>
#include <deque>
#include <functional>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <unordered_map>
#include <vector>

#include "gf_math.hpp"
#include "kernels.hpp"
#include "mec.h"

namespace mec {
namespace core {

using mec::Field;
using mec::Mat;

// Thread-local error text (mec_last_error) and status helpers.
extern thread_local std::string g_err;
int fail(int code, const char *fmt, ...) __attribute__((format(printf, 2, 3)));
int hip_fail(hipError_t e, const char *what);

#define HIP_TRY(expr)                                     \
    do {                                                  \
        hipError_t e_ = (expr);                           \
        if (e_ != hipSuccess) return hip_fail(e_, #expr); \
    } while (0)

// Restores the caller's current device on scope exit.
struct DeviceGuard {
    int prev = -1;
    bool ok = true;
    explicit DeviceGuard(int dev) {
        if (hipGetDevice(&prev) != hipSuccess) prev = -1;
        if (prev != dev) ok = hipSetDevice(dev) == hipSuccess;
    }
    ~DeviceGuard() {
        int cur = -1;
        if (prev >= 0 && hipGetDevice(&cur) == hipSuccess && cur != prev) (void)hipSetDevice(prev);
    }
};

// Staging resources for the single-stripe host entry points (one per
// concurrent caller; server workers share one context, worker.cc:128-137):
// a stream and (k + m) chunk slots of pinned host memory mapped into the
// GPU — unregistered chunks are copied into the slots and the kernel codes
// them there over PCIe (no HBM round trip, one launch per call).
struct Lane {
    hipStream_t stream = nullptr;
    hipEvent_t done = nullptr;  // system-scope release: host memory written by the lane's launches is visible
    uint8_t *host = nullptr;    // (k + m) chunk slots, pinned + mapped
    uint8_t *hdev = nullptr;    // their device address
    size_t bytes = 0;
};

// Pinned host + device copy of a gather table (per-stripe chunk pointers)
// for the device-memory pointer batches.  `done` is recorded after the last
// launch that reads it; the slot is reused only after it fired.
struct TableSlot {
    std::mutex mu;
    uint64_t *host = nullptr;  // pinned + GPU-mapped
    uint64_t *hdev = nullptr;  // device address of host (small zero-copy batches read it in place)
    uint64_t *dev = nullptr;
    size_t cap = 0;  // entries
    hipEvent_t done = nullptr;    // the launches that read dev have finished (on the caller's stream)
    hipEvent_t copied = nullptr;  // dev holds this call's tables (on the context's copy stream)
    bool pending = false;
    uint64_t *xdev = nullptr;  // 32-bit slab offset rows expanded to pointers (mec_*_batch32)
    size_t xcap = 0;           // bytes
};
constexpr int kTableSlots = 4;

// Double-buffered host pipeline of the host-memory pointer batches over
// unregistered chunks: a sub-batch is packed into pinned, GPU-mapped
// staging, coded there by the kernel over PCIe, and unpacked; packing the
// next sub-batch overlaps the kernel on the current one.
struct HostPipe {
    std::mutex mu;
    hipStream_t stream[2] = {nullptr, nullptr};
    hipEvent_t done[2] = {nullptr, nullptr};
    uint8_t *host[2] = {nullptr, nullptr};  // pinned + mapped
    uint8_t *hdev[2] = {nullptr, nullptr};  // device addresses of host[]
    size_t bytes = 0;  // per buffer
};

// One pending single-stripe host request (mec_*_host while coalescing).
struct Request;

constexpr uint32_t kMaxLeaders = 4;

struct Coalescer {
    std::mutex mu;
    std::condition_variable cv;
    std::deque<Request *> queue;
    uint32_t leaders = 0;    // batches in flight (at most kMaxLeaders)
    std::atomic<uint32_t> max_batch{0};  // 0 = coalescing off (read lock-free on every host call)
    uint64_t batches = 0, requests = 0;  // statistics
};

// queue.hip: device-side submission queue for single-stripe host calls.
constexpr uint32_t kQMaxSrc = 32, kQMaxDst = 4, kQMaxSlots = 1024;
constexpr uint32_t kQMaxParts = 64;  // workgroups per slot (one call's chunk spread over CUs)
// a timed-out call waits at most this many call timeouts (at least 10 s)
// for the resident grid to leave before it gives up with MEC_EHIP (queue_try)
constexpr uint64_t kQDrainFactor = 4;
constexpr uint32_t kQBmRows = kQMaxDst * 8;  // bitmatrix output packet rows (outputs x w <= 8)
// A job's descriptor (host -> GPU): sources, outputs, chunk bytes,
// accumulate, w (0: byte-wise GF(2^8); 1..8: Jerasure bitmatrix over w
// packets), packet bytes, trace, -; then chunk addresses and tables.
struct QDesc {
    uint32_t hdr[8];
    uint64_t src[kQMaxSrc];  // device addresses of registered chunks (0 = zeros)
    uint64_t dst[kQMaxDst];  // (0 = unwanted output)
    union {
        // byte-wise: the v_perm tables of coefficient (output r, source j)
        // at (r * sources + j) * 5 dwords (t0 t1 u0 u1 v, gf8_kernel.hpp),
        // built on the host (a table per GF(2^8) value, computed once)
        uint32_t tab_w[kQMaxDst * kQMaxSrc * 5];
        uint32_t mask_w[kQMaxSrc * kQBmRows / 4];  // bitmatrix bytes [source][output*w + l], bit x
    };
};
struct alignas(128) QSlot {  // in GPU-mapped coherent host memory
    // host -> GPU: (number of the posted job << 16) | (sources << 8) |
    // outputs — the poll that sees a job also sizes its descriptor read
    // (host-memory slots; device-memory slots carry it in QDevSlot)
    uint64_t seq;
    uint64_t pad0[15];
    uint64_t done[kQMaxParts];  // GPU -> host: number of the last job each part finished
    QDesc d;                    // the descriptor (host-memory slots; the host's staging copy otherwise)
    // GPU -> host when hdr[6] (trace) is set: part 0's s_memrealtime when it
    // took the job, after its acquire fence, with the descriptor in LDS,
    // when thread 0's source loads had returned, and with its output stores
    // acknowledged (just before its done store)
    uint64_t trace[5];
};
// The host -> GPU half of a slot in device memory (uncached), written by the
// host through the PCIe BAR: part 0 then polls HBM and reads the
// descriptor from HBM instead of over PCIe (queue_try, MEC_QUEUE_DEVSLOT).
struct alignas(256) QDevSlot {
    uint64_t seq;
    uint64_t pad0[7];
    QDesc d;
};
// The one-pass kernel's permute tables (gf8_mg_kernel), one entry per
// distinct > 4-row matrix: suballocated from device arena blocks with a
// pinned host mirror (the image stays there as the source of its async
// upload), uploaded on the calling stream; `ready` fires when the upload
// has landed, so a hit from another stream waits for it on the device.
// At most `cap` bytes: matrices past it (a decode that walks through many
// erasure patterns) run as 4-row launches with their coefficients in
// kernel arguments instead of growing the cache.
struct MgEntry {
    const uint32_t *dev = nullptr;
    hipEvent_t ready = nullptr;
    bool landed = false;
};
struct MgCache {
    std::mutex mu;
    std::unordered_map<std::string, MgEntry> map;
    std::vector<uint8_t *> dev_blocks, host_blocks;
    size_t block_used = 0;   // bytes used in the last block
    size_t bytes = 0;        // bytes handed to entries
    size_t cap = 0;          // MEC_MG_CACHE_BYTES at mec_create (default 64 MiB)
    uint64_t uncached = 0;   // launches that fell back past the cap
};
constexpr size_t kMgBlock = size_t(4) << 20;

// Run-time compiled bit-sliced kernels of wide matrices (jit.cpp).
struct JitKernel {
    std::atomic<int> state{0};  // 0 compiling, 1 ready, -1 failed
    hipModule_t mod = nullptr;
    hipFunction_t fn = nullptr;
    double compile_ms = 0;
    std::string err;
    uint32_t tpb = 1;  // gathered: tiles per block it was built for (> 1: looped)
    // the last launch on each stream this kernel ran on (device-scope
    // events): jit_release waits for these, and nothing else, before it
    // unloads the module
    std::mutex ev_mu;
    std::vector<std::pair<hipStream_t, hipEvent_t>> ev;
};
// Shared with the compile jobs a context queued: a job may still sit in the
// process-wide queue when its context is destroyed, so it holds this (and
// its JitKernel) by shared_ptr; a cancelled context's queued jobs skip the
// compile, and jit_release waits only for a compile already running.
struct JitShared {
    std::mutex mu;
    std::condition_variable cv;
    bool cancelled = false;
    uint32_t pending = 0;  // queued or running
    uint32_t running = 0;
    uint64_t ready = 0, failed = 0;
    double compile_ms = 0;
};
struct JitCache {
    std::mutex mu;  // the map
    std::unordered_map<std::string, std::shared_ptr<JitKernel>> map;
    size_t cap = 512;        // MEC_JIT_MAX_KERNELS: matrices per context
    uint32_t max_queued = 16;  // MEC_JIT_MAX_QUEUED: compiles waiting per context
    std::string arch = "gfx950";  // the device's gcnArchName (hiprtc --offload-arch)
    std::shared_ptr<JitShared> sh = std::make_shared<JitShared>();
    std::atomic<uint64_t> launches{0};
};

// Grid-wide control words, after the slots in the same mapped allocation.
enum : uint32_t { kQCtlStop = 0, kQCtlExit = 1, kQCtlWords = 2 };
struct HostQueue {
    QSlot *host = nullptr, *dev = nullptr;
    QDevSlot *dslot = nullptr;        // device-memory slot halves (large-BAR devices), else null
    // per slot, host side, on its own cache line (16 server workers posting
    // at ~1 M calls/s would otherwise bounce one line of flags)
    struct alignas(64) HostSlotState {
        std::atomic<bool> busy{false};
        uint64_t seqno = 0;  // number of the last job posted
        std::atomic<uint64_t> calls{0};
    };
    HostSlotState *hs = nullptr;
    uint32_t *ctl_host = nullptr, *ctl_dev = nullptr;  // [kQCtlStop] host -> GPU, [kQCtlExit] leader -> grid
    uint64_t *act = nullptr;          // device memory: per-slot time of the last job (s_memrealtime)
    // device memory, per slot: [0, slots) the job part 0 took (`go`, read by
    // the slot's other parts), [slots, 2 slots) the launch epoch in which
    // part 0 left the grid (`left`: the other parts leave after it)
    uint64_t *link = nullptr;
    uint64_t epoch = 0;               // launches so far (the `left` epoch)
    uint32_t slots = 0, parts = 1, max_chunk = 0, threads = 0;
    std::atomic<uint64_t> timeouts{0};  // calls that timed out (each stops the queue for good)
    uint32_t solo_max = 0;            // larger chunks use the queue only beside other queue calls
    std::atomic<uint32_t> inflight{0};
    std::atomic<bool> broken{false};  // a call timed out: the queue is stopped for good
    uint64_t idle_ticks = 0, timeout_ms = 5000;
    std::atomic<bool> trace{false};   // mec_queue_trace_enable
    // MEC_QUEUE_PUSH=<bytes>: for chunks up to that size the caller streams
    // the job's sources through the BAR into this per-slot device area
    // (uncached, next to the device-memory descriptor), so part 0 reads them
    // from HBM instead of across PCIe (§4.5)
    uint8_t *push = nullptr;
    uint32_t push_max = 0;
    size_t push_chunk = 0;  // bytes per source in the area (chunk rounded up to 64)
    hipStream_t stream = nullptr;
    std::mutex mu;  // launches
    std::atomic<uint64_t> launches{0};
};

}  // namespace core
}  // namespace mec

struct mec_ctx {
    int family;
    uint32_t k, m, w, cs, packet;
    int device;
    mec::Mat A;  // m x k (Jerasure) or (k+m) x k (ISA-L)
    std::mutex plan_mu;
    std::unordered_map<uint64_t, std::shared_ptr<mec::LinearPlan>> plans;
    // lock-free index of `plans` for the per-call lookup (mec.cpp get_plan):
    // open addressing on the present mask, entries only ever added (the
    // plans live in `plans` until mec_destroy); a full table falls back to
    // the mutex
    static constexpr size_t kPlanSlots = 4096;
    std::unique_ptr<std::atomic<uint64_t>[]> plan_keys{new std::atomic<uint64_t>[kPlanSlots]()};
    std::unique_ptr<std::atomic<const mec::LinearPlan *>[]> plan_vals{new std::atomic<const mec::LinearPlan *>[kPlanSlots]()};
    std::mutex lane_mu;
    std::vector<mec::core::Lane *> lanes_free;
    std::vector<mec::core::Lane *> lanes_all;
    // pipelined dense host batch (mec_encode_host_batch): HBM buffers, and
    // pinned host staging the caller's pageable bytes are copied through
    std::mutex batch_mu;
    hipStream_t bstream[2] = {nullptr, nullptr};
    uint8_t *bdev[2] = {nullptr, nullptr};
    uint8_t *bpin[2] = {nullptr, nullptr};
    hipEvent_t bdone[2] = {nullptr, nullptr};
    size_t bbytes = 0;
    // pointer batches (batch.cpp)
    std::mutex tab_mu;
    uint32_t tab_next = 0;
    hipStream_t tab_stream = nullptr;  // table uploads (batch.cpp table_upload), created at first use
    mec::core::TableSlot tabs[mec::core::kTableSlots];
    mec::core::HostPipe pipe;
    mec::core::Coalescer coal;
    // host-call statistics, striped over cache lines by calling thread
    struct alignas(64) CallCounters {
        std::atomic<uint64_t> zc{0}, staged{0};
    };
    static constexpr int kCounterStripes = 16;
    CallCounters calls[kCounterStripes];
    std::mutex hq_mu;
    mec::core::HostQueue *hq = nullptr;  // mec_set_host_queue
    // multi-GPU context (multi.cpp): one ordinary context per device
    std::vector<mec_ctx *> shards;
    std::atomic<uint32_t> rr{0};
    // mec_set_probe: MEC_PROBE_XOR runs strided byte-wise launches as their
    // arithmetic-free twin (measurement only)
    std::atomic<int> probe{0};
    // device copies of the permute tables of > 4-row matrices
    // (gf8_mg_kernel), keyed by (rows, k, rows per group, coefficient
    // bytes); bounded (mec.cpp mg_tables)
    mec::core::MgCache mg;
    // bit-sliced kernels compiled for this context's wide matrices
    mec::core::JitCache jit;

    bool byte_wise() const { return family != MEC_CAUCHY_GOOD; }
    mec::Scheme scheme() const {
        return family == MEC_RS_VANDERMONDE ? mec::Scheme::kJerasureRS
               : family == MEC_CAUCHY_GOOD  ? mec::Scheme::kJerasureCauchy
                                            : mec::Scheme::kIsal;
    }
    // coefficient of parity row i (0..m-1), data column j
    uint8_t coef(uint32_t i, uint32_t j) const {
        return byte_wise() && family != MEC_RS_VANDERMONDE ? A[size_t(k + i) * k + j] : A[size_t(i) * k + j];
    }
};

namespace mec {
namespace core {

inline bool has_device(const mec_ctx *c) { return c->device >= 0; }

// The calling thread's stripe of the per-call counters.
inline mec_ctx::CallCounters &call_counters(mec_ctx *c) {
    static thread_local const int stripe = int(std::hash<std::thread::id>()(std::this_thread::get_id()) % mec_ctx::kCounterStripes);
    return c->calls[stripe];
}
inline void count_zc(mec_ctx *c) { call_counters(c).zc.fetch_add(1, std::memory_order_relaxed); }
inline void count_staged(mec_ctx *c) { call_counters(c).staged.fetch_add(1, std::memory_order_relaxed); }

#define CHECK_CTX(c)                                                          \
    do {                                                                      \
        if (!(c)) return fail(MEC_EINVAL, "null context");                    \
        if (!has_device(c)) return fail(MEC_ENODEV, "context has no device"); \
    } while (0)

// Strided chunk addressing of a launch: source j of stripe s at
// src + s * sss + src_off[j], output r at dst + s * dss + dst_off[r].
struct Layout {
    const uint8_t *src = nullptr;
    uint8_t *dst = nullptr;
    int64_t sss = 0, dss = 0;
    std::vector<int64_t> src_off, dst_off;
    size_t ns = 0, nd = 0;

    static Layout strided(const uint8_t *src, int64_t sss, std::vector<int64_t> so, uint8_t *dst, int64_t dss,
                          std::vector<int64_t> dof) {
        Layout l;
        l.src = src;
        l.dst = dst;
        l.sss = sss;
        l.dss = dss;
        l.ns = so.size();
        l.nd = dof.size();
        l.src_off = std::move(so);
        l.dst_off = std::move(dof);
        return l;
    }
};

void bit_block(const Field &f, unsigned e, uint32_t w, uint8_t *mask, size_t mstride);
// A one-pass launch (gf8_mg_kernel) of coef (nd x ns, nd > 4, GF(2^8)):
// structure, rows per group and the device copy of its tables into L.
// MEC_OK, kMgUncached (the cache is full: the caller codes the rows in
// groups of 4 instead) or an error.
constexpr int kMgUncached = 1;
int mg_prepare(mec_ctx *c, const Mat &coef, size_t nd, size_t ns, Gf8MgLaunch &L, hipStream_t stream);
void mg_release(mec_ctx *c);
// jit.cpp: wide byte-wise outputs through a run-time compiled bit-sliced
// kernel.  jit_kernel: the kernel for this matrix, or nullptr (compiling,
// failed, capped, MEC_BITSLICE=0) — the caller then runs gf8_mg_kernel.
bool jit_wanted(const mec_ctx *c, size_t nd, size_t ns, const Mat &coef, bool gathered);
bool coef_vand(const Mat &coef, size_t nd, size_t ns);
JitKernel *jit_kernel(mec_ctx *c, const Mat &coef, size_t nd, size_t ns, bool accumulate, bool gather,
                      bool twin = false);
int jit_launch(mec_ctx *c, JitKernel *k, const BsLaunch &L, hipStream_t stream);
void jit_init(mec_ctx *c);
void jit_release(mec_ctx *c);
// Byte-wise outputs beyond 4 per launch go through gf8_mg_kernel (every
// source read once) unless MEC_WIDE=0 or the chunk has a sub-16-byte tail.
bool mg_wanted(const mec_ctx *c, size_t nd);
// outputs (^)= coef (nd x ns over GF(2^w)) * sources, every stripe.
int apply(mec_ctx *c, const Layout &lay, const Mat &coef, uint32_t n_stripes, bool accumulate, hipStream_t stream);
int apply(mec_ctx *c, const uint8_t *src, int64_t sss, const std::vector<int64_t> &src_off, uint8_t *dst,
          int64_t dss, const std::vector<int64_t> &dst_off, const Mat &coef, uint32_t n_stripes, bool accumulate,
          hipStream_t stream);
// Cached decode plan for a present-chunk mask (reference survivor choice).
int get_plan(mec_ctx *c, uint64_t present, const mec::LinearPlan *&out);  // owned by the context
Mat encode_rows(const mec_ctx *c, const std::vector<uint32_t> &rows, const std::vector<uint32_t> &cols);
std::vector<uint32_t> mask_rows(const mec_ctx *c, uint32_t parity_mask);
Lane *lane_acquire(mec_ctx *c, int &rc);
void lane_release(mec_ctx *c, Lane *l);

struct LaneHold {
    mec_ctx *c;
    Lane *l;
    ~LaneHold() {
        if (l) lane_release(c, l);
    }
};

// hostmem.cpp: registered (GPU-mapped) host ranges.  zc_device_address:
// device address of [p, p + len) if it lies in one registered range.
// zc_translate: every non-zero entry of ptrs (chunks of len bytes) replaced
// by its device address; false (ptrs partly rewritten) if any is not
// registered.
bool zc_device_address(const void *p, size_t len, uint64_t &dev);
bool zc_any_registered();
bool zc_translate(uint64_t *ptrs, size_t n, size_t len);

// multi.cpp: multi-GPU contexts.  shard_run runs fn(shard, s0, s1) on every
// shard's contiguous stripe range concurrently and returns the first error
// (its text prefixed with the device); shard_pick round-robins.
bool is_multi(const mec_ctx *c);
mec_ctx *shard_pick(mec_ctx *c);
int shard_run(mec_ctx *c, uint32_t n, const std::function<int(mec_ctx *, uint32_t, uint32_t)> &fn);

// Wait for a lane's single-call work, its host-memory outputs visible to
// the host: an event recorded with an explicit system-scope release
// (hipEventReleaseToSystem) after the launch, then waited for — the call's
// own completion point does not depend on how the runtime scopes a
// kernel's end-of-dispatch release (the r05 zero-copy audit).
// MEC_SYNC_SPIN=1 polls the event for up to 200 us first: +8 % calls/s for
// one staged caller, but -14 % at 16 workers x RS(8,2)@4K (the pollers
// compete for the cores the callers need) -- profiles/r01/host/sync_ab.log.
hipError_t lane_sync(Lane *l);

// batch.cpp: memcpy of n bytes split over a few threads when large
// (MEC_COPY_THREADS).
void par_memcpy(void *dst, const void *src, size_t n);

// queue.hip.  queue_try: run one zero-copy call (addrs = ns sources then nd
// outputs, device addresses) through the resident kernel; false = not
// eligible, no free slot, or a timed-out job that was withdrawn (nothing
// done: the caller takes the launch path), else rc holds the result.
// hsrc (optional): the sources' host addresses, for MEC_QUEUE_PUSH.
bool queue_try(mec_ctx *c, const uint64_t *addrs, size_t ns, size_t nd, const Mat &coef, bool accumulate, int &rc,
               const uint8_t *const *hsrc = nullptr);
// Stop the resident kernel and free the queue; false if the grid was still
// running at the drain cap (the queue's memory is then leaked, and so must
// be anything its jobs can address: mec_destroy keeps the staging lanes).
bool queue_stop(mec_ctx *c);

// batch.cpp
void batch_release(mec_ctx *c);  // frees table slots and the host pipeline
bool coalescing(mec_ctx *c);
int submit_encode(mec_ctx *c, const uint8_t *const *data, uint8_t *const *parity);
int submit_decode(mec_ctx *c, uint8_t *const *chunks, uint64_t present);
int submit_update(mec_ctx *c, uint32_t index, const uint8_t *delta, uint8_t *const *parity);

}  // namespace core
}  // namespace mec
