// mec.cpp — libmec C ABI (include/mec.h): coding contexts, plan caching,
// kernel dispatch, strided device entry points and single-stripe host
// staging.  Pointer-table batches, the host pipeline and the request
// coalescer live in batch.cpp.
#include "ctx.hpp"
#include "knobs.hpp"
#include "launch_plan.hpp"

#include <chrono>
#include <cstdarg>
#include <cstdlib>
#include <cstdio>
#include <cstring>

namespace mec {
namespace core {

thread_local std::string g_err;

int fail(int code, const char *fmt, ...) {
    char buf[512];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof buf, fmt, ap);
    va_end(ap);
    g_err = buf;
    return code;
}

int hip_fail(hipError_t e, const char *what) {
    return fail(MEC_EHIP, "%s: %s", what, hipGetErrorString(e));
}

// Bitmatrix rows of GF(2^w) coefficient e: mask[l] bit x = bit l of e * 2^x
// (jerasure_matrix_to_bitmatrix, jerasure.c:271-297).
void bit_block(const Field &f, unsigned e, uint32_t w, uint8_t *mask, size_t mstride) {
    uint8_t cols[8];
    for (uint32_t x = 0; x < w; ++x) {
        cols[x] = uint8_t(e);
        e = f.mul(e, 2 % f.size());
    }
    for (uint32_t l = 0; l < w; ++l) {
        uint8_t mb = 0;
        for (uint32_t x = 0; x < w; ++x) mb |= uint8_t((cols[x] >> l & 1) << x);
        mask[l * mstride] = mb;
    }
}

// The device copy of coef's multi-group permute tables (gf8_mg_kernel):
// looked up, or built into the arena's pinned mirror and uploaded with an
// async copy on `stream` (no blocking hipMalloc / hipMemcpy on the null
// stream inside a stream-ordered call; an arena block is allocated once per
// 4 MiB of tables).  kMgUncached past the cache's cap.
int mg_tables(mec_ctx *c, const Mat &coef, size_t rows, size_t ns, int R, hipStream_t stream, const uint32_t *&out) {
    std::string key(reinterpret_cast<const char *>(coef.data()), rows * ns);
    key += char(rows);
    key += char(ns);
    key += char(R);
    MgCache &M = c->mg;
    std::lock_guard<std::mutex> g(M.mu);
    auto it = M.map.find(key);
    if (it != M.map.end()) {
        MgEntry &e = it->second;
        if (!e.landed) {
            const hipError_t q = hipEventQuery(e.ready);
            if (q == hipSuccess) e.landed = true;
            else if (q == hipErrorNotReady) HIP_TRY(hipStreamWaitEvent(stream, e.ready, 0));
            else return hip_fail(q, "mg tables upload");
        }
        out = e.dev;
        return MEC_OK;
    }
    std::vector<uint32_t> img;
    mec::gf8_mg_tables(coef.data(), int(rows), int(ns), R, img);
    const size_t bytes = (img.size() * sizeof(uint32_t) + 255) & ~size_t(255);
    if (M.bytes + bytes > M.cap || bytes > kMgBlock) {
        M.uncached++;
        return kMgUncached;
    }
    DeviceGuard dg(c->device);
    if (M.dev_blocks.empty() || M.block_used + bytes > kMgBlock) {
        uint8_t *d = nullptr, *h = nullptr;
        HIP_TRY(hipMalloc(reinterpret_cast<void **>(&d), kMgBlock));
        const hipError_t e = hipHostMalloc(reinterpret_cast<void **>(&h), kMgBlock, hipHostMallocDefault);
        if (e != hipSuccess) {
            (void)hipFree(d);
            return hip_fail(e, "mg tables staging");
        }
        M.dev_blocks.push_back(d);
        M.host_blocks.push_back(h);
        M.block_used = 0;
    }
    uint8_t *hd = M.host_blocks.back() + M.block_used, *dd = M.dev_blocks.back() + M.block_used;
    std::memcpy(hd, img.data(), img.size() * sizeof(uint32_t));
    MgEntry e;
    HIP_TRY(hipEventCreateWithFlags(&e.ready, hipEventDisableTiming));
    hipError_t err = hipMemcpyAsync(dd, hd, img.size() * sizeof(uint32_t), hipMemcpyHostToDevice, stream);
    if (err == hipSuccess) err = hipEventRecord(e.ready, stream);
    if (err != hipSuccess) {
        (void)hipEventDestroy(e.ready);
        return hip_fail(err, "mg tables upload");
    }
    e.dev = reinterpret_cast<const uint32_t *>(dd);
    M.block_used += bytes;
    M.bytes += bytes;
    M.map.emplace(key, e);
    out = e.dev;
    return MEC_OK;
}

void mg_release(mec_ctx *c) {
    MgCache &M = c->mg;
    for (auto &kv : M.map)
        if (kv.second.ready) {
            (void)hipEventSynchronize(kv.second.ready);
            (void)hipEventDestroy(kv.second.ready);
        }
    M.map.clear();
    for (uint8_t *d : M.dev_blocks) (void)hipFree(d);
    for (uint8_t *h : M.host_blocks) (void)hipHostFree(h);
    M.dev_blocks.clear();
    M.host_blocks.clear();
}

int mg_prepare(mec_ctx *c, const Mat &coef, size_t nd, size_t ns, Gf8MgLaunch &L, hipStream_t stream) {
    bool vand = true;  // row 0 and column 0 all ones (Jerasure / ISA-L RS parity rows)
    for (size_t j = 0; j < ns && vand; ++j) vand = coef[j] == 1;
    for (size_t r = 0; r < nd && vand; ++r) vand = coef[r * ns] == 1;
    L.vand = vand;
    L.group_rows = mec::detail::mg_group_rows(int(nd), int(ns), vand);
    return mg_tables(c, coef, nd, ns, L.group_rows, stream, L.tabs);
}

bool mg_wanted(const mec_ctx *c, size_t nd) {
    return c->byte_wise() && nd > size_t(mec::kMaxRows) && c->cs % 16 == 0 &&
           mec::detail::knob(mec::detail::kKnobWide) != 0;
}

// outputs (^)= coef (nd x ns over GF(2^w)) * sources, every stripe.
int apply(mec_ctx *c, const Layout &lay, const Mat &coef, uint32_t n_stripes, bool accumulate, hipStream_t stream) {
    const size_t ns = lay.ns, nd = lay.nd;
    if (nd == 0 || n_stripes == 0) return MEC_OK;
    if (ns == 0) {  // all-zero input: outputs are zero (or unchanged when accumulating)
        if (accumulate) return MEC_OK;
        for (uint32_t s = 0; s < n_stripes; ++s)
            for (size_t r = 0; r < nd; ++r)
                HIP_TRY(hipMemsetAsync(lay.dst + int64_t(s) * lay.dss + lay.dst_off[r], 0, c->cs, stream));
        return MEC_OK;
    }
    const bool probe = c->probe.load(std::memory_order_relaxed) == MEC_PROBE_XOR;
    if (mg_wanted(c, nd) && jit_wanted(c, nd, ns, coef, false)) {
        // more than 4 outputs: the matrix's own bit-sliced kernel once built
        // (its arithmetic-free twin under MEC_PROBE_XOR); MEC_WIDE=0 turns
        // every one-pass form off, as on the pointer-batch path (run_gather)
        if (JitKernel *jk = jit_kernel(c, coef, nd, ns, accumulate, false, probe)) {
            mec::BsLaunch L{};
            L.src = lay.src;
            L.dst = lay.dst;
            L.src_stripe_stride = lay.sss;
            L.dst_stripe_stride = lay.dss;
            L.k = int(ns);
            L.rows = int(nd);
            L.len = c->cs;
            L.n_stripes = n_stripes;
            L.vand = coef_vand(coef, nd, ns);
            for (size_t j = 0; j < ns; ++j) L.src_off[j] = lay.src_off[j];
            for (size_t r = 0; r < nd; ++r) L.dst_off[r] = lay.dst_off[r];
            return jit_launch(c, jk, L, stream);
        }
    }
    if (mg_wanted(c, nd) && !probe) {
        // more than 4 outputs: one pass over the sources (gf8_mg_kernel)
        mec::Gf8MgLaunch L{};
        L.src = lay.src;
        L.dst = lay.dst;
        L.src_stripe_stride = lay.sss;
        L.dst_stripe_stride = lay.dss;
        L.k = int(ns);
        L.rows = int(nd);
        L.len = c->cs;
        L.n_stripes = n_stripes;
        L.accumulate = accumulate;
        for (size_t j = 0; j < ns; ++j) L.src_off[j] = lay.src_off[j];
        for (size_t r = 0; r < nd; ++r) L.dst_off[r] = lay.dst_off[r];
        const int rc = mg_prepare(c, coef, nd, ns, L, stream);
        if (rc == MEC_OK) {
            HIP_TRY(mec::launch_gf8_mg(L, stream));
            return MEC_OK;
        }
        if (rc != kMgUncached) return rc;
        // past the table cache's cap: groups of 4 rows below
    }
    const size_t step = c->byte_wise() ? size_t(mec::kMaxRows) : size_t(mec::kMaxBmOut);
    for (size_t r0 = 0; r0 < nd; r0 += step) {
        const int rows = int(std::min<size_t>(step, nd - r0));
        if (c->byte_wise()) {
            mec::Gf8Launch L{};
            L.src = lay.src;
            L.dst = lay.dst;
            L.src_stripe_stride = lay.sss;
            L.dst_stripe_stride = lay.dss;
            L.k = int(ns);
            L.rows = rows;
            L.len = c->cs;
            L.n_stripes = n_stripes;
            L.accumulate = accumulate;
            L.probe = probe;
            for (size_t j = 0; j < ns; ++j) L.src_off[j] = lay.src_off[j];
            for (int i = 0; i < rows; ++i) L.dst_off[i] = lay.dst_off[r0 + i];
            for (int i = 0; i < rows; ++i)
                for (size_t j = 0; j < ns; ++j) L.coef[i][j] = mec::gf8_coef(coef[(r0 + i) * ns + j]);
            HIP_TRY(mec::launch_gf8(L, stream));
        } else {
            const Field &f = Field::get(int(c->w));
            mec::BmLaunch L{};
            L.src = lay.src;
            L.dst = lay.dst;
            L.src_stripe_stride = lay.sss;
            L.dst_stripe_stride = lay.dss;
            L.k = int(ns);
            L.rows = rows;
            L.w = int(c->w);
            L.packet = c->packet;
            L.n_stripes = n_stripes;
            L.accumulate = accumulate;
            for (size_t j = 0; j < ns; ++j) L.src_off[j] = lay.src_off[j];
            for (int i = 0; i < rows; ++i) L.dst_off[i] = lay.dst_off[r0 + i];
            for (int i = 0; i < rows; ++i)
                for (size_t j = 0; j < ns; ++j)
                    bit_block(f, coef[(r0 + i) * ns + j], c->w, &L.mask[j][i * c->w], 1);
            HIP_TRY(mec::launch_bm(L, stream));
        }
    }
    return MEC_OK;
}

int apply(mec_ctx *c, const uint8_t *src, int64_t sss, const std::vector<int64_t> &src_off, uint8_t *dst,
          int64_t dss, const std::vector<int64_t> &dst_off, const Mat &coef, uint32_t n_stripes, bool accumulate,
          hipStream_t stream) {
    return apply(c, Layout::strided(src, sss, src_off, dst, dss, dst_off), coef, n_stripes, accumulate, stream);
}

// Plan index slot of a present mask (keys stored as mask + 1: 0 = empty).
size_t plan_slot(uint64_t key) { return size_t((key * 0x9E3779B97F4A7C15ull) >> 52) & (mec_ctx::kPlanSlots - 1); }

const mec::LinearPlan *plan_lookup(const mec_ctx *c, uint64_t present) {
    const uint64_t key = present + 1;
    for (size_t i = plan_slot(key), n = 0; n < 64; ++n, i = (i + 1) & (mec_ctx::kPlanSlots - 1)) {
        const uint64_t k = c->plan_keys[i].load(std::memory_order_acquire);
        if (k == key) return c->plan_vals[i].load(std::memory_order_acquire);
        if (k == 0) return nullptr;
    }
    return nullptr;
}

// Cached decode plan: the per-call lookup reads the lock-free index (16
// server workers decoding at ~1 M calls/s contended on a mutex here);
// building and inserting a new pattern's plan takes plan_mu.
int get_plan(mec_ctx *c, uint64_t present, const mec::LinearPlan *&out) {
    const uint64_t full = (uint64_t(1) << (c->k + c->m)) - 1;
    present &= full;
    if ((out = plan_lookup(c, present))) return MEC_OK;
    {
        std::lock_guard<std::mutex> g(c->plan_mu);
        auto it = c->plans.find(present);
        if (it != c->plans.end()) {
            out = it->second.get();
            return MEC_OK;
        }
    }
    auto plan = std::make_shared<mec::LinearPlan>();
    std::string err;
    int rc = mec::plan_decode(c->scheme(), c->A, int(c->k), int(c->m), int(c->w), present, *plan, err);
    if (rc != MEC_OK) return fail(rc, "decode: %s", err.c_str());
    std::lock_guard<std::mutex> g(c->plan_mu);
    auto ins = c->plans.emplace(present, plan);
    out = ins.first->second.get();
    if (ins.second) {  // publish in the index: value first, then the key (release)
        const uint64_t key = present + 1;
        for (size_t i = plan_slot(key), n = 0; n < 64; ++n, i = (i + 1) & (mec_ctx::kPlanSlots - 1)) {
            const uint64_t k = c->plan_keys[i].load(std::memory_order_relaxed);
            if (k == key) break;
            if (k == 0) {
                c->plan_vals[i].store(out, std::memory_order_relaxed);
                c->plan_keys[i].store(key, std::memory_order_release);
                break;
            }
        }
    }
    return MEC_OK;
}

Mat encode_rows(const mec_ctx *c, const std::vector<uint32_t> &rows, const std::vector<uint32_t> &cols) {
    Mat m(rows.size() * cols.size());
    for (size_t r = 0; r < rows.size(); ++r)
        for (size_t j = 0; j < cols.size(); ++j) m[r * cols.size() + j] = c->coef(rows[r], cols[j]);
    return m;
}

std::vector<uint32_t> mask_rows(const mec_ctx *c, uint32_t parity_mask) {
    std::vector<uint32_t> rows;
    if (parity_mask == 0) parity_mask = (c->m >= 32) ? 0xffffffffu : ((1u << c->m) - 1);
    for (uint32_t i = 0; i < c->m; ++i)
        if (parity_mask >> i & 1) rows.push_back(i);
    return rows;
}

Lane *lane_acquire(mec_ctx *c, int &rc) {
    {
        std::lock_guard<std::mutex> g(c->lane_mu);
        if (!c->lanes_free.empty()) {
            Lane *l = c->lanes_free.back();
            c->lanes_free.pop_back();
            return l;
        }
    }
    Lane *l = new Lane;
    l->bytes = size_t(c->k + c->m) * c->cs;
    hipError_t e = hipStreamCreateWithFlags(&l->stream, hipStreamNonBlocking);
    if (e == hipSuccess) e = hipEventCreateWithFlags(&l->done, hipEventDisableTiming | hipEventReleaseToSystem);
    if (e == hipSuccess) e = hipHostMalloc(reinterpret_cast<void **>(&l->host), l->bytes, hipHostMallocMapped);
    if (e == hipSuccess) e = hipHostGetDevicePointer(reinterpret_cast<void **>(&l->hdev), l->host, 0);
    if (e != hipSuccess) {
        rc = hip_fail(e, "staging lane");
        if (l->host) (void)hipHostFree(l->host);
        if (l->done) (void)hipEventDestroy(l->done);
        if (l->stream) (void)hipStreamDestroy(l->stream);
        delete l;
        return nullptr;
    }
    std::lock_guard<std::mutex> g(c->lane_mu);
    c->lanes_all.push_back(l);
    return l;
}

hipError_t lane_sync(Lane *l) {
    static const bool spin = [] {
        const char *e = std::getenv("MEC_SYNC_SPIN");
        return e && e[0] && e[0] != '0';
    }();
    const hipError_t r = hipEventRecord(l->done, l->stream);
    if (r != hipSuccess) return r;
    if (spin) {
        const auto t0 = std::chrono::steady_clock::now();
        while (std::chrono::steady_clock::now() - t0 < std::chrono::microseconds(200)) {
            const hipError_t e = hipEventQuery(l->done);
            if (e != hipErrorNotReady) return e;
        }
    }
    return hipEventSynchronize(l->done);
}

void lane_release(mec_ctx *c, Lane *l) {
    std::lock_guard<std::mutex> g(c->lane_mu);
    c->lanes_free.push_back(l);
}

// Zero-copy single stripe (hostmem.cpp): when every source and output chunk
// lies in a registered host range, one strided launch addresses the chunks
// by their absolute device addresses (offsets from the first output) and
// codes them in place over PCIe.  `taken` = false: not eligible, nothing
// done.  No source (every data chunk is Coding::zeros) writes zero outputs.
int zc_single(mec_ctx *c, const std::vector<const uint8_t *> &srcs, const std::vector<uint8_t *> &outs,
              const Mat &coef, bool accumulate, bool &taken) {
    taken = false;
    if (outs.empty() || !zc_any_registered()) return MEC_OK;
    const size_t cs = c->cs;
    std::vector<uint64_t> a(srcs.size() + outs.size());
    for (size_t t = 0; t < srcs.size(); ++t) a[t] = uint64_t(uintptr_t(srcs[t]));
    for (size_t r = 0; r < outs.size(); ++r) a[srcs.size() + r] = uint64_t(uintptr_t(outs[r]));
    if (!zc_translate(a.data(), a.size(), cs)) return MEC_OK;
    taken = true;
    if (srcs.empty()) {
        if (!accumulate)
            for (uint8_t *o : outs) std::memset(o, 0, cs);
        return MEC_OK;
    }
    {
        int qrc = MEC_OK;
        if (c->hq && queue_try(c, a.data(), srcs.size(), outs.size(), coef, accumulate, qrc, srcs.data())) {
            if (qrc == MEC_OK) count_zc(c);
            return qrc;
        }
    }
    DeviceGuard dg(c->device);
    int rc = MEC_OK;
    LaneHold h{c, lane_acquire(c, rc)};
    if (!h.l) return rc;
    const uint64_t base = a[srcs.size()];
    std::vector<int64_t> so(srcs.size()), dof(outs.size());
    for (size_t t = 0; t < so.size(); ++t) so[t] = int64_t(a[t] - base);
    for (size_t r = 0; r < dof.size(); ++r) dof[r] = int64_t(a[srcs.size() + r] - base);
    uint8_t *b = reinterpret_cast<uint8_t *>(uintptr_t(base));
    rc = apply(c, b, 0, so, b, 0, dof, coef, 1, accumulate, h.l->stream);
    if (rc != MEC_OK) return rc;
    HIP_TRY(lane_sync(h.l));
    count_zc(c);
    return MEC_OK;
}


// Run one staged single-stripe call whose chunks sit in lane l's mapped
// pinned buffer (offsets so / dof): the resident queue kernel
// (mec_set_host_queue) codes them in place when it can take the call,
// otherwise one launch on the lane's stream and a wait.  A queue call that
// never completes leaves its workgroup owning the buffer, so the lane is
// then retired instead of returned to the pool.
int lane_run(mec_ctx *c, LaneHold &h, const std::vector<int64_t> &so, const std::vector<int64_t> &dof,
             const Mat &coef, bool accumulate) {
    Lane *l = h.l;
    if (c->hq) {
        const uint64_t base = uint64_t(uintptr_t(l->hdev));
        std::vector<uint64_t> a(so.size() + dof.size());
        for (size_t t = 0; t < so.size(); ++t) a[t] = base + uint64_t(so[t]);
        for (size_t r = 0; r < dof.size(); ++r) a[so.size() + r] = base + uint64_t(dof[r]);
        std::vector<const uint8_t *> hs(so.size());
        for (size_t t = 0; t < so.size(); ++t) hs[t] = l->host + so[t];
        int qrc = MEC_OK;
        if (queue_try(c, a.data(), so.size(), dof.size(), coef, accumulate, qrc, hs.data())) {
            if (qrc != MEC_OK) h.l = nullptr;
            return qrc;
        }
    }
    int rc = apply(c, l->hdev, 0, so, l->hdev, 0, dof, coef, 1, accumulate, l->stream);
    if (rc != MEC_OK) return rc;
    HIP_TRY(lane_sync(l));
    return MEC_OK;
}


}  // namespace core
}  // namespace mec

using namespace mec::core;

extern "C" {

int mec_abi_version(void) { return MEC_ABI_VERSION; }

const char *mec_last_error(void) { return g_err.c_str(); }

int mec_create(int family, uint32_t k, uint32_t m, uint32_t chunk_size, int device, mec_ctx **out) {
    if (!out) return fail(MEC_EINVAL, "out is null");
    *out = nullptr;
    if (family < MEC_RS_VANDERMONDE || family > MEC_ISAL_CAUCHY) return fail(MEC_EINVAL, "unknown family %d", family);
    if (k < 1 || m < 1 || k + m > MEC_MAX_CHUNKS)
        return fail(MEC_EINVAL, "Only support N up to %u for RS coding (k=%u, m=%u)", MEC_MAX_CHUNKS, k, m);
    if (chunk_size == 0) return fail(MEC_EINVAL, "chunk_size is 0");
    std::unique_ptr<mec_ctx> c(new mec_ctx);
    c->family = family;
    c->k = k;
    c->m = m;
    c->cs = chunk_size;
    c->device = device;
    switch (family) {
        case MEC_RS_VANDERMONDE: {
            int w = mec::rs_getw(k, m, chunk_size);
            if (w != 8)
                return fail(MEC_EINVAL, "chunkSize is not a multiple of %d bytes is of supported", 8);
            c->w = 8;
            if (!mec::jerasure_rs_matrix(int(k), int(m), c->A))
                return fail(MEC_EINVAL, "No coding matrix can be generated with k=%u, m=%u, w=8", k, m);
            break;
        }
        case MEC_CAUCHY_GOOD: {
            int w = mec::cauchy_getw(k, m, chunk_size);
            if (w < 0) return fail(MEC_EINVAL, "Cannot find a suitable w for k=%u,m=%u,chunkSize=%u", k, m, chunk_size);
            if (w > 8) return fail(MEC_EINVAL, "Cauchy w=%d > 8 is not supported", w);
            c->w = uint32_t(w);
            if (!mec::jerasure_cauchy_matrix(int(k), int(m), w, c->A))
                return fail(MEC_EINVAL, "No coding matrix can be generated with k=%u, m=%u, w=%d", k, m, w);
            break;
        }
        case MEC_ISAL_RS:
            c->w = 8;
            c->A = mec::isal_rs_matrix(int(k), int(m));
            break;
        case MEC_ISAL_CAUCHY:
            c->w = 8;
            c->A = mec::isal_cauchy_matrix(int(k), int(m));
            break;
    }
    c->packet = family == MEC_CAUCHY_GOOD ? chunk_size / c->w : chunk_size;
    jit_init(c.get());
    {  // one-pass table cache cap (read here, never on a launch path)
        const char *e = std::getenv("MEC_MG_CACHE_BYTES");
        c->mg.cap = e && *e ? size_t(std::strtoull(e, nullptr, 10)) : (size_t(64) << 20);
    }
    if (device >= 0) {
        int n = 0;
        hipError_t e = hipGetDeviceCount(&n);
        if (e != hipSuccess || device >= n)
            return fail(MEC_ENODEV, "HIP device %d not available (%s)", device,
                        e == hipSuccess ? "count" : hipGetErrorString(e));
        hipDeviceProp_t prop;
        e = hipGetDeviceProperties(&prop, device);
        if (e != hipSuccess) return hip_fail(e, "hipGetDeviceProperties");
        if (std::strncmp(prop.gcnArchName, "gfx950", 6) != 0)
            return fail(MEC_ENODEV, "device %d is %s; libmec is built for gfx950 only", device, prop.gcnArchName);
        c->jit.arch = prop.gcnArchName;  // hiprtc compiles for exactly this target
    }
    *out = c.release();
    return MEC_OK;
}

void mec_destroy(mec_ctx *c) {
    if (!c) return;
    for (mec_ctx *s : c->shards) mec_destroy(s);
    c->shards.clear();
    if (has_device(c)) {
        DeviceGuard g(c->device);
        // the resident kernel returns before anything is freed; a grid still
        // running at the drain cap (a hung job) may yet read a staging lane's
        // sources and write its outputs, so the lanes are leaked with it
        const bool drained = queue_stop(c);
        batch_release(c);
        for (Lane *l : c->lanes_all) {
            if (!drained) break;
            (void)hipStreamSynchronize(l->stream);
            (void)hipHostFree(l->host);
            (void)hipEventDestroy(l->done);
            (void)hipStreamDestroy(l->stream);
            delete l;
        }
        for (int i = 0; i < 2; ++i) {
            if (c->bstream[i]) {
                (void)hipStreamSynchronize(c->bstream[i]);
                (void)hipStreamDestroy(c->bstream[i]);
            }
            if (c->bdev[i]) (void)hipFree(c->bdev[i]);
            if (c->bpin[i]) (void)hipHostFree(c->bpin[i]);
            if (c->bdone[i]) (void)hipEventDestroy(c->bdone[i]);
        }
        jit_release(c);
        mg_release(c);
    }
    delete c;
}

int mec_get_info(const mec_ctx *c, mec_info *out) {
    if (!c || !out) return fail(MEC_EINVAL, "null argument");
    out->family = c->family;
    out->k = c->k;
    out->m = c->m;
    out->w = c->w;
    out->chunk_size = c->cs;
    out->packet_size = c->packet;
    out->device = c->device;
    return MEC_OK;
}

int mec_get_matrix(const mec_ctx *c, int32_t *out, size_t capacity) {
    if (!c || !out) return fail(MEC_EINVAL, "null argument");
    if (capacity < c->A.size()) return fail(MEC_EINVAL, "capacity %zu < %zu", capacity, c->A.size());
    for (size_t i = 0; i < c->A.size(); ++i) out[i] = c->A[i];
    return int(c->A.size());
}

int mec_get_bitmatrix(const mec_ctx *c, int32_t *out, size_t capacity) {
    if (!c || !out) return fail(MEC_EINVAL, "null argument");
    if (c->family != MEC_CAUCHY_GOOD) return fail(MEC_EINVAL, "bitmatrix exists for MEC_CAUCHY_GOOD only");
    const uint32_t w = c->w, cols = c->k * w;
    const size_t n = size_t(c->m) * w * cols;
    if (capacity < n) return fail(MEC_EINVAL, "capacity %zu < %zu", capacity, n);
    const Field &f = Field::get(int(w));
    for (uint32_t i = 0; i < c->m; ++i)
        for (uint32_t j = 0; j < c->k; ++j) {
            unsigned e = c->A[size_t(i) * c->k + j];
            for (uint32_t x = 0; x < w; ++x) {
                for (uint32_t l = 0; l < w; ++l) out[size_t(i * w + l) * cols + j * w + x] = (e >> l) & 1;
                e = f.mul(e, 2 % f.size());
            }
        }
    return int(n);
}

int mec_encode(mec_ctx *c, const uint8_t *data, int64_t dss_, int64_t dcs, uint8_t *parity, int64_t pss, int64_t pcs,
               uint32_t n_stripes, uint32_t parity_mask, void *stream) {
    CHECK_CTX(c);
    if ((!data || !parity) && n_stripes) return fail(MEC_EINVAL, "null buffer");
    DeviceGuard dg(c->device);
    std::vector<uint32_t> rows = mask_rows(c, parity_mask), cols(c->k);
    for (uint32_t j = 0; j < c->k; ++j) cols[j] = j;
    std::vector<int64_t> so(c->k), dof(rows.size());
    for (uint32_t j = 0; j < c->k; ++j) so[j] = int64_t(j) * dcs;
    for (size_t r = 0; r < rows.size(); ++r) dof[r] = int64_t(rows[r]) * pcs;
    return apply(c, data, dss_, so, parity, pss, dof, encode_rows(c, rows, cols), n_stripes, false,
                 hipStream_t(stream));
}

int mec_decode_split(mec_ctx *c, const uint8_t *in, int64_t iss, int64_t ics, uint8_t *out, int64_t oss, int64_t ocs,
                     uint32_t n_stripes, uint64_t present_mask, void *stream) {
    CHECK_CTX(c);
    if ((!in || !out) && n_stripes) return fail(MEC_EINVAL, "null buffer");
    const mec::LinearPlan *plan = nullptr;
    int rc = get_plan(c, present_mask, plan);
    if (rc != MEC_OK) return rc;
    if (plan->dst.empty()) return MEC_OK;
    DeviceGuard dg(c->device);
    std::vector<int64_t> so(plan->src.size()), dof(plan->dst.size());
    for (size_t t = 0; t < so.size(); ++t) so[t] = int64_t(plan->src[t]) * ics;
    for (size_t r = 0; r < dof.size(); ++r) dof[r] = int64_t(plan->dst[r]) * ocs;
    return apply(c, in, iss, so, out, oss, dof, plan->coef, n_stripes, false, hipStream_t(stream));
}

int mec_decode(mec_ctx *c, uint8_t *chunks, int64_t ss, int64_t cs, uint32_t n_stripes, uint64_t present_mask,
               void *stream) {
    return mec_decode_split(c, chunks, ss, cs, chunks, ss, cs, n_stripes, present_mask, stream);
}

int mec_encode_update(mec_ctx *c, uint32_t data_index, const uint8_t *delta, int64_t delta_ss, uint8_t *parity,
                      int64_t pss, int64_t pcs, uint32_t n_stripes, uint32_t parity_mask, void *stream) {
    CHECK_CTX(c);
    if ((!delta || !parity) && n_stripes) return fail(MEC_EINVAL, "null buffer");
    if (data_index >= c->k) return fail(MEC_EINVAL, "data_index %u >= k %u", data_index, c->k);
    DeviceGuard dg(c->device);
    std::vector<uint32_t> rows = mask_rows(c, parity_mask), cols{data_index};
    std::vector<int64_t> so{0}, dof(rows.size());
    for (size_t r = 0; r < rows.size(); ++r) dof[r] = int64_t(rows[r]) * pcs;
    return apply(c, delta, delta_ss, so, parity, pss, dof, encode_rows(c, rows, cols), n_stripes, true,
                 hipStream_t(stream));
}

int mec_xor(uint8_t *dst, const uint8_t *a, const uint8_t *b, uint64_t len, void *stream) {
    if ((!dst || !a || !b) && len) return fail(MEC_EINVAL, "null buffer");
    HIP_TRY(mec::launch_xor(dst, a, b, len, hipStream_t(stream)));
    return MEC_OK;
}

int mec_set_probe(mec_ctx *c, int mode) {
    if (!c) return fail(MEC_EINVAL, "null context");
    if (mode != MEC_PROBE_OFF && mode != MEC_PROBE_XOR) return fail(MEC_EINVAL, "unknown probe mode %d", mode);
    if (mode == MEC_PROBE_XOR && !c->byte_wise())
        return fail(MEC_EINVAL, "the XOR twin exists for byte-wise families only");
    c->probe.store(mode, std::memory_order_relaxed);
    // a multi-device context launches on its shards
    for (mec_ctx *sh : c->shards) sh->probe.store(mode, std::memory_order_relaxed);
    return MEC_OK;
}

int mec_set_knob(const char *name, const char *value) {
    if (!name) return fail(MEC_EINVAL, "null knob name");
    switch (mec::detail::set_knob(name, value)) {
        case mec::detail::KnobStatus::kOk: return MEC_OK;
        case mec::detail::KnobStatus::kUnknown: return fail(MEC_EINVAL, "unknown knob %s", name);
        default: return fail(MEC_EINVAL, "%s=%s is not an accepted value", name, value ? value : "(null)");
    }
}

int mec_fill_random(uint8_t *dst, uint64_t len, uint64_t seed, uint64_t word_offset, void *stream) {
    if (!dst && len) return fail(MEC_EINVAL, "null buffer");
    HIP_TRY(mec::launch_fill(dst, len, seed, word_offset, hipStream_t(stream)));
    return MEC_OK;
}

// ---- host-memory, one stripe ------------------------------------------------

int mec_encode_host(mec_ctx *c, const uint8_t *const *data, uint8_t *const *parity) {
    CHECK_CTX(c);
    if (is_multi(c)) return mec_encode_host(shard_pick(c), data, parity);
    if (!data || !parity) return fail(MEC_EINVAL, "null pointer array");
    std::vector<uint32_t> rows, cols;
    for (uint32_t i = 0; i < c->m; ++i)
        if (parity[i]) rows.push_back(i);
    if (rows.empty()) return MEC_OK;
    for (uint32_t j = 0; j < c->k; ++j)
        if (data[j]) cols.push_back(j);
    // concurrent calls batched into one launch (mec_set_coalescing)
    if (coalescing(c)) return submit_encode(c, data, parity);
    {
        std::vector<const uint8_t *> zs;
        std::vector<uint8_t *> zo;
        for (uint32_t j : cols) zs.push_back(data[j]);
        for (uint32_t i : rows) zo.push_back(parity[i]);
        bool taken;
        int zrc = zc_single(c, zs, zo, encode_rows(c, rows, cols), false, taken);
        if (taken) return zrc;
    }
    count_staged(c);
    DeviceGuard dg(c->device);
    int rc = MEC_OK;
    LaneHold h{c, lane_acquire(c, rc)};
    if (!h.l) return rc;
    const size_t cs = c->cs;
    if (cols.empty()) {  // every data chunk is Coding::zeros
        for (uint32_t i : rows) std::memset(parity[i], 0, cs);
        return MEC_OK;
    }
    std::vector<int64_t> so(cols.size()), dof(rows.size());
    for (size_t t = 0; t < cols.size(); ++t) {
        so[t] = int64_t(cols[t]) * int64_t(cs);
        std::memcpy(h.l->host + so[t], data[cols[t]], cs);
    }
    for (size_t r = 0; r < rows.size(); ++r) dof[r] = int64_t(c->k + rows[r]) * int64_t(cs);
    rc = lane_run(c, h, so, dof, encode_rows(c, rows, cols), false);
    if (rc != MEC_OK) return rc;
    for (size_t r = 0; r < rows.size(); ++r) std::memcpy(parity[rows[r]], h.l->host + dof[r], cs);
    return MEC_OK;
}

int mec_decode_host(mec_ctx *c, uint8_t *const *chunks, uint64_t present_mask) {
    CHECK_CTX(c);
    if (is_multi(c)) return mec_decode_host(shard_pick(c), chunks, present_mask);
    if (!chunks) return fail(MEC_EINVAL, "null pointer array");
    const mec::LinearPlan *plan = nullptr;
    int rc = get_plan(c, present_mask, plan);
    if (rc != MEC_OK) return rc;
    if (plan->dst.empty()) return MEC_OK;
    for (uint32_t i = 0; i < c->k + c->m; ++i)
        if (!chunks[i]) return fail(MEC_EINVAL, "chunk %u pointer is NULL", i);
    if (coalescing(c)) return submit_decode(c, chunks, present_mask);
    {
        std::vector<const uint8_t *> zs;
        std::vector<uint8_t *> zo;
        for (int t : plan->src) zs.push_back(chunks[t]);
        for (int r : plan->dst) zo.push_back(chunks[r]);
        bool taken;
        int zrc = zc_single(c, zs, zo, plan->coef, false, taken);
        if (taken) return zrc;
    }
    count_staged(c);
    DeviceGuard dg(c->device);
    LaneHold h{c, lane_acquire(c, rc)};
    if (!h.l) return rc;
    const size_t cs = c->cs;
    std::vector<int64_t> so(plan->src.size()), dof(plan->dst.size());
    for (size_t t = 0; t < so.size(); ++t) {
        so[t] = int64_t(plan->src[t]) * int64_t(cs);
        std::memcpy(h.l->host + so[t], chunks[plan->src[t]], cs);
    }
    for (size_t r = 0; r < dof.size(); ++r) dof[r] = int64_t(plan->dst[r]) * int64_t(cs);
    rc = lane_run(c, h, so, dof, plan->coef, false);
    if (rc != MEC_OK) return rc;
    for (size_t r = 0; r < dof.size(); ++r) std::memcpy(chunks[plan->dst[r]], h.l->host + dof[r], cs);
    return MEC_OK;
}

int mec_encode_update_host(mec_ctx *c, uint32_t data_index, const uint8_t *delta, uint8_t *const *parity) {
    CHECK_CTX(c);
    if (is_multi(c)) return mec_encode_update_host(shard_pick(c), data_index, delta, parity);
    if (!delta || !parity) return fail(MEC_EINVAL, "null pointer");
    if (data_index >= c->k) return fail(MEC_EINVAL, "data_index %u >= k %u", data_index, c->k);
    std::vector<uint32_t> rows, cols{data_index};
    for (uint32_t i = 0; i < c->m; ++i)
        if (parity[i]) rows.push_back(i);
    if (rows.empty()) return MEC_OK;
    if (coalescing(c)) return submit_update(c, data_index, delta, parity);
    {
        std::vector<uint8_t *> zo;
        for (uint32_t i : rows) zo.push_back(parity[i]);
        bool taken;
        int zrc = zc_single(c, {delta}, zo, encode_rows(c, rows, cols), true, taken);
        if (taken) return zrc;
    }
    count_staged(c);
    DeviceGuard dg(c->device);
    int rc = MEC_OK;
    LaneHold h{c, lane_acquire(c, rc)};
    if (!h.l) return rc;
    const size_t cs = c->cs;
    std::vector<int64_t> so{0}, dof(rows.size());
    std::memcpy(h.l->host, delta, cs);
    for (size_t r = 0; r < rows.size(); ++r) {
        dof[r] = int64_t(1 + r) * int64_t(cs);
        std::memcpy(h.l->host + dof[r], parity[rows[r]], cs);
    }
    rc = lane_run(c, h, so, dof, encode_rows(c, rows, cols), true);
    if (rc != MEC_OK) return rc;
    for (size_t r = 0; r < rows.size(); ++r) std::memcpy(parity[rows[r]], h.l->host + dof[r], cs);
    return MEC_OK;
}

int mec_encode_host_batch(mec_ctx *c, const uint8_t *data, uint8_t *parity, uint32_t n_stripes,
                          uint32_t parity_mask) {
    CHECK_CTX(c);
    if ((!data || !parity) && n_stripes) return fail(MEC_EINVAL, "null buffer");
    if (!n_stripes) return MEC_OK;
    if (is_multi(c)) {
        const size_t dbytes = size_t(c->k) * c->cs, pbytes = size_t(c->m) * c->cs;
        return shard_run(c, n_stripes, [&](mec_ctx *sc, uint32_t s0, uint32_t s1) {
            return mec_encode_host_batch(sc, data + s0 * dbytes, parity + s0 * pbytes, s1 - s0, parity_mask);
        });
    }
    DeviceGuard dg(c->device);
    std::lock_guard<std::mutex> bg(c->batch_mu);
    const size_t cs = c->cs, dbytes = size_t(c->k) * cs, pbytes = size_t(c->m) * cs;
    const size_t per = dbytes + pbytes;
    for (int i = 0; i < 2; ++i)
        if (!c->bstream[i]) HIP_TRY(hipStreamCreateWithFlags(&c->bstream[i], hipStreamNonBlocking));
    uint64_t zd, zp;
    if (n_stripes && zc_device_address(data, size_t(n_stripes) * dbytes, zd) &&
        zc_device_address(parity, size_t(n_stripes) * pbytes, zp)) {
        // zero-copy: one strided launch over the registered host buffers
        std::vector<uint32_t> rows = mask_rows(c, parity_mask), cols(c->k);
        for (uint32_t j = 0; j < c->k; ++j) cols[j] = j;
        std::vector<int64_t> so(c->k), dof(rows.size());
        for (uint32_t j = 0; j < c->k; ++j) so[j] = int64_t(j) * int64_t(cs);
        for (size_t r = 0; r < rows.size(); ++r) dof[r] = int64_t(rows[r]) * int64_t(cs);
        int rc = MEC_OK;
        LaneHold h{c, lane_acquire(c, rc)};
        if (!h.l) return rc;
        rc = apply(c, reinterpret_cast<const uint8_t *>(uintptr_t(zd)), int64_t(dbytes), so,
                   reinterpret_cast<uint8_t *>(uintptr_t(zp)), int64_t(pbytes), dof, encode_rows(c, rows, cols),
                   n_stripes, false, h.l->stream);
        const hipError_t e = lane_sync(h.l);  // no launch may outlive the call (the caller owns the buffers)
        if (rc != MEC_OK) return rc;
        HIP_TRY(e);
        count_zc(c);
        return MEC_OK;
    }
    count_staged(c);
    // Staged: the caller's pageable bytes are copied by the host (a few
    // threads) into library-owned pinned buffers, DMA'd to HBM, coded there,
    // and the parity comes back the same way; two sub-batches in flight.  No
    // DMA ever reads or writes the caller's pageable memory (the runtime
    // would pin it on the fly; round 6 saw such a copy fault).
    const uint32_t sub = uint32_t(std::max<size_t>(1, std::min<size_t>(n_stripes, (size_t(256) << 20) / per)));
    const size_t need = size_t(sub) * per;
    if (c->bbytes < need) {
        for (int i = 0; i < 2; ++i) {
            if (c->bstream[i]) (void)hipStreamSynchronize(c->bstream[i]);
            if (c->bdev[i]) (void)hipFree(c->bdev[i]);
            if (c->bpin[i]) (void)hipHostFree(c->bpin[i]);
            c->bdev[i] = c->bpin[i] = nullptr;
        }
        c->bbytes = 0;
        for (int i = 0; i < 2; ++i) {
            HIP_TRY(hipMalloc(&c->bdev[i], need));
            HIP_TRY(hipHostMalloc(reinterpret_cast<void **>(&c->bpin[i]), need, hipHostMallocDefault));
        }
        c->bbytes = need;
    }
    for (int i = 0; i < 2; ++i)
        if (!c->bdone[i]) HIP_TRY(hipEventCreateWithFlags(&c->bdone[i], hipEventDisableTiming | hipEventReleaseToSystem));
    std::vector<uint32_t> rows = mask_rows(c, parity_mask), cols(c->k);
    for (uint32_t j = 0; j < c->k; ++j) cols[j] = j;
    const Mat coef = encode_rows(c, rows, cols);
    std::vector<int64_t> so(c->k), dof(rows.size());
    for (uint32_t j = 0; j < c->k; ++j) so[j] = int64_t(j) * int64_t(cs);
    for (size_t r = 0; r < rows.size(); ++r) dof[r] = int64_t(rows[r]) * int64_t(cs);
    // on any failure both streams are drained before returning, so no copy
    // queued here still writes into a buffer afterwards
    auto drain = [&](int rc) {
        (void)hipStreamSynchronize(c->bstream[0]);
        (void)hipStreamSynchronize(c->bstream[1]);
        return rc;
    };
    // sub-batch i uses buffers b = i & 1: data [ns][k][cs] then parity [ns][m][cs]
    auto enqueue = [&](uint32_t s0, uint32_t ns, int b) -> int {
        uint8_t *hp = c->bpin[b], *dd = c->bdev[b];
        par_memcpy(hp, data + size_t(s0) * dbytes, size_t(ns) * dbytes);
        hipError_t e = hipMemcpyAsync(dd, hp, size_t(ns) * dbytes, hipMemcpyHostToDevice, c->bstream[b]);
        if (e != hipSuccess) return hip_fail(e, "hipMemcpyAsync H2D");
        uint8_t *dp = dd + size_t(sub) * dbytes;
        const int rc = apply(c, dd, int64_t(dbytes), so, dp, int64_t(pbytes), dof, coef, ns, false, c->bstream[b]);
        if (rc != MEC_OK) return rc;
        e = hipMemcpyAsync(hp + size_t(sub) * dbytes, dp, size_t(ns) * pbytes, hipMemcpyDeviceToHost, c->bstream[b]);
        if (e == hipSuccess) e = hipEventRecord(c->bdone[b], c->bstream[b]);
        return e == hipSuccess ? MEC_OK : hip_fail(e, "hipMemcpyAsync D2H");
    };
    auto finish = [&](uint32_t s0, uint32_t ns, int b) -> int {
        HIP_TRY(hipEventSynchronize(c->bdone[b]));
        par_memcpy(parity + size_t(s0) * pbytes, c->bpin[b] + size_t(sub) * dbytes, size_t(ns) * pbytes);
        return MEC_OK;
    };
    std::vector<std::pair<uint32_t, uint32_t>> items;
    for (uint32_t s0 = 0; s0 < n_stripes; s0 += sub) items.emplace_back(s0, std::min(sub, n_stripes - s0));
    for (size_t i = 0; i < items.size(); ++i) {
        const int b = int(i & 1);
        if (i >= 2) {
            const int rc = finish(items[i - 2].first, items[i - 2].second, b);
            if (rc != MEC_OK) return drain(rc);
        }
        const int rc = enqueue(items[i].first, items[i].second, b);
        if (rc != MEC_OK) return drain(rc);
    }
    for (size_t i = items.size() >= 2 ? items.size() - 2 : 0; i < items.size(); ++i) {
        const int rc = finish(items[i].first, items[i].second, int(i & 1));
        if (rc != MEC_OK) return drain(rc);
    }
    return MEC_OK;
}

}  // extern "C"
