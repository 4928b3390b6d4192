// batch.cpp — libmec pointer-array batches (mec_encode_batch,
// mec_decode_batch, mec_encode_update_batch), the host-memory pipeline
// behind them, and the request coalescer for the single-stripe host entry
// points.
//
// MemEC's chunks do not sit in one strided array: a stripe's k + m chunks
// are separate `Chunk*` (ChunkPool slots, chunk_pool.cc:22-95, or temp
// chunks, chunk_pool.hh:38-53), and every stripe of a reconstruction batch
// can have its own erasure pattern (recovery_worker.cc:210-296).  A batch
// is therefore a list of per-stripe chunk pointers.  Stripes are grouped by
// their linear map — (present data columns, wanted parities) for encode,
// the present mask for decode, (data column, wanted parities) for delta
// updates — and each group becomes one gather launch that reads its chunk
// addresses from a device table (one row of pointers per stripe, scalar
// loads, uniform per block).  Decode plans are cached per pattern, so a
// batch of mixed erasures costs one host-side plan per distinct pattern
// (the reference rebuilds matrices per call, jerasure.c:223, 958).
#include <emmintrin.h>
#include <unistd.h>

#include <atomic>
#include <condition_variable>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <thread>

#include "ctx.hpp"
#include "knobs.hpp"

namespace mec {
namespace core {

// Stripes sharing one linear map: outputs (^)= coef * sources.
struct Group {
    Mat coef;
    uint32_t ns = 0, nd = 0;
    bool accumulate = false;
    uint32_t n = 0;
    std::vector<uint64_t> ptrs;  // n rows of [ns sources | nd outputs]
    std::vector<int32_t> owner;  // per stripe: index of the request / stripe it came from
    const LinearPlan *plan = nullptr;  // decode groups: survivor / output chunk indices (owned by the context)
    std::vector<uint32_t> cols, rows;  // encode / update groups: source columns, output rows
};

struct GroupSet {
    std::unordered_map<uint64_t, size_t> index;
    std::vector<Group> groups;
    Group &get(uint64_t sig, bool &fresh) {
        auto it = index.find(sig);
        fresh = it == index.end();
        if (!fresh) return groups[it->second];
        index.emplace(sig, groups.size());
        groups.emplace_back();
        return groups.back();
    }
};

inline uint32_t full_mask32(uint32_t n) { return n >= 32 ? 0xffffffffu : ((1u << n) - 1); }

std::vector<uint32_t> bits_of(uint64_t mask, uint32_t n) {
    std::vector<uint32_t> v;
    for (uint32_t i = 0; i < n; ++i)
        if (mask >> i & 1) v.push_back(i);
    return v;
}

// encode: data[j] == NULL is the Coding::zeros sentinel (skipped),
// parity[i] == NULL or outside pmask is not wanted.
void add_encode(mec_ctx *c, GroupSet &G, const uint8_t *const *data, uint8_t *const *parity, uint32_t pmask,
                int32_t owner) {
    uint32_t sm = 0, dm = 0;
    for (uint32_t j = 0; j < c->k; ++j)
        if (data[j]) sm |= 1u << j;
    for (uint32_t i = 0; i < c->m; ++i)
        if (parity[i] && (pmask >> i & 1)) dm |= 1u << i;
    if (!dm) return;
    bool fresh;
    Group &g = G.get(uint64_t(sm) | uint64_t(dm) << 32, fresh);
    if (fresh) {
        g.cols = bits_of(sm, c->k);
        g.rows = bits_of(dm, c->m);
        g.coef = encode_rows(c, g.rows, g.cols);
        g.ns = uint32_t(g.cols.size());
        g.nd = uint32_t(g.rows.size());
    }
    for (uint32_t j : g.cols) g.ptrs.push_back(uint64_t(uintptr_t(data[j])));
    for (uint32_t i : g.rows) g.ptrs.push_back(uint64_t(uintptr_t(parity[i])));
    g.owner.push_back(owner);
    ++g.n;
}

// delta update: parity[i] ^= A[i][j] * delta for wanted parities.
void add_update(mec_ctx *c, GroupSet &G, uint32_t j, const uint8_t *delta, uint8_t *const *parity, uint32_t pmask,
                int32_t owner) {
    uint32_t dm = 0;
    for (uint32_t i = 0; i < c->m; ++i)
        if (parity[i] && (pmask >> i & 1)) dm |= 1u << i;
    if (!dm) return;
    bool fresh;
    Group &g = G.get(uint64_t(j) | uint64_t(dm) << 8, fresh);
    if (fresh) {
        g.rows = bits_of(dm, c->m);
        g.coef = encode_rows(c, g.rows, {j});
        g.ns = 1;
        g.nd = uint32_t(g.rows.size());
        g.accumulate = true;
    }
    g.ptrs.push_back(uint64_t(uintptr_t(delta)));
    for (uint32_t i : g.rows) g.ptrs.push_back(uint64_t(uintptr_t(parity[i])));
    g.owner.push_back(owner);
    ++g.n;
}

// decode: MEC_OK (queued or nothing to do), MEC_ETOOMANY, or a plan error.
int add_decode(mec_ctx *c, GroupSet &G, uint8_t *const *chunks, uint64_t present, int32_t owner) {
    const uint32_t n = c->k + c->m;
    const uint64_t full = (uint64_t(1) << n) - 1;
    present &= full;
    const uint32_t failed = uint32_t(__builtin_popcountll(~present & full));
    if (failed > c->m) return fail(MEC_ETOOMANY, "Too many failure to recover (%u>%u)", failed, c->m);
    if (failed == 0) return MEC_OK;
    for (uint32_t i = 0; i < n; ++i)
        if (!chunks[i]) return fail(MEC_EINVAL, "chunk %u pointer is NULL", i);
    auto it = G.index.find(present);
    if (it == G.index.end()) {
        const LinearPlan *plan = nullptr;
        int rc = get_plan(c, present, plan);
        if (rc != MEC_OK) return rc;
        bool fresh;
        Group &g = G.get(present, fresh);
        g.plan = plan;
        g.coef = plan->coef;
        g.ns = uint32_t(plan->src.size());
        g.nd = uint32_t(plan->dst.size());
        it = G.index.find(present);
    }
    Group &g = G.groups[it->second];
    for (int t : g.plan->src) g.ptrs.push_back(uint64_t(uintptr_t(chunks[t])));
    for (int r : g.plan->dst) g.ptrs.push_back(uint64_t(uintptr_t(chunks[r])));
    g.owner.push_back(owner);
    ++g.n;
    return MEC_OK;
}

// ---------------------------------------------------------------------------
// device-resident execution: the caller's pointer rows are uploaded as they
// are, every stripe carries a descriptor index, and each group of <= 4
// output rows is ONE gathered launch whatever the mix of patterns
// ---------------------------------------------------------------------------

// The linear maps of a device batch: map p reads sources ssel[p] (entries of
// the stripe's source row) and writes outputs dsel[p] with coef[p]
// (dsel.size() x K over GF(2^w)).
struct MapSet {
    uint32_t K = 0;
    bool accumulate = false;
    std::vector<std::vector<uint8_t>> ssel, dsel;
    std::vector<Mat> coef;
    size_t rows() const {
        size_t r = 0;
        for (const auto &d : dsel) r = std::max(r, d.size());
        return r;
    }
    uint32_t add(std::vector<uint8_t> s, std::vector<uint8_t> d, Mat c) {
        ssel.push_back(std::move(s));
        dsel.push_back(std::move(d));
        coef.push_back(std::move(c));
        return uint32_t(ssel.size() - 1);
    }
};

// Descriptor blobs [row group][map] (layout in kernels.hpp).
// Rows per descriptor group: 4 byte-wise (the gf8 kernels' R; more groups
// run in the same launch), 8 bitmatrix (a launch keeps 8 x w packet slices).
size_t group_rows(const mec_ctx *c) { return c->byte_wise() ? size_t(kMaxRows) : size_t(kBmGatherRows); }

size_t build_descs(const mec_ctx *c, const MapSet &M, std::vector<uint32_t> &out, uint32_t &desc_dw) {
    const size_t GR = group_rows(c);
    const size_t groups = (M.rows() + GR - 1) / GR, nm = M.ssel.size();
    const uint32_t K = M.K;
    desc_dw = c->byte_wise() ? uint32_t(kGf8DescHead + kMaxRows * K * 8) : uint32_t(kBmDescHead + kMaxSrc * 2 * c->w);
    out.assign(groups * nm * desc_dw, 0);
    auto put_byte = [](uint32_t *w, size_t idx, uint8_t v) { w[idx / 4] |= uint32_t(v) << (8 * (idx % 4)); };
    for (size_t g = 0; g < groups; ++g)
        for (size_t q = 0; q < nm; ++q) {
            uint32_t *D = out.data() + (g * nm + q) * desc_dw;
            const size_t nd = M.dsel[q].size();
            const uint32_t sel_dw = c->byte_wise() ? 8 : 0, dsel_dw = c->byte_wise() ? 16 : 8;
            for (uint32_t j = 0; j < K; ++j) put_byte(D + sel_dw, j, M.ssel[q][j]);
            for (size_t i = 0; i < GR; ++i) {
                const size_t r = g * GR + i;
                put_byte(D + dsel_dw, i, r < nd ? M.dsel[q][r] : kNoRow);
            }
            if (c->byte_wise()) {
                for (int i = 0; i < kMaxRows; ++i) {
                    const size_t r = g * kMaxRows + i;
                    for (uint32_t j = 0; j < K; ++j) {
                        const uint8_t e = r < nd ? M.coef[q][r * K + j] : 0;
                        const uint32_t b = uint32_t(i) * K + j;
                        const Gf8Coef cf = gf8_coef(e);
                        uint32_t *t = D + kGf8DescHead + b * 8;
                        t[0] = cf.t0;
                        t[1] = cf.t1;
                        t[2] = cf.u0;
                        t[3] = cf.u1;
                        t[4] = cf.v;
                        if (e == 0) D[4 + b / 32] |= 1u << (b % 32);
                        if (e == 1) D[b / 32] |= 1u << (b % 32);
                    }
                }
            } else {
                const Field &f = Field::get(int(c->w));
                for (size_t i = 0; i < GR; ++i) {
                    const size_t r = g * GR + i;
                    if (r >= nd) continue;
                    for (uint32_t j = 0; j < K; ++j) {
                        uint8_t mask[8];
                        bit_block(f, M.coef[q][r * K + j], c->w, mask, 1);
                        for (uint32_t l = 0; l < c->w; ++l)
                            put_byte(D + kBmDescHead + j * 2 * c->w, i * c->w + l, mask[l]);
                    }
                }
            }
        }
    return groups;
}

// Pinned + device staging of one call's tables, reused round-robin.  With
// `mapped` the kernels read the tables in place from the pinned buffer (no
// copy; small zero-copy batches, where the copy would be most of the call)
// and `base` is its device address; otherwise `base` is the HBM copy, made
// on the context's own copy stream and waited for by `st` through an event,
// so the copy of one call's tables overlaps the launches of the call before
// (on `st` the copy sat between them: RS(16,8)@4 KiB, 131072 stripes,
// 25 MB of rows, 0.45 ms of copy after each 2.1 ms launch, 63 % of 8 TB/s
// per call against 76.5 for the kernel, profiles/r05/vrow/prof4k/).  A slot
// is reused only after its previous launches finished (`done`).
void table_memcpy(void *dst, const void *src, size_t n);

int table_upload(mec_ctx *c, const std::vector<std::pair<const void *, size_t>> &parts, TableSlot *&slot,
                 std::vector<size_t> &offs, hipStream_t st, bool mapped, uint8_t *&base,
                 const std::function<int(TableSlot &, uint8_t *, hipStream_t)> &after_copy = nullptr) {
    size_t total = 0;
    offs.clear();
    for (const auto &pr : parts) {
        offs.push_back(total);
        total += (pr.second + 255) & ~size_t(255);
    }
    uint32_t idx;
    hipStream_t cs = nullptr;
    {
        std::lock_guard<std::mutex> lk(c->tab_mu);
        idx = c->tab_next++ % kTableSlots;
        if (!mapped && !c->tab_stream) HIP_TRY(hipStreamCreateWithFlags(&c->tab_stream, hipStreamNonBlocking));
        cs = c->tab_stream;
    }
    TableSlot &t = c->tabs[idx];
    t.mu.lock();
    slot = &t;
    if (t.pending) {
        HIP_TRY(hipEventSynchronize(t.done));
        t.pending = false;
    }
    if (!t.done) HIP_TRY(hipEventCreateWithFlags(&t.done, hipEventDisableTiming));
    if (!t.copied) HIP_TRY(hipEventCreateWithFlags(&t.copied, hipEventDisableTiming));
    if (t.cap < total) {
        if (t.host) (void)hipHostFree(t.host);
        if (t.dev) (void)hipFree(t.dev);
        t.host = t.hdev = nullptr;
        t.dev = nullptr;
        t.cap = 0;
        const size_t cap = std::max<size_t>(total, size_t(1) << 20);
        HIP_TRY(hipHostMalloc(reinterpret_cast<void **>(&t.host), cap, hipHostMallocMapped));
        HIP_TRY(hipHostGetDevicePointer(reinterpret_cast<void **>(&t.hdev), t.host, 0));
        HIP_TRY(hipMalloc(reinterpret_cast<void **>(&t.dev), cap));
        t.cap = cap;
    }
    uint8_t *h = reinterpret_cast<uint8_t *>(t.host);
    for (size_t i = 0; i < parts.size(); ++i)
        if (parts[i].second) table_memcpy(h + offs[i], parts[i].first, parts[i].second);
    if (mapped) {
        base = reinterpret_cast<uint8_t *>(t.hdev);
        return MEC_OK;
    }
    HIP_TRY(hipMemcpyAsync(t.dev, t.host, total, hipMemcpyHostToDevice, cs));
    if (after_copy) {  // device-side work on the copied tables, on the copy stream too
        const int rc = after_copy(t, reinterpret_cast<uint8_t *>(t.dev), cs);
        if (rc != MEC_OK) return rc;
    }
    HIP_TRY(hipEventRecord(t.copied, cs));
    // While st still runs earlier launches, wait for the copy on the host —
    // it overlaps those launches — so this call's launch queues behind them
    // with no cross-stream dependency: a device-side wait on the copy's
    // event cost 10-11 us between back-to-back launches even when the copy
    // had finished long before (rocprofv3 kernel + copy traces,
    // profiles/r06/batch/profcopy_*), 2.5 % of an RS(8,2)@4 KiB x 65536
    // batch; interleaved A/B (profiles/r06/batch/tabwait_r06e.jsonl): that
    // batch 79.9-80.6 -> 80.9-81.5 % of 8 TB/s, its 32-bit offset form
    // 79.9-80.4 -> 81.1-81.7, RS(10,4)@1 MiB unchanged.  An idle stream
    // keeps the device-side wait (no host block for a lone call).
    // MEC_TAB_WAIT=0 forces the device-side wait.
    if (detail::knob(detail::kKnobTabWait) != 0 && hipStreamQuery(st) == hipErrorNotReady) {
        HIP_TRY(hipEventSynchronize(t.copied));
    } else {
        (void)hipGetLastError();  // a hipStreamQuery "not ready" leaves no error behind
        HIP_TRY(hipStreamWaitEvent(st, t.copied, 0));
    }
    base = reinterpret_cast<uint8_t *>(t.dev);
    return MEC_OK;
}

struct SlotHold {
    TableSlot *t = nullptr;
    hipStream_t st = nullptr;
    ~SlotHold() {
        if (!t) return;
        // recorded even after a failed launch so the slot is never reused early
        if (hipEventRecord(t->done, st) == hipSuccess) t->pending = true;
        t->mu.unlock();
    }
};

// stab / dtab: host arrays of n rows of device chunk pointers; pat: per-stripe
// map index (nullptr = map 0).
// 1 if the chunk pointers of the first stripes (a sample: the shape only
// steers the launch, never the result) are all 128-byte (cache-line)
// aligned, else 2.  16-byte alignment is not enough: chunks at 16 or 64 mod
// 128 run 6-14 % faster with the 4-wave shape (tools/gather_ab.py,
// profiles/r02/host/gather_ab_hdr.log; tools/align_probe.hip).
uint8_t gather_shape(const void *tab, uint32_t stride, uint32_t n) {
    const uint64_t *t = static_cast<const uint64_t *>(tab);
    uint64_t bits = 0;
    const size_t cnt = size_t(std::min<uint32_t>(n, 64)) * stride;
    for (size_t i = 0; i < cnt; ++i) bits |= t[i];
    return (bits & 127) ? 2 : 1;
}

// 32-bit slab offset rows (mec_*_batch32): entry = base + (off << shift),
// kNullOff = NULL.  The rows cross PCIe at half the size of pointer rows and
// are expanded to pointers on the device (launch_expand_rows), so every
// gathered kernel reads the same pointer table as for mec_*_batch.
struct Off32 {
    uint64_t base;
    uint32_t shift;
};
constexpr uint32_t kMaxOffShift = 12;

uint8_t gather_shape32(const uint32_t *tab, uint32_t stride, uint32_t n, const Off32 &o) {
    uint64_t bits = 0;
    const size_t cnt = size_t(std::min<uint32_t>(n, 64)) * stride;
    for (size_t i = 0; i < cnt; ++i)
        if (tab[i] != kNullOff) bits |= o.base + (uint64_t(tab[i]) << o.shift);
    return (bits & 127) ? 2 : 1;
}

int run_gather(mec_ctx *c, const MapSet &M, const void *stab, uint32_t sstride, const void *dtab, uint32_t dstride,
               const uint16_t *pat, uint32_t n, hipStream_t st, bool mapped_tables = false, bool device_mem = true,
               const Off32 *o32 = nullptr) {
    if (M.ssel.empty() || M.rows() == 0 || n == 0) return MEC_OK;
    const size_t es = o32 ? 4 : 8;  // bytes per row entry on the host
    // a single map with no skipped stripe runs from kernel arguments;
    // anything else through per-stripe descriptors (and byte-wise maps with
    // more than 4 outputs too: the descriptor kernel codes every row group
    // from one read of the sources)
    bool one_map = M.ssel.size() == 1;
    if (one_map && pat)
        for (uint32_t s = 0; s < n && one_map; ++s) one_map = pat[s] == 0;
    // one map and more than 4 byte-wise outputs: the one-pass kernel reads
    // the pointer rows itself, with the map's tables and structure (row 0 /
    // column 0 XORs, groups of 3, 4 or 8) like a strided launch
    const bool one_pass = one_map && M.K >= 1 && mg_wanted(c, M.rows());
    // (bitmatrix maps: up to 8 outputs per gathered bm_kernel launch)
    const bool single =
        one_map && (M.rows() <= size_t(c->byte_wise() ? kMaxRows : kMaxBmOut) || one_pass);
    std::vector<uint32_t> descs;
    uint32_t desc_dw = 0;
    const size_t groups = single ? 0 : build_descs(c, M, descs, desc_dw);
    const bool same = stab == dtab && sstride == dstride;
    std::vector<std::pair<const void *, size_t>> parts = {
        {stab, size_t(n) * sstride * es},
        {same ? nullptr : dtab, same ? 0 : size_t(n) * dstride * es},
        {single ? nullptr : pat, (pat && !single) ? size_t(n) * 2 : 0},
        {descs.data(), descs.size() * sizeof(uint32_t)}};
    SlotHold hold;
    hold.st = st;
    std::vector<size_t> offs;
    uint8_t *dev = nullptr;
    // 32-bit offset rows: expanded into the slot's pointer table right after
    // the copy, on the copy stream, so the coding launch waits for one event
    const size_t ne_s = size_t(n) * sstride, ne_d = same ? 0 : size_t(n) * dstride;
    auto expand = [&](TableSlot &t, uint8_t *d, hipStream_t cs) -> int {
        const size_t need = (ne_s + ne_d) * 8;
        if (t.xcap < need) {
            if (t.xdev) (void)hipFree(t.xdev);
            t.xdev = nullptr;
            t.xcap = 0;
            HIP_TRY(hipMalloc(reinterpret_cast<void **>(&t.xdev), std::max<size_t>(need, size_t(1) << 20)));
            t.xcap = std::max<size_t>(need, size_t(1) << 20);
        }
        HIP_TRY(launch_expand_rows(reinterpret_cast<const uint32_t *>(d + offs[0]), t.xdev, o32->base, o32->shift, ne_s, cs));
        if (!same)
            HIP_TRY(launch_expand_rows(reinterpret_cast<const uint32_t *>(d + offs[1]), t.xdev + ne_s, o32->base,
                                       o32->shift, ne_d, cs));
        return MEC_OK;
    };
    int rc = o32 ? table_upload(c, parts, hold.t, offs, st, mapped_tables, dev, expand)
                 : table_upload(c, parts, hold.t, offs, st, mapped_tables, dev);
    if (rc != MEC_OK) return rc;
    const uint64_t *dstab = reinterpret_cast<const uint64_t *>(dev + offs[0]);
    const uint64_t *ddtab = reinterpret_cast<const uint64_t *>(dev + offs[same ? 0 : 1]);
    if (o32) {
        dstab = hold.t->xdev;
        ddtab = same ? hold.t->xdev : hold.t->xdev + ne_s;
    }
    auto shape_of = [&]() -> uint8_t {
        if (!device_mem) return 0;
        if (o32)
            return std::max(gather_shape32(static_cast<const uint32_t *>(stab), sstride, n, *o32),
                            gather_shape32(static_cast<const uint32_t *>(dtab), dstride, n, *o32));
        return std::max(gather_shape(stab, sstride, n), gather_shape(dtab, dstride, n));
    };
    const size_t rows = M.rows(), nm = M.ssel.size();
    if (single) {
        // one map for every stripe: the map goes in kernel arguments
        // (gf8_kernel / bm_kernel gather mode), only the pointers are read
        const std::vector<uint8_t> &ss = M.ssel[0], &ds = M.dsel[0];
        const Mat &cf = M.coef[0];
        if (one_pass && jit_wanted(c, ds.size(), M.K, cf, true)) {
            if (JitKernel *jk = jit_kernel(c, cf, ds.size(), M.K, M.accumulate, true)) {
                BsLaunch L{};
                L.stab = dstab;
                L.dtab = ddtab;
                L.sstride = sstride;
                L.dstride = dstride;
                L.k = int(M.K);
                L.rows = int(ds.size());
                L.len = c->cs;
                L.n_stripes = n;
                L.vand = coef_vand(cf, ds.size(), M.K);
                for (uint32_t j = 0; j < M.K; ++j) L.src_off[j] = ss[j];
                for (size_t r = 0; r < ds.size(); ++r) L.dst_off[r] = ds[r];
                return jit_launch(c, jk, L, st);
            }
        }
        if (one_pass) {
            Gf8MgLaunch L{};
            L.stab = dstab;
            L.dtab = ddtab;
            L.sstride = sstride;
            L.dstride = dstride;
            L.k = int(M.K);
            L.rows = int(ds.size());
            L.len = c->cs;
            L.n_stripes = n;
            L.accumulate = M.accumulate;
            for (uint32_t j = 0; j < M.K; ++j) L.src_off[j] = ss[j];
            for (size_t r = 0; r < ds.size(); ++r) L.dst_off[r] = ds[r];
            rc = mg_prepare(c, cf, ds.size(), M.K, L, st);
            if (rc == MEC_OK) {
                HIP_TRY(launch_gf8_mg(L, st));
                return MEC_OK;
            }
            if (rc != kMgUncached) return rc;
            // past the table cache's cap: 4-row launches below
        }
        const size_t step = c->byte_wise() ? size_t(kMaxRows) : size_t(kMaxBmOut);
        for (size_t r0 = 0; r0 < ds.size(); r0 += step) {
            const int nr = int(std::min<size_t>(step, ds.size() - r0));
            if (c->byte_wise()) {
                Gf8Launch L{};
                L.stab = dstab;
                L.dtab = ddtab;
                L.sstride = sstride;
                L.dstride = dstride;
                L.k = int(M.K);
                L.rows = nr;
                L.len = c->cs;
                L.n_stripes = n;
                L.accumulate = M.accumulate;
                L.gshape = shape_of();
                for (uint32_t j = 0; j < M.K; ++j) L.src_off[j] = ss[j];
                for (int i = 0; i < nr; ++i) {
                    L.dst_off[i] = ds[r0 + i];
                    for (uint32_t j = 0; j < M.K; ++j) L.coef[i][j] = gf8_coef(cf[(r0 + i) * M.K + j]);
                }
                HIP_TRY(launch_gf8(L, st));
            } else {
                const Field &f = Field::get(int(c->w));
                BmLaunch L{};
                L.stab = dstab;
                L.dtab = ddtab;
                L.sstride = sstride;
                L.dstride = dstride;
                L.k = int(M.K);
                L.rows = nr;
                L.w = int(c->w);
                L.packet = c->packet;
                L.n_stripes = n;
                L.accumulate = M.accumulate;
                L.gshape = shape_of();
                for (uint32_t j = 0; j < M.K; ++j) L.src_off[j] = ss[j];
                for (int i = 0; i < nr; ++i) {
                    L.dst_off[i] = ds[r0 + i];
                    for (uint32_t j = 0; j < M.K; ++j) bit_block(f, cf[(r0 + i) * M.K + j], c->w, &L.mask[j][i * c->w], 1);
                }
                HIP_TRY(launch_bm(L, st));
            }
        }
        return MEC_OK;
    }
    GatherLaunch L{};
    L.stab = dstab;
    L.dtab = ddtab;
    L.sstride = sstride;
    L.dstride = dstride;
    L.pat = pat ? reinterpret_cast<const uint16_t *>(dev + offs[2]) : nullptr;
    L.n_stripes = n;
    L.k = int(M.K);
    L.accumulate = M.accumulate;
    if (c->byte_wise()) {  // every row group in one launch (rows past a map's own are kNoRow)
        L.rows = int(std::min<size_t>(kMaxRows, rows));
        L.desc = dev + offs[3];
        L.desc_dw = desc_dw;
        L.groups = uint32_t(groups);
        L.group_maps = uint32_t(nm);
        L.w = 0;
        L.len = c->cs;
        HIP_TRY(launch_gf8_gather(L, st));
        return MEC_OK;
    }
    for (size_t g = 0; g < groups; ++g) {  // bitmatrix: groups of up to 8 outputs
        L.rows = int(std::min<size_t>(kBmGatherRows, rows - g * kBmGatherRows));
        L.desc = dev + offs[3] + g * nm * desc_dw * sizeof(uint32_t);
        L.desc_dw = desc_dw;
        {
            L.w = int(c->w);
            L.len = c->packet;
            HIP_TRY(launch_bm_gather(L, st));
        }
    }
    return MEC_OK;
}

// ---------------------------------------------------------------------------
// host-memory execution over unregistered chunks: pack into pinned,
// GPU-mapped staging -> kernel over PCIe -> unpack, two buffers in flight
// ---------------------------------------------------------------------------
constexpr size_t kPipeBytes = size_t(64) << 20;  // per staging buffer

struct Copy {
    void *dst;
    const void *src;
};

// Threads for packing / unpacking staged chunks (MEC_COPY_THREADS, default 8).
unsigned copy_threads() {
    const int64_t e = detail::knob(detail::kKnobCopyThreads);
    const int64_t v = e != detail::kKnobUnset ? e : 8;
    return unsigned(std::max<int64_t>(1, std::min<int64_t>(v, 64)));
}

// memcpy with non-temporal stores for the staged paths' big copies: what
// they write (staging read by DMA or a kernel, outputs handed back) is not
// read again by this thread, so the stores skip the cache and its
// read-for-ownership.  Callers fence (_mm_sfence) before anyone else reads.
static void nt_copy(void *dst, const void *src, size_t n) {
    auto *d = static_cast<uint8_t *>(dst);
    auto *s = static_cast<const uint8_t *>(src);
    const size_t head = (0 - reinterpret_cast<uintptr_t>(d)) & 15;
    if (n < 1024) {
        std::memcpy(d, s, n);
        return;
    }
    std::memcpy(d, s, head);
    d += head;
    s += head;
    n -= head;
    for (; n >= 64; n -= 64, d += 64, s += 64) {
        const __m128i a = _mm_loadu_si128(reinterpret_cast<const __m128i *>(s));
        const __m128i b = _mm_loadu_si128(reinterpret_cast<const __m128i *>(s + 16));
        const __m128i c = _mm_loadu_si128(reinterpret_cast<const __m128i *>(s + 32));
        const __m128i e = _mm_loadu_si128(reinterpret_cast<const __m128i *>(s + 48));
        _mm_stream_si128(reinterpret_cast<__m128i *>(d), a);
        _mm_stream_si128(reinterpret_cast<__m128i *>(d + 16), b);
        _mm_stream_si128(reinterpret_cast<__m128i *>(d + 32), c);
        _mm_stream_si128(reinterpret_cast<__m128i *>(d + 48), e);
    }
    std::memcpy(d, s, n);
}

// Long-lived helper threads for the big host copies of the staged paths.
// Spawning the helpers per copy cost about a tenth of a staged RS(10,4)
// 1 MiB-chunk batch (73 sub-batches x 2 copies x 8 thread starts).  One job
// at a time (bandwidth is shared anyway); the caller works too, and chunks
// are claimed in runs so slow threads do not hold the job back.  Against
// threads spawned per copy: staged pointer batches +4-10 %, dense batches
// equal or +1 % (profiles/r06/host/copy_pool_ab_r06{m,n,o,p}).  The
// pool is deliberately leaked (its threads wait on it until the process
// ends) and rebuilt in a forked child, which inherits no threads.
class CopyPool {
public:
    static CopyPool &get() {
        static std::mutex mu;
        static CopyPool *pool = nullptr;
        std::lock_guard<std::mutex> lk(mu);
        if (!pool || pool->pid_ != getpid()) pool = new CopyPool;
        return *pool;
    }

    void run(const Copy *ops, size_t n, size_t len, unsigned helpers) {
        std::lock_guard<std::mutex> job(job_mu_);
        while (threads_ < helpers) {
            std::thread(&CopyPool::worker, this, threads_).detach();
            ++threads_;
        }
        {
            std::lock_guard<std::mutex> lk(mu_);
            ops_ = ops;
            n_ = n;
            len_ = len;
            next_.store(0, std::memory_order_relaxed);
            helpers_ = helpers;
            active_ = helpers;
            ++gen_;
        }
        cv_.notify_all();
        drain();
        std::unique_lock<std::mutex> lk(mu_);
        idle_cv_.wait(lk, [&] { return active_ == 0; });
    }

private:
    // claims runs of >= 1 MiB: per-chunk claims of 4 KiB chunks scattered
    // each thread's writes and cost 30 % (profiles/r06/host/copy_pool_ab_r06m)
    void drain() {
        const size_t run = std::max<size_t>(1, (size_t(1) << 20) / len_);
        for (size_t a; (a = next_.fetch_add(run, std::memory_order_relaxed)) < n_;)
            for (size_t i = a, b = std::min(n_, a + run); i < b; ++i) nt_copy(ops_[i].dst, ops_[i].src, len_);
        _mm_sfence();
    }
    void worker(unsigned id) {
        uint64_t seen = 0;
        std::unique_lock<std::mutex> lk(mu_);
        for (;;) {
            cv_.wait(lk, [&] { return gen_ != seen; });
            seen = gen_;
            if (id >= helpers_) continue;  // not asked to help with this job
            lk.unlock();
            drain();
            lk.lock();
            if (--active_ == 0) idle_cv_.notify_one();
        }
    }

    const pid_t pid_ = getpid();
    std::mutex job_mu_, mu_;
    std::condition_variable cv_, idle_cv_;
    unsigned threads_ = 0, helpers_ = 0, active_ = 0;
    uint64_t gen_ = 0;
    const Copy *ops_ = nullptr;
    size_t n_ = 0, len_ = 0;
    std::atomic<size_t> next_{0};
};

// memcpy of many equal-sized chunks, split over a few threads when large.
void copy_chunks(const std::vector<Copy> &ops, size_t len) {
    const size_t bytes = ops.size() * len;
    unsigned nt = 1;
    if (bytes >= (size_t(8) << 20)) nt = std::min<unsigned>(copy_threads(), std::max(1u, std::thread::hardware_concurrency() / 2));
    nt = std::min<unsigned>(nt, unsigned(ops.size()));
    if (nt <= 1) {
        for (const Copy &o : ops) nt_copy(o.dst, o.src, len);
        _mm_sfence();
        return;
    }
    CopyPool::get().run(ops.data(), ops.size(), len, nt - 1);
}

// A call's tables (pointer rows: 5 MB per RS(8,2)@4 KiB batch of 65536
// stripes) into the slot's pinned staging: from 1 MiB on over a few pool
// threads in 256 KiB pieces, so the host prepares the next call's rows well
// inside the launch before it (one thread copying them, plus a one-map
// decode's planning, took longer than that 0.44 ms launch: rocprofv3
// traces, profiles/r06/batch/).
void table_memcpy(void *dst, const void *src, size_t n) {
    constexpr size_t kPiece = size_t(256) << 10;
    if (n < (size_t(1) << 20)) {
        std::memcpy(dst, src, n);
        return;
    }
    const unsigned nt = std::min<unsigned>({4u, copy_threads(), std::max(1u, std::thread::hardware_concurrency() / 2)});
    std::vector<Copy> ops;
    for (size_t o = 0; o + kPiece <= n; o += kPiece)
        ops.push_back({static_cast<uint8_t *>(dst) + o, static_cast<const uint8_t *>(src) + o});
    if (nt <= 1) {
        for (const Copy &o : ops) nt_copy(o.dst, o.src, kPiece);
        _mm_sfence();
    } else {
        CopyPool::get().run(ops.data(), ops.size(), kPiece, std::min<unsigned>(nt - 1, unsigned(ops.size())));
    }
    const size_t done = n / kPiece * kPiece;
    std::memcpy(static_cast<uint8_t *>(dst) + done, static_cast<const uint8_t *>(src) + done, n - done);
}

void par_memcpy(void *dst, const void *src, size_t n) {
    if (n == 0) return;
    constexpr size_t kPiece = size_t(1) << 20;
    if (n < (size_t(8) << 20)) {
        std::memcpy(dst, src, n);
        return;
    }
    std::vector<Copy> ops;
    for (size_t o = 0; o + kPiece <= n; o += kPiece)
        ops.push_back({static_cast<uint8_t *>(dst) + o, static_cast<const uint8_t *>(src) + o});
    copy_chunks(ops, kPiece);
    const size_t done = n / kPiece * kPiece;
    std::memcpy(static_cast<uint8_t *>(dst) + done, static_cast<const uint8_t *>(src) + done, n - done);
}

int pipe_ready(mec_ctx *c, size_t bytes) {
    HostPipe &P = c->pipe;
    for (int b = 0; b < 2; ++b) {
        if (!P.stream[b]) HIP_TRY(hipStreamCreateWithFlags(&P.stream[b], hipStreamNonBlocking));
        // system-scope release: the outputs the kernel wrote to the mapped
        // staging are read by the host right after the wait (lane_sync)
        if (!P.done[b]) HIP_TRY(hipEventCreateWithFlags(&P.done[b], hipEventDisableTiming | hipEventReleaseToSystem));
    }
    if (P.bytes >= bytes) return MEC_OK;
    for (int b = 0; b < 2; ++b) {
        if (P.host[b]) (void)hipHostFree(P.host[b]);
        P.host[b] = P.hdev[b] = nullptr;
    }
    P.bytes = 0;
    for (int b = 0; b < 2; ++b) {
        HIP_TRY(hipHostMalloc(reinterpret_cast<void **>(&P.host[b]), bytes, hipHostMallocMapped));
        HIP_TRY(hipHostGetDevicePointer(reinterpret_cast<void **>(&P.hdev[b]), P.host[b], 0));
    }
    P.bytes = bytes;
    return MEC_OK;
}

struct Item {
    Group *g;
    uint32_t s0, n;
};

// Zero-copy execution (hostmem.cpp): every chunk of every group lies in a
// registered host range, so each group is one gathered launch over the
// chunks' device addresses, on a lane stream; returns kNotZeroCopy (and
// does nothing) otherwise.
constexpr int kNotZeroCopy = 1;

int run_zerocopy(mec_ctx *c, std::vector<Group> &gs) {
    const size_t cs = c->cs;
    std::vector<std::vector<uint64_t>> rows(gs.size());
    for (size_t q = 0; q < gs.size(); ++q) {
        rows[q] = gs[q].ptrs;
        if (!zc_translate(rows[q].data(), rows[q].size(), cs)) return kNotZeroCopy;
    }
    int rc = MEC_OK;
    LaneHold h{c, lane_acquire(c, rc)};
    if (!h.l) return rc;
    for (size_t q = 0; q < gs.size() && rc == MEC_OK; ++q) {
        const Group &g = gs[q];
        if (!g.n || !g.nd) continue;
        const uint32_t row = g.ns + g.nd;
        if (!g.ns) {  // every source is Coding::zeros: zero outputs (host pointers)
            if (g.accumulate) continue;
            for (uint32_t s = 0; s < g.n; ++s)
                for (uint32_t r = 0; r < g.nd; ++r) std::memset(reinterpret_cast<void *>(g.ptrs[size_t(s) * row + g.ns + r]), 0, cs);
            continue;
        }
        MapSet M;
        M.K = g.ns;
        M.accumulate = g.accumulate;
        std::vector<uint8_t> ss(g.ns), ds(g.nd);
        for (uint32_t j = 0; j < g.ns; ++j) ss[j] = uint8_t(j);
        for (uint32_t i = 0; i < g.nd; ++i) ds[i] = uint8_t(g.ns + i);
        M.add(ss, ds, g.coef);
        // small batches (coalesced single-stripe calls) read their pointer
        // rows in place from pinned memory: one launch, no table copy
        rc = run_gather(c, M, rows[q].data(), row, rows[q].data(), row, nullptr, g.n, h.l->stream, g.n <= 256, false);
    }
    // no launch may outlive the call (the caller owns the chunks)
    hipError_t e = lane_sync(h.l);
    if (rc == MEC_OK && e != hipSuccess) rc = hip_fail(e, "hipStreamSynchronize");
    if (rc == MEC_OK) count_zc(c);
    return rc;
}

int run_host(mec_ctx *c, std::vector<Group> &gs) {
    if (zc_any_registered()) {
        const int zrc = run_zerocopy(c, gs);
        if (zrc != kNotZeroCopy) return zrc;
    }
    count_staged(c);
    HostPipe &P = c->pipe;
    std::lock_guard<std::mutex> lk(P.mu);
    const size_t cs = c->cs;
    std::vector<Item> items;
    size_t need = 0;
    for (Group &g : gs) {
        if (!g.n || !g.nd) continue;
        if (!g.ns) {
            if (g.accumulate) continue;
            for (uint32_t s = 0; s < g.n; ++s)
                for (uint32_t r = 0; r < g.nd; ++r) std::memset(reinterpret_cast<void *>(g.ptrs[size_t(s) * g.nd + r]), 0, cs);
            continue;
        }
        const size_t per = size_t(g.ns + g.nd) * cs;
        need = std::max(need, per);
        const uint32_t sub = uint32_t(std::max<size_t>(1, kPipeBytes / per));
        for (uint32_t s0 = 0; s0 < g.n; s0 += sub) items.push_back({&g, s0, std::min(sub, g.n - s0)});
    }
    if (items.empty()) return MEC_OK;
    int rc = pipe_ready(c, std::max(need, kPipeBytes));
    if (rc != MEC_OK) return rc;

    auto row = [](const Item &it, uint32_t s) { return &it.g->ptrs[size_t(it.s0 + s) * (it.g->ns + it.g->nd)]; };
    // staging layout: sources [n][ns][cs], then outputs [n][nd][cs]
    auto enqueue = [&](const Item &it, int b) -> int {
        const Group &g = *it.g;
        uint8_t *h = P.host[b], *d = P.hdev[b];
        const size_t srcb = size_t(it.n) * g.ns * cs;
        std::vector<Copy> ops;
        ops.reserve(size_t(it.n) * (g.ns + (g.accumulate ? g.nd : 0)));
        for (uint32_t s = 0; s < it.n; ++s) {
            const uint64_t *r = row(it, s);
            for (uint32_t j = 0; j < g.ns; ++j)
                ops.push_back({h + (size_t(s) * g.ns + j) * cs, reinterpret_cast<const void *>(r[j])});
            if (g.accumulate)
                for (uint32_t i = 0; i < g.nd; ++i)
                    ops.push_back({h + srcb + (size_t(s) * g.nd + i) * cs, reinterpret_cast<const void *>(r[g.ns + i])});
        }
        copy_chunks(ops, cs);
        std::vector<int64_t> so(g.ns), dof(g.nd);
        for (uint32_t j = 0; j < g.ns; ++j) so[j] = int64_t(j) * int64_t(cs);
        for (uint32_t i = 0; i < g.nd; ++i) dof[i] = int64_t(i) * int64_t(cs);
        int r = apply(c, d, int64_t(g.ns * cs), so, d + srcb, int64_t(g.nd * cs), dof, g.coef, it.n, g.accumulate,
                      P.stream[b]);
        if (r != MEC_OK) return r;
        HIP_TRY(hipEventRecord(P.done[b], P.stream[b]));
        return MEC_OK;
    };
    auto finish = [&](const Item &it, int b) -> int {
        HIP_TRY(hipEventSynchronize(P.done[b]));
        const Group &g = *it.g;
        const size_t srcb = size_t(it.n) * g.ns * cs;
        std::vector<Copy> ops;
        ops.reserve(size_t(it.n) * g.nd);
        for (uint32_t s = 0; s < it.n; ++s) {
            const uint64_t *r = row(it, s);
            for (uint32_t i = 0; i < g.nd; ++i)
                ops.push_back({reinterpret_cast<void *>(r[g.ns + i]), P.host[b] + srcb + (size_t(s) * g.nd + i) * cs});
        }
        copy_chunks(ops, cs);
        return MEC_OK;
    };
    size_t i = 0;
    for (; i < items.size() && rc == MEC_OK; ++i) {
        const int b = int(i & 1);
        if (i >= 2) rc = finish(items[i - 2], b);
        if (rc == MEC_OK) rc = enqueue(items[i], b);
    }
    // drain what is still in flight (also after an error: no DMA may
    // outlive this call)
    for (size_t q = (i >= 2 ? i - 2 : 0); q < i; ++q) {
        const int b = int(q & 1);
        if (rc == MEC_OK)
            rc = finish(items[q], b);
        else
            (void)hipStreamSynchronize(P.stream[b]);
    }
    return rc;
}

// ---------------------------------------------------------------------------
// coalescer: concurrent single-stripe host calls become one batch
// ---------------------------------------------------------------------------
}  // namespace core
}  // namespace mec

struct mec::core::Request {
    int op;  // 0 encode, 1 decode, 2 update
    const uint8_t *const *data;
    uint8_t *const *out;  // parity (encode/update) or chunks (decode)
    uint64_t present;
    uint32_t index;
    const uint8_t *delta;
    int rc = MEC_OK;
    bool done = false;
    std::string err;
};

namespace mec {
namespace core {

void execute(mec_ctx *c, std::vector<Request *> &batch) {
    GroupSet enc, dec, upd;
    const uint32_t all = full_mask32(c->m);
    for (size_t q = 0; q < batch.size(); ++q) {
        Request *r = batch[q];
        if (r->op == 0) {
            add_encode(c, enc, r->data, r->out, all, int32_t(q));
        } else if (r->op == 1) {
            r->rc = add_decode(c, dec, r->out, r->present, int32_t(q));
            if (r->rc != MEC_OK) r->err = g_err;
        } else {
            add_update(c, upd, r->index, r->delta, r->out, all, int32_t(q));
        }
    }
    std::vector<Group> gs;
    for (GroupSet *G : {&enc, &dec, &upd})
        for (Group &g : G->groups) gs.push_back(std::move(g));
    DeviceGuard dg(c->device);
    const int rc = run_host(c, gs);
    if (rc != MEC_OK) {
        for (Request *r : batch)
            if (r->rc == MEC_OK) {
                r->rc = rc;
                r->err = g_err;
            }
    }
    std::lock_guard<std::mutex> lk(c->coal.mu);
    c->coal.batches++;
    c->coal.requests += batch.size();
}

// Leader/follower group commit: a caller that finds fewer than kMaxLeaders
// batches in flight takes everything queued (up to max_batch) and runs it;
// callers arriving meanwhile queue up for the next batch, so the batch size
// grows with the offered load and an idle system pays no wait.  Several
// batches in flight keep the GPU and the host copies overlapped.
int submit(mec_ctx *c, Request &req) {
    Coalescer &C = c->coal;
    std::unique_lock<std::mutex> lk(C.mu);
    C.queue.push_back(&req);
    while (!req.done) {
        if (C.leaders < kMaxLeaders && !C.queue.empty()) {
            ++C.leaders;
            std::vector<Request *> batch;
            const uint32_t cap = std::max<uint32_t>(1, C.max_batch);
            while (!C.queue.empty() && batch.size() < cap) {
                batch.push_back(C.queue.front());
                C.queue.pop_front();
            }
            lk.unlock();
            execute(c, batch);
            lk.lock();
            for (Request *r : batch) r->done = true;
            --C.leaders;
            C.cv.notify_all();
        } else {
            C.cv.wait(lk);
        }
    }
    if (req.rc != MEC_OK) g_err = req.err;
    return req.rc;
}

bool coalescing(mec_ctx *c) { return c->coal.max_batch.load(std::memory_order_relaxed) > 0; }

int submit_encode(mec_ctx *c, const uint8_t *const *data, uint8_t *const *parity) {
    Request r{0, data, parity, 0, 0, nullptr};
    return submit(c, r);
}
int submit_decode(mec_ctx *c, uint8_t *const *chunks, uint64_t present) {
    Request r{1, nullptr, chunks, present, 0, nullptr};
    return submit(c, r);
}
int submit_update(mec_ctx *c, uint32_t index, const uint8_t *delta, uint8_t *const *parity) {
    Request r{2, nullptr, parity, 0, index, delta};
    return submit(c, r);
}

void batch_release(mec_ctx *c) {
    for (TableSlot &t : c->tabs) {
        if (t.pending && t.done) (void)hipEventSynchronize(t.done);
        if (t.done) (void)hipEventDestroy(t.done);
        if (t.copied) (void)hipEventDestroy(t.copied);
        if (t.host) (void)hipHostFree(t.host);
        if (t.dev) (void)hipFree(t.dev);
        if (t.xdev) (void)hipFree(t.xdev);
    }
    if (c->tab_stream) {
        (void)hipStreamSynchronize(c->tab_stream);
        (void)hipStreamDestroy(c->tab_stream);
    }
    HostPipe &P = c->pipe;
    for (int b = 0; b < 2; ++b) {
        if (P.stream[b]) {
            (void)hipStreamSynchronize(P.stream[b]);
            (void)hipStreamDestroy(P.stream[b]);
        }
        if (P.done[b]) (void)hipEventDestroy(P.done[b]);
        if (P.host[b]) (void)hipHostFree(P.host[b]);
    }
}

// The maps of a device decode batch: one per distinct erasure pattern
// (cached plans), pat[s] its index or kSkipStripe (nothing missing, or the
// stripe failed: its status goes to note(s, rc)).  is_null(s, i): chunk i
// of stripe s is NULL.
// Whether any of n row entries is NULL (kNullOff for 32-bit offset rows):
// one vectorised pass, so a batch with none skips the per-stripe checks
// (65536 stripes x 6 entries cost a decode batch ~0.1 ms per call).
template <typename T>
bool any_null_entry(const T *e, size_t n, T null) {
    bool z = false;
    for (size_t i = 0; i < n; ++i) z |= e[i] == null;
    return z;
}

template <typename IsNull, typename Note>
void decode_maps(mec_ctx *c, const uint64_t *present_masks, uint32_t n_stripes, IsNull is_null, MapSet &M,
                 std::vector<uint16_t> &pat, Note note, bool maybe_null = true) {
    const uint32_t n = c->k + c->m;
    const uint64_t full = (uint64_t(1) << n) - 1;
    M.K = c->k;
    // every stripe with one pattern and no NULL entry (a failed server: each
    // stripe lost the same chunks): one plan, no per-stripe map (pat empty =
    // map 0 for all)
    if (!maybe_null && n_stripes > 0) {
        const uint64_t p0 = present_masks[0] & full;
        bool uniform = true;
        for (uint32_t s = 1; s < n_stripes; ++s) uniform &= (present_masks[s] & full) == p0;
        const uint32_t failed = uint32_t(__builtin_popcountll(~p0 & full));
        const LinearPlan *plan = nullptr;
        if (uniform && failed > 0 && failed <= c->m && get_plan(c, p0, plan) == MEC_OK) {
            std::vector<uint8_t> ss(plan->src.begin(), plan->src.end());
            std::vector<uint8_t> ds(plan->dst.begin(), plan->dst.end());
            M.add(ss, ds, plan->coef);
            pat.clear();
            for (uint32_t s = 0; s < n_stripes; ++s) note(s, MEC_OK);
            return;
        }
    }
    pat.assign(n_stripes, kSkipStripe);
    std::unordered_map<uint64_t, uint16_t> ids;
    std::pair<uint64_t, uint16_t> seen[16];
    for (auto &e : seen) e = {~uint64_t(0), kSkipStripe};  // no present mask has every bit set
    // runs of stripes with one pattern (a reconstruction batch is mostly
    // one long run): the pattern's checks and plan once per run, per stripe
    // only the NULL check and the two stores
    for (uint32_t s = 0; s < n_stripes;) {
        const uint64_t present = present_masks[s] & full;
        uint32_t e = s + 1;
        while (e < n_stripes && (present_masks[e] & full) == present) ++e;
        const uint32_t failed = uint32_t(__builtin_popcountll(~present & full));
        if (failed > c->m) {
            for (; s < e; ++s) note(s, fail(MEC_ETOOMANY, "Too many failure to recover (%u>%u)", failed, c->m));
            continue;
        }
        if (failed == 0) {
            for (; s < e; ++s) note(s, MEC_OK);
            continue;
        }
        int prc = MEC_OK;
        uint16_t id = kSkipStripe;
        for (; s < e; ++s) {
            bool nul = false;
            if (maybe_null)
                for (uint32_t i = 0; i < n; ++i) nul |= is_null(s, i);
            if (nul) {
                uint32_t i = 0;
                while (!is_null(s, i)) ++i;
                note(s, fail(MEC_EINVAL, "chunk %u pointer is NULL", i));
                continue;
            }
            if (id == kSkipStripe && prc == MEC_OK) {  // the run's plan, at its first stripe that needs it
                // a 16-entry direct-mapped cache in front of the map: mixed
                // batches change pattern at almost every stripe
                const uint32_t slot = uint32_t((present * 0x9E3779B97F4A7C15ull) >> 60);
                if (seen[slot].first == present) {
                    id = seen[slot].second;
                    pat[s] = id;
                    note(s, MEC_OK);
                    continue;
                }
                auto it = ids.find(present);
                if (it == ids.end()) {
                    const LinearPlan *plan = nullptr;
                    prc = get_plan(c, present, plan);
                    if (prc == MEC_OK) {
                        if (M.ssel.size() >= kSkipStripe) {
                            prc = fail(MEC_EINVAL, "too many distinct erasure patterns in one batch");
                        } else {
                            std::vector<uint8_t> ss(plan->src.begin(), plan->src.end());
                            std::vector<uint8_t> ds(plan->dst.begin(), plan->dst.end());
                            it = ids.emplace(present, uint16_t(M.add(ss, ds, plan->coef))).first;
                        }
                    }
                }
                if (prc == MEC_OK) {
                    id = it->second;
                    seen[slot] = {present, id};
                }
            }
            if (prc != MEC_OK) {
                note(s, prc);  // g_err still holds the plan's message
                continue;
            }
            pat[s] = id;
            note(s, MEC_OK);
        }
    }
}

}  // namespace core
}  // namespace mec

using namespace mec;
using namespace mec::core;

extern "C" {

int mec_encode_batch(mec_ctx *c, const uint8_t *const *data, uint8_t *const *parity, uint32_t n_stripes,
                     uint32_t parity_mask, int mem_kind, void *stream) {
    CHECK_CTX(c);
    if (mem_kind != MEC_MEM_DEVICE && mem_kind != MEC_MEM_HOST) return fail(MEC_EINVAL, "bad mem_kind %d", mem_kind);
    if (n_stripes == 0) return MEC_OK;
    if (!data || !parity) return fail(MEC_EINVAL, "null pointer array");
    if (mem_kind == MEC_MEM_HOST && is_multi(c))
        return shard_run(c, n_stripes, [&](mec_ctx *sc, uint32_t s0, uint32_t s1) {
            return mec_encode_batch(sc, data + size_t(s0) * c->k, parity + size_t(s0) * c->m, s1 - s0, parity_mask,
                                    MEC_MEM_HOST, nullptr);
        });
    const uint32_t pm = parity_mask ? parity_mask : full_mask32(c->m);
    DeviceGuard dg(c->device);
    if (mem_kind == MEC_MEM_DEVICE) {
        // one map: all k columns (NULL sources read as zero), the masked rows
        // (NULL outputs are skipped in the kernel)
        MapSet M;
        M.K = c->k;
        std::vector<uint32_t> rows = bits_of(pm, c->m), cols = bits_of(full_mask32(c->k), c->k);
        std::vector<uint8_t> ss(cols.begin(), cols.end()), ds(rows.begin(), rows.end());
        M.add(ss, ds, encode_rows(c, rows, cols));
        return run_gather(c, M, data, c->k, parity, c->m, nullptr, n_stripes, hipStream_t(stream));
    }
    GroupSet G;
    for (uint32_t s = 0; s < n_stripes; ++s)
        add_encode(c, G, data + size_t(s) * c->k, parity + size_t(s) * c->m, pm, int32_t(s));
    return run_host(c, G.groups);
}

int mec_decode_batch(mec_ctx *c, uint8_t *const *chunks, const uint64_t *present_masks, uint32_t n_stripes,
                     int32_t *results, int mem_kind, void *stream) {
    CHECK_CTX(c);
    if (mem_kind != MEC_MEM_DEVICE && mem_kind != MEC_MEM_HOST) return fail(MEC_EINVAL, "bad mem_kind %d", mem_kind);
    if (n_stripes == 0) return MEC_OK;
    if (!chunks || !present_masks) return fail(MEC_EINVAL, "null pointer array");
    if (mem_kind == MEC_MEM_HOST && is_multi(c)) {
        // every shard reports its stripes' results; like one context, the
        // call returns the first failing stripe's status (with its text)
        std::vector<int32_t> res(n_stripes, MEC_OK);
        const size_t row = size_t(c->k) + c->m;
        std::mutex emu;
        std::vector<std::pair<uint32_t, std::string>> errs;  // (first stripe of the shard, its error)
        const int rc = shard_run(c, n_stripes, [&](mec_ctx *sc, uint32_t s0, uint32_t s1) -> int {
            const int r = mec_decode_batch(sc, chunks + s0 * row, present_masks + s0, s1 - s0, res.data() + s0,
                                           MEC_MEM_HOST, nullptr);
            if (r == MEC_OK) return MEC_OK;
            bool per_stripe = false;
            for (uint32_t s = s0; s < s1 && !per_stripe; ++s) per_stripe = res[s] == r;
            if (!per_stripe) return r;  // not attributable to a stripe: a real failure
            std::lock_guard<std::mutex> lk(emu);
            errs.emplace_back(s0, g_err);
            return MEC_OK;
        });
        if (results) std::copy(res.begin(), res.end(), results);
        if (rc != MEC_OK) return rc;
        for (uint32_t s = 0; s < n_stripes; ++s)
            if (res[s] != MEC_OK) {
                std::string text;
                uint32_t best = 0;
                for (const auto &e : errs)
                    if (e.first <= s && e.first >= best) {
                        best = e.first;
                        text = e.second;
                    }
                // the shard numbers its stripes from its range start
                g_err = "shard starting at stripe " + std::to_string(best) + ": " + text;
                return res[s];
            }
        return MEC_OK;
    }
    int first = MEC_OK;
    std::string first_err;
    const uint32_t n = c->k + c->m;
    auto note = [&](uint32_t s, int rc) {
        if (results) results[s] = rc;
        if (rc != MEC_OK && first == MEC_OK) {
            first = rc;
            first_err = "stripe " + std::to_string(s) + ": " + g_err;
        }
    };
    DeviceGuard dg(c->device);
    int rc = MEC_OK;
    if (mem_kind == MEC_MEM_DEVICE) {
        MapSet M;
        std::vector<uint16_t> pat;
        decode_maps(c, present_masks, n_stripes, [&](uint32_t s, uint32_t i) { return !chunks[size_t(s) * n + i]; }, M,
                    pat, note,
                    any_null_entry(reinterpret_cast<const uintptr_t *>(chunks), size_t(n_stripes) * n, uintptr_t(0)));
        rc = run_gather(c, M, chunks, n, chunks, n, pat.empty() ? nullptr : pat.data(), n_stripes, hipStream_t(stream));
    } else {
        GroupSet G;
        for (uint32_t s = 0; s < n_stripes; ++s) note(s, add_decode(c, G, chunks + size_t(s) * n, present_masks[s], int32_t(s)));
        rc = run_host(c, G.groups);
    }
    if (rc != MEC_OK) {
        if (results)
            for (uint32_t s = 0; s < n_stripes; ++s)
                if (results[s] == MEC_OK) results[s] = rc;
        return rc;
    }
    if (first != MEC_OK) g_err = first_err;
    return first;
}

int mec_encode_update_batch(mec_ctx *c, const uint32_t *data_index, const uint8_t *const *delta,
                            uint8_t *const *parity, uint32_t n_stripes, uint32_t parity_mask, int mem_kind,
                            void *stream) {
    CHECK_CTX(c);
    if (mem_kind != MEC_MEM_DEVICE && mem_kind != MEC_MEM_HOST) return fail(MEC_EINVAL, "bad mem_kind %d", mem_kind);
    if (n_stripes == 0) return MEC_OK;
    if (!data_index || !delta || !parity) return fail(MEC_EINVAL, "null pointer array");
    for (uint32_t s = 0; s < n_stripes; ++s)
        if (data_index[s] >= c->k) return fail(MEC_EINVAL, "stripe %u: data_index %u >= k %u", s, data_index[s], c->k);
    if (mem_kind == MEC_MEM_HOST && is_multi(c))
        return shard_run(c, n_stripes, [&](mec_ctx *sc, uint32_t s0, uint32_t s1) {
            return mec_encode_update_batch(sc, data_index + s0, delta + s0, parity + size_t(s0) * c->m, s1 - s0,
                                           parity_mask, MEC_MEM_HOST, nullptr);
        });
    const uint32_t pm = parity_mask ? parity_mask : full_mask32(c->m);
    DeviceGuard dg(c->device);
    if (mem_kind == MEC_MEM_DEVICE) {
        // map j = delta column j (one source, the masked rows); the stripe's
        // data_index picks it, a NULL delta skips the stripe
        MapSet M;
        M.K = 1;
        M.accumulate = true;
        const std::vector<uint32_t> rows = bits_of(pm, c->m);
        const std::vector<uint8_t> ds(rows.begin(), rows.end());
        std::vector<int> id_of(c->k, -1);
        std::vector<uint16_t> pat(n_stripes);
        for (uint32_t s = 0; s < n_stripes; ++s) {
            if (!delta[s]) {
                pat[s] = kSkipStripe;
                continue;
            }
            const uint32_t j = data_index[s];
            if (id_of[j] < 0) id_of[j] = int(M.add({0}, ds, encode_rows(c, rows, {j})));
            pat[s] = uint16_t(id_of[j]);
        }
        return run_gather(c, M, delta, 1, parity, c->m, pat.data(), n_stripes, hipStream_t(stream));
    }
    GroupSet G;
    for (uint32_t s = 0; s < n_stripes; ++s) {
        if (!delta[s]) continue;  // an all-zero delta changes nothing
        add_update(c, G, data_index[s], delta[s], parity + size_t(s) * c->m, pm, int32_t(s));
    }
    return run_host(c, G.groups);
}

// ---- 32-bit slab offsets (device memory) ----------------------------------

#define MEC_CHECK_OFF32(c, base, shift)                                                        \
    do {                                                                                        \
        if (!(base)) return fail(MEC_EINVAL, "null slab base");                                \
        if ((shift) > kMaxOffShift) return fail(MEC_EINVAL, "unit_shift %u > %u", (shift), kMaxOffShift); \
    } while (0)

int mec_encode_batch32(mec_ctx *c, uint8_t *base, uint32_t unit_shift, const uint32_t *data_off,
                       const uint32_t *parity_off, uint32_t n_stripes, uint32_t parity_mask, void *stream) {
    CHECK_CTX(c);
    if (n_stripes == 0) return MEC_OK;
    MEC_CHECK_OFF32(c, base, unit_shift);
    if (!data_off || !parity_off) return fail(MEC_EINVAL, "null offset array");
    const uint32_t pm = parity_mask ? parity_mask : full_mask32(c->m);
    DeviceGuard dg(c->device);
    MapSet M;
    M.K = c->k;
    std::vector<uint32_t> rows = bits_of(pm, c->m), cols = bits_of(full_mask32(c->k), c->k);
    std::vector<uint8_t> ss(cols.begin(), cols.end()), ds(rows.begin(), rows.end());
    M.add(ss, ds, encode_rows(c, rows, cols));
    const Off32 o{uint64_t(uintptr_t(base)), unit_shift};
    return run_gather(c, M, data_off, c->k, parity_off, c->m, nullptr, n_stripes, hipStream_t(stream), false, true, &o);
}

int mec_decode_batch32(mec_ctx *c, uint8_t *base, uint32_t unit_shift, const uint32_t *chunk_off,
                       const uint64_t *present_masks, uint32_t n_stripes, int32_t *results, void *stream) {
    CHECK_CTX(c);
    if (n_stripes == 0) return MEC_OK;
    MEC_CHECK_OFF32(c, base, unit_shift);
    if (!chunk_off || !present_masks) return fail(MEC_EINVAL, "null offset array");
    int first = MEC_OK;
    std::string first_err;
    const uint32_t n = c->k + c->m;
    auto note = [&](uint32_t s, int rc) {
        if (results) results[s] = rc;
        if (rc != MEC_OK && first == MEC_OK) {
            first = rc;
            first_err = "stripe " + std::to_string(s) + ": " + g_err;
        }
    };
    DeviceGuard dg(c->device);
    MapSet M;
    std::vector<uint16_t> pat;
    decode_maps(c, present_masks, n_stripes,
                [&](uint32_t s, uint32_t i) { return chunk_off[size_t(s) * n + i] == kNullOff; }, M, pat, note,
                any_null_entry(chunk_off, size_t(n_stripes) * n, kNullOff));
    const Off32 o{uint64_t(uintptr_t(base)), unit_shift};
    const int rc = run_gather(c, M, chunk_off, n, chunk_off, n, pat.empty() ? nullptr : pat.data(), n_stripes,
                              hipStream_t(stream), false, true, &o);
    if (rc != MEC_OK) {
        if (results)
            for (uint32_t s = 0; s < n_stripes; ++s)
                if (results[s] == MEC_OK) results[s] = rc;
        return rc;
    }
    if (first != MEC_OK) g_err = first_err;
    return first;
}

int mec_encode_update_batch32(mec_ctx *c, uint8_t *base, uint32_t unit_shift, const uint32_t *data_index,
                              const uint32_t *delta_off, const uint32_t *parity_off, uint32_t n_stripes,
                              uint32_t parity_mask, void *stream) {
    CHECK_CTX(c);
    if (n_stripes == 0) return MEC_OK;
    MEC_CHECK_OFF32(c, base, unit_shift);
    if (!data_index || !delta_off || !parity_off) return fail(MEC_EINVAL, "null offset array");
    for (uint32_t s = 0; s < n_stripes; ++s)
        if (data_index[s] >= c->k) return fail(MEC_EINVAL, "stripe %u: data_index %u >= k %u", s, data_index[s], c->k);
    const uint32_t pm = parity_mask ? parity_mask : full_mask32(c->m);
    DeviceGuard dg(c->device);
    MapSet M;
    M.K = 1;
    M.accumulate = true;
    const std::vector<uint32_t> rows = bits_of(pm, c->m);
    const std::vector<uint8_t> ds(rows.begin(), rows.end());
    std::vector<int> id_of(c->k, -1);
    std::vector<uint16_t> pat(n_stripes);
    for (uint32_t s = 0; s < n_stripes; ++s) {
        if (delta_off[s] == kNullOff) {
            pat[s] = kSkipStripe;
            continue;
        }
        const uint32_t j = data_index[s];
        if (id_of[j] < 0) id_of[j] = int(M.add({0}, ds, encode_rows(c, rows, {j})));
        pat[s] = uint16_t(id_of[j]);
    }
    const Off32 o{uint64_t(uintptr_t(base)), unit_shift};
    return run_gather(c, M, delta_off, 1, parity_off, c->m, pat.data(), n_stripes, hipStream_t(stream), false, true, &o);
}

int mec_set_coalescing(mec_ctx *c, uint32_t max_batch) {
    CHECK_CTX(c);
    for (mec_ctx *sc : c->shards) (void)mec_set_coalescing(sc, max_batch);
    std::lock_guard<std::mutex> lk(c->coal.mu);
    c->coal.max_batch.store(max_batch, std::memory_order_relaxed);
    return MEC_OK;
}

int mec_get_stats(const mec_ctx *cc, mec_stats *out) {
    if (!cc || !out) return fail(MEC_EINVAL, "null argument");
    mec_ctx *c = const_cast<mec_ctx *>(cc);
    std::lock_guard<std::mutex> lk(c->coal.mu);
    out->coalesced_batches = c->coal.batches;
    out->coalesced_requests = c->coal.requests;
    out->zero_copy_calls = out->staged_calls = out->queue_calls = 0;
    for (const auto &k : c->calls) {
        out->zero_copy_calls += k.zc.load(std::memory_order_relaxed);
        out->staged_calls += k.staged.load(std::memory_order_relaxed);
    }
    if (c->hq)
        for (uint32_t i = 0; i < c->hq->slots; ++i) out->queue_calls += c->hq->hs[i].calls.load(std::memory_order_relaxed);
    out->queue_launches = c->hq ? c->hq->launches.load() : 0;
    out->queue_slots = c->hq ? c->hq->slots : 0;
    out->queue_parts = c->hq ? c->hq->parts : 0;
    out->queue_broken = c->hq && c->hq->broken.load() ? 1u : 0u;
    out->queue_devslot = c->hq && c->hq->dslot ? 1u : 0u;
    out->queue_timeouts = c->hq ? c->hq->timeouts.load() : 0;
    {
        std::lock_guard<std::mutex> pk(c->plan_mu);
        out->cached_plans = c->plans.size();
    }
    {
        std::lock_guard<std::mutex> mk(c->mg.mu);
        out->mg_cache_bytes = c->mg.bytes;
        out->mg_cache_tables = c->mg.map.size();
        out->mg_cache_uncached = c->mg.uncached;
    }
    {
        JitShared &js = *c->jit.sh;
        std::lock_guard<std::mutex> jk(js.mu);
        out->jit_kernels = js.ready;
        out->jit_failed = js.failed;
        out->jit_pending = js.pending;
        out->jit_compile_ms = uint64_t(js.compile_ms + 0.5);
        out->jit_launches = c->jit.launches.load();
    }
    for (mec_ctx *sc : c->shards) {  // a multi context reports its shards' sums
        mec_stats t{};
        (void)mec_get_stats(sc, &t);
        out->coalesced_batches += t.coalesced_batches;
        out->coalesced_requests += t.coalesced_requests;
        out->cached_plans += t.cached_plans;
        out->zero_copy_calls += t.zero_copy_calls;
        out->staged_calls += t.staged_calls;
        out->queue_calls += t.queue_calls;
        out->queue_launches += t.queue_launches;
        out->queue_slots += t.queue_slots;
        out->queue_parts = std::max(out->queue_parts, t.queue_parts);
        out->queue_broken |= t.queue_broken;
        out->queue_devslot |= t.queue_devslot;
        out->queue_timeouts += t.queue_timeouts;
        out->mg_cache_bytes += t.mg_cache_bytes;
        out->mg_cache_tables += t.mg_cache_tables;
        out->mg_cache_uncached += t.mg_cache_uncached;
        out->jit_kernels += t.jit_kernels;
        out->jit_failed += t.jit_failed;
        out->jit_pending += t.jit_pending;
        out->jit_compile_ms += t.jit_compile_ms;
        out->jit_launches += t.jit_launches;
    }
    return MEC_OK;
}

}  // extern "C"
