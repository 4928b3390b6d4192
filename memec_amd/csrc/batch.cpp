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
#include <cstring>
#include <thread>

#include "ctx.hpp"

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
    std::shared_ptr<LinearPlan> plan;  // decode groups: survivor / output chunk indices
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
    const std::vector<uint32_t> cols = bits_of(sm, c->k), rows = bits_of(dm, c->m);
    if (fresh) {
        g.coef = encode_rows(c, rows, cols);
        g.ns = uint32_t(cols.size());
        g.nd = uint32_t(rows.size());
    }
    for (uint32_t j : cols) g.ptrs.push_back(uint64_t(uintptr_t(data[j])));
    for (uint32_t i : rows) g.ptrs.push_back(uint64_t(uintptr_t(parity[i])));
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
    const std::vector<uint32_t> rows = bits_of(dm, c->m);
    if (fresh) {
        g.coef = encode_rows(c, rows, {j});
        g.ns = 1;
        g.nd = uint32_t(rows.size());
        g.accumulate = true;
    }
    g.ptrs.push_back(uint64_t(uintptr_t(delta)));
    for (uint32_t i : rows) g.ptrs.push_back(uint64_t(uintptr_t(parity[i])));
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
        std::shared_ptr<LinearPlan> plan;
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
// device-resident execution: one table upload, one gather launch per group
// ---------------------------------------------------------------------------
int run_device(mec_ctx *c, std::vector<Group> &gs, hipStream_t st) {
    size_t total = 0;
    for (Group &g : gs) {
        if (!g.n || !g.nd) continue;
        if (!g.ns) {  // every source is the zeros sentinel: outputs are zero
            if (g.accumulate) continue;
            for (uint32_t s = 0; s < g.n; ++s)
                for (uint32_t r = 0; r < g.nd; ++r)
                    HIP_TRY(hipMemsetAsync(reinterpret_cast<void *>(g.ptrs[size_t(s) * g.nd + r]), 0, c->cs, st));
            continue;
        }
        total += g.ptrs.size();
    }
    if (!total) return MEC_OK;
    uint32_t idx;
    {
        std::lock_guard<std::mutex> lk(c->tab_mu);
        idx = c->tab_next++ % kTableSlots;
    }
    TableSlot &t = c->tabs[idx];
    std::lock_guard<std::mutex> lk(t.mu);
    if (t.pending) {
        HIP_TRY(hipEventSynchronize(t.done));
        t.pending = false;
    }
    if (!t.done) HIP_TRY(hipEventCreateWithFlags(&t.done, hipEventDisableTiming));
    if (t.cap < total) {
        if (t.host) (void)hipHostFree(t.host);
        if (t.dev) (void)hipFree(t.dev);
        t.host = nullptr;
        t.dev = nullptr;
        t.cap = 0;
        const size_t cap = std::max<size_t>(total, 4096);
        HIP_TRY(hipHostMalloc(reinterpret_cast<void **>(&t.host), cap * sizeof(uint64_t), hipHostMallocDefault));
        HIP_TRY(hipMalloc(reinterpret_cast<void **>(&t.dev), cap * sizeof(uint64_t)));
        t.cap = cap;
    }
    size_t off = 0;
    for (Group &g : gs) {
        if (!g.n || !g.nd || !g.ns) continue;
        std::memcpy(t.host + off, g.ptrs.data(), g.ptrs.size() * sizeof(uint64_t));
        off += g.ptrs.size();
    }
    HIP_TRY(hipMemcpyAsync(t.dev, t.host, total * sizeof(uint64_t), hipMemcpyHostToDevice, st));
    off = 0;
    int rc = MEC_OK;
    for (Group &g : gs) {
        if (!g.n || !g.nd || !g.ns) continue;
        rc = apply(c, Layout::gather(t.dev + off, g.ns, g.nd), g.coef, g.n, g.accumulate, st);
        if (rc != MEC_OK) break;
        off += g.ptrs.size();
    }
    // recorded even after a failed launch so the slot is never reused early
    HIP_TRY(hipEventRecord(t.done, st));
    t.pending = true;
    return rc;
}

// ---------------------------------------------------------------------------
// host-memory execution: pack -> H2D -> kernel -> D2H -> unpack, two
// buffers in flight
// ---------------------------------------------------------------------------
constexpr size_t kPipeBytes = size_t(64) << 20;   // per staging buffer
constexpr size_t kDirectChunk = size_t(256) << 10; // chunks this large are DMA'd in place

struct Copy {
    void *dst;
    const void *src;
};

// memcpy of many equal-sized chunks, split over a few threads when large.
void copy_chunks(const std::vector<Copy> &ops, size_t len) {
    const size_t bytes = ops.size() * len;
    unsigned nt = 1;
    if (bytes >= (size_t(8) << 20)) nt = std::min<unsigned>(8, std::max(1u, std::thread::hardware_concurrency() / 2));
    nt = std::min<unsigned>(nt, unsigned(ops.size()));
    auto work = [&](unsigned t) {
        const size_t a = ops.size() * t / nt, b = ops.size() * (t + 1) / nt;
        for (size_t i = a; i < b; ++i) std::memcpy(ops[i].dst, ops[i].src, len);
    };
    if (nt <= 1) {
        work(0);
        return;
    }
    std::vector<std::thread> th;
    for (unsigned t = 1; t < nt; ++t) th.emplace_back(work, t);
    work(0);
    for (auto &x : th) x.join();
}

int pipe_ready(mec_ctx *c, size_t bytes) {
    HostPipe &P = c->pipe;
    for (int b = 0; b < 2; ++b) {
        if (!P.stream[b]) HIP_TRY(hipStreamCreateWithFlags(&P.stream[b], hipStreamNonBlocking));
        if (!P.done[b]) HIP_TRY(hipEventCreateWithFlags(&P.done[b], hipEventDisableTiming));
    }
    if (P.bytes >= bytes) return MEC_OK;
    for (int b = 0; b < 2; ++b) {
        if (P.host[b]) (void)hipHostFree(P.host[b]);
        if (P.dev[b]) (void)hipFree(P.dev[b]);
        P.host[b] = P.dev[b] = nullptr;
    }
    P.bytes = 0;
    for (int b = 0; b < 2; ++b) {
        HIP_TRY(hipHostMalloc(reinterpret_cast<void **>(&P.host[b]), bytes, hipHostMallocDefault));
        HIP_TRY(hipMalloc(reinterpret_cast<void **>(&P.dev[b]), bytes));
    }
    P.bytes = bytes;
    return MEC_OK;
}

struct Item {
    Group *g;
    uint32_t s0, n;
    bool direct;
};

int run_host(mec_ctx *c, std::vector<Group> &gs) {
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
        for (uint32_t s0 = 0; s0 < g.n; s0 += sub) items.push_back({&g, s0, std::min(sub, g.n - s0), cs >= kDirectChunk});
    }
    if (items.empty()) return MEC_OK;
    int rc = pipe_ready(c, std::max(need, kPipeBytes));
    if (rc != MEC_OK) return rc;

    auto row = [](const Item &it, uint32_t s) { return &it.g->ptrs[size_t(it.s0 + s) * (it.g->ns + it.g->nd)]; };
    // staging layout: sources [n][ns][cs], then outputs [n][nd][cs]
    auto enqueue = [&](const Item &it, int b) -> int {
        const Group &g = *it.g;
        uint8_t *h = P.host[b], *d = P.dev[b];
        const size_t srcb = size_t(it.n) * g.ns * cs, outb = size_t(it.n) * g.nd * cs;
        hipStream_t st = P.stream[b];
        if (it.direct) {
            for (uint32_t s = 0; s < it.n; ++s) {
                const uint64_t *r = row(it, s);
                for (uint32_t j = 0; j < g.ns; ++j)
                    HIP_TRY(hipMemcpyAsync(d + (size_t(s) * g.ns + j) * cs, reinterpret_cast<const void *>(r[j]), cs,
                                           hipMemcpyHostToDevice, st));
                if (g.accumulate)
                    for (uint32_t i = 0; i < g.nd; ++i)
                        HIP_TRY(hipMemcpyAsync(d + srcb + (size_t(s) * g.nd + i) * cs,
                                               reinterpret_cast<const void *>(r[g.ns + i]), cs, hipMemcpyHostToDevice, st));
            }
        } else {
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
            HIP_TRY(hipMemcpyAsync(d, h, srcb + (g.accumulate ? outb : 0), hipMemcpyHostToDevice, st));
        }
        std::vector<int64_t> so(g.ns), dof(g.nd);
        for (uint32_t j = 0; j < g.ns; ++j) so[j] = int64_t(j) * int64_t(cs);
        for (uint32_t i = 0; i < g.nd; ++i) dof[i] = int64_t(i) * int64_t(cs);
        int r = apply(c, d, int64_t(g.ns * cs), so, d + srcb, int64_t(g.nd * cs), dof, g.coef, it.n, g.accumulate, st);
        if (r != MEC_OK) return r;
        if (it.direct) {
            for (uint32_t s = 0; s < it.n; ++s) {
                const uint64_t *rw = row(it, s);
                for (uint32_t i = 0; i < g.nd; ++i)
                    HIP_TRY(hipMemcpyAsync(reinterpret_cast<void *>(rw[g.ns + i]), d + srcb + (size_t(s) * g.nd + i) * cs,
                                           cs, hipMemcpyDeviceToHost, st));
            }
        } else {
            HIP_TRY(hipMemcpyAsync(h + srcb, d + srcb, outb, hipMemcpyDeviceToHost, st));
        }
        HIP_TRY(hipEventRecord(P.done[b], st));
        return MEC_OK;
    };
    auto finish = [&](const Item &it, int b) -> int {
        HIP_TRY(hipEventSynchronize(P.done[b]));
        if (it.direct) return MEC_OK;
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

int run(mec_ctx *c, std::vector<Group> &gs, int kind, hipStream_t st) {
    if (kind == MEC_MEM_DEVICE) return run_device(c, gs, st);
    return run_host(c, gs);
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

// Leader/follower group commit: the first caller to find no batch in
// flight takes everything queued (up to max_batch) and runs it; callers
// arriving meanwhile queue up for the next batch, so the batch size grows
// with the offered load and an idle system pays no wait.
int submit(mec_ctx *c, Request &req) {
    Coalescer &C = c->coal;
    std::unique_lock<std::mutex> lk(C.mu);
    C.queue.push_back(&req);
    while (!req.done) {
        if (!C.leader_active) {
            C.leader_active = true;
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
            C.leader_active = false;
            C.cv.notify_all();
        } else {
            C.cv.wait(lk);
        }
    }
    if (req.rc != MEC_OK) g_err = req.err;
    return req.rc;
}

bool coalescing(mec_ctx *c) {
    std::lock_guard<std::mutex> lk(c->coal.mu);
    return c->coal.max_batch > 0;
}

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
        if (t.host) (void)hipHostFree(t.host);
        if (t.dev) (void)hipFree(t.dev);
    }
    HostPipe &P = c->pipe;
    for (int b = 0; b < 2; ++b) {
        if (P.stream[b]) {
            (void)hipStreamSynchronize(P.stream[b]);
            (void)hipStreamDestroy(P.stream[b]);
        }
        if (P.done[b]) (void)hipEventDestroy(P.done[b]);
        if (P.host[b]) (void)hipHostFree(P.host[b]);
        if (P.dev[b]) (void)hipFree(P.dev[b]);
    }
}

}  // namespace core
}  // namespace mec

using namespace mec::core;

extern "C" {

int mec_encode_batch(mec_ctx *c, const uint8_t *const *data, uint8_t *const *parity, uint32_t n_stripes,
                     uint32_t parity_mask, int mem_kind, void *stream) {
    CHECK_CTX(c);
    if (mem_kind != MEC_MEM_DEVICE && mem_kind != MEC_MEM_HOST) return fail(MEC_EINVAL, "bad mem_kind %d", mem_kind);
    if (n_stripes == 0) return MEC_OK;
    if (!data || !parity) return fail(MEC_EINVAL, "null pointer array");
    const uint32_t pm = parity_mask ? parity_mask : full_mask32(c->m);
    GroupSet G;
    for (uint32_t s = 0; s < n_stripes; ++s)
        add_encode(c, G, data + size_t(s) * c->k, parity + size_t(s) * c->m, pm, int32_t(s));
    DeviceGuard dg(c->device);
    return run(c, G.groups, mem_kind, hipStream_t(stream));
}

int mec_decode_batch(mec_ctx *c, uint8_t *const *chunks, const uint64_t *present_masks, uint32_t n_stripes,
                     int32_t *results, int mem_kind, void *stream) {
    CHECK_CTX(c);
    if (mem_kind != MEC_MEM_DEVICE && mem_kind != MEC_MEM_HOST) return fail(MEC_EINVAL, "bad mem_kind %d", mem_kind);
    if (n_stripes == 0) return MEC_OK;
    if (!chunks || !present_masks) return fail(MEC_EINVAL, "null pointer array");
    GroupSet G;
    int first = MEC_OK;
    std::string first_err;
    const uint32_t n = c->k + c->m;
    for (uint32_t s = 0; s < n_stripes; ++s) {
        const int rc = add_decode(c, G, chunks + size_t(s) * n, present_masks[s], int32_t(s));
        if (results) results[s] = rc;
        if (rc != MEC_OK && first == MEC_OK) {
            first = rc;
            first_err = "stripe " + std::to_string(s) + ": " + g_err;
        }
    }
    DeviceGuard dg(c->device);
    const int rc = run(c, G.groups, mem_kind, hipStream_t(stream));
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
    const uint32_t pm = parity_mask ? parity_mask : full_mask32(c->m);
    GroupSet G;
    for (uint32_t s = 0; s < n_stripes; ++s) {
        if (data_index[s] >= c->k) return fail(MEC_EINVAL, "stripe %u: data_index %u >= k %u", s, data_index[s], c->k);
        if (!delta[s]) continue;  // an all-zero delta changes nothing
        add_update(c, G, data_index[s], delta[s], parity + size_t(s) * c->m, pm, int32_t(s));
    }
    DeviceGuard dg(c->device);
    return run(c, G.groups, mem_kind, hipStream_t(stream));
}

int mec_set_coalescing(mec_ctx *c, uint32_t max_batch) {
    CHECK_CTX(c);
    std::lock_guard<std::mutex> lk(c->coal.mu);
    c->coal.max_batch = max_batch;
    return MEC_OK;
}

int mec_get_stats(const mec_ctx *cc, mec_stats *out) {
    if (!cc || !out) return fail(MEC_EINVAL, "null argument");
    mec_ctx *c = const_cast<mec_ctx *>(cc);
    std::lock_guard<std::mutex> lk(c->coal.mu);
    out->coalesced_batches = c->coal.batches;
    out->coalesced_requests = c->coal.requests;
    {
        std::lock_guard<std::mutex> pk(c->plan_mu);
        out->cached_plans = c->plans.size();
    }
    return MEC_OK;
}

}  // extern "C"
