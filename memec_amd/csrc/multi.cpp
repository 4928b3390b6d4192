// multi.cpp — multi-GPU contexts for one host process (mec_create_multi).
//
// MemEC runs one server process per node and keeps its chunks in host
// memory (ChunkPool slabs, chunk_pool.cc:22-95), so the way such a process
// uses several GPUs is to spread its host-memory calls over them: each GPU
// reads its share of the stripes over its own PCIe link (zero-copy on
// registered memory, or through its own mapped staging).  A multi context
// owns one ordinary context per listed device ("shards"):
//   * host-memory batches are cut into contiguous stripe ranges, one per
//     shard, run concurrently (GPU g gets [g*N/G, (g+1)*N/G), the same
//     partition as memec_amd.shard.shard_range);
//   * single-stripe host calls go to the shards round-robin;
//   * device-memory calls run on the first device (the parent context).
// Stripes are independent, so no data moves between GPUs.
#include <functional>
#include <thread>

#include "ctx.hpp"

namespace mec {
namespace core {

bool is_multi(const mec_ctx *c) { return !c->shards.empty(); }

mec_ctx *shard_pick(mec_ctx *c) {
    const uint32_t i = c->rr.fetch_add(1, std::memory_order_relaxed);
    return c->shards[i % c->shards.size()];
}

int shard_run(mec_ctx *c, uint32_t n, const std::function<int(mec_ctx *, uint32_t, uint32_t)> &fn) {
    const size_t G = c->shards.size();
    std::vector<int> rc(G, MEC_OK);
    std::vector<std::string> err(G);
    std::vector<std::thread> th;
    for (size_t g = 0; g < G; ++g) {
        const uint32_t s0 = uint32_t(uint64_t(n) * g / G), s1 = uint32_t(uint64_t(n) * (g + 1) / G);
        if (s0 == s1) continue;
        th.emplace_back([&, g, s0, s1] {
            rc[g] = fn(c->shards[g], s0, s1);
            if (rc[g] != MEC_OK) err[g] = g_err;  // g_err is thread-local
        });
    }
    for (auto &t : th) t.join();
    for (size_t g = 0; g < G; ++g)
        if (rc[g] != MEC_OK) {
            g_err = "device " + std::to_string(c->shards[g]->device) + ": " + err[g];
            return rc[g];
        }
    return MEC_OK;
}

}  // namespace core
}  // namespace mec

using namespace mec::core;

extern "C" {

int mec_create_multi(int family, uint32_t k, uint32_t m, uint32_t chunk_size, const int *devices, uint32_t n_devices,
                     mec_ctx **out) {
    if (!out) return fail(MEC_EINVAL, "out is null");
    *out = nullptr;
    if (!devices || n_devices == 0) return fail(MEC_EINVAL, "empty device list");
    for (uint32_t i = 0; i < n_devices; ++i)
        if (devices[i] < 0) return fail(MEC_EINVAL, "device %d: a multi context needs GPUs", devices[i]);
    mec_ctx *parent = nullptr;
    int rc = mec_create(family, k, m, chunk_size, devices[0], &parent);
    if (rc != MEC_OK) return rc;
    for (uint32_t i = 0; i < n_devices; ++i) {
        mec_ctx *s = nullptr;
        rc = mec_create(family, k, m, chunk_size, devices[i], &s);
        if (rc != MEC_OK) {
            mec_destroy(parent);  // also destroys the shards made so far
            return rc;
        }
        parent->shards.push_back(s);
    }
    *out = parent;
    return MEC_OK;
}

}  // extern "C"
