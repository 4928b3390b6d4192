// hostmem.cpp — host memory the GPU addresses directly (zero-copy).
//
// MemEC's chunks start and end in host memory (ChunkPool slabs fed from
// sockets, chunk_pool.cc:22-95).  Host memory registered with
// mec_host_register is mapped into the GPU's address space, so the coding
// kernels read the k source chunks over PCIe and write the outputs straight
// back — no staging copy through HBM and one launch per call.  Measured on
// MI355X (tools/zerocopy_probe.hip, profiles/r01/host/zerocopy_probe.log): the RS(10,4)
// stream reads host memory at 54.7 GB/s of data (PCIe Gen5 x16 both ways)
// against 40.4 GB/s for H2D + kernel + D2H, and a single RS(8,2) 4 KiB
// stripe takes 13.5 us instead of 20.6 us.
//
// The registry maps registered host ranges to their device addresses; the
// host entry points (mec_*_host, mec_*_batch with MEC_MEM_HOST,
// mec_encode_host_batch) take the zero-copy path when every chunk of the
// call lies in a registered range; otherwise they copy the chunks into
// pinned, GPU-mapped staging and code there (still no HBM round trip).
// Registration is Portable: on ROCm the locked range has one device address
// valid on every GPU, so a multi-device context shares this registry.
#include <algorithm>
#include <atomic>
#include <functional>
#include <mutex>
#include <thread>

#include "ctx.hpp"
#include "registry.hpp"

namespace mec {
namespace core {
namespace {

using reg::Range;

// The registry as an immutable snapshot (ranges sorted by begin, disjoint),
// replaced as a whole by mec_host_register / mec_host_unregister under
// reg_mu and read without a lock: every zero-copy host call looks up each of
// its chunks here, and 16 server workers taking a reader lock per chunk
// bounced one cache line ~10^7 times a second.  Readers announce themselves
// on one of kStripes counters (each on its own cache line; a thread keeps
// its stripe, so with fewer threads than stripes nobody shares one) before
// loading the snapshot pointer, and a writer that has published a new
// snapshot frees the old one once it has seen every stripe at zero: a reader
// that could still hold the old pointer incremented its stripe before the
// writer's exchange (both sequentially consistent), so its count is not zero
// until it is done (replaced snapshots were never freed).
struct Snapshot {
    std::vector<Range> r;
};
constexpr size_t kStripes = 64;
struct alignas(64) ReaderStripe {
    std::atomic<uint64_t> n{0};
};
ReaderStripe g_readers[kStripes];
std::mutex reg_mu;
std::atomic<const Snapshot *> reg_snap{nullptr};

struct ReadGuard {
    ReaderStripe &s;
    ReadGuard() : s(g_readers[stripe()]) { s.n.fetch_add(1, std::memory_order_seq_cst); }
    ~ReadGuard() { s.n.fetch_sub(1, std::memory_order_release); }
    static size_t stripe() {
        static thread_local const size_t i = std::hash<std::thread::id>()(std::this_thread::get_id()) % kStripes;
        return i;
    }
    const Snapshot *snap() const { return reg_snap.load(std::memory_order_seq_cst); }
};

// Caller holds reg_mu: publish `r` as the new snapshot and free the old one
// once no reader can hold it.
void publish(std::vector<Range> r) {
    const Snapshot *n = r.empty() ? nullptr : new Snapshot{std::move(r)};
    const Snapshot *old = reg_snap.exchange(n, std::memory_order_seq_cst);
    if (!old) return;
    for (ReaderStripe &s : g_readers)
        while (s.n.load(std::memory_order_seq_cst) != 0) std::this_thread::yield();
    delete old;
}

const std::vector<Range> &ranges(const Snapshot *s) {
    static const std::vector<Range> none;
    return s ? s->r : none;
}

}  // namespace

bool zc_device_address(const void *p, size_t len, uint64_t &dev) {
    ReadGuard g;
    const Snapshot *s = g.snap();
    return s && reg::lookup(s->r, reinterpret_cast<uintptr_t>(p), len, dev);
}

bool zc_any_registered() { return reg_snap.load(std::memory_order_acquire) != nullptr; }

bool zc_translate(uint64_t *ptrs, size_t n, size_t len) {
    ReadGuard g;
    const Snapshot *s = g.snap();
    if (!s) return false;
    for (size_t i = 0; i < n; ++i) {
        if (!ptrs[i]) continue;  // NULL = zero source / unwanted output
        uint64_t d;
        if (!reg::lookup(s->r, uintptr_t(ptrs[i]), len, d)) return false;
        ptrs[i] = d;
    }
    return true;
}

}  // namespace core
}  // namespace mec

using namespace mec::core;

extern "C" {

int mec_host_register(void *ptr, size_t len) {
    if (!ptr || !len) return fail(MEC_EINVAL, "null or empty range");
    const uintptr_t a = reinterpret_cast<uintptr_t>(ptr);
    // held across hipHostRegister so two threads cannot both pass the
    // overlap check with ranges that overlap each other
    std::lock_guard<std::mutex> lk(reg_mu);
    const std::vector<Range> &cur = ranges(reg_snap.load(std::memory_order_acquire));
    Range hit{};
    switch (mec::reg::can_insert(cur, a, len, &hit)) {
        case mec::reg::Insert::kOk: break;
        case mec::reg::Insert::kOverlap:
            return fail(MEC_EINVAL, "[%p, +%zu) overlaps the registered range [%p, %p)%s", ptr, len,
                        reinterpret_cast<void *>(hit.begin), reinterpret_cast<void *>(hit.end),
                        hit.begin == a ? " (already registered)" : "; unregister it first");
        default: return fail(MEC_EINVAL, "range [%p, +%zu) wraps the address space", ptr, len);
    }
    HIP_TRY(hipHostRegister(ptr, len, hipHostRegisterMapped | hipHostRegisterPortable));
    void *dev = nullptr;
    hipError_t e = hipHostGetDevicePointer(&dev, ptr, 0);
    if (e != hipSuccess) {
        (void)hipHostUnregister(ptr);
        return hip_fail(e, "hipHostGetDevicePointer");
    }
    publish(mec::reg::with(cur, a, len, reinterpret_cast<uintptr_t>(dev)));
    return MEC_OK;
}

int mec_host_unregister(void *ptr) {
    {
        std::lock_guard<std::mutex> lk(reg_mu);
        bool found = false;
        std::vector<Range> r = mec::reg::without(ranges(reg_snap.load(std::memory_order_acquire)),
                                                 reinterpret_cast<uintptr_t>(ptr), found);
        if (!found) return fail(MEC_EINVAL, "%p does not begin a registered range", ptr);
        publish(std::move(r));
    }
    HIP_TRY(hipHostUnregister(ptr));
    return MEC_OK;
}

}  // extern "C"
