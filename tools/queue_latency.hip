// queue_latency.hip — where a single caller's queue call spends its time
// (one worker issuing synchronous single-stripe calls, as
// server/worker/worker.cc:128-137 does).
//
//   queue_latency <rs|cauchy|isal_rs> k m chunk calls [registered=1] [nd=1]
//
// One thread issues `calls` mec_encode_host calls, each writing `nd` parity
// chunks (the SEAL pattern: encode(index) for one parity, nd = 1) on a
// registered ChunkPool-like slab (zero-copy) or malloc'd chunks (staged),
// with mec_queue_trace_enable on.  Per call:
//   pre       API entry -> job posted           (host)
//   poll      posted -> part 0 took the job     (PCIe poll of the slot)
//   fence     took -> its acquire fence done     (device)
//   desc      fence -> descriptor + tables in LDS (device: one read over PCIe)
//   load      tables -> thread 0's source loads returned (device: one read over PCIe)
//   code      loads returned -> output stores acked (device: math, stores, their acks)
//   complete  stores acked -> host saw done     (done release + host poll)
//   post      done seen -> API return            (host)
// Device and host clocks are related by a calibration kernel that reads a
// host word the host keeps rewriting with CLOCK_MONOTONIC (midpoint of the
// read's device-side window, best of 256).  Prints one JSON line with the
// median and p90 of every segment (microseconds) and calls/s.
#include <hip/hip_runtime.h>
#include <time.h>

#include <algorithm>
#include <atomic>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <thread>
#include <vector>

#include "mec.h"

static uint64_t mono_ns() {
    timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return uint64_t(ts.tv_sec) * 1000000000ull + uint64_t(ts.tv_nsec);
}

__global__ void calib_kernel(const uint64_t *host_word, uint64_t *out, int n) {
    for (int i = 0; i < n; ++i) {
        const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
        const uint64_t v = __hip_atomic_load(host_word, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the read has returned
        const uint64_t t1 = __builtin_amdgcn_s_memrealtime();
        out[3 * i] = t0;
        out[3 * i + 1] = v;
        out[3 * i + 2] = t1;
    }
}

#define CK(x)                                                                  \
    do {                                                                       \
        hipError_t e_ = (x);                                                   \
        if (e_ != hipSuccess) {                                                \
            fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));            \
            exit(1);                                                           \
        }                                                                      \
    } while (0)
#define MK(x)                                                                  \
    do {                                                                       \
        if ((x) != MEC_OK) {                                                   \
            fprintf(stderr, "%s: %s\n", #x, mec_last_error());                 \
            exit(1);                                                           \
        }                                                                      \
    } while (0)

// device ticks -> host CLOCK_MONOTONIC ns: host = ticks * ns_per_tick - offset
static double calibrate(double ns_per_tick, double &window_ns) {
    uint64_t *word = nullptr, *dword = nullptr, *out = nullptr;
    CK(hipHostMalloc((void **)&word, 64, hipHostMallocMapped | hipHostMallocCoherent));
    CK(hipHostGetDevicePointer((void **)&dword, word, 0));
    const int n = 256;
    CK(hipMalloc((void **)&out, sizeof(uint64_t) * 3 * n));
    std::atomic<bool> stop(false);
    std::thread writer([&] {
        while (!stop.load(std::memory_order_relaxed)) __atomic_store_n(word, mono_ns(), __ATOMIC_RELEASE);
    });
    hipLaunchKernelGGL(calib_kernel, dim3(1), dim3(1), 0, 0, dword, out, n);
    CK(hipDeviceSynchronize());
    stop = true;
    writer.join();
    std::vector<uint64_t> h(3 * n);
    CK(hipMemcpy(h.data(), out, sizeof(uint64_t) * 3 * n, hipMemcpyDeviceToHost));
    double best_w = 1e18, off = 0;
    for (int i = 8; i < n; ++i) {  // the first reads warm the path
        const double w = double(h[3 * i + 2] - h[3 * i]) * ns_per_tick;
        if (w < best_w && h[3 * i + 1]) {
            best_w = w;
            off = 0.5 * double(h[3 * i] + h[3 * i + 2]) * ns_per_tick - double(h[3 * i + 1]);
        }
    }
    window_ns = best_w;
    CK(hipFree(out));
    CK(hipHostFree(word));
    return off;
}

static double pct(std::vector<double> v, double p) {
    if (v.empty()) return 0;
    std::sort(v.begin(), v.end());
    return v[std::min(v.size() - 1, size_t(p * (v.size() - 1) + 0.5))];
}

int main(int argc, char **argv) {
    if (argc < 6) {
        fprintf(stderr, "usage: %s <rs|cauchy|isal_rs> k m chunk calls [registered=1] [nd=1] [traced=1]\n", argv[0]);
        return 2;
    }
    const int fam = !strcmp(argv[1], "cauchy") ? MEC_CAUCHY_GOOD : !strcmp(argv[1], "isal_rs") ? MEC_ISAL_RS
                                                                                                 : MEC_RS_VANDERMONDE;
    const uint32_t k = atoi(argv[2]), m = atoi(argv[3]), cs = atoi(argv[4]);
    const int calls = atoi(argv[5]);
    const bool reg = argc > 6 ? atoi(argv[6]) != 0 : true;
    const uint32_t nd = argc > 7 ? uint32_t(atoi(argv[7])) : 1u;
    // traced = 0: no device stamps (the trace's own stores delay the done
    // store); only the host-side total and calls/s are reported
    const bool traced = argc > 8 ? atoi(argv[8]) != 0 : true;
    CK(hipSetDevice(0));
    int khz = 0;
    CK(hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, 0));
    const double ns_per_tick = 1e6 / double(khz);
    double window = 0;
    const double off = calibrate(ns_per_tick, window);

    mec_ctx *c = nullptr;
    MK(mec_create(fam, k, m, cs, 0, &c));
    MK(mec_set_host_queue(c, 8));
    MK(mec_queue_trace_enable(c, traced ? 1 : 0));
    const size_t slot = 8 + size_t(cs);  // ChunkPool slot: 8-byte header + data (chunk_pool.cc:22-47)
    const size_t bytes = ((k + m) * slot + 4095) / 4096 * 4096;
    uint8_t *slab = (uint8_t *)aligned_alloc(4096, bytes);
    for (size_t i = 0; i < bytes; ++i) slab[i] = uint8_t(i * 131 >> 3);
    if (reg) MK(mec_host_register(slab, bytes));
    std::vector<const uint8_t *> data(k);
    std::vector<uint8_t *> par(m, nullptr);
    for (uint32_t j = 0; j < k; ++j) data[j] = slab + j * slot + 8;
    std::vector<double> seg[9];
    const int warm = std::min(2000, calls / 4 + 1);
    uint64_t t_start = 0;
    for (int it = 0; it < warm + calls; ++it) {
        if (it == warm) t_start = mono_ns();
        for (uint32_t i = 0; i < m; ++i) par[i] = i < nd ? slab + (k + (it + i) % m) * slot + 8 : nullptr;
        const uint64_t a = mono_ns();
        MK(mec_encode_host(c, data.data(), par.data()));
        const uint64_t b = mono_ns();
        if (!traced) {
            if (it >= warm) seg[8].push_back(double(b - a) * 1e-3);
            continue;
        }
        mec_queue_trace tr;
        if (mec_queue_last_trace(&tr) != MEC_OK || it < warm) continue;  // launch path (no trace)
        const double take = double(tr.dev_take) * ns_per_tick - off;
        const double fence = double(tr.dev_fence) * ns_per_tick - off;
        const double desc = double(tr.dev_desc) * ns_per_tick - off;
        const double loaded = tr.dev_loaded ? double(tr.dev_loaded) * ns_per_tick - off : desc;
        const double end = double(tr.dev_end) * ns_per_tick - off;
        seg[0].push_back((double(tr.host_post_ns) - double(a)) * 1e-3);
        seg[1].push_back((take - double(tr.host_post_ns)) * 1e-3);
        seg[2].push_back((fence - take) * 1e-3);
        seg[3].push_back((desc - fence) * 1e-3);
        seg[4].push_back((loaded - desc) * 1e-3);
        seg[5].push_back((end - loaded) * 1e-3);
        seg[6].push_back((double(tr.host_seen_ns) - end) * 1e-3);
        seg[7].push_back((double(b) - double(tr.host_seen_ns)) * 1e-3);
        seg[8].push_back(double(b - a) * 1e-3);
    }
    const double dt = double(mono_ns() - t_start) * 1e-9;
    const char *names[9] = {"pre", "poll", "fence", "desc", "load", "code", "complete", "post", "total"};
    printf("{\"bench\": \"queue_latency\", \"family\": \"%s\", \"k\": %u, \"m\": %u, \"chunk\": %u, \"outputs\": %u, "
           "\"registered\": %d, \"calls\": %d, \"trace_on\": %d, \"traced\": %zu, \"calls_per_s\": %.1f, \"clock_window_us\": %.3f",
           argv[1], k, m, cs, nd, reg ? 1 : 0, calls, traced ? 1 : 0, seg[8].size(), calls / dt, window * 1e-3);
    for (int i = traced ? 0 : 8; i < 9; ++i)
        printf(", \"%s_us\": [%.3f, %.3f]", names[i], pct(seg[i], 0.5), pct(seg[i], 0.9));
    printf("}\n");
    if (reg) mec_host_unregister(slab);
    free(slab);
    mec_destroy(c);
    return 0;
}
