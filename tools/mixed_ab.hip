// mixed_ab.hip — the resident queue beside full-device launches in one
// process (the queue's grid holds up to half the device's
// resident workgroups and keeps spinning for MEC_QUEUE_IDLE_MS after a call,
// so device-memory launches of the same process may get only part of the
// CUs).  Three phases of `secs` seconds each:
//   launches  RS(10,4)@1 MiB encode of `stripes` device-resident stripes,
//             back to back on one stream (GB/s of the algorithmic bytes)
//   queue     W worker threads, single-stripe RS(8,2)@4 KiB encode(index)
//             calls on registered slabs through the resident queue (calls/s)
//   both      the two at once
//
//   mixed_ab [stripes=1024] [workers=4] [secs=3] [queue_slots=32]
#include <hip/hip_runtime.h>
#include <time.h>

#include <atomic>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <thread>
#include <vector>

#include "mec.h"

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

static double now() {
    timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return ts.tv_sec + ts.tv_nsec * 1e-9;
}

int main(int argc, char **argv) {
    const uint32_t stripes = argc > 1 ? atoi(argv[1]) : 1024;
    const int W = argc > 2 ? atoi(argv[2]) : 4;
    const double secs = argc > 3 ? atof(argv[3]) : 3.0;
    const uint32_t slots = argc > 4 ? atoi(argv[4]) : 32;
    CK(hipSetDevice(0));
    // device-resident encode: RS(10,4) @ 1 MiB (BASELINE configs[1] shape)
    const uint32_t K = 10, M = 4, CS = 1 << 20;
    mec_ctx *big = nullptr;
    MK(mec_create(MEC_RS_VANDERMONDE, K, M, CS, 0, &big));
    uint8_t *data = nullptr, *par = nullptr;
    CK(hipMalloc((void **)&data, size_t(stripes) * K * CS));
    CK(hipMalloc((void **)&par, size_t(stripes) * M * CS));
    MK(mec_fill_random(data, size_t(stripes) * K * CS, 7, 0, nullptr));
    hipStream_t st;
    CK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
    const double alg = double(stripes) * (K + M) * CS;
    // single-stripe queue calls: RS(8,2) @ 4 KiB on registered slabs
    const uint32_t k = 8, m = 2, cs = 4096;
    mec_ctx *small = nullptr;
    MK(mec_create(MEC_RS_VANDERMONDE, k, m, cs, 0, &small));
    MK(mec_set_host_queue(small, slots));
    std::atomic<int> phase(0);  // 0 idle, 1 run, 2 stop
    std::vector<uint64_t> calls(W, 0);
    std::vector<std::thread> th;
    for (int w = 0; w < W; ++w)
        th.emplace_back([&, w] {
            const size_t slot = 8 + cs, bytes = ((k + m) * slot + 4095) / 4096 * 4096;
            uint8_t *slab = (uint8_t *)aligned_alloc(4096, bytes);
            memset(slab, w + 1, bytes);
            MK(mec_host_register(slab, bytes));
            std::vector<const uint8_t *> d(k);
            std::vector<uint8_t *> p(m, nullptr);
            for (uint32_t j = 0; j < k; ++j) d[j] = slab + j * slot + 8;
            uint64_t it = 0;
            for (;;) {
                const int ph = phase.load(std::memory_order_relaxed);
                if (ph == 2) break;
                if (ph == 0) {
                    std::this_thread::yield();
                    continue;
                }
                for (uint32_t i = 0; i < m; ++i) p[i] = i == it % m ? slab + (k + i) * slot + 8 : nullptr;
                MK(mec_encode_host(small, d.data(), p.data()));
                calls[w]++;
                it++;
            }
            mec_host_unregister(slab);
            free(slab);
        });
    auto run_launches = [&](double dur, double &gbps) {
        hipEvent_t e0, e1;
        CK(hipEventCreate(&e0));
        CK(hipEventCreate(&e1));
        int n = 0;
        const double t0 = now();
        CK(hipEventRecord(e0, st));
        while (now() - t0 < dur) {
            MK(mec_encode(big, data, int64_t(K) * CS, CS, par, int64_t(M) * CS, CS, stripes, 0, st));
            ++n;
            if (n % 4 == 0) CK(hipStreamSynchronize(st));
        }
        CK(hipEventRecord(e1, st));
        CK(hipEventSynchronize(e1));
        float ms = 0;
        CK(hipEventElapsedTime(&ms, e0, e1));
        gbps = alg * n / (ms * 1e-3) / 1e9;
        CK(hipEventDestroy(e0));
        CK(hipEventDestroy(e1));
        return n;
    };
    auto count = [&] {
        uint64_t s = 0;
        for (auto c : calls) s += c;
        return s;
    };
    double g_alone = 0, g_mixed = 0;
    // warm both paths
    run_launches(0.5, g_alone);
    phase = 1;
    std::this_thread::sleep_for(std::chrono::milliseconds(300));
    phase = 0;
    std::this_thread::sleep_for(std::chrono::milliseconds(200));  // queue idles out (MEC_QUEUE_IDLE_MS)
    // launches alone
    run_launches(secs, g_alone);
    // queue alone
    uint64_t c0 = count();
    double t0 = now();
    phase = 1;
    std::this_thread::sleep_for(std::chrono::duration<double>(secs));
    phase = 0;
    const double q_alone = (count() - c0) / (now() - t0);
    std::this_thread::sleep_for(std::chrono::milliseconds(200));
    // both
    c0 = count();
    t0 = now();
    phase = 1;
    run_launches(secs, g_mixed);
    phase = 0;
    const double q_mixed = (count() - c0) / (now() - t0);
    phase = 2;
    for (auto &x : th) x.join();
    printf("{\"bench\": \"mixed_ab\", \"launch\": \"RS(10,4)@1MiB encode x %u stripes\", \"queue\": \"RS(8,2)@4KiB "
           "encode(index), %d workers, %u slots\", \"launch_GBps_alone\": %.1f, \"launch_GBps_mixed\": %.1f, "
           "\"launch_frac_alone\": %.4f, \"launch_frac_mixed\": %.4f, \"queue_calls_alone\": %.0f, "
           "\"queue_calls_mixed\": %.0f}\n",
           stripes, W, slots, g_alone, g_mixed, g_alone / 8000.0, g_mixed / 8000.0, q_alone, q_mixed);
    mec_destroy(small);
    mec_destroy(big);
    CK(hipFree(data));
    CK(hipFree(par));
    return 0;
}
