// bar_probe.hip — experiment (single-caller latency): can the
// queue's slot (sequence word + descriptor) live in device memory that the
// host writes through the PCIe BAR, so part 0 polls HBM and reads the
// descriptor from HBM instead of crossing PCIe twice?
//
// For each flag placement — pinned host memory (the product today),
// fine-grained device memory (hipExtMallocWithFlags Finegrained), plain
// device memory (hipMalloc) — if the CPU can store to it (checked under a
// SIGSEGV guard):
//   ping   host stores i into `in`, a one-wave kernel polling `in`
//          (system-scope relaxed loads, bounded) stores i into `out` (pinned
//          host memory), the host spins on `out`: median round trip, 2000
//          rounds
//   desc   the kernel reads a 512-byte block at `in` (32 lanes x 16 B) and
//          times it with s_memrealtime (median of 256)
// Every loop on the device is bounded (a missed flag ends the kernel with a
// count of misses).
//
//   bar_probe [rounds=2000]
#include <hip/hip_runtime.h>
#include <setjmp.h>
#include <signal.h>
#include <time.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#define CK(x)                                                                  \
    do {                                                                       \
        hipError_t e_ = (x);                                                   \
        if (e_ != hipSuccess) {                                                \
            fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));            \
            exit(1);                                                           \
        }                                                                      \
    } while (0)

static uint64_t mono_ns() {
    timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return uint64_t(ts.tv_sec) * 1000000000ull + uint64_t(ts.tv_nsec);
}

static sigjmp_buf g_jb;
static void on_segv(int) { siglongjmp(g_jb, 1); }

// true if the CPU can store to and load from p
static bool cpu_can_touch(volatile uint32_t *p) {
    struct sigaction sa {}, old {};
    sa.sa_handler = on_segv;
    sigemptyset(&sa.sa_mask);
    sigaction(SIGSEGV, &sa, &old);
    sigaction(SIGBUS, &sa, nullptr);
    bool ok = false;
    if (sigsetjmp(g_jb, 1) == 0) {
        p[0] = 0x5a5a1234u;
        ok = p[0] == 0x5a5a1234u;
    }
    sigaction(SIGSEGV, &old, nullptr);
    signal(SIGBUS, SIG_DFL);
    return ok;
}

// rounds of: wait for *in == i (bounded), then *out = i
__global__ void ping_kernel(const uint32_t *in, uint32_t *out, int rounds, uint32_t *misses) {
    if (threadIdx.x != 0) return;
    uint32_t miss = 0;
    for (int i = 1; i <= rounds; ++i) {
        const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
        while (__hip_atomic_load(in, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) != uint32_t(i)) {
            if (__builtin_amdgcn_s_memrealtime() - t0 > 100000) {  // 1 ms at 100 MHz: give up on this round
                ++miss;
                break;
            }
        }
        __hip_atomic_store(out, uint32_t(i), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
    misses[0] = miss;
}

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

// 32 lanes read 16 B each of `in` (512 B), n times; lane 0 records the ticks
__global__ void desc_kernel(const u32x4 *in, uint64_t *ticks, uint32_t *sink, int n) {
    uint32_t acc = 0;
    for (int i = 0; i < n; ++i) {
        const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
        u32x4 v{0, 0, 0, 0};
        if (threadIdx.x < 32) {
            // system scope: must not hit a stale L2 line (the host writes it)
            const uint32_t *p = reinterpret_cast<const uint32_t *>(in + threadIdx.x);
            v.x = __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            v.y = __hip_atomic_load(p + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            v.z = __hip_atomic_load(p + 2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            v.w = __hip_atomic_load(p + 3, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        }
        acc ^= v.x ^ v.y ^ v.z ^ v.w;
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        const uint64_t t1 = __builtin_amdgcn_s_memrealtime();
        if (threadIdx.x == 0) ticks[i] = t1 - t0;
    }
    sink[threadIdx.x] = acc;
}

// release cost: 256 lanes store `bytes` to pinned host memory (one job's
// output), wait for the acks, barrier, then thread 0 times a system-scope
// release fence (the L2 writeback the queue's done store pays) and the
// done store after it; n rounds, ticks of the fence and of the fence+store
__global__ void release_kernel(uint32_t *out, uint32_t words, uint32_t *done, uint64_t *ticks, int n) {
    for (int i = 0; i < n; ++i) {
        for (uint32_t w = threadIdx.x; w < words; w += blockDim.x) out[w] = uint32_t(i) ^ w;
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        if (threadIdx.x == 0) {
            const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
            const uint64_t t1 = __builtin_amdgcn_s_memrealtime();
            __hip_atomic_store(done, uint32_t(i), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            const uint64_t t2 = __builtin_amdgcn_s_memrealtime();
            ticks[2 * i] = t1 - t0;
            ticks[2 * i + 1] = t2 - t0;
        }
        __syncthreads();
    }
}

struct Place {
    const char *name;
    uint32_t *host;  // CPU address
    uint32_t *dev;   // device address
};

int main(int argc, char **argv) {
    const int rounds = argc > 1 ? atoi(argv[1]) : 2000;
    CK(hipSetDevice(0));
    int large_bar = -1;
    (void)hipDeviceGetAttribute(&large_bar, hipDeviceAttributeIsLargeBar, 0);
    std::vector<Place> places;
    {
        uint32_t *h = nullptr, *d = nullptr;
        CK(hipHostMalloc((void **)&h, 4096, hipHostMallocMapped | hipHostMallocCoherent));
        CK(hipHostGetDevicePointer((void **)&d, h, 0));
        places.push_back({"pinned_host", h, d});
    }
    {
        uint32_t *d = nullptr;
        CK(hipExtMallocWithFlags((void **)&d, 4096, hipDeviceMallocFinegrained));
        places.push_back({"device_finegrained", d, d});
    }
    {
        uint32_t *d = nullptr;
        CK(hipExtMallocWithFlags((void **)&d, 4096, hipDeviceMallocUncached));
        places.push_back({"device_uncached", d, d});
    }
    {
        uint32_t *d = nullptr;
        CK(hipMalloc((void **)&d, 4096));
        places.push_back({"device_coarse", d, d});
    }
    uint32_t *out_h = nullptr, *out_d = nullptr, *misses = nullptr, *sink = nullptr;
    uint64_t *ticks = nullptr;
    CK(hipHostMalloc((void **)&out_h, 64, hipHostMallocMapped | hipHostMallocCoherent));
    CK(hipHostGetDevicePointer((void **)&out_d, out_h, 0));
    CK(hipMalloc((void **)&misses, 64));
    CK(hipMalloc((void **)&sink, 4096));
    CK(hipMalloc((void **)&ticks, 256 * sizeof(uint64_t)));
    int clk_khz = 100000;
    (void)hipDeviceGetAttribute(&clk_khz, hipDeviceAttributeWallClockRate, 0);
    const double ns_per_tick = 1e6 / clk_khz;
    hipStream_t st;
    CK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
    for (const Place &pl : places) {
        hipPointerAttribute_t attr{};
        (void)hipPointerGetAttributes(&attr, pl.dev);
        const bool touch = cpu_can_touch(reinterpret_cast<volatile uint32_t *>(pl.host));
        printf("{\"place\": \"%s\", \"large_bar\": %d, \"mem_type\": %d, \"cpu_access\": %s", pl.name, large_bar,
               int(attr.type), touch ? "true" : "false");
        if (!touch) {
            printf("}\n");
            fflush(stdout);
            continue;
        }
        // desc: host fills the 512 B, the device times its read
        for (int i = 0; i < 128; ++i) reinterpret_cast<volatile uint32_t *>(pl.host)[i] = uint32_t(i * 2654435761u);
        __atomic_thread_fence(__ATOMIC_SEQ_CST);
        hipLaunchKernelGGL(desc_kernel, dim3(1), dim3(64), 0, st, reinterpret_cast<const u32x4 *>(pl.dev), ticks, sink,
                           256);
        CK(hipStreamSynchronize(st));
        std::vector<uint64_t> tk(256);
        CK(hipMemcpy(tk.data(), ticks, tk.size() * 8, hipMemcpyDeviceToHost));
        std::sort(tk.begin() + 1, tk.end());
        const double desc_us = tk[128] * ns_per_tick * 1e-3;
        // ping
        reinterpret_cast<volatile uint32_t *>(pl.host)[0] = 0;
        __atomic_store_n(out_h, 0u, __ATOMIC_SEQ_CST);
        CK(hipMemsetAsync(misses, 0, 4, st));
        hipLaunchKernelGGL(ping_kernel, dim3(1), dim3(64), 0, st, pl.dev, out_d, rounds, misses);
        std::vector<double> rt;
        rt.reserve(rounds);
        int host_miss = 0;
        for (int i = 1; i <= rounds; ++i) {
            const uint64_t t0 = mono_ns();
            __atomic_thread_fence(__ATOMIC_SEQ_CST);
            reinterpret_cast<volatile uint32_t *>(pl.host)[0] = uint32_t(i);
            __builtin_ia32_sfence();
            bool seen = false;
            while (mono_ns() - t0 < 5000000ull) {  // 5 ms
                if (__atomic_load_n(out_h, __ATOMIC_ACQUIRE) == uint32_t(i)) {
                    seen = true;
                    break;
                }
            }
            rt.push_back((mono_ns() - t0) * 1e-3);
            if (!seen && ++host_miss >= 5) break;  // the device does not see the flag: stop (its rounds time out)
        }
        CK(hipStreamSynchronize(st));
        uint32_t dmiss = 0;
        CK(hipMemcpy(&dmiss, misses, 4, hipMemcpyDeviceToHost));
        std::sort(rt.begin(), rt.end());
        printf(", \"desc512_us_median\": %.3f, \"ping_us_median\": %.3f, \"ping_us_p10\": %.3f, \"ping_us_p90\": %.3f, "
               "\"device_misses\": %u, \"host_misses\": %d}\n",
               desc_us, rt[rt.size() / 2], rt[rt.size() / 10], rt[rt.size() * 9 / 10], dmiss, host_miss);
        fflush(stdout);
    }
    // release cost after a 4 KiB job output to pinned host memory
    {
        uint32_t *oh = nullptr, *od = nullptr;
        CK(hipHostMalloc((void **)&oh, 1 << 16, hipHostMallocMapped | hipHostMallocCoherent));
        CK(hipHostGetDevicePointer((void **)&od, oh, 0));
        uint64_t *rt = nullptr;
        CK(hipMalloc((void **)&rt, 2 * 256 * sizeof(uint64_t)));
        for (uint32_t bytes : {4096u, 65536u}) {
            hipLaunchKernelGGL(release_kernel, dim3(1), dim3(256), 0, st, od, bytes / 4, out_d, rt, 256);
            CK(hipStreamSynchronize(st));
            std::vector<uint64_t> t(512);
            CK(hipMemcpy(t.data(), rt, t.size() * 8, hipMemcpyDeviceToHost));
            std::vector<double> f, fs;
            for (int i = 1; i < 256; ++i) {
                f.push_back(t[2 * i] * ns_per_tick * 1e-3);
                fs.push_back(t[2 * i + 1] * ns_per_tick * 1e-3);
            }
            std::sort(f.begin(), f.end());
            std::sort(fs.begin(), fs.end());
            printf("{\"release_after_output_bytes\": %u, \"release_fence_us_median\": %.3f, \"fence_plus_done_store_acked_us_median\": %.3f}\n",
                   bytes, f[f.size() / 2], fs[fs.size() / 2]);
            fflush(stdout);
        }
    }
    return 0;
}
