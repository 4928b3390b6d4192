// wide_r8_probe.hip — experiment: the wide (m > 4) one-pass kernel with
// row groups of 4 (libmec's choice) against one group of 8 rows.  R = 8
// extracts each source's bit fields once instead of twice but runs at
// 160-180 VGPRs (2-3 waves per SIMD) against 128-150 (3-4).  Same
// gf8_mg_kernel body (gf8_kernel.hpp), same permute-table image (row r of
// the image is row r whatever the group size when rows % R == 0), the
// product's launch rules otherwise; the outputs of both arms are compared.
//
//   wide_r8_probe [stripes=16384] [rounds=3]
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#include "gf8_kernel.hpp"
#include "mec.h"

using namespace mec;
using namespace mec::detail;

#define CK(x)                                                                  \
    do {                                                                       \
        hipError_t e_ = (x);                                                   \
        if (e_ != hipSuccess) {                                                \
            fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));            \
            exit(1);                                                           \
        }                                                                      \
    } while (0)

template <int K>
float time_arm(int R, const Gf8MgLaunch &L) {
    auto go = [&] { return R == 8 ? run_gf8_mg<K, 8>(L, 0) : run_gf8_mg<K, 4>(L, 0); };
    CK(go());
    CK(hipDeviceSynchronize());
    float best = 1e30f;
    for (int r = 0; r < 5; ++r) {
        hipEvent_t e0, e1;
        CK(hipEventCreate(&e0));
        CK(hipEventCreate(&e1));
        CK(hipEventRecord(e0, 0));
        CK(go());
        CK(hipEventRecord(e1, 0));
        CK(hipEventSynchronize(e1));
        float ms = 0;
        CK(hipEventElapsedTime(&ms, e0, e1));
        best = ms < best ? ms : best;
        CK(hipEventDestroy(e0));
        CK(hipEventDestroy(e1));
    }
    return best;
}

template <int K>
void shape(int family, const char *name, uint32_t n, int rounds) {
    constexpr int M = 8;
    const uint64_t CS = 65536;
    mec_ctx *c = nullptr;
    if (mec_create(family, K, M, uint32_t(CS), 0, &c) != MEC_OK) {
        fprintf(stderr, "%s\n", mec_last_error());
        exit(1);
    }
    std::vector<int32_t> A(size_t(K + M) * K);
    const int na = mec_get_matrix(c, A.data(), A.size());
    const int off = na == K * M ? 0 : K * K;  // ISA-L matrices carry the identity on top
    std::vector<uint8_t> coef(size_t(M) * K);
    for (int i = 0; i < M * K; ++i) coef[size_t(i)] = uint8_t(A[size_t(off + i)]);
    std::vector<uint32_t> img;
    gf8_mg_tables(coef.data(), M, K, 8, img);  // M % 8 == 0: the same image at R = 4
    uint32_t *tabs = nullptr;
    CK(hipMalloc((void **)&tabs, img.size() * 4));
    CK(hipMemcpy(tabs, img.data(), img.size() * 4, hipMemcpyHostToDevice));
    uint8_t *data = nullptr, *p4 = nullptr, *p8 = nullptr;
    CK(hipMalloc((void **)&data, size_t(n) * K * CS));
    CK(hipMalloc((void **)&p4, size_t(n) * M * CS));
    CK(hipMalloc((void **)&p8, size_t(n) * M * CS));
    mec_fill_random(data, size_t(n) * K * CS, 3, 0, nullptr);
    Gf8MgLaunch L{};
    L.src = data;
    L.src_stripe_stride = int64_t(K) * CS;
    L.dst_stripe_stride = int64_t(M) * CS;
    for (int j = 0; j < K; ++j) L.src_off[j] = int64_t(j) * CS;
    for (int r = 0; r < M; ++r) L.dst_off[r] = int64_t(r) * CS;
    L.k = K;
    L.rows = M;
    L.len = CS;
    L.n_stripes = n;
    L.accumulate = false;
    L.vand = family != MEC_ISAL_CAUCHY;
    L.tabs = tabs;
    const double alg = double(n) * (K + M) * CS;
    for (int rd = 0; rd < rounds; ++rd)
        for (int R : {4, 8}) {
            L.dst = R == 8 ? p8 : p4;
            L.group_rows = R;
            const float ms = time_arm<K>(R, L);
            printf("{\"round\": %d, \"shape\": \"%s\", \"R\": %d, \"ms\": %.4f, \"frac\": %.4f}\n", rd, name, R, ms,
                   alg / (ms * 1e-3) / 8e12);
            fflush(stdout);
        }
    std::vector<uint8_t> a(size_t(n) * M * CS), b(a.size());
    CK(hipMemcpy(a.data(), p4, a.size(), hipMemcpyDeviceToHost));
    CK(hipMemcpy(b.data(), p8, b.size(), hipMemcpyDeviceToHost));
    printf("{\"shape\": \"%s\", \"outputs_equal\": %s}\n", name, a == b ? "true" : "false");
    CK(hipFree(data));
    CK(hipFree(p4));
    CK(hipFree(p8));
    CK(hipFree(tabs));
    mec_destroy(c);
}

int main(int argc, char **argv) {
    const uint32_t n = argc > 1 ? atoi(argv[1]) : 16384;
    const int rounds = argc > 2 ? atoi(argv[2]) : 3;
    CK(hipSetDevice(0));
    shape<16>(MEC_RS_VANDERMONDE, "RS(16,8)@64KiB encode", n, rounds);
    shape<12>(MEC_ISAL_RS, "ISA-L RS(12,8)@64KiB encode", n, rounds);
    shape<12>(MEC_ISAL_CAUCHY, "ISA-L Cauchy(12,8)@64KiB encode", n, rounds);
    shape<10>(MEC_RS_VANDERMONDE, "RS(10,8)@64KiB encode", n, rounds);
    shape<16>(MEC_ISAL_CAUCHY, "ISA-L Cauchy(16,8)@64KiB encode", n, rounds);
    shape<20>(MEC_RS_VANDERMONDE, "RS(20,8)@64KiB encode", n / 2, rounds);
    shape<20>(MEC_ISAL_CAUCHY, "ISA-L Cauchy(20,8)@64KiB encode", n / 2, rounds);
    return 0;
}
