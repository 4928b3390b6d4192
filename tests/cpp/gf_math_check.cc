// gf_math_check.cc — host-side check of libmec's decode planning
// (memec_amd/csrc/gf_math.cpp), built with AddressSanitizer and UBSan by
// tests/test_host_sanitized.py.
//
// For every code family and every (k, m) with k + m <= 32 (RS: w = 8;
// Cauchy: every w from the smallest with 2^w >= k + m up to 8), random
// symbols are encoded with the family's matrix, erasure patterns are
// applied (all of them for small codes, a random sample otherwise), and the
// plan from plan_decode must rebuild exactly the erased symbols from the
// chunks it names.  Patterns with more than m erasures must be refused.
// Prints "ok <plans checked>" and exits 0, or the first failure and 1.
#include <cstdio>
#include <cstdlib>
#include <random>
#include <string>
#include <vector>

#include "gf_math.hpp"
#include "mec.h"

using namespace mec;

namespace {

constexpr int kSymbols = 6;  // symbols per chunk

struct Code {
    Scheme s;
    const char *name;
    int k, m, w;
    Mat A;  // m x k (Jerasure) or (k+m) x k (ISA-L)
    uint8_t coef(int i, int j) const { return s == Scheme::kIsal ? A[size_t(k + i) * k + j] : A[size_t(i) * k + j]; }
};

long checked = 0;

bool check_pattern(const Code &c, const std::vector<std::vector<uint8_t>> &chunks, uint64_t present) {
    const int n = c.k + c.m;
    LinearPlan plan;
    std::string err;
    const int rc = plan_decode(c.s, c.A, c.k, c.m, c.w, present, plan, err);
    const int erased = n - __builtin_popcountll(present & ((uint64_t(1) << n) - 1));
    if (erased > c.m) {
        if (rc == MEC_OK) {
            std::printf("FAIL %s k=%d m=%d w=%d: %d erasures accepted\n", c.name, c.k, c.m, c.w, erased);
            return false;
        }
        return true;
    }
    if (rc != MEC_OK) {
        // ISA-L's gf_gen_rs_matrix is not MDS for every (k, m): a singular
        // survivor set is reported, not mis-decoded
        if (c.s == Scheme::kIsal && rc == MEC_ESINGULAR) return true;
        std::printf("FAIL %s k=%d m=%d w=%d present=%llx: %s\n", c.name, c.k, c.m, c.w,
                    (unsigned long long)present, err.c_str());
        return false;
    }
    const Field &f = Field::get(c.w);
    for (int i : plan.src)
        if (!(present >> i & 1)) {
            std::printf("FAIL %s: plan reads erased chunk %d\n", c.name, i);
            return false;
        }
    for (size_t r = 0; r < plan.dst.size(); ++r)
        for (int t = 0; t < kSymbols; ++t) {
            uint8_t v = 0;
            for (size_t q = 0; q < plan.src.size(); ++q)
                v ^= f.mul(plan.coef[r * plan.src.size() + q], chunks[plan.src[q]][t]);
            if (v != chunks[plan.dst[r]][t]) {
                std::printf("FAIL %s k=%d m=%d w=%d present=%llx: chunk %d symbol %d\n", c.name, c.k, c.m, c.w,
                            (unsigned long long)present, plan.dst[r], t);
                return false;
            }
        }
    // every erased chunk is rebuilt
    for (int i = 0; i < n; ++i) {
        if (present >> i & 1) continue;
        bool found = false;
        for (int d : plan.dst) found |= d == i;
        if (!found) {
            std::printf("FAIL %s: erased chunk %d not rebuilt\n", c.name, i);
            return false;
        }
    }
    ++checked;
    return true;
}

bool check_code(const Code &c, std::mt19937_64 &rng) {
    const int n = c.k + c.m;
    const Field &f = Field::get(c.w);
    std::vector<std::vector<uint8_t>> chunks(n, std::vector<uint8_t>(kSymbols));
    for (int j = 0; j < c.k; ++j)
        for (auto &x : chunks[j]) x = uint8_t(rng() % unsigned(f.size()));
    for (int i = 0; i < c.m; ++i)
        for (int t = 0; t < kSymbols; ++t) {
            uint8_t v = 0;
            for (int j = 0; j < c.k; ++j) v ^= f.mul(c.coef(i, j), chunks[j][t]);
            chunks[c.k + i][t] = v;
        }
    const uint64_t full = (uint64_t(1) << n) - 1;
    if (n <= 10) {  // every pattern, too-many ones included
        for (uint64_t present = 0; present <= full; ++present)
            if (!check_pattern(c, chunks, present)) return false;
        return true;
    }
    for (int trial = 0; trial < 24; ++trial) {
        const int e = 1 + int(rng() % unsigned(c.m + 1));  // up to m + 1 erasures
        uint64_t present = full;
        for (int q = 0; q < e;) {
            const int i = int(rng() % unsigned(n));
            if (present >> i & 1) {
                present &= ~(uint64_t(1) << i);
                ++q;
            }
        }
        if (!check_pattern(c, chunks, present)) return false;
    }
    return true;
}

}  // namespace

int main() {
    std::mt19937_64 rng(2024);
    for (int k = 1; k < 32; ++k)
        for (int m = 1; k + m <= 32; ++m) {
            Code rs{Scheme::kJerasureRS, "jerasure-rs", k, m, 8, {}};
            if (!jerasure_rs_matrix(k, m, rs.A)) {
                std::printf("FAIL no RS matrix k=%d m=%d\n", k, m);
                return 1;
            }
            if (!check_code(rs, rng)) return 1;
            int w0 = 1;
            while ((1 << w0) < k + m) ++w0;
            for (int w = w0; w <= 8; ++w) {
                Code cr{Scheme::kJerasureCauchy, "jerasure-cauchy", k, m, w, {}};
                if (!jerasure_cauchy_matrix(k, m, w, cr.A)) {
                    std::printf("FAIL no Cauchy matrix k=%d m=%d w=%d\n", k, m, w);
                    return 1;
                }
                if (!check_code(cr, rng)) return 1;
            }
            Code ir{Scheme::kIsal, "isal-rs", k, m, 8, isal_rs_matrix(k, m)};
            if (!check_code(ir, rng)) return 1;
            Code ic{Scheme::kIsal, "isal-cauchy", k, m, 8, isal_cauchy_matrix(k, m)};
            if (!check_code(ic, rng)) return 1;
        }
    std::printf("ok %ld\n", checked);
    return 0;
}
