// gf_math.hpp — host-side GF(2^w) arithmetic, code-matrix construction and
// decode planning for libmec.  Clean-room C++; produces the
// same matrices as the reference (pinned by tests/golden) and caches nothing
// itself — the context caches plans per erasure pattern.
#pragma once

#include <cstdint>
#include <string>
#include <vector>

namespace mec {

// GF(2^w), 1 <= w <= 8, with gf_complete's default polynomials
// (gf_w4.c:2045, gf_w8.c:2376, gf_wgen.c:936-944).
class Field {
public:
    static const Field &get(int w);
    int w() const { return w_; }
    int size() const { return 1 << w_; }
    uint8_t mul(unsigned a, unsigned b) const { return mul_[(a << w_) | b]; }
    uint8_t inv(unsigned a) const { return inv_[a]; }
    uint8_t div(unsigned a, unsigned b) const { return mul(a, inv(b)); }
    // Ones in the w x w GF(2) matrix of "multiply by c" (cauchy_n_ones).
    int ones(unsigned c) const;

private:
    explicit Field(int w);
    int w_;
    std::vector<uint8_t> mul_, inv_;
};

using Mat = std::vector<uint8_t>;  // row-major, entries in GF(2^w)

// Reference getW rules (rscoding.cc:189-220, cauchycoding.cc:182-205).
int rs_getw(uint32_t k, uint32_t m, uint32_t chunk);
int cauchy_getw(uint32_t k, uint32_t m, uint32_t chunk);

// Jerasure reed_sol_vandermonde_coding_matrix (w = 8): m x k.
bool jerasure_rs_matrix(int k, int m, Mat &out);
// Jerasure cauchy_good_general_coding_matrix: m x k over GF(2^w).
bool jerasure_cauchy_matrix(int k, int m, int w, Mat &out);
// ISA-L gf_gen_rs_matrix / gf_gen_cauchy1_matrix: (k+m) x k, identity on top.
Mat isal_rs_matrix(int k, int m);
Mat isal_cauchy_matrix(int k, int m);

// n x n inverse by Gauss-Jordan; false if singular.
bool invert(const Mat &a, int n, const Field &f, Mat &inv);
// (r x n) * (n x c)
Mat matmul(const Mat &a, const Mat &b, int r, int n, int c, const Field &f);

// outputs = coef (dst.size() x src.size()) * sources, over GF(2^w).
struct LinearPlan {
    std::vector<int> src;  // chunk indices read
    std::vector<int> dst;  // chunk indices written
    Mat coef;
};

// Decode plans reproducing the reference plugin's arithmetic exactly:
//  * Jerasure RS: jerasure_matrix_decode with row_k_ones = 1
//    (jerasure.c:167-268): survivors = first k present chunks; the last
//    erased data chunk via coding row 0 when it is present.
//  * Jerasure Cauchy: jerasure_schedule_decode_lazy (jerasure.c:947-973,
//    718-945): erased data i is replaced by the lowest unused present coding
//    chunk; the (bit)matrix is the inverse of that selection.
//  * ISA-L: first k present chunks (rscoding.cc:155-177); erased parity
//    uses encode_row x inverse (the reference's parity rows are a bug).
// A = coding matrix (m x k) for Jerasure, (k+m) x k for ISA-L.
enum class Scheme { kJerasureRS, kJerasureCauchy, kIsal };
int plan_decode(Scheme s, const Mat &A, int k, int m, int w, uint64_t present,
                LinearPlan &plan, std::string &err);

}  // namespace mec
