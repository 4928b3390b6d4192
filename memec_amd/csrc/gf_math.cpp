// gf_math.cpp — see gf_math.hpp.
#include "gf_math.hpp"

#include <algorithm>
#include <array>
#include <mutex>
#include <numeric>

#include "mec.h"

namespace mec {

namespace {
// gf_complete defaults incl. the x^w term.
constexpr int kPoly[9] = {0, 0x3, 0x7, 0xb, 0x13, 0x25, 0x43, 0x89, 0x11d};

unsigned slow_mul(unsigned a, unsigned b, int w) {
    unsigned r = 0;
    for (int i = 0; i < w; ++i)
        if (b >> i & 1) r ^= a << i;
    for (int i = 2 * w - 2; i >= w; --i)
        if (r >> i & 1) r ^= unsigned(kPoly[w]) << (i - w);
    return r;
}
}  // namespace

Field::Field(int w) : w_(w), mul_(size_t(1) << (2 * w)), inv_(size_t(1) << w, 0) {
    const unsigned n = 1u << w;
    for (unsigned a = 0; a < n; ++a)
        for (unsigned b = 0; b < n; ++b) {
            unsigned p = slow_mul(a, b, w);
            mul_[(a << w) | b] = uint8_t(p);
            if (p == 1) inv_[a] = uint8_t(b);
        }
}

const Field &Field::get(int w) {
    static std::once_flag once[9];
    static Field *fields[9];
    std::call_once(once[w], [w] { fields[w] = new Field(w); });
    return *fields[w];
}

int Field::ones(unsigned c) const {
    int n = 0;
    for (int x = 0; x < w_; ++x) {
        n += __builtin_popcount(c);
        c = mul(c, 2 % size());
    }
    return n;
}

static int log2_ceil(uint32_t n) {
    int w = 1;
    while ((1u << w) < n) ++w;
    return w;
}

int rs_getw(uint32_t k, uint32_t m, uint32_t chunk) {
    int w = log2_ceil(k + m);
    w = w < 8 ? 8 : w < 16 ? 16 : w < 32 ? 32 : -1;
    if (w < 0 || chunk % uint32_t(w)) return -1;
    return w;
}

int cauchy_getw(uint32_t k, uint32_t m, uint32_t chunk) {
    for (int w = log2_ceil(k + m); w <= 32; ++w)
        if (chunk % uint32_t(w) == 0) return w;
    return -1;
}

// ---------------------------------------------------------------------------
// Jerasure RS: systematic distribution matrix derived from the extended
// Vandermonde matrix by column operations (reed_sol.c:175-300).  The steps
// (pivot choice, column scaling, elimination, the two normalisations) are
// what make the matrix unique, so they are followed exactly.
// ---------------------------------------------------------------------------
bool jerasure_rs_matrix(int k, int m, Mat &out) {
    const Field &f = Field::get(8);
    const int R = k + m, C = k;
    if (k < 1 || m < 1 || R > 256) return false;
    std::vector<std::array<uint8_t, 256>> V(R);
    for (auto &row : V) row.fill(0);
    V[0][0] = 1;
    if (R > 1) V[R - 1][C - 1] = 1;
    for (int r = 1; r < R - 1; ++r) {
        uint8_t p = 1;
        for (int c = 0; c < C; ++c) {
            V[r][c] = p;
            p = f.mul(p, unsigned(r));
        }
    }
    auto scale_col = [&](int c, uint8_t s, int from) {
        for (int r = from; r < R; ++r) V[r][c] = f.mul(s, V[r][c]);
    };
    auto axpy_col = [&](int dstc, int srcc, uint8_t e) {  // col dst += e * col src
        for (int r = 0; r < R; ++r) V[r][dstc] ^= f.mul(e, V[r][srcc]);
    };
    for (int i = 1; i < C; ++i) {
        int piv = i;
        while (piv < R && V[piv][i] == 0) ++piv;
        if (piv == R) return false;
        if (piv != i) std::swap(V[piv], V[i]);
        if (V[i][i] != 1) scale_col(i, f.inv(V[i][i]), 0);
        for (int c = 0; c < C; ++c)
            if (c != i && V[i][c] != 0) axpy_col(c, i, V[i][c]);
    }
    for (int c = 0; c < C; ++c)  // row C becomes all ones (rows >= C only)
        if (V[C][c] != 1) scale_col(c, f.inv(V[C][c]), C);
    for (int r = C + 1; r < R; ++r)  // first column becomes all ones
        if (V[r][0] != 1) {
            uint8_t s = f.inv(V[r][0]);
            for (int c = 0; c < C; ++c) V[r][c] = f.mul(V[r][c], s);
        }
    out.assign(size_t(m) * k, 0);
    for (int i = 0; i < m; ++i)
        for (int j = 0; j < k; ++j) out[size_t(i) * k + j] = V[C + i][j];
    return true;
}

// ---------------------------------------------------------------------------
// Jerasure Cauchy "good" matrix (cauchy.c:131-238).
// m == 2 uses the cbest lists, which are the nonzero field elements ordered
// by (bitmatrix ones, value) (checked against the reference for w = 2..8).
// ---------------------------------------------------------------------------
bool jerasure_cauchy_matrix(int k, int m, int w, Mat &out) {
    if (w < 1 || w > 8 || k < 1 || m < 1) return false;
    const Field &f = Field::get(w);
    const int n = f.size();
    out.assign(size_t(m) * k, 0);
    if (m == 2 && w >= 2 && k <= n - 1) {
        std::vector<int> best(n - 1);
        std::iota(best.begin(), best.end(), 1);
        std::stable_sort(best.begin(), best.end(), [&](int a, int b) {
            int oa = f.ones(a), ob = f.ones(b);
            return oa != ob ? oa < ob : a < b;
        });
        for (int j = 0; j < k; ++j) {
            out[j] = 1;
            out[k + j] = uint8_t(best[j]);
        }
        return true;
    }
    if (k + m > n) return false;
    for (int i = 0; i < m; ++i)
        for (int j = 0; j < k; ++j) out[size_t(i) * k + j] = f.inv(unsigned(i ^ (m + j)));
    for (int j = 0; j < k; ++j) {  // columns scaled so row 0 is ones
        uint8_t s = f.inv(out[j]);
        if (out[j] == 1) continue;
        for (int i = 0; i < m; ++i) out[size_t(i) * k + j] = f.mul(out[size_t(i) * k + j], s);
    }
    for (int i = 1; i < m; ++i) {  // each later row: divide by its best element
        uint8_t *row = &out[size_t(i) * k];
        auto row_ones = [&](uint8_t s) {
            int t = 0;
            for (int j = 0; j < k; ++j) t += f.ones(f.mul(row[j], s));
            return t;
        };
        int best = row_ones(1), best_j = -1;
        for (int j = 0; j < k; ++j) {
            if (row[j] == 1) continue;
            int t = row_ones(f.inv(row[j]));
            if (t < best) { best = t; best_j = j; }
        }
        if (best_j >= 0) {
            uint8_t s = f.inv(row[best_j]);
            for (int j = 0; j < k; ++j) row[j] = f.mul(row[j], s);
        }
    }
    return true;
}

Mat isal_rs_matrix(int k, int m) {
    const Field &f = Field::get(8);
    Mat a(size_t(k + m) * k, 0);
    for (int i = 0; i < k; ++i) a[size_t(i) * k + i] = 1;
    uint8_t gen = 1;
    for (int i = k; i < k + m; ++i) {
        uint8_t p = 1;
        for (int j = 0; j < k; ++j) {
            a[size_t(i) * k + j] = p;
            p = f.mul(p, gen);
        }
        gen = f.mul(gen, 2);
    }
    return a;
}

Mat isal_cauchy_matrix(int k, int m) {
    const Field &f = Field::get(8);
    Mat a(size_t(k + m) * k, 0);
    for (int i = 0; i < k; ++i) a[size_t(i) * k + i] = 1;
    for (int i = k; i < k + m; ++i)
        for (int j = 0; j < k; ++j) a[size_t(i) * k + j] = f.inv(unsigned(i ^ j));
    return a;
}

bool invert(const Mat &a, int n, const Field &f, Mat &inv) {
    Mat t(a);
    inv.assign(size_t(n) * n, 0);
    for (int i = 0; i < n; ++i) inv[size_t(i) * n + i] = 1;
    auto row = [n](Mat &x, int r) { return &x[size_t(r) * n]; };
    for (int c = 0; c < n; ++c) {
        int p = c;
        while (p < n && row(t, p)[c] == 0) ++p;
        if (p == n) return false;
        if (p != c)
            for (int j = 0; j < n; ++j) {
                std::swap(row(t, p)[j], row(t, c)[j]);
                std::swap(row(inv, p)[j], row(inv, c)[j]);
            }
        uint8_t s = f.inv(row(t, c)[c]);
        for (int j = 0; j < n; ++j) {
            row(t, c)[j] = f.mul(row(t, c)[j], s);
            row(inv, c)[j] = f.mul(row(inv, c)[j], s);
        }
        for (int r = 0; r < n; ++r) {
            uint8_t e = row(t, r)[c];
            if (r == c || e == 0) continue;
            for (int j = 0; j < n; ++j) {
                row(t, r)[j] ^= f.mul(e, row(t, c)[j]);
                row(inv, r)[j] ^= f.mul(e, row(inv, c)[j]);
            }
        }
    }
    return true;
}

Mat matmul(const Mat &a, const Mat &b, int r, int n, int c, const Field &f) {
    Mat out(size_t(r) * c, 0);
    for (int i = 0; i < r; ++i)
        for (int t = 0; t < n; ++t) {
            uint8_t e = a[size_t(i) * n + t];
            if (!e) continue;
            for (int j = 0; j < c; ++j) out[size_t(i) * c + j] ^= f.mul(e, b[size_t(t) * c + j]);
        }
    return out;
}

// ---------------------------------------------------------------------------
// Decode planning.  Every chunk value is tracked as a linear form over the
// chosen sources; the plan's rows are the forms of the erased chunks.
// ---------------------------------------------------------------------------
int plan_decode(Scheme s, const Mat &A, int k, int m, int w, uint64_t present,
                LinearPlan &plan, std::string &err) {
    const int n = k + m;
    const Field &f = Field::get(w);
    std::vector<bool> erased(n);
    int ne = 0;
    for (int i = 0; i < n; ++i) {
        erased[i] = !(present >> i & 1);
        ne += erased[i];
    }
    plan = LinearPlan{};
    if (ne > m) {
        err = "Too many failure to recover (" + std::to_string(ne) + ">" + std::to_string(m) + ")";
        return MEC_ETOOMANY;
    }
    if (ne == 0) return MEC_OK;
    for (int i = 0; i < n; ++i)
        if (erased[i]) plan.dst.push_back(i);

    if (s == Scheme::kJerasureCauchy) {
        // sources: data i, or (if erased) the lowest unused present coding chunk
        int next = k;
        for (int i = 0; i < k; ++i) {
            if (!erased[i]) { plan.src.push_back(i); continue; }
            while (erased[next]) ++next;
            plan.src.push_back(next++);
        }
    } else {
        for (int i = 0; i < n && int(plan.src.size()) < k; ++i)
            if (!erased[i]) plan.src.push_back(i);
    }
    // generator rows of the sources (k x k), in source order
    auto gen_row = [&](int chunk, uint8_t *dst) {
        if (s == Scheme::kIsal) {
            std::copy_n(&A[size_t(chunk) * k], k, dst);
        } else if (chunk < k) {
            std::fill_n(dst, k, 0);
            dst[chunk] = 1;
        } else {
            std::copy_n(&A[size_t(chunk - k) * k], k, dst);
        }
    };
    Mat G(size_t(k) * k), Ginv;
    for (int i = 0; i < k; ++i) gen_row(plan.src[i], &G[size_t(i) * k]);

    // forms[c] = coefficients over the k sources for chunk c's value
    std::vector<Mat> form(n);
    std::vector<int> pos(n, -1);
    for (int i = 0; i < k; ++i) {
        pos[plan.src[i]] = i;
        form[plan.src[i]].assign(k, 0);
        form[plan.src[i]][i] = 1;
    }
    auto need_inverse = [&]() -> bool {
        if (!Ginv.empty()) return true;
        if (!invert(G, k, f, Ginv)) {
            err = "decoding matrix is singular";
            return false;
        }
        return true;
    };
    bool broken = false;
    auto combine = [&](const uint8_t *coef, const int *ids) {  // sum coef[t] * form[ids[t]]
        Mat r(k, 0);
        for (int t = 0; t < k; ++t) {
            if (!coef[t]) continue;
            const Mat &fm = form[ids[t]];
            if (fm.size() != size_t(k)) { broken = true; continue; }
            for (int j = 0; j < k; ++j) r[j] ^= f.mul(coef[t], fm[j]);
        }
        return r;
    };
    std::vector<int> ident(k);
    std::iota(ident.begin(), ident.end(), 0);

    if (s == Scheme::kJerasureRS) {
        int edd = 0, last = k;
        for (int i = 0; i < k; ++i)
            if (erased[i]) { ++edd; last = i; }
        if (erased[k]) last = k;
        if (edd > 1 || (edd > 0 && erased[k]))
            if (!need_inverse()) return MEC_ESINGULAR;
        for (int i = 0; edd > 0 && i < last; ++i)
            if (erased[i]) {
                form[i].assign(Ginv.begin() + size_t(i) * k, Ginv.begin() + size_t(i + 1) * k);
                --edd;
            }
        if (edd > 0) {  // last erased data drive from coding row 0 (row_k_ones)
            std::vector<int> ids(k);
            for (int t = 0; t < k; ++t) ids[t] = t < last ? t : t + 1;
            form[last] = combine(&A[0], ids.data());
        }
        for (int i = 0; i < m; ++i)
            if (erased[k + i]) form[k + i] = combine(&A[size_t(i) * k], ident.data());
    } else {
        bool data_lost = false;
        for (int i = 0; i < k; ++i) data_lost |= erased[i];
        if (data_lost || s == Scheme::kIsal) {
            if (!need_inverse()) return MEC_ESINGULAR;
            // data chunk d = row d of G^-1 (columns are source positions)
            for (int d = 0; d < k; ++d)
                if (erased[d] || s == Scheme::kIsal)
                    form[d].assign(Ginv.begin() + size_t(d) * k, Ginv.begin() + size_t(d + 1) * k);
        }
        for (int c = k; c < n; ++c)
            if (erased[c]) {
                const uint8_t *row = s == Scheme::kIsal ? &A[size_t(c) * k] : &A[size_t(c - k) * k];
                form[c] = combine(row, ident.data());
            }
    }
    if (broken) {
        err = "internal: decode form references an unknown chunk";
        return MEC_EINVAL;
    }
    plan.coef.assign(plan.dst.size() * size_t(k), 0);
    for (size_t r = 0; r < plan.dst.size(); ++r)
        std::copy_n(form[plan.dst[r]].begin(), k, plan.coef.begin() + r * k);
    return MEC_OK;
}

}  // namespace mec
