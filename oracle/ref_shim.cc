// ref_shim.cc — C entry points over the REAL reference coding path.
//
// TEST INFRASTRUCTURE ONLY.  Compiled by oracle/ref.mk against the reference
// sources where they lie under /root/reference (nothing is copied into this
// repo); the output goes to oracle/_ref/ (git-ignored).  Used in this
// container to generate tests/golden/ fixtures and to cross-check the C
// restatement in oracle/oracle.c, and (prebuilt, travelling with the tree)
// by bench.py's cpu_baseline leg on the GPU box host.  Never built there,
// never part of the product path.
//
// It drives MemEC's own plugin exactly as its test does
// (test/common/coding/coding.cc:149-274): Coding::instantiate -> encode(index)
// / decode(chunks, bitmap), with Chunk buffers from TempChunkPool.
#include <cstdint>
#include <cstdlib>
#include <cstring>

#include "common/coding/coding.hh"
#include "common/ds/bitmask_array.hh"
#include "common/ds/chunk_pool.hh"
#include "common/ds/chunk_util.hh"

extern "C" {
#include "galois.h"
#include "jerasure.h"
#include "reed_sol.h"
#include "cauchy.h"
}

namespace {
struct RefHandle {
    Coding *coding;
    uint32_t k, m, cs;
};
}  // namespace

extern "C" {

void *ref_instantiate(int scheme, uint32_t k, uint32_t m, uint32_t chunk_size) {
    CodingParams params;
    CodingScheme s = scheme == 7 ? CS_CAUCHY : CS_RS;
    params.setScheme(s);
    params.setK(k);
    params.setM(m);
    ChunkUtil::init(chunk_size, k);
    Coding *c = Coding::instantiate(s, params, chunk_size);
    if (!c) return nullptr;
    RefHandle *h = new RefHandle{c, k, m, chunk_size};
    return h;
}

void ref_destroy(void *hp) {
    RefHandle *h = (RefHandle *)hp;
    delete h->coding;  // Coding::destroy reads an unset scheme (Appendix B #1)
    delete h;
}

// data: k chunks of cs bytes, dense.  zero_mask bit j => pass Coding::zeros
// for data j (the server's delta-encode form).  Writes parity `index`
// (1-based) into out.
void ref_encode(void *hp, const uint8_t *data, uint32_t zero_mask, uint32_t index,
                uint8_t *out) {
    RefHandle *h = (RefHandle *)hp;
    TempChunkPool pool;
    Chunk *d[64];
    for (uint32_t j = 0; j < h->k; j++) {
        if (zero_mask >> j & 1) {
            d[j] = Coding::zeros;
        } else {
            d[j] = pool.alloc();
            memcpy(ChunkUtil::getData(d[j]), data + (size_t)j * h->cs, h->cs);
        }
    }
    Chunk *p = pool.alloc();
    h->coding->encode(d, p, index);
    memcpy(out, ChunkUtil::getData(p), h->cs);
    pool.free(p);
    for (uint32_t j = 0; j < h->k; j++)
        if (!(zero_mask >> j & 1)) pool.free(d[j]);
}

// chunks: (k+m) chunks dense, in/out.  Missing chunks are cleared first
// (server_peer_res_worker.cc:818-828) and rebuilt in place.
int ref_decode(void *hp, uint8_t *chunks, uint64_t present_mask) {
    RefHandle *h = (RefHandle *)hp;
    uint32_t n = h->k + h->m;
    TempChunkPool pool;
    Chunk *c[64];
    BitmaskArray bm(1, n);
    for (uint32_t i = 0; i < n; i++) {
        c[i] = pool.alloc();
        if (present_mask >> i & 1) {
            memcpy(ChunkUtil::getData(c[i]), chunks + (size_t)i * h->cs, h->cs);
            bm.set(i, 0);
        }
    }
    bool ok = h->coding->decode(c, &bm);
    for (uint32_t i = 0; i < n; i++) {
        memcpy(chunks + (size_t)i * h->cs, ChunkUtil::getData(c[i]), h->cs);
        pool.free(c[i]);
    }
    return ok ? 0 : -1;
}

void ref_bitwise_xor(uint8_t *dst, const uint8_t *a, const uint8_t *b, uint32_t len) {
    Coding::bitwiseXOR((char *)dst, (char *)a, (char *)b, len);
}

int ref_gf_mul(int a, int b, int w) { return galois_single_multiply(a, b, w); }
int ref_gf_div(int a, int b, int w) { return galois_single_divide(a, b, w); }

int ref_rs_matrix(int k, int m, int w, int *out) {
    int *mat = reed_sol_vandermonde_coding_matrix(k, m, w);
    if (!mat) return -1;
    memcpy(out, mat, sizeof(int) * k * m);
    free(mat);
    return 0;
}

int ref_cauchy_matrix(int k, int m, int w, int *out) {
    int *mat = cauchy_good_general_coding_matrix(k, m, w);
    if (!mat) return -1;
    memcpy(out, mat, sizeof(int) * k * m);
    free(mat);
    return 0;
}

int ref_cauchy_n_ones(int n, int w) { return cauchy_n_ones(n, w); }

int ref_bitmatrix(int k, int m, int w, const int *matrix, int *out) {
    int *bm = jerasure_matrix_to_bitmatrix(k, m, w, (int *)matrix);
    if (!bm) return -1;
    memcpy(out, bm, sizeof(int) * k * m * w * w);
    free(bm);
    return 0;
}

// Returns op count; ops[5*i..5*i+4].
int ref_smart_schedule(int k, int m, int w, const int *bitmatrix, int *ops, int max_ops) {
    int **s = jerasure_smart_bitmatrix_to_schedule(k, m, w, (int *)bitmatrix);
    int n = 0;
    for (; s[n][0] >= 0; n++) {
        if (n < max_ops) memcpy(ops + 5 * n, s[n], sizeof(int) * 5);
    }
    jerasure_free_schedule(s);
    return n;
}

int ref_invert_matrix(int *mat, int *inv, int n, int w) { return jerasure_invert_matrix(mat, inv, n, w); }
int ref_invert_bitmatrix(int *mat, int *inv, int n) { return jerasure_invert_bitmatrix(mat, inv, n); }

}  // extern "C"

// Timing entry points (tools/speed_fidelity.py): chunks allocated once, so
// a timed encode is exactly one Coding::encode call on resident chunks.
extern "C" {
void *ref_alloc_chunks(uint32_t n) {
    Chunk **c = new Chunk *[n];
    TempChunkPool pool;
    for (uint32_t i = 0; i < n; i++) c[i] = pool.alloc();
    return c;
}
char *ref_chunk_data(void *chunks, uint32_t i) { return ChunkUtil::getData(((Chunk **)chunks)[i]); }
void ref_encode_chunks(void *hp, void *chunks, uint32_t first, uint32_t index) {
    RefHandle *h = (RefHandle *)hp;
    Chunk **c = (Chunk **)chunks + first;
    h->coding->encode(c, c[h->k + index - 1], index);
}
}

// Batch drivers for bench.py's cpu_baseline leg (kind "reference"): the
// reference's own plugin run the way test/common/coding/batch_performance.cc
// runs it (worker pthreads, chunks allocated once per worker, then a loop of
// Coding calls on them), over disjoint stripe ranges.  Returns the wall time
// in seconds of `passes` timed passes (setup and copies untimed), or < 0 on a
// decode failure.
//   encode: one Coding::encode(data, parity, 1) per stripe per pass — the
//           plugin computes every parity of the stripe in that call
//           (rscoding.cc:51-95, cauchycoding.cc:49-85); the remaining
//           parities are then written out once, untimed, for verification.
//   decode: one Coding::decode(chunks, status) per stripe per pass on the
//           chunks whose present bit is clear (rebuilt in place).
#include <atomic>
#include <chrono>
#include <thread>
#include <vector>
namespace {
Chunk **stripes_in(const RefHandle *h, const uint8_t *src, uint32_t n) {
    const uint32_t per = h->k + h->m;
    Chunk **c = new Chunk *[(size_t)n * per];
    TempChunkPool pool;
    for (uint32_t s = 0; s < n; s++)
        for (uint32_t i = 0; i < per; i++) {
            c[(size_t)s * per + i] = pool.alloc();
            if (src) memcpy(ChunkUtil::getData(c[(size_t)s * per + i]), src + ((size_t)s * per + i) * h->cs, h->cs);
        }
    return c;
}
void stripes_free(const RefHandle *h, Chunk **c, uint32_t n) {
    TempChunkPool pool;
    for (size_t i = 0; i < (size_t)n * (h->k + h->m); i++) pool.free(c[i]);
    delete[] c;
}
template <typename F>
double run_workers(uint32_t n, uint32_t threads, F body) {
    std::vector<std::thread> th;
    const auto t0 = std::chrono::steady_clock::now();
    for (uint32_t t = 0; t < threads; t++)
        th.emplace_back([=] { body((uint64_t)n * t / threads, (uint64_t)n * (t + 1) / threads); });
    for (auto &x : th) x.join();
    return std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
}
}  // namespace
extern "C" {
// data: [n][k][cs] dense; parity: [n][m][cs] dense (written).
double ref_encode_batch_mt(void *hp, const uint8_t *data, uint8_t *parity, uint32_t n, uint32_t threads,
                           uint32_t passes) {
    RefHandle *h = (RefHandle *)hp;
    const uint32_t per = h->k + h->m;
    std::vector<uint8_t> dense((size_t)n * per * h->cs, 0);
    for (uint32_t s = 0; s < n; s++)
        memcpy(&dense[(size_t)s * per * h->cs], data + (size_t)s * h->k * h->cs, (size_t)h->k * h->cs);
    Chunk **c = stripes_in(h, dense.data(), n);
    const double dt = run_workers(n, threads, [&](uint64_t a, uint64_t b) {
        for (uint32_t p = 0; p < passes; p++)
            for (uint64_t s = a; s < b; s++) {
                Chunk **st = c + s * per;
                h->coding->encode(st, st[h->k], 1);
            }
    });
    run_workers(n, threads, [&](uint64_t a, uint64_t b) {  // untimed: the other parities
        for (uint64_t s = a; s < b; s++)
            for (uint32_t i = 2; i <= h->m; i++) h->coding->encode(c + s * per, c[s * per + h->k + i - 1], i);
    });
    for (uint32_t s = 0; s < n; s++) {
        Chunk **st = c + (size_t)s * per;
        for (uint32_t i = 0; i < h->m; i++)
            memcpy(parity + ((size_t)s * h->m + i) * h->cs, ChunkUtil::getData(st[h->k + i]), h->cs);
    }
    stripes_free(h, c, n);
    return dt;
}

// chunks: [n][k+m][cs] dense codewords; on return the erased chunks hold
// the reference's reconstruction.
double ref_decode_batch_mt(void *hp, uint8_t *chunks, uint32_t n, uint64_t present_mask, uint32_t threads,
                           uint32_t passes) {
    RefHandle *h = (RefHandle *)hp;
    const uint32_t per = h->k + h->m;
    Chunk **c = stripes_in(h, chunks, n);
    for (uint32_t s = 0; s < n; s++)
        for (uint32_t i = 0; i < per; i++)
            if (!(present_mask >> i & 1)) memset(ChunkUtil::getData(c[(size_t)s * per + i]), 0, h->cs);
    std::atomic<bool> all{true};
    const double dt = run_workers(n, threads, [&](uint64_t a, uint64_t b) {
        BitmaskArray bm(1, per);
        for (uint32_t i = 0; i < per; i++)
            if (present_mask >> i & 1) bm.set(i, 0);
        bool good = true;
        for (uint32_t p = 0; p < passes; p++)
            for (uint64_t s = a; s < b; s++) good = h->coding->decode(c + s * per, &bm) && good;
        if (!good) all = false;
    });
    for (uint32_t s = 0; s < n; s++)
        for (uint32_t i = 0; i < per; i++)
            memcpy(chunks + ((size_t)s * per + i) * h->cs, ChunkUtil::getData(c[(size_t)s * per + i]), h->cs);
    stripes_free(h, c, n);
    return all ? dt : -1.0;
}
// delta: [n][cs] (one data column j per stripe); parity: [n][m][cs] in/out.
// The server's delta path per stripe, as every parity server runs it
// (parity_chunk_buffer.cc:342-353, 387-393): for each parity index i,
// data = Coding::zeros except column j, ChunkUtil::clear(tmp),
// Coding::encode(data, tmp, i), then parity_i ^= tmp (Coding::bitwiseXOR).
double ref_update_batch_mt(void *hp, const uint8_t *delta, uint8_t *parity, uint32_t j, uint32_t n,
                           uint32_t threads, uint32_t passes) {
    RefHandle *h = (RefHandle *)hp;
    const uint32_t per = h->k + h->m;
    std::vector<uint8_t> dense((size_t)n * per * h->cs, 0);
    for (uint32_t s = 0; s < n; s++) {
        memcpy(&dense[((size_t)s * per + j) * h->cs], delta + (size_t)s * h->cs, h->cs);
        memcpy(&dense[((size_t)s * per + h->k) * h->cs], parity + (size_t)s * h->m * h->cs, (size_t)h->m * h->cs);
    }
    Chunk **c = stripes_in(h, dense.data(), n);
    const double dt = run_workers(n, threads, [&](uint64_t a, uint64_t b) {
        TempChunkPool pool;
        Chunk *tmp = pool.alloc();
        Chunk *d[64];
        for (uint32_t p = 0; p < passes; p++)
            for (uint64_t s = a; s < b; s++) {
                Chunk **st = c + s * per;
                for (uint32_t x = 0; x < h->k; x++) d[x] = Coding::zeros;
                d[j] = st[j];
                for (uint32_t i = 1; i <= h->m; i++) {
                    ChunkUtil::clear(tmp);
                    h->coding->encode(d, tmp, i);
                    char *par = ChunkUtil::getData(st[h->k + i - 1]);
                    Coding::bitwiseXOR(par, par, ChunkUtil::getData(tmp), h->cs);
                }
            }
        pool.free(tmp);
    });
    for (uint32_t s = 0; s < n; s++)
        for (uint32_t i = 0; i < h->m; i++)
            memcpy(parity + ((size_t)s * h->m + i) * h->cs, ChunkUtil::getData(c[(size_t)s * per + h->k + i]), h->cs);
    stripes_free(h, c, n);
    return dt;
}
}  // extern "C"
