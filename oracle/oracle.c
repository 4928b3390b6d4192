/*
 * oracle.c — CPU restatement of MemEC's erasure-coding hot path.
 *
 * TEST INFRASTRUCTURE ONLY (see oracle.h).  This file is never linked into
 * the product library; it is the checker for tests/ and the timed
 * "reference CPU path" (cpu_baseline kind "port") for bench.py.
 *
 * Speed fidelity: like MemEC's default build (common/coding/Makefile:41-45,
 * gcc -O3 without -DINTEL_SSE*), the w=8 region multiply is the single
 * 256x256 product-table byte loop (gf_w8.c:1047-1050) and region XOR is a
 * 64-bit word loop (gf.c:974-978).  Compile with -O3 and no SIMD flags.
 */
#include "oracle.h"

#include <pthread.h>
#include <stdlib.h>
#include <string.h>

/* ------------------------------------------------------------------------ */
/* GF(2^w), w <= 8                                                           */
/* ------------------------------------------------------------------------ */

/* Default primitive polynomials, including the x^w term:
 *   w=4: 0x13  (gf_w4.c:2045)      w=8: 0x11d (gf_w8.c:2376)
 *   w=1,2,3,5,6,7: gf_wgen.c:936-944 (octal 1, 7, 013, 045, 0103, 0211). */
int orc_gf_poly(int w)
{
    static const int polys[9] = {0, 0x3, 0x7, 0xb, 0x13, 0x25, 0x43, 0x89, 0x11d};
    return (w >= 1 && w <= 8) ? polys[w] : -1;
}

int orc_gf_mul(int a, int b, int w)
{
    int poly = orc_gf_poly(w);
    int acc = 0;
    int top = 1 << w;
    a &= top - 1;
    b &= top - 1;
    while (b) {
        if (b & 1) acc ^= a;
        b >>= 1;
        a <<= 1;
        if (a & top) a ^= poly;
    }
    return acc;
}

static int gf_inverse(int a, int w)
{
    int x;
    if (a == 0) return 0;
    for (x = 1; x < (1 << w); x++)
        if (orc_gf_mul(a, x, w) == 1) return x;
    return 0;
}

/* galois_single_divide (galois.c:257-272): a / b, 0 when b == 0. */
int orc_gf_div(int a, int b, int w)
{
    if (b == 0) return -1;
    if (a == 0) return 0;
    return orc_gf_mul(a, gf_inverse(b, w), w);
}

/* 256x256 product table for w = 8 (gf_w8_table_init, gf_w8.c:1207-1290). */
static uint8_t g_mt8[256][256];
static pthread_once_t g_mt8_once = PTHREAD_ONCE_INIT;

static void mt8_build(void)
{
    int a, b;
    for (a = 0; a < 256; a++)
        for (b = 0; b < 256; b++)
            g_mt8[a][b] = (uint8_t)orc_gf_mul(a, b, 8);
}

/* ------------------------------------------------------------------------ */
/* MemEC getW                                                                */
/* ------------------------------------------------------------------------ */

static int min_w_for(uint32_t n)
{
    int w = 1;
    while ((1u << w) < n) w++;
    return w;
}

/* rscoding.cc:189-220: smallest w in {8,16,32} with 2^w >= k+m; chunk % w. */
int orc_rs_getw(uint32_t k, uint32_t m, uint32_t chunk_size)
{
    int w = min_w_for(k + m);
    if (w < 8) w = 8;
    else if (w < 16) w = 16;
    else if (w < 32) w = 32;
    else return -1;
    if (chunk_size % (uint32_t)w) return -1;
    return w;
}

/* cauchycoding.cc:182-205: smallest w >= log2(k+m) dividing chunk, w <= 32. */
int orc_cauchy_getw(uint32_t k, uint32_t m, uint32_t chunk_size)
{
    int w = min_w_for(k + m);
    while (chunk_size % (uint32_t)w) {
        w++;
        if (w > 32) return -1;
    }
    return w;
}

/* ------------------------------------------------------------------------ */
/* Jerasure Reed-Solomon Vandermonde coding matrix                           */
/* ------------------------------------------------------------------------ */

/* reed_sol_extended_vandermonde_matrix (reed_sol.c:175-203) followed by
 * reed_sol_big_vandermonde_distribution_matrix (reed_sol.c:205-300); the
 * coding matrix is rows k..k+m-1 (reed_sol_vandermonde_coding_matrix,
 * reed_sol.c:78-98). */
int orc_rs_vandermonde_matrix(int k, int m, int w, int *out)
{
    int rows = k + m, cols = k;
    int r, c, i, t;
    int *d;

    if (cols >= rows || w > 8 || (1 << w) < rows) return -1;
    d = (int *)calloc((size_t)rows * cols, sizeof(int));
    if (!d) return -1;
#define D(rr, cc) d[(rr) * cols + (cc)]
    /* extended Vandermonde: row 0 = e0, last row = e_{cols-1}, row r = r^c */
    D(0, 0) = 1;
    if (rows > 1) D(rows - 1, cols - 1) = 1;
    for (r = 1; r < rows - 1; r++) {
        int p = 1;
        for (c = 0; c < cols; c++) {
            D(r, c) = p;
            p = orc_gf_mul(p, r, w);
        }
    }
    /* column operations that turn the top cols x cols block into identity */
    for (i = 1; i < cols; i++) {
        int piv = i, inv;
        while (piv < rows && D(piv, i) == 0) piv++;
        if (piv >= rows) { free(d); return -1; }
        if (piv != i)
            for (c = 0; c < cols; c++) { t = D(piv, c); D(piv, c) = D(i, c); D(i, c) = t; }
        if (D(i, i) != 1) {
            inv = orc_gf_div(1, D(i, i), w);
            for (r = 0; r < rows; r++) D(r, i) = orc_gf_mul(inv, D(r, i), w);
        }
        for (c = 0; c < cols; c++) {
            int e = D(i, c);
            if (c == i || e == 0) continue;
            for (r = 0; r < rows; r++) D(r, c) ^= orc_gf_mul(e, D(r, i), w);
        }
    }
    /* scale columns so that row `cols` is all ones (only rows >= cols) */
    for (c = 0; c < cols; c++) {
        int e = D(cols, c);
        if (e != 1) {
            int inv = orc_gf_div(1, e, w);
            for (r = cols; r < rows; r++) D(r, c) = orc_gf_mul(inv, D(r, c), w);
        }
    }
    /* scale rows cols+1.. so that their first element is one */
    for (r = cols + 1; r < rows; r++) {
        int e = D(r, 0);
        if (e != 1) {
            int inv = orc_gf_div(1, e, w);
            for (c = 0; c < cols; c++) D(r, c) = orc_gf_mul(D(r, c), inv, w);
        }
    }
    memcpy(out, d + (size_t)cols * cols, sizeof(int) * (size_t)m * k);
#undef D
    free(d);
    return 0;
}

/* ------------------------------------------------------------------------ */
/* Jerasure Cauchy "good" coding matrix                                      */
/* ------------------------------------------------------------------------ */

/* cauchy_n_ones (cauchy.c:89-129): ones in the w x w bitmatrix of n. */
int orc_cauchy_n_ones(int n, int w)
{
    int x, ones = 0, e = n;
    for (x = 0; x < w; x++) {
        ones += __builtin_popcount((unsigned)e);
        e = orc_gf_mul(e, 2, w);
    }
    return ones;
}

/* The cbest_w tables (cauchy.c:240-271) list every nonzero element of
 * GF(2^w) ordered by (cauchy_n_ones, value); verified equal for w = 2..8 in
 * tests/test_oracle.py against the values dumped from the reference. */
static void cbest_list(int w, int *list)
{
    int n = (1 << w) - 1, i, j;
    for (i = 0; i < n; i++) list[i] = i + 1;
    for (i = 1; i < n; i++) {
        int v = list[i], ov = orc_cauchy_n_ones(v, w);
        j = i - 1;
        while (j >= 0) {
            int oj = orc_cauchy_n_ones(list[j], w);
            if (oj < ov || (oj == ov && list[j] < v)) break;
            list[j + 1] = list[j];
            j--;
        }
        list[j + 1] = v;
    }
}

/* cauchy_good_general_coding_matrix (cauchy.c:209-238) with
 * cauchy_original_coding_matrix (cauchy.c:131-147) and
 * cauchy_improve_coding_matrix (cauchy.c:166-207). */
int orc_cauchy_good_matrix(int k, int m, int w, int *out)
{
    int i, j, x;
    static const int cbest_max_k[9] = {-1, -1, 3, 7, 15, 31, 63, 127, 255};

    if (w < 1 || w > 8) return -1;
    if (m == 2 && k <= cbest_max_k[w]) {
        int list[255];
        cbest_list(w, list);
        for (j = 0; j < k; j++) {
            out[j] = 1;
            out[k + j] = list[j];
        }
        return 0;
    }
    if (k + m > (1 << w)) return -1;
    for (i = 0; i < m; i++)
        for (j = 0; j < k; j++)
            out[i * k + j] = orc_gf_div(1, i ^ (m + j), w);
    /* improve: normalise every column so row 0 is ones */
    for (j = 0; j < k; j++) {
        if (out[j] != 1) {
            int s = orc_gf_div(1, out[j], w);
            for (i = 0; i < m; i++) out[i * k + j] = orc_gf_mul(out[i * k + j], s, w);
        }
    }
    /* then scale each later row by the inverse of the element that
     * minimises the row's bitmatrix ones */
    for (i = 1; i < m; i++) {
        int *row = out + i * k;
        int best = 0, best_j = -1;
        for (j = 0; j < k; j++) best += orc_cauchy_n_ones(row[j], w);
        for (j = 0; j < k; j++) {
            int s, tot = 0;
            if (row[j] == 1) continue;
            s = orc_gf_div(1, row[j], w);
            for (x = 0; x < k; x++) tot += orc_cauchy_n_ones(orc_gf_mul(row[x], s, w), w);
            if (tot < best) { best = tot; best_j = j; }
        }
        if (best_j != -1) {
            int s = orc_gf_div(1, row[best_j], w);
            for (j = 0; j < k; j++) row[j] = orc_gf_mul(row[j], s, w);
        }
    }
    return 0;
}

/* jerasure_matrix_to_bitmatrix (jerasure.c:271-297):
 * B[i*w+l][j*w+x] = bit l of (A[i][j] * 2^x). */
void orc_matrix_to_bitmatrix(int k, int m, int w, const int *matrix, int *bm)
{
    int i, j, x, l, cols = k * w;
    for (i = 0; i < m; i++)
        for (j = 0; j < k; j++) {
            int e = matrix[i * k + j];
            for (x = 0; x < w; x++) {
                for (l = 0; l < w; l++)
                    bm[(i * w + l) * cols + j * w + x] = (e >> l) & 1;
                e = orc_gf_mul(e, 2, w);
            }
        }
}

/* jerasure_invert_matrix (jerasure.c:373-458).  mat is destroyed. */
int orc_invert_matrix(int *mat, int *inv, int n, int w)
{
    int i, j, c;
    for (i = 0; i < n * n; i++) inv[i] = 0;
    for (i = 0; i < n; i++) inv[i * n + i] = 1;
    for (i = 0; i < n; i++) {
        int *ri = mat + i * n, *vi = inv + i * n;
        if (ri[i] == 0) {
            for (j = i + 1; j < n && mat[j * n + i] == 0; j++) ;
            if (j == n) return -1;
            for (c = 0; c < n; c++) {
                int t = ri[c]; ri[c] = mat[j * n + c]; mat[j * n + c] = t;
                t = vi[c]; vi[c] = inv[j * n + c]; inv[j * n + c] = t;
            }
        }
        if (ri[i] != 1) {
            int s = orc_gf_div(1, ri[i], w);
            for (c = 0; c < n; c++) {
                ri[c] = orc_gf_mul(ri[c], s, w);
                vi[c] = orc_gf_mul(vi[c], s, w);
            }
        }
        for (j = i + 1; j < n; j++) {
            int f = mat[j * n + i];
            if (f == 0) continue;
            for (c = 0; c < n; c++) {
                mat[j * n + c] ^= orc_gf_mul(f, ri[c], w);
                inv[j * n + c] ^= orc_gf_mul(f, vi[c], w);
            }
        }
    }
    for (i = n - 1; i >= 0; i--)
        for (j = 0; j < i; j++) {
            int f = mat[j * n + i];
            if (f == 0) continue;
            mat[j * n + i] = 0;
            for (c = 0; c < n; c++) inv[j * n + c] ^= orc_gf_mul(f, inv[i * n + c], w);
        }
    return 0;
}

/* jerasure_invert_bitmatrix (jerasure.c:1043-1098).  mat is destroyed. */
int orc_invert_bitmatrix(int *mat, int *inv, int n)
{
    int i, j, c;
    for (i = 0; i < n * n; i++) inv[i] = 0;
    for (i = 0; i < n; i++) inv[i * n + i] = 1;
    for (i = 0; i < n; i++) {
        if (mat[i * n + i] == 0) {
            for (j = i + 1; j < n && mat[j * n + i] == 0; j++) ;
            if (j == n) return -1;
            for (c = 0; c < n; c++) {
                int t = mat[i * n + c]; mat[i * n + c] = mat[j * n + c]; mat[j * n + c] = t;
                t = inv[i * n + c]; inv[i * n + c] = inv[j * n + c]; inv[j * n + c] = t;
            }
        }
        for (j = i + 1; j < n; j++)
            if (mat[j * n + i])
                for (c = 0; c < n; c++) { mat[j * n + c] ^= mat[i * n + c]; inv[j * n + c] ^= inv[i * n + c]; }
    }
    for (i = n - 1; i >= 0; i--)
        for (j = 0; j < i; j++)
            if (mat[j * n + i])
                for (c = 0; c < n; c++) { mat[j * n + c] ^= mat[i * n + c]; inv[j * n + c] ^= inv[i * n + c]; }
    return 0;
}

/* jerasure_smart_bitmatrix_to_schedule (jerasure.c:1235-1353).
 * Rows are emitted cheapest-first; a row is either built from scratch
 * (copy + XORs of its ones) or from a previously built row plus the XOR of
 * the columns in which the two differ, whichever is cheaper. */
int orc_smart_schedule(int k, int m, int w, const int *bm, int *ops, int max_ops)
{
    int R = m * w, C = k * w;
    int *cost = malloc(sizeof(int) * R), *base = malloc(sizeof(int) * R);
    int *next = malloc(sizeof(int) * R), *prev = malloc(sizeof(int) * R);
    int head = 0, pick = 0, best, r, c, nops = 0;

#define EMIT(sd, sp, dd, dp, x) do { if (nops >= max_ops) goto fail; \
        ops[5*nops+0] = (sd); ops[5*nops+1] = (sp); ops[5*nops+2] = (dd); \
        ops[5*nops+3] = (dp); ops[5*nops+4] = (x); nops++; } while (0)

    best = C + 1;
    for (r = 0; r < R; r++) {
        int ones = 0;
        for (c = 0; c < C; c++) ones += bm[r * C + c];
        cost[r] = ones;
        base[r] = -1;
        next[r] = r + 1;
        prev[r] = r - 1;
        if (ones < best) { best = ones; pick = r; }
    }
    next[R - 1] = -1;

    while (head != -1) {
        const int *row;
        r = pick;
        /* unlink r */
        if (prev[r] == -1) {
            head = next[r];
            if (head != -1) prev[head] = -1;
        } else {
            next[prev[r]] = next[r];
            if (next[r] != -1) prev[next[r]] = prev[r];
        }
        row = bm + r * C;
        if (base[r] == -1) {
            int started = 0;
            for (c = 0; c < C; c++)
                if (row[c]) { EMIT(c / w, c % w, k + r / w, r % w, started); started = 1; }
        } else {
            const int *brow = bm + base[r] * C;
            EMIT(k + base[r] / w, base[r] % w, k + r / w, r % w, 0);
            for (c = 0; c < C; c++)
                if (row[c] ^ brow[c]) EMIT(c / w, c % w, k + r / w, r % w, 1);
        }
        best = C + 1;
        for (c = head; c != -1; c = next[c]) {
            const int *orow = bm + c * C;
            int diff = 1, j;
            for (j = 0; j < C; j++) diff += row[j] ^ orow[j];
            if (diff < cost[c]) { base[c] = r; cost[c] = diff; }
            if (cost[c] < best) { best = cost[c]; pick = c; }
        }
    }
#undef EMIT
    free(cost); free(base); free(next); free(prev);
    return nops;
fail:
    free(cost); free(base); free(next); free(prev);
    return -1;
}

/* ------------------------------------------------------------------------ */
/* Region primitives                                                         */
/* ------------------------------------------------------------------------ */

/* gf_multby_one with xor (gf.c:894-989): bytes up to 8-byte alignment of
 * dst, then 64-bit words (gf.c:974-978), then a byte tail. */
static void region_xor(const uint8_t *src, uint8_t *dst, size_t n)
{
    size_t head = (8 - ((uintptr_t)dst & 7)) & 7, i, words;
    const uint64_t *s64;
    uint64_t *d64;
    if (head > n) head = n;
    for (i = 0; i < head; i++) dst[i] ^= src[i];
    words = (n - head) / 8;
    s64 = (const uint64_t *)(src + head);
    d64 = (uint64_t *)(dst + head);
    for (i = 0; i < words; i++) d64[i] ^= s64[i];
    for (i = head + words * 8; i < n; i++) dst[i] ^= src[i];
}

void orc_xor(uint8_t *dst, const uint8_t *a, const uint8_t *b, size_t len)
{
    size_t i = 0;
    for (; i + 8 <= len; i += 8) {
        uint64_t x, y;
        memcpy(&x, a + i, 8);
        memcpy(&y, b + i, 8);
        x ^= y;
        memcpy(dst + i, &x, 8);
    }
    for (; i < len; i++) dst[i] = a[i] ^ b[i];
}

/* gf_w8_table_multiply_region (gf_w8.c:1033-1056). */
static void region_mul8(const uint8_t *src, uint8_t *dst, int c, size_t n, int accumulate)
{
    size_t i;
    pthread_once(&g_mt8_once, mt8_build);
    if (accumulate)
        for (i = 0; i < n; i++) dst[i] ^= g_mt8[src[i]][c];
    else
        for (i = 0; i < n; i++) dst[i] = g_mt8[src[i]][c];
}

/* jerasure_matrix_dotprod for w = 8 (jerasure.c:574-633): unit terms are
 * copied/XORed first, then every other nonzero term is table-multiplied. */
static void dotprod8(int k, const int *row, const int *src_ids, int dest_id,
                     uint8_t *const *data, uint8_t *const *coding, size_t size)
{
    uint8_t *dst = dest_id < k ? data[dest_id] : coding[dest_id - k];
    int have = 0, j;
    for (j = 0; j < k; j++) {
        int id = src_ids ? src_ids[j] : j;
        const uint8_t *src = id < k ? data[id] : coding[id - k];
        if (row[j] != 1) continue;
        if (!have) { memcpy(dst, src, size); have = 1; }
        else region_xor(src, dst, size);
    }
    for (j = 0; j < k; j++) {
        int id = src_ids ? src_ids[j] : j;
        const uint8_t *src = id < k ? data[id] : coding[id - k];
        if (row[j] == 0 || row[j] == 1) continue;
        region_mul8(src, dst, row[j], size, have);
        have = 1;
    }
}

/* jerasure_matrix_encode (jerasure.c:299-312). */
void orc_rs_encode(int k, int m, const int *matrix, const uint8_t *const *data,
                   uint8_t *const *coding, size_t size)
{
    int i;
    for (i = 0; i < m; i++)
        dotprod8(k, matrix + i * k, NULL, k + i, (uint8_t *const *)data, coding, size);
}

/* jerasure_matrix_decode with row_k_ones = 1 (jerasure.c:167-268), as
 * called by RSCoding::decode (rscoding.cc:182). */
int orc_rs_decode(int k, int m, const int *matrix, const int *erased,
                  uint8_t *const *data, uint8_t *const *coding, size_t size)
{
    int i, j, n_erased = 0, edd = 0, last = k;
    int dm_ids[64], *dec = NULL;

    for (i = 0; i < k + m; i++) n_erased += erased[i] ? 1 : 0;
    if (n_erased > m) return -1;
    for (i = 0; i < k; i++)
        if (erased[i]) { edd++; last = i; }
    if (erased[k]) last = k;

    if (edd > 1 || (edd > 0 && erased[k])) {
        /* jerasure_make_decoding_matrix (jerasure.c:98-126) */
        int *sub = malloc(sizeof(int) * k * k);
        dec = malloc(sizeof(int) * k * k);
        for (i = 0, j = 0; j < k; i++)
            if (!erased[i]) dm_ids[j++] = i;
        for (i = 0; i < k; i++) {
            if (dm_ids[i] < k) {
                for (j = 0; j < k; j++) sub[i * k + j] = 0;
                sub[i * k + dm_ids[i]] = 1;
            } else {
                for (j = 0; j < k; j++) sub[i * k + j] = matrix[(dm_ids[i] - k) * k + j];
            }
        }
        if (orc_invert_matrix(sub, dec, k, 8) < 0) { free(sub); free(dec); return -1; }
        free(sub);
    }
    for (i = 0; edd > 0 && i < last; i++)
        if (erased[i]) {
            dotprod8(k, dec + i * k, dm_ids, i, data, coding, size);
            edd--;
        }
    if (edd > 0) {
        int ids[64];
        for (i = 0; i < k; i++) ids[i] = i < last ? i : i + 1;
        dotprod8(k, matrix, ids, last, data, coding, size);
    }
    for (i = 0; i < m; i++)
        if (erased[k + i]) dotprod8(k, matrix + i * k, NULL, k + i, data, coding, size);
    free(dec);
    return 0;
}

/* ------------------------------------------------------------------------ */
/* Cauchy-RS: scheduled packet XOR                                           */
/* ------------------------------------------------------------------------ */

/* jerasure_do_scheduled_operations (jerasure.c:1162-1185), looped over the
 * region as jerasure_schedule_encode does (jerasure.c:1187-1201). */
void orc_schedule_run(int k, int w, const int *ops, int nops, uint8_t *const *ptrs_in,
                      size_t size, size_t packetsize)
{
    uint8_t *ptrs[64];
    size_t done;
    int i, n = 64;
    (void)k;
    for (i = 0; i < n; i++) ptrs[i] = ptrs_in[i];
    for (done = 0; done < size; done += packetsize * (size_t)w) {
        for (i = 0; i < nops; i++) {
            const int *o = ops + 5 * i;
            const uint8_t *s = ptrs[o[0]] + (size_t)o[1] * packetsize;
            uint8_t *d = ptrs[o[2]] + (size_t)o[3] * packetsize;
            if (o[4]) region_xor(s, d, packetsize);
            else memcpy(d, s, packetsize);
        }
        for (i = 0; i < n; i++) if (ptrs[i]) ptrs[i] += packetsize * (size_t)w;
    }
}

void orc_crs_encode(int k, int m, int w, const int *ops, int nops,
                    const uint8_t *const *data, uint8_t *const *coding,
                    size_t size, size_t packetsize)
{
    uint8_t *ptrs[64];
    int i;
    memset(ptrs, 0, sizeof(ptrs));
    for (i = 0; i < k; i++) ptrs[i] = (uint8_t *)data[i];
    for (i = 0; i < m; i++) ptrs[k + i] = coding[i];
    orc_schedule_run(k, w, ops, nops, ptrs, size, packetsize);
}

/* jerasure_schedule_decode_lazy with smart = 1 (jerasure.c:947-973):
 * set_up_ptrs/ids_for_scheduled_decoding (jerasure.c:718-815) and
 * jerasure_generate_decoding_schedule (jerasure.c:817-945). */
int orc_crs_decode(int k, int m, int w, const int *bm, const int *erased,
                   uint8_t *const *data, uint8_t *const *coding,
                   size_t size, size_t packetsize)
{
    int row_ids[64], to_row[64];
    uint8_t *ptrs[64];
    int i, j, x, y, z, ddf = 0, cdf = 0, kw = k * w, blk = k * w * w;
    int *real, *ops, nops, max_ops;

    for (i = 0; i < k + m; i++) {
        if (!erased[i]) continue;
        if (i < k) ddf++; else cdf++;
    }
    if (ddf + cdf > m) return -1;
    if (ddf + cdf == 0) return 0;

    memset(ptrs, 0, sizeof(ptrs));
    j = k;
    x = k;
    for (i = 0; i < k; i++) {
        if (!erased[i]) {
            row_ids[i] = i; to_row[i] = i; ptrs[i] = data[i];
        } else {
            while (erased[j]) j++;
            row_ids[i] = j; to_row[j] = i; ptrs[i] = coding[j - k];
            j++;
            row_ids[x] = i; to_row[i] = x; ptrs[x] = data[i];
            x++;
        }
    }
    for (i = k; i < k + m; i++)
        if (erased[i]) { row_ids[x] = i; to_row[i] = x; ptrs[x] = coding[i - k]; x++; }

    real = calloc((size_t)(ddf + cdf) * blk, sizeof(int));
    if (ddf > 0) {
        int *sub = calloc((size_t)k * blk, sizeof(int));
        int *inv = malloc(sizeof(int) * (size_t)k * blk);
        for (i = 0; i < k; i++) {
            int *p = sub + (size_t)i * blk;
            if (row_ids[i] == i) {
                for (x = 0; x < w; x++) p[x * kw + i * w + x] = 1;
            } else {
                memcpy(p, bm + (size_t)(row_ids[i] - k) * blk, sizeof(int) * blk);
            }
        }
        orc_invert_bitmatrix(sub, inv, kw);
        for (i = 0; i < ddf; i++)
            memcpy(real + (size_t)i * blk, inv + (size_t)row_ids[k + i] * blk, sizeof(int) * blk);
        free(sub);
        free(inv);
    }
    for (x = 0; x < cdf; x++) {
        int drive = row_ids[x + ddf + k] - k;
        int *p = real + (size_t)(ddf + x) * blk;
        const int *src = bm + (size_t)drive * blk;
        memcpy(p, src, sizeof(int) * blk);
        for (i = 0; i < k; i++) {
            if (row_ids[i] == i) continue;
            for (j = 0; j < w; j++) memset(p + j * kw + i * w, 0, sizeof(int) * w);
        }
        for (i = 0; i < k; i++) {
            const int *b1;
            if (row_ids[i] == i) continue;
            b1 = real + (size_t)(to_row[i] - k) * blk;
            for (j = 0; j < w; j++) {
                int *b2 = p + j * kw;
                for (y = 0; y < w; y++)
                    if (src[j * kw + i * w + y])
                        for (z = 0; z < kw; z++) b2[z] ^= b1[z + y * kw];
            }
        }
    }
    max_ops = kw * (ddf + cdf) * w + 1;
    ops = malloc(sizeof(int) * 5 * (size_t)max_ops);
    nops = orc_smart_schedule(k, ddf + cdf, w, real, ops, max_ops);
    orc_schedule_run(k, w, ops, nops, ptrs, size, packetsize);
    free(ops);
    free(real);
    return 0;
}

/* ------------------------------------------------------------------------ */
/* ISA-L 2.14 base family                                                    */
/* ------------------------------------------------------------------------ */

static uint8_t isal_mul(uint8_t a, uint8_t b) { return (uint8_t)orc_gf_mul(a, b, 8); }

/* gf_gen_rs_matrix (erasure_code/ec_base.c:62-79). */
void orc_isal_gen_rs_matrix(uint8_t *a, int rows, int k)
{
    int i, j;
    uint8_t gen = 1;
    memset(a, 0, (size_t)rows * k);
    for (i = 0; i < k; i++) a[i * k + i] = 1;
    for (i = k; i < rows; i++) {
        uint8_t p = 1;
        for (j = 0; j < k; j++) { a[i * k + j] = p; p = isal_mul(p, gen); }
        gen = isal_mul(gen, 2);
    }
}

/* gf_gen_cauchy1_matrix (erasure_code/ec_base.c:81-97). */
void orc_isal_gen_cauchy1_matrix(uint8_t *a, int rows, int k)
{
    int i, j;
    memset(a, 0, (size_t)rows * k);
    for (i = 0; i < k; i++) a[i * k + i] = 1;
    for (i = k; i < rows; i++)
        for (j = 0; j < k; j++) a[i * k + j] = (uint8_t)gf_inverse(i ^ j, 8);
}

/* gf_invert_matrix (erasure_code/ec_base.c:117-170), Gauss-Jordan. */
int orc_isal_invert_matrix(uint8_t *in, uint8_t *out, int n)
{
    int i, j, c;
    memset(out, 0, (size_t)n * n);
    for (i = 0; i < n; i++) out[i * n + i] = 1;
    for (i = 0; i < n; i++) {
        uint8_t s;
        if (in[i * n + i] == 0) {
            for (j = i + 1; j < n && in[j * n + i] == 0; j++) ;
            if (j == n) return -1;
            for (c = 0; c < n; c++) {
                uint8_t t = in[i * n + c]; in[i * n + c] = in[j * n + c]; in[j * n + c] = t;
                t = out[i * n + c]; out[i * n + c] = out[j * n + c]; out[j * n + c] = t;
            }
        }
        s = (uint8_t)gf_inverse(in[i * n + i], 8);
        for (c = 0; c < n; c++) {
            in[i * n + c] = isal_mul(in[i * n + c], s);
            out[i * n + c] = isal_mul(out[i * n + c], s);
        }
        for (j = 0; j < n; j++) {
            uint8_t f;
            if (j == i) continue;
            f = in[j * n + i];
            for (c = 0; c < n; c++) {
                out[j * n + c] ^= isal_mul(f, out[i * n + c]);
                in[j * n + c] ^= isal_mul(f, in[i * n + c]);
            }
        }
    }
    return 0;
}

/* ec_encode_data_base (erasure_code/ec_base.c:308-323), coefficients given
 * directly (ec_init_tables expands each into a 32-byte nibble table). */
void orc_isal_encode(int len, int k, int rows, const uint8_t *coef,
                     const uint8_t *const *src, uint8_t *const *dst)
{
    int l, i, j;
    pthread_once(&g_mt8_once, mt8_build);
    for (l = 0; l < rows; l++)
        for (i = 0; i < len; i++) {
            uint8_t s = 0;
            for (j = 0; j < k; j++) s ^= g_mt8[src[j][i]][coef[l * k + j]];
            dst[l][i] = s;
        }
}

/* ec_encode_data_update_base (erasure_code/ec_base.c:325-339). */
void orc_isal_encode_update(int len, int k, int rows, int col, const uint8_t *coef,
                            const uint8_t *src, uint8_t *const *dst)
{
    int l, i;
    pthread_once(&g_mt8_once, mt8_build);
    for (l = 0; l < rows; l++)
        for (i = 0; i < len; i++) dst[l][i] ^= g_mt8[src[i]][coef[l * k + col]];
}

/* RSCoding/CauchyCoding::decode with USE_ISAL (rscoding.cc:155-177,
 * cauchycoding.cc:145-168): survivors = first k present chunks; erased data
 * row e = inverse row e.  Erased parity p uses encode_row(p) x inverse
 * (the reference reads inverse row p, past k rows: a bug). */
int orc_isal_decode(int k, int m, const uint8_t *enc, const int *erased,
                    uint8_t *const *chunks, size_t size)
{
    uint8_t sub[32 * 32], inv[32 * 32], rows[32 * 32];
    const uint8_t *alive[32];
    uint8_t *missing[32];
    int i, j, t, na = 0, ne = 0;
    for (i = 0; i < k + m; i++) ne += erased[i] ? 1 : 0;
    if (ne > m) return -1;
    if (ne == 0) return 0;
    for (i = 0; i < k + m && na < k; i++)
        if (!erased[i]) { memcpy(sub + na * k, enc + i * k, k); alive[na++] = chunks[i]; }
    if (orc_isal_invert_matrix(sub, inv, k) < 0) return -1;
    ne = 0;
    for (i = 0; i < k + m; i++) {
        if (!erased[i]) continue;
        if (i < k) {
            memcpy(rows + ne * k, inv + i * k, k);
        } else {
            for (j = 0; j < k; j++) {
                uint8_t s = 0;
                for (t = 0; t < k; t++) s ^= isal_mul(enc[i * k + t], inv[t * k + j]);
                rows[ne * k + j] = s;
            }
        }
        missing[ne++] = chunks[i];
    }
    orc_isal_encode((int)size, k, ne, rows, alive, missing);
    return 0;
}

/* ------------------------------------------------------------------------ */
/* Helpers                                                                   */
/* ------------------------------------------------------------------------ */

static uint64_t splitmix_at(uint64_t seed, uint64_t q)
{
    uint64_t z = seed + (q + 1) * 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

/* Byte i of the stream is byte (i % 8) (little endian) of word
 * word_offset + i / 8.  Identical to the device fill (mec_fill_random). */
void orc_fill_splitmix(uint8_t *buf, size_t n, uint64_t seed, uint64_t word_offset)
{
    size_t i;
    for (i = 0; i < n; i += 8) {
        uint64_t v = splitmix_at(seed, word_offset + i / 8);
        size_t b, lim = n - i < 8 ? n - i : 8;
        for (b = 0; b < lim; b++) buf[i + b] = (uint8_t)(v >> (8 * b));
    }
}

struct batch_job {
    int family, k, m, w, nops;
    uint32_t cs;
    const int *matrix, *ops;
    const uint8_t *data;
    uint8_t *parity;
    uint32_t s0, s1;
};

static void *batch_worker(void *arg)
{
    struct batch_job *jb = (struct batch_job *)arg;
    const uint8_t *d[64];
    uint8_t *p[64];
    uint32_t s;
    int i;
    for (s = jb->s0; s < jb->s1; s++) {
        for (i = 0; i < jb->k; i++) d[i] = jb->data + ((size_t)s * jb->k + i) * jb->cs;
        for (i = 0; i < jb->m; i++) p[i] = jb->parity + ((size_t)s * jb->m + i) * jb->cs;
        if (jb->family == 0)
            orc_rs_encode(jb->k, jb->m, jb->matrix, d, p, jb->cs);
        else
            orc_crs_encode(jb->k, jb->m, jb->w, jb->ops, jb->nops, d, p, jb->cs, jb->cs / jb->w);
    }
    return NULL;
}

int orc_encode_batch_mt(int family, int k, int m, uint32_t chunk_size,
                        const uint8_t *data, uint8_t *parity, uint32_t n_stripes, int threads)
{
    int matrix[32 * 32], *bm = NULL, *ops = NULL, nops = 0, w, t, rc = 0;
    pthread_t tid[256];
    struct batch_job jobs[256];

    if (threads < 1) threads = 1;
    if (threads > 256) threads = 256;
    pthread_once(&g_mt8_once, mt8_build);
    if (family == 0) {
        w = orc_rs_getw((uint32_t)k, (uint32_t)m, chunk_size);
        if (w != 8 || orc_rs_vandermonde_matrix(k, m, 8, matrix)) return -1;
    } else {
        int max_ops;
        w = orc_cauchy_getw((uint32_t)k, (uint32_t)m, chunk_size);
        if (w < 1 || w > 8 || orc_cauchy_good_matrix(k, m, w, matrix)) return -1;
        bm = malloc(sizeof(int) * (size_t)k * m * w * w);
        orc_matrix_to_bitmatrix(k, m, w, matrix, bm);
        max_ops = k * m * w * w + 1;
        ops = malloc(sizeof(int) * 5 * (size_t)max_ops);
        nops = orc_smart_schedule(k, m, w, bm, ops, max_ops);
    }
    for (t = 0; t < threads; t++) {
        jobs[t].family = family; jobs[t].k = k; jobs[t].m = m; jobs[t].w = w;
        jobs[t].cs = chunk_size; jobs[t].matrix = matrix; jobs[t].ops = ops; jobs[t].nops = nops;
        jobs[t].data = data; jobs[t].parity = parity;
        jobs[t].s0 = (uint32_t)((uint64_t)n_stripes * t / threads);
        jobs[t].s1 = (uint32_t)((uint64_t)n_stripes * (t + 1) / threads);
        if (pthread_create(&tid[t], NULL, batch_worker, &jobs[t])) { rc = -1; threads = t; break; }
    }
    for (t = 0; t < threads; t++) pthread_join(tid[t], NULL);
    free(bm);
    free(ops);
    return rc;
}

struct dec_job {
    int family, k, m, w, rc;
    uint32_t cs;
    const int *matrix, *bm, *erased;
    uint8_t *chunks;
    uint32_t s0, s1;
};

static void *dec_worker(void *arg)
{
    struct dec_job *jb = (struct dec_job *)arg;
    uint8_t *d[64], *p[64];
    uint32_t s;
    int i, n = jb->k + jb->m;
    for (s = jb->s0; s < jb->s1; s++) {
        for (i = 0; i < jb->k; i++) d[i] = jb->chunks + ((size_t)s * n + i) * jb->cs;
        for (i = 0; i < jb->m; i++) p[i] = jb->chunks + ((size_t)s * n + jb->k + i) * jb->cs;
        if (jb->family == 0) {
            if (orc_rs_decode(jb->k, jb->m, jb->matrix, jb->erased, d, p, jb->cs)) jb->rc = -1;
        } else {
            if (orc_crs_decode(jb->k, jb->m, jb->w, jb->bm, jb->erased, d, p, jb->cs, jb->cs / jb->w)) jb->rc = -1;
        }
    }
    return NULL;
}

/* Multi-threaded in-place decode of a dense [s][k+m][cs] batch, one erasure
 * pattern (erased[i] != 0: chunk i lost) for every stripe; each stripe
 * rebuilds its decoding matrix / schedule as the reference does per call
 * (rscoding.cc:182 -> jerasure.c:223; cauchycoding.cc:173 -> jerasure.c:958).
 * Threads take disjoint stripes (batch_performance.cc:143-154). */
int orc_decode_batch_mt(int family, int k, int m, uint32_t chunk_size, uint8_t *chunks,
                        uint32_t n_stripes, const int *erased, int threads)
{
    int matrix[32 * 32], *bm = NULL, w, t, rc = 0;
    pthread_t tid[256];
    struct dec_job jobs[256];

    if (threads < 1) threads = 1;
    if (threads > 256) threads = 256;
    pthread_once(&g_mt8_once, mt8_build);
    if (family == 0) {
        w = orc_rs_getw((uint32_t)k, (uint32_t)m, chunk_size);
        if (w != 8 || orc_rs_vandermonde_matrix(k, m, 8, matrix)) return -1;
    } else {
        w = orc_cauchy_getw((uint32_t)k, (uint32_t)m, chunk_size);
        if (w < 1 || w > 8 || orc_cauchy_good_matrix(k, m, w, matrix)) return -1;
        bm = malloc(sizeof(int) * (size_t)k * m * w * w);
        orc_matrix_to_bitmatrix(k, m, w, matrix, bm);
    }
    for (t = 0; t < threads; t++) {
        jobs[t].family = family; jobs[t].k = k; jobs[t].m = m; jobs[t].w = w; jobs[t].rc = 0;
        jobs[t].cs = chunk_size; jobs[t].matrix = matrix; jobs[t].bm = bm; jobs[t].erased = erased;
        jobs[t].chunks = chunks;
        jobs[t].s0 = (uint32_t)((uint64_t)n_stripes * t / threads);
        jobs[t].s1 = (uint32_t)((uint64_t)n_stripes * (t + 1) / threads);
        if (pthread_create(&tid[t], NULL, dec_worker, &jobs[t])) { rc = -1; threads = t; break; }
    }
    for (t = 0; t < threads; t++) {
        pthread_join(tid[t], NULL);
        if (jobs[t].rc) rc = -1;
    }
    free(bm);
    return rc;
}
