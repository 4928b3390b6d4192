/* ref_isal_shim.c — C entry points over ISA-L 2.14's base (C) erasure-code
 * functions, compiled from /root/reference/lib/isa-l-2.14.0/erasure_code/
 * ec_base.c by oracle/ref.mk.
 *
 * TEST INFRASTRUCTURE ONLY (fixture generation in this container).
 *
 * MemEC's USE_ISAL=1 plugin build is NOT built here: its ec_encode_data /
 * ec_init_tables come from the yasm multibinary dispatcher
 * (ec_multibinary.asm, ec_highlevel_func.c) and yasm is absent from the
 * image.  These entry points instead call the reference's own portable
 * functions in the order the plugin does (rscoding.cc:81-89,155-177,226-228):
 * gf_gen_*_matrix, gf_invert_matrix, gf_vect_mul_init (the 32-byte tables
 * ec_init_tables builds), ec_encode_data_base, ec_encode_data_update_base. */
#include <stdlib.h>
#include <string.h>
#include "erasure_code.h"

void ref_isal_gen_rs_matrix(unsigned char *a, int rows, int k) { gf_gen_rs_matrix(a, rows, k); }
void ref_isal_gen_cauchy1_matrix(unsigned char *a, int rows, int k) { gf_gen_cauchy1_matrix(a, rows, k); }
int ref_isal_invert_matrix(unsigned char *in, unsigned char *out, int n) { return gf_invert_matrix(in, out, n); }
unsigned char ref_isal_gf_mul(unsigned char a, unsigned char b) { return gf_mul(a, b); }

static void tables(int k, int rows, const unsigned char *coef, unsigned char *tbl)
{
    int i;
    for (i = 0; i < k * rows; i++) gf_vect_mul_init(coef[i], tbl + 32 * i);
}

/* coef: rows*k; src: k pointers; dst: rows pointers. */
void ref_isal_encode(int len, int k, int rows, const unsigned char *coef,
                     unsigned char **src, unsigned char **dst)
{
    unsigned char tbl[32 * 32 * 32];
    tables(k, rows, coef, tbl);
    ec_encode_data_base(len, k, rows, tbl, src, dst);
}

void ref_isal_encode_update(int len, int k, int rows, int col, const unsigned char *coef,
                            unsigned char *src, unsigned char **dst)
{
    unsigned char tbl[32 * 32 * 32];
    tables(k, rows, coef, tbl);
    ec_encode_data_update_base(len, k, rows, col, tbl, src, dst);
}

/* MemEC's USE_ISAL plugin bodies, step for step, over the base functions
 * above (ec_init_tables == gf_vect_mul_init per coefficient,
 * ec_highlevel_func.c:33-43; ec_encode_data == ec_encode_data_base).
 * family 0 = RSCoding (gf_gen_rs_matrix, rscoding.cc:226-228),
 * 1 = CauchyCoding (gf_gen_cauchy1_matrix, cauchycoding.cc:211-213). */
#define ISAL_N_MAX 32

static void plugin_matrix(int family, int k, int m, unsigned char *enc)
{
    if (family == 0)
        gf_gen_rs_matrix(enc, m + k, k);
    else
        gf_gen_cauchy1_matrix(enc, m + k, k);
}

/* RSCoding::encode / CauchyCoding::encode with USE_ISAL (rscoding.cc:51-95,
 * cauchycoding.cc:49-85).  data: k chunk pointers; parity: the caller's
 * parity chunk for `index` (1-based), read-modify-written by the RS update
 * branch, overwritten otherwise.  The other m-1 parities go to scratch. */
void ref_isal_plugin_encode(int family, int k, int m, int chunk, unsigned char **data,
                            unsigned char *parity, unsigned index, unsigned startOff, unsigned endOff)
{
    unsigned char enc[ISAL_N_MAX * ISAL_N_MAX], tbl[ISAL_N_MAX * ISAL_N_MAX * 32];
    unsigned char *code[ISAL_N_MAX], *scratch;
    int i;
    unsigned c;
    memset(enc, 0, sizeof(enc));
    plugin_matrix(family, k, m, enc);
    tables(k, m, enc + k * k, tbl);
    scratch = (unsigned char *)calloc((size_t)m, (size_t)chunk);
    for (i = 0; i < m; i++)
        code[i] = (unsigned)i == index - 1 ? parity : scratch + (size_t)i * chunk;
    if (family == 0 && !(startOff == 0 && endOff == 0)) {
        /* rscoding.cc:85-88: in-place XOR update per touched data column */
        for (c = startOff / chunk; c <= (endOff - 1) / chunk; c++)
            ec_encode_data_update_base(chunk, k, m, (int)c, tbl, data[c], code);
    } else {
        /* rscoding.cc:83, cauchycoding.cc:79 (Cauchy ignores the offsets) */
        ec_encode_data_base(chunk, k, m, tbl, data, code);
    }
    free(scratch);
}

/* RSCoding::decode / CauchyCoding::decode with USE_ISAL (rscoding.cc:97-187,
 * cauchycoding.cc:87-180).  chunks: k+m pointers, rebuilt in place where
 * bit i of present is clear.  Returns 1 (true) / 0 (false) as the plugin.
 *
 * The plugin reads row erasures[i] of the k x k inverse for EVERY erased
 * chunk (rscoding.cc:173-175); for an erased parity (index >= k) that row
 * lies past the k*k bytes gf_invert_matrix writes, in the uninitialised
 * rest of the stack array.  Here that rest is zero, so such a chunk comes
 * out all-zero — the deterministic stand-in for undefined bytes. */
int ref_isal_plugin_decode(int family, int k, int m, int chunk, unsigned char **chunks, unsigned long long present)
{
    unsigned char enc[ISAL_N_MAX * ISAL_N_MAX];
    unsigned char decodeMatrix[ISAL_N_MAX * ISAL_N_MAX], invertedMatrix[ISAL_N_MAX * ISAL_N_MAX];
    unsigned char gftbl[ISAL_N_MAX * ISAL_N_MAX * 32];
    unsigned char *alive[ISAL_N_MAX], *missing[ISAL_N_MAX];
    int erasures[ISAL_N_MAX + 1], failed = 0, pos = 0, rpos = 0, i;
    for (i = 0; i < k + m; i++)
        if (!(present >> i & 1)) failed++;
    if (failed > m) return 0;
    if (failed == 0) return 1;
    memset(enc, 0, sizeof(enc));
    plugin_matrix(family, k, m, enc);
    for (i = 0; i < k + m; i++) {
        if (!(present >> i & 1)) {
            erasures[pos] = i;
            missing[pos++] = chunks[i];
        } else {
            alive[rpos++] = chunks[i];
        }
    }
    erasures[failed] = -1;
    memset(invertedMatrix, 0, sizeof(invertedMatrix));
    {
        int r, oi = 0;
        pos = 0;
        for (r = 0; r < k + m; r++) {
            if (r != erasures[pos])
                memcpy(decodeMatrix + k * oi++, enc + k * r, (size_t)k);
            else
                pos++;
        }
    }
    if (gf_invert_matrix(decodeMatrix, invertedMatrix, k) < 0) return 0;
    memset(decodeMatrix, 0, sizeof(decodeMatrix));
    for (i = 0; i < failed; i++)
        memcpy(decodeMatrix + k * i, invertedMatrix + k * erasures[i], (size_t)k);
    tables(k, failed, decodeMatrix, gftbl);
    ec_encode_data_base(chunk, k, failed, gftbl, alive, missing);
    return 1;
}
