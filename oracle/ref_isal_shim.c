/* ref_isal_shim.c — C entry points over ISA-L 2.14's base (C) erasure-code
 * functions, compiled from /root/reference/lib/isa-l-2.14.0/erasure_code/
 * ec_base.c by oracle/ref.mk.
 *
 * TEST INFRASTRUCTURE ONLY (fixture generation in this container).
 *
 * These are ISA-L's own portable functions, called directly: gf_gen_*_matrix,
 * gf_invert_matrix, gf_vect_mul_init (the 32-byte tables ec_init_tables
 * builds), ec_encode_data_base, ec_encode_data_update_base.  MemEC's USE_ISAL
 * plugin itself (the glue around these calls) is built separately, from its
 * own sources, into libmemec_ref_isal.so (oracle/ref_isal_plugin.cc). */
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
