// ref_isal_plugin.cc — C entry points over MemEC's REAL USE_ISAL=1 plugin.
//
// TEST INFRASTRUCTURE ONLY (fixture generation in this container; never
// part of the product path).  oracle/Makefile `ref` compiles MemEC's own
// common/coding/*.cc with -DUSE_ISAL (as common/coding/Makefile:27-30 does
// for `make USE_ISAL=1`) over ISA-L 2.14's ec_base.c and ec_highlevel_func.c
// (ec_init_tables, ec_highlevel_func.c:33-43), all from their sources under
// /root/reference, into oracle/_ref/libmemec_ref_isal.so.
//
// The one piece of ISA-L that cannot be built here is its multibinary
// dispatcher (ec_multibinary.asm needs yasm, absent from the image).  It
// resolves ec_encode_data / ec_encode_data_update at run time to one of
// ISA-L's own *_base / *_sse / *_avx / *_avx2 targets, all of which compute
// the same bytes; the link binds the two names to the *_base targets with
// --defsym (no code is written for them).  The SIMD variants that
// ec_highlevel_func.c defines are dropped by --gc-sections.
//
// So RSCoding / CauchyCoding's encode (rscoding.cc:51-95,
// cauchycoding.cc:49-85, incl. the startOff/endOff update branch) and decode
// (rscoding.cc:97-187, cauchycoding.cc:87-180, incl. the survivor-row choice
// and the parity-erasure read past the k x k inverse) below are the
// reference's own code, driven the way test/common/coding/coding.cc drives
// the plugin.
#include <cstdint>
#include <cstdlib>
#include <cstring>

#include "common/coding/coding.hh"
#include "common/ds/bitmask_array.hh"
#include "common/ds/chunk_pool.hh"
#include "common/ds/chunk_util.hh"

namespace {
struct RefHandle {
    Coding *coding;
    uint32_t k, m, cs;
};
}  // namespace

extern "C" {

// scheme: 4 = CS_RS (gf_gen_rs_matrix, rscoding.cc:226-228), 7 = CS_CAUCHY
// (gf_gen_cauchy1_matrix, cauchycoding.cc:211-213).
void *refi_instantiate(int scheme, uint32_t k, uint32_t m, uint32_t chunk_size) {
    CodingParams params;
    CodingScheme s = scheme == 7 ? CS_CAUCHY : CS_RS;
    params.setScheme(s);
    params.setK(k);
    params.setM(m);
    ChunkUtil::init(chunk_size, k);
    Coding *c = Coding::instantiate(s, params, chunk_size);
    if (!c) return nullptr;
    return new RefHandle{c, k, m, chunk_size};
}

void refi_destroy(void *hp) {
    RefHandle *h = (RefHandle *)hp;
    delete h->coding;  // Coding::destroy reads an unset scheme
    delete h;
}

// Coding::encode(data, parity, index, startOff, endOff) with the caller's
// parity chunk holding `parity` on entry (the RS update branch XORs into it,
// rscoding.cc:85-88); the chunk's bytes after the call are written back.
// zero_mask bit j => data j is Coding::zeros (the server's delta form).
void refi_encode(void *hp, const uint8_t *data, uint32_t zero_mask, uint8_t *parity, uint32_t index,
                 uint32_t start_off, uint32_t end_off) {
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
    memcpy(ChunkUtil::getData(p), parity, h->cs);
    h->coding->encode(d, p, index, start_off, end_off);
    memcpy(parity, ChunkUtil::getData(p), h->cs);
    pool.free(p);
    for (uint32_t j = 0; j < h->k; j++)
        if (!(zero_mask >> j & 1)) pool.free(d[j]);
}

// Coding::decode(chunks, status) on (k+m) dense chunks; chunks whose present
// bit is clear are cleared first (server_peer_res_worker.cc:818-828) and
// rebuilt in place.  Returns 0 (true) / -1 (false).
int refi_decode(void *hp, uint8_t *chunks, uint64_t present_mask) {
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

// The same decode after filling the stack below the caller with `poison`:
// the plugin reads rows erasures[i] >= k of a k x k inverse it keeps in an
// uninitialised 32 x 32 stack array (rscoding.cc:173-175,
// cauchycoding.cc:164-166), so for an erased PARITY chunk its output depends
// on whatever that stack held.  Poisoning makes the defect show the same way
// on every run (make_golden.py records that it does); erased DATA chunks
// never touch those rows.
__attribute__((noinline)) static void poison_stack(uint8_t poison) {
    volatile uint8_t pad[1 << 16];
    for (size_t i = 0; i < sizeof(pad); i++) pad[i] = poison;
}
int refi_decode_poisoned(void *hp, uint8_t *chunks, uint64_t present_mask, uint8_t poison) {
    poison_stack(poison);
    return refi_decode(hp, chunks, present_mask);
}

}  // extern "C"
