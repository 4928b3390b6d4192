// bitslice.hpp — bit-sliced GF(2^8) matrix programs for wide codes (more
// than 4 outputs), compiled at run time per matrix (jit.cpp).
//
// c * x over GF(2^8) is linear over GF(2): as an 8 x 8 bit matrix
// B_c[l][x] = bit l of c * 2^x (jerasure_matrix_to_bitmatrix,
// jerasure.c:271-297, applied to the byte-wise families), so output byte bit
// l is the XOR of the input bits x with B_c[l][x] = 1.  Bit-sliced, 32 bytes
// at once: a lane's 32 bytes of a chunk (two 16-byte units 1 KiB apart, so a
// wave's loads stay 1 KiB-contiguous) are 8 dwords; an 8 x 8 bit transpose
// across them (3 swap stages, 2 shifts + 2 v_bitop3 bit-field inserts per
// swap) turns them into 8 planes, plane x holding bit x of all 32 bytes.  An
// output plane (r, l) is then the XOR of source planes (j, x) over the ones
// of the (8 nd) x (8 ns) bitmatrix, and an inverse transpose puts the bytes
// back.  The XORs use the "four Russians" split: per source, the 15 non-zero
// XOR combinations of planes 0-3 and of planes 4-7 are formed once (the ones
// the matrix uses), and every output plane takes one of each — one 3-input
// v_bitop3 XOR per (source, output plane), the combination indices being
// compile-time constants of this matrix's program.  Per source dword that is
// 6 (transpose) + 22/8 (combinations) + R (accumulate) operations against 5 +
// 4.5 R for the v_perm products of gf8_mg_kernel: R = 8 rows, 16 sources,
// ~20 against ~41 (SURVEY §7 hard part (c)).
//
// A program is straight-line SSA over 32-bit values (BsOp), generated here
// from the coefficients, interpreted on the CPU by bs_run (tests: every
// program checked against GF(2^8) products before any device runs it) and
// emitted as HIP source by bs_source (compiled with hiprtc for gfx950).
#pragma once

#include <cstdint>
#include <string>
#include <vector>

namespace mec {

enum class BsOpc : uint8_t {
    kLoad,     // v = dword d of source j's 32 bytes (a = j, b = d)
    kLoadOut,  // v = dword d of output r's old 32 bytes (accumulate; a = r, b = d)
    kShl,      // v = a << imm
    kShr,      // v = a >> imm
    kBfi,      // v = (imm & a) | (~imm & b)     (v_bitop3 0xCA with a literal mask)
    kXor2,     // v = a ^ b
    kXor3,     // v = a ^ b ^ c                  (v_bitop3 0x96)
    kStore,    // dword d of output r = a (a = value, b = r, c = d)
};

struct BsOp {
    BsOpc op;
    int32_t a, b, c;
    uint32_t imm;
};

struct BsProgram {
    int ns = 0, nd = 0;
    bool accumulate = false;
    std::vector<BsOp> ops;  // value i is defined by ops[i] (kStore defines none)
    // operation counts (VALU estimate per lane per 32 bytes of every chunk)
    uint32_t n_transpose = 0, n_combine = 0, n_accumulate = 0;
};

// The program for outputs (^)= coef (nd x ns, row-major over GF(2^8) with
// the 0x11d polynomial) * sources.
BsProgram bs_build(const uint8_t *coef, int nd, int ns, bool accumulate);
// The arithmetic-free twin of a bs_build program (mec_set_probe): the same
// loads and stores, every output the plain XOR of the sources (8 dwords x
// ns / 2 three-input XORs), so a launch measures what the access pattern
// alone sustains.  Not a code.
BsProgram bs_build_twin(int nd, int ns, bool accumulate);
// CPU interpreter: src = ns chunks of 32 bytes, out = nd chunks of 32 bytes
// (read too when accumulating).  Bytes [0, 16) are unit 0, [16, 32) unit 1.
void bs_run(const BsProgram &p, const uint8_t *const *src, uint8_t *const *out);
// HIP source of the kernel `mec_bs` (one-wave blocks, 2 KiB of every chunk
// per block; strided or gathered addressing, BsParams below).
// waves > 0: compiled for at least that many waves per SIMD
// (amdgpu_waves_per_eu; the register budget shrinks accordingly).
// prefetch > 0: at most that many sources' loads issued ahead of the
// combine (0: every load first).
// loop (gathered only): the block walks p.tpb tiles per pointer-row read;
// otherwise it codes one tile, straight-line (launch with tpb = 1).
// fence: between sources, an empty asm that takes every value live across
// the boundary (the output planes' running XORs) and the next source's
// loaded units, so the compiler cannot start a source's transposes and
// combinations before the previous source's are consumed (one source's
// combinations live at a time).
// vrow (gathered): the block's whole pointer row arrives in one vector load
// (one lane per entry, read back with v_readlane at each use); otherwise
// each entry is a scalar load at its use, and the compiler waits on each.
std::string bs_source(const BsProgram &p, bool gather, int waves = 0, int prefetch = 0, bool loop = false,
                      bool fence = false, bool vrow = false);

// Kernel arguments of every generated kernel (the same layout in the
// generated source, bs_source).  Strided: source j of stripe s at src + s *
// sss + src_off[j]; gathered (stab != 0): at stab[(s0 + s) * sstride +
// src_off[j]] (0 = an all-zero chunk), output r likewise.
struct BsParams {
    const uint8_t *src;
    uint8_t *dst;
    int64_t sss, dss;
    const uint64_t *stab, *dtab;
    uint32_t sstride, dstride;
    uint32_t chunk, tiles, xcd, win, s0, tpb;  // tiles = blocks per stripe, each tpb 2 KiB tiles; xcd: XCD runs
    int64_t src_off[32];
    int64_t dst_off[32];
};

}  // namespace mec
