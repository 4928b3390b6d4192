// bitslice.cpp — bit-sliced GF(2^8) programs for wide codes: generation,
// CPU interpretation and HIP source emission (see bitslice.hpp).
#include "bitslice.hpp"

#include <cstdio>
#include <cstring>
#include <string>

#include "gf_math.hpp"

namespace mec {
namespace {

// The three swap stages of an 8 x 8 bit transpose over 8 dwords (each dword
// carrying 4 independent byte rows): rows (i, i + d) exchange the bit block
// under mask m (shifted by s into a).  Hacker's Delight transpose8, SWAR.
struct Stage {
    int d, s;
    uint32_t m;
};
constexpr Stage kStages[3] = {{4, 4, 0x0F0F0F0Fu}, {2, 2, 0x33333333u}, {1, 1, 0x55555555u}};

struct Builder {
    BsProgram p;
    int emit(BsOpc op, int a = -1, int b = -1, int c = -1, uint32_t imm = 0) {
        p.ops.push_back(BsOp{op, a, b, c, imm});
        return int(p.ops.size()) - 1;
    }
    // rows r[0..7] -> transposed in place (value ids); 4 ops per swap
    void transpose(int (&r)[8], uint32_t &count) {
        for (const Stage &st : kStages)
            for (int i = 0; i < 8; ++i) {
                if (i & st.d) continue;
                const int a = r[i], b = r[i + st.d];
                // a' = bits (m << s) from b << s, the rest from a;
                // b' = bits m from a >> s, the rest from b
                const int bs = emit(BsOpc::kShl, b, -1, -1, uint32_t(st.s));
                const int na = emit(BsOpc::kBfi, bs, a, -1, st.m << st.s);
                const int as = emit(BsOpc::kShr, a, -1, -1, uint32_t(st.s));
                const int nb = emit(BsOpc::kBfi, as, b, -1, st.m);
                r[i] = na;
                r[i + st.d] = nb;
                count += 4;
            }
    }
};

// Accumulator of one output plane: terms folded two at a time into 3-input
// XORs (a pending term waits for a partner).
struct Acc {
    int v = -1, pend = -1;
};

void acc_add(Builder &B, Acc &a, int t, uint32_t &count) {
    if (a.v < 0) {
        a.v = t;
        return;
    }
    if (a.pend < 0) {
        a.pend = t;
        return;
    }
    a.v = B.emit(BsOpc::kXor3, a.v, a.pend, t);
    a.pend = -1;
    ++count;
}

int acc_value(Builder &B, Acc &a, uint32_t &count) {
    if (a.pend >= 0) {
        a.v = B.emit(BsOpc::kXor2, a.v, a.pend);
        a.pend = -1;
        ++count;
    }
    return a.v;
}

}  // namespace

BsProgram bs_build(const uint8_t *coef, int nd, int ns, bool accumulate) {
    Builder B;
    B.p.ns = ns;
    B.p.nd = nd;
    B.p.accumulate = accumulate;
    const Field &f = Field::get(8);
    // rowbits[(r * 8 + l) * ns + j] = byte x-bits of row l of block (r, j)
    std::vector<uint8_t> rowbits(size_t(nd) * 8 * ns, 0);
    for (int r = 0; r < nd; ++r)
        for (int j = 0; j < ns; ++j) {
            const unsigned c = coef[size_t(r) * ns + j];
            for (int x = 0; x < 8; ++x) {
                const unsigned e = f.mul(c, 1u << x);
                for (int l = 0; l < 8; ++l)
                    if (e >> l & 1) rowbits[(size_t(r) * 8 + l) * ns + j] |= uint8_t(1u << x);
            }
        }
    std::vector<Acc> acc(size_t(nd) * 8);
    for (int j = 0; j < ns; ++j) {
        int P[8];
        for (int d = 0; d < 8; ++d) P[d] = B.emit(BsOpc::kLoad, j, d);
        B.transpose(P, B.p.n_transpose);
        // the combinations this source's rows use: lo = planes 0-3, hi = 4-7
        bool need[2][16] = {};
        for (int q = 0; q < nd * 8; ++q) {
            const uint8_t bits = rowbits[size_t(q) * ns + j];
            need[0][bits & 15] = true;
            need[1][bits >> 4] = true;
        }
        int comb[2][16];
        for (int h = 0; h < 2; ++h) {
            // a combination needs its smaller parts: mark downwards
            for (int idx = 15; idx > 0; --idx)
                if (need[h][idx] && (idx & (idx - 1))) need[h][idx & (idx - 1)] = true;
            comb[h][0] = -1;
            for (int idx = 1; idx < 16; ++idx) {
                comb[h][idx] = -1;
                if (!need[h][idx]) continue;
                const int low = __builtin_ctz(unsigned(idx));
                const int rest = idx & (idx - 1);
                if (!rest) {
                    comb[h][idx] = P[4 * h + low];
                } else {
                    comb[h][idx] = B.emit(BsOpc::kXor2, comb[h][rest], P[4 * h + low]);
                    ++B.p.n_combine;
                }
            }
        }
        for (int q = 0; q < nd * 8; ++q) {
            const uint8_t bits = rowbits[size_t(q) * ns + j];
            if (bits & 15) acc_add(B, acc[q], comb[0][bits & 15], B.p.n_accumulate);
            if (bits >> 4) acc_add(B, acc[q], comb[1][bits >> 4], B.p.n_accumulate);
        }
    }
    for (int r = 0; r < nd; ++r) {
        int O[8];
        int zero = -1;
        for (int l = 0; l < 8; ++l) {
            int v = acc[size_t(r) * 8 + l].v < 0 ? -1 : acc_value(B, acc[size_t(r) * 8 + l], B.p.n_accumulate);
            if (v < 0) {  // an all-zero output plane (an all-zero coefficient row)
                if (zero < 0) zero = B.emit(BsOpc::kXor2, -1, -1);
                v = zero;
            }
            O[l] = v;
        }
        B.transpose(O, B.p.n_transpose);
        for (int d = 0; d < 8; ++d) {
            int v = O[d];
            if (accumulate) {
                const int old = B.emit(BsOpc::kLoadOut, r, d);
                v = B.emit(BsOpc::kXor2, v, old);
            }
            B.emit(BsOpc::kStore, v, r, d);
        }
    }
    return B.p;
}

BsProgram bs_build_twin(int nd, int ns, bool accumulate) {
    Builder B;
    B.p.ns = ns;
    B.p.nd = nd;
    B.p.accumulate = accumulate;
    int x[8];
    for (int j = 0; j < ns; ++j) {
        for (int d = 0; d < 8; ++d) {
            const int v = B.emit(BsOpc::kLoad, j, d);
            x[d] = j == 0 ? v : B.emit(BsOpc::kXor2, x[d], v);
        }
    }
    for (int r = 0; r < nd; ++r)
        for (int d = 0; d < 8; ++d) {
            int v = x[d];
            if (accumulate) v = B.emit(BsOpc::kXor2, v, B.emit(BsOpc::kLoadOut, r, d));
            B.emit(BsOpc::kStore, v, r, d);
        }
    return B.p;
}

void bs_run(const BsProgram &p, const uint8_t *const *src, uint8_t *const *out) {
    std::vector<uint32_t> v(p.ops.size(), 0);
    auto dword = [](const uint8_t *b, int d) {
        uint32_t x;
        std::memcpy(&x, b + 4 * d, 4);
        return x;
    };
    std::vector<std::vector<uint8_t>> old(size_t(p.nd));
    if (p.accumulate)
        for (int r = 0; r < p.nd; ++r) old[size_t(r)].assign(out[r], out[r] + 32);
    for (size_t i = 0; i < p.ops.size(); ++i) {
        const BsOp &o = p.ops[i];
        switch (o.op) {
            case BsOpc::kLoad: v[i] = dword(src[o.a], o.b); break;
            case BsOpc::kLoadOut: v[i] = dword(old[size_t(o.a)].data(), o.b); break;
            case BsOpc::kShl: v[i] = v[size_t(o.a)] << o.imm; break;
            case BsOpc::kShr: v[i] = v[size_t(o.a)] >> o.imm; break;
            case BsOpc::kBfi: v[i] = (o.imm & v[size_t(o.a)]) | (~o.imm & v[size_t(o.b)]); break;
            case BsOpc::kXor2: v[i] = (o.a < 0 ? 0 : v[size_t(o.a)]) ^ (o.b < 0 ? 0 : v[size_t(o.b)]); break;
            case BsOpc::kXor3: v[i] = v[size_t(o.a)] ^ v[size_t(o.b)] ^ v[size_t(o.c)]; break;
            case BsOpc::kStore: std::memcpy(out[o.b] + 4 * o.c, &v[size_t(o.a)], 4); break;
        }
    }
}

std::string bs_source(const BsProgram &p, bool gather, int waves, int prefetch, bool loop, bool fence, bool vrow) {
    std::string s;
    s.reserve(p.ops.size() * 48 + 4096);
    s += gather ? "#define MEC_GATHER 1\n" : "#define MEC_GATHER 0\n";
    s += gather && vrow ? "#define MEC_VROW 1\n" : "#define MEC_VROW 0\n";
    if (waves > 0) s += "#define MEC_WAVES __attribute__((amdgpu_waves_per_eu(" + std::to_string(waves) + ")))\n";
    else s += "#define MEC_WAVES\n";
    s += R"HIP(
typedef unsigned int u32;
typedef unsigned long long u64;
typedef long long i64;
typedef u32 u32x4 __attribute__((ext_vector_type(4)));
struct BsParams {
    const unsigned char *src;
    unsigned char *dst;
    i64 sss, dss;
    const u64 *stab, *dtab;
    u32 sstride, dstride;
    u32 chunk, tiles, xcd, win, s0, tpb;
    i64 src_off[32];
    i64 dst_off[32];
};
__device__ __forceinline__ __amdgpu_buffer_rsrc_t mec_rsrc(u64 a, u32 bytes) {
    return __builtin_amdgcn_make_buffer_rsrc((void *)a, 0, a ? (int)bytes : 0, 0x00020000);
}
__device__ __forceinline__ u64 mec_uniform64(u64 v) {
    const u32 lo = __builtin_amdgcn_readfirstlane((u32)v), hi = __builtin_amdgcn_readfirstlane((u32)(v >> 32));
    return ((u64)hi << 32) | lo;
}
#define LD(r, o) __builtin_amdgcn_raw_buffer_load_b128(r, o, 0, 2)
__device__ __forceinline__ void mec_st(u32 a, u32 b, u32 c, u32 d, __amdgpu_buffer_rsrc_t r, u32 o) {
    __builtin_amdgcn_raw_buffer_store_b128((u32x4){a, b, c, d}, r, o, 0, 18);
}
#define BFI(m, a, b) ((u32)__builtin_amdgcn_bitop3_b32(m, a, b, 0xCA))
#define X3(a, b, c) ((u32)__builtin_amdgcn_bitop3_b32(a, b, c, 0x96))
extern "C" __global__ __launch_bounds__(64) MEC_WAVES void mec_bs(const BsParams p) {
    u32 bid = blockIdx.x;
    if (!MEC_GATHER && p.win > 1) {  // in-place layouts: windows taken round-robin (stream_common.hpp block_order)
        const u32 per = gridDim.x / p.win;
        if (bid < per * p.win) bid = (bid % p.win) * per + bid / p.win;
    } else if (p.xcd) {  // blocks dealt round-robin over the 8 XCDs: each XCD one contiguous run (plan_bs)
        const u32 per = gridDim.x >> 3;
        if (bid < per * 8u) bid = (bid & 7u) * per + (bid >> 3);
    }
    // block b of a stripe codes tiles [b * tpb, (b + 1) * tpb): its chunk
    // addresses (pointer-row loads when gathered) are read once
    const u32 stripe = bid / p.tiles, tile0 = (bid - stripe * p.tiles) * p.tpb;
    if (tile0 * 2048u >= p.chunk) return;
    const u64 gs = (u64)p.s0 + stripe;
#if MEC_GATHER && !MEC_VROW
    auto src_at = [&](int j) -> u64 { return mec_uniform64(p.stab[gs * p.sstride + p.src_off[j]]); };
    auto dst_at = [&](int r) -> u64 { return mec_uniform64(p.dtab[gs * p.dstride + p.dst_off[r]]); };
#elif !MEC_GATHER
    auto src_at = [&](int j) -> u64 { return (u64)(p.src + (i64)stripe * p.sss + p.src_off[j]); };
    auto dst_at = [&](int r) -> u64 { return (u64)(p.dst + (i64)stripe * p.dss + p.dst_off[r]); };
#endif
)HIP";
    if (gather && vrow) {
        // the block's pointer row in one vector load: lane j < 32 fetches
        // source j's entry, lane 32 + r output r's; each use reads its lane
        // back into SGPRs (v_readlane), so no source waits on a scalar load
        s += "    i64 mo = -1;\n";
        for (int j = 0; j < p.ns; ++j)
            s += "    mo = threadIdx.x == " + std::to_string(j) + "u ? p.src_off[" + std::to_string(j) + "] : mo;\n";
        for (int r = 0; r < p.nd; ++r)
            s += "    mo = threadIdx.x == " + std::to_string(32 + r) + "u ? p.dst_off[" + std::to_string(r) + "] : mo;\n";
        s += "    const u64 *mrow = threadIdx.x < 32u ? p.stab + gs * p.sstride : p.dtab + gs * p.dstride;\n"
             "    const u64 mptr = mo >= 0 ? mrow[mo] : 0ull;\n"
             "    auto lane64 = [&](int l) -> u64 {\n"
             "        return ((u64)(u32)__builtin_amdgcn_readlane((int)(u32)(mptr >> 32), l) << 32) |\n"
             "               (u32)__builtin_amdgcn_readlane((int)(u32)mptr, l);\n"
             "    };\n"
             "    auto src_at = [&](int j) -> u64 { return lane64(j); };\n"
             "    auto dst_at = [&](int r) -> u64 { return lane64(32 + r); };\n";
    }
    char buf[320];
    // source units: the first `depth` sources' loads up front, then each
    // further source's loads just before the combine of the source `depth`
    // places earlier (depth 0: all loads first)
    const int depth = prefetch > 0 && prefetch < p.ns ? prefetch : p.ns;
    // chunk addresses at each load / store (24 buffer resources held at
    // once would be 96 SGPRs and spill into VGPR lanes)
    auto emit_load = [&](int j) {
        std::snprintf(buf, sizeof buf,
                      "    u32x4 sa%d = LD(mec_rsrc(sp%d, p.chunk), off), sb%d = LD(mec_rsrc(sp%d, p.chunk), off + 1024u);\n",
                      j, j, j, j);
        s += buf;
    };
    // value names (renamed at fences) and each value's last use
    std::vector<std::string> nm(p.ops.size());
    std::vector<size_t> last(p.ops.size(), 0);
    for (size_t i = 0; i < p.ops.size(); ++i) {
        nm[i] = "v" + std::to_string(i);
        const BsOp &o = p.ops[i];
        auto use = [&](int x) {
            if (x >= 0) last[size_t(x)] = i;
        };
        switch (o.op) {
            case BsOpc::kShl:
            case BsOpc::kShr: use(o.a); break;
            case BsOpc::kBfi:
            case BsOpc::kXor2: use(o.a); use(o.b); break;
            case BsOpc::kXor3: use(o.a); use(o.b); use(o.c); break;
            case BsOpc::kStore: use(o.a); break;
            default: break;
        }
    }
    int nfence = 0;
    auto emit_fence = [&](size_t i0, int j) {  // before op i0, where source j starts
        std::vector<size_t> live;
        for (size_t x = 0; x < i0; ++x)
            if (p.ops[x].op != BsOpc::kStore && last[x] >= i0) live.push_back(x);
        for (size_t g = 0; g < live.size(); g += 8) {
            std::string decl, cons;
            for (size_t t = g; t < live.size() && t < g + 8; ++t) {
                const std::string w = "f" + std::to_string(nfence) + "_" + std::to_string(live[t]);
                decl += "    u32 " + w + " = " + nm[live[t]] + ";\n";
                cons += std::string(cons.empty() ? "" : ", ") + "\"+v\"(" + w + ")";
                nm[live[t]] = w;
            }
            s += decl + "    __asm__ volatile(\"\" : " + cons + ");\n";
        }
        std::snprintf(buf, sizeof buf, "    __asm__ volatile(\"\" : \"+v\"(sa%d), \"+v\"(sb%d));\n", j, j);
        s += buf;
        ++nfence;
    };
    // (gathered: with vrow each use reads its entry back from the row's
    // lane (two VGPRs held across a tile loop); without, the entry is
    // re-read per use, from the scalar cache after the first)
    for (int j = 0; j < p.ns; ++j) {
        std::snprintf(buf, sizeof buf, "#define sp%d src_at(%d)\n", j, j);
        s += buf;
    }
    for (int r = 0; r < p.nd; ++r) {
        std::snprintf(buf, sizeof buf, "#define dp%d dst_at(%d)\n", r, r);
        s += buf;
    }
    // looped gathered kernels walk the block's tiles; the others take one
    // tile per block (straight-line: the loop costs registers).  With vrow no
    // lane leaves before the row's last v_readlane: lanes past the chunk's
    // end run on, their loads reading zeros and their stores dropped by the
    // buffer resource's bounds (num_records = chunk)
    const char *past = gather && vrow ? "" : loop ? "    if (off >= p.chunk) break;\n" : "    if (off >= p.chunk) return;\n";
    if (gather && loop)
        s += std::string("    for (u32 t = 0; t < p.tpb; ++t) {\n"
                         "    if ((tile0 + t) * 2048u >= p.chunk) break;\n"
                         "    const u32 off = (tile0 + t) * 2048u + threadIdx.x * 16u;\n") + past;
    else
        s += std::string("    {\n"
                         "    const u32 off = tile0 * 2048u + threadIdx.x * 16u;\n") + past;
    for (int j = 0; j < depth; ++j) emit_load(j);
    int next_load = depth;
    for (int r = 0; r < p.nd; ++r) {
        if (p.accumulate) {
            std::snprintf(buf, sizeof buf,
                          "    const u32x4 oa%d = LD(mec_rsrc(dp%d, p.chunk), off), ob%d = LD(mec_rsrc(dp%d, p.chunk), off + 1024u);\n",
                          r, r, r, r);
            s += buf;
        }
    }
    static const char comp[4] = {'x', 'y', 'z', 'w'};
    // stores gathered per output, emitted once its 8 dwords exist
    std::vector<std::vector<int>> stored(size_t(p.nd), std::vector<int>(8, -1));
    for (size_t i = 0; i < p.ops.size(); ++i) {
        const BsOp &o = p.ops[i];
        if (o.op == BsOpc::kLoad && o.b == 0 && o.a > 0 && next_load < p.ns && next_load <= o.a + depth - 1) {
            emit_load(next_load++);  // source o.a starts: keep `depth` sources in flight
        }
        if (fence && o.op == BsOpc::kLoad && o.b == 0 && o.a > 0) emit_fence(i, o.a);
        auto N = [&](int x) { return nm[size_t(x)].c_str(); };
        switch (o.op) {
            case BsOpc::kLoad:
                std::snprintf(buf, sizeof buf, "    const u32 v%zu = s%c%d.%c;\n", i, o.b < 4 ? 'a' : 'b', o.a, comp[o.b & 3]);
                break;
            case BsOpc::kLoadOut:
                std::snprintf(buf, sizeof buf, "    const u32 v%zu = o%c%d.%c;\n", i, o.b < 4 ? 'a' : 'b', o.a, comp[o.b & 3]);
                break;
            case BsOpc::kShl: std::snprintf(buf, sizeof buf, "    const u32 v%zu = %s << %u;\n", i, N(o.a), o.imm); break;
            case BsOpc::kShr: std::snprintf(buf, sizeof buf, "    const u32 v%zu = %s >> %u;\n", i, N(o.a), o.imm); break;
            case BsOpc::kBfi:
                std::snprintf(buf, sizeof buf, "    const u32 v%zu = BFI(0x%08xu, %s, %s);\n", i, o.imm, N(o.a), N(o.b));
                break;
            case BsOpc::kXor2:
                if (o.a < 0)
                    std::snprintf(buf, sizeof buf, "    const u32 v%zu = 0u;\n", i);
                else
                    std::snprintf(buf, sizeof buf, "    const u32 v%zu = %s ^ %s;\n", i, N(o.a), N(o.b));
                break;
            case BsOpc::kXor3:
                std::snprintf(buf, sizeof buf, "    const u32 v%zu = X3(%s, %s, %s);\n", i, N(o.a), N(o.b), N(o.c));
                break;
            case BsOpc::kStore: {
                stored[size_t(o.b)][size_t(o.c)] = o.a;
                buf[0] = 0;
                bool all = true;
                for (int d = 0; d < 8; ++d) all = all && stored[size_t(o.b)][size_t(d)] >= 0;
                if (all) {
                    const std::vector<int> &w = stored[size_t(o.b)];
                    std::snprintf(buf, sizeof buf,
                                  "    mec_st(%s, %s, %s, %s, mec_rsrc(dp%d, p.chunk), off);\n"
                                  "    mec_st(%s, %s, %s, %s, mec_rsrc(dp%d, p.chunk), off + 1024u);\n",
                                  N(w[0]), N(w[1]), N(w[2]), N(w[3]), o.b, N(w[4]), N(w[5]), N(w[6]), N(w[7]), o.b);
                }
                break;
            }
        }
        s += buf;
    }
    s += "    }\n}\n";
    return s;
}

}  // namespace mec
