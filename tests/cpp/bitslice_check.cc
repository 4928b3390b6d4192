// bitslice_check.cc — CPU check of the bit-sliced GF(2^8) programs
// (memec_amd/csrc/bitslice.cpp) before any device runs one: for random and
// structured coefficient matrices of every wide shape (5..31 outputs, k + m
// <= 32), the program interpreted over random 32-byte chunks equals the
// byte-wise GF(2^8) products (0x11d), overwrite and accumulate; the emitted
// HIP source is generated for each.  Prints "ok <programs> <ops>".
// With a directory argument it also writes the RS(16,8)-shaped encode
// program's kernel in its three addressing forms as the JIT builds them by
// default (strided without scheduling fences, gathered straight-line and
// gathered looping over tiles with them), and the strided form with fences,
// as <dir>/bs_{strided,gather1,gather4,strided_fence}.hip, for a gfx950
// compile check (tests/test_abi.py).
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <vector>

#include "bitslice.hpp"
#include "gf_math.hpp"

using namespace mec;

int main(int argc, char **argv) {
    const Field &f = Field::get(8);
    std::mt19937_64 rng(12345);
    long programs = 0, ops = 0;
    for (int nd = 1; nd <= 31; ++nd)
        for (int ns = 1; ns + nd <= 32; ++ns)
            for (int kind = 0; kind < 3; ++kind)
                for (int acc = 0; acc < 2; ++acc) {
                    std::vector<uint8_t> coef(size_t(nd) * ns);
                    for (size_t i = 0; i < coef.size(); ++i) {
                        const uint8_t c = uint8_t(rng());
                        // kind 1: Vandermonde-like ones in row 0 / column 0; kind 2: sparse with zeros
                        coef[i] = kind == 1 && (i < size_t(ns) || i % size_t(ns) == 0) ? 1 : kind == 2 && (c & 3) == 0 ? 0 : c;
                    }
                    BsProgram p = bs_build(coef.data(), nd, ns, acc != 0);
                    for (int trial = 0; trial < 3; ++trial) {
                        std::vector<std::vector<uint8_t>> src(size_t(ns), std::vector<uint8_t>(32)),
                            out(size_t(nd), std::vector<uint8_t>(32));
                        std::vector<const uint8_t *> sp;
                        std::vector<uint8_t *> op;
                        for (auto &c : src) {
                            for (auto &b : c) b = uint8_t(rng());
                            sp.push_back(c.data());
                        }
                        for (auto &c : out) {
                            for (auto &b : c) b = uint8_t(rng());
                            op.push_back(c.data());
                        }
                        std::vector<std::vector<uint8_t>> want = out;
                        for (int r = 0; r < nd; ++r)
                            for (int b = 0; b < 32; ++b) {
                                uint8_t x = acc ? want[size_t(r)][size_t(b)] : 0;
                                for (int j = 0; j < ns; ++j) x ^= f.mul(coef[size_t(r) * ns + j], src[size_t(j)][size_t(b)]);
                                want[size_t(r)][size_t(b)] = x;
                            }
                        bs_run(p, sp.data(), op.data());
                        if (out != want) {
                            std::printf("MISMATCH nd=%d ns=%d kind=%d acc=%d trial=%d\n", nd, ns, kind, acc, trial);
                            return 1;
                        }
                    }
                    if (nd >= 5 && kind == 0 && acc == 0 && (ns == 16 || ns == 12) && nd == 8)
                        std::printf("shape %dx%d: %zu ops (transpose %u, combine %u, accumulate %u), source %zu bytes\n", nd,
                                    ns, p.ops.size(), p.n_transpose, p.n_combine, p.n_accumulate, bs_source(p, false).size());
                    (void)bs_source(p, (programs & 1) != 0);
                    ++programs;
                    ops += long(p.ops.size());
                }
    if (argc > 1) {
        std::vector<uint8_t> coef(8 * 16);
        for (size_t i = 0; i < coef.size(); ++i) coef[i] = i < 16 || i % 16 == 0 ? 1 : uint8_t(rng() | 2);
        const BsProgram p = bs_build(coef.data(), 8, 16, false);
        const struct {
            const char *name;
            bool gather, loop;
            int prefetch;
            bool fence, vrow;
        } forms[] = {{"strided", false, false, 4, false, false}, {"gather1", true, false, 4, true, true},
                     {"gather4", true, true, 4, true, true},     {"strided_fence", false, false, 4, true, false},
                     {"gather1_srow", true, false, 4, true, false}};
        for (const auto &fm : forms) {
            const std::string path = std::string(argv[1]) + "/bs_" + fm.name + ".hip";
            FILE *out = std::fopen(path.c_str(), "w");
            if (!out) return 2;
            const std::string src = bs_source(p, fm.gather, 0, fm.prefetch, fm.loop, fm.fence, fm.vrow);
            std::fwrite(src.data(), 1, src.size(), out);
            std::fclose(out);
        }
    }
    std::printf("ok %ld %ld\n", programs, ops);
    return 0;
}
