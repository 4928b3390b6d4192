// coding_test.cc — exercises the drop-in Coding adapter the way MemEC's own
// coding test does (test/common/coding/coding.cc:76-286): instantiate a
// scheme through Coding::instantiate, encode every parity with the 1-based
// index, apply a data delta through a Coding::zeros delta-encode +
// bitwiseXOR, then rebuild 1, 2 and 3 lost chunks with decode() and
// compare.  Extended beyond the reference: parity-only and mixed
// erasures, too-many-failures, forceSeal, and several worker threads
// sharing one instance (server.cc:107, worker.cc:128-137).
//
//   coding_test <rs|cauchy> [k m chunk]
#include <pthread.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <vector>

#include "coding.hh"
#include "mec.h"

static int fails = 0;
#define EXPECT(cond, ...)                                   \
    do {                                                    \
        if (!(cond)) {                                      \
            fprintf(stderr, "FAIL %s:%d: ", __FILE__, __LINE__); \
            fprintf(stderr, __VA_ARGS__);                   \
            fprintf(stderr, "\n");                          \
            fails++;                                        \
        }                                                   \
    } while (0)

struct Stripe {
    uint32_t k, m, cs;
    TempChunkPool pool;
    std::vector<Chunk *> c;
    bool reg;  // CODING_TEST_REGISTER=1: chunks registered (zero-copy / host queue)
    Stripe(uint32_t k_, uint32_t m_, uint32_t cs_) : k(k_), m(m_), cs(cs_), c(k_ + m_) {
        reg = getenv("CODING_TEST_REGISTER") && atoi(getenv("CODING_TEST_REGISTER"));
        for (auto &x : c) {
            if (!reg) {
                x = pool.alloc();
                continue;
            }
            // whole pages per chunk, so no two registrations share a page
            const size_t bytes = (ChunkUtil::chunkSize + 8 + 4095) / 4096 * 4096;
            x = (Chunk *)aligned_alloc(4096, bytes);
            ChunkUtil::clear(x);
            if (mec_host_register(x, bytes) != MEC_OK) {
                fprintf(stderr, "mec_host_register: %s\n", mec_last_error());
                exit(1);
            }
        }
    }
    ~Stripe() {
        for (auto &x : c) {
            if (reg) mec_host_unregister(x);
            pool.free(x);  // free() either way
        }
    }
    char *data(uint32_t i) { return ChunkUtil::getData(c[i]); }
};

static void fill_pattern(Stripe &s, uint64_t seed) {
    uint64_t x = seed * 0x9E3779B97F4A7C15ull + 1;
    for (uint32_t i = 0; i < s.k; i++)
        for (uint32_t b = 0; b < s.cs; b++) {
            x ^= x << 13;
            x ^= x >> 7;
            x ^= x << 17;
            s.data(i)[b] = char(b < s.cs / 2 ? (3 * i + 5) : (x >> 24));
        }
}

static void encode_all(Coding *coding, Stripe &s) {
    for (uint32_t i = 0; i < s.m; i++) coding->encode(&s.c[0], s.c[s.k + i], i + 1);
}

// Lose `lost` (indices), decode into a copy, compare with the original.
static void check_decode(Coding *coding, Stripe &orig, const std::vector<uint32_t> &lost, bool expect_ok) {
    Stripe t(orig.k, orig.m, orig.cs);
    BitmaskArray bitmap(1, orig.k + orig.m);
    for (uint32_t i = 0; i < orig.k + orig.m; i++) {
        bool gone = false;
        for (uint32_t l : lost) gone |= (l == i);
        if (gone) continue;
        memcpy(t.data(i), orig.data(i), orig.cs);
        bitmap.set(i, 0);
    }
    bool ok = coding->decode(&t.c[0], &bitmap);
    EXPECT(ok == expect_ok, "decode returned %d (lost %zu chunks)", ok, lost.size());
    if (!ok) return;
    for (uint32_t i = 0; i < orig.k + orig.m; i++)
        EXPECT(memcmp(t.data(i), orig.data(i), orig.cs) == 0, "chunk %u differs after decode (lost %zu)", i,
               lost.size());
}

struct ThreadArg {
    Coding *coding;
    Stripe *ref;
    int rounds;
    int bad;
};

static void *worker(void *p) {
    ThreadArg *a = (ThreadArg *)p;
    for (int r = 0; r < a->rounds; r++) {
        Stripe s(a->ref->k, a->ref->m, a->ref->cs);
        for (uint32_t i = 0; i < s.k; i++) memcpy(s.data(i), a->ref->data(i), s.cs);
        encode_all(a->coding, s);
        for (uint32_t i = 0; i < s.m; i++)
            if (memcmp(s.data(s.k + i), a->ref->data(s.k + i), s.cs)) a->bad++;
    }
    return 0;
}

// splitmix64 stream (oracle.c orc_fill_splitmix == mec_fill_random)
static void fill_splitmix(char *buf, size_t n, uint64_t seed) {
    for (size_t i = 0; i < n; i += 8) {
        uint64_t z = seed + (i / 8 + 1) * 0x9E3779B97F4A7C15ull;
        z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
        z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
        z ^= z >> 31;
        for (size_t b = 0; b < 8 && i + b < n; b++) buf[i + b] = char(z >> (8 * b));
    }
}

// coding_test encode-offsets <rs|cauchy> k m chunk index startOff endOff
//                            data_seed parity_seed out.bin
// One Coding::encode(data, parity, index, startOff, endOff) on a parity
// chunk that already holds bytes (the server's delta call shape,
// parity_chunk_buffer.cc:349-353); writes the parity chunk to out.bin.
static int encode_offsets(int argc, char **argv) {
    if (argc < 12) return 2;
    CodingScheme scheme = strcmp(argv[2], "cauchy") == 0 ? CS_CAUCHY : CS_RS;
    const uint32_t k = atoi(argv[3]), m = atoi(argv[4]), cs = atoi(argv[5]), index = atoi(argv[6]);
    const uint32_t st = strtoul(argv[7], 0, 10), ed = strtoul(argv[8], 0, 10);
    CodingParams params;
    params.setScheme(scheme);
    params.setK(k);
    params.setM(m);
    ChunkUtil::init(cs, k);
    Coding *coding = Coding::instantiate(scheme, params, cs);
    if (!coding) return 1;
    {
        Stripe s(k, m, cs);
        std::vector<char> data(size_t(k) * cs);
        fill_splitmix(data.data(), data.size(), strtoull(argv[9], 0, 10));
        for (uint32_t j = 0; j < k; j++) memcpy(s.data(j), &data[size_t(j) * cs], cs);
        fill_splitmix(s.data(k), cs, strtoull(argv[10], 0, 10));
        coding->encode(&s.c[0], s.c[k], index, st, ed);
        FILE *f = fopen(argv[11], "wb");
        if (!f || fwrite(s.data(k), 1, cs, f) != cs) return 1;
        fclose(f);
    }
    Coding::destroy(coding);
    return 0;
}

// coding_test sweep <rs|cauchy> cases.txt stripes.bin out.bin
// One case per line "k m chunk present_mask column": the next (k + m) *
// chunk bytes of stripes.bin are one stripe (any bytes, codeword or not).
// Per case out.bin gets: the m parities Coding::encode computes from the
// first k chunks (index 1..m); the m parities of the server's delta form
// (chunk `column` as the only data chunk, Coding::zeros elsewhere,
// parity_chunk_buffer.cc:342-353); then the k + m chunks after
// Coding::decode on the stripe with every chunk outside present_mask lost
// (cleared first, server_peer_res_worker.cc:818-828); then one byte,
// decode()'s return value.  tests/test_coding_adapter.py compares every
// byte with MemEC's own plugin.
static int sweep(int argc, char **argv) {
    if (argc < 6) return 2;
    CodingScheme scheme = strcmp(argv[2], "cauchy") == 0 ? CS_CAUCHY : CS_RS;
    FILE *cf = fopen(argv[3], "r"), *sf = fopen(argv[4], "rb"), *of = fopen(argv[5], "wb");
    if (!cf || !sf || !of) return 1;
    unsigned k, m, cs, col;
    unsigned long long present;
    while (fscanf(cf, "%u %u %u %llu %u", &k, &m, &cs, &present, &col) == 5) {
        CodingParams params;
        params.setScheme(scheme);
        params.setK(k);
        params.setM(m);
        ChunkUtil::init(cs, k);
        Coding *coding = Coding::instantiate(scheme, params, cs);
        if (!coding) return 1;
        {
            Stripe in(k, m, cs), enc(k, m, cs), dlt(k, m, cs), dec(k, m, cs);
            for (uint32_t i = 0; i < k + m; i++)
                if (fread(in.data(i), 1, cs, sf) != cs) return 1;
            for (uint32_t j = 0; j < k; j++) memcpy(enc.data(j), in.data(j), cs);
            encode_all(coding, enc);
            std::vector<Chunk *> d(k, Coding::zeros);
            memcpy(dlt.data(col), in.data(col), cs);
            d[col] = dlt.c[col];
            for (uint32_t i = 0; i < m; i++) coding->encode(&d[0], dlt.c[k + i], i + 1);
            BitmaskArray bitmap(1, k + m);
            for (uint32_t i = 0; i < k + m; i++) {
                if (!(present >> i & 1)) continue;  // lost: stays cleared
                memcpy(dec.data(i), in.data(i), cs);
                bitmap.set(i, 0);
            }
            const char ok = coding->decode(&dec.c[0], &bitmap) ? 1 : 0;
            for (uint32_t i = 0; i < m; i++) fwrite(enc.data(k + i), 1, cs, of);
            for (uint32_t i = 0; i < m; i++) fwrite(dlt.data(k + i), 1, cs, of);
            for (uint32_t i = 0; i < k + m; i++) fwrite(dec.data(i), 1, cs, of);
            fwrite(&ok, 1, 1, of);
        }
        Coding::destroy(coding);
    }
    fclose(cf);
    fclose(sf);
    return fclose(of) == 0 ? 0 : 1;
}

int main(int argc, char **argv) {
    if (argc > 1 && strcmp(argv[1], "encode-offsets") == 0) return encode_offsets(argc, argv);
    if (argc > 1 && strcmp(argv[1], "sweep") == 0) return sweep(argc, argv);
    if (argc < 2) {
        fprintf(stderr, "usage: %s <rs|cauchy> [k m chunk]\n", argv[0]);
        return 2;
    }
    CodingScheme scheme = strcmp(argv[1], "cauchy") == 0 ? CS_CAUCHY : CS_RS;
    uint32_t k = argc > 2 ? atoi(argv[2]) : 8, m = argc > 3 ? atoi(argv[3]) : 3;
    uint32_t cs = argc > 4 ? atoi(argv[4]) : 4096;
    CodingParams params;
    params.setScheme(scheme);
    params.setK(k);
    params.setM(m);
    ChunkUtil::init(cs, k);
    Coding *coding = Coding::instantiate(scheme, params, cs);
    EXPECT(coding != 0, "instantiate");
    if (!coding) return 1;

    Stripe s(k, m, cs);
    fill_pattern(s, 1);
    encode_all(coding, s);

    // out-of-range index writes nothing (idx - k == index - 1 never matches)
    {
        Stripe t(k, m, cs);
        memset(t.data(k), 0x5a, cs);
        coding->encode(&s.c[0], t.c[k], 0);
        coding->encode(&s.c[0], t.c[k], m + 1);
        bool untouched = true;
        for (uint32_t b = 0; b < cs; b++) untouched &= t.data(k)[b] == 0x5a;
        EXPECT(untouched, "index 0 / m+1 must not write the parity chunk");
    }

    // delta: change bytes [3012, cs) of data chunk 1 (coding.cc:155-181 uses
    // chunks 1..m); parity += encode(delta as the only non-zero column)
    {
        const uint32_t st = cs > 3012 ? 3012 : cs / 2, ed = cs;
        Stripe d(k, m, cs);
        std::vector<Chunk *> cols(k, Coding::zeros);
        char *old = s.data(1) + st;
        std::vector<char> before(old, old + (ed - st));
        memset(old, 0x42, ed - st);
        memset(d.data(1), 0, cs);
        Coding::bitwiseXOR(d.data(1) + st, old, before.data(), ed - st);
        cols[1] = d.c[1];
        for (uint32_t i = 0; i < m; i++) {
            ChunkUtil::clear(d.c[k + i]);
            coding->encode(&cols[0], d.c[k + i], i + 1, 1 * cs + st, 1 * cs + ed);
            Coding::bitwiseXOR(s.c[k + i], d.c[k + i], s.c[k + i], cs);
        }
        Stripe fresh(k, m, cs);
        for (uint32_t i = 0; i < k; i++) memcpy(fresh.data(i), s.data(i), cs);
        encode_all(coding, fresh);
        for (uint32_t i = 0; i < m; i++)
            EXPECT(memcmp(fresh.data(k + i), s.data(k + i), cs) == 0, "delta-updated parity %u != re-encode", i);
    }

    // 1, 2, 3 (up to m) data failures as in the reference test, then parity
    // and mixed patterns it never covers
    check_decode(coding, s, {1}, true);
    if (m >= 2) check_decode(coding, s, {1, 2}, true);
    if (m >= 3) check_decode(coding, s, {1, 2, 3}, true);
    check_decode(coding, s, {k}, true);
    if (m >= 2) check_decode(coding, s, {0, k + m - 1}, true);
    std::vector<uint32_t> all_parity;
    for (uint32_t i = 0; i < m; i++) all_parity.push_back(k + i);
    check_decode(coding, s, all_parity, true);
    std::vector<uint32_t> too_many;
    for (uint32_t i = 0; i <= m; i++) too_many.push_back(i);
    check_decode(coding, s, too_many, false);
    check_decode(coding, s, {}, true);

    // forceSeal (coding.cc:120-185): data chunk 2 is sealed but parity 1 has
    // not seen it.  forceSeal passes its 0-based parity loop index as the
    // 1-based `index` (Appendix B #11), so parity 1 receives coding row 0's
    // contribution of chunk 2 — the reference's caller behaviour, kept.
    if (m >= 2) {
        Stripe t(k, m, cs);
        for (uint32_t i = 0; i < k + m; i++) memcpy(t.data(i), s.data(i), cs);
        std::vector<Chunk *> cols(k, Coding::zeros);
        cols[2] = t.c[2];
        Stripe d(k, m, cs);
        coding->encode(&cols[0], d.c[k + 1], 2);  // chunk 2's term in parity 1
        Coding::bitwiseXOR(t.c[k + 1], d.c[k + 1], t.c[k + 1], cs);
        Stripe e(k, m, cs);
#ifdef USE_ISAL
        // ISA-L RS: forceSeal's encode(..., 0, chunkSize) selects columns
        // [0, (chunkSize-1)/chunkSize] = {0} only (rscoding.cc:85-88); column
        // 0 is Coding::zeros here, so the parity is left as it was.  ISA-L
        // Cauchy ignores the offsets (cauchycoding.cc:78-79).
        if (scheme == CS_CAUCHY) coding->encode(&cols[0], e.c[k], 1);
#else
        coding->encode(&cols[0], e.c[k], 1);  // chunk 2's term in parity 0
#endif
        std::vector<char> expected(cs);
        Coding::bitwiseXOR(expected.data(), t.data(k + 1), e.data(k), cs);
        std::vector<char> storage((m + 1) * k, 1);
        std::vector<bool *> ind(m + 1);
        for (uint32_t i = 0; i <= m; i++) ind[i] = (bool *)&storage[i * k];
        ind[1][2] = false;
        Chunk *tmp = TempChunkPool().alloc();
        uint32_t fixed = Coding::forceSeal(coding, &t.c[0], tmp, &ind[0], k, m);
        EXPECT(fixed == 1, "forceSeal fixed %u", fixed);
        EXPECT(memcmp(t.data(k + 1), expected.data(), cs) == 0, "forceSeal result differs from the reference rule");
        EXPECT(ind[1][2], "seal indicator not set");
        free(tmp);
    }

    // several workers sharing one instance
    {
        const int T = 4;
        pthread_t th[T];
        ThreadArg args[T];
        for (int t = 0; t < T; t++) {
            args[t] = ThreadArg{coding, &s, 8, 0};
            pthread_create(&th[t], 0, worker, &args[t]);
        }
        for (int t = 0; t < T; t++) {
            pthread_join(th[t], 0);
            EXPECT(args[t].bad == 0, "thread %d: %d mismatches", t, args[t].bad);
        }
    }

    Coding::destroy(coding);
    printf("%s k=%u m=%u chunk=%u: %s\n", argv[1], k, m, cs, fails ? "FAILED" : "ok");
    return fails ? 1 : 0;
}
