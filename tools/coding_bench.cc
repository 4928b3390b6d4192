// coding_bench.cc — MemEC's server-side calling pattern through the drop-in
// Coding adapter: W worker threads share ONE Coding instance (server.cc:107,
// worker.cc:128-137) and each issues single-stripe calls on its own chunks,
// as test/common/coding/batch_performance.cc drives the reference plugin.
//
//   coding_bench <rs|cauchy> <k> <m> <chunk> <workers> <seconds> <mode>
//     mode = seal   : full parity of a stripe, encode(index) for every parity
//                     (parity_chunk_buffer.cc:349 on SEAL)
//            delta  : one data column against Coding::zeros, one parity index
//                     (the UPDATE path, parity_chunk_buffer.cc:342-353)
//            decode : rebuild 1..m lost chunks (worker.cc:49)
//
// Prints one JSON line: calls/s, data GiB/s (data bytes the calls cover),
// and the adapter's coalescing setting (env MEMEC_GPU_COALESCE).
//
// Built twice from this one file: against the drop-in adapter + libmec
// (tools/coding_bench.sh), and with -DCODING_BENCH_REF against MemEC's own
// plugin (common/coding + Jerasure + gf_complete compiled from the
// reference sources, oracle/Makefile `ref` -> oracle/_ref/coding_bench_ref),
// so both sides of a comparison run the same threads, calls and chunks.
#include <pthread.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include <atomic>
#include <vector>

#ifdef CODING_BENCH_REF
#include "common/coding/coding.hh"
#include "common/ds/bitmask_array.hh"
#include "common/ds/chunk_pool.hh"
#include "common/ds/chunk_util.hh"
#else
#include "coding.hh"
#include "mec.h"
#endif

static Coding *coding;
static uint32_t K, M, CS;
static double seconds;
static int mode;  // 0 seal, 1 delta, 2 decode
static std::atomic<bool> stop_flag(false);

static double now() {
    timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return ts.tv_sec + ts.tv_nsec * 1e-9;
}

struct Worker {
    pthread_t th;
    uint64_t calls = 0, bytes = 0;
    int id = 0;
};

static bool registered;  // MEMEC_GPU_REGISTER=1: chunks in a registered slab

static void *run(void *arg) {
    Worker *w = (Worker *)arg;
    TempChunkPool pool;
    std::vector<Chunk *> c(K + M);
    char *slab = 0;
    const size_t slot = 8 + size_t(CS);
#ifndef CODING_BENCH_REF
    if (registered) {
        // one ChunkPool-like slab per worker (slot = 8-byte header + data,
        // chunk_pool.cc:22-47), mapped for zero-copy coding
        slab = (char *)aligned_alloc(4096, ((K + M) * slot + 4095) / 4096 * 4096);
        memset(slab, 0, (K + M) * slot);
        if (mec_host_register(slab, (K + M) * slot) != MEC_OK) {
            fprintf(stderr, "mec_host_register: %s\n", mec_last_error());
            exit(1);
        }
        for (uint32_t i = 0; i < K + M; i++) c[i] = (Chunk *)(slab + i * slot);
    } else
#endif
    {
        for (auto &x : c) x = pool.alloc();
    }
    for (auto &x : c) {
        char *d = ChunkUtil::getData(x);
        for (uint32_t b = 0; b < CS; b++) d[b] = char((b * 131 + w->id * 7) >> 3);
    }
    std::vector<Chunk *> dz(K, Coding::zeros);
    BitmaskArray status(1, K + M);
    uint64_t it = 0;
    while (!stop_flag.load(std::memory_order_relaxed)) {
        if (mode == 0) {
            for (uint32_t i = 0; i < M; i++) coding->encode(&c[0], c[K + i], i + 1);
            w->calls += M;
            w->bytes += uint64_t(K) * CS;
        } else if (mode == 1) {
            const uint32_t j = uint32_t(it % K);
            dz[j] = c[j];
            coding->encode(&dz[0], c[K + uint32_t(it % M)], uint32_t(it % M) + 1);
            dz[j] = Coding::zeros;
            w->calls += 1;
            w->bytes += CS;
        } else {
            for (uint32_t i = 0; i < K + M; i++) status.set(0, i);
            const uint32_t lost = 1 + uint32_t(it % M);
            for (uint32_t q = 0; q < lost; q++) status.unset(0, uint32_t((it * 3 + q * 5) % (K + M)));
            if (!coding->decode(&c[0], &status)) {
                fprintf(stderr, "decode failed\n");
                exit(1);
            }
            w->calls += 1;
            w->bytes += uint64_t(K) * CS;
        }
        it++;
    }
#ifndef CODING_BENCH_REF
    if (registered) {
        mec_host_unregister(slab);
        free(slab);
    } else
#endif
    {
        for (auto &x : c) pool.free(x);
    }
    return 0;
}

int main(int argc, char **argv) {
    if (argc < 8) {
        fprintf(stderr, "usage: %s <rs|cauchy> k m chunk workers seconds <seal|delta|decode>\n", argv[0]);
        return 2;
    }
    const CodingScheme scheme = strcmp(argv[1], "rs") == 0 ? CS_RS : CS_CAUCHY;
    K = atoi(argv[2]);
    M = atoi(argv[3]);
    CS = atoi(argv[4]);
    const int W = atoi(argv[5]);
    seconds = atof(argv[6]);
    mode = strcmp(argv[7], "seal") == 0 ? 0 : strcmp(argv[7], "delta") == 0 ? 1 : 2;
    CodingParams params;
    params.setScheme(scheme);
    params.setK(K);
    params.setM(M);
    params.setN(K + M);
    ChunkUtil::init(CS, K);
    registered = getenv("MEMEC_GPU_REGISTER") && atoi(getenv("MEMEC_GPU_REGISTER"));
    coding = Coding::instantiate(scheme, params, CS);
    std::vector<Worker> ws(W);
    const double t0 = now();
    for (int i = 0; i < W; i++) {
        ws[i].id = i;
        pthread_create(&ws[i].th, 0, run, &ws[i]);
    }
    while (now() - t0 < seconds) {
        timespec ts = {0, 20 * 1000 * 1000};
        nanosleep(&ts, 0);
    }
    stop_flag = true;
    uint64_t calls = 0, bytes = 0;
    for (int i = 0; i < W; i++) {
        pthread_join(ws[i].th, 0);
        calls += ws[i].calls;
        bytes += ws[i].bytes;
    }
    const double dt = now() - t0;
    const char *co = getenv("MEMEC_GPU_COALESCE");
    const char *push = getenv("MEC_QUEUE_PUSH");
#ifdef CODING_BENCH_REF
    const char *which = "reference";  // MemEC's own plugin, CPU
#else
    const char *which = "coding_adapter";
#endif
    printf("{\"bench\": \"%s\", \"scheme\": \"%s\", \"k\": %u, \"m\": %u, \"chunk\": %u, \"workers\": %d, "
           "\"mode\": \"%s\", \"coalesce\": %s, \"queue_push\": %s, \"registered\": %d, \"calls_per_s\": %.1f, "
           "\"data_GiBps\": %.4f}\n",
           which, argv[1], K, M, CS, W, argv[7], co ? co : "0", push && *push ? push : "0", registered ? 1 : 0, calls / dt,
           bytes / dt / 1073741824.0);
    Coding::destroy(coding);
    return 0;
}
