// gpu_coding.cc — RSCoding / CauchyCoding bodies over libmec.
#include "gpu_coding.hh"
#include "boundary_ds.hh"

#include <stdio.h>
#include <stdlib.h>

static int adapter_device() {
    const char *e = getenv("MEMEC_GPU_DEVICE");
    return e ? atoi(e) : 0;
}

// MEMEC_GPU_DEVICES=0,1,2,3: one server process drives several GPUs
// (mec_create_multi: host-memory calls spread over them); empty = one
// device (MEMEC_GPU_DEVICE).
static int adapter_devices(int *out, int cap) {
    const char *e = getenv("MEMEC_GPU_DEVICES");
    int n = 0;
    while (e && *e && n < cap) {
        char *end = 0;
        const long v = strtol(e, &end, 10);
        if (end == e) break;
        out[n++] = int(v);
        e = *end == ',' ? end + 1 : end;
    }
    return n;
}

// One instance is shared by every server worker thread (server.cc:107,
// worker.cc:128-137), each issuing single-stripe calls.  Each call is one
// launch on the calling thread's own stream, coding the chunks in place
// (registered memory) or in mapped pinned staging, so concurrent calls
// already overlap; batching them through the coalescer measured 2-4x
// slower at 16 workers (profiles/r01/host/coding_bench_staged.jsonl), so
// it is off unless MEMEC_GPU_COALESCE = max requests per batch is set.
static unsigned adapter_coalesce() {
    const char *e = getenv("MEMEC_GPU_COALESCE");
    return e ? unsigned(atoi(e)) : 0u;
}

// Resident submission-queue kernel for single-stripe calls on registered
// chunks (mec_set_host_queue), on by default with 32 slots: with 16 workers
// it serves 2.9x (RS(8,2)@4 KiB seal) to 3.4x (RS(10,4)@4 KiB delta) the
// calls/s of per-call launches (profiles/r01/host/queue_ab.log).
// MEMEC_GPU_QUEUE = slots, 0 = off.
static unsigned adapter_queue() {
    const char *e = getenv("MEMEC_GPU_QUEUE");
    return e ? unsigned(atoi(e)) : 32u;
}

GpuMatrixCoding::GpuMatrixCoding(int family, const char *name, uint32_t k, uint32_t m, uint32_t chunkSize)
    : _name(name), _family(family), _k(k), _m(m), _chunkSize(chunkSize), _ctx(0) {
    // Parameter errors exit(-1) with a message, like rscoding.cc:26-29 and
    // rscoding.cc:205-213 / cauchycoding.cc:193-196.
    int devs[64];
    const int nd = adapter_devices(devs, 64);
    int rc = nd > 0 ? mec_create_multi(family, k, m, chunkSize, devs, uint32_t(nd), &_ctx)
                    : mec_create(family, k, m, chunkSize, adapter_device(), &_ctx);
    if (rc != MEC_OK) {
        fprintf(stderr, "%s: %s\n", _name, mec_last_error());
        exit(-1);
    }
    if (adapter_coalesce() && mec_set_coalescing(_ctx, adapter_coalesce()) != MEC_OK)
        fprintf(stderr, "%s: coalescing unavailable: %s\n", _name, mec_last_error());
    if (adapter_queue() && mec_set_host_queue(_ctx, adapter_queue()) != MEC_OK)
        fprintf(stderr, "%s: host queue unavailable: %s\n", _name, mec_last_error());
}

GpuMatrixCoding::~GpuMatrixCoding() { mec_destroy(_ctx); }

// rscoding.cc:51-95 / cauchycoding.cc:49-85: only parity `index` (1-based)
// is written; an out-of-range index writes nothing (as idx-k == index-1
// never matches there).  Coding::zeros columns are skipped outright — they
// contribute nothing — which turns the server's single-column delta encodes
// into one scale of one chunk.
void GpuMatrixCoding::encode(Chunk **dataChunks, Chunk *parityChunk, uint32_t index, uint32_t startOff,
                             uint32_t endOff) {
    if (index < 1 || index > _m) return;
    uint8_t *parity[32] = {0};
    parity[index - 1] = (uint8_t *)ChunkUtil::getData(parityChunk);
    int rc;
    if (_family == MEC_ISAL_RS && (startOff != 0 || endOff != 0)) {
        // USE_ISAL RSCoding: ec_encode_data_update over the touched columns,
        // XORed in place (rscoding.cc:82-89).  USE_ISAL CauchyCoding ignores
        // the offsets and overwrites with a full encode (cauchycoding.cc:78-79),
        // as the Jerasure builds do (Appendix B #3).
        rc = MEC_OK;
        for (uint32_t i = startOff / _chunkSize; rc == MEC_OK && i <= (endOff - 1) / _chunkSize && i < _k; i++) {
            if (dataChunks[i] == Coding::zeros) continue;
            rc = mec_encode_update_host(_ctx, i, (const uint8_t *)ChunkUtil::getData(dataChunks[i]), parity);
        }
        if (rc != MEC_OK) encode_failed(rc);
        return;
    }
    const uint8_t *data[32];
    for (uint32_t j = 0; j < _k; j++)
        data[j] = dataChunks[j] == Coding::zeros ? 0 : (const uint8_t *)ChunkUtil::getData(dataChunks[j]);
    rc = mec_encode_host(_ctx, data, parity);
    if (rc != MEC_OK) encode_failed(rc);
}

// The reference's encode cannot fail (it returns void, rscoding.cc:51), so
// its callers go on to XOR the parity into their buffers
// (parity_chunk_buffer.cc:349-393).  libmec already retries on the launch
// path when its queue fails; a call that still fails would leave stale
// parity behind silently, so the process stops instead.
void GpuMatrixCoding::encode_failed(int rc) const {
    fprintf(stderr, "%s::encode: %s (rc %d); aborting rather than leaving parity unwritten\n", _name,
            mec_last_error(), rc);
    abort();
}

// rscoding.cc:97-187 / cauchycoding.cc:87-180.
bool GpuMatrixCoding::decode(Chunk **chunks, BitmaskArray *chunkStatus) {
    uint32_t failed = 0;
    uint64_t present = 0;
    for (uint32_t i = 0; i < _k + _m; i++) {
        if (chunkStatus->check(i))
            present |= uint64_t(1) << i;
        else
            failed++;
    }
    if (failed > _m) {
        fprintf(stderr, "%s: Too many failure to recover (%d>%d)!!\n", _name, failed, _m);
        return false;
    }
    if (failed == 0) return true;
    uint8_t *ptrs[32];
    for (uint32_t i = 0; i < _k + _m; i++) ptrs[i] = (uint8_t *)ChunkUtil::getData(chunks[i]);
    int rc = mec_decode_host(_ctx, ptrs, present);
    if (rc != MEC_OK) {
        // The reference ignores jerasure's return code; a device failure is
        // reported instead of silently returning unrepaired chunks.
        fprintf(stderr, "%s::decode: %s\n", _name, mec_last_error());
        return false;
    }
    return true;
}
