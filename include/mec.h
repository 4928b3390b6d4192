/*
 * mec.h — libmec: MI355X-native erasure-coding engine for MemEC's stripe
 * encode/decode path.  Plain C ABI: opaque context, plain pointers and sizes,
 * int status codes (never exit()).
 *
 * Which reference interface each entry point replaces (paths relative to the
 * mtyiu/memec root):
 *
 *   mec_create / mec_destroy     Coding::instantiate / Coding::destroy
 *                                (common/coding/coding.cc:12-54, :56-86) and
 *                                the RSCoding / CauchyCoding constructors
 *                                (rscoding.cc:20-43, cauchycoding.cc:20-39)
 *   mec_encode                   Coding::encode (coding.hh:31) ->
 *                                RSCoding::encode (rscoding.cc:51-95),
 *                                CauchyCoding::encode (cauchycoding.cc:49-85),
 *                                batched over stripes, device-resident
 *   mec_decode                   Coding::decode (coding.hh:40) ->
 *                                RSCoding::decode (rscoding.cc:97-187),
 *                                CauchyCoding::decode (cauchycoding.cc:87-180)
 *   mec_encode_update            the USE_ISAL delta path
 *                                ec_encode_data_update (rscoding.cc:81-89) and
 *                                the server's single-column delta encode
 *                                (parity_chunk_buffer.cc:340-415)
 *   mec_xor                      Coding::bitwiseXOR (coding.cc:88-118)
 *   mec_encode_host /            the same calls on host-resident chunks, one
 *   mec_decode_host /            stripe per call, as server/ issues them; the
 *   mec_encode_update_host       C++ Coding adapter (memec_amd/csrc/coding/)
 *                                forwards its virtual methods here
 *   mec_encode_host_batch        host-memory (PCIe-inclusive) batched encode
 *   mec_encode_batch /           the libmec batch ABI of SURVEY §8(b): many
 *   mec_decode_batch /           stripes given as per-stripe chunk pointer
 *   mec_encode_update_batch      rows (Chunk** as server/ holds them), device
 *                                or host memory; replaces a loop of
 *                                Coding::encode / Coding::decode calls
 *                                (parity_chunk_buffer.cc:349, worker.cc:49,
 *                                server_peer_res_worker.cc:836-838) and the
 *                                server's delta encodes
 *                                (parity_chunk_buffer.cc:342-353,
 *                                degraded_chunk_buffer.cc:645-656)
 *   mec_create_multi             one server process driving several GPUs: its
 *                                host-memory calls spread over them (SURVEY
 *                                §8e; the reference has no GPU, one Coding
 *                                per server process, server.cc:107)
 *   mec_set_coalescing           batching of concurrent mec_*_host calls from
 *                                the server's worker threads, which share one
 *                                Coding instance (server.cc:107,
 *                                worker.cc:128-137)
 *
 * Memory: the device entry points take device pointers (hipMalloc / torch
 * CUDA tensors) and a hipStream_t passed as void* (NULL = default stream);
 * they are asynchronous on that stream.  The *_host entry points take host
 * pointers and return when the result is in host memory.  A call with zero
 * stripes (or zero bytes) touches no memory and succeeds; its buffer
 * pointers may then be NULL (an empty torch tensor's data_ptr is 0).
 *
 * Layout of the batched device entry points ("strided"): chunk c of stripe s
 * starts at  base + s * stripe_stride + c * chunk_stride  (bytes).  Dense
 * [stripe][chunk][bytes] is chunk_stride = chunk_size,
 * stripe_stride = chunks_per_stripe * chunk_size.
 *
 * Code families (mec_family):
 *   MEC_RS_VANDERMONDE  Jerasure reed_sol_vandermonde_coding_matrix, GF(2^8)
 *                       poly 0x11d, byte-wise (MemEC CS_RS, default build)
 *   MEC_CAUCHY_GOOD     Jerasure cauchy_good_general_coding_matrix as a
 *                       bitmatrix over w packets of chunk_size/w bytes
 *                       (MemEC CS_CAUCHY, default build)
 *   MEC_ISAL_RS         ISA-L gf_gen_rs_matrix, byte-wise GF(2^8)
 *                       (MemEC CS_RS with USE_ISAL=1)
 *   MEC_ISAL_CAUCHY     ISA-L gf_gen_cauchy1_matrix, byte-wise GF(2^8)
 *                       (MemEC CS_CAUCHY with USE_ISAL=1)
 */
#ifndef MEC_H
#define MEC_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define MEC_ABI_VERSION 6
#define MEC_MAX_CHUNKS 32 /* k + m <= 32: RS_N_MAX / CRS_N_MAX (rscoding.hh:5, cauchycoding.hh:5) */

typedef enum {
    MEC_OK = 0,
    MEC_EINVAL = -1,     /* bad argument (the reference exit(-1)s here) */
    MEC_ENOMEM = -2,     /* host or device allocation failed */
    MEC_EHIP = -3,       /* HIP runtime error (message in mec_last_error) */
    MEC_ETOOMANY = -4,   /* more than m chunks missing: decode returns false */
    MEC_ESINGULAR = -5,  /* decoding matrix not invertible */
    MEC_ENODEV = -6      /* no usable gfx950 device / kernels missing */
} mec_status;

typedef enum {
    MEC_RS_VANDERMONDE = 0,
    MEC_CAUCHY_GOOD = 1,
    MEC_ISAL_RS = 2,
    MEC_ISAL_CAUCHY = 3
} mec_family;

typedef enum {
    MEC_MEM_DEVICE = 0, /* device pointers; asynchronous on the given stream */
    MEC_MEM_HOST = 1    /* host pointers (pageable or registered); synchronous */
} mec_mem_kind;

typedef struct mec_ctx mec_ctx;

typedef struct {
    uint64_t coalesced_batches;  /* batches run by the coalescer */
    uint64_t coalesced_requests; /* single-stripe requests they carried */
    uint64_t cached_plans;       /* decode plans cached (one per erasure pattern) */
    uint64_t zero_copy_calls;    /* host calls coded in place over PCIe (registered memory) */
    uint64_t staged_calls;       /* host calls copied through pinned, GPU-mapped staging */
    uint64_t queue_calls;        /* zero-copy calls served by the resident queue kernel */
    uint64_t queue_launches;     /* launches of the resident queue kernel (idle exits relaunch) */
    uint32_t queue_slots;        /* slots actually running (mec_set_host_queue may grant fewer) */
    uint32_t queue_parts;        /* workgroups per slot (one per 16 KiB of chunk, at most 64) */
    uint32_t queue_broken;       /* 1: a call timed out and the queue stopped for good */
    uint32_t queue_devslot;      /* 1: slot descriptors in device memory, written through the BAR */
    uint64_t queue_timeouts;     /* calls that hit MEC_QUEUE_TIMEOUT_MS */
    /* one-pass (> 4 output) permute tables: device bytes held, matrices
     * cached, and launches that ran as 4-row groups because the cache was at
     * its cap (MEC_MG_CACHE_BYTES at mec_create, default 64 MiB; ABI 5) */
    uint64_t mg_cache_bytes;
    uint64_t mg_cache_tables;
    uint64_t mg_cache_uncached;
    /* wide codes' run-time compiled bit-sliced kernels (MEC_BITSLICE): built,
     * failed (those matrices stay on the one-pass kernel), still compiling,
     * total compile milliseconds, and launches that ran one (ABI 5) */
    uint64_t jit_kernels;
    uint64_t jit_failed;
    uint64_t jit_pending;
    uint64_t jit_compile_ms;
    uint64_t jit_launches;
} mec_stats;

typedef struct {
    int32_t family;
    uint32_t k, m;
    uint32_t w;           /* field width (8 for byte-wise families) */
    uint32_t chunk_size;  /* bytes */
    uint32_t packet_size; /* chunk_size / w for MEC_CAUCHY_GOOD, else chunk_size */
    int32_t device;
} mec_info;

/* ---- lifecycle ---------------------------------------------------------- */

int mec_abi_version(void);
/* Create a coding context on HIP device `device`.  Applies the reference's
 * getW rules: RS w = 8 (rscoding.cc:189-220); Cauchy w = smallest w >=
 * log2(k+m) dividing chunk_size (cauchycoding.cc:182-205), w <= 8 here.
 * MEC_EINVAL where the reference would exit(-1). */
int mec_create(int family, uint32_t k, uint32_t m, uint32_t chunk_size, int device,
               mec_ctx **out);
/* Frees the context.  With a host queue (mec_set_host_queue) the resident
 * kernel is stopped first; if it does not leave within max(timeout, 1 s) —
 * a job that never completes — its memory and the context's staging lanes
 * are leaked rather than freed under it, a message goes to stderr, and
 * mec_destroy returns while that kernel may still read the job's source
 * chunks and write its outputs: the caller must keep registered chunks of
 * a call that failed with MEC_EHIP alive.  Run-time compiles the context
 * queued (wide codes) are cancelled; one already running is waited for, and
 * each compiled kernel's module is unloaded after its last launch on each
 * stream it ran on (no device-wide synchronize). */
void mec_destroy(mec_ctx *ctx);
/* Thread-local description of the last failure on this thread. */
const char *mec_last_error(void);
int mec_get_info(const mec_ctx *ctx, mec_info *out);
/* Coding matrix: m*k int32 (Jerasure families) or (k+m)*k (ISA-L families,
 * identity on top, as gf_gen_*_matrix produces). */
int mec_get_matrix(const mec_ctx *ctx, int32_t *out, size_t capacity);
/* MEC_CAUCHY_GOOD only: (m*w) x (k*w) 0/1 int32 bitmatrix
 * (jerasure_matrix_to_bitmatrix, jerasure.c:271-297). */
int mec_get_bitmatrix(const mec_ctx *ctx, int32_t *out, size_t capacity);

/* ---- device-resident batched entry points -------------------------------- */

/* Encode n_stripes stripes.  Writes parity i (0-based) for every bit i set in
 * parity_mask (0 = all m), overwriting it (jerasure.c:603,625 overwrite too).
 * Data and parity must not overlap. */
int mec_encode(mec_ctx *ctx,
               const uint8_t *data, int64_t data_stripe_stride, int64_t data_chunk_stride,
               uint8_t *parity, int64_t parity_stripe_stride, int64_t parity_chunk_stride,
               uint32_t n_stripes, uint32_t parity_mask, void *stream);

/* Multi-GPU context for one host process (MemEC runs one server process
 * per node, chunks in host memory).  devices[0..n_devices-1] are HIP
 * ordinals (a device may repeat).  Host-memory batches (mec_encode_batch /
 * mec_decode_batch / mec_encode_update_batch with MEC_MEM_HOST,
 * mec_encode_host_batch) are cut into contiguous stripe ranges, one per
 * device ([g*N/G, (g+1)*N/G)), and run concurrently, each GPU over its own
 * PCIe link; single-stripe host calls go to the devices round-robin;
 * device-memory calls run on devices[0].  No data moves between GPUs
 * (stripes are independent).  mec_get_stats sums the devices; destroy with
 * mec_destroy. */
int mec_create_multi(int family, uint32_t k, uint32_t m, uint32_t chunk_size,
                     const int *devices, uint32_t n_devices, mec_ctx **out);

/* Decode n_stripes stripes in place.  chunks holds all k+m chunks of every
 * stripe (strided).  Bit i of present_mask set <=> chunk i is present
 * (BitmaskArray::check(i), bitmask_array.cc:52-56).  Every missing chunk is
 * rebuilt, exactly as the reference plugin computes it (same survivors, same
 * decoding matrix).  MEC_ETOOMANY if more than m are missing; MEC_OK and no
 * work if none is. */
int mec_decode(mec_ctx *ctx, uint8_t *chunks, int64_t stripe_stride, int64_t chunk_stride,
               uint32_t n_stripes, uint64_t present_mask, void *stream);

/* Decode with survivors and outputs in separate buffers: reads the chunks
 * named by present_mask from `in`, writes the missing ones to `out` (its
 * chunk slot c for missing chunk c). */
int mec_decode_split(mec_ctx *ctx,
                     const uint8_t *in, int64_t in_stripe_stride, int64_t in_chunk_stride,
                     uint8_t *out, int64_t out_stripe_stride, int64_t out_chunk_stride,
                     uint32_t n_stripes, uint64_t present_mask, void *stream);

/* Delta / update encode: parity_i ^= A[i][data_index] * delta for every bit
 * i in parity_mask (0 = all).  Byte-wise families: one GF(2^8) scale per
 * parity.  MEC_CAUCHY_GOOD: the column's bitmatrix block.  `delta` is one
 * chunk per stripe. */
int mec_encode_update(mec_ctx *ctx, uint32_t data_index,
                      const uint8_t *delta, int64_t delta_stripe_stride,
                      uint8_t *parity, int64_t parity_stripe_stride, int64_t parity_chunk_stride,
                      uint32_t n_stripes, uint32_t parity_mask, void *stream);

/* dst = a ^ b over len bytes (device pointers; dst may alias a or b). */
int mec_xor(uint8_t *dst, const uint8_t *a, const uint8_t *b, uint64_t len, void *stream);

/* Benchmark / test utility: fill len device bytes with the splitmix64
 * stream (word q = mix(seed + (q + 1) * 0x9E3779B97F4A7C15), little endian,
 * starting at word word_offset).  Same stream as the oracle's fill. */
int mec_fill_random(uint8_t *dst, uint64_t len, uint64_t seed, uint64_t word_offset, void *stream);

/* ---- host-memory entry points (one stripe; synchronous) ------------------- */

/* data[j] == NULL means an all-zero chunk (the Coding::zeros sentinel,
 * coding.cc:14-16): it is neither copied nor multiplied.  parity[i] == NULL
 * means parity i is not wanted.  Each non-NULL parity[i] receives
 * chunk_size bytes, overwritten. */
int mec_encode_host(mec_ctx *ctx, const uint8_t *const *data, uint8_t *const *parity);
/* chunks[0..k+m-1]: present chunks are read, missing ones (bit clear) are
 * written in place. */
int mec_decode_host(mec_ctx *ctx, uint8_t *const *chunks, uint64_t present_mask);
/* parity[i] ^= A[i][data_index] * delta for non-NULL parity[i]. */
int mec_encode_update_host(mec_ctx *ctx, uint32_t data_index, const uint8_t *delta,
                           uint8_t *const *parity);

/* Host-resident batch (dense [stripe][k][cs] data, [stripe][m][cs] parity);
 * returns when the parity is in host memory.  Registered memory (both
 * buffers inside mec_host_register ranges) is coded zero-copy; otherwise
 * pipelined H2D -> kernel -> D2H over internal streams. */
int mec_encode_host_batch(mec_ctx *ctx, const uint8_t *data, uint8_t *parity,
                          uint32_t n_stripes, uint32_t parity_mask);

/* Zero-copy host memory.  Pins [ptr, ptr + len) and maps it into the GPU's
 * address space (hipHostRegister, mapped + portable).  Every host entry
 * point (mec_*_host, mec_encode_host_batch, the pointer-array batches with
 * MEC_MEM_HOST) whose chunks all lie in registered ranges runs its kernel
 * directly on the host chunks over PCIe: no staging copy, one launch per
 * call.  A server registers its ChunkPool slab once (chunk_pool.cc:22-47,
 * the 8-byte chunk headers included); chunks outside registered ranges are
 * copied into pinned, GPU-mapped staging and coded there.  Registered ranges
 * are disjoint: a range overlapping a registered one (the same ptr included)
 * is refused with MEC_EINVAL, so memory freed without mec_host_unregister
 * cannot leave a stale mapping behind a later range.  mec_host_unregister
 * takes the same ptr (MEC_EINVAL if no registered range begins there).
 * Registration is meant for long-lived ranges: each call copies the range
 * list and waits for concurrent lookups to leave the one it replaces, and
 * the HIP runtime appears to register / unregister only while no kernel is
 * resident
 * (measured: up to the 50 ms idle exit of a busy host queue, longer while
 * another context keeps its queue busy) — register slabs at setup. */
int mec_host_register(void *ptr, size_t len);
int mec_host_unregister(void *ptr);

/* ---- pointer-array batches ------------------------------------------------
 *
 * A batch is n_stripes rows of chunk pointers, row-major (stripe s's chunk
 * c at array[s * chunks_per_row + c]), as the server holds Chunk* arrays.
 * mem_kind MEC_MEM_DEVICE: device pointers, work enqueued on `stream`
 * (the pointer arrays themselves are host arrays, consumed before return).
 * MEC_MEM_HOST: host pointers; synchronous, `stream` ignored.  Zero-copy
 * when every chunk lies in a mec_host_register range, otherwise staged
 * through pinned, GPU-mapped host buffers.
 * Stripes are grouped by their linear map (same sources / outputs); each
 * group is one gather launch. */

/* data: n_stripes * k pointers, NULL = the all-zero Coding::zeros chunk
 * (neither read nor multiplied).  parity: n_stripes * m pointers, NULL = not
 * wanted; parity_mask (0 = all m) filters further.  Wanted parities are
 * overwritten. */
int mec_encode_batch(mec_ctx *ctx, const uint8_t *const *data, uint8_t *const *parity, uint32_t n_stripes,
                     uint32_t parity_mask, int mem_kind, void *stream);

/* chunks: n_stripes * (k + m) pointers; present_masks[s] bit i set <=> chunk
 * i of stripe s is present.  Each stripe's missing chunks are rebuilt in
 * place exactly as mec_decode would (the reference's survivors and decoding
 * matrix); stripes may have different erasure patterns.  results (optional,
 * n_stripes entries) receives each stripe's status: MEC_OK or
 * MEC_ETOOMANY (more than m missing; the reference's decode() == false) /
 * MEC_EINVAL.  Decodable stripes are decoded even when others fail; the
 * return value is the first failure, or MEC_OK. */
int mec_decode_batch(mec_ctx *ctx, uint8_t *const *chunks, const uint64_t *present_masks, uint32_t n_stripes,
                     int32_t *results, int mem_kind, void *stream);

/* Delta encode: parity[s * m + i] ^= A[i][data_index[s]] * delta[s] for every
 * non-NULL parity pointer in parity_mask (0 = all).  delta[s] == NULL is an
 * all-zero delta (no work). */
int mec_encode_update_batch(mec_ctx *ctx, const uint32_t *data_index, const uint8_t *const *delta,
                            uint8_t *const *parity, uint32_t n_stripes, uint32_t parity_mask, int mem_kind,
                            void *stream);

/* ---- pointer batches as 32-bit slab offsets (device memory; ABI 6) -------
 *
 * The same batches as mec_encode_batch / mec_decode_batch /
 * mec_encode_update_batch with MEC_MEM_DEVICE, for chunks that live in one
 * device slab (a ChunkPool-like slab, chunk_pool.cc:22-55): chunk = base +
 * ((uint64_t)off << unit_shift), off == MEC_NULL_OFF is NULL (the
 * Coding::zeros source / an unwanted output / a skipped delta), unit_shift
 * <= 12 (3: 8-byte units, a 32 GiB slab; MemEC's chunk data is 8-byte
 * aligned).  The offset rows cross PCIe at half the size of pointer rows and
 * are expanded to pointers on the device before the coding launch; results
 * equal the pointer-row calls' bit for bit.  Work is enqueued on `stream`;
 * the offset arrays are consumed before return. */
#define MEC_NULL_OFF 0xFFFFFFFFu
int mec_encode_batch32(mec_ctx *ctx, uint8_t *base, uint32_t unit_shift, const uint32_t *data_off,
                       const uint32_t *parity_off, uint32_t n_stripes, uint32_t parity_mask, void *stream);
int mec_decode_batch32(mec_ctx *ctx, uint8_t *base, uint32_t unit_shift, const uint32_t *chunk_off,
                       const uint64_t *present_masks, uint32_t n_stripes, int32_t *results, void *stream);
int mec_encode_update_batch32(mec_ctx *ctx, uint8_t *base, uint32_t unit_shift, const uint32_t *data_index,
                              const uint32_t *delta_off, const uint32_t *parity_off, uint32_t n_stripes,
                              uint32_t parity_mask, void *stream);

/* Coalesce concurrent mec_encode_host / mec_decode_host /
 * mec_encode_update_host calls on this context: while one batch runs,
 * arriving calls queue, and the next caller to lead takes up to max_batch
 * of them as one host batch.  An idle context adds no wait.  0 = off
 * (default): every call is its own launch. */
int mec_set_coalescing(mec_ctx *ctx, uint32_t max_batch);

/* Device-side submission queue for single-stripe host calls (queue.hip).
 * slots > 0 starts a resident kernel with `parts` workgroups per slot (one
 * per 16 KiB of chunk, at most 64; MEC_QUEUE_PARTS overrides).  Each
 * slot's sequence word and descriptor live in device memory that the host
 * writes through the PCIe BAR when the device has a large BAR
 * (mec_stats.queue_devslot = 1; MEC_QUEUE_DEVSLOT=0 keeps them in
 * GPU-mapped host memory), its completion words in host memory;
 * mec_encode_host / mec_decode_host /
 * mec_encode_update_host calls of every family (RS and ISA-L byte-wise,
 * Jerasure Cauchy-RS as bitmatrix jobs) with chunks of at most
 * MEC_QUEUE_MAX_CHUNK bytes (default 1 MiB) are then posted to a free slot instead of
 * launching a kernel: no HIP runtime call on the caller's path (calls
 * beyond `slots` concurrent callers take the launch path).  Registered
 * chunks (mec_host_register) are coded in place; other host chunks are
 * copied through a mapped pinned staging buffer.
 * Slots: every workgroup must be resident at once, and the resident grid
 * takes at most half of what the device can hold (launches beside it keep
 * CUs), so `slots` is reduced to that (mec_stats.queue_slots reports the
 * number running, e.g. 2 slots at 1 MiB chunks; the call still returns
 * MEC_OK).
 * Idle: the kernel exits after MEC_QUEUE_IDLE_MS (default 50) without work
 * and is relaunched by the next call.
 * Timeout: a call not completed within MEC_QUEUE_TIMEOUT_MS (default 5000)
 * withdraws its job, stops the queue FOR GOOD (mec_stats.queue_broken = 1,
 * queue_timeouts counts them; every later call takes the launch path until
 * mec_set_host_queue is called again) and waits for the resident kernel to
 * leave, at most max(4 x MEC_QUEUE_TIMEOUT_MS, 10 s).  Then: a job every part of its
 * slot finished returns MEC_OK; a job no part took is coded on the launch
 * path; anything else — some parts finished, the kernel faulted, or it is
 * still running at the cap — returns MEC_EHIP and the outputs are undefined
 * (a still-running kernel may write them later; the slot stays reserved and
 * mec_destroy leaks the queue's memory rather than free it under the
 * kernel).
 * 0 stops the queue.  Not to be called concurrently with other calls on the
 * context.  Replaces nothing in the reference: its workers call the CPU
 * plugin directly (worker.cc:128-137). */
int mec_set_host_queue(mec_ctx *ctx, uint32_t slots);

/* Latency breakdown of single-stripe queue calls (measurement only; no
 * reference counterpart).  While enabled, part 0 of the slot that runs a
 * call records its device clock (s_memrealtime, 100 MHz ticks) when it took
 * the job, when the descriptor and coefficient tables were ready, and when
 * its output stores were acknowledged (and after its acquire fence); the
 * calling thread's last such call,
 * with its host CLOCK_MONOTONIC times of posting the job and seeing it
 * done, is read back with mec_queue_last_trace (once; MEC_EINVAL when none
 * is pending).  Device and host clocks are not related here: a tool
 * calibrates the offset (tools/queue_latency.hip). */
typedef struct {
    uint64_t host_post_ns;  /* before the sequence-number store that posts the job */
    uint64_t host_seen_ns;  /* when every part's done word was seen */
    uint64_t dev_take;      /* device ticks: job taken (seq seen) */
    uint64_t dev_fence;     /* its system-scope acquire fence done */
    uint64_t dev_desc;      /* descriptor (incl. coefficient tables) in LDS */
    uint64_t dev_loaded;    /* thread 0's first source loads returned (byte-wise jobs; 0 otherwise) */
    uint64_t dev_end;       /* output stores acknowledged, before the done store */
    uint32_t parts, pad;
} mec_queue_trace;
int mec_queue_trace_enable(mec_ctx *ctx, int on);
int mec_queue_last_trace(mec_queue_trace *out);
int mec_get_stats(const mec_ctx *ctx, mec_stats *out);

/* ---- measurement and experiments (no reference counterpart) --------------- */

#define MEC_PROBE_OFF 0
#define MEC_PROBE_XOR 1
/* MEC_PROBE_XOR: this context's strided byte-wise launches (mec_encode,
 * mec_decode, mec_decode_split, mec_encode_update, and the single-stripe
 * host calls' launches) run their arithmetic-free
 * twin — the same kernel, launch shape, loads and stores with every GF(2^8)
 * product replaced by a plain XOR — so a bench can measure, live, the rate
 * the same memory stream reaches without the coding arithmetic.  The
 * outputs are NOT codes while it is on.  MEC_PROBE_OFF (default) restores
 * normal coding.  MEC_EINVAL for MEC_CAUCHY_GOOD. */
int mec_set_probe(mec_ctx *ctx, int mode);

/* Launch-shape experiment overrides.  libmec reads MEC_SGROUP, MEC_WINDOWS,
 * MEC_BLOCK, MEC_GBLOCK, MEC_GWPC, MEC_BM_VW, MEC_WPC, MEC_COPY_THREADS,
 * MEC_WIDE, MEC_MG_ROWS, MEC_BITSLICE, MEC_BS_WAVES, MEC_BS_PREFETCH,
 * MEC_BS_TPB, MEC_BS_FENCE, MEC_BS_XCD, MEC_BS_VROW,
 * MEC_TILE_SKEW, MEC_WBATCH, MEC_TAB_WAIT, MEC_GXCD, MEC_GU from the environment once, at first use, never on a launch path; this
 * call changes one at run time (same name and value syntax as the
 * variable; value NULL = unset, i.e. the built-in rule).  Each stored
 * value is one atomic word, so a concurrent launch sees the old or the new
 * value of it; MEC_SGROUP's group and run are two words, and a launch racing
 * a change may see one of each (experiments set knobs between launches).
 * MEC_EINVAL for an unknown name or a value outside the knob's accepted set
 * (memec_amd/csrc/knobs.cpp); the launch planner then also keeps every
 * launch inside its kernel's invariants whatever the accepted values. */
int mec_set_knob(const char *name, const char *value);

#ifdef __cplusplus
}
#endif
#endif /* MEC_H */
