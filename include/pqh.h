/*
 * pqh.h -- the GPU batch boundary of pq_huffman_amd (C ABI, plain pointers and sizes).
 *
 * The reference has no FFI layer: its boundary is its C headers + CLI + file formats
 * (SURVEY.md 8b).  Its hot loops become the calls below; each names the reference code
 * it replaces.  All d_* pointers are DEVICE pointers owned by the caller; every call is
 * asynchronous on the context's HIP stream unless it says otherwise.  Calls return 0
 * (PQH_OK) or a negative pqh_status_t -- never assert or exit.  There is no CPU fallback:
 * without a usable GPU the calls return PQH_ERR_NO_DEVICE.
 *
 * Device data formats (shared with the CLI tools and the Python layer):
 *   codes        n x m row-major, uint8 (K <= 256) or uint16 (K <= 65536)
 *   counts       uint32 [m][K] (non-context) or [m][K*K] (context, index prev*K + cur)
 *   stream       byte stream exactly as huffman_indices.bin after its 8-byte header:
 *                vector-major, part-minor, MSB-first, zero padded at the end
 *   chunk index  (sidecar for parallel decode; not part of huffman_indices.bin)
 *                u64 bit offset of vector j*C for every chunk j, and in context mode
 *                the m codes of vector j*C-1 (row of chunk_prev) for j > 0
 */
#ifndef _PQH_H
#define _PQH_H

#include <stddef.h>
#include <stdint.h>

#include "fast_nn_block.h"
#include "huffman.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef enum {
    PQH_OK = 0,
    PQH_ERR_ARG = -1,
    PQH_ERR_NO_DEVICE = -2,
    PQH_ERR_HIP = -3,
    PQH_ERR_UNSUPPORTED = -4,
    PQH_ERR_CODE_TOO_LONG = -5,  /* a Huffman code longer than 56 bits (needs N >= F(58)) */
    PQH_ERR_CORRUPT = -6,        /* invalid code in a stream */
    PQH_ERR_NOMEM = -7,
    PQH_ERR_CAPACITY = -8,       /* output buffer too small */
    PQH_ERR_REMOTE = -9,         /* another rank's part of a sharded call failed */
    PQH_ERR_COMM = -10           /* a collective hook of a sharded call failed */
} pqh_status_t;

typedef struct pqh_ctx pqh_ctx_t;

/* ---- context: one per device, one host thread per context ----------------------- */
/* creates the context with a private non-blocking stream */
int pqh_ctx_create(pqh_ctx_t** ctx, int device);
/* Like pqh_ctx_create, but the context's own stream may only use `cus` compute units,
 * spread evenly over the device (hipExtStreamCreateWithCUMask) -- for running the
 * latency-bound code-table build beside the next batch's assignment. */
int pqh_ctx_create_cu_limited(pqh_ctx_t** ctx, int device, int cus);
/* As pqh_ctx_create_cu_limited; complement != 0 takes every compute unit the cus-subset does
 * NOT use, so two contexts (cus, 0) and (cus, 1) run side by side on disjoint CUs.
 * cus < 0: every compute unit on a CU-masked stream, which HIP gives a hardware queue of its
 * own (streams without a mask share GPU_MAX_HW_QUEUES queues). */
int pqh_ctx_create_cu_split(pqh_ctx_t** ctx, int device, int cus, int complement);
/* the context's current HIP stream (e.g. for torch.cuda.ExternalStream) */
void* pqh_ctx_stream(const pqh_ctx_t* ctx);
int pqh_ctx_destroy(pqh_ctx_t* ctx);
/* Free the context's grow-only device scratch (workspace, the tiled encoder's tile images,
 * the one-pass encoder's look-back state, the sort's state) after synchronising its stream;
 * later calls allocate again as needed.  The largest is the encoder's: ~56 B per encoded
 * row (one worst-case image per 256-row tile) for pqh_encode_write*. */
int pqh_ctx_release_scratch(pqh_ctx_t* ctx);
/* run all later calls on hip_stream, taken literally: NULL is the device's default
 * (legacy, synchronising) stream -- what torch's current stream usually is. */
int pqh_ctx_set_stream(pqh_ctx_t* ctx, void* hip_stream);
int pqh_ctx_sync(pqh_ctx_t* ctx);
/* Per-context launch shapes of the kernels this context launches (results never change;
 * 0 restores the library default, which the PQH_* environment variable of the same name
 * can set process-wide):
 *   PQH_TUNE_ASSIGN_WGS_PER_CU  workgroups per CU of the K = 256 assignment grid (<= its
 *                               occupancy limit, 3): fewer leave SIMD room for kernels
 *                               running beside it on other streams (PQH_ASSIGN_WGS_PER_CU);
 *   PQH_TUNE_HIST_SPLIT         the context histogram's split of the previous-symbol range
 *                               (1, 2, 4 or 8): LDS per workgroup = 128 KB / split at K = 256
 *                               (PQH_HIST_SPLIT);
 *   PQH_TUNE_HIST_BLOCK         its workgroup size, 256 or 1024 threads (PQH_HIST_BLOCK);
 *   PQH_TUNE_ENC_IMPL           the whole-stream encoder of pqh_encode_write*: 1 = tiled
 *                               (tiles in context scratch, scan, placement), 2 = one pass
 *                               with a decoupled look-back (PQH_ENC_IMPL=onepass).
 * A histogram that runs beside the assignment grid (on another stream) fits best at
 * split 4, 256 threads. */
enum { PQH_TUNE_ASSIGN_WGS_PER_CU = 1, PQH_TUNE_HIST_SPLIT = 2, PQH_TUNE_HIST_BLOCK = 3,
       PQH_TUNE_ENC_IMPL = 4 };
int pqh_ctx_set_tuning(pqh_ctx_t* ctx, int key, double value);
const char* pqh_status_string(int status);
const char* pqh_ctx_last_error(const pqh_ctx_t* ctx);
int pqh_device_count(int* count);

/* ---- PQ assignment (replaces yael kmeans' assignment, pq_encoder.c:270-273, and
 *      copy_cluster_indices :192-205) ----------------------------------------------- */
typedef struct pqh_pq pqh_pq_t;

/* centroids: host [m][k][dsub] fp32 (pq_centroids.fvecsl order). */
int pqh_pq_create(pqh_ctx_t* ctx, const float* centroids, int m, int k, int dsub, pqh_pq_t** pq);
int pqh_pq_destroy(pqh_pq_t* pq);

/* codes[v][i] = argmin_k sum_j (x[v][i*dsub+j] - c[i][k][j])^2, fp32 direct form, j
 * order, first minimum wins (oracle definition).  x rows are ld_x floats apart.
 * d_counts (optional, may be NULL): uint32 [m][k] non-context histogram accumulated
 * (+=) from the produced codes (huffman_encoder.c:139-164) -- fused in the kernel.
 * mode: 0 = MFMA screening + exact re-rank (default), 1 = exact VALU kernel only.
 * ctx: any context of the codebook's device; the launch uses its stream and scratch, so
 * contexts on different streams may assign concurrently. */
int pqh_pq_assign(pqh_ctx_t* ctx, const pqh_pq_t* pq, const float* d_x, long long n,
                  long long ld_x, void* d_codes, uint32_t* d_counts, int mode);
/* pqh_pq_assign writing the codes PART-MAJOR: codes of part i at d_codes[i * ld_codes + v]
 * (ld_codes >= n elements): each subspace's codes are contiguous, so the kernel stores
 * whole 128-byte lines (when d_codes is 128-byte aligned and ld_codes a multiple of 128
 * codes; any layout is correct) and a part's histogram reads one contiguous run (pqh_histogram_parts,
 * pqh_encode_write_parts consume this layout; pqh_transpose_codes converts to rows).
 * d_counts: as pqh_pq_assign (K <= 256 only). */
int pqh_pq_assign_parts(pqh_ctx_t* ctx, const pqh_pq_t* pq, const float* d_x, long long n,
                        long long ld_x, void* d_codes, long long ld_codes, uint32_t* d_counts,
                        int mode);
/* diagnostics of the last pqh_pq_assign (synchronises): vectors x parts re-ranked
 * exactly because the screening could not separate the best two centroids. */
int pqh_pq_last_rerank_count(pqh_ctx_t* ctx, unsigned long long* count);

/* mean squared reconstruction error (pq_encoder.c:82-119); synchronises. */
int pqh_pq_error(pqh_ctx_t* ctx, const pqh_pq_t* pq, const float* d_x, long long n,
                 long long ld_x, const void* d_codes, double* error_out);
/* x_hat[v] = concat_i c[i][codes[v][i]] (decode codes -> floats). */
int pqh_pq_reconstruct(pqh_ctx_t* ctx, const pqh_pq_t* pq, const void* d_codes, long long n,
                       float* d_out, long long ld_out);

/* ---- k-means training (replaces the training half of yael kmeans, pq_encoder.c:265-274) */
/* `iters` Lloyd iterations per subspace on the GPU: exact fp32 assignment (as
 * pqh_pq_assign) then centroid means; an empty cluster keeps its centroid.  Sums are
 * 64-bit fixed point (x * 2^s, s = 61 - ceil(log2(max|x| * n))), so the result is exact
 * and the same on every run.  centroids: host [m][k][dsub], initial in, trained out.
 * d_x rows are ld_x floats apart (subspace i = columns [i*dsub, (i+1)*dsub)).  Synchronous. */
int pqh_kmeans_train(pqh_ctx_t* ctx, const float* d_x, long long n, long long ld_x, int m,
                     int k, int dsub, int iters, float* centroids);

/* ---- symbol histograms (huffman_encoder.c:139-205) ------------------------------- */
/* counts += histogram of codes.  context: pairs (codes[v-1][i], codes[v][i]) for v >= 1,
 * plus (d_prev_row[i], codes[0][i]) when d_prev_row != NULL (the one-vector halo of a
 * shard boundary).  d_counts must be zeroed by the caller before the first call. */
int pqh_histogram(pqh_ctx_t* ctx, const void* d_codes, long long n, int m, int k, int context,
                  const void* d_prev_row, uint32_t* d_counts);
/* counts = histogram of codes (overwrites; no zeroing by the caller).  Same arguments. */
int pqh_histogram_set(pqh_ctx_t* ctx, const void* d_codes, long long n, int m, int k,
                      int context, const void* d_prev_row, uint32_t* d_counts);
/* The context histogram in two halves, for a pipelined caller that keeps the short first
 * half on its critical stream and moves the reduce to another (ordered by an event): the
 * per-chunk partial counts of the (prev, cur) pairs into d_partials (device,
 * pqh_histogram_partial_bytes(n, m, k) bytes, K <= 256), then counts (+)= their sum
 * (set != 0: overwrite).  Same pairs as pqh_histogram with context = 1. */
long long pqh_histogram_partial_bytes(long long n, int m, int k);
/* The same histograms over PART-MAJOR codes (pqh_pq_assign_parts: part i's codes at
 * d_codes[i * ld_codes + v]); set != 0 overwrites the counts.  d_prev_row stays a row of m
 * codes. */
int pqh_histogram_parts(pqh_ctx_t* ctx, const void* d_codes, long long ld_codes, long long n,
                        int m, int k, int context, const void* d_prev_row, uint32_t* d_counts,
                        int set);
int pqh_histogram_partial_parts(pqh_ctx_t* ctx, const void* d_codes, long long ld_codes,
                                long long n, int m, int k, const void* d_prev_row,
                                void* d_partials);
int pqh_histogram_partial(pqh_ctx_t* ctx, const void* d_codes, long long n, int m, int k,
                          const void* d_prev_row, void* d_partials);
int pqh_histogram_reduce(pqh_ctx_t* ctx, const void* d_partials, long long n, int m, int k,
                         uint32_t* d_counts, int set);

/* ---- code tables ------------------------------------------------------------------ */
/* Device-resident Huffman code tables of m parts: encode entries + decode lookup tables. */
typedef struct pqh_tables pqh_tables_t;

/* allocate tables for m parts of alphabet k (context: k must be 256) */
int pqh_tables_alloc(pqh_ctx_t* ctx, int m, int k, int context, pqh_tables_t** tables);
int pqh_tables_destroy(pqh_tables_t* tables);
/* Build every code on the GPU from device counts (pqh_histogram layout) -- the reference
 * codebook construction (huffman_codebook_[context_]encode_init, huffman_encode.c:141-269)
 * with its exact heap tie-breaks, one lane per alphabet; asynchronous, no host round trip.
 * Codes longer than 56 bits set an error reported by pqh_tables_status.  `ctx` may be any
 * context on the tables' device; the build is ordered on ctx's stream. */
int pqh_tables_build(pqh_ctx_t* ctx, pqh_tables_t* tables, const uint32_t* d_counts);
/* pqh_tables_build with the tree builder chosen by the caller (PQH_TREES_DEFAULT: the
 * PQH_TREE_IMPL environment choice, "lane" | "wave" | "grp").  K <= 256: GROUP = 16 lanes per
 * tree, four trees per wavefront, at most 32 VGPRs so it runs beside the assignment grid (the
 * default); LANE = one lane per tree; WAVE = one wavefront per tree with the heap in
 * registers.  K > 256: LANE = one lane per tree, otherwise one wavefront per tree.  Every
 * choice builds the same tables. */
enum { PQH_TREES_DEFAULT = 0, PQH_TREES_LANE = 1, PQH_TREES_WAVE = 2, PQH_TREES_GROUP = 3 };
int pqh_tables_build_impl(pqh_ctx_t* ctx, pqh_tables_t* t, const uint32_t* d_counts, int which);
/* The two halves of pqh_tables_build_impl, for callers that run them on different streams:
 * the Huffman trees (code table) on ctx's stream, then -- after the caller orders it behind
 * the trees (an event) -- the decode tables and the encoder's gather copy on ctx's stream.
 * With the K <= 256 group builder (PQH_TREES_GROUP, the default) the tree build writes the
 * encoder's gather copy itself, so pqh_encode* may run as soon as pqh_tables_build_trees is
 * done, concurrently with pqh_tables_build_luts (pqh_tables_encode_ready says which case
 * holds); pqh_decode always needs pqh_tables_build_luts. */
int pqh_tables_build_trees(pqh_ctx_t* ctx, pqh_tables_t* t, const uint32_t* d_counts, int which);
int pqh_tables_build_luts(pqh_ctx_t* ctx, pqh_tables_t* t);
/* 1 if the last pqh_tables_build_trees completed the encoder's tables (no LUT build needed
 * before pqh_encode*), else 0. */
int pqh_tables_encode_ready(const pqh_tables_t* t);
/* Two table sets (same m, K, mode) built by one launch of the default tree build (K <= 256:
 * the group builder, K > 256: one wavefront per tree): twice the trees in one latency-bound
 * pass, for a caller whose table builds are the bound; then both sets' decode tables.  Same
 * tables as two pqh_tables_build calls. */
int pqh_tables_build_pair(pqh_ctx_t* ctx, pqh_tables_t* t, const uint32_t* d_counts,
                          pqh_tables_t* t2, const uint32_t* d_counts2);
/* Load codes from m host codebooks (e.g. huffman_codebooks.bin read by huffman_codebook_load). */
int pqh_tables_upload(pqh_ctx_t* ctx, pqh_tables_t* tables, const huffman_codebook_t* codebooks);
/* alloc + upload */
int pqh_tables_create(pqh_ctx_t* ctx, const huffman_codebook_t* codebooks, int m,
                      pqh_tables_t** tables);
/* Synchronises; PQH_ERR_CODE_TOO_LONG if a GPU build of these tables since the last call
 * produced a code > 56 bits (the error is sticky until read here: a build issues no
 * zeroing dispatch of its own). */
int pqh_tables_status(pqh_ctx_t* ctx, const pqh_tables_t* tables);
/* Synchronises; fills m caller-provided structs with malloc'd host codebooks equal to the
 * tables (free with huffman_codebook_destroy) -- for huffman_codebook_save and stats. */
int pqh_tables_codebooks(pqh_ctx_t* ctx, const pqh_tables_t* tables, huffman_codebook_t* codebooks);

/* counts (host, double [m][items], huffman_encoder.c layout) -> host codebooks, built with
 * the reference's exact heap tie-breaks (huffman_encode.c:141-269).  Threads over parts
 * and context rows; codebooks must hold m uninitialised structs. */
int pqh_codebooks_build(const double* counts, int m, int k, int context,
                        huffman_codebook_t* codebooks, int num_threads);

/* ---- encode (huffman_encoder.c:207-238 + bitstream.c:71-150) --------------------- */
/* Total bits of the stream (device, u64) without writing it -- for placing shards before
 * they are written (multi-GPU); pqh_encode_write does not need it.
 * raw_first: context mode writes row 0 raw (8 bits per part, huffman_encoder.c:234) --
 * set for the shard holding global row 0; other shards pass d_prev_row instead. */
int pqh_encode_size(pqh_ctx_t* ctx, const pqh_tables_t* t, const void* d_codes, long long n,
                    int raw_first, const void* d_prev_row, unsigned long long* d_total_bits);
/* Write the stream at bit offset `bit_offset` of d_out (no pqh_encode_size needed): every
 * word of [bit_offset, bit_offset + bits) is stored exactly once, zero padding the last word
 * -- the buffer needs no zeroing.  By default 256-row tiles are coded into context scratch
 * (~56 B per row, grow-only; pqh_ctx_release_scratch frees it), scanned and placed; when that
 * scratch cannot be allocated (or PQH_ENC_IMPL=onepass) one pass whose workgroups find their
 * offsets by a decoupled look-back, with O(n / 256) state.  Bits of d_out before bit_offset in the first word are kept (they are
 * merged), so shards written at adjacent offsets into one buffer compose.
 * chunk_vectors > 0 also emits the chunk index: d_chunk_offsets[ceil(n/C)] (bit offsets
 * relative to d_out bit 0) and, in context mode, d_chunk_prev[ceil(n/C)][m] codes.
 * d_total_bits (optional, device u64): the number of bits written. */
int pqh_encode_write(pqh_ctx_t* ctx, const pqh_tables_t* t, const void* d_codes, long long n,
                     int raw_first, const void* d_prev_row, unsigned long long bit_offset,
                     unsigned char* d_out, unsigned long long out_bytes, int chunk_vectors,
                     unsigned long long* d_chunk_offsets, void* d_chunk_prev,
                     unsigned long long* d_total_bits);

/* pqh_encode_write for one shard of a multi-GPU stream, with the shard's GLOBAL bit offset
 * read from device memory (the exclusive scan of the shards' pqh_encode_size totals, e.g.
 * an all-gather + prefix sum on the device): no host round trip.  The shard is written at
 * bit (offset % 32) of d_out, whose word 0 is the global stream's word offset / 32, so the
 * shards' buffers compose by OR-ing their boundary words. */
int pqh_encode_write_at(pqh_ctx_t* ctx, const pqh_tables_t* t, const void* d_codes, long long n,
                        int raw_first, const void* d_prev_row,
                        const unsigned long long* d_global_bit_offset, unsigned char* d_out,
                        unsigned long long out_bytes, int chunk_vectors,
                        unsigned long long* d_chunk_offsets, void* d_chunk_prev,
                        unsigned long long* d_total_bits);

/* pqh_encode_write over PART-MAJOR codes (pqh_pq_assign_parts; part i of vector v at
 * d_codes[i * ld_codes + v]): the same stream, chunk index and chunk_prev rows.  The row
 * encoder only: K <= 256 and m = 8 or 16 (else PQH_ERR_UNSUPPORTED). */
int pqh_encode_write_parts(pqh_ctx_t* ctx, const pqh_tables_t* t, const void* d_codes,
                           long long ld_codes, long long n, int raw_first, const void* d_prev_row,
                           unsigned long long bit_offset, unsigned char* d_out,
                           unsigned long long out_bytes, int chunk_vectors,
                           unsigned long long* d_chunk_offsets, void* d_chunk_prev,
                           unsigned long long* d_total_bits);
/* part-major codes [m][ld_parts] -> rows [n][m] (pq_indices.bvecsl order); code_bytes 1 or 2. */
int pqh_transpose_codes(pqh_ctx_t* ctx, const void* d_parts, long long ld_parts, long long n, int m,
                        int code_bytes, void* d_rows);

/* Synchronises; PQH_ERR_CAPACITY if a pqh_encode_write since the last call had to drop
 * words because out_bytes was too small (nothing is written out of bounds). */
int pqh_encode_status(pqh_ctx_t* ctx);

/* ---- decode (huffman_decoder.c:211-255, huffman_decode.c:137-191) ---------------- */
/* Decodes n vectors from d_stream using the chunk index (C = chunk_vectors).  Context
 * mode: chunk 0 starts raw when raw_first, else from d_chunk_prev row 0.
 * Returns PQH_ERR_CORRUPT (after synchronising) if an invalid code was met. */
int pqh_decode(pqh_ctx_t* ctx, const pqh_tables_t* t, const unsigned char* d_stream,
               unsigned long long stream_bytes, long long n, int raw_first, int chunk_vectors,
               const unsigned long long* d_chunk_offsets, const void* d_chunk_prev,
               void* d_codes);
/* Synchronises; PQH_ERR_CORRUPT if a pqh_decode / pqh_decode_tree on this context since
 * the last call met an invalid code (sticky until read here, like pqh_encode_status). */
int pqh_decode_status(pqh_ctx_t* ctx);
/* Build the chunk index of an existing stream (one produced without a sidecar, e.g. by
 * the reference encoder) with a sequential table walk on the HOST copy of the stream
 * (index building only; the symbols themselves are decoded on the GPU). */
int pqh_chunk_index_host(const pqh_tables_t* t, const unsigned char* stream,
                         unsigned long long stream_bytes, long long n, int raw_first,
                         int chunk_vectors, unsigned long long* chunk_offsets,
                         void* chunk_prev);

/* ---- sort mode (huffman_encoder.c:301-317: qsort + strncmp) ---------------------- */
/* Stable sort of the n rows by key(row) = row with every byte after its first 0 zeroed
 * (strncmp order), uint8 codes only.
 * Workspace (grown in the context, kept between calls): the in-tree radix sort (2 <= m
 * <= 8, n < 2^31) takes 32 bytes per row + 8 KB plus a persistent 2 KB-per-8192-row
 * tile-state array, and sorts in place (d_tmp unused, may be NULL).  Other shapes, or
 * PQH_SORT_IMPL=rocprim, use rocPRIM's radix_sort_pairs: 24 bytes per row + its temp
 * storage, plus n*m bytes for the gathered rows unless d_tmp (n*m bytes) is given.
 * If the in-tree sort cannot allocate its workspace it retries on the rocPRIM path
 * before returning PQH_ERR_NOMEM. */
int pqh_sort_rows(pqh_ctx_t* ctx, void* d_codes, long long n, int m, void* d_tmp);

/* ---- multi-GPU row shards ------------------------------------------
 * One process per GPU; rank r owns a contiguous row range, described by a block_t
 * (src/fast_nn_block.h:4-25: id = first global row, size = rows; data / indices unused on
 * the device path).  The only exchanges are small: the one-row halo (context mode), the
 * histogram all-reduce that feeds the shared code tables (huffman_encoder.c:139-205 over
 * the whole input), and an all-gather of the shards' bit lengths whose exclusive scan places
 * every shard in the global stream (the bit cursor of bitstream.c:71-101).  The transport is
 * the caller's communicator, passed as hooks (RCCL, MPI, torch.distributed, gloo ...). */

/* rank `rank`'s rows of n_total over `world` ranks: sizes differ by at most one row.
 * Fills block->id / size (capacity = size, num_dimensions 0, data / indices NULL). */
int pqh_shard_block(long long n_total, int world, int rank, block_t* block);

/* Collective hooks over DEVICE buffers, ordered on `stream` (the context's): return 0 on
 * success.  all_reduce_sum_u32: in-place sum over ranks; all_gather: d_recv[world][bytes]
 * = every rank's d_send[bytes], in rank order. */
typedef struct {
    void* user;
    int world, rank;
    int (*all_reduce_sum_u32)(void* user, uint32_t* d_buf, long long count, void* stream);
    int (*all_gather)(void* user, const void* d_send, void* d_recv, long long bytes,
                      void* stream);
} pqh_shard_comm_t;

/* Scratch bytes pqh_shard_encode needs in d_scratch (device, 16-byte aligned). */
long long pqh_shard_scratch_bytes(int world, int m);

/* One rank's encode of its shard (uint8 codes, K <= 256 -- context mode needs K = 256):
 *   context mode: all-gather of every rank's (non-empty flag, last row) -> on the device,
 *     the halo of this shard = the last row of the nearest non-empty rank before it, and the
 *     raw first row (huffman_encoder.c:234) belongs to the first non-empty rank (a shard may
 *     be empty, e.g. a slice of the distributed sort);
 *   histogram of the shard (+ the halo pair) -> all_reduce_sum_u32 -> GPU code tables
 *   (identical on every rank: no broadcast) -> the shard's exact bit length -> all_gather
 *   of the lengths -> exclusive scan on the device -> pqh_encode_write_at.
 * Asynchronous: no host round trip (unless raw_first is non-NULL, which reads back at the
 * end whether this shard wrote the raw first row).
 * Outputs: d_counts [m][items] the GLOBAL histogram; tables built from it; d_out holds the
 * shard's bits at (global offset % 32) with word 0 = the global stream's word offset / 32
 * (buffers compose by OR-ing boundary words: pqh_shard_stitch); d_offsets[2] (device u64) =
 * {this shard's global bit offset, the global stream's length in bits}; the chunk index
 * (optional, chunk_vectors > 0) is relative to d_out bit 0.
 * Errors: PQH_ERR_ARG at once (before any collective) when ctx, comm, m, k, context,
 * d_counts, d_offsets or d_scratch are unusable -- the arguments the collectives need.  Any
 * other failure of this rank (its shard, tables or output arguments, or a library call)
 * keeps the rank in the collective sequence with an empty contribution and the sentinel
 * length ~0, and is returned here; every rank's d_offsets then reads {0, ~0}, which
 * pqh_shard_status reports as PQH_ERR_REMOTE -- no rank is left waiting in a collective. */
int pqh_shard_encode(pqh_ctx_t* ctx, const pqh_shard_comm_t* comm, const block_t* shard,
                     const void* d_codes, int m, int k, int context, pqh_tables_t* tables,
                     uint32_t* d_counts, unsigned char* d_out, unsigned long long out_bytes,
                     int chunk_vectors, unsigned long long* d_chunk_offsets, void* d_chunk_prev,
                     unsigned long long* d_offsets, void* d_scratch, int* raw_first);
/* pqh_shard_encode in two phases, for a caller that pipelines batches (bench.py): phase 1
 * (halo, histogram, all-reduce, code tables) and phase 2 (length, all-gather, offsets,
 * write) may run on different streams -- ordered by the caller -- with other batches'
 * collectives between them.  Both take the same d_scratch; phase 2's `status` is phase 1's
 * return value (a nonzero status sends the sentinel length).  pqh_shard_encode = phase 1 +
 * phase 2.  A collective hook failure returns PQH_ERR_COMM. */
int pqh_shard_encode_tables(pqh_ctx_t* ctx, const pqh_shard_comm_t* comm, const block_t* shard,
                            const void* d_codes, int m, int k, int context,
                            pqh_tables_t* tables, uint32_t* d_counts, void* d_scratch);
int pqh_shard_encode_write(pqh_ctx_t* ctx, const pqh_shard_comm_t* comm, const block_t* shard,
                           const void* d_codes, int m, int k, int context, pqh_tables_t* tables,
                           unsigned char* d_out, unsigned long long out_bytes, int chunk_vectors,
                           unsigned long long* d_chunk_offsets, void* d_chunk_prev,
                           unsigned long long* d_offsets, void* d_scratch, int status,
                           int* raw_first);
/* The two phases for PART-MAJOR codes (pqh_pq_assign_parts: part i's codes at
 * d_codes[i * ld_codes + v], ld_codes >= the shard's rows), so a multi-rank pipeline runs the
 * single-rank one (bench.py): phase 2 takes m = 8 or 16 (the row encoder reading part runs).
 * d_partials (phase 1, optional, context mode): the shard's partial pair counts taken by
 * pqh_histogram_partial_parts(d_codes, ld_codes, n, m, k, NULL, d_partials) -- e.g. on the
 * assignment stream, ordered before this call by the caller; phase 1 then reduces them and
 * adds the shard-boundary pair itself instead of running the histogram.  NULL: phase 1 runs
 * the part-major histogram (with the halo pair).  Same errors and outputs as above. */
int pqh_shard_encode_tables_parts(pqh_ctx_t* ctx, const pqh_shard_comm_t* comm,
                                  const block_t* shard, const void* d_codes, long long ld_codes,
                                  int m, int k, int context, pqh_tables_t* tables,
                                  uint32_t* d_counts, void* d_scratch, const void* d_partials);
int pqh_shard_encode_write_parts(pqh_ctx_t* ctx, const pqh_shard_comm_t* comm,
                                 const block_t* shard, const void* d_codes, long long ld_codes,
                                 int m, int k, int context, pqh_tables_t* tables,
                                 unsigned char* d_out, unsigned long long out_bytes,
                                 int chunk_vectors, unsigned long long* d_chunk_offsets,
                                 void* d_chunk_prev, unsigned long long* d_offsets, void* d_scratch,
                                 int status, int* raw_first);
/* Synchronises; PQH_ERR_REMOTE if some rank's pqh_shard_encode behind d_offsets failed. */
int pqh_shard_status(pqh_ctx_t* ctx, const unsigned long long* d_offsets);

/* Host: (this rank's global bit offset, the global length) from every rank's bit length. */
int pqh_shard_offsets(const unsigned long long* lengths, int world, int rank,
                      unsigned long long* offset, unsigned long long* total);
/* Host: the global stream (huffman_indices.bin after its 8-byte header) from the ranks'
 * shard buffers: buffer r holds its bits at offsets[r] % 32, its byte 0 being global byte
 * (offsets[r] / 32) * 4; bits outside each range are zero.  out (zeroed here) needs
 * ceil(sum(bits) / 8) bytes. */
int pqh_shard_stitch(int world, const unsigned char* const* bufs,
                     const unsigned long long* offsets, const unsigned long long* bits,
                     unsigned char* out, unsigned long long out_bytes);
/* Host: for shards that may be empty (sorted slices): the rank whose last row is this
 * shard's halo (-1: none) and whether this shard writes the raw first row. */
int pqh_shard_halo_source(const int* nonempty, int world, int rank, int* prev_rank,
                          int* raw_first);

/* ---- forest builder of tree mode (compute_nn_fast.c + mst_builder.c) ---- */
/* compute_nn_fast's block geometry (blocks_info_init / dimension_info_build,
 * fast_nn_blocks_info.c:52-112) over n device rows of d floats (row stride ld_x): split i
 * is coordinate num_split-1-i; h_starts / h_ends [num_split][blocks_per_dim] receive the
 * block ranges the reference stores in dimension_infos[i].block_starts / block_ends.
 * blocks_per_dim <= 32, num_split <= 8. */
int pqh_knn_blocks_info(pqh_ctx_t* ctx, const float* d_x, long long n, long long ld_x, int d,
                        int num_split, int blocks_per_dim, double overlap, float* h_starts,
                        float* h_ends);
/* compute_nn_fast with one block per pass (run, compute_nn_fast.c:510-620; the CLI's
 * --num-dimensions-at-pass 0): every block's exact kNN among its rows, merged per row in
 * block order into a num_nn max-heap (fast_nn_heap_push) and sorted -- d_indices / d_dists
 * [n][num_nn] as nn_indices.ivecsl / nn_dist.fvecsl hold them (never-filled slots:
 * 0xFFFFFFFF / +inf).  The in-block neighbours are the smallest direct-form fp32 squared
 * distances (get_real_dist, :304-311), lower block position first on ties (the reference
 * calls yael's knn_full_thread here: parity unpinned at that call).  d <= 128,
 * num_nn <= 63.  h_block_sizes (may be NULL): [blocks_per_dim^num_split] rows per block. */
int pqh_knn_fast(pqh_ctx_t* ctx, const float* d_x, long long n, long long ld_x, int d,
                 int num_nn, int num_split, int blocks_per_dim, const float* h_starts,
                 const float* h_ends, uint32_t* d_indices, float* d_dists,
                 long long* h_block_sizes);
/* mst_builder's forest (load_mst_edges_from_nn_files + minimum_spanning_tree,
 * mst.c:80-236): the first `take` neighbours of each of the n rows of the kNN lists
 * (num_nn per row, device), re-scored first when penalty > 0 (Hamming distance of the
 * device PQ codes d_pq [n][pq_m] times penalty, or the Hamming distance alone when
 * infinite), Kruskal in distance order.  Outputs tree_save_file's arrays (mst.c:253-265):
 * h_targets [*num_edges <= 2 (n - 1)] grouped by source, h_counts [n].  Synchronises.
 * PQH_ERR_ARG for a neighbour id outside the rows. */
int pqh_mst_build(pqh_ctx_t* ctx, const uint32_t* d_indices, const float* d_dists, long long n,
                  int num_nn, int take, const uint8_t* d_pq, int pq_m, float penalty,
                  uint32_t* h_targets, int* h_counts, long long* num_edges);

/* compute_nn_fast as a whole (the CLI, csrc/tools/compute_nn_fast.c): .fvecs rows in,
 * <out_template>nn_indices.ivecsl / nn_dist.fvecsl out.  options may be NULL (the reference
 * CLI's defaults, compute_nn_fast.c:164-175: 5 splits, 3 blocks, overlap 0.3).  A
 * blocks_info_cache that loads supplies the geometry; otherwise it is written
 * (fast_nn_blocks_info.c:124-172 layout).  with_blocks_stat writes blocks_stat.txt. */
typedef struct {
    int num_split;               /* --num-dims */
    int blocks_per_dim;          /* --num-blocks-per-dim */
    double overlap;              /* --block-overlap-fraction */
    const char* blocks_info_cache;
    int with_blocks_stat;
} pqh_knn_options_t;
int pqh_knn_fast_files(const char* input_fvecs, const char* out_template, int num_nn,
                       const pqh_knn_options_t* options);
/* mst_builder as a whole (mst_builder.c:98-131): <nn_template>nn_indices.ivecsl +
 * nn_dist.fvecsl (+ <pq_template>pq_indices.bvecsl, may be NULL) in; <out_template>mst.tree,
 * and with PQ codes stats.json / stats_num_children.json (appended) plus the indices stats
 * line on stdout. */
int pqh_mst_files(const char* nn_template, const char* out_template, int take,
                  const char* pq_template, float penalty);

/* ---- tree-ordered context coding (huffman_encoder.c --tree: :240-286, :321-375) ---- */
/* DFS order of a stored forest (mst.tree: tree_load_file, mst.c:273-288 -- num_edges
 * u32 targets grouped by source, children_counts[v] of them per vertex) exactly as
 * tree_collect_vertices_dfs (mst.c:290-364), plus each stream row's coding context, the
 * traverser's active parent (mst.c:366-405): parents[p] = the parent's vertex id, or -1 for
 * a root.  Host; returns num_roots (>= 1 when num_vertices > 0) or PQH_ERR_ARG.
 * parents may be NULL. */
int pqh_tree_order(long long num_vertices, long long num_edges, const uint32_t* edge_targets,
                   const int* children_counts, uint32_t* vertices, int* num_children,
                   long long* parents);
/* pqh_tree_order on the device, for a forest (no self-loop, every edge stored in both
 * directions once, no cycle): device counts/targets in, device vertices / num_children /
 * parents (may be NULL) out, *num_roots on the host.  PQH_ERR_UNSUPPORTED for a graph that is
 * not such a forest (nothing written; pqh_tree_order walks any graph), PQH_ERR_ARG for
 * counts that are negative or do not sum to num_edges.  Synchronises. */
int pqh_tree_order_device(pqh_ctx_t* ctx, long long num_vertices, long long num_edges,
                          const uint32_t* d_edge_targets, const int* d_children_counts,
                          uint32_t* d_vertices, int* d_num_children, long long* d_parents,
                          int* num_roots);
/* d_rows[p] = d_codes[d_vertices[p]] (stream order) and d_tree_prev[p][i] =
 * d_codes[d_parents[p]][i], 0xFFFF for a root.  Ids outside [0, n) are reported by
 * pqh_tree_status (nothing is read for them). */
int pqh_tree_gather(pqh_ctx_t* ctx, const void* d_codes, long long n, int m, int k,
                    const uint32_t* d_vertices, const long long* d_parents, void* d_rows,
                    uint16_t* d_tree_prev);
/* Synchronises; PQH_ERR_ARG if the last pqh_tree_gather met an id outside the rows. */
int pqh_tree_status(pqh_ctx_t* ctx);
/* counts[i][prev][cur] += pairs (d_tree_prev[p][i], d_rows[p][i]) of the non-root rows
 * (tree_collect_indices_stats, mst.c:442-490); K = 256, u8 rows. */
int pqh_histogram_tree(pqh_ctx_t* ctx, const void* d_rows, const uint16_t* d_tree_prev,
                       long long n, int m, int k, uint32_t* d_counts);
/* encode_tree_data (huffman_encoder.c:240-286): context tables, each row coded in its
 * d_tree_prev context, roots raw 8 bits per part.  Same buffer rules as pqh_encode_write;
 * chunk_vectors > 0 emits the chunk bit offsets (the tree decoder's index). */
int pqh_encode_tree_write(pqh_ctx_t* ctx, const pqh_tables_t* t, const void* d_rows,
                          const uint16_t* d_tree_prev, long long n,
                          unsigned long long bit_offset, unsigned char* d_out,
                          unsigned long long out_bytes, int chunk_vectors,
                          unsigned long long* d_chunk_offsets, unsigned long long* d_total_bits);
/* Decode-side index from the child counts (decoded children stream): parent_pos[p] = the
 * stream position of row p's context (-1: root; huffman_decoder.c:214-247), and per chunk
 * of C rows the rows whose context precedes the chunk: ext_offsets[chunks + 1] into
 * ext_positions (may be NULL to count).  Host; returns the ext count or PQH_ERR_ARG. */
long long pqh_tree_ext_index(long long n, const int* num_children, int chunk_vectors,
                             long long* parent_pos, long long* ext_offsets,
                             long long* ext_positions);
/* pqh_tree_ext_index on the device, from device child counts (child_bytes 1, 2 or 4: u8,
 * u16 or i32): d_parent_pos[n], d_ext_offsets[chunks + 1] and, unless NULL,
 * d_ext_positions (room for n); returns the ext count or a negative status.  Same results
 * as the host walk for any counts.  Synchronises. */
long long pqh_tree_ext_index_device(pqh_ctx_t* ctx, long long n, const void* d_num_children,
                                    int child_bytes, int chunk_vectors, long long* d_parent_pos,
                                    long long* d_ext_offsets, long long* d_ext_positions);
/* huffman_decoder --tree on the GPU: rows in stream order.  One lane per chunk (offsets
 * from pqh_encode_tree_write); a context inside the chunk is read from the chunk's own
 * decoded rows, one before it from d_ext_rows[d_ext_offsets[j]...] (m codes each, the rows
 * at ext_positions).  stream_bytes is the stream's exact length (d_stream readable up to the
 * next multiple of 4 bytes); a chunk whose offset or symbols pass stream_bytes * 8 bits (a
 * truncated file, a stale sidecar) is an error.  Errors are reported by pqh_decode_status. */
int pqh_decode_tree(pqh_ctx_t* ctx, const pqh_tables_t* t, const unsigned char* d_stream,
                    unsigned long long stream_bytes, long long n, int chunk_vectors,
                    const unsigned long long* d_chunk_offsets, const long long* d_parent_pos,
                    const long long* d_ext_offsets, const unsigned char* d_ext_rows,
                    void* d_rows);

/* ---- whole-file host helpers used by the CLI tools ------------------------------- */
typedef struct {
    int context;           /* order-1 context coding (default 1) */
    int sort;              /* 0 none, 1 strncmp sort (default 1) */
    int chunk_vectors;     /* decode chunk size for the sidecar (default 64) */
    int only_estimate;     /* stats only (huffman_encoder --only-estimate) */
} pqh_encode_options_t;

/* Runs histogram -> GPU codebooks -> encode on host codes (n x m, K=256).  Produces the
 * reference files under out_prefix: huffman_codebooks.bin, huffman_indices.bin,
 * huffman_stats.txt (appended), and the decode sidecar huffman_chunks.bin. */
int pqh_encode_files(const unsigned char* codes, long long n, int m,
                     const pqh_encode_options_t* options, const char* out_prefix);
/* huffman_encoder --tree <tree_path>: tree-ordered context coding of host codes (n x m,
 * K = 256) over the forest stored in mst.tree (sorted first when sort != 0, as the CLI
 * does).  Writes the reference's tree-mode files under out_prefix: huffman_codebooks.bin,
 * huffman_indices.bin, huffman_stats.txt, huffman_children_codebooks.bin,
 * huffman_children.bin, huffman_children_stats.txt, plus the decode sidecar
 * huffman_tree_chunks.bin (pqh extension: chunk bit offsets + ext context rows). */
int pqh_encode_tree_files(const unsigned char* codes, long long n, int m, int sort,
                          const char* tree_path, const char* out_prefix);
/* huffman_decoder --tree: decodes the tree-mode files under in_prefix into rows in stream
 * (DFS) order, as the reference decoder writes them.  Needs the decode sidecar
 * huffman_tree_chunks.bin that pqh_encode_tree_files writes (PQH_ERR_ARG without it). */
int pqh_decode_tree_files(const char* in_prefix, unsigned char** codes_out, long long* n_out,
                          int* m_out);
/* Decodes huffman_indices.bin (+ sidecar when present) under in_prefix into codes
 * (n x m host buffer, n from the file header). */
int pqh_decode_files(const char* in_prefix, unsigned char** codes_out, long long* n_out,
                     int* m_out);

#ifdef __cplusplus
}
#endif

#endif /* _PQH_H */
