// pqh_shard.hip -- the multi-GPU row-shard protocol of the encode path behind the C ABI
// (include/pqh.h "multi-GPU row shards").
//
// The reference encodes one file on one host (huffman_encoder.c:139-238); sharded over
// ranks the only data that crosses ranks is small:
//   * the one-row halo: the pair (last row of the previous shard, first row of this one) is
//     counted (huffman_encoder.c:166-205) and coded with that row as context (:220-238), and
//     only the shard holding global row 0 writes it raw (:234);
//   * the histogram all-reduce feeding the shared code tables (built identically on every
//     rank, so no broadcast);
//   * an all-gather of the shards' bit lengths, whose exclusive scan is the bit cursor of
//     bitstream.c:71-101 at each shard's start.
// The transport is the caller's (pqh_shard_comm_t hooks over device buffers).
#include <cstring>
#include <vector>

#include "pqh_internal.h"

namespace {

// d_offsets = {sum of the lengths of the ranks before `rank`, sum of all lengths}; a rank
// that failed locally sent the sentinel length ~0: then {0, ~0} (pqh_shard_status reports it)
__global__ void shard_prefix(const unsigned long long* __restrict__ lengths, int world, int rank,
                             unsigned long long* __restrict__ offsets,
                             uint32_t* __restrict__ out_word0) {
    if (threadIdx.x != 0 || blockIdx.x != 0) return;
    // word 0 of the shard's output: the bits before its offset belong to the previous shard
    // and stay zero here (the placement ORs its first bits into it) -- no memset dispatch
    if (out_word0) *out_word0 = 0u;
    unsigned long long before = 0, all = 0;
    bool failed = false;
    for (int r = 0; r < world; ++r) {
        failed |= lengths[r] == ~0ull;
        before += r < rank ? lengths[r] : 0ull;
        all += lengths[r];
    }
    offsets[0] = failed ? 0ull : before;
    offsets[1] = failed ? ~0ull : all;
}

constexpr long long kHaloData = 16;   // a halo record: flag byte, pad, the row at byte 16

long long halo_record_bytes(int m) { return ((kHaloData + m + 15) / 16) * 16; }

// The halo of this shard, decided on the device from every rank's record (flag byte = the
// shard is non-empty, its last row at byte 16): the last row of the nearest non-empty rank
// before this one goes to `row`, and *rawf = 1 when there is none -- this shard then holds
// global row 0 and writes it raw (huffman_encoder.c:234); pqh_shard_halo_source's rule.
__global__ void shard_halo_pick(const unsigned char* __restrict__ recs, long long recb, int world,
                                int rank, int m, unsigned char* __restrict__ row,
                                int* __restrict__ rawf) {
    int prev = -1;
    for (int r = 0; r < rank && r < world; ++r)
        if (recs[r * recb]) prev = r;
    if (threadIdx.x == 0) *rawf = prev < 0 ? 1 : 0;
    for (int i = threadIdx.x; i < m; i += blockDim.x)
        row[i] = prev >= 0 ? recs[prev * recb + kHaloData + i] : (unsigned char)0;
}

// this shard's halo record, all recb bytes written (no memset dispatch): the flag byte
// (1 = the shard is non-empty), zero padding, and its last row at byte kHaloData, from
// row-major codes (ldc = 0) or part-major ones (part i's codes at i * ldc); n = 0: all zero
__global__ void shard_last_row(const unsigned char* __restrict__ codes, long long ldc, long long n,
                               int m, unsigned char* __restrict__ rec, long long recb) {
    for (long long i = threadIdx.x; i < recb; i += blockDim.x) {
        unsigned char v = 0;
        if (i == 0) v = n > 0 ? 1 : 0;
        else if (n > 0 && i >= kHaloData && i < kHaloData + m) {
            const long long j = i - kHaloData;
            v = ldc ? codes[j * ldc + n - 1] : codes[(n - 1) * m + j];
        }
        rec[i] = v;
    }
}

// the shard-boundary pair (halo row, first row) of every part, one count each, when this
// shard does not hold global row 0 (*rawf == 0): what the histogram's prev_row adds, for
// counts reduced from partials that were taken without the halo (pqh_histogram_partial_parts
// on the assignment stream, before the halo exchange)
__global__ void shard_halo_pair(uint32_t* __restrict__ counts, const unsigned char* __restrict__ halo,
                                const int* __restrict__ rawf, const unsigned char* __restrict__ codes,
                                long long ldc, int m, int k) {
    if (*rawf) return;
    for (int i = threadIdx.x; i < m; i += blockDim.x) {
        const unsigned p = halo[i], c = ldc ? codes[(long long)i * ldc] : codes[i];
        if (p < (unsigned)k && c < (unsigned)k) counts[(long long)i * k * k + p * (unsigned)k + c] += 1u;
    }
}

}  // namespace

extern "C" {

int pqh_shard_block(long long n_total, int world, int rank, block_t* block) {
    if (!block || n_total < 0 || world <= 0 || rank < 0 || rank >= world) return PQH_ERR_ARG;
    const long long base = n_total / world, extra = n_total % world;
    block->id = (long long)rank * base + (rank < extra ? rank : extra);
    block->size = base + (rank < extra ? 1 : 0);
    block->capacity = block->size;
    block->num_dimensions = 0;
    block->data = nullptr;
    block->indices = nullptr;
    return PQH_OK;
}

// scratch: [send record][world records][halo row (a record's size)][send length]
//          [world lengths][raw-first flag, 64 B][pad to 256 B]
// (round 5: the shard's length comes from the encoder's tile pass, so the copy of the local
// histogram that round 4 kept here for it is gone)
long long pqh_shard_scratch_bytes(int world, int m) {
    if (world <= 0 || m <= 0) return PQH_ERR_ARG;
    return ((halo_record_bytes(m) * (world + 2) + 8ll * (world + 1) + 64 + 255) / 256) * 256;
}

int pqh_shard_offsets(const unsigned long long* lengths, int world, int rank,
                      unsigned long long* offset, unsigned long long* total) {
    if (!lengths || world <= 0 || rank < 0 || rank >= world || !offset || !total)
        return PQH_ERR_ARG;
    unsigned long long before = 0, all = 0;
    for (int r = 0; r < world; ++r) {
        if (r < rank) before += lengths[r];
        all += lengths[r];
    }
    *offset = before;
    *total = all;
    return PQH_OK;
}

int pqh_shard_stitch(int world, const unsigned char* const* bufs,
                     const unsigned long long* offsets, const unsigned long long* bits,
                     unsigned char* out, unsigned long long out_bytes) {
    if (world <= 0 || !bufs || !offsets || !bits || (!out && out_bytes)) return PQH_ERR_ARG;
    unsigned long long total = 0;
    for (int r = 0; r < world; ++r) total += bits[r];
    if (out_bytes < (total + 7) / 8) return PQH_ERR_CAPACITY;
    memset(out, 0, (size_t)((total + 7) / 8));
    for (int r = 0; r < world; ++r) {
        if (!bits[r]) continue;
        if (!bufs[r] || offsets[r] + bits[r] > total) return PQH_ERR_ARG;
        const unsigned long long start = (offsets[r] / 32) * 4;          // buffer byte 0
        const unsigned long long end = (offsets[r] + bits[r] + 7) / 8;   // past the last byte
        for (unsigned long long j = start; j < end; ++j) out[j] |= bufs[r][j - start];
    }
    return PQH_OK;
}

int pqh_shard_halo_source(const int* nonempty, int world, int rank, int* prev_rank,
                          int* raw_first) {
    if (!nonempty || world <= 0 || rank < 0 || rank >= world || !prev_rank || !raw_first)
        return PQH_ERR_ARG;
    int prev = -1, first = -1;
    for (int r = 0; r < world; ++r) {
        if (!nonempty[r]) continue;
        if (first < 0) first = r;
        if (r < rank) prev = r;
    }
    *prev_rank = prev;
    *raw_first = first == rank ? 1 : 0;
    return PQH_OK;
}

namespace {
// the scratch layout (pqh_shard_scratch_bytes)
struct ShardScratch {
    unsigned char* halo_send;
    unsigned char* halo_recv;
    unsigned char* halo_row;
    unsigned long long* len_send;
    unsigned long long* len_recv;
    int* rawf;
    long long recb;
    ShardScratch(void* d, int world, int m) {
        unsigned char* p = static_cast<unsigned char*>(d);
        recb = halo_record_bytes(m);
        halo_send = p;
        halo_recv = p + recb;
        halo_row = p + recb * (world + 1);
        len_send = reinterpret_cast<unsigned long long*>(p + recb * (world + 2));
        len_recv = len_send + 1;
        rawf = reinterpret_cast<int*>(len_recv + world);
    }
};

// Without these the collective sequence itself cannot run (or would not match the other
// ranks' sizes): refused before the first collective.
bool shard_fatal(const pqh_ctx_t* ctx, const pqh_shard_comm_t* comm, int m, int k, int context,
                 const void* d_scratch) {
    return !ctx || !comm || comm->world <= 0 || comm->rank < 0 || comm->rank >= comm->world ||
           !comm->all_gather || !comm->all_reduce_sum_u32 || m <= 0 || k <= 0 || k > 256 ||
           (context && k != 256) || !d_scratch || (reinterpret_cast<uintptr_t>(d_scratch) & 15u);
}

bool shard_local_bad(const block_t* shard, const void* d_codes, const pqh_tables_t* tables, int m,
                     int k, int context) {
    return !shard || shard->size < 0 || (shard->size > 0 && !d_codes) || !tables ||
           tables->m != m || tables->k != k || (tables->context ? 1 : 0) != (context ? 1 : 0);
}
}  // namespace

// Phase 1: halo, histogram, all-reduce, code tables.  Any failure after the fatal checks is
// local: the rank stays in the collective sequence (an empty halo record, a histogram
// counting nothing), the error is returned and must be handed to phase 2 (status), which
// then sends the sentinel length so every rank sees it (pqh_shard_status).
static int shard_tables_impl(pqh_ctx_t* ctx, const pqh_shard_comm_t* comm, const block_t* shard,
                             const void* d_codes, long long ldc, int m, int k, int context,
                             pqh_tables_t* tables, uint32_t* d_counts, void* d_scratch,
                             const void* d_partials) {
    if (shard_fatal(ctx, comm, m, k, context, d_scratch) || !d_counts) return PQH_ERR_ARG;
    int rc = pqh_use_device(ctx);
    if (rc) return rc;
    int err = shard_local_bad(shard, d_codes, tables, m, k, context) ? PQH_ERR_ARG : PQH_OK;
    if (!err && ldc && (ldc < shard->size || (d_partials && !context))) err = PQH_ERR_ARG;
    auto local = [&](int r) {   // the first local failure is kept
        if (r && !err) err = r;
    };
    const long long n = err ? 0 : shard->size;
    const int world = comm->world, rank = comm->rank;
    ShardScratch sc(d_scratch, world, m);
    void* const st = ctx->stream;
    // the halo (context mode): every rank's (non-empty flag, last row); the halo row and the
    // raw-first flag are picked on the device -- no host round trip
    if (context) {
        // (n = 0 -- an empty shard or a local failure: an all-zero record, "no rows")
        hipLaunchKernelGGL(shard_last_row, dim3(1), dim3(64), 0, ctx->stream,
                           static_cast<const unsigned char*>(d_codes), ldc, err ? 0ll : n, m,
                           sc.halo_send, (long long)sc.recb);
        local(hipGetLastError() == hipSuccess ? PQH_OK : PQH_ERR_HIP);
        if (comm->all_gather(comm->user, sc.halo_send, sc.halo_recv, sc.recb, st))
            return pqh_set_error(ctx, PQH_ERR_COMM, "shard halo all-gather failed");
        hipLaunchKernelGGL(shard_halo_pick, dim3(1), dim3(64), 0, ctx->stream, sc.halo_recv,
                           sc.recb, world, rank, m, sc.halo_row, sc.rawf);
        local(hipGetLastError() == hipSuccess ? PQH_OK : PQH_ERR_HIP);
    }
    // the shard's histogram (+ the halo pair), summed over ranks -> identical tables
    const long long items = context ? (long long)k * k : k;
    if (err) {
        local(hipMemsetAsync(d_counts, 0, (size_t)m * items * 4, ctx->stream) == hipSuccess
                  ? PQH_OK : PQH_ERR_HIP);
    } else if (d_partials) {
        // the partial counts were taken on another stream, without the halo: reduce them,
        // then add the boundary pair
        local(pqh_histogram_reduce(ctx, d_partials, n, m, k, d_counts, 1));
        if (n > 0 && !err) {
            hipLaunchKernelGGL(shard_halo_pair, dim3(1), dim3(64), 0, ctx->stream, d_counts,
                               sc.halo_row, sc.rawf, static_cast<const unsigned char*>(d_codes),
                               ldc, m, k);
            local(hipGetLastError() == hipSuccess ? PQH_OK : PQH_ERR_HIP);
        }
    } else if (context) {
        local(pqh_histogram_set_dev_ld(ctx, d_codes, ldc, n, m, k, sc.halo_row, sc.rawf, d_counts));
    } else {
        local(ldc ? pqh_histogram_parts(ctx, d_codes, ldc, n, m, k, 0, nullptr, d_counts, 1)
                  : pqh_histogram_set(ctx, d_codes, n, m, k, 0, nullptr, d_counts));
    }
    if (comm->all_reduce_sum_u32(comm->user, d_counts, (long long)m * items, st))
        return pqh_set_error(ctx, PQH_ERR_COMM, "shard histogram all-reduce failed");
    if (!err) local(pqh_tables_build(ctx, tables, d_counts));
    return err;
}

int pqh_shard_encode_tables(pqh_ctx_t* ctx, const pqh_shard_comm_t* comm, const block_t* shard,
                            const void* d_codes, int m, int k, int context,
                            pqh_tables_t* tables, uint32_t* d_counts, void* d_scratch) {
    return shard_tables_impl(ctx, comm, shard, d_codes, 0, m, k, context, tables, d_counts,
                             d_scratch, nullptr);
}

int pqh_shard_encode_tables_parts(pqh_ctx_t* ctx, const pqh_shard_comm_t* comm,
                                  const block_t* shard, const void* d_codes, long long ld_codes,
                                  int m, int k, int context, pqh_tables_t* tables,
                                  uint32_t* d_counts, void* d_scratch, const void* d_partials) {
    if (ld_codes <= 0) return PQH_ERR_ARG;
    return shard_tables_impl(ctx, comm, shard, d_codes, ld_codes, m, k, context, tables, d_counts,
                             d_scratch, d_partials);
}

// Phase 2: the shard's exact length, everyone's (all-gather; the sentinel ~0 when status,
// the rank's phase-1 result, or this phase fails locally), the exclusive scan on the device,
// and the write.
static int shard_write_impl(pqh_ctx_t* ctx, const pqh_shard_comm_t* comm, const block_t* shard,
                            const void* d_codes, long long ldc, int m, int k, int context,
                            pqh_tables_t* tables, unsigned char* d_out, unsigned long long out_bytes,
                            int chunk_vectors, unsigned long long* d_chunk_offsets,
                            void* d_chunk_prev, unsigned long long* d_offsets, void* d_scratch,
                            int status, int* raw_first_out) {
    if (shard_fatal(ctx, comm, m, k, context, d_scratch) || !d_offsets) return PQH_ERR_ARG;
    int rc = pqh_use_device(ctx);
    if (rc) return rc;
    int err = status;
    if (!err && (shard_local_bad(shard, d_codes, tables, m, k, context) || !d_out || out_bytes < 4 ||
                 (reinterpret_cast<uintptr_t>(d_out) & 3)))
        err = PQH_ERR_ARG;
    // (part-major codes: the 8-byte-row encoder's shapes, m = 8 or 16 u8 codes)
    if (!err && ldc && (ldc < shard->size || (m != 8 && m != 16) ||
                        (reinterpret_cast<uintptr_t>(d_chunk_prev) & 7)))
        err = PQH_ERR_ARG;
    const long long n = err ? 0 : shard->size;
    const int world = comm->world, rank = comm->rank;
    ShardScratch sc(d_scratch, world, m);
    // the shard's exact length from the tiled encoder's first half (its tiles coded into
    // scratch, their bit counts scanned -- nothing depends on the offset yet), all-gathered;
    // the sentinel ~0 when status, the rank's phase-1 result, or this phase fails locally
    const void* prev = context ? sc.halo_row : nullptr;
    const int* rawf = context ? sc.rawf : nullptr;
    if (!err) {
        const int r = pqh_encode_tiles_dev_ld(ctx, tables, d_codes, ldc, n, prev, rawf,
                                              chunk_vectors, d_chunk_offsets, d_chunk_prev,
                                              sc.len_send);
        if (r) err = r;
    }
    if (err) (void)hipMemsetAsync(sc.len_send, 0xFF, 8, ctx->stream);   // the sentinel length
    if (comm->all_gather(comm->user, sc.len_send, sc.len_recv, 8, ctx->stream))
        return pqh_set_error(ctx, PQH_ERR_COMM, "shard length all-gather failed");
    // (word 0 of d_out = the global word offset / 32: shard_prefix zeroes it)
    hipLaunchKernelGGL(shard_prefix, dim3(1), dim3(64), 0, ctx->stream, sc.len_recv, world, rank,
                       d_offsets, err ? nullptr : reinterpret_cast<uint32_t*>(d_out));
    PQH_LAUNCH_CHECK(ctx);
    if (err) return err;
    rc = pqh_encode_place_dev_ld(ctx, tables, d_codes, ldc, n, prev, rawf, d_offsets, d_out,
                                 out_bytes, chunk_vectors, d_chunk_offsets, d_chunk_prev,
                                 sc.len_send);
    if (rc) return rc;
    if (raw_first_out) {   // (optional: the one host read, at the end)
        int rf = rank == 0 ? 1 : 0;
        if (context) {
            PQH_HIP(ctx, hipMemcpyAsync(&rf, sc.rawf, 4, hipMemcpyDeviceToHost, ctx->stream));
            PQH_HIP(ctx, hipStreamSynchronize(ctx->stream));
        }
        *raw_first_out = rf;
    }
    return PQH_OK;
}

int pqh_shard_encode_write(pqh_ctx_t* ctx, const pqh_shard_comm_t* comm, const block_t* shard,
                           const void* d_codes, int m, int k, int context, pqh_tables_t* tables,
                           unsigned char* d_out, unsigned long long out_bytes, int chunk_vectors,
                           unsigned long long* d_chunk_offsets, void* d_chunk_prev,
                           unsigned long long* d_offsets, void* d_scratch, int status,
                           int* raw_first_out) {
    return shard_write_impl(ctx, comm, shard, d_codes, 0, m, k, context, tables, d_out, out_bytes,
                            chunk_vectors, d_chunk_offsets, d_chunk_prev, d_offsets, d_scratch,
                            status, raw_first_out);
}

int pqh_shard_encode_write_parts(pqh_ctx_t* ctx, const pqh_shard_comm_t* comm,
                                 const block_t* shard, const void* d_codes, long long ld_codes,
                                 int m, int k, int context, pqh_tables_t* tables,
                                 unsigned char* d_out, unsigned long long out_bytes,
                                 int chunk_vectors, unsigned long long* d_chunk_offsets,
                                 void* d_chunk_prev, unsigned long long* d_offsets, void* d_scratch,
                                 int status, int* raw_first_out) {
    if (ld_codes <= 0) return PQH_ERR_ARG;
    return shard_write_impl(ctx, comm, shard, d_codes, ld_codes, m, k, context, tables, d_out,
                            out_bytes, chunk_vectors, d_chunk_offsets, d_chunk_prev, d_offsets,
                            d_scratch, status, raw_first_out);
}

int pqh_shard_encode(pqh_ctx_t* ctx, const pqh_shard_comm_t* comm, const block_t* shard,
                     const void* d_codes, int m, int k, int context, pqh_tables_t* tables,
                     uint32_t* d_counts, unsigned char* d_out, unsigned long long out_bytes,
                     int chunk_vectors, unsigned long long* d_chunk_offsets, void* d_chunk_prev,
                     unsigned long long* d_offsets, void* d_scratch, int* raw_first_out) {
    if (shard_fatal(ctx, comm, m, k, context, d_scratch) || !d_counts || !d_offsets)
        return PQH_ERR_ARG;
    const int rc1 = pqh_shard_encode_tables(ctx, comm, shard, d_codes, m, k, context, tables,
                                            d_counts, d_scratch);
    // (a failed collective hook leaves the sequence unfinishable: phase 2 is not attempted)
    if (rc1 == PQH_ERR_COMM) return rc1;
    const int rc2 = pqh_shard_encode_write(ctx, comm, shard, d_codes, m, k, context, tables, d_out,
                                           out_bytes, chunk_vectors, d_chunk_offsets, d_chunk_prev,
                                           d_offsets, d_scratch, rc1, raw_first_out);
    return rc1 ? rc1 : rc2;
}

int pqh_shard_status(pqh_ctx_t* ctx, const unsigned long long* d_offsets) {
    if (!ctx || !d_offsets) return PQH_ERR_ARG;
    int rc = pqh_use_device(ctx);
    if (rc) return rc;
    unsigned long long total = 0;
    PQH_HIP(ctx, hipMemcpyAsync(&total, d_offsets + 1, 8, hipMemcpyDeviceToHost, ctx->stream));
    PQH_HIP(ctx, hipStreamSynchronize(ctx->stream));
    return total == ~0ull ? pqh_set_error(ctx, PQH_ERR_REMOTE, "a rank's shard encode failed")
                          : PQH_OK;
}

}  // extern "C"
