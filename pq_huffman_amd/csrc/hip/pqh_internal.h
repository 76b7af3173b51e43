// pqh_internal.h -- shared internals of the pq_huffman_amd GPU library (not installed).
#pragma once

#include <hip/hip_runtime.h>

#include <cstdarg>
#include <cstdint>
#include <cstdio>

#include "pqh.h"

// The kernels are written for gfx950 (CDNA4) only: wave64 DPP controls that exist only on
// GFX9/CDNA (row_bcast:15/31, wave_shr:1 in the scans, the encoder's look-back and the wave
// histogram), v_permlane32_swap, the 32x32x16 bf16 MFMA.  A device pass for any other target
// stops here instead of miscompiling.
#if defined(__HIP_DEVICE_COMPILE__) && !defined(__gfx950__)
#error "pq_huffman_amd device code targets gfx950 only (--offload-arch=gfx950)"
#endif

struct pqh_tables;

struct pqh_ctx {
    int device = 0;
    int num_cus = 256;
    hipStream_t stream = nullptr;
    bool own_stream = false;
    char err[512] = {0};
    // grow-only scratch (stream ordered use, allocated outside timed regions)
    void* ws = nullptr;
    size_t ws_bytes = 0;
    // [0] / [4] re-rank counters of alternate assignment launches, [1] decode error,
    // [2] encode capacity error, [3] scratch total bits, [6] re-rank count of the exact path,
    // [7] tree-order id error
    unsigned long long* d_diag = nullptr;
    // one-pass encoder look-back state: [lb_cap] block states, [lb_cap] tails, ticket
    unsigned long long* lb_state = nullptr;
    long long lb_cap = 0;
    unsigned lb_epoch = 0;
    unsigned long long lb_ticket_base = 0;
    // work-queue heads of the assignment kernel: kXcds per subspace, kSchedStride words
    // apart; two sets used by alternate launches, each launch zeroing the other set (and the
    // other re-rank counter, d_diag[0] / d_diag[4]) for the next one -- no memset dispatches
    uint32_t* d_sched = nullptr;
    unsigned long long assign_launches = 0;
    // radix sort look-back state: [sort_cap * 256] per-(block, digit) status words, ticket
    unsigned long long* sort_state = nullptr;
    long long sort_cap = 0;
    unsigned sort_epoch = 0;
    unsigned long long sort_ticket_base = 0;
    int rerank_slot = 0;              // d_diag slot of the last assignment's re-rank count
    // pqh_ctx_set_tuning (0: the library / environment default)
    double tune_wgs_per_cu = 0.0;
    int tune_hist_split = 0;
    int tune_hist_block = 0;
    int tune_enc_impl = 0;   // 1 tiled, 2 one-pass (0: PQH_ENC_IMPL or tiled)
    // the tiled encoder's scratch: one worst-case slot per tile (grow-only)
    void* enc_scr = nullptr;
    size_t enc_scr_bytes = 0;
};
constexpr int kSchedMax = 64;      // subspaces with a work queue (more: static schedule)
constexpr int kXcds = 8;
constexpr int kSchedStride = 64;   // u32 words = 256 B
constexpr long long kSchedSet = (long long)kSchedMax * kXcds * kSchedStride;   // words per set

int pqh_set_error(pqh_ctx* ctx, int code, const char* fmt, ...);
int pqh_ensure_ws(pqh_ctx* ctx, size_t bytes);
int pqh_ensure_enc_scratch(pqh_ctx* ctx, size_t bytes);
int pqh_use_device(pqh_ctx* ctx);
int pqh_kmeans_fixed_shift(float max_abs, long long n);
// k-means iteration pieces (pqh_kmeans.hip), shared by the one-shot and the streamed trainers
int pqh_kmeans_absmax_launch(pqh_ctx* ctx, const float* d_x, long long n, long long ld_x, int d,
                             unsigned* d_max);
int pqh_kmeans_accum_launch(pqh_ctx* ctx, const float* d_x, long long n, long long ld_x, int m,
                            int k, int dsub, const void* d_codes, int s, long long* d_sums,
                            unsigned long long* d_cnt);
int pqh_kmeans_update_launch(pqh_ctx* ctx, const long long* d_sums, const unsigned long long* d_cnt,
                             long long cells, int dsub, int s, float* d_cent);
// the error pass over n rows, its 256-row block partials added to *sum in row order (so a
// caller streaming chunks of a multiple of 256 rows gets pqh_pq_error's sum bit for bit)
int pqh_pq_error_accum(pqh_ctx* ctx, const pqh_pq_t* pq, const float* d_x, long long n,
                       long long ld_x, const void* d_codes, double* sum);
// pqh_shard_encode's histogram / size / write with this shard's raw-first flag in device
// memory (1: row 0 raw, no halo pair; 0: row 0 in the context of d_prev_row) -- pqh_huff.hip
extern "C" {
int pqh_histogram_set_dev(pqh_ctx_t* ctx, const void* d_codes, long long n, int m, int k,
                          const void* d_prev_row, const int* d_rawf, uint32_t* d_counts);
// the same with codes row-major (ldc = 0) or part-major (part i at d_codes + i * ldc)
int pqh_histogram_set_dev_ld(pqh_ctx_t* ctx, const void* d_codes, long long ldc, long long n,
                             int m, int k, const void* d_prev_row, const int* d_rawf,
                             uint32_t* d_counts);
int pqh_encode_write_at_dev_ld(pqh_ctx_t* ctx, const pqh_tables_t* t, const void* d_codes,
                               long long ldc, long long n, const void* d_prev_row,
                               const int* d_rawf, const unsigned long long* d_global_bit_offset,
                               unsigned char* d_out, unsigned long long out_bytes,
                               int chunk_vectors, unsigned long long* d_chunk_offsets,
                               void* d_chunk_prev);
// its two halves (tiled encoder): the tiles and the exact length, then the placement at the
// device offset (pqh_shard_encode_write runs the length all-gather between them)
int pqh_encode_tiles_dev_ld(pqh_ctx_t* ctx, const pqh_tables_t* t, const void* d_codes,
                            long long ldc, long long n, const void* d_prev_row, const int* d_rawf,
                            int chunk_vectors, unsigned long long* d_chunk_offsets,
                            void* d_chunk_prev, unsigned long long* d_total_bits);
int pqh_encode_place_dev_ld(pqh_ctx_t* ctx, const pqh_tables_t* t, const void* d_codes,
                            long long ldc, long long n, const void* d_prev_row, const int* d_rawf,
                            const unsigned long long* d_global_bit_offset, unsigned char* d_out,
                            unsigned long long out_bytes, int chunk_vectors,
                            unsigned long long* d_chunk_offsets, void* d_chunk_prev,
                            unsigned long long* d_total_bits);
int pqh_encode_size_dev(pqh_ctx_t* ctx, const pqh_tables_t* t, const void* d_codes, long long n,
                        const void* d_prev_row, const int* d_rawf,
                        unsigned long long* d_total_bits);
int pqh_encode_write_at_dev(pqh_ctx_t* ctx, const pqh_tables_t* t, const void* d_codes,
                            long long n, const void* d_prev_row, const int* d_rawf,
                            const unsigned long long* d_global_bit_offset, unsigned char* d_out,
                            unsigned long long out_bytes, int chunk_vectors,
                            unsigned long long* d_chunk_offsets, void* d_chunk_prev);
}

#define PQH_HIP(ctx, expr)                                                                \
    do {                                                                                  \
        hipError_t _e = (expr);                                                           \
        if (_e != hipSuccess)                                                             \
            return pqh_set_error((ctx), PQH_ERR_HIP, "%s:%d %s: %s", __FILE__, __LINE__,  \
                                 #expr, hipGetErrorString(_e));                          \
    } while (0)

// Wave issue priority of a kernel (s_setprio takes an immediate): the latency-bound kernels
// that run beside the assignment grid raise theirs.  pqh_prio(name, default) reads the
// PQH_PRIO_<NAME> override (0..3) -- an experiment knob; the defaults are the measured best.
int pqh_prio(const char* name, int def);
__device__ __forceinline__ void pqh_set_prio(int p) {
    switch (p) {
        case 1: __builtin_amdgcn_s_setprio(1); break;
        case 2: __builtin_amdgcn_s_setprio(2); break;
        case 3: __builtin_amdgcn_s_setprio(3); break;
        default: break;
    }
}

// A workgroup barrier that orders this wave's LDS accesses (atomics, stores, reads) before
// every other wave's accesses after it.  The explicit lgkmcnt(0) matters: the compiler has
// been seen to emit a bare s_barrier after LDS atomics whose results are unused (a histogram
// lost counts that way), so every barrier that hands LDS data between waves uses this.
__device__ __forceinline__ void lds_barrier() {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __syncthreads();
}

// PQH_DEBUG_SYNC=1: synchronise and check after every launch, so an asynchronous fault is
// reported by the call that caused it (diagnostics only).
// the u16 gather entry of a u64 code-table entry (enc16 above)
__device__ __forceinline__ uint16_t pqh_enc16_of(unsigned long long e) {
    const unsigned len = (unsigned)(e >> 56);
    return len == 0 ? (uint16_t)0 : len <= 12 ? (uint16_t)((len << 12) | (unsigned)(e & 0xFFFu))
                                              : (uint16_t)0xFFFFu;
}

bool pqh_debug_sync();
#define PQH_LAUNCH_CHECK(ctx)                                                             \
    do {                                                                                  \
        PQH_HIP(ctx, hipGetLastError());                                                  \
        if (pqh_debug_sync()) PQH_HIP(ctx, hipStreamSynchronize((ctx)->stream));          \
    } while (0)

// Device-side code tables shared by the encode and decode kernels (pqh_tables.hip).
//   enc [m][items] u64: (len << 56) | code (right-aligned, len <= 56; 0 = no code)
//   enc32 [m][items] u32: the same entry as len << 26 | code when len <= 26, else ~0u
//   enc16 [m][items] u16: len << 12 | code when 1 <= len <= 12, 0 (no code), else 0xFFFF
//   Decode: two-level lookup per alphabet (tables = m * roots, roots = K in context mode)
//   lut1 [tables][1 << l1_bits] u16 (rows packed at the table set's own W1 = l1_bits, for
//        every alphabet): (len << 12) | sym for 1 <= len <= W1 (replicated);
//        (15 << 12) | sub = a longer code, subtable `sub` of this alphabet; 0 = invalid
//   meta [tables] u32: l2base << 9 | noL2 << 8 | w2 << 4 | W1 -- the alphabet's subtables
//        are 2^w2-entry blocks at lut2[l2base + (sub << w2)] holding (len2 << 12) | sym,
//        15 << 12 = even longer (linear search in longs), 0 = invalid
//   longs [tables][k] {code, len, sym}, long_cnt [tables]: codes beyond both levels
struct pqh_long_code {
    unsigned long long code;
    uint32_t len;
    uint32_t sym;
};

struct pqh_tables {
    pqh_ctx* ctx = nullptr;
    int m = 0, k = 0, context = 0, roots = 1, l1_bits = 9, l2_bits = 8;
    long long items = 0, tables = 0;
    long long lut2_cap = 0;
    unsigned long long* d_enc = nullptr;
    uint32_t* d_enc32 = nullptr;     // [m][items] len << 26 | code (len <= 26), else ~0u
    // [m][items] the encoder's first gather: len << 12 | code for 1 <= len <= 12, 0 = no code,
    // 0xFFFF = longer (read d_enc32) -- half the bytes of d_enc32, so the context tables of
    // a 16-part set (2 MB) stay in an XCD's 4 MB L2 beside the streams that pass through it
    uint16_t* d_enc16 = nullptr;
    bool enc32_by_trees = false;     // the last tree build wrote d_enc32 (the LUT build skips it)
                                     // (escape: read d_enc) -- the encoder's gather table
    uint16_t* d_lut1 = nullptr;
    uint16_t* d_lut2 = nullptr;
    uint32_t* d_meta = nullptr;
    pqh_long_code* d_long = nullptr;
    uint32_t* d_long_cnt = nullptr;
    // [0] error word (sticky until pqh_tables_status); [2..3] / [4..5] two LUT pool heads
    // (u64): a decode-table build allocates from slot pool_slot and zeroes the other slot for
    // the next build (its own was zeroed by the build before it, by its tree kernel, or at
    // allocation)
    uint32_t* d_err = nullptr;
    int pool_slot = 0;
};
