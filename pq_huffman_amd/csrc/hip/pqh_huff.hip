// pqh_huff.hip -- symbol histograms, Huffman stream encode and chunked decode on gfx950.
//
//  hist_ctx / hist_plain   huffman_encoder.c:139-205 (collect_*_stats)
//  enc_size + scan         code-length pass: per 256-vector block bit totals, then an
//                          exclusive scan -> every block's bit offset (the serial bit
//                          cursor of bitstream.c:71-101 made parallel)
//  enc_write               encode_*_data (huffman_encoder.c:207-238): each block scans its
//                          per-vector lengths in LDS, ORs its codes into an LDS image of
//                          its bit range, stores interior words and ORs its two edge words
// (code tables and decode: pqh_tables.hip)
// Stream words are assembled MSB-first in 32-bit registers and byte-swapped on store, so
// memory holds exactly the bytes bitstream.c writes.
#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <thread>
#include <vector>

#include "pqh_internal.h"

namespace {

constexpr int kEncBlock = 256;   // vectors per encode workgroup (one thread each)
constexpr int kMaxCodeLen = 56;
constexpr int kHistChunk = 32768; // vectors per context-histogram workgroup (< 65536)

template <typename CodeT>
__device__ __forceinline__ unsigned ld_code(const CodeT* c, long long i) { return (unsigned)c[i]; }

// ---------------------------------------------------------------- histograms
template <typename CodeT>
__global__ void __launch_bounds__(1024)
hist_ctx(const CodeT* __restrict__ codes, long long n, int m_total, int k,
         const CodeT* __restrict__ prev_row, uint32_t* __restrict__ counts) {
    extern __shared__ uint32_t pairs[];   // k*k u16 counters packed two per word
    const int m = blockIdx.y;
    const int words = (k * k + 1) / 2;
    for (int w = threadIdx.x; w < words; w += blockDim.x) pairs[w] = 0;
    __syncthreads();
    const long long v0 = (long long)blockIdx.x * kHistChunk;
    const long long v1 = min(n, v0 + kHistChunk);
    for (long long v = v0 + threadIdx.x; v < v1; v += blockDim.x) {
        unsigned prev;
        if (v > 0) prev = ld_code(codes, (v - 1) * m_total + m);
        else if (prev_row) prev = ld_code(prev_row, m);
        else continue;
        const unsigned cur = ld_code(codes, v * m_total + m);
        if (prev >= (unsigned)k || cur >= (unsigned)k) continue;  // out-of-alphabet codes
        const unsigned bin = prev * (unsigned)k + cur;
        atomicAdd(&pairs[bin >> 1], 1u << ((bin & 1u) * 16));
    }
    __syncthreads();
    uint32_t* out = counts + (long long)m * k * k;
    for (int w = threadIdx.x; w < words; w += blockDim.x) {
        const uint32_t c = pairs[w];
        if (c & 0xFFFFu) atomicAdd(&out[2 * w], c & 0xFFFFu);
        if (c >> 16) atomicAdd(&out[2 * w + 1], c >> 16);
    }
}

template <typename CodeT>
__global__ void __launch_bounds__(256)
hist_plain(const CodeT* __restrict__ codes, long long n, int m_total, int k,
           uint32_t* __restrict__ counts) {
    extern __shared__ uint32_t bins[];
    const int m = blockIdx.y;
    for (int i = threadIdx.x; i < k; i += blockDim.x) bins[i] = 0;
    __syncthreads();
    const long long per = (n + gridDim.x - 1) / gridDim.x;
    const long long v0 = (long long)blockIdx.x * per, v1 = min(n, v0 + per);
    for (long long v = v0 + threadIdx.x; v < v1; v += blockDim.x) {
        const unsigned c = ld_code(codes, v * m_total + m);
        if (c < (unsigned)k) atomicAdd(&bins[c], 1u);
    }
    __syncthreads();
    for (int i = threadIdx.x; i < k; i += blockDim.x)
        if (bins[i]) atomicAdd(&counts[(long long)m * k + i], bins[i]);
}

// ---------------------------------------------------------------- encode
// one symbol's (code, len): context row 0 of the stream is raw 8 bits (huffman_encoder.c:234)
template <typename CodeT>
__device__ __forceinline__ unsigned long long sym_entry(const CodeT* codes, long long v, int i,
                                                        int m_total, int k, int context,
                                                        int raw_first, const CodeT* prev_row,
                                                        const unsigned long long* enc,
                                                        long long items) {
    const unsigned s = ld_code(codes, v * m_total + i);
    if (s >= (unsigned)k) return 0;  // out-of-alphabet symbol: no code (length 0)
    if (!context) return enc[(long long)i * items + s];
    unsigned prev;
    if (v > 0) {
        prev = ld_code(codes, (v - 1) * m_total + i);
    } else if (!raw_first && prev_row) {
        prev = ld_code(prev_row, i);
    } else {
        return (8ull << 56) | (s & 0xFFu);
    }
    if (prev >= (unsigned)k) return 0;
    return enc[(long long)i * items + (long long)prev * k + s];
}

template <typename CodeT>
__global__ void __launch_bounds__(kEncBlock)
enc_size(const CodeT* __restrict__ codes, long long n, int m_total, int k, int context,
         int raw_first, const CodeT* __restrict__ prev_row, const unsigned long long* __restrict__ enc,
         long long items, uint32_t* __restrict__ block_bits) {
    __shared__ uint32_t red[kEncBlock / 64];
    const long long v = (long long)blockIdx.x * kEncBlock + threadIdx.x;
    uint32_t bits = 0;
    if (v < n)
        for (int i = 0; i < m_total; ++i)
            bits += (uint32_t)(sym_entry(codes, v, i, m_total, k, context, raw_first, prev_row,
                                         enc, items) >> 56);
    for (int off = 32; off >= 1; off >>= 1) bits += __shfl_xor(bits, off);
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = bits;
    __syncthreads();
    if (threadIdx.x == 0) {
        uint32_t s = 0;
        for (int w = 0; w < kEncBlock / 64; ++w) s += red[w];
        block_bits[blockIdx.x] = s;
    }
}

// exclusive scan of nb block totals by one workgroup (nb ~ n/256)
__global__ void __launch_bounds__(1024)
scan_blocks(const uint32_t* __restrict__ block_bits, long long nb,
            unsigned long long* __restrict__ block_off, unsigned long long* __restrict__ total) {
    __shared__ unsigned long long wsum[16];
    __shared__ unsigned long long carry;
    if (threadIdx.x == 0) carry = 0;
    __syncthreads();
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    for (long long base = 0; base < nb; base += blockDim.x) {
        const long long i = base + threadIdx.x;
        unsigned long long x = i < nb ? block_bits[i] : 0;
        unsigned long long incl = x;
        for (int off = 1; off < 64; off <<= 1) {
            unsigned long long y = __shfl_up(incl, off);
            if (lane >= off) incl += y;
        }
        if (lane == 63) wsum[wid] = incl;
        __syncthreads();
        unsigned long long before = carry;
        for (int w = 0; w < wid; ++w) before += wsum[w];
        if (i < nb) block_off[i] = before + incl - x;
        __syncthreads();
        if (threadIdx.x == blockDim.x - 1) carry = before + incl;
        __syncthreads();
    }
    if (threadIdx.x == 0) *total = carry;
}

__device__ __forceinline__ uint32_t bswap32(uint32_t x) { return __builtin_bswap32(x); }

template <typename CodeT>
__global__ void __launch_bounds__(kEncBlock)
enc_write(const CodeT* __restrict__ codes, long long n, int m_total, int k, int context,
          int raw_first, const CodeT* __restrict__ prev_row, const unsigned long long* __restrict__ enc,
          long long items, const unsigned long long* __restrict__ block_off,
          const uint32_t* __restrict__ block_bits, unsigned long long bit_offset,
          uint32_t* __restrict__ out_words, long long out_words_cap, int chunk_vectors,
          unsigned long long* __restrict__ chunk_off, CodeT* __restrict__ chunk_prev,
          unsigned long long* __restrict__ err) {
    extern __shared__ uint32_t img[];   // LDS image of this block's bit range
    __shared__ uint32_t wsum[kEncBlock / 64];
    const long long v = (long long)blockIdx.x * kEncBlock + threadIdx.x;
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    const unsigned long long b0 = bit_offset + block_off[blockIdx.x];
    const unsigned long long b1 = b0 + block_bits[blockIdx.x];
    const long long w0 = (long long)(b0 >> 5);
    const long long nwords = b1 > b0 ? (long long)((b1 - 1) >> 5) - w0 + 1 : 0;
    for (long long w = threadIdx.x; w < nwords; w += blockDim.x) img[w] = 0;

    uint32_t bits = 0;
    if (v < n)
        for (int i = 0; i < m_total; ++i)
            bits += (uint32_t)(sym_entry(codes, v, i, m_total, k, context, raw_first, prev_row,
                                         enc, items) >> 56);
    uint32_t incl = bits;
    for (int off = 1; off < 64; off <<= 1) {
        uint32_t y = __shfl_up(incl, off);
        if (lane >= off) incl += y;
    }
    if (lane == 63) wsum[wid] = incl;
    __syncthreads();
    uint32_t before = 0;
    for (int w = 0; w < wid; ++w) before += wsum[w];
    unsigned long long pos = b0 + before + incl - bits;

    if (v < n) {
        if (chunk_vectors > 0 && v % chunk_vectors == 0) {
            const long long j = v / chunk_vectors;
            chunk_off[j] = pos;
            if (context && chunk_prev)
                for (int i = 0; i < m_total; ++i)
                    chunk_prev[j * m_total + i] =
                        v > 0 ? codes[(v - 1) * m_total + i] : (prev_row ? prev_row[i] : (CodeT)0);
        }
        for (int i = 0; i < m_total; ++i) {
            const unsigned long long e = sym_entry(codes, v, i, m_total, k, context, raw_first,
                                                   prev_row, enc, items);
            int len = (int)(e >> 56);
            const unsigned long long code = e & ((1ull << 56) - 1);
            while (len > 0) {
                const int o = (int)(pos & 31);
                const int take = min(len, 32 - o);
                const uint32_t piece = (uint32_t)((code >> (len - take)) & ((1ull << take) - 1));
                atomicOr(&img[(long long)(pos >> 5) - w0], piece << (32 - o - take));
                pos += take;
                len -= take;
            }
        }
    }
    __syncthreads();
    if (w0 + nwords > out_words_cap) {   // caller's buffer too small: write nothing, flag
        if (threadIdx.x == 0) atomicOr(err, 2ull);
        return;
    }
    for (long long w = threadIdx.x; w < nwords; w += blockDim.x) {
        const uint32_t val = bswap32(img[w]);
        if (w == 0 || w == nwords - 1) {
            if (val) atomicOr(&out_words[w0 + w], val);
        } else {
            out_words[w0 + w] = val;
        }
    }
}

}  // namespace

extern "C" {

int pqh_histogram(pqh_ctx_t* ctx, const void* d_codes, long long n, int m, int k, int context,
                  const void* d_prev_row, uint32_t* d_counts) {
    if (!ctx || m <= 0 || k <= 0 || n < 0 || !d_counts || (n > 0 && !d_codes)) return PQH_ERR_ARG;
    if (context && k > 256) return PQH_ERR_UNSUPPORTED;
    int rc = pqh_use_device(ctx);
    if (rc) return rc;
    if (n == 0) return PQH_OK;
    if (context) {
        const unsigned chunks = (unsigned)((n + kHistChunk - 1) / kHistChunk);
        const size_t lds = (size_t)((k * k + 1) / 2) * 4;
        PQH_HIP(ctx, hipFuncSetAttribute((const void*)hist_ctx<uint8_t>,
                                         hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
        hipLaunchKernelGGL(hist_ctx<uint8_t>, dim3(chunks, m), dim3(1024), lds, ctx->stream,
                           static_cast<const uint8_t*>(d_codes), n, m, k,
                           static_cast<const uint8_t*>(d_prev_row), d_counts);
    } else {
        const unsigned blocks = (unsigned)std::min<long long>((n + 4095) / 4096, 512);
        if (k <= 256)
            hipLaunchKernelGGL(hist_plain<uint8_t>, dim3(blocks, m), dim3(256), k * 4, ctx->stream,
                               static_cast<const uint8_t*>(d_codes), n, m, k, d_counts);
        else
            hipLaunchKernelGGL(hist_plain<uint16_t>, dim3(blocks, m), dim3(256), k * 4, ctx->stream,
                               static_cast<const uint16_t*>(d_codes), n, m, k, d_counts);
    }
    PQH_LAUNCH_CHECK(ctx);
    return PQH_OK;
}

// workspace layout for encode: [block_bits u32 nb][pad][block_off u64 nb]
static int enc_ws(pqh_ctx* ctx, long long n, uint32_t** bb, unsigned long long** bo) {
    const long long nb = (n + kEncBlock - 1) / kEncBlock;
    const size_t a = ((size_t)nb * 4 + 255) & ~(size_t)255;
    int rc = pqh_ensure_ws(ctx, a + (size_t)nb * 8 + 256);
    if (rc) return rc;
    *bb = static_cast<uint32_t*>(ctx->ws);
    *bo = reinterpret_cast<unsigned long long*>(static_cast<char*>(ctx->ws) + a);
    return PQH_OK;
}

static int run_size(pqh_ctx* ctx, const pqh_tables* t, const void* d_codes, long long n,
                    int raw_first, const void* d_prev_row, unsigned long long* d_total) {
    uint32_t* bb;
    unsigned long long* bo;
    int rc = enc_ws(ctx, n, &bb, &bo);
    if (rc) return rc;
    const long long nb = (n + kEncBlock - 1) / kEncBlock;
    if (t->k <= 256)
        hipLaunchKernelGGL(enc_size<uint8_t>, dim3((unsigned)nb), dim3(kEncBlock), 0, ctx->stream,
                           static_cast<const uint8_t*>(d_codes), n, t->m, t->k, t->context,
                           raw_first, static_cast<const uint8_t*>(d_prev_row), t->d_enc, t->items, bb);
    else
        hipLaunchKernelGGL(enc_size<uint16_t>, dim3((unsigned)nb), dim3(kEncBlock), 0, ctx->stream,
                           static_cast<const uint16_t*>(d_codes), n, t->m, t->k, t->context,
                           raw_first, static_cast<const uint16_t*>(d_prev_row), t->d_enc, t->items, bb);
    PQH_LAUNCH_CHECK(ctx);
    hipLaunchKernelGGL(scan_blocks, dim3(1), dim3(1024), 0, ctx->stream, bb, nb, bo, d_total);
    PQH_LAUNCH_CHECK(ctx);
    ctx->enc_key = {d_codes, n, t, raw_first, d_prev_row};
    return PQH_OK;
}

int pqh_encode_size(pqh_ctx_t* ctx, const pqh_tables_t* t, const void* d_codes, long long n,
                    int raw_first, const void* d_prev_row, unsigned long long* d_total_bits) {
    if (!ctx || !t || n < 0 || !d_total_bits || (n > 0 && !d_codes)) return PQH_ERR_ARG;
    int rc = pqh_use_device(ctx);
    if (rc) return rc;
    if (n == 0) {
        PQH_HIP(ctx, hipMemsetAsync(d_total_bits, 0, 8, ctx->stream));
        return PQH_OK;
    }
    return run_size(ctx, t, d_codes, n, raw_first, d_prev_row, d_total_bits);
}

int pqh_encode_write(pqh_ctx_t* ctx, const pqh_tables_t* t, const void* d_codes, long long n,
                     int raw_first, const void* d_prev_row, unsigned long long bit_offset,
                     unsigned char* d_out, unsigned long long out_bytes, int chunk_vectors,
                     unsigned long long* d_chunk_offsets, void* d_chunk_prev) {
    if (!ctx || !t || n < 0 || (n > 0 && (!d_codes || !d_out))) return PQH_ERR_ARG;
    if ((reinterpret_cast<uintptr_t>(d_out) & 3u) || (out_bytes & 3u))
        return pqh_set_error(ctx, PQH_ERR_ARG, "stream buffer must be 4-byte aligned and sized");
    if (chunk_vectors > 0 && !d_chunk_offsets) return PQH_ERR_ARG;
    int rc = pqh_use_device(ctx);
    if (rc) return rc;
    if (n == 0) return PQH_OK;
    const pqh_enc_key& key = ctx->enc_key;
    if (key.codes != d_codes || key.n != n || key.t != t || key.raw_first != raw_first ||
        key.prev != d_prev_row) {
        rc = run_size(ctx, t, d_codes, n, raw_first, d_prev_row, ctx->d_diag + 3);
        if (rc) return rc;
    }
    uint32_t* bb;
    unsigned long long* bo;
    rc = enc_ws(ctx, n, &bb, &bo);
    if (rc) return rc;
    const long long nb = (n + kEncBlock - 1) / kEncBlock;
    const size_t lds = ((size_t)kEncBlock * t->m * kMaxCodeLen / 32 + 4) * 4;
    if (lds > 64 * 1024) return PQH_ERR_UNSUPPORTED;
    uint32_t* words = reinterpret_cast<uint32_t*>(d_out);
    if (t->k <= 256)
        hipLaunchKernelGGL(enc_write<uint8_t>, dim3((unsigned)nb), dim3(kEncBlock), lds, ctx->stream,
                           static_cast<const uint8_t*>(d_codes), n, t->m, t->k, t->context,
                           raw_first, static_cast<const uint8_t*>(d_prev_row), t->d_enc, t->items, bo,
                           bb, bit_offset, words, (long long)(out_bytes / 4), chunk_vectors,
                           d_chunk_offsets, static_cast<uint8_t*>(d_chunk_prev), ctx->d_diag + 2);
    else
        hipLaunchKernelGGL(enc_write<uint16_t>, dim3((unsigned)nb), dim3(kEncBlock), lds, ctx->stream,
                           static_cast<const uint16_t*>(d_codes), n, t->m, t->k, t->context,
                           raw_first, static_cast<const uint16_t*>(d_prev_row), t->d_enc, t->items, bo,
                           bb, bit_offset, words, (long long)(out_bytes / 4), chunk_vectors,
                           d_chunk_offsets, static_cast<uint16_t*>(d_chunk_prev), ctx->d_diag + 2);
    PQH_LAUNCH_CHECK(ctx);
    return PQH_OK;
}

int pqh_encode_status(pqh_ctx_t* ctx) {
    unsigned long long e = 0;
    PQH_HIP(ctx, hipMemcpyAsync(&e, ctx->d_diag + 2, 8, hipMemcpyDeviceToHost, ctx->stream));
    PQH_HIP(ctx, hipStreamSynchronize(ctx->stream));
    PQH_HIP(ctx, hipMemsetAsync(ctx->d_diag + 2, 0, 8, ctx->stream));
    return e ? pqh_set_error(ctx, PQH_ERR_CAPACITY, "stream buffer too small") : PQH_OK;
}

int pqh_codebooks_build(const double* counts, int m, int k, int context,
                        huffman_codebook_t* codebooks, int num_threads) {
    if (!counts || m <= 0 || k <= 0 || !codebooks) return PQH_ERR_ARG;
    const long long items = context ? (long long)k * k : k;
    auto work = [&](int i) {
        if (context) huffman_codebook_context_encode_init(&codebooks[i], k, counts + i * items);
        else huffman_codebook_encode_init(&codebooks[i], k, counts + i * items);
    };
    if (num_threads <= 1 || m == 1) {
        for (int i = 0; i < m; ++i) work(i);
        return PQH_OK;
    }
    std::vector<std::thread> pool;
    const int nt = std::min(num_threads, m);
    for (int w = 0; w < nt; ++w)
        pool.emplace_back([&, w] {
            for (int i = w; i < m; i += nt) work(i);
        });
    for (auto& th : pool) th.join();
    return PQH_OK;
}

}  // extern "C"
