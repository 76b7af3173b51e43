// pqh_sort.hip -- the default sort mode of the reference encoder on the GPU.
//
// huffman_encoder.c:301-317 sorts the N code rows with qsort and a strncmp comparator over
// the M bytes of a row (glibc's qsort is a merge sort here, so the order is stable).
// strncmp stops at the first 0 byte, so the order is exactly a stable sort by
//     key(row) = the row's bytes, every byte after its first 0 cleared,
// compared as an unsigned big-endian byte string (verified by the oracle's
// orc_sort_rows against reference-built fixtures).
//
// GPU: LSD over 8-byte key chunks, least significant chunk first.  Each pass builds the
// chunk's big-endian u64 key for every row (through the current permutation) and runs a
// stable radix sort of (key, row index) pairs (rocPRIM onesweep radix sort -- a library
// primitive, like a plain GEMM); stability of every pass makes the composition a stable
// sort by the whole key.  A final gather permutes the rows.  M = 8: one pass.
#include <rocprim/device/device_radix_sort.hpp>

#include "pqh_internal.h"

namespace {

// key chunk c of row idx[v] (bytes 8c .. 8c+7, big-endian, zeroed after the row's first 0)
__global__ void __launch_bounds__(256)
sort_keys(const uint8_t* __restrict__ codes, long long n, int m, int c,
          const uint32_t* __restrict__ idx, unsigned long long* __restrict__ keys) {
    const long long v = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (v >= n) return;
    const uint8_t* row = codes + (long long)(idx ? idx[v] : v) * m;
    int z = m;   // first zero byte
    for (int j = 0; j < m; ++j)
        if (row[j] == 0) {
            z = j;
            break;
        }
    unsigned long long key = 0;
#pragma unroll
    for (int q = 0; q < 8; ++q) {
        const int j = 8 * c + q;
        const unsigned long long b = (j < m && j <= z) ? row[j] : 0u;
        key |= b << (56 - 8 * q);
    }
    keys[v] = key;
}

__global__ void __launch_bounds__(256)
iota_u32(uint32_t* __restrict__ a, long long n) {
    const long long v = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (v < n) a[v] = (uint32_t)v;
}

__global__ void __launch_bounds__(256)
gather_rows(const uint8_t* __restrict__ src, long long n, int m, const uint32_t* __restrict__ idx,
            uint8_t* __restrict__ dst) {
    const long long v = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (v >= n) return;
    const uint8_t* a = src + (long long)idx[v] * m;
    uint8_t* b = dst + v * m;
    if ((m & 7) == 0) {
        for (int j = 0; j < m; j += 8)
            *reinterpret_cast<unsigned long long*>(b + j) =
                *reinterpret_cast<const unsigned long long*>(a + j);
    } else {
        for (int j = 0; j < m; ++j) b[j] = a[j];
    }
}

}  // namespace

extern "C" {

int pqh_sort_rows(pqh_ctx_t* ctx, void* d_codes, long long n, int m, void* d_tmp) {
    if (!ctx || n < 0 || m <= 0 || (n > 0 && !d_codes)) return PQH_ERR_ARG;
    if (n >= (1ll << 32)) return pqh_set_error(ctx, PQH_ERR_UNSUPPORTED, "sort: n >= 2^32 rows");
    int rc = pqh_use_device(ctx);
    if (rc) return rc;
    if (n <= 1) return PQH_OK;
    // workspace: keys in/out (u64), index in/out (u32), rocPRIM temp, row buffer if no d_tmp
    size_t temp = 0;
    if (rocprim::radix_sort_pairs(nullptr, temp, (unsigned long long*)nullptr,
                                  (unsigned long long*)nullptr, (uint32_t*)nullptr,
                                  (uint32_t*)nullptr, (size_t)n, 0u, 64u, ctx->stream) != hipSuccess)
        return pqh_set_error(ctx, PQH_ERR_HIP, "sort: temp storage query failed");
    auto al = [](size_t x) { return (x + 255) & ~(size_t)255; };
    const size_t kb = al((size_t)n * 8), ib = al((size_t)n * 4), rb = d_tmp ? 0 : al((size_t)n * m);
    rc = pqh_ensure_ws(ctx, 2 * kb + 2 * ib + al(temp) + rb);
    if (rc) return rc;
    char* w = static_cast<char*>(ctx->ws);
    unsigned long long* k0 = reinterpret_cast<unsigned long long*>(w);
    unsigned long long* k1 = reinterpret_cast<unsigned long long*>(w + kb);
    uint32_t* i0 = reinterpret_cast<uint32_t*>(w + 2 * kb);
    uint32_t* i1 = reinterpret_cast<uint32_t*>(w + 2 * kb + ib);
    void* tmp = w + 2 * kb + 2 * ib;
    uint8_t* rows = d_tmp ? static_cast<uint8_t*>(d_tmp)
                          : reinterpret_cast<uint8_t*>(w + 2 * kb + 2 * ib + al(temp));
    const unsigned blocks = (unsigned)((n + 255) / 256);
    uint8_t* codes = static_cast<uint8_t*>(d_codes);
    hipLaunchKernelGGL(iota_u32, dim3(blocks), dim3(256), 0, ctx->stream, i0, n);
    PQH_LAUNCH_CHECK(ctx);
    const int passes = (m + 7) / 8;
    for (int c = passes - 1; c >= 0; --c) {   // least significant chunk first
        hipLaunchKernelGGL(sort_keys, dim3(blocks), dim3(256), 0, ctx->stream, codes, n, m, c, i0, k0);
        PQH_LAUNCH_CHECK(ctx);
        size_t tb = temp;
        PQH_HIP(ctx, rocprim::radix_sort_pairs(tmp, tb, k0, k1, i0, i1, (size_t)n, 0u, 64u,
                                               ctx->stream));
        std::swap(i0, i1);
    }
    hipLaunchKernelGGL(gather_rows, dim3(blocks), dim3(256), 0, ctx->stream, codes, n, m, i0, rows);
    PQH_LAUNCH_CHECK(ctx);
    PQH_HIP(ctx, hipMemcpyAsync(codes, rows, (size_t)n * m, hipMemcpyDeviceToDevice, ctx->stream));
    return PQH_OK;
}

}  // extern "C"
