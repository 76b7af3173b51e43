// pqh_kmeans.hip -- Lloyd k-means per subspace on the GPU.
//
// Replaces the training half of yael kmeans() called at pq_encoder.c:265-274 (10
// iterations).  yael is absent and its Berkeley init is time-seeded, so the build trains a
// deterministic Lloyd instead (init chosen by the caller, see pq_encoder's --seed):
//   repeat iters times:
//     code[v][i] = exact fp32 argmin (pqh_pq_assign: the oracle's assignment)
//     c[i][q] = mean of the subvectors assigned to q (an empty cluster keeps its centroid)
// The sums are accumulated in 64-bit FIXED POINT, x * 2^s rounded to an integer with
// s = 61 - ceil(log2(max|x| * n)): integer addition is exact and order independent, so the
// GPU's atomic accumulation gives the same bits on every run and equals the oracle's
// sequential restatement (oracle/pqh_oracle.c orc_kmeans).  mean = (float)(sum / count *
// 2^-s), evaluated in double.
#include <algorithm>
#include <cmath>
#include <cstring>
#include <vector>

#include "pqh_internal.h"

namespace {

__global__ void __launch_bounds__(256)
absmax_kernel(const float* __restrict__ x, long long n, long long ldx, int d,
              unsigned* __restrict__ out) {
    unsigned best = 0;   // |x| bits (non-negative floats order as unsigned)
    const long long total = n * d;
    for (long long e = (long long)blockIdx.x * blockDim.x + threadIdx.x; e < total;
         e += (long long)gridDim.x * blockDim.x) {
        const float v = x[(e / d) * ldx + e % d];
        const unsigned b = __float_as_uint(v) & 0x7FFFFFFFu;
        best = max(best, b > 0x7F800000u ? 0x7F800000u : b);   // NaN counts as inf
    }
    for (int off = 32; off >= 1; off >>= 1) best = max(best, (unsigned)__shfl_xor(best, off));
    if ((threadIdx.x & 63) == 0) atomicMax(out, best);
}

// per (block of vectors, subspace): fixed-point sums in LDS, flushed with global atomics
template <typename CodeT, bool LDS>
__global__ void __launch_bounds__(256)
kmeans_accum(const float* __restrict__ x, long long n, long long ldx, int m, int k, int dsub,
             const CodeT* __restrict__ codes, int s, long long* __restrict__ sums,
             unsigned long long* __restrict__ counts) {
    extern __shared__ __attribute__((aligned(16))) char lds[];
    long long* ls = reinterpret_cast<long long*>(lds);
    unsigned* lc = reinterpret_cast<unsigned*>(lds + (size_t)k * dsub * 8);
    const int i = blockIdx.y;
    if (LDS) {
        for (int q = threadIdx.x; q < k * dsub; q += blockDim.x) ls[q] = 0;
        for (int q = threadIdx.x; q < k; q += blockDim.x) lc[q] = 0;
        __syncthreads();
    }
    const long long per = (n + gridDim.x - 1) / gridDim.x;
    const long long v0 = (long long)blockIdx.x * per, v1 = min(n, v0 + per);
    long long* gs = sums + (long long)i * k * dsub;
    unsigned long long* gc = counts + (long long)i * k;
    for (long long v = v0 + threadIdx.x; v < v1; v += blockDim.x) {
        const int c = (int)codes[v * m + i];
        const float* xp = x + v * ldx + (long long)i * dsub;
        for (int j = 0; j < dsub; ++j) {
            const long long f = __double2ll_rn(ldexp((double)xp[j], s));
            if (LDS) atomicAdd(reinterpret_cast<unsigned long long*>(&ls[c * dsub + j]), (unsigned long long)f);
            else atomicAdd(reinterpret_cast<unsigned long long*>(&gs[(long long)c * dsub + j]), (unsigned long long)f);
        }
        if (LDS) atomicAdd(&lc[c], 1u);
        else atomicAdd(&gc[c], 1ull);
    }
    if (LDS) {
        __syncthreads();
        for (int q = threadIdx.x; q < k * dsub; q += blockDim.x)
            if (ls[q]) atomicAdd(reinterpret_cast<unsigned long long*>(&gs[q]), (unsigned long long)ls[q]);
        for (int q = threadIdx.x; q < k; q += blockDim.x)
            if (lc[q]) atomicAdd(&gc[q], (unsigned long long)lc[q]);
    }
}

__global__ void __launch_bounds__(256)
kmeans_update(const long long* __restrict__ sums, const unsigned long long* __restrict__ counts,
              long long cells, int dsub, int s, float* __restrict__ cent) {
    const long long e = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= cells * dsub) return;
    const unsigned long long cnt = counts[e / dsub];
    if (cnt) cent[e] = (float)ldexp((double)sums[e] / (double)cnt, -s);
}

}  // namespace

// The three launches of an iteration, shared by pqh_kmeans_train (device-resident rows) and
// the streamed trainer pq_train_rows (pqh_pq_host.cpp, rows a chunk at a time): the
// fixed-point sums are exact integers, so accumulating chunk by chunk gives the same bits.
int pqh_kmeans_absmax_launch(pqh_ctx* ctx, const float* d_x, long long n, long long ld_x, int d,
                             unsigned* d_max) {
    if (n <= 0) return PQH_OK;
    hipLaunchKernelGGL(absmax_kernel, dim3(1024), dim3(256), 0, ctx->stream, d_x, n, ld_x, d, d_max);
    return hipGetLastError() == hipSuccess ? PQH_OK : PQH_ERR_HIP;
}

int pqh_kmeans_accum_launch(pqh_ctx* ctx, const float* d_x, long long n, long long ld_x, int m,
                            int k, int dsub, const void* d_codes, int s, long long* d_sums,
                            unsigned long long* d_cnt) {
    if (n <= 0) return PQH_OK;
    const bool lds = (size_t)k * dsub * 8 + (size_t)k * 4 <= 48 * 1024;
    const size_t lds_bytes = lds ? (size_t)k * dsub * 8 + (size_t)k * 4 : 0;
    const unsigned bx = (unsigned)std::min<long long>(std::max<long long>(1, n / 4096), 256);
    if (k <= 256) {
        if (lds)
            hipLaunchKernelGGL((kmeans_accum<uint8_t, true>), dim3(bx, m), dim3(256), lds_bytes,
                               ctx->stream, d_x, n, ld_x, m, k, dsub,
                               static_cast<const uint8_t*>(d_codes), s, d_sums, d_cnt);
        else
            hipLaunchKernelGGL((kmeans_accum<uint8_t, false>), dim3(bx, m), dim3(256), 0,
                               ctx->stream, d_x, n, ld_x, m, k, dsub,
                               static_cast<const uint8_t*>(d_codes), s, d_sums, d_cnt);
    } else {
        if (lds)
            hipLaunchKernelGGL((kmeans_accum<uint16_t, true>), dim3(bx, m), dim3(256), lds_bytes,
                               ctx->stream, d_x, n, ld_x, m, k, dsub,
                               static_cast<const uint16_t*>(d_codes), s, d_sums, d_cnt);
        else
            hipLaunchKernelGGL((kmeans_accum<uint16_t, false>), dim3(bx, m), dim3(256), 0,
                               ctx->stream, d_x, n, ld_x, m, k, dsub,
                               static_cast<const uint16_t*>(d_codes), s, d_sums, d_cnt);
    }
    return hipGetLastError() == hipSuccess ? PQH_OK : PQH_ERR_HIP;
}

int pqh_kmeans_update_launch(pqh_ctx* ctx, const long long* d_sums, const unsigned long long* d_cnt,
                             long long cells, int dsub, int s, float* d_cent) {
    hipLaunchKernelGGL(kmeans_update, dim3((unsigned)((cells * dsub + 255) / 256)), dim3(256), 0,
                       ctx->stream, d_sums, d_cnt, cells, dsub, s, d_cent);
    return hipGetLastError() == hipSuccess ? PQH_OK : PQH_ERR_HIP;
}

extern "C" {

int pqh_kmeans_train(pqh_ctx_t* ctx, const float* d_x, long long n, long long ld_x, int m,
                     int k, int dsub, int iters, float* centroids) {
    if (!ctx || !centroids || m <= 0 || k <= 0 || dsub <= 0 || iters < 0 || n < 0 ||
        (n > 0 && !d_x) || ld_x < (long long)m * dsub)
        return PQH_ERR_ARG;
    int rc = pqh_use_device(ctx);
    if (rc) return rc;
    if (n == 0 || iters == 0) return PQH_OK;
    const long long cells = (long long)m * k;
    const size_t esz = k <= 256 ? 1 : 2;
    // device buffers: codes, sums, counts, centroids, absmax
    void* d_codes = nullptr;
    long long* d_sums = nullptr;
    unsigned long long* d_cnt = nullptr;
    float* d_cent = nullptr;
    unsigned* d_max = nullptr;
    auto cleanup = [&] {
        (void)hipFree(d_codes);
        (void)hipFree(d_sums);
        (void)hipFree(d_cnt);
        (void)hipFree(d_cent);
        (void)hipFree(d_max);
    };
    if (hipMalloc(&d_codes, (size_t)n * m * esz) != hipSuccess ||
        hipMalloc(&d_sums, (size_t)cells * dsub * 8) != hipSuccess ||
        hipMalloc(&d_cnt, (size_t)cells * 8) != hipSuccess ||
        hipMalloc(&d_cent, (size_t)cells * dsub * 4) != hipSuccess ||
        hipMalloc(&d_max, 4) != hipSuccess) {
        cleanup();
        return pqh_set_error(ctx, PQH_ERR_NOMEM, "kmeans buffers");
    }
    // fixed-point exponent from max |x| over the training data
    unsigned hmax = 0;
    int s;
    {
        hipError_t e = hipMemsetAsync(d_max, 0, 4, ctx->stream);
        if (e == hipSuccess && pqh_kmeans_absmax_launch(ctx, d_x, n, ld_x, m * dsub, d_max))
            e = hipErrorLaunchFailure;
        if (e == hipSuccess) e = hipMemcpyAsync(&hmax, d_max, 4, hipMemcpyDeviceToHost, ctx->stream);
        if (e == hipSuccess) e = hipStreamSynchronize(ctx->stream);
        if (e != hipSuccess) {
            cleanup();
            return pqh_set_error(ctx, PQH_ERR_HIP, "kmeans absmax: %s", hipGetErrorString(e));
        }
        float fmax;
        std::memcpy(&fmax, &hmax, 4);
        s = pqh_kmeans_fixed_shift(fmax, n);
    }
    for (int it = 0; it < iters; ++it) {
        pqh_pq_t* pq = nullptr;
        rc = pqh_pq_create(ctx, centroids, m, k, dsub, &pq);
        if (!rc) rc = pqh_pq_assign(ctx, pq, d_x, n, ld_x, d_codes, nullptr, 0);
        if (pq) pqh_pq_destroy(pq);
        if (rc) {
            cleanup();
            return rc;
        }
        hipError_t e = hipMemsetAsync(d_sums, 0, (size_t)cells * dsub * 8, ctx->stream);
        if (e == hipSuccess) e = hipMemsetAsync(d_cnt, 0, (size_t)cells * 8, ctx->stream);
        if (e == hipSuccess)
            e = hipMemcpyAsync(d_cent, centroids, (size_t)cells * dsub * 4, hipMemcpyHostToDevice,
                               ctx->stream);
        if (e == hipSuccess && pqh_kmeans_accum_launch(ctx, d_x, n, ld_x, m, k, dsub, d_codes, s,
                                                       d_sums, d_cnt))
            e = hipErrorLaunchFailure;
        if (e == hipSuccess && pqh_kmeans_update_launch(ctx, d_sums, d_cnt, cells, dsub, s, d_cent))
            e = hipErrorLaunchFailure;
        if (e == hipSuccess)
            e = hipMemcpyAsync(centroids, d_cent, (size_t)cells * dsub * 4, hipMemcpyDeviceToHost,
                               ctx->stream);
        if (e == hipSuccess) e = hipStreamSynchronize(ctx->stream);
        if (e != hipSuccess) {
            cleanup();
            return pqh_set_error(ctx, PQH_ERR_HIP, "kmeans iteration: %s", hipGetErrorString(e));
        }
    }
    cleanup();
    return PQH_OK;
}

}  // extern "C"
