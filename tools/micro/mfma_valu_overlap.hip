// Diagnostic microbenchmark (not product code): do independent v_min3_f32 and
// v_mfma_f32_32x32x16_bf16 from the waves of one SIMD overlap on gfx950?  Times a loop of
// MFMAs only, min3s only, and both interleaved, with 1..3 waves per SIMD (256 CUs x 4 SIMDs).
#include <hip/hip_runtime.h>
#include <cstdio>

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

template <int MODE>   // 1: MFMA, 2: VALU, 3: both
__global__ void kern(int iters, float* sink) {
    bf16x8 a, b;
    for (int j = 0; j < 8; ++j) { a[j] = (__bf16)(threadIdx.x * 0.001f + j); b[j] = (__bf16)(j * 0.5f); }
    f32x16 acc0 = {}, acc1 = {};
    unsigned v[8];
    for (int j = 0; j < 8; ++j) v[j] = 0x3f800000u + threadIdx.x + j;
    const unsigned p = 0x3f000000u | threadIdx.x, q = 0x3e000000u ^ threadIdx.x;
    for (int i = 0; i < iters; ++i) {
        if (MODE & 1) {   // 4 MFMAs: two independent chains of two
            acc0 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, acc0, 0, 0, 0);
            acc1 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, acc1, 0, 0, 0);
            acc0 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(b, a, acc0, 0, 0, 0);
            acc1 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(b, a, acc1, 0, 0, 0);
        }
        if (MODE & 2) {   // 32 min3s over 8 independent chains
#pragma unroll
            for (int r = 0; r < 4; ++r)
#pragma unroll
                for (int j = 0; j < 8; ++j)
                    asm volatile("v_min3_f32 %0, %0, %1, %2" : "+v"(v[j]) : "v"(p), "v"(q));
        }
    }
    float s = 0;
    for (int j = 0; j < 16; ++j) s += acc0[j] + acc1[j];
    for (int j = 0; j < 8; ++j) s += __uint_as_float(v[j]);
    sink[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

template <int MODE>
float run(int wps, int iters, float* d) {
    hipEvent_t e0, e1;
    hipEventCreate(&e0); hipEventCreate(&e1);
    hipLaunchKernelGGL(kern<MODE>, dim3(256), dim3(256 * wps), 0, 0, iters, d);
    hipEventRecord(e0, 0);
    hipLaunchKernelGGL(kern<MODE>, dim3(256), dim3(256 * wps), 0, 0, iters, d);
    hipEventRecord(e1, 0);
    hipEventSynchronize(e1);
    float ms = 0;
    hipEventElapsedTime(&ms, e0, e1);
    return ms;
}

int main() {
    float* d;
    hipMalloc(&d, 256 * 1024 * 4);
    const int iters = 20000;
    for (int wps = 1; wps <= 3; ++wps) {
        const float m = run<1>(wps, iters, d), v = run<2>(wps, iters, d), b = run<3>(wps, iters, d);
        // per wave-iteration: 4 MFMAs and/or 32 min3s; ns per iteration per SIMD
        const double it = (double)iters * wps;
        printf("waves/SIMD %d: mfma-only %.2f ns, min3-only %.2f ns, both %.2f ns per iteration "
               "(sum %.2f, max %.2f)\n", wps, m * 1e6 / it, v * 1e6 / it, b * 1e6 / it,
               (m + v) * 1e6 / it, (m > v ? m : v) * 1e6 / it);
    }
    return 0;
}
