// Diagnostic microbenchmark (not product code): VALU throughput per SIMD on gfx950 for the
// integer ops of the assignment kernel's key reduction (v_med3_u32, v_min_u32,
// v_and_or_b32) and v_fma_f32, with 1..4 waves per SIMD.  Each lane runs 8 independent
// chains so a wave's own dependencies never limit it.  Prints cycles per wave-instruction
// per SIMD (s_memtime ticks of one workgroup's wave 0, all waves busy the whole time).
#include <hip/hip_runtime.h>
#include <cstdio>

template <int OP>
__global__ void valu_rate(int iters, unsigned long long* out, unsigned* sink) {
    unsigned a[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) a[j] = threadIdx.x * 7u + j;
    unsigned b = threadIdx.x | 1u, c = threadIdx.x ^ 0x5555u;
    float f[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) f[j] = (float)(threadIdx.x + j);
    __syncthreads();
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    for (int i = 0; i < iters; ++i) {
#pragma unroll
        for (int r = 0; r < 4; ++r)
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                if (OP == 0) asm volatile("v_med3_u32 %0, %0, %1, %2" : "+v"(a[j]) : "v"(b), "v"(c));
                if (OP == 1) asm volatile("v_min_u32 %0, %0, %1" : "+v"(a[j]) : "v"(b));
                if (OP == 2) asm volatile("v_and_or_b32 %0, %0, %1, %2" : "+v"(a[j]) : "v"(b), "v"(c));
                if (OP == 3) asm volatile("v_fma_f32 %0, %0, %1, %1" : "+v"(f[j]) : "v"(1.0001f));
                if (OP == 4) {   // the assignment kernel's mix: one 32x32x16 MFMA per 24 VALU
                    asm volatile("v_med3_u32 %0, %0, %1, %2" : "+v"(a[j]) : "v"(b), "v"(c));
                    asm volatile("v_min_u32 %0, %0, %1" : "+v"(a[j]) : "v"(b));
                    asm volatile("v_and_or_b32 %0, %0, %1, %2" : "+v"(a[j]) : "v"(b), "v"(c));
                }
            }
        if (OP == 4) {
            typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
            typedef float f32x16 __attribute__((ext_vector_type(16)));
            bf16x8 av, bv;
#pragma unroll
            for (int j = 0; j < 8; ++j) { av[j] = (__bf16)f[j]; bv[j] = (__bf16)f[7 - j]; }
            f32x16 acc = {0};
            acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(av, bv, acc, 0, 0, 0);
            f[i & 7] += acc[0];
        }
    }
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    __syncthreads();
    if (threadIdx.x == 0 && blockIdx.x == 0) out[0] = t1 - t0;
    unsigned s = 0;
#pragma unroll
    for (int j = 0; j < 8; ++j) s += a[j] + __float_as_uint(f[j]);
    sink[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

int main() {
    unsigned long long* d_out;
    unsigned* d_sink;
    hipMalloc(&d_out, 64);
    hipMalloc(&d_sink, 256 * 1024 * 4);
    const int iters = 2000;
    const char* names[5] = {"v_med3_u32", "v_min_u32", "v_and_or_b32", "v_fma_f32", "mix 96:1mfma"};
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    for (int op = 0; op < 5; ++op)
        for (int wps : {1, 2, 3, 4}) {
            const int threads = 64 * 4 * wps;   // wps waves on each of the 4 SIMDs
            auto k = op == 0 ? valu_rate<0> : op == 1 ? valu_rate<1> : op == 2 ? valu_rate<2>
                     : op == 3 ? valu_rate<3> : valu_rate<4>;
            hipLaunchKernelGGL(k, dim3(256), dim3(threads), 0, 0, iters, d_out, d_sink);
            hipEventRecord(e0, 0);
            hipLaunchKernelGGL(k, dim3(256), dim3(threads), 0, 0, iters, d_out, d_sink);
            hipEventRecord(e1, 0);
            hipEventSynchronize(e1);
            float ms = 0;
            hipEventElapsedTime(&ms, e0, e1);
            unsigned long long h = 0;
            hipMemcpy(&h, d_out, 8, hipMemcpyDeviceToHost);
            const double insts = (double)iters * (op == 4 ? 96 : 32) * wps;   // VALU per SIMD
            printf("%-13s waves/SIMD %d: %.2f ticks per VALU wave-instruction per SIMD "
                   "(%.3f ns each; kernel %.3f ms, %.0f ticks/us)\n",
                   names[op], wps, (double)h / insts, ms * 1e6 / insts, ms, h / (ms * 1e3));
        }
    return 0;
}
