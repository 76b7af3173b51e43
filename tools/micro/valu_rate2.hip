// Diagnostic microbenchmark (not product code): wave64 VALU issue rate per SIMD on gfx950
// for the candidate key-reduction instructions, 1/2/4 waves per SIMD, 8 independent chains
// per lane.  Reports ns per wave-instruction per SIMD from the event-timed kernel
// (256 workgroups = one per CU; every SIMD runs `wps` waves for the whole kernel).
#include <hip/hip_runtime.h>
#include <cstdio>

#define OPS(X)                                                                         \
    X(0, "v_min3_u32", asm volatile("v_min3_u32 %0, %0, %1, %2" : "+v"(a[j]) : "v"(b), "v"(c)))   \
    X(1, "v_min3_f32", asm volatile("v_min3_f32 %0, %0, %1, %2" : "+v"(a[j]) : "v"(b), "v"(c)))   \
    X(2, "v_med3_f32", asm volatile("v_med3_f32 %0, %0, %1, %2" : "+v"(a[j]) : "v"(b), "v"(c)))   \
    X(3, "v_min_f32", asm volatile("v_min_f32 %0, %0, %1" : "+v"(a[j]) : "v"(b)))                 \
    X(4, "v_fma_f32", asm volatile("v_fma_f32 %0, %0, %1, %2" : "+v"(a[j]) : "v"(b), "v"(c)))     \
    X(5, "v_add_f32", asm volatile("v_add_f32 %0, %0, %1" : "+v"(a[j]) : "v"(b)))                 \
    X(6, "v_and_or_b32", asm volatile("v_and_or_b32 %0, %0, %1, %2" : "+v"(a[j]) : "v"(b), "v"(c))) \
    X(7, "v_pk_minimum3_f16", asm volatile("v_pk_minimum3_f16 %0, %0, %1, %2" : "+v"(a[j]) : "v"(b), "v"(c))) \
    X(8, "v_mov_b32", asm volatile("v_mov_b32 %0, %1" : "=v"(a[j]) : "v"(b)))                    \
    X(9, "v_perm_b32", asm volatile("v_perm_b32 %0, %0, %1, %2" : "+v"(a[j]) : "v"(b), "v"(c)))

template <int OP>
__global__ void rate(int iters, unsigned* sink) {
    unsigned a[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) a[j] = 0x3f800000u + threadIdx.x * 7u + j;
    unsigned b = 0x3f000000u | threadIdx.x, c = 0x3e000000u ^ threadIdx.x;
    for (int i = 0; i < iters; ++i) {
#pragma unroll
        for (int r = 0; r < 4; ++r)
#pragma unroll
            for (int j = 0; j < 8; ++j) {
#define CASE(N, NAME, STMT) if (OP == N) { STMT; }
                OPS(CASE)
#undef CASE
            }
    }
    unsigned s = 0;
#pragma unroll
    for (int j = 0; j < 8; ++j) s += a[j];
    sink[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

int main() {
    unsigned* d_sink;
    hipMalloc(&d_sink, 256 * 1024 * 4);
    const int iters = 4000;
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
#define RUN(N, NAME, STMT)                                                                    \
    for (int wps : {1, 2, 4}) {                                                               \
        const int threads = 64 * 4 * wps;                                                     \
        hipLaunchKernelGGL(rate<N>, dim3(256), dim3(threads), 0, 0, iters, d_sink);           \
        hipEventRecord(e0, 0);                                                                \
        hipLaunchKernelGGL(rate<N>, dim3(256), dim3(threads), 0, 0, iters, d_sink);           \
        hipEventRecord(e1, 0);                                                                \
        hipEventSynchronize(e1);                                                              \
        float ms = 0;                                                                         \
        hipEventElapsedTime(&ms, e0, e1);                                                     \
        const double insts = (double)iters * 32 * wps;                                        \
        printf("%-18s waves/SIMD %d: %.3f ns per wave-instruction per SIMD\n", NAME, wps,    \
               ms * 1e6 / insts);                                                             \
    }
    OPS(RUN)
#undef RUN
    return 0;
}
