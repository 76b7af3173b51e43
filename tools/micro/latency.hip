// Diagnostic microbenchmark (not product code): dependent-chain latencies of one wave on
// gfx950 -- LDS pointer chase (stride-16 interleaved lanes, like the tree builder), VALU
// chain, and LDS chase with a 144 KB dynamic allocation.
#include <hip/hip_runtime.h>
#include <cstdio>

__global__ void lds_chase(int steps, int active, unsigned long long* out, int* sink) {
    extern __shared__ unsigned int mem[];
    const int t = threadIdx.x;
    for (int i = t; i < 4096; i += blockDim.x) mem[i] = ((i / 16 + 7) % 256) * 16 + (i % 16);
    __syncthreads();
    if (t >= active) return;
    unsigned int p = t;
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    for (int s = 0; s < steps; ++s) p = mem[p];
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    if (t == 0) out[0] = t1 - t0;
    sink[t] = (int)p;
}

__global__ void valu_chain(int steps, unsigned long long* out, int* sink) {
    unsigned int p = threadIdx.x;
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    for (int s = 0; s < steps; ++s) {
        p = p * 2654435761u + 12345u;
        p ^= p >> 13;
    }
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    if (threadIdx.x == 0) out[0] = t1 - t0;
    sink[threadIdx.x] = (int)p;
}

int main() {
    unsigned long long* d_out;
    int* d_sink;
    hipMalloc(&d_out, 64);
    hipMalloc(&d_sink, 4096);
    unsigned long long h;
    const int steps = 10000;
    for (int lds_kb : {16, 144}) {
        if (lds_kb > 64)
            hipFuncSetAttribute((const void*)lds_chase, hipFuncAttributeMaxDynamicSharedMemorySize,
                                lds_kb * 1024);
        for (int active : {1, 16, 64}) {
            hipLaunchKernelGGL(lds_chase, dim3(1), dim3(64), lds_kb * 1024, 0, steps, active, d_out, d_sink);
            hipLaunchKernelGGL(lds_chase, dim3(1), dim3(64), lds_kb * 1024, 0, steps, active, d_out, d_sink);
            hipMemcpy(&h, d_out, 8, hipMemcpyDeviceToHost);
            printf("lds_chase lds=%dKB active=%d: %.1f cycles/step\n", lds_kb, active, (double)h / steps);
        }
    }
    hipLaunchKernelGGL(valu_chain, dim3(1), dim3(64), 0, 0, steps, d_out, d_sink);
    hipLaunchKernelGGL(valu_chain, dim3(1), dim3(64), 0, 0, steps, d_out, d_sink);
    hipMemcpy(&h, d_out, 8, hipMemcpyDeviceToHost);
    printf("valu_chain (mul+add+shr+xor): %.1f cycles/step\n", (double)h / steps);
    hipError_t e = hipDeviceSynchronize();
    printf("status %s\n", hipGetErrorString(e));
    return 0;
}
