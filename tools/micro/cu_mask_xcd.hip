// Diagnostic (not product code): which XCDs do the CUs of a hipExtStreamCreateWithCUMask mask
// map to?  Launches many workgroups on streams masked to (a) CUs 0-31, (b) every 8th CU,
// (c) every 4th CU, records each workgroup's XCC_ID and prints the histogram.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

__global__ void who(unsigned* out) {
    if (threadIdx.x == 0) {
        const unsigned xcc = __builtin_amdgcn_s_getreg((3 << 11) | 20) & 15;   // XCC_ID
        atomicAdd(&out[xcc], 1u);
    }
}

static void run(const char* name, const std::vector<int>& cus) {
    std::vector<uint32_t> mask(8, 0u);
    for (int c : cus) mask[c / 32] |= 1u << (c % 32);
    hipStream_t s;
    if (hipExtStreamCreateWithCUMask(&s, (uint32_t)mask.size(), mask.data()) != hipSuccess) {
        printf("%s: mask failed\n", name);
        return;
    }
    unsigned* d;
    hipMalloc(&d, 16 * 4);
    hipMemsetAsync(d, 0, 64, s);
    hipLaunchKernelGGL(who, dim3(4096), dim3(64), 0, s, d);
    unsigned h[16];
    hipMemcpyAsync(h, d, 64, hipMemcpyDeviceToHost, s);
    hipStreamSynchronize(s);
    printf("%-22s XCC histogram:", name);
    for (int i = 0; i < 8; ++i) printf(" %u", h[i]);
    printf("\n");
    hipFree(d);
    hipStreamDestroy(s);
}

int main() {
    std::vector<int> a, b, c, e;
    for (int i = 0; i < 32; ++i) a.push_back(i);
    for (int i = 0; i < 256; i += 8) b.push_back(i);
    for (int i = 0; i < 256; i += 4) c.push_back(i);
    for (int i = 32; i < 64; ++i) e.push_back(i);
    run("CUs 0-31", a);
    run("CUs 32-63", e);
    run("every 8th CU", b);
    run("every 4th CU", c);
    return 0;
}
