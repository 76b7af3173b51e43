// Diagnostic (not product code): the round-4 decoder variant that decoded wrong symbols
// (EXPERIMENTS.md section 5) read its stream window from LDS at a BIT POSITION, peeking the
// next bits as a 64-bit shift of the word pair (w[i] << 32 | w[i + 1]).  This kernel
// reproduces only that reader, in the decoder's shape: one-wave workgroups, a stream window
// staged byte-swapped into LDS, and per lane a dependent chain of peeks whose next position
// depends on the value peeked (as a symbol's length does).  Every lane runs the chain with
// the pair form (FORM 0) or with v_alignbit_b32 (FORM 1); the host recomputes every chain
// and counts the mismatches per workgroup.
//   hipcc --offload-arch=gfx950 -O3 -o lds_peek64 lds_peek64.hip && ./lds_peek64
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <vector>

constexpr int kWin = 1536;     // window words per workgroup (the SIFT decoder's size)
constexpr int kSteps = 64;     // peeks per lane (8 rows x 8 parts)

template <int FORM>
__global__ void __launch_bounds__(64)
peek_chain(const uint32_t* __restrict__ stream, uint32_t* __restrict__ out) {
    __shared__ uint32_t win[kWin + 4];
    const int lane = threadIdx.x;
    const uint32_t* src = stream + (size_t)blockIdx.x * kWin;
    for (int w = lane; w < kWin; w += 64) win[w] = __builtin_bswap32(src[w]);
    if (lane < 4) win[kWin + lane] = 0;
    __syncthreads();
    uint32_t pos = (uint32_t)lane * 700u;   // lane's chain start (bits)
    uint32_t acc = 0;
    for (int s = 0; s < kSteps; ++s) {
        const uint32_t i = pos >> 5, sh = pos & 31;
        const uint32_t w0 = win[i], w1 = win[i + 1];
        uint32_t v;
        if (FORM == 0) {
            const unsigned long long pair = ((unsigned long long)w0 << 32) | w1;
            v = (uint32_t)((pair << sh) >> 32);   // the next 32 bits at pos
        } else {
            v = sh ? __builtin_amdgcn_alignbit(w0, w1, 32 - sh) : w0;
        }
        acc = acc * 31u + (v >> 23);
        pos += 1 + (v >> 28);                      // a "code length" of 1..16 bits
    }
    out[(size_t)blockIdx.x * 64 + lane] = acc ^ pos;
}

static uint32_t host_chain(const uint32_t* src, int lane) {
    std::vector<uint32_t> win(kWin + 4, 0);
    for (int w = 0; w < kWin; ++w) win[w] = __builtin_bswap32(src[w]);
    uint32_t pos = (uint32_t)lane * 700u, acc = 0;
    for (int s = 0; s < kSteps; ++s) {
        const uint32_t i = pos >> 5, sh = pos & 31;
        const unsigned long long pair = ((unsigned long long)win[i] << 32) | win[i + 1];
        const uint32_t v = (uint32_t)((pair << sh) >> 32);
        acc = acc * 31u + (v >> 23);
        pos += 1 + (v >> 28);
    }
    return acc ^ pos;
}

int main() {
    const int blocks = 4096;
    std::vector<uint32_t> h((size_t)blocks * kWin);
    uint64_t x = 0x9E3779B97F4A7C15ull;
    for (auto& w : h) {
        x ^= x << 13; x ^= x >> 7; x ^= x << 17;
        w = (uint32_t)x;
    }
    uint32_t *d_s, *d_o;
    hipMalloc(&d_s, h.size() * 4);
    hipMalloc(&d_o, (size_t)blocks * 64 * 4);
    hipMemcpy(d_s, h.data(), h.size() * 4, hipMemcpyHostToDevice);
    std::vector<uint32_t> want((size_t)blocks * 64);
    for (int b = 0; b < blocks; ++b)
        for (int l = 0; l < 64; ++l) want[(size_t)b * 64 + l] = host_chain(&h[(size_t)b * kWin], l);
    for (int form = 0; form < 2; ++form) {
        for (int rep = 0; rep < 3; ++rep) {
            hipMemset(d_o, 0, (size_t)blocks * 64 * 4);
            if (form == 0) hipLaunchKernelGGL(peek_chain<0>, dim3(blocks), dim3(64), 0, 0, d_s, d_o);
            else hipLaunchKernelGGL(peek_chain<1>, dim3(blocks), dim3(64), 0, 0, d_s, d_o);
            hipDeviceSynchronize();
            std::vector<uint32_t> got((size_t)blocks * 64);
            hipMemcpy(got.data(), d_o, got.size() * 4, hipMemcpyDeviceToHost);
            long bad = 0, bad_lo = 0, first_bad = -1;
            for (size_t q = 0; q < got.size(); ++q)
                if (got[q] != want[q]) {
                    ++bad;
                    if (q / 64 < 512) ++bad_lo;
                    if (first_bad < 0) first_bad = (long)(q / 64);
                }
            printf("form %s rep %d: %ld of %zu lane chains wrong (%ld in workgroups < 512), first bad "
                   "workgroup %ld\n", form ? "alignbit" : "pair64", rep, bad, got.size(), bad_lo,
                   first_bad);
        }
    }
    hipFree(d_s);
    hipFree(d_o);
    return 0;
}
