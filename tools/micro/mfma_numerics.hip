// Diagnostic (not product code): the rounding model of v_mfma_f32_32x32x16_bf16 on gfx950.
// The assignment kernel's acceptance bound (pqh_assign.hip, TauCoef) charges the MFMA's
// fp32 accumulation of ||c||^2 + 16 bf16 products per instruction; this measures which
// model the hardware follows, on random and on cancellation-heavy operands:
//   chain  -- acc = fma(a_k, b_k, acc) for k = 0..15 in order (one rounding per product)
//   rchain -- the same, k = 15..0
//   once   -- the exact sum of the 16 products and C, rounded to fp32 once
//   prods  -- the exact sum of the 16 products rounded once, then + C rounded
// and the largest error against the exact sum, in units of 2^-24 * (|C| + sum |a_k b_k|).
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <vector>

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

// one 32x32x16 MFMA per tile; A [tiles][32][16], B [tiles][16][32], C/D [tiles][32][32]
__global__ void mfma_tiles(const __bf16* A, const __bf16* B, const float* C, float* D) {
    const int t = blockIdx.x, l = threadIdx.x, r = l & 31, h = l >> 5;
    bf16x8 a, b;
    for (int j = 0; j < 8; ++j) {
        a[j] = A[(t * 32 + r) * 16 + 8 * h + j];
        b[j] = B[(t * 16 + 8 * h + j) * 32 + r];
    }
    f32x16 c;
    for (int v = 0; v < 16; ++v) c[v] = C[(t * 32 + (v & 3) + 8 * (v >> 2) + 4 * h) * 32 + r];
    f32x16 d = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
    for (int v = 0; v < 16; ++v) D[(t * 32 + (v & 3) + 8 * (v >> 2) + 4 * h) * 32 + r] = d[v];
}

static float bf(float x) {   // round to bf16 (RNE), back to float
    unsigned u;
    std::memcpy(&u, &x, 4);
    u = (u + 0x7FFFu + ((u >> 16) & 1u)) & 0xFFFF0000u;
    float y;
    std::memcpy(&y, &u, 4);
    return y;
}

int main(int argc, char** argv) {
    const int tiles = argc > 1 ? std::atoi(argv[1]) : 4096;
    std::mt19937_64 rng(12345);
    std::normal_distribution<double> nd(0.0, 1.0);
    for (int mode = 0; mode < 3; ++mode) {
        // 0: random normal operands, C ~ 100; 1: SIFT-like (a in [0,255] integers, b ~ c
        // halves), C = ||c||^2-like (cancellation); 2: wide exponent spread
        std::vector<float> A(tiles * 512), B(tiles * 512), C(tiles * 1024), D(tiles * 1024);
        std::vector<__bf16> Ab(A.size()), Bb(B.size());
        for (size_t i = 0; i < A.size(); ++i) {
            float v = mode == 1 ? bf((float)(rng() % 256)) : bf((float)nd(rng) * (mode == 2 ? std::ldexp(1.0, (int)(rng() % 40) - 20) : 1.0));
            A[i] = v;
            Ab[i] = (__bf16)v;
        }
        for (size_t i = 0; i < B.size(); ++i) {
            float v = bf((float)(mode == 1 ? -2.0 * (rng() % 256) : nd(rng) * (mode == 2 ? std::ldexp(1.0, (int)(rng() % 40) - 20) : 1.0)));
            B[i] = v;
            Bb[i] = (__bf16)v;
        }
        for (size_t i = 0; i < C.size(); ++i)
            C[i] = mode == 1 ? (float)(16 * 128 * 128 + (rng() % 100000)) : (float)(nd(rng) * 100.0);
        __bf16 *dA, *dB;
        float *dC, *dD;
        hipMalloc(&dA, Ab.size() * 2);
        hipMalloc(&dB, Bb.size() * 2);
        hipMalloc(&dC, C.size() * 4);
        hipMalloc(&dD, D.size() * 4);
        hipMemcpy(dA, Ab.data(), Ab.size() * 2, hipMemcpyHostToDevice);
        hipMemcpy(dB, Bb.data(), Bb.size() * 2, hipMemcpyHostToDevice);
        hipMemcpy(dC, C.data(), C.size() * 4, hipMemcpyHostToDevice);
        hipLaunchKernelGGL(mfma_tiles, dim3(tiles), dim3(64), 0, 0, dA, dB, dC, dD);
        hipMemcpy(D.data(), dD, D.size() * 4, hipMemcpyDeviceToHost);
        long long n = 0, m_chain = 0, m_rchain = 0, m_once = 0, m_prods = 0;
        double worst = 0.0;
        for (int t = 0; t < tiles; ++t)
            for (int i = 0; i < 32; ++i)
                for (int j = 0; j < 32; ++j) {
                    const float c = C[(t * 32 + i) * 32 + j];
                    float ch = c, rc = c;
                    long double ex = c, ps = 0, mag = std::fabs(c);
                    for (int k = 0; k < 16; ++k) {
                        const float a = A[(t * 32 + i) * 16 + k], b = B[(t * 16 + k) * 32 + j];
                        ch = std::fmaf(a, b, ch);
                        ex += (long double)a * b;
                        ps += (long double)a * b;
                        mag += std::fabs((long double)a * b);
                    }
                    for (int k = 15; k >= 0; --k)
                        rc = std::fmaf(A[(t * 32 + i) * 16 + k], B[(t * 16 + k) * 32 + j], rc);
                    const float d = D[(t * 32 + i) * 32 + j];
                    ++n;
                    m_chain += d == ch;
                    m_rchain += d == rc;
                    m_once += d == (float)ex;
                    m_prods += d == (float)((long double)(float)ps + c);
                    if (mag > 0) {
                        const double e = (double)(std::fabs((long double)d - ex) / (mag * 0x1p-24L));
                        if (e > worst) worst = e;
                    }
                }
        std::printf("mode %d: n %lld  chain %.6f  rchain %.6f  once %.6f  prods+C %.6f  worst err %.3f x 2^-24 (|C| + sum|ab|)\n",
                    mode, n, (double)m_chain / n, (double)m_rchain / n, (double)m_once / n,
                    (double)m_prods / n, worst);
        hipFree(dA);
        hipFree(dB);
        hipFree(dC);
        hipFree(dD);
    }
    return 0;
}
