// pqh_assign.hip -- PQ nearest-centroid assignment on gfx950.
//
// Replaces the assignment half of yael kmeans() called at pq_encoder.c:270-272 plus
// copy_cluster_indices (pq_encoder.c:192-205); fuses the non-context symbol histogram
// (huffman_encoder.c:139-164).
//
// Result definition (= the oracle, oracle/pqh_oracle.c): for every vector v and part i,
//   D_k = sum_j (x_j - c_kj)^2 in fp32, j ascending, product and sum rounded separately,
//   code = the first k reaching min_k D_k.
//
// Kernel design (DESIGN.md "pq_assign"):
//  * One wave per subspace, its centroid sub-codebook resident in VGPRs as MFMA A
//    fragments; a workgroup = up to 8 subspace waves over the same 32-vector block, so
//    every input row is read from HBM once per workgroup (512 B per SIFT vector).
//  * Screening score S_k = ||c_k||^2 - 2 x.c_k computed exactly-as-bounded by
//    v_mfma_f32_32x32x16_bf16: the accumulator starts at ||c_k||^2 (fp32, the C operand,
//    read from LDS) and the K dimension is [xh . ch | xh . cl]  (+ xl . ch only if the
//    block has any x that is not bf16-exact -- SIFT-like integer data skips that pass);
//    x = xh + xl + r, c = ch + cl + r' (bf16 splits).  Scores are signed and ordered as
//    floats (v_min3_f32 / v_med3_f32).
//  * Each lane's 128 scores (8 tiles x 16 accumulator registers) are reduced over two
//    partitions of that grid on the raw score bits (P: tile halves, Q: register pairs);
//    their group minima give the smallest and second smallest score and the winner's
//    cell (see `reduce`), and the two half-waves merge.  If the runner-up is further than a rigorous error bound tau
//    from the winner the winner IS the fp32 direct-form argmin; otherwise (and for any
//    non-finite input) the wave re-ranks all K centroids of that vector with the exact
//    fp32 direct form and first-index tie break.
#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <type_traits>
#include <vector>

#include "pqh_internal.h"

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

namespace {

#ifndef PQH_ASSIGN_WPG
#define PQH_ASSIGN_WPG 4
#endif
#ifndef PQH_ASSIGN_OCC_LARGE   // K = 4096: waves per SIMD
#define PQH_ASSIGN_OCC_LARGE 2
#endif
#ifndef PQH_ASSIGN_RING   // K = 4096: A-fragment tiles in flight from L2 (ring depth)
#define PQH_ASSIGN_RING 4
#endif
#ifndef PQH_ASSIGN_NB
#define PQH_ASSIGN_NB 2
#endif
#ifndef PQH_ASSIGN_OCC
#define PQH_ASSIGN_OCC (PQH_ASSIGN_NB == 1 ? 4 : 3)
#endif
#ifndef PQH_ASSIGN_DEFER
#define PQH_ASSIGN_DEFER 1
#endif
#ifndef PQH_ASSIGN_RQ
#define PQH_ASSIGN_RQ 128
#endif
constexpr int kRqLds = PQH_ASSIGN_RQ;   // deferred re-rank queue entries per wave (LDS)
constexpr int kWavesPerWG = PQH_ASSIGN_WPG;   // subspace waves per workgroup
constexpr int kNB = PQH_ASSIGN_NB;            // 32-vector blocks screened together per step
#ifndef PQH_ASSIGN_CLDS
#define PQH_ASSIGN_CLDS 0
#endif
#ifndef PQH_ASSIGN_SHAREA   // K = 4096: the workgroup's waves share one LDS ring of A tiles
#define PQH_ASSIGN_SHAREA 0    // (measured slower: 3.55 vs 2.6-2.9 ms per 1M rows alone, EXPERIMENTS.md)
#endif
constexpr int kAG = 8;            // (SHAREA) A tiles per ring group: one barrier per group
#ifndef PQH_ASSIGN_XAUX   // cache policy of the x slices' LDS DMA (2 = nt; experiment knob)
#define PQH_ASSIGN_XAUX 0
#endif
constexpr bool kCentLds = PQH_ASSIGN_CLDS != 0;

template <int D>
struct Plan {
    static constexpr int MAIN = 2 * D;                // xh.ch | xh.cl (||c||^2: the C operand)
    static constexpr int PM = (MAIN + 15) / 16;       // main MFMA passes
    static constexpr int PL = (D + 15) / 16;          // lo passes (xl . ch)
    // The lo pass reuses the main passes' A fragments: main slots [0, D) hold ch, and the lo
    // B operand is xl in slots [0, D) and zero elsewhere, so A pass p gives xl . ch over
    // dims [16p, 16p + 16) and the cl slots meet zeros.
    static constexpr int PA = PM;                     // distinct A fragments per tile
};

// Scores and keys are fp32 values carried as their bit patterns (unsigned) and ordered as
// floats: a key is a score with its low mantissa bits replaced by an index, which keeps the
// order of scores whose truncations differ (truncation moves a positive value down and a
// negative one up, monotonically) and makes every key distinct.
#ifndef PQH_ASSIGN_ASMMIN
#define PQH_ASSIGN_ASMMIN 0
#endif
#if PQH_ASSIGN_ASMMIN
// (PQH_ASSIGN_ASMMIN=1, the round-5 form) min/med written in asm so the compiler neither
// canonicalises nor reorders them.  The compiler cannot tell what an asm VALU is, so it pads
// the VALU that reads an asm result with an s_nop (a transcendental's forwarding hazard):
// ~20 per 32-vector block.
__device__ __forceinline__ unsigned med3u(unsigned a, unsigned b, unsigned c) {
    unsigned r;
    asm("v_med3_f32 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "v"(c));
    return r;
}

// v_min3_f32 of MFMA results.  The compiler's hazard recognizer does not look into inline
// asm, so an asm read of an accumulator gets none of the wait states an MFMA result needs
// (it would read stale values).  `after` is a compiler-generated value computed from the
// same accumulator (its read got the wait states); as an extra operand it keeps this asm
// behind that read, when the whole result is available.
__device__ __forceinline__ unsigned min3d(unsigned a, unsigned b, unsigned c, unsigned after) {
    unsigned r;
    asm("v_min3_f32 %0, %1, %2, %3 ; after %4" : "=v"(r) : "v"(a), "v"(b), "v"(c), "v"(after));
    return r;
}

__device__ __forceinline__ unsigned min3u(unsigned a, unsigned b, unsigned c) {
    unsigned r;
    asm("v_min3_f32 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "v"(c));
    return r;
}

__device__ __forceinline__ unsigned minu(unsigned a, unsigned b) {
    unsigned r;
    asm("v_min_f32 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
    return r;
}

__device__ __forceinline__ unsigned maxu(unsigned a, unsigned b) {
    unsigned r;
    asm("v_max_f32 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
    return r;
}
#else
// Compiler-generated gfx950 v_minimum3_f32 / v_maximum3_f32 (IEEE-754 2019 minimum /
// maximum: NaN-propagating, so unlike fminf they need no canonicalising max before them --
// checked in the ISA) and v_med3_f32, so the hazard recognizer sees every read: MFMA results
// get exactly their wait states and no asm result costs an s_nop.  min and max of non-NaN
// values are exact and order-free (-0 < +0 in both partitions alike), so the compiler's
// freedom to re-associate them changes no result; a NaN score (non-finite input or
// overflow) fails the gap test either way and is re-ranked.
__device__ __forceinline__ unsigned med3u(unsigned a, unsigned b, unsigned c) {
    return __float_as_uint(
        __builtin_amdgcn_fmed3f(__uint_as_float(a), __uint_as_float(b), __uint_as_float(c)));
}
__device__ __forceinline__ unsigned min3u(unsigned a, unsigned b, unsigned c) {
    return __float_as_uint(__builtin_elementwise_minimum(
        __builtin_elementwise_minimum(__uint_as_float(a), __uint_as_float(b)), __uint_as_float(c)));
}
__device__ __forceinline__ unsigned min3d(unsigned a, unsigned b, unsigned c, unsigned) {
    return min3u(a, b, c);
}
__device__ __forceinline__ unsigned minu(unsigned a, unsigned b) {
    return __float_as_uint(__builtin_elementwise_minimum(__uint_as_float(a), __uint_as_float(b)));
}
__device__ __forceinline__ unsigned maxu(unsigned a, unsigned b) {
    return __float_as_uint(__builtin_elementwise_maximum(__uint_as_float(a), __uint_as_float(b)));
}
#endif

// min(a, b) of two accumulator values as a compiler-generated instruction (v_med3_f32
// with -inf: the compiler inserts the MFMA wait states before it) -- the anchor of min3d.
// `ninf` holds -inf in a register the compiler cannot see into (an asm v_mov), so the
// med3 is not rewritten into a min with canonicalising maxes.
__device__ __forceinline__ unsigned anchor_min(unsigned a, unsigned b, float ninf) {
    return __float_as_uint(__builtin_amdgcn_fmed3f(__uint_as_float(a), __uint_as_float(b), ninf));
}

// a 32-bit constant in a VGPR the compiler cannot see into (so (x & mask) | s stays one
// v_and_or_b32 with the mask in a register instead of a literal and + an add)
__device__ __forceinline__ unsigned opaque_u32(unsigned v) {
    unsigned r;
    asm volatile("v_mov_b32 %0, %1" : "=v"(r) : "i"(v));
    return r;
}

// a wave-uniform value in an SGPR the compiler cannot split into SGPR + constant (so a
// key's index goes into one v_and_or_b32, not an and + an or3 with an inline constant)
__device__ __forceinline__ unsigned opaque_s32(int v) {
    unsigned r;
    asm("s_mov_b32 %0, %1" : "=s"(r) : "s"(v));
    return r;
}

__device__ __forceinline__ float opaque_ninf() {
    float r;
    asm volatile("v_mov_b32 %0, 0xff800000" : "=v"(r));
    return r;
}

// max(|a|, |b|) in one instruction (fmaxf(fabsf, fabsf) adds two canonicalising maxes)
__device__ __forceinline__ float max_abs(float a, float b) {
    float r;
    asm("v_max_f32_e64 %0, |%1|, |%2|" : "=v"(r) : "v"(a), "v"(b));
    return r;
}

// The index bits of Q-group j's key: register j of the tile's lower half is accumulator row
// (j & 3) + 8 (j >> 2) (tile_row), so the winner's row is an OR of its two keys' low bits.
__device__ __forceinline__ unsigned q_code_bits(int j) {
    return (unsigned)((j & 3) | ((j & 4) << 1));
}

// The running smallest (m1) and second smallest (m2 >= m1) keys after two more distinct keys
// (3 VALU instead of two med3 + min folds): the new minimum is min3(m1, k0, k1); the new
// second is the smaller of m2 and the second smallest of {m1, k0, k1} -- the minimum of the
// four values lies in {m1, k0, k1}, and the rest's smallest is either that triple's second or
// m2.
#ifndef PQH_ASSIGN_FOLD4
__device__ __forceinline__ void fold2(unsigned& m1, unsigned& m2, unsigned k0, unsigned k1) {
    m2 = minu(med3u(m1, k0, k1), m2);
    m1 = min3u(m1, k0, k1);
}
#else   // (the round-5 form, 4 VALU: A/B builds)
__device__ __forceinline__ void fold2(unsigned& m1, unsigned& m2, unsigned k0, unsigned k1) {
    m2 = med3u(m1, m2, k0);
    m1 = minu(m1, k0);
    m2 = med3u(m1, m2, k1);
    m1 = minu(m1, k1);
}
#endif

// Smallest and second smallest of 8 distinct keys (10 VALU): two triples and a pair give
// their (min, second); every key but the overall minimum is >= one of the three seconds or
// is the second smallest of the three minima, and each of those is a key other than the
// minimum, so their minimum is the second key.
__device__ __forceinline__ void top2_8(const unsigned* k, unsigned& m1, unsigned& m2) {
    const unsigned a1 = min3u(k[0], k[1], k[2]), a2 = med3u(k[0], k[1], k[2]);
    const unsigned b1 = min3u(k[3], k[4], k[5]), b2 = med3u(k[3], k[4], k[5]);
    const unsigned c1 = minu(k[6], k[7]), c2 = maxu(k[6], k[7]);
    m1 = min3u(a1, b1, c1);
    m2 = minu(min3u(a2, b2, c2), med3u(a1, b1, c1));
}

// main-layout B slot value for vector-side quantities
template <int D>
__device__ __forceinline__ float main_slot(int s, const float* xh) {
    if (s < D) return xh[s];
    if (s < 2 * D) return xh[s - D];
    return 0.0f;
}

// Exact fp32 direct-form distance (no contraction: __fadd_rn/__fmul_rn).
template <int D>
__device__ __forceinline__ float exact_dist(const float* x, const float* c) {
#pragma clang fp contract(off)
    float acc = 0.0f;
#pragma unroll
    for (int j = 0; j < D; ++j) {
        float d = __fsub_rn(x[j], c[j]);
        acc = __fadd_rn(acc, __fmul_rn(d, d));
    }
    return acc;
}

// diagnostics (PQH_ASSIGN_STAMPS builds only): per wave of the last pq_assign_mfma launch,
// {s_memrealtime at start, at end, blocks done | s_memtime lifetime << 16, XCC id}
constexpr int kStampWaves = 8192;
__device__ unsigned long long g_assign_stamps[kStampWaves][4];
// re-rank phases per wave (PQH_ASSIGN_STAMPS): ticks {x rows arrived, screening, candidate
// rounds} summed over the wave's batches, and the rounds
__device__ unsigned long long g_assign_rr[kStampWaves][4];
#ifdef PQH_ASSIGN_STAMPS
#define PQH_RR_STAMP(var)                                                \
    do {                                                                 \
        asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");      \
        var = __builtin_amdgcn_s_memrealtime();                          \
    } while (0)
#endif

// ---- screening steps shared by pq_assign_mfma and pq_rerank_window: a deferred vector is
// re-screened by the same instruction sequence, so its scores are bitwise the same.
// D = 16, 32 ("HALF"): lane (r, h) holds dims [16p + 8h, 16p + 8h + 8) of vector r for
// every 16-dim piece p -- exactly the B-fragment slots it feeds -- as xs[8p .. 8p + 8);
// other D: both half-waves hold all D dims.
template <int D>
struct Slice {
    static constexpr bool HALF = D % 16 == 0;
    static constexpr int NP = HALF ? D / 16 : 1;    // 16-dim pieces
    static constexpr int XD = HALF ? D / 2 : D;     // values per lane
    // dim of the lane's value j
    static __device__ __forceinline__ int dim(int j, int h) {
        return HALF ? 16 * (j >> 3) + 8 * h + (j & 7) : j;
    }
};

// the value of lane l ^ 32 (a VALU lane swap, no LDS round trip)
__device__ __forceinline__ unsigned partner32(unsigned v) {
    const auto sw = __builtin_amdgcn_permlane32_swap(v, v, false, false);
    return (threadIdx.x & 32) ? sw[0] : sw[1];
}

// ||x||^2: fp32 fma chain over the lane's slice (HALF: plus the partner half-wave's, lower +
// upper, so both halves round the same sum; a VALU lane swap, no LDS round trip).  The main
// loop and the re-rank tail both use this, so their biases are bitwise the same.
template <int D>
__device__ __forceinline__ float norm_part(const float* xs) {
    float X = 0.0f;
#pragma unroll
    for (int j = 0; j < Slice<D>::XD; ++j) X = fmaf(xs[j], xs[j], X);
    return X;
}

template <int D>
__device__ __forceinline__ float norm_x(const float* xs) {
    float X = norm_part<D>(xs);
    if constexpr (Slice<D>::HALF) {
        const auto sw = __builtin_amdgcn_permlane32_swap(__float_as_uint(X), __float_as_uint(X),
                                                         false, false);
        X = __uint_as_float(sw[0]) + __uint_as_float(sw[1]);
    }
    return X;
}

// whether some x of the lane's slice is not bf16-exact: a float whose low 16 bits are zero
// converts to bf16 exactly (denormals are preserved, .amdhsa_float_denorm_mode_32 3), any
// other leaves a non-zero remainder x - float(bf16(x))
template <int D>
__device__ __forceinline__ bool has_lo(const float* xs) {
    constexpr int XD = Slice<D>::XD;
    unsigned o = __float_as_uint(xs[0]);
    int j = 1;
    for (; j + 1 < XD; j += 2)   // v_or3_b32: two values per instruction
        asm("v_or3_b32 %0, %1, %2, %3"
            : "=v"(o) : "v"(o), "v"(__float_as_uint(xs[j])), "v"(__float_as_uint(xs[j + 1])));
    for (; j < XD; ++j) o |= __float_as_uint(xs[j]);
    return (o & 0xFFFFu) != 0;
}

// ||x||^2, the bf16 split x = xh + xl (+ r), and whether this lane's slice has any bf16
// remainder (the re-rank tail's form of the main loop's prologue).
template <int D>
__device__ __forceinline__ void split_x(const float* xs, float& X, bool& lo, float* xh, float* xl) {
    constexpr int XD = Slice<D>::XD;
    X = norm_x<D>(xs);
    lo = false;
#pragma unroll
    for (int j = 0; j < XD; ++j) {
        __bf16 hb = (__bf16)xs[j];
        xh[j] = (float)hb;
        float rem = xs[j] - xh[j];
        xl[j] = (float)(__bf16)rem;
        lo |= rem != 0.0f;
    }
}

// Error bound E0 of the screening score S_k = D_k - X against the fp32 direct-form
// distance D_k (DESIGN.md "pq_assign error bound"), P = sqrt(X) sqrt(Cmax):
//   E0 = split + 2^-22 Cmax + 2^-17 (2.02 P + 1.01 Cmax + 1.05 X).
// split is what the bf16 halves leave out of 2 x.c: with a bf16 remainder in some x of the
// block 2^-13 P; without one (x = xh) exactly 2 |x . r'_k| with r'_k = c_k - ch_k - cl_k,
// <= 2 sqrt(X) R, R = max_k ||r'_k|| measured on the host (R <= 2^-16 sqrt(Cmax), so this is
// never looser than the 2^-15 P it replaces; typically ~3x tighter, fewer re-ranks).  The
// acceptance gap tau = 2.2 E0 is evaluated as a1 sqrt(X) + (c X + b) with per-subspace
// coefficients (TauCoef); every term is positive, so inflating each coefficient by 2^-20
// covers the rounding of the coefficients and of the two fmas, and the 1e-5 on sqrt(Cmax)
// covers v_sqrt_f32 (1 ulp) against the correctly rounded root.
struct TauCoef {
    float a_nolo, a_lo, b, c;
};

// cm = Cmax, sc = sqrt(Cmax), r2 = 2 R (all rounded up on the host)
__device__ __forceinline__ TauCoef tau_coef(float cm, float sc, float r2) {
    constexpr float up = 1.0f + 0x1p-20f;
    const float s = 2.2f * 1.00001f;
    return {s * (r2 + 2.02f * 0x1p-17f * sc) * up, s * sc * (0x1p-13f + 2.02f * 0x1p-17f) * up,
            2.2f * cm * (0x1p-22f + 1.01f * 0x1p-17f) * up + 1e-30f,
            2.2f * 1.05f * 0x1p-17f * up};
}

__device__ __forceinline__ float screen_tau(float X, bool any_lo, const TauCoef& q) {
#ifdef PQH_ASSIGN_TAU_SCALE   // diagnostic builds only (breaks exactness): re-rank rate sweeps
    return PQH_ASSIGN_TAU_SCALE *
           fmaf(any_lo ? q.a_lo : q.a_nolo, __builtin_amdgcn_sqrtf(X), fmaf(q.c, X, q.b));
#endif
    return fmaf(any_lo ? q.a_lo : q.a_nolo, __builtin_amdgcn_sqrtf(X), fmaf(q.c, X, q.b));
}

template <int D>
__device__ __forceinline__ void build_b(const float* xh, const float* xl, int h,
                                        bf16x8* Bm, bf16x8* Bl) {
    using P = Plan<D>;
    if constexpr (Slice<D>::HALF) {
        // pass p < NP: slots 16p + 8h + j = dims of piece p (the lane's xs[8p + j]); passes
        // NP .. 2 NP - 1 repeat them (x . cl); lo pass p: the remainders of piece p
        constexpr int NP = Slice<D>::NP;
#pragma unroll
        for (int p = 0; p < NP; ++p) {
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                Bm[p][j] = (__bf16)xh[8 * p + j];
                Bl[p][j] = (__bf16)xl[8 * p + j];
            }
            Bm[NP + p] = Bm[p];
        }
    } else {
#pragma unroll
        for (int p = 0; p < P::PM; ++p)
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                float v0 = main_slot<D>(16 * p + j, xh);
                float v1 = main_slot<D>(16 * p + 8 + j, xh);
                Bm[p][j] = (__bf16)(h ? v1 : v0);
            }
#pragma unroll
        for (int p = 0; p < P::PL; ++p)
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                int s0 = 16 * p + j, s1 = 16 * p + 8 + j;
                float v0 = s0 < D ? xl[s0 < D ? s0 : 0] : 0.0f;
                float v1 = s1 < D ? xl[s1 < D ? s1 : 0] : 0.0f;
                Bl[p][j] = (__bf16)(h ? v1 : v0);
            }
    }
}

// The main loop's B operands, straight from x: the same bf16 values as split_x + build_b
// (xh = bf16(x), xl = bf16(x - xh)), with packed conversions; xl only when LO.
template <int D, bool LO>
__device__ __forceinline__ void make_b(const float* xs, int h, bf16x8* Bm, bf16x8* Bl) {
    using P = Plan<D>;
    if constexpr (Slice<D>::HALF) {
        typedef float f32x8 __attribute__((ext_vector_type(8)));
        constexpr int NP = Slice<D>::NP;
#pragma unroll
        for (int p = 0; p < NP; ++p) {
            f32x8 xv;
#pragma unroll
            for (int j = 0; j < 8; ++j) xv[j] = xs[8 * p + j];
            Bm[p] = __builtin_convertvector(xv, bf16x8);
            Bm[NP + p] = Bm[p];
            if constexpr (LO) {
                f32x8 rem;
#pragma unroll
                for (int j = 0; j < 8; ++j) rem[j] = xs[8 * p + j] - (float)Bm[p][j];
                Bl[p] = __builtin_convertvector(rem, bf16x8);
            }
        }
    } else if constexpr (D % 2 == 0) {
        // Even D without the half split (Deep's dsub 6): every B slot pair (2w, 2w + 1) of a
        // pass holds a pair of consecutive dims (d, d + 1), d even, or zeros, so the lane
        // converts its D/2 dim pairs once (packed v_cvt_pk_bf16_f32) and picks each word for its
        // half-wave with one select: D/2 + 4 VALU per pass instead of a convert and a select
        // per slot.  The same bf16 values as build_b (round to nearest even both ways).
        typedef float f32x2 __attribute__((ext_vector_type(2)));
        typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
        typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
        constexpr int NQ = D / 2;
        unsigned ph[NQ], pl[NQ];
#pragma unroll
        for (int q = 0; q < NQ; ++q) {
            const f32x2 v = {xs[2 * q], xs[2 * q + 1]};
            const bf16x2 hb = __builtin_convertvector(v, bf16x2);
            ph[q] = __builtin_bit_cast(unsigned, hb);
            if constexpr (LO) {
                const f32x2 r = {xs[2 * q] - (float)hb[0], xs[2 * q + 1] - (float)hb[1]};
                pl[q] = __builtin_bit_cast(unsigned, __builtin_convertvector(r, bf16x2));
            }
        }
        // main-layout word of slot s (even): dims s, s + 1 (s < D), again for the x . cl
        // half (D <= s < 2D), else zero
        auto mword = [&](int s) -> unsigned {
            return s < D ? ph[s / 2] : s < 2 * D ? ph[(s - D) / 2] : 0u;
        };
#pragma unroll
        for (int p = 0; p < P::PM; ++p) {
            u32x4 wv;
#pragma unroll
            for (int w = 0; w < 4; ++w) {
                const unsigned v0 = mword(16 * p + 2 * w), v1 = mword(16 * p + 8 + 2 * w);
                wv[w] = h ? v1 : v0;
            }
            Bm[p] = __builtin_bit_cast(bf16x8, wv);
        }
        if constexpr (LO) {
#pragma unroll
            for (int p = 0; p < P::PL; ++p) {
                u32x4 wv;
#pragma unroll
                for (int w = 0; w < 4; ++w) {
                    const int s0 = 16 * p + 2 * w, s1 = 16 * p + 8 + 2 * w;
                    const unsigned v0 = s0 < D ? pl[s0 / 2] : 0u, v1 = s1 < D ? pl[s1 / 2] : 0u;
                    wv[w] = h ? v1 : v0;
                }
                Bl[p] = __builtin_bit_cast(bf16x8, wv);
            }
        }
    } else {
        constexpr int XD = Slice<D>::XD;
        float xh[XD], xl[XD];
#pragma unroll
        for (int j = 0; j < XD; ++j) {
            xh[j] = (float)(__bf16)xs[j];
            xl[j] = LO ? (float)(__bf16)(xs[j] - xh[j]) : 0.0f;
        }
        build_b<D>(xh, xl, h, Bm, Bl);
    }
}

// the 32 x 32 score tile: centroid rows (A fragments a[0 .. PA)) x the block's vectors (B),
// accumulated onto the rows' ||c||^2 (cn: this lane's 16 rows of the tile)
template <int D>
__device__ __forceinline__ f32x16 tile_scores_a(const bf16x8* a, const bf16x8* Bm,
                                                const bf16x8* Bl, bool lo_pass, const f32x16& cn) {
    using P = Plan<D>;
    f32x16 acc = cn;
#pragma unroll
    for (int p = 0; p < P::PM; ++p)
        acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[p], Bm[p], acc, 0, 0, 0);
    if (lo_pass) {
#pragma unroll
        for (int p = 0; p < P::PL; ++p)
            acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[p], Bl[p], acc, 0, 0, 0);
    }
    return acc;
}

// this lane's 16 rows of ||c||^2 for tile t (LDS image [tile][half][16]: every lane of a
// half-wave reads the same 64 bytes, a broadcast)
// (four 16-byte reads: with one 64-byte vector read the compiler loses track of which LDS
// array it reads and waits for the in-flight LDS DMA of the next chunk's x before every tile)
__device__ __forceinline__ f32x16 tile_norms(const float* Cn, int t, int h) {
    const f32x4* p = reinterpret_cast<const f32x4*>(Cn + (t * 2 + h) * 16);
    const f32x4 a = p[0], b = p[1], c = p[2], d = p[3];
    return f32x16{a[0], a[1], a[2], a[3], b[0], b[1], b[2], b[3],
                  c[0], c[1], c[2], c[3], d[0], d[1], d[2], d[3]};
}

// A fragment p of tile t, [PA][KT][64 lanes] per subspace: from the workgroup's LDS copy
// (K = 256) or straight from L2 (K = 4096: 256 KB per subspace, streamed)
template <int KT>
__device__ __forceinline__ bf16x8 frag_at(const uint4* src, int p, int t, int lane) {
    return *reinterpret_cast<const bf16x8*>(&src[(p * KT + t) * 64 + lane]);
}

// tile t with its A fragments read from `src` (LDS copy or global)
template <int D, int KT>
__device__ __forceinline__ f32x16 tile_scores(const uint4* src, const float* Cn, int lane, int t,
                                              const bf16x8* Bm, const bf16x8* Bl, bool lo_pass) {
    using P = Plan<D>;
    bf16x8 a[P::PA];
#pragma unroll
    for (int p = 0; p < P::PA; ++p) a[p] = frag_at<KT>(src, p, t, lane);
    return tile_scores_a<D>(a, Bm, Bl, lo_pass, tile_norms(Cn, t, lane >> 5));
}

// centroid row of accumulator register i of tile t for half-wave h (32x32x16 output layout)
__device__ __forceinline__ int tile_row(int t, int i, int h) {
    return 32 * t + (i & 3) + 8 * (i >> 2) + 4 * h;
}

// KT = centroid tiles of 32 (8: K = 256, A fragments in LDS; 128: K = 4096, A fragments
// streamed from L2 a few tiles ahead, no fused histogram)
// (dsub 32 and K = 4096 hold more live state per wave: two waves per SIMD, no spills)
template <int D, int KT, typename CodeT>
__global__ void __launch_bounds__(64 * kWavesPerWG, D == 32 ? 2 : KT > 8 ? PQH_ASSIGN_OCC_LARGE : PQH_ASSIGN_OCC)
pq_assign_mfma(const float* __restrict__ x, long long n, long long ldx, int m_total,
               const bf16x8* __restrict__ afrag, const float* __restrict__ cnorm,
               const float* __restrict__ cent,
               const float* __restrict__ cmax, const float* __restrict__ sqrt_cmax,
               CodeT* __restrict__ codes, uint32_t* __restrict__ counts,
               unsigned long long* __restrict__ rerank, uint32_t* __restrict__ sched, int gx,
               unsigned long long* __restrict__ rerank_next, uint32_t* __restrict__ sched_next,
               int prio, long long ldc) {
    using P = Plan<D>;
    constexpr int K = KT * 32;
    constexpr bool kLdsA = KT <= 8;
    // P-key index bits (tile and half: 2 KT groups) and the key truncation they cost
    constexpr int PB = KT <= 8 ? 4 : 8;
    constexpr unsigned PMASK = (1u << PB) - 1;
    static_assert(2 * KT <= (1 << PB), "P-group index must fit the key's low bits");
    // the fused histogram's per-wave counters (non-context counts only): dynamic LDS that the
    // launch allocates only when counts are requested, so the context path's workgroups
    // leave those 4 KB to the kernels running beside the grid
    extern __shared__ uint32_t hist_dyn[];
    auto hist = [&](int w) -> uint32_t* { return hist_dyn + w * K; };
    // the subspace's A fragments, shared by the workgroup's waves (16 KB at D = 16): keeping
    // them out of VGPRs is what lets several waves share each SIMD
    __shared__ uint4 As[kLdsA ? P::PA * KT * 64 : 1];
    // ||c_k||^2 (fp32) of the subspace in accumulator order: [tile][half-wave][16 registers]
    __shared__ __attribute__((aligned(64))) float Cn[KT * 2 * 16];
    // each wave's re-rank queue (the LDS budget stays at 32 KB, so a workgroup still fits on
    // a CU beside a code-table build's 112 KB)
    __shared__ uint2 rqs[kWavesPerWG][kRqLds];
#ifndef PQH_ASSIGN_XLDS
#define PQH_ASSIGN_XLDS 1
#endif
    // the next chunk's x slices, prefetched by LDS DMA instead of into registers (16 fewer
    // VGPRs live across the step at D = 16): [wave][block][16-byte piece][64 lanes x 4]
    constexpr bool kXLds = PQH_ASSIGN_XLDS && KT <= 8 && Slice<D>::XD % 4 == 0;
    __shared__ __attribute__((aligned(16))) float xst[kXLds ? kWavesPerWG : 1][kXLds ? kNB : 1]
                                                     [kXLds ? Slice<D>::XD / 4 : 1][kXLds ? 256 : 1];
    // (PQH_ASSIGN_CLDS, K = 256) the fp32 centroids for the exact re-rank's candidate rows
    __shared__ __attribute__((aligned(16))) float Cf[kLdsA && kCentLds ? K * D : 1];
    // K = 4096 (SHAREA): the A fragments stream through an LDS ring of 2 kAG tiles that the
    // workgroup's waves fill together by LDS DMA and all read -- one L2 fetch of a tile per
    // workgroup instead of one per wave (the streamed kernel was bound by those L2 reads:
    // 256 KB per 64 vectors, 32 GB per 1M-row launch).  Tile t sits in slot t % (2 kAG):
    // Ar[(slot * PA + p) * 64 + lane].  The waves then run their chunks in lockstep (one
    // barrier per group), on a static workgroup schedule.
    constexpr bool kShareA = !kLdsA && PQH_ASSIGN_SHAREA != 0;
    constexpr int kAR = 2 * kAG;
    __shared__ __attribute__((aligned(16))) uint4 Ar[kShareA ? kAR * P::PA * 64 : 1];

    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);   // (uniform: SGPR math)
    // One subspace per workgroup, gx workgroups per subspace, 1-D grid.  Workgroup L is
    // placed on XCD L % 8 and, within it, round robin over the CUs, so L, L + 256, L + 512 ...
    // tend to share a CU.  The waves of a SIMD run at very different speeds (VALU issue goes
    // to the oldest wave first); only waves of the SAME subspace can even that out through
    // the subspace's work queue, so with gx % 8 == 0 subspace m = (L / 8) % m_total, which
    // gives every CU's resident workgroups one subspace (speed only -- any bijection is
    // correct).
    const int L = blockIdx.x;
    const bool inter = (gx & 7) == 0;
    const int m = inter ? (L >> 3) % m_total : L / gx;
    const int bx = inter ? (L / (8 * m_total)) * 8 + (L & 7) : L % gx;
    const int r = lane & 31;
    const int h = lane >> 5;
    pqh_set_prio(prio);   // (pqh_prio "ASSIGN": against the kernels running beside it)
    if (L == 0 && wave == 0) {   // the next launch's queue heads and re-rank counter
        // (agent-scope stores: written through to where the next launch's atomics act)
        if (sched_next)   // every subspace's heads, not only this launch's m_total: the next
                          // launch on this context may have more subspaces
            for (int q = lane; q < kSchedMax * kXcds; q += 64)
                __hip_atomic_store(sched_next + q * kSchedStride, 0u, __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_AGENT);
        if (lane == 0)
            __hip_atomic_store(rerank_next, 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    {
        const uint4* src = reinterpret_cast<const uint4*>(afrag) + (long long)m * P::PA * KT * 64;
        if constexpr (kLdsA)
            for (int i = threadIdx.x; i < P::PA * KT * 64; i += blockDim.x) As[i] = src[i];
        for (int i = threadIdx.x; i < KT * 2 * 16; i += blockDim.x)
            Cn[i] = cnorm[(long long)m * KT * 2 * 16 + i];
        if (kLdsA && counts)
            for (int i = lane; i < K; i += 64) hist(wave)[i] = 0;
        if constexpr (kLdsA && kCentLds)
            for (int i = threadIdx.x; i < K * D; i += blockDim.x) Cf[i] = cent[(long long)m * K * D + i];
        __syncthreads();   // the only workgroup barrier
    }
    // where the A fragments come from: the LDS copy, or this subspace's slice in global
    const uint4* const asrc =
        kLdsA ? As : reinterpret_cast<const uint4*>(afrag) + (long long)m * P::PA * KT * 64;
    // (K = 4096: the subspace's fragments as a buffer; built from wave-uniform values)
    const auto arsrc = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<uint4*>(reinterpret_cast<const uint4*>(afrag) + (long long)m * P::PA * KT * 64),
        0, P::PA * KT * 64 * 16, 0x00020000);
#ifdef PQH_ASSIGN_STAMPS
    const unsigned long long st0 = __builtin_amdgcn_s_memtime();
    const unsigned long long rt0 = __builtin_amdgcn_s_memrealtime();
    unsigned long long nbdone = 0, rr_ticks = 0, rr_batches = 0;
    unsigned long long rr_x = 0, rr_scr = 0, rr_cand = 0, rr_rounds = 0;
#endif
    const float cm = cmax[m];
    const float sc = sqrt_cmax[m];
    const TauCoef tq = tau_coef(cm, sc, sqrt_cmax[m_total + m]);   // ([m, 2m): 2 R)
    const float ninf = opaque_ninf();
    // the P-key mask: an inline constant for 4 index bits, a register for 8
    const unsigned keymask = PB == 4 ? ~PMASK : opaque_u32(~PMASK);
    // fp32 centroids (L2-resident, 16 KB at dsub 16; or the workgroup's LDS copy)
    const float* cl = kLdsA && kCentLds ? Cf : cent + (long long)m * K * D;
    // block and chunk indices are 32-bit, so their tests are scalar compares (a 64-bit signed
    // compare of wave-uniform values is a VALU instruction pair): 0.2436 -> 0.2413 ms per 1M
    // (the host splits launches at 2^30 rows)
    const int n32 = (int)n;
    const int nblk = (n32 + 31) / 32;
    const int nfull = n32 / 32;   // blocks with 32 valid rows
    unsigned long long slow_count = 0;

    // x slice of a block.  D == 16 (SIFT): lane (r, h) holds dims [8h, 8h + 8) of vector r
    // -- exactly the B-fragment slots it feeds -- so each lane splits 8 values and no
    // half-wave selects are needed; other D: both half-waves hold all D dims.
    constexpr bool HALF = Slice<D>::HALF;
    constexpr int XD = Slice<D>::XD;
    // Branch-free loads (the row index is clamped; the block's validity is applied when
    // the slice is used), so the prefetch stays in flight across a whole block.
    // The lane's slice of row r of block 0; a block's rows are a uniform offset away.  Only
    // the last, partial block clamps its rows (to n - 1), on a wave-uniform branch.
    // Addresses are a wave-uniform 64-bit base (SGPRs) plus the lane's 32-bit byte offset
    // within the block (global loads / stores with an SGPR base): no per-lane 64-bit math.
    // (ld_x < 2^22 on the host, so the offsets fit 24 bits.)
    const unsigned ldx4 = (unsigned)ldx * 4u;
    const unsigned xh_off = HALF ? 32u * (unsigned)h : 0u;
    const unsigned xlane_off = __umul24((unsigned)r, ldx4) + xh_off;
    const char* const xm = reinterpret_cast<const char*>(x + (long long)m * D);
    // codes: row-major [n][m_total] (ldc = 0: pq_indices.bvecsl order), or part-major
    // [m_total][ldc] -- then a wave's 64 codes of a chunk are 64 contiguous bytes (whole
    // lines from one wave instead of one byte in every 8 from 8 subspaces' workgroups)
    const long long crs = ldc ? 1 : m_total;   // (uniform) row stride in codes
    CodeT* const cbase = codes + (ldc ? (long long)m * ldc : (long long)m);
    const unsigned code_lane_off = (unsigned)r * (unsigned)crs * (unsigned)sizeof(CodeT);
    const unsigned code_pair_off = (unsigned)lane * (unsigned)crs * (unsigned)sizeof(CodeT);
    auto load_x = [&](int b, float* dst) {
#ifdef PQH_ASSIGN_NOMEM   // diagnostic: every chunk re-reads the first 64 blocks (cache hits)
        b &= 63;
#endif
        long long row0 = (long long)b * 32;
        unsigned off = xlane_off;
        if (b >= nfull) {   // (uniform) the last, partial block: rows past n read row n - 1
            row0 = row0 < n - 1 ? row0 : n - 1;
            const long long left = n - 1 - row0;
            const unsigned last = (unsigned)(left < 31 ? left : 31);
            off = __umul24(min((unsigned)r, last), ldx4) + xh_off;
        }
        const float* xp = reinterpret_cast<const float*>(xm + row0 * (long long)ldx4 + off);
        if constexpr (XD % 4 == 0) {
#pragma unroll
            for (int j = 0; j < XD; j += 4) {
                // (plain loads: the 8 subspaces read the two 64-B halves of each row's lines,
                // and non-temporal loads re-fetch the line per half -- 1.6x the HBM bytes)
                // HALF: piece j / 8 sits 16 dims after the previous one
                const f32x4 q = *reinterpret_cast<const f32x4*>(xp + (HALF ? 16 * (j >> 3) + (j & 7) : j));
                dst[j] = q.x; dst[j + 1] = q.y; dst[j + 2] = q.z; dst[j + 3] = q.w;
            }
        } else {
#pragma unroll
            for (int j = 0; j < XD; ++j) dst[j] = xp[j];
        }
    };
    // the same slices into xst[wave][slot] by LDS DMA (16 bytes per lane and piece)
    auto load_x_lds = [&](int b, int slot) {
#ifdef PQH_ASSIGN_NOMEM   // diagnostic: every chunk re-reads the first 64 blocks (cache hits)
        b &= 63;
#endif
        long long row0 = (long long)b * 32;
        unsigned off = xlane_off;
        if (b >= nfull) {
            row0 = row0 < n - 1 ? row0 : n - 1;
            const long long left = n - 1 - row0;
            const unsigned last = (unsigned)(left < 31 ? left : 31);
            off = __umul24(min((unsigned)r, last), ldx4) + xh_off;
        }
        const float* xp = reinterpret_cast<const float*>(xm + row0 * (long long)ldx4 + off);
#pragma unroll
        for (int j = 0; j < XD; j += 4) {
#if defined(__HIP_DEVICE_COMPILE__)   // (the host pass rejects the 16-byte form)
            __builtin_amdgcn_global_load_lds(
                xp + (HALF ? 16 * (j >> 3) + (j & 7) : j),
                (__attribute__((address_space(3))) void*)(&xst[wave][slot][j / 4][0]), 16, 0,
                PQH_ASSIGN_XAUX);
#else
            (void)xp;
#endif
        }
    };
    auto read_x_lds = [&](int slot, float* dst) {
#pragma unroll
        for (int j = 0; j < XD; j += 4) {
            const f32x4 q = *reinterpret_cast<const f32x4*>(&xst[wave][slot][j / 4][lane * 4]);
            dst[j] = q.x; dst[j + 1] = q.y; dst[j + 2] = q.z; dst[j + 3] = q.w;
        }
    };
    // (SHAREA) tile t's A fragments from the LDS ring, and one group's DMA into it: the group's
    // kAG * PA pieces of 1 KB (64 lanes x 16 B) spread over the workgroup's waves
    auto read_ring = [&](int t, bf16x8* a) {
#pragma unroll
        for (int p = 0; p < P::PA; ++p)
            a[p] = *reinterpret_cast<const bf16x8*>(&Ar[((t % kAR) * P::PA + p) * 64 + lane]);
    };
    auto dma_group = [&](int g) {
        if constexpr (kShareA) {
            const uint4* src = reinterpret_cast<const uint4*>(afrag) + (long long)m * P::PA * KT * 64;
            static_assert((kAG * P::PA) % kWavesPerWG == 0, "whole pieces per wave");
#pragma unroll
            for (int i = 0; i < (kAG * P::PA) / kWavesPerWG; ++i) {
                const int q = wave + i * kWavesPerWG;
                const int t = g * kAG + q / P::PA, p = q % P::PA;
#if defined(__HIP_DEVICE_COMPILE__)
                __builtin_amdgcn_global_load_lds(
                    src + (p * KT + t) * 64 + lane,
                    (__attribute__((address_space(3))) void*)(&Ar[((t % kAR) * P::PA + p) * 64]),
                    16, 0, 0);
#else
                (void)src; (void)t; (void)p;
#endif
            }
        }
    };
    // Deferred re-rank: a vector whose screening gap is too small is appended to this wave's
    // LDS queue and finished after the wave's last chunk (tail_rerank); only when the queue
    // is full, or x is not finite, does the wave re-rank inline.
    unsigned qn = 0;

    // One step = a chunk of kNB consecutive 32-vector blocks, screened together: each tile's
    // A fragments are read from LDS once for all kNB blocks, and the kNB independent MFMA
    // chains and key reductions give the SIMD work to overlap.  The kernel is VALU-issue
    // bound (a wave64 VALU instruction takes ~4 cycles of its SIMD), so the per-block work
    // outside the key reduction is kept to a few dozen instructions: the B operands come
    // straight from x by packed conversions, the lo pass is decided once per chunk (a lo pass
    // over bf16-exact x adds exact zeros, so the blocks without a remainder keep their exact
    // scores and their tighter bound), and the winner's tile rides in its key.
    auto body = [&](auto lo_c, long long blk0, float (*xs)[XD], const float* Xg,
                    const bool* any_lo) {
        constexpr bool LO = decltype(lo_c)::value;
        bf16x8 Bm[kNB][P::PM], Bl[kNB][P::PL];
#pragma unroll
        for (int b = 0; b < kNB; ++b) make_b<D, LO>(xs[b], h, Bm[b], Bl[b]);
        // The lane's 128 scores of a block form an 8 x 16 grid: tile t (row) x accumulator
        // register i (column).  Instead of ranking every score with its index attached, two
        // partitions of the grid are reduced on the raw score bits:
        //   P-groups (t, g): the 8 registers i in [8g, 8g + 8) of tile t -- 16 minima;
        //   Q-groups j:      registers j and j + 8 of every tile        -- 8 running minima.
        // A P-group and a Q-group share exactly one cell, so the smallest and second
        // smallest score of the lane are
        //   S1 = min P = min Q,   S2 = min(second min P, second min Q)
        // (if the runner-up shares the winner's P-group it lies in another Q-group, and vice
        // versa), and the winner's cell is (argmin P, argmin Q).  A score is touched by one
        // min3 of each partition -- 1 VALU per score instead of 2.25 for keys + tournament --
        // and only the 24 group minima get index bits (the winner's P-group in the low 4
        // bits, its Q-group as row bits in the low 4).
        unsigned pm1[kNB], pm2[kNB], qg[kNB][8];
        // streamed K = 4096: the P-groups span tile pairs and the Q-groups split by tile
        // parity (reduce_pair): qh = the odd tiles' Q minima, pp = the even tile's P minima
        unsigned qh[kNB][8], pp[kNB][2];
        auto load_a = [&](int t, bf16x8* a) {
#ifdef PQH_ASSIGN_KTNOMEM   // diagnostic: every tile re-reads tile t % 4 (cache hits)
            if constexpr (!kLdsA) t &= 3;
#endif
            if constexpr (kLdsA) {
#pragma unroll
                for (int p = 0; p < P::PA; ++p) a[p] = frag_at<KT>(asrc, p, t, lane);
            } else {
                // buffer loads: the tile's offset in a scalar register, the lane's constant
                // (no per-tile 64-bit address arithmetic on the VALU)
#pragma unroll
                for (int p = 0; p < P::PA; ++p) {
                    typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
                    const u32x4 v = __builtin_amdgcn_raw_buffer_load_b128(
                        arsrc, (int)((p * KT * 64 + lane) * 16), t * 1024, 0);
                    a[p] = __builtin_bit_cast(bf16x8, v);
                }
            }
        };
        // first: the tile that starts the running minima (compile-time in the unrolled
        // K = 256 loop; the streamed K = 4096 loop starts them at +inf instead)
        auto reduce = [&](const f32x16& acc, int t, int b, bool first) {
            unsigned a[16];
#pragma unroll
            for (int i = 0; i < 16; ++i) a[i] = __float_as_uint(acc[i]);
            // P: the tile's two group minima, keyed (P-group index 2t + g in the low 4 bits)
            // and folded into the running top two of the P keys
            // (e0, e1: the compiler-generated first reads of the tile's results, see min3d)
            const unsigned e0 = anchor_min(a[6], a[7], ninf), e1 = anchor_min(a[14], a[15], ninf);
            const unsigned k0 =
                (min3u(min3d(a[0], a[1], a[2], e0), min3d(a[3], a[4], a[5], e0), e0) & keymask) |
                (unsigned)(2 * t);
            const unsigned k1 =
                (min3u(min3d(a[8], a[9], a[10], e1), min3d(a[11], a[12], a[13], e1), e1) & keymask) |
                (PB == 4 ? (unsigned)(2 * t + 1) : opaque_s32(2 * t + 1));
            if (first) {
                pm1[b] = minu(k0, k1);
                pm2[b] = maxu(k0, k1);
            } else {
                fold2(pm1[b], pm2[b], k0, k1);
            }
            // Q: running minima of the register pairs (j, j + 8)
#pragma unroll
            for (int j = 0; j < 8; ++j)
                qg[b][j] = first ? min3d(a[j], a[j + 8], a[j + 8], e1)
                                 : min3d(qg[b][j], a[j], a[j + 8], e1);
        };
        // Streamed K = 4096, tiles 2s and 2s + 1 (par = t & 1): P-group (s, g) = registers
        // [8g, 8g + 8) of BOTH tiles (16 cells, one key and one top-two fold per pair of
        // tiles), Q-group (j, par) = registers j and j + 8 of the tiles of parity par; a P-
        // and a Q-group still share exactly one cell (tile 2s + par, register j + 8g).  The
        // even tile's two half minima wait in pp for the odd tile: 40 VALU per tile pair
        // instead of 44.
        auto reduce_pair = [&](const f32x16& acc, int t, int b, int par) {
            unsigned a[16];
#pragma unroll
            for (int i = 0; i < 16; ++i) a[i] = __float_as_uint(acc[i]);
            const unsigned e0 = anchor_min(a[6], a[7], ninf), e1 = anchor_min(a[14], a[15], ninf);
            if (par == 0) {
                pp[b][0] = min3u(min3d(a[0], a[1], a[2], e0), min3d(a[3], a[4], a[5], e0), e0);
                pp[b][1] = min3u(min3d(a[8], a[9], a[10], e1), min3d(a[11], a[12], a[13], e1), e1);
#pragma unroll
                for (int j = 0; j < 8; ++j) qg[b][j] = min3d(qg[b][j], a[j], a[j + 8], e1);
            } else {
                const unsigned w0 =
                    minu(min3u(pp[b][0], min3d(a[0], a[1], a[2], e0), min3d(a[3], a[4], a[5], e0)), e0);
                const unsigned w1 =
                    minu(min3u(pp[b][1], min3d(a[8], a[9], a[10], e1), min3d(a[11], a[12], a[13], e1)), e1);
                // P index 2s + g = t - 1 + g (7 bits)
                const unsigned k0 = (w0 & keymask) | opaque_s32(t - 1);
                const unsigned k1 = (w1 & keymask) | opaque_s32(t);
                fold2(pm1[b], pm2[b], k0, k1);
#pragma unroll
                for (int j = 0; j < 8; ++j) qh[b][j] = min3d(qh[b][j], a[j], a[j + 8], e1);
            }
        };
        // Software pipeline over the tiles: block b's MFMA chain for tile t + 1 is issued
        // right after its tile-t keys are reduced, so it runs while the other block's keys
        // are (the scheduling barriers keep the compiler from sinking the chain behind them).
        f32x16 acc[kNB];
#ifdef PQH_ASSIGN_PF2
        // experiment: A fragments and ||c||^2 read two tiles ahead (double-buffered operands)
        if constexpr (kLdsA) {
            bf16x8 a[2][P::PA];
            f32x16 cn[2];
            load_a(0, a[0]);
            cn[0] = tile_norms(Cn, 0, h);
            load_a(1, a[1]);
            cn[1] = tile_norms(Cn, 1, h);
#pragma unroll
            for (int b = 0; b < kNB; ++b) acc[b] = tile_scores_a<D>(a[0], Bm[b], Bl[b], LO, cn[0]);
#pragma unroll
            for (int t = 0; t < KT; ++t) {
                // buffer t & 1 (tile t) was consumed by MFMAs already issued: refill it with
                // tile t + 2 while tile t + 1's MFMAs read the other buffer
                if (t + 2 < KT) {
                    load_a(t + 2, a[t & 1]);
                    cn[t & 1] = tile_norms(Cn, t + 2, h);
                }
                __builtin_amdgcn_sched_barrier(0);
#pragma unroll
                for (int b = 0; b < kNB; ++b) {
                    reduce(acc[b], t, b, t == 0);
                    if (t + 1 < KT)
                        acc[b] = tile_scores_a<D>(a[(t + 1) & 1], Bm[b], Bl[b], LO, cn[(t + 1) & 1]);
                    __builtin_amdgcn_sched_barrier(0);
                }
            }
        } else
#endif
        if constexpr (kLdsA) {
            bf16x8 a[P::PA];
            load_a(0, a);
            f32x16 cn = tile_norms(Cn, 0, h);
#pragma unroll
            for (int b = 0; b < kNB; ++b) acc[b] = tile_scores_a<D>(a, Bm[b], Bl[b], LO, cn);
#pragma unroll
            for (int t = 0; t < KT; ++t) {
                if (t + 1 < KT) {
                    load_a(t + 1, a);
                    cn = tile_norms(Cn, t + 1, h);
                }
#pragma unroll
                for (int b = 0; b < kNB; ++b) {
                    reduce(acc[b], t, b, t == 0);
                    if (t + 1 < KT) acc[b] = tile_scores_a<D>(a, Bm[b], Bl[b], LO, cn);
                    __builtin_amdgcn_sched_barrier(0);
                }
            }
        } else if constexpr (kShareA) {
            // the LDS ring: group g + 1 was requested a group ago; at the last tile of group g
            // every wave has issued the MFMAs that read group g, so after the barrier group
            // g's slots take group g + 2 (past the last group: the next chunk's 0 and 1)
            constexpr int NG = KT / kAG;
#pragma unroll
            for (int b = 0; b < kNB; ++b) {
                pm1[b] = pm2[b] = 0x7F800000u;
#pragma unroll
                for (int j = 0; j < 8; ++j) qg[b][j] = qh[b][j] = 0x7F800000u;
            }
            bf16x8 a[P::PA];
            read_ring(0, a);
            f32x16 cn = tile_norms(Cn, 0, h);
#pragma unroll
            for (int b = 0; b < kNB; ++b) acc[b] = tile_scores_a<D>(a, Bm[b], Bl[b], LO, cn);
#pragma unroll 1
            for (int g = 0; g < NG; ++g) {
#pragma unroll
                for (int u = 0; u < kAG; ++u) {
                    const int t = g * kAG + u;
                    if (u == kAG - 1) {
                        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // this wave's DMAs
                        lds_barrier();                                      // everyone's
                        dma_group(g + 2 < NG ? g + 2 : g + 2 - NG);
                    }
                    // (past the last tile: the next chunk's tile 0, whose scores are never
                    // reduced -- an unconditional MFMA keeps the accumulators in place)
                    read_ring((t + 1) & (KT - 1), a);
                    cn = tile_norms(Cn, (t + 1) & (KT - 1), h);
#pragma unroll
                    for (int b = 0; b < kNB; ++b) {
                        reduce_pair(acc[b], t, b, u & 1);
                        acc[b] = tile_scores_a<D>(a, Bm[b], Bl[b], LO, cn);
                        __builtin_amdgcn_sched_barrier(0);
                    }
                }
            }
        } else {
            // A fragments from L2 into a ring of kRing tile sets, kRing - 1 tiles ahead of use
            constexpr int kRing = PQH_ASSIGN_RING;
            static_assert(KT % kRing == 0, "the ring unrolls the tile loop");
#pragma unroll
            for (int b = 0; b < kNB; ++b) {
                pm1[b] = pm2[b] = 0x7F800000u;   // +inf: any key is smaller
#pragma unroll
                for (int j = 0; j < 8; ++j) qg[b][j] = qh[b][j] = 0x7F800000u;
            }
            static_assert(kRing % 2 == 0, "tile pairs within a ring turn");
            bf16x8 ar[kRing][P::PA];
#pragma unroll
            for (int u = 0; u < kRing - 1; ++u) load_a(u, ar[u]);
            f32x16 cn = tile_norms(Cn, 0, h);
#pragma unroll
            for (int b = 0; b < kNB; ++b) acc[b] = tile_scores_a<D>(ar[0], Bm[b], Bl[b], LO, cn);
#pragma unroll 1
            for (int t0 = 0; t0 < KT; t0 += kRing) {
#pragma unroll
                for (int u = 0; u < kRing; ++u) {
                    const int t = t0 + u;
                    // unconditional: past the last tile the ring wraps to tiles 0, 1, ...
                    // whose scores are never reduced (a conditional load or MFMA made the
                    // compiler copy the accumulators at every ring turn)
                    load_a((t + kRing - 1) & (KT - 1), ar[(u + kRing - 1) % kRing]);
                    cn = tile_norms(Cn, (t + 1) & (KT - 1), h);
#pragma unroll
                    for (int b = 0; b < kNB; ++b) {
                        reduce_pair(acc[b], t, b, u & 1);
                        acc[b] = tile_scores_a<D>(ar[(u + 1) % kRing], Bm[b], Bl[b], LO, cn);
                        __builtin_amdgcn_sched_barrier(0);
                    }
                }
            }
        }
        // the lane's 128 centroids per block: keyed group minima, top two of each partition,
        // and the winner's row bits from its two keys
        unsigned own1[kNB], own2[kNB], cbits[kNB];
#pragma unroll
        for (int b = 0; b < kNB; ++b) {
            if constexpr (kLdsA) {
                unsigned qk[8];
#pragma unroll
                for (int j = 0; j < 8; ++j) qk[j] = (qg[b][j] & ~15u) | q_code_bits(j);
                unsigned q1, q2;
                top2_8(qk, q1, q2);
                own1[b] = pm1[b];
                own2[b] = minu(pm2[b], q2);
                // the winner's row (tile_row): 16 (2t + g) from its P key, the rest from its Q key
                cbits[b] = ((pm1[b] & PMASK) << 4) | (q1 & 15u) | ((unsigned)h << 2);
            } else {
                // 16 Q keys: (j, par) with the row bits 32 par + q_code_bits(j) (6 bits)
                unsigned qe[8], qo[8];
#pragma unroll
                for (int j = 0; j < 8; ++j) {
                    qe[j] = (qg[b][j] & ~63u) | q_code_bits(j);
                    qo[j] = (qh[b][j] & ~63u) | 32u | q_code_bits(j);
                }
                unsigned e1_, e2_, o1_, o2_;
                top2_8(qe, e1_, e2_);
                top2_8(qo, o1_, o2_);
                const unsigned q1 = minu(e1_, o1_);
                const unsigned q2 = min3u(maxu(e1_, o1_), e2_, o2_);
                own1[b] = pm1[b];
                own2[b] = minu(pm2[b], q2);
                // row 64 s + 16 g (P index 2s + g) + 32 par + (j & 3) + 8 (j >> 2) + 4 h
                const unsigned pi = pm1[b] & PMASK;
                cbits[b] = ((pi >> 1) << 6) | ((pi & 1u) << 4) | (q1 & 63u) | ((unsigned)h << 2);
            }
        }
        // The two half-waves hold the two halves of a vector's centroids.  Blocks are merged
        // in pairs by one v_permlane32_swap per value: swap(block b0's, block b0 + 1's) leaves
        // both halves of block b0's vector r in lane r and both halves of block b0 + 1's in
        // lane r + 32 (s[0]: the lower half's value, s[1]: the upper's), so everything after
        // the merge -- gap test, re-rank decision, store, histogram -- runs once per vector
        // on all 64 lanes.  (An odd block count merges its last block with itself: both
        // halves then hold the same vector and the lower half stores.)
        constexpr int NG = (kNB + 1) / 2;
#pragma unroll
        for (int g = 0; g < NG; ++g) {
            const int ba = 2 * g, bb = 2 * g + 1 < kNB ? 2 * g + 1 : 2 * g;
            const bool pair = ba != bb;
            const auto s1 = __builtin_amdgcn_permlane32_swap(own1[ba], own1[bb], false, false);
            const auto s2 = __builtin_amdgcn_permlane32_swap(own2[ba], own2[bb], false, false);
            const auto sc = __builtin_amdgcn_permlane32_swap(cbits[ba], cbits[bb], false, false);
            const unsigned b1 = minu((unsigned)s1[0], (unsigned)s1[1]);
            const unsigned b2 = minu(minu((unsigned)s2[0], (unsigned)s2[1]),
                                     maxu((unsigned)s1[0], (unsigned)s1[1]));
            // (equal keys in the two halves: K2 = K1, the gap test fails, the slow path decides)
            // (keys order as floats: the lower half won iff its key is the minimum)
            int code = (int)((unsigned)s1[0] == b1 ? (unsigned)sc[0] : (unsigned)sc[1]);
            // the lane's vector: block ba + h (pair) or ba, row r
            const long long rowl = (blk0 + ba) * 32 + (pair ? lane : r);
            const bool valid = rowl < n;   // rows past n hold row n - 1 (clamped loads)
            const bool own_lane = pair || h == 0;
            const float Xl = Xg[g];
            const bool finite = isfinite(Xl);
            const float tau = screen_tau(Xl, pair && h ? any_lo[bb] : any_lo[ba], tq);
            // a key differs from its score by less than 2^PB ulp (2^(PB-23) relative):
            // 2^(PB-21) of the larger magnitude covers both keys of the gap (and the rounding
            // of K2 - K1)
            constexpr float kKeySlack = PB == 4 ? 0x1p-17f : 0x1p-13f;
            const float K1 = __uint_as_float(b1), K2 = __uint_as_float(b2);
            const float KA = max_abs(K1, K2);
            const bool slow = !(K2 - K1 > fmaf(kKeySlack, KA, tau)) || !finite;

            unsigned long long need = __ballot(slow && valid && own_lane);
            bool deferred = false;
            if (need) {
                slow_count += __popcll(need);
                // finite vectors go to the queue with their candidate window: every centroid
                // that can be the fp32 argmin (or tie with it) screens below
                // K1 + tau + 2^-16 |K1| -- see the tail; non-finite ones stay inline
                const unsigned long long fin = need & __ballot(finite);
                const unsigned cnt = (unsigned)__popcll(fin);
                if (PQH_ASSIGN_DEFER && cnt && qn + cnt <= (unsigned)kRqLds) {
                    if (slow && valid && own_lane && finite) {
                        const float thr = fmaf(2.0f * kKeySlack, fabsf(K1), K1 + tau);
                        rqs[wave][qn + __builtin_amdgcn_mbcnt_hi((unsigned)(fin >> 32),
                                      __builtin_amdgcn_mbcnt_lo((unsigned)fin, 0u))] =
                            make_uint2((uint32_t)rowl, __float_as_uint(thr));
                    }
                    qn += cnt;
                    deferred = finite;
                    need &= ~fin;
                }
                unsigned long long todo = need;
                while (todo) {   // inline exact re-rank: non-finite x, or a full queue
                    const int rs = __ffsll((long long)todo) - 1;
                    todo &= todo - 1;
                    float xv[D];   // the vector's slice, re-read (a uniform address)
                    const long long vrow = (blk0 + ba) * 32 + (pair ? rs : (rs & 31));
                    const float* xr = x + vrow * ldx + (long long)m * D;
#pragma unroll
                    for (int j = 0; j < D; ++j) xv[j] = xr[j];
                    float best = INFINITY;
                    int bidx = 0x7FFFFFFF;
#pragma unroll 1
                    for (int q = 0; q < K / 64; ++q) {   // rare path: keep its registers few
                        const int c = lane + 64 * q;
                        const float dd = exact_dist<D>(xv, cl + c * D);
                        if (dd < best) { best = dd; bidx = c; }
                    }
#pragma unroll
                    for (int off = 32; off >= 1; off >>= 1) {
                        const float ob = __shfl_xor(best, off);
                        const int oi = __shfl_xor(bidx, off);
                        if (ob < best || (ob == best && oi < bidx)) { best = ob; bidx = oi; }
                    }
                    if (lane == rs) code = bidx == 0x7FFFFFFF ? 0 : bidx;
                }
            }
            // every lane stores its vector's code (the lower half only for a self-merged
            // block), unless the vector waits in the queue
            if (valid && own_lane && !(slow && deferred)) {
                *reinterpret_cast<CodeT*>(reinterpret_cast<char*>(cbase + (blk0 + ba) * 32 * crs) +
                                          (pair ? code_pair_off : code_lane_off)) = (CodeT)code;
                if (kLdsA && counts) atomicAdd(&hist(wave)[code], 1u);
            }
        }
    };
    // per chunk: ||x||^2, finiteness and bf16 remainders of its blocks, then the tile loop
    // with or without the lo pass
    auto step = [&](long long blk0, float (*xs)[XD]) {
#ifdef PQH_ASSIGN_NOCOMPUTE   // diagnostic: the kernel's memory traffic alone
#pragma unroll
        for (int b = 0; b < kNB; ++b) {
            const long long vv = (blk0 + b) * 32 + r;
            float q = 0.0f;
#pragma unroll
            for (int j = 0; j < XD; ++j) q += xs[b][j];
            if (vv < n && h == 0) cbase[vv * crs] = (CodeT)(int)q;
        }
        return;
#endif
        // ||x||^2 of the lane's vector after the block merge (see body): a pair's partial sums
        // are merged by the same swap as the keys (lower + upper, bitwise norm_x's sum)
        constexpr int NG = (kNB + 1) / 2;
        float Xg[NG];
        bool any_lo[kNB];
        bool chunk_lo = false;
#pragma unroll
        for (int g = 0; g < NG; ++g) {
            const int ba = 2 * g, bb = 2 * g + 1 < kNB ? 2 * g + 1 : 2 * g;
            if (ba == bb) {
                Xg[g] = norm_x<D>(xs[ba]);
            } else if constexpr (Slice<D>::HALF) {
                const auto sw = __builtin_amdgcn_permlane32_swap(
                    __float_as_uint(norm_part<D>(xs[ba])), __float_as_uint(norm_part<D>(xs[bb])),
                    false, false);
                Xg[g] = __uint_as_float(sw[0]) + __uint_as_float(sw[1]);
            } else {
                const float xa_ = norm_x<D>(xs[ba]), xb_ = norm_x<D>(xs[bb]);
                Xg[g] = h ? xb_ : xa_;
            }
        }
#pragma unroll
        for (int b = 0; b < kNB; ++b) {
            any_lo[b] = __any(has_lo<D>(xs[b]));
            chunk_lo |= any_lo[b];
        }
        if (chunk_lo)
            body(std::true_type{}, blk0, xs, Xg, any_lo);
        else
            body(std::false_type{}, blk0, xs, Xg, any_lo);
    };

    // Chunk schedule (a chunk = kNB blocks = one step).  Wave w of the subspace (w = bx
    // * kWavesPerWG + wave) starts on chunk w.  sched == nullptr: static stride over chunks.
    // Otherwise the remaining chunks are handed out by tickets, so waves that share their CU
    // with other work (a concurrent stream) simply take fewer chunks.  The dynamic region is
    // split into kXcds ranges with a head each; a wave drains the range of the XCD it runs on
    // first (XCC_ID; placement only affects speed), then moves on to the next range -- one
    // shared head per subspace saturated at a few dequeues per microsecond.  The ticket for
    // the next chunk is requested a whole step ahead, and the next chunk's x is loaded
    // during the current one.
    const int wave_id = bx * kWavesPerWG + wave;
    const int waves_m = gx * kWavesPerWG;
    const int nchunk = (nblk + kNB - 1) / kNB;
    const int R = nchunk > waves_m ? (nchunk - waves_m + kXcds - 1) / kXcds : 0;
    uint32_t* head = sched && !kShareA ? sched + (long long)m * kXcds * kSchedStride : nullptr;
    int xr = head ? (int)(__builtin_amdgcn_s_getreg((3 << 11) | 20) & (kXcds - 1)) : 0;
    int tries = head && R > 0 ? 0 : kXcds;
    auto ticket = [&]() -> unsigned {
        unsigned t = __builtin_nondeterministic_value(0u);   // lane 0 only: no select,
                                                             // so no wait at the join
        if (lane == 0)
            t = __hip_atomic_fetch_add(head + xr * kSchedStride, 1u, __ATOMIC_RELAXED,
                                       __HIP_MEMORY_SCOPE_AGENT);
        return t;
    };
    unsigned traw = 0;
    if (tries < kXcds) traw = ticket();
    auto next_dyn = [&]() -> int {
        while (tries < kXcds) {
            const int t = (int)__builtin_amdgcn_readfirstlane(traw);
            const int lo = waves_m + xr * R;
            if (t < std::min(R, nchunk - lo)) {
                traw = ticket();           // prefetch the one after
                return lo + t;
            }
            if (++tries < kXcds) {         // this range is empty: the next XCD's
                xr = (xr + 1) & (kXcds - 1);
                traw = ticket();
            }
#ifdef PQH_ASSIGN_ENDPRIO   // (experiment) the end phase: waves past their home range first
            __builtin_amdgcn_s_setprio(PQH_ASSIGN_ENDPRIO);
#endif
        }
        return -1;
    };
    // One batch of queued vectors (lane r: entry r; invalid lanes idle): re-screen, collect
    // the candidates at or below the entry's threshold, evaluate them exactly (see the tail).
    auto rerank32 = [&](const uint2 ent, const bool valid) {
#ifdef PQH_ASSIGN_STAMPS
        const unsigned long long rr0 = __builtin_amdgcn_s_memrealtime();
#endif
        const long long v = (long long)ent.x;
        const float thr = __uint_as_float(ent.y);
        float xv[D];
        const float* xp = x + v * ldx + (long long)m * D;
        if constexpr (D % 4 == 0) {
#pragma unroll
            for (int j = 0; j < D; j += 4) {
                const float4 q = *reinterpret_cast<const float4*>(xp + j);
                xv[j] = q.x; xv[j + 1] = q.y; xv[j + 2] = q.z; xv[j + 3] = q.w;
            }
        } else {
#pragma unroll
            for (int j = 0; j < D; ++j) xv[j] = xp[j];
        }
        float xs[XD];
#pragma unroll
        for (int j = 0; j < XD; ++j)   // (static indices: a dynamic one puts xv in scratch)
            xs[j] = valid ? (h ? xv[Slice<D>::dim(j, 1)] : xv[Slice<D>::dim(j, 0)]) : 0.0f;
        float X;
        bool lo;
        float xh[XD], xl[XD];
        split_x<D>(xs, X, lo, xh, xl);
#ifdef PQH_ASSIGN_STAMPS
        unsigned long long rr1, rr2, rr3;
        asm volatile("" ::"v"(X), "v"(xh[0]));
        PQH_RR_STAMP(rr1);
        rr_x += rr1 - rr0;
#endif
        bf16x8 Bm[P::PM];
        bf16x8 Bl[P::PL];
        build_b<D>(xh, xl, h, Bm, Bl);
        const bool lo_pass = __any(lo);
        float best = INFINITY;
        int bidx = 0x7FFFFFFF;
        // Eight tiles at a time: screen them all (a candidate bit mask per tile pair), then
        // evaluate the candidates kCand per lane per round, their centroid rows loaded
        // together -- the tail's time is L2 round trips, so they are few (one or two rounds
        // per vector instead of one per tile holding a candidate).
        constexpr int kGT = KT < 8 ? KT : 8;
        constexpr int kCand = D <= 16 ? 4 : 2;
#pragma unroll 1
        for (int t0 = 0; t0 < KT; t0 += kGT) {
            uint32_t cw[(kGT + 1) / 2];   // tiles t0 + 2w (bits 0-15) and t0 + 2w + 1 (16-31)
#pragma unroll
            for (int w = 0; w < (kGT + 1) / 2; ++w) cw[w] = 0u;
#pragma unroll 1
            for (int u = 0; u < kGT; ++u) {   // (rolled: the tail keeps its registers few)
                const f32x16 acc = tile_scores<D, KT>(asrc, Cn, lane, t0 + u, Bm, Bl, lo_pass);
                uint32_t bits = 0;
#pragma unroll
                for (int i = 0; i < 16; ++i) bits |= (acc[i] <= thr ? 1u : 0u) << i;
                bits = (valid ? bits : 0u) << (16 * (u & 1));
#pragma unroll
                for (int w = 0; w < (kGT + 1) / 2; ++w) cw[w] |= w == (u >> 1) ? bits : 0u;
            }
#ifdef PQH_ASSIGN_STAMPS
            asm volatile("" ::"v"(cw[0]));
            PQH_RR_STAMP(rr2);
            rr_scr += rr2 - rr1;
#endif
            for (;;) {
                int kc[kCand];
                bool hc[kCand];
#pragma unroll
                for (int c = 0; c < kCand; ++c) {   // the lane's next candidate, if any
                    hc[c] = false;
                    kc[c] = 0;
#pragma unroll
                    for (int w = 0; w < (kGT + 1) / 2; ++w) {
                        if (!hc[c] && cw[w]) {
                            const int i = __builtin_ctz(cw[w]);
                            cw[w] &= cw[w] - 1;
                            hc[c] = true;
                            kc[c] = tile_row(t0 + 2 * w + (i >> 4), i & 15, h);
                        }
                    }
                }
                if (!__any(hc[0])) break;
#ifdef PQH_ASSIGN_STAMPS
                ++rr_rounds;
#endif
                float cr[kCand][D];   // (lanes without a candidate read row 0)
#pragma unroll
                for (int c = 0; c < kCand; ++c) {
                    const float* cp = cl + kc[c] * D;
                    if constexpr (D % 4 == 0) {
#pragma unroll
                        for (int j = 0; j < D; j += 4) {
                            const float4 q = *reinterpret_cast<const float4*>(cp + j);
                            cr[c][j] = q.x; cr[c][j + 1] = q.y; cr[c][j + 2] = q.z; cr[c][j + 3] = q.w;
                        }
                    } else {
#pragma unroll
                        for (int j = 0; j < D; ++j) cr[c][j] = cp[j];
                    }
                }
#pragma unroll
                for (int c = 0; c < kCand; ++c) {
                    const float dd = exact_dist<D>(xv, cr[c]);
                    const int k = kc[c];
                    if (hc[c] && (dd < best || (dd == best && k < bidx))) { best = dd; bidx = k; }
                }
            }
#ifdef PQH_ASSIGN_STAMPS
            asm volatile("" ::"v"(best));
            PQH_RR_STAMP(rr3);
            rr_cand += rr3 - rr2;
            rr1 = rr3;
#endif
        }
        const float ob = __uint_as_float(partner32(__float_as_uint(best)));
        const int oi = (int)partner32((unsigned)bidx);
        if (ob < best || (ob == best && oi < bidx)) { best = ob; bidx = oi; }
        if (valid && h == 0) {
            const int code = bidx == 0x7FFFFFFF ? 0 : bidx;
            cbase[v * crs] = (CodeT)code;
            if (kLdsA && counts) atomicAdd(&hist(wave)[code], 1u);
        }
#ifdef PQH_ASSIGN_STAMPS
        rr_ticks += __builtin_amdgcn_s_memrealtime() - rr0;
        ++rr_batches;
#endif
    };
    if constexpr (kShareA) {
        // lockstep waves: workgroup bx takes super-chunks sc = bx, bx + gx, ... of kWavesPerWG
        // chunks, wave w chunk kWavesPerWG sc + w (past nchunk: clamped rows, nothing stored)
        const int nsuper = (nchunk + kWavesPerWG - 1) / kWavesPerWG;
        int sc = bx;
        dma_group(0);
        dma_group(1);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        lds_barrier();
        int chs = sc * kWavesPerWG + wave;
        float xq[kNB][XD];
#pragma unroll
        for (int b = 0; b < kNB; ++b) load_x(chs * kNB + b, xq[b]);
        while (sc < nsuper) {   // (uniform in the workgroup)
            float xa[kNB][XD];
#pragma unroll
            for (int b = 0; b < kNB; ++b)
#pragma unroll
                for (int j = 0; j < XD; ++j) xa[b][j] = xq[b][0 * j + j];
            const int nsc = sc + gx;
            const int nch = nsc * kWavesPerWG + wave;
            const int pre = nsc < nsuper ? nch : chs;   // branch-free: re-load at the end
#pragma unroll
            for (int b = 0; b < kNB; ++b) load_x(pre * kNB + b, xq[b]);
            step((long long)chs * kNB, xa);
            while (qn >= 32u) {
                rerank32(rqs[wave][qn - 32u + (unsigned)r], true);
                qn -= 32u;
            }
            sc = nsc;
            chs = nch;
        }
        // (the last group barrier requested the next chunk's first tiles: let them land
        // before the workgroup's LDS is released)
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    int ch = kShareA ? nchunk : wave_id;
    float xn[kXLds ? 1 : kNB][XD];
#pragma unroll
    for (int b = 0; b < kNB; ++b) {
        if constexpr (kXLds)
            load_x_lds(ch * kNB + b, b);
        else
            load_x(ch * kNB + b, xn[b]);
    }
    while (ch < nchunk) {
        float xa[kNB][XD];
        if constexpr (kXLds) {
#pragma unroll
            for (int b = 0; b < kNB; ++b) read_x_lds(b, xa[b]);
            // the slices are in registers before the next chunk's DMA overwrites them (a DMA
            // write is not ordered with this wave's LDS reads)
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        } else {
#pragma unroll
            for (int b = 0; b < kNB; ++b)
#pragma unroll
                for (int j = 0; j < XD; ++j) xa[b][j] = xn[b][0 * j + j];
        }
        int nc;
        if (!head) {
            nc = ch + waves_m;
        } else {
            const int c = next_dyn();
            nc = c < 0 ? nchunk : c;
        }
        const int pre = nc < nchunk ? nc : ch;   // branch-free: re-load at the end
#pragma unroll
        for (int b = 0; b < kNB; ++b) {
            if constexpr (kXLds)
                load_x_lds(pre * kNB + b, b);
            else
                load_x(pre * kNB + b, xn[b]);
        }
        step((long long)ch * kNB, xa);
        while (qn >= 32u) {   // full batches of deferred vectors: done while the SIMD is busy
            rerank32(rqs[wave][qn - 32u + (unsigned)r], true);
            qn -= 32u;
        }
#ifdef PQH_ASSIGN_STAMPS
        nbdone += kNB;
#endif
        ch = nc;
    }
#ifdef PQH_ASSIGN_STAMPS
    const unsigned long long rt_loop = __builtin_amdgcn_s_memrealtime();
#endif
    // Tail: this wave's queued vectors, 32 at a time.  thr = K1 + tau + 2^-16 |K1| bounds the
    // screened score of every centroid whose fp32 direct-form distance can equal the minimum
    // (S_k <= D_k - X + E0 <= D_min - X + E0 <= S_k1 + 2 E0 <= K1 + 2^-19 |K1| + 2 E0 < thr):
    // the vectors are re-screened with the main loop's own instruction sequence (bitwise the
    // same scores: same norms, and a lo pass adds exact zeros for bf16-exact x), the centroids
    // screening at or below thr are collected per lane, and only those few are evaluated in
    // exact fp32 direct form (first index among equal distances) -- instead of all K.
    // Full batches were finished in the chunk loop (while the SIMD had other waves to run);
    // the wave's last, partial batch runs here, without waiting for the workgroup's other waves.
#ifdef PQH_ASSIGN_TAILPRIO   // (experiment) the re-rank tail ahead of other waves' main loops
    __builtin_amdgcn_s_setprio(PQH_ASSIGN_TAILPRIO);
#endif
    if (qn) {   // (qn < 32 here)
        const bool valid = (unsigned)r < qn;
        rerank32(valid ? rqs[wave][r] : make_uint2(0u, 0u), valid);
    }
#ifdef PQH_ASSIGN_STAMPS
    {
        const unsigned gw = (unsigned)((m * gx + bx) * kWavesPerWG + wave);
        if (lane == 0 && gw < (unsigned)kStampWaves) {
            g_assign_rr[gw][0] = rr_x;
            g_assign_rr[gw][1] = rr_scr;
            g_assign_rr[gw][2] = rr_cand;
            g_assign_rr[gw][3] = rr_rounds;
            g_assign_stamps[gw][0] = rt0;   // 100 MHz, chip-wide
            g_assign_stamps[gw][1] = __builtin_amdgcn_s_memrealtime();
            g_assign_stamps[gw][2] = nbdone | ((__builtin_amdgcn_s_memtime() - st0) << 16);
            g_assign_stamps[gw][3] = (__builtin_amdgcn_s_getreg((3 << 11) | 20) & 15) |
                                     ((rt_loop - rt0) << 8) |   // chunk loop done
                                     (rr_ticks << 32) | (rr_batches << 56);   // re-rank batches
        }
    }
#endif
    if (kLdsA && counts) {
        __builtin_amdgcn_wave_barrier();
        for (int i = lane; i < K; i += 64) {
            uint32_t c = hist(wave)[i];
            if (c) atomicAdd(&counts[(long long)m * K + i], c);
        }
    }
    if (lane == 0 && slow_count) atomicAdd(rerank, slow_count);
}

// Exact VALU kernel: one thread per (vector, part); any K, any dsub.  Used for shapes the
// MFMA kernel is not instantiated for, for inputs with non-finite centroids, and as the
// independent cross-check of the MFMA kernel in the GPU tests.
template <typename CodeT>
__global__ void pq_assign_exact(const float* __restrict__ x, long long n, long long ldx, int m_total,
                                int k, int dsub, const float* __restrict__ cent,
                                CodeT* __restrict__ codes, uint32_t* __restrict__ counts,
                                long long ldc) {
#pragma clang fp contract(off)
    const long long gid = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (gid >= n * m_total) return;
    const long long v = gid / m_total;
    const int m = (int)(gid % m_total);
    const float* xp = x + v * ldx + (long long)m * dsub;
    const float* cb = cent + (long long)m * k * dsub;
    float best = INFINITY;
    int code = 0;
    for (int c = 0; c < k; ++c) {
        float acc = 0.0f;
        for (int j = 0; j < dsub; ++j) {
            float d = __fsub_rn(xp[j], cb[(long long)c * dsub + j]);
            acc = __fadd_rn(acc, __fmul_rn(d, d));
        }
        if (acc < best) { best = acc; code = c; }
    }
    codes[ldc ? (long long)m * ldc + v : gid] = (CodeT)code;   // (ldc: part-major)
    if (counts) atomicAdd(&counts[(long long)m * k + code], 1u);
}

// Reconstruction error partial sums (pq_encoder.c:82-119): per (vector) double sums,
// reduced per block; host adds the block sums in order.
template <typename CodeT>
__global__ void pq_error_kernel(const float* __restrict__ x, long long n, long long ldx, int m_total,
                                int k, int dsub, const float* __restrict__ cent,
                                const CodeT* __restrict__ codes, double* __restrict__ partial) {
#pragma clang fp contract(off)
    __shared__ double red[256];
    const long long v = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    double s = 0.0;
    if (v < n) {
        for (int i = 0; i < m_total; ++i) {
            const float* c = cent + ((long long)i * k + codes[v * m_total + i]) * dsub;
            for (int j = 0; j < dsub; ++j) {
                float delta = __fsub_rn(x[v * ldx + (long long)i * dsub + j], c[j]);
                s += (double)delta * (double)delta;
            }
        }
    }
    red[threadIdx.x] = s;
    __syncthreads();
    for (int w = 128; w > 0; w >>= 1) {
        if ((int)threadIdx.x < w) red[threadIdx.x] += red[threadIdx.x + w];
        __syncthreads();
    }
    if (threadIdx.x == 0) partial[blockIdx.x] = red[0];
}

template <typename CodeT>
__global__ void pq_reconstruct_kernel(const CodeT* __restrict__ codes, long long n, int m_total,
                                      int k, int dsub, const float* __restrict__ cent,
                                      float* __restrict__ out, long long ldo) {
    const long long gid = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    const long long d = (long long)m_total * dsub;
    if (gid >= n * d) return;
    const long long v = gid / d;
    const int col = (int)(gid % d);
    const int i = col / dsub, j = col % dsub;
    out[v * ldo + col] = cent[((long long)i * k + codes[v * m_total + i]) * dsub + j];
}

uint16_t bf16_rne(float f) {
    uint32_t u;
    memcpy(&u, &f, 4);
    if ((u & 0x7F800000u) == 0x7F800000u) return (uint16_t)(u >> 16);  // inf/nan
    u += 0x7FFFu + ((u >> 16) & 1u);
    return (uint16_t)(u >> 16);
}

float bf16_to_f(uint16_t b) {
    uint32_t u = (uint32_t)b << 16;
    float f;
    memcpy(&f, &u, 4);
    return f;
}

}  // namespace

struct pqh_pq {
    pqh_ctx* ctx = nullptr;
    int m = 0, k = 0, dsub = 0;
    bool mfma_ok = false;
    float* d_cent = nullptr;
    bf16x8* d_afrag = nullptr;
    float* d_cn = nullptr;     // ||c||^2 in accumulator order, [m][tile][half][16]
    float* d_cmax = nullptr;
    float* d_sqc = nullptr;
};

namespace {

// A[row][slot] of one subspace for the pass layout of Plan<D> (-2 ch | -2 cl, both exact
// bf16) and the rows' ||c||^2 in accumulator order (the C operand of each tile's chain)
template <int D>
void build_afrag(const float* c, int k, std::vector<uint16_t>& out, std::vector<float>& cn,
                 int m, float& cmax_out, float& r2_out) {
    using P = Plan<D>;
    const int slots = 16 * P::PM;
    std::vector<uint16_t> main((size_t)k * slots, 0);
    std::vector<double> norm(k);
    double cmax = 0.0, rmax = 0.0;
    for (int row = 0; row < k; ++row) {
        const float* cr = c + (size_t)row * D;
        double q = 0.0, rq = 0.0;
        for (int j = 0; j < D; ++j) {
            q += (double)cr[j] * (double)cr[j];
            uint16_t hi = bf16_rne(cr[j]);
            uint16_t lw = bf16_rne(cr[j] - bf16_to_f(hi));
            main[(size_t)row * slots + j] = bf16_rne(-2.0f * bf16_to_f(hi));       // exact
            main[(size_t)row * slots + D + j] = bf16_rne(-2.0f * bf16_to_f(lw));   // exact
            // the split's remainder r' (exact in double: three floats' sum)
            const double r = (double)cr[j] - (double)bf16_to_f(hi) - (double)bf16_to_f(lw);
            rq += r * r;
        }
        norm[row] = q;
        cmax = q > cmax ? q : cmax;
        rmax = rq > rmax ? rq : rmax;
    }
    cmax_out = (float)(cmax * (1.0 + 1e-6)) + 1e-30f;
    // 2 max_k ||r'_k||, rounded up (the 1e-6 covers the double sum and root)
    r2_out = (float)(2.0 * std::sqrt(rmax) * (1.0 + 1e-6)) + 1e-30f;
    // fragment order [m][PA][tile][lane][8]
    const int kt = k / 32;
    const size_t base = (size_t)m * P::PA * kt * 64 * 8;
    for (int p = 0; p < P::PA; ++p)
        for (int t = 0; t < kt; ++t)
            for (int lane = 0; lane < 64; ++lane)
                for (int j = 0; j < 8; ++j) {
                    int row = 32 * t + (lane & 31);
                    int slot = 16 * p + 8 * (lane >> 5) + j;
                    out[base + (((size_t)p * kt + t) * 64 + lane) * 8 + j] =
                        main[(size_t)row * slots + slot];
                }
    // accumulator register i of half-wave h holds row tile_row(t, i, h)
    for (int t = 0; t < kt; ++t)
        for (int h = 0; h < 2; ++h)
            for (int i = 0; i < 16; ++i)
                cn[(size_t)m * kt * 32 + (t * 2 + h) * 16 + i] =
                    (float)norm[32 * t + (i & 3) + 8 * (i >> 2) + 4 * h];
}

template <int D>
int pa_of() { return Plan<D>::PA; }

int plan_pa(int dsub) {
    switch (dsub) {
        case 4: return pa_of<4>();
        case 6: return pa_of<6>();
        case 8: return pa_of<8>();
        case 12: return pa_of<12>();
        case 16: return pa_of<16>();
        case 32: return pa_of<32>();
        default: return 0;
    }
}

// workgroups per CU of the persistent assignment grid: the occupancy limit, or fewer
// (PQH_ASSIGN_WGS_PER_CU, a fraction allowed: an experiment knob -- with three waves of 166
// VGPRs on every SIMD, no 32-VGPR wave of the kernels running beside the grid fits)
double assign_wgs_per_cu(const pqh_ctx* ctx, int occ) {
    double v = ctx->tune_wgs_per_cu;   // pqh_ctx_set_tuning, else the environment
    if (!(v > 0.0)) {
        const char* e = getenv("PQH_ASSIGN_WGS_PER_CU");
        v = e ? atof(e) : 0.0;
    }
    return v > 0.0 && v < occ ? v : (double)occ;
}

template <typename CodeT>
int launch_mfma(pqh_ctx* ctx, pqh_pq* pq, const float* x, long long n, long long ldx,
                CodeT* codes, uint32_t* counts, long long ldc) {
    const long long nblk = (n + 31) / 32;
    const int groups = pq->m;   // grid y: one subspace per workgroup
    dim3 block(64 * kWavesPerWG);
    // alternate launches use alternate queue-head sets and re-rank counters; each zeroes the
    // other's for the next launch (the stream orders the launches)
    const int ring = (int)(ctx->assign_launches++ & 1);
    unsigned long long* rr = ctx->d_diag + (ring ? 4 : 0);
    unsigned long long* rr_next = ctx->d_diag + (ring ? 0 : 4);
    ctx->rerank_slot = ring ? 4 : 0;
#ifdef PQH_ASSIGN_STATIC   // diagnostic: static chunk stride, no work queues
    uint32_t* sched = nullptr;
#else
    uint32_t* sched = pq->m <= kSchedMax ? ctx->d_sched + ring * kSchedSet : nullptr;
#endif
    const int prio = pqh_prio("ASSIGN", 0);
    // grid = the workgroups that are resident at once (persistent, grid-stride over the
    // 32-vector blocks): more would only queue behind the first wave of workgroups
#define PQH_CASE(DD) PQH_CASE_KT(DD, 8)
#define PQH_CASE_KT(DD, KTT)                                                                \
    case DD: {                                                                              \
        int per_cu = 1;                                                                     \
        const size_t dyn = KTT <= 8 && counts ? (size_t)kWavesPerWG * 256 * 4 : 0;         \
        if (hipOccupancyMaxActiveBlocksPerMultiprocessor(                                   \
                &per_cu, (const void*)(pq_assign_mfma<DD, KTT, CodeT>), (int)block.x, dyn) != \
                hipSuccess || per_cu < 1)                                                   \
            per_cu = 1;                                                                     \
        long long gx = (long long)((double)ctx->num_cus * assign_wgs_per_cu(ctx, per_cu) / groups); \
        gx = std::max(1ll, std::min(gx, ((nblk + kNB - 1) / kNB + kWavesPerWG - 1) / kWavesPerWG)); \
        if (gx >= 16) gx &= ~7ll;   /* CU-uniform subspace placement (see the kernel) */   \
        hipLaunchKernelGGL((pq_assign_mfma<DD, KTT, CodeT>), dim3((unsigned)(gx * groups)), block, \
                           dyn, ctx->stream, x, n, ldx, pq->m, pq->d_afrag, pq->d_cn, pq->d_cent, \
                           pq->d_cmax, pq->d_sqc, codes, counts, rr, sched, (int)gx,         \
                           rr_next, sched ? ctx->d_sched + (1 - ring) * kSchedSet : nullptr, \
                           prio, ldc);                                                        \
        PQH_LAUNCH_CHECK(ctx);                                                              \
        break;                                                                              \
    }
    if (pq->k == 4096) {   // A fragments streamed from L2; u16 codes; no fused histogram
        if constexpr (sizeof(CodeT) == 2) {
            switch (pq->dsub) {
                PQH_CASE_KT(16, 128)
                default: return PQH_ERR_UNSUPPORTED;
            }
        } else {
            return PQH_ERR_UNSUPPORTED;
        }
    } else if constexpr (sizeof(CodeT) == 1) {
        switch (pq->dsub) {
            PQH_CASE(4)
            PQH_CASE(6)
            PQH_CASE(8)
            PQH_CASE(12)
            PQH_CASE(16)
            PQH_CASE(32)
            default: return PQH_ERR_UNSUPPORTED;
        }
    } else {
        return PQH_ERR_UNSUPPORTED;
    }
#undef PQH_CASE
#undef PQH_CASE_KT
    PQH_LAUNCH_CHECK(ctx);
    return PQH_OK;
}

template <typename CodeT>
int launch_exact(pqh_ctx* ctx, pqh_pq* pq, const float* x, long long n, long long ldx,
                 CodeT* codes, uint32_t* counts, long long ldc) {
    const long long total = n * pq->m;
    if (total == 0) return PQH_OK;
    hipLaunchKernelGGL((pq_assign_exact<CodeT>), dim3((unsigned)((total + 255) / 256)), dim3(256),
                       0, ctx->stream, x, n, ldx, pq->m, pq->k, pq->dsub, pq->d_cent, codes,
                       counts, ldc);
    PQH_LAUNCH_CHECK(ctx);
    return PQH_OK;
}

}  // namespace

extern "C" {

int pqh_pq_create(pqh_ctx_t* ctx, const float* centroids, int m, int k, int dsub, pqh_pq_t** out) {
    if (!ctx || !centroids || !out || m <= 0 || k <= 0 || dsub <= 0 || k > 65536)
        return PQH_ERR_ARG;
    int rc = pqh_use_device(ctx);
    if (rc) return rc;
    pqh_pq* pq = new pqh_pq();
    pq->ctx = ctx;
    pq->m = m;
    pq->k = k;
    pq->dsub = dsub;
    const size_t nc = (size_t)m * k * dsub;
    bool finite = true;
    for (size_t i = 0; i < nc; ++i) finite &= std::isfinite(centroids[i]);
    const int pa = plan_pa(dsub);
    // MFMA screening: K = 256 at dsub 4, 6, 8, 12, 16, 32; K = 4096 at dsub 16
    pq->mfma_ok = finite && pa > 0 && (k == 256 || (k == 4096 && dsub == 16));
    if (hipMalloc(&pq->d_cent, nc * sizeof(float)) != hipSuccess) {
        delete pq;
        return pqh_set_error(ctx, PQH_ERR_NOMEM, "hipMalloc centroids");
    }
    (void)hipMemcpy(pq->d_cent, centroids, nc * sizeof(float), hipMemcpyHostToDevice);
    if (pq->mfma_ok) {
        std::vector<uint16_t> frag((size_t)m * pa * (k / 32) * 64 * 8);
        std::vector<float> cn((size_t)m * (k / 32) * 32);
        // sqc: [0, m) sqrt(Cmax), [m, 2m) 2 R (the split remainder's bound, see TauCoef)
        std::vector<float> cmax(m), sqc(2 * (size_t)m);
        for (int i = 0; i < m; ++i) {
            const float* c = centroids + (size_t)i * k * dsub;
            float& r2 = sqc[(size_t)m + i];
            switch (dsub) {
                case 4: build_afrag<4>(c, k, frag, cn, i, cmax[i], r2); break;
                case 6: build_afrag<6>(c, k, frag, cn, i, cmax[i], r2); break;
                case 8: build_afrag<8>(c, k, frag, cn, i, cmax[i], r2); break;
                case 12: build_afrag<12>(c, k, frag, cn, i, cmax[i], r2); break;
                case 16: build_afrag<16>(c, k, frag, cn, i, cmax[i], r2); break;
                case 32: build_afrag<32>(c, k, frag, cn, i, cmax[i], r2); break;
            }
            sqc[i] = (float)(std::sqrt((double)cmax[i]) * (1.0 + 1e-6)) + 1e-30f;
        }
        if (hipMalloc(&pq->d_afrag, frag.size() * 2) != hipSuccess ||
            hipMalloc(&pq->d_cn, cn.size() * sizeof(float)) != hipSuccess ||
            hipMalloc(&pq->d_cmax, m * sizeof(float)) != hipSuccess ||
            hipMalloc(&pq->d_sqc, 2 * (size_t)m * sizeof(float)) != hipSuccess) {
            pqh_pq_destroy(pq);
            return pqh_set_error(ctx, PQH_ERR_NOMEM, "hipMalloc fragments");
        }
        (void)hipMemcpy(pq->d_afrag, frag.data(), frag.size() * 2, hipMemcpyHostToDevice);
        (void)hipMemcpy(pq->d_cn, cn.data(), cn.size() * sizeof(float), hipMemcpyHostToDevice);
        (void)hipMemcpy(pq->d_cmax, cmax.data(), m * sizeof(float), hipMemcpyHostToDevice);
        (void)hipMemcpy(pq->d_sqc, sqc.data(), 2 * (size_t)m * sizeof(float), hipMemcpyHostToDevice);
    }
    *out = pq;
    return PQH_OK;
}

int pqh_pq_destroy(pqh_pq_t* pq) {
    if (!pq) return PQH_OK;
    (void)hipSetDevice(pq->ctx->device);
    (void)hipStreamSynchronize(pq->ctx->stream);
    (void)hipFree(pq->d_cent);
    (void)hipFree(pq->d_afrag);
    (void)hipFree(pq->d_cn);
    (void)hipFree(pq->d_cmax);
    (void)hipFree(pq->d_sqc);
    delete pq;
    return PQH_OK;
}

}  // extern "C"

// ldc = 0: row-major codes [n][m] (pq_indices.bvecsl); ldc >= n: part-major [m][ldc]
static int assign_impl(pqh_ctx_t* ctx, const pqh_pq_t* cpq, const float* d_x, long long n,
                       long long ld_x, void* d_codes, long long ldc, uint32_t* d_counts, int mode) {
    pqh_pq* pq = const_cast<pqh_pq*>(cpq);
    // any context of the codebook's device may run the assignment (its stream, its
    // work-queue heads and counters), so several streams can assign concurrently
    if (!ctx || !pq || pq->ctx->device != ctx->device || (n > 0 && (!d_x || !d_codes)) || n < 0 ||
        ld_x < (long long)pq->m * pq->dsub || (ldc != 0 && ldc < n))
        return PQH_ERR_ARG;
    int rc = pqh_use_device(ctx);
    if (rc) return rc;
    bool mfma = mode == 0 && pq->mfma_ok && n > 0;
    if (mfma && pq->dsub % 4 == 0 &&
        ((ld_x % 4) != 0 || (reinterpret_cast<uintptr_t>(d_x) & 15u) != 0))
        mfma = false;  // vector loads need 16-byte aligned subspace slices
    if (ld_x >= (1ll << 22)) mfma = false;   // its lane offsets within a block are 24-bit
    // the other paths re-rank nothing: their count is d_diag[6] = 0
    if (!mfma) {
        ctx->rerank_slot = 6;
        PQH_HIP(ctx, hipMemsetAsync(ctx->d_diag + 6, 0, sizeof(unsigned long long), ctx->stream));
    }
    if (n == 0) return PQH_OK;
    if (ldc && pq->k > 256 && d_counts) return PQH_ERR_UNSUPPORTED;
    // the MFMA kernel queues re-rank rows as 32-bit indices: at most 2^30 rows a launch
    constexpr long long kLaunchRows = 1ll << 30;
    auto pieces = [&](auto* c, uint32_t* counts) {
        for (long long off = 0; off < n; off += kLaunchRows) {
            const int r = launch_mfma(ctx, pq, d_x + off * ld_x, std::min(kLaunchRows, n - off),
                                      ld_x, c + (ldc ? off : off * pq->m), counts, ldc);
            if (r) return r;
        }
        return (int)PQH_OK;
    };
    if (pq->k <= 256) {
        uint8_t* c = static_cast<uint8_t*>(d_codes);
        return mfma ? pieces(c, d_counts) : launch_exact(ctx, pq, d_x, n, ld_x, c, d_counts, ldc);
    }
    uint16_t* c16 = static_cast<uint16_t*>(d_codes);
    if (!mfma) return launch_exact(ctx, pq, d_x, n, ld_x, c16, d_counts, ldc);
    // K = 4096: the screening kernel keeps no per-workgroup histogram (16 KB of counters per
    // wave); the requested counts come from the histogram kernel over the codes just written
    rc = pieces(c16, nullptr);
    if (rc || !d_counts) return rc;
    return pqh_histogram(ctx, d_codes, n, pq->m, pq->k, 0, nullptr, d_counts);
}

extern "C" {

int pqh_pq_assign(pqh_ctx_t* ctx, const pqh_pq_t* pq, const float* d_x, long long n,
                  long long ld_x, void* d_codes, uint32_t* d_counts, int mode) {
    return assign_impl(ctx, pq, d_x, n, ld_x, d_codes, 0, d_counts, mode);
}

int pqh_pq_assign_parts(pqh_ctx_t* ctx, const pqh_pq_t* pq, const float* d_x, long long n,
                        long long ld_x, void* d_codes, long long ld_codes, uint32_t* d_counts,
                        int mode) {
    if (ld_codes < n || ld_codes <= 0) return PQH_ERR_ARG;
    return assign_impl(ctx, pq, d_x, n, ld_x, d_codes, ld_codes, d_counts, mode);
}

// diagnostics: the per-wave stamps of the last assignment launch (PQH_ASSIGN_STAMPS builds;
// zeros otherwise); out holds max_waves * 4 values
int pqh_debug_assign_stamps(pqh_ctx_t* ctx, unsigned long long* out, int max_waves) {
    if (!ctx || !out || max_waves <= 0) return PQH_ERR_ARG;
    PQH_HIP(ctx, hipStreamSynchronize(ctx->stream));
    const int w = std::min(max_waves, kStampWaves);
    PQH_HIP(ctx, hipMemcpyFromSymbol(out, HIP_SYMBOL(g_assign_stamps), (size_t)w * 4 * 8));
    return PQH_OK;
}

// diagnostics: the per-wave re-rank phase sums of the last launch (PQH_ASSIGN_STAMPS builds)
int pqh_debug_assign_rr(pqh_ctx_t* ctx, unsigned long long* out, int max_waves) {
    if (!ctx || !out || max_waves <= 0) return PQH_ERR_ARG;
    PQH_HIP(ctx, hipStreamSynchronize(ctx->stream));
    const int w = std::min(max_waves, kStampWaves);
    PQH_HIP(ctx, hipMemcpyFromSymbol(out, HIP_SYMBOL(g_assign_rr), (size_t)w * 4 * 8));
    return PQH_OK;
}

int pqh_pq_last_rerank_count(pqh_ctx_t* ctx, unsigned long long* count) {
    if (!ctx || !count) return PQH_ERR_ARG;
    PQH_HIP(ctx, hipMemcpyAsync(count, ctx->d_diag + ctx->rerank_slot, sizeof(unsigned long long),
                                hipMemcpyDeviceToHost, ctx->stream));
    PQH_HIP(ctx, hipStreamSynchronize(ctx->stream));
    return PQH_OK;
}

int pqh_pq_error(pqh_ctx_t* ctx, const pqh_pq_t* pq, const float* d_x, long long n,
                 long long ld_x, const void* d_codes, double* error_out) {
    if (!ctx || !pq || !error_out || n <= 0) return PQH_ERR_ARG;
    double s = 0.0;
    const int rc = pqh_pq_error_accum(ctx, pq, d_x, n, ld_x, d_codes, &s);
    if (rc) return rc;
    *error_out = s / (double)n;
    return PQH_OK;
}

}  // extern "C"

int pqh_pq_error_accum(pqh_ctx* ctx, const pqh_pq_t* pq, const float* d_x, long long n,
                       long long ld_x, const void* d_codes, double* sum) {
    if (!ctx || !pq || !sum || n <= 0) return PQH_ERR_ARG;
    int rc = pqh_use_device(ctx);
    if (rc) return rc;
    const long long blocks = (n + 255) / 256;
    rc = pqh_ensure_ws(ctx, blocks * sizeof(double));
    if (rc) return rc;
    double* part = static_cast<double*>(ctx->ws);
    if (pq->k <= 256)
        hipLaunchKernelGGL(pq_error_kernel<uint8_t>, dim3((unsigned)blocks), dim3(256), 0, ctx->stream,
                           d_x, n, ld_x, pq->m, pq->k, pq->dsub, pq->d_cent,
                           static_cast<const uint8_t*>(d_codes), part);
    else
        hipLaunchKernelGGL(pq_error_kernel<uint16_t>, dim3((unsigned)blocks), dim3(256), 0, ctx->stream,
                           d_x, n, ld_x, pq->m, pq->k, pq->dsub, pq->d_cent,
                           static_cast<const uint16_t*>(d_codes), part);
    PQH_LAUNCH_CHECK(ctx);
    std::vector<double> h(blocks);
    PQH_HIP(ctx, hipMemcpyAsync(h.data(), part, blocks * sizeof(double), hipMemcpyDeviceToHost,
                                ctx->stream));
    PQH_HIP(ctx, hipStreamSynchronize(ctx->stream));
    double s = *sum;
    for (double v : h) s += v;
    *sum = s;
    return PQH_OK;
}

extern "C" {

int pqh_pq_reconstruct(pqh_ctx_t* ctx, const pqh_pq_t* pq, const void* d_codes, long long n,
                       float* d_out, long long ld_out) {
    if (!ctx || !pq || n < 0 || ld_out < (long long)pq->m * pq->dsub) return PQH_ERR_ARG;
    int rc = pqh_use_device(ctx);
    if (rc) return rc;
    const long long total = n * pq->m * pq->dsub;
    if (!total) return PQH_OK;
    const unsigned blocks = (unsigned)((total + 255) / 256);
    if (pq->k <= 256)
        hipLaunchKernelGGL(pq_reconstruct_kernel<uint8_t>, dim3(blocks), dim3(256), 0, ctx->stream,
                           static_cast<const uint8_t*>(d_codes), n, pq->m, pq->k, pq->dsub,
                           pq->d_cent, d_out, ld_out);
    else
        hipLaunchKernelGGL(pq_reconstruct_kernel<uint16_t>, dim3(blocks), dim3(256), 0, ctx->stream,
                           static_cast<const uint16_t*>(d_codes), n, pq->m, pq->k, pq->dsub,
                           pq->d_cent, d_out, ld_out);
    PQH_LAUNCH_CHECK(ctx);
    return PQH_OK;
}

}  // extern "C"
