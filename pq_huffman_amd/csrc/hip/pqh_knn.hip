// pqh_knn.hip -- the forest builder of tree mode on gfx950: compute_nn_fast's blocked kNN
// graph and mst_builder's minimum spanning forest.
//
//  knn geometry   blocks_info_init / dimension_info_build (fast_nn_blocks_info.c:52-112):
//                 split i is coordinate ns-1-i; block b of a split covers the sorted values
//                 [N b/nb - ov, N (b+1)/nb + ov] (ov = N overlap / 2), outer ends pushed out
//                 by 1.  The column is sorted on the device (rocPRIM radix sort); see
//                 "near-equal values" below for the one case that needs the host qsort.
//  block members  is_vector_in_block (:187-239) for every (row, block) at once: per row and
//                 split a bit mask of the blocks whose range holds the coordinate, the rows'
//                 (block, row) pairs emitted in ascending block id, stably sorted by block
//                 -> every block's rows in row order (block_loader2_thread, :84-150 of
//                 fast_nn_block_loader2.c).
//  block kNN      knn_full_thread (compute_nn_fast.c:479-481, yael -- absent here, so the
//                 in-block neighbours are defined by the oracle: the num_nn_real + 1 smallest
//                 direct-form fp32 distances (get_real_dist, :304-311), the lower block
//                 position first among equal distances).  One wave per 64 queries of a
//                 block: queries in VGPRs, 64-row candidate tiles in LDS read as broadcasts,
//                 a per-lane sorted top-KMAX list kept by a compare-exchange network.
//  merge          run_merge_block (:485-508) + fast_nn_heap_push/_sort
//                 (fast_nn_temp_file.c:11-63): one lane per row replays its blocks' lists
//                 in block order into its max-heap (LDS), then heap-sorts it.
//  mst            load_mst_edges_from_nn_files + minimum_spanning_tree (mst.c:80-236): PQ
//                 penalty re-scoring and the per-row sort, the global edge sort by distance as
//                 a stable radix sort, Boruvka under that order (= Kruskal's forest, see
//                 "minimum spanning forest"), the adjacency by a stable sort by source --
//                 all on the device.
//
// Near-equal values: the reference sorts with comparators that call two floats equal when
// they differ by less than 1e-9 (fast_nn_blocks_info.c:41-50, mst.c:15-26).  For any array
// without two DISTINCT values that close, glibc's merge sort with that comparator gives
// exactly the stable sort by value that the device computes; the device checks every
// adjacent pair of the sorted values, and if such a pair exists the affected sort is redone
// by glibc qsort on the host with the reference comparator (so the result stays the
// reference's), never silently approximated.
#include <rocprim/device/device_radix_sort.hpp>
#include <rocprim/device/device_scan.hpp>

#include <cmath>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "pqh_internal.h"

namespace {

constexpr int kQ = 64;   // queries (lanes) per kNN workgroup = candidate rows per LDS tile

struct DevBuf {   // device allocations of one call, released on every exit path
    std::vector<void*> ptrs;
    ~DevBuf() {
        for (void* p : ptrs) (void)hipFree(p);
    }
    template <typename T>
    T* get(size_t count) {
        void* p = nullptr;
        if (hipMalloc(&p, count ? count * sizeof(T) : 16) != hipSuccess) return nullptr;
        ptrs.push_back(p);
        return static_cast<T*>(p);
    }
};

// ------------------------------------------------------------------ geometry
__global__ void __launch_bounds__(256)
knn_column(const float* __restrict__ x, long long n, long long ld, int coord,
           uint32_t* __restrict__ keys) {
    const long long v = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (v >= n) return;
    float f = x[v * ld + coord];
    if (f == 0.0f) f = 0.0f;   // -0 sorts with +0 (the comparator calls them equal)
    const uint32_t b = __float_as_uint(f);
    keys[v] = (b & 0x80000000u) ? ~b : (b | 0x80000000u);   // order-preserving bits
}

__device__ __forceinline__ float key_float(uint32_t k) {
    return __uint_as_float((k & 0x80000000u) ? (k & 0x7FFFFFFFu) : ~k);
}

// flag[0] |= 1 when two adjacent sorted values are distinct but closer than 1e-9 (the
// comparator's "equal" band; float difference, as the reference computes it)
__global__ void __launch_bounds__(256)
near_equal_check(const uint32_t* __restrict__ keys, long long n, int* __restrict__ flag) {
    const long long v = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (v + 1 >= n) return;
    if (keys[v] == keys[v + 1]) return;
    const float a = key_float(keys[v]), b = key_float(keys[v + 1]);
    if (fabs((double)(b - a)) < 1e-9) atomicOr(flag, 1);
}

// the block bounds of one split from its sorted values (dimension_info_build, :70-81)
__global__ void knn_bounds(const uint32_t* __restrict__ sorted, long long n, int nb, long long ov,
                           float* __restrict__ starts, float* __restrict__ ends) {
    const int b = threadIdx.x;
    if (b >= nb) return;
    long long s = n * b / nb - ov;
    s = s < 0 ? 0 : (s > n ? n : s);
    long long e = n * (b + 1) / nb + ov;
    e = e < 0 ? 0 : (e > n ? n : e);
    e = e < n - 1 ? e : n - 1;
    float sv = key_float(sorted[s < n ? s : n - 1]);
    float ev = key_float(sorted[e]);
    if (b == 0) sv = (float)((double)key_float(sorted[0]) - 1.0);
    if (b == nb - 1) ev = (float)((double)key_float(sorted[n - 1]) + 1.0);
    starts[b] = sv;
    ends[b] = ev;
}

// ------------------------------------------------------------------ block members
struct Geo {
    int ns, nb;
    const float* starts;   // [ns][nb]
    const float* ends;
};

// per row and split, the mask of blocks holding the coordinate; count = product of popcounts
__global__ void __launch_bounds__(256)
knn_masks(const float* __restrict__ x, long long n, long long ld, Geo g,
          uint32_t* __restrict__ masks, uint32_t* __restrict__ count) {
    const long long v = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (v >= n) return;
    unsigned long long c = 1;
    for (int i = 0; i < g.ns; ++i) {
        const float val = x[v * ld + (g.ns - 1 - i)];
        uint32_t mk = 0;
        for (int b = 0; b < g.nb; ++b)
            if (!(val < g.starts[i * g.nb + b] || val > g.ends[i * g.nb + b])) mk |= 1u << b;
        masks[v * g.ns + i] = mk;
        c *= (unsigned long long)__popc(mk);
    }
    count[v] = (uint32_t)c;
}

// the row's (block, emission index) pairs in ascending block id: split 0 is the most
// significant digit (weight nb^(ns-1)), so an odometer over the masks' set bits with split
// ns-1 fastest enumerates them in order
__global__ void __launch_bounds__(256)
knn_emit(const uint32_t* __restrict__ masks, long long n, Geo g,
         const unsigned long long* __restrict__ off, uint32_t* __restrict__ keys,
         uint32_t* __restrict__ vals, uint32_t* __restrict__ erow) {
    const long long v = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (v >= n) return;
    unsigned long long e = off[v];
    if (off[v + 1] == e) return;
    uint32_t mk[8], cur[8];
    for (int i = 0; i < g.ns; ++i) {
        mk[i] = masks[v * g.ns + i];
        cur[i] = mk[i] & (0u - mk[i]);   // lowest set bit
    }
    for (;;) {
        uint32_t B = 0;
        for (int i = 0; i < g.ns; ++i) B = B * (uint32_t)g.nb + (uint32_t)(__ffs(cur[i]) - 1);
        keys[e] = B;
        vals[e] = (uint32_t)e;
        erow[e] = (uint32_t)v;
        ++e;
        int i = g.ns - 1;   // advance: next set bit of the fastest digit, carry to slower ones
        for (; i >= 0; --i) {
            const uint32_t rest = mk[i] & ~((cur[i] << 1) - 1u);
            if (rest) {
                cur[i] = rest & (0u - rest);
                break;
            }
            cur[i] = mk[i] & (0u - mk[i]);
        }
        if (i < 0) break;
    }
}

// sorted pair p: its row, and the emission index's position p
__global__ void __launch_bounds__(256)
knn_place(const uint32_t* __restrict__ sorted_vals, long long np, const uint32_t* __restrict__ erow,
          uint32_t* __restrict__ rows, uint32_t* __restrict__ inv) {
    const long long p = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (p >= np) return;
    const uint32_t e = sorted_vals[p];
    rows[p] = erow[e];
    inv[e] = (uint32_t)p;
}

// boff[b] = first sorted pair of block b (lower bound in the sorted keys)
__global__ void __launch_bounds__(256)
knn_block_offsets(const uint32_t* __restrict__ keys, long long np, long long nblocks,
                  long long* __restrict__ boff) {
    const long long b = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (b > nblocks) return;
    long long lo = 0, hi = np;
    while (lo < hi) {
        const long long mid = (lo + hi) >> 1;
        if ((long long)keys[mid] < b) lo = mid + 1;
        else hi = mid;
    }
    boff[b] = lo;
}

// ------------------------------------------------------------------ block kNN
// One wave = up to 64 queries of one block (tile list built on the host).  Every lane keeps
// its top-KMAX (distance, block position) list sorted ascending -- equal distances in
// position order, because candidates arrive in position order and a new entry goes after
// equal ones -- in registers, updated by a compare-exchange network with static indices.
// The first kk = min(num_nn, S - 1) + 1 entries are the block kNN (kk <= KMAX).
// Per 64-candidate tile: the rows are staged in LDS zero-padded to DMAX dimensions (a zero
// term adds +0 to a non-negative sum: exact), every lane computes its 64 distances from
// broadcast b128 reads, and appends the ones below its current kk-th distance to an LDS
// buffer; the network then runs once per buffered entry of the busiest lane -- after the
// first tiles a handful per tile instead of one per candidate.
template <int DMAX, int KMAX>
__global__ void __launch_bounds__(kQ)
knn_block_topk(const float* __restrict__ x, long long ld, int d, int num_nn,
               const uint32_t* __restrict__ rows, const long long* __restrict__ boff,
               const long long* __restrict__ tile_block, const long long* __restrict__ tile_q0,
               int stride, float* __restrict__ out_dist, uint32_t* __restrict__ out_row) {
    static_assert(DMAX % 4 == 0, "b128 reads");
    __shared__ __attribute__((aligned(16))) float cand[kQ * DMAX];
    __shared__ float2 buf[kQ * kQ];   // per lane: (distance, position bits) of this tile
    const int lane = threadIdx.x;
    const long long b = tile_block[blockIdx.x];
    const long long base = boff[b];
    const int S = (int)(boff[b + 1] - base);
    const int q = (int)tile_q0[blockIdx.x] + lane;
    const bool valid = q < S;
    const int kk = (num_nn < S - 1 ? num_nn : S - 1) + 1;
    const uint32_t* brows = rows + base;
    float qv[DMAX];
    {
        const float* xq = x + (long long)brows[valid ? q : 0] * ld;
#pragma unroll
        for (int j = 0; j < DMAX; ++j) qv[j] = j < d ? xq[j] : 0.0f;
    }
    float ld_[KMAX];
    uint32_t lp_[KMAX];
#pragma unroll
    for (int j = 0; j < KMAX; ++j) {
        ld_[j] = INFINITY;
        lp_[j] = 0xFFFFFFFFu;
    }
    float thr = INFINITY;   // the current kk-th distance
    for (int c0 = 0; c0 < S; c0 += kQ) {
        const int nc = S - c0 < kQ ? S - c0 : kQ;
        __syncthreads();
        for (int f = lane; f < nc * DMAX; f += kQ) {   // stage the tile (rows in block order)
            const int r = f / DMAX, j = f - r * DMAX;
            cand[f] = j < d ? x[(long long)brows[c0 + r] * ld + j] : 0.0f;
        }
        __syncthreads();
        int cnt = 0;
        for (int c = 0; c < nc; ++c) {
            const float4* cr = reinterpret_cast<const float4*>(cand + c * DMAX);
            float acc = 0.0f;   // get_real_dist: (x - y)^2 summed in dimension order
#pragma unroll
            for (int j4 = 0; j4 < DMAX / 4; ++j4) {
                const float4 y = cr[j4];
                float t = __fsub_rn(qv[4 * j4], y.x);
                acc = __fadd_rn(acc, __fmul_rn(t, t));
                t = __fsub_rn(qv[4 * j4 + 1], y.y);
                acc = __fadd_rn(acc, __fmul_rn(t, t));
                t = __fsub_rn(qv[4 * j4 + 2], y.z);
                acc = __fadd_rn(acc, __fmul_rn(t, t));
                t = __fsub_rn(qv[4 * j4 + 3], y.w);
                acc = __fadd_rn(acc, __fmul_rn(t, t));
                // (a group of 8 reads at a time: hoisting all of them costs DMAX registers)
                if ((j4 & 7) == 7) __builtin_amdgcn_sched_barrier(0);
            }
            if (valid && acc < thr) {
                buf[lane * kQ + cnt] = make_float2(acc, __uint_as_float((uint32_t)(c0 + c)));
                ++cnt;
            }
        }
        for (int i = 0; __any(i < cnt); ++i) {
            {   // (a lane with no entry left carries +inf: nothing moves)
                const float2 e = i < cnt ? buf[lane * kQ + i] : make_float2(INFINITY, 0.0f);
                float cd = e.x;   // the entry goes before the first strictly larger one, and
                uint32_t cp = __float_as_uint(e.y);   // every later slot shifts by one: the
                bool mv = false;                      // displaced entry is carried (in place)
#pragma unroll
                for (int j = 0; j < KMAX; ++j) {
                    const bool sw = mv || ld_[j] > cd;   // (selects: fminf/fmaxf canonicalise)
                    mv = sw;
                    const float dj = ld_[j];
                    const uint32_t pj = lp_[j];
                    ld_[j] = sw ? cd : dj;
                    lp_[j] = sw ? cp : pj;
                    cd = sw ? dj : cd;
                    cp = sw ? pj : cp;
                }
            }
        }
        // the kk-th entry (kk is uniform: a static select chain)
#pragma unroll
        for (int j = 0; j < KMAX; ++j) thr = j == kk - 1 ? ld_[j] : thr;
    }
    if (!valid) return;
    const long long pair = base + q;
#pragma unroll
    for (int j = 0; j < KMAX; ++j) {
        if (j < kk) {
            out_dist[pair * stride + j] = ld_[j];
            out_row[pair * stride + j] = brows[lp_[j]];
        }
    }
}

// ------------------------------------------------------------------ block kNN, MFMA screen
// The default in-block kNN (PQH_KNN_IMPL=valu: knn_block_topk above).  Three steps:
//  knn_split     every row once: x = hi + lo as two bf16 rows zero-padded to DP dimensions
//                (DP = d rounded up to 16) and ||x||^2 in fp32.
//  knn_screen    one wave per 32 queries of a block (v_mfma_f32_32x32x16_bf16, A = 32
//                candidate rows, B = the 32 queries, K = 16 dimensions; hi*hi + lo*hi +
//                hi*lo per 16 dimensions): the approximate distance
//                d' = ||q||^2 + ||c||^2 - 2 q.c  of every (query, candidate) pair, twice.
//                Pass 1 keeps, per half-wave lane, the kk smallest d' of its candidates; the
//                smaller of the two halves' kk-th values, T, is >= the block's kk-th smallest
//                d'.  Pass 2 lists every candidate with d' <= T + 2 E (E bounds |d' - D| for
//                the oracle's fp32 distance D of every candidate of this query): that list
//                holds every candidate whose D can be among the kk smallest (if D_c <= D_(kk)
//                then d'_c <= D_(kk) + E <= T + 2 E, because kk candidates have D <= d' + E
//                <= T + E).
//  knn_select    one lane per query: the listed candidates' exact direct-form distances and
//                the kk smallest by (distance, block position); a list that overflowed its
//                CH slots makes the lane scan the whole block instead.
// E = (3 2^-18 + (3 DP + 3 d + 8) 2^-24) (||q||^2 + Cmax) * 1.25, Cmax = the block's largest
// ||c||^2: the bf16 split drops ql.cl + (qh + ql).rc + rq.c (each <= 2^-18 |q||c| summed,
// Cauchy-Schwarz), the fp32 accumulation of 3 DP products, the fp32 norms (d + 1 roundings)
// and the final fma, and the oracle's own direct-form rounding ((d + 2) 2^-24 D, D <=
// 2 (||q||^2 + ||c||^2)); every term is <= its coefficient times ||q||^2 + Cmax.
typedef __bf16 kbf16x8 __attribute__((ext_vector_type(8)));
typedef float kf32x16 __attribute__((ext_vector_type(16)));
constexpr int kScreenQ = 32;   // queries per screening wave (the MFMA's columns)

__device__ __forceinline__ float raw_min(float a, float b) {   // (no canonicalising maxes)
    float r;
    asm("v_min_f32 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
    return r;
}
__device__ __forceinline__ float raw_max(float a, float b) {
    float r;
    asm("v_max_f32 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
    return r;
}

// one lane per (row, 8-column group): a wave reads and writes contiguous rows.  ||x||^2 is
// summed as 8-term sequential partials combined by a butterfly -- any order is within the
// screen's bound E (|error| <= (d - 1) u sum x^2 for every summation order)
template <int DP>
__global__ void __launch_bounds__(256)
knn_split(const float* __restrict__ x, long long n, long long ld, int d,
          kbf16x8* __restrict__ xhi, kbf16x8* __restrict__ xlo, float* __restrict__ norm,
          float* __restrict__ xpad) {
    constexpr int G = DP / 8;   // lanes per row (2..16, a power of two)
    const long long t = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    const long long v = t / G;
    const int g = (int)(t % G);
    const bool in = v < n;
    const float* xr = x + (in ? v : 0) * ld;
    float f[8];
    float nn = 0.0f;
    kbf16x8 hi, lo;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        const int c = 8 * g + j;
        f[j] = in && c < d ? xr[c] : 0.0f;
        nn = __fadd_rn(nn, __fmul_rn(f[j], f[j]));
        const __bf16 h = (__bf16)f[j];
        hi[j] = h;
        lo[j] = (__bf16)(f[j] - (float)h);
    }
#pragma unroll
    for (int o = 1; o < G; o <<= 1) nn = __fadd_rn(nn, __shfl_xor(nn, o, G));
    if (!in) return;
    float4* xp = reinterpret_cast<float4*>(xpad + v * DP + 8 * g);
    xp[0] = make_float4(f[0], f[1], f[2], f[3]);
    xp[1] = make_float4(f[4], f[5], f[6], f[7]);
    xhi[v * G + g] = hi;
    xlo[v * G + g] = lo;
    if (g == 0) norm[v] = nn;
}

// cmax[b] = the largest ||c||^2 of block b (non-negative floats order as their bits); the
// pairs are sorted by block, so a wave reduces its runs and each run head does one atomic
__global__ void __launch_bounds__(256)
knn_block_cmax(const uint32_t* __restrict__ keys_sorted, const uint32_t* __restrict__ rows,
               long long np, const float* __restrict__ norm, uint32_t* __restrict__ cmax) {
    const long long p = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    const bool in = p < np;
    const uint32_t key = in ? keys_sorted[p] : 0xFFFFFFFFu;
    uint32_t val = in ? __float_as_uint(norm[rows[p]]) : 0u;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const uint32_t k2 = __shfl_down(key, o), v2 = __shfl_down(val, o);
        if (k2 == key) val = v2 > val ? v2 : val;
    }
    const uint32_t kprev = __shfl_up(key, 1);
    if (in && ((threadIdx.x & 63) == 0 || kprev != key)) atomicMax(&cmax[key], val);
}

template <int DP, int KMAX>
__global__ void __launch_bounds__(64)
knn_screen(const kbf16x8* __restrict__ xhi, const kbf16x8* __restrict__ xlo,
           const float* __restrict__ norm, const uint32_t* __restrict__ rows,
           const long long* __restrict__ boff, const uint32_t* __restrict__ cmax_bits,
           const long long* __restrict__ tile_block, const long long* __restrict__ tile_q0,
           int num_nn, int d, int ch, uint32_t* __restrict__ cand, uint32_t* __restrict__ ccount) {
    constexpr int NSTEP = DP / 16;
    constexpr int G = DP / 8;   // bf16x8 groups per row
    __shared__ __attribute__((aligned(16))) float tnorm[kScreenQ];
    __shared__ float pbuf[64 * 16];   // pass 1: a tile's values below the lane's threshold
    const int lane = threadIdx.x, r = lane & 31, h = lane >> 5;
    const long long b = tile_block[blockIdx.x];
    const long long base = boff[b];
    const int S = (int)(boff[b + 1] - base);
    const int q = (int)tile_q0[blockIdx.x] + r;
    const bool valid = q < S;
    const int kk = (num_nn < S - 1 ? num_nn : S - 1) + 1;
    const uint32_t* brows = rows + base;
    const uint32_t qrow = brows[valid ? q : 0];
    kbf16x8 bh[NSTEP], bl[NSTEP];
#pragma unroll
    for (int s = 0; s < NSTEP; ++s) {
        bh[s] = xhi[(long long)qrow * G + 2 * s + h];
        bl[s] = xlo[(long long)qrow * G + 2 * s + h];
    }
    const float nq = norm[qrow];
    const float cmax = __uint_as_float(cmax_bits[b]);
    auto tile = [&](int c0, kf32x16& acc, float* nc) {
        const int cr = c0 + r < S ? c0 + r : S - 1;   // this lane's A row (clamped)
        const uint32_t crow = brows[cr];
        __syncthreads();
        if (h == 0) tnorm[r] = norm[crow];
        acc = kf32x16{};
#pragma unroll
        for (int s = 0; s < NSTEP; ++s) {
            const kbf16x8 ah = xhi[(long long)crow * G + 2 * s + h];
            const kbf16x8 al = xlo[(long long)crow * G + 2 * s + h];
            acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah, bh[s], acc, 0, 0, 0);
            acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(al, bh[s], acc, 0, 0, 0);
            acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah, bl[s], acc, 0, 0, 0);
        }
        __syncthreads();
#pragma unroll
        for (int g = 0; g < 4; ++g) {   // rows 8g + 4h .. +4 of the tile
            const float4 v4 = *reinterpret_cast<const float4*>(tnorm + 8 * g + 4 * h);
            nc[4 * g] = v4.x; nc[4 * g + 1] = v4.y; nc[4 * g + 2] = v4.z; nc[4 * g + 3] = v4.w;
        }
    };
    // pass 1: the KMAX smallest d' of this lane's candidates (values only)
    float lst[KMAX];
#pragma unroll
    for (int j = 0; j < KMAX; ++j) lst[j] = INFINITY;
    for (int c0 = 0; c0 < S; c0 += kScreenQ) {
        kf32x16 acc;
        float nc[16];
        tile(c0, acc, nc);
        // the tile's values below the lane's current KMAX-th go to its LDS buffer; the
        // network then runs once per entry of the fullest lane (not once per register)
        const float thr = lst[KMAX - 1];
        int cnt = 0;
#pragma unroll
        for (int i = 0; i < 16; ++i) {
            const int row = c0 + (i & 3) + 8 * (i >> 2) + 4 * h;
            const float dp = fmaf(-2.0f, acc[i], nq + nc[i]);
            if (valid && row < S && dp < thr) pbuf[lane * 16 + cnt++] = dp;
        }
        for (int e = 0; __any(e < cnt); ++e) {
            float cd = e < cnt ? pbuf[lane * 16 + e] : INFINITY;
#pragma unroll
            for (int j = 0; j < KMAX; ++j) {
                const float lo = raw_min(lst[j], cd), hi = raw_max(lst[j], cd);
                lst[j] = lo;
                cd = hi;
            }
        }
    }
    float tloc = INFINITY;
#pragma unroll
    for (int j = 0; j < KMAX; ++j) tloc = j == kk - 1 ? lst[j] : tloc;
    const auto sw = __builtin_amdgcn_permlane32_swap(__float_as_uint(tloc), __float_as_uint(tloc),
                                                     false, false);
    const float T = raw_min(__uint_as_float(sw[0]), __uint_as_float(sw[1]));
    const float E = (3.0f * 0x1p-18f + (float)(3 * DP + 3 * d + 8) * 0x1p-24f) * (nq + cmax) * 1.25f;
    const float U = T + 2.0f * E;   // (T = +inf: every candidate is listed)
    // pass 2: list the candidates with d' <= U (block positions, ascending per half)
    uint32_t cnt = 0;
    uint32_t* my = cand + ((long long)(base + q) * 2 + h) * ch;
    for (int c0 = 0; c0 < S; c0 += kScreenQ) {
        kf32x16 acc;
        float nc[16];
        tile(c0, acc, nc);
#pragma unroll
        for (int i = 0; i < 16; ++i) {
            const int row = c0 + (i & 3) + 8 * (i >> 2) + 4 * h;
            const float dp = fmaf(-2.0f, acc[i], nq + nc[i]);
            if (valid && row < S && !(dp > U)) {
                if (cnt < (uint32_t)ch) my[cnt] = (uint32_t)row;
                ++cnt;
            }
        }
    }
    if (valid) ccount[(base + q) * 2 + h] = cnt;
}

// one lane per (block, query) pair: exact distances of the listed candidates (or of the whole
// block after an overflow), the kk smallest by (distance, position), in the output lists
template <int DP, int KMAX>
__global__ void __launch_bounds__(64)
knn_select(const float* __restrict__ xpad, int num_nn,
           const uint32_t* __restrict__ rows, const uint32_t* __restrict__ keys_sorted,
           const long long* __restrict__ boff, long long np, int ch,
           const uint32_t* __restrict__ cand, const uint32_t* __restrict__ ccount, int stride,
           float* __restrict__ out_dist, uint32_t* __restrict__ out_row) {
    const long long p = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (p >= np) return;
    const long long b = keys_sorted[p];
    const long long base = boff[b];
    const int S = (int)(boff[b + 1] - base);
    const int kk = (num_nn < S - 1 ? num_nn : S - 1) + 1;
    const uint32_t* brows = rows + base;
    float qv[DP];   // (rows zero-padded to DP: a zero term adds +0, exact)
    {
        const float4* xq = reinterpret_cast<const float4*>(xpad + (long long)rows[p] * DP);
#pragma unroll
        for (int j = 0; j < DP / 4; ++j) {
            const float4 v4 = xq[j];
            qv[4 * j] = v4.x; qv[4 * j + 1] = v4.y; qv[4 * j + 2] = v4.z; qv[4 * j + 3] = v4.w;
        }
    }
    float ld_[KMAX];
    uint32_t lp_[KMAX];
#pragma unroll
    for (int j = 0; j < KMAX; ++j) {
        ld_[j] = INFINITY;
        lp_[j] = 0xFFFFFFFFu;
    }
    const uint32_t n0 = ccount[p * 2], n1 = ccount[p * 2 + 1];
    const bool full = n0 > (uint32_t)ch || n1 > (uint32_t)ch;
    const int total = full ? S : (int)(n0 + n1);
    for (int t = 0; t < total; ++t) {
        const uint32_t pos = full ? (uint32_t)t
                                  : cand[(p * 2 + (t < (int)n0 ? 0 : 1)) * ch + (t < (int)n0 ? t : t - n0)];
        const float4* xc = reinterpret_cast<const float4*>(xpad + (long long)brows[pos] * DP);
        float acc = 0.0f;   // get_real_dist, dimension order
#pragma unroll
        for (int j = 0; j < DP / 4; ++j) {
            const float4 c4 = xc[j];
            float tt = __fsub_rn(qv[4 * j], c4.x);
            acc = __fadd_rn(acc, __fmul_rn(tt, tt));
            tt = __fsub_rn(qv[4 * j + 1], c4.y);
            acc = __fadd_rn(acc, __fmul_rn(tt, tt));
            tt = __fsub_rn(qv[4 * j + 2], c4.z);
            acc = __fadd_rn(acc, __fmul_rn(tt, tt));
            tt = __fsub_rn(qv[4 * j + 3], c4.w);
            acc = __fadd_rn(acc, __fmul_rn(tt, tt));
            if ((j & 7) == 7) __builtin_amdgcn_sched_barrier(0);
        }
        float cd = acc;   // carried up the list in (distance, position) order
        uint32_t cp = pos;
#pragma unroll
        for (int j = 0; j < KMAX; ++j) {
            const bool sw = ld_[j] > cd || (ld_[j] == cd && lp_[j] > cp);
            const float dj = ld_[j];
            const uint32_t pj = lp_[j];
            ld_[j] = sw ? cd : dj;
            lp_[j] = sw ? cp : pj;
            cd = sw ? dj : cd;
            cp = sw ? pj : cp;
        }
    }
#pragma unroll
    for (int j = 0; j < KMAX; ++j) {
        if (j < kk) {
            out_dist[p * stride + j] = ld_[j];
            out_row[p * stride + j] = brows[lp_[j]];
        }
    }
}

// knn_select's wave form (the default): one wave per (block, query) pair, a lane per listed
// candidate (64 at a time): the exact direct-form distances in parallel (the query row is
// wave-uniform), then a bitonic sort of the 64 (distance, position) keys across the lanes,
// merged into the running 64 smallest (min with the reversed new list, then a bitonic
// clean), so after the last round lanes 0 .. kk-1 hold the kk smallest in order.
__device__ __forceinline__ bool key_less(float da, uint32_t pa, float db, uint32_t pb) {
    return da < db || (da == db && pa < pb);
}

// one compare-exchange stage of a bitonic network across the wave: partner = lane ^ j; the
// lane keeps the smaller key when (lane & j) == 0 and the block is ascending
__device__ __forceinline__ void bitonic_step(float& d, uint32_t& p, int lane, int j, bool up) {
    const float od = __shfl_xor(d, j);
    const uint32_t op = (uint32_t)__shfl_xor((int)p, j);
    const bool lower = (lane & j) == 0;
    const bool other_less = key_less(od, op, d, p);
    const bool take = (lower == up) ? other_less : !other_less && !(od == d && op == p);
    if (take) {
        d = od;
        p = op;
    }
}

template <int DP>
__global__ void __launch_bounds__(256)
knn_select_wave(const float* __restrict__ xpad, int num_nn, const uint32_t* __restrict__ rows,
                const uint32_t* __restrict__ keys_sorted, const long long* __restrict__ boff,
                long long np, int ch, const uint32_t* __restrict__ cand,
                const uint32_t* __restrict__ ccount, int stride, float* __restrict__ out_dist,
                uint32_t* __restrict__ out_row) {
    const int lane = threadIdx.x & 63;
    const long long p = (long long)blockIdx.x * 4 + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    if (p >= np) return;
    const long long b = keys_sorted[p];
    const long long base = boff[b];
    const int S = (int)(boff[b + 1] - base);
    const int kk = (num_nn < S - 1 ? num_nn : S - 1) + 1;
    const uint32_t* brows = rows + base;
    const float4* xq = reinterpret_cast<const float4*>(xpad + (long long)rows[p] * DP);
    const uint32_t n0 = ccount[p * 2], n1 = ccount[p * 2 + 1];
    const bool full = n0 > (uint32_t)ch || n1 > (uint32_t)ch;
    const int total = full ? S : (int)(n0 + n1);
    float kd = INFINITY;          // the running 64 smallest keys, ascending by lane
    uint32_t kp = 0xFFFFFFFFu;
    for (int t0 = 0; t0 < total; t0 += 64) {
        const int t = t0 + lane;
        float d = INFINITY;
        uint32_t pos = 0xFFFFFFFFu;
        if (t < total) {
            pos = full ? (uint32_t)t
                       : cand[(p * 2 + (t < (int)n0 ? 0 : 1)) * ch + (t < (int)n0 ? t : t - (int)n0)];
            const float4* xc = reinterpret_cast<const float4*>(xpad + (long long)brows[pos] * DP);
            float acc = 0.0f;   // get_real_dist, dimension order
#pragma unroll
            for (int j = 0; j < DP / 4; ++j) {
                const float4 q4 = xq[j], c4 = xc[j];
                float tt = __fsub_rn(q4.x, c4.x);
                acc = __fadd_rn(acc, __fmul_rn(tt, tt));
                tt = __fsub_rn(q4.y, c4.y);
                acc = __fadd_rn(acc, __fmul_rn(tt, tt));
                tt = __fsub_rn(q4.z, c4.z);
                acc = __fadd_rn(acc, __fmul_rn(tt, tt));
                tt = __fsub_rn(q4.w, c4.w);
                acc = __fadd_rn(acc, __fmul_rn(tt, tt));
            }
            d = acc;
        }
        // sort the 64 new keys ascending (bitonic)
        for (int k = 2; k <= 64; k <<= 1)
            for (int j = k >> 1; j > 0; j >>= 1) bitonic_step(d, pos, lane, j, (lane & k) == 0);
        if (t0 == 0) {
            kd = d;
            kp = pos;
        } else {   // the 64 smallest of both: min with the reversed new list (bitonic), clean
            const float rd = __shfl(d, 63 - lane);
            const uint32_t rp = (uint32_t)__shfl((int)pos, 63 - lane);
            if (key_less(rd, rp, kd, kp)) {
                kd = rd;
                kp = rp;
            }
            for (int j = 32; j > 0; j >>= 1) bitonic_step(kd, kp, lane, j, true);
        }
    }
    if (lane < kk) {
        out_dist[p * stride + lane] = kd;
        out_row[p * stride + lane] = brows[kp];
    }
}

// ------------------------------------------------------------------ merge
struct NnItem {
    uint32_t index;
    float dist;
};

// fast_nn_heap_push_impl (fast_nn_temp_file.c:23-46): the item replaces the root and sinks
// while a child is strictly heavier (the right one when it is the heavier of the two).
// Heap slot i at h[i * S] (S = kQ in the merge: the lanes' heaps interleaved, so lanes at the
// same slot read consecutive words).
template <int S>
__device__ __forceinline__ void nn_sift(NnItem* h, NnItem it, int k) {
    int i = 0;
    for (;;) {
        const int l = 2 * i + 1, r = 2 * i + 2;
        int sw;
        if (r < k && h[r * S].dist > h[l * S].dist && h[r * S].dist > it.dist) sw = r;
        else if (l < k && h[l * S].dist > it.dist) sw = l;
        else break;
        h[i * S] = h[sw * S];
        i = sw;
    }
    h[i * S] = it;
}

// one lane per row: its blocks' lists (entries 1 .. kk-1) in block order into the heap, then
// fast_nn_heap_sort into the output row
__global__ void __launch_bounds__(kQ)
knn_merge(long long n, int num_nn, const unsigned long long* __restrict__ off,
          const uint32_t* __restrict__ inv, const uint32_t* __restrict__ keys_sorted,
          const long long* __restrict__ boff, int stride, const float* __restrict__ ldist,
          const uint32_t* __restrict__ lrow, uint32_t* __restrict__ out_idx,
          float* __restrict__ out_dist) {
    extern __shared__ NnItem heaps[];
    const long long v = (long long)blockIdx.x * kQ + threadIdx.x;
    if (v >= n) return;
    NnItem* h = heaps + threadIdx.x;   // slot j at h[j * kQ]
    for (int j = 0; j < num_nn; ++j) h[j * kQ] = NnItem{0xFFFFFFFFu, INFINITY};
    // a row in one block gets distinct indices only: the reference's duplicate scan never
    // fires for it
    const bool single = off[v + 1] - off[v] == 1;
    for (unsigned long long e = off[v]; e < off[v + 1]; ++e) {
        const long long p = inv[e];
        const long long b = keys_sorted[p];
        const long long S = boff[b + 1] - boff[b];
        const int kk = (int)((num_nn < S - 1 ? num_nn : S - 1) + 1);
        // the list's entries eight at a time, their loads issued together (the merge is
        // bound by these loads' latency, not by the heap work)
        for (int j0 = 1; j0 < kk; j0 += 8) {
            NnItem its[8];
#pragma unroll
            for (int u = 0; u < 8; ++u) {
                const int j = j0 + u < kk ? j0 + u : j0;
                its[u] = NnItem{lrow[p * stride + j], ldist[p * stride + j]};
            }
#pragma unroll
            for (int u = 0; u < 8; ++u) {
                if (j0 + u >= kk) break;
                const NnItem it = its[u];
                if (!(it.dist < h[0].dist)) continue;
                bool dup = false;
                if (!single)
                    for (int q = 0; q < num_nn; ++q) dup |= h[q * kQ].index == it.index;
                if (!dup) nn_sift<kQ>(h, it, num_nn);
            }
        }
    }
    for (int k = num_nn - 1; k >= 0; --k) {
        out_idx[v * num_nn + k] = h[0].index;
        out_dist[v * num_nn + k] = h[0].dist;
        nn_sift<kQ>(h, h[k * kQ], k);
    }
}

// ------------------------------------------------------------------ mst edges
// Row v's first `take` neighbours as edges; with a PQ penalty every neighbour is re-scored
// (dist += Hamming * penalty, = Hamming when infinite: mst.c:117-130) and the row stably
// sorted by the new distance first (qsort at :133-135).  flag bit 1: a neighbour id outside
// the rows; bit 2: a row holds two distinct re-scored distances closer than 1e-9.
__global__ void __launch_bounds__(kQ)
mst_row_edges(const uint32_t* __restrict__ idx, const float* __restrict__ dist, long long n,
              int num_nn, int take, const uint8_t* __restrict__ pq, int pq_m, float penalty,
              uint32_t* __restrict__ keys, uint32_t* __restrict__ vals, uint32_t* __restrict__ src,
              uint32_t* __restrict__ dst, float* __restrict__ edist, int* __restrict__ flag) {
    extern __shared__ NnItem rowbuf[];
    const long long v = (long long)blockIdx.x * kQ + threadIdx.x;
    if (v >= n) return;
    NnItem* r = rowbuf + threadIdx.x * num_nn;
    int bad = 0;
    for (int j = 0; j < num_nn; ++j) {
        NnItem it{idx[v * num_nn + j], dist[v * num_nn + j]};
        if (it.index >= n) {
            bad |= 1;
            it.index = 0;
        }
        if (penalty > 0.0f) {
            int ham = 0;
            for (int i = 0; i < pq_m; ++i)
                ham += pq[v * pq_m + i] != pq[(long long)it.index * pq_m + i];
            if (isinf(penalty)) it.dist = (float)ham;
            else it.dist = __fadd_rn(it.dist, __fmul_rn((float)ham, penalty));
            int p = j;   // stable insertion: after equal distances
            while (p > 0 && r[p - 1].dist > it.dist) {
                r[p] = r[p - 1];
                --p;
            }
            r[p] = it;
        } else {
            r[j] = it;
        }
    }
    if (penalty > 0.0f)
        for (int j = 0; j + 1 < num_nn; ++j) {
            const float df = r[j + 1].dist - r[j].dist;
            if (df != 0.0f && fabs((double)df) < 1e-9) bad |= 2;
        }
    for (int j = 0; j < take; ++j) {
        const long long e = v * take + j;
        float f = r[j].dist;
        if (f == 0.0f) f = 0.0f;
        const uint32_t bits = __float_as_uint(f);
        keys[e] = (bits & 0x80000000u) ? ~bits : (bits | 0x80000000u);
        vals[e] = (uint32_t)e;
        src[e] = (uint32_t)v;
        dst[e] = r[j].index;
        edist[e] = r[j].dist;
    }
    if (bad) atomicOr(flag, bad);
}

__global__ void __launch_bounds__(256)
gather_pairs(const uint32_t* __restrict__ order, long long ne, const uint32_t* __restrict__ src,
             const uint32_t* __restrict__ dst, uint2* __restrict__ out) {
    const long long e = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= ne) return;
    const uint32_t q = order[e];
    out[e] = make_uint2(src[q], dst[q]);
}

// ------------------------------------------------------------------ minimum spanning forest
// Boruvka over the edges in rank order (rank = position in the stable distance sort, i.e.
// the order Kruskal scans them, mst.c:191-201): under that strict order the forest is
// unique, so the edges Boruvka keeps are exactly Kruskal's, and listed by rank they are in
// Kruskal's acceptance order.  Components are labelled by a root vertex; every round each
// component takes its smallest-rank outgoing edge (atomicMin of the rank), hooks to the
// other side's component, a mutual pair keeps its smaller root, and pointer jumping
// relabels every vertex.
__global__ void __launch_bounds__(256)
bv_reset(long long n, uint32_t* __restrict__ best, uint32_t* __restrict__ hook) {
    const long long v = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (v >= n) return;
    best[v] = 0xFFFFFFFFu;
    hook[v] = (uint32_t)v;
}

__global__ void __launch_bounds__(256)
bv_iota(long long n, uint32_t* __restrict__ a) {
    const long long v = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (v < n) a[v] = (uint32_t)v;
}

__global__ void __launch_bounds__(256)
bv_edges(const uint2* __restrict__ pairs, long long ne, const uint32_t* __restrict__ comp,
         uint32_t* __restrict__ best, int* __restrict__ any) {
    const long long e = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    bool cross = false;
    if (e < ne) {
        const uint2 pr = pairs[e];
        const uint32_t ca = comp[pr.x], cb = comp[pr.y];
        if (ca != cb) {
            cross = true;
            // (best only decreases: an edge above the current value cannot win; edges come
            // in rank order, so most lanes skip the atomic)
            if ((uint32_t)e < best[ca]) atomicMin(&best[ca], (uint32_t)e);
            if ((uint32_t)e < best[cb]) atomicMin(&best[cb], (uint32_t)e);
        }
    }
    const unsigned long long b = __ballot(cross);
    if (b && (int)(threadIdx.x & 63) == __ffsll((unsigned long long)b) - 1) *any = 1;
}

__global__ void __launch_bounds__(256)
bv_hook(const uint2* __restrict__ pairs, long long n, const uint32_t* __restrict__ comp,
        const uint32_t* __restrict__ best, uint32_t* __restrict__ hook, uint32_t* __restrict__ kept) {
    const long long c = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (c >= n || comp[c] != (uint32_t)c || best[c] == 0xFFFFFFFFu) return;
    const uint32_t e = best[c];
    const uint2 pr = pairs[e];
    const uint32_t ca = comp[pr.x];
    hook[c] = ca == (uint32_t)c ? comp[pr.y] : ca;
    kept[e] = 1u;
}

// two components that chose the same edge hook to each other: the smaller root stays a root
__global__ void __launch_bounds__(256)
bv_mutual(long long n, uint32_t* __restrict__ hook) {
    const long long c = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (c >= n) return;
    const uint32_t h = hook[c];
    if (h != (uint32_t)c && hook[h] == (uint32_t)c && (uint32_t)c < h) hook[c] = (uint32_t)c;
}

__global__ void __launch_bounds__(256)
bv_jump(long long n, uint32_t* __restrict__ hook, int* __restrict__ changed) {
    const long long c = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (c >= n) return;
    const uint32_t h = hook[c], hh = hook[h];
    if (hh != h) {
        hook[c] = hh;
        *changed = 1;
    }
}

__global__ void __launch_bounds__(256)
bv_relabel(long long n, const uint32_t* __restrict__ hook, uint32_t* __restrict__ comp) {
    const long long v = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (v < n) comp[v] = hook[comp[v]];
}

// kept edge k (rank order): forward copy k (key = source), reversed copy K + k (key = target)
__global__ void __launch_bounds__(256)
bv_emit(const uint2* __restrict__ pairs, long long ne, const uint32_t* __restrict__ kept,
        const uint32_t* __restrict__ kidx, uint32_t K, uint32_t* __restrict__ keys,
        uint32_t* __restrict__ vals, uint32_t* __restrict__ other, int* __restrict__ counts) {
    const long long e = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= ne || !kept[e]) return;
    const uint32_t k = kidx[e];
    const uint2 pr = pairs[e];
    keys[k] = pr.x;
    vals[k] = k;
    other[k] = pr.y;
    keys[K + k] = pr.y;
    vals[K + k] = K + k;
    other[K + k] = pr.x;
    atomicAdd(&counts[pr.x], 1);
    atomicAdd(&counts[pr.y], 1);
}

__global__ void __launch_bounds__(256)
bv_targets(const uint32_t* __restrict__ vals_sorted, long long m, const uint32_t* __restrict__ other,
           uint32_t* __restrict__ targets) {
    const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < m) targets[i] = other[vals_sorted[i]];
}

// ------------------------------------------------------------------ host helpers
int radix_sort_u32(pqh_ctx* ctx, DevBuf& buf, uint32_t* k_in, uint32_t* k_out, uint32_t* v_in,
                   uint32_t* v_out, long long n) {
    size_t temp = 0;
    PQH_HIP(ctx, rocprim::radix_sort_pairs(nullptr, temp, k_in, k_out, v_in, v_out, (size_t)n,
                                           0u, 32u, ctx->stream));
    void* t = buf.get<char>(temp);
    if (!t) return pqh_set_error(ctx, PQH_ERR_NOMEM, "knn: sort temp (%zu B)", temp);
    PQH_HIP(ctx, rocprim::radix_sort_pairs(t, temp, k_in, k_out, v_in, v_out, (size_t)n, 0u, 32u,
                                           ctx->stream));
    return PQH_OK;
}

int float_cmp_ref(const void* a, const void* b) {   // fast_nn_blocks_info.c:41-50
    const float v = *(const float*)a - *(const float*)b;
    if (fabs(v) < 1e-9) return 0;
    return v < 0 ? -1 : 1;
}

struct HostEdge {   // mst_edge_t (mst.h)
    uint32_t source, target;
    float dist;
};

int edge_dist_cmp_ref(const void* a, const void* b) {   // mst.c:15-26
    const float diff = ((const HostEdge*)a)->dist - ((const HostEdge*)b)->dist;
    if (fabs(diff) < 1e-9) return 0;
    return diff < 0 ? -1 : 1;
}

template <int DMAX, int KMAX>
void launch_topk(pqh_ctx* ctx, long long tiles, const float* x, long long ld, int d, int num_nn,
                 const uint32_t* rows, const long long* boff, const long long* tb,
                 const long long* tq, int stride, float* od, uint32_t* orow) {
    hipLaunchKernelGGL((knn_block_topk<DMAX, KMAX>), dim3((unsigned)tiles), dim3(kQ), 0,
                       ctx->stream, x, ld, d, num_nn, rows, boff, tb, tq, stride, od, orow);
}

template <int DMAX>
void launch_topk_k(pqh_ctx* ctx, int kmax, long long tiles, const float* x, long long ld, int d,
                   int num_nn, const uint32_t* rows, const long long* boff, const long long* tb,
                   const long long* tq, int stride, float* od, uint32_t* orow) {
    if (kmax <= 8) launch_topk<DMAX, 8>(ctx, tiles, x, ld, d, num_nn, rows, boff, tb, tq, stride, od, orow);
    else if (kmax <= 16) launch_topk<DMAX, 16>(ctx, tiles, x, ld, d, num_nn, rows, boff, tb, tq, stride, od, orow);
    else if (kmax <= 32) launch_topk<DMAX, 32>(ctx, tiles, x, ld, d, num_nn, rows, boff, tb, tq, stride, od, orow);
    else if (kmax <= 52) launch_topk<DMAX, 52>(ctx, tiles, x, ld, d, num_nn, rows, boff, tb, tq, stride, od, orow);
    else launch_topk<DMAX, 64>(ctx, tiles, x, ld, d, num_nn, rows, boff, tb, tq, stride, od, orow);
}

}  // namespace

extern "C" {

int pqh_knn_blocks_info(pqh_ctx_t* ctx, const float* d_x, long long n, long long ld_x, int d,
                        int num_split, int blocks_per_dim, double overlap, float* h_starts,
                        float* h_ends) {
    if (!ctx || !d_x || n <= 0 || d <= 0 || ld_x < d || num_split <= 0 || num_split > d ||
        num_split > 8 || blocks_per_dim <= 0 || blocks_per_dim > 32 || !h_starts || !h_ends ||
        n >= (1ll << 32))
        return PQH_ERR_ARG;
    int rc = pqh_use_device(ctx);
    if (rc) return rc;
    DevBuf buf;
    uint32_t* k0 = buf.get<uint32_t>(n);
    uint32_t* k1 = buf.get<uint32_t>(n);
    uint32_t* i0 = buf.get<uint32_t>(n);
    uint32_t* i1 = buf.get<uint32_t>(n);
    float* dse = buf.get<float>(2 * blocks_per_dim);
    int* flag = buf.get<int>(1);
    if (!k0 || !k1 || !i0 || !i1 || !dse || !flag)
        return pqh_set_error(ctx, PQH_ERR_NOMEM, "knn_blocks_info: %lld rows", n);
    const unsigned g = (unsigned)((n + 255) / 256);
    const long long ov = (long long)(n * overlap / 2);
    for (int i = 0; i < num_split; ++i) {
        const int coord = num_split - 1 - i;
        hipLaunchKernelGGL(knn_column, dim3(g), dim3(256), 0, ctx->stream, d_x, n, ld_x, coord, k0);
        PQH_LAUNCH_CHECK(ctx);
        if ((rc = radix_sort_u32(ctx, buf, k0, k1, i0, i1, n))) return rc;   // (values unused)
        PQH_HIP(ctx, hipMemsetAsync(flag, 0, sizeof(int), ctx->stream));
        hipLaunchKernelGGL(near_equal_check, dim3(g), dim3(256), 0, ctx->stream, k1, n, flag);
        PQH_LAUNCH_CHECK(ctx);
        hipLaunchKernelGGL(knn_bounds, dim3(1), dim3(64), 0, ctx->stream, k1, n, blocks_per_dim,
                           ov, dse, dse + blocks_per_dim);
        PQH_LAUNCH_CHECK(ctx);
        int hflag = 0;
        PQH_HIP(ctx, hipMemcpyAsync(&hflag, flag, sizeof(int), hipMemcpyDeviceToHost, ctx->stream));
        PQH_HIP(ctx, hipMemcpyAsync(h_starts + i * blocks_per_dim, dse, sizeof(float) * blocks_per_dim,
                                    hipMemcpyDeviceToHost, ctx->stream));
        PQH_HIP(ctx, hipMemcpyAsync(h_ends + i * blocks_per_dim, dse + blocks_per_dim,
                                    sizeof(float) * blocks_per_dim, hipMemcpyDeviceToHost, ctx->stream));
        PQH_HIP(ctx, hipStreamSynchronize(ctx->stream));
        if (hflag) {   // near-equal distinct values: the reference's own qsort decides
            std::vector<float> col((size_t)n);
            PQH_HIP(ctx, hipMemcpy2DAsync(col.data(), sizeof(float), d_x + coord, ld_x * sizeof(float),
                                          sizeof(float), (size_t)n, hipMemcpyDeviceToHost, ctx->stream));
            PQH_HIP(ctx, hipStreamSynchronize(ctx->stream));
            qsort(col.data(), (size_t)n, sizeof(float), float_cmp_ref);
            for (int b = 0; b < blocks_per_dim; ++b) {
                long long s = n * b / blocks_per_dim - ov;
                s = s < 0 ? 0 : (s > n ? n : s);
                long long e = n * (b + 1) / blocks_per_dim + ov;
                e = e < 0 ? 0 : (e > n ? n : e);
                h_starts[i * blocks_per_dim + b] = col[(size_t)(s < n ? s : n - 1)];
                h_ends[i * blocks_per_dim + b] = col[(size_t)(e < n - 1 ? e : n - 1)];
            }
            h_starts[i * blocks_per_dim] = (float)((double)col[0] - 1.0);
            h_ends[i * blocks_per_dim + blocks_per_dim - 1] = (float)((double)col[(size_t)n - 1] + 1.0);
        }
    }
    return PQH_OK;
}

int pqh_knn_fast(pqh_ctx_t* ctx, const float* d_x, long long n, long long ld_x, int d,
                 int num_nn, int num_split, int blocks_per_dim, const float* h_starts,
                 const float* h_ends, uint32_t* d_indices, float* d_dists,
                 long long* h_block_sizes) {
    if (!ctx || !d_x || n <= 0 || d <= 0 || ld_x < d || num_nn <= 0 || num_nn > 63 ||
        num_split <= 0 || num_split > d || num_split > 8 || blocks_per_dim <= 0 ||
        blocks_per_dim > 32 || !h_starts || !h_ends || !d_indices || !d_dists || n >= (1ll << 32))
        return PQH_ERR_ARG;
    if (d > 128) return pqh_set_error(ctx, PQH_ERR_UNSUPPORTED, "knn_fast: d = %d > 128", d);
    long long nblocks = 1;
    for (int i = 0; i < num_split; ++i) {
        nblocks *= blocks_per_dim;
        if (nblocks >= (1ll << 31)) return PQH_ERR_ARG;
    }
    int rc = pqh_use_device(ctx);
    if (rc) return rc;
    DevBuf buf;
    const size_t gb = sizeof(float) * num_split * blocks_per_dim;
    float* dg = buf.get<float>(2 * (size_t)num_split * blocks_per_dim);
    uint32_t* masks = buf.get<uint32_t>((size_t)n * num_split);
    uint32_t* cnt = buf.get<uint32_t>(n + 1);
    unsigned long long* off = buf.get<unsigned long long>(n + 1);
    if (!dg || !masks || !cnt || !off) return pqh_set_error(ctx, PQH_ERR_NOMEM, "knn_fast: %lld rows", n);
    PQH_HIP(ctx, hipMemcpyAsync(dg, h_starts, gb, hipMemcpyHostToDevice, ctx->stream));
    PQH_HIP(ctx, hipMemcpyAsync(dg + num_split * blocks_per_dim, h_ends, gb, hipMemcpyHostToDevice,
                                ctx->stream));
    const Geo geo{num_split, blocks_per_dim, dg, dg + num_split * blocks_per_dim};
    const unsigned g = (unsigned)((n + 255) / 256);
    hipLaunchKernelGGL(knn_masks, dim3(g), dim3(256), 0, ctx->stream, d_x, n, ld_x, geo, masks, cnt);
    PQH_LAUNCH_CHECK(ctx);
    PQH_HIP(ctx, hipMemsetAsync(cnt + n, 0, sizeof(uint32_t), ctx->stream));
    {   // off[v] = pairs of the rows before v (off[n] = all)
        size_t temp = 0;
        PQH_HIP(ctx, rocprim::exclusive_scan(nullptr, temp, cnt, off, 0ull, (size_t)n + 1,
                                             rocprim::plus<unsigned long long>(), ctx->stream));
        void* t = buf.get<char>(temp);
        if (!t) return pqh_set_error(ctx, PQH_ERR_NOMEM, "knn_fast: scan temp");
        PQH_HIP(ctx, rocprim::exclusive_scan(t, temp, cnt, off, 0ull, (size_t)n + 1,
                                             rocprim::plus<unsigned long long>(), ctx->stream));
    }
    unsigned long long npairs = 0;
    PQH_HIP(ctx, hipMemcpyAsync(&npairs, off + n, 8, hipMemcpyDeviceToHost, ctx->stream));
    PQH_HIP(ctx, hipStreamSynchronize(ctx->stream));
    if (npairs >= (1ull << 32))
        return pqh_set_error(ctx, PQH_ERR_UNSUPPORTED, "knn_fast: %llu (block, row) pairs", npairs);
    const long long np = (long long)npairs;
    uint32_t* keys = buf.get<uint32_t>(np);
    uint32_t* keys_s = buf.get<uint32_t>(np);
    uint32_t* vals = buf.get<uint32_t>(np);
    uint32_t* vals_s = buf.get<uint32_t>(np);
    uint32_t* erow = buf.get<uint32_t>(np);
    uint32_t* rows = buf.get<uint32_t>(np);
    uint32_t* inv = buf.get<uint32_t>(np);
    long long* boff = buf.get<long long>(nblocks + 1);
    const int stride = num_nn + 1;
    float* ldist = buf.get<float>((size_t)np * stride);
    uint32_t* lrow = buf.get<uint32_t>((size_t)np * stride);
    if (!keys || !keys_s || !vals || !vals_s || !erow || !rows || !inv || !boff || !ldist || !lrow)
        return pqh_set_error(ctx, PQH_ERR_NOMEM, "knn_fast: %lld pairs", np);
    const unsigned gp = (unsigned)((np + 255) / 256);
    if (np > 0) {
        hipLaunchKernelGGL(knn_emit, dim3(g), dim3(256), 0, ctx->stream, masks, n, geo, off, keys,
                           vals, erow);
        PQH_LAUNCH_CHECK(ctx);
        if ((rc = radix_sort_u32(ctx, buf, keys, keys_s, vals, vals_s, np))) return rc;
        hipLaunchKernelGGL(knn_place, dim3(gp), dim3(256), 0, ctx->stream, vals_s, np, erow, rows, inv);
        PQH_LAUNCH_CHECK(ctx);
    }
    hipLaunchKernelGGL(knn_block_offsets, dim3((unsigned)((nblocks + 256) / 256)), dim3(256), 0,
                       ctx->stream, keys_s, np, nblocks, boff);
    PQH_LAUNCH_CHECK(ctx);
    // the tile list: (block, first query) of every 64 queries of every block
    std::vector<long long> hb((size_t)nblocks + 1);
    PQH_HIP(ctx, hipMemcpyAsync(hb.data(), boff, sizeof(long long) * (nblocks + 1),
                                hipMemcpyDeviceToHost, ctx->stream));
    PQH_HIP(ctx, hipStreamSynchronize(ctx->stream));
    long long max_s = 0;
    for (long long b = 0; b < nblocks; ++b) {
        const long long S = hb[b + 1] - hb[b];
        if (h_block_sizes) h_block_sizes[b] = S;
        max_s = S > max_s ? S : max_s;
    }
    const int kmax = (int)((num_nn < max_s - 1 ? num_nn : max_s - 1) + 1);
    // the tile list: (block, first query) of every tq queries of every block
    auto tiles_of = [&](int tqn, std::vector<long long>& tb, std::vector<long long>& tq) {
        for (long long b = 0; b < nblocks; ++b)
            for (long long q0 = 0; q0 < hb[b + 1] - hb[b]; q0 += tqn) {
                tb.push_back(b);
                tq.push_back(q0);
            }
    };
    auto upload = [&](const std::vector<long long>& v, long long** dv) -> int {
        *dv = buf.get<long long>(v.size());
        if (!*dv) return pqh_set_error(ctx, PQH_ERR_NOMEM, "knn_fast: tiles");
        PQH_HIP(ctx, hipMemcpyAsync(*dv, v.data(), sizeof(long long) * v.size(),
                                    hipMemcpyHostToDevice, ctx->stream));
        return PQH_OK;
    };
    static const bool valu_impl = [] {
        const char* e = std::getenv("PQH_KNN_IMPL");
        return e && std::strcmp(e, "valu") == 0;
    }();
    if (np > 0 && valu_impl) {   // exact VALU distances for every pair (knn_block_topk)
        std::vector<long long> tb, tq;
        tiles_of(kQ, tb, tq);
        const long long tiles = (long long)tb.size();
        long long *dtb = nullptr, *dtq = nullptr;
        if ((rc = upload(tb, &dtb)) || (rc = upload(tq, &dtq))) return rc;
        if (d <= 8)
            launch_topk_k<8>(ctx, kmax, tiles, d_x, ld_x, d, num_nn, rows, boff, dtb, dtq, stride, ldist, lrow);
        else if (d <= 16)
            launch_topk_k<16>(ctx, kmax, tiles, d_x, ld_x, d, num_nn, rows, boff, dtb, dtq, stride, ldist, lrow);
        else if (d <= 32)
            launch_topk_k<32>(ctx, kmax, tiles, d_x, ld_x, d, num_nn, rows, boff, dtb, dtq, stride, ldist, lrow);
        else if (d <= 64)
            launch_topk_k<64>(ctx, kmax, tiles, d_x, ld_x, d, num_nn, rows, boff, dtb, dtq, stride, ldist, lrow);
        else if (d <= 96)
            launch_topk_k<96>(ctx, kmax, tiles, d_x, ld_x, d, num_nn, rows, boff, dtb, dtq, stride, ldist, lrow);
        else
            launch_topk_k<128>(ctx, kmax, tiles, d_x, ld_x, d, num_nn, rows, boff, dtb, dtq, stride, ldist, lrow);
        PQH_LAUNCH_CHECK(ctx);
    } else if (np > 0) {   // MFMA screen + exact selection
        const int dp = d <= 16 ? 16 : d <= 32 ? 32 : d <= 64 ? 64 : 128;
        const int ch = 2 * kmax + 16;   // listed candidates per half-wave lane before a full scan
        kbf16x8* xhi = buf.get<kbf16x8>((size_t)n * (dp / 8));
        kbf16x8* xlo = buf.get<kbf16x8>((size_t)n * (dp / 8));
        float* nrm = buf.get<float>(n);
        float* xpad = buf.get<float>((size_t)n * dp);
        uint32_t* cmx = buf.get<uint32_t>(nblocks);
        uint32_t* cand = buf.get<uint32_t>((size_t)np * 2 * ch);
        uint32_t* ccnt = buf.get<uint32_t>((size_t)np * 2);
        if (!xhi || !xlo || !nrm || !xpad || !cmx || !cand || !ccnt)
            return pqh_set_error(ctx, PQH_ERR_NOMEM, "knn_fast: screen buffers (%lld pairs)", np);
        std::vector<long long> tb, tq;
        tiles_of(kScreenQ, tb, tq);
        const long long tiles = (long long)tb.size();
        long long *dtb = nullptr, *dtq = nullptr;
        if ((rc = upload(tb, &dtb)) || (rc = upload(tq, &dtq))) return rc;
        PQH_HIP(ctx, hipMemsetAsync(cmx, 0, sizeof(uint32_t) * nblocks, ctx->stream));
        const unsigned gn = (unsigned)((n * (dp / 8) + 255) / 256);
#define PQH_KNN_SPLIT(DP_)                                                                       \
    hipLaunchKernelGGL(knn_split<DP_>, dim3(gn), dim3(256), 0, ctx->stream, d_x, n, ld_x, d, xhi,   \
                       xlo, nrm, xpad)
        if (dp == 16) PQH_KNN_SPLIT(16);
        else if (dp == 32) PQH_KNN_SPLIT(32);
        else if (dp == 64) PQH_KNN_SPLIT(64);
        else PQH_KNN_SPLIT(128);
#undef PQH_KNN_SPLIT
        PQH_LAUNCH_CHECK(ctx);
        hipLaunchKernelGGL(knn_block_cmax, dim3(gp), dim3(256), 0, ctx->stream, keys_s, rows, np, nrm, cmx);
        PQH_LAUNCH_CHECK(ctx);
#define PQH_KNN_SCREEN(DP_, K_)                                                                  \
    hipLaunchKernelGGL((knn_screen<DP_, K_>), dim3((unsigned)tiles), dim3(64), 0, ctx->stream, xhi, \
                       xlo, nrm, rows, boff, cmx, dtb, dtq, num_nn, d, ch, cand, ccnt)
#define PQH_KNN_SCREEN_K(DP_)                                                                    \
    do {                                                                                         \
        if (kmax <= 8) PQH_KNN_SCREEN(DP_, 8);                                                    \
        else if (kmax <= 16) PQH_KNN_SCREEN(DP_, 16);                                             \
        else if (kmax <= 32) PQH_KNN_SCREEN(DP_, 32);                                             \
        else if (kmax <= 52) PQH_KNN_SCREEN(DP_, 52);                                             \
        else PQH_KNN_SCREEN(DP_, 64);                                                             \
    } while (0)
        if (dp == 16) PQH_KNN_SCREEN_K(16);
        else if (dp == 32) PQH_KNN_SCREEN_K(32);
        else if (dp == 64) PQH_KNN_SCREEN_K(64);
        else PQH_KNN_SCREEN_K(128);
#undef PQH_KNN_SCREEN_K
#undef PQH_KNN_SCREEN
        PQH_LAUNCH_CHECK(ctx);
        const unsigned gs = (unsigned)((np + 63) / 64);
        static const bool lane_select = [] {
            const char* e = std::getenv("PQH_KNN_SELECT");
            return e && std::strcmp(e, "lane") == 0;
        }();
        if (!lane_select) {   // one wave per query (default)
            const unsigned gw = (unsigned)((np + 3) / 4);
#define PQH_KNN_SELECT_W(DP_)                                                                    \
    hipLaunchKernelGGL((knn_select_wave<DP_>), dim3(gw), dim3(256), 0, ctx->stream, xpad, num_nn,  \
                       rows, keys_s, boff, np, ch, cand, ccnt, stride, ldist, lrow)
            if (dp == 16) PQH_KNN_SELECT_W(16);
            else if (dp == 32) PQH_KNN_SELECT_W(32);
            else if (dp == 64) PQH_KNN_SELECT_W(64);
            else PQH_KNN_SELECT_W(128);
#undef PQH_KNN_SELECT_W
            PQH_LAUNCH_CHECK(ctx);
        } else {
#define PQH_KNN_SELECT(DM_, K_)                                                                  \
    hipLaunchKernelGGL((knn_select<DM_, K_>), dim3(gs), dim3(64), 0, ctx->stream, xpad, num_nn,    \
                       rows, keys_s, boff, np, ch, cand, ccnt, stride, ldist, lrow)
#define PQH_KNN_SELECT_K(DM_)                                                                    \
    do {                                                                                         \
        if (kmax <= 8) PQH_KNN_SELECT(DM_, 8);                                                    \
        else if (kmax <= 16) PQH_KNN_SELECT(DM_, 16);                                             \
        else if (kmax <= 32) PQH_KNN_SELECT(DM_, 32);                                             \
        else if (kmax <= 52) PQH_KNN_SELECT(DM_, 52);                                             \
        else PQH_KNN_SELECT(DM_, 64);                                                             \
    } while (0)
        if (dp == 16) PQH_KNN_SELECT_K(16);
        else if (dp == 32) PQH_KNN_SELECT_K(32);
        else if (dp == 64) PQH_KNN_SELECT_K(64);
        else PQH_KNN_SELECT_K(128);
#undef PQH_KNN_SELECT_K
#undef PQH_KNN_SELECT
        PQH_LAUNCH_CHECK(ctx);
        }
    }
    hipLaunchKernelGGL(knn_merge, dim3((unsigned)((n + kQ - 1) / kQ)), dim3(kQ),
                       sizeof(NnItem) * kQ * num_nn, ctx->stream, n, num_nn, off, inv, keys_s, boff,
                       stride, ldist, lrow, d_indices, d_dists);
    PQH_LAUNCH_CHECK(ctx);
    PQH_HIP(ctx, hipStreamSynchronize(ctx->stream));   // the call's buffers are freed on return
    return PQH_OK;
}

int pqh_mst_build(pqh_ctx_t* ctx, const uint32_t* d_indices, const float* d_dists, long long n,
                  int num_nn, int take, const uint8_t* d_pq, int pq_m, float penalty,
                  uint32_t* h_targets, int* h_counts, long long* num_edges) {
    if (!ctx || !d_indices || !d_dists || n <= 0 || num_nn <= 0 || num_nn > 63 || take <= 0 ||
        take > num_nn || !h_targets || !h_counts || !num_edges || n >= (1ll << 32) ||
        (penalty > 0.0f && (!d_pq || pq_m <= 0)))
        return PQH_ERR_ARG;
    int rc = pqh_use_device(ctx);
    if (rc) return rc;
    const long long ne = n * take;
    if (ne >= (1ll << 32)) return pqh_set_error(ctx, PQH_ERR_UNSUPPORTED, "mst: %lld edges", ne);
    DevBuf buf;
    uint32_t* keys = buf.get<uint32_t>(ne);
    uint32_t* keys_s = buf.get<uint32_t>(ne);
    uint32_t* vals = buf.get<uint32_t>(ne);
    uint32_t* vals_s = buf.get<uint32_t>(ne);
    uint32_t* src = buf.get<uint32_t>(ne);
    uint32_t* dst = buf.get<uint32_t>(ne);
    float* edist = buf.get<float>(ne);
    uint2* pairs = buf.get<uint2>(ne);
    int* flag = buf.get<int>(2);
    if (!keys || !keys_s || !vals || !vals_s || !src || !dst || !edist || !pairs || !flag)
        return pqh_set_error(ctx, PQH_ERR_NOMEM, "mst: %lld edges", ne);
    PQH_HIP(ctx, hipMemsetAsync(flag, 0, 2 * sizeof(int), ctx->stream));
    hipLaunchKernelGGL(mst_row_edges, dim3((unsigned)((n + kQ - 1) / kQ)), dim3(kQ),
                       sizeof(NnItem) * kQ * num_nn, ctx->stream, d_indices, d_dists, n, num_nn,
                       take, d_pq, pq_m, penalty, keys, vals, src, dst, edist, flag);
    PQH_LAUNCH_CHECK(ctx);
    if ((rc = radix_sort_u32(ctx, buf, keys, keys_s, vals, vals_s, ne))) return rc;
    const unsigned ge = (unsigned)((ne + 255) / 256);
    hipLaunchKernelGGL(near_equal_check, dim3(ge), dim3(256), 0, ctx->stream, keys_s, ne, flag + 1);
    PQH_LAUNCH_CHECK(ctx);
    hipLaunchKernelGGL(gather_pairs, dim3(ge), dim3(256), 0, ctx->stream, vals_s, ne, src, dst, pairs);
    PQH_LAUNCH_CHECK(ctx);
    int hflag[2] = {0, 0};
    PQH_HIP(ctx, hipMemcpyAsync(hflag, flag, sizeof(hflag), hipMemcpyDeviceToHost, ctx->stream));
    PQH_HIP(ctx, hipStreamSynchronize(ctx->stream));
    if (hflag[0] & 1) return pqh_set_error(ctx, PQH_ERR_ARG, "mst: a neighbour id outside the rows");
    if ((hflag[0] & 2) || hflag[1]) {
        // distinct distances inside the comparator's 1e-9 band: the reference's qsorts decide
        std::vector<uint32_t> hi((size_t)n * num_nn);
        std::vector<float> hd((size_t)n * num_nn);
        std::vector<uint8_t> hp(penalty > 0.0f ? (size_t)n * pq_m : 0);
        PQH_HIP(ctx, hipMemcpyAsync(hi.data(), d_indices, hi.size() * 4, hipMemcpyDeviceToHost, ctx->stream));
        PQH_HIP(ctx, hipMemcpyAsync(hd.data(), d_dists, hd.size() * 4, hipMemcpyDeviceToHost, ctx->stream));
        if (!hp.empty())
            PQH_HIP(ctx, hipMemcpyAsync(hp.data(), d_pq, hp.size(), hipMemcpyDeviceToHost, ctx->stream));
        PQH_HIP(ctx, hipStreamSynchronize(ctx->stream));
        std::vector<HostEdge> all((size_t)ne), row((size_t)num_nn);
        for (long long v = 0; v < n; ++v) {
            for (int j = 0; j < num_nn; ++j) {
                HostEdge& e = row[j];
                e.source = (uint32_t)v;
                e.target = hi[(size_t)v * num_nn + j];
                e.dist = hd[(size_t)v * num_nn + j];
                if (penalty > 0.0f) {
                    int ham = 0;
                    for (int i = 0; i < pq_m; ++i)
                        ham += hp[(size_t)v * pq_m + i] != hp[(size_t)e.target * pq_m + i];
                    if (std::isinf(penalty)) e.dist = (float)ham;
                    else e.dist += ham * penalty;
                }
            }
            if (penalty > 0.0f) qsort(row.data(), (size_t)num_nn, sizeof(HostEdge), edge_dist_cmp_ref);
            for (int j = 0; j < take; ++j) all[(size_t)v * take + j] = row[j];
        }
        qsort(all.data(), (size_t)ne, sizeof(HostEdge), edge_dist_cmp_ref);
        std::vector<uint2> ed((size_t)ne);
        for (long long e = 0; e < ne; ++e) ed[e] = make_uint2(all[e].source, all[e].target);
        PQH_HIP(ctx, hipMemcpyAsync(pairs, ed.data(), sizeof(uint2) * ne, hipMemcpyHostToDevice, ctx->stream));
        PQH_HIP(ctx, hipStreamSynchronize(ctx->stream));   // (ed goes out of scope)
    }
    // Boruvka on the device (the same forest as Kruskal's scan, mst.c:185-201)
    uint32_t* comp = buf.get<uint32_t>(n);
    uint32_t* best = buf.get<uint32_t>(n);
    uint32_t* hook = buf.get<uint32_t>(n);
    uint32_t* kept = buf.get<uint32_t>(ne + 1);
    uint32_t* kidx = buf.get<uint32_t>(ne + 1);
    int* fl = buf.get<int>(2);
    if (!comp || !best || !hook || !kept || !kidx || !fl)
        return pqh_set_error(ctx, PQH_ERR_NOMEM, "mst: forest buffers");
    const unsigned gn = (unsigned)((n + 255) / 256);
    hipLaunchKernelGGL(bv_iota, dim3(gn), dim3(256), 0, ctx->stream, n, comp);
    PQH_LAUNCH_CHECK(ctx);
    PQH_HIP(ctx, hipMemsetAsync(kept, 0, sizeof(uint32_t) * (ne + 1), ctx->stream));
    for (int round = 0; round < 64; ++round) {
        PQH_HIP(ctx, hipMemsetAsync(fl, 0, 2 * sizeof(int), ctx->stream));
        hipLaunchKernelGGL(bv_reset, dim3(gn), dim3(256), 0, ctx->stream, n, best, hook);
        hipLaunchKernelGGL(bv_edges, dim3(ge), dim3(256), 0, ctx->stream, pairs, ne, comp, best, fl);
        hipLaunchKernelGGL(bv_hook, dim3(gn), dim3(256), 0, ctx->stream, pairs, n, comp, best, hook, kept);
        hipLaunchKernelGGL(bv_mutual, dim3(gn), dim3(256), 0, ctx->stream, n, hook);
        PQH_LAUNCH_CHECK(ctx);
        int any = 0;
        PQH_HIP(ctx, hipMemcpyAsync(&any, fl, sizeof(int), hipMemcpyDeviceToHost, ctx->stream));
        PQH_HIP(ctx, hipStreamSynchronize(ctx->stream));
        if (!any) break;
        for (int j = 0; j < 64; ++j) {   // pointer jumping to the roots
            PQH_HIP(ctx, hipMemsetAsync(fl + 1, 0, sizeof(int), ctx->stream));
            hipLaunchKernelGGL(bv_jump, dim3(gn), dim3(256), 0, ctx->stream, n, hook, fl + 1);
            PQH_LAUNCH_CHECK(ctx);
            int changed = 0;
            PQH_HIP(ctx, hipMemcpyAsync(&changed, fl + 1, sizeof(int), hipMemcpyDeviceToHost, ctx->stream));
            PQH_HIP(ctx, hipStreamSynchronize(ctx->stream));
            if (!changed) break;
        }
        hipLaunchKernelGGL(bv_relabel, dim3(gn), dim3(256), 0, ctx->stream, n, hook, comp);
        PQH_LAUNCH_CHECK(ctx);
    }
    {   // kidx = exclusive scan of the kept flags (kidx[ne] = K)
        size_t temp = 0;
        PQH_HIP(ctx, rocprim::exclusive_scan(nullptr, temp, kept, kidx, 0u, (size_t)ne + 1,
                                             rocprim::plus<uint32_t>(), ctx->stream));
        void* t = buf.get<char>(temp);
        if (!t) return pqh_set_error(ctx, PQH_ERR_NOMEM, "mst: scan temp");
        PQH_HIP(ctx, rocprim::exclusive_scan(t, temp, kept, kidx, 0u, (size_t)ne + 1,
                                             rocprim::plus<uint32_t>(), ctx->stream));
    }
    uint32_t K = 0;
    PQH_HIP(ctx, hipMemcpyAsync(&K, kidx + ne, 4, hipMemcpyDeviceToHost, ctx->stream));
    PQH_HIP(ctx, hipStreamSynchronize(ctx->stream));
    const long long m2 = 2 * (long long)K;
    uint32_t* akeys = buf.get<uint32_t>(m2);
    uint32_t* akeys_s = buf.get<uint32_t>(m2);
    uint32_t* avals = buf.get<uint32_t>(m2);
    uint32_t* avals_s = buf.get<uint32_t>(m2);
    uint32_t* other = buf.get<uint32_t>(m2);
    uint32_t* tg = buf.get<uint32_t>(m2);
    int* cnt = buf.get<int>(n);
    if (!akeys || !akeys_s || !avals || !avals_s || !other || !tg || !cnt)
        return pqh_set_error(ctx, PQH_ERR_NOMEM, "mst: adjacency buffers");
    PQH_HIP(ctx, hipMemsetAsync(cnt, 0, sizeof(int) * n, ctx->stream));
    hipLaunchKernelGGL(bv_emit, dim3(ge), dim3(256), 0, ctx->stream, pairs, ne, kept, kidx, K, akeys,
                       avals, other, cnt);
    PQH_LAUNCH_CHECK(ctx);
    if (m2 > 0) {
        // both directions stably by source (mst.c:204-214): forward copies first, then the
        // reversed ones, each in acceptance order
        if ((rc = radix_sort_u32(ctx, buf, akeys, akeys_s, avals, avals_s, m2))) return rc;
        hipLaunchKernelGGL(bv_targets, dim3((unsigned)((m2 + 255) / 256)), dim3(256), 0, ctx->stream,
                           avals_s, m2, other, tg);
        PQH_LAUNCH_CHECK(ctx);
        PQH_HIP(ctx, hipMemcpyAsync(h_targets, tg, sizeof(uint32_t) * m2, hipMemcpyDeviceToHost, ctx->stream));
    }
    PQH_HIP(ctx, hipMemcpyAsync(h_counts, cnt, sizeof(int) * n, hipMemcpyDeviceToHost, ctx->stream));
    PQH_HIP(ctx, hipStreamSynchronize(ctx->stream));
    *num_edges = m2;
    return PQH_OK;
}

}  // extern "C"
