// pqh_tree_dev.hip -- tree mode's DFS order on the device (pqh_tree_order_device).
//
// tree_collect_vertices_dfs (mst.c:290-364) walks a stored forest with a stack, marking a
// vertex when it is pushed: roots are the lowest unvisited ids, a vertex's unvisited
// neighbours are pushed in adjacency order and therefore visited in REVERSE adjacency order.
// On a forest that is the preorder in which every tree is rooted at its smallest vertex id,
// trees come in root-id order and the children of a vertex in reverse adjacency order; the
// traverser's active parent of a row (mst.c:366-405) is the vertex's tree parent.  Computed
// without a sequential walk:
//   twins      every directed edge u->v paired with v->u (a radix sort of the undirected
//              keys); a self-loop, a repeated edge or an unpaired edge is not a forest --
//              PQH_ERR_UNSUPPORTED, and the caller walks on the host (pqh_tree_order)
//   tours      succ(u->v) = the edge after v->u in v's list (cyclic): the faces of the
//              graph's rotation system, one Euler tour per tree of a forest
//   ranking    pointer jumping on (the tour's smallest edge id m, distance to it) keys: m is
//              the first edge of the component's smallest vertex; pos(e) = distance from m
//   forest?    every vertex's edges on one tour (then tours = components) and
//              edges / 2 = vertices - isolated - tours (then every component is a tree)
//   parents    u->v goes down when it precedes v->u on the tour; subtree size = half the
//              distance between the two
//   preorder   off(c) = 1 + sizes of the children after c in its parent's list (a scan over
//              the edges); pre(v) = the tree's offset + the sum of off over v's ancestors --
//              a prefix sum along the tours (+off at the edge down, -off at the edge back)
//
// pqh_tree_ext_index_device: the decoder's traverser (huffman_decoder.c:214-247) over the
// decoded child counts, without a walk.  Row p pops one slot of the stack's top entry (its
// context) unless the stack is empty (a root), then pushes nch[p] slots.  With
// E(p) = sum_{q<=p} (nch[q] - 1), p is a root exactly when E(p - 1) is a new strict minimum
// below 0 (E falls by at most one per row); the stack depth is D(p) = E(p) + roots so far,
// and the depth after p's pop is L(p) = D(p) - nch[p].  The slot p pops sits at depth
// D(p - 1) = L(p) + 1 and was pushed by the last row q < p with L(q) < D(p - 1): p's context
// is the nearest earlier row with L(q) <= L(p) (a min-tree search).
#include <rocprim/device/device_radix_sort.hpp>
#include <rocprim/device/device_scan.hpp>

#include <algorithm>
#include <climits>
#include <vector>

#include "pqh_internal.h"

namespace {

#define G1(n) dim3((unsigned)(((n) + 255) / 256)), dim3(256)

// one atomic per wave for a count of lanes
__device__ inline void wave_count(bool pred, int* ctr) {
    const unsigned long long b = __ballot(pred);
    if (b && (int)(threadIdx.x & 63) == __ffsll((unsigned long long)b) - 1) atomicAdd(ctr, __popcll(b));
}

__global__ void __launch_bounds__(256)
td_vertex_init(long long n, const int* __restrict__ counts, uint32_t* __restrict__ parent,
               uint32_t* __restrict__ rootL, int* __restrict__ flags) {
    const long long v = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    const bool in = v < n;
    const int c = in ? counts[v] : 1;
    if (c < 0) flags[0] = 1;
    wave_count(in && c == 0, flags + 2);   // isolated vertices
    if (!in) return;
    parent[v] = (uint32_t)v;
    rootL[v] = 0;
}

// the source of every edge (CSR rows), and the undirected key of every edge
__global__ void __launch_bounds__(256)
td_edges(const uint32_t* __restrict__ first, long long n, const uint32_t* __restrict__ tg,
         uint32_t* __restrict__ src, unsigned long long* __restrict__ key, uint32_t* __restrict__ idx) {
    const long long v = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (v >= n) return;
    for (uint32_t e = first[v]; e < first[v + 1]; ++e) {
        src[e] = (uint32_t)v;
        const uint32_t t = tg[e];
        const uint32_t a = (uint32_t)v < t ? (uint32_t)v : t, b = (uint32_t)v < t ? t : (uint32_t)v;
        key[e] = ((unsigned long long)a << 32) | b;
        idx[e] = e;
    }
}

// twins from the sorted keys: every key exactly twice, from two different sources
__global__ void __launch_bounds__(256)
td_twins(const unsigned long long* __restrict__ ks, const uint32_t* __restrict__ is, long long ne,
         const uint32_t* __restrict__ src, uint32_t* __restrict__ twin, int* __restrict__ bad) {
    const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= ne) return;
    if ((i & 1) == 0) {
        const bool ok = i + 1 < ne && ks[i] == ks[i + 1] && (uint32_t)(ks[i] >> 32) != (uint32_t)ks[i] &&
                        src[is[i]] != src[is[i + 1]];
        if (!ok) {
            *bad = 1;
            return;
        }
        twin[is[i]] = is[i + 1];
        twin[is[i + 1]] = is[i];
    } else if (i + 1 < ne && ks[i] == ks[i + 1]) {
        *bad = 1;
    }
}

// succ(u->v) = the edge after v->u in v's list, cyclic; key = (own id, distance 0)
__global__ void __launch_bounds__(256)
td_succ(const uint32_t* __restrict__ first, const uint32_t* __restrict__ tg,
        const uint32_t* __restrict__ twin, long long ne, uint32_t* __restrict__ succ,
        uint32_t* __restrict__ jmp, unsigned long long* __restrict__ key) {
    const long long e = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= ne) return;
    const uint32_t v = tg[e], t = twin[e];
    const uint32_t s = t + 1 == first[v + 1] ? first[v] : t + 1;
    succ[e] = s;
    jmp[e] = s;
    key[e] = (unsigned long long)e << 32;
}

// one pointer-jumping round: the window [e, e + 2 span) from [e, e + span) and
// [j, j + span), j = e + span; key = (smallest edge id, distance to its first occurrence)
__global__ void __launch_bounds__(256)
td_jump(long long ne, unsigned span, const uint32_t* __restrict__ j0,
        const unsigned long long* __restrict__ k0, uint32_t* __restrict__ j1,
        unsigned long long* __restrict__ k1) {
    const long long e = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= ne) return;
    const uint32_t j = j0[e];
    const unsigned long long a = k0[e], b = k0[j] + span;
    k1[e] = a < b ? a : b;
    j1[e] = j0[j];
}

// forest test: all edges of a vertex on one tour; tours counted (edges at distance 0)
__global__ void __launch_bounds__(256)
td_verify(const uint32_t* __restrict__ first, const uint32_t* __restrict__ src,
          const unsigned long long* __restrict__ key, long long ne, int* __restrict__ flags) {
    const long long e = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    const bool in = e < ne;
    unsigned long long k = 1;
    if (in) {
        k = key[e];
        if ((k >> 32) != (key[first[src[e]]] >> 32)) flags[0] = 1;
    }
    wave_count(in && (uint32_t)k == 0u, flags + 3);
}

// position on the tour from its smallest edge m: L - d, with L - 1 = d(succ(m))
__device__ inline uint32_t tour_pos(const unsigned long long* __restrict__ key,
                                    const uint32_t* __restrict__ succ, uint32_t e) {
    const unsigned long long k = key[e];
    const uint32_t d = (uint32_t)k;
    if (!d) return 0u;
    return (uint32_t)key[succ[(uint32_t)(k >> 32)]] + 1u - d;
}

// parents (the edge down), subtree sizes, tour lengths of the roots
__global__ void __launch_bounds__(256)
td_parents(const uint32_t* __restrict__ tg, const uint32_t* __restrict__ src,
           const uint32_t* __restrict__ twin, const uint32_t* __restrict__ succ,
           const unsigned long long* __restrict__ key, long long ne, uint32_t* __restrict__ parent,
           uint32_t* __restrict__ size, uint32_t* __restrict__ posdown, uint32_t* __restrict__ rootof,
           uint32_t* __restrict__ rootL) {
    const long long e = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= ne) return;
    const uint32_t pe = tour_pos(key, succ, (uint32_t)e), pt = tour_pos(key, succ, twin[e]);
    if (pe < pt) {   // e = u->v comes first: v's parent is u
        const uint32_t v = tg[e];
        parent[v] = src[e];
        size[v] = (pt - pe + 1) / 2;
        posdown[v] = pe;
        rootof[v] = src[(uint32_t)(key[e] >> 32)];
    }
    if (pe == 0) rootL[src[e]] = (uint32_t)key[succ[e]] + 1u;
}

// per root: (vertex count << 32) | tour length, scanned into the trees' offsets
__global__ void __launch_bounds__(256)
td_roots(long long n, const uint32_t* __restrict__ parent, const uint32_t* __restrict__ rootL,
         uint32_t* __restrict__ size, unsigned long long* __restrict__ rinfo) {
    const long long v = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (v > n) return;
    unsigned long long x = 0ull;
    if (v < n && parent[v] == (uint32_t)v) {
        const uint32_t len = rootL[v];
        size[v] = len / 2 + 1;
        x = ((unsigned long long)(len / 2 + 1) << 32) | len;
    }
    rinfo[v] = x;
}

// w(e) = size of the child below a down edge, 0 for the edge to the parent
__global__ void __launch_bounds__(256)
td_weights(const uint32_t* __restrict__ tg, const uint32_t* __restrict__ src,
           const uint32_t* __restrict__ parent, const uint32_t* __restrict__ size, long long ne,
           uint32_t* __restrict__ w) {
    const long long e = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= ne) return;
    const uint32_t c = tg[e];
    w[e] = parent[c] == src[e] ? size[c] : 0u;
}

// off(c) = 1 + sizes of the children after c in its parent's list (W = inclusive sums;
// differences mod 2^32 are exact, each below n)
__global__ void __launch_bounds__(256)
td_offsets(const uint32_t* __restrict__ first, const uint32_t* __restrict__ tg,
           const uint32_t* __restrict__ src, const uint32_t* __restrict__ parent,
           const uint32_t* __restrict__ W, long long ne, uint32_t* __restrict__ offc) {
    const long long e = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= ne) return;
    const uint32_t c = tg[e], v = src[e];
    if (parent[c] != v) return;
    offc[c] = 1u + (W[first[v + 1] - 1] - W[e]);
}

// the tours laid out one after another (trees in root-id order): +off(child) at the edge
// down, -off(child) at the edge back up
__global__ void __launch_bounds__(256)
td_tour(const uint32_t* __restrict__ tg, const uint32_t* __restrict__ src,
        const uint32_t* __restrict__ twin, const uint32_t* __restrict__ succ,
        const unsigned long long* __restrict__ key, const unsigned long long* __restrict__ rbase,
        const uint32_t* __restrict__ offc, long long ne, int* __restrict__ val) {
    const long long e = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= ne) return;
    const uint32_t pe = tour_pos(key, succ, (uint32_t)e), pt = tour_pos(key, succ, twin[e]);
    const uint32_t r = src[(uint32_t)(key[e] >> 32)];
    val[(uint32_t)rbase[r] + pe] = pe < pt ? (int)offc[tg[e]] : -(int)offc[src[e]];
}

__global__ void __launch_bounds__(256)
td_output(long long n, const uint32_t* __restrict__ first, const uint32_t* __restrict__ parent,
          const uint32_t* __restrict__ posdown, const uint32_t* __restrict__ rootof,
          const unsigned long long* __restrict__ rbase, const int* __restrict__ S,
          uint32_t* __restrict__ vertices, int* __restrict__ num_children,
          long long* __restrict__ parents) {
    const long long v = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (v >= n) return;
    const bool rt = parent[v] == (uint32_t)v;
    long long pre;
    if (rt) {
        pre = (long long)(rbase[v] >> 32);
    } else {
        const unsigned long long b = rbase[rootof[v]];
        pre = (long long)(b >> 32) + S[(uint32_t)b + posdown[v]];
    }
    const int deg = (int)(first[v + 1] - first[v]);
    vertices[pre] = (uint32_t)v;
    num_children[pre] = rt ? deg : deg - 1;
    if (parents) parents[pre] = rt ? -1ll : (long long)parent[v];
}

struct Arena {
    char* base = nullptr;
    size_t used = 0;
    template <typename T>
    T* take(size_t count) {
        T* p = reinterpret_cast<T*>(base ? base + used : nullptr);
        used += (count * sizeof(T) + 255) & ~size_t(255);
        return p;
    }
};

// ---------------------------------------------------------------- decoder's traverser
template <typename T>
__global__ void __launch_bounds__(256)
tx_vals(const T* __restrict__ nch, long long n, long long* __restrict__ val) {
    const long long p = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (p < n) val[p] = (long long)nch[p] - 1;
}

// roots (E(p-1) a new strict minimum below 0), as 0/1 for a sum scan
__global__ void __launch_bounds__(256)
tx_roots(const long long* __restrict__ E, const long long* __restrict__ PM, long long n,
         long long* __restrict__ root) {
    const long long p = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (p >= n) return;
    const long long before = p >= 2 && PM[p - 2] < 0 ? PM[p - 2] : 0;   // min(0, E(0..p-2))
    root[p] = (p == 0 || E[p - 1] < before) ? 1 : 0;
}

// L(p) = E(p) + R(p) - nch[p] (level 0 of the min tree); roots marked for the query
template <typename T>
__global__ void __launch_bounds__(256)
tx_levels0(const T* __restrict__ nch, const long long* __restrict__ E,
           const long long* __restrict__ R, long long n, long long* __restrict__ L) {
    const long long p = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (p < n) L[p] = E[p] + R[p] - (long long)nch[p];
}

__global__ void __launch_bounds__(256)
tx_level_up(const long long* __restrict__ lo, long long nlo, long long* __restrict__ hi, long long nhi) {
    const long long j = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= nhi) return;
    const long long a = lo[2 * j];
    const long long b = 2 * j + 1 < nlo ? lo[2 * j + 1] : LLONG_MAX;
    hi[j] = a < b ? a : b;
}

// context row of p: the nearest earlier row with L <= L(p) (climb to the first block holding
// one, then descend to its rightmost); roots have none.  Ext flag: a context before p's chunk.
__global__ void __launch_bounds__(256)
tx_query(const long long* __restrict__ levels, const long long* __restrict__ loff, int nlev,
         const long long* __restrict__ rootflag, long long n, int C,
         long long* __restrict__ parent_pos, long long* __restrict__ ext) {
    const long long p = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (p >= n) return;
    long long q = -1;
    if (!rootflag[p]) {
        const long long x = levels[p];
        int k = 0;
        long long j = p - 1;
        while (j >= 0 && levels[loff[k] + j] > x) {
            if (j & 1) {
                j -= 1;
            } else {
                j = j / 2 - 1;
                ++k;
                if (k >= nlev) { j = -1; break; }
            }
        }
        if (j >= 0) {
            while (k > 0) {
                --k;
                j = 2 * j + 1;   // the right child, unless it is past the level's end
                if (j >= loff[k + 1] - loff[k] || levels[loff[k] + j] > x) j -= 1;
            }
            q = j;
        }
    }
    parent_pos[p] = q;
    ext[p] = (q >= 0 && q < p - p % C) ? 1 : 0;
}

// the contexts before their chunk, in row order (the encoder gathers these rows)
__global__ void __launch_bounds__(256)
tx_compact(const long long* __restrict__ ext, const long long* __restrict__ S,
           const long long* __restrict__ parent_pos, long long n, long long* __restrict__ pos) {
    const long long p = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (p < n && ext[p]) pos[S[p] - 1] = parent_pos[p];
}

__global__ void __launch_bounds__(256)
tx_offsets(const long long* __restrict__ S, long long n, int C, long long chunks,
           long long* __restrict__ eo) {
    const long long c = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (c > chunks) return;
    const long long end = c * C < n ? c * C : n;   // rows before chunk c
    eo[c] = end > 0 ? S[end - 1] : 0;
}

int ceil_log2(long long x) {
    int r = 0;
    while ((1ll << r) < x) ++r;
    return r;
}

}  // namespace

extern "C" int pqh_tree_order_device(pqh_ctx_t* ctx, long long n, long long ne,
                                     const uint32_t* d_targets, const int* d_counts,
                                     uint32_t* d_vertices, int* d_num_children,
                                     long long* d_parents, int* num_roots) {
    if (!ctx || n <= 0 || ne < 0 || !d_counts || (ne > 0 && !d_targets) || !d_vertices ||
        !d_num_children || !num_roots || n >= (1ll << 31) || ne >= (1ll << 31))
        return PQH_ERR_ARG;
    int rc = pqh_use_device(ctx);
    if (rc) return rc;
    hipStream_t st = ctx->stream;
    const size_t en = ne > 0 ? (size_t)ne : 1;
    // temporary storage of the library calls
    size_t t_scan32 = 0, t_sort = 0, t_scanw = 0, t_scan64 = 0, t_scanv = 0;
    PQH_HIP(ctx, rocprim::exclusive_scan(nullptr, t_scan32, (const int*)nullptr, (uint32_t*)nullptr,
                                         0u, (size_t)n + 1, rocprim::plus<uint32_t>(), st));
    PQH_HIP(ctx, rocprim::radix_sort_pairs(nullptr, t_sort, (unsigned long long*)nullptr,
                                           (unsigned long long*)nullptr, (uint32_t*)nullptr,
                                           (uint32_t*)nullptr, en, 0u, 64u, st));
    PQH_HIP(ctx, rocprim::inclusive_scan(nullptr, t_scanw, (const uint32_t*)nullptr, (uint32_t*)nullptr,
                                         en, rocprim::plus<uint32_t>(), st));
    PQH_HIP(ctx, rocprim::exclusive_scan(nullptr, t_scan64, (const unsigned long long*)nullptr,
                                         (unsigned long long*)nullptr, 0ull, (size_t)n + 1,
                                         rocprim::plus<unsigned long long>(), st));
    PQH_HIP(ctx, rocprim::inclusive_scan(nullptr, t_scanv, (const int*)nullptr, (int*)nullptr, en,
                                         rocprim::plus<int>(), st));
    const size_t t_max = std::max({t_scan32, t_sort, t_scanw, t_scan64, t_scanv});
    // one scratch block (the context's grow-only workspace), carved twice: once to size it
    uint32_t *first, *parent, *size, *posdown, *rootof, *rootL, *offc;
    int *cnt1, *flags;
    unsigned long long *rinfo, *rbase;
    uint32_t *src, *idx, *idx2, *twin, *succ;
    unsigned long long *key, *key2;
    void* temp;
    auto carve = [&](Arena& a) {
        first = a.take<uint32_t>(n + 1);
        cnt1 = a.take<int>(n + 1);
        parent = a.take<uint32_t>(n);
        size = a.take<uint32_t>(n);
        posdown = a.take<uint32_t>(n);
        rootof = a.take<uint32_t>(n);
        rootL = a.take<uint32_t>(n);
        offc = a.take<uint32_t>(n);
        rinfo = a.take<unsigned long long>(n + 1);
        rbase = a.take<unsigned long long>(n + 1);
        flags = a.take<int>(8);
        src = a.take<uint32_t>(en);
        idx = a.take<uint32_t>(en);
        idx2 = a.take<uint32_t>(en);
        twin = a.take<uint32_t>(en);
        succ = a.take<uint32_t>(en);
        key = a.take<unsigned long long>(en);
        key2 = a.take<unsigned long long>(en);
        temp = a.take<char>(t_max);
    };
    Arena sizing;
    carve(sizing);
    if ((rc = pqh_ensure_ws(ctx, sizing.used))) return rc;
    Arena arena;
    arena.base = static_cast<char*>(ctx->ws);
    carve(arena);
    // flags: [0] bad counts / not a forest, [2] isolated vertices, [3] tours
    int hb[8] = {0};
    auto read_flags = [&]() -> int {
        PQH_HIP(ctx, hipMemcpyAsync(hb, flags, sizeof(hb), hipMemcpyDeviceToHost, st));
        PQH_HIP(ctx, hipStreamSynchronize(st));
        return PQH_OK;
    };
    // CSR offsets (restore_tree_edges_pointers, mst.c:52-61); counts >= 0 summing to ne
    PQH_HIP(ctx, hipMemsetAsync(flags, 0, sizeof(hb), st));
    PQH_HIP(ctx, hipMemcpyAsync(cnt1, d_counts, sizeof(int) * n, hipMemcpyDeviceToDevice, st));
    PQH_HIP(ctx, hipMemsetAsync(cnt1 + n, 0, sizeof(int), st));
    size_t tb = t_max;
    PQH_HIP(ctx, rocprim::exclusive_scan(temp, tb, cnt1, first, 0u, (size_t)n + 1,
                                         rocprim::plus<uint32_t>(), st));
    hipLaunchKernelGGL(td_vertex_init, G1(n), 0, st, n, d_counts, parent, rootL, flags);
    PQH_LAUNCH_CHECK(ctx);
    uint32_t total = 0;
    PQH_HIP(ctx, hipMemcpyAsync(&total, first + n, 4, hipMemcpyDeviceToHost, st));
    if ((rc = read_flags())) return rc;
    if (hb[0] || (long long)total != ne) return PQH_ERR_ARG;
    const int isolated = hb[2];
    unsigned long long* kf = key;
    int* val = reinterpret_cast<int*>(idx2);   // (both free once the jumping is done)
    uint32_t* W = idx;
    if (ne > 0) {
        hipLaunchKernelGGL(td_edges, G1(n), 0, st, first, n, d_targets, src, key, idx);
        PQH_LAUNCH_CHECK(ctx);
        tb = t_max;
        PQH_HIP(ctx, rocprim::radix_sort_pairs(temp, tb, key, key2, idx, idx2, (size_t)ne, 0u, 64u, st));
        // twins; an out-of-range target never pairs (no edge leaves it), so every target is
        // a vertex once this passes
        hipLaunchKernelGGL(td_twins, G1(ne), 0, st, key2, idx2, ne, src, twin, flags);
        PQH_LAUNCH_CHECK(ctx);
        if ((rc = read_flags())) return rc;
        if (hb[0]) return PQH_ERR_UNSUPPORTED;   // not a simple graph of paired edges
        hipLaunchKernelGGL(td_succ, G1(ne), 0, st, first, d_targets, twin, ne, succ, idx, key);
        PQH_LAUNCH_CHECK(ctx);
        uint32_t *ja = idx, *jb = idx2;
        unsigned long long *ka = key, *kb = key2;
        for (int round = 0, rounds = ceil_log2(ne); round < rounds; ++round) {
            hipLaunchKernelGGL(td_jump, G1(ne), 0, st, ne, 1u << round, ja, ka, jb, kb);
            std::swap(ja, jb);
            std::swap(ka, kb);
        }
        PQH_LAUNCH_CHECK(ctx);
        kf = ka;
        hipLaunchKernelGGL(td_verify, G1(ne), 0, st, first, src, kf, ne, flags);
        PQH_LAUNCH_CHECK(ctx);
        if ((rc = read_flags())) return rc;
        // every component on a tour of its own, and a tree: E = V - 1 for each
        if (hb[0] || ne / 2 != n - isolated - hb[3]) return PQH_ERR_UNSUPPORTED;
        hipLaunchKernelGGL(td_parents, G1(ne), 0, st, d_targets, src, twin, succ, kf, ne, parent,
                           size, posdown, rootof, rootL);
        PQH_LAUNCH_CHECK(ctx);
    }
    hipLaunchKernelGGL(td_roots, G1(n + 1), 0, st, n, parent, rootL, size, rinfo);
    PQH_LAUNCH_CHECK(ctx);
    tb = t_max;
    PQH_HIP(ctx, rocprim::exclusive_scan(temp, tb, rinfo, rbase, 0ull, (size_t)n + 1,
                                         rocprim::plus<unsigned long long>(), st));
    if (ne > 0) {
        hipLaunchKernelGGL(td_weights, G1(ne), 0, st, d_targets, src, parent, size, ne, W);
        PQH_LAUNCH_CHECK(ctx);
        tb = t_max;
        PQH_HIP(ctx, rocprim::inclusive_scan(temp, tb, W, W, (size_t)ne, rocprim::plus<uint32_t>(), st));
        hipLaunchKernelGGL(td_offsets, G1(ne), 0, st, first, d_targets, src, parent, W, ne, offc);
        PQH_LAUNCH_CHECK(ctx);
        hipLaunchKernelGGL(td_tour, G1(ne), 0, st, d_targets, src, twin, succ, kf, rbase, offc, ne, val);
        PQH_LAUNCH_CHECK(ctx);
        tb = t_max;
        PQH_HIP(ctx, rocprim::inclusive_scan(temp, tb, val, val, (size_t)ne, rocprim::plus<int>(), st));
    }
    hipLaunchKernelGGL(td_output, G1(n), 0, st, n, first, parent, posdown, rootof, rbase, val,
                       d_vertices, d_num_children, d_parents);
    PQH_LAUNCH_CHECK(ctx);
    PQH_HIP(ctx, hipStreamSynchronize(st));
    *num_roots = isolated + hb[3];
    return PQH_OK;
}

extern "C" long long pqh_tree_ext_index_device(pqh_ctx_t* ctx, long long n,
                                               const void* d_num_children, int child_bytes,
                                               int chunk_vectors, long long* d_parent_pos,
                                               long long* d_ext_offsets,
                                               long long* d_ext_positions) {
    if (!ctx || n < 0 || chunk_vectors <= 0 || (child_bytes != 1 && child_bytes != 2 && child_bytes != 4) ||
        (n > 0 && (!d_num_children || !d_parent_pos || !d_ext_offsets)))
        return PQH_ERR_ARG;
    int rc = pqh_use_device(ctx);
    if (rc) return rc;
    hipStream_t st = ctx->stream;
    const long long chunks = (n + chunk_vectors - 1) / chunk_vectors;
    if (n == 0) {
        PQH_HIP(ctx, hipMemsetAsync(d_ext_offsets, 0, 8, st));
        PQH_HIP(ctx, hipStreamSynchronize(st));
        return 0;
    }
    size_t t_sum = 0, t_min = 0;
    PQH_HIP(ctx, rocprim::inclusive_scan(nullptr, t_sum, (const long long*)nullptr, (long long*)nullptr,
                                         (size_t)n, rocprim::plus<long long>(), st));
    PQH_HIP(ctx, rocprim::inclusive_scan(nullptr, t_min, (const long long*)nullptr, (long long*)nullptr,
                                         (size_t)n, rocprim::minimum<long long>(), st));
    const size_t t_max = std::max(t_sum, t_min);
    int nlev = 1;
    long long tot = n;
    std::vector<long long> loff(1, 0);   // level k at loff[k], loff[nlev] = the total
    for (long long len = n; len > 1; len = (len + 1) / 2) {
        loff.push_back(tot);
        tot += (len + 1) / 2;
        ++nlev;
    }
    loff.push_back(tot);
    long long *E, *PM, *R, *lev, *ext, *S, *dloff;
    void* temp;
    auto carve = [&](Arena& a) {
        E = a.take<long long>(n);
        PM = a.take<long long>(n);
        R = a.take<long long>(n);
        lev = a.take<long long>(tot);
        ext = a.take<long long>(n);
        S = a.take<long long>(n);
        dloff = a.take<long long>(nlev + 1);
        temp = a.take<char>(t_max);
    };
    Arena sizing;
    carve(sizing);
    if ((rc = pqh_ensure_ws(ctx, sizing.used))) return rc;
    Arena arena;
    arena.base = static_cast<char*>(ctx->ws);
    carve(arena);
    PQH_HIP(ctx, hipMemcpyAsync(dloff, loff.data(), sizeof(long long) * (nlev + 1), hipMemcpyHostToDevice, st));
#define PQH_TX(T)                                                                                \
    do {                                                                                         \
        const T* nc = static_cast<const T*>(d_num_children);                                    \
        hipLaunchKernelGGL(tx_vals<T>, G1(n), 0, st, nc, n, E);                                  \
        size_t tb = t_max;                                                                       \
        PQH_HIP(ctx, rocprim::inclusive_scan(temp, tb, E, E, (size_t)n, rocprim::plus<long long>(), st)); \
        tb = t_max;                                                                              \
        PQH_HIP(ctx, rocprim::inclusive_scan(temp, tb, E, PM, (size_t)n,                         \
                                             rocprim::minimum<long long>(), st));               \
        hipLaunchKernelGGL(tx_roots, G1(n), 0, st, E, PM, n, R);                                  \
    } while (0)
    if (child_bytes == 1) PQH_TX(uint8_t);
    else if (child_bytes == 2) PQH_TX(uint16_t);
    else PQH_TX(int32_t);
#undef PQH_TX
    PQH_LAUNCH_CHECK(ctx);
    // PM <- the root flags (kept for the query), R <- their running count; then level 0
    PQH_HIP(ctx, hipMemcpyAsync(PM, R, sizeof(long long) * n, hipMemcpyDeviceToDevice, st));
    {
        size_t tb = t_max;
        PQH_HIP(ctx, rocprim::inclusive_scan(temp, tb, R, R, (size_t)n, rocprim::plus<long long>(), st));
    }
    if (child_bytes == 1)
        hipLaunchKernelGGL(tx_levels0<uint8_t>, G1(n), 0, st, static_cast<const uint8_t*>(d_num_children), E, R, n, lev);
    else if (child_bytes == 2)
        hipLaunchKernelGGL(tx_levels0<uint16_t>, G1(n), 0, st, static_cast<const uint16_t*>(d_num_children), E, R, n, lev);
    else
        hipLaunchKernelGGL(tx_levels0<int32_t>, G1(n), 0, st, static_cast<const int32_t*>(d_num_children), E, R, n, lev);
    PQH_LAUNCH_CHECK(ctx);
    for (int k = 1; k < nlev; ++k) {
        const long long nlo = loff[k] - loff[k - 1];
        const long long nhi = loff[k + 1] - loff[k];
        hipLaunchKernelGGL(tx_level_up, G1(nhi), 0, st, lev + loff[k - 1], nlo, lev + loff[k], nhi);
    }
    PQH_LAUNCH_CHECK(ctx);
    hipLaunchKernelGGL(tx_query, G1(n), 0, st, lev, dloff, nlev, PM, n, chunk_vectors, d_parent_pos, ext);
    PQH_LAUNCH_CHECK(ctx);
    {
        size_t tb = t_max;
        PQH_HIP(ctx, rocprim::inclusive_scan(temp, tb, ext, S, (size_t)n, rocprim::plus<long long>(), st));
    }
    hipLaunchKernelGGL(tx_offsets, G1(chunks + 1), 0, st, S, n, chunk_vectors, chunks, d_ext_offsets);
    if (d_ext_positions)
        hipLaunchKernelGGL(tx_compact, G1(n), 0, st, ext, S, d_parent_pos, n, d_ext_positions);
    PQH_LAUNCH_CHECK(ctx);
    long long total = 0;
    PQH_HIP(ctx, hipMemcpyAsync(&total, S + n - 1, 8, hipMemcpyDeviceToHost, st));
    PQH_HIP(ctx, hipStreamSynchronize(st));
    return total;
}
