// pqh_tree_dev.hip -- tree mode's DFS order on the device (pqh_tree_order_device).
//
// tree_collect_vertices_dfs (mst.c:290-364) walks a stored forest with a stack, marking a
// vertex when it is pushed: roots are the lowest unvisited ids, a vertex's unvisited
// neighbours are pushed in adjacency order and therefore visited in REVERSE adjacency order.
// On a forest that is the preorder in which every tree is rooted at its smallest vertex id,
// trees come in root-id order and the children of a vertex in reverse adjacency order; the
// traverser's active parent of a row (mst.c:366-405) is the vertex's tree parent.  Computed
// without a sequential walk:
//   twins      every directed edge u->v paired with v->u (a stable radix sort of the
//              undirected keys); a self-loop, a repeated edge or an unpaired edge is not a
//              forest -- PQH_ERR_UNSUPPORTED, and the caller walks on the host (pqh_tree_order)
//   tour       succ(u->v) = the edge after v->u in v's list (cyclic): one Euler tour per tree
//   roots      the minimum vertex over each tour (pointer jumping); the tour is cut before
//              the root's first edge and list-ranked (pointer jumping)
//   parents    u->v is a tree edge down when it precedes v->u in the tour; subtree sizes from
//              the two ranks; a graph with a cycle leaves a vertex without exactly one edge
//              down into it, or more tours than the forest count allows -> not a forest
//   preorder   pre(c) = pre(v) + 1 + the sizes of the children after c in v's list (a scan
//              over the edges), accumulated to the root by pointer jumping, plus the sizes of
//              the trees with smaller roots
#include <rocprim/device/device_radix_sort.hpp>
#include <rocprim/device/device_scan.hpp>

#include <vector>

#include "pqh_internal.h"

namespace {

constexpr uint32_t kNil = 0xFFFFFFFFu;

struct DevBuf {
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

#define G1(n) dim3((unsigned)(((n) + 255) / 256)), dim3(256)

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

// twins from the sorted keys: keys must come in pairs of opposite directions
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

__global__ void __launch_bounds__(256)
td_succ(const uint32_t* __restrict__ first, const uint32_t* __restrict__ tg,
        const uint32_t* __restrict__ twin, long long ne, uint32_t* __restrict__ succ,
        uint32_t* __restrict__ mn, uint32_t* __restrict__ src) {
    const long long e = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= ne) return;
    const uint32_t v = tg[e], t = twin[e];
    const uint32_t deg = first[v + 1] - first[v];
    const uint32_t i = t - first[v];
    succ[e] = first[v] + (i + 1 == deg ? 0 : i + 1);
    mn[e] = src[e];
}

// one pointer-jumping round of the minimum over a tour (cycles): mn'[e] = min(mn[e], mn[j[e]]),
// j'[e] = j[j[e]]
__global__ void __launch_bounds__(256)
td_min_round(long long ne, const uint32_t* __restrict__ j0, const uint32_t* __restrict__ m0,
             uint32_t* __restrict__ j1, uint32_t* __restrict__ m1) {
    const long long e = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= ne) return;
    const uint32_t j = j0[e];
    m1[e] = min(m0[e], m0[j]);
    j1[e] = j0[j];
}

// cut each tour before its root's first edge: the edge into the root that precedes it
__global__ void __launch_bounds__(256)
td_cut(const uint32_t* __restrict__ first, const uint32_t* __restrict__ twin,
       const uint32_t* __restrict__ root, long long ne, uint32_t* __restrict__ succ,
       uint32_t* __restrict__ rank) {
    const long long e = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= ne) return;
    const uint32_t r = root[e];
    const uint32_t last_in = twin[first[r + 1] - 1];   // (r's last edge reversed)
    if ((uint32_t)e == last_in) succ[e] = kNil;
    rank[e] = succ[e] == kNil ? 0u : 1u;
}

// list ranking: distance to the tour's end
__global__ void __launch_bounds__(256)
td_rank_round(long long ne, const uint32_t* __restrict__ j0, const uint32_t* __restrict__ r0,
              uint32_t* __restrict__ j1, uint32_t* __restrict__ r1, int* __restrict__ more) {
    const long long e = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= ne) return;
    const uint32_t j = j0[e];
    if (j == kNil) {
        j1[e] = kNil;
        r1[e] = r0[e];
        return;
    }
    r1[e] = r0[e] + r0[j];
    j1[e] = j0[j];
    if (j0[j] != kNil) *more = 1;
}

// per vertex: parent, the number of edges down into it, subtree size; the tree's edge count
// and root; isolated vertices are roots of their own tree
__global__ void __launch_bounds__(256)
td_parents(const uint32_t* __restrict__ first, const uint32_t* __restrict__ tg,
           const uint32_t* __restrict__ src, const uint32_t* __restrict__ twin,
           const uint32_t* __restrict__ rank, const uint32_t* __restrict__ root, long long ne,
           uint32_t* __restrict__ parent, uint32_t* __restrict__ size, uint32_t* __restrict__ downs,
           uint32_t* __restrict__ tedges) {
    const long long e = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= ne) return;
    const uint32_t t = twin[e];
    // positions from the tour start: pos = (tour edges - 1) - rank; compare ranks instead
    if (rank[e] > rank[t]) {   // e = u->v comes first: v's parent is u
        const uint32_t v = tg[e];
        parent[v] = src[e];
        size[v] = (rank[e] - rank[t] + 1) / 2;
        atomicAdd(&downs[v], 1u);
    }
    if ((uint32_t)e == first[root[e]]) tedges[root[e]] = rank[e] + 1;   // the tour's length
}

__global__ void __launch_bounds__(256)
td_vertex_init(long long n, const int* __restrict__ counts, uint32_t* __restrict__ parent,
               uint32_t* __restrict__ size, uint32_t* __restrict__ downs, uint32_t* __restrict__ tedges,
               int* __restrict__ bad) {
    const long long v = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (v >= n) return;
    if (counts[v] < 0) *bad = 1;
    parent[v] = (uint32_t)v;
    size[v] = 0;
    downs[v] = 0;
    tedges[v] = 0;
}

// vertex checks and the per-edge weight for the children offsets: w(e) = size of the child
// below a down edge, 0 for the edge to the parent
__global__ void __launch_bounds__(256)
td_check(long long n, const uint32_t* __restrict__ first, const uint32_t* __restrict__ parent,
         const uint32_t* __restrict__ downs, const uint32_t* __restrict__ tedges,
         uint32_t* __restrict__ size, uint32_t* __restrict__ isroot, int* __restrict__ bad,
         int* __restrict__ roots) {
    const long long v = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (v >= n) return;
    const bool deg0 = first[v + 1] == first[v];
    const bool rt = parent[v] == (uint32_t)v;
    if (rt) {
        atomicAdd(roots, 1);
        if (downs[v] != 0) *bad = 1;
        // a root heads a tour over its whole tree: 2 (size - 1) edges
        size[v] = deg0 ? 1u : tedges[v] / 2 + 1;
        if (!deg0 && tedges[v] == 0) *bad = 1;   // (a vertex that is no tour's minimum)
    } else if (downs[v] != 1) {
        *bad = 1;
    }
    isroot[v] = rt ? size[v] : 0u;
}

__global__ void __launch_bounds__(256)
td_weights(const uint32_t* __restrict__ tg, const uint32_t* __restrict__ src,
           const uint32_t* __restrict__ parent, const uint32_t* __restrict__ size, long long ne,
           unsigned long long* __restrict__ w) {
    const long long e = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= ne) return;
    const uint32_t c = tg[e];
    w[e] = (parent[c] == src[e] && c != src[e]) ? size[c] : 0ull;
}

// off(c) = 1 + sizes of the children after c in its parent's list (incl. prefix sums W)
__global__ void __launch_bounds__(256)
td_offsets(const uint32_t* __restrict__ first, const uint32_t* __restrict__ tg,
           const uint32_t* __restrict__ src, const uint32_t* __restrict__ parent,
           const unsigned long long* __restrict__ W, long long ne, unsigned long long* __restrict__ acc) {
    const long long e = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= ne) return;
    const uint32_t c = tg[e], v = src[e];
    if (parent[c] != v || c == v) return;
    const uint32_t end = first[v + 1] - 1;
    acc[c] = 1ull + (W[end] - W[e]);
}

__global__ void __launch_bounds__(256)
td_acc_init(long long n, const uint32_t* __restrict__ parent, unsigned long long* __restrict__ acc,
            uint32_t* __restrict__ up) {
    const long long v = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (v >= n) return;
    up[v] = parent[v];
    if (parent[v] == (uint32_t)v) acc[v] = 0ull;
}

__global__ void __launch_bounds__(256)
td_acc_round(long long n, const uint32_t* __restrict__ u0, const unsigned long long* __restrict__ a0,
             uint32_t* __restrict__ u1, unsigned long long* __restrict__ a1, int* __restrict__ more) {
    const long long v = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (v >= n) return;
    const uint32_t u = u0[v];
    if (u == u0[u]) {   // u is a root: done (its acc is 0)
        u1[v] = u;
        a1[v] = a0[v];
        return;
    }
    a1[v] = a0[v] + a0[u];
    u1[v] = u0[u];
    *more = 1;
}

__global__ void __launch_bounds__(256)
td_output(long long n, const uint32_t* __restrict__ first, const uint32_t* __restrict__ parent,
          const uint32_t* __restrict__ up, const unsigned long long* __restrict__ acc,
          const unsigned long long* __restrict__ toff, uint32_t* __restrict__ vertices,
          int* __restrict__ num_children, long long* __restrict__ parents) {
    const long long v = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (v >= n) return;
    const bool rt = parent[v] == (uint32_t)v;
    const uint32_t r = rt ? (uint32_t)v : up[v];
    const long long pre = (long long)(toff[r] + acc[v]);
    const int deg = (int)(first[v + 1] - first[v]);
    vertices[pre] = (uint32_t)v;
    num_children[pre] = rt ? deg : deg - 1;
    if (parents) parents[pre] = rt ? -1ll : (long long)parent[v];
}

}  // namespace

static int ceil_log2(long long x) {
    int r = 0;
    while ((1ll << r) < x) ++r;
    return r;
}

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
    DevBuf buf;
    uint32_t* first = buf.get<uint32_t>(n + 1);
    uint32_t* parent = buf.get<uint32_t>(n);
    uint32_t* size = buf.get<uint32_t>(n);
    uint32_t* downs = buf.get<uint32_t>(n);
    uint32_t* tedges = buf.get<uint32_t>(n);
    uint32_t* isroot = buf.get<uint32_t>(n + 1);
    unsigned long long* toff = buf.get<unsigned long long>(n + 1);
    unsigned long long* acc = buf.get<unsigned long long>(n);
    unsigned long long* acc2 = buf.get<unsigned long long>(n);
    uint32_t* up = buf.get<uint32_t>(n);
    uint32_t* up2 = buf.get<uint32_t>(n);
    int* cnt1 = buf.get<int>(n + 1);
    // flags: [0] bad input or not a forest, [1] list ranking unfinished, [2] root count,
    // [3] parent chains unfinished
    int* flags = buf.get<int>(8);
    if (!first || !parent || !size || !downs || !tedges || !isroot || !toff || !acc || !acc2 ||
        !up || !up2 || !cnt1 || !flags)
        return pqh_set_error(ctx, PQH_ERR_NOMEM, "tree order: %lld vertices", n);
    int hb[8] = {0};
    auto read_flags = [&]() -> int {
        PQH_HIP(ctx, hipMemcpyAsync(hb, flags, sizeof(hb), hipMemcpyDeviceToHost, st));
        PQH_HIP(ctx, hipStreamSynchronize(st));
        return PQH_OK;
    };
    // CSR offsets (restore_tree_edges_pointers, mst.c:52-61); counts must be >= 0 and sum to ne
    PQH_HIP(ctx, hipMemsetAsync(flags, 0, sizeof(hb), st));
    PQH_HIP(ctx, hipMemcpyAsync(cnt1, d_counts, sizeof(int) * n, hipMemcpyDeviceToDevice, st));
    PQH_HIP(ctx, hipMemsetAsync(cnt1 + n, 0, sizeof(int), st));
    {
        size_t temp = 0;
        PQH_HIP(ctx, rocprim::exclusive_scan(nullptr, temp, cnt1, first, 0u, (size_t)n + 1,
                                             rocprim::plus<uint32_t>(), st));
        void* t = buf.get<char>(temp);
        if (!t) return pqh_set_error(ctx, PQH_ERR_NOMEM, "tree order: scan");
        PQH_HIP(ctx, rocprim::exclusive_scan(t, temp, cnt1, first, 0u, (size_t)n + 1,
                                             rocprim::plus<uint32_t>(), st));
    }
    hipLaunchKernelGGL(td_vertex_init, G1(n), 0, st, n, d_counts, parent, size, downs, tedges, flags);
    PQH_LAUNCH_CHECK(ctx);
    uint32_t total = 0;
    PQH_HIP(ctx, hipMemcpyAsync(&total, first + n, 4, hipMemcpyDeviceToHost, st));
    if ((rc = read_flags())) return rc;
    if (hb[0] || (long long)total != ne) return PQH_ERR_ARG;
    if (ne > 0) {
        uint32_t* src = buf.get<uint32_t>(ne);
        unsigned long long* key = buf.get<unsigned long long>(ne);
        unsigned long long* key2 = buf.get<unsigned long long>(ne);
        uint32_t* idx = buf.get<uint32_t>(ne);
        uint32_t* idx2 = buf.get<uint32_t>(ne);
        uint32_t* twin = buf.get<uint32_t>(ne);
        uint32_t* succ = buf.get<uint32_t>(ne);
        uint32_t* j2 = buf.get<uint32_t>(ne);
        uint32_t* mn = buf.get<uint32_t>(ne);
        uint32_t* mn2 = buf.get<uint32_t>(ne);
        unsigned long long* W = buf.get<unsigned long long>(ne);
        if (!src || !key || !key2 || !idx || !idx2 || !twin || !succ || !j2 || !mn || !mn2 || !W)
            return pqh_set_error(ctx, PQH_ERR_NOMEM, "tree order: %lld edges", ne);
        hipLaunchKernelGGL(td_edges, G1(n), 0, st, first, n, d_targets, src, key, idx);
        PQH_LAUNCH_CHECK(ctx);
        {
            size_t temp = 0;
            PQH_HIP(ctx, rocprim::radix_sort_pairs(nullptr, temp, key, key2, idx, idx2, (size_t)ne,
                                                   0u, 64u, st));
            void* t = buf.get<char>(temp);
            if (!t) return PQH_ERR_NOMEM;
            PQH_HIP(ctx, rocprim::radix_sort_pairs(t, temp, key, key2, idx, idx2, (size_t)ne, 0u, 64u, st));
        }
        // twins; an out-of-range target never pairs (no edge leaves it), so every target is
        // a vertex once this passes
        hipLaunchKernelGGL(td_twins, G1(ne), 0, st, key2, idx2, ne, src, twin, flags);
        PQH_LAUNCH_CHECK(ctx);
        if ((rc = read_flags())) return rc;
        if (hb[0]) return PQH_ERR_UNSUPPORTED;   // not a simple graph of paired edges
        hipLaunchKernelGGL(td_succ, G1(ne), 0, st, first, d_targets, twin, ne, succ, mn, src);
        PQH_LAUNCH_CHECK(ctx);
        // the minimum vertex of every tour (its tree's root): pointer jumping
        PQH_HIP(ctx, hipMemcpyAsync(j2, succ, sizeof(uint32_t) * ne, hipMemcpyDeviceToDevice, st));
        uint32_t *ja = j2, *ma = mn, *jb = idx, *mb = mn2;   // (idx is free now)
        for (int round = 0, rounds = ceil_log2(ne); round < rounds; ++round) {
            hipLaunchKernelGGL(td_min_round, G1(ne), 0, st, ne, ja, ma, jb, mb);
            std::swap(ja, jb);
            std::swap(ma, mb);
        }
        PQH_LAUNCH_CHECK(ctx);
        uint32_t* root = ma;
        // cut every tour before its root's first edge and rank the edges to the tour's end
        uint32_t* rank = mb;
        hipLaunchKernelGGL(td_cut, G1(ne), 0, st, first, twin, root, ne, succ, rank);
        PQH_LAUNCH_CHECK(ctx);
        uint32_t *jr = succ, *jr2 = ja, *ra = rank, *rb = jb;   // (the jump buffers are free)
        for (int round = 0, rounds = ceil_log2(ne) + 1; round < rounds; ++round) {
            if (round + 1 == rounds) PQH_HIP(ctx, hipMemsetAsync(flags + 1, 0, sizeof(int), st));
            hipLaunchKernelGGL(td_rank_round, G1(ne), 0, st, ne, jr, ra, jr2, rb, flags + 1);
            std::swap(jr, jr2);
            std::swap(ra, rb);
        }
        PQH_LAUNCH_CHECK(ctx);
        hipLaunchKernelGGL(td_parents, G1(ne), 0, st, first, d_targets, src, twin, ra, root, ne,
                           parent, size, downs, tedges);
        PQH_LAUNCH_CHECK(ctx);
        hipLaunchKernelGGL(td_check, G1(n), 0, st, n, first, parent, downs, tedges, size, isroot,
                           flags, flags + 2);
        PQH_LAUNCH_CHECK(ctx);
        hipLaunchKernelGGL(td_weights, G1(ne), 0, st, d_targets, src, parent, size, ne, W);
        PQH_LAUNCH_CHECK(ctx);
        {   // W = inclusive prefix sums of the weights
            size_t temp = 0;
            PQH_HIP(ctx, rocprim::inclusive_scan(nullptr, temp, W, W, (size_t)ne,
                                                 rocprim::plus<unsigned long long>(), st));
            void* t = buf.get<char>(temp);
            if (!t) return PQH_ERR_NOMEM;
            PQH_HIP(ctx, rocprim::inclusive_scan(t, temp, W, W, (size_t)ne,
                                                 rocprim::plus<unsigned long long>(), st));
        }
        hipLaunchKernelGGL(td_offsets, G1(ne), 0, st, first, d_targets, src, parent, W, ne, acc);
        PQH_LAUNCH_CHECK(ctx);
    } else {
        hipLaunchKernelGGL(td_check, G1(n), 0, st, n, first, parent, downs, tedges, size, isroot,
                           flags, flags + 2);
        PQH_LAUNCH_CHECK(ctx);
    }
    if ((rc = read_flags())) return rc;
    // a forest: every tour cut once, one edge down into each non-root, and exactly the
    // non-roots' parent edges in the graph (then parent chains are checked acyclic below)
    if (hb[0] || hb[1] || 2ll * (n - hb[2]) != ne) return PQH_ERR_UNSUPPORTED;
    // tree offsets in root-id order; preorder by accumulating the offsets up to the root
    PQH_HIP(ctx, hipMemsetAsync(isroot + n, 0, sizeof(uint32_t), st));
    {
        size_t temp = 0;
        PQH_HIP(ctx, rocprim::exclusive_scan(nullptr, temp, isroot, toff, 0ull, (size_t)n + 1,
                                             rocprim::plus<unsigned long long>(), st));
        void* t = buf.get<char>(temp);
        if (!t) return PQH_ERR_NOMEM;
        PQH_HIP(ctx, rocprim::exclusive_scan(t, temp, isroot, toff, 0ull, (size_t)n + 1,
                                             rocprim::plus<unsigned long long>(), st));
    }
    unsigned long long all = 0;
    PQH_HIP(ctx, hipMemcpyAsync(&all, toff + n, 8, hipMemcpyDeviceToHost, st));
    hipLaunchKernelGGL(td_acc_init, G1(n), 0, st, n, parent, acc, up);
    PQH_LAUNCH_CHECK(ctx);
    unsigned long long *aa = acc, *ab = acc2;
    uint32_t *ua = up, *ub = up2;
    for (int round = 0, rounds = ceil_log2(n) + 1; round < rounds; ++round) {
        if (round + 1 == rounds) PQH_HIP(ctx, hipMemsetAsync(flags + 3, 0, sizeof(int), st));
        hipLaunchKernelGGL(td_acc_round, G1(n), 0, st, n, ua, aa, ub, ab, flags + 3);
        std::swap(ua, ub);
        std::swap(aa, ab);
    }
    PQH_LAUNCH_CHECK(ctx);
    if ((rc = read_flags())) return rc;
    if (hb[3] || (long long)all != n) return PQH_ERR_UNSUPPORTED;
    hipLaunchKernelGGL(td_output, G1(n), 0, st, n, first, parent, ua, aa, toff, d_vertices,
                       d_num_children, d_parents);
    PQH_LAUNCH_CHECK(ctx);
    PQH_HIP(ctx, hipStreamSynchronize(st));   // (before the scratch is freed)
    *num_roots = hb[2];
    return PQH_OK;
}
