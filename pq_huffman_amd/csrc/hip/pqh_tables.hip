// pqh_tables.hip -- Huffman code tables built on the GPU, and the chunked stream decoder.
//
//  huff_trees   huffman_codebook_init_encoder + collect_codes (huffman_encode.c:33-192,
//               :100-132) for every (part, previous-symbol) alphabet at once: one lane per
//               tree simulates the reference's binary heap step for step -- same push
//               (sift up while strictly lighter), same pop (left child unless the right one
//               is strictly lighter), leaves pushed in symbol order, first pop = child 0 --
//               so the tree, and therefore every code, is the reference's.  Heap entries
//               carry (weight << 16 | node) so a comparison is one LDS read; all per-tree
//               arrays are interleaved tree-minor so the 32 lanes of a wave hit 32
//               consecutive LDS words.
//  lut_build    two-level decode tables per alphabet: a first level of up to 2^11
//               entries (2^9 in context mode, where there are K*m alphabets), second-level
//               subtables for the prefixes of longer codes, ranges taken from a pool head.
//  dec_chunks   huffman_decoder.c:211-255: one lane per chunk of C vectors; a symbol costs
//               one table load instead of one trie step per bit (huffman_decode.c:137-191).
#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <type_traits>
#include <vector>

#include "pqh_internal.h"
#include "pqh_heap_asm.h"

namespace {

constexpr int kMaxCodeLen = 56;
constexpr unsigned long long kCodeMask = (1ull << 56) - 1;
constexpr int kL1Max = 13;                      // decode first level: 2^W1 entries, W1 <= 13
constexpr long long kL2BaseMax = 1ll << 23;     // (meta holds l2base in 23 bits)

// ------------------------------------------------------------------- tree building
// A tree's heap lives in LDS, interleaved tree-minor (entry i of lane t at [i * TPW + t]) so
// the lanes of a wave touch consecutive words.  Keys are (weight << NB | node): a 32-bit key
// (NB = 9) when the tree's total weight is below 2^23, else 64-bit (NB = 16).  Comparisons
// use the weight only, exactly as the reference heap does.
// SPLIT (64-bit keys in a u32 column): entry i is the words [2i * TPW] (low) and
// [(2i + 1) * TPW] (high) of the lane's own u32 column, so a 64-bit heap touches only the
// slots of its own tree and the u32 sentinel heaps of the other lanes of the workgroup --
// whose branch may run after this one -- keep their sentinels.
template <typename Key, int NB, int TPW, int CAP, bool SPLIT = false>
struct LdsHeap {
    using Word = typename std::conditional<SPLIT, uint32_t, Key>::type;
    Word* h;
    int size;
    __device__ __forceinline__ Key get(int i) const {
        if constexpr (SPLIT)
            return (Key)h[2 * i * TPW] | ((Key)h[(2 * i + 1) * TPW] << 32);
        else
            return h[i * TPW];
    }
    __device__ __forceinline__ void set(int i, Key v) {
        if constexpr (SPLIT) {
            h[2 * i * TPW] = (uint32_t)v;
            h[(2 * i + 1) * TPW] = (uint32_t)(v >> 32);
        } else {
            h[i * TPW] = v;
        }
    }
    // huffman_encode.c:33-46: sift up while strictly lighter than the parent.  The first
    // three ancestors are read in one round trip (most pushes stop within them).
    __device__ __forceinline__ void push(Key e) {
        int i = size++;
        const Key w = e >> NB;
        const int p1 = (i - 1) >> 1, p2 = (p1 - 1) >> 1, p3 = (p2 - 1) >> 1;
        Key a1 = get(max(p1, 0)), a2 = get(max(p2, 0)), a3 = get(max(p3, 0));
        asm volatile("" : "+v"(a1), "+v"(a2), "+v"(a3));   // one wait for all three
        if (i > 0 && w < (a1 >> NB)) {
            set(i, a1);
            i = p1;
            if (i > 0 && w < (a2 >> NB)) {
                set(i, a2);
                i = p2;
                if (i > 0 && w < (a3 >> NB)) {
                    set(i, a3);
                    i = p3;
                    while (i > 0) {
                        const int p = (i - 1) >> 1;
                        const Key hp = get(p);
                        if (w >= (hp >> NB)) break;
                        set(i, hp);
                        i = p;
                    }
                }
            }
        }
        set(i, e);
    }
    // huffman_encode.c:48-76: the last entry sifts down from the root; at each level the
    // left child is the candidate unless the right one is strictly lighter, and the entry
    // moves while strictly heavier than the candidate.  Children and grandchildren are read
    // together, so two levels cost one LDS round trip.
    __device__ __forceinline__ Key pop() {
        const Key top = get(0);
        const Key last = get(--size);
        const Key w = last >> NB;
        constexpr int lim = CAP - 1;
        int i = 0;
        for (;;) {
            const int l = 2 * i + 1;
            if (l >= size) break;
            const int g = 2 * l + 1;
            const Key kl = get(l), kr = get(min(l + 1, lim));
            Key g0 = get(min(g, lim)), g1 = get(min(g + 1, lim));
            Key g2 = get(min(g + 2, lim)), g3 = get(min(g + 3, lim));
            asm volatile("" : "+v"(g0), "+v"(g1), "+v"(g2), "+v"(g3));   // keep the loads together
            const bool pr = l + 1 < size && (kr >> NB) < (kl >> NB);
            const Key kc = pr ? kr : kl;
            if (!(w > (kc >> NB))) break;
            set(i, kc);
            i = l + (pr ? 1 : 0);
            const int l2 = 2 * i + 1;
            if (l2 >= size) break;
            const Key a = pr ? g2 : g0, b = pr ? g3 : g1;
            const bool pr2 = l2 + 1 < size && (b >> NB) < (a >> NB);
            const Key kc2 = pr2 ? b : a;
            if (!(w > (kc2 >> NB))) break;
            set(i, kc2);
            i = l2 + (pr2 ? 1 : 0);
        }
        set(i, last);
        return top;
    }
};

// Count scan: calls f(symbol, count) for every nonzero count in symbol order.
// zero(symbol) is called for the symbols that never occur (their code table entry).
template <typename F, typename Z>
__device__ __forceinline__ void scan_counts(const uint32_t* __restrict__ cnt, int k, F&& f,
                                            Z&& zero) {
    const int kv = (k & 31) ? 0 : k;           // vector part (count rows are 16-B aligned)
    const uint4* cnt4 = reinterpret_cast<const uint4*>(cnt);
    for (int s0 = 0; s0 < kv; s0 += 32) {      // 128 B of counts in flight per lane
        uint4 q[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) q[u] = cnt4[(s0 >> 2) + u];
#pragma unroll
        for (int u = 0; u < 32; ++u) {
            const uint32_t c = u % 4 == 0 ? q[u / 4].x : u % 4 == 1 ? q[u / 4].y
                             : u % 4 == 2 ? q[u / 4].z : q[u / 4].w;
            if (c) f(s0 + u, c);
            else zero(s0 + u);
        }
    }
    for (int s = kv; s < k; ++s) {             // small / odd alphabets
        const uint32_t c = cnt[s];
        if (c) f(s, c);
        else zero(s);
    }
}

// Merge loop of huffman_codebook_init_encoder (huffman_encode.c:150-190) on one lane's heap:
// the nz leaves (counts lcnt, in symbol order) are pushed, then pop two / push their sum
// until one node is left.  Returns the node count; kid[q - nz] = children of internal node q.
template <typename Key, int NB, int TPW, int CAP, bool SPLIT = false>
__device__ __forceinline__ int merge_tree(typename LdsHeap<Key, NB, TPW, CAP, SPLIT>::Word* heap_base,
                                          const uint32_t* lcnt, int nz, uint32_t* kid) {
    LdsHeap<Key, NB, TPW, CAP, SPLIT> hp{heap_base, 0};
    for (int j = 0; j < nz; ++j) hp.push(((Key)lcnt[j * TPW] << NB) | (Key)j);
    int next = nz;
    const Key nmask = ((Key)1 << NB) - 1;
    if (hp.size == 1) {  // lone symbol: code "0" (huffman_encode.c:168-177)
        const Key e = hp.pop();
        kid[0] = (uint32_t)(e & nmask) | 0xFFFF0000u;
        hp.push(((e >> NB) << NB) | (Key)next);
        ++next;
    }
    while (hp.size > 1) {
        const Key a = hp.pop();
        const Key b = hp.pop();
        kid[(next - nz) * TPW] = (uint32_t)(a & nmask) | ((uint32_t)(b & nmask) << 16);
        hp.push((((a >> NB) + (b >> NB)) << NB) | (Key)next);
        ++next;
    }
    return next;
}

// Sentinel heap for K <= 256 and tree totals below 2^22 (the common case): u32 keys
// weight << 10 | tie << 9 | node.  Every slot past the heap holds 0xFFFFFFFF, so children
// need no bounds checks.  The reference rules (huffman_encode.c:33-76) become single
// integer ops: "left child unless the right one is strictly lighter" is
// min(left, right | TIE) (the tie bit makes an equal-weight right child lose), and "move
// while strictly heavier" is child < (last & ~LOW) (weights compared, low bits ignored).
template <int TPW>
struct SentinelHeap {
    static constexpr uint32_t kTie = 1u << 9, kLow = (1u << 10) - 1, kMax = 0xFFFFFFFFu;
    static constexpr int kSlots = 512;         // heap < 256 entries; reads clamp to slot 511
    uint32_t* h;                               // this lane's slot 0 (stride TPW)
    int size;
    __device__ __forceinline__ uint32_t get(int i) const { return h[min(i, kSlots - 1) * TPW]; }
    __device__ __forceinline__ void set(int i, uint32_t v) { h[i * TPW] = v; }
    // sift up while strictly lighter than the parent; three ancestors per LDS round trip
    __device__ __forceinline__ void push(uint32_t e) {
        int i = size++;
        bool act = true;
        while (true) {
            const int p1 = (i - 1) >> 1, p2 = (p1 - 1) >> 1, p3 = (p2 - 1) >> 1;
            uint32_t a1 = get(max(p1, 0)), a2 = get(max(p2, 0)), a3 = get(max(p3, 0));
            asm volatile("" : "+v"(a1), "+v"(a2), "+v"(a3));
            bool mv = act && i > 0 && e < (a1 & ~kLow);
            if (mv) { set(i, a1); i = p1; }
            act = mv;
            mv = act && i > 0 && e < (a2 & ~kLow);
            if (mv) { set(i, a2); i = p2; }
            act = mv;
            mv = act && i > 0 && e < (a3 & ~kLow);
            if (mv) { set(i, a3); i = p3; }
            act = mv;
            if (!__any(act)) break;
        }
        set(i, e);
    }
    __device__ __forceinline__ uint32_t pop() {
        const uint32_t top = get(0);
        const uint32_t last = get(--size);
        set(size, kMax);                       // the vacated slot becomes a sentinel
        const uint32_t lw = last & ~kLow;      // child < lw  <=>  child weight < last weight
        int i = 0;
        bool act = true;
        while (true) {
            const int c = 2 * i + 1, g = 4 * i + 3;
            uint32_t kl = get(c), kr = get(c + 1);
            uint32_t g0 = get(g), g1 = get(g + 1), g2 = get(g + 2), g3 = get(g + 3);
            asm volatile("" : "+v"(kl), "+v"(kr), "+v"(g0), "+v"(g1), "+v"(g2), "+v"(g3));
            const uint32_t kc = min(kl, kr | kTie);
            const bool pr = (kc & kTie) != 0;
            bool mv = act && kc < lw;
            if (mv) { set(i, kc & ~kTie); i = c + (int)pr; }
            act = mv;
            const uint32_t kc2 = min(pr ? g2 : g0, (pr ? g3 : g1) | kTie);
            mv = act && kc2 < lw;
            if (mv) { set(i, kc2 & ~kTie); i = 2 * i + 1 + (int)((kc2 & kTie) != 0); }
            act = mv;
            if (!__any(act)) break;
        }
        set(i, last);
        return top;
    }
};

// ---- one wavefront per tree: the heap in registers ------------------------------------
// The reference heap (huffman_encode.c:33-76) simulated with its entries spread over the
// lanes of five VGPRs: slot s lives in register (s + 1) >> 6 at lane (s + 1) & 63, so every
// heap depth but the seventh has one fixed register (depth 7 has two, picked by bit 6).
// The tree's control state (slot index, keys being sifted) is wave-uniform and lives in
// SGPRs; a heap read is one v_readlane with a scalar lane index, a write a lane select --
// no LDS round trip on the serial chain of sifts, which is what bounds a tree build (one
// lane per tree through LDS: ~4,000 cycles a merge).  The sifts are unrolled by depth so
// every access names its register statically.
// Keys are the SentinelHeap's: weight << 10 | tie << 9 | node, u32 while the tree's total
// weight is below 2^22, else u64 (two words per slot); slots past the heap hold all ones, so
// children need no bounds checks.
template <typename Key>
__device__ __forceinline__ Key lane_read(const Key& v, int ln) {
    if constexpr (sizeof(Key) == 4) {
        return (Key)__builtin_amdgcn_readlane((int)v, ln);
    } else {
        const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)v, ln);
        const uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(v >> 32), ln);
        return ((Key)hi << 32) | lo;
    }
}

template <typename Key>
struct WaveHeap {
    static constexpr Key kTie = (Key)1 << 9, kLow = ((Key)1 << 10) - 1, kMax = ~(Key)0;
    Key r0, r1, r2, r3, r4;   // slots with s + 1 in 1..63 | 64..127 | 128..191 | 192..255 | 256
    int size;
    int me;                    // this lane's id
    __device__ __forceinline__ void init() {
        r0 = r1 = r2 = r3 = r4 = kMax;
        size = 0;
        me = (int)(threadIdx.x & 63);
    }
    // register of slot s (as a value: a uniform select, no branch)
    __device__ __forceinline__ Key reg(int s) const {
        const int r = (s + 1) >> 6;
        return r == 0 ? r0 : r == 1 ? r1 : r == 2 ? r2 : r == 3 ? r3 : r4;
    }
    __device__ __forceinline__ Key get(int s) const {
        return s < 256 ? lane_read(reg(s), (s + 1) & 63) : kMax;   // past 255: never in the heap
    }
    __device__ __forceinline__ void set(int s, Key v) {
        const int r = (s + 1) >> 6;
        const bool hit = me == ((s + 1) & 63);
        r0 = hit && r == 0 ? v : r0;
        r1 = hit && r == 1 ? v : r1;
        r2 = hit && r == 2 ? v : r2;
        r3 = hit && r == 3 ? v : r3;
        r4 = hit && r == 4 ? v : r4;
    }
    // sift up while strictly lighter than the parent (huffman_encode.c:33-46)
    __device__ __forceinline__ void push(Key e) {
        int i = size++;
        while (i > 0) {
            const int p = (i - 1) >> 1;
            const Key hp = get(p);
            if (!(e < (hp & ~kLow))) break;
            set(i, hp);
            i = p;
        }
        set(i, e);
    }
    // the last entry sifts down from the root: the left child unless the right one is
    // strictly lighter (min(left, right | TIE)), moving while it is strictly heavier than
    // that child (huffman_encode.c:48-76).  Both children share a register.
    __device__ __forceinline__ Key pop() {
        const Key top = lane_read(r0, 1);
        const Key last = get(--size);
        set(size, kMax);   // the vacated slot becomes a sentinel
        const Key lw = last & ~kLow;
        int i = 0;
        while (i < 128) {
            const int c = 2 * i + 1;
            const Key rc = reg(c);
            const Key kl = lane_read(rc, (c + 1) & 63);
            const Key kr = c + 1 < 256 ? lane_read(rc, (c + 2) & 63) : kMax;
            const Key kc = min(kl, kr | kTie);
            if (!(kc < lw)) break;
            set(i, kc & ~kTie);
            i = c + ((kc & kTie) ? 1 : 0);
        }
        set(i, last);
        return top;
    }
};

// The u32-key heap (tree totals below 2^22: every bench and test alphabet but the heaviest)
// with its sifts as generated inline asm (pqh_heap_asm.h): the heap occupies v40..v47, the
// operands are SGPRs.  Same slot layout and semantics as WaveHeap<uint32_t>.
typedef uint32_t u32x8 __attribute__((ext_vector_type(8)));
struct WaveHeapAsm {
    u32x8 h;
    int size;
    __device__ __forceinline__ void init() {
        h = u32x8(0xFFFFFFFFu);
        size = 0;
    }
    __device__ __forceinline__ void push(uint32_t e) {
        uint32_t i = (uint32_t)size++, p, ln, hp, hw, t, d, m0s;
        asm volatile(PQH_HEAP_PUSH_ASM
                     : [i] "+&s"(i), [p] "=&s"(p), [ln] "=&s"(ln), [hp] "=&s"(hp), [hw] "=&s"(hw),
                       [t] "=&s"(t), [d] "=&s"(d), [m0s] "=&s"(m0s), "+{v[40:47]}"(h)
                     : [e] "s"(e)
                     : "scc");
    }
    __device__ __forceinline__ uint32_t pop() {
        const uint32_t sz = (uint32_t)(--size);
        uint32_t top, i, c, ln, kl, kr, kc, lw, last, t, m0s;
        asm volatile(PQH_HEAP_POP_ASM
                     : [top] "=&s"(top), [i] "=&s"(i), [c] "=&s"(c), [ln] "=&s"(ln),
                       [kl] "=&s"(kl), [kr] "=&s"(kr), [kc] "=&s"(kc), [lw] "=&s"(lw),
                       [last] "=&s"(last), [t] "=&s"(t), [m0s] "=&s"(m0s), "+{v[40:47]}"(h)
                     : [sz] "s"(sz)
                     : "scc");
        return top;
    }
};

template <typename Key>
struct HeapFor { using type = WaveHeap<Key>; };
template <>
struct HeapFor<uint32_t> { using type = WaveHeapAsm; };

__device__ unsigned long long g_tree_stamps[16];

template <typename Key>
__device__ __forceinline__ int wave_merge(uint32_t lc0, uint32_t lc1, uint32_t lc2, uint32_t lc3,
                                          int nz, uint32_t* kid, int lane, bool stamp_tree) {
    typename HeapFor<Key>::type hp;
    hp.init();
    const bool stamp = stamp_tree;
    for (int j = 0; j < nz; ++j) {
        const uint32_t lcr = (j >> 6) == 0 ? lc0 : (j >> 6) == 1 ? lc1 : (j >> 6) == 2 ? lc2 : lc3;
        hp.push(((Key)(uint32_t)__builtin_amdgcn_readlane((int)lcr, j & 63) << 10) | (Key)j);
    }
    if (stamp && lane == 0) g_tree_stamps[2] = __builtin_amdgcn_s_memtime();
    int next = nz;
    constexpr Key kNode = 511, kW = ~(Key)1023;
    if (hp.size == 1) {   // lone symbol: code "0" (huffman_encode.c:168-177)
        const Key e = hp.pop();
        if (lane == 0) kid[0] = (uint32_t)(e & kNode) | 0xFFFF0000u;
        hp.push((e & kW) | (Key)next);
        ++next;
    }
    while (hp.size > 1) {
        const Key a = hp.pop();
        const Key b = hp.pop();
        if (lane == 0) kid[next - nz] = (uint32_t)(a & kNode) | ((uint32_t)(b & kNode) << 16);
        hp.push(((a & kW) + (b & kW)) | (Key)next);
        ++next;
    }
    return next;
}

__device__ __forceinline__ void wave_sync_lds() {
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    __builtin_amdgcn_wave_barrier();
}

// One wavefront per (part, context) alphabet, K <= 256: counts -> code table entries
// len << 56 | code for every symbol (0 for symbols that never occur).  Four trees per
// workgroup; waves are independent (no workgroup barrier).  Codes come from the merge record
// by pointer jumping over the tree (code(v) = code(anc) << len | bits) -- eight parallel
// rounds instead of a serial walk from the root.
constexpr int kTreeWaves = 4;
// A tree build's first workgroup of each table set zeroes that set's two LUT pool heads
// (d_err[2..5]), which the decode-table build that follows it allocates from: no memset
// dispatch in front of the build.  (A fused tree + LUT build zeroes only the slot it does
// not use -- huff_trees_grp.)  The error word d_err[0] is sticky until pqh_tables_status.
__device__ __forceinline__ void reset_pool_head(uint32_t* err) {
    reinterpret_cast<unsigned long long*>(err + 2)[0] = 0ull;
    reinterpret_cast<unsigned long long*>(err + 2)[1] = 0ull;
}

__global__ void __launch_bounds__(64 * kTreeWaves)
huff_trees_wave(const uint32_t* __restrict__ counts, int k, long long trees,
                unsigned long long* __restrict__ enc, uint32_t* __restrict__ err) {
    __shared__ uint32_t s_kid[kTreeWaves][256];
    __shared__ uint32_t s_leaf[kTreeWaves][256];              // count, then the symbol
    __shared__ uint32_t s_al[kTreeWaves][512];                // anc | len << 16
    __shared__ unsigned long long s_code[kTreeWaves][512];
    const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
    if (blockIdx.x == 0 && threadIdx.x == 0) reset_pool_head(err);
    const long long tree = (long long)blockIdx.x * kTreeWaves + w;
    if (tree >= trees) return;   // no workgroup barriers below
    const uint32_t* cnt = counts + tree * k;
    unsigned long long* out = enc + tree * k;
    if (tree == 0 && lane == 0) g_tree_stamps[0] = __builtin_amdgcn_s_memtime();
    uint32_t* kid = s_kid[w];
    uint32_t* leaf = s_leaf[w];
    uint32_t* al = s_al[w];
    unsigned long long* code = s_code[w];
    // nonzero counts in symbol order (huffman_encode.c:158), compacted by ballot
    int nz = 0;
    unsigned long long total = 0;
    uint32_t cg[4];
#pragma unroll
    for (int g = 0; g < 4; ++g) {
        const int sy = 64 * g + lane;
        cg[g] = sy < k ? cnt[sy] : 0u;
    }
#pragma unroll
    for (int g = 0; g < 4; ++g) {
        const int sy = 64 * g + lane;
        const unsigned long long mask = __ballot(cg[g] != 0u);
        const int pos = nz + (int)__builtin_amdgcn_mbcnt_hi((unsigned)(mask >> 32),
                                                            __builtin_amdgcn_mbcnt_lo((unsigned)mask, 0u));
        if (cg[g]) {
            leaf[pos] = cg[g];
            kid[pos] = (uint32_t)sy;   // (kid is free until the merges: symbols parked here)
        } else if (sy < k) {
            out[sy] = 0ull;            // a symbol that never occurs has no code
        }
        nz += __popcll(mask);
        unsigned long long v = cg[g];
#pragma unroll
        for (int off = 32; off >= 1; off >>= 1) v += __shfl_xor(v, off);
        total += v;
    }
    if (nz == 0) return;
    wave_sync_lds();
    const uint32_t lc0 = leaf[lane], lc1 = leaf[64 + lane], lc2 = leaf[128 + lane],
                   lc3 = leaf[192 + lane];
    uint32_t sym[4];
#pragma unroll
    for (int g = 0; g < 4; ++g) sym[g] = kid[64 * g + lane];
    wave_sync_lds();
    const bool stamp = tree == 0;
    if (stamp && lane == 0) g_tree_stamps[1] = __builtin_amdgcn_s_memtime();
    const int next = total < (1ull << 22)
                         ? wave_merge<uint32_t>(lc0, lc1, lc2, lc3, nz, kid, lane, stamp)
                         : wave_merge<unsigned long long>(lc0, lc1, lc2, lc3, nz, kid, lane, stamp);
    if (stamp && lane == 0) g_tree_stamps[3] = __builtin_amdgcn_s_memtime();
    wave_sync_lds();
    // the parent links: child 0 gets bit 0, child 1 bit 1 (huffman_encode.c:100-132)
    const int root = next - 1;
    for (int q = nz + lane; q < next; q += 64) {
        const uint32_t kk = kid[q - nz];
        const uint32_t a = kk & 0xFFFFu, b = kk >> 16;
        al[a] = (uint32_t)q | (1u << 16);
        code[a] = 0ull;
        if (b != 0xFFFFu) {
            al[b] = (uint32_t)q | (1u << 16);
            code[b] = 1ull;
        }
    }
    if (lane == 0) {
        al[root] = 0xFFFFu;   // no ancestor, length 0
        code[root] = 0ull;
    }
    wave_sync_lds();
    // pointer jumping: after round r every node's link spans 2^r levels (depth <= 255)
    for (int round = 0; round < 9; ++round) {
        uint32_t nal[8];
        unsigned long long ncode[8];
        bool live = false;
#pragma unroll
        for (int u = 0; u < 8; ++u) {
            const int v = lane + 64 * u;
            nal[u] = 0xFFFFu;
            ncode[u] = 0ull;
            if (v < next) {
                const uint32_t x = al[v];
                nal[u] = x;
                ncode[u] = code[v];
                const uint32_t anc = x & 0xFFFFu;
                if (anc != 0xFFFFu) {
                    const uint32_t y = al[anc];
                    const uint32_t len = (x >> 16) & 0xFFu, len2 = (y >> 16) & 0xFFu;
                    const uint32_t nl = min(len + len2, 255u);
                    ncode[u] = (len < 64 ? code[anc] << len : 0ull) | ncode[u];
                    nal[u] = (y & 0xFFFFu) | (nl << 16);
                    live = true;
                }
            }
        }
        wave_sync_lds();
#pragma unroll
        for (int u = 0; u < 8; ++u) {
            const int v = lane + 64 * u;
            if (v < next) {
                al[v] = nal[u];
                code[v] = ncode[u];
            }
        }
        wave_sync_lds();
        if (!__any(live)) break;
    }
    bool too_long = false;
#pragma unroll
    for (int g = 0; g < 4; ++g) {
        const int j = 64 * g + lane;
        if (j < nz) {
            const unsigned long long len = (al[j] >> 16) & 0xFFu;
            if (len > (unsigned long long)kMaxCodeLen) too_long = true;
            else out[sym[g]] = (len << 56) | (code[j] & kCodeMask);
        }
    }
    if (too_long) atomicOr(err, 1u);
    if (tree == 0 && lane == 0) {
        g_tree_stamps[4] = __builtin_amdgcn_s_memtime();
        g_tree_stamps[5] = (unsigned long long)nz;
        g_tree_stamps[6] = (unsigned long long)next;
    }
}

// diagnostics: s_memtime stamps of the first workgroup's phases (pqh_debug_stamps):
// [0..6] huff_trees tree 0, [8..13] dec_chunks workgroup 0 lane 0 (g_tree_stamps, above)

// Compact per-tree layout for K <= 256 (3.5 KB, so 32 trees fit one workgroup and the
// whole build occupies 64 CUs -- it can run beside the next batch's assignment):
//   heap u32 [512]  (sentinel heap; after the merges the internal nodes' codes, u64 [255])
//   kid  u32 [256]  (children of internal node q at q - nz; the leaf counts before that)
//   lsym u16 [256]  (symbol of leaf j)
// all interleaved tree-minor (element e of lane t at [e * TPW + t]).
template <int TPW>
__global__ void __launch_bounds__(64)
huff_trees_small(const uint32_t* __restrict__ counts, int k, long long trees,
                 unsigned long long* __restrict__ enc, uint32_t* __restrict__ err,
                 long long trees2, const uint32_t* __restrict__ counts2,
                 unsigned long long* __restrict__ enc2, uint32_t* __restrict__ err2) {
    // trees [0, trees) from counts -> enc; a paired build (pqh_tables_build_pair) adds trees
    // [trees, trees + trees2) of a second table set
    if ((long long)blockIdx.x * TPW >= trees) {
        const long long b = (long long)blockIdx.x - (trees + TPW - 1) / TPW;
        counts = counts2 + b * TPW * k;
        enc = enc2 + b * TPW * k;
        err = err2;
        trees = trees2 - b * TPW;
        if (b == 0 && threadIdx.x == 0) reset_pool_head(err);
    } else {
        if (blockIdx.x == 0 && threadIdx.x == 0) reset_pool_head(err);
        trees -= (long long)blockIdx.x * TPW;
        counts += (long long)blockIdx.x * TPW * k;
        enc += (long long)blockIdx.x * TPW * k;
    }
    extern __shared__ __attribute__((aligned(16))) char lds[];
    uint32_t* heap_all = reinterpret_cast<uint32_t*>(lds);
    uint32_t* kid_all = heap_all + 512 * TPW;
    uint16_t* lsym_all = reinterpret_cast<uint16_t*>(kid_all + 256 * TPW);
    const int t = threadIdx.x;
    {   // the whole workgroup fills the heap slots with sentinels
        uint4* z = reinterpret_cast<uint4*>(heap_all);
        for (int q = t; q < 512 * TPW / 4; q += blockDim.x) z[q] = make_uint4(~0u, ~0u, ~0u, ~0u);
        __syncthreads();
    }
    if (t >= TPW) return;  // no barriers below
    if (t >= trees) return;   // (counts / enc / trees are this workgroup's, above)
    const uint32_t* cnt = counts + (long long)t * k;
    unsigned long long* out = enc + (long long)t * k;
    const bool stamp = blockIdx.x == 0 && t == 0;
#ifdef PQH_LAT_PRIO   // (experiment) latency-bound waves first in issue arbitration
    __builtin_amdgcn_s_setprio(PQH_LAT_PRIO);
#endif
    if (stamp) g_tree_stamps[0] = __builtin_amdgcn_s_memtime();
    uint32_t* kid = kid_all + t;
    uint32_t* lcnt = kid;                      // leaf counts until the first merge
    uint16_t* lsym = lsym_all + t;
    unsigned long long total = 0;
    int nz = 0;
    scan_counts(cnt, k, [&](int s, uint32_t c) {
        lsym[nz * TPW] = (uint16_t)s;
        lcnt[nz * TPW] = c;
        total += c;
        ++nz;
    }, [&](int s) { out[s] = 0ull; });   // no code (the table set is not memset)
    if (nz == 0) return;
    if (stamp) g_tree_stamps[1] = __builtin_amdgcn_s_memtime();
    int next;
    // u32 heap: key payloads are the leaf's symbol (< 256) or 256 + the internal node's
    // creation index, so the code pass reads no symbol table; the 64-bit heap's are node ids.
    // The packing weight << 10 | tie << 9 | payload holds because (1) k <= 256 (the host
    // launches this kernel, like huff_trees_grp, only for k <= 256 -- checked again here), so
    // symbols fit 8 bits and the <= 255 internal nodes give payloads <= 256 + 254 < 512, and
    // (2) the tree's total weight is < 2^22, so every node weight (<= total) shifted by 10
    // stays below 2^32; heavier trees take the 64-bit path.
    if (k > 256) {
        atomicOr(err, 2u);
        return;
    }
    const bool symp = total < (1ull << 22);
    if (symp) {
        SentinelHeap<TPW> hp{heap_all + t, 0};
        for (int j = 0; j < nz; ++j) hp.push((lcnt[j * TPW] << 10) | (uint32_t)lsym[j * TPW]);
        if (stamp) g_tree_stamps[2] = __builtin_amdgcn_s_memtime();
        next = nz;
        if (hp.size == 1) {  // lone symbol: code "0" (huffman_encode.c:168-177)
            const uint32_t e = hp.pop();
            kid[0] = (e & 511u) | 0xFFFF0000u;
            hp.push((e & ~1023u) | (uint32_t)(256 + next - nz));
            ++next;
        }
        while (hp.size > 1) {
            const uint32_t a = hp.pop();
            const uint32_t b = hp.pop();
            kid[(next - nz) * TPW] = (a & 511u) | ((b & 511u) << 16);
            hp.push(((a & ~1023u) + (b & ~1023u)) | (uint32_t)(256 + next - nz));
            ++next;
        }
    } else {   // heavy tree: 64-bit keys (u64 [256] as word pairs of the lane's own column)
        next = merge_tree<unsigned long long, 16, TPW, 256, true>(heap_all + t, lcnt, nz, kid);
    }
    if (stamp) g_tree_stamps[3] = __builtin_amdgcn_s_memtime();
    // codes top-down in reverse creation order (parents are created after their children):
    // depth << 56 | code, child 0 appends bit 0 (huffman_encode.c:100-132); internal nodes
    // keep theirs in the dead heap, leaves go straight to the code table
    constexpr unsigned long long kMask = (1ull << 56) - 1;
    unsigned long long* icode = reinterpret_cast<unsigned long long*>(heap_all) + t;
    icode[(next - 1 - nz) * TPW] = 0;         // root
    bool too_long = false;
    for (int q = next - 1; q >= nz; --q) {
        const unsigned long long e = icode[(q - nz) * TPW];
        const uint32_t kk = kid[(q - nz) * TPW];
        const unsigned long long d = min((e >> 56) + 1, 255ull);
        const unsigned long long c = (e & kMask) << 1;
#pragma unroll
        for (int b = 0; b < 2; ++b) {
            const uint32_t ch = b ? kk >> 16 : kk & 0xFFFFu;
            if (ch == 0xFFFFu) continue;
            const unsigned long long v = (d << 56) | ((c | (unsigned long long)b) & kMask);
            const int base = symp ? 256 : nz;   // first internal payload
            if ((int)ch >= base) {
                icode[((int)ch - base) * TPW] = v;
            } else if (d > (unsigned long long)kMaxCodeLen) {
                too_long = true;
            } else {
                out[symp ? ch : lsym[ch * TPW]] = v;
            }
        }
    }
    if (too_long) atomicOr(err, 1u);
    if (stamp) {
        g_tree_stamps[4] = __builtin_amdgcn_s_memtime();
        g_tree_stamps[5] = (unsigned long long)nz;
        g_tree_stamps[6] = (unsigned long long)next;
    }
}

// ---- sixteen lanes per tree, four trees per wavefront (K <= 256; the default build) -------
// The heap of huffman_encode.c:33-76 in LDS, each sift read a stretch at a time by the
// tree's 16 lanes, so a heap level costs no LDS round trip of its own:
//   push  lane l reads ancestor l + 1 of the new slot (the whole path: one round trip); the
//         ancestors the entry passes are those strictly heavier than it -- a prefix of the
//         path (weights fall towards the root), so the group's ballot popcount is the stop
//         level -- and they move down one level in one write;
//   pop   lane q = 1..15 stands for node q of the 4-level subtree below the hole (heap
//         numbering, q = 1 the hole itself) and reads that node's two children in one
//         ds_read2: kc = the reference's candidate (left unless the right is strictly
//         lighter: min(left, right | TIE)), mv = the sinking entry moves past it.  Lane q is
//         on the sink's path iff every ancestor p of q in the stretch chose the side towards
//         q and moved: two compares of the group's ballots against lane constants A(q) (the
//         ancestors' bits) and E(q) (the directions towards q) -- no serial walk down the
//         path.  Lanes on the path move their candidate up; the one whose candidate does not
//         move takes the sinking entry.  If a depth-3 lane moved, the next stretch starts at
//         its candidate's slot (two stretches cover a 256-entry heap).
// Keys are the SentinelHeap's (weight << 10 | tie << 9 | payload, slots past the heap all
// ones; payload = the leaf's symbol or 256 + the internal node's creation index), u32 when
// every tree of the wavefront weighs < 2^22, else u64.  The codes come from the merge record
// by pointer jumping.  At most 32 VGPRs: the persistent assignment grid (3 waves x 160 VGPRs
// per SIMD) leaves exactly that, so the build runs beside it instead of between its launches.
constexpr int kGrpTrees = 4;                        // trees per wavefront
constexpr int kGrpHeapBytes = 4096;                 // heap (<= 257 slots) / codes u64 [512]
constexpr int kGrpKidBytes = 1024;                  // kid u32 [256]
constexpr int kGrpLeafBytes = 2048;                 // leaf keys u64 [256] / links u16 [512]
constexpr int kGrpTreeBytes = kGrpHeapBytes + kGrpKidBytes + kGrpLeafBytes;

// the 16 ballot bits of this lane's group
__device__ __forceinline__ uint32_t grp_bits(bool pred, int gsh) {
    return (uint32_t)(__ballot(pred) >> gsh) & 0xFFFFu;
}

// 1-based heap positions (slot s of the reference heap at h[s + 1]); h[0] = 0 makes a
// missing ancestor read as lighter than anything, positions past the heap hold all ones.
struct GrpHeap {
    static constexpr uint32_t kTie = 1u << 9, kLow = 1023u, kMax = ~0u;
    static constexpr int kDummy = 1023;   // lanes off the write set store here (never read)
    uint32_t* h;     // this tree's positions
    int n;           // entries
    int gl;          // lane in the group
    int gsh;         // the group's first bit in a ballot
    int dq, off;     // node gl of a stretch below hole I: (I << dq) + off (lane 0: past the heap)
    uint32_t A, E;   // ancestors of node gl in a stretch, and the directions towards gl
    // ancestor gl + 1 of the position a push fills (0 when there is none)
    __device__ __forceinline__ uint32_t anc() const { return h[(n + 1) >> (gl + 1)]; }
    // huffman_encode.c:33-46 (sift up while strictly lighter), `a` = anc(): lanes below the
    // stop level move their ancestor down, the stop level takes e -- one store, no branch
    __device__ __forceinline__ void push(uint32_t e, uint32_t a) {
        const int s = __popc((uint32_t)(__ballot(e < (a & ~kLow)) >> gsh) & 0xFFFFu);
        h[gl <= s ? (n + 1) >> gl : kDummy] = gl < s ? a : e;
        ++n;
    }
    // one stretch below hole I: lane gl's node, its candidate child, whether the sinking
    // entry passes it; the lanes on the sink's path store (branch-free); returns the ballot
    // bits of the group's path lanes
    __device__ __forceinline__ uint32_t stretch(int G, uint32_t kl, uint32_t kr, uint32_t lw,
                                                uint32_t last, bool act, uint32_t& mm,
                                                uint32_t& md) {
        const uint32_t t = kr | kTie;
        const uint32_t kc = min(kl, t);
        const bool mv = kc < lw;
        mm = (uint32_t)(__ballot(mv) >> gsh);
        md = (uint32_t)(__ballot(t < kl) >> gsh);
        const bool on = act && (((md ^ E) | ~mm) & A) == 0;
        h[on ? G : kDummy] = mv ? (kc & ~kTie) : last;
        return (uint32_t)(__ballot(on) >> gsh);
    }
    // huffman_encode.c:48-76: the last entry sinks from the root, moving while strictly
    // heavier than the candidate child (left unless the right one is strictly lighter).
    // Two stretches cover every sink: the second's deepest nodes (level 7) have no children
    // in a heap of < 256 entries, and at 256 entries position 256 is the sinking entry itself.
    __device__ __forceinline__ uint32_t pop() {
        // the root, the last entry and the first stretch's children in one round trip; the
        // sentinel store sits between them in LDS order (LDS is in order)
        const int G1 = gl ? gl : 256;   // stretch 1 below the root: node gl
        const int g1 = min(G1, 129);     // (nodes past 128 have no children in the heap)
        const uint32_t top = h[1];
        const uint32_t last = h[n];
        h[gl ? kDummy : n] = kMax;       // the vacated position becomes a sentinel
        uint32_t kl = h[2 * g1], kr = h[2 * g1 + 1];
        --n;
        const uint32_t lw = last & ~kLow;
        uint32_t mm, md;
        const uint32_t onm = stretch(G1, kl, kr, lw, last, gl != 0, mm, md);
        const uint32_t deep = onm & mm & 0xFF00u;   // the path left the stretch below level 3
        if (__any(deep)) {
            const int p = deep ? __ffs(deep) - 1 : 8;
            const int I = 2 * p + (int)((md >> p) & 1u);   // the hole, level 4
            const int G = (I << dq) + off;
            const int g = min(G, 129);
            kl = h[2 * g];
            kr = h[2 * g + 1];
            (void)stretch(G, kl, kr, lw, last, deep != 0u, mm, md);
        }
        return top;
    }
};

// leaves (pushed in symbol order), merges; returns the internal-node count
__device__ __forceinline__ int grp_merge(GrpHeap& hp, const unsigned long long* lkey, int nz,
                                         uint32_t* kid, bool stamp) {
    constexpr uint32_t kLow = GrpHeap::kLow;
    for (int j = 0; j < nz; ++j) {
        const uint32_t a = hp.anc();
        const uint32_t e = (uint32_t)lkey[j];   // (read in the same round trip as the ancestors)
        hp.push(e, a);
    }
    if (stamp) g_tree_stamps[2] = __builtin_amdgcn_s_memtime();
    int next = 0;
    if (hp.n == 1) {   // lone symbol: code "0" (huffman_encode.c:168-177)
        const uint32_t e = hp.pop();
        if (hp.gl == 0) kid[0] = (e & 511u) | 0xFFFF0000u;
        hp.push((e & ~kLow) | 256u, hp.anc());
        next = 1;
    }
    while (hp.n > 1) {
        const uint32_t a = hp.pop();
        const uint32_t b = hp.pop();
        kid[hp.gl ? 255 : next] = (a & 511u) | ((b & 511u) << 16);   // (255: never a node)
        hp.push(((a & ~kLow) + (b & ~kLow)) | (uint32_t)(256 + next), hp.anc());
        ++next;
    }
    return next;
}

// A tree weighing 2^22 or more (counts accumulated over more than ~4M rows): the same heap
// with u64 keys, sifted by one lane (the group's other lanes wait) -- the cooperative u64
// sifts would take the build past its 32-VGPR budget, and such trees are rare.
__device__ __forceinline__ int grp_merge_heavy(unsigned long long* h, const unsigned long long* lkey,
                                               int nz, uint32_t* kid) {
    using Key = unsigned long long;
    constexpr Key kTie = 1ull << 9, kLow = 1023ull, kMax = ~0ull;
    int n = 0;
    auto push = [&](Key e) {
        int i = n++;
        while (i > 0) {
            const int p = (i - 1) >> 1;
            const Key hp = h[p];
            if (!(e < (hp & ~kLow))) break;
            h[i] = hp;
            i = p;
        }
        h[i] = e;
    };
    auto pop = [&]() -> Key {
        const Key top = h[0];
        const Key last = h[--n];
        h[n] = kMax;
        const Key lw = last & ~kLow;
        int i = 0;
        while (i < 128) {
            const Key kl = h[2 * i + 1], kr = h[2 * i + 2];
            const Key kc = min(kl, kr | kTie);
            if (!(kc < lw)) break;
            h[i] = kc & ~kTie;
            i = 2 * i + 1 + ((kc & kTie) ? 1 : 0);
        }
        h[i] = last;
        return top;
    };
    for (int j = 0; j < nz; ++j) push(lkey[j]);
    int next = 0;
    if (n == 1) {   // lone symbol
        const Key e = pop();
        kid[0] = (uint32_t)(e & 511) | 0xFFFF0000u;
        push((e & ~kLow) | 256ull);
        next = 1;
    }
    while (n > 1) {
        const Key a = pop();
        const Key b = pop();
        kid[next] = (uint32_t)(a & 511) | ((uint32_t)(b & 511) << 16);
        push(((a & ~kLow) + (b & ~kLow)) | (Key)(256 + next));
        ++next;
    }
    return next;
}

// Pointers of the decode tables lut_grp writes (the layout of lut_build, below).
struct GrpLut {
    uint32_t* enc32;
    uint16_t* enc16;   // (written with enc32)
    uint16_t* lut1;
    uint16_t* lut2;
    uint32_t* meta;
    pqh_long_code* longs;
    uint32_t* long_cnt;
    unsigned long long* pool_head;
    long long lut2_cap;
    int w1, l2_bits;
    int prio;   // wave issue priority (pqh_prio)
};

__device__ __forceinline__ void grp_luts(const GrpLut& L, long long t, int k, int lane, int gl,
                                         int gsh, const unsigned long long* code, char* scratch);

__global__ void __launch_bounds__(64) __attribute__((amdgpu_num_vgpr(32)))
huff_trees_grp(const uint32_t* __restrict__ counts, int k, long long trees,
               unsigned long long* __restrict__ enc, uint32_t* __restrict__ err,
               long long trees2, const uint32_t* __restrict__ counts2,
               unsigned long long* __restrict__ enc2, uint32_t* __restrict__ err2, int prio,
               uint32_t* __restrict__ e32, uint32_t* __restrict__ e32_2,
               uint16_t* __restrict__ e16, uint16_t* __restrict__ e16_2, GrpLut lut,
               unsigned long long* __restrict__ pool_next) {
    // trees [0, trees) from counts -> enc (and the encoder's u32 gather copy e32); a paired
    // build adds [trees, trees + trees2)
    const long long blocks1 = (trees + kGrpTrees - 1) / kGrpTrees;
    // lut.lut1 set: the decode tables too, each group right after its tree (unpaired builds);
    // its pool slot was zeroed before this launch, the other one is zeroed here for the next
    const bool fuse = lut.lut1 != nullptr;
    if (((long long)blockIdx.x == 0 || (long long)blockIdx.x == blocks1) && threadIdx.x == 0) {
        if (fuse) *pool_next = 0ull;
        else reset_pool_head((long long)blockIdx.x == 0 ? err : err2);
    }
    if ((long long)blockIdx.x >= blocks1) {
        const long long b = (long long)blockIdx.x - blocks1;
        counts = counts2 + b * kGrpTrees * k;
        enc = enc2 + b * kGrpTrees * k;
        e32 = e32_2 + b * kGrpTrees * k;
        e16 = e16_2 + b * kGrpTrees * k;
        err = err2;
        trees = trees2 - b * kGrpTrees;
    } else {
        trees -= (long long)blockIdx.x * kGrpTrees;
        counts += (long long)blockIdx.x * kGrpTrees * k;
        enc += (long long)blockIdx.x * kGrpTrees * k;
        e32 += (long long)blockIdx.x * kGrpTrees * k;
        e16 += (long long)blockIdx.x * kGrpTrees * k;
    }
    __shared__ __attribute__((aligned(16))) char lds[kGrpTrees * kGrpTreeBytes];
    const int lane = threadIdx.x, grp = lane >> 4, gl = lane & 15, gsh = grp * 16;
    char* base = lds + grp * kGrpTreeBytes;
    uint32_t* kid = reinterpret_cast<uint32_t*>(base + kGrpHeapBytes);
    unsigned long long* lkey = reinterpret_cast<unsigned long long*>(base + kGrpHeapBytes + kGrpKidBytes);
    {   // sentinels: every heap slot all ones (u32 and u64 views alike)
        uint4* z = reinterpret_cast<uint4*>(base);
        for (int q = gl; q < kGrpHeapBytes / 16; q += 16) z[q] = make_uint4(~0u, ~0u, ~0u, ~0u);
    }
    if (grp >= trees) return;   // no workgroup barriers below
    // latency-bound: issue ahead of the (older, VALU-bound) assignment waves on the SIMD
    pqh_set_prio(prio);
    const bool stamp = blockIdx.x == 0 && lane == 0;
    if (stamp) g_tree_stamps[0] = __builtin_amdgcn_s_memtime();
    const uint32_t* cnt = counts + (long long)grp * k;
    // nonzero counts in symbol order (huffman_encode.c:158): key count << 10 | symbol
    int nz = 0;
    unsigned long long total = 0;
    for (int s0 = 0; s0 < k; s0 += 16) {
        const int s = s0 + gl;
        const uint32_t c = s < k ? cnt[s] : 0u;
        const uint32_t mb = grp_bits(c != 0u, gsh);
        if (c) lkey[nz + __popc(mb & ((1u << gl) - 1u))] = ((unsigned long long)c << 10) | (unsigned)s;
        nz += __popc(mb);
        total += c;
    }
#pragma unroll
    for (int off = 8; off >= 1; off >>= 1) total += __shfl_xor(total, off, 16);
    const bool heavy = total >= (1ull << 22);   // (uniform in the group)
    if (stamp) g_tree_stamps[1] = __builtin_amdgcn_s_memtime();
    uint16_t* par = reinterpret_cast<uint16_t*>(lkey);   // (after the leaves are pushed)
    unsigned long long* code = reinterpret_cast<unsigned long long*>(base);   // (after the merges)
    int nint = 0;
    if (nz > 0 && !heavy) {
        // lane constants of the stretch: node gl's depth, its ancestors and the directions
        // towards it; lane 0 stands for no node (its node lies past the heap and its
        // direction bit, 0, never matches E)
        const int dq = gl ? 31 - __clz(gl) : 8;
        const int off = gl ? gl - (1 << dq) : 0;
        uint32_t A = gl ? 0u : 1u, E = gl ? 0u : 1u;
        for (int j = 1; j <= (gl ? dq : 0); ++j) {
            A |= 1u << (gl >> j);
            E |= (uint32_t)((gl >> (j - 1)) & 1) << (gl >> j);
        }
        uint32_t* h = reinterpret_cast<uint32_t*>(base);
        if (gl == 0) h[0] = 0u;   // position 0: the missing ancestor
        GrpHeap hp{h, 0, gl, gsh, dq, off, A, E};
        nint = grp_merge(hp, lkey, nz, kid, stamp);
    } else if (nz > 0) {
        if (gl == 0) nint = grp_merge_heavy(reinterpret_cast<unsigned long long*>(base), lkey, nz, kid);
        nint = __shfl(nint, 0, 16);
    }
    wave_sync_lds();
    if (stamp) g_tree_stamps[3] = __builtin_amdgcn_s_memtime();
    // codes (huffman_encode.c:100-132: child 0 appends bit 0, child 1 bit 1) by pointer
    // jumping over the parent links of node ids sym | 256 + q: code[v] = len << 56 | the bits
    // of the path from par[v] down to v; len saturates at 255 and any len > 56 is reported
    for (int v = gl; v < 512; v += 16) par[v] = 0xFFFFu;
    wave_sync_lds();
    const int root = 256 + nint - 1;
    for (int q = gl; q < nint; q += 16) {
        const uint32_t kk = kid[q];
        par[kk & 0xFFFFu] = (uint16_t)(256 + q);
        code[kk & 0xFFFFu] = 1ull << 56;
        if ((kk >> 16) != 0xFFFFu) {
            par[kk >> 16] = (uint16_t)(256 + q);
            code[kk >> 16] = (1ull << 56) | 1ull;
        }
    }
    wave_sync_lds();
    for (bool live = nint > 0; __any(live);) {
        live = false;
        for (int v = gl; v < 256 + nint; v += 16) {
            const int u = par[v];
            if (u == 0xFFFF || u == root) continue;   // absent leaf / the root's child (done)
            const unsigned long long ev = code[v], eu = code[u];
            const int pu = par[u];
            const unsigned lv = (unsigned)(ev >> 56), lu = (unsigned)(eu >> 56);
            const unsigned long long hi = lv < 56 ? ((eu & kCodeMask) << lv) : 0ull;
            const unsigned long long len = min((unsigned long long)(lv + lu), 255ull);
            code[v] = (len << 56) | ((hi | (ev & kCodeMask)) & kCodeMask);
            par[v] = (uint16_t)pu;
            live = true;
        }
        wave_sync_lds();
    }
    // (the group index made opaque, so the pointers below are formed here and not kept
    // live across the merges: the build stays within the VGPRs the assignment grid leaves)
    int grp2 = grp;
    asm volatile("" : "+v"(grp2));
    unsigned long long* out = enc + (long long)grp2 * k;
    uint32_t* out32 = e32 + (long long)grp2 * k;
    uint16_t* out16 = e16 + (long long)grp2 * k;
    bool too_long = false;
    for (int s = gl; s < k; s += 16) {
        unsigned long long e = 0;
        if (par[s] != 0xFFFFu) {
            e = code[s];
            if ((e >> 56) > (unsigned long long)kMaxCodeLen) {
                too_long = true;
                e = 0;
            }
        }
        out[s] = e;
        if (fuse) code[s] = e;   // (the LUT build's input: 0 for absent and refused codes)
        // the encoder's gather copy here too, so an encode may start before the decode
        // tables (lut_grp / lut_build then skip it)
        const unsigned len = (unsigned)(e >> 56);
        out32[s] = len <= 26 ? (uint32_t)((len << 26) | (uint32_t)(e & ((1ull << 26) - 1))) : ~0u;
        out16[s] = pqh_enc16_of(e);
    }
    if (too_long) atomicOr(err, 1u);
    if (stamp) {
        g_tree_stamps[4] = __builtin_amdgcn_s_memtime();
        g_tree_stamps[5] = (unsigned long long)nz;
        g_tree_stamps[6] = (unsigned long long)(nz + nint);
    }
    if (fuse) {
        // the codes of symbols 0..k-1 stay at base; the internal nodes' codes, kid and the
        // parent links after them are dead, so lut_grp's 3 KB scratch goes at base + 2 KB
        wave_sync_lds();
        // (lane values made opaque here, so nothing of the LUT build is computed before
        // the merges and held through them: the tree phase keeps its 32-VGPR budget)
        char* b2 = base;
        int ln2 = lane, gl2 = gl, gsh2 = gsh;
        asm volatile("" : "+v"(b2), "+v"(ln2), "+v"(gl2), "+v"(gsh2));
        grp_luts(lut, (long long)blockIdx.x * kGrpTrees + grp2, k, ln2, gl2, gsh2,
                 reinterpret_cast<const unsigned long long*>(b2), b2 + 2048);
    }
}

// The decode tables of lut_build for four alphabets per 64-thread workgroup (16 lanes each):
// the same tables from <= 32 VGPRs and 20 KB of LDS, so -- like huff_trees_grp -- it runs
// beside the assignment grid instead of waiting for its end (context mode, W1 <= 9).
__global__ void __launch_bounds__(64)
lut_grp(const unsigned long long* __restrict__ enc, int k, long long tables, GrpLut lut,
        unsigned long long* __restrict__ pool_next) {
    __shared__ __attribute__((aligned(16))) char lds[kGrpTrees * (2048 + 3072 + 16)];
    const int lane = threadIdx.x, grp = lane >> 4, gl = lane & 15, gsh = grp * 16;
    const long long t = (long long)blockIdx.x * kGrpTrees + grp;
    if (blockIdx.x == 0 && lane == 0) *pool_next = 0ull;   // (the next build's slot)
    if (t >= tables) return;   // no workgroup barriers below
    pqh_set_prio(lut.prio);
    char* base = lds + grp * (2048 + 3072 + 16);
    unsigned long long* code = reinterpret_cast<unsigned long long*>(base);
    const unsigned long long* e = enc + t * k;
#pragma unroll 1
    for (int s = gl; s < k; s += 16) code[s] = e[s];
    wave_sync_lds();
    grp_luts(lut, t, k, lane, gl, gsh, code, base + 2048);
}

// lut_build's tables for alphabet t from its k code entries `code` (LDS), by the tree's 16
// lanes; `scratch` = 3 KB of LDS (the L1 image u16 [2^w1 <= 512], the per-prefix widest
// remainder / subtable id u32 [512]) + a counter word after them.  Same entries as
// lut_build (whose comments give the format); only the pool ranges' placement may differ.
// shuffles within a lane's 16-lane group from an explicit lane id (so a caller can pass an
// opaque copy: the fused tree build must not compute these addresses before its merges)
__device__ __forceinline__ uint32_t g16_from(uint32_t v, int src_lane) {
    return (uint32_t)__builtin_amdgcn_ds_bpermute(src_lane << 2, (int)v);
}

__device__ __forceinline__ void grp_luts(const GrpLut& L, long long t, int k, int lane, int gl,
                                         int gsh, const unsigned long long* code, char* scratch) {
    const int w1 = L.w1, np = 1 << w1;                 // (w1 <= 9 here)
    uint16_t* img = reinterpret_cast<uint16_t*>(scratch);
    uint32_t* pre = reinterpret_cast<uint32_t*>(scratch + 1024);
    uint32_t* nlong = reinterpret_cast<uint32_t*>(scratch + 3072);
    for (int q = gl; q < 512 / 8; q += 16) reinterpret_cast<uint4*>(img)[q] = make_uint4(0, 0, 0, 0);
    for (int q = gl; q < 512 / 4; q += 16) reinterpret_cast<uint4*>(pre)[q] = make_uint4(0, 0, 0, 0);
    if (gl == 0) *nlong = 0;
    wave_sync_lds();
    // the widest remainder (capped at l2_bits) past W1 bits, per W1-bit prefix
#pragma unroll 1
    for (int s = gl; s < k; s += 16) {
        const unsigned long long v = code[s];
        const int len = (int)(v >> 56);
        if (len > w1)
            atomicMax(&pre[(unsigned)((v & kCodeMask) >> (len - w1))], (uint32_t)min(len - w1, L.l2_bits));
    }
    wave_sync_lds();
    // subtable ids in prefix order: lane gl's np / 16 prefixes, a group scan of their counts
    const int per = np / 16, p0 = gl * per;
    uint32_t c_id = 0, w2 = 0;
#pragma unroll 1
    for (int p = p0; p < p0 + per; ++p) {
        const uint32_t x = pre[p];
        c_id += x ? 1u : 0u;
        w2 = max(w2, x);
    }
    uint32_t incl = c_id;
#pragma unroll
    for (int off = 1; off < 16; off <<= 1) {
        const uint32_t y = g16_from(incl, gl >= off ? lane - off : lane);
        if (gl >= off) incl += y;
    }
#pragma unroll
    for (int off = 8; off >= 1; off >>= 1) w2 = max(w2, g16_from(w2, lane ^ off));
    const uint32_t nsub = g16_from(incl, lane | 15);
    uint32_t id = incl - c_id;
    // the pool range (sub ids must fit 12 bits; an alphabet without long codes takes none)
    unsigned long long l0 = 0;
    const bool ok = nsub < 4095;
    const unsigned long long size = ok ? (unsigned long long)nsub << w2 : 0ull;
    if (gl == 0 && size) l0 = atomicAdd(L.pool_head, size);
    l0 = ((unsigned long long)g16_from((uint32_t)(l0 >> 32), lane & ~15) << 32) |
         g16_from((uint32_t)l0, lane & ~15);
    const bool fits = ok && l0 + size <= (unsigned long long)L.lut2_cap;
    if (gl == 0)
        L.meta[t] = fits ? (uint32_t)((l0 << 9) | (w2 << 4) | (uint32_t)w1)
                         : (0x100u | (w2 << 4) | (uint32_t)w1);
    const bool subs = fits && w2 > 0;
    uint16_t* const sub0 = L.lut2 + (subs ? (long long)l0 : 0);   // this alphabet's subtables
    // (entries past the pool's end are dropped, as lut_build does)
    const int room = subs ? (int)min((long long)nsub << w2, L.lut2_cap - (long long)l0) : 0;
#pragma unroll 1
    for (int p = p0; p < p0 + per; ++p) {   // long prefixes: their L1 entry, their sub id
        if (pre[p]) {
            img[p] = (uint16_t)((15u << 12) | (subs ? id : 0xFFFu));
            pre[p] = id++;
        }
    }
    if (subs) {   // zero the subtables (the fill below is ordered after these stores)
#pragma clang loop unroll(disable) vectorize(disable) interleave(disable)
        for (int q = gl; q < room; q += 16) sub0[q] = 0;
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
    }
    wave_sync_lds();
    uint16_t* const L1 = L.lut1 + (t << L.w1);
#pragma unroll 1
    for (int s = gl; s < k; s += 16) {
        const unsigned long long v = code[s];
        const int len = (int)(v >> 56);
        if (L.enc32) {   // (null: the tree build wrote them)
            L.enc32[t * k + s] = len <= 26 ? (uint32_t)(((unsigned long long)len << 26) | (v & kCodeMask)) : ~0u;
            L.enc16[t * k + s] = pqh_enc16_of(v);
        }
        if (!len) continue;
        const unsigned long long cbits = v & kCodeMask;
        if (len <= w1) {   // replicated over the 2^(W1 - len) patterns that start with it
            const unsigned first = (unsigned)(cbits << (w1 - len));
            const uint16_t val = (uint16_t)((len << 12) | s);
#pragma clang loop unroll(disable) vectorize(disable) interleave(disable)
            for (unsigned j = 0; j < (1u << (w1 - len)); ++j) img[first + j] = val;
            continue;
        }
        const unsigned p = (unsigned)(cbits >> (len - w1));
        const int rem = len - w1;
        if (subs) {
            const int sb = (int)(pre[p] << w2);
            if (rem <= (int)w2) {
                const int b0 = sb + (int)((unsigned)(cbits & ((1ull << rem) - 1)) << (w2 - rem));
                const uint16_t val = (uint16_t)((rem << 12) | s);
#pragma clang loop unroll(disable) vectorize(disable) interleave(disable)
                for (int j = b0; j < b0 + (1 << (w2 - rem)) && j < room; ++j) sub0[j] = val;
                continue;
            }
            const int q = sb + (int)((cbits >> (rem - w2)) & ((1u << w2) - 1));
            if (q < room) sub0[q] = (uint16_t)(15u << 12);
        }
        const uint32_t idx = atomicAdd(nlong, 1u);
        L.longs[t * k + idx] = {cbits, (uint32_t)len, (uint32_t)s};
    }
    wave_sync_lds();
#pragma unroll 1
    for (int q = gl; q < np / 8; q += 16)   // the first level, 16 B per lane and store
        reinterpret_cast<uint4*>(L1)[q] = reinterpret_cast<const uint4*>(img)[q];
    if (gl == 0) L.long_cnt[t] = *nlong;
}

template <int KMAX, int TPW>
__global__ void __launch_bounds__(64)
huff_trees(const uint32_t* __restrict__ counts, int k, long long trees,
           unsigned long long* __restrict__ enc, uint32_t* __restrict__ err) {
    extern __shared__ __attribute__((aligned(16))) char lds[];
    // per tree: ncode u64 [2 KMAX] (the heap aliases it), kid u32 [KMAX], lcnt u32 [KMAX],
    // lsym u16 [KMAX]; all interleaved tree-minor
    unsigned long long* ncode_all = reinterpret_cast<unsigned long long*>(lds);
    uint32_t* kid_all = reinterpret_cast<uint32_t*>(ncode_all + 2 * KMAX * TPW);
    uint32_t* lcnt_all = kid_all + KMAX * TPW;
    uint16_t* lsym_all = reinterpret_cast<uint16_t*>(lcnt_all + KMAX * TPW);
    const int t = threadIdx.x;
    if (blockIdx.x == 0 && t == 0) reset_pool_head(err);
    if (KMAX <= 256) {   // the whole workgroup fills the sentinel-heap slots (ncode region)
        uint4* z = reinterpret_cast<uint4*>(ncode_all);
        for (int q = t; q < 2 * KMAX * TPW / 2; q += blockDim.x)
            z[q] = make_uint4(~0u, ~0u, ~0u, ~0u);
        __syncthreads();
    }
    if (t >= TPW) return;  // no barriers below
    const long long tree = (long long)blockIdx.x * TPW + t;
    if (tree >= trees) return;
    const uint32_t* cnt = counts + tree * k;
    unsigned long long* out = enc + tree * k;
    unsigned long long* ncode = ncode_all + t;
    const bool stamp = tree == 0;
    if (stamp) g_tree_stamps[0] = __builtin_amdgcn_s_memtime();
    uint32_t* kid = kid_all + t;
    uint16_t* lsym = lsym_all + t;

    // nonzero symbols in symbol order, with their counts
    uint32_t* lcnt = lcnt_all + t;
    unsigned long long total = 0;
    int nz = 0;
    scan_counts(cnt, k, [&](int s, uint32_t c) {
        lsym[nz * TPW] = (uint16_t)s;
        lcnt[nz * TPW] = c;
        total += c;
        ++nz;
    }, [&](int s) { out[s] = 0ull; });   // no code (the table set is not memset)
    if (nz == 0) return;
    if (stamp) g_tree_stamps[1] = __builtin_amdgcn_s_memtime();
    int next;
    if (KMAX <= 256 && total < (1ull << 22)) {
        // sentinel heap in the ncode region (1024 u32 slots per lane = 4 KB = ncode's 512 u64)
        SentinelHeap<TPW> hp{reinterpret_cast<uint32_t*>(ncode_all) + t, 0};   // pre-filled
        for (int j = 0; j < nz; ++j) hp.push((lcnt[j * TPW] << 10) | (uint32_t)j);
        if (stamp) g_tree_stamps[2] = __builtin_amdgcn_s_memtime();
        next = nz;
        if (hp.size == 1) {  // lone symbol: code "0" (huffman_encode.c:168-177)
            const uint32_t e = hp.pop();
            kid[0] = (e & 511u) | 0xFFFF0000u;
            hp.push((e & ~1023u) | (uint32_t)next);
            ++next;
        }
        while (hp.size > 1) {
            const uint32_t a = hp.pop();
            const uint32_t b = hp.pop();
            kid[(next - nz) * TPW] = (a & 511u) | ((b & 511u) << 16);
            hp.push(((a & ~1023u) + (b & ~1023u)) | (uint32_t)next);
            ++next;
        }
    } else if (KMAX <= 256 && total < (1ull << 23)) {
        next = merge_tree<uint32_t, 9, TPW, KMAX>(reinterpret_cast<uint32_t*>(ncode_all) + t,
                                                  lcnt, nz, kid);
    } else {
        next = merge_tree<unsigned long long, 16, TPW, KMAX>(ncode, lcnt, nz, kid);
    }

    if (stamp) g_tree_stamps[3] = __builtin_amdgcn_s_memtime();
    // codes top-down in reverse creation order (parents are created after their children):
    // ncode[q] = depth << 56 | code, child 0 appends bit 0 (huffman_encode.c:100-132)
    constexpr unsigned long long kMask = (1ull << 56) - 1;
    ncode[(next - 1) * TPW] = 0;   // root: the heap is dead, its storage is reused
    for (int q = next - 1; q >= nz; --q) {
        const unsigned long long e = ncode[q * TPW];
        const uint32_t kk = kid[(q - nz) * TPW];
        const unsigned long long d = min((e >> 56) + 1, 255ull);
        const unsigned long long c = (e & kMask) << 1;
        ncode[(kk & 0xFFFFu) * TPW] = (d << 56) | (c & kMask);
        if ((kk >> 16) != 0xFFFFu) ncode[(kk >> 16) * TPW] = (d << 56) | ((c | 1ull) & kMask);
    }
    bool too_long = false;
    for (int j = 0; j < nz; ++j) {
        const unsigned long long e = ncode[j * TPW];
        if ((e >> 56) > (unsigned long long)kMaxCodeLen) too_long = true;
        else out[lsym[j * TPW]] = e;
    }
    if (too_long) atomicOr(err, 1u);
    if (stamp) {
        g_tree_stamps[4] = __builtin_amdgcn_s_memtime();
        g_tree_stamps[5] = (unsigned long long)nz;
        g_tree_stamps[6] = (unsigned long long)next;
    }
}

// ---- one wavefront per large tree (K > 256), the heap in LDS, each sift read in parallel --
// The per-lane builds serialise every heap level on an LDS round trip (a K = 4,096 tree:
// ~3 ms of its 4,095 merges' pops).  Here the wave owns one tree and reads a whole stretch of
// a sift at once:
//   push  lane l reads ancestor l + 1 of the new slot (<= 12 levels: one round trip); the
//         ancestors the entry passes are exactly the lanes whose weight is strictly above
//         it (monotone along the path, so a ballot's popcount), and they move down one
//         level in one write;
//   pop   lane q (subtree position q = 1..63 below the current slot, 6 levels) reads its
//         node's two children (adjacent slots, one ds_read2) and picks the reference's
//         candidate (left unless the right is strictly lighter); a scalar chase down the
//         lanes' choices finds how far the last entry sinks, and the lanes on the path move
//         their candidates up in one write.
// Keys as SentinelHeap's, u64: weight << 16 | tie << 15 | node; slots past the heap hold all
// ones.  Same results as huff_trees / huff_trees_small (tie rules of huffman_encode.c:33-76).
struct ParHeap {
    using Key = unsigned long long;
    static constexpr Key kTie = 1ull << 15, kLow = (1ull << 16) - 1, kMaxKey = ~0ull;
    Key* h;     // slots [0, cap]; slot cap and every slot >= size hold kMaxKey
    int cap;
    int size;
    // pop's lane constants for subtree position q = lane: its ancestors in the stretch (bit p
    // for position p) and, among them, those whose path to q takes the right child
    unsigned long long anc = 0, dir = 0;
    __device__ __forceinline__ void init_masks(int lane) {
        const int q = lane;
        const int d = q ? 31 - __clz(q) : 0;
        for (int j = 0; j < d; ++j) {
            const int p = q >> (j + 1);
            anc |= 1ull << p;
            if ((q >> j) & 1) dir |= 1ull << p;
        }
    }
    __device__ __forceinline__ void push(Key e, int lane) {
        const int i = size++;
        const int anc = ((i + 1) >> (lane + 1)) - 1;   // lane l: ancestor l + 1 (-1: none)
        const bool va = lane < 16 && anc >= 0;
        const Key av = va ? h[anc] : 0ull;
        const bool mv = va && e < (av & ~kLow);       // strictly lighter than that ancestor
        const int s = __popcll(__ballot(mv));
        if (lane < s) h[((i + 1) >> lane) - 1] = av;   // ancestor l + 1 moves down to slot l
        if (lane == 0) h[((i + 1) >> s) - 1] = e;
    }
    __device__ __forceinline__ Key pop(int lane) {
        --size;
        // this lane's subtree position q = lane (1..63: six levels below the current slot)
        const int q = lane;
        const int d = q ? 31 - __clz(q) : 0;
        int i = 0;
        Key top = 0, last = 0, lw = 0;
        for (int round = 0;; ++round) {
            const int g = ((i + 1) << d) + (q - (1 << d)) - 1;
            const int c0 = 2 * g + 1;
            if (round == 0) {   // (the first stretch's reads go out with these two)
                top = h[0];
                last = h[size];
            }
            Key kl = kMaxKey, kr = kMaxKey;
            if (q >= 1 && c0 < cap) {
                kl = h[c0];
                kr = h[c0 + 1];
            }
            asm volatile("" : "+v"(kl), "+v"(kr), "+v"(top), "+v"(last));   // one wait for all
            if (round == 0) {
                lw = last & ~kLow;
                if (lane == 0) h[size] = kMaxKey;   // the vacated slot becomes a sentinel
            }
            if (c0 == size) kl = kMaxKey;           // (read before the sentinel landed)
            if (c0 + 1 == size) kr = kMaxKey;
            const Key kc = kl < (kr | kTie) ? kl : (kr | kTie);
            const bool mv = q >= 1 && kc < lw;
            // reached: every ancestor of q in the stretch moved toward q -- from two wave
            // ballots (who moves, who took the right child) and the lane's constant masks of
            // its ancestors (anc) and of the directions towards it (dir): no LDS round trip
            const unsigned long long M = __ballot(mv);
            const unsigned long long Rt = __ballot((kc & kTie) != 0);
            const bool reached = q >= 1 && (anc & (~M | (Rt ^ dir))) == 0ull;
            if (reached && mv) h[g] = kc & ~kTie;   // the candidates move up one level
            const unsigned long long stop = __ballot(reached && !mv);
            if (stop) {                              // `last` settles where the path ends
                if (reached && !mv) h[g] = last;
                break;
            }
            // the path left the stretch below its depth-5 position: continue there (at the
            // chosen child of the one reached depth-5 lane that moved)
            const unsigned long long deep = __ballot(reached && mv && q >= 32);
            const int qd = __ffsll((long long)deep) - 1;
            const int pq = 2 * qd + (int)((Rt >> qd) & 1ull);
            i = ((i + 1) << 6) + (pq - 64) - 1;
        }
        return top;
    }
};

template <int KMAX>
__global__ void __launch_bounds__(64)
huff_trees_par(const uint32_t* __restrict__ counts, int k, long long trees,
               unsigned long long* __restrict__ enc, uint32_t* __restrict__ err,
               const uint32_t* __restrict__ counts2, unsigned long long* __restrict__ enc2,
               uint32_t* __restrict__ err2) {
    // trees [0, trees) from counts -> enc; a paired build (pqh_tables_build_pair) continues
    // with the second table set's trees at workgroups trees, trees + 1, ...
    if ((long long)blockIdx.x >= trees) {
        counts = counts2 - trees * k;
        enc = enc2 - trees * k;
        err = err2;
    }
    if (((long long)blockIdx.x == 0 || (long long)blockIdx.x == trees) && threadIdx.x == 0)
        reset_pool_head(err);
    using Key = ParHeap::Key;
    // 104 KB at K = 4,096, so a build fits on a CU beside the K = 4,096 assignment grid's two
    // workgroups (~40 KB): the heap and the node codes share one region -- the heap lives
    // during the merges, the codes after them -- and the leaf counts are parked in it before
    // the pushes (leaf j's count sits at slot j, read before push j can write there)
    extern __shared__ __attribute__((aligned(16))) char lds[];
    Key* heap = reinterpret_cast<Key*>(lds);                              // [KMAX + 1] |
    unsigned long long* ncode = heap;                                    // [2 KMAX]
    uint32_t* kid = reinterpret_cast<uint32_t*>(ncode + 2 * KMAX);       // [KMAX]
    uint16_t* lsym = reinterpret_cast<uint16_t*>(kid + KMAX);            // [KMAX]
    uint16_t* par = lsym + KMAX;                                         // [2 KMAX]
    const int lane = threadIdx.x;
    const long long tree = blockIdx.x;   // (a paired build's grid covers both sets exactly)
    const uint32_t* cnt = counts + tree * k;
    unsigned long long* out = enc + tree * k;
    const bool stamp = tree == 0 && lane == 0;
    if (stamp) g_tree_stamps[0] = __builtin_amdgcn_s_memtime();
    // nonzero symbols in symbol order (their counts parked in ncode); no code for the rest
    int nz = 0;
    for (int s0 = 0; s0 < k; s0 += 64) {
        const int s = s0 + lane;
        const uint32_t c = s < k ? cnt[s] : 0u;
        const unsigned long long b = __ballot(c != 0u);
        if (c) {
            const int pos = nz + (int)__builtin_amdgcn_mbcnt_hi(
                                     (uint32_t)(b >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)b, 0u));
            lsym[pos] = (uint16_t)s;
            ncode[pos] = c;
        } else if (s < k) {
            out[s] = 0ull;
        }
        nz += __popcll(b);
    }
    if (nz == 0) return;
    ParHeap hp{heap, KMAX, 0};
    hp.init_masks(lane);
    constexpr Key kNode = ParHeap::kTie - 1;
    if (stamp) g_tree_stamps[1] = __builtin_amdgcn_s_memtime();
    for (int j = 0; j < nz; ++j) hp.push((ncode[j] << 16) | (Key)j, lane);
    // the slots past the heap become sentinels (they held the parked counts and older data)
    __builtin_amdgcn_wave_barrier();
    for (int q = nz + lane; q <= KMAX; q += 64) heap[q] = ParHeap::kMaxKey;
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    __builtin_amdgcn_wave_barrier();
    if (stamp) g_tree_stamps[2] = __builtin_amdgcn_s_memtime();
    int next = nz;
    if (hp.size == 1) {   // lone symbol: code "0" (huffman_encode.c:168-177)
        const Key e = hp.pop(lane);
        if (lane == 0) kid[0] = (uint32_t)(e & kNode) | 0xFFFF0000u;
        hp.push((e & ~ParHeap::kLow) | (Key)next, lane);
        ++next;
    }
    while (hp.size > 1) {
        const Key a = hp.pop(lane);
        const Key b = hp.pop(lane);
        if (lane == 0) kid[next - nz] = (uint32_t)(a & kNode) | ((uint32_t)(b & kNode) << 16);
        hp.push(((a & ~ParHeap::kLow) + (b & ~ParHeap::kLow)) | (Key)next, lane);
        ++next;
    }
    if (stamp) g_tree_stamps[3] = __builtin_amdgcn_s_memtime();
    // codes (huffman_encode.c:100-132: child 0 appends bit 0) by pointer jumping over the
    // parent links: e[v] = len << 56 | the path's bits from par[v] down to v (len saturates
    // at 255; any len > 56 is reported, so a truncated code never reaches a table)
    for (int q = nz + lane; q < next; q += 64) {
        const uint32_t kk = kid[q - nz];
        par[kk & 0xFFFFu] = (uint16_t)q;
        ncode[kk & 0xFFFFu] = 1ull << 56;
        if ((kk >> 16) != 0xFFFFu) {
            par[kk >> 16] = (uint16_t)q;
            ncode[kk >> 16] = (1ull << 56) | 1ull;
        }
    }
    if (lane == 0) {
        par[next - 1] = (uint16_t)(next - 1);   // the root: its own parent, empty path
        ncode[next - 1] = 0;
    }
    for (int span = 1; span < next; span <<= 1) {   // (in place: a node's link and path
        for (int v = lane; v < next; v += 64) {      //  are read before either is rewritten)
            const int u = par[v];
            const unsigned long long ev = ncode[v], eu = ncode[u];
            const int pu = par[u];
            const unsigned lv = (unsigned)(ev >> 56), lu = (unsigned)(eu >> 56);
            const unsigned long long hi = lv < 56 ? ((eu & kCodeMask) << lv) : 0ull;
            const unsigned long long len = min((unsigned long long)(lv + lu), 255ull);
            ncode[v] = (len << 56) | ((hi | (ev & kCodeMask)) & kCodeMask);
            par[v] = (uint16_t)pu;
        }
    }
    if (stamp) {
        g_tree_stamps[4] = __builtin_amdgcn_s_memtime();
        g_tree_stamps[5] = (unsigned long long)nz;
        g_tree_stamps[6] = (unsigned long long)next;
    }
    bool too_long = false;
    for (int j = lane; j < nz; j += 64) {
        const unsigned long long e = ncode[j];
        if ((e >> 56) > (unsigned long long)kMaxCodeLen) too_long = true;
        else out[lsym[j]] = e;
    }
    if (too_long) atomicOr(err, 1u);
}

// Two-level decode tables, one block per alphabet.
//   L1: 2^W1 u16 entries per alphabet, W1 fixed for the table set (9 in context mode, 11
//       otherwise) so a lookup never waits for per-alphabet metadata:
//       (len << 12) | sym for codes of len <= W1 (replicated), 15 << 12 | sub for the
//       prefix of longer codes, 0 for bit patterns no code starts with.
//   L2: per alphabet `nsub` subtables of one width w2 (the widest prefix needs, <= 8):
//       entry (rem << 12) | sym, or 15 << 12 for codes longer than W1 + w2 (long list).
//   meta[alphabet] = l2base << 9 | noL2 << 8 | w2 << 4 | W1   (l2base < 2^23)
// lut_build sizes every alphabet, takes its L2 range from the pool and writes the entries.

// per W1-prefix: widest remainder (capped at l2_bits) of the codes longer than W1
__device__ void block_w2max(const unsigned long long* e, int k, int w1, int l2_bits,
                            uint32_t* w2max /* LDS [1 << kL1Max] */) {
    for (int i = threadIdx.x; i < (1 << w1); i += blockDim.x) w2max[i] = 0;
    lds_barrier();
    for (int s = threadIdx.x; s < k; s += blockDim.x) {
        const unsigned long long v = e[s];
        const int len = (int)(v >> 56);
        if (len > w1) {
            const unsigned p = (unsigned)((v & kCodeMask) >> (len - w1));
            atomicMax(&w2max[p], (uint32_t)min(len - w1, l2_bits));
        }
    }
    lds_barrier();   // (the atomics' results are unused: an explicit LDS wait before the barrier)
}

// One workgroup per alphabet: size its second level, take the pool range with one atomic
// on the build's pool head (zeroed with the error word before the trees), write both levels.
// (Pool ranges are taken in completion order, so two builds may place an alphabet's
// subtables differently; the tables they describe are the same.  An alphabet whose range
// would pass the pool's end keeps only L1: its long codes go to the long list.)
__global__ void __launch_bounds__(256)
lut_build(const unsigned long long* __restrict__ enc, uint32_t* __restrict__ enc32,
          uint16_t* __restrict__ enc16, int k, int w1,
          int l2_bits, uint32_t* __restrict__ meta, uint16_t* __restrict__ lut1,
          uint16_t* __restrict__ lut2, long long lut2_cap, pqh_long_code* __restrict__ longs,
          uint32_t* __restrict__ long_cnt, unsigned long long* __restrict__ pool_head,
          unsigned long long* __restrict__ pool_next) {
    if (blockIdx.x == 0 && threadIdx.x == 0) *pool_next = 0ull;   // (the next build's slot)
    // w2max[2^W1], sub_id[2^W1]: dynamic LDS sized by the set's W1 (8 KB at the K = 256
    // W1 = 9 / 11, 64 KB only at K = 4096's W1 = 13), so a build beside the assignment grid
    // takes only what its alphabet needs
    extern __shared__ uint32_t lut_dyn[];
    uint32_t* const w2max = lut_dyn;
    uint32_t* const sub_id = lut_dyn + (1 << w1);
    __shared__ uint32_t nlong, nsub, w2s;
    __shared__ unsigned long long base_s;
    __shared__ uint32_t part[256];
    const long long t = blockIdx.x;
    const unsigned long long* e = enc + t * k;
    uint16_t* L1 = lut1 + (t << w1);
    block_w2max(e, k, w1, l2_bits, w2max);
    // subtable ids in prefix order: per-thread chunk counts, then a block-wide exclusive
    // scan (wave scans + the four wave totals; 256 threads)
    const int np = 1 << w1;
    const int per = (np + blockDim.x - 1) / blockDim.x;
    const int p0 = threadIdx.x * per, p1 = min(np, p0 + per);
    uint32_t c_id = 0;
    for (int p = p0; p < p1; ++p) c_id += w2max[p] ? 1u : 0u;
    {
        const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
        uint32_t incl = c_id;
        for (int off = 1; off < 64; off <<= 1) {
            const uint32_t y = __shfl_up(incl, off);
            if (lane >= off) incl += y;
        }
        if (lane == 63) part[wid] = incl;
        __syncthreads();
        uint32_t before = 0, all = 0;
        for (int w = 0; w < (int)blockDim.x / 64; ++w) {
            const uint32_t x = part[w];
            before += w < wid ? x : 0u;
            all += x;
        }
        if (threadIdx.x == 0) {
            nsub = all;
            nlong = 0;
        }
        c_id = before + incl - c_id;
    }
    {   // the widest remainder over the prefixes: the subtables' width
        uint32_t w = 0;
        for (int p = p0; p < p1; ++p) w = max(w, w2max[p]);
        for (int off = 32; off >= 1; off >>= 1) w = max(w, (uint32_t)__shfl_xor(w, off));
        __syncthreads();   // (part[] was read above)
        if ((threadIdx.x & 63) == 0) part[threadIdx.x >> 6] = w;
        __syncthreads();
        if (threadIdx.x == 0) {
            uint32_t w2 = 0;
            for (int q = 0; q < (int)blockDim.x / 64; ++q) w2 = max(w2, part[q]);
            w2s = w2;
            // sub ids must fit 12 bits; an alphabet without long codes takes no range
            const bool ok = nsub < 4095;
            const unsigned long long size = ok ? (unsigned long long)nsub << w2 : 0ull;
            const unsigned long long l0 = size ? atomicAdd(pool_head, size) : 0ull;
            const bool fits = ok && l0 + size <= (unsigned long long)lut2_cap;
            base_s = fits ? l0 : ~0ull;
            meta[t] = fits ? (uint32_t)((l0 << 9) | (w2 << 4) | (uint32_t)w1)
                           : (0x100u | (w2 << 4) | (uint32_t)w1);
        }
    }
    __syncthreads();
    const int w2 = (int)w2s;
    const bool subs = base_s != ~0ull && w2 > 0;
    const long long l2base = subs ? (long long)base_s : 0;
    for (int p = p0; p < p1; ++p)
        if (w2max[p]) sub_id[p] = c_id++;
    for (int i = threadIdx.x; i < np; i += blockDim.x) L1[i] = 0;
    __syncthreads();
    if (subs) {   // zero this alphabet's subtables
        const long long entries = (long long)nsub << w2;
        for (long long q = threadIdx.x; q < entries; q += blockDim.x)
            if (l2base + q < lut2_cap) lut2[l2base + q] = 0;
    }
    __syncthreads();
    for (int s = threadIdx.x; s < k; s += blockDim.x) {
        const unsigned long long v = e[s];
        const int len = (int)(v >> 56);
        if (enc32) {   // (null: the tree build wrote them)
            enc32[t * k + s] = len <= 26 ? (uint32_t)(((unsigned long long)len << 26) | (v & kCodeMask))
                                         : ~0u;
            enc16[t * k + s] = pqh_enc16_of(v);
        }
        if (!len) continue;
        const unsigned long long code = v & kCodeMask;
        if (len <= w1) {
            const unsigned first = (unsigned)(code << (w1 - len));
            const uint16_t val = (uint16_t)((len << 12) | s);
            for (unsigned j = 0; j < (1u << (w1 - len)); ++j) L1[first + j] = val;
            continue;
        }
        const unsigned p = (unsigned)(code >> (len - w1));
        const int rem = len - w1;
        if (subs) {
            L1[p] = (uint16_t)((15u << 12) | sub_id[p]);
            const long long sb = l2base + ((long long)sub_id[p] << w2);
            if (rem <= w2) {
                const unsigned rest = (unsigned)(code & ((1ull << rem) - 1));
                const long long base = sb + ((long long)rest << (w2 - rem));
                const uint16_t val = (uint16_t)((rem << 12) | s);
                for (unsigned j = 0; j < (1u << (w2 - rem)); ++j)
                    if (base + j < lut2_cap) lut2[base + j] = val;
                continue;
            }
            const unsigned rest = (unsigned)((code >> (rem - w2)) & ((1u << w2) - 1));
            if (sb + rest < lut2_cap) lut2[sb + rest] = (uint16_t)(15u << 12);
        } else {
            L1[p] = (uint16_t)((15u << 12) | 0xFFFu);
        }
        const uint32_t idx = atomicAdd(&nlong, 1u);
        longs[t * k + idx] = {code, (uint32_t)len, (uint32_t)s};
    }
    lds_barrier();
    if (threadIdx.x == 0) long_cnt[t] = nlong;
}

// ------------------------------------------------------------------- decoding
// Bit reader over a word array: a 64-bit MSB-first buffer refilled one 32-bit word at a
// time, branch-free (the next word is always read; the array is readable up to `lim`).
// WIN = the words are this workgroup's LDS window (the compiler then emits ds_read).
struct BitReader {
    const uint32_t* words;
    long long lim;             // last readable index
    long long next;            // next word to load
    unsigned long long buf;
    int have;
    __device__ __forceinline__ uint32_t load(long long i) const {
        return __builtin_bswap32(words[min(i, lim)]);
    }
    __device__ __forceinline__ void init(const uint32_t* w, long long l, unsigned long long p) {
        words = w;
        lim = l;
        const long long wi = (long long)(p >> 5);
        const int o = (int)(p & 31);
        buf = (((unsigned long long)load(wi) << 32) | load(wi + 1)) << o;
        have = 64 - o;
        next = wi + 2;
    }
    __device__ __forceinline__ unsigned long long pos() const {
        return (unsigned long long)next * 32 - (unsigned long long)have;
    }
    __device__ __forceinline__ void skip(int nb) {   // nb <= 32
        const uint32_t w = load(next);
        buf <<= nb;
        have -= nb;
        const bool need = have <= 32;
        buf |= need ? ((unsigned long long)w << (32 - have)) : 0ull;
        next += need ? 1 : 0;
        have += need ? 32 : 0;
    }
    __device__ __forceinline__ void skip_long(int nb) {   // nb may exceed 32
        while (nb > 0) {
            const int step = nb < 32 ? nb : 32;
            skip(step);
            nb -= step;
        }
    }
    __device__ __forceinline__ uint32_t peek(int nb) const { return (uint32_t)(buf >> (64 - nb)); }
    __device__ unsigned long long peek_long(int nb) const {  // nb <= 56
        const unsigned long long p = pos();
        const long long wi = (long long)(p >> 5);
        const int o = (int)(p & 31);
        const unsigned long long hi = ((unsigned long long)load(wi) << 32) | load(wi + 1);
        const unsigned long long lo = load(wi + 2);
        const unsigned long long w64 = o ? ((hi << o) | (lo >> (32 - o))) : hi;
        return w64 >> (64 - nb);
    }
};

// Decoder tables as seen by one workgroup.
struct DecTables {
    const uint32_t* meta;      // LDS copy
    const uint16_t* lut1;      // LDS copy (non-context) or global
    const uint16_t* lut2;
    long long lut2_cap;
    const pqh_long_code* longs;
    const uint32_t* long_cnt;
    int k;
    int w1;                    // fixed first-level width of the table set
};

// one symbol of alphabet `tab` (huffman_decode.c:137-191 as table lookups); false = invalid.
// The L1 lookup depends only on (tab, next W1 bits); the metadata read runs beside it and
// is needed only for the second level.
__device__ __forceinline__ bool dec_symbol(BitReader& br, const DecTables& T, long long tab,
                                           unsigned& sym) {
    const int w1 = T.w1;
    const uint16_t e = T.lut1[(tab << w1) + br.peek(w1)];
    const uint32_t mt = T.meta[tab];
    const int len = e >> 12;
    sym = e & 0xFFFu;
    if (len >= 1 && len <= w1) {
        br.skip(len);
        return sym < (unsigned)T.k;
    }
    if (len != 15) return false;
    bool slow = true;
    if (sym != 0xFFFu) {
        const int w2 = (int)((mt >> 4) & 15u);
        const long long li = (long long)(mt >> 9) + ((long long)sym << w2) +
                             (br.peek(w1 + w2) & ((1u << w2) - 1u));
        if (w2 < 1 || (mt & 0x100u) || li >= T.lut2_cap) return false;
        const uint16_t e2 = T.lut2[li];
        const int len2 = e2 >> 12;
        if (len2 >= 1 && len2 <= w2) {
            sym = e2 & 0xFFFu;
            br.skip(w1 + len2);
            slow = false;
        } else if (len2 != 15) {
            return false;
        }
    }
    if (slow) {   // codes beyond both levels: rare, linear search
        const uint32_t cnt = T.long_cnt[tab];
        bool found = false;
        for (uint32_t q = 0; q < cnt; ++q) {
            const pqh_long_code lc = T.longs[tab * T.k + q];
            if (br.peek_long((int)lc.len) == lc.code) {
                sym = lc.sym;
                br.skip_long((int)lc.len);
                found = true;
                break;
            }
        }
        if (!found) return false;
    }
    return sym < (unsigned)T.k;   // never false for a well-formed table
}

// Per-lane decode of [v0, v1) in batches of S vectors staged in LDS; every lane of the
// workgroup runs the batch loop (barriers).  `src` is the LDS window or the global stream.
template <int MT, typename CodeT>
__device__ __forceinline__ void decode_lanes(const uint32_t* src, long long src_lim,
                                             unsigned long long start, bool live, long long j,
                                             long long j0, long long jn, long long n, int m,
                                             int k, int context, int raw_first,
                                             int chunk_vectors, int S,
                                             const CodeT* __restrict__ chunk_prev,
                                             const DecTables& T, CodeT* stage,
                                             CodeT* __restrict__ out, bool& ok) {
    const int lane = threadIdx.x;
    const long long v0 = j * chunk_vectors;
    const long long v1 = min(n, v0 + chunk_vectors);
    BitReader br;
    br.init(src, src_lim, live ? start : 0);
    unsigned prev[MT ? MT : 16];
    bool warm = context && j == 0 && raw_first && live;
#pragma unroll
    for (int i = 0; i < (MT ? MT : 16); ++i)
        prev[i] = (live && i < m && context && !warm) ? (unsigned)chunk_prev[j * m + i] : 0u;
    const int roots = context ? k : 1;
    const long long run = (long long)S * m;   // staged codes per lane per batch

    for (int s0 = 0; s0 < chunk_vectors; s0 += S) {
        long long va = v0 + s0;
        const long long vb = live ? min(v1, va + S) : va;
        if (warm && va < vb) {   // global row 0 of a context stream: ceil(log2 K) raw bits
            int warm_bits = 1;   // per part (huffman_decode.c:73-76; the encoder writes 8)
            while ((1 << warm_bits) < k) ++warm_bits;
            for (int i = 0; i < m; ++i) {
                prev[i] = br.peek(warm_bits);
                br.skip(warm_bits);
            }
            CodeT* o = stage + lane * run;
            for (int i = 0; i < m; ++i) o[i] = (CodeT)prev[i];
            ++va;
            warm = false;
        }
        for (long long v = va; v < vb && ok; ++v) {
#pragma unroll
            for (int i = 0; i < (MT ? MT : 16); ++i) {
                if (!MT && i >= m) break;
                const long long tab = (long long)i * roots + (context ? prev[i] : 0u);
                unsigned sym;
                if (!dec_symbol(br, T, tab, sym)) {
                    ok = false;
                    break;
                }
                prev[i] = sym;
            }
            CodeT* o = stage + lane * run + (v - v0 - s0) * m;
            if constexpr (sizeof(CodeT) == 1 && MT % 4 == 0 && MT > 0) {
#pragma unroll
                for (int q = 0; q < MT / 4; ++q)
                    reinterpret_cast<uint32_t*>(o)[q] = prev[4 * q] | (prev[4 * q + 1] << 8) |
                                                        (prev[4 * q + 2] << 16) | (prev[4 * q + 3] << 24);
            } else {
#pragma unroll
                for (int i = 0; i < (MT ? MT : 16); ++i)
                    if (MT || i < m) o[i] = (CodeT)prev[i];
            }
        }
        __syncthreads();
        // write back: lane-run r holds rows (j0 + r) * C + s0 ... of at most S rows
        if (S == chunk_vectors && (run * (long long)sizeof(CodeT)) % 4 == 0) {
            // runs are contiguous: one linear copy of the workgroup's rows
            const long long rows = min(n, (j0 + 64) * chunk_vectors) - j0 * chunk_vectors;
            const long long nbytes = rows * m * (long long)sizeof(CodeT);
            char* dst = reinterpret_cast<char*>(out + j0 * chunk_vectors * m);
            const long long n4 = nbytes / 4;
            for (long long q = lane; q < n4; q += 64)
                __builtin_nontemporal_store(reinterpret_cast<const uint32_t*>(stage)[q],
                                            reinterpret_cast<uint32_t*>(dst) + q);
            for (long long q = n4 * 4 + lane; q < nbytes; q += 64)
                dst[q] = reinterpret_cast<const char*>(stage)[q];
        } else {
            for (long long q = lane; q < 64 * run; q += 64) {
                const long long r = q / run, w = q % run;
                const long long row = (j0 + r) * chunk_vectors + s0 + w / m;
                if (r < jn && s0 + w / m < chunk_vectors && row < n) out[row * m + w % m] = stage[q];
            }
        }
        __syncthreads();
    }
}

// One lane per chunk of C vectors (huffman_decoder.c:211-255).  The workgroup's 64 chunks
// are contiguous in the stream, so their bits are first copied into an LDS window with
// coalesced non-temporal loads (global fallback when the window is too small); decoded
// codes are staged in LDS and written back coalesced, S vectors per lane at a time.  The
// only global loads in the symbol loop are then the table lookups, and no store sits in
// front of them in the vmcnt queue.  MT = parts at compile time (0 = runtime m <= 16).
template <int MT, typename CodeT, bool L1_IN_LDS>
__global__ void __launch_bounds__(64)
dec_chunks(const uint32_t* __restrict__ words, long long nwords, long long n, int m_rt, int k,
           int context, int raw_first, int chunk_vectors,
           const unsigned long long* __restrict__ chunk_off, const CodeT* __restrict__ chunk_prev,
           const uint16_t* __restrict__ lut1_g, const uint16_t* __restrict__ lut2,
           const uint32_t* __restrict__ meta_g, int w1, long long tables, long long lut2_cap,
           const pqh_long_code* __restrict__ longs,
           const uint32_t* __restrict__ long_cnt, CodeT* __restrict__ out,
           unsigned long long* __restrict__ err, int win_words, int S) {
    extern __shared__ __attribute__((aligned(16))) char lds[];
    const int m = MT ? MT : m_rt;
    const long long meta_b = (tables * 4 + 15) & ~15ll;
    const long long l1_b = L1_IN_LDS ? (((tables << w1) * 2 + 15) & ~15ll) : 0;
    uint32_t* meta = reinterpret_cast<uint32_t*>(lds);
    uint16_t* l1s = reinterpret_cast<uint16_t*>(lds + meta_b);
    uint32_t* win = reinterpret_cast<uint32_t*>(lds + meta_b + l1_b);
    CodeT* stage = reinterpret_cast<CodeT*>(lds + meta_b + l1_b + ((long long)win_words + 4) * 4);
    const int lane = threadIdx.x;
    const bool stamp = blockIdx.x == 0 && lane == 0;
#ifdef PQH_LAT_PRIO   // (experiment) latency-bound waves first in issue arbitration
    __builtin_amdgcn_s_setprio(PQH_LAT_PRIO);
#endif
    if (stamp) g_tree_stamps[8] = __builtin_amdgcn_s_memtime();
    for (long long t = lane; t < tables; t += 64) meta[t] = meta_g[t];
    if constexpr (L1_IN_LDS) {
        const long long n16 = ((tables << w1) * 2 + 15) / 16;
        const uint4* src = reinterpret_cast<const uint4*>(lut1_g);
        uint4* dst = reinterpret_cast<uint4*>(l1s);
        for (long long i = lane; i < n16; i += 64) dst[i] = src[i];
    }
    const long long chunks = (n + chunk_vectors - 1) / chunk_vectors;
    const long long j0 = (long long)blockIdx.x * 64;
    const long long jn = min(chunks - j0, 64ll);
    if (stamp) g_tree_stamps[9] = __builtin_amdgcn_s_memtime();
    // stream window of this workgroup's chunks
    const unsigned long long b_lo = chunk_off[j0];
    const unsigned long long b_hi = j0 + 64 < chunks ? chunk_off[j0 + 64] : (unsigned long long)nwords * 32;
    const long long w_lo = (long long)(b_lo >> 5);
    const long long w_hi = min(nwords, (long long)((b_hi + 31) >> 5) + 2);
    const bool in_lds = w_hi - w_lo <= win_words;
    if (in_lds) {   // streamed once: non-temporal, so the code tables keep the L2
        const long long nw = w_hi - w_lo;
        for (long long w0 = 0; w0 < nw; w0 += 8 * 64) {   // 8 loads in flight per lane
            uint32_t r[8];
#pragma unroll
            for (int u = 0; u < 8; ++u) {
                const long long w = w0 + u * 64 + lane;
                r[u] = w < nw ? __builtin_nontemporal_load(words + w_lo + w) : 0u;
            }
#pragma unroll
            for (int u = 0; u < 8; ++u) {
                const long long w = w0 + u * 64 + lane;
                if (w < nw) win[w] = r[u];
            }
        }
        if (lane < 4) win[nw + lane] = 0;   // zero pad read past the window
    }
    __syncthreads();

    if (stamp) {
        g_tree_stamps[10] = __builtin_amdgcn_s_memtime();
        g_tree_stamps[13] = in_lds;
    }
    DecTables T{meta, L1_IN_LDS ? l1s : lut1_g, lut2, lut2_cap, longs, long_cnt, k, w1};
    const long long j = j0 + lane;
    const bool live = lane < jn;
    bool ok = true;
    const unsigned long long start = live ? chunk_off[j] : 0;
    if (in_lds)
        decode_lanes<MT, CodeT>(win, w_hi - w_lo + 3, live ? start - (unsigned long long)w_lo * 32 : 0,
                                live, j, j0, jn, n, m, k, context, raw_first, chunk_vectors, S,
                                chunk_prev, T, stage, out, ok);
    else
        decode_lanes<MT, CodeT>(words, nwords - 1, start, live, j, j0, jn, n, m, k, context,
                                raw_first, chunk_vectors, S, chunk_prev, T, stage, out, ok);
    if (stamp) g_tree_stamps[11] = __builtin_amdgcn_s_memtime();
    if (!ok) atomicOr(err, 1ull);
}

// ---- slim decoder for 8-part u8 rows (the bench shape): <= 32 VGPRs, so, like the table
// builds, it runs beside the assignment grid.  One lane per chunk of C <= 32 vectors, 64
// chunks per workgroup; the chunks' stream window in LDS (or, if it does not fit, the
// global stream at 32-bit offsets from the window's first word); a row is decoded into one
// u64, staged in LDS and written back as whole rows; the context row is that u64.  Table
// lookups as dec_symbol (first level, second level, long list).
template <bool LDS>
struct BitRd {   // MSB-first reader over words [0, lim] (32-bit indices)
    const uint32_t* w;
    uint32_t lim;
    uint32_t next;
    unsigned long long buf;
    int have;
    __device__ __forceinline__ uint32_t load(uint32_t i) const { return __builtin_bswap32(w[min(i, lim)]); }
    __device__ __forceinline__ void init(unsigned long long p) {
        const uint32_t wi = (uint32_t)(p >> 5);
        const int o = (int)(p & 31);
        buf = (((unsigned long long)load(wi) << 32) | load(wi + 1)) << o;
        have = 64 - o;
        next = wi + 2;
    }
    __device__ __forceinline__ uint32_t peek(int nb) const { return (uint32_t)(buf >> (64 - nb)); }
    __device__ __forceinline__ void skip(int nb) {   // nb <= 32
        const uint32_t x = load(next);
        buf <<= nb;
        have -= nb;
        const bool need = have <= 32;
        buf |= need ? ((unsigned long long)x << (32 - have)) : 0ull;
        next += need ? 1u : 0u;
        have += need ? 32 : 0;
    }
    __device__ __forceinline__ unsigned long long peek56() const {   // the next 56 bits
        const unsigned long long p = (unsigned long long)next * 32 - (unsigned long long)have;
        const uint32_t wi = (uint32_t)(p >> 5);
        const int o = (int)(p & 31);
        const unsigned long long hi = ((unsigned long long)load(wi) << 32) | load(wi + 1);
        const unsigned long long lo = load(wi + 2);
        return (o ? ((hi << o) | (lo >> (32 - o))) : hi) >> 8;
    }
};

// The LDS window's reader: the window holds the stream words already byte-swapped (MSB-first
// as integers, done once when they are staged), and the reader keeps only the bit position, so
// a peek is one two-word LDS read and a funnel shift and a skip one add (the 64-bit buffer of
// BitRd costs ~17 VALU per skip: the refill's shifts and selects).  Words past `lim` read as
// the last one (the window's zero pad).
struct PosRd {
    const uint32_t* w;
    uint32_t lim;
    uint32_t pos;
    __device__ __forceinline__ uint32_t word(uint32_t i) const { return w[min(i, lim)]; }
    __device__ __forceinline__ void init(unsigned long long p) { pos = (uint32_t)p; }
    __device__ __forceinline__ uint32_t peek(int nb) const {   // 1 <= nb <= 32
        // words i and i + 1 in one ds_read2 (i clamped so both are in [0, lim]: past the
        // window's data both are its zero pad), then one 64-bit shift
        const uint32_t i = min(pos >> 5, lim - 1);
        const unsigned long long ab = ((unsigned long long)w[i] << 32) | w[i + 1];
        return (uint32_t)((ab << (pos & 31u)) >> 32) >> (32 - nb);
    }
    __device__ __forceinline__ void skip(int nb) { pos += (uint32_t)nb; }
    __device__ __forceinline__ unsigned long long peek56() const {   // the next 56 bits
        const uint32_t i = pos >> 5;
        const int o = (int)(pos & 31u);
        const unsigned long long hi = ((unsigned long long)word(i) << 32) | word(i + 1);
        const unsigned long long lo = word(i + 2);
        return (o ? ((hi << o) | (lo >> (32 - o))) : hi) >> 8;
    }
};

// codes beyond both table levels: linear search of the alphabet's long list against the
// next 56 stream bits; returns len << 16 | sym, or 0 if none matches (inlined: a call would
// cost the kernel its register budget)
__device__ __forceinline__ uint32_t dec_long(const pqh_long_code* __restrict__ longs, uint32_t cnt,
                                          unsigned long long bits56) {
    for (uint32_t q = 0; q < cnt; ++q) {
        const pqh_long_code lc = longs[q];
        if (lc.len >= 1 && lc.len <= 56 && (bits56 >> (56 - lc.len)) == lc.code)
            return (lc.len << 16) | lc.sym;
    }
    return 0;
}

struct Row8Tabs {
    const uint16_t* lut1;
    const uint16_t* lut2;
    const uint32_t* meta;
    const pqh_long_code* longs;
    const uint32_t* long_cnt;
    long long lut2_cap;
    int w1, k;
    int prio;   // wave issue priority (pqh_prio)
};

// one symbol of alphabet tab, or -1 (invalid)
#ifndef PQH_DEC_SYM_OLD
// A wave decodes 64 chains in lock step, so a branch taken by any lane costs every lane: with
// W1 = 9 about 3 % of a SIFT batch's symbols are longer than the first level, so 87 % of the
// wave's symbol steps run the second level.  This form keeps that path short: the alphabet's
// meta word is loaded with the first-level entry (8 KB per table set: cache-resident), so the
// second level is one dependent load, and every path but the long list ends in the same
// single skip.  Same results as the round-5 form (PQH_DEC_SYM_OLD).
template <typename Rd>
__device__ __forceinline__ int dec_sym8(Rd& br, const Row8Tabs& T, unsigned tab) {
    const int w1 = T.w1;
    const uint32_t mt = T.meta[tab];
    const uint32_t p32 = br.peek(32);   // (>= 33 bits are buffered; W1 + w2 <= 25)
    const uint16_t e = T.lut1[(tab << w1) + (p32 >> (32 - w1))];
    // (both loads complete here: without this the compiler sinks the meta load into the
    // second-level branch, behind the first-level load's result)
    asm volatile("" ::"v"(mt), "v"(e));
    const int len = e >> 12;
    unsigned sym = e & 0xFFFu;
    int adv = -1;   // bits to skip; 0: the long list; -1: invalid
    if (len >= 1 && len <= w1) {
        adv = len;
    } else if (len == 15) {
        adv = 0;
        if (sym != 0xFFFu) {   // second level
            const int w2 = (int)((mt >> 4) & 15u);
            const long long li = (long long)(mt >> 9) + ((long long)sym << w2) +
                                 ((p32 >> (32 - w1 - w2)) & ((1u << w2) - 1u));
            adv = -1;
            if (w2 >= 1 && !(mt & 0x100u) && li < T.lut2_cap) {
                const uint16_t e2 = T.lut2[li];
                const int len2 = e2 >> 12;
                if (len2 >= 1 && len2 <= w2) {
                    adv = w1 + len2;
                    sym = e2 & 0xFFFu;
                } else if (len2 == 15) {
                    adv = 0;
                }
            }
        }
    }
    if (adv == 0) {   // codes beyond both levels: the alphabet's long list
        const uint32_t f = dec_long(T.longs + (long long)tab * T.k, T.long_cnt[tab], br.peek56());
        if (!f) return -1;
        for (int nb = (int)(f >> 16); nb > 0; nb -= 32) br.skip(nb < 32 ? nb : 32);
        sym = f & 0xFFFFu;
        return sym < (unsigned)T.k ? (int)sym : -1;
    }
    if (adv < 0) return -1;
    br.skip(adv);
    return sym < (unsigned)T.k ? (int)sym : -1;
}
#else
template <typename Rd>
__device__ __forceinline__ int dec_sym8(Rd& br, const Row8Tabs& T, unsigned tab) {
    const int w1 = T.w1;
    const uint16_t e = T.lut1[(tab << w1) + br.peek(w1)];
    const int len = e >> 12;
    unsigned sym = e & 0xFFFu;
    if (len >= 1 && len <= w1) {
        br.skip(len);
        return sym < (unsigned)T.k ? (int)sym : -1;
    }
    if (len != 15) return -1;
    if (sym != 0xFFFu) {   // second level
        const uint32_t mt = T.meta[tab];
        const int w2 = (int)((mt >> 4) & 15u);
        const long long li = (long long)(mt >> 9) + ((long long)sym << w2) +
                             (br.peek(w1 + w2) & ((1u << w2) - 1u));
        if (w2 < 1 || (mt & 0x100u) || li >= T.lut2_cap) return -1;
        const uint16_t e2 = T.lut2[li];
        const int len2 = e2 >> 12;
        if (len2 >= 1 && len2 <= w2) {
            br.skip(w1 + len2);
            sym = e2 & 0xFFFu;
            return sym < (unsigned)T.k ? (int)sym : -1;
        }
        if (len2 != 15) return -1;
    }
    const uint32_t f = dec_long(T.longs + (long long)tab * T.k, T.long_cnt[tab], br.peek56());
    if (!f) return -1;
    for (int nb = (int)(f >> 16); nb > 0; nb -= 32) br.skip(nb < 32 ? nb : 32);
    sym = f & 0xFFFFu;
    return sym < (unsigned)T.k ? (int)sym : -1;
}

#endif

// One lane's chunk: rows of NW u64 words, SB-bit symbols packed little-end first (SB = 8:
// u8 codes, 8 NW parts; SB = 16: u16 codes, 4 NW parts), so a row is decoded into NW
// registers, staged in LDS and stored whole; the context row is those registers.
template <bool CTX, bool LDS, int NW, int SB>
__device__ __forceinline__ bool dec_row_lane(const uint32_t* src, uint32_t lim,
                                             unsigned long long start, long long j, long long n,
                                             int chunk_vectors, int raw_first,
                                             const unsigned long long* __restrict__ chunk_prev,
                                             const Row8Tabs& T, unsigned long long* st) {
    constexpr int PW = 64 / SB;   // parts per word
    constexpr unsigned SMASK = (1u << SB) - 1u;
    // (LDS: the window's words are byte-swapped when staged; global: BitRd swaps per load)
    using Rd = typename std::conditional<LDS, PosRd, BitRd<false>>::type;
    Rd br{};
    br.w = src;
    br.lim = lim;
    br.init(start);
    const long long v0 = j * chunk_vectors;
    const int cnt = (int)min((long long)chunk_vectors, n - v0);
    unsigned long long prev[NW];
#pragma unroll
    for (int w = 0; w < NW; ++w) prev[w] = 0;
    int s = 0;
    if (CTX) {
        if (j == 0 && raw_first) {   // global row 0: ceil(log2 K) raw bits per part
            int wb = 1;              // (huffman_decode.c:73-76; the encoder writes 8)
            while ((1 << wb) < T.k) ++wb;
#pragma unroll
            for (int w = 0; w < NW; ++w) {
#pragma unroll 1
                for (int i = 0; i < PW; ++i) {
                    prev[w] |= (unsigned long long)br.peek(wb) << (SB * i);
                    br.skip(wb);
                }
                st[w] = prev[w];
            }
            s = 1;
        } else {
#pragma unroll
            for (int w = 0; w < NW; ++w) prev[w] = chunk_prev[j * NW + w];
        }
    }
    const unsigned roots = CTX ? (unsigned)T.k : 1u;
    for (; s < cnt; ++s) {
#pragma unroll
        for (int w = 0; w < NW; ++w) {
            unsigned long long row = 0;
#pragma unroll 1
            for (int i = 0; i < PW; ++i) {   // (rolled: one copy of the lookup code, fewer registers)
                const unsigned part = (unsigned)(w * PW + i);
                const unsigned tab =
                    part * roots + (CTX ? (unsigned)(prev[w] >> (SB * i)) & SMASK : 0u);
                const int sym = dec_sym8(br, T, tab);
                if (sym < 0) return false;
                row |= (unsigned long long)sym << (SB * i);
            }
            prev[w] = row;
            st[s * NW + w] = row;
        }
    }
    return true;
}

template <bool CTX, int NW, int SB>
__global__ void __launch_bounds__(64)
dec_rows(const uint32_t* __restrict__ words, long long nwords, long long n, int raw_first,
         int chunk_vectors, const unsigned long long* __restrict__ chunk_off,
         const unsigned long long* __restrict__ chunk_prev, Row8Tabs T,
         unsigned long long* __restrict__ out, unsigned long long* __restrict__ err, int win_words) {
    extern __shared__ __attribute__((aligned(16))) char lds[];
    unsigned long long* stage = reinterpret_cast<unsigned long long*>(lds);   // [64][C][NW]
    uint32_t* win = reinterpret_cast<uint32_t*>(lds + 64 * 8 * NW * chunk_vectors);
    const int lane = threadIdx.x;
    pqh_set_prio(T.prio);   // latency-bound: issue ahead of the assignment's waves
    const long long chunks = (n + chunk_vectors - 1) / chunk_vectors;
    const long long j0 = (long long)blockIdx.x * 64;
    const long long jn = min(chunks - j0, 64ll);
    const unsigned long long b_lo = chunk_off[j0];
    const unsigned long long b_hi = j0 + 64 < chunks ? chunk_off[j0 + 64] : (unsigned long long)nwords * 32;
    const long long w_lo = (long long)(b_lo >> 5);
    const long long w_hi = min(nwords, (long long)((b_hi + 31) >> 5) + 2);
    const long long nw = w_hi - w_lo;
    const bool in_lds = nw <= win_words;
    if (in_lds) {   // streamed once: non-temporal, so the code tables keep the L2
#pragma unroll 1
        for (long long w0 = 0; w0 < nw; w0 += 4 * 64) {
            uint32_t r[4];
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                const long long w = w0 + u * 64 + lane;
                r[u] = w < nw ? __builtin_nontemporal_load(words + w_lo + w) : 0u;
            }
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                const long long w = w0 + u * 64 + lane;
                if (w < nw) win[w] = __builtin_bswap32(r[u]);   // (MSB-first: PosRd)
            }
        }
        if (lane < 4) win[nw + lane] = 0;   // zero pad read past the window
    }
    __syncthreads();
    const long long j = j0 + lane;
    bool ok = true;
    if (lane < jn) {
        const unsigned long long start = chunk_off[j] - (unsigned long long)w_lo * 32;
        unsigned long long* st = stage + (long long)lane * chunk_vectors * NW;
        ok = in_lds ? dec_row_lane<CTX, true, NW, SB>(win, (uint32_t)(nw + 3), start, j, n,
                                                      chunk_vectors, raw_first, chunk_prev, T, st)
                    : dec_row_lane<CTX, false, NW, SB>(words + w_lo, (uint32_t)(nwords - 1 - w_lo),
                                                       start, j, n, chunk_vectors, raw_first,
                                                       chunk_prev, T, st);
    }
    __syncthreads();
    // the workgroup's rows are contiguous: whole-row stores
    const long long r0 = j0 * chunk_vectors * NW;
    const long long words_out = (min(n, (j0 + 64) * chunk_vectors) - j0 * chunk_vectors) * NW;
#pragma unroll 1
    for (long long q = lane; q < words_out; q += 64) __builtin_nontemporal_store(stage[q], out + r0 + q);
    if (!ok) atomicOr(err, 1ull);
}

// diagnostics only (pqh_debug_poison_lds): fills a whole CU's LDS (160 KB) with `value`, so a
// kernel launched after it on any CU finds that pattern, not zeros or an earlier kernel's
// data, in whatever LDS it reads before writing -- a test for stale-LDS reads
__global__ void __launch_bounds__(1024)
lds_poison(uint32_t value, int words, uint32_t* __restrict__ sink) {
    extern __shared__ __attribute__((aligned(16))) char lds[];
    volatile uint32_t* w = reinterpret_cast<volatile uint32_t*>(lds);
    for (int i = threadIdx.x; i < words; i += blockDim.x) w[i] = value;
    lds_barrier();
    if (threadIdx.x == 0 && w[(blockIdx.x * 977u) % (unsigned)words] != value) sink[0] = 1u;
}

}  // namespace

extern "C" {

int pqh_tables_alloc(pqh_ctx_t* ctx, int m, int k, int context, pqh_tables_t** out) {
    if (!ctx || !out || m <= 0 || k <= 0 || k > 4096) return PQH_ERR_ARG;
    if (context && k != 256)
        return pqh_set_error(ctx, PQH_ERR_UNSUPPORTED,
                             "context coding needs K=256 (huffman_encoder.c:187,234)");
    int rc = pqh_use_device(ctx);
    if (rc) return rc;
    pqh_tables* t = new pqh_tables();
    t->ctx = ctx;
    t->m = m;
    t->k = k;
    t->context = context;
    t->roots = context ? k : 1;
    t->items = (long long)t->roots * k;
    t->tables = (long long)m * t->roots;
    // first-level width W1 (the table set's lut1 rows are 2^W1 entries, packed): 9 in context
    // mode (1 KB per alphabet, K * m alphabets), 11 for K <= 256, 13 for K = 4,096 (codes
    // average ~12 bits there: with 11, most symbols took the second level, whose subtables
    // -- up to 2^12 entries per long prefix -- made the K = 4,096 decode read ~27x its stream)
    t->l1_bits = context ? 9 : (k > 256 ? 13 : 11);
    // Second-level width: 8 bits for K <= 256 (codes past W1 + 8 bits are rare); 12 bits
    // for larger alphabets, whose rarest symbols sit ~log2(N) bits deep -- with 8 bits
    // (19 covered) a K = 4096 stream spent its decode in the long-code list (133 ms per
    // 1M vectors).  A larger pool for those few alphabets.
    t->l2_bits = k > 256 ? 12 : 8;
    t->lut2_cap = std::min<long long>(k > 256 ? t->tables * (1ll << 20) : t->tables * 2048 + 65536,
                                      kL2BaseMax - 1);
    if (hipMalloc(&t->d_enc, (size_t)m * t->items * 8) != hipSuccess ||
        hipMalloc(&t->d_enc32, (size_t)m * t->items * 4) != hipSuccess ||
        hipMalloc(&t->d_enc16, (size_t)m * t->items * 2) != hipSuccess ||
        hipMalloc(&t->d_lut1, (size_t)(t->tables << t->l1_bits) * 2 + 16) != hipSuccess ||
        hipMalloc(&t->d_lut2, (size_t)t->lut2_cap * 2) != hipSuccess ||
        hipMalloc(&t->d_meta, (size_t)t->tables * 4 + 16) != hipSuccess ||
        hipMalloc(&t->d_long, (size_t)t->tables * k * sizeof(pqh_long_code)) != hipSuccess ||
        hipMalloc(&t->d_long_cnt, (size_t)t->tables * 4) != hipSuccess ||
        hipMalloc(&t->d_err, 32) != hipSuccess) {
        pqh_tables_destroy(t);
        return pqh_set_error(ctx, PQH_ERR_NOMEM, "hipMalloc tables");
    }
    // the error word starts clear (builds leave it sticky; pqh_tables_status clears it);
    // synchronised, as a build may run on another context's stream
    if (hipMemsetAsync(t->d_err, 0, 32, ctx->stream) != hipSuccess ||
        hipStreamSynchronize(ctx->stream) != hipSuccess) {
        pqh_tables_destroy(t);
        return pqh_set_error(ctx, PQH_ERR_HIP, "hipMemsetAsync tables");
    }
    *out = t;
    return PQH_OK;
}

int pqh_tables_destroy(pqh_tables_t* t) {
    if (!t) return PQH_OK;
    if (t->ctx) {
        (void)hipSetDevice(t->ctx->device);
        (void)hipStreamSynchronize(t->ctx->stream);
    }
    void* bufs[] = {t->d_enc, t->d_enc32, t->d_enc16, t->d_lut1, t->d_lut2, t->d_meta, t->d_long,
                    t->d_long_cnt, t->d_err};
    for (void* b : bufs)
        if (b) (void)hipFree(b);
    delete t;
    return PQH_OK;
}

// the LUT pool head a build allocates from (slot pool_slot) and the other slot
static unsigned long long* pool_slot_ptr(pqh_tables* t, int slot) {
    return reinterpret_cast<unsigned long long*>(t->d_err + 2) + slot;
}

static GrpLut grp_lut_of(pqh_tables* t) {
    return GrpLut{t->enc32_by_trees ? nullptr : t->d_enc32, t->d_enc16, t->d_lut1, t->d_lut2,
                  t->d_meta, t->d_long, t->d_long_cnt, pool_slot_ptr(t, t->pool_slot),
                  t->lut2_cap, t->l1_bits, t->l2_bits, pqh_prio("LUTS", 3)};
}

static void launch_lut_grp(pqh_ctx* ctx, pqh_tables* t) {
    const GrpLut lut = grp_lut_of(t);
    hipLaunchKernelGGL(lut_grp, dim3((unsigned)((t->tables + kGrpTrees - 1) / kGrpTrees)), dim3(64),
                       0, ctx->stream, t->d_enc, t->k, t->tables, lut,
                       pool_slot_ptr(t, t->pool_slot ^ 1));
}

static int launch_luts(pqh_ctx* ctx, pqh_tables* t) {
    // the 16-lane build for context tables (W1 = 9), lut_build otherwise
    // (PQH_LUT_IMPL=block: lut_build for every table set)
    const char* impl = std::getenv("PQH_LUT_IMPL");
    if (!(impl && std::strcmp(impl, "block") == 0) && t->l1_bits <= 9 && t->k == 256) {
        launch_lut_grp(ctx, t);
        PQH_LAUNCH_CHECK(ctx);
        t->pool_slot ^= 1;   // (the kernel zeroed the other slot for the next build)
        return PQH_OK;
    }
    // (the pool head, d_err[2..3], was zeroed with the error word before the trees)
    const size_t lds = (size_t)2 * 4 << t->l1_bits;   // w2max + sub_id
    if (lds > 48 * 1024) {
        static const bool big = [] {
            return hipFuncSetAttribute((const void*)lut_build,
                                       hipFuncAttributeMaxDynamicSharedMemorySize,
                                       (int)((size_t)2 * 4 << kL1Max)) == hipSuccess;
        }();
        if (!big) return pqh_set_error(ctx, PQH_ERR_HIP, "lut_build: dynamic LDS attribute");
    }
    hipLaunchKernelGGL(lut_build, dim3((unsigned)t->tables), dim3(256), lds, ctx->stream, t->d_enc,
                       t->enc32_by_trees ? nullptr : t->d_enc32, t->d_enc16, t->k, t->l1_bits, t->l2_bits, t->d_meta, t->d_lut1, t->d_lut2,
                       t->lut2_cap, t->d_long, t->d_long_cnt, pool_slot_ptr(t, t->pool_slot),
                       pool_slot_ptr(t, t->pool_slot ^ 1));
    PQH_LAUNCH_CHECK(ctx);
    t->pool_slot ^= 1;   // (the kernel zeroed the other slot for the next build)
    return PQH_OK;
}

int pqh_tables_build(pqh_ctx_t* ctx, pqh_tables_t* t, const uint32_t* d_counts) {
    return pqh_tables_build_impl(ctx, t, d_counts, PQH_TREES_DEFAULT);
}

static int build_trees(pqh_ctx_t* ctx, pqh_tables_t* t, const uint32_t* d_counts, int which,
                       pqh_tables_t* t2 = nullptr, const uint32_t* d_counts2 = nullptr,
                       bool* fused = nullptr);

int pqh_tables_build_impl(pqh_ctx_t* ctx, pqh_tables_t* t, const uint32_t* d_counts, int which) {
    // trees and decode tables in one launch where the group builders serve both (context
    // tables, K = 256; PQH_FUSE_LUTS=0: two launches); else the trees, then launch_luts
    bool fused = false;
    const int rc = build_trees(ctx, t, d_counts, which, nullptr, nullptr, &fused);
    return rc ? rc : fused ? PQH_OK : launch_luts(ctx, t);
}

int pqh_tables_build_trees(pqh_ctx_t* ctx, pqh_tables_t* t, const uint32_t* d_counts, int which) {
    return build_trees(ctx, t, d_counts, which);
}

int pqh_tables_build_pair(pqh_ctx_t* ctx, pqh_tables_t* t, const uint32_t* d_counts,
                          pqh_tables_t* t2, const uint32_t* d_counts2) {
    if (!t || !t2 || t == t2 || !d_counts2 || t2->k != t->k || t2->m != t->m ||
        t2->context != t->context || !t2->ctx || t2->ctx->device != t->ctx->device ||
        (reinterpret_cast<uintptr_t>(d_counts2) & 15u))
        return PQH_ERR_ARG;
    int rc = build_trees(ctx, t, d_counts, PQH_TREES_DEFAULT, t2, d_counts2);
    if (!rc) rc = launch_luts(ctx, t);
    return rc ? rc : launch_luts(ctx, t2);
}

int pqh_tables_build_luts(pqh_ctx_t* ctx, pqh_tables_t* t) {
    if (!ctx || !t || !t->ctx || t->ctx->device != ctx->device) return PQH_ERR_ARG;
    const int rc = pqh_use_device(ctx);
    return rc ? rc : launch_luts(ctx, t);
}

// the code tables' trees (d_enc) on ctx's stream; the decode tables follow (launch_luts)
static int build_trees(pqh_ctx_t* ctx, pqh_tables_t* t, const uint32_t* d_counts, int which,
                       pqh_tables_t* t2, const uint32_t* d_counts2, bool* fused) {
    // any context of the tables' device may run the build (on its own stream), so the
    // builds of consecutive batches can overlap on different streams
    if (!ctx || !t || !d_counts || !t->ctx || t->ctx->device != ctx->device) return PQH_ERR_ARG;
    if (which < PQH_TREES_DEFAULT || which > PQH_TREES_GROUP) return PQH_ERR_ARG;
    int rc = pqh_use_device(ctx);
    if (rc) return rc;
    // (no memset: the tree kernel zeroes each set's LUT pool head; the error word is sticky)
    if (reinterpret_cast<uintptr_t>(d_counts) & 15u) return PQH_ERR_ARG;
    t->enc32_by_trees = false;   // (set below by the builds that write the gather copy)
    if (t2) t2->enc32_by_trees = false;
    const long long trees = t->tables;
    // Three builds of the same trees (K <= 256):
    //  * 16 lanes per tree, four trees per wavefront (huff_trees_grp, the default): two LDS
    //    round trips per pop, <= 32 VGPRs, so it runs beside the assignment grid;
    //  * one lane per tree through LDS (huff_trees_small, PQH_TREE_IMPL=lane): 128
    //    wavefronts of 16 trees, a heap level per LDS round trip (0.64 ms alone);
    //  * one wavefront per tree with the heap in registers (huff_trees_wave,
    //    PQH_TREE_IMPL=wave): 0.40 ms alone, but 52 VGPRs.
    const char* impl = which == PQH_TREES_WAVE ? "wave"
                     : which == PQH_TREES_LANE ? "lane"
                     : which == PQH_TREES_GROUP ? "grp" : std::getenv("PQH_TREE_IMPL");
    if (t->k <= 256 && impl && std::strcmp(impl, "wave") == 0 && !t2) {
        // writes every entry (0 for symbols that never occur): no memset
        hipLaunchKernelGGL(huff_trees_wave, dim3((unsigned)((trees + kTreeWaves - 1) / kTreeWaves)),
                           dim3(64 * kTreeWaves), 0, ctx->stream, d_counts, t->k, trees, t->d_enc,
                           t->d_err);
        PQH_LAUNCH_CHECK(ctx);
        return PQH_OK;
    }
    if (t->k <= 256 && !(impl && std::strcmp(impl, "lane") == 0)) {
        const long long blocks = (trees + kGrpTrees - 1) / kGrpTrees +
                                 (t2 ? (t2->tables + kGrpTrees - 1) / kGrpTrees : 0);
        static const bool fuse_env = [] {
            const char* f = std::getenv("PQH_FUSE_LUTS");
            const char* l = std::getenv("PQH_LUT_IMPL");
            return !(f && std::strcmp(f, "0") == 0) && !(l && std::strcmp(l, "block") == 0);
        }();
        const bool fuse = fused && fuse_env && !t2 && t->k == 256 && t->l1_bits <= 9;
        t->enc32_by_trees = true;   // (before grp_lut_of: the trees write the gather copies)
        GrpLut lut{};
        unsigned long long* next = nullptr;
        if (fuse) {
            lut = grp_lut_of(t);                      // slot pool_slot, zeroed beforehand
            next = pool_slot_ptr(t, t->pool_slot ^ 1);   // zeroed by this launch
        }
        hipLaunchKernelGGL(huff_trees_grp, dim3((unsigned)blocks), dim3(64), 0, ctx->stream, d_counts,
                           t->k, trees, t->d_enc, t->d_err, t2 ? t2->tables : 0ll,
                           t2 ? d_counts2 : d_counts, t2 ? t2->d_enc : t->d_enc,
                           t2 ? t2->d_err : t->d_err, pqh_prio("TREES", 3), t->d_enc32,
                           t2 ? t2->d_enc32 : t->d_enc32, t->d_enc16, t2 ? t2->d_enc16 : t->d_enc16,
                           lut, next);
        PQH_LAUNCH_CHECK(ctx);
        if (t2) t2->enc32_by_trees = true;
        if (fuse) {
            t->pool_slot ^= 1;
            *fused = true;
        }
        return PQH_OK;
    }
    // (every build writes every entry, 0 for symbols that never occur: no memset)
    if (t->k <= 256) {
        // trees per workgroup: fewer = more, smaller workgroups (3.5 KB of LDS per tree), so
        // the build spreads over more CUs and leaves each CU's LDS to concurrent kernels
        // (16 = 56 KB: beside three assignment workgroups; PQH_TREE_TPW = 8 / 16 / 32)
        static const int tpw_env = [] {
            const char* e = std::getenv("PQH_TREE_TPW");
            const int v = e ? std::atoi(e) : 0;
            return v == 8 || v == 16 || v == 32 ? v : 16;
        }();
        auto launch = [&](auto tpw_c) -> int {
            constexpr int TPW = decltype(tpw_c)::value;
            const size_t lds = (size_t)TPW * (512 * 4 + 256 * 4 + 256 * 2);
            PQH_HIP(ctx, hipFuncSetAttribute((const void*)huff_trees_small<TPW>,
                                             hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
            const long long blocks = (trees + TPW - 1) / TPW + (t2 ? (t2->tables + TPW - 1) / TPW : 0);
            hipLaunchKernelGGL((huff_trees_small<TPW>), dim3((unsigned)blocks), dim3(64), lds,
                               ctx->stream, d_counts, t->k, trees, t->d_enc, t->d_err,
                               t2 ? t2->tables : 0ll, t2 ? d_counts2 : d_counts,
                               t2 ? t2->d_enc : t->d_enc, t2 ? t2->d_err : t->d_err);
            return PQH_OK;
        };
        rc = tpw_env == 8 ? launch(std::integral_constant<int, 8>{})
           : tpw_env == 32 ? launch(std::integral_constant<int, 32>{})
                           : launch(std::integral_constant<int, 16>{});
        if (rc) return rc;
    } else if (!(impl && std::strcmp(impl, "lane") == 0)) {
        // K > 256: one wavefront per tree, sifts read in parallel (huff_trees_par)
        const size_t lds = (size_t)2 * 4096 * 8 + (size_t)4096 * (4 + 2 + 4);   // 104 KB
        PQH_HIP(ctx, hipFuncSetAttribute((const void*)huff_trees_par<4096>,
                                         hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
        const long long all = trees + (t2 ? t2->tables : 0);
        hipLaunchKernelGGL((huff_trees_par<4096>), dim3((unsigned)all), dim3(64), lds, ctx->stream,
                           d_counts, t->k, trees, t->d_enc, t->d_err, t2 ? d_counts2 : d_counts,
                           t2 ? t2->d_enc : t->d_enc, t2 ? t2->d_err : t->d_err);
    } else {   // (PQH_TREE_IMPL=lane: one lane per tree through LDS)
        if (t2) return pqh_set_error(ctx, PQH_ERR_UNSUPPORTED, "paired K > 256 build: lane builder");
        constexpr int TPW = 1;
        const size_t lds = (size_t)4096 * TPW * (16 + 4 + 4 + 2);
        PQH_HIP(ctx, hipFuncSetAttribute((const void*)huff_trees<4096, TPW>,
                                         hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
        hipLaunchKernelGGL((huff_trees<4096, TPW>), dim3((unsigned)((trees + TPW - 1) / TPW)), dim3(64),
                           lds, ctx->stream, d_counts, t->k, trees, t->d_enc, t->d_err);
    }
    PQH_LAUNCH_CHECK(ctx);
    return PQH_OK;
}

// diagnostics only: phase stamps (s_memtime) of tree 0 of the last huff_trees launch
int pqh_debug_tree_stamps(pqh_ctx_t* ctx, unsigned long long* out16) {
    if (!ctx || !out16) return PQH_ERR_ARG;
    PQH_HIP(ctx, hipStreamSynchronize(ctx->stream));
    PQH_HIP(ctx, hipMemcpyFromSymbol(out16, HIP_SYMBOL(g_tree_stamps), 16 * sizeof(unsigned long long)));
    return PQH_OK;
}

// diagnostics only: every CU's LDS filled with `value` (lds_poison), on ctx's stream; a
// test runs it right before a kernel under test.  4 workgroups per CU, each holding all of
// the CU's LDS, so every CU runs at least one.
int pqh_debug_poison_lds(pqh_ctx_t* ctx, unsigned value) {
    if (!ctx) return PQH_ERR_ARG;
    int rc = pqh_use_device(ctx);
    if (rc) return rc;
    const int bytes = 160 * 1024;
    PQH_HIP(ctx, hipFuncSetAttribute((const void*)lds_poison,
                                     hipFuncAttributeMaxDynamicSharedMemorySize, bytes));
    hipLaunchKernelGGL(lds_poison, dim3((unsigned)(4 * ctx->num_cus)), dim3(1024), bytes,
                       ctx->stream, (uint32_t)value, bytes / 4,
                       reinterpret_cast<uint32_t*>(ctx->d_diag + 5));
    PQH_LAUNCH_CHECK(ctx);
    return PQH_OK;
}

int pqh_tables_encode_ready(const pqh_tables_t* t) { return t && t->enc32_by_trees ? 1 : 0; }

int pqh_tables_upload(pqh_ctx_t* ctx, pqh_tables_t* t, const huffman_codebook_t* cbs) {
    if (!ctx || !t || !cbs) return PQH_ERR_ARG;
    for (int i = 0; i < t->m; ++i)
        if (cbs[i].alphabet_size != t->k || (cbs[i].is_context ? 1 : 0) != t->context) return PQH_ERR_ARG;
    int rc = pqh_use_device(ctx);
    if (rc) return rc;
    std::vector<unsigned long long> h((size_t)t->m * t->items, 0);
    for (int i = 0; i < t->m; ++i)
        for (long long it = 0; it < t->items; ++it) {
            const huffman_code_item_t& c = cbs[i].items[it];
            if (c.bit_length <= 0) continue;
            if (c.bit_length > kMaxCodeLen)
                return pqh_set_error(ctx, PQH_ERR_CODE_TOO_LONG, "code of %d bits", c.bit_length);
            unsigned long long v = 0;
            for (int b = 0; b < c.bit_length; ++b) v = (v << 1) | ((c.code[b >> 3] >> (7 - (b & 7))) & 1u);
            h[(size_t)i * t->items + it] = ((unsigned long long)c.bit_length << 56) | v;
        }
    PQH_HIP(ctx, hipMemsetAsync(t->d_err, 0, 32, ctx->stream));   // error word + LUT pool heads
    PQH_HIP(ctx, hipMemcpyAsync(t->d_enc, h.data(), h.size() * 8, hipMemcpyHostToDevice, ctx->stream));
    t->enc32_by_trees = false;   // the LUT build writes the gather copy
    rc = launch_luts(ctx, t);
    if (rc) return rc;
    PQH_HIP(ctx, hipStreamSynchronize(ctx->stream));  // h goes out of scope
    return PQH_OK;
}

int pqh_tables_create(pqh_ctx_t* ctx, const huffman_codebook_t* cbs, int m, pqh_tables_t** out) {
    if (!ctx || !cbs || m <= 0 || !out) return PQH_ERR_ARG;
    int rc = pqh_tables_alloc(ctx, m, cbs[0].alphabet_size, cbs[0].is_context ? 1 : 0, out);
    if (rc) return rc;
    rc = pqh_tables_upload(ctx, *out, cbs);
    if (rc) {
        pqh_tables_destroy(*out);
        *out = nullptr;
    }
    return rc;
}

int pqh_tables_status(pqh_ctx_t* ctx, const pqh_tables_t* t) {
    if (!ctx || !t) return PQH_ERR_ARG;
    uint32_t e = 0;
    PQH_HIP(ctx, hipMemcpyAsync(&e, t->d_err, 4, hipMemcpyDeviceToHost, ctx->stream));
    PQH_HIP(ctx, hipStreamSynchronize(ctx->stream));
    if (e) PQH_HIP(ctx, hipMemsetAsync(t->d_err, 0, 4, ctx->stream));   // (sticky until read)
    if (e & 2u) return pqh_set_error(ctx, PQH_ERR_UNSUPPORTED, "a k <= 256 tree builder ran with k > 256");
    return e ? pqh_set_error(ctx, PQH_ERR_CODE_TOO_LONG, "a Huffman code exceeds 56 bits") : PQH_OK;
}

int pqh_tables_codebooks(pqh_ctx_t* ctx, const pqh_tables_t* t, huffman_codebook_t* cbs) {
    if (!ctx || !t || !cbs) return PQH_ERR_ARG;
    int rc = pqh_tables_status(ctx, t);
    if (rc) return rc;
    std::vector<unsigned long long> h((size_t)t->m * t->items);
    PQH_HIP(ctx, hipMemcpyAsync(h.data(), t->d_enc, h.size() * 8, hipMemcpyDeviceToHost, ctx->stream));
    PQH_HIP(ctx, hipStreamSynchronize(ctx->stream));
    for (int i = 0; i < t->m; ++i) {
        huffman_codebook_t& cb = cbs[i];
        cb.alphabet_size = t->k;
        cb.is_context = t->context;
        cb.num_items = (int)t->items;
        cb.items = (huffman_code_item_t*)calloc((size_t)t->items, sizeof(huffman_code_item_t));
        long long bytes = 0;
        for (long long it = 0; it < t->items; ++it) bytes += ((h[(size_t)i * t->items + it] >> 56) + 7) / 8;
        cb.codefield = (byte_t*)calloc((size_t)(bytes > 0 ? bytes : 1), 1);
        byte_t* p = cb.codefield;
        for (long long it = 0; it < t->items; ++it) {
            const unsigned long long v = h[(size_t)i * t->items + it];
            const int L = (int)(v >> 56);
            cb.items[it].bit_length = L;
            if (!L) continue;
            const unsigned long long code = v & kCodeMask;
            for (int b = 0; b < L; ++b)
                if ((code >> (L - 1 - b)) & 1ull) p[b >> 3] |= (byte_t)(0x80u >> (b & 7));
            cb.items[it].code = p;
            p += (L + 7) / 8;
        }
    }
    return PQH_OK;
}

int pqh_decode(pqh_ctx_t* ctx, const pqh_tables_t* t, const unsigned char* d_stream,
               unsigned long long stream_bytes, long long n, int raw_first, int chunk_vectors,
               const unsigned long long* d_chunk_offsets, const void* d_chunk_prev, void* d_codes) {
    if (!ctx || !t || n < 0 || chunk_vectors <= 0 ||
        (n > 0 && (!d_stream || !d_chunk_offsets || !d_codes)))
        return PQH_ERR_ARG;
    if (reinterpret_cast<uintptr_t>(d_stream) & 3u) return PQH_ERR_ARG;
    if (t->context && !raw_first && !d_chunk_prev) return PQH_ERR_ARG;
    if (t->m > 16) return PQH_ERR_UNSUPPORTED;
    int rc = pqh_use_device(ctx);
    if (rc) return rc;
    if (n == 0) return PQH_OK;
    // (no memset: d_diag[1] is sticky until pqh_decode_status reads it)
    const long long chunks = (n + chunk_vectors - 1) / chunk_vectors;
    const long long nwords = (long long)(stream_bytes / 4);
    const unsigned blocks = (unsigned)((chunks + 63) / 64);
    if (reinterpret_cast<uintptr_t>(d_codes) & 3u) return PQH_ERR_ARG;
    const size_t l1_bytes = (size_t)(t->tables << t->l1_bits) * 2;
    const size_t meta_bytes = ((size_t)t->tables * 4 + 15) & ~(size_t)15;
    const bool lds_l1 = meta_bytes + l1_bytes <= 48 * 1024;
    const size_t esz = t->k <= 256 ? 1 : 2;
    // stream window: the workgroup's 64 chunks at up to 12 (K <= 256; Huffman averages
    // at most ~8.x bits) or 14 bits per symbol, at most 16 KB -- a larger span reads the
    // global stream instead; staging: S vectors per lane, at most 16 KB
    const long long sym_bits = t->k <= 256 ? 12 : 14;
    const int win_words = (int)std::min<long long>(4096, std::max<long long>(
        256, (64ll * chunk_vectors * t->m * sym_bits + 31) / 32 + 8));
    int S = chunk_vectors;
    while (S > 1 && (size_t)64 * S * t->m * esz > 16 * 1024) S = (S + 1) / 2;
    const size_t lds = meta_bytes + (lds_l1 ? ((l1_bytes + 15) & ~(size_t)15) : 0) +
                       ((size_t)win_words + 4) * 4 + (size_t)64 * S * t->m * esz + 16;
    if (lds > 160 * 1024) return PQH_ERR_UNSUPPORTED;
    // whole-row decoders (<= 32 VGPRs: they run beside the assignment grid): rows of 8 or 16
    // u8 codes, or of 8 u16 codes, chunks of C <= 32 vectors, 8-byte aligned rows
    const int esz_b = (int)esz;
    const int row_bytes = t->m * esz_b;
    if ((row_bytes == 8 || row_bytes == 16) && (esz_b == 1 || t->m == 8) && chunk_vectors <= 32 &&
        nwords < (1ll << 31) && !(reinterpret_cast<uintptr_t>(d_codes) & 7) &&
        !(reinterpret_cast<uintptr_t>(d_chunk_prev) & 7)) {
        const int nw_row = row_bytes / 8;
        const int ww = (int)std::min<long long>(4096 - 1024 * (nw_row - 1), std::max<long long>(
            256, (64ll * chunk_vectors * t->m * sym_bits + 31) / 32 + 8));
        const size_t lds_r = (size_t)64 * row_bytes * chunk_vectors + ((size_t)ww + 4) * 4;
        const Row8Tabs T{t->d_lut1, t->d_lut2, t->d_meta, t->d_long, t->d_long_cnt, t->lut2_cap,
                         t->l1_bits, t->k, pqh_prio("DECODE", 3)};
        const uint32_t* wp = reinterpret_cast<const uint32_t*>(d_stream);
        const unsigned long long* cp = static_cast<const unsigned long long*>(d_chunk_prev);
        unsigned long long* op = static_cast<unsigned long long*>(d_codes);
#define PQH_DEC_ROWS(CTX, NW, SB)                                                               \
    do {                                                                                         \
        if (lds_r > 64 * 1024)                                                                   \
            PQH_HIP(ctx, hipFuncSetAttribute((const void*)(dec_rows<CTX, NW, SB>),               \
                                             hipFuncAttributeMaxDynamicSharedMemorySize,         \
                                             (int)lds_r));                                       \
        hipLaunchKernelGGL((dec_rows<CTX, NW, SB>), dim3(blocks), dim3(64), lds_r, ctx->stream,   \
                           wp, nwords, n, raw_first, chunk_vectors, d_chunk_offsets, cp, T, op,  \
                           ctx->d_diag + 1, ww);                                                 \
    } while (0)
        if (esz_b == 2)
            PQH_DEC_ROWS(false, 2, 16);
        else if (nw_row == 1 && t->context)
            PQH_DEC_ROWS(true, 1, 8);
        else if (nw_row == 1)
            PQH_DEC_ROWS(false, 1, 8);
        else if (t->context)
            PQH_DEC_ROWS(true, 2, 8);
        else
            PQH_DEC_ROWS(false, 2, 8);
#undef PQH_DEC_ROWS
        PQH_LAUNCH_CHECK(ctx);
        return PQH_OK;
    }
#define PQH_DEC(MT, T, L)                                                                        \
    do {                                                                                         \
        if (lds > 64 * 1024)                                                                     \
            PQH_HIP(ctx, hipFuncSetAttribute((const void*)(dec_chunks<MT, T, L>),                \
                                             hipFuncAttributeMaxDynamicSharedMemorySize,         \
                                             (int)lds));                                         \
        hipLaunchKernelGGL((dec_chunks<MT, T, L>), dim3(blocks), dim3(64), lds, ctx->stream,      \
                           reinterpret_cast<const uint32_t*>(d_stream), nwords, n, t->m, t->k,   \
                           t->context, raw_first, chunk_vectors, d_chunk_offsets,                \
                           static_cast<const T*>(d_chunk_prev), t->d_lut1, t->d_lut2, t->d_meta, \
                           t->l1_bits, t->tables, t->lut2_cap, t->d_long,                        \
                           t->d_long_cnt, static_cast<T*>(d_codes), ctx->d_diag + 1, win_words,  \
                           S);                                                                   \
    } while (0)
    if (t->k <= 256) {
        if (t->m == 8) {
            if (lds_l1) PQH_DEC(8, uint8_t, true); else PQH_DEC(8, uint8_t, false);
        } else if (t->m == 16) {
            if (lds_l1) PQH_DEC(16, uint8_t, true); else PQH_DEC(16, uint8_t, false);
        } else {
            if (lds_l1) PQH_DEC(0, uint8_t, true); else PQH_DEC(0, uint8_t, false);
        }
    } else {
        if (lds_l1) PQH_DEC(0, uint16_t, true); else PQH_DEC(0, uint16_t, false);
    }
#undef PQH_DEC
    PQH_LAUNCH_CHECK(ctx);
    return PQH_OK;
}

int pqh_decode_status(pqh_ctx_t* ctx) {
    unsigned long long e = 0;
    PQH_HIP(ctx, hipMemcpyAsync(&e, ctx->d_diag + 1, 8, hipMemcpyDeviceToHost, ctx->stream));
    PQH_HIP(ctx, hipStreamSynchronize(ctx->stream));
    if (e) PQH_HIP(ctx, hipMemsetAsync(ctx->d_diag + 1, 0, 8, ctx->stream));   // (sticky until read)
    return e ? pqh_set_error(ctx, PQH_ERR_CORRUPT, "invalid code in stream") : PQH_OK;
}

// Chunk index of a stream that came without a sidecar: a sequential walk over a HOST copy
// of the code table (index building only; the symbols are decoded by pqh_decode).
int pqh_chunk_index_host(const pqh_tables_t* t, const unsigned char* stream,
                         unsigned long long stream_bytes, long long n, int raw_first,
                         int chunk_vectors, unsigned long long* chunk_offsets, void* chunk_prev) {
    if (!t || n < 0 || chunk_vectors <= 0 || (n > 0 && (!stream || !chunk_offsets))) return PQH_ERR_ARG;
    if (t->context && !chunk_prev) return PQH_ERR_ARG;
    pqh_ctx* ctx = t->ctx;
    std::vector<unsigned long long> enc((size_t)t->m * t->items);
    PQH_HIP(ctx, hipMemcpyAsync(enc.data(), t->d_enc, enc.size() * 8, hipMemcpyDeviceToHost, ctx->stream));
    PQH_HIP(ctx, hipStreamSynchronize(ctx->stream));
    // per-table canonical lookup: (len, code) -> symbol, via sorted vectors per length
    const int W = 16;
    std::vector<int32_t> lut((size_t)t->tables << W, -1);
    std::vector<std::vector<std::pair<unsigned long long, int>>> longs(t->tables);
    for (long long tab = 0; tab < t->tables; ++tab)
        for (int s = 0; s < t->k; ++s) {
            const unsigned long long v = enc[(size_t)tab * t->k + s];
            const int L = (int)(v >> 56);
            if (!L) continue;
            const unsigned long long code = v & kCodeMask;
            if (L <= W) {
                for (unsigned long long e = code << (W - L); e < (code + 1) << (W - L); ++e)
                    lut[((size_t)tab << W) + e] = (L << 16) | s;
            } else {
                longs[tab].push_back({(code << 8) | (unsigned long long)L, s});
            }
        }
    const unsigned long long total = stream_bytes * 8;
    auto peek = [&](unsigned long long p, int nb) -> unsigned long long {
        unsigned long long r = 0;
        for (int b = 0; b < nb; ++b) {
            const unsigned long long q = p + b;
            r = (r << 1) | (q < total ? (unsigned long long)((stream[q >> 3] >> (7 - (q & 7))) & 1u) : 0ull);
        }
        return r;
    };
    std::vector<unsigned> prev(t->m, 0);
    bool warm = t->context && raw_first;
    int warm_bits = 1;
    while ((1 << warm_bits) < t->k) ++warm_bits;
    unsigned long long pos = 0;
    for (long long v = 0; v < n; ++v) {
        if (v % chunk_vectors == 0) {
            const long long j = v / chunk_vectors;
            chunk_offsets[j] = pos;
            if (t->context)
                for (int i = 0; i < t->m; ++i) {
                    if (t->k <= 256) static_cast<uint8_t*>(chunk_prev)[j * t->m + i] = (uint8_t)prev[i];
                    else static_cast<uint16_t*>(chunk_prev)[j * t->m + i] = (uint16_t)prev[i];
                }
        }
        for (int i = 0; i < t->m; ++i) {
            unsigned sym;
            if (warm) {
                sym = (unsigned)peek(pos, warm_bits);
                pos += warm_bits;
            } else {
                const long long tab = (long long)i * t->roots + (t->context ? prev[i] : 0);
                const int32_t e = lut[((size_t)tab << W) + peek(pos, W)];
                if (e >= 0) {
                    pos += (unsigned)e >> 16;
                    sym = (unsigned)e & 0xFFFFu;
                } else {
                    bool found = false;
                    sym = 0;
                    for (auto& lc : longs[tab]) {
                        const int L = (int)(lc.first & 0xFF);
                        if (peek(pos, L) == (lc.first >> 8)) {
                            pos += L;
                            sym = (unsigned)lc.second;
                            found = true;
                            break;
                        }
                    }
                    if (!found) return PQH_ERR_CORRUPT;
                }
                if (pos > total) return PQH_ERR_CORRUPT;
            }
            prev[i] = sym;
        }
        warm = false;
    }
    return PQH_OK;
}

}  // extern "C"

// ---------------------------------------------------------------- tree-mode decode
// huffman_decoder --tree (huffman_decoder.c:214-247): row p is decoded in the context of the
// row at stream position parent_pos[p] (the traverser replayed over the children stream),
// a root starting every part with the raw warm-up bits.  One lane per chunk of C rows from
// the encoder's chunk index; the chunk's rows are staged in LDS, so a parent inside the
// chunk is read back from there, and the parents that lie before the chunk come from the
// ext sidecar (ext_rows[ext_off[j] ...], in row order) -- every chunk decodes independently.
namespace {
__global__ void __launch_bounds__(64)
dec_tree(const uint32_t* __restrict__ words, long long nwords, long long n, int m, int k,
         int chunk_vectors, const unsigned long long* __restrict__ chunk_off,
         const long long* __restrict__ parent_pos, const long long* __restrict__ ext_off,
         const uint8_t* __restrict__ ext_rows, const uint16_t* __restrict__ lut1,
         const uint16_t* __restrict__ lut2, const uint32_t* __restrict__ meta, int w1,
         long long lut2_cap, const pqh_long_code* __restrict__ longs,
         const uint32_t* __restrict__ long_cnt, uint8_t* __restrict__ out,
         unsigned long long* __restrict__ err, unsigned long long total_bits) {
    extern __shared__ uint8_t tstage[];   // [64 lanes][C rows][m]
    const long long chunks = (n + chunk_vectors - 1) / chunk_vectors;
    const long long j = (long long)blockIdx.x * 64 + threadIdx.x;
    if (j >= chunks) return;               // no barriers below: lanes are independent
    const long long v0 = j * chunk_vectors;
    const long long v1 = min(n, v0 + chunk_vectors);
    uint8_t* st = tstage + (long long)threadIdx.x * chunk_vectors * m;
    DecTables T{meta, lut1, lut2, lut2_cap, longs, long_cnt, k, w1};
    BitReader br;
    br.init(words, nwords - 1, chunk_off[j]);
    long long e = ext_off[j];
    const long long e_end = ext_off[j + 1];
    int warm_bits = 1;
    while ((1 << warm_bits) < k) ++warm_bits;
    // a chunk that starts past the stream's end (a truncated file or a stale sidecar) reads
    // nothing; one whose symbols run past it is reported below -- never decoded silently
    bool ok = chunk_off[j] <= total_bits;
    for (long long p = v0; p < v1 && ok; ++p) {
        const long long pp = parent_pos[p];
        const uint8_t* prow = nullptr;
        if (pp >= v0 && pp < p) {
            prow = st + (pp - v0) * m;
        } else if (pp >= 0) {
            if (pp >= p || e >= e_end) { ok = false; break; }   // inconsistent sidecar
            prow = ext_rows + e * m;
            ++e;
        }
        uint8_t* o = st + (p - v0) * m;
        for (int i = 0; i < m; ++i) {
            unsigned sym;
            if (!prow) {
                sym = br.peek(warm_bits);
                br.skip(warm_bits);
            } else if (!dec_symbol(br, T, (long long)i * k + prow[i], sym)) {
                ok = false;
                break;
            }
            o[i] = (uint8_t)sym;
        }
    }
    if (br.pos() > total_bits) ok = false;
    const long long nb = (v1 - v0) * m;
    uint8_t* dst = out + v0 * m;
    for (long long q = 0; q < nb; ++q) dst[q] = ok ? st[q] : 0;
    if (!ok) atomicOr(err, 1ull);
}
}  // namespace

int pqh_decode_tree(pqh_ctx_t* ctx, const pqh_tables_t* t, const unsigned char* d_stream,
                    unsigned long long stream_bytes, long long n, int chunk_vectors,
                    const unsigned long long* d_chunk_offsets, const long long* d_parent_pos,
                    const long long* d_ext_offsets, const unsigned char* d_ext_rows,
                    void* d_rows) {
    if (!ctx || !t || !t->context || t->k > 256 || n < 0 || chunk_vectors <= 0 ||
        (n > 0 && (!d_stream || !d_chunk_offsets || !d_parent_pos || !d_ext_offsets || !d_rows)))
        return PQH_ERR_ARG;
    if (reinterpret_cast<uintptr_t>(d_stream) & 3u) return PQH_ERR_ARG;
    const size_t lds = (size_t)64 * chunk_vectors * t->m;
    if (lds > 160 * 1024) return PQH_ERR_UNSUPPORTED;
    int rc = pqh_use_device(ctx);
    if (rc) return rc;
    if (n == 0) return PQH_OK;
    const long long chunks = (n + chunk_vectors - 1) / chunk_vectors;
    if (lds > 64 * 1024)
        PQH_HIP(ctx, hipFuncSetAttribute((const void*)dec_tree,
                                         hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
    hipLaunchKernelGGL(dec_tree, dim3((unsigned)((chunks + 63) / 64)), dim3(64), lds, ctx->stream,
                       reinterpret_cast<const uint32_t*>(d_stream), (long long)((stream_bytes + 3) / 4),
                       n, t->m, t->k, chunk_vectors, d_chunk_offsets, d_parent_pos,
                       d_ext_offsets, d_ext_rows, t->d_lut1, t->d_lut2, t->d_meta, t->l1_bits,
                       t->lut2_cap, t->d_long, t->d_long_cnt, static_cast<uint8_t*>(d_rows),
                       ctx->d_diag + 1, stream_bytes * 8ull);
    PQH_LAUNCH_CHECK(ctx);
    return PQH_OK;
}
