// pqh_sort.hip -- the default sort mode of the reference encoder on the GPU.
//
// huffman_encoder.c:301-317 sorts the N code rows with qsort and a strncmp comparator over
// the M bytes of a row (glibc's qsort is a merge sort here, so the order is stable).
// strncmp stops at the first 0 byte, so the order is exactly a stable sort by
//     key(row) = the row's bytes, every byte after its first 0 cleared,
// compared as an unsigned big-endian byte string (verified by the oracle's
// orc_sort_rows against reference-built fixtures).
//
// GPU, 2 <= M <= 16 (the CLI's M = 8 and configs[3]'s M = 16 among them): a hand-written LSD
// radix sort, one pass per key byte, least significant first (stable passes compose into a
// stable sort by the whole key).  Each element is the row itself (one u64 word for M <= 8,
// two for M <= 16); a pass derives its key byte from the row (cleared past the row's first 0
// byte), so the first pass reads the codes and the last writes the sorted rows in place -- no
// index permutation and no gather.  One kernel counts the digits
// of the first pass's byte (`sort_digits`); each pass (`sort_pass`) is one kernel over
// 4,096-row tiles taken in ticket order: a wave ranks its rows among equal digits with 8
// ballots per 64 rows (stable: rows are ranked in index order), counts the next pass's
// digits, chains the workgroup's per-digit counts across tiles by a decoupled look-back (one
// lane per digit, 16 tiles per round), and scatters every row to digit base + earlier tiles
// + earlier waves + its rank.  Measured (1M x 8, alone): 0.25 ms, as the rocPRIM path
// (PQH_SORT_IMPL=rocprim); a pass is ~29 us, of which the look-back ~11 and the scatter ~8
// (PQH_SORT_DIAG timing runs).
// Other M (1, > 16): the same passes over (key chunk, row index) pairs -- LSD over 8-byte
// chunks of the key, least significant chunk first: `sort_chunk_keys` gathers each row's chunk
// (cleared past the row's first 0 byte) in the current order and counts its last byte, then
// one pass per byte of the chunk carries the pair -- and a final gather of the rows.
// (PQH_SORT_IMPL=rocprim: the same chunk order with rocPRIM pair sorts; a cross-check.)
#include <rocprim/device/device_radix_sort.hpp>

#include <algorithm>
#include <cstdlib>
#include <cstring>

#include "pqh_internal.h"

namespace {

// key chunk c of row idx[v] (bytes 8c .. 8c+7, big-endian, zeroed after the row's first 0)
__global__ void __launch_bounds__(256)
sort_keys(const uint8_t* __restrict__ codes, long long n, int m, int c,
          const uint32_t* __restrict__ idx, unsigned long long* __restrict__ keys) {
    const long long v = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (v >= n) return;
    const uint8_t* row = codes + (long long)(idx ? idx[v] : v) * m;
    int z = m;   // first zero byte
    for (int j = 0; j < m; ++j)
        if (row[j] == 0) {
            z = j;
            break;
        }
    unsigned long long key = 0;
#pragma unroll
    for (int q = 0; q < 8; ++q) {
        const int j = 8 * c + q;
        const unsigned long long b = (j < m && j <= z) ? row[j] : 0u;
        key |= b << (56 - 8 * q);
    }
    keys[v] = key;
}

__global__ void __launch_bounds__(256)
iota_u32(uint32_t* __restrict__ a, long long n) {
    const long long v = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (v < n) a[v] = (uint32_t)v;
}

__global__ void __launch_bounds__(256)
gather_rows(const uint8_t* __restrict__ src, long long n, int m, const uint32_t* __restrict__ idx,
            uint8_t* __restrict__ dst) {
    const long long v = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (v >= n) return;
    const uint8_t* a = src + (long long)idx[v] * m;
    uint8_t* b = dst + v * m;
    if ((m & 7) == 0) {
        for (int j = 0; j < m; j += 8)
            *reinterpret_cast<unsigned long long*>(b + j) =
                *reinterpret_cast<const unsigned long long*>(a + j);
    } else {
        for (int j = 0; j < m; ++j) b[j] = a[j];
    }
}

// ---------------------------------------------------------------- 2 <= m <= 8
#ifndef PQH_SORT_THREADS
#define PQH_SORT_THREADS 512
#endif
#ifndef PQH_SORT_ITEMS   // (8: 100 VGPRs, so a pass's waves fit beside two assignment waves;
#define PQH_SORT_ITEMS 8   //  16: 141 VGPRs -- the sort stage 0.40 vs 0.36 ms in the bench)
#endif
#ifndef PQH_SORT_WIN
#define PQH_SORT_WIN 16
#endif
constexpr int kSortThreads = PQH_SORT_THREADS;
constexpr int kSortWaves = kSortThreads / 64;
constexpr int kSortItems = PQH_SORT_ITEMS;                 // rows per lane
constexpr int kSortTile = kSortThreads * kSortItems;       // rows per workgroup (4,096)
constexpr int kLookWin = PQH_SORT_WIN;                     // tiles read per look-back round
constexpr unsigned long long kStAgg = 1ull << 46, kStPre = 1ull << 47;
constexpr unsigned long long kStVal = (1ull << 46) - 1;

// row v of the codes as W little-endian u64 words (byte j at bits 8 (j % 8) of word j / 8);
// bytes >= m are 0
template <int W>
__device__ __forceinline__ void sort_load_row(const uint8_t* __restrict__ codes, long long v, int m,
                                              unsigned long long* r) {
    if (W == 1 && m == 8) {
        r[0] = reinterpret_cast<const unsigned long long*>(codes)[v];
    } else if (W == 2 && m == 16) {
        const uint4 q = reinterpret_cast<const uint4*>(codes)[v];
        r[0] = (unsigned long long)q.x | ((unsigned long long)q.y << 32);
        r[1] = (unsigned long long)q.z | ((unsigned long long)q.w << 32);
    } else {
#pragma unroll
        for (int w = 0; w < W; ++w) r[w] = 0;
        for (int j = 0; j < m; ++j) r[j >> 3] |= (unsigned long long)codes[v * m + j] << (8 * (j & 7));
    }
}

// the index of the row's first 0 byte (W * 8 if none): the lowest flag of the zero-byte test
// is exact (only flags above a zero byte can be false)
template <int W>
__device__ __forceinline__ int sort_first_zero(const unsigned long long* r) {
    int z = 8 * W;
#pragma unroll
    for (int w = W - 1; w >= 0; --w) {
        const unsigned long long zb = (r[w] - 0x0101010101010101ull) & ~r[w] & 0x8080808080808080ull;
        if (zb) z = 8 * w + ((__ffsll((long long)zb) - 1) >> 3);
    }
    return z;
}

// key byte j of the row: its byte j while no 0 byte comes before it (strncmp stops there),
// else 0
template <int W>
__device__ __forceinline__ unsigned row_digit(const unsigned long long* r, int z, int j) {
    const unsigned b = (unsigned)(r[j >> 3] >> (8 * (j & 7))) & 0xFFu;
    return j <= z ? b : 0u;
}

// lanes (among `valid`) holding the same 8-bit value as this lane
__device__ __forceinline__ unsigned long long match_digit(unsigned d, bool valid) {
    unsigned long long match = __ballot(valid);
#pragma unroll
    for (int b = 0; b < 8; ++b) {
        const unsigned long long bal = __ballot((d >> b) & 1u);
        match &= ((d >> b) & 1u) ? bal : ~bal;
    }
    return match;
}

__device__ __forceinline__ uint32_t lanes_below(unsigned long long match) {
    return __builtin_amdgcn_mbcnt_hi((uint32_t)(match >> 32),
                                     __builtin_amdgcn_mbcnt_lo((uint32_t)match, 0u));
}

// digit counts of the first pass's byte position j (counts[256], zeroed by the caller); the
// passes count the next pass's byte as they go
template <int W>
__global__ void __launch_bounds__(256)
sort_digits(const uint8_t* __restrict__ codes, long long n, int m, int j, uint32_t* __restrict__ counts) {
    __shared__ uint32_t h[4][256];   // one histogram per wave
    for (int i = threadIdx.x; i < 4 * 256; i += blockDim.x) (&h[0][0])[i] = 0;
    lds_barrier();
    const int wave = threadIdx.x >> 6;
    constexpr int kPer = 8;   // rows per thread, loaded together
    for (long long v0 = (long long)blockIdx.x * blockDim.x * kPer + threadIdx.x; v0 < n;
         v0 += (long long)gridDim.x * blockDim.x * kPer) {
        unsigned long long row[kPer][W];
#pragma unroll
        for (int i = 0; i < kPer; ++i) {
            const long long v = v0 + (long long)i * blockDim.x;
#pragma unroll
            for (int w = 0; w < W; ++w) row[i][w] = 0;
            if (v < n) sort_load_row<W>(codes, v, m, row[i]);
        }
#pragma unroll
        for (int i = 0; i < kPer; ++i)
            if (v0 + (long long)i * blockDim.x < n)
                atomicAdd(&h[wave][row_digit<W>(row[i], sort_first_zero<W>(row[i]), j)], 1u);
    }
    lds_barrier();
    const uint32_t c = h[0][threadIdx.x] + h[1][threadIdx.x] + h[2][threadIdx.x] + h[3][threadIdx.x];
    if (c) atomicAdd(counts + threadIdx.x, c);
}

// the last pass's rows (W u64 words each) -> m bytes per row (m other than 8 and 16)
template <int W>
__global__ void __launch_bounds__(256)
sort_unpack(const unsigned long long* __restrict__ rows, long long n, int m, uint8_t* __restrict__ codes) {
    const long long v = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (v >= n) return;
    for (int q = 0; q < m; ++q) codes[v * m + q] = (uint8_t)(rows[v * W + (q >> 3)] >> (8 * (q & 7)));
}

// (pair passes) chunk c of row idx[v] as a little-endian word -- key byte q of the chunk at
// bits 8q, cleared past the row's first 0 byte -- and the digit counts of the chunk's last
// byte nb - 1 (counts[256], zeroed by the caller).  The first chunk (idx null) runs in row
// order: it writes the identity into idx_out and each row's first-0 position into zpos, which
// the later chunks' gathers use instead of rescanning the row.  W8: m % 8 == 0 and the codes
// 8-byte aligned (the chunk is one u64 load).
template <bool W8>
__global__ void __launch_bounds__(256)
sort_chunk_keys(const uint8_t* __restrict__ codes, long long n, int m, int c, int nb,
                const uint32_t* __restrict__ idx, uint32_t* __restrict__ idx_out,
                uint16_t* __restrict__ zpos, unsigned long long* __restrict__ keys,
                uint32_t* __restrict__ counts) {
    __shared__ uint32_t h[256];
    h[threadIdx.x] = 0;
    lds_barrier();
    const long long v = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    unsigned long long key = 0;
    if (v < n) {
        const long long r = idx ? (long long)idx[v] : v;
        const uint8_t* row = codes + r * m;
        int z;   // the row's first 0 byte (m if none)
        if (!idx) {
            idx_out[v] = (uint32_t)v;
            z = m;
            if (W8) {
                for (int w = 0; w < m / 8; ++w) {
                    const unsigned long long q = reinterpret_cast<const unsigned long long*>(row)[w];
                    const unsigned long long zb = (q - 0x0101010101010101ull) & ~q & 0x8080808080808080ull;
                    if (zb) {
                        z = 8 * w + ((__ffsll((long long)zb) - 1) >> 3);
                        break;
                    }
                }
            } else {
                for (int j = 0; j < m; ++j)
                    if (row[j] == 0) {
                        z = j;
                        break;
                    }
            }
            zpos[v] = (uint16_t)z;
        } else {
            z = zpos[r];
        }
        if (W8) {
            key = reinterpret_cast<const unsigned long long*>(row)[c];
        } else {
            key = 0;
            for (int q = 0; q < nb; ++q) key |= (unsigned long long)row[8 * c + q] << (8 * q);
        }
        // bytes 8c + q > z cleared
        const int keep = z - 8 * c + 1;   // bytes of the chunk kept
        if (keep <= 0) key = 0;
        else if (keep < 8) key &= (1ull << (8 * keep)) - 1;
        keys[v] = key;
    }
    // one LDS add per distinct digit of the wave (skewed codes share digits: a plain atomic
    // per lane serialises on the popular bins)
    const unsigned d = (unsigned)(key >> (8 * (nb - 1))) & 0xFFu;
    const unsigned long long match = match_digit(d, v < n);
    if (v < n && lanes_below(match) == 0) atomicAdd(&h[d], (uint32_t)__popcll(match));
    lds_barrier();
    if (h[threadIdx.x]) atomicAdd(counts + threadIdx.x, h[threadIdx.x]);
}

__device__ __forceinline__ void st_store(unsigned long long* p, unsigned long long v) {
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ unsigned long long st_load(const unsigned long long* p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// one stable counting pass by byte position j (digit counts of j in `counts`, the next
// pass's byte j - 1 counted into `counts_next`).  Elements are rows of W u64 words.  FIRST:
// rows come from the codes; LAST: the rows go to the codes (never both in one launch: m >= 2)
// IDX: elements are (key chunk, row index) pairs (W = 1, never FIRST): the chunk from rin /
// iin to rout / iout
template <bool FIRST, bool LAST, int W, bool IDX = false>
__global__ void __launch_bounds__(kSortThreads)
sort_pass(const uint8_t* __restrict__ codes_in, uint8_t* __restrict__ codes_out, long long n, int m,
          int j, const unsigned long long* __restrict__ rin, unsigned long long* __restrict__ rout,
          const uint32_t* __restrict__ counts, uint32_t* __restrict__ counts_next,
          unsigned long long* __restrict__ state, unsigned long long* __restrict__ ticket,
          unsigned long long ticket_base, unsigned epoch, int diag,
          const uint32_t* __restrict__ iin = nullptr, uint32_t* __restrict__ iout = nullptr) {
    static_assert(!IDX || (W == 1 && !FIRST), "pairs carry one key word");
    __shared__ uint32_t wcnt[kSortWaves][256];   // per-wave digit counters, then bases
    __shared__ uint32_t hnext[LAST ? 1 : 2][256];   // the next pass's digit counts
    __shared__ uint32_t wsum[4];
    __shared__ long long s_tile;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    if (tid == 0) s_tile = (long long)(atomicAdd(ticket, 1ull) - ticket_base);
    for (int i = tid; i < kSortWaves * 256; i += kSortThreads) (&wcnt[0][0])[i] = 0;
    if (!LAST)
        for (int i = tid; i < 2 * 256; i += kSortThreads) (&hnext[0][0])[i] = 0;
    lds_barrier();
    const long long tile = s_tile;
    const long long base = tile * kSortTile + (long long)wave * 64 * kSortItems;
    unsigned long long row[kSortItems][W];
    uint32_t rank[kSortItems];
    uint32_t id[IDX ? kSortItems : 1];   // (IDX) the pair's row index
    uint8_t dig[kSortItems];   // this pass's key byte of each row
    // every load first (the ranking below needs each key; issuing them all up front keeps
    // the tile's reads in flight together)
#pragma unroll
    for (int it = 0; it < kSortItems; ++it) {
        const long long v = base + it * 64 + lane;
#pragma unroll
        for (int w = 0; w < W; ++w) row[it][w] = 0;
        if (v < n) {
            if (FIRST) {
                sort_load_row<W>(codes_in, v, m, row[it]);
            } else if (W == 2) {
                const uint4 q = reinterpret_cast<const uint4*>(rin)[v];
                row[it][0] = (unsigned long long)q.x | ((unsigned long long)q.y << 32);
                row[it][W - 1] = (unsigned long long)q.z | ((unsigned long long)q.w << 32);
            } else {
                row[it][0] = rin[v];
                if constexpr (IDX) id[it] = iin[v];
            }
        }
    }
#pragma unroll
    for (int it = 0; it < kSortItems; ++it) {
        const bool valid = base + it * 64 + lane < n;
        const int z = sort_first_zero<W>(row[it]);
        if (!LAST && valid) atomicAdd(&hnext[wave & 1][row_digit<W>(row[it], z, j - 1)], 1u);
        // lanes with this lane's digit, among the valid ones, in lane order
        const unsigned d = row_digit<W>(row[it], z, j);
        dig[it] = (uint8_t)d;
        const unsigned long long match = match_digit(d, valid);
        const uint32_t below = lanes_below(match);
        // every lane reads the counter, then the group's lowest lane adds the group's size
        // (one wave: its LDS operations complete in order)
        const uint32_t old = wcnt[wave][d];
        if (valid && below == 0) wcnt[wave][d] = old + (uint32_t)__popcll(match);
        rank[it] = old + below;
    }
    lds_barrier();
    // one lane per digit (the first 4 waves): wave prefixes, the tile's count, the look-back
    // over earlier tiles (kLookWin of them per round), the digit base
    const unsigned dg = (unsigned)tid & 255u;
    uint32_t c[kSortWaves], tot = 0;
    unsigned long long excl = 0;
    uint32_t x = 0;
    if (tid < 256) {
#pragma unroll
        for (int w = 0; w < kSortWaves; ++w) {
            c[w] = wcnt[w][dg];
            tot += c[w];
        }
        if (!LAST) {
            const uint32_t hn = hnext[0][dg] + hnext[1][dg];
            if (hn) atomicAdd(counts_next + dg, hn);
        }
        unsigned long long* my = state + tile * 256 + dg;
        if (diag & 1) {
        } else if (tile == 0) {
            st_store(my, ((unsigned long long)epoch << 48) | kStPre | tot);
        } else {
            st_store(my, ((unsigned long long)epoch << 48) | kStAgg | tot);
            long long p = tile - 1;
            for (;;) {
                unsigned long long sw[kLookWin];
#pragma unroll
                for (int i = 0; i < kLookWin; ++i)
                    sw[i] = p - i >= 0 ? st_load(state + (p - i) * 256 + dg)
                                       : (((unsigned long long)epoch << 48) | kStPre);
                int i = 0;
                bool done = false;
                for (; i < kLookWin; ++i) {
                    const unsigned long long st = sw[i];
                    if ((unsigned)(st >> 48) != epoch || !(st & (kStAgg | kStPre))) break;
                    excl += st & kStVal;
                    if (st & kStPre) {
                        done = true;
                        break;
                    }
                }
                if (done) break;
                p -= i;
                if (i < kLookWin) __builtin_amdgcn_s_sleep(1);
            }
            st_store(my, ((unsigned long long)epoch << 48) | kStPre | (excl + tot));
        }
        x = counts[dg];
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const uint32_t y = __shfl_up(x, o);
            if (lane >= o) x += y;
        }
        if (lane == 63) wsum[wave] = x;
    }
    lds_barrier();   // (also: every wave has read its counters)
    if (tid < 256) {
        uint32_t gb = x - counts[dg];
        for (int w = 0; w < wave; ++w) gb += wsum[w];
        uint32_t run = gb + (uint32_t)excl;
#pragma unroll
        for (int w = 0; w < kSortWaves; ++w) {
            wcnt[w][dg] = run;
            run += c[w];
        }
    }
    lds_barrier();
    if (diag & 2) {   // (diagnostic: no scatter)
        if (rank[0] == 0xFFFFFFFFu) rout[0] = row[0][0] + row[kSortItems - 1][W - 1];
        return;
    }
#pragma unroll
    for (int it = 0; it < kSortItems; ++it) {
        const long long v = base + it * 64 + lane;
        if (v >= n) continue;
        long long dst = (long long)wcnt[wave][dig[it]] + rank[it];
        if (diag) dst = dst < n ? dst : n - 1;   // (diagnostic runs: bases are wrong, stay in range)
        // (the last pass writes 8- and 16-byte rows straight into the codes; other m go
        // through sort_unpack)
        unsigned long long* dstp = !IDX && LAST && m == 8 * W
                                       ? reinterpret_cast<unsigned long long*>(codes_out) : rout;
        if constexpr (IDX) iout[dst] = id[it];
        if (W == 2) {
            reinterpret_cast<uint4*>(dstp)[dst] =
                make_uint4((uint32_t)row[it][0], (uint32_t)(row[it][0] >> 32),
                           (uint32_t)row[it][W - 1], (uint32_t)(row[it][W - 1] >> 32));
        } else {
            dstp[dst] = row[it][0];
        }
    }
}

// the look-back's per-tile state for `tiles` tiles (grown on demand; tags are epochs)
int sort_state_for(pqh_ctx_t* ctx, long long tiles) {
    if (tiles > ctx->sort_cap) {
        PQH_HIP(ctx, hipStreamSynchronize(ctx->stream));   // no launch may still use it
        if (ctx->sort_state) (void)hipFree(ctx->sort_state);
        ctx->sort_state = nullptr;
        ctx->sort_cap = 0;
        const long long cap = tiles + tiles / 4 + 16;
        if (hipMalloc(&ctx->sort_state, (size_t)(cap * 256 + 1) * 8) != hipSuccess) {
            ctx->sort_state = nullptr;
            (void)hipGetLastError();
            return pqh_set_error(ctx, PQH_ERR_NOMEM, "sort: cannot allocate the tile state");
        }
        PQH_HIP(ctx, hipMemsetAsync(ctx->sort_state, 0, (size_t)(cap * 256 + 1) * 8, ctx->stream));
        ctx->sort_cap = cap;
        ctx->sort_epoch = 0;
        ctx->sort_ticket_base = 0;
    }
    return PQH_OK;
}

// the next pass's epoch (wrap: clear the tags)
int sort_next_epoch(pqh_ctx_t* ctx) {
    if (++ctx->sort_epoch >= 0xFFFF) {
        PQH_HIP(ctx, hipMemsetAsync(ctx->sort_state, 0, (size_t)ctx->sort_cap * 256 * 8, ctx->stream));
        ctx->sort_epoch = 1;
    }
    return PQH_OK;
}

int sort_diag() {   // PQH_SORT_DIAG (timing diagnostics only: wrong results)
    static const int diag = [] {
        const char* e = std::getenv("PQH_SORT_DIAG");
        return e ? std::atoi(e) : 0;
    }();
    return diag;
}

template <int W>
int sort_rows_radix(pqh_ctx_t* ctx, uint8_t* codes, long long n, int m) {
    const long long tiles = (n + kSortTile - 1) / kSortTile;
    int rc = sort_state_for(ctx, tiles);
    if (rc) return rc;
    auto al = [](size_t x) { return (x + 255) & ~(size_t)255; };
    const size_t eb = al((size_t)n * 8 * W);
    rc = pqh_ensure_ws(ctx, 2 * eb + al(16 * 256 * 4));
    if (rc) return rc;
    char* w = static_cast<char*>(ctx->ws);
    unsigned long long* r0 = reinterpret_cast<unsigned long long*>(w);
    unsigned long long* r1 = reinterpret_cast<unsigned long long*>(w + eb);
    uint32_t* dcnt = reinterpret_cast<uint32_t*>(w + 2 * eb);
    PQH_HIP(ctx, hipMemsetAsync(dcnt, 0, (size_t)m * 256 * 4, ctx->stream));
    const unsigned dgrid = (unsigned)std::min<long long>((n + 2047) / 2048, 1024);
    hipLaunchKernelGGL(sort_digits<W>, dim3(dgrid), dim3(256), 0, ctx->stream, codes, n, m, m - 1,
                       dcnt + (m - 1) * 256);
    PQH_LAUNCH_CHECK(ctx);
    unsigned long long* ticket = ctx->sort_state + ctx->sort_cap * 256;
    const int diag = sort_diag();
    for (int p = 0; p < m; ++p) {   // byte m - 1 first
        const int j = m - 1 - p;
        rc = sort_next_epoch(ctx);
        if (rc) return rc;
        const bool first = p == 0, last = p == m - 1;
        // (first: codes -> r0; middle: ping-pong; last: -> codes, or r0/r1 + unpack)
        const unsigned long long* rin = (p & 1) ? r0 : r1;
        unsigned long long* rout = (p & 1) ? r1 : r0;
#define PQH_SORT_PASS(F, L)                                                                       \
    hipLaunchKernelGGL((sort_pass<F, L, W>), dim3((unsigned)tiles), dim3(kSortThreads), 0,          \
                       ctx->stream, codes, codes, n, m, j, rin, rout, dcnt + j * 256,              \
                       dcnt + (j > 0 ? j - 1 : 0) * 256, ctx->sort_state, ticket,                  \
                       ctx->sort_ticket_base, ctx->sort_epoch, diag)
        if (first) PQH_SORT_PASS(true, false);
        else if (last) PQH_SORT_PASS(false, true);
        else PQH_SORT_PASS(false, false);
#undef PQH_SORT_PASS
        PQH_LAUNCH_CHECK(ctx);
        ctx->sort_ticket_base += (unsigned long long)tiles;
        if (last && m != 8 * W) {
            hipLaunchKernelGGL(sort_unpack<W>, dim3((unsigned)((n + 255) / 256)), dim3(256), 0,
                               ctx->stream, rout, n, m, codes);
            PQH_LAUNCH_CHECK(ctx);
        }
    }
    return PQH_OK;
}

// m = 1 or m > 16: (key chunk, index) pair passes, chunk by chunk from the last, then the rows
// gathered through the final permutation (into d_tmp or the workspace) and copied back
int sort_rows_pairs(pqh_ctx_t* ctx, uint8_t* codes, long long n, int m, void* d_tmp) {
    const long long tiles = (n + kSortTile - 1) / kSortTile;
    int rc = sort_state_for(ctx, tiles);
    if (rc) return rc;
    auto al = [](size_t x) { return (x + 255) & ~(size_t)255; };
    const size_t kb = al((size_t)n * 8), ib = al((size_t)n * 4), zb = al((size_t)n * 2);
    const size_t rb = d_tmp ? 0 : al((size_t)n * m);
    rc = pqh_ensure_ws(ctx, 2 * kb + 2 * ib + zb + al(8 * 256 * 4) + rb);
    if (rc) return rc;
    char* w = static_cast<char*>(ctx->ws);
    unsigned long long* kin = reinterpret_cast<unsigned long long*>(w);
    unsigned long long* kout = reinterpret_cast<unsigned long long*>(w + kb);
    uint32_t* iin = reinterpret_cast<uint32_t*>(w + 2 * kb);
    uint32_t* iout = reinterpret_cast<uint32_t*>(w + 2 * kb + ib);
    uint16_t* zpos = reinterpret_cast<uint16_t*>(w + 2 * kb + 2 * ib);
    uint32_t* dcnt = reinterpret_cast<uint32_t*>(w + 2 * kb + 2 * ib + zb);
    uint8_t* rows = d_tmp ? static_cast<uint8_t*>(d_tmp)
                          : reinterpret_cast<uint8_t*>(w + 2 * kb + 2 * ib + zb + al(8 * 256 * 4));
    const bool w8 = (m & 7) == 0 && (reinterpret_cast<uintptr_t>(codes) & 7) == 0;
    unsigned long long* ticket = ctx->sort_state + ctx->sort_cap * 256;
    const int diag = sort_diag();
    const unsigned blocks = (unsigned)((n + 255) / 256);
    const int chunks = (m + 7) / 8;
    for (int c = chunks - 1; c >= 0; --c) {   // least significant chunk first
        const int nb = std::min(8, m - 8 * c);
        PQH_HIP(ctx, hipMemsetAsync(dcnt, 0, 8 * 256 * 4, ctx->stream));
        // (first chunk: the identity order, written into iin)
        hipLaunchKernelGGL(w8 ? sort_chunk_keys<true> : sort_chunk_keys<false>, dim3(blocks),
                           dim3(256), 0, ctx->stream, codes, n, m, c, nb,
                           c == chunks - 1 ? nullptr : iin, iin, zpos, kin, dcnt + (nb - 1) * 256);
        PQH_LAUNCH_CHECK(ctx);
        for (int j = nb - 1; j >= 0; --j) {   // the chunk's last byte first
            rc = sort_next_epoch(ctx);
            if (rc) return rc;
#define PQH_SORT_PAIR_PASS(L)                                                                     \
    hipLaunchKernelGGL((sort_pass<false, L, 1, true>), dim3((unsigned)tiles), dim3(kSortThreads),  \
                       0, ctx->stream, codes, codes, n, m, j, kin, kout, dcnt + j * 256,           \
                       dcnt + (j > 0 ? j - 1 : 0) * 256, ctx->sort_state, ticket,                  \
                       ctx->sort_ticket_base, ctx->sort_epoch, diag, iin, iout)
            if (j == 0) PQH_SORT_PAIR_PASS(true);
            else PQH_SORT_PAIR_PASS(false);
#undef PQH_SORT_PAIR_PASS
            PQH_LAUNCH_CHECK(ctx);
            ctx->sort_ticket_base += (unsigned long long)tiles;
            std::swap(kin, kout);
            std::swap(iin, iout);
        }
    }
    hipLaunchKernelGGL(gather_rows, dim3(blocks), dim3(256), 0, ctx->stream, codes, n, m, iin, rows);
    PQH_LAUNCH_CHECK(ctx);
    PQH_HIP(ctx, hipMemcpyAsync(codes, rows, (size_t)n * m, hipMemcpyDeviceToDevice, ctx->stream));
    return PQH_OK;
}
}  // namespace

extern "C" {

int pqh_sort_rows(pqh_ctx_t* ctx, void* d_codes, long long n, int m, void* d_tmp) {
    if (!ctx || n < 0 || m <= 0 || (n > 0 && !d_codes)) return PQH_ERR_ARG;
    if (n >= (1ll << 32)) return pqh_set_error(ctx, PQH_ERR_UNSUPPORTED, "sort: n >= 2^32 rows");
    int rc = pqh_use_device(ctx);
    if (rc) return rc;
    if (n <= 1) return PQH_OK;
    static const bool force_lib = [] {
        const char* e = std::getenv("PQH_SORT_IMPL");
        return e && !std::strcmp(e, "rocprim");
    }();
    const uintptr_t addr = reinterpret_cast<uintptr_t>(d_codes);
    if (m >= 2 && m <= 16 && n < (1ll << 31) && !force_lib &&
        (m != 8 || (addr & 7) == 0) && (m != 16 || (addr & 15) == 0)) {
        rc = m <= 8 ? sort_rows_radix<1>(ctx, static_cast<uint8_t*>(d_codes), n, m)
                    : sort_rows_radix<2>(ctx, static_cast<uint8_t*>(d_codes), n, m);
        if (rc != PQH_ERR_NOMEM) return rc;
        // out of device memory for the in-tree sort's 16 (m <= 8) or 32 B/row: the rocPRIM
        // path below needs 24 B/row + its temp when the caller passes d_tmp
    } else if (n < (1ll << 31) && m < 65535 && !force_lib) {
        rc = sort_rows_pairs(ctx, static_cast<uint8_t*>(d_codes), n, m, d_tmp);
        if (rc != PQH_ERR_NOMEM) return rc;
    }
    // workspace: keys in/out (u64), index in/out (u32), rocPRIM temp, row buffer if no d_tmp
    size_t temp = 0;
    if (rocprim::radix_sort_pairs(nullptr, temp, (unsigned long long*)nullptr,
                                  (unsigned long long*)nullptr, (uint32_t*)nullptr,
                                  (uint32_t*)nullptr, (size_t)n, 0u, 64u, ctx->stream) != hipSuccess)
        return pqh_set_error(ctx, PQH_ERR_HIP, "sort: temp storage query failed");
    auto al = [](size_t x) { return (x + 255) & ~(size_t)255; };
    const size_t kb = al((size_t)n * 8), ib = al((size_t)n * 4), rb = d_tmp ? 0 : al((size_t)n * m);
    rc = pqh_ensure_ws(ctx, 2 * kb + 2 * ib + al(temp) + rb);
    if (rc) return rc;
    char* w = static_cast<char*>(ctx->ws);
    unsigned long long* k0 = reinterpret_cast<unsigned long long*>(w);
    unsigned long long* k1 = reinterpret_cast<unsigned long long*>(w + kb);
    uint32_t* i0 = reinterpret_cast<uint32_t*>(w + 2 * kb);
    uint32_t* i1 = reinterpret_cast<uint32_t*>(w + 2 * kb + ib);
    void* tmp = w + 2 * kb + 2 * ib;
    uint8_t* rows = d_tmp ? static_cast<uint8_t*>(d_tmp)
                          : reinterpret_cast<uint8_t*>(w + 2 * kb + 2 * ib + al(temp));
    const unsigned blocks = (unsigned)((n + 255) / 256);
    uint8_t* codes = static_cast<uint8_t*>(d_codes);
    hipLaunchKernelGGL(iota_u32, dim3(blocks), dim3(256), 0, ctx->stream, i0, n);
    PQH_LAUNCH_CHECK(ctx);
    const int passes = (m + 7) / 8;
    for (int c = passes - 1; c >= 0; --c) {   // least significant chunk first
        hipLaunchKernelGGL(sort_keys, dim3(blocks), dim3(256), 0, ctx->stream, codes, n, m, c, i0, k0);
        PQH_LAUNCH_CHECK(ctx);
        size_t tb = temp;
        PQH_HIP(ctx, rocprim::radix_sort_pairs(tmp, tb, k0, k1, i0, i1, (size_t)n, 0u, 64u,
                                               ctx->stream));
        std::swap(i0, i1);
    }
    hipLaunchKernelGGL(gather_rows, dim3(blocks), dim3(256), 0, ctx->stream, codes, n, m, i0, rows);
    PQH_LAUNCH_CHECK(ctx);
    PQH_HIP(ctx, hipMemcpyAsync(codes, rows, (size_t)n * m, hipMemcpyDeviceToDevice, ctx->stream));
    return PQH_OK;
}

}  // extern "C"
