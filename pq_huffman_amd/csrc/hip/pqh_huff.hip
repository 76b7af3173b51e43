// pqh_huff.hip -- symbol histograms, Huffman stream encode and chunked decode on gfx950.
//
//  hist_ctx / hist_plain   huffman_encoder.c:139-205 (collect_*_stats)
//  enc_size + scan         code-length pass: per 256-vector block bit totals, then an
//                          exclusive scan -> every block's bit offset (the serial bit
//                          cursor of bitstream.c:71-101 made parallel)
//  enc_write               encode_*_data (huffman_encoder.c:207-238): each block scans its
//                          per-vector lengths in LDS, ORs its codes into an LDS image of
//                          its bit range, stores interior words and ORs its two edge words
// (code tables and decode: pqh_tables.hip)
// Stream words are assembled MSB-first in 32-bit registers and byte-swapped on store, so
// memory holds exactly the bytes bitstream.c writes.
#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <thread>
#include <vector>

#include "pqh_internal.h"

namespace {

constexpr int kEncBlock = 512;   // vectors per encode workgroup (one thread each)
constexpr int kMaxCodeLen = 56;
constexpr int kHistChunk = 61440; // vectors per context-histogram workgroup (< 65536)

template <typename CodeT>
__device__ __forceinline__ unsigned ld_code(const CodeT* c, long long i) { return (unsigned)c[i]; }

// ---------------------------------------------------------------- histograms
// Multi-round workgroups (large inputs): a workgroup counts `rounds` consecutive chunks into
// the same u16-pair LDS image, so the partials are bounded by the grid, not by n.  A chunk
// adds at most kHistChunk counts, so the image cannot overflow while every counter starts a
// chunk at <= kHistCarry = 65535 - kHistChunk = 4095: between chunks each counter above that
// is added to the u32 accumulator `acc` (a memory-side global atomic) and cleared.  Each
// flush moves >= 4096 counts, so a chunk causes at most 15 of them per workgroup.
constexpr unsigned kHistCarry = 65535u - (unsigned)kHistChunk;
static_assert(kHistCarry == 4095u, "the flush test reads the top nibble of each u16");

__device__ __forceinline__ void hist_flush_carry(uint32_t* pairs, int words, unsigned base_bin,
                                                 int k, uint32_t* __restrict__ acc) {
    // The chunk's counts are in.  (lds_barrier's explicit wait matters: in the part-major
    // instance of hist_ctx_w the compiler put no lgkmcnt wait before a bare barrier here, so
    // another wave's last LDS atomics could land after this flush read the counter and be
    // overwritten by `keep` -- 64 or 128 counts of a hot pair lost on some runs.)
    lds_barrier();
    for (int w = threadIdx.x; w < words; w += blockDim.x) {
        const uint32_t x = pairs[w];
        if (!(x & 0xF000F000u)) continue;   // both halves <= 4095
        uint32_t keep = x;
        const unsigned bin = base_bin + 2u * (unsigned)w;
        if (x & 0xF000u) {
            atomicAdd(&acc[bin], x & 0xFFFFu);
            keep &= 0xFFFF0000u;
        }
        if (x & 0xF0000000u) {
            atomicAdd(&acc[bin + 1], x >> 16);
            keep &= 0xFFFFu;
        }
        pairs[w] = keep;   // (this thread owns the word between the barriers)
    }
    lds_barrier();
}

// Context histogram, pass 1: workgroup (chunk of kHistChunk vectors, part, prev-range z)
// counts its (prev, cur) pairs with prev in [z k / split, (z + 1) k / split) in LDS as u16
// pairs (a chunk cannot overflow 16 bits) and stores the packed counters as its slice of
// the chunk's private partial -- plain coalesced stores, no global atomics.  split = 2
// halves the LDS (64 KB at K = 256), so a workgroup fits on a CU beside the assignment's and
// the code-table builds' workgroups; every split re-reads the chunk's rows (L2 hits).
// The grid is 1-D and XCD-aware: workgroup L runs on XCD L % 8, and the m * split workgroups
// of a chunk all get L % 8 = chunk % 8, so the chunk's rows are fetched from HBM into one
// XCD's L2 once instead of once per XCD.
// BLK = 1024 threads (20 rows per load group), or 256 threads with 8-row groups: <= 32
// VGPRs and one wave per SIMD, so it fits on a CU beside the assignment grid's waves.
template <typename CodeT, int BLK = 1024, int kSub = 20>
__global__ void __launch_bounds__(BLK)
hist_ctx(const CodeT* __restrict__ codes, long long n, int m_total, int k,
         const CodeT* __restrict__ prev_row, const int* __restrict__ d_rawf,
         uint32_t* __restrict__ partial, int split, int chunks, int rounds,
         uint32_t* __restrict__ acc, int prio) {
    extern __shared__ uint32_t pairs[];   // (k / split) * k u16 counters packed two per word
    pqh_set_prio(prio);
    if (d_rawf && *d_rawf) prev_row = nullptr;   // decided on the device (pqh_shard_encode)
    const int per_chunk = m_total * split;
    const int q = (int)(blockIdx.x >> 3);
    // group g = chunks [g rounds, (g + 1) rounds), its partial image g
    const int groups = (chunks + rounds - 1) / rounds;
    const int grp = (q / per_chunk) * 8 + (int)(blockIdx.x & 7);
    if (grp >= groups) return;   // (uniform: the XCD's list is shorter)
    const int m = (q % per_chunk) / split;
    const int zs = q % split;
    const int prows = k / split;
    const unsigned plo = (unsigned)(zs * prows);
    const int all_words = (k * k + 1) / 2;
    const int words = split == 1 ? all_words : prows * k / 2;
#pragma clang loop unroll_count(4) vectorize(disable) interleave(disable)
    for (int w = threadIdx.x; w < words; w += blockDim.x) pairs[w] = 0;
    constexpr int kRun = kHistChunk / BLK;    // consecutive vectors per thread, taken kSub
    static_assert(kRun % kSub == 0 && kSub % 2 == 0, "whole 16-byte row pairs per group");
    const int c_end = min(chunks, (grp + 1) * rounds);
#pragma unroll 1
    for (int chunk = grp * rounds; chunk < c_end; ++chunk) {
    if (chunk > grp * rounds)   // the previous chunk's counters above the carry go to acc
        hist_flush_carry(pairs, words, (unsigned)m * (unsigned)(k * k) + plo * (unsigned)k, k, acc);
    const long long v0 = (long long)chunk * kHistChunk + (long long)threadIdx.x * kRun;
    auto count = [&](unsigned prev, unsigned cur) {
        if (prev >= (unsigned)k || cur >= (unsigned)k) return;   // absent / out of alphabet
        const unsigned pr = prev - plo;
        if (pr >= (unsigned)prows) return;                       // another split's range
        const unsigned bin = pr * (unsigned)k + cur;
        atomicAdd(&pairs[bin >> 1], 1u << ((bin & 1u) * 16));
    };
    unsigned prevc = v0 > 0 ? (v0 - 1 < n ? ld_code(codes, (v0 - 1) * m_total + m) : ~0u)
                            : (prev_row ? (unsigned)prev_row[m] : ~0u);
    const bool full = sizeof(CodeT) == 1 && v0 + kRun <= n;
    const bool wide = full && m_total == 8;
    // other part counts that are a multiple of 4 (configs[3]: M = 16): the dword of the row
    // that holds part m, kSub rows' dwords issued before their counter updates
    const bool dw = full && m_total != 8 && (m_total & 3) == 0 &&
                    (reinterpret_cast<uintptr_t>(codes) & 3) == 0;
    lds_barrier();   // the counters are zeroed (one barrier on every path: `wide` varies)
    if (dw) {
        const int rw = m_total >> 2;   // dwords per row
        const uint32_t* rows = reinterpret_cast<const uint32_t*>(codes) + v0 * rw + (m >> 2);
        const int sh = 8 * (m & 3);
#pragma unroll 1
        for (int g = 0; g < kRun / kSub; ++g) {
            uint32_t q[kSub];
#pragma unroll
            for (int u = 0; u < kSub; ++u) q[u] = rows[(long long)(g * kSub + u) * rw];
#pragma unroll
            for (int u = 0; u < kSub; ++u) {
                const unsigned c = (q[u] >> sh) & 0xFFu;
                count(prevc, c);
                prevc = c;
            }
        }
    } else if (wide) {
        // this thread's part-m codes of kSub consecutive rows per group, all of a group's
        // loads issued before its counter updates (8-byte rows of u8 codes: 16 B per load)
        const uint4* rows = reinterpret_cast<const uint4*>(codes + v0 * 8);
        const int sh = 8 * (m & 3);
#pragma unroll 1
        for (int g = 0; g < kRun / kSub; ++g) {
            uint4 q[kSub / 2];
#pragma unroll
            for (int u = 0; u < kSub / 2; ++u) q[u] = rows[g * (kSub / 2) + u];
#pragma unroll
            for (int u = 0; u < kSub / 2; ++u) {
                const unsigned a = m < 4 ? q[u].x : q[u].y, b = m < 4 ? q[u].z : q[u].w;
                const unsigned ca = (a >> sh) & 0xFFu, cb = (b >> sh) & 0xFFu;
                count(prevc, ca);
                count(ca, cb);
                prevc = cb;
            }
        }
    } else {
        for (int u = 0; u < kRun; ++u) {
            const long long v = v0 + u;
            const unsigned cur = v < n ? ld_code(codes, v * m_total + m) : ~0u;
            count(prevc, cur);
            prevc = cur;
        }
    }
    }   // chunk
    lds_barrier();
    uint32_t* out = partial + ((long long)m * groups + grp) * all_words + (long long)zs * words;
    if ((words & 3) == 0) {
        const uint4* src = reinterpret_cast<const uint4*>(pairs);
        uint4* dst = reinterpret_cast<uint4*>(out);
#pragma clang loop unroll_count(2) vectorize(disable) interleave(disable)
        for (int w = threadIdx.x; w < words / 4; w += blockDim.x) dst[w] = src[w];
    } else {
#pragma clang loop unroll(disable) vectorize(disable) interleave(disable)
        for (int w = threadIdx.x; w < words; w += blockDim.x) out[w] = pairs[w];
    }
}

// the value of lane l - 1 (lane 0: `first`), a DPP wave shift -- no LDS round trip
__device__ __forceinline__ unsigned wave_shr1(unsigned v, unsigned first) {
    return (unsigned)__builtin_amdgcn_update_dpp((int)first, (int)v, 0x138, 0xF, 0xF, false);
}

// Context histogram, pass 1, wave-contiguous form (u8 codes, m % 4 == 0, 4-byte aligned):
// same workgroups, LDS counters and partials as hist_ctx, but wave w of the workgroup counts
// the rows [w R, (w + 1) R) of the chunk in tiles of 64 (or, at m = 8, 128) consecutive rows,
// lane l holding row(s) l of the tile, so each load instruction covers 1 KB of consecutive
// rows (16 cache lines) instead of one line per lane; a row's predecessor is the previous
// lane's row (a DPP wave shift), the tile's first row's the previous tile's last (readlane).
// G tiles' loads are issued before their counter updates.
// ldc > 0: the codes are part-major ([m_total][ldc], pqh_pq_assign_parts): part m's rows are
// contiguous, so a lane's 4-byte load holds 4 consecutive rows (256 rows per wave load, no
// byte of another part read).
template <int BLK, int G, bool PM = false>
__global__ void __launch_bounds__(BLK)
hist_ctx_w(const uint8_t* __restrict__ codes, long long n, int m_total, int k,
           const uint8_t* __restrict__ prev_row, const int* __restrict__ d_rawf,
           uint32_t* __restrict__ partial, int split, int chunks, int rounds,
           uint32_t* __restrict__ acc, int prio, long long ldc_arg) {
    const long long ldc = PM ? ldc_arg : 0;   // (row-major instances: the old register budget)
    extern __shared__ uint32_t pairs[];   // (k / split) * k u16 counters packed two per word
    pqh_set_prio(prio);
    if (d_rawf && *d_rawf) prev_row = nullptr;   // decided on the device (pqh_shard_encode)
    const int per_chunk = m_total * split;
    const int q = (int)(blockIdx.x >> 3);
    // group g = chunks [g rounds, (g + 1) rounds), its partial image g
    const int groups = (chunks + rounds - 1) / rounds;
    const int grp = (q / per_chunk) * 8 + (int)(blockIdx.x & 7);
    if (grp >= groups) return;   // (uniform: the XCD's list is shorter)
    const int m = (q % per_chunk) / split;
    const int zs = q % split;
    const int prows = k / split;
    const unsigned plo = (unsigned)(zs * prows);
    const int all_words = (k * k + 1) / 2;
    const int words = split == 1 ? all_words : prows * k / 2;
#pragma clang loop unroll_count(4) vectorize(disable) interleave(disable)
    for (int w = threadIdx.x; w < words; w += blockDim.x) pairs[w] = 0;
    auto count = [&](unsigned prev, unsigned cur) {
        if (prev >= (unsigned)k || cur >= (unsigned)k) return;   // absent / out of alphabet
        const unsigned pr = prev - plo;
        if (pr >= (unsigned)prows) return;                       // another split's range
        const unsigned bin = pr * (unsigned)k + cur;
        atomicAdd(&pairs[bin >> 1], 1u << ((bin & 1u) * 16));
    };
    const int lane = threadIdx.x & 63;
    constexpr int kR = kHistChunk / (BLK / 64);   // rows per wave
    static_assert(kR % (128 * G) == 0, "whole tile groups per wave");
    // (uniform values through readfirstlane: SGPR bases, 32-bit per-lane offsets)
    const int wv = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
    const int sh = 8 * (m & 3);
    const int c_end = min(chunks, (grp + 1) * rounds);
    bool first = true;
#pragma unroll 1
    for (int chunk = grp * rounds; chunk < c_end; ++chunk) {
    if (!first)   // the previous chunk's counters above the carry go to acc
        hist_flush_carry(pairs, words, (unsigned)m * (unsigned)(k * k) + plo * (unsigned)k, k, acc);
    const long long w0 = (long long)chunk * kHistChunk + (long long)wv * kR;
    const int cnt = (int)max(0ll, min(n - w0, (long long)kR));   // rows this wave counts
    const uint8_t* const pm = codes + (long long)m * ldc;        // (ldc > 0) part m's codes
    unsigned carry = w0 > 0 ? (w0 - 1 < n ? (unsigned)(PM ? pm[w0 - 1] : codes[(w0 - 1) * m_total + m]) : ~0u)
                            : (prev_row ? (unsigned)prev_row[m] : ~0u);
    carry = (unsigned)__builtin_amdgcn_readfirstlane((int)carry);
    if (first) lds_barrier();   // the counters are zeroed
    first = false;
    if (PM && cnt == kR && !(reinterpret_cast<uintptr_t>(pm + w0) & 3)) {
        // part-major: lane l holds rows 4l .. 4l + 3 of a 256-row tile (one 4-byte load)
        static_assert(kR % (256 * G) == 0, "whole 256-row tile groups per wave");
        const uint32_t* p4 = reinterpret_cast<const uint32_t*>(pm + w0);
#pragma unroll 1
        for (int t0 = 0; t0 < kR / 256; t0 += G) {
            uint32_t v[G];
#pragma unroll
            for (int u = 0; u < G; ++u) v[u] = p4[(t0 + u) * 64 + lane];
#pragma unroll
            for (int u = 0; u < G; ++u) {
                const unsigned c0 = v[u] & 0xFFu, c1 = (v[u] >> 8) & 0xFFu,
                               c2 = (v[u] >> 16) & 0xFFu, c3 = v[u] >> 24;
                count(wave_shr1(c3, carry), c0);
                count(c0, c1);
                count(c1, c2);
                count(c2, c3);
                carry = (unsigned)__builtin_amdgcn_readlane((int)c3, 63);
            }
        }
    } else if (PM && cnt > 0) {
        // part-major, a partial or unaligned range: one row per lane
#pragma unroll 1
        for (int r0 = 0; r0 < cnt; r0 += 64) {
            const unsigned c = r0 + lane < cnt ? (unsigned)pm[w0 + r0 + lane] : ~0u;
            count(wave_shr1(c, carry), c);
            carry = (unsigned)__builtin_amdgcn_readlane((int)c, 63);
        }
    } else if (!PM && m_total == 8 && cnt == kR) {
        // two 8-byte rows per lane: one 16-byte load covers rows 2l, 2l + 1 of a 128-row tile
        const uint4* pr = reinterpret_cast<const uint4*>(codes + w0 * 8);
#pragma unroll 1
        for (int t0 = 0; t0 < kR / 128; t0 += G) {
            uint4 v[G];
#pragma unroll
            for (int u = 0; u < G; ++u) v[u] = pr[(t0 + u) * 64 + lane];
#pragma unroll
            for (int u = 0; u < G; ++u) {
                const unsigned a = m < 4 ? v[u].x : v[u].y, b = m < 4 ? v[u].z : v[u].w;
                const unsigned ca = (a >> sh) & 0xFFu, cb = (b >> sh) & 0xFFu;
                count(wave_shr1(cb, carry), ca);
                count(ca, cb);
                carry = (unsigned)__builtin_amdgcn_readlane((int)cb, 63);
            }
        }
    } else if (!PM && cnt > 0) {
        // one row per lane: the dword of row r that holds part m (rows past the wave's range
        // clamp their load and count nothing)
        const int rw = m_total >> 2;
        const uint32_t* c32 = reinterpret_cast<const uint32_t*>(codes + w0 * m_total) + (m >> 2);
#pragma unroll 1
        for (int r0 = 0; r0 < cnt; r0 += 64 * 2 * G) {
            uint32_t v[2 * G];
#pragma unroll
            for (int u = 0; u < 2 * G; ++u) v[u] = c32[min(r0 + u * 64 + lane, cnt - 1) * rw];
#pragma unroll
            for (int u = 0; u < 2 * G; ++u) {
                const unsigned c = r0 + u * 64 + lane < cnt ? (v[u] >> sh) & 0xFFu : ~0u;
                count(wave_shr1(c, carry), c);
                carry = (unsigned)__builtin_amdgcn_readlane((int)c, 63);
            }
        }
    }
    }   // chunk
    lds_barrier();
    uint32_t* out = partial + ((long long)m * groups + grp) * all_words + (long long)zs * words;
    if ((words & 3) == 0) {
        const uint4* src = reinterpret_cast<const uint4*>(pairs);
        uint4* dst = reinterpret_cast<uint4*>(out);
#pragma clang loop unroll_count(2) vectorize(disable) interleave(disable)
        for (int w = threadIdx.x; w < words / 4; w += blockDim.x) dst[w] = src[w];
    } else {
#pragma clang loop unroll(disable) vectorize(disable) interleave(disable)
        for (int w = threadIdx.x; w < words; w += blockDim.x) out[w] = pairs[w];
    }
}

// Context histogram, pass 2: counts[m][bin] += sum of the chunks' partials (one thread per
// packed word, so every counter has a single writer)
__global__ void __launch_bounds__(256)
hist_ctx_reduce(const uint32_t* __restrict__ partial, int chunks, int words, long long items,
                uint32_t* __restrict__ counts, int set, uint32_t* __restrict__ acc) {
    const int m = blockIdx.y;
    const int w = blockIdx.x * blockDim.x + threadIdx.x;
    if (w >= words) return;
    const uint32_t* p = partial + (long long)m * chunks * words + w;
    uint32_t lo = 0, hi = 0;
#pragma unroll 8
    for (int c = 0; c < chunks; ++c) {
        const uint32_t x = p[(long long)c * words];
        lo += x & 0xFFFFu;
        hi += x >> 16;
    }
    if (acc) {   // the multi-round form's carries; cleared for the next launch
        uint32_t* a = acc + (long long)m * items + 2 * w;
        lo += a[0];
        a[0] = 0;
        if (2 * w + 1 < items) {
            hi += a[1];
            a[1] = 0;
        }
    }
    uint32_t* out = counts + (long long)m * items;
    if (set) {   // every counter has exactly one writer: a plain store overwrites
        out[2 * w] = lo;
        if (2 * w + 1 < items) out[2 * w + 1] = hi;
    } else {
        if (lo) out[2 * w] += lo;
        if (hi && 2 * w + 1 < items) out[2 * w + 1] += hi;
    }
}

template <typename CodeT>
__global__ void __launch_bounds__(256)
hist_plain(const CodeT* __restrict__ codes, long long n, int m_total, int k,
           uint32_t* __restrict__ counts, long long ldc) {
    extern __shared__ uint32_t bins[];
    const int m = blockIdx.y;
    for (int i = threadIdx.x; i < k; i += blockDim.x) bins[i] = 0;
    lds_barrier();
    const long long per = (n + gridDim.x - 1) / gridDim.x;
    const long long v0 = (long long)blockIdx.x * per, v1 = min(n, v0 + per);
    for (long long v = v0 + threadIdx.x; v < v1; v += blockDim.x) {
        const unsigned c = ld_code(codes, ldc ? (long long)m * ldc + v : v * m_total + m);
        if (c < (unsigned)k) atomicAdd(&bins[c], 1u);
    }
    lds_barrier();
    for (int i = threadIdx.x; i < k; i += blockDim.x)
        if (bins[i]) atomicAdd(&counts[(long long)m * k + i], bins[i]);
}

// Non-context histogram of 8-part u16 rows (K > 256, configs[4]): a workgroup counts `rows`
// consecutive rows -- one 16-byte load per row, coalesced across the workgroup -- into u16
// pair counters for all 8 parts in LDS (8 x K/2 words: 64 KB at K = 4,096; a workgroup's
// rows stay below 65,536, so no counter overflows) and stores the image as its slice of the
// partials [part][group][K/2 words]; hist_ctx_reduce sums them.  (hist_plain flushed every
// non-zero bin of every workgroup by a global atomic: ~32 MB of atomic traffic per 1M rows
// for 128 KB of counts.)
__global__ void __launch_bounds__(256)
hist_plain_rows16(const uint16_t* __restrict__ codes, long long n, int k, long long rows,
                  uint32_t* __restrict__ partial, int groups) {
    extern __shared__ uint32_t bins[];   // [8][k / 2]
    const int words = k / 2;
    for (int w = threadIdx.x; w < 8 * words; w += blockDim.x) bins[w] = 0;
    lds_barrier();
    const long long r0 = (long long)blockIdx.x * rows, r1 = min(n, r0 + rows);
    const uint4* rp = reinterpret_cast<const uint4*>(codes);
    auto count = [&](uint32_t pair, int part) {
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            const unsigned c = h ? pair >> 16 : pair & 0xFFFFu;
            if (c < (unsigned)k) {
                const unsigned bin = (unsigned)(part + h) * (unsigned)k + c;
                atomicAdd(&bins[bin >> 1], 1u << ((bin & 1u) * 16));
            }
        }
    };
#pragma unroll 1
    for (long long r = r0 + threadIdx.x; r < r1; r += 4 * (long long)blockDim.x) {
        uint4 q[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) {   // four rows' loads in flight before their counts
            const long long rr = r + (long long)u * blockDim.x;
            q[u] = rr < r1 ? rp[rr] : make_uint4(~0u, ~0u, ~0u, ~0u);
        }
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            count(q[u].x, 0);
            count(q[u].y, 2);
            count(q[u].z, 4);
            count(q[u].w, 6);
        }
    }
    lds_barrier();
    for (int w = threadIdx.x; w < 8 * words; w += blockDim.x) {
        const int part = w / words, ww = w - part * words;
        partial[((long long)part * groups + blockIdx.x) * words + ww] = bins[w];
    }
}

// part-major codes [m][ldc] -> rows [n][m] (one thread per row: coalesced loads of each part,
// one 8- or 16-byte store per row where the row allows)
template <typename CodeT>
__global__ void __launch_bounds__(256)
transpose_codes(const CodeT* __restrict__ parts, long long ldc, long long n, int m,
                CodeT* __restrict__ rows) {
    const long long v = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (v >= n) return;
    if (sizeof(CodeT) == 1 && (m == 8 || m == 16)) {
        unsigned long long w[2] = {0, 0};
        for (int i = 0; i < m; ++i)
            w[i >> 3] |= (unsigned long long)(uint8_t)parts[(long long)i * ldc + v] << (8 * (i & 7));
        unsigned long long* d = reinterpret_cast<unsigned long long*>(rows) + v * (m / 8);
        d[0] = w[0];
        if (m == 16) d[1] = w[1];
    } else {
        for (int i = 0; i < m; ++i) rows[v * m + i] = parts[(long long)i * ldc + v];
    }
}

// ---------------------------------------------------------------- encode
// one symbol's (code, len): context row 0 of the stream is raw 8 bits (huffman_encoder.c:234)
template <typename CodeT>
__device__ __forceinline__ unsigned long long sym_entry(const CodeT* codes, long long v, int i,
                                                        int m_total, int k, int context,
                                                        int raw_first, const CodeT* prev_row,
                                                        const unsigned long long* enc,
                                                        long long items,
                                                        const uint16_t* tree_prev,
                                                        long long ldc = 0) {
    // (ldc > 0: part-major codes, part i of row v at i * ldc + v)
    auto at = [&](long long row) { return ld_code(codes, ldc ? (long long)i * ldc + row : row * m_total + i); };
    const unsigned s = at(v);
    if (s >= (unsigned)k) return 0;  // out-of-alphabet symbol: no code (length 0)
    if (!context) return enc[(long long)i * items + s];
    unsigned prev;
    if (tree_prev) {   // tree order: the row's context is its parent's code (0xFFFF: root)
        prev = tree_prev[v * m_total + i];
        if (prev == 0xFFFFu) return (8ull << 56) | (s & 0xFFu);
    } else if (v > 0) {
        prev = at(v - 1);
    } else if (!raw_first && prev_row) {
        prev = ld_code(prev_row, i);
    } else {
        return (8ull << 56) | (s & 0xFFu);
    }
    if (prev >= (unsigned)k) return 0;
    return enc[(long long)i * items + (long long)prev * k + s];
}

template <typename CodeT>
__global__ void __launch_bounds__(kEncBlock)
enc_size(const CodeT* __restrict__ codes, long long n, int m_total, int k, int context,
         int raw_first, const CodeT* __restrict__ prev_row, const int* __restrict__ d_rawf,
         const unsigned long long* __restrict__ enc,
         long long items, uint32_t* __restrict__ block_bits,
         const uint16_t* __restrict__ tree_prev) {
    __shared__ uint32_t red[kEncBlock / 64];
    if (d_rawf) raw_first = *d_rawf;   // decided on the device (pqh_shard_encode)
    const long long v = (long long)blockIdx.x * kEncBlock + threadIdx.x;
    uint32_t bits = 0;
    if (v < n)
        for (int i = 0; i < m_total; ++i)
            bits += (uint32_t)(sym_entry(codes, v, i, m_total, k, context, raw_first, prev_row,
                                         enc, items, tree_prev) >> 56);
    for (int off = 32; off >= 1; off >>= 1) bits += __shfl_xor(bits, off);
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = bits;
    lds_barrier();
    if (threadIdx.x == 0) {
        uint32_t s = 0;
        for (int w = 0; w < kEncBlock / 64; ++w) s += red[w];
        block_bits[blockIdx.x] = s;
    }
}

// Exclusive scan of nb block totals by one 256-thread workgroup (nb ~ n/256: 3,907 tiles at
// 1M rows, 488K at 125M).  Thread t owns the contiguous run [t*per, (t+1)*per): it sums its
// run, the 256 run sums are scanned once, then it writes its run's offsets.  Two passes over
// the totals and no per-element barriers; four waves fit beside the assignment grid, where a
// 1,024-thread workgroup waited for a whole CU's wave slots.
constexpr int kScanThreads = 256;
__global__ void __launch_bounds__(kScanThreads)
scan_blocks(const uint32_t* __restrict__ block_bits, long long nb,
            unsigned long long* __restrict__ block_off, unsigned long long* __restrict__ total) {
    __shared__ unsigned long long wsum[kScanThreads / 64];
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    const long long per = (nb + kScanThreads - 1) / kScanThreads;
    const long long lo = min(nb, per * threadIdx.x), hi = min(nb, lo + per);
    unsigned long long run = 0;
#pragma unroll 8
    for (long long i = lo; i < hi; ++i) run += block_bits[i];
    unsigned long long incl = run;
    for (int off = 1; off < 64; off <<= 1) {
        const unsigned long long y = __shfl_up(incl, off);
        if (lane >= off) incl += y;
    }
    if (lane == 63) wsum[wid] = incl;
    lds_barrier();
    unsigned long long acc = incl - run;
    for (int w = 0; w < wid; ++w) acc += wsum[w];
    if (threadIdx.x == kScanThreads - 1) *total = acc + run;
#pragma unroll 8
    for (long long i = lo; i < hi; ++i) {
        block_off[i] = acc;
        acc += block_bits[i];
    }
}

// Large inputs (more than kScanOneWg counts: past 4.2M rows of 256-row tiles) scan in two
// launches of one workgroup per segment of kScanSeg counts, all loads coalesced:
// scan_seg_sums writes each segment's sum; scan_seg_write adds up the sums before its
// segment (at most a few thousand) and scans its own segment, 16 consecutive counts per
// thread.  (One workgroup at 125M rows -- 488K counts, 1,907 per thread -- took 0.9 ms.)
constexpr int kScanSeg = 16 * kScanThreads;
constexpr long long kScanOneWg = 16384;
__global__ void __launch_bounds__(kScanThreads)
scan_seg_sums(const uint32_t* __restrict__ bits, long long nb,
              unsigned long long* __restrict__ seg_sum) {
    __shared__ unsigned long long wsum[kScanThreads / 64];
    const long long base = (long long)blockIdx.x * kScanSeg;
    unsigned long long v = 0;
#pragma unroll 4
    for (int i = threadIdx.x; i < kScanSeg; i += kScanThreads) {
        const long long j = base + i;
        v += j < nb ? bits[j] : 0u;
    }
    for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o);
    if ((threadIdx.x & 63) == 0) wsum[threadIdx.x >> 6] = v;
    lds_barrier();
    if (threadIdx.x == 0) {
        unsigned long long t = 0;
        for (int w = 0; w < kScanThreads / 64; ++w) t += wsum[w];
        seg_sum[blockIdx.x] = t;
    }
}

__global__ void __launch_bounds__(kScanThreads)
scan_seg_write(const uint32_t* __restrict__ bits, long long nb,
               const unsigned long long* __restrict__ seg_sum,
               unsigned long long* __restrict__ block_off, unsigned long long* __restrict__ total) {
    __shared__ unsigned long long wsum[kScanThreads / 64];
    __shared__ unsigned long long s_base;
    const int seg = (int)blockIdx.x;
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    unsigned long long b = 0;   // the segments before this one
    for (int i = threadIdx.x; i < seg; i += kScanThreads) b += seg_sum[i];
    for (int o = 32; o >= 1; o >>= 1) b += __shfl_xor(b, o);
    if (lane == 0) wsum[wid] = b;
    lds_barrier();
    if (threadIdx.x == 0) {
        unsigned long long t = 0;
        for (int w = 0; w < kScanThreads / 64; ++w) t += wsum[w];
        s_base = t;
    }
    lds_barrier();
    const long long j0 = (long long)seg * kScanSeg + 16ll * threadIdx.x;
    uint32_t v[16];
    if (j0 + 16 <= nb) {   // (16-count runs are 64-byte aligned)
        const uint4* p = reinterpret_cast<const uint4*>(bits + j0);
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const uint4 x = p[q];
            v[4 * q] = x.x; v[4 * q + 1] = x.y; v[4 * q + 2] = x.z; v[4 * q + 3] = x.w;
        }
    } else {
#pragma unroll
        for (int i = 0; i < 16; ++i) v[i] = j0 + i < nb ? bits[j0 + i] : 0u;
    }
    unsigned long long run = 0;
#pragma unroll
    for (int i = 0; i < 16; ++i) run += v[i];
    unsigned long long incl = run;
    for (int o = 1; o < 64; o <<= 1) {
        const unsigned long long y = __shfl_up(incl, o);
        if (lane >= o) incl += y;
    }
    if (lane == 63) wsum[wid] = incl;
    lds_barrier();
    unsigned long long acc = s_base + incl - run;
    for (int w = 0; w < wid; ++w) acc += wsum[w];
#pragma unroll
    for (int i = 0; i < 16; ++i) {
        if (j0 + i < nb) block_off[j0 + i] = acc;
        acc += v[i];
    }
    if (seg == (int)gridDim.x - 1 && threadIdx.x == kScanThreads - 1) *total = acc;
}

// the exclusive scan of nb counts and their total; seg: ceil(nb / kScanSeg) u64 of scratch
static void launch_scan(hipStream_t st, const uint32_t* bits, long long nb,
                        unsigned long long* off, unsigned long long* total,
                        unsigned long long* seg) {
    if (nb <= kScanOneWg) {
        hipLaunchKernelGGL(scan_blocks, dim3(1), dim3(kScanThreads), 0, st, bits, nb, off, total);
        return;
    }
    const unsigned nseg = (unsigned)((nb + kScanSeg - 1) / kScanSeg);
    hipLaunchKernelGGL(scan_seg_sums, dim3(nseg), dim3(kScanThreads), 0, st, bits, nb, seg);
    hipLaunchKernelGGL(scan_seg_write, dim3(nseg), dim3(kScanThreads), 0, st, bits, nb, seg, off,
                       total);
}

__device__ __forceinline__ uint32_t bswap32(uint32_t x) { return __builtin_bswap32(x); }

// Inclusive wave64 scan of u32 with DPP row shifts and row broadcasts (no LDS permutes, no
// lane-address registers): rows of 16 scan by row_shr 1/2/4/8, then row 15's / 31's
// totals are broadcast into the rows after them.
__device__ __forceinline__ uint32_t wave_incl_scan(uint32_t v) {
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x111, 0xF, 0xF, false);   // row_shr:1
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x112, 0xF, 0xF, false);   // row_shr:2
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x114, 0xF, 0xF, false);   // row_shr:4
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x118, 0xF, 0xF, false);   // row_shr:8
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x142, 0xA, 0xF, false);   // row_bcast:15
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x143, 0xC, 0xF, false);   // row_bcast:31
    return v;
}

// decoupled look-back state words: epoch (16 bits) | status (2) | value (46)
constexpr unsigned long long kLbAgg = 1ull << 46, kLbPrefix = 2ull << 46;
constexpr unsigned long long kLbValue = (1ull << 46) - 1;
__device__ __forceinline__ unsigned long long lb_pack(unsigned epoch, unsigned long long status,
                                                      unsigned long long v) {
    return ((unsigned long long)epoch << 48) | status | v;
}
// Every value handed between workgroups travels inside the 64-bit atomic word itself, so
// relaxed agent-scope atomics suffice (coherent sc1 accesses): release/acquire would add a
// whole-L2 writeback (buffer_wbl2) per publish and an L2 invalidate (buffer_inv) per poll.
__device__ __forceinline__ void lb_store(unsigned long long* p, unsigned long long v) {
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ unsigned long long lb_load(const unsigned long long* p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// tail word of a block: epoch | ready (bit 32) | the word's bits from blocks <= it
__device__ __forceinline__ uint32_t lb_wait_tail(const unsigned long long* tails, long long b,
                                                 unsigned epoch) {
    for (;;) {
        const unsigned long long t = lb_load(tails + b);
        if ((unsigned)(t >> 48) == epoch && (t >> 32 & 1ull)) return (uint32_t)t;
        __builtin_amdgcn_s_sleep(1);
    }
}

// m codes of row v (MAXM >= m) with wide loads when the row is 8-byte aligned
template <typename CodeT, int MAXM>
__device__ __forceinline__ void load_row(const CodeT* __restrict__ codes, long long v, int m,
                                         unsigned (&out)[MAXM]) {
    const CodeT* row = codes + v * m;
    if (m * (int)sizeof(CodeT) == 8 * ((m * (int)sizeof(CodeT)) / 8) &&
        !(reinterpret_cast<uintptr_t>(row) & 7)) {
        constexpr int per = 8 / sizeof(CodeT);
        unsigned long long w[(MAXM * sizeof(CodeT) + 7) / 8];
#pragma unroll
        for (int q = 0; q < (MAXM * (int)sizeof(CodeT) + 7) / 8; ++q)
            w[q] = q * 8 < m * (int)sizeof(CodeT) ? reinterpret_cast<const unsigned long long*>(row)[q] : 0ull;
#pragma unroll
        for (int i = 0; i < MAXM; ++i)
            out[i] = (unsigned)((w[i / per] >> (8 * sizeof(CodeT) * (i % per))) &
                                ((1ull << (8 * sizeof(CodeT))) - 1));
    } else {
#pragma unroll
        for (int i = 0; i < MAXM; ++i) out[i] = i < m ? (unsigned)row[i] : 0u;
    }
}

// The m table entries of vector v as the u32 gather copy (len << 26 | code; ~0u = a code
// longer than 26 bits, read from the u64 table when it is emitted), all loads issued together
// (huffman_encoder.c:207-238: context index (prev << 8) + cur; context row 0 raw 8 bits).
// u32 entries keep a vector's m entries in m registers, not 2m.
template <typename CodeT, int MAXM>
__device__ __forceinline__ void gather_entries(const CodeT* __restrict__ codes, long long v, int m,
                                               int k, int context, int raw_first,
                                               const CodeT* __restrict__ prev_row,
                                               const uint32_t* __restrict__ enc32,
                                               long long items, uint32_t (&e32)[MAXM],
                                               const uint16_t* __restrict__ tree_prev) {
    unsigned cur[MAXM], prv[MAXM];
    load_row<CodeT, MAXM>(codes, v, m, cur);
    bool raw = context && v == 0 && (raw_first || !prev_row);
    if (tree_prev) {   // tree order: explicit parent row (0xFFFF in part 0: a root, raw)
        load_row<uint16_t, MAXM>(tree_prev, v, m, prv);
        raw = prv[0] == 0xFFFFu;
    } else if (context && v > 0) {
        load_row<CodeT, MAXM>(codes, v - 1, m, prv);
    } else {
#pragma unroll
        for (int i = 0; i < MAXM; ++i) prv[i] = (context && prev_row && i < m) ? (unsigned)prev_row[i] : 0u;
    }
#pragma unroll
    for (int i = 0; i < MAXM; ++i) {
        const bool ok = i < m && cur[i] < (unsigned)k && (!context || prv[i] < (unsigned)k) && !raw;
        const long long idx = i * items + (context ? (long long)prv[i] * k + cur[i] : (long long)cur[i]);
        e32[i] = ok ? enc32[idx] : 0u;
    }
    if (raw) {
#pragma unroll
        for (int i = 0; i < MAXM; ++i) e32[i] = i < m ? ((8u << 26) | (cur[i] & 0xFFu)) : 0u;
    }
}

// One-pass encoder (huffman_encoder.c:207-238 + the bit cursor of bitstream.c:71-101).
// Workgroups take tickets in launch order (so every predecessor has started), sum their
// kEncBlock vectors' code lengths, and find their bit offset by a decoupled look-back over the
// predecessors' published aggregates / prefixes.  Each workgroup ORs its codes into an LDS
// image of its bit range and stores every word it owns exactly once: the word it shares with
// its successor is published as a "tail" instead, and the successor merges it into its own
// first word.  So no word is written twice, nothing needs zeroing and no global atomics are
// used; the call's first word is merged with the memory content when bit_offset is not
// word-aligned (shards composed into one buffer).  MAXM > 0 keeps the m table entries of a
// vector in registers (m <= MAXM).  (Diagnostics: g_enc_stamps holds s_memtime phase
// stamps of the mid-grid workgroup, read by pqh_debug_enc_stamps.)
__device__ unsigned long long g_enc_stamps[8];

//
// TILE = true (the default encoder, see encode_write_impl): the same kernel without any
// inter-workgroup waiting.  Workgroup `id` = blockIdx.x codes tile id of the input into its
// LDS image starting at bit 0, stores the image's words whole into its slot of the scratch
// (out_words + id * cap_words, cap_words = the slot's words, a tile's worst case), its bit
// count into tile_bits[id] (`state` as u32) and its chunk offsets relative to the tile; a
// scan of the tile counts and enc_place then put every tile at its offset.
template <typename CodeT, int MAXM, int BLK, bool ROW8 = false, int CS = 1, bool PM = false,
          bool TILE = false>
__global__ void __launch_bounds__(BLK)
enc_onepass(const CodeT* __restrict__ codes, long long n, int m_total, int k, int context,
            int raw_first, const CodeT* __restrict__ prev_row, const int* __restrict__ d_rawf,
            const unsigned long long* __restrict__ enc, const uint32_t* __restrict__ enc32,
            const uint16_t* __restrict__ enc16, long long items,
            unsigned long long bit_offset_arg,
            const unsigned long long* __restrict__ d_bit_offset,
            uint32_t* __restrict__ out_words, long long cap_words,
            int chunk_vectors, unsigned long long* __restrict__ chunk_off,
            CodeT* __restrict__ chunk_prev, unsigned long long* __restrict__ err,
            unsigned long long* __restrict__ state, unsigned long long* __restrict__ tails,
            unsigned long long* __restrict__ ticket, unsigned long long ticket_base,
            unsigned epoch, long long nb, unsigned long long* __restrict__ total_out,
            const uint16_t* __restrict__ tree_prev, int prio, long long ldc_arg) {
    const long long ldc = PM ? ldc_arg : 0;   // (row-major instances: the old register budget)
    // ROW8: n counts 8-byte rows of 8 u8 codes, CS of them per vector (m_total = 8 CS: a
    // 16-part vector is two consecutive 8-part rows, which are also consecutive in the
    // stream); a row's context row is CS rows back and its parts are (row % CS) * 8 + i.
    // ldc > 0 (ROW8 only): the codes are part-major [m_total][ldc]; a row is gathered from
    // its 8 parts' runs (coalesced byte loads across the wave's consecutive rows).
    auto row8_at = [&](long long vec, unsigned hf) -> unsigned long long {
        if (!PM) return reinterpret_cast<const unsigned long long*>(codes)[vec * CS + hf];
        unsigned long long r = 0;
#pragma unroll
        for (int i = 0; i < 8; ++i)
            r |= (unsigned long long)(uint8_t)codes[(long long)(hf * 8 + i) * ldc + vec] << (8 * i);
        return r;
    };
    extern __shared__ uint32_t img[];   // LDS image of this block's bit range
    pqh_set_prio(prio);
    __shared__ uint32_t wsum[BLK / 64];
    __shared__ long long s_id;
    __shared__ unsigned long long s_excl;
    __shared__ uint32_t s_head;
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    if (d_rawf) raw_first = *d_rawf;   // decided on the device (pqh_shard_encode)
    // d_bit_offset: the shard's GLOBAL bit offset, produced on the device (multi-GPU, no host
    // round trip); the shard's own buffer starts at its word, so only offset % 32 matters
    const unsigned long long bit_offset =
        TILE ? 0ull : d_bit_offset ? (*d_bit_offset & 31ull) : bit_offset_arg;
    if constexpr (!TILE) {
        if (tid == 0) s_id = (long long)(atomicAdd(ticket, 1ull) - ticket_base);
        lds_barrier();
    }
    const long long id = TILE ? (long long)blockIdx.x : s_id;
    const long long v = id * BLK + tid;
    const bool stamp = id == nb / 2 && tid == 0;
    if (stamp) g_enc_stamps[0] = __builtin_amdgcn_s_memtime();

    // code entries of this vector (gathered once)
    uint32_t ent[MAXM > 0 ? MAXM : 1];
    uint32_t bits = 0;
    if constexpr (ROW8) tree_prev = nullptr;   // (the 8-byte-row path: no tree order)
    if (v < n) {
        if constexpr (ROW8) {
            // m = 8 u8 codes: the row (and its context row) is one 8-byte load; entry loads
            // are a uniform base plus a 32-bit offset (m * items * 4 B < 4 GB)
            static_assert(MAXM == 8 && sizeof(CodeT) == 1, "8-byte rows");
            const unsigned half = (unsigned)(v % CS);   // (CS = 1: 0)
            const unsigned long long row = row8_at(v / CS, half);
            unsigned long long prow = 0;
            bool raw = false;
            if (context) {
                if (v >= CS) {
                    prow = row8_at(v / CS - 1, half);
                } else if (!raw_first && prev_row) {
#pragma unroll
                    for (int i = 0; i < 8; ++i)
                        prow |= (unsigned long long)prev_row[half * 8 + i] << (8 * i);
                } else {
                    raw = true;   // row 0 raw, 8 bits per part (huffman_encoder.c:234)
                }
            }
            const unsigned ibase = half * 8u * (unsigned)items;
#pragma unroll
            for (int i = 0; i < 8; ++i) {
                const unsigned cur = (unsigned)(row >> (8 * i)) & 0xFFu;
                const unsigned prv = (unsigned)(prow >> (8 * i)) & 0xFFu;
                const bool ok = cur < (unsigned)k && (!context || prv < (unsigned)k);
                const unsigned idx = ibase + (unsigned)i * (unsigned)items + (context ? prv * (unsigned)k + cur : cur);
                // the u16 copy first (half the table bytes in L2), the u32 entry only for
                // codes longer than 12 bits (escape 0xFFFF)
                if (enc16) {
                    const uint32_t h = ok ? (uint32_t)enc16[idx] : 0u;
                    ent[i] = raw ? ((8u << 26) | cur)
                                 : h != 0xFFFFu ? ((h >> 12) << 26) | (h & 0xFFFu) : enc32[idx];
                } else {   // (PQH_ENC16=0: the u32 copy only)
                    ent[i] = raw ? ((8u << 26) | cur) : ok ? enc32[idx] : 0u;
                }
            }
#pragma unroll
            for (int i = 0; i < 8; ++i)
                bits += ent[i] != ~0u ? ent[i] >> 26
                                      : (uint32_t)(sym_entry(codes, v / CS, (int)half * 8 + i,
                                                             8 * CS, k, context, raw_first,
                                                             prev_row, enc, items, nullptr,
                                                             ldc) >> 56);
        } else if constexpr (MAXM > 0) {
            gather_entries<CodeT, MAXM>(codes, v, m_total, k, context, raw_first, prev_row,
                                        enc32, items, ent, tree_prev);
#pragma unroll
            for (int i = 0; i < MAXM; ++i)
                bits += ent[i] != ~0u ? ent[i] >> 26
                                      : (uint32_t)(sym_entry(codes, v, i, m_total, k, context,
                                                             raw_first, prev_row, enc, items,
                                                             tree_prev) >> 56);
        } else {
            for (int i = 0; i < m_total; ++i)
                bits += (uint32_t)(sym_entry(codes, v, i, m_total, k, context, raw_first,
                                             prev_row, enc, items, tree_prev) >> 56);
        }
    }
    const uint32_t incl = wave_incl_scan(bits);
    if (lane == 63) wsum[wid] = incl;
    lds_barrier();
    if (stamp) g_enc_stamps[1] = __builtin_amdgcn_s_memtime();
    uint32_t before = 0, block_bits = 0;
    for (int w = 0; w < BLK / 64; ++w) {
        before += w < wid ? wsum[w] : 0u;
        block_bits += wsum[w];
    }
    // decoupled look-back, one wave wide: lane l inspects predecessor p - l; the walk stops
    // at the nearest published inclusive prefix, adding the aggregates in front of it
    // (TILE: none -- the tile starts at its own bit 0)
    if (TILE) {
        if (tid == 0) {
            s_excl = 0;
            reinterpret_cast<uint32_t*>(state)[id] = block_bits;
        }
    } else if (wid == 0) {
        unsigned long long excl = 0;
        if (id == 0) {
            if (lane == 0) lb_store(state, lb_pack(epoch, kLbPrefix, block_bits));
        } else {
            if (lane == 0) lb_store(state + id, lb_pack(epoch, kLbAgg, block_bits));
            long long p = id - 1;
            for (;;) {
                const long long q = p - lane;
                const unsigned long long st = q >= 0 ? lb_load(state + q) : lb_pack(epoch, kLbPrefix, 0);
                const bool ready = (unsigned)(st >> 48) == epoch && (st & (3ull << 46));
                const unsigned long long pref = __ballot(ready && (st & kLbPrefix));
                const unsigned long long notready = __ballot(!ready);
                // lanes up to the nearest prefix (or all 64) must be ready
                const int f = pref ? __ffsll((long long)pref) - 1 : 63;
                const unsigned long long need = f == 63 ? ~0ull : ((2ull << f) - 1);
                if (notready & need) {
                    __builtin_amdgcn_s_sleep(1);
                    continue;
                }
                // the aggregates before the prefix lane (block totals: < 2^23 for 64 of them)
                // summed in 32 bits, the prefix itself read from its lane
                const uint32_t a = (!pref || lane < f) ? (uint32_t)(st & kLbValue) : 0u;
                excl += (uint32_t)__builtin_amdgcn_readlane((int)wave_incl_scan(a), 63);
                if (pref) {
                    const unsigned long long lo = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)st, f);
                    const unsigned long long hi = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(st >> 32), f);
                    excl += ((hi << 32) | lo) & kLbValue;
                    break;
                }
                p -= 64;
            }
            if (lane == 0) lb_store(state + id, lb_pack(epoch, kLbPrefix, excl + block_bits));
        }
        if (lane == 0) s_excl = excl;
    }
    lds_barrier();
    if (stamp) g_enc_stamps[2] = __builtin_amdgcn_s_memtime();
    const unsigned long long bs = bit_offset + s_excl, be = bs + block_bits;
    const long long wa = (long long)(bs >> 5);
    const long long wz = block_bits ? (long long)((be - 1) >> 5) : wa;
    const long long nwords = block_bits ? wz - wa + 1 : 0;
    const bool head_pred = (bs & 31) && bs > bit_offset;    // earlier blocks' bits in word wa
    const bool head_mem = (bs & 31) && bs == bit_offset;    // the caller's bits in word wa
    const bool overflow = nwords > 0 && wz >= cap_words;
    for (long long w = tid; w < nwords; w += BLK) img[w] = 0;
    lds_barrier();

    unsigned long long pos = bs + before + incl - bits;
    if (v < n) {
        const long long vv = ROW8 ? v / CS : v;   // the vector
        if (chunk_vectors > 0 && (!ROW8 || v % CS == 0) && vv % chunk_vectors == 0) {
            const long long j = vv / chunk_vectors;
            chunk_off[j] = pos;
            if (context && chunk_prev) {
                if (ROW8 && vv > 0) {   // (chunk_prev rows are 8 CS bytes: aligned)
                    for (int q = 0; q < CS; ++q)
                        reinterpret_cast<unsigned long long*>(chunk_prev)[j * CS + q] =
                            row8_at(vv - 1, (unsigned)q);
                } else {
                    for (int i = 0; i < m_total; ++i)
                        chunk_prev[j * m_total + i] =
                            vv > 0 ? codes[(vv - 1) * m_total + i] : (prev_row ? prev_row[i] : (CodeT)0);
                }
            }
        }
        // assemble this vector's bits in registers: words wholly inside its range are
        // plain LDS stores (no other thread touches them); only the first and the last,
        // shared with the neighbouring vectors, are OR-ed
        long long w = (long long)(pos >> 5) - wa;
        unsigned long long acc = 0;   // pending bits, right-aligned
        int nacc = (int)(pos & 31);   // (the bits before `pos` in the first word are zeros)
        bool first = true;
        auto emit = [&](uint32_t word) {
            if (first) atomicOr(&img[w], word);
            else img[w] = word;
            first = false;
            ++w;
        };
        auto append = [&](unsigned long long code, int len) {   // len <= 32
            acc = (acc << len) | code;
            nacc += len;
            if (nacc >= 32) {
                emit((uint32_t)(acc >> (nacc - 32)));
                nacc -= 32;
                acc &= (1ull << nacc) - 1;
            }
        };
        auto put = [&](unsigned long long e) {
            const int len = (int)(e >> 56);
            const unsigned long long code = e & ((1ull << 56) - 1);
            if (len > 32) {
                append(code >> 32, len - 32);
                append(code & 0xFFFFFFFFull, 32);
            } else if (len > 0) {
                append(code, len);
            }
        };
        if constexpr (MAXM > 0 || ROW8) {
#pragma unroll
            for (int i = 0; i < MAXM; ++i) {   // length 0 past m_total
                if (ent[i] != ~0u) {
                    if (ent[i] >> 26) append(ent[i] & ((1u << 26) - 1), (int)(ent[i] >> 26));
                } else if (ROW8) {   // a code longer than 26 bits: its u64 entry
                    put(sym_entry(codes, v / CS, (int)(v % CS) * 8 + i, 8 * CS, k, context,
                                  raw_first, prev_row, enc, items, nullptr, ldc));
                } else {
                    put(sym_entry(codes, v, i, m_total, k, context, raw_first, prev_row, enc,
                                  items, tree_prev));
                }
            }
        } else {
            for (int i = 0; i < m_total; ++i)
                put(sym_entry(codes, v, i, m_total, k, context, raw_first, prev_row, enc, items,
                              tree_prev));
        }
        if (nacc > 0) atomicOr(&img[w], (uint32_t)(acc << (32 - nacc)));
        pos += bits;
    }
    lds_barrier();
    if (stamp) g_enc_stamps[3] = __builtin_amdgcn_s_memtime();
    if constexpr (TILE) {   // the whole image into the tile's scratch slot
        uint32_t* slot = out_words + id * cap_words;
        for (long long w = tid; w < nwords; w += BLK) slot[w] = img[w];
        return;
    }
    // tail / head exchange with the neighbours (one lane)
    if (tid == 0) {
        const bool tail_open = (be & 31) != 0;   // last word not complete: successor's head
        uint32_t pred = 0;
        if (head_mem) pred = bswap32(out_words[wa]);   // nobody else writes word wa yet
        if (nwords == 0) {
            // empty block: forward the open word unchanged
            if (head_pred) pred = lb_wait_tail(tails, id - 1, epoch);
            lb_store(tails + id, ((unsigned long long)epoch << 48) | (1ull << 32) | pred);
            s_head = pred;
        } else if (nwords > 1) {
            // the tail does not depend on the predecessor: publish it first
            lb_store(tails + id, ((unsigned long long)epoch << 48) | (1ull << 32) |
                                     (tail_open ? img[nwords - 1] : 0u));
            if (head_pred) pred = lb_wait_tail(tails, id - 1, epoch);
            s_head = img[0] | pred;
        } else {
            if (head_pred) pred = lb_wait_tail(tails, id - 1, epoch);
            s_head = img[0] | pred;
            lb_store(tails + id, ((unsigned long long)epoch << 48) | (1ull << 32) |
                                     (tail_open ? s_head : 0u));
        }
        if (id == nb - 1) *total_out = be - bit_offset;
        if (overflow) atomicOr(err, 2ull);
    }
    lds_barrier();
    if (stamp) g_enc_stamps[4] = __builtin_amdgcn_s_memtime();
    const bool last = id == nb - 1;
    if (!overflow) {
        // words this block owns: [wa, wz], minus an open last word unless this is the last block
        const long long wend = ((be & 31) && !last) ? nwords - 1 : nwords;
        for (long long w = tid; w < wend; w += BLK)
            __builtin_nontemporal_store(bswap32(w == 0 ? s_head : img[w]), out_words + wa + w);
        if (nwords == 0 && last && (be & 31) && tid == 0)   // empty last block closes the word
            out_words[wa] = bswap32(s_head);
    }
    if (stamp) g_enc_stamps[5] = __builtin_amdgcn_s_memtime();
}

// `take` (1..32) bits of a tile's MSB-first image starting at bit r, right-aligned (the slot
// has one readable word past its last: masked off)
__device__ __forceinline__ uint32_t slot_bits(const uint32_t* __restrict__ src, unsigned long long r,
                                              int take) {
    const long long w = (long long)(r >> 5);
    const int sh = (int)(r & 31);
    const uint32_t x = sh ? (src[w] << sh) | (src[w + 1] >> (32 - sh)) : src[w];
    return x >> (32 - take);
}

// Places every tile's image (enc_onepass<..., TILE = true>) at its offset in the stream:
// workgroup t writes the stream words whose first bit lies in tile t -- a word that runs past
// the tile's end takes the next tiles' first bits from their slots -- so every word has one
// writer and no workgroup waits for another.  The stream's first word, when bit_offset is
// not word-aligned, is merged with its memory content (shards composed into one buffer).
// Also adds the tile's offset to its chunks' tile-relative bit offsets.
__global__ void __launch_bounds__(256)
enc_place(const uint32_t* __restrict__ scratch, long long slot_words,
          const uint32_t* __restrict__ tile_bits, const unsigned long long* __restrict__ tile_off,
          long long nb, unsigned long long bit_offset_arg,
          const unsigned long long* __restrict__ d_bit_offset, uint32_t* __restrict__ out_words,
          long long cap_words, long long rows_per_tile, long long rows_per_chunk,
          long long chunks, unsigned long long* __restrict__ chunk_off,
          unsigned long long* __restrict__ err, const unsigned long long* __restrict__ total) {
    const long long t = blockIdx.x;
    const unsigned long long bo = d_bit_offset ? (*d_bit_offset & 31ull) : bit_offset_arg;
    const unsigned long long gs = bo + tile_off[t];          // the tile's first stream bit
    const unsigned long long nbits = tile_bits[t];
    const unsigned long long ge = gs + nbits;
    if (t == 0 && threadIdx.x == 0 && ((bo + *total + 31) >> 5) > (unsigned long long)cap_words)
        atomicOr(err, 2ull);
    // (the stream must fit: checked from the total by every workgroup, nothing written if not)
    if (((bo + *total + 31) >> 5) > (unsigned long long)cap_words) return;
    if (chunk_off && rows_per_chunk > 0) {
        const long long r0 = t * rows_per_tile, r1 = r0 + rows_per_tile;
        const long long j0 = (r0 + rows_per_chunk - 1) / rows_per_chunk;
        const long long j1 = min(chunks, (r1 + rows_per_chunk - 1) / rows_per_chunk);
        for (long long j = j0 + threadIdx.x; j < j1; j += blockDim.x) chunk_off[j] += gs;
    }
    if (!nbits) return;
    const uint32_t* src = scratch + t * slot_words;
    // the word holding the stream's first bit, when that is not word-aligned: memory bits + ours
    if (gs == bo && (bo & 31) && threadIdx.x == 0) {
        const int room = 32 - (int)(bo & 31);
        const int take = nbits < (unsigned long long)room ? (int)nbits : room;
        const uint32_t mine = slot_bits(src, 0, take) << (room - take);
        const long long w = (long long)(bo >> 5);
        out_words[w] = __builtin_bswap32(__builtin_bswap32(out_words[w]) | mine);
        // (a tile shorter than the rest of that word: the next tiles' bits are placed by
        // the general loop below only for words they own, so merge them here too)
        unsigned long long filled = (unsigned long long)take;
        long long tt = t + 1;
        uint32_t more = 0;
        while (filled < (unsigned long long)room && tt < nb) {
            const unsigned long long b2 = tile_bits[tt];
            const int tk = (int)min<unsigned long long>(b2, (unsigned long long)room - filled);
            if (tk > 0)
                more |= slot_bits(scratch + tt * slot_words, 0, tk) << (room - (int)filled - tk);
            filled += (unsigned long long)tk;
            ++tt;
        }
        if (more) out_words[w] = __builtin_bswap32(__builtin_bswap32(out_words[w]) | more);
    }
    const long long wa = (long long)((gs + 31) >> 5), wz = (long long)((ge + 31) >> 5);   // [wa, wz)
    for (long long w = wa + threadIdx.x; w < wz; w += blockDim.x) {
        const unsigned long long r = ((unsigned long long)w << 5) - gs;   // < nbits
        uint32_t word;
        if (r + 32 <= nbits) {
            word = slot_bits(src, r, 32);
        } else {   // the tile's last word: its bits, then the next tiles' first bits
            const int have = (int)(nbits - r);
            word = slot_bits(src, r, have) << (32 - have);
            int filled = have;
            for (long long tt = t + 1; filled < 32 && tt < nb; ++tt) {
                const unsigned long long b2 = tile_bits[tt];
                const int tk = (int)min<unsigned long long>(b2, (unsigned long long)(32 - filled));
                if (tk > 0) word |= slot_bits(scratch + tt * slot_words, 0, tk) << (32 - filled - tk);
                filled += tk;
            }
        }
        __builtin_nontemporal_store(__builtin_bswap32(word), out_words + w);
    }
}

}  // namespace

// The context histogram's shape for n rows: its prev-range split, and the workgroup groups.
// Up to 4 groups' worth of chunks (3.9M rows at m = 8) every chunk is a workgroup of its own
// (one round); past that the chunks are spread over a fixed number of groups per (part,
// split) -- ~256 workgroups in all, one per CU -- each counting its chunks in rounds, so the partial images
// (and the reduce's reads) no longer grow with n; the u32 carry accumulator follows them.
struct HistPlan {
    int split, rounds, groups;
    long long chunks;
    size_t partial_bytes, acc_offset, total_bytes;
};

static int hist_split(int k, int ctx_split) {
    static const int split_env = [] {   // PQH_HIST_SPLIT = 1, 2, 4 or 8; default 2 for even k
        const char* e = std::getenv("PQH_HIST_SPLIT");
        const int v = e ? std::atoi(e) : 2;
        return v == 1 || v == 4 || v == 8 ? v : 2;
    }();
    const int want = ctx_split > 0 ? ctx_split : split_env;   // pqh_ctx_set_tuning first
    return k % (2 * want) == 0 ? want : (k % 4 == 0 ? 2 : 1);
}

static HistPlan hist_plan(long long n, int m, int k, int ctx_split = 0) {
    HistPlan p{};
    p.split = hist_split(k, ctx_split);
    p.chunks = (n + kHistChunk - 1) / kHistChunk;
    static const int target = [] {   // PQH_HIST_WGS: the multi-round grid's workgroups
        const char* e = std::getenv("PQH_HIST_WGS");
        const int v = e ? std::atoi(e) : 256;
        return v >= 8 ? v : 256;
    }();
    // groups per (part, split), independent of the split: the partials' layout (and the
    // reduce that reads them, possibly on another context with another split) depends only on
    // n, m and k
    const int gt = std::max(8, (target / (m * 2)) / 8 * 8);
    if (p.chunks <= 4ll * gt) {
        p.rounds = 1;
        p.groups = (int)p.chunks;
    } else {
        p.rounds = (int)((p.chunks + gt - 1) / gt);
        p.groups = (int)((p.chunks + p.rounds - 1) / p.rounds);
    }
    const size_t words = (size_t)((k * k + 1) / 2);
    p.partial_bytes = (size_t)m * p.groups * words * 4;
    p.acc_offset = (p.partial_bytes + 255) & ~(size_t)255;
    p.total_bytes = p.rounds > 1 ? p.acc_offset + (size_t)m * k * k * 4 : p.partial_bytes;
    return p;
}

extern "C" {

// phase: 0 = partials + reduce (pqh_histogram*), 1 = the context partials only, into
// d_partials (pqh_histogram_partial), 2 = the reduce of d_partials only (pqh_histogram_reduce)
static int histogram_impl(pqh_ctx_t* ctx, const void* d_codes, long long n, int m, int k,
                          int context, const void* d_prev_row, uint32_t* d_counts, int set,
                          const int* d_rawf = nullptr, int phase = 0,
                          uint32_t* d_partials = nullptr, long long ldc = 0) {
    if (ldc && ldc < n) return PQH_ERR_ARG;
    if (!ctx || m <= 0 || k <= 0 || n < 0) return PQH_ERR_ARG;
    if (phase != 1 && !d_counts) return PQH_ERR_ARG;
    if (phase != 2 && n > 0 && !d_codes) return PQH_ERR_ARG;
    if (phase && (!context || !d_partials)) return PQH_ERR_ARG;
    if (context && k > 256) return PQH_ERR_UNSUPPORTED;
    int rc = pqh_use_device(ctx);
    if (rc) return rc;
    const long long items = context ? (long long)k * k : k;
    // (8-part u16 rows, K > 256: per-workgroup partials + a reduce that overwrites)
    const bool wide16 = !context && k > 256 && !ldc && m == 8 && k % 2 == 0 && k <= 4096 &&
                        !(reinterpret_cast<uintptr_t>(d_codes) & 15);
    if (set && (n == 0 || (!context && !wide16)) && phase != 1)   // the plain kernel and an empty input only add
        PQH_HIP(ctx, hipMemsetAsync(d_counts, 0, (size_t)m * items * 4, ctx->stream));
    if (n == 0) return PQH_OK;
    if (context) {
        const HistPlan hp = hist_plan(n, m, k, ctx->tune_hist_split);
        const int words = (k * k + 1) / 2;
        const int split = hp.split;
        const size_t lds = (size_t)(split == 1 ? words : (k / split) * k / 2) * 4;
        uint32_t* partial = d_partials;
        if (!partial) {
            rc = pqh_ensure_ws(ctx, hp.total_bytes);
            if (rc) return rc;
            partial = static_cast<uint32_t*>(ctx->ws);
        }
        uint32_t* acc = hp.rounds > 1
                            ? reinterpret_cast<uint32_t*>(reinterpret_cast<char*>(partial) + hp.acc_offset)
                            : nullptr;
        if (phase == 2) {
            hipLaunchKernelGGL(hist_ctx_reduce, dim3((unsigned)((words + 255) / 256), m), dim3(256),
                               0, ctx->stream, partial, hp.groups, words, (long long)k * k,
                               d_counts, set, acc);
            PQH_LAUNCH_CHECK(ctx);
            return PQH_OK;
        }
        // the carry accumulator starts at zero (the reduce clears it again after reading)
        if (acc) PQH_HIP(ctx, hipMemsetAsync(acc, 0, (size_t)m * k * k * 4, ctx->stream));
        const int chunks = (int)hp.chunks, rounds = hp.rounds;
        const unsigned grid = 8u * (((unsigned)hp.groups + 7u) / 8u) * (unsigned)(m * split);
        // 1024-thread workgroups; PQH_HIST_BLOCK=256: 256 threads with <= 32 VGPRs, which fit
        // beside the assignment grid (measured: histogram 0.19 vs 0.075 ms in the bench -- a
        // quarter of the loads in flight -- and the bench 2,119 vs 2,534 Mvec/s)
        const char* hb_env = std::getenv("PQH_HIST_BLOCK");
        const int hb_v = ctx->tune_hist_block ? ctx->tune_hist_block : (hb_env ? std::atoi(hb_env) : 0);
        // the wave-contiguous form for u8 codes with m % 4 == 0 (aligned rows; PQH_HIST_IMPL=
        // thread keeps the per-thread runs of hist_ctx)
        static const int form_env = [] {   // 1: thread, 2: wave (any m % 4 == 0), 0: default
            const char* e = std::getenv("PQH_HIST_IMPL");
            return !e ? 0 : !std::strcmp(e, "thread") ? 1 : !std::strcmp(e, "wave") ? 2 : 0;
        }();
        const bool thread_form = form_env == 1;
        const uintptr_t al = reinterpret_cast<uintptr_t>(d_codes);
        // (measured alone, tools/bench_hist.py: 0.027 vs 0.035 ms per 1M rows at m = 8, 0.052
        // vs 0.108 at m = 16; the Deep bench 1,300 vs 1,218 Mvec/s)
        const bool slim = hb_v == 256;
        // (part-major codes: always the wave form, which reads each part's run directly)
        const bool wave_form = ldc || (!thread_form && m % 4 == 0 && (al & (m == 8 ? 15u : 3u)) == 0);
        if (wave_form && slim) {
            // 256 threads, <= 32 VGPRs: fits on a CU beside the assignment grid (one wave
            // per SIMD, 64 KB of LDS beside its ~75 KB), for a histogram off stream A
            auto kf = ldc ? hist_ctx_w<256, 3, true> : hist_ctx_w<256, 3, false>;
            PQH_HIP(ctx, hipFuncSetAttribute((const void*)kf,
                                             hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
            hipLaunchKernelGGL(kf, dim3(grid), dim3(256), lds, ctx->stream,
                               static_cast<const uint8_t*>(d_codes), n, m, k,
                               static_cast<const uint8_t*>(d_prev_row), d_rawf, partial, split,
                               chunks, rounds, acc, pqh_prio("HIST", 0), ldc);
        } else if (wave_form) {
            auto kf = ldc ? hist_ctx_w<1024, 5, true> : hist_ctx_w<1024, 5, false>;
            PQH_HIP(ctx, hipFuncSetAttribute((const void*)kf,
                                             hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
            hipLaunchKernelGGL(kf, dim3(grid), dim3(1024), lds, ctx->stream,
                               static_cast<const uint8_t*>(d_codes), n, m, k,
                               static_cast<const uint8_t*>(d_prev_row), d_rawf, partial, split,
                               chunks, rounds, acc, pqh_prio("HIST", 0), ldc);
        } else if (!slim) {
            PQH_HIP(ctx, hipFuncSetAttribute((const void*)hist_ctx<uint8_t>,
                                             hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
            hipLaunchKernelGGL(hist_ctx<uint8_t>, dim3(grid), dim3(1024), lds, ctx->stream,
                               static_cast<const uint8_t*>(d_codes), n, m, k,
                               static_cast<const uint8_t*>(d_prev_row), d_rawf, partial, split,
                               chunks, rounds, acc, pqh_prio("HIST", 0));
        } else {
            PQH_HIP(ctx, hipFuncSetAttribute((const void*)hist_ctx<uint8_t, 256, 8>,
                                             hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
            hipLaunchKernelGGL((hist_ctx<uint8_t, 256, 8>), dim3(grid), dim3(256), lds, ctx->stream,
                               static_cast<const uint8_t*>(d_codes), n, m, k,
                               static_cast<const uint8_t*>(d_prev_row), d_rawf, partial, split,
                               chunks, rounds, acc, pqh_prio("HIST", 0));
        }
        PQH_LAUNCH_CHECK(ctx);
        if (phase == 0)
            hipLaunchKernelGGL(hist_ctx_reduce, dim3((unsigned)((words + 255) / 256), m), dim3(256),
                               0, ctx->stream, partial, hp.groups, words, (long long)k * k,
                               d_counts, set, acc);
    } else if (wide16) {
        // 8-part u16 rows: per-workgroup partial images + hist_ctx_reduce (no global atomics)
        const long long rows = std::max<long long>(1, std::min<long long>(16384, (n + 63) / 64));
        const int groups = (int)((n + rows - 1) / rows);
        const int words = k / 2;
        rc = pqh_ensure_ws(ctx, (size_t)8 * groups * words * 4);
        if (rc) return rc;
        uint32_t* partial = static_cast<uint32_t*>(ctx->ws);
        const size_t lds = (size_t)8 * words * 4;
        PQH_HIP(ctx, hipFuncSetAttribute((const void*)hist_plain_rows16,
                                         hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
        hipLaunchKernelGGL(hist_plain_rows16, dim3((unsigned)groups), dim3(256), lds, ctx->stream,
                           static_cast<const uint16_t*>(d_codes), n, k, rows, partial, groups);
        PQH_LAUNCH_CHECK(ctx);
        hipLaunchKernelGGL(hist_ctx_reduce, dim3((unsigned)((words + 255) / 256), m), dim3(256), 0,
                           ctx->stream, partial, groups, words, (long long)k, d_counts,
                           set ? 1 : 0, nullptr);
    } else {
        const unsigned blocks = (unsigned)std::min<long long>((n + 4095) / 4096, 512);
        if (k <= 256)
            hipLaunchKernelGGL(hist_plain<uint8_t>, dim3(blocks, m), dim3(256), k * 4, ctx->stream,
                               static_cast<const uint8_t*>(d_codes), n, m, k, d_counts, ldc);
        else
            hipLaunchKernelGGL(hist_plain<uint16_t>, dim3(blocks, m), dim3(256), k * 4, ctx->stream,
                               static_cast<const uint16_t*>(d_codes), n, m, k, d_counts, ldc);
    }
    PQH_LAUNCH_CHECK(ctx);
    return PQH_OK;
}

long long pqh_histogram_partial_bytes(long long n, int m, int k) {
    if (n < 0 || m <= 0 || k <= 0 || k > 256) return -1;
    return (long long)hist_plan(n, m, k).total_bytes;
}

int pqh_histogram_partial(pqh_ctx_t* ctx, const void* d_codes, long long n, int m, int k,
                          const void* d_prev_row, void* d_partials) {
    return histogram_impl(ctx, d_codes, n, m, k, 1, d_prev_row, nullptr, 0, nullptr, 1,
                          static_cast<uint32_t*>(d_partials));
}

int pqh_histogram_reduce(pqh_ctx_t* ctx, const void* d_partials, long long n, int m, int k,
                         uint32_t* d_counts, int set) {
    return histogram_impl(ctx, nullptr, n, m, k, 1, nullptr, d_counts, set ? 1 : 0, nullptr, 2,
                          static_cast<uint32_t*>(const_cast<void*>(d_partials)));
}

int pqh_histogram(pqh_ctx_t* ctx, const void* d_codes, long long n, int m, int k, int context,
                  const void* d_prev_row, uint32_t* d_counts) {
    return histogram_impl(ctx, d_codes, n, m, k, context, d_prev_row, d_counts, 0);
}

int pqh_histogram_set(pqh_ctx_t* ctx, const void* d_codes, long long n, int m, int k,
                      int context, const void* d_prev_row, uint32_t* d_counts) {
    return histogram_impl(ctx, d_codes, n, m, k, context, d_prev_row, d_counts, 1);
}

int pqh_histogram_parts(pqh_ctx_t* ctx, const void* d_codes, long long ld_codes, long long n,
                        int m, int k, int context, const void* d_prev_row, uint32_t* d_counts,
                        int set) {
    if (ld_codes <= 0) return PQH_ERR_ARG;
    return histogram_impl(ctx, d_codes, n, m, k, context, d_prev_row, d_counts, set ? 1 : 0,
                          nullptr, 0, nullptr, ld_codes);
}

int pqh_histogram_partial_parts(pqh_ctx_t* ctx, const void* d_codes, long long ld_codes,
                                long long n, int m, int k, const void* d_prev_row,
                                void* d_partials) {
    if (ld_codes <= 0) return PQH_ERR_ARG;
    return histogram_impl(ctx, d_codes, n, m, k, 1, d_prev_row, nullptr, 0, nullptr, 1,
                          static_cast<uint32_t*>(d_partials), ld_codes);
}

// workspace layout for encode: [block_bits u32 nb][pad][block_off u64 nb][scan segments]
static size_t scan_seg_bytes(long long nb) { return (size_t)((nb + kScanSeg - 1) / kScanSeg) * 8; }
static int enc_ws(pqh_ctx* ctx, long long n, uint32_t** bb, unsigned long long** bo) {
    const long long nb = (n + kEncBlock - 1) / kEncBlock;
    const size_t a = ((size_t)nb * 4 + 255) & ~(size_t)255;
    int rc = pqh_ensure_ws(ctx, a + (size_t)nb * 8 + scan_seg_bytes(nb) + 256);
    if (rc) return rc;
    *bb = static_cast<uint32_t*>(ctx->ws);
    *bo = reinterpret_cast<unsigned long long*>(static_cast<char*>(ctx->ws) + a);
    return PQH_OK;
}

static int run_size(pqh_ctx* ctx, const pqh_tables* t, const void* d_codes, long long n,
                    int raw_first, const void* d_prev_row, unsigned long long* d_total,
                    const int* d_rawf = nullptr) {
    uint32_t* bb;
    unsigned long long* bo;
    int rc = enc_ws(ctx, n, &bb, &bo);
    if (rc) return rc;
    const long long nb = (n + kEncBlock - 1) / kEncBlock;
    if (t->k <= 256)
        hipLaunchKernelGGL(enc_size<uint8_t>, dim3((unsigned)nb), dim3(kEncBlock), 0, ctx->stream,
                           static_cast<const uint8_t*>(d_codes), n, t->m, t->k, t->context,
                           raw_first, static_cast<const uint8_t*>(d_prev_row), d_rawf, t->d_enc,
                           t->items, bb, nullptr);
    else
        hipLaunchKernelGGL(enc_size<uint16_t>, dim3((unsigned)nb), dim3(kEncBlock), 0, ctx->stream,
                           static_cast<const uint16_t*>(d_codes), n, t->m, t->k, t->context,
                           raw_first, static_cast<const uint16_t*>(d_prev_row), d_rawf, t->d_enc,
                           t->items, bb, nullptr);
    PQH_LAUNCH_CHECK(ctx);
    launch_scan(ctx->stream, bb, nb, bo, d_total, bo + nb);
    PQH_LAUNCH_CHECK(ctx);
    return PQH_OK;
}

int pqh_encode_size(pqh_ctx_t* ctx, const pqh_tables_t* t, const void* d_codes, long long n,
                    int raw_first, const void* d_prev_row, unsigned long long* d_total_bits) {
    if (!ctx || !t || n < 0 || !d_total_bits || (n > 0 && !d_codes)) return PQH_ERR_ARG;
    int rc = pqh_use_device(ctx);
    if (rc) return rc;
    if (n == 0) {
        PQH_HIP(ctx, hipMemsetAsync(d_total_bits, 0, 8, ctx->stream));
        return PQH_OK;
    }
    return run_size(ctx, t, d_codes, n, raw_first, d_prev_row, d_total_bits);
}

static int encode_write_impl(pqh_ctx_t* ctx, const pqh_tables_t* t, const void* d_codes,
                             long long n, int raw_first, const void* d_prev_row,
                             unsigned long long bit_offset,
                             const unsigned long long* d_bit_offset, unsigned char* d_out,
                             unsigned long long out_bytes, int chunk_vectors,
                             unsigned long long* d_chunk_offsets, void* d_chunk_prev,
                             unsigned long long* d_total_bits,
                             const uint16_t* tree_prev = nullptr, const int* d_rawf = nullptr,
                             long long ldc = 0, int phase = 0) {
    // phase (tiled encoder only): 0 = the whole write; 1 = the tiles and the scan (the
    // total in *d_total_bits; d_out and the offset unused); 2 = the placement of phase 1's
    // tiles at the offset, with the same arguments and nothing else run on ctx between
    // (pqh_shard_encode_write: the length all-gather runs between them)
    if (!ctx || !t || n < 0 || (n > 0 && !d_codes) || (n > 0 && phase != 1 && !d_out))
        return PQH_ERR_ARG;
    if (phase && !d_total_bits) return PQH_ERR_ARG;
    if (ldc && (ldc < n || t->k > 256 || (t->m != 8 && t->m != 16) || tree_prev ||
                (reinterpret_cast<uintptr_t>(d_chunk_prev) & 7)))
        return ldc < n ? PQH_ERR_ARG : PQH_ERR_UNSUPPORTED;   // part-major: the row encoder only
    if (phase != 1 && ((reinterpret_cast<uintptr_t>(d_out) & 3u) || (out_bytes & 3u)))
        return pqh_set_error(ctx, PQH_ERR_ARG, "stream buffer must be 4-byte aligned and sized");
    if (chunk_vectors > 0 && !d_chunk_offsets) return PQH_ERR_ARG;
    int rc = pqh_use_device(ctx);
    if (rc) return rc;
    if (n == 0) {
        if (d_total_bits && phase != 2) PQH_HIP(ctx, hipMemsetAsync(d_total_bits, 0, 8, ctx->stream));
        return PQH_OK;
    }
    // 8-byte rows: m = 8 (one row per vector) or m = 16 (two rows per vector), u8 codes,
    // aligned, no tree order: the <= 32-VGPR row encoder on 256 rows per workgroup, which fits
    // on a CU beside the assignment grid's waves; other shapes the generic encoder (m <= 8:
    // 256 vectors per workgroup, wider rows 512)
    const bool row8 = t->k <= 256 && (t->m == 8 || t->m == 16) && !tree_prev &&
                      (ldc || !(reinterpret_cast<uintptr_t>(d_codes) & 7)) &&
                      !(reinterpret_cast<uintptr_t>(d_chunk_prev) & 7);
    const int cs = row8 ? t->m / 8 : 1;
    const long long rows = n * cs;
    const int blk = row8 || t->m <= 8 ? 256 : kEncBlock;
    const long long nb = (rows + blk - 1) / blk;
    const size_t lds = ((size_t)blk * (row8 ? 8 : t->m) * kMaxCodeLen / 32 + 4) * 4;
    if (lds > 160 * 1024) return PQH_ERR_UNSUPPORTED;
    unsigned long long* total = d_total_bits ? d_total_bits : ctx->d_diag + 3;
    uint32_t* words = reinterpret_cast<uint32_t*>(d_out);
    const int enc_prio = pqh_prio("ENCODE", 0);
    // The tiled encoder (default): tiles coded into scratch slots with no inter-workgroup
    // waiting, a scan of their bit counts, then enc_place.  PQH_ENC_IMPL=onepass: the
    // single-kernel decoupled look-back form.
    static const bool onepass_env = [] {
        const char* e = std::getenv("PQH_ENC_IMPL");
        return e && !std::strcmp(e, "onepass");
    }();
    const bool onepass = ctx->tune_enc_impl ? ctx->tune_enc_impl == 2 : onepass_env;
    static const bool no16 = [] {   // (diagnostic A/B: PQH_ENC16=0 gathers the u32 copy only)
        const char* e = std::getenv("PQH_ENC16");
        return e && !std::strcmp(e, "0");
    }();
    const uint16_t* const enc16 = no16 ? nullptr : t->d_enc16;
    // The tiled encoder's scratch holds one worst-case tile image per 256 rows (56 B per
    // row, 7 GB at 125M rows).  A whole write (phase 0) that cannot get it falls back to the
    // one-pass encoder, which needs O(tiles) state; the two-phase shard write keeps its tiles
    // between the phases, so it has no such fallback and reports PQH_ERR_NOMEM.
    const long long slot = (long long)(lds / 4);   // a tile's worst-case image, + 4 words
    bool tiled = !onepass || phase;
    if (tiled && phase == 0 &&
        pqh_ensure_enc_scratch(ctx, ((size_t)nb * slot + 64) * 4) == PQH_ERR_NOMEM) {
        tiled = false;
        pqh_set_error(ctx, PQH_OK, "");
    }
    if (tiled) {
        int rc2 = pqh_ensure_enc_scratch(ctx, ((size_t)nb * slot + 64) * 4);
        if (rc2) return rc2;
        const size_t a = ((size_t)nb * 4 + 255) & ~(size_t)255;
        rc2 = pqh_ensure_ws(ctx, a + (size_t)nb * 8 + scan_seg_bytes(nb) + 256);
        if (rc2) return rc2;
        uint32_t* tile_bits = static_cast<uint32_t*>(ctx->ws);
        unsigned long long* tile_off =
            reinterpret_cast<unsigned long long*>(static_cast<char*>(ctx->ws) + a);
        uint32_t* scr = static_cast<uint32_t*>(ctx->enc_scr);
        unsigned long long* tb = reinterpret_cast<unsigned long long*>(tile_bits);
        const long long chunks = chunk_vectors > 0 ? (n + chunk_vectors - 1) / chunk_vectors : 0;
        auto place = [&]() -> int {
            hipLaunchKernelGGL(enc_place, dim3((unsigned)nb), dim3(256), 0, ctx->stream, scr, slot,
                               tile_bits, tile_off, nb, bit_offset, d_bit_offset, words,
                               (long long)(out_bytes / 4), (long long)blk,
                               chunk_vectors > 0 ? (long long)chunk_vectors * cs : 0ll, chunks,
                               d_chunk_offsets, ctx->d_diag + 2, total);
            PQH_LAUNCH_CHECK(ctx);
            return PQH_OK;
        };
        if (phase == 2) return place();
#define PQH_ENC_T(T, MAXM, R8, CS, PMV)                                                          \
    do {                                                                                         \
        constexpr int B = MAXM > 0 && MAXM <= 8 ? 256 : kEncBlock;                               \
        auto kf = enc_onepass<T, MAXM, B, R8, CS, PMV, true>;                                    \
        if (lds > 64 * 1024)                                                                     \
            PQH_HIP(ctx, hipFuncSetAttribute((const void*)kf,                                    \
                                             hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds)); \
        hipLaunchKernelGGL(kf, dim3((unsigned)nb), dim3(B), lds, ctx->stream,                   \
                           static_cast<const T*>(d_codes), R8 ? rows : n, t->m, t->k, t->context, \
                           raw_first, static_cast<const T*>(d_prev_row), d_rawf, t->d_enc,       \
                           t->d_enc32, enc16, t->items, 0ull, nullptr, scr, slot, chunk_vectors,     \
                           d_chunk_offsets, static_cast<T*>(d_chunk_prev), ctx->d_diag + 2, tb,  \
                           nullptr, nullptr, 0ull, 0u, nb, nullptr, tree_prev, enc_prio, ldc);   \
    } while (0)
        if (ldc) {
            if (cs == 2) PQH_ENC_T(uint8_t, 8, true, 2, true);
            else PQH_ENC_T(uint8_t, 8, true, 1, true);
        } else if (t->k <= 256) {
            if (row8 && cs == 2) PQH_ENC_T(uint8_t, 8, true, 2, false);
            else if (row8) PQH_ENC_T(uint8_t, 8, true, 1, false);
            else if (t->m <= 8) PQH_ENC_T(uint8_t, 8, false, 1, false);
            else if (t->m <= 16) PQH_ENC_T(uint8_t, 16, false, 1, false);
            else PQH_ENC_T(uint8_t, 0, false, 1, false);
        } else {
            if (t->m <= 8) PQH_ENC_T(uint16_t, 8, false, 1, false);
            else if (t->m <= 16) PQH_ENC_T(uint16_t, 16, false, 1, false);
            else PQH_ENC_T(uint16_t, 0, false, 1, false);
        }
#undef PQH_ENC_T
        PQH_LAUNCH_CHECK(ctx);
        launch_scan(ctx->stream, tile_bits, nb, tile_off, total, tile_off + nb);
        PQH_LAUNCH_CHECK(ctx);
        return phase == 1 ? PQH_OK : place();
    }
    // look-back state: grow-only, epoch-tagged so it never needs clearing between calls
    if (nb > ctx->lb_cap) {
        PQH_HIP(ctx, hipStreamSynchronize(ctx->stream));   // no launch may still use it
        if (ctx->lb_state) (void)hipFree(ctx->lb_state);
        ctx->lb_state = nullptr;
        const long long cap = nb + nb / 4 + 64;
        PQH_HIP(ctx, hipMalloc(&ctx->lb_state, (size_t)(2 * cap + 1) * 8));
        PQH_HIP(ctx, hipMemsetAsync(ctx->lb_state, 0, (size_t)(2 * cap + 1) * 8, ctx->stream));
        ctx->lb_cap = cap;
        ctx->lb_epoch = 0;
        ctx->lb_ticket_base = 0;
    }
    if (++ctx->lb_epoch >= 0xFFFF) {   // wrap: clear the tags (never matched by a new epoch)
        PQH_HIP(ctx, hipMemsetAsync(ctx->lb_state, 0, (size_t)(2 * ctx->lb_cap) * 8, ctx->stream));
        ctx->lb_epoch = 1;
    }
    unsigned long long* st = ctx->lb_state;
    unsigned long long* tails = st + ctx->lb_cap;
    unsigned long long* ticket = st + 2 * ctx->lb_cap;
#define PQH_ENC(T, MAXM, R8, CS) PQH_ENC_PM(T, MAXM, R8, CS, false)
#define PQH_ENC_PM(T, MAXM, R8, CS, PMV)                                                          \
    do {                                                                                          \
        constexpr int B = MAXM > 0 && MAXM <= 8 ? 256 : kEncBlock;                                \
        if (lds > 64 * 1024)                                                                      \
            PQH_HIP(ctx, hipFuncSetAttribute((const void*)(enc_onepass<T, MAXM, B, R8, CS, PMV>), \
                                             hipFuncAttributeMaxDynamicSharedMemorySize,          \
                                             (int)lds));                                          \
        hipLaunchKernelGGL((enc_onepass<T, MAXM, B, R8, CS, PMV>), dim3((unsigned)nb), dim3(B), lds, \
                           ctx->stream, static_cast<const T*>(d_codes), R8 ? rows : n, t->m, t->k, \
                           t->context, raw_first, static_cast<const T*>(d_prev_row), d_rawf,     \
                           t->d_enc,                                                              \
                           t->d_enc32, enc16, t->items, bit_offset, d_bit_offset, words,           \
                           (long long)(out_bytes / 4),                                            \
                           chunk_vectors, d_chunk_offsets, static_cast<T*>(d_chunk_prev),         \
                           ctx->d_diag + 2, st, tails, ticket, ctx->lb_ticket_base,               \
                           (unsigned)ctx->lb_epoch, nb, total, tree_prev, enc_prio, ldc);         \
    } while (0)
    if (ldc) {   // part-major codes: the row encoder (checked above)
        if (cs == 2) PQH_ENC_PM(uint8_t, 8, true, 2, true);
        else PQH_ENC_PM(uint8_t, 8, true, 1, true);
    } else if (t->k <= 256) {
        if (row8 && cs == 2) PQH_ENC(uint8_t, 8, true, 2);
        else if (row8) PQH_ENC(uint8_t, 8, true, 1);
        else if (t->m <= 8) PQH_ENC(uint8_t, 8, false, 1);
        else if (t->m <= 16) PQH_ENC(uint8_t, 16, false, 1);
        else PQH_ENC(uint8_t, 0, false, 1);
    } else {
        if (t->m <= 8) PQH_ENC(uint16_t, 8, false, 1);
        else if (t->m <= 16) PQH_ENC(uint16_t, 16, false, 1);
        else PQH_ENC(uint16_t, 0, false, 1);
    }
#undef PQH_ENC
#undef PQH_ENC_PM
    PQH_LAUNCH_CHECK(ctx);
    ctx->lb_ticket_base += (unsigned long long)nb;
    return PQH_OK;
}

int pqh_encode_write(pqh_ctx_t* ctx, const pqh_tables_t* t, const void* d_codes, long long n,
                     int raw_first, const void* d_prev_row, unsigned long long bit_offset,
                     unsigned char* d_out, unsigned long long out_bytes, int chunk_vectors,
                     unsigned long long* d_chunk_offsets, void* d_chunk_prev,
                     unsigned long long* d_total_bits) {
    return encode_write_impl(ctx, t, d_codes, n, raw_first, d_prev_row, bit_offset, nullptr,
                             d_out, out_bytes, chunk_vectors, d_chunk_offsets, d_chunk_prev,
                             d_total_bits);
}

int pqh_transpose_codes(pqh_ctx_t* ctx, const void* d_parts, long long ld_parts, long long n, int m,
                        int code_bytes, void* d_rows) {
    if (!ctx || n < 0 || m <= 0 || ld_parts < n || (code_bytes != 1 && code_bytes != 2) ||
        (n > 0 && (!d_parts || !d_rows)))
        return PQH_ERR_ARG;
    if (code_bytes == 1 && (m == 8 || m == 16) && (reinterpret_cast<uintptr_t>(d_rows) & 7))
        return pqh_set_error(ctx, PQH_ERR_ARG, "transpose: 8- and 16-byte rows must be 8-byte aligned");
    int rc = pqh_use_device(ctx);
    if (rc) return rc;
    if (n == 0) return PQH_OK;
    const unsigned blocks = (unsigned)((n + 255) / 256);
    if (code_bytes == 1)
        hipLaunchKernelGGL(transpose_codes<uint8_t>, dim3(blocks), dim3(256), 0, ctx->stream,
                           static_cast<const uint8_t*>(d_parts), ld_parts, n, m,
                           static_cast<uint8_t*>(d_rows));
    else
        hipLaunchKernelGGL(transpose_codes<uint16_t>, dim3(blocks), dim3(256), 0, ctx->stream,
                           static_cast<const uint16_t*>(d_parts), ld_parts, n, m,
                           static_cast<uint16_t*>(d_rows));
    PQH_LAUNCH_CHECK(ctx);
    return PQH_OK;
}

int pqh_encode_write_parts(pqh_ctx_t* ctx, const pqh_tables_t* t, const void* d_codes,
                           long long ld_codes, long long n, int raw_first, const void* d_prev_row,
                           unsigned long long bit_offset, unsigned char* d_out,
                           unsigned long long out_bytes, int chunk_vectors,
                           unsigned long long* d_chunk_offsets, void* d_chunk_prev,
                           unsigned long long* d_total_bits) {
    if (ld_codes <= 0) return PQH_ERR_ARG;
    return encode_write_impl(ctx, t, d_codes, n, raw_first, d_prev_row, bit_offset, nullptr,
                             d_out, out_bytes, chunk_vectors, d_chunk_offsets, d_chunk_prev,
                             d_total_bits, nullptr, nullptr, ld_codes);
}

int pqh_encode_write_at(pqh_ctx_t* ctx, const pqh_tables_t* t, const void* d_codes, long long n,
                        int raw_first, const void* d_prev_row,
                        const unsigned long long* d_global_bit_offset, unsigned char* d_out,
                        unsigned long long out_bytes, int chunk_vectors,
                        unsigned long long* d_chunk_offsets, void* d_chunk_prev,
                        unsigned long long* d_total_bits) {
    if (!d_global_bit_offset) return PQH_ERR_ARG;
    return encode_write_impl(ctx, t, d_codes, n, raw_first, d_prev_row, 0, d_global_bit_offset,
                             d_out, out_bytes, chunk_vectors, d_chunk_offsets, d_chunk_prev,
                             d_total_bits);
}

// pqh_shard_encode's variants: this shard's raw-first flag lives in device memory (decided
// on the device from the all-gathered halo records); 1 = write row 0 raw and count no halo
// pair, 0 = row 0 in the context of d_prev_row
int pqh_histogram_set_dev(pqh_ctx_t* ctx, const void* d_codes, long long n, int m, int k,
                          const void* d_prev_row, const int* d_rawf, uint32_t* d_counts) {
    return histogram_impl(ctx, d_codes, n, m, k, 1, d_prev_row, d_counts, 1, d_rawf);
}

int pqh_histogram_set_dev_ld(pqh_ctx_t* ctx, const void* d_codes, long long ldc, long long n,
                             int m, int k, const void* d_prev_row, const int* d_rawf,
                             uint32_t* d_counts) {
    return histogram_impl(ctx, d_codes, n, m, k, 1, d_prev_row, d_counts, 1, d_rawf, 0, nullptr,
                          ldc);
}

int pqh_encode_write_at_dev_ld(pqh_ctx_t* ctx, const pqh_tables_t* t, const void* d_codes,
                               long long ldc, long long n, const void* d_prev_row,
                               const int* d_rawf, const unsigned long long* d_global_bit_offset,
                               unsigned char* d_out, unsigned long long out_bytes,
                               int chunk_vectors, unsigned long long* d_chunk_offsets,
                               void* d_chunk_prev) {
    if (!d_global_bit_offset) return PQH_ERR_ARG;
    return encode_write_impl(ctx, t, d_codes, n, 0, d_prev_row, 0, d_global_bit_offset, d_out,
                             out_bytes, chunk_vectors, d_chunk_offsets, d_chunk_prev, nullptr,
                             nullptr, d_rawf, ldc);
}

// pqh_shard_encode_write's two halves of pqh_encode_write_at_dev_ld: phase 1 codes the tiles
// and leaves the shard's exact length in *d_total_bits (before any offset is known), phase 2
// places them at *d_global_bit_offset -- the length all-gather runs between (no size pass)
int pqh_encode_tiles_dev_ld(pqh_ctx_t* ctx, const pqh_tables_t* t, const void* d_codes,
                            long long ldc, long long n, const void* d_prev_row, const int* d_rawf,
                            int chunk_vectors, unsigned long long* d_chunk_offsets,
                            void* d_chunk_prev, unsigned long long* d_total_bits) {
    return encode_write_impl(ctx, t, d_codes, n, 0, d_prev_row, 0, nullptr, nullptr, 0,
                             chunk_vectors, d_chunk_offsets, d_chunk_prev, d_total_bits, nullptr,
                             d_rawf, ldc, 1);
}

int pqh_encode_place_dev_ld(pqh_ctx_t* ctx, const pqh_tables_t* t, const void* d_codes,
                            long long ldc, long long n, const void* d_prev_row, const int* d_rawf,
                            const unsigned long long* d_global_bit_offset, unsigned char* d_out,
                            unsigned long long out_bytes, int chunk_vectors,
                            unsigned long long* d_chunk_offsets, void* d_chunk_prev,
                            unsigned long long* d_total_bits) {
    if (!d_global_bit_offset) return PQH_ERR_ARG;
    return encode_write_impl(ctx, t, d_codes, n, 0, d_prev_row, 0, d_global_bit_offset, d_out,
                             out_bytes, chunk_vectors, d_chunk_offsets, d_chunk_prev, d_total_bits,
                             nullptr, d_rawf, ldc, 2);
}

int pqh_encode_size_dev(pqh_ctx_t* ctx, const pqh_tables_t* t, const void* d_codes, long long n,
                        const void* d_prev_row, const int* d_rawf,
                        unsigned long long* d_total_bits) {
    if (!ctx || !t || n < 0 || !d_total_bits || (n > 0 && !d_codes)) return PQH_ERR_ARG;
    int rc = pqh_use_device(ctx);
    if (rc) return rc;
    if (n == 0) {
        PQH_HIP(ctx, hipMemsetAsync(d_total_bits, 0, 8, ctx->stream));
        return PQH_OK;
    }
    return run_size(ctx, t, d_codes, n, 0, d_prev_row, d_total_bits, d_rawf);
}

int pqh_encode_write_at_dev(pqh_ctx_t* ctx, const pqh_tables_t* t, const void* d_codes,
                            long long n, const void* d_prev_row, const int* d_rawf,
                            const unsigned long long* d_global_bit_offset, unsigned char* d_out,
                            unsigned long long out_bytes, int chunk_vectors,
                            unsigned long long* d_chunk_offsets, void* d_chunk_prev) {
    if (!d_global_bit_offset) return PQH_ERR_ARG;
    return encode_write_impl(ctx, t, d_codes, n, 0, d_prev_row, 0, d_global_bit_offset, d_out,
                             out_bytes, chunk_vectors, d_chunk_offsets, d_chunk_prev, nullptr,
                             nullptr, d_rawf);
}

// diagnostics only: phase stamps of the mid-grid workgroup of the last one-pass encode
int pqh_debug_enc_stamps(pqh_ctx_t* ctx, unsigned long long* out8) {
    if (!ctx || !out8) return PQH_ERR_ARG;
    PQH_HIP(ctx, hipStreamSynchronize(ctx->stream));
    PQH_HIP(ctx, hipMemcpyFromSymbol(out8, HIP_SYMBOL(g_enc_stamps), 8 * sizeof(unsigned long long)));
    return PQH_OK;
}

int pqh_encode_status(pqh_ctx_t* ctx) {
    unsigned long long e = 0;
    PQH_HIP(ctx, hipMemcpyAsync(&e, ctx->d_diag + 2, 8, hipMemcpyDeviceToHost, ctx->stream));
    PQH_HIP(ctx, hipStreamSynchronize(ctx->stream));
    PQH_HIP(ctx, hipMemsetAsync(ctx->d_diag + 2, 0, 8, ctx->stream));
    return e ? pqh_set_error(ctx, PQH_ERR_CAPACITY, "stream buffer too small") : PQH_OK;
}

int pqh_codebooks_build(const double* counts, int m, int k, int context,
                        huffman_codebook_t* codebooks, int num_threads) {
    if (!counts || m <= 0 || k <= 0 || !codebooks) return PQH_ERR_ARG;
    const long long items = context ? (long long)k * k : k;
    auto work = [&](int i) {
        if (context) huffman_codebook_context_encode_init(&codebooks[i], k, counts + i * items);
        else huffman_codebook_encode_init(&codebooks[i], k, counts + i * items);
    };
    if (num_threads <= 1 || m == 1) {
        for (int i = 0; i < m; ++i) work(i);
        return PQH_OK;
    }
    std::vector<std::thread> pool;
    const int nt = std::min(num_threads, m);
    for (int w = 0; w < nt; ++w)
        pool.emplace_back([&, w] {
            for (int i = w; i < m; i += nt) work(i);
        });
    for (auto& th : pool) th.join();
    return PQH_OK;
}

}  // extern "C"

// ---------------------------------------------------------------- tree-ordered coding
// Tree mode (huffman_encoder.c:240-286 + mst.c:407-490): the stream walks the rows in the DFS
// order of a spanning forest and codes each row in the context of its forest parent.  The
// order and parents come from pqh_tree_order (host); the device gathers the rows into stream
// order with their parents' codes beside them (tree_prev, 0xFFFF for a root), after which
// the histogram and the encoder are the context-mode ones with an explicit context row.
namespace {

constexpr int kTreeChunk = 61440;   // vectors per tree-histogram workgroup (< 65536: u16)

template <typename CodeT>
__global__ void __launch_bounds__(256)
tree_gather(const CodeT* __restrict__ codes, long long n, int m,
            const uint32_t* __restrict__ vertices, const long long* __restrict__ parents,
            CodeT* __restrict__ rows, uint16_t* __restrict__ tree_prev,
            unsigned long long* __restrict__ err) {
    const long long p = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (p >= n) return;
    const long long v = vertices[p];
    const long long par = parents[p];
    const bool bad = v >= n || par >= n;
    if (bad) atomicOr(err, 1ull);   // an id outside the rows: reported, nothing read
    if (sizeof(CodeT) == 1 && (m & 7) == 0) {   // whole 8-byte groups: wide loads and stores
        for (int q = 0; q < m / 8; ++q) {
            const unsigned long long c =
                bad ? 0ull : reinterpret_cast<const unsigned long long*>(codes + v * m)[q];
            const unsigned long long pc =
                (bad || par < 0) ? 0ull : reinterpret_cast<const unsigned long long*>(codes + par * m)[q];
            reinterpret_cast<unsigned long long*>(rows + p * m)[q] = c;
            unsigned long long w[2];
#pragma unroll
            for (int h = 0; h < 2; ++h) {
                w[h] = 0;
#pragma unroll
                for (int b = 0; b < 4; ++b)
                    w[h] |= (unsigned long long)((bad || par < 0) ? 0xFFFFu
                                                 : (unsigned)((pc >> (8 * (4 * h + b))) & 0xFFu))
                            << (16 * b);
            }
            reinterpret_cast<unsigned long long*>(tree_prev + p * m)[2 * q] = w[0];
            reinterpret_cast<unsigned long long*>(tree_prev + p * m)[2 * q + 1] = w[1];
        }
        return;
    }
    for (int i = 0; i < m; ++i) {
        rows[p * m + i] = bad ? CodeT(0) : codes[v * m + i];
        tree_prev[p * m + i] = (bad || par < 0) ? uint16_t(0xFFFF) : uint16_t(codes[par * m + i]);
    }
}

// (parent code, code) pair counts of one part over a chunk of stream rows, as packed u16
// counters in LDS (k * k / 2 words; 128 KB at K = 256), flushed with one global atomic per
// non-zero counter (tree_collect_indices_stats, mst.c:442-490; roots are not counted).
template <typename CodeT>
__global__ void __launch_bounds__(1024)
hist_tree(const CodeT* __restrict__ rows, const uint16_t* __restrict__ tree_prev, long long n,
          int m_total, int k, uint32_t* __restrict__ counts) {
    extern __shared__ uint32_t pairs[];
    const int m = blockIdx.y;
    const int words = (k * k + 1) / 2;
    for (int w = threadIdx.x; w < words; w += blockDim.x) pairs[w] = 0;
    lds_barrier();
    const long long p0 = (long long)blockIdx.x * kTreeChunk;
    const long long p1 = p0 + kTreeChunk < n ? p0 + kTreeChunk : n;
    for (long long p = p0 + threadIdx.x; p < p1; p += blockDim.x) {
        const unsigned prev = tree_prev[p * m_total + m];
        const unsigned cur = (unsigned)rows[p * m_total + m];
        if (prev >= (unsigned)k || cur >= (unsigned)k) continue;   // root / out of alphabet
        const unsigned bin = prev * (unsigned)k + cur;
        atomicAdd(&pairs[bin >> 1], 1u << ((bin & 1u) * 16));
    }
    lds_barrier();
    uint32_t* out = counts + (long long)m * k * k;
    for (int w = threadIdx.x; w < words; w += blockDim.x) {
        const uint32_t c = pairs[w];
        if (c & 0xFFFFu) atomicAdd(&out[2 * w], c & 0xFFFFu);
        if ((c >> 16) && 2 * w + 1 < k * k) atomicAdd(&out[2 * w + 1], c >> 16);
    }
}

}  // namespace

int pqh_tree_gather(pqh_ctx_t* ctx, const void* d_codes, long long n, int m, int k,
                    const uint32_t* d_vertices, const long long* d_parents, void* d_rows,
                    uint16_t* d_tree_prev) {
    if (!ctx || n < 0 || m <= 0 || k <= 0 || k > 4096) return PQH_ERR_ARG;
    if (n > 0 && (!d_codes || !d_vertices || !d_parents || !d_rows || !d_tree_prev))
        return PQH_ERR_ARG;
    int rc = pqh_use_device(ctx);
    if (rc) return rc;
    if (n == 0) return PQH_OK;
    const unsigned blocks = (unsigned)((n + 255) / 256);
    if (k <= 256)
        hipLaunchKernelGGL(tree_gather<uint8_t>, dim3(blocks), dim3(256), 0, ctx->stream,
                           static_cast<const uint8_t*>(d_codes), n, m, d_vertices, d_parents,
                           static_cast<uint8_t*>(d_rows), d_tree_prev, ctx->d_diag + 7);
    else
        hipLaunchKernelGGL(tree_gather<uint16_t>, dim3(blocks), dim3(256), 0, ctx->stream,
                           static_cast<const uint16_t*>(d_codes), n, m, d_vertices, d_parents,
                           static_cast<uint16_t*>(d_rows), d_tree_prev, ctx->d_diag + 7);
    PQH_LAUNCH_CHECK(ctx);
    return PQH_OK;
}

int pqh_tree_status(pqh_ctx_t* ctx) {
    if (!ctx) return PQH_ERR_ARG;
    unsigned long long e = 0;
    PQH_HIP(ctx, hipMemcpyAsync(&e, ctx->d_diag + 7, 8, hipMemcpyDeviceToHost, ctx->stream));
    PQH_HIP(ctx, hipStreamSynchronize(ctx->stream));
    PQH_HIP(ctx, hipMemsetAsync(ctx->d_diag + 7, 0, 8, ctx->stream));
    return e ? pqh_set_error(ctx, PQH_ERR_ARG, "tree order names a row outside the input") : PQH_OK;
}

int pqh_histogram_tree(pqh_ctx_t* ctx, const void* d_rows, const uint16_t* d_tree_prev,
                       long long n, int m, int k, uint32_t* d_counts) {
    if (!ctx || n < 0 || m <= 0 || k <= 0 || !d_counts) return PQH_ERR_ARG;
    if (k > 256) return PQH_ERR_UNSUPPORTED;   // context alphabets are K = 256 (mst.c:440)
    if (n > 0 && (!d_rows || !d_tree_prev)) return PQH_ERR_ARG;
    int rc = pqh_use_device(ctx);
    if (rc) return rc;
    if (n == 0) return PQH_OK;
    const unsigned chunks = (unsigned)((n + kTreeChunk - 1) / kTreeChunk);
    const size_t lds = (size_t)((k * k + 1) / 2) * 4;
    PQH_HIP(ctx, hipFuncSetAttribute((const void*)hist_tree<uint8_t>,
                                     hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
    hipLaunchKernelGGL(hist_tree<uint8_t>, dim3(chunks, m), dim3(1024), lds, ctx->stream,
                       static_cast<const uint8_t*>(d_rows), d_tree_prev, n, m, k, d_counts);
    PQH_LAUNCH_CHECK(ctx);
    return PQH_OK;
}

int pqh_encode_tree_write(pqh_ctx_t* ctx, const pqh_tables_t* t, const void* d_rows,
                          const uint16_t* d_tree_prev, long long n,
                          unsigned long long bit_offset, unsigned char* d_out,
                          unsigned long long out_bytes, int chunk_vectors,
                          unsigned long long* d_chunk_offsets, unsigned long long* d_total_bits) {
    if (!ctx || !t || !t->context || t->k > 256 || (n > 0 && !d_tree_prev)) return PQH_ERR_ARG;
    return encode_write_impl(ctx, t, d_rows, n, 1, nullptr, bit_offset, nullptr, d_out,
                             out_bytes, chunk_vectors, d_chunk_offsets, nullptr, d_total_bits,
                             d_tree_prev);
}
