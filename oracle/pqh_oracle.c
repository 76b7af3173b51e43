/*
 * pqh_oracle.c -- TEST INFRASTRUCTURE ONLY: the CPU oracle for the pq_huffman hot path.
 *
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load this
 * (as oracle/_build/liboracle.so, via ctypes).  The product (pq_huffman_amd) never links
 * or calls it.  It is a plain, scalar, array-oriented restatement of the reference
 * algorithm, written independently of the product's drop-in library so that the two do
 * not share bugs.  Every function cites the reference code it restates.
 *
 * Pinning (see tests/test_oracle_golden.py):
 *   - Huffman/bitstream/codebook/stats: pinned byte-for-byte against outputs of the
 *     reference itself built from /root/reference/src (oracle/ref.mk -> oracle/_ref),
 *     committed as fixtures under tests/golden/ by oracle/gen_golden.py, and against the
 *     reference's embedded known-answer tests (bitstream.c:196-228,
 *     huffman_encode.c:280-323, huffman_decode.c:193-288, huffman_codebook.c:145-221).
 *   - PQ assignment: "parity unpinned" at the yael boundary.  The reference assigns
 *     inside yael kmeans() (pq_encoder.c:270-272; yael v438 is not vendored and absent
 *     here).  The oracle defines assignment as the direct-form fp32 distance
 *     sum_j (x_j - c_kj)^2 accumulated in j order with separate rounding of the product
 *     and the sum (the form of compute_nn_fast.c:304-311 get_real_dist, compiled
 *     -ffp-contract=off like gcc -std=c99 does), argmin with the FIRST minimum winning.
 */
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

/* ------------------------------------------------------------------------------------
 * Huffman tree: restates huffman_encode.c:33-76 (binary heap with its exact tie-breaks),
 * :141-192 (tree build, 1-symbol special case) and :100-132 (code assignment: child 1
 * first, bit 1 for child 1).
 * ---------------------------------------------------------------------------------- */
typedef struct {
    int alphabet;
    double* cnt;   /* 2*alphabet nodes */
    int* sym;      /* symbol id for leaves, -1 for internal */
    int* ch0;
    int* ch1;
    int* heap;
    int hsize;
} orc_tree_t;

static void orc_heap_push(orc_tree_t* t, int e) {
    int i = t->hsize++;
    while (i > 0) {
        int p = (i + 1) / 2 - 1;
        if (t->cnt[e] >= t->cnt[t->heap[p]]) break;      /* huffman_encode.c:38 */
        t->heap[i] = t->heap[p];
        i = p;
    }
    t->heap[i] = e;
}

static int orc_heap_pop(orc_tree_t* t) {
    int res = t->heap[0];
    int last = t->heap[--t->hsize];
    int i = 0;
    while (i < t->hsize) {
        int l = 2 * i + 1, r = 2 * i + 2;
        if (l < t->hsize && t->cnt[last] > t->cnt[t->heap[l]] &&
            (r >= t->hsize || t->cnt[t->heap[l]] <= t->cnt[t->heap[r]])) {   /* :56-59 */
            t->heap[i] = t->heap[l];
            i = l;
        } else if (r < t->hsize && t->cnt[last] > t->cnt[t->heap[r]] &&
                   t->cnt[t->heap[r]] <= t->cnt[t->heap[l]]) {                 /* :63-66 */
            t->heap[i] = t->heap[r];
            i = r;
        } else {
            break;
        }
    }
    t->heap[i] = last;
    return res;
}

/* returns root node index or -1 when no symbol has a positive count */
static int orc_build_tree(orc_tree_t* t, int alphabet, const double* counts) {
    int nn = 2 * alphabet + 1;
    t->alphabet = alphabet;
    t->cnt = calloc(nn, sizeof(double));
    t->sym = malloc(nn * sizeof(int));
    t->ch0 = malloc(nn * sizeof(int));
    t->ch1 = malloc(nn * sizeof(int));
    t->heap = malloc((alphabet + 1) * sizeof(int));
    t->hsize = 0;
    for (int i = 0; i < nn; ++i) {
        t->ch0[i] = t->ch1[i] = -1;
        t->sym[i] = i < alphabet ? i : -1;
        t->cnt[i] = i < alphabet ? counts[i] : 0.0;
    }
    for (int i = 0; i < alphabet; ++i) {
        if (counts[i] > 0.0f) orc_heap_push(t, i);          /* huffman_encode.c:158 */
    }
    int used = alphabet;
    if (t->hsize == 1) {                                    /* :168-177 */
        int leaf = orc_heap_pop(t);
        int nd = used++;
        t->cnt[nd] = t->cnt[leaf];
        t->ch0[nd] = leaf;
        orc_heap_push(t, nd);
    }
    while (t->hsize > 1) {                                  /* :179-188 */
        int z = orc_heap_pop(t);
        int o = orc_heap_pop(t);
        int nd = used++;
        t->cnt[nd] = t->cnt[z] + t->cnt[o];
        t->ch0[nd] = z;
        t->ch1[nd] = o;
        orc_heap_push(t, nd);
    }
    return t->hsize ? t->heap[0] : -1;
}

static void orc_free_tree(orc_tree_t* t) {
    free(t->cnt); free(t->sym); free(t->ch0); free(t->ch1); free(t->heap);
}

static void orc_assign_codes(const orc_tree_t* t, int node, int depth, unsigned char* cur,
                             int* lens, unsigned char* codes, int stride, int* maxlen) {
    if (node < 0) return;
    if (t->sym[node] >= 0) {
        int s = t->sym[node];
        lens[s] = depth;
        if (depth > *maxlen) *maxlen = depth;
        int nb = (depth + 7) / 8;
        if (nb > stride) nb = stride;
        memcpy(codes + (size_t)s * stride, cur, nb);
        return;
    }
    int byte = depth / 8, bit = 7 - depth % 8;
    cur[byte] |= (unsigned char)(1u << bit);                /* child 1 first, bit 1 */
    orc_assign_codes(t, t->ch1[node], depth + 1, cur, lens, codes, stride, maxlen);
    cur[byte] &= (unsigned char)~(1u << bit);
    orc_assign_codes(t, t->ch0[node], depth + 1, cur, lens, codes, stride, maxlen);
}

/* Codebook for `rows` independent trees of `alphabet` symbols (rows = alphabet for a
 * context codebook, huffman_encode.c:235-269; rows = 1 otherwise).  lens[rows*alphabet],
 * codes[rows*alphabet][stride] left-aligned MSB-first, zero padded.  Returns max length
 * (or -1 if some code needs more than stride bytes). */
int orc_codebook(int alphabet, int rows, const double* counts, int* lens, unsigned char* codes,
                 int stride) {
    int maxlen = 0;
    unsigned char* cur = calloc(alphabet + 8, 1);
    memset(codes, 0, (size_t)rows * alphabet * stride);
    for (int r = 0; r < rows; ++r) {
        orc_tree_t t;
        int root = orc_build_tree(&t, alphabet, counts + (size_t)r * alphabet);
        for (int s = 0; s < alphabet; ++s) lens[(size_t)r * alphabet + s] = 0;
        memset(cur, 0, alphabet + 8);
        orc_assign_codes(&t, root, 0, cur, lens + (size_t)r * alphabet,
                         codes + (size_t)r * alphabet * stride, stride, &maxlen);
        orc_free_tree(&t);
    }
    free(cur);
    return maxlen > stride * 8 ? -1 : maxlen;
}

/* ------------------------------------------------------------------------------------
 * Bit writer: restates bitstream.c bit-serial writer, MSB-first within bytes, zero pad on
 * destroy (bitstream.c:71-150).  The 128 MiB buffering is not observable in outputs.
 * ---------------------------------------------------------------------------------- */
typedef struct {
    unsigned char* buf;
    long long cap;
    long long bits;
    int overflow;
} orc_bw_t;

static void orc_bw_put(orc_bw_t* w, const unsigned char* data, long long nbits) {
    for (long long i = 0; i < nbits; ++i) {
        int b = (data[i / 8] >> (7 - i % 8)) & 1;
        long long pos = w->bits + i;
        if (pos / 8 >= w->cap) { w->overflow = 1; continue; }
        if (b) w->buf[pos / 8] |= (unsigned char)(1u << (7 - pos % 8));
        else w->buf[pos / 8] &= (unsigned char)~(1u << (7 - pos % 8));
    }
    w->bits += nbits;
}

/* varint bit length, huffman_codebook.c:43-59 */
static long long orc_put_varint(unsigned char* out, long long pos, unsigned v) {
    unsigned rest = v;
    int cont = 1;
    for (int i = 0; i < 4 && cont; ++i) {
        unsigned char byte = rest & 0x7f;
        cont = (rest != byte);
        if (cont) byte |= 0x80;
        out[pos++] = byte;
        rest >>= 7;
    }
    return pos;
}

/* huffman_codebook_save (huffman_codebook.c:74-94) into a byte buffer; returns bytes
 * written or -1 if cap is too small. */
long long orc_codebook_serialize(int alphabet, int is_context, const int* lens,
                                 const unsigned char* codes, int stride, unsigned char* out,
                                 long long cap) {
    long long items = is_context ? (long long)alphabet * alphabet : alphabet;
    long long need = 5 + items * 4;
    long long codebits = 0;
    for (long long i = 0; i < items; ++i) codebits += lens[i];
    need += (codebits + 7) / 8;
    if (need > cap) return -1;
    long long pos = 0;
    memcpy(out, &alphabet, 4);
    pos = 4;
    out[pos++] = (unsigned char)is_context;
    for (long long i = 0; i < items; ++i) pos = orc_put_varint(out, pos, (unsigned)lens[i]);
    orc_bw_t w = {out + pos, cap - pos, 0, 0};
    memset(out + pos, 0, (codebits + 7) / 8);
    for (long long i = 0; i < items; ++i) orc_bw_put(&w, codes + i * stride, lens[i]);
    return pos + (w.bits + 7) / 8;
}

/* ------------------------------------------------------------------------------------
 * Histograms: huffman_encoder.c:139-164 (non-context, counts[i*K + c]) and :166-205
 * (context, counts[i*K*K + (prev<<8) + cur], v >= 1).  Codes are u8 (esize 1) or u16.
 * ---------------------------------------------------------------------------------- */
static inline unsigned orc_sym(const void* c, int es, long long i) {
    return es == 1 ? ((const unsigned char*)c)[i] : ((const unsigned short*)c)[i];
}

void orc_histogram(const void* codes, int esize, long long n, int m, int k, int context,
                   double* counts) {
    long long per = context ? (long long)k * k : k;
    memset(counts, 0, sizeof(double) * per * m);
    for (long long v = context ? 1 : 0; v < n; ++v) {
        for (int i = 0; i < m; ++i) {
            unsigned cur = orc_sym(codes, esize, v * m + i);
            long long idx = cur;
            if (context) idx += (long long)orc_sym(codes, esize, (v - 1) * m + i) * k;
            counts[i * per + idx] += 1;
        }
    }
}

/* ------------------------------------------------------------------------------------
 * Stream encode: encode_non_context_data / encode_context_data (huffman_encoder.c:207-238);
 * row-major over vectors, then parts; context: row 0 raw 8 bits per part (:234).
 * codetab: per part [items][stride].  Returns total bits or -1 on overflow.
 * ---------------------------------------------------------------------------------- */
long long orc_encode(const void* codes, int esize, long long n, int m, int k, int context,
                     const int* lens, const unsigned char* codetab, int stride,
                     unsigned char* out, long long cap) {
    long long per = context ? (long long)k * k : k;
    orc_bw_t w = {out, cap, 0, 0};
    memset(out, 0, cap);
    for (long long v = 0; v < n; ++v) {
        for (int i = 0; i < m; ++i) {
            unsigned cur = orc_sym(codes, esize, v * m + i);
            if (context && v == 0) {
                unsigned char raw = (unsigned char)cur;
                orc_bw_put(&w, &raw, 8);
                continue;
            }
            long long idx = cur;
            if (context) idx += (long long)orc_sym(codes, esize, (v - 1) * m + i) * k;
            long long item = i * per + idx;
            orc_bw_put(&w, codetab + item * stride, lens[item]);
        }
    }
    return w.overflow ? -1 : w.bits;
}

/* ------------------------------------------------------------------------------------
 * Decode: restates the trie decoder (huffman_decode.c:30-191) driven by the CLI loop
 * (huffman_decoder.c:211-255, non-tree): per part a persistent decoder; context mode
 * warms up with ceil(log2 K) raw bits (huffman_decode.c:73-76).  Returns 0, or -1 on an
 * invalid code, -2 on running out of stream.
 * ---------------------------------------------------------------------------------- */
typedef struct {
    int* c0;
    int* c1;
    int* sym;
    int nodes;
    int cap;
} orc_trie_t;

static int orc_trie_node(orc_trie_t* t) {
    if (t->nodes == t->cap) {
        t->cap = t->cap ? t->cap * 2 : 1024;
        t->c0 = realloc(t->c0, t->cap * sizeof(int));
        t->c1 = realloc(t->c1, t->cap * sizeof(int));
        t->sym = realloc(t->sym, t->cap * sizeof(int));
    }
    t->c0[t->nodes] = t->c1[t->nodes] = -1;
    t->sym[t->nodes] = -1;
    return t->nodes++;
}

static int orc_decode_impl(const unsigned char* stream, long long stream_bytes, long long n,
                           int m, int k, int context, const int* lens,
                           const unsigned char* codetab, int stride, void* out, int esize,
                           const long long* parent_pos);

int orc_decode(const unsigned char* stream, long long stream_bytes, long long n, int m, int k,
               int context, const int* lens, const unsigned char* codetab, int stride,
               void* out, int esize) {
    return orc_decode_impl(stream, stream_bytes, n, m, k, context, lens, codetab, stride, out,
                           esize, NULL);
}

/* Tree-mode decode (huffman_decoder.c:214-247 with --tree): row v's context is the decoded
 * row at stream position parent_pos[v] (the traverser driven by the children stream), a
 * root (-1) restarts every part with HUFFMAN_NO_SYMBOL, i.e. the raw warm-up bits. */
int orc_decode_tree(const unsigned char* stream, long long stream_bytes, long long n, int m,
                    int k, const int* lens, const unsigned char* codetab, int stride,
                    void* out, const long long* parent_pos) {
    return orc_decode_impl(stream, stream_bytes, n, m, k, 1, lens, codetab, stride, out, 1,
                           parent_pos);
}

static int orc_decode_impl(const unsigned char* stream, long long stream_bytes, long long n,
                           int m, int k, int context, const int* lens,
                           const unsigned char* codetab, int stride, void* out, int esize,
                           const long long* parent_pos) {
    long long per = context ? (long long)k * k : k;
    int roots_per_part = context ? k : 1;
    orc_trie_t trie = {0};
    int* roots = malloc(sizeof(int) * m * roots_per_part);
    for (int i = 0; i < m; ++i) {
        for (int r = 0; r < roots_per_part; ++r) {
            int root = orc_trie_node(&trie);
            roots[i * roots_per_part + r] = root;
            for (int s = 0; s < k; ++s) {
                long long item = i * per + (long long)r * k + s;
                int L = lens[item];
                if (L == 0) continue;
                int nd = root;
                for (int b = 0; b < L; ++b) {
                    int bit = (codetab[item * stride + b / 8] >> (7 - b % 8)) & 1;
                    int nx = bit ? trie.c1[nd] : trie.c0[nd];
                    if (nx < 0) {
                        nx = orc_trie_node(&trie);
                        if (bit) trie.c1[nd] = nx; else trie.c0[nd] = nx;
                    }
                    nd = nx;
                }
                trie.sym[nd] = s;
            }
        }
    }
    int warm = 1;
    while ((1 << warm) < k) ++warm;
    int* prev = malloc(sizeof(int) * m);
    for (int i = 0; i < m; ++i) prev[i] = -1;
    long long pos = 0, total = stream_bytes * 8;
    int rc = 0;
    for (long long v = 0; v < n && !rc; ++v) {
        if (parent_pos)
            for (int i = 0; i < m; ++i)
                prev[i] = parent_pos[v] < 0 ? -1 : ((unsigned char*)out)[parent_pos[v] * m + i];
        for (int i = 0; i < m; ++i) {
            int s;
            if (context && prev[i] < 0) {
                if (pos + warm > total) { rc = -2; break; }
                s = 0;
                for (int b = 0; b < warm; ++b, ++pos) s = (s << 1) | ((stream[pos / 8] >> (7 - pos % 8)) & 1);
            } else {
                int nd = roots[i * roots_per_part + (context ? prev[i] : 0)];
                for (;;) {
                    if (pos >= total) { rc = -2; break; }
                    int bit = (stream[pos / 8] >> (7 - pos % 8)) & 1;
                    ++pos;
                    nd = bit ? trie.c1[nd] : trie.c0[nd];
                    if (nd < 0) { rc = -1; break; }
                    if (trie.sym[nd] >= 0) break;
                }
                if (rc) break;
                s = trie.sym[nd];
            }
            prev[i] = s;
            if (esize == 1) ((unsigned char*)out)[v * m + i] = (unsigned char)s;
            else ((unsigned short*)out)[v * m + i] = (unsigned short)s;
        }
    }
    free(prev); free(roots); free(trie.c0); free(trie.c1); free(trie.sym);
    return rc;
}

/* ------------------------------------------------------------------------------------
 * Sort mode: qsort(rows, strncmp(.,.,m)) (huffman_encoder.c:301-317).  strncmp stops at
 * the first 0 byte, so the order is the stable order of key(row) = row with every byte
 * after the first 0 set to 0 (glibc 2.35 qsort = stable merge sort).  Restated with an
 * explicit stable merge sort so the result does not depend on the libc.
 * ---------------------------------------------------------------------------------- */
static int orc_rowcmp(const unsigned char* a, const unsigned char* b, int m) {
    for (int i = 0; i < m; ++i) {
        if (a[i] != b[i]) return (int)a[i] - (int)b[i];
        if (a[i] == 0) return 0;
    }
    return 0;
}

static void orc_msort(unsigned char* a, unsigned char* tmp, long long n, int m) {
    if (n < 2) return;
    long long h = n / 2;
    orc_msort(a, tmp, h, m);
    orc_msort(a + h * m, tmp, n - h, m);
    long long i = 0, j = h, o = 0;
    while (i < h && j < n) {
        if (orc_rowcmp(a + j * m, a + i * m, m) < 0) { memcpy(tmp + o * m, a + j * m, m); ++j; }
        else { memcpy(tmp + o * m, a + i * m, m); ++i; }
        ++o;
    }
    while (i < h) { memcpy(tmp + o * m, a + i * m, m); ++i; ++o; }
    while (j < n) { memcpy(tmp + o * m, a + j * m, m); ++j; ++o; }
    memcpy(a, tmp, n * m);
}

void orc_sort_rows(unsigned char* rows, long long n, int m) {
    unsigned char* tmp = malloc((size_t)(n > 0 ? n : 1) * m);
    orc_msort(rows, tmp, n, m);
    free(tmp);
}

/* ------------------------------------------------------------------------------------
 * PQ assignment (see header): direct form, j order, separate rounding, first minimum.
 * x: n x d (row-major fp32), centroids: [m][k][d/m] (pq_centroids.fvecsl order,
 * pq_encoder.c:227-255).  codes: n x m (esize 1 or 2), dists (optional): n x m.
 * threads <= 0: all OpenMP threads.
 * ---------------------------------------------------------------------------------- */
void orc_pq_assign(const float* x, long long n, int d, int m, int k, const float* cent,
                   void* codes, int esize, float* dists, int threads) {
    int ds = d / m;
#ifdef _OPENMP
    if (threads <= 0) threads = omp_get_max_threads();
#pragma omp parallel for schedule(static) num_threads(threads)
#endif
    for (long long v = 0; v < n; ++v) {
        for (int i = 0; i < m; ++i) {
            const float* xs = x + v * d + (long long)i * ds;
            const float* cb = cent + (size_t)i * k * ds;
            float best = INFINITY;
            int code = 0;
            for (int c = 0; c < k; ++c) {
                float acc = 0.0f; /* SSE fp32: each step rounded, no contraction */
                for (int j = 0; j < ds; ++j) {
                    float diff = xs[j] - cb[(size_t)c * ds + j];
                    float sq = diff * diff;
                    acc = acc + sq;
                }
                if (acc < best) { best = acc; code = c; }
            }
            if (esize == 1) ((unsigned char*)codes)[v * m + i] = (unsigned char)code;
            else ((unsigned short*)codes)[v * m + i] = (unsigned short)code;
            if (dists) dists[v * m + i] = best;
        }
    }
}

/* Deterministic Lloyd k-means (the build's replacement for yael's training, SURVEY 8f-2;
 * NOT the reference's algorithm -- yael is absent): iters x { exact assignment as
 * orc_pq_assign; centroid = mean of its members, accumulated in 64-bit fixed point
 * x * 2^s, s = 61 - ceil(log2(max|x| * n)) clamped to [-126, 100]; empty clusters keep
 * their centroid }.  The GPU trainer (pqh_kmeans.hip) must match this bit for bit. */
int orc_kmeans_shift(float max_abs, long long n) {
    if (!(max_abs > 0.0f) || n <= 0) return 40;
    if (isinf(max_abs)) return -126;
    double b = (double)max_abs * (double)n;
    int s = 61 - (int)ceil(log2(b));
    if (s < -126) s = -126;
    if (s > 100) s = 100;
    return s;
}

void orc_kmeans(const float* x, long long n, int d, int m, int k, int iters, float* cent,
                int threads) {
    int ds = d / m;
    float mx = 0.0f;
    for (long long e = 0; e < n * d; ++e) {
        float a = fabsf(x[e]);
        if (isnan(a)) a = INFINITY;
        if (a > mx) mx = a;
    }
    int s = orc_kmeans_shift(mx, n);
    int esize = k <= 256 ? 1 : 2;
    void* codes = malloc((size_t)n * m * esize + 1);
    long long* sums = (long long*)malloc(sizeof(long long) * (size_t)m * k * ds);
    unsigned long long* cnt = (unsigned long long*)malloc(sizeof(unsigned long long) * (size_t)m * k);
    for (int it = 0; it < iters; ++it) {
        orc_pq_assign(x, n, d, m, k, cent, codes, esize, NULL, threads);
        memset(sums, 0, sizeof(long long) * (size_t)m * k * ds);
        memset(cnt, 0, sizeof(unsigned long long) * (size_t)m * k);
        for (long long v = 0; v < n; ++v)
            for (int i = 0; i < m; ++i) {
                unsigned c = orc_sym(codes, esize, v * m + i);
                cnt[(size_t)i * k + c]++;
                for (int j = 0; j < ds; ++j)
                    sums[((size_t)i * k + c) * ds + j] +=
                        llrint(ldexp((double)x[v * d + (long long)i * ds + j], s));
            }
        for (size_t q = 0; q < (size_t)m * k; ++q)
            if (cnt[q])
                for (int j = 0; j < ds; ++j)
                    cent[q * ds + j] = (float)ldexp((double)sums[q * ds + j] / (double)cnt[q], -s);
    }
    free(codes);
    free(sums);
    free(cnt);
}

/* compute_error (pq_encoder.c:82-119): mean over vectors of sum (double) of squared fp32
 * deltas. */
double orc_compute_error(const float* x, long long n, int d, int m, int k, const float* cent,
                         const void* codes, int esize) {
    int ds = d / m;
    double sum = 0.0;
    for (long long v = 0; v < n; ++v) {
        for (int i = 0; i < m; ++i) {
            unsigned c = orc_sym(codes, esize, v * m + i);
            for (int j = 0; j < ds; ++j) {
                float delta = x[v * d + (long long)i * ds + j] - cent[((size_t)i * k + c) * ds + j];
                sum += 1.0 * delta * delta;
            }
        }
    }
    return sum / n;
}

/* huffman_estimate_size (huffman_encode.c:271-277) per part */
double orc_estimate_size(const int* lens, const double* counts, long long items) {
    double r = 0;
    for (long long i = 0; i < items; ++i) r += counts[i] * lens[i];
    return r;
}

/* huffman_stats_print_file (stats.c:38-76) into buf; returns length. */
static int orc_stats_impl(char* buf, int cap, double bits, int m, long long n) {
    return snprintf(buf, cap, "\"length_bit\": %.1lf, \"length_bytes\": %.1lf, "
                    "\"compression_rate\": %.3lf, \"bits_per_byte\": %.2lf",
                    bits, bits / 8, bits / (n * m * 8), bits / (n * m));
}

int orc_stats_json(long long n, int m, int k, int num_roots, const double* partial, char* buf,
                   int cap) {
    int p = snprintf(buf, cap, "{\"num_vectors\": %lld, \"m\": %d, \"k_star\": %d, ", n, m, k);
    double add = 8.0 * num_roots, sum = 0.0;
    for (int i = 0; i < m; ++i) sum += partial[i];
    p += orc_stats_impl(buf + p, cap - p, sum + add * m, m, n);
    if (num_roots) p += snprintf(buf + p, cap - p, ", \"num_roots\": %d", num_roots);
    p += snprintf(buf + p, cap - p, ", \"partials\": [");
    for (int i = 0; i < m; ++i) {
        if (i) p += snprintf(buf + p, cap - p, ", ");
        p += snprintf(buf + p, cap - p, "{");
        p += orc_stats_impl(buf + p, cap - p, partial[i] + add, 1, n);
        p += snprintf(buf + p, cap - p, "}");
    }
    p += snprintf(buf + p, cap - p, "]}\n");
    return p;
}

/* Raw writer check: concatenate num writes (data packed per write, ceil(len/8) bytes each)
 * MSB-first and zero-pad (bitstream.c:71-150).  Returns bytes written. */
long long orc_bitstream_write(const unsigned char* data, const long long* lens, int num,
                              unsigned char* out, long long cap) {
    orc_bw_t w = {out, cap, 0, 0};
    memset(out, 0, cap);
    const unsigned char* p = data;
    for (int i = 0; i < num; ++i) {
        orc_bw_put(&w, p, lens[i]);
        p += (lens[i] + 7) / 8;
    }
    return w.overflow ? -1 : (w.bits + 7) / 8;
}

/* ------------------------------------------------------------------------------------
 * Tree mode (huffman_encoder.c --tree <mst.tree>).
 * orc_tree_order: tree_collect_vertices_dfs (mst.c:290-364) over the loaded forest
 * (tree_load_file + restore_tree_edges_pointers, mst.c:52-61,273-288): adjacency of vertex
 * v = targets[sum(counts[<v]) ...][counts[v]]; returns num_roots.
 * orc_tree_parents: the tree_traverser (mst.c:366-405) replayed over num_children; ids[p]
 * is what gets pushed (vertex ids for the encoder, NULL = stream positions for the decoder,
 * huffman_decoder.c:245).  out[p] = the active parent before row p, -1 if none.
 * ---------------------------------------------------------------------------------- */
int orc_tree_order(long long nv, long long ne, const unsigned* targets, const int* counts,
                   unsigned* vertices, int* num_children) {
    long long* first = malloc(sizeof(long long) * (nv + 1));
    unsigned* stack = malloc(sizeof(unsigned) * (nv ? nv : 1));
    char* seen = calloc(nv ? nv : 1, 1);
    first[0] = 0;
    for (long long v = 0; v < nv; ++v) first[v + 1] = first[v] + counts[v];
    if (first[nv] != ne) { free(first); free(stack); free(seen); return -1; }
    long long done = 0, sp = 0;
    unsigned root = 0;
    int roots = 0;
    while (done < nv) {
        if (sp == 0) {
            while (root < nv && seen[root]) ++root;
            stack[sp++] = root;
            seen[root] = 1;
            ++roots;
        }
        unsigned cur = stack[--sp];
        vertices[done] = cur;
        int c = 0;
        for (long long e = first[cur]; e < first[cur + 1]; ++e) c += !seen[targets[e]];
        num_children[done++] = c;
        for (long long e = first[cur]; e < first[cur + 1]; ++e)
            if (!seen[targets[e]]) { seen[targets[e]] = 1; stack[sp++] = targets[e]; }
    }
    free(first); free(stack); free(seen);
    return roots;
}

void orc_tree_parents(long long n, const unsigned* ids, const int* num_children,
                      long long* out) {
    long long* sv = malloc(sizeof(long long) * (n ? n : 1));
    int* sc = malloc(sizeof(int) * (n ? n : 1));
    long long sp = 0;
    for (long long p = 0; p < n; ++p) {
        out[p] = sp ? sv[sp - 1] : -1;
        if (sp && --sc[sp - 1] == 0) --sp;
        if (num_children[p]) { sv[sp] = ids ? ids[p] : p; sc[sp] = num_children[p]; ++sp; }
    }
    free(sv); free(sc);
}

/* tree_collect_indices_stats (mst.c:442-490): pairs (codes[parent], codes[vertex]). */
void orc_tree_histogram(const unsigned char* codes, long long n, int m, int k,
                        const unsigned* vertices, const long long* parents, double* counts) {
    long long per = (long long)k * k;
    memset(counts, 0, sizeof(double) * per * m);
    for (long long p = 0; p < n; ++p) {
        if (parents[p] < 0) continue;
        for (int i = 0; i < m; ++i)
            counts[i * per + (long long)codes[parents[p] * m + i] * k + codes[(long long)vertices[p] * m + i]] += 1;
    }
}

/* encode_tree_data (huffman_encoder.c:240-286): rows in DFS order, context = parent's code,
 * roots raw 8 bits per part.  Returns total bits or -1 on overflow. */
long long orc_tree_encode(const unsigned char* codes, long long n, int m, int k,
                          const unsigned* vertices, const long long* parents, const int* lens,
                          const unsigned char* codetab, int stride, unsigned char* out,
                          long long cap) {
    long long per = (long long)k * k;
    orc_bw_t w = {out, cap, 0, 0};
    memset(out, 0, cap);
    for (long long p = 0; p < n; ++p) {
        const unsigned char* cur = codes + (long long)vertices[p] * m;
        for (int i = 0; i < m; ++i) {
            if (parents[p] < 0) { orc_bw_put(&w, cur + i, 8); continue; }
            long long item = i * per + (long long)codes[parents[p] * m + i] * k + cur[i];
            orc_bw_put(&w, codetab + item * stride, lens[item]);
        }
    }
    return w.overflow ? -1 : w.bits;
}

/* ------------------------------------------------------------------------------------
 * Forest builder (tree mode's kNN graph and minimum spanning forest).
 *
 * orc_knn_blocks_info: blocks_info_init + dimension_info_build (fast_nn_blocks_info.c:52-112):
 * split i (0 <= i < ns) is coordinate ns-1-i; its sorted values (qsort with float_cmp,
 * :41-50 -- the same glibc qsort, so near-equal values land where the reference puts them)
 * give block b the range [v[N b/nb - ov], v[min(N (b+1)/nb + ov, N-1)]], ov = (long long)
 * (N overlap / 2), with the outer ends pushed out by 1.0.  starts/ends: [ns][nb] floats.
 * ---------------------------------------------------------------------------------- */
static int orc_float_cmp(const void* a, const void* b) {
    float v = *(const float*)a - *(const float*)b;
    if (fabs(v) < 1e-9) return 0;
    return v < 0 ? -1 : 1;
}

void orc_knn_blocks_info(const float* x, long long n, int d, int ns, int nb, double overlap,
                         float* starts, float* ends) {
    float* vals = malloc(sizeof(float) * (n ? n : 1));
    for (int i = 0; i < ns; ++i) {
        const int coord = ns - 1 - i;
        for (long long v = 0; v < n; ++v) vals[v] = x[v * d + coord];
        qsort(vals, n, sizeof(float), orc_float_cmp);
        const long long ov = (long long)(n * overlap / 2);
        for (int b = 0; b < nb; ++b) {
            long long s = n * b / nb - ov;
            s = s < 0 ? 0 : (s > n ? n : s);
            starts[i * nb + b] = vals[s];
            long long e = n * (b + 1) / nb + ov;
            e = e < 0 ? 0 : (e > n ? n : e);
            ends[i * nb + b] = vals[e < n - 1 ? e : n - 1];
        }
        starts[i * nb] = vals[0] - 1.0;
        ends[i * nb + nb - 1] = vals[n - 1] + 1.0;
    }
    free(vals);
}

/* is_vector_in_block (fast_nn_blocks_info.c:187-239): block id digit of split i is
 * (B / nb^(ns-1-i)) % nb; inside means start <= x <= end on every split. */
int orc_in_block(const float* vec, int ns, int nb, const float* starts, const float* ends,
                 long long block) {
    for (int i = 0; i < ns; ++i) {
        const int coord = ns - 1 - i;
        long long mask = 1;
        for (int q = 0; q < coord; ++q) mask *= nb;
        const long long b = block / mask % nb;
        const float val = vec[coord];
        if (val < starts[i * nb + b] || val > ends[i * nb + b]) return 0;
    }
    return 1;
}

typedef struct { unsigned index; float dist; } orc_nn_t;

/* fast_nn_heap_push_impl / _push / _sort (fast_nn_temp_file.c:11-63): a max-heap of num_nn
 * (index, dist) items, initialised to (UINT_MAX, +inf) (:93-108); a candidate enters when
 * it is strictly closer than the root and its index is not in the heap. */
static void orc_nn_sift(orc_nn_t* heap, orc_nn_t item, int k) {
    int i = 0;
    for (;;) {
        const int l = 2 * i + 1, r = 2 * i + 2;
        int sw;
        if (r < k && heap[r].dist > heap[l].dist && heap[r].dist > item.dist) sw = r;
        else if (l < k && heap[l].dist > item.dist) sw = l;
        else break;
        heap[i] = heap[sw];
        i = sw;
    }
    heap[i] = item;
}

static void orc_nn_push(orc_nn_t* heap, orc_nn_t item, int k) {
    if (item.dist >= heap[0].dist) return;
    for (int q = 0; q < k; ++q)
        if (heap[q].index == item.index) return;
    orc_nn_sift(heap, item, k);
}

static void orc_nn_sort(orc_nn_t* heap, int k, unsigned* idx, float* dist) {
    while (--k >= 0) {
        idx[k] = heap[0].index;
        dist[k] = heap[0].dist;
        orc_nn_sift(heap, heap[k], k);
    }
}

static float orc_l2(const float* a, const float* b, int d) {
    float acc = 0.0f;   /* get_real_dist (compute_nn_fast.c:304-311), separate roundings */
    for (int j = 0; j < d; ++j) {
        const float t = a[j] - b[j];
        acc = acc + t * t;
    }
    return acc;
}

/* compute_nn_fast run/run_block/run_merge_block (compute_nn_fast.c:469-620) with one block
 * per pass (--num-dimensions-at-pass 0): blocks in id order, each block's members in row
 * order; the block kNN (yael knn_full_thread, :479-481 -- parity unpinned: yael is absent)
 * is defined as the num_nn_real + 1 smallest direct-form fp32 distances with the lower
 * block position first among equal distances; entries 1.. are pushed into the row's heap
 * (:490-507); temp_file_to_result sorts the heaps (fast_nn_temp_file.c:253-301).
 * Also reports (optional, may be NULL) every block's size. */
void orc_knn_fast(const float* x, long long n, int d, int num_nn, int ns, int nb,
                  const float* starts, const float* ends, unsigned* out_idx, float* out_dist,
                  long long* block_sizes, long long* log_row, unsigned* log_idx,
                  float* log_dist, long long* log_n) {
    /* log_*: when given, the heap pushes in the reference's order (single-threaded) */
    orc_nn_t* heaps = malloc(sizeof(orc_nn_t) * (size_t)(n ? n : 1) * num_nn);
    for (long long q = 0; q < n * num_nn; ++q) { heaps[q].index = 0xFFFFFFFFu; heaps[q].dist = INFINITY; }
    long long* mem = malloc(sizeof(long long) * (n ? n : 1));
    long long nblocks = 1;
    for (int i = 0; i < ns; ++i) nblocks *= nb;
    for (long long B = 0; B < nblocks; ++B) {
        long long S = 0;
        for (long long v = 0; v < n; ++v)
            if (orc_in_block(x + v * d, ns, nb, starts, ends, B)) mem[S++] = v;
        if (block_sizes) block_sizes[B] = S;
        if (S == 0) continue;
        const int nreal = (int)(num_nn < S - 1 ? num_nn : S - 1);
        const int kk = nreal + 1;
        #pragma omp parallel for schedule(dynamic, 16) if (!log_n)
        for (long long q = 0; q < S; ++q) {
            long long li[kk];   /* sorted by (dist, position) */
            float ld[kk];
            int cnt = 0;
            const float* xq = x + mem[q] * d;
            for (long long c = 0; c < S; ++c) {
                const float dd = orc_l2(xq, x + mem[c] * d, d);
                if (cnt == kk && !(dd < ld[kk - 1])) continue;
                int p = cnt < kk ? cnt++ : kk - 1;
                while (p > 0 && ld[p - 1] > dd) { ld[p] = ld[p - 1]; li[p] = li[p - 1]; --p; }
                ld[p] = dd;
                li[p] = c;
            }
            orc_nn_t* heap = heaps + mem[q] * num_nn;
            for (int j = 1; j < cnt; ++j) {
                orc_nn_t it = {(unsigned)mem[li[j]], ld[j]};
                if (log_n) {
                    log_row[*log_n] = mem[q];
                    log_idx[*log_n] = it.index;
                    log_dist[*log_n] = it.dist;
                    ++*log_n;
                }
                orc_nn_push(heap, it, num_nn);
            }
        }
    }
    for (long long v = 0; v < n; ++v)
        orc_nn_sort(heaps + v * num_nn, num_nn, out_idx + v * num_nn, out_dist + v * num_nn);
    free(mem);
    free(heaps);
}

/* mst_builder (mst_builder.c:98-131): load_mst_edges_from_nn_files (mst.c:80-171) keeps the
 * first `take` of each row's num_nn neighbours -- with a PQ penalty the row is first re-scored
 * (dist += Hamming(codes) * penalty, or = Hamming for an infinite penalty) and sorted;
 * minimum_spanning_tree (mst.c:173-236): qsort by distance (mst_dist_comparator, :15-26),
 * Kruskal over a DSU, then both directions of every kept edge sorted by source
 * (mst_source_comparator, :28-32).  glibc qsort as the reference calls it.  Outputs the
 * tree_save_file arrays (mst.c:253-265): edge targets (2 (kept) of them) and per-vertex
 * edge counts.  Returns the edge count, -1 for a neighbour id outside the rows. */
typedef struct { unsigned source, target; float dist; } orc_edge_t;

static int orc_edge_dist_cmp(const void* a, const void* b) {
    const float diff = ((const orc_edge_t*)a)->dist - ((const orc_edge_t*)b)->dist;
    if (fabs(diff) < 1e-9) return 0;
    return diff < 0 ? -1 : 1;
}

static int orc_edge_src_cmp(const void* a, const void* b) {
    const long long x = ((const orc_edge_t*)a)->source, y = ((const orc_edge_t*)b)->source;
    return (int)(x - y);
}

static unsigned orc_dsu_find(unsigned* parent, unsigned v) {
    unsigned r = v;
    while (parent[r] != r) r = parent[r];
    while (parent[v] != r) { const unsigned nx = parent[v]; parent[v] = r; v = nx; }
    return r;
}

long long orc_mst(long long n, int num_nn, int take, const unsigned* idx, const float* dist,
                  int pq_m, float penalty, const unsigned char* pq, unsigned* targets,
                  int* counts) {
    orc_edge_t* e = malloc(sizeof(orc_edge_t) * (size_t)(n * take > 0 ? n * take : 1));
    orc_edge_t* row = malloc(sizeof(orc_edge_t) * (size_t)(num_nn ? num_nn : 1));
    for (long long v = 0; v < n; ++v) {
        for (int j = 0; j < num_nn; ++j) {
            row[j].source = (unsigned)v;
            row[j].target = idx[v * num_nn + j];
            row[j].dist = dist[v * num_nn + j];
            if (row[j].target >= n) { free(e); free(row); return -1; }
            if (penalty > 0.0f) {
                int ham = 0;
                for (int i = 0; i < pq_m; ++i)
                    ham += pq[v * pq_m + i] != pq[(long long)row[j].target * pq_m + i];
                if (isinf(penalty)) row[j].dist = ham;
                else row[j].dist += ham * penalty;
            }
        }
        if (penalty > 0.0f) qsort(row, num_nn, sizeof(orc_edge_t), orc_edge_dist_cmp);
        memcpy(e + v * take, row, sizeof(orc_edge_t) * take);
    }
    free(row);
    const long long ne = n * take;
    qsort(e, ne, sizeof(orc_edge_t), orc_edge_dist_cmp);
    unsigned* parent = malloc(sizeof(unsigned) * (n ? n : 1));
    for (long long v = 0; v < n; ++v) { parent[v] = (unsigned)v; counts[v] = 0; }
    long long good = 0;
    for (long long q = 0; good + 1 < n && q < ne; ++q) {
        const unsigned a = orc_dsu_find(parent, e[q].source), b = orc_dsu_find(parent, e[q].target);
        if (a == b) continue;
        ++counts[e[q].source];
        parent[b] = a;
        const orc_edge_t t = e[q]; e[q] = e[good]; e[good] = t;
        ++good;
    }
    for (long long q = 0; q < good; ++q) {
        e[good + q].source = e[q].target;
        e[good + q].target = e[q].source;
        e[good + q].dist = e[q].dist;
        ++counts[e[q].target];
    }
    qsort(e, 2 * good, sizeof(orc_edge_t), orc_edge_src_cmp);
    for (long long q = 0; q < 2 * good; ++q) targets[q] = e[q].target;
    free(parent);
    free(e);
    return 2 * good;
}
