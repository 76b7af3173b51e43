/* huffman_encode.c -- codebook construction, drop-in for the reference's
 * src/huffman_encode.c:8-277.
 *
 * Bit-identical codes are a format requirement, so the tree is built with the same
 * binary-heap discipline as the reference (huffman_encode.c:33-76):
 *   push: sift up while the new weight is strictly smaller than the parent's;
 *   pop:  move the last element down, preferring the left child unless the right child
 *         is strictly lighter;
 * positive-count leaves are pushed in symbol order (:158), the first pop becomes child 0
 * and the second child 1 (:180-186), a lone symbol hangs under a new root as child 0
 * (:168-177).  Codes are read off the tree depth-first visiting child 1 (bit 1) before
 * child 0 (:100-132); items[i].code points into codefield in that visiting order.
 * Implementation: flat node arrays and an explicit DFS stack instead of the reference's
 * pointer tree and recursion.
 */
#include "huffman.h"

#include <stdlib.h>
#include <string.h>

typedef struct {
    double* w;
    int* sym;   /* leaf symbol, -1 for internal */
    int* kid0;
    int* kid1;
    int* heap;
    int heap_size;
    int used;
} hf_forest_t;

static void hf_alloc(hf_forest_t* f, int alphabet) {
    int cap = 2 * alphabet + 2;
    f->w = (double*)malloc(sizeof(double) * cap);
    f->sym = (int*)malloc(sizeof(int) * cap);
    f->kid0 = (int*)malloc(sizeof(int) * cap);
    f->kid1 = (int*)malloc(sizeof(int) * cap);
    f->heap = (int*)malloc(sizeof(int) * (alphabet + 2));
}

static void hf_free(hf_forest_t* f) {
    free(f->w); free(f->sym); free(f->kid0); free(f->kid1); free(f->heap);
}

static void hf_sift_in(hf_forest_t* f, int node) {
    int pos = f->heap_size++;
    double w = f->w[node];
    while (pos > 0) {
        int up = (pos - 1) >> 1;
        if (!(w < f->w[f->heap[up]])) break;
        f->heap[pos] = f->heap[up];
        pos = up;
    }
    f->heap[pos] = node;
}

static int hf_take_min(hf_forest_t* f) {
    int top = f->heap[0];
    int moving = f->heap[--f->heap_size];
    double w = f->w[moving];
    int pos = 0, n = f->heap_size;
    for (;;) {
        int l = 2 * pos + 1, r = l + 1, next = -1;
        if (l < n) {
            double wl = f->w[f->heap[l]];
            if (r < n) {
                double wr = f->w[f->heap[r]];
                if (wl <= wr) { if (w > wl) next = l; }
                else if (w > wr) next = r;
            } else if (w > wl) {
                next = l;
            }
        }
        if (next < 0) break;
        f->heap[pos] = f->heap[next];
        pos = next;
    }
    f->heap[pos] = moving;
    return top;
}

/* builds the tree of one alphabet; returns the root (or -1 when every count is <= 0) */
static int hf_build(hf_forest_t* f, int alphabet, const double* counts) {
    f->heap_size = 0;
    for (int s = 0; s < alphabet; ++s) {
        f->w[s] = counts[s];
        f->sym[s] = s;
        f->kid0[s] = f->kid1[s] = -1;
    }
    f->used = alphabet;
    for (int s = 0; s < alphabet; ++s)
        if (counts[s] > 0.0) hf_sift_in(f, s);
    if (f->heap_size == 1) {
        int leaf = hf_take_min(f);
        int root = f->used++;
        f->w[root] = f->w[leaf];
        f->sym[root] = -1;
        f->kid0[root] = leaf;
        f->kid1[root] = -1;
        hf_sift_in(f, root);
    }
    while (f->heap_size > 1) {
        int a = hf_take_min(f);
        int b = hf_take_min(f);
        int nd = f->used++;
        f->w[nd] = f->w[a] + f->w[b];
        f->sym[nd] = -1;
        f->kid0[nd] = a;
        f->kid1[nd] = b;
        hf_sift_in(f, nd);
    }
    return f->heap_size ? f->heap[0] : -1;
}

typedef struct { int node, depth, bit; } hf_visit_t;

/* depth-first, child 1 first.  pass 0: lengths + byte total; pass 1: emit codes. */
static long long hf_walk(const hf_forest_t* f, int root, huffman_code_item_t* items,
                         byte_t* field, long long field_pos, byte_t* path, hf_visit_t* stack,
                         int emit, long long* bytes_out) {
    if (root < 0) return field_pos;
    int top = 0;
    stack[top++] = (hf_visit_t){root, 0, 0};
    long long bytes = 0;
    while (top) {
        hf_visit_t v = stack[--top];
        if (v.depth > 0) {
            int d = v.depth - 1;
            byte_t m = (byte_t)(0x80u >> (d & 7));
            if (v.bit) path[d >> 3] |= m; else path[d >> 3] &= (byte_t)~m;
        }
        if (f->sym[v.node] >= 0) {
            int nb = (v.depth + 7) >> 3;
            bytes += nb;
            if (emit) {
                huffman_code_item_t* it = &items[f->sym[v.node]];
                it->bit_length = v.depth;
                if (nb) {
                    memcpy(field + field_pos, path, (size_t)nb);
                    if (v.depth & 7) field[field_pos + nb - 1] &= (byte_t)(0xFF00u >> (v.depth & 7));
                    it->code = field + field_pos;
                } else {
                    it->code = NULL;
                }
                field_pos += nb;
            }
            continue;
        }
        if (f->kid0[v.node] >= 0) stack[top++] = (hf_visit_t){f->kid0[v.node], v.depth + 1, 0};
        if (f->kid1[v.node] >= 0) stack[top++] = (hf_visit_t){f->kid1[v.node], v.depth + 1, 1};
    }
    if (bytes_out) *bytes_out += bytes;
    return field_pos;
}

static void hf_codebook_init(huffman_codebook_t* cb, int alphabet, int rows,
                             const double* counts) {
    cb->alphabet_size = alphabet;
    cb->is_context = rows > 1 ? 1 : 0;
    cb->num_items = alphabet * rows;
    cb->items = (huffman_code_item_t*)calloc((size_t)cb->num_items, sizeof(huffman_code_item_t));
    hf_forest_t f;
    hf_alloc(&f, alphabet);
    hf_visit_t* stack = (hf_visit_t*)malloc(sizeof(hf_visit_t) * (2 * alphabet + 2));
    byte_t* path = (byte_t*)calloc((size_t)alphabet / 8 + 2, 1);
    int* roots = (int*)malloc(sizeof(int) * rows);
    /* pass 0: sizes.  Trees are rebuilt for pass 1 to keep memory O(alphabet). */
    long long total = 0;
    for (int r = 0; r < rows; ++r) {
        roots[r] = hf_build(&f, alphabet, counts + (size_t)r * alphabet);
        hf_walk(&f, roots[r], NULL, NULL, 0, path, stack, 0, &total);
    }
    cb->codefield = (byte_t*)malloc((size_t)(total > 0 ? total : 1));
    long long pos = 0;
    for (int r = 0; r < rows; ++r) {
        int root = hf_build(&f, alphabet, counts + (size_t)r * alphabet);
        pos = hf_walk(&f, root, cb->items + (size_t)r * alphabet, cb->codefield, pos, path,
                      stack, 1, NULL);
    }
    free(roots);
    free(path);
    free(stack);
    hf_free(&f);
}

void huffman_codebook_encode_init(huffman_codebook_t* codebook, int alphabet_size,
                                  const double* symbol_counts) {
    hf_codebook_init(codebook, alphabet_size, 1, symbol_counts);
}

void huffman_codebook_context_encode_init(huffman_codebook_t* codebook, int alphabet_size,
                                          const double* symbol_counts) {
    hf_codebook_init(codebook, alphabet_size, alphabet_size, symbol_counts);
    codebook->is_context = 1;
}

double huffman_estimate_size(const huffman_codebook_t* codebook, const double* symbol_counts) {
    double bits = 0;
    for (int i = 0; i < codebook->num_items; ++i)
        bits += symbol_counts[i] * codebook->items[i].bit_length;
    return bits;
}
