/* huffman_decode.c -- the stateful symbol decoder, drop-in for the reference's
 * src/huffman_decode.c:8-191.
 *
 * Semantics kept: one trie per codebook (per previous symbol in context mode); a
 * context decoder with no previous symbol is "warming" and takes the next
 * ceil(log2 alphabet) bits (at least 1) as a raw symbol (:73-76, :138-152); an unknown
 * branch returns HUFFMAN_INVALID_SYMBOL and resets the decoder (:154-157); a finished
 * symbol becomes the context of the next one (:158-161).
 * Implementation: one node pool with int links instead of malloc'd nodes; bulk decoding
 * of whole streams is on the GPU (pqh.h pqh_decode).
 */
#include "huffman.h"

#include <stdlib.h>

struct _huffman_decoder {
    int* link;       /* 2 per node, -1 = none */
    int* leaf;       /* symbol or -1 */
    int nodes, cap;
    int alphabet;
    int is_context;
    int warm_bits;   /* raw bits of a context-less symbol */
    int prev;        /* previous symbol or HUFFMAN_NO_SYMBOL */
    int cur;         /* current node, -1 = none */
    int warm_value, warm_count;
};

static int hd_node(huffman_decoder_t* d) {
    if (d->nodes == d->cap) {
        d->cap = d->cap ? d->cap * 2 : 512;
        d->link = (int*)realloc(d->link, sizeof(int) * 2 * d->cap);
        d->leaf = (int*)realloc(d->leaf, sizeof(int) * d->cap);
    }
    d->link[2 * d->nodes] = d->link[2 * d->nodes + 1] = -1;
    d->leaf[d->nodes] = HUFFMAN_NO_SYMBOL;
    return d->nodes++;
}

static void hd_insert(huffman_decoder_t* d, int root, int symbol, const huffman_code_item_t* it) {
    int nd = root;
    for (int b = 0; b < it->bit_length; ++b) {
        int bit = (it->code[b >> 3] >> (7 - (b & 7))) & 1;
        int nx = d->link[2 * nd + bit];
        if (nx < 0) {
            nx = hd_node(d);
            d->link[2 * nd + bit] = nx;
        }
        nd = nx;
    }
    if (it->bit_length > 0) d->leaf[nd] = symbol;
}

huffman_decoder_t* huffman_decoder_create(const huffman_codebook_t* cb) {
    huffman_decoder_t* d = (huffman_decoder_t*)calloc(1, sizeof(huffman_decoder_t));
    d->alphabet = cb->alphabet_size;
    d->is_context = cb->is_context;
    d->warm_bits = 1;
    while ((1 << d->warm_bits) < d->alphabet) ++d->warm_bits;
    int roots = d->is_context ? d->alphabet : 1;
    for (int r = 0; r < roots; ++r) hd_node(d);   /* roots are nodes 0 .. roots-1 */
    for (int r = 0; r < roots; ++r)
        for (int s = 0; s < d->alphabet; ++s)
            hd_insert(d, r, s, &cb->items[(size_t)r * d->alphabet * d->is_context + s]);
    d->prev = HUFFMAN_NO_SYMBOL;
    d->cur = d->is_context ? -1 : 0;
    return d;
}

huffman_decoder_t* huffman_decoder_destroy(huffman_decoder_t* d) {
    free(d->link);
    free(d->leaf);
    free(d);
    return NULL;
}

void huffman_decoder_set_prev_symbol(huffman_decoder_t* d, int prev_symbol) {
    if (!d->is_context) {
        d->cur = 0;
        return;
    }
    d->warm_value = 0;
    d->warm_count = 0;
    d->prev = prev_symbol;
    d->cur = prev_symbol == HUFFMAN_NO_SYMBOL ? -1 : prev_symbol;
}

void huffman_decoder_reset(huffman_decoder_t* d) {
    huffman_decoder_set_prev_symbol(d, HUFFMAN_NO_SYMBOL);
}

int huffman_decoder_push_bit(huffman_decoder_t* d, int bit_value) {
    if (d->is_context && d->prev == HUFFMAN_NO_SYMBOL) {
        d->warm_value = (d->warm_value << 1) | (bit_value & 1);
        if (++d->warm_count < d->warm_bits) return HUFFMAN_NO_SYMBOL;
        int s = d->warm_value;
        if (s >= d->alphabet) {          /* the reference asserts here (:145) */
            huffman_decoder_reset(d);
            return HUFFMAN_INVALID_SYMBOL;
        }
        huffman_decoder_set_prev_symbol(d, s);
        return s;
    }
    int nx = d->cur < 0 ? -1 : d->link[2 * d->cur + (bit_value & 1)];
    if (nx < 0) {
        huffman_decoder_reset(d);
        return HUFFMAN_INVALID_SYMBOL;
    }
    d->cur = nx;
    int s = d->leaf[nx];
    if (s == HUFFMAN_NO_SYMBOL) return HUFFMAN_NO_SYMBOL;
    huffman_decoder_set_prev_symbol(d, s);
    return s;
}

int huffman_decoder_push_bits(huffman_decoder_t* d, const byte_t* bits, int bit_length) {
    int r = HUFFMAN_NO_SYMBOL, b = 0;
    for (; b < bit_length && r == HUFFMAN_NO_SYMBOL; ++b)
        r = huffman_decoder_push_bit(d, (bits[b >> 3] >> (7 - (b & 7))) & 1);
    return b == bit_length ? r : HUFFMAN_INVALID_SYMBOL;
}

int huffman_decoder_read_symbol(huffman_decoder_t* d, bit_stream_t* stream) {
    int s = HUFFMAN_NO_SYMBOL;
    while (s == HUFFMAN_NO_SYMBOL) s = huffman_decoder_push_bit(d, bit_stream_read_bit(stream));
    return s;
}
