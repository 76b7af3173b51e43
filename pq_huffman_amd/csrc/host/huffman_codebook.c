/* huffman_codebook.c -- codebook dump/save/load, drop-in for the reference's
 * src/huffman_codebook.c:6-143.
 * File layout per codebook (huffman_codebook.c:74-94): i32 alphabet, u8 is_context,
 * num_items varint bit lengths (7 bits per byte, low group first, 0x80 = more, at most
 * 4 bytes: :43-72), then all codes concatenated MSB-first, zero padded to a byte. */
#include "huffman.h"

#include <stdint.h>
#include <stdlib.h>
#include <string.h>

void huffman_dump_code(const huffman_code_item_t* item, FILE* f) {
    if (!item->code) {
        fputc('-', f);
        return;
    }
    for (int b = 0; b < item->bit_length; ++b) fputc('0' + ((item->code[b >> 3] >> (7 - (b & 7))) & 1), f);
    fprintf(f, " (%d)", item->bit_length);
}

void huffman_codebook_dump(const huffman_codebook_t* cb, FILE* f) {
    for (int i = 0; i < cb->num_items; ++i) {
        if (cb->is_context) fprintf(f, "%d -> %d: ", i / cb->alphabet_size, i % cb->alphabet_size);
        else fprintf(f, "%d: ", i);
        huffman_dump_code(cb->items + i, f);
        fputc('\n', f);
    }
}

void huffman_counts_context_dump(const double* counts, int alphabet, FILE* f) {
    for (int a = 0; a < alphabet; ++a)
        for (int b = 0; b < alphabet; ++b)
            fprintf(f, "%d -> %d: %lf\n", a, b, counts[a * alphabet + b]);
}

static int put_varint(byte_t* out, unsigned v) {
    int n = 0;
    for (;;) {
        byte_t low = (byte_t)(v & 0x7f);
        v >>= 7;
        if (v == 0 || n == 3) {   /* the 4th byte keeps 0x80 if bits remain (:46-58) */
            out[n++] = (byte_t)(low | (v ? 0x80 : 0));
            if (v) fprintf(stderr, "Cannot write bit_length of code because it's too large\n");
            return n;
        }
        out[n++] = (byte_t)(low | 0x80);
    }
}

void huffman_codebook_save(const huffman_codebook_t* cb, FILE* file) {
    int32_t alphabet = cb->alphabet_size;
    byte_t ctx = (byte_t)cb->is_context;
    fwrite(&alphabet, sizeof(alphabet), 1, file);
    fwrite(&ctx, 1, 1, file);
    byte_t* lens = (byte_t*)malloc((size_t)cb->num_items * 4 + 1);
    size_t lp = 0;
    long long total_bits = 0;
    for (int i = 0; i < cb->num_items; ++i) {
        lp += put_varint(lens + lp, (unsigned)cb->items[i].bit_length);
        total_bits += cb->items[i].bit_length;
    }
    fwrite(lens, 1, lp, file);
    free(lens);
    size_t nbytes = (size_t)((total_bits + 7) >> 3);
    byte_t* packed = (byte_t*)calloc(nbytes + 1, 1);
    long long pos = 0;
    for (int i = 0; i < cb->num_items; ++i) {
        const huffman_code_item_t* it = cb->items + i;
        for (int b = 0; b < it->bit_length; ++b, ++pos)
            if ((it->code[b >> 3] >> (7 - (b & 7))) & 1) packed[pos >> 3] |= (byte_t)(0x80u >> (pos & 7));
    }
    fwrite(packed, 1, nbytes, file);
    free(packed);
}

void huffman_codebook_load(huffman_codebook_t* cb, FILE* file) {
    int32_t alphabet = 0;
    byte_t ctx = 0;
    if (fread(&alphabet, sizeof(alphabet), 1, file) != 1) alphabet = 0;
    if (fread(&ctx, 1, 1, file) != 1) ctx = 0;
    cb->alphabet_size = alphabet;
    cb->is_context = ctx;
    cb->num_items = ctx ? alphabet * alphabet : alphabet;
    cb->items = (huffman_code_item_t*)calloc((size_t)(cb->num_items > 0 ? cb->num_items : 1),
                                             sizeof(huffman_code_item_t));
    long long total_bits = 0, field_bytes = 0;
    for (int i = 0; i < cb->num_items; ++i) {
        unsigned v = 0;
        for (int k = 0; k < 4; ++k) {
            int c = fgetc(file);
            byte_t byte = c == EOF ? 0 : (byte_t)c;
            v |= (unsigned)(byte & 0x7f) << (7 * k);
            if (!(byte & 0x80)) break;
        }
        cb->items[i].bit_length = (int)v;
        total_bits += v;
        field_bytes += (v + 7) / 8;
    }
    size_t nbytes = (size_t)((total_bits + 7) >> 3);
    byte_t* packed = (byte_t*)calloc(nbytes + 1, 1);
    if (nbytes && fread(packed, 1, nbytes, file) != nbytes) {
        /* truncated file: leave the missing bits zero */
    }
    cb->codefield = (byte_t*)calloc((size_t)(field_bytes > 0 ? field_bytes : 1), 1);
    byte_t* next = cb->codefield;
    long long pos = 0;
    for (int i = 0; i < cb->num_items; ++i) {
        int L = cb->items[i].bit_length;
        if (!L) {
            cb->items[i].code = NULL;
            continue;
        }
        for (int b = 0; b < L; ++b, ++pos)
            if ((packed[pos >> 3] >> (7 - (pos & 7))) & 1) next[b >> 3] |= (byte_t)(0x80u >> (b & 7));
        cb->items[i].code = next;
        next += (L + 7) / 8;
    }
    free(packed);
}

void huffman_codebook_destroy(huffman_codebook_t* cb) {
    free(cb->codefield);
    free(cb->items);
    cb->codefield = NULL;
    cb->items = NULL;
    cb->alphabet_size = 0;
    cb->is_context = 0;
}
