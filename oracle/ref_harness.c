/*
 * ref_harness.c -- TEST INFRASTRUCTURE ONLY (oracle side, never shipped, never linked
 * by pq_huffman_amd).
 *
 * A thin driver compiled TOGETHER WITH the reference's own library sources
 * (/root/reference/src/{huffman_encode,huffman_codebook,huffman_decode,bitstream,
 * stats,misc,vecs_io}.c) by oracle/ref.mk into oracle/_ref/libref.so.  It exposes the
 * reference library behind a ctypes-friendly surface so golden fixtures can be produced
 * for cases the reference CLI cannot run as shipped:
 *
 *   * --no-context encoding: huffman_encoder.c:402-405 reads items[j] for j < 65536 on a
 *     256-item codebook (out of bounds, segfaults).  refh_encode_dir() restates the
 *     CLI's run() (huffman_encoder.c:306-439, non-tree branches, no sorting) calling
 *     only the reference library, without that debug loop.
 *   * alphabets other than 256 (K=4096, 16-bit codes): the library layer
 *     (huffman_encode.c, huffman_codebook.c, huffman_decode.c) is alphabet-generic,
 *     only the CLI hard-wires k*=256 (huffman_encoder.c:89).
 *
 * Nothing here re-implements an algorithm: every codebook, bit and stat comes from the
 * reference functions.
 */
#include <assert.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "bitstream.h"
#include "huffman.h"
#include "stats.h"
#include "vecs_io.h"

/* Build a codebook from counts with the reference builder and export code lengths and
 * left-aligned code bytes (code_stride bytes per item, zero padded). */
int refh_build_codebook(int alphabet, int context, const double* counts,
                        int* lengths_out, unsigned char* codes_out, int code_stride) {
    huffman_codebook_t cb;
    if (context) {
        huffman_codebook_context_encode_init(&cb, alphabet, counts);
    } else {
        huffman_codebook_encode_init(&cb, alphabet, counts);
    }
    int overflow = 0;
    for (int i = 0; i < cb.num_items; ++i) {
        lengths_out[i] = cb.items[i].bit_length;
        int nbytes = (cb.items[i].bit_length + 7) / 8;
        if (nbytes > code_stride) {
            overflow = 1;
            nbytes = code_stride;
        }
        memset(codes_out + (size_t)i * code_stride, 0, code_stride);
        if (cb.items[i].code) {
            memcpy(codes_out + (size_t)i * code_stride, cb.items[i].code, nbytes);
        }
    }
    huffman_codebook_destroy(&cb);
    return overflow ? -1 : 0;
}

/* Write one codebook file (huffman_codebook_save) for counts; used for the codebook
 * serialisation fixtures. */
int refh_save_codebook_file(int alphabet, int context, const double* counts, const char* path) {
    huffman_codebook_t cb;
    if (context) {
        huffman_codebook_context_encode_init(&cb, alphabet, counts);
    } else {
        huffman_codebook_encode_init(&cb, alphabet, counts);
    }
    FILE* f = fopen(path, "wb");
    if (!f) {
        huffman_codebook_destroy(&cb);
        return -1;
    }
    huffman_codebook_save(&cb, f);
    fclose(f);
    huffman_codebook_destroy(&cb);
    return 0;
}

static unsigned sym_at(const void* codes, int elem_size, long long idx) {
    if (elem_size == 1) {
        return ((const unsigned char*)codes)[idx];
    }
    return ((const unsigned short*)codes)[idx];
}

/* Restatement of huffman_encoder.c run() for the non-tree, non-sorting modes, calling
 * only reference library functions.  Writes huffman_codebooks.bin, huffman_indices.bin
 * and huffman_stats.txt under out_prefix (a directory path ending in '/').
 * codes: n x m symbols (elem_size 1 or 2 bytes), alphabet k.  context only for k=256
 * (the CLI's (prev << 8) + cur indexing, huffman_encoder.c:187,230). */
int refh_encode_dir(const char* out_prefix, const void* codes, int elem_size, long long n, int m,
                    int k, int context) {
    if (context && k != 256) {
        return -2;
    }
    int alphabet = context ? k * k : k;
    double* stats = calloc((size_t)m * alphabet, sizeof(double));
    int num_roots = 0;
    if (context) {
        for (long long v = 1; v < n; ++v) {
            for (int i = 0; i < m; ++i) {
                unsigned prev = sym_at(codes, elem_size, (v - 1) * m + i);
                unsigned cur = sym_at(codes, elem_size, v * m + i);
                stats[(size_t)i * alphabet + (prev << 8) + cur] += 1;
            }
        }
        num_roots = 1;
    } else {
        for (long long v = 0; v < n; ++v) {
            for (int i = 0; i < m; ++i) {
                stats[(size_t)i * alphabet + sym_at(codes, elem_size, v * m + i)] += 1;
            }
        }
    }

    huffman_stats_t encode_stats;
    huffman_stats_init(&encode_stats, n, m, k);
    encode_stats.num_roots = num_roots;
    huffman_codebook_t* cbs = malloc(sizeof(*cbs) * m);
    for (int i = 0; i < m; ++i) {
        double* part = stats + (size_t)alphabet * i;
        if (context) {
            huffman_codebook_context_encode_init(cbs + i, k, part);
        } else {
            huffman_codebook_encode_init(cbs + i, k, part);
        }
        huffman_stats_push(&encode_stats, i, huffman_estimate_size(&cbs[i], part));
    }
    size_t plen = strlen(out_prefix);
    char* path = malloc(plen + 64);

    snprintf(path, plen + 64, "%shuffman_stats.txt", out_prefix);
    huffman_stats_print_filename(&encode_stats, path);
    huffman_stats_destroy(&encode_stats);

    snprintf(path, plen + 64, "%shuffman_codebooks.bin", out_prefix);
    FILE* cf = fopen(path, "wb");
    unsigned int m_int = m;
    fwrite(&m_int, sizeof(m_int), 1, cf);
    for (int i = 0; i < m; ++i) {
        huffman_codebook_save(cbs + i, cf);
    }
    fclose(cf);

    snprintf(path, plen + 64, "%shuffman_indices.bin", out_prefix);
    FILE* ef = fopen(path, "wb");
    unsigned long long nll = n;
    fwrite(&nll, sizeof(nll), 1, ef);
    bit_stream_t* stream = bit_stream_create_from_file(ef);
    for (long long v = 0; v < n; ++v) {
        for (int i = 0; i < m; ++i) {
            unsigned cur = sym_at(codes, elem_size, v * m + i);
            if (context) {
                if (v > 0) {
                    unsigned prev = sym_at(codes, elem_size, (v - 1) * m + i);
                    const huffman_code_item_t* it = &cbs[i].items[(prev << 8) + cur];
                    bit_stream_write(stream, it->code, it->bit_length);
                } else {
                    unsigned char raw = (unsigned char)cur;
                    bit_stream_write(stream, &raw, BYTE_NUM_BITS);
                }
            } else {
                const huffman_code_item_t* it = &cbs[i].items[cur];
                bit_stream_write(stream, it->code, it->bit_length);
            }
        }
    }
    stream = bit_stream_destroy(stream);
    fclose(ef);

    for (int i = 0; i < m; ++i) {
        huffman_codebook_destroy(cbs + i);
    }
    free(cbs);
    free(path);
    free(stats);
    return 0;
}

/* Decode a directory written by the reference (or by refh_encode_dir) with the reference
 * trie decoder (huffman_decoder.c run() loop, non-tree): out gets n x m symbols. */
int refh_decode_dir(const char* in_prefix, void* out, int elem_size, long long n) {
    size_t plen = strlen(in_prefix);
    char* path = malloc(plen + 64);
    snprintf(path, plen + 64, "%shuffman_codebooks.bin", in_prefix);
    FILE* cf = fopen(path, "rb");
    if (!cf) {
        free(path);
        return -1;
    }
    unsigned int m = 0;
    fread(&m, sizeof(m), 1, cf);
    huffman_codebook_t* cbs = malloc(sizeof(*cbs) * m);
    huffman_decoder_t** decs = malloc(sizeof(*decs) * m);
    for (unsigned i = 0; i < m; ++i) {
        huffman_codebook_load(cbs + i, cf);
        decs[i] = huffman_decoder_create(cbs + i);
    }
    fclose(cf);
    snprintf(path, plen + 64, "%shuffman_indices.bin", in_prefix);
    FILE* ef = fopen(path, "rb");
    fseek(ef, sizeof(long long), SEEK_CUR);
    bit_stream_t* stream = bit_stream_create_from_file(ef);
    int rc = 0;
    for (long long v = 0; v < n && rc == 0; ++v) {
        for (unsigned i = 0; i < m; ++i) {
            int s = huffman_decoder_read_symbol(decs[i], stream);
            if (s < 0) {
                rc = -3;
                break;
            }
            if (elem_size == 1) {
                ((unsigned char*)out)[v * m + i] = (unsigned char)s;
            } else {
                ((unsigned short*)out)[v * m + i] = (unsigned short)s;
            }
        }
    }
    stream = bit_stream_destroy(stream);
    fclose(ef);
    for (unsigned i = 0; i < m; ++i) {
        decs[i] = huffman_decoder_destroy(decs[i]);
        huffman_codebook_destroy(cbs + i);
    }
    free(decs);
    free(cbs);
    free(path);
    return rc;
}

/* Write bits through the reference bitstream with a tiny buffer (exercises the
 * mid-stream flush path, bitstream.c:71-101) -- the _BITSTREAM_TEST sequence. */
int refh_bitstream_write(const char* path, const unsigned char* data, const long long* bit_lengths,
                         int num_writes, long long buffer_bytes) {
    FILE* f = fopen(path, "wb");
    if (!f) {
        return -1;
    }
    bit_stream_t* s = bit_stream_create_from_file_buffered(f, buffer_bytes);
    const unsigned char* p = data;
    for (int i = 0; i < num_writes; ++i) {
        bit_stream_write(s, p, bit_lengths[i]);
        p += (bit_lengths[i] + 7) / 8;
    }
    s = bit_stream_destroy(s);
    fclose(f);
    return 0;
}
