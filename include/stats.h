/*
 * stats.h -- drop-in for the reference's src/stats.h:6-23 (JSON line of estimated
 * Huffman sizes, stats.c:38-76; appended to huffman_stats.txt).
 */
#ifndef _HUFFMAN_STATS_H
#define _HUFFMAN_STATS_H

#include <stdio.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct _huffman_stats {
    long long num_vectors;
    int m;
    int k_star;

    double sum_length;
    double* partial_lengths;
    int num_roots;
} huffman_stats_t;

void huffman_stats_init(huffman_stats_t* stats, long long num_vectors, int m, int k_star);
void huffman_stats_destroy(huffman_stats_t* stats);

void huffman_stats_push(huffman_stats_t* stats, int part, double length);

void huffman_stats_print(const huffman_stats_t* stats);
void huffman_stats_print_filename(const huffman_stats_t* stats, const char* filename);
void huffman_stats_print_file(const huffman_stats_t* stats, FILE* file);

#ifdef __cplusplus
}
#endif

#endif /* _HUFFMAN_STATS_H */
