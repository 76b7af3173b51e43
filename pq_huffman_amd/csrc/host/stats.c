/* stats.c -- drop-in for the reference's src/stats.c:5-76: one JSON line of estimated
 * Huffman sizes.  Number formats (%.1lf/%.3lf/%.2lf) and key order are part of the
 * format; files are appended to, not truncated. */
#include "stats.h"

#include <stdlib.h>

void huffman_stats_init(huffman_stats_t* stats, long long num_vectors, int m, int k_star) {
    stats->num_vectors = num_vectors;
    stats->m = m;
    stats->k_star = k_star;
    stats->sum_length = 0.0;
    stats->partial_lengths = (double*)calloc(m > 0 ? m : 1, sizeof(double));
    stats->num_roots = 0;
}

void huffman_stats_destroy(huffman_stats_t* stats) {
    free(stats->partial_lengths);
    stats->partial_lengths = NULL;
    stats->num_vectors = 0;
    stats->m = 0;
    stats->k_star = 0;
    stats->sum_length = 0.0;
    stats->num_roots = 0;
}

void huffman_stats_push(huffman_stats_t* stats, int part, double length) {
    stats->sum_length += length;
    stats->partial_lengths[part] = length;
}

static void print_lengths(FILE* f, const huffman_stats_t* s, double bits, int m) {
    double symbols = (double)s->num_vectors * m;
    fprintf(f, "\"length_bit\": %.1lf, \"length_bytes\": %.1lf, ", bits, bits / 8);
    fprintf(f, "\"compression_rate\": %.3lf, \"bits_per_byte\": %.2lf", bits / (symbols * 8),
            bits / symbols);
}

void huffman_stats_print_file(const huffman_stats_t* stats, FILE* file) {
    double root_bits = 8.0 * stats->num_roots;   /* raw first symbol per root and part */
    fprintf(file, "{\"num_vectors\": %lld, \"m\": %d, \"k_star\": %d, ", stats->num_vectors,
            stats->m, stats->k_star);
    print_lengths(file, stats, stats->sum_length + root_bits * stats->m, stats->m);
    if (stats->num_roots) fprintf(file, ", \"num_roots\": %d", stats->num_roots);
    fprintf(file, ", \"partials\": [");
    for (int i = 0; i < stats->m; ++i) {
        fprintf(file, i ? ", {" : "{");
        print_lengths(file, stats, stats->partial_lengths[i] + root_bits, 1);
        fprintf(file, "}");
    }
    fprintf(file, "]}\n");
}

void huffman_stats_print(const huffman_stats_t* stats) { huffman_stats_print_file(stats, stdout); }

void huffman_stats_print_filename(const huffman_stats_t* stats, const char* filename) {
    FILE* f = fopen(filename, "a");
    if (!f) return;
    huffman_stats_print_file(stats, f);
    fclose(f);
}
