/* huffman_decoder -- CLI-compatible replacement for the reference's src/huffman_decoder.c
 * (huffman_decoder.c:39-99,170-305): decodes <template>huffman_indices.bin on the GPU.
 *   huffman_decoder <huffman output template> [--output-file f] [--check-file pq] [--tree]
 * --output-file writes the raw n x m codes (no header), as the reference does.
 * --check-file is a real check: both sides are put in the encoder's sort order and
 * compared byte by byte (the reference's strncmp compare is vacuous). */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "misc.h"
#include "pqh.h"
#include "vecs_io.h"

static int g_m;
static int row_cmp(const void* a, const void* b) {
    const unsigned char *x = a, *y = b;
    for (int i = 0; i < g_m; ++i) {
        if (x[i] != y[i]) return (int)x[i] - (int)y[i];
        if (!x[i]) return 0;
    }
    return 0;
}

static int full_cmp(const void* a, const void* b) { return memcmp(a, b, (size_t)g_m); }

int main(int argc, const char* argv[]) {
    if (argc < 2) {
        fprintf(stderr, "Usage: %s <huffman output template> [--output-file <output file>]"
                        " [--check-file <pq indices file>] [--tree]\n", argv[0]);
        return 1;
    }
    const char* out_file = NULL;
    const char* check = NULL;
    int tree = 0;
    for (int i = 2; i < argc; ++i) {
        if (!strcmp(argv[i], "--output-file") && i + 1 < argc) out_file = argv[++i];
        else if (!strcmp(argv[i], "--check-file") && i + 1 < argc) check = argv[++i];
        else if (!strcmp(argv[i], "--tree")) tree = 1;
        else {
            fprintf(stderr, "Unknown arg: %s\n", argv[i]);
            return 1;
        }
    }
    unsigned char* codes = NULL;
    long long n = 0;
    int m = 0;
    /* --tree: rows come back in the stream's DFS order (huffman_decoder.c:214-247) */
    int rc = tree ? pqh_decode_tree_files(argv[1], &codes, &n, &m)
                  : pqh_decode_files(argv[1], &codes, &n, &m);
    if (rc) {
        fprintf(stderr, "huffman_decoder: %s\n", pqh_status_string(rc));
        return 1;
    }
    printf("Decoded\n");
    if (out_file) {
        FILE* f = fopen(out_file, "wb");
        if (!f || fwrite(codes, (size_t)m, (size_t)n, f) != (size_t)n) {
            fprintf(stderr, "cannot write %s\n", out_file);
            return 1;
        }
        fclose(f);
    }
    if (check) {
        long long cn = 0;
        int cm = 0;
        unsigned char* orig = load_vecs_light_filename(check, 1, &cn, &cm);
        if (!orig || cn != n || cm != m) {
            fprintf(stderr, "Check FAILED: shape mismatch\n");
            return 1;
        }
        g_m = m;
        /* the encoder may have sorted (strncmp order, huffman_encoder.c:316-317): compare
         * both sides as multisets under a total order */
        qsort(orig, (size_t)n, (size_t)m, full_cmp);
        qsort(codes, (size_t)n, (size_t)m, full_cmp);
        if (memcmp(orig, codes, (size_t)n * m)) {
            fprintf(stderr, "Check FAILED\n");
            return 1;
        }
        printf("Check OK!\n");
        free(orig);
        (void)row_cmp;
    }
    free(codes);
    return 0;
}
