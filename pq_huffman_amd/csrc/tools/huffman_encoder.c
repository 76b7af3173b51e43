/* huffman_encoder -- CLI-compatible replacement for the reference's src/huffman_encoder.c
 * (usage and outputs of huffman_encoder.c:42-102,306-439) running histogram, encode and
 * the sidecar chunk index on the GPU through libpqh.
 *   huffman_encoder <pq-output-template> <output-template> <m>
 *                   [--no-sort] [--no-context] [--only-estimate] [--shuffle] [--tree <path>]
 * --tree <mst.tree> codes the rows in the stored forest's DFS order (pqh_encode_tree_files).
 * --shuffle (time-seeded rand(), not reproducible) is out of scope and rejected. */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "misc.h"
#include "pqh.h"
#include "vecs_io.h"

static void usage(const char* argv0) {
    fprintf(stderr, "Usage: %s <pq-output-template> <output-template> <m>"
                    " [--no-sort] [--no-context] [--only-estimate] [--tree <tree path>]\n", argv0);
    exit(1);
}

int main(int argc, const char* argv[]) {
    if (argc < 4) {
        fprintf(stderr, "Too few positional arguments\n");
        usage(argv[0]);
    }
    pqh_encode_options_t opt = {1, 1, 64, 0};
    int m = atoi(argv[3]);
    const char* tree = NULL;
    for (int i = 4; i < argc; ++i) {
        if (!strcmp(argv[i], "--only-estimate")) opt.only_estimate = 1;
        else if (!strcmp(argv[i], "--no-sort")) opt.sort = 0;
        else if (!strcmp(argv[i], "--no-context")) opt.context = 0;
        else if (!strcmp(argv[i], "--tree") && i + 1 < argc) tree = argv[++i];
        else if (!strcmp(argv[i], "--shuffle")) {
            fprintf(stderr, "%s: not supported by this build (see DESIGN.md scope)\n", argv[i]);
            return 1;
        } else {
            fprintf(stderr, "Unknown arg: %s\n", argv[i]);
            usage(argv[0]);
        }
    }
    char* in = concat(argv[1], "pq_indices.bvecsl");
    long long n = 0;
    int d = 0;
    byte_t* codes = load_vecs_light_filename(in, 1, &n, &d);
    if (!codes || d != m) {
        fprintf(stderr, "cannot read %s (or its dimension %d != m %d)\n", in, d, m);
        return 1;
    }
    int rc;
    if (tree) {
        if (!opt.context || opt.only_estimate) {
            fprintf(stderr, "--tree needs context coding and a full encode\n");
            return 1;
        }
        printf("use tree encoder\n");
        rc = pqh_encode_tree_files(codes, n, m, opt.sort, tree, argv[2]);
    } else {
        printf("use %s encoder\n", opt.context ? "context" : "non-context");
        rc = pqh_encode_files(codes, n, m, &opt, argv[2]);
    }
    if (rc) {
        fprintf(stderr, "huffman_encoder: %s\n", pqh_status_string(rc));
        return 1;
    }
    free(codes);
    free(in);
    return 0;
}
