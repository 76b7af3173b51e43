/* compute_nn_fast -- CLI-compatible replacement for the reference's src/compute_nn_fast.c
 * (usage and outputs of compute_nn_fast.c:120-235,623-658): the blocked kNN graph of an
 * .fvecs file on the GPU through libpqh (pqh_knn_fast_files).
 *   compute_nn_fast <input dataset path> <output files template> <num_nn> [optional args]
 * Geometry: --num-dims, --num-blocks-per-dim, --block-overlap-fraction, --blocks-info-cache,
 * --with-blocks-stat as the reference.  --num-threads, --temp-file, --[no-]delete-temp-file,
 * --[no-]init-temp-file and --num-dimensions-at-pass only steer the reference's CPU/disk
 * staging (the results do not depend on them) and are accepted and ignored; a partial run
 * (--blocks-from / --blocks-to) is out of scope and rejected. */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "pqh.h"

static void usage(const char* argv0) {
    fprintf(stderr, "Usage: %s  <input dataset path> <output files template> <num_nn> [optional args]\n",
            argv0);
    exit(1);
}

int main(int argc, const char* argv[]) {
    if (argc < 4) {
        fprintf(stderr, "Too few required args\n");
        usage(argv[0]);
    }
    pqh_knn_options_t opt = {5, 3, 0.3, NULL, 0};
    const int num_nn = atoi(argv[3]);
    for (int i = 4; i < argc; ++i) {
        const char* a = argv[i];
        const int has = i + 1 < argc;
        if (!strcmp(a, "--num-dims") && has) opt.num_split = atoi(argv[++i]);
        else if (!strcmp(a, "--num-blocks-per-dim") && has) opt.blocks_per_dim = atoi(argv[++i]);
        else if (!strcmp(a, "--block-overlap-fraction") && has) opt.overlap = atof(argv[++i]);
        else if (!strcmp(a, "--blocks-info-cache") && has) opt.blocks_info_cache = argv[++i];
        else if (!strcmp(a, "--with-blocks-stat")) opt.with_blocks_stat = 1;
        else if ((!strcmp(a, "--num-threads") || !strcmp(a, "--temp-file") ||
                  !strcmp(a, "--num-dimensions-at-pass")) && has) ++i;
        else if (!strcmp(a, "--delete-temp-file") || !strcmp(a, "--no-delete-temp-file") ||
                 !strcmp(a, "--init-temp-file") || !strcmp(a, "--no-init-temp-file")) {
        } else if (!strcmp(a, "--blocks-from") || !strcmp(a, "--blocks-to")) {
            fprintf(stderr, "%s: partial runs are not supported by this build\n", a);
            return 1;
        } else {
            fprintf(stderr, "Unknown arg %s\n", a);
            return 1;
        }
    }
    const int rc = pqh_knn_fast_files(argv[1], argv[2], num_nn, &opt);
    if (rc) {
        fprintf(stderr, "compute_nn_fast failed: %s\n", pqh_status_string(rc));
        return 1;
    }
    return 0;
}
