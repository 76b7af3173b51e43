/* mst_builder -- CLI-compatible replacement for the reference's src/mst_builder.c (usage and
 * outputs of mst_builder.c:28-141): the minimum spanning forest of a kNN graph on the GPU
 * through libpqh (pqh_mst_files).
 *   mst_builder <nn-input-template> <output-template> <num-nn-to-use>
 *               [--pq-template <pq output template>] [--pq-penalty <pq penalty size>] */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "pqh.h"

static void usage(const char* argv0) {
    fprintf(stderr, "Usage: %s <nn-input-template> <output-template> <num-nn-to-use>"
                    " [--pq-template <pq output template>]"
                    " [--pq-penalty <pq penalty size>]\n", argv0);
    exit(1);
}

int main(int argc, const char* argv[]) {
    if (argc < 4) {
        fprintf(stderr, "Too few arguments\n");
        usage(argv[0]);
    }
    const char* pq = NULL;
    float penalty = 0.0f;
    for (int i = 4; i < argc; ++i) {
        if (!strcmp(argv[i], "--pq-template") && i + 1 < argc) pq = argv[++i];
        else if (!strcmp(argv[i], "--pq-penalty") && i + 1 < argc) penalty = (float)atof(argv[++i]);
        else {
            fprintf(stderr, "Unknown argument: %s\n", argv[i]);
            usage(argv[0]);
        }
    }
    const int rc = pqh_mst_files(argv[1], argv[2], atoi(argv[3]), pq, penalty);
    if (rc) {
        fprintf(stderr, "mst_builder failed: %s\n", pqh_status_string(rc));
        return 1;
    }
    return 0;
}
