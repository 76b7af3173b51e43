/* prepend_vecsl_meta -- the reference's converter from header-less vector files to the
 * light .xvecsl format (src/prepend_vecsl_meta.c:12-71; vecs_io.c:70-76 for the header).
 *   prepend_vecsl_meta <file.{b,i,f,l}vecsl> <num_vectors> <num_dimensions>
 * The file must hold exactly num_vectors x num_dimensions elements (1, 4, 4 or 8 bytes by
 * the letter before "vecsl"); it is rewritten as u32 N, u32 D, then the same payload.  A
 * file already 8 bytes longer is reported as processed and left alone.  The payload is
 * streamed to a temporary file next to it (the reference holds it in memory), then written
 * back into the SAME file after the header, as the reference rewrites it in place
 * (prepend_vecsl_meta.c:65-68): the inode, its mode, owner and hard links are kept, and a
 * symlink still points at the rewritten file.  Messages and exit codes follow the reference
 * (an extension it asserts on is reported with exit status 1). */
#define _FILE_OFFSET_BITS 64
#define _POSIX_C_SOURCE 200809L
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "vecs_io.h"

static long long element_size_of(const char* filename) {
    const size_t len = strlen(filename);
    if (len < 7) return -1;
    const char* ext = filename + len - 7;   /* ".?vecsl" */
    if (ext[0] != '.' || strcmp(ext + 2, "vecsl")) return -1;
    switch (ext[1]) {
        case 'i':
        case 'f': return 4;
        case 'l': return 8;
        case 'b': return 1;
        default: return 0;
    }
}

int main(int argc, const char* argv[]) {
    if (argc < 4) {
        fprintf(stderr, "Usage: %s <filename> <num_vectors> <num_dimensions>\n", argv[0]);
        return 1;
    }
    const char* filename = argv[1];
    const int num_vectors = atoi(argv[2]);
    const int num_dimensions = atoi(argv[3]);
    const long long esz = element_size_of(filename);
    if (esz < 0) {
        fprintf(stderr, "Not an .xvecsl file name: %s\n", filename);
        return 1;
    }
    if (esz == 0) {
        fprintf(stderr, "Unknown extension type: '%s'\n", filename + strlen(filename) - 7);
        return 1;
    }
    FILE* in = fopen(filename, "rb");
    if (!in) {
        fprintf(stderr, "File %s not found\n", filename);
        return 1;
    }
    const long long elements = 1LL * num_vectors * num_dimensions;
    fseeko(in, 0, SEEK_END);
    const long long size = (long long)ftello(in);
    if (size == elements * esz + 8) {
        printf("File %s already processed\n", filename);
        fclose(in);
        return 0;
    }
    if (size != elements * esz) {
        fprintf(stderr, "Invalid size/dimension of file %s. File size if %lld (expected %lld)\n",
                filename, size, elements * esz);
        fclose(in);
        return 1;
    }
    fseeko(in, 0, SEEK_SET);
    const size_t tlen = strlen(filename) + 16;
    char* tmp = (char*)malloc(tlen);
    snprintf(tmp, tlen, "%s.pqh_tmp", filename);
    FILE* out = fopen(tmp, "wb");
    if (!out) {
        fprintf(stderr, "Cannot write %s\n", tmp);
        fclose(in);
        return 1;
    }
    enum { kBuf = 1 << 22 };
    char* buf = (char*)malloc(kBuf);
    long long left = elements * esz;
    int bad = 0;
    while (left > 0 && !bad) {   /* 1. the payload -> the temporary copy */
        const size_t want = left < kBuf ? (size_t)left : (size_t)kBuf;
        const size_t got = fread(buf, 1, want, in);
        if (got != want) {
            fprintf(stderr, "Cannot read enough data from %s: requested %lld, got %lld",
                    filename, elements, (elements * esz - left + (long long)got) / esz);
            bad = 1;
        } else if (fwrite(buf, 1, got, out) != got) {
            fprintf(stderr, "Cannot write %s\n", tmp);
            bad = 1;
        }
        left -= (long long)got;
    }
    fclose(in);
    if (fclose(out) || bad) {
        if (!bad) fprintf(stderr, "Cannot write %s\n", tmp);
        remove(tmp);
        free(buf);
        free(tmp);
        return 1;
    }
    /* 2. header + payload back into the original file, in place */
    FILE* src = fopen(tmp, "rb");
    FILE* dst = src ? fopen(filename, "r+b") : NULL;
    if (!dst) {
        fprintf(stderr, "Cannot replace %s\n", filename);
        if (src) fclose(src);
        remove(tmp);
        free(buf);
        free(tmp);
        return 1;
    }
    save_vecs_light_meta_file(dst, num_vectors, num_dimensions);
    left = elements * esz;
    while (left > 0 && !bad) {
        const size_t want = left < kBuf ? (size_t)left : (size_t)kBuf;
        if (fread(buf, 1, want, src) != want || fwrite(buf, 1, want, dst) != want) bad = 1;
        left -= (long long)want;
    }
    fclose(src);
    if (fclose(dst) || bad) {
        /* the original is partly rewritten: keep the copy of its payload */
        fprintf(stderr, "Cannot replace %s (its payload is kept in %s)\n", filename, tmp);
        free(buf);
        free(tmp);
        return 1;
    }
    remove(tmp);
    free(buf);
    free(tmp);
    return 0;
}
