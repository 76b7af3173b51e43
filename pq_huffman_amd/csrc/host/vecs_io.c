/* vecs_io.c -- drop-in for the reference's src/vecs_io.c:8-76: light .xvecsl files
 * (u32 N, u32 D, raw payload).  The header fields are 32-bit on disk (vecs_io.c:45). */
#include "vecs_io.h"

#include <stdint.h>
#include <stdlib.h>

void load_vecs_light_meta_file(FILE* file, long long* num_elements_out, int* num_dimensions_out) {
    uint32_t hdr[2] = {0, 0};
    size_t got = fread(hdr, sizeof(uint32_t), 2, file);
    if (got < 1) hdr[0] = 0;
    if (got < 2) hdr[1] = 0;
    if (num_elements_out) *num_elements_out = hdr[0];
    if (num_dimensions_out) *num_dimensions_out = (int)hdr[1];
}

void load_vecs_light_meta_filename(const char* filename, long long* num_elements_out,
                                   int* num_dimensions_out) {
    FILE* f = fopen(filename, "rb");
    if (!f) {
        if (num_elements_out) *num_elements_out = 0;
        if (num_dimensions_out) *num_dimensions_out = 0;
        return;
    }
    load_vecs_light_meta_file(f, num_elements_out, num_dimensions_out);
    fclose(f);
}

byte_t* load_vecs_light_file(FILE* file, size_t element_size, long long* num_elements_out,
                             int* num_dimensions_out) {
    long long n = 0;
    int d = 0;
    load_vecs_light_meta_file(file, &n, &d);
    if (num_elements_out) *num_elements_out = n;
    if (num_dimensions_out) *num_dimensions_out = d;
    size_t count = (size_t)n * (size_t)d;
    byte_t* data = (byte_t*)malloc(count * element_size > 0 ? count * element_size : 1);
    if (count && fread(data, element_size, count, file) != count) {
        free(data);
        return NULL;
    }
    return data;
}

byte_t* load_vecs_light_filename(const char* filename, size_t element_size,
                                 long long* num_elements_out, int* num_dimensions_out) {
    FILE* f = fopen(filename, "rb");
    if (!f) return NULL;
    byte_t* r = load_vecs_light_file(f, element_size, num_elements_out, num_dimensions_out);
    fclose(f);
    return r;
}

long long load_vecs_num_vectors_filename(const char* filename) {
    long long n = 0;
    load_vecs_light_meta_filename(filename, &n, NULL);
    return n;
}

int load_vecs_num_dimensions_filename(const char* filename) {
    int d = 0;
    load_vecs_light_meta_filename(filename, NULL, &d);
    return d;
}

void save_vecs_light_meta_file(FILE* file, long long num_elements, int num_dimensions) {
    uint32_t hdr[2] = {(uint32_t)num_elements, (uint32_t)num_dimensions};
    fwrite(hdr, sizeof(uint32_t), 2, file);
}
