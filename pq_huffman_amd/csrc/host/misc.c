/* misc.c -- drop-in for the reference's src/misc.c:8-50 (misc.h). */
#include "misc.h"

#include <stdio.h>
#include <stdlib.h>
#include <string.h>

int imin(int a, int b) { return b < a ? b : a; }

long long iminll(long long a, long long b) { return b < a ? b : a; }

long long iclampll(long long value, long long min_value, long long max_value) {
    if (value <= min_value) return min_value;
    if (value >= max_value) return max_value;
    return value;
}

char* concat(const char* prefix, const char* suffix) {
    size_t a = strlen(prefix), b = strlen(suffix);
    char* out = (char*)malloc(a + b + 1);
    memcpy(out, prefix, a);
    memcpy(out + a, suffix, b + 1);
    return out;
}

long long load_num_elements(const char* filename, long long element_size) {
    FILE* f = fopen(filename, "rb");
    if (!f) return -1;
    fseek(f, 0, SEEK_END);
    long long size = ftell(f);
    fclose(f);
    if (element_size <= 0 || size % element_size) return -1;
    return size / element_size;
}
