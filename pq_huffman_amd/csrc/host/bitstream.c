/* bitstream.c -- drop-in for the reference's src/bitstream.c:27-194 (bitstream.h).
 *
 * Same observable behaviour: MSB-first bits, whole bytes flushed when the buffer fills
 * (the partial byte carried to the front), zero pad to a byte when a write stream is
 * destroyed, read streams seek the file back over unread whole bytes on destroy, and
 * reading past the end prints "bit_stream: eof" and exits(1) (bitstream.c:159-162).
 * Writes move whole bytes with shifts instead of one bit per iteration
 * (bitstream.c:80-98); a 1-byte buffer no longer spins forever (bitstream.c:131-147
 * computes a zero batch length there).
 */
#include "bitstream.h"

#include <stdlib.h>
#include <string.h>

enum { BS_DEFAULT_BYTES = 128 * 1024 * 1024, BS_UNKNOWN = 0, BS_READ = 1, BS_WRITE = 2 };

struct _bit_stream {
    FILE* file;
    byte_t* buf;
    long long cap;   /* bytes */
    long long bits;  /* write: filled bits; read: valid bits in buf */
    long long rpos;  /* read position in bits */
    int mode;
};

bit_stream_t* bit_stream_create_from_file(FILE* file) {
    return bit_stream_create_from_file_buffered(file, BS_DEFAULT_BYTES);
}

bit_stream_t* bit_stream_create_from_file_buffered(FILE* file, long long buffer_size_bytes) {
    bit_stream_t* s = (bit_stream_t*)calloc(1, sizeof(bit_stream_t));
    s->file = file;
    s->cap = buffer_size_bytes > 2 ? buffer_size_bytes : 2;
    s->buf = (byte_t*)malloc(s->cap);
    s->mode = BS_UNKNOWN;
    return s;
}

int bit_stream_flush(bit_stream_t* s, int add_pad) {
    if (add_pad && (s->bits & 7)) s->bits += 8 - (s->bits & 7); /* low bits already zero */
    long long whole = s->bits >> 3;
    if (whole && fwrite(s->buf, 1, (size_t)whole, s->file) != (size_t)whole) {
        perror("bit_stream: cannot flush");
        abort();
    }
    if (s->bits & 7) s->buf[0] = s->buf[whole];
    s->bits -= whole << 3;
    return 1;
}

/* append nbits (MSB-first from data) at the fill position; caller guarantees room */
static void bs_put(bit_stream_t* s, const byte_t* data, long long nbits) {
    long long cur = s->bits >> 3;
    int off = (int)(s->bits & 7);
    long long full = nbits >> 3;
    int rem = (int)(nbits & 7);
    if (off == 0) {
        memcpy(s->buf + cur, data, (size_t)full);
        if (rem) s->buf[cur + full] = data[full] & (byte_t)(0xFF00u >> rem);
    } else {
        byte_t* o = s->buf + cur;
        for (long long i = 0; i < full; ++i) {
            o[i] |= (byte_t)(data[i] >> off);
            o[i + 1] = (byte_t)(data[i] << (8 - off));
        }
        if (rem) {
            byte_t v = data[full] & (byte_t)(0xFF00u >> rem);
            o[full] |= (byte_t)(v >> off);
            if (off + rem > 8) o[full + 1] = (byte_t)(v << (8 - off));
        }
    }
    s->bits += nbits;
}

int bit_stream_write(bit_stream_t* s, const byte_t* data, long long bit_length) {
    if (s->mode == BS_READ) {
        fprintf(stderr, "bit_stream: write on a read stream\n");
        abort();
    }
    s->mode = BS_WRITE;
    long long room_bits = (s->cap - 1) * 8; /* keep one byte for the carried partial byte */
    while (bit_length > 0) {
        if (s->bits + bit_length > s->cap * 8 - 8) bit_stream_flush(s, 0);
        long long piece = bit_length;
        if (s->bits + piece > s->cap * 8 - 8) piece = (room_bits - s->bits) & ~7LL;
        if (piece <= 0) piece = 8 > bit_length ? bit_length : 8;
        bs_put(s, data, piece);
        data += piece >> 3;
        bit_length -= piece;
    }
    return 1;
}

static void bs_refill(bit_stream_t* s) {
    size_t got = fread(s->buf, 1, (size_t)s->cap, s->file);
    s->bits = (long long)got * 8;
    if (got != (size_t)s->cap && ferror(s->file)) perror("bit_stream: error reading file");
    if (got == 0 && feof(s->file)) {
        fprintf(stderr, "bit_stream: eof\n");
        exit(1);
    }
    s->rpos = 0;
    s->mode = BS_READ;
}

int bit_stream_read_bit(bit_stream_t* s) {
    if (s->mode == BS_WRITE) {
        fprintf(stderr, "bit_stream: read on a write stream\n");
        abort();
    }
    if (s->rpos == s->bits) {
        bs_refill(s);
        if (s->rpos == s->bits) return EOF;
    }
    long long p = s->rpos++;
    return (s->buf[p >> 3] >> (7 - (p & 7))) & 1;
}

void bit_stream_read(bit_stream_t* s, byte_t* data, long long bit_length) {
    for (long long i = 0; i < bit_length; ++i) {
        byte_t mask = (byte_t)(0x80u >> (i & 7));
        if (bit_stream_read_bit(s) > 0) data[i >> 3] |= mask;
        else data[i >> 3] &= (byte_t)~mask;
    }
}

bit_stream_t* bit_stream_destroy_file(bit_stream_t* s, int close_file) {
    if (s->mode == BS_WRITE) {
        bit_stream_flush(s, 1);
    } else if (s->mode == BS_READ) {
        long long unread_bytes = (s->bits - s->rpos) / 8;
        if (unread_bytes) fseek(s->file, -unread_bytes, SEEK_CUR);
    }
    if (close_file) fclose(s->file);
    free(s->buf);
    free(s);
    return NULL;
}

bit_stream_t* bit_stream_destroy(bit_stream_t* s) { return bit_stream_destroy_file(s, 0); }
