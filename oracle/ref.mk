# oracle/ref.mk -- TEST INFRASTRUCTURE: build the reference's Huffman/bitstream half from its
# own sources where they lie (/root/reference/src), outputs only into oracle/_ref/.
#
#   make -f oracle/ref.mk            (from the repo root)
#
# Nothing is copied out of the reference; no stand-in headers are written.  The PQ half
# (pq_encoder.c) is NOT buildable here: it needs yael v438 (yael/kmeans.h, .profile:9-11),
# which is not vendored and not in this image -- see DESIGN.md "Oracle".
# Reference build flags are `-std=c99 -g` (src/Makefile:9, no -O); we build both that
# (as-shipped, *_O0) and -O2 (calibration of the CPU baseline).

REF ?= /root/reference/src
OUT := oracle/_ref
CC  := gcc
CFLAGS_O0 := -std=c99 -g -w -I$(REF)
CFLAGS_O2 := -std=c99 -O2 -w -I$(REF)

LIBSRC := $(REF)/huffman_encode.c $(REF)/huffman_decode.c $(REF)/huffman_codebook.c \
          $(REF)/bitstream.c $(REF)/stats.c $(REF)/misc.c $(REF)/vecs_io.c
TREESRC := $(REF)/mst.c $(REF)/dsu.c

BINS := $(OUT)/huffman_encoder $(OUT)/huffman_decoder \
        $(OUT)/relink/huffman_encoder $(OUT)/relink/huffman_decoder \
        $(OUT)/huffman_encoder_O0 $(OUT)/huffman_decoder_O0 \
        $(OUT)/bitstream_test $(OUT)/huffman_encode_test $(OUT)/huffman_decode_test \
        $(OUT)/huffman_codebook_test $(OUT)/libref.so \
        $(OUT)/mst_builder $(OUT)/libref_knn.so $(OUT)/prepend_vecsl_meta

.PHONY: all clean
all: $(BINS)

$(OUT):
	mkdir -p $(OUT)

$(OUT)/huffman_encoder: $(REF)/huffman_encoder.c $(LIBSRC) $(TREESRC) | $(OUT)
	$(CC) $(CFLAGS_O2) -o $@ $^ -lm
$(OUT)/huffman_decoder: $(REF)/huffman_decoder.c $(LIBSRC) $(TREESRC) | $(OUT)
	$(CC) $(CFLAGS_O2) -o $@ $^ -lm
$(OUT)/huffman_encoder_O0: $(REF)/huffman_encoder.c $(LIBSRC) $(TREESRC) | $(OUT)
	$(CC) $(CFLAGS_O0) -o $@ $^ -lm
$(OUT)/huffman_decoder_O0: $(REF)/huffman_decoder.c $(LIBSRC) $(TREESRC) | $(OUT)
	$(CC) $(CFLAGS_O0) -o $@ $^ -lm

# the reference CLIs relinked against libpqh -- its own
# huffman_encoder.c / huffman_decoder.c (+ mst.c, dsu.c: the forest loader libpqh does not
# replace) compiled against include/*.h (`-I-`: quote includes skip the source's own
# directory, so huffman.h, bitstream.h, stats.h, misc.h, vecs_io.h come from include/),
# linked with -lpqh instead of the reference's library objects.
PQH_LIB := pq_huffman_amd/lib
CFLAGS_RELINK := -std=c99 -O2 -w -Iinclude -I- -I$(REF)
$(OUT)/relink:
	mkdir -p $(OUT)/relink
$(OUT)/relink/%: $(REF)/%.c $(TREESRC) $(PQH_LIB)/libpqh.so | $(OUT)/relink
	$(CC) $(CFLAGS_RELINK) -o $@ $< $(TREESRC) -L$(PQH_LIB) -lpqh \
	    -Wl,-rpath,$(abspath $(PQH_LIB)) -lm

# embedded `#ifdef _X_TEST` mains (src/bitstream.c:196, huffman_encode.c:280,
# huffman_decode.c:193, huffman_codebook.c:145); not built by the reference Makefile
$(OUT)/bitstream_test: $(REF)/bitstream.c $(REF)/misc.c | $(OUT)
	$(CC) $(CFLAGS_O2) -D_BITSTREAM_TEST -o $@ $^ -lm
$(OUT)/huffman_encode_test: $(LIBSRC) | $(OUT)
	$(CC) $(CFLAGS_O2) -D_HUFFMAN_ENCODE_TEST -o $@ $^ -lm
$(OUT)/huffman_decode_test: $(LIBSRC) | $(OUT)
	$(CC) $(CFLAGS_O2) -D_HUFFMAN_DECODE_TEST -o $@ $^ -lm
$(OUT)/huffman_codebook_test: $(LIBSRC) | $(OUT)
	$(CC) $(CFLAGS_O2) -D_HUFFMAN_CODEBOOK_TEST -o $@ $^ -lm

$(OUT)/libref.so: oracle/ref_harness.c $(LIBSRC) | $(OUT)
	$(CC) $(CFLAGS_O2) -fPIC -shared -o $@ $^ -lm

# the light-header converter as shipped (prepend_vecsl_meta.c + vecs_io.c + misc.c)
$(OUT)/prepend_vecsl_meta: $(REF)/prepend_vecsl_meta.c $(REF)/vecs_io.c $(REF)/misc.c | $(OUT)
	$(CC) $(CFLAGS_O2) -o $@ $^ -lm

# the forest builder's yael-free parts: mst_builder as shipped (mst_builder.c + mst.c + dsu.c
# + the library), and the kNN block geometry / heap merge of compute_nn_fast behind
# oracle/ref_knn_harness.c (compute_nn_fast.c itself includes yael/nn.h: not buildable)
$(OUT)/mst_builder: $(REF)/mst_builder.c $(LIBSRC) $(TREESRC) | $(OUT)
	$(CC) $(CFLAGS_O2) -o $@ $^ -lm
KNNSRC := $(REF)/fast_nn_blocks_info.c $(REF)/fast_nn_temp_file.c $(REF)/fast_nn_block.c \
          $(REF)/misc.c $(REF)/vecs_io.c
$(OUT)/libref_knn.so: oracle/ref_knn_harness.c $(KNNSRC) | $(OUT)
	$(CC) -std=gnu99 -O2 -w -I$(REF) -fPIC -shared -o $@ $^ -lm -lpthread

clean:
	rm -rf $(OUT)
