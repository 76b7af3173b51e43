"""CPU tests of the drop-in C library (libpqh.so host side: huffman.h, bitstream.h,
vecs_io.h, stats.h, pq.h) against the reference-generated golden fixtures, plus the
export check of every symbol include/*.h declares.  No GPU calls."""
import ctypes
import os
import re
import subprocess
import tempfile

import numpy as np
import pytest

from conftest import GOLD, ROOT, golden
from pq_huffman_amd import capi
from pq_huffman_amd.capi import HuffmanCodebook, HuffmanStats, lib
from pq_huffman_amd.codec import Codebooks, _libc

HEADERS = ["misc.h", "bitstream.h", "huffman.h", "vecs_io.h", "stats.h", "fast_nn_block.h",
           "pq.h", "pqh.h"]


def _declared_functions():
    names = set()
    for h in HEADERS:
        text = open(os.path.join(ROOT, "include", h)).read()
        text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
        for m in re.finditer(r"^[A-Za-z_][\w \*]*?\b([a-z_][a-z0-9_]*)\s*\(", text, re.M):
            if not text[m.start():m.end()].lstrip().startswith(("typedef", "#", "return")):
                names.add(m.group(1))
    return names


def test_library_exports_every_declared_function():
    names = _declared_functions()
    assert len(names) > 70
    out = subprocess.check_output(["nm", "-D", "--defined-only", capi.LIB_PATH], text=True)
    exported = {line.split()[-1] for line in out.splitlines() if " T " in line}
    missing = sorted(names - exported)
    assert not missing, missing
    declared_in_py = {n for n, _, _ in capi.SIGNATURES}
    assert names <= declared_in_py | {"usleep"}, sorted(names - declared_in_py)
    lib()  # binds every signature


CASES = ["fib1024", "fib32ctx", "enc_test_many", "enc_test_one", "enc_test_zero",
         "ties_small_ints", "ties_all_equal", "ties_powers", "single_symbol", "empty",
         "geometric", "ctx16_mixed"]


def _codes_of(cb: HuffmanCodebook, stride):
    lens = np.zeros(cb.num_items, np.int32)
    codes = np.zeros((cb.num_items, stride), np.uint8)
    for i in range(cb.num_items):
        L = cb.items[i].bit_length
        lens[i] = L
        for b in range((L + 7) // 8):
            codes[i, b] = cb.items[i].code[b]
    return lens, codes


@pytest.mark.parametrize("case", CASES)
def test_codebook_build_and_save_match_reference(case):
    g = golden("codebooks.npz")
    k, c = (int(v) for v in g[case + "__alphabet"])
    cbs = Codebooks(g[case + "__counts"][None, :], k, bool(c), threads=1)
    lens, codes = _codes_of(cbs.arr[0], g[case + "__codes"].shape[1])
    assert np.array_equal(lens, g[case + "__lens"])
    assert np.array_equal(codes, g[case + "__codes"])
    # huffman_codebooks.bin of one part = u32 m + the reference's saved codebook
    assert cbs.file_bytes() == np.uint32(1).tobytes() + g[case + "__file"].tobytes()


@pytest.mark.parametrize("case", CASES)
def test_codebook_load_resave(case, tmp_path):
    g = golden("codebooks.npz")
    path = str(tmp_path / "cb.bin")
    with open(path, "wb") as f:
        f.write(np.uint32(1).tobytes() + g[case + "__file"].tobytes())
    cbs = Codebooks.load_file(path)
    lens, codes = _codes_of(cbs.arr[0], g[case + "__codes"].shape[1])
    assert np.array_equal(lens, g[case + "__lens"])
    assert np.array_equal(codes, g[case + "__codes"])
    assert cbs.file_bytes()[4:] == g[case + "__file"].tobytes()


@pytest.mark.parametrize("buf", [2, 3, 64])
def test_bitstream_writer_matches_reference(buf, tmp_path):
    g = golden("bitstream.npz")
    lens, data = g[f"buf{buf}__lens"], g[f"buf{buf}__data"]
    path = str(tmp_path / "bs.bin").encode()
    f = _libc.fopen(path, b"wb")
    s = lib().bit_stream_create_from_file_buffered(ctypes.c_void_p(f), buf)
    off = 0
    for L in lens:
        lib().bit_stream_write(s, data[off:].ctypes.data_as(ctypes.c_void_p), int(L))
        off += (int(L) + 7) // 8
    lib().bit_stream_destroy(s)
    _libc.fclose(ctypes.c_void_p(f))
    assert open(path, "rb").read() == g[f"buf{buf}__out"].tobytes()


def test_bitstream_one_byte_buffer_terminates(tmp_path):
    """The reference loops forever here (bitstream.c:131-147); the drop-in must not."""
    path = str(tmp_path / "bs1.bin").encode()
    f = _libc.fopen(path, b"wb")
    s = lib().bit_stream_create_from_file_buffered(ctypes.c_void_p(f), 1)
    data = np.array([0xAB, 0xCD, 0xEF, 0x12], np.uint8)
    for L in (3, 17, 9, 30):
        lib().bit_stream_write(s, data.ctypes.data_as(ctypes.c_void_p), L)
    lib().bit_stream_destroy(s)
    _libc.fclose(ctypes.c_void_p(f))
    assert len(open(path, "rb").read()) == (3 + 17 + 9 + 30 + 7) // 8


def test_bitstream_reader_roundtrip(tmp_path):
    rng = np.random.default_rng(0)
    bits = rng.integers(0, 2, 1000).astype(np.uint8)
    packed = np.packbits(bits)
    path = str(tmp_path / "r.bin")
    packed.tofile(path)
    f = _libc.fopen(path.encode(), b"rb")
    s = lib().bit_stream_create_from_file_buffered(ctypes.c_void_p(f), 7)
    got = [lib().bit_stream_read_bit(s) for _ in range(1000)]
    lib().bit_stream_destroy(s)
    _libc.fclose(ctypes.c_void_p(f))
    assert np.array_equal(np.array(got, np.uint8), bits)


def test_decoder_known_answer():
    """huffman_decode.c:196-221 through the drop-in decoder API."""
    cbs = Codebooks(np.array([[1.0, 4, 3, 8, 3, 8]]), 6, False, threads=1)
    dec = lib().huffman_decoder_create(ctypes.byref(cbs.arr[0]))
    seq = [0, 1, 0, 2, 0, 1, 0, 3, 0, 1, 0, 2, 0, 1, 0, 4, 0, 1, 0, 2, 0, 1, 0, 3, 0, 1, 0, 2,
           0, 1, 0]
    out = []
    for s in seq:
        it = cbs.arr[0].items[s]
        out.append(lib().huffman_decoder_push_bits(dec, ctypes.cast(it.code, ctypes.c_void_p),
                                                   it.bit_length))
    lib().huffman_decoder_destroy(dec)
    assert "".join(chr(97 + s) for s in out) == "abacabadabacabaeabacabadabacaba"


def test_context_decoder_known_answer():
    """huffman_decode.c:223-279: 6x6 context codebook, 3 raw warm-up bits."""
    counts = np.array([1, 4, 3, 8, 3, 8, 3, 9, 4, 5, 2, 4, 9, 4, 3, 2, 8, 7, 6, 5, 4, 3, 2, 1,
                       5, 4, 2, 6, 9, 4, 3, 7, 3, 6, 9, 3], float)
    cbs = Codebooks(counts[None], 6, True, threads=1)
    dec = lib().huffman_decoder_create(ctypes.byref(cbs.arr[0]))
    for start in range(6):
        lib().huffman_decoder_reset(dec)
        prev = -1
        got, want = [], []
        for sym in range(6):
            if prev < 0:
                b = np.array([start << 5], np.uint8)
                r = lib().huffman_decoder_push_bits(dec, b.ctypes.data_as(ctypes.c_void_p), 3)
            else:
                it = cbs.arr[0].items[prev * 6 + start]
                r = lib().huffman_decoder_push_bits(dec, ctypes.cast(it.code, ctypes.c_void_p),
                                                    it.bit_length)
            got.append(r)
            want.append(start)
            it = cbs.arr[0].items[start * 6 + sym]
            got.append(lib().huffman_decoder_push_bits(dec, ctypes.cast(it.code, ctypes.c_void_p),
                                                       it.bit_length))
            want.append(sym)
            prev = sym
        assert got == want
    lib().huffman_decoder_destroy(dec)


@pytest.mark.parametrize("name", ["m8_n1000", "m16_n1000", "m8_n1", "m3_n2"])
@pytest.mark.parametrize("mode", ["nosort_ctx", "nosort_noctx", "sort_ctx"])
def test_codebooks_and_stats_from_reference_counts(oracle, name, mode):
    """Host codebooks (pqh_codebooks_build, threaded) + huffman_codebooks.bin + stats line
    from the same counts the reference saw."""
    g = golden(f"huff_{name}.npz")
    ctx = mode != "nosort_noctx"
    codes = oracle.sort_rows(g["input"]) if mode == "sort_ctx" else g["input"]
    counts = oracle.histogram(codes, 256, ctx)
    cbs = Codebooks(counts, 256, ctx)
    assert cbs.file_bytes() == g[mode + "__codebooks"].tobytes()
    st = HuffmanStats()
    lib().huffman_stats_init(ctypes.byref(st), len(codes), codes.shape[1], 256)
    st.num_roots = 1 if ctx else 0
    for i, e in enumerate(cbs.estimate()):
        lib().huffman_stats_push(ctypes.byref(st), i, float(e))
    with tempfile.TemporaryDirectory() as d:
        p = os.path.join(d, "stats.txt")
        lib().huffman_stats_print_filename(ctypes.byref(st), p.encode())
        assert open(p).read() == g[mode + "__stats"].tobytes().decode()
    lib().huffman_stats_destroy(ctypes.byref(st))


def test_vecs_light_roundtrip(tmp_path):
    a = np.arange(35, dtype=np.uint8).reshape(7, 5)
    p = str(tmp_path / "x.bvecsl")
    with open(p, "wb") as f:
        np.array([7, 5], np.uint32).tofile(f)
        a.tofile(f)
    n = ctypes.c_longlong()
    d = ctypes.c_int()
    ptr = lib().load_vecs_light_filename(p.encode(), 1, ctypes.byref(n), ctypes.byref(d))
    assert (n.value, d.value) == (7, 5)
    got = np.ctypeslib.as_array(ctypes.cast(ptr, ctypes.POINTER(ctypes.c_uint8)), (35,))
    assert np.array_equal(got.reshape(7, 5), a)
    assert lib().load_vecs_num_vectors_filename(p.encode()) == 7


def test_fvecs_and_centroids_io(tmp_path):
    from datagen import write_fvecs
    x = np.random.default_rng(1).random((9, 12)).astype(np.float32)
    p = str(tmp_path / "a.fvecs")
    write_fvecs(p, x)
    n = ctypes.c_longlong()
    d = ctypes.c_int()
    ptr = lib().fvecs_load(p.encode(), ctypes.byref(n), ctypes.byref(d))
    got = np.ctypeslib.as_array(ctypes.cast(ptr, ctypes.POINTER(ctypes.c_float)), (9 * 12,))
    assert (n.value, d.value) == (9, 12)
    assert np.array_equal(got.reshape(9, 12), x)


def test_block_matches_reference_behaviour():
    """block_t (fast_nn_block.c:6-71): capacity starts at 100 whatever initial_capacity says
    (:11), grows to (capacity + 1) * 2 on a full push (:42-44), keeps rows and global ids in
    push order; set_id empties the block (:68-71); destroy resets every field (:24-39)."""
    from pq_huffman_amd.capi import Block
    b = Block()
    lib().block_init(ctypes.byref(b), 7, 3, 5000, 0xFF)
    assert (b.id, b.num_dimensions, b.capacity, b.size) == (7, 3, 100, 0)
    rows = np.arange(3 * 250, dtype=np.float32).reshape(250, 3)
    caps = []
    for i in range(250):
        lib().block_push(ctypes.byref(b), 1000 + i, rows[i].ctypes.data_as(ctypes.c_void_p))
        caps.append(b.capacity)
    assert sorted(set(caps)) == [100, 202, 406]
    assert caps.index(202) == 100 and caps.index(406) == 202
    data = np.ctypeslib.as_array(b.data, (250 * 3,)).reshape(250, 3)
    ids = np.ctypeslib.as_array(b.indices, (250,))
    assert np.array_equal(data, rows) and np.array_equal(ids, np.arange(1000, 1250))
    lib().block_set_id(ctypes.byref(b), 9)
    assert (b.id, b.size, b.capacity) == (9, 0, 406)
    lib().block_destroy(ctypes.byref(b))
    assert (b.id, b.num_dimensions, b.capacity, b.size) == (-1, 0, 0, 0)
    assert not b.data and not b.indices
    # data-only block: no index array, rows still stored
    lib().block_init(ctypes.byref(b), 0, 2, 0, 0x01)
    assert not b.indices and b.data
    lib().block_destroy(ctypes.byref(b))


def test_shard_host_protocol():
    """pqh_shard_block / _offsets / _halo_source / _stitch (the host half of the multi-GPU
    protocol): row ranges partition the rows, offsets are the exclusive scan,
    the ragged halo comes from the nearest non-empty rank before, and stitching word-aligned
    shard buffers reproduces one stream."""
    from pq_huffman_amd.capi import Block
    L = lib()
    for n_total in (0, 1, 7, 1000, 10 ** 9 + 7):
        for world in (1, 3, 8):
            spans = []
            for r in range(world):
                b = Block()
                assert L.pqh_shard_block(n_total, world, r, ctypes.byref(b)) == 0
                spans.append((b.id, b.size))
            assert spans[0][0] == 0 and sum(s for _, s in spans) == n_total
            assert all(spans[i][0] + spans[i][1] == spans[i + 1][0] for i in range(world - 1))
            assert max(s for _, s in spans) - min(s for _, s in spans) <= 1
    b = Block()
    assert L.pqh_shard_block(10, 2, 2, ctypes.byref(b)) != 0           # rank out of range
    lens = (ctypes.c_ulonglong * 4)(13, 0, 40, 7)
    off, tot = ctypes.c_ulonglong(), ctypes.c_ulonglong()
    assert L.pqh_shard_offsets(lens, 4, 2, ctypes.byref(off), ctypes.byref(tot)) == 0
    assert (off.value, tot.value) == (13, 60)
    prev, raw = ctypes.c_int(), ctypes.c_int()
    has = (ctypes.c_int * 5)(0, 1, 0, 0, 1)
    for rank, want in ((0, (-1, 0)), (1, (-1, 1)), (3, (1, 0)), (4, (1, 0))):
        assert L.pqh_shard_halo_source(has, 5, rank, ctypes.byref(prev), ctypes.byref(raw)) == 0
        assert (prev.value, raw.value) == want
    # three shards of a 90-bit stream: 13 bits, 0 bits, 77 bits at global bit 13
    rng = np.random.default_rng(4)
    bits = rng.integers(0, 2, 90).astype(np.uint8)
    def buf(goff, nb):
        out = np.zeros(((goff % 32) + nb + 31) // 32 * 4 + 4, np.uint8)
        for j in range(nb):
            if bits[goff + j]:
                p = goff % 32 + j
                out[p // 8] |= 1 << (7 - p % 8)
        return out
    parts = [(buf(0, 13), 0, 13), (np.zeros(4, np.uint8), 13, 0), (buf(13, 77), 13, 77)]
    ptrs = (ctypes.c_void_p * 3)(*[p[0].ctypes.data for p in parts])
    offs = (ctypes.c_ulonglong * 3)(*[p[1] for p in parts])
    nbs = (ctypes.c_ulonglong * 3)(*[p[2] for p in parts])
    out = np.full(12, 0xAA, np.uint8)
    assert L.pqh_shard_stitch(3, ptrs, offs, nbs, out.ctypes.data, 12) == 0
    assert np.array_equal(out, np.packbits(bits))
    assert L.pqh_shard_stitch(3, ptrs, offs, nbs, out.ctypes.data, 11) != 0   # too small


def test_histogram_partials_bounded_by_the_grid():
    """pqh_histogram_partial_bytes: one partial image per 61,440-row chunk up to 64 chunks,
    then a fixed number of images (the multi-round form) + the u32 carry accumulator, so the
    125M-row shard of configs[2] needs ~18 MB instead of 2.1 GB (no GPU call)."""
    from pq_huffman_amd.capi import lib
    img = 32768 * 4
    assert lib().pqh_histogram_partial_bytes(1_000_000, 8, 256) == 17 * 8 * img
    big = lib().pqh_histogram_partial_bytes(125_000_000, 8, 256)
    assert big <= 16 * 8 * img + 8 * 65536 * 4 + 256
    assert lib().pqh_histogram_partial_bytes(10**10, 16, 256) <= 8 * 16 * img + 16 * 65536 * 4 + 256
