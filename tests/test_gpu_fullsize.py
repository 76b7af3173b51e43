"""Full-size parity of the exact path behind the bench line, and configs[2]'s per-rank
shard on one GPU.

The bench step (bench.py) is pq_assign (MFMA screen + exact re-rank) -> pqh_histogram_set
-> pqh_tables_build (GPU heap simulation) -> pqh_encode_write (one pass, chunk index) ->
pqh_decode (chunked).  Here the same calls, on the bench's own data generator and
centroids, are compared with the CPU oracle on every row:
  * all 1,000,000 PQ codes (oracle: fp32 direct form, first minimum -- SURVEY.md 8c),
  * the codebook file bytes and the stream bytes (huffman_encoder.c:398-428),
  * decode == codes (huffman_decoder.c:211-255),
for SIFT-like integer data (bf16-exact: no lo pass) and for Deep-like unit-norm data (every
x has a bf16 remainder: the lo pass and its tighter bound are active).

configs[2] (1B rows over 8 GPUs) is a 125M-row, 64 GB shard per rank: the shard is run on
one GPU through the same calls; the round trip must be exact, the stream length must equal
the codebook estimate, the GPU histogram and codebooks must equal the oracle's, and the PQ
codes must equal the oracle's on sampled windows of rows."""
import numpy as np
import pytest

import datagen

pytestmark = pytest.mark.gpu


def _bench_default_chunk():
    """bench.py's --chunk default: the decode-chunk size the timed bench line runs at"""
    import bench
    return bench.parse([]).chunk


BENCH_CHUNK = _bench_default_chunk()


@pytest.fixture(scope="module")
def gpu():
    import torch
    from pq_huffman_amd import codec
    assert torch.cuda.is_available()
    return torch, codec, codec.Context(0)


def _bench_path(gpu, x, cent, chunk=8, ctxm=True, sort=False):
    """the bench's per-batch calls, in its order, on one stream (bench.py front/back):
    assignment [-> sort] -> histogram -> GPU code tables -> one-pass encode -> decode"""
    torch, codec, ctx = gpu
    n = x.shape[0]
    m, k, _ = cent.shape
    pq = codec.PQ(ctx, cent)
    codes = torch.empty((n, m), dtype=torch.uint8 if k <= 256 else torch.int16, device=x.device)
    pq.assign(x, codes)
    if sort:   # stable strncmp-key sort of the rows, in place (huffman_encoder.c:301-317)
        codec.sort_rows(ctx, codes, torch.empty_like(codes))
    counts = torch.empty((m, k * k if ctxm else k), dtype=torch.int32, device=x.device)
    codec.histogram(ctx, codes, k, ctxm, counts=counts, accumulate=False)
    tabs = codec.Tables(ctx, m, k, ctxm).build(counts)
    chunks = (n + chunk - 1) // chunk
    out = torch.empty(n * m * 56 // 8 + 64, dtype=torch.uint8, device=x.device)
    coff = torch.empty(chunks, dtype=torch.int64, device=x.device)
    cprev = torch.empty((chunks, m), dtype=torch.uint8, device=x.device) if ctxm else None
    tot = torch.zeros(1, dtype=torch.int64, device=x.device)
    raw_first = 1 if ctxm else 0
    codec.encode_write(ctx, tabs, codes, out, 0, raw_first, None, chunk, coff, cprev, total=tot)
    codec.encode_status(ctx)
    enc = codec.Encoded(out, int(tot.item()), chunk, coff, cprev, n, raw_first)
    dec = codec.decode(ctx, tabs, enc)
    codec.decode_status(ctx)
    tabs.status()
    return pq, codes, counts, tabs, enc, dec


def _bench_path_parts(gpu, x, cent, chunk=8):
    """bench.py's DEFAULT per-batch calls at one rank (--code-layout parts, --hist-split on),
    issued exactly as front()/back() issue them: pqh_pq_assign_parts into a 128-padded
    [m][ld] buffer -> pqh_histogram_partial_parts + pqh_histogram_reduce -> code trees + decode
    tables -> pqh_encode_write_parts (the part-major row encoder) -> pqh_decode.  Returns the
    codes as rows (pqh_transpose_codes: the pq_indices.bvecsl layout) and the part buffer."""
    torch, codec, ctx = gpu
    n = x.shape[0]
    m, k, _ = cent.shape
    pq = codec.PQ(ctx, cent)
    ldp = (n + 127) // 128 * 128
    parts = torch.empty((m, ldp), dtype=torch.uint8, device=x.device)[:, :n]
    pq.assign_parts(x, parts)
    hp = torch.empty(codec.histogram_partial_bytes(n, m, k), dtype=torch.uint8, device=x.device)
    codec.histogram_partial_parts(ctx, parts, n, k, hp)
    counts = torch.empty((m, k * k), dtype=torch.int32, device=x.device)
    codec.histogram_reduce(ctx, hp, n, m, k, counts)
    tabs = codec.Tables(ctx, m, k, True)
    tabs.build_trees(counts)
    tabs.build_luts()
    chunks = (n + chunk - 1) // chunk
    out = torch.empty(n * m * 56 // 8 + 64, dtype=torch.uint8, device=x.device)
    coff = torch.empty(chunks, dtype=torch.int64, device=x.device)
    cprev = torch.empty((chunks, m), dtype=torch.uint8, device=x.device)
    tot = torch.zeros(1, dtype=torch.int64, device=x.device)
    codec.encode_write_parts(ctx, tabs, parts, n, out, 0, 1, None, chunk, coff, cprev, total=tot)
    codec.encode_status(ctx)
    enc = codec.Encoded(out, int(tot.item()), chunk, coff, cprev, n, 1)
    dec = codec.decode(ctx, tabs, enc)
    codec.decode_status(ctx)
    tabs.status()
    rows = codec.transpose_codes(ctx, parts, n)
    return pq, rows, parts, counts, tabs, enc, dec


def _check_chunk_index(torch, oracle, rows_h, ocb, enc, chunk):
    """every chunk offset is the oracle's bit position of its first row (the cumulative
    code lengths of the rows before it; row 0 raw), every chunk context row its predecessor"""
    n, m = rows_h.shape
    r = rows_h.astype(np.int64)
    lens = np.empty(n, np.int64)
    lens[0] = 8 * m                                    # row 0 raw (huffman_encoder.c:234)
    idx = r[:-1] * ocb.k + r[1:]                       # (prev << 8) + cur per part
    lens[1:] = ocb.lens[np.arange(m)[None, :], idx].sum(axis=1)
    starts = np.concatenate([[0], np.cumsum(lens)])
    want = starts[0:len(rows_h):chunk]
    assert np.array_equal(enc.chunk_offsets.cpu().numpy(), want)
    cp = enc.chunk_prev.cpu().numpy()
    assert np.array_equal(cp[1:], rows_h[chunk - 1:len(rows_h) - 1:chunk][:len(cp) - 1])


def _check_against_oracle(gpu, oracle, xh, cent, codes, tabs, enc, dec, ctxm=True, sort=False):
    torch, codec, ctx = gpu
    assert torch.equal(dec, codes)
    k = cent.shape[1]
    hc = codes.cpu().numpy()
    if k > 256:
        hc = hc.view(np.uint16)
    want, _ = oracle.pq_assign(xh, cent, threads=0)
    if sort:
        want = oracle.sort_rows(want)
    bad = int((hc != want).sum())
    assert bad == 0, f"{bad} PQ codes differ from the oracle"
    ocb = oracle.build_codebooks(want, k, ctxm)
    assert tabs.codebooks().file_bytes() == oracle.codebooks_file(ocb)
    stream, bits = oracle.encode(want, ocb)
    assert enc.bits == bits
    assert enc.stream[:len(stream)].cpu().numpy().tobytes() == stream


def test_bench_path_sift1m_all_rows(gpu, oracle):
    import bench
    torch, codec, ctx = gpu
    dev = torch.device("cuda", 0)
    x = bench.make_data(torch, 1_000_000, 128, 0x5EED, 0, dev)
    cent = bench.train_centroids(torch, bench.make_data(torch, 200_000, 128, 0x5EED, 0, dev),
                                 8, 256)
    pq, codes, counts, tabs, enc, dec = _bench_path(gpu, x, cent)
    assert pq.rerank_count() > 0
    _check_against_oracle(gpu, oracle, x.cpu().numpy(), cent, codes, tabs, enc, dec)


def _check_parts_against_oracle(gpu, oracle, xh, cent, rows, counts, tabs, enc, dec, chunk):
    """the part-major pipeline's every output against the oracle: codes, pair counts,
    codebook file, stream bytes and bit count, chunk index, decode"""
    torch, codec, ctx = gpu
    k = cent.shape[1]
    want, _ = oracle.pq_assign(xh, cent, threads=0)
    got = rows.cpu().numpy()
    bad = int((got != want).sum())
    assert bad == 0, f"{bad} part-major PQ codes differ from the oracle"
    assert np.array_equal(codec.counts_to_host(counts), oracle.histogram(want, k, True))
    ocb = oracle.build_codebooks(want, k, True)
    assert tabs.codebooks().file_bytes() == oracle.codebooks_file(ocb)
    stream, bits = oracle.encode(want, ocb)
    assert enc.bits == bits
    assert enc.stream[:len(stream)].cpu().numpy().tobytes() == stream
    _check_chunk_index(torch, oracle, want, ocb, enc, chunk)
    assert torch.equal(dec, rows)


def test_bench_parts_path_sift1m_all_rows(gpu, oracle):
    """the pipeline bench.py TIMES at one rank (part-major codes, split histogram), on the
    bench's own data and centroids, against the oracle on all 1,000,000 rows
    (src/pq_encoder.c:192-213, src/huffman_encoder.c:166-238,398-428)."""
    import bench
    torch, codec, ctx = gpu
    dev = torch.device("cuda", 0)
    x = bench.make_data(torch, 1_000_000, 128, 0x5EED, 0, dev)
    cent = bench.train_centroids(torch, bench.make_data(torch, 200_000, 128, 0x5EED, 0, dev),
                                 8, 256)
    pq, rows, parts, counts, tabs, enc, dec = _bench_path_parts(gpu, x, cent, chunk=BENCH_CHUNK)
    assert pq.rerank_count() > 0
    _check_parts_against_oracle(gpu, oracle, x.cpu().numpy(), cent, rows, counts, tabs, enc,
                                dec, BENCH_CHUNK)


def test_bench_parts_path_deep1m_all_rows(gpu, oracle):
    """`bench.py --config deep` as timed: 16 part-major runs, each vector encoded as two
    8-part rows gathered from them (the lo pass active: unit-norm floats)."""
    import bench
    torch, codec, ctx = gpu
    dev = torch.device("cuda", 0)
    x = bench.make_deep(torch, 1_000_000, 96, 0x5EED, 0, dev)
    cent = bench.train_centroids(torch, bench.make_deep(torch, 200_000, 96, 0x5EED, 0, dev),
                                 16, 256)
    pq, rows, parts, counts, tabs, enc, dec = _bench_path_parts(gpu, x, cent, chunk=BENCH_CHUNK)
    _check_parts_against_oracle(gpu, oracle, x.cpu().numpy(), cent, rows, counts, tabs, enc,
                                dec, BENCH_CHUNK)


def test_bench_path_deep1m_all_rows(gpu, oracle):
    """configs[3] shape (96-d, M = 16, dsub = 6) on 1M non-integer rows: the lo pass."""
    torch, codec, ctx = gpu
    xh = datagen.deep_like(1_000_000, 96, seed=31)
    assert (xh.view(np.uint32) & 0xFFFF).any(axis=1).all()   # every row has a remainder
    cent = datagen.lloyd_centroids(xh, 16, 256, iters=2, sample=30000, seed=5)
    x = torch.from_numpy(xh).cuda()
    pq, codes, counts, tabs, enc, dec = _bench_path(gpu, x, cent)
    _check_against_oracle(gpu, oracle, xh, cent, codes, tabs, enc, dec)


def test_bench_path_k4096_1m_all_rows(gpu, oracle):
    """configs[4] as `bench.py --config k4096` runs it, on all 1,000,000 rows: K = 4,096
    assignment (u16 codes, centroid tiles from L2) -> non-context histogram -> huff_trees_par
    code tables -> one-pass encode -> chunked decode; every code, the codebook file and the
    stream bytes against the oracle (src/huffman_encode.c:141-192, src/huffman_encoder.c:207-218)."""
    import bench
    torch, codec, ctx = gpu
    dev = torch.device("cuda", 0)
    x = bench.make_data(torch, 1_000_000, 128, 0x5EED, 0, dev)
    cent = bench.train_centroids(torch, bench.make_data(torch, 200_000, 128, 0x5EED, 0, dev),
                                 8, 4096)
    pq, codes, counts, tabs, enc, dec = _bench_path(gpu, x, cent, ctxm=False)
    assert pq.rerank_count() > 0
    _check_against_oracle(gpu, oracle, x.cpu().numpy(), cent, codes, tabs, enc, dec, ctxm=False)


def test_bench_path_sort_1m_all_rows(gpu, oracle):
    """`bench.py --sort` (the reference's default sort + context mode) on all 1,000,000 rows:
    assignment -> stable strncmp-key sort on the device -> context histogram -> GPU code tables
    -> encode -> decode, against the oracle's sorted codes, codebooks and stream
    (src/huffman_encoder.c:301-318, src/huffman_encode.c:235-269)."""
    import bench
    torch, codec, ctx = gpu
    dev = torch.device("cuda", 0)
    x = bench.make_data(torch, 1_000_000, 128, 0x5EED, 0, dev)
    cent = bench.train_centroids(torch, bench.make_data(torch, 200_000, 128, 0x5EED, 0, dev),
                                 8, 256)
    pq, codes, counts, tabs, enc, dec = _bench_path(gpu, x, cent, sort=True)
    _check_against_oracle(gpu, oracle, x.cpu().numpy(), cent, codes, tabs, enc, dec, sort=True)


def test_bench_path_deep_sort_1m_all_rows(gpu, oracle):
    """configs[3] in the reference's default sort + context mode (`bench.py --config deep
    --sort`): 16-byte rows through the hand-written radix sort (two words per row, 16
    passes), then the context path, against the oracle on all 1,000,000 rows."""
    torch, codec, ctx = gpu
    xh = datagen.deep_like(1_000_000, 96, seed=33)
    cent = datagen.lloyd_centroids(xh, 16, 256, iters=2, sample=30000, seed=6)
    x = torch.from_numpy(xh).cuda()
    pq, codes, counts, tabs, enc, dec = _bench_path(gpu, x, cent, sort=True)
    _check_against_oracle(gpu, oracle, xh, cent, codes, tabs, enc, dec, sort=True)


def test_configs2_shard_125m_rows(gpu, oracle):
    """BASELINE.json configs[2]: the per-rank shard (1e9 / 8 = 125M rows x 128-d, 64 GB)."""
    import bench
    torch, codec, ctx = gpu
    dev = torch.device("cuda", 0)
    n = 125_000_000
    x = bench.make_data(torch, n, 128, 0x5EED, 3, dev)
    cent = bench.train_centroids(torch, bench.make_data(torch, 200_000, 128, 0x5EED, 0, dev),
                                 8, 256)
    pq, codes, counts, tabs, enc, dec = _bench_path(gpu, x, cent, chunk=64)
    assert torch.equal(dec, codes)
    hc = codes.cpu().numpy()
    ch = codec.counts_to_host(counts)
    assert np.array_equal(ch, oracle.histogram(hc, 256, True).reshape(ch.shape))
    cbs = tabs.codebooks(ch)
    assert int(cbs.estimate().sum()) + 8 * 8 == enc.bits        # + row 0 raw
    ocb = oracle.build_codebooks(hc, 256, True)
    assert cbs.file_bytes() == oracle.codebooks_file(ocb)
    # PQ codes on windows: the first rows, rows around 2^26 and 2^31 / 32 blocks, the last
    for lo in (0, (1 << 26) - 50_000, 67_108_864 - 7, n - 100_000):
        w = slice(lo, lo + 100_000)
        want, _ = oracle.pq_assign(x[w].cpu().numpy(), cent, threads=0)
        assert np.array_equal(hc[w], want), lo
    # stream bits on a window: the oracle encodes rows [a - 1, b) -- row a - 1 raw, rows
    # [a, b) in context -- and the chunk index places rows [a, b) in the GPU stream
    a = (n // 2) // 64 * 64
    b = a + 200_000
    start = int(enc.chunk_offsets[a // 64].item())
    stop = int(enc.chunk_offsets[b // 64].item())
    ostream, obits = oracle.encode(np.ascontiguousarray(hc[a - 1:b]), ocb)
    assert obits - 8 * 8 == stop - start
    gbytes = enc.stream[start // 8:(stop + 7) // 8 + 1].cpu().numpy()
    gbits = np.unpackbits(gbytes)[start % 8:start % 8 + (stop - start)]
    assert np.array_equal(gbits, np.unpackbits(np.frombuffer(ostream, np.uint8))[64:obits])

    # The pipeline bench.py times on this shard (part-major codes, multi-round split
    # histogram, part-major row encoder), on the same rows: every code, the pair counts, every
    # stream byte and every chunk offset equal the row path's just checked above.
    row_stream = enc.stream[:(enc.bits + 7) // 8]
    row_coff = enc.chunk_offsets
    del dec, pq
    torch.cuda.empty_cache()
    pq2, rows2, parts2, counts2, tabs2, enc2, dec2 = _bench_path_parts(gpu, x, cent, chunk=64)
    assert torch.equal(rows2, codes)
    assert torch.equal(counts2, counts)
    assert tabs2.codebooks().file_bytes() == oracle.codebooks_file(ocb)
    assert enc2.bits == enc.bits
    assert torch.equal(enc2.stream[:(enc2.bits + 7) // 8], row_stream)
    assert torch.equal(enc2.chunk_offsets, row_coff)
    assert torch.equal(dec2, codes)


def test_encode_segmented_scan_5m_rows(gpu, oracle):
    """More than 16,384 encoder tiles (5M rows): the tiles' bit offsets come from the
    two-launch segmented scan (scan_seg_sums + scan_seg_write) instead of the one-workgroup
    scan.  For the row encoder and the part-major encoder alike: the bit count, every stream
    byte and the chunk index equal the oracle's (huffman_encoder.c:207-238), and the decode is
    exact."""
    torch, codec, ctx = gpu
    n, m, k, chunk = 5_000_003, 8, 256, 4
    rng = np.random.default_rng(91)
    base = np.minimum(rng.geometric(0.03, size=(n, m)) - 1, k - 1)
    codes_h = np.empty((n, m), np.uint8)
    for j in range(m):
        codes_h[:, j] = rng.permutation(k)[base[:, j]].astype(np.uint8)
    cd = torch.from_numpy(codes_h).cuda()
    counts = codec.histogram(ctx, cd, k, True)
    tabs = codec.Tables(ctx, m, k, True).build(counts)
    ocb = oracle.build_codebooks(codes_h, k, True)
    assert tabs.codebooks().file_bytes() == oracle.codebooks_file(ocb)
    stream, bits = oracle.encode(codes_h, ocb)
    enc = codec.encode(ctx, tabs, cd, chunk_vectors=chunk)
    assert enc.bits == bits
    assert enc.stream[:len(stream)].cpu().numpy().tobytes() == stream
    _check_chunk_index(torch, oracle, codes_h, ocb, enc, chunk)
    # the part-major encoder on the same rows
    ld = (n + 127) // 128 * 128
    parts = torch.empty((m, ld), dtype=torch.uint8, device=cd.device)
    parts[:, :n] = cd.t()
    out = torch.zeros_like(enc.stream)
    coff = torch.empty_like(enc.chunk_offsets)
    cprev = torch.empty_like(enc.chunk_prev)
    tot = torch.zeros(1, dtype=torch.int64, device=cd.device)
    codec.encode_write_parts(ctx, tabs, parts[:, :n], n, out, 0, 1, None, chunk, coff, cprev,
                             total=tot)
    codec.encode_status(ctx)
    assert int(tot.item()) == bits
    assert out[:len(stream)].cpu().numpy().tobytes() == stream
    assert torch.equal(coff, enc.chunk_offsets) and torch.equal(cprev, enc.chunk_prev)
    dec = codec.decode(ctx, tabs, enc)
    codec.decode_status(ctx)
    assert torch.equal(dec, cd)
