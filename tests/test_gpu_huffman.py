"""GPU parity of histogram / encode / decode (C ABI) against the reference-generated golden
files and the oracle: byte-exact huffman_indices.bin, exact round trips, shard composition,
full-size properties."""
import os
import subprocess

import numpy as np
import pytest

from conftest import ROOT, golden
import datagen

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def gpu():
    import torch
    from pq_huffman_amd import codec
    assert torch.cuda.is_available()
    return torch, codec, codec.Context(0)


def _codebooks_from_gpu_hist(gpu, codes, k, ctx_mode):
    torch, codec, ctx = gpu
    codes = np.ascontiguousarray(codes)
    if codes.dtype == np.uint16:
        codes = codes.view(np.int16)
    cd = torch.from_numpy(codes).cuda()
    counts = codec.histogram(ctx, cd, k, ctx_mode)
    return cd, codec.Codebooks(codec.counts_to_host(counts), k, ctx_mode)


@pytest.mark.parametrize("name", ["m8_n1000", "m16_n1000", "m8_n1", "m3_n2"])
@pytest.mark.parametrize("mode", ["nosort_ctx", "nosort_noctx"])
@pytest.mark.parametrize("chunk", [1, 7, 64])
def test_encode_decode_vs_reference_files(gpu, name, mode, chunk):
    torch, codec, ctx = gpu
    g = golden(f"huff_{name}.npz")
    ctxm = mode == "nosort_ctx"
    cd, cbs = _codebooks_from_gpu_hist(gpu, g["input"], 256, ctxm)
    assert cbs.file_bytes() == g[mode + "__codebooks"].tobytes()
    tabs = codec.Tables.from_codebooks(ctx, cbs)
    enc = codec.encode(ctx, tabs, cd, chunk_vectors=chunk)
    assert codec.indices_file_bytes(enc) == g[mode + "__indices"].tobytes()
    dec = codec.decode(ctx, tabs, enc)
    codec.decode_status(ctx)
    assert np.array_equal(dec.cpu().numpy(), g["input"])


def test_k4096_noctx_vs_reference(gpu):
    torch, codec, ctx = gpu
    g = golden("huff_k4096_m8_n2000.npz")
    cd, cbs = _codebooks_from_gpu_hist(gpu, g["input"], 4096, False)
    assert cbs.file_bytes() == g["nosort_noctx__codebooks"].tobytes()
    tabs = codec.Tables.from_codebooks(ctx, cbs)
    enc = codec.encode(ctx, tabs, cd, chunk_vectors=16)
    assert codec.indices_file_bytes(enc) == g["nosort_noctx__indices"].tobytes()
    dec = codec.decode(ctx, tabs, enc)
    assert np.array_equal(dec.cpu().numpy().view(np.uint16), g["input"])


@pytest.mark.parametrize("ctxm", [True, False])
def test_histogram_set_overwrites(gpu, oracle, ctxm):
    """pqh_histogram_set: counts = histogram, whatever the buffer held (the bench's form);
    n = 0 gives zeros.  Sizes span several 61,440-vector chunks plus a partial one."""
    torch, codec, ctx = gpu
    for n in (130001, 5, 0):
        codes = datagen.skewed_codes(max(n, 1), 8, seed=9)[:n]
        cd = torch.from_numpy(np.ascontiguousarray(codes)).cuda().reshape(n, 8)
        items = 256 * 256 if ctxm else 256
        junk = torch.full((8, items), 12345, dtype=torch.int32, device="cuda")
        codec.histogram(ctx, cd, 256, ctxm, counts=junk, accumulate=False)
        want = (oracle.histogram(codes, 256, ctxm) if n else np.zeros((8, items), np.int64))
        assert np.array_equal(codec.counts_to_host(junk), want)


@pytest.mark.parametrize("m", [4, 8, 12, 16])
def test_context_histogram_part_counts_and_offsets(gpu, oracle, m):
    """The context histogram's kernel forms: wave-contiguous rows for m % 4 == 0 (aligned),
    per-thread runs otherwise; full and partial waves and chunks (n spans three 61,440-row
    chunks), a sliced start row (unaligned for the wave form at m = 8), and the halo row."""
    torch, codec, ctx = gpu
    n = 130001
    codes = datagen.skewed_codes(n, m, seed=11 + m)
    cd = torch.from_numpy(np.ascontiguousarray(codes)).cuda().reshape(n, m)
    got = codec.counts_to_host(codec.histogram(ctx, cd, 256, True))
    assert np.array_equal(got, oracle.histogram(codes, 256, True))
    for s in (1, 3, 64):   # rows [s, n) with row s - 1 as the halo
        part = codec.histogram(ctx, cd[s:], 256, True, prev_row=cd[s - 1])
        want = oracle.histogram(codes[s - 1:], 256, True)
        want -= oracle.histogram(codes[s - 1:s], 256, True)   # (the raw row's own count: none)
        assert np.array_equal(codec.counts_to_host(part), want), s


@pytest.mark.parametrize("m", [8, 16])
def test_histogram_partial_then_reduce(gpu, oracle, m):
    """pqh_histogram_partial + pqh_histogram_reduce (the bench's split histogram) == the
    one-call context histogram: set and accumulate, with and without the halo row, n = 0."""
    torch, codec, ctx = gpu
    n = 130001
    codes = datagen.skewed_codes(n, m, seed=71 + m)
    cd = torch.from_numpy(np.ascontiguousarray(codes)).cuda()
    parts = torch.empty(codec.histogram_partial_bytes(n, m, 256), dtype=torch.uint8, device="cuda")
    junk = torch.full((m, 65536), 777, dtype=torch.int32, device="cuda")
    codec.histogram_partial(ctx, cd, 256, parts)
    codec.histogram_reduce(ctx, parts, n, m, 256, junk)
    whole = codec.counts_to_host(junk)
    assert np.array_equal(whole, oracle.histogram(codes, 256, True))
    codec.histogram_partial(ctx, cd[1:], 256, parts, prev_row=cd[0])
    codec.histogram_reduce(ctx, parts, n - 1, m, 256, junk, accumulate=True)
    assert np.array_equal(codec.counts_to_host(junk), 2 * whole)
    codec.histogram_reduce(ctx, parts, 0, m, 256, junk)   # n = 0 with set: zeros
    assert not codec.counts_to_host(junk).any()


@pytest.mark.parametrize("ctxm", [True, False])
def test_histogram_vs_oracle_with_halo(gpu, oracle, ctxm):
    torch, codec, ctx = gpu
    codes = datagen.skewed_codes(70001, 8, seed=8)
    cd = torch.from_numpy(codes).cuda()
    got = codec.counts_to_host(codec.histogram(ctx, cd, 256, ctxm))
    assert np.array_equal(got, oracle.histogram(codes, 256, ctxm))
    if ctxm:  # shard [40000:) with the halo row 39999 == the pairs of the whole array
        a = codec.histogram(ctx, cd[:40000], 256, True)
        codec.histogram(ctx, cd[40000:], 256, True, prev_row=cd[39999], counts=a)
        assert np.array_equal(codec.counts_to_host(a), got)


@pytest.mark.parametrize("ctxm", [True, False])
def test_sharded_encode_composes(gpu, oracle, ctxm):
    """Two shards written at their global bit offsets into one buffer == one-shot stream
    (the multi-GPU concatenation rule)."""
    torch, codec, ctx = gpu
    codes = datagen.skewed_codes(9000, 8, seed=31)
    cd, cbs = _codebooks_from_gpu_hist(gpu, codes, 256, ctxm)
    tabs = codec.Tables.from_codebooks(ctx, cbs)
    whole = codec.encode(ctx, tabs, cd, chunk_vectors=32)
    cut = 4321
    a, b = cd[:cut], cd[cut:]
    ta = int(codec.encode_size(ctx, tabs, a, 1, None).item())
    tb = int(codec.encode_size(ctx, tabs, b, 0, cd[cut - 1] if ctxm else None).item())
    assert ta + tb == whole.bits
    out = torch.zeros_like(whole.stream)
    codec.encode_write(ctx, tabs, a, out, 0, 1, None, 0)
    codec.encode_write(ctx, tabs, b, out, ta, 0, cd[cut - 1] if ctxm else None, 0)
    assert torch.equal(out, whole.stream)
    stream, bits = oracle.encode(codes, oracle.build_codebooks(codes, 256, ctxm))
    assert bits == whole.bits
    assert out[:len(stream)].cpu().numpy().tobytes() == stream


@pytest.mark.parametrize("ctxm", [True, False])
def test_sharded_encode_device_offsets(gpu, oracle, ctxm):
    """Three shards, each written into a buffer of its own by pqh_encode_write_at with its
    global bit offset in device memory (the multi-GPU path: no host round trip), stitched
    by shard.stitch == the oracle's one-shot stream; each shard decodes from its own chunk
    index."""
    torch, codec, ctx = gpu
    from pq_huffman_amd import shard
    codes = datagen.skewed_codes(7001, 8, seed=41)
    cd, cbs = _codebooks_from_gpu_hist(gpu, codes, 256, ctxm)
    tabs = codec.Tables.from_codebooks(ctx, cbs)
    cuts = [0, 2500, 4999, 7001]
    totals, parts = [], []
    for r in range(3):
        piece = cd[cuts[r]:cuts[r + 1]]
        prev = cd[cuts[r] - 1] if (ctxm and r > 0) else None
        totals.append(codec.encode_size(ctx, tabs, piece, 1 if r == 0 else 0, prev))
        parts.append((piece, prev))
    offs = torch.cumsum(torch.cat(totals), 0) - torch.cat(totals)   # device prefix sum
    shards = []
    for r, (piece, prev) in enumerate(parts):
        goff = offs[r:r + 1].clone()
        out = torch.zeros(piece.shape[0] * 8 * 7 + 64, dtype=torch.uint8, device="cuda")
        nch = (piece.shape[0] + 15) // 16
        coff = torch.empty(nch, dtype=torch.int64, device="cuda")
        cprev = torch.empty((nch, 8), dtype=torch.uint8, device="cuda") if ctxm else None
        tot = torch.zeros(1, dtype=torch.int64, device="cuda")
        codec.encode_write_at(ctx, tabs, piece, out, goff, 1 if r == 0 else 0, prev, 16,
                              coff, cprev, total=tot)
        codec.encode_status(ctx)
        g = int(goff.item())
        bits = int(tot.item())
        assert bits == int(totals[r].item())
        enc = codec.Encoded(out, -1, 16, coff, cprev, piece.shape[0], 1 if r == 0 else 0)
        dec = codec.decode(ctx, tabs, enc)
        codec.decode_status(ctx)
        assert torch.equal(dec, piece), r
        shards.append((out.cpu().numpy().tobytes(), g, bits))
    total_bits = sum(s[2] for s in shards)
    stream, obits = oracle.encode(codes, oracle.build_codebooks(codes, 256, ctxm))
    assert obits == total_bits
    assert shard.stitch(shards, total_bits)[:len(stream)] == stream


def test_corrupt_stream_is_reported(gpu):
    torch, codec, ctx = gpu
    codes = np.zeros((100, 2), np.uint8)
    codes[::2, 0] = 1
    cd, cbs = _codebooks_from_gpu_hist(gpu, codes, 256, False)
    tabs = codec.Tables.from_codebooks(ctx, cbs)
    enc = codec.encode(ctx, tabs, cd, chunk_vectors=10)
    # part 1 has a single symbol: code "0"; a 1 bit there is invalid
    good = enc.stream.clone()
    enc.stream[:] = 0xFF
    codec.decode(ctx, tabs, enc)
    # the error is sticky: a good decode after it does not clear it, the status call does
    enc.stream.copy_(good)
    assert torch.equal(codec.decode(ctx, tabs, enc), cd)
    with pytest.raises(Exception):
        codec.decode_status(ctx)
    codec.decode_status(ctx)


@pytest.mark.parametrize("ctxm", [True, False])
def test_full_size_roundtrip_sift1m(gpu, oracle, ctxm):
    """SIFT1M-shaped: assign (MFMA) -> hist -> codebooks -> encode -> decode; exact round
    trip, total bits == the codebook estimate, stream byte-equal to the oracle's."""
    torch, codec, ctx = gpu
    n = 1_000_000
    x = datagen.sift_like(n, 128, seed=77)
    cent = datagen.lloyd_centroids(x, 8, 256, iters=2, sample=20000)
    pq = codec.PQ(ctx, cent)
    xd = torch.from_numpy(x).cuda()
    codes = pq.assign(xd)
    counts = codec.histogram(ctx, codes, 256, ctxm)
    cbs = codec.Codebooks(codec.counts_to_host(counts), 256, ctxm)
    tabs = codec.Tables.from_codebooks(ctx, cbs)
    enc = codec.encode(ctx, tabs, codes, chunk_vectors=64)
    dec = codec.decode(ctx, tabs, enc)
    codec.decode_status(ctx)
    assert torch.equal(dec, codes)
    est = cbs.estimate().sum() + (8 * 8 if ctxm else 0)
    assert enc.bits == int(est)
    hc = codes.cpu().numpy()
    stream, bits = oracle.encode(hc, oracle.build_codebooks(hc, 256, ctxm))
    assert bits == enc.bits
    assert enc.stream[:len(stream)].cpu().numpy().tobytes() == stream
    # the PQ codes themselves: oracle on a 20k-row sample
    sel = np.random.default_rng(0).choice(n, 20000, replace=False)
    want, _ = oracle.pq_assign(x[sel], cent, threads=0)
    assert np.array_equal(hc[sel], want)


@pytest.mark.parametrize("case", ["enc_test_many", "enc_test_one", "enc_test_zero",
                                  "ties_small_ints", "ties_all_equal", "ties_powers",
                                  "single_symbol", "empty", "geometric"])
@pytest.mark.parametrize("impl", ["grp", "lane", "wave"])
def test_gpu_tree_builder_vs_reference_codebooks(gpu, case, impl, monkeypatch):
    """pqh_tables_build (GPU heap simulation, both builds) == the reference's codebook bytes."""
    monkeypatch.setenv("PQH_TREE_IMPL", impl)
    torch, codec, ctx = gpu
    g = golden("codebooks.npz")
    k, c = (int(v) for v in g[case + "__alphabet"])
    counts = torch.from_numpy(g[case + "__counts"].astype(np.int32)[None]).cuda()
    tabs = codec.Tables(ctx, 1, k, bool(c)).build(counts)
    cbs = tabs.codebooks()
    assert cbs.file_bytes() == np.uint32(1).tobytes() + g[case + "__file"].tobytes()


@pytest.mark.parametrize("ctxm", [True, False])
@pytest.mark.parametrize("impl", ["grp", "lane", "wave"])
def test_gpu_tree_builder_vs_host_builder_ties(gpu, ctxm, impl, monkeypatch):
    """2048 tie-heavy context trees (or 8 plain ones): GPU tables == host codebooks."""
    monkeypatch.setenv("PQH_TREE_IMPL", impl)
    torch, codec, ctx = gpu
    rng = np.random.default_rng(17)
    items = 256 * 256 if ctxm else 256
    counts = rng.integers(0, 4, (8, items)).astype(np.int64)
    counts[:, : items // 3] *= rng.integers(0, 50, (8, items // 3))
    if ctxm:
        counts[0, 5 * 256:6 * 256] = 0      # an empty context row
        counts[1, 7 * 256:8 * 256] = 0
        counts[1, 7 * 256 + 3] = 9          # a one-symbol context row
    else:
        counts[2] = 0
        counts[2, 77] = 5                   # a one-symbol part
    host = codec.Codebooks(counts.astype(np.float64), 256, ctxm)
    dev = codec.Tables(ctx, 8, 256, ctxm).build(torch.from_numpy(counts.astype(np.int32)).cuda())
    assert dev.codebooks().file_bytes() == host.file_bytes()


@pytest.mark.parametrize("impl", ["grp", "lane"])
def test_gpu_tree_builder_random_shapes(gpu, impl, monkeypatch):
    """2048 context alphabets of random size (0 to 256 symbols) and shape -- tie-heavy small
    counts, geometric, Zipf, a few dominant symbols, all equal -- GPU tables == host codebooks
    (every sift depth of the 16-lane stretches, heaps of 1 to 256 entries)."""
    monkeypatch.setenv("PQH_TREE_IMPL", impl)
    torch, codec, ctx = gpu
    rng = np.random.default_rng(57)
    counts = np.zeros((8, 256 * 256), np.int64)
    for t in range(8 * 256):
        nzc = int(rng.choice([0, 1, 2, 3, 7, 16, 17, 31, 64, 100, 200, 255, 256]))
        sym = rng.choice(256, nzc, replace=False)
        kind = t % 5
        if kind == 0:
            w = rng.integers(1, 4, nzc)
        elif kind == 1:
            w = 2 ** rng.integers(0, 12, nzc)
        elif kind == 2:
            w = np.floor(5e4 / (np.arange(nzc) + 1) ** 1.2).astype(np.int64) + 1
        elif kind == 3:
            w = rng.integers(1, 6, nzc)
            w[: max(1, nzc // 20)] = rng.integers(10_000, 20_000)
        else:
            w = np.full(nzc, 7)
        counts[t // 256, (t % 256) * 256 + sym] = w
    dev = codec.Tables(ctx, 8, 256, True).build(torch.from_numpy(counts.astype(np.int32)).cuda())
    host = codec.Codebooks(counts.astype(np.float64), 256, True)
    assert dev.codebooks().file_bytes() == host.file_bytes()


@pytest.mark.parametrize("impl", ["grp", "lane"])
def test_encode_after_trees_only(gpu, oracle, impl):
    """The group tree build writes the encoder's gather copy itself (encode_ready): an encode
    issued right after build_trees, before the decode tables, gives the one-shot stream; the
    lane build does not claim it.  Then the decode tables decode that stream."""
    torch, codec, ctx = gpu
    codes = datagen.skewed_codes(20001, 8, seed=21)
    cd = torch.from_numpy(codes).cuda()
    counts = codec.histogram(ctx, cd, 256, True)
    ref = codec.encode(ctx, codec.Tables(ctx, 8, 256, True).build(counts), cd, chunk_vectors=8)
    t = codec.Tables(ctx, 8, 256, True).build_trees(counts, trees=impl)
    assert t.encode_ready() == (impl == "grp")
    if impl == "grp":
        enc = codec.encode(ctx, t, cd, chunk_vectors=8)
        assert codec.indices_file_bytes(enc) == codec.indices_file_bytes(ref)
    t.build_luts()
    assert not t.encode_ready() or impl == "grp"
    dec = codec.decode(ctx, t, ref)
    assert np.array_equal(dec.cpu().numpy(), codes)


@pytest.mark.parametrize("luts", ["grp", "block"])
def test_gpu_decode_tables_long_codes(gpu, luts, monkeypatch):
    """Context decode tables (lut_grp, the default, and lut_build, PQH_LUT_IMPL=block) for
    alphabets whose codes reach ~30 bits: first level (W1 = 9), second-level subtables and
    the long-code list all used; every row round-trips (huffman_decode.c:137-191)."""
    monkeypatch.setenv("PQH_LUT_IMPL", luts)
    torch, codec, ctx = gpu
    rng = np.random.default_rng(61)
    m, k, n = 8, 256, 30000
    w = np.maximum(1, np.floor(2.0 ** 20 / 1.5 ** np.arange(k))).astype(np.int64)
    counts = np.zeros((m, k * k), np.int64)
    for i in range(m):
        for c in range(k):
            counts[i, c * k:(c + 1) * k] = np.roll(w, (7 * c + i) % k)   # every pair coded
    tabs = codec.Tables(ctx, m, k, True).build(torch.from_numpy(counts.astype(np.int32)).cuda())
    host = codec.Codebooks(counts.astype(np.float64), k, True)
    assert tabs.codebooks().file_bytes() == host.file_bytes()
    codes = torch.from_numpy(rng.integers(0, k, (n, m)).astype(np.uint8)).cuda()
    for chunk in (1, 8, 33):
        enc = codec.encode(ctx, tabs, codes, chunk_vectors=chunk)
        codec.encode_status(ctx)
        dec = codec.decode(ctx, tabs, enc)
        codec.decode_status(ctx)
        assert torch.equal(dec, codes)


@pytest.mark.parametrize("impl", ["grp", "lane", "wave"])
def test_gpu_tree_builder_mixed_heavy_light(gpu, impl, monkeypatch):
    """Context alphabets of one workgroup that take different heaps: frequent previous
    symbols give trees past 2^22 (64-bit keys), rare ones stay on the u32 sentinel heap.
    (Regression: the 64-bit heap once overwrote its neighbours' sentinels.)"""
    monkeypatch.setenv("PQH_TREE_IMPL", impl)
    torch, codec, ctx = gpu
    rng = np.random.default_rng(31)
    codes = torch.from_numpy(rng.zipf(1.3, (20000, 8)).clip(1, 256).astype(np.uint8) - 1).cuda()
    c = codec.histogram(ctx, codes, 256, True)
    c = c * 1000 + (c > 0).to(c.dtype) * 5
    tabs = codec.Tables(ctx, 8, 256, True).build(c)
    host = codec.Codebooks(c.cpu().numpy().astype(np.float64), 256, True)
    assert tabs.codebooks().file_bytes() == host.file_bytes()


@pytest.mark.parametrize("ctxm", [True, False])
def test_gpu_tree_builder_pair(gpu, ctxm):
    """pqh_tables_build_pair: two table sets from two histograms (tie-heavy, and heavy with
    64-bit keys) in one tree launch == each set's host codebooks; the pair's decode tables
    decode both sets' streams."""
    torch, codec, ctx = gpu
    rng = np.random.default_rng(29)
    codes = torch.from_numpy(rng.zipf(1.3, (20000, 8)).clip(1, 256).astype(np.uint8) - 1).cuda()
    c1 = codec.histogram(ctx, codes, 256, ctxm)                 # tie-heavy small counts
    c2 = c1 * 1000 + (c1 > 0).to(c1.dtype) * 5                  # totals past 2^22: 64-bit keys
    t1 = codec.Tables(ctx, 8, 256, ctxm)
    t2 = codec.Tables(ctx, 8, 256, ctxm)
    t1.build_pair(c1, t2, c2)
    t1.status()
    t2.status()
    for t, c in ((t1, c1), (t2, c2)):
        host = codec.Codebooks(c.cpu().numpy().astype(np.float64), 256, ctxm)
        assert t.codebooks().file_bytes() == host.file_bytes()
        enc = codec.encode(ctx, t, codes, chunk_vectors=8)
        assert torch.equal(codec.decode(ctx, t, enc), codes)
    codec.decode_status(ctx)


def test_gpu_tree_builder_pair_k4096(gpu):
    """pqh_tables_build_pair at K = 4096 (one huff_trees_par launch over both sets' 16 trees):
    each set == its host codebooks, and each set's decode tables decode its stream."""
    torch, codec, ctx = gpu
    k = 4096
    codes = datagen.skewed_codes(30000, 8, k=k, seed=83)
    cd = torch.from_numpy(codes.view(np.int16)).cuda()
    c1 = codec.histogram(ctx, cd, k, False)
    c2 = c1 * 3 + (c1 > 0).to(c1.dtype)
    t1, t2 = codec.Tables(ctx, 8, k, False), codec.Tables(ctx, 8, k, False)
    t1.build_pair(c1, t2, c2)
    for t, c in ((t1, c1), (t2, c2)):
        t.status()
        host = codec.Codebooks(c.cpu().numpy().astype(np.float64), k, False)
        assert t.codebooks().file_bytes() == host.file_bytes()
        enc = codec.encode(ctx, t, cd, chunk_vectors=8)
        assert torch.equal(codec.decode(ctx, t, enc), cd)


@pytest.mark.parametrize("ctxm", [True, False])
@pytest.mark.parametrize("impl", ["grp", "lane", "wave"])
def test_gpu_tree_builder_heavy_and_rebuilt(gpu, ctxm, impl, monkeypatch):
    """Trees whose total weight reaches 2^22 (64-bit heap keys) with ties, and a table set
    rebuilt from a histogram with fewer symbols: every entry is rewritten (the build does not
    memset), so the second build equals the host codebooks of the second histogram."""
    monkeypatch.setenv("PQH_TREE_IMPL", impl)
    torch, codec, ctx = gpu
    rng = np.random.default_rng(23)
    items = 256 * 256 if ctxm else 256
    heavy = rng.integers(0, 3, (8, items)).astype(np.int64) * 3_000_000
    heavy[:, ::7] += 5                        # ties among light and heavy leaves
    heavy[3, : items // 2] = 0
    sparse = np.zeros((8, items), np.int64)
    sparse[:, ::5] = rng.integers(1, 9, (8, len(range(0, items, 5))))
    tabs = codec.Tables(ctx, 8, 256, ctxm)
    for counts in (heavy, sparse):
        assert counts.max() < 2 ** 31
        tabs.build(torch.from_numpy(counts.astype(np.int32)).cuda())
        host = codec.Codebooks(counts.astype(np.float64), 256, ctxm)
        assert tabs.codebooks().file_bytes() == host.file_bytes()


@pytest.mark.parametrize("impl", ["lane", "par"])
def test_gpu_tree_builder_k4096_vs_host(gpu, impl, monkeypatch):
    """K = 4096 trees (huff_trees_par: one wave per tree, sifts read in parallel; and the
    one-lane build, PQH_TREE_IMPL=lane): tie-heavy, heavy (64-bit weights), skewed,
    one-symbol and empty parts, then a sparser rebuild -- GPU tables == host codebooks."""
    monkeypatch.setenv("PQH_TREE_IMPL", impl)
    torch, codec, ctx = gpu
    rng = np.random.default_rng(41)
    k = 4096
    a = rng.integers(0, 4, (8, k)).astype(np.int64)
    a[0] *= rng.integers(0, 50, k)                            # ties among small counts
    a[1] = rng.integers(0, 3, k) * 3_000_000 + (np.arange(k) % 7 == 0) * 5   # heavy + light
    a[2] = 0
    a[2, 4000] = 11                                           # one symbol
    a[3] = 0                                                  # empty part
    a[4] = np.floor(1e6 / (np.arange(k) + 1) ** 1.1).astype(np.int64)   # Zipf-like
    a[5] = 1                                                  # all equal
    a[6, ::3] = 0
    a[7] = rng.integers(1, 2 ** 20, k)
    b = np.zeros_like(a)
    b[:, ::9] = rng.integers(1, 5, (8, len(range(0, k, 9))))
    tabs = codec.Tables(ctx, 8, k, False)
    for counts in (a, b):
        assert counts.max() < 2 ** 31
        tabs.build(torch.from_numpy(counts.astype(np.int32)).cuda())
        host = codec.Codebooks(counts.astype(np.float64), k, False)
        assert tabs.codebooks().file_bytes() == host.file_bytes()


def _run(args, cwd=None):
    r = subprocess.run(args, capture_output=True, text=True, cwd=cwd)
    assert r.returncode == 0, r.stdout + r.stderr
    return r.stdout


@pytest.mark.parametrize("mode,flags", [("sort_ctx", []),
                                        ("nosort_ctx", ["--no-sort"]),
                                        ("nosort_noctx", ["--no-sort", "--no-context"])])
def test_cli_tools_match_reference_files(tmp_path, mode, flags):
    g = golden("huff_m8_n1000.npz")
    bind = os.path.join(ROOT, "pq_huffman_amd", "bin")
    pqdir, out = tmp_path / "pq", tmp_path / "out"
    pqdir.mkdir()
    out.mkdir()
    datagen.write_vecsl(str(pqdir / "pq_indices.bvecsl"), g["input"])
    _run([os.path.join(bind, "huffman_encoder"), str(pqdir) + "/", str(out) + "/", "8"] + flags)
    assert (out / "huffman_codebooks.bin").read_bytes() == g[mode + "__codebooks"].tobytes()
    assert (out / "huffman_indices.bin").read_bytes() == g[mode + "__indices"].tobytes()
    assert (out / "huffman_stats.txt").read_text() == g[mode + "__stats"].tobytes().decode()
    dec = tmp_path / "dec.bin"
    _run([os.path.join(bind, "huffman_decoder"), str(out) + "/", "--output-file", str(dec),
          "--check-file", str(pqdir / "pq_indices.bvecsl")])
    want = g[mode + "__decoded"].reshape(1000, 8)      # sort mode decodes the sorted rows
    assert np.array_equal(np.fromfile(dec, np.uint8).reshape(1000, 8), want)
    # without the sidecar the decoder rebuilds the chunk index from the stream
    (out / "huffman_chunks.bin").unlink()
    _run([os.path.join(bind, "huffman_decoder"), str(out) + "/", "--output-file", str(dec)])
    assert np.array_equal(np.fromfile(dec, np.uint8).reshape(1000, 8), want)


@pytest.mark.parametrize("chunk", [None, "97"])
def test_cli_pq_encoder_fixed_centroids(tmp_path, oracle, chunk, monkeypatch):
    """pq_encoder --centroids streams the .fvecs file to the GPU (pq_encode_rows; chunk 97:
    eleven chunks of a 1,000-row file) and writes the reference's files."""
    if chunk:
        monkeypatch.setenv("PQH_ENCODE_CHUNK", chunk)
    g = golden("pq_sift_n1000_m8_k256.npz")
    bind = os.path.join(ROOT, "pq_huffman_amd", "bin")
    datagen.write_fvecs(str(tmp_path / "x.fvecs"), g["x"])
    cfile = tmp_path / "c.fvecsl"
    datagen.write_vecsl(str(cfile), g["centroids"].reshape(8 * 256, 16))
    _run([os.path.join(bind, "pq_encoder"), str(tmp_path / "x.fvecs"), str(tmp_path) + "/", "8",
          "--centroids", str(cfile), "--compute-error"])
    raw = (tmp_path / "pq_indices.bvecsl").read_bytes()
    assert np.frombuffer(raw[:8], np.uint32).tolist() == [1000, 8]
    assert np.array_equal(np.frombuffer(raw[8:], np.uint8).reshape(1000, 8), g["codes"])
    err = float((tmp_path / "pq_error").read_text().strip())
    want = oracle.compute_error(g["x"], g["centroids"], g["codes"])
    assert abs(err - want) <= 1e-6 * want


def _zero_heavy_rows(n, m, seed):
    """Rows that exercise the strncmp key: many zeros at every position, repeated rows and
    rows equal up to their first zero (whose tails must keep input order)."""
    rng = np.random.default_rng(seed)
    a = rng.integers(0, 4, size=(n, m)).astype(np.uint8)
    a[rng.random((n, m)) < 0.3] = 0
    half = a[1::4]
    a[1::4] = a[0::4][: len(half)]          # exact duplicates
    a[2::4, 0] = 0                          # ties decided by input order alone
    return np.ascontiguousarray(a)


@pytest.mark.parametrize("n,m", [(1, 8), (2, 8), (1000, 8), (1000, 16), (777, 3), (513, 12),
                                 (300, 1), (2000, 24), (2048, 8), (2049, 8), (4097, 2),
                                 (50_000, 8), (30_001, 7), (100_000, 4), (300_000, 8),
                                 (8193, 16), (40_000, 9), (20_001, 15), (300_000, 16),
                                 (4097, 1), (300_000, 1), (4099, 17), (50_000, 32),
                                 (300_000, 32), (20_001, 41), (30_000, 64)])
def test_gpu_sort_rows_vs_oracle(gpu, oracle, n, m):
    """2 <= m <= 16 runs the hand-written radix passes (one or two words per row; tiles of
    4,096 rows chained by the look-back: the sizes straddle tile edges), m = 1 and m > 16
    the same passes over (key chunk, row index) pairs, chunk by chunk."""
    torch, codec, ctx = gpu
    for seed in (1, 2):
        a = _zero_heavy_rows(n, m, seed)
        d = torch.from_numpy(a.copy()).cuda()
        codec.sort_rows(ctx, d)
        assert np.array_equal(d.cpu().numpy(), oracle.sort_rows(a))


@pytest.mark.parametrize("m", [8, 32])
def test_gpu_sort_rows_radix_vs_rocprim(gpu, m):
    """The radix passes and the rocPRIM path (PQH_SORT_IMPL=rocprim) give the same rows, on
    skewed full-alphabet codes and on heavy ties spread over many tiles (m = 32: the pair
    passes)."""
    import sys
    import tempfile
    torch, codec, ctx = gpu
    a = datagen.skewed_codes(200_000, m, 256, seed=11)
    a[::3] = a[0]                                  # one row repeated across every tile
    d = torch.from_numpy(a.copy()).cuda()
    codec.sort_rows(ctx, d)
    code = ("import numpy as np, torch, sys; sys.path.insert(0, %r); "
            "from pq_huffman_amd import codec; c = codec.Context(0); "
            "a = np.load(sys.argv[1]); d = torch.from_numpy(a).cuda(); codec.sort_rows(c, d); "
            "np.save(sys.argv[1], d.cpu().numpy())") % ROOT
    with tempfile.TemporaryDirectory() as td:
        f = os.path.join(td, "a.npy")
        np.save(f, a)
        r = subprocess.run([sys.executable, "-c", code, f], capture_output=True, text=True,
                           env=dict(os.environ, PQH_SORT_IMPL="rocprim"), timeout=300)
        assert r.returncode == 0, r.stderr
        np.testing.assert_array_equal(d.cpu().numpy(), np.load(f))


@pytest.mark.parametrize("m", [8, 16, 32])
def test_gpu_sort_full_size_vs_oracle(gpu, oracle, m):
    torch, codec, ctx = gpu
    a = datagen.skewed_codes(1_000_000, m, 256, seed=5, stay=0)
    a[::5] = a[7]                                   # one key repeated across every tile
    d = torch.from_numpy(a).cuda()
    tmp = torch.empty_like(d)
    codec.sort_rows(ctx, d, tmp)
    assert np.array_equal(d.cpu().numpy(), oracle.sort_rows(a))


@pytest.mark.parametrize("name", ["m8_n1000", "m16_n1000", "m8_n1", "m3_n2"])
def test_sort_ctx_mode_vs_reference_files(gpu, name):
    """Default reference mode: GPU sort, then the GPU histogram / codebooks / encode."""
    torch, codec, ctx = gpu
    g = golden(f"huff_{name}.npz")
    cd = torch.from_numpy(np.ascontiguousarray(g["input"])).cuda()
    codec.sort_rows(ctx, cd)
    assert np.array_equal(cd.cpu().numpy(), g["sort_ctx__decoded"].reshape(g["input"].shape))
    counts = codec.histogram(ctx, cd, 256, True)
    cbs = codec.Codebooks(codec.counts_to_host(counts), 256, True)
    assert cbs.file_bytes() == g["sort_ctx__codebooks"].tobytes()
    tabs = codec.Tables.from_codebooks(ctx, cbs)
    enc = codec.encode(ctx, tabs, cd, chunk_vectors=16)
    assert codec.indices_file_bytes(enc) == g["sort_ctx__indices"].tobytes()


def test_gpu_sort_key_words_and_local_sort(gpu, oracle):
    """The pieces of the multi-GPU sort mode that run on the GPU: sort_key_words on device
    tensors orders rows like the oracle, and sort_rows_distributed with the library sort
    (one rank) is the oracle's stable strncmp sort.  The multi-rank protocol itself is
    covered by the gloo tests (test_shard_gloo.py)."""
    torch, codec, ctx = gpu
    from pq_huffman_amd import shard
    for n, m in ((1000, 8), (777, 3), (513, 16)):
        a = _zero_heavy_rows(n, m, 3)
        w = shard.sort_key_words(torch.from_numpy(a).cuda()).cpu().numpy()
        np.testing.assert_array_equal(w, shard.sort_key_words(torch.from_numpy(a)).numpy())
        order = np.lexsort(tuple(w[:, j] for j in range(w.shape[1] - 1, -1, -1)))
        assert np.array_equal(a[order], oracle.sort_rows(a))
        out = shard.sort_rows_distributed(torch.from_numpy(a).cuda(), 1, 0,
                                          shard.library_sort(ctx))
        torch.cuda.synchronize()
        assert np.array_equal(out.cpu().numpy(), oracle.sort_rows(a))


def _long_codes(n, m, seed):
    """skewed codes with long constant runs: (0, 0) and (255, 255) pairs far above the
    multi-round form's 4,095 carry threshold in every chunk they cover"""
    codes = datagen.skewed_codes(n, m, seed=seed, stay=0)
    codes[300_000:500_000] = 0
    codes[900_000:1_030_000] = 255
    codes[1_500_000:1_500_000 + 61_440] = 7   # one whole chunk of one pair (61,440 counts)
    return codes


@pytest.mark.parametrize("m", [6, 8, 16])
def test_context_histogram_multi_round(gpu, oracle, m):
    """Past 4 groups' worth of chunks the context histogram counts several chunks per
    workgroup in one u16 image, moving counters above 4,095 into a u32 accumulator between
    chunks: its partials stay bounded by the grid (not by n).  4.2M rows (69 chunks: 5 to 9
    rounds) with long constant runs, wave form (m = 8, 16) and thread form (m = 6), one call
    and partial + reduce, set and accumulate, with a halo row."""
    torch, codec, ctx = gpu
    n = 4_200_001
    codes = _long_codes(n, m, 90 + m)
    cd = torch.from_numpy(np.ascontiguousarray(codes)).cuda()
    want = oracle.histogram(codes, 256, True)
    assert want.max() > 100_000
    got = codec.counts_to_host(codec.histogram(ctx, cd, 256, True))
    assert np.array_equal(got, want)
    # the bounded partial buffer: far below one image per chunk
    assert codec.histogram_partial_bytes(n, m, 256) < 69 * m * 32768 * 4 // 2
    parts = torch.empty(codec.histogram_partial_bytes(n, m, 256), dtype=torch.uint8, device="cuda")
    junk = torch.full((m, 65536), 777, dtype=torch.int32, device="cuda")
    for rep in range(2):   # the reduce clears the accumulator for the next launch
        codec.histogram_partial(ctx, cd, 256, parts)
        codec.histogram_reduce(ctx, parts, n, m, 256, junk)
        assert np.array_equal(codec.counts_to_host(junk), want), rep
    codec.histogram_partial(ctx, cd[1:], 256, parts, prev_row=cd[0])
    codec.histogram_reduce(ctx, parts, n - 1, m, 256, junk, accumulate=True)
    assert np.array_equal(codec.counts_to_host(junk), 2 * want)


@pytest.mark.parametrize("m,k,ctxm", [(8, 256, True), (16, 256, True), (8, 256, False),
                                      (6, 256, True), (8, 4096, False)])
def test_onepass_encoder_and_scratch_release(gpu, oracle, m, k, ctxm):
    """The one-pass look-back encoder (the fallback when the tiled encoder's scratch cannot be
    allocated; PQH_TUNE_ENC_IMPL = 2) writes the oracle's stream and chunk index, like the
    tiled default; pqh_ctx_release_scratch frees the scratch and the next encode allocates
    it again (huffman_encoder.c:207-238, bitstream.c:71-101)."""
    torch, codec, _ = gpu
    ctx = codec.Context(0)
    n = 300_007
    codes = datagen.skewed_codes(n, m, k=k, seed=140 + m, stay=0)
    if k > 256:
        cd = torch.from_numpy(codes.astype(np.uint16).view(np.int16)).cuda()
    else:
        cd = torch.from_numpy(np.ascontiguousarray(codes.astype(np.uint8))).cuda()
    tabs = codec.Tables(ctx, m, k, ctxm).build(codec.histogram(ctx, cd, k, ctxm))
    ocb = oracle.build_codebooks(codes, k, ctxm)
    want, bits = oracle.encode(codes, ocb)
    runs = {}
    for impl in (2, 1, 2):
        ctx.set_tuning(enc_impl=impl)
        enc = codec.encode(ctx, tabs, cd, chunk_vectors=4)
        assert enc.bits == bits, impl
        assert enc.stream[:len(want)].cpu().numpy().tobytes() == want, impl
        runs.setdefault(impl, enc.chunk_offsets.cpu().numpy())
        assert np.array_equal(runs[impl], enc.chunk_offsets.cpu().numpy())
        dec = codec.decode(ctx, tabs, enc)
        codec.decode_status(ctx)
        assert torch.equal(dec, cd), impl
        ctx.release_scratch()
    assert np.array_equal(runs[1], runs[2])


def test_fused_and_split_table_builds_alternate(gpu, oracle):
    """One table set rebuilt by the fused tree + decode-table launch (pqh_tables_build) and by
    the split pair (build_trees, build_luts) in turn, on two contexts: every build decodes the
    oracle's stream exactly, and its code tables and codebook file equal the oracle's (the two
    LUT pool heads alternate between builds; no memset dispatch in front of a build)
    (huffman_encode.c:141-192, huffman_decode.c:137-191)."""
    torch, codec, ctx = gpu
    ctx2 = codec.Context(0)
    m, k, n = 8, 256, 120_011
    codes = datagen.skewed_codes(n, m, k=k, seed=991, stay=0)
    cd = torch.from_numpy(np.ascontiguousarray(codes.astype(np.uint8))).cuda()
    counts = codec.histogram(ctx, cd, k, True)
    ocb = oracle.build_codebooks(codes, k, True)
    want, bits = oracle.encode(codes, ocb)
    tabs = codec.Tables(ctx, m, k, True)
    # ("luts": the decode tables rebuilt alone, after a fused build)
    for step, how in enumerate(["fused", "split", "split", "fused", "luts", "fused", "fused",
                                "luts", "split"]):
        c = ctx if step % 2 == 0 else ctx2
        if how == "fused":
            tabs.build(counts, c)
        elif how == "luts":
            tabs.build_luts(c)
        else:
            tabs.build_trees(counts, c).build_luts(c)
        torch.cuda.synchronize()
        tabs.status()
        enc = codec.encode(ctx, tabs, cd, chunk_vectors=4)
        assert enc.bits == bits, (step, how)
        assert enc.stream[:len(want)].cpu().numpy().tobytes() == want, (step, how)
        dec = codec.decode(ctx, tabs, enc)
        codec.decode_status(ctx)
        assert torch.equal(dec, cd), (step, how)
    assert tabs.codebooks(codec.counts_to_host(counts)).file_bytes() == oracle.codebooks_file(ocb)
    ctx2.close()
