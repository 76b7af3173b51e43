"""Stale-LDS hunt: every CU's LDS is filled with a poison pattern (pqh_debug_poison_lds)
right before the kernel under test, so any read of LDS that the kernel did not write first
shows up as a wrong result instead of reading zeros or an earlier workgroup's identical data.

Covers the kernels whose workgroups hand data through LDS: the row decoders (dec_rows: the
staged stream window with its zero pad, the staged rows), the any-shape decoder
(dec_chunks), the context histograms (u16-pair counters, multi-round carries) and the
one-pass encoder (the LDS bit image) and the row sort.  Each result must equal the unpoisoned run, which the
other test files pin to the oracle (huffman_decode.c:137-191, huffman_encoder.c:166-238)."""
import ctypes

import numpy as np
import pytest

import datagen

pytestmark = pytest.mark.gpu

POISON = (0xFFFFFFFF, 0xA5A5A5A5, 0x00000001)


@pytest.fixture(scope="module")
def gpu():
    import torch
    from pq_huffman_amd import codec
    assert torch.cuda.is_available()
    return torch, codec, codec.Context(0)


def _poison(codec, ctx, value):
    from pq_huffman_amd.capi import lib
    assert lib().pqh_debug_poison_lds(ctx.ptr, ctypes.c_uint(value)) == 0


def _encode(torch, codec, ctx, rows, tabs, chunk):
    n, m = rows.shape
    chunks = (n + chunk - 1) // chunk
    out = torch.zeros(n * m * 7 + 64, dtype=torch.uint8, device="cuda")
    coff = torch.empty(chunks, dtype=torch.int64, device="cuda")
    cprev = torch.empty((chunks, m), dtype=rows.dtype, device="cuda") if tabs.context else None
    tot = torch.zeros(1, dtype=torch.int64, device="cuda")
    codec.encode_write(ctx, tabs, rows, out, 0, 1, None, chunk, coff, cprev, total=tot)
    codec.encode_status(ctx)
    return codec.Encoded(out, int(tot.item()), chunk, coff, cprev, n, 1)


@pytest.mark.parametrize("m,k,ctxm,chunk", [(8, 256, True, 8), (8, 256, False, 8),
                                            (16, 256, True, 8), (8, 4096, False, 8),
                                            (8, 256, True, 32), (6, 256, True, 8)])
def test_decode_after_lds_poison(gpu, m, k, ctxm, chunk):
    """1M rows: dec_rows (8/16 u8 parts, 8 u16 parts, C = 8 and 32) and dec_chunks (m = 6)"""
    torch, codec, ctx = gpu
    n = 1_000_000
    codes = datagen.skewed_codes(n, m, k=k, seed=70 + m, stay=0)
    if k > 256:
        rows = torch.from_numpy(codes.astype(np.uint16).view(np.int16)).cuda()
    else:
        rows = torch.from_numpy(np.ascontiguousarray(codes.astype(np.uint8))).cuda()
    counts = codec.histogram(ctx, rows, k, ctxm)
    tabs = codec.Tables(ctx, m, k, ctxm).build(counts)
    enc = _encode(torch, codec, ctx, rows, tabs, chunk)
    for value in POISON:
        _poison(codec, ctx, value)
        dec = codec.decode(ctx, tabs, enc)
        codec.decode_status(ctx)
        assert torch.equal(dec, rows), hex(value)


@pytest.mark.parametrize("m,n", [(8, 1_000_000), (8, 4_200_001), (16, 1_000_003)])
def test_histograms_after_lds_poison(gpu, m, n):
    """context histograms (rows and part-major, one round and multi-round) and the plain one"""
    torch, codec, ctx = gpu
    codes = datagen.skewed_codes(n, m, seed=80 + m, stay=0)
    codes[1000:70_000] = 3
    rows = torch.from_numpy(np.ascontiguousarray(codes)).cuda()
    parts = rows.t().contiguous()
    want_ctx = codec.histogram(ctx, rows, 256, True)
    want_plain = codec.histogram(ctx, rows, 256, False)
    for value in POISON:
        _poison(codec, ctx, value)
        assert torch.equal(codec.histogram(ctx, rows, 256, True), want_ctx), hex(value)
        _poison(codec, ctx, value)
        assert torch.equal(codec.histogram_parts(ctx, parts, n, 256, True), want_ctx), hex(value)
        _poison(codec, ctx, value)
        hp = torch.empty(codec.histogram_partial_bytes(n, m, 256), dtype=torch.uint8, device="cuda")
        codec.histogram_partial_parts(ctx, parts, n, 256, hp)
        red = torch.empty((m, 65536), dtype=torch.int32, device="cuda")
        _poison(codec, ctx, value)
        codec.histogram_reduce(ctx, hp, n, m, 256, red)
        assert torch.equal(red, want_ctx), hex(value)
        _poison(codec, ctx, value)
        assert torch.equal(codec.histogram(ctx, rows, 256, False), want_plain), hex(value)


@pytest.mark.parametrize("m", [8, 16])
def test_encode_after_lds_poison(gpu, m):
    """the one-pass encoder's LDS bit image (zeroed per workgroup) and tails"""
    torch, codec, ctx = gpu
    n = 1_000_000
    codes = datagen.skewed_codes(n, m, seed=90 + m, stay=0)
    rows = torch.from_numpy(np.ascontiguousarray(codes)).cuda()
    tabs = codec.Tables(ctx, m, 256, True).build(codec.histogram(ctx, rows, 256, True))
    ref = _encode(torch, codec, ctx, rows, tabs, 8)
    nb = (ref.bits + 7) // 8
    for value in POISON:
        _poison(codec, ctx, value)
        got = _encode(torch, codec, ctx, rows, tabs, 8)
        assert got.bits == ref.bits
        assert torch.equal(got.stream[:nb], ref.stream[:nb]), hex(value)
        assert torch.equal(got.chunk_offsets, ref.chunk_offsets)


@pytest.mark.parametrize("m,n", [(8, 1_000_000), (16, 600_001), (12, 300_007), (3, 200_003)])
def test_sort_after_lds_poison(gpu, oracle, m, n):
    """the stable strncmp-key row sort (pqh_sort.hip: the per-chunk key histograms, the
    pass kernels' LDS digit counters and the next pass's counts) after every CU's LDS is
    poisoned: the rows equal the oracle's sort (huffman_encoder.c:301-317)"""
    torch, codec, ctx = gpu
    codes = datagen.skewed_codes(n, m, seed=100 + m, stay=0)
    codes[np.random.default_rng(m).random(codes.shape) < 0.25] = 0   # runs of equal keys
    want = oracle.sort_rows(codes)
    for value in POISON:
        rows = torch.from_numpy(np.ascontiguousarray(codes)).cuda()
        _poison(codec, ctx, value)
        codec.sort_rows(ctx, rows, torch.empty_like(rows))
        assert np.array_equal(rows.cpu().numpy(), want), hex(value)
