"""Part-major codes (pqh_pq_assign_parts and its consumers): the assignment stores each
subspace's codes contiguously, so every store is a whole line from one wave (row-major
pq_indices.bvecsl order, src/pq_encoder.c:192-213, interleaves the 8 subspaces' bytes and
their workgroups write each line 8 times).  Every consumer of the layout must give the
row-major path's results bit for bit: the codes themselves (oracle-checked through the row
path), the histograms (huffman_encoder.c:139-205), the stream and chunk index
(huffman_encoder.c:207-238)."""
import numpy as np
import pytest

import datagen

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def gpu():
    import torch
    from pq_huffman_amd import codec
    assert torch.cuda.is_available()
    return torch, codec, codec.Context(0)


def _parts_of(torch, rows, pad=0):
    """rows (n, m) -> a part-major (m, n + pad) buffer holding them (padding garbage)"""
    n, m = rows.shape
    p = torch.full((m, n + pad), 0xA5, dtype=rows.dtype, device=rows.device)
    p[:, :n] = rows.t()
    return p


@pytest.mark.parametrize("kind,d,m,k", [("sift", 128, 8, 256), ("deep", 96, 16, 256),
                                        ("sift", 128, 8, 4096)])
def test_assign_parts_equals_rows(gpu, oracle, kind, d, m, k):
    torch, codec, ctx = gpu
    n = 50_001
    x = datagen.sift_like(n, d, seed=3) if kind == "sift" else datagen.deep_like(n, d, seed=4)
    cent = datagen.lloyd_centroids(x, m, 256, iters=1, sample=4000) if k == 256 else \
        np.ascontiguousarray(x[np.random.default_rng(2).choice(n, k, replace=False)]
                             .reshape(k, m, d // m).transpose(1, 0, 2) + 0.25, np.float32)
    pq = codec.PQ(ctx, cent)
    xd = torch.from_numpy(x).cuda()
    rows = pq.assign(xd)
    for pad, mode in ((0, 0), (77, 0), (3, 1)):
        parts = torch.full((m, n + pad), 0x5A, dtype=rows.dtype, device="cuda")
        pq.assign_parts(xd, parts, mode=mode)
        assert torch.equal(parts[:, :n].t(), rows), (pad, mode)
        assert (parts[:, n:] == 0x5A).all()           # nothing past n written
        assert torch.equal(codec.transpose_codes(ctx, parts, n), rows)
    if k == 256:   # the fused non-context histogram works for either layout
        c1 = torch.zeros((m, k), dtype=torch.int32, device="cuda")
        c2 = torch.zeros((m, k), dtype=torch.int32, device="cuda")
        pq.assign(xd, counts=c1)
        pq.assign_parts(xd, counts=c2)
        assert torch.equal(c1, c2)
    want, _ = oracle.pq_assign(x, cent, threads=0)
    got = rows.cpu().numpy()
    assert np.array_equal(got.view(np.uint16) if k > 256 else got, want)


@pytest.mark.parametrize("m,n", [(8, 130_001), (16, 70_001), (6, 61_441), (8, 4_200_001)])
def test_histogram_parts_equals_rows(gpu, m, n):
    """context (wave form on part runs, aligned and ragged ranges, multi-round at 4.2M rows)
    and plain histograms, with and without the halo row, one call and partial + reduce"""
    torch, codec, ctx = gpu
    codes = datagen.skewed_codes(n, m, seed=40 + m, stay=0)
    codes[1000:70_000] = 3                               # long runs: carries in the rounds form
    rows = torch.from_numpy(np.ascontiguousarray(codes)).cuda()
    for pad in (0, 5):
        parts = _parts_of(torch, rows, pad)
        for ctxm in (True, False):
            want = codec.histogram(ctx, rows, 256, ctxm)
            got = codec.histogram_parts(ctx, parts, n, 256, ctxm)
            assert torch.equal(got, want), (pad, ctxm)
        halo = rows[7].clone()
        want = codec.histogram(ctx, rows[8:], 256, True, prev_row=halo)
        got = codec.histogram_parts(ctx, parts[:, 8:], n - 8, 256, True, prev_row=halo)
        assert torch.equal(got, want)
        hp = torch.empty(codec.histogram_partial_bytes(n, m, 256), dtype=torch.uint8, device="cuda")
        codec.histogram_partial_parts(ctx, parts, n, 256, hp)
        red = torch.empty((m, 65536), dtype=torch.int32, device="cuda")
        codec.histogram_reduce(ctx, hp, n, m, 256, red)
        assert torch.equal(red, codec.histogram(ctx, rows, 256, True))


@pytest.mark.parametrize("m,ctxm", [(8, True), (8, False), (16, True), (16, False)])
def test_encode_parts_equals_rows(gpu, m, ctxm):
    """the row encoder reading part runs: the same stream bytes, bit count, chunk offsets
    and chunk context rows as the row-major encoder; halo row and raw first row"""
    torch, codec, ctx = gpu
    n = 100_003
    codes = datagen.skewed_codes(n, m, seed=60 + m, stay=0)
    rows = torch.from_numpy(np.ascontiguousarray(codes)).cuda()
    counts = codec.histogram(ctx, rows, 256, ctxm)
    tabs = codec.Tables(ctx, m, 256, ctxm).build(counts)
    parts = _parts_of(torch, rows, 9)
    chunk = 8
    nch = (n + chunk - 1) // chunk
    for raw_first, halo in ((1, None), (0, rows[5].clone())):
        outs = []
        for part_major in (False, True):
            out = torch.zeros(n * m * 7 + 64, dtype=torch.uint8, device="cuda")
            coff = torch.zeros(nch, dtype=torch.int64, device="cuda")
            cprev = torch.zeros((nch, m), dtype=torch.uint8, device="cuda") if ctxm else None
            tot = torch.zeros(1, dtype=torch.int64, device="cuda")
            if part_major:
                codec.encode_write_parts(ctx, tabs, parts, n, out, 0, raw_first, halo, chunk, coff,
                                         cprev, total=tot)
            else:
                codec.encode_write(ctx, tabs, rows, out, 0, raw_first, halo, chunk, coff, cprev,
                                   total=tot)
            codec.encode_status(ctx)
            outs.append((out, coff, cprev, int(tot.item())))
        (o0, c0, p0, t0), (o1, c1, p1, t1) = outs
        assert t0 == t1 and t0 > 0
        assert torch.equal(o0[:(t0 + 7) // 8], o1[:(t1 + 7) // 8])
        assert torch.equal(c0, c1)
        if ctxm:
            assert torch.equal(p0, p1)
