"""BASELINE.json configs[3] and configs[4] end to end on the GPU, checked against the oracle.

configs[3]: Deep1B-style 96-d fp32, M = 16, K = 256 (dsub = 6: the MFMA assignment's
            one-pass plan), order-1 context Huffman with GPU-built code tables.
configs[4]: M = 8, K = 4096 (12-bit codes, u16): the MFMA assignment with centroid tiles
            streamed from L2, non-context Huffman with GPU-built code tables over a
            4,096-symbol alphabet.

Each: GPU assignment == oracle codes (bit-exact), GPU histogram == oracle histogram,
GPU code tables == the oracle's codebooks (file bytes), encode == the oracle's stream,
decode == the codes.  The sizes keep the oracle's share of the run to seconds."""
import numpy as np
import pytest

import datagen

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def gpu():
    import torch
    from pq_huffman_amd import codec
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch, codec, codec.Context(0)


def _roundtrip(gpu, oracle, x, cent, k, ctxm, chunk):
    torch, codec, ctx = gpu
    n, m = x.shape[0], cent.shape[0]
    pq = codec.PQ(ctx, cent)
    codes = pq.assign(torch.from_numpy(x).cuda())
    hc = codes.cpu().numpy()
    want, _ = oracle.pq_assign(x, cent, threads=0)
    assert np.array_equal(hc, want), "assignment != oracle"
    counts = codec.histogram(ctx, codes, k, ctxm)
    assert np.array_equal(codec.counts_to_host(counts), oracle.histogram(want, k, ctxm))
    tabs = codec.Tables(ctx, m, k, ctxm).build(counts)          # GPU trees
    tabs.status()
    ocb = oracle.build_codebooks(want, k, ctxm)
    assert tabs.codebooks(codec.counts_to_host(counts)).file_bytes() == \
        oracle.codebooks_file(ocb), "GPU code tables != oracle codebooks"
    enc = codec.encode(ctx, tabs, codes, chunk_vectors=chunk)
    codec.encode_status(ctx)
    stream, bits = oracle.encode(want, ocb)
    assert enc.bits == bits
    assert enc.stream[:len(stream)].cpu().numpy().tobytes() == stream
    dec = codec.decode(ctx, tabs, enc)
    codec.decode_status(ctx)
    assert torch.equal(dec, codes)
    return pq.rerank_count()


def test_config_deep96_m16_context(gpu, oracle):
    n = 100_000
    x = datagen.deep_like(n, 96, seed=31)
    cent = datagen.lloyd_centroids(x, 16, 256, iters=2, sample=20000)
    _roundtrip(gpu, oracle, x, cent, 256, True, 8)


def test_config_m8_k4096_noncontext(gpu, oracle):
    n = 6000
    x = datagen.sift_like(n, 128, seed=32)
    rng = np.random.default_rng(33)
    # 4,096 centroids per subspace: distinct data rows plus small offsets (no training)
    rows = x[rng.choice(n, 4096, replace=False)].reshape(4096, 8, 16).transpose(1, 0, 2)
    cent = np.ascontiguousarray(rows + rng.normal(0, 0.5, rows.shape)).astype(np.float32)
    assert _roundtrip(gpu, oracle, x, cent, 4096, False, 16) > 0   # the screening ran
