"""Multi-rank protocol of the encode path (pq_huffman_amd/shard.py) on CPU:
world_size 2 and 3 over gloo.  Each rank takes its row shard (pqh_shard_block), exchanges
the one-vector halo (the ragged halo's source: pqh_shard_halo_source), all-reduces its
histogram, builds the (oracle) code tables from the global counts, encodes its shard at the
all-gathered bit offset (pqh_shard_offsets), and rank 0 stitches the shard buffers
(pqh_shard_stitch).  The stitched stream and the reduced histogram must equal the oracle's
single-process results bit for bit.  The library's host half of the protocol runs here;
the per-shard bit packer is test code standing in for the GPU encoder, which needs a GPU
(its two-rank run of the whole library protocol, pqh_shard_encode, is test_gpu_zz_shard.py)."""
import os

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from oracle import oracle_ctypes as orc
from pq_huffman_amd import shard
from tests.datagen import skewed_codes


def _init(rank, world, store_file):
    """Rendezvous through a FileStore in the test's tmp_path: no TCP port is picked, released
    and bound again later (the race a free-port probe leaves open)."""
    dist.init_process_group("gloo", init_method=f"file://{store_file}", rank=rank,
                            world_size=world)


def _pack(codes, cbs, raw_first, prev_row, bit_off):
    """Reference bit order (huffman_encoder.c:207-238): vector-major, part-minor, MSB first."""
    n, m = codes.shape
    bits = []
    for v in range(n):
        for i in range(m):
            cur = int(codes[v, i])
            if cbs.context:
                if v == 0 and raw_first:
                    bits.extend((cur >> (7 - b)) & 1 for b in range(8))
                    continue
                prev = int(codes[v - 1, i]) if v > 0 else int(prev_row[i])
                item = prev * cbs.k + cur
            else:
                item = cur
            L = int(cbs.lens[i, item])
            cb = cbs.codes[i, item]
            bits.extend((int(cb[b // 8]) >> (7 - b % 8)) & 1 for b in range(L))
    total = bit_off + len(bits)
    buf = np.zeros((total + 31) // 32 * 4, np.uint8)
    for j, b in enumerate(bits):
        if b:
            p = bit_off + j
            buf[p // 8] |= 1 << (7 - p % 8)
    return buf.tobytes(), len(bits)


def _local_hist(codes, k, context, prev_row):
    m = codes.shape[1]
    per = k * k if context else k
    h = np.zeros((m, per), np.int64)
    for v in range(codes.shape[0]):
        for i in range(m):
            cur = int(codes[v, i])
            if context:
                if v == 0:
                    if prev_row is None:
                        continue
                    prev = int(prev_row[i])
                else:
                    prev = int(codes[v - 1, i])
                h[i, prev * k + cur] += 1
            else:
                h[i, cur] += 1
    return h


def _worker(rank, world, store_file, n, m, k, context, q):
    _init(rank, world, store_file)
    try:
        codes = skewed_codes(n, m, k, seed=11)
        b, e = shard.row_range(n, world, rank)
        mine = codes[b:e]
        halo = shard.exchange_halo(torch.from_numpy(mine[-1].astype(np.int64)), world, rank)
        prev = halo.numpy() if (context and halo is not None) else None
        counts = torch.from_numpy(_local_hist(mine, k, context, prev))
        shard.reduce_counts(counts, world)
        cnt = counts.numpy().astype(np.float64)
        items = k * k if context else k
        lens = np.zeros((m, items), np.int32)
        cds = np.zeros((m, items, 8), np.uint8)
        for i in range(m):
            lens[i], cds[i] = orc.codebook(k, cnt[i], context, 8)
        cbs = orc.Codebooks(k, context, lens, cds, 8)
        # exact bit length first (the size pass), then place the shard
        _, nbits = _pack(mine, cbs, shard.raw_first(rank), prev, 0)
        goff, total = shard.bit_offsets(torch.tensor([nbits], dtype=torch.int64), world, rank)
        # the host-sync-free form the GPU bench feeds to pqh_encode_write_at
        goff_d, total_d = shard.bit_offsets_device(torch.tensor([nbits], dtype=torch.int64),
                                                   world, rank)
        assert (int(goff_d.item()), int(total_d.item())) == (goff, total)
        buf, nb2 = _pack(mine, cbs, shard.raw_first(rank), prev, shard.local_bit_offset(goff))
        assert nb2 == nbits
        pieces = [None] * world
        dist.all_gather_object(pieces, (buf, goff, nbits))
        if rank == 0:
            q.put((shard.stitch(pieces, total), cnt))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,context", [(2, True), (2, False), (3, True)])
def test_sharded_encode_matches_single_process(world, context, tmp_path):
    n, m, k = 301, 4, 256
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    store_file = tmp_path / "store"
    procs = [ctx.Process(target=_worker, args=(r, world, str(store_file), n, m, k, context, q))
             for r in range(world)]
    for p in procs:
        p.start()
    stream, counts = q.get(timeout=120)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    codes = skewed_codes(n, m, k, seed=11)
    np.testing.assert_array_equal(counts, orc.histogram(codes, k, context))
    cbs = orc.build_codebooks(codes, k, context)
    ref, bits = orc.encode(codes, cbs)
    assert stream == ref


def test_row_range_partitions():
    for n in (0, 1, 7, 100, 1001):
        for world in (1, 2, 3, 8):
            rs = [shard.row_range(n, world, r) for r in range(world)]
            assert rs[0][0] == 0 and rs[-1][1] == n
            assert all(rs[i][1] == rs[i + 1][0] for i in range(world - 1))
            sizes = [e - b for b, e in rs]
            assert max(sizes) - min(sizes) <= 1


def test_stitch_word_alignment():
    # two shards: 13 bits then 40 bits; second starts at global bit 13 -> local offset 13
    a = np.zeros(4, np.uint8); a[0] = 0b10110011; a[1] = 0b11111000
    b_bits = [1, 0] * 20
    b = np.zeros(8, np.uint8)
    for j, bit in enumerate(b_bits):
        p = 13 + j
        if bit:
            b[p // 8] |= 1 << (7 - p % 8)
    out = shard.stitch([(a.tobytes(), 0, 13), (b.tobytes(), 13, 40)], 53)
    ref_bits = [1, 0, 1, 1, 0, 0, 1, 1, 1, 1, 1, 1, 1] + b_bits
    ref = np.zeros(7, np.uint8)
    for j, bit in enumerate(ref_bits):
        if bit:
            ref[j // 8] |= 1 << (7 - j % 8)
    assert out == ref.tobytes()


# ---- sort mode across ranks: sample sort + ragged halo (shard.sort_rows_distributed) -----

def _sort_codes(kind, n, m, k):
    codes = skewed_codes(n, m, k, seed=5)
    if kind == "zeros":      # many 0 bytes: long runs of equal strncmp keys, ties everywhere
        rng = np.random.default_rng(6)
        codes[rng.random(codes.shape) < 0.3] = 0
    elif kind == "onekey":   # every row starts with 0: one key, all rows land on one rank
        codes[:, 0] = 0
    return codes


def _local_sort(t):
    return torch.from_numpy(orc.sort_rows(t.numpy())) if t.shape[0] else t


def _sort_worker(rank, world, store_file, kind, n, m, k, q):
    _init(rank, world, store_file)
    try:
        codes = _sort_codes(kind, n, m, k)
        b, e = shard.row_range(n, world, rank)
        mine = shard.sort_rows_distributed(torch.from_numpy(codes[b:e]), world, rank,
                                           _local_sort, samples=16).numpy()
        # the context-mode encode protocol on the (possibly empty) sorted slices
        last = torch.from_numpy(mine[-1].copy()) if len(mine) else None
        halo, raw = shard.halo_ragged(last, world, rank)
        # the halo keeps the codes' dtype: the library reads prev_row as m code bytes
        assert halo is None or (halo.dtype == torch.uint8 and halo.shape == (m,))
        prev = halo.numpy() if halo is not None else None
        counts = torch.from_numpy(_local_hist(mine, k, True, prev))
        shard.reduce_counts(counts, world)
        cnt = counts.numpy().astype(np.float64)
        lens = np.zeros((m, k * k), np.int32)
        cds = np.zeros((m, k * k, 8), np.uint8)
        for i in range(m):
            lens[i], cds[i] = orc.codebook(k, cnt[i], True, 8)
        cbs = orc.Codebooks(k, True, lens, cds, 8)
        _, nbits = _pack(mine, cbs, raw, prev, 0)
        goff, total = shard.bit_offsets(torch.tensor([nbits], dtype=torch.int64), world, rank)
        buf, _ = _pack(mine, cbs, raw, prev, shard.local_bit_offset(goff))
        pieces = [None] * world
        dist.all_gather_object(pieces, (buf, goff, nbits))
        slices = [None] * world
        dist.all_gather_object(slices, mine)
        if rank == 0:
            q.put((np.concatenate(slices), shard.stitch(pieces, total), [len(s) for s in slices]))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,kind,m", [(2, "skewed", 8), (3, "zeros", 8), (3, "zeros", 16),
                                          (2, "onekey", 4), (3, "skewed", 3)])
def test_distributed_sort_mode_matches_single_process(world, kind, m, tmp_path):
    """Sample sort across gloo ranks, then the sort+context encode on the sorted slices:
    the concatenated slices equal the oracle's stable strncmp-key sort of all rows, and the
    stitched stream equals the oracle's single-process sort+context stream
    (huffman_encoder.c:301-317, :220-238)."""
    n, k = 400, 256
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    store_file = tmp_path / "store"
    procs = [ctx.Process(target=_sort_worker, args=(r, world, str(store_file), kind, n, m, k, q))
             for r in range(world)]
    for p in procs:
        p.start()
    rows, stream, sizes = q.get(timeout=120)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    want = orc.sort_rows(_sort_codes(kind, n, m, k))
    np.testing.assert_array_equal(rows, want)
    assert sum(sizes) == n
    if kind == "onekey":
        assert sorted(sizes)[:-1] == [0] * (world - 1)    # the empty-slice path ran
    cbs = orc.build_codebooks(want, k, True)
    ref, _ = orc.encode(want, cbs)
    assert stream == ref


def test_sort_key_words_order():
    """sort_key_words orders rows like the stable strncmp comparator of the oracle."""
    for m in (3, 8, 12):
        codes = _sort_codes("zeros", 500, m, 256)
        w = shard.sort_key_words(torch.from_numpy(codes)).numpy()
        order = np.lexsort(tuple(w[:, j] for j in range(w.shape[1] - 1, -1, -1)), axis=0)
        np.testing.assert_array_equal(codes[order], orc.sort_rows(codes))
