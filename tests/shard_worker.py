"""One rank of the library's sharded encode (pqh_shard_encode through shard.shard_encode),
run by tests/test_gpu_zz_shard.py under torch.distributed.run with the gloo backend and every
rank on cuda:0 (a fresh process per rank).  Writes rank 0's result to --out (.npz):
the stitched stream (pqh_shard_stitch of every rank's buffer), the global histogram, and
the rows the ranks encoded, for the test to compare with the oracle's one-shot results.

  --case even|ragged|sort|fail|parts|parts_ragged   --mode ctx|noctx
even: contiguous shards; ragged: rank 1 holds no rows; fail: rank 1's call fails locally
(an output buffer too small) -- both ranks must return, rank 1 with its error and rank 0
through pqh_shard_status; sort: the distributed sample sort
(shard.sort_rows_distributed with the library's stable radix sort) then the sorted slices,
whose halo also goes through shard.halo_ragged into codec.histogram / encode_size (the
library's halo must agree); parts / parts_ragged: the two-phase calls on part-major codes
(pqh_shard_encode_tables_parts with the partial pair counts, pqh_shard_encode_write_parts),
and each shard decoded through its own chunk index."""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

import numpy as np  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--case", default="even")
    ap.add_argument("--mode", default="ctx")
    ap.add_argument("--n", type=int, default=20011)
    ap.add_argument("--out", required=True)
    a = ap.parse_args()
    import torch
    import torch.distributed as dist
    import datagen
    from pq_huffman_amd import codec, shard

    dist.init_process_group("gloo")
    world, rank = dist.get_world_size(), dist.get_rank()
    torch.cuda.set_device(0)
    ctxm = a.mode == "ctx"
    m, k = 8, 256
    allc = datagen.skewed_codes(a.n, m, k, seed=77)
    if a.case == "sort":
        allc[np.random.default_rng(3).random(allc.shape) < 0.2] = 0   # strncmp-key ties
    ctx = codec.Context(0)
    if a.case in ("ragged", "parts_ragged"):
        b, e = (0, a.n) if rank == 0 else (a.n, a.n)
    else:
        b, e = shard.row_range(a.n, world, rank)
    mine = torch.from_numpy(np.ascontiguousarray(allc[b:e])).cuda()
    if a.case == "sort":
        mine = shard.sort_rows_distributed(mine, world, rank, shard.library_sort(ctx))
    n = mine.shape[0]
    items = k * k if ctxm else k
    counts = torch.zeros((m, items), dtype=torch.int32, device="cuda")
    tabs = codec.Tables(ctx, m, k, ctxm)
    out = torch.zeros(n * m * 7 + 64, dtype=torch.uint8, device="cuda")
    comm = shard.TorchComm(world, rank)
    if a.case == "fail":
        from pq_huffman_amd.capi import PqhError
        bad = out[:2] if rank == 1 else out            # rank 1: out_bytes < 4 (local failure)
        try:
            offsets, _ = shard.shard_encode(ctx, comm, mine, tabs, counts, bad, first_row=b,
                                            raw_first=False)
            assert rank != 1, "rank 1's bad buffer was accepted"
            try:
                shard.status(ctx, offsets)
                raise AssertionError("rank 0 did not see rank 1's failure")
            except PqhError as e:
                assert "another rank" in str(e), str(e)
        except PqhError as e:
            assert rank == 1 and "invalid argument" in str(e), str(e)
        dist.barrier()
        if rank == 0:
            np.savez(a.out, failed=np.int64(1))
        tabs.close()
        ctx.close()
        dist.destroy_process_group()
        return
    if a.case.startswith("parts"):
        # the two phases on PART-MAJOR codes (bench.py's multi-rank pipeline): context mode
        # hands phase 1 the partial pair counts taken without the halo (as the assignment
        # stream does), non-context lets phase 1 run the part-major histogram itself
        ld = (n + 127) // 128 * 128 + 64
        pm = torch.full((m, max(ld, 1)), 0xA5, dtype=torch.uint8, device="cuda")
        pm[:, :n] = mine.t()
        pm = pm[:, :n]
        hp = None
        if ctxm:
            hp = torch.empty(max(codec.histogram_partial_bytes(n, m, k), 4), dtype=torch.uint8,
                             device="cuda")
            if n:
                codec.histogram_partial_parts(ctx, pm, n, k, hp)
        scratch = shard.scratch_for(comm, m, torch.device("cuda", 0))
        st = shard.shard_encode_tables(ctx, comm, pm, tabs, counts, scratch, first_row=b,
                                       parts_n=n, partials=hp)
        assert st == 0, st
        chunks = (n + 7) // 8
        coff = torch.empty(max(chunks, 1), dtype=torch.int64, device="cuda")
        cprev = torch.empty((max(chunks, 1), m), dtype=torch.uint8, device="cuda") if ctxm else None
        offsets = torch.zeros(2, dtype=torch.int64, device="cuda")
        shard.shard_encode_write(ctx, comm, pm, tabs, out, 8, coff, cprev, offsets, scratch,
                                 status=st, first_row=b, parts_n=n)
        shard.status(ctx, offsets)
        raw = 1 if b == 0 else 0
        if n:   # the shard's own decode through its chunk index (halo row as chunk 0's context)
            enc = codec.Encoded(out, -1, 8, coff, cprev, n, raw)
            dec = codec.decode(ctx, tabs, enc)
            codec.decode_status(ctx)
            assert torch.equal(dec, mine), "part-major shard does not decode to its rows"
    else:
        offsets, raw = shard.shard_encode(ctx, comm, mine, tabs, counts, out, first_row=b,
                                          check=True)
    torch.cuda.synchronize()
    goff, total = (int(v) for v in offsets.cpu().tolist())
    # every rank's length, for the stitch on rank 0
    lens = [None] * world
    dist.all_gather_object(lens, (goff, total))
    nxt = [g for g, _ in lens] + [total]
    bits = nxt[rank + 1] - goff
    if a.case == "sort" and ctxm:
        # the ragged halo through the Python protocol: device tensors in the codes' dtype,
        # fed to the library's histogram and size -- must match what shard_encode did
        halo, raw2 = shard.halo_ragged(mine[-1] if n else None, world, rank,
                                       device=torch.device("cuda", 0))
        assert raw2 == raw, (raw2, raw)
        assert halo is None or (halo.dtype == torch.uint8 and halo.is_cuda)
        c2 = codec.histogram(ctx, mine, k, True, prev_row=halo)
        shard.reduce_counts(c2, world)
        assert torch.equal(c2, counts), "halo_ragged histogram != pqh_shard_encode's"
        t2 = codec.encode_size(ctx, tabs, mine, raw, halo)
        assert int(t2.item()) == bits, (int(t2.item()), bits)
    nb = (goff % 32 + bits + 7) // 8 + 4
    parts = [None] * world
    dist.all_gather_object(parts, (out[:nb].cpu().numpy().tobytes(), goff, bits,
                                   mine.cpu().numpy()))
    if rank == 0:
        stream = shard.stitch([(p[0], p[1], p[2]) for p in parts], total)
        np.savez(a.out, stream=np.frombuffer(stream, np.uint8), total=np.int64(total),
                 counts=counts.cpu().numpy(), rows=np.concatenate([p[3] for p in parts]))
    dist.barrier()
    tabs.close()
    ctx.close()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
