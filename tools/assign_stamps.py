"""Per-wave timeline of pq_assign_mfma (diagnostic; needs a PQH_ASSIGN_STAMPS build, see
tools/build_variants.sh): start/end spread, lifetime and blocks per wave, per XCD."""
import ctypes
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402
import bench  # noqa: E402
from pq_huffman_amd import codec  # noqa: E402
from pq_huffman_amd.capi import lib  # noqa: E402


def main():
    dev = torch.device("cuda", 0)
    n, d, m, k = int(os.environ.get("BENCH_ASSIGN_N", 1_000_000)), 128, 8, 256
    x = bench.make_data(torch, n, d, 1234, 0, dev)
    cent = bench.train_centroids(torch, x, m, k)
    ctx = codec.Context(0)
    pq = codec.PQ(ctx, cent)
    codes = torch.empty((n, m), dtype=torch.uint8, device=dev)
    for _ in range(5):
        pq.assign(x, codes)
    torch.cuda.synchronize()
    W = 8192
    buf = (ctypes.c_ulonglong * (W * 4))()
    lib().pqh_debug_assign_stamps(ctx.ptr, buf, W)
    a = np.frombuffer(buf, dtype=np.uint64).reshape(W, 4).astype(np.int64)
    rbuf = (ctypes.c_ulonglong * (W * 4))()
    lib().pqh_debug_assign_rr(ctx.ptr, rbuf, W)
    rr = np.frombuffer(rbuf, dtype=np.uint64).reshape(W, 4).astype(np.int64)
    idx = np.nonzero(a[:, 1] > 0)[0]
    rr = rr[a[:, 1] > 0]
    a = a[a[:, 1] > 0]
    wps = int(os.environ.get("STAMPS_WAVES_PER_SUBSPACE", 384))   # gx * 4 (gx = 96 on 256 CUs)
    sub = idx // wps
    t0 = a[:, 0].min()
    st, en, nb, xcc = a[:, 0] - t0, a[:, 1] - t0, a[:, 2] & 0xFFFF, a[:, 3] & 15
    loop_end = st + ((a[:, 3] >> 8) & 0xFFFFFF)   # the chunk loop's end (the tail after it)
    rr_t, rr_n = (a[:, 3] >> 32) & 0xFFFFFF, (a[:, 3] >> 56) & 0xFF   # re-rank batches
    tail = en - loop_end
    cyc = a[:, 2] >> 16          # s_memtime lifetime (shader clock)
    life = en - st               # s_memrealtime: 100 MHz ticks, comparable across CUs
    print(f"waves {len(a)}  span {en.max()} ticks of 10 ns")
    for name, v in (("start", st), ("end", en), ("loopend", loop_end), ("tail", tail), ("rr_ticks", rr_t), ("rr_batch", rr_n),
                    ("rr_per_batch", rr_t // np.maximum(rr_n, 1)),
                    ("life", life), ("blocks", nb), ("cycles", cyc)):
        q = np.percentile(v, [0, 5, 25, 50, 75, 95, 100]).astype(int)
        print(f"{name:7s} p0/5/25/50/75/95/100: {list(q)}")
    for c in range(8):
        sel = xcc == c
        if sel.any():
            print(f"xcc {c}: waves {sel.sum()} blocks {nb[sel].sum()} start p50/max {int(np.median(st[sel]))}/"
                  f"{st[sel].max()} end p5/p50/max {int(np.percentile(en[sel], 5))}/{int(np.median(en[sel]))}/"
                  f"{en[sel].max()}")
    nbat = np.maximum((a[:, 3] >> 56) & 0xFF, 1)
    for name, v in (("rr_x/batch", rr[:, 0] // nbat), ("rr_screen/batch", rr[:, 1] // nbat),
                    ("rr_cand/batch", rr[:, 2] // nbat), ("rr_rounds/batch", rr[:, 3] / nbat)):
        q = np.percentile(v, [0, 5, 25, 50, 75, 95, 100]).round(1)
        print(f"{name:16s} p0/5/25/50/75/95/100: {list(q)}")
    for c in range(m):
        sel = sub == c
        if sel.any():
            print(f"subspace {c}: waves {sel.sum()} blocks {nb[sel].sum()} loopend p50/max "
                  f"{int(np.median(loop_end[sel]))}/{loop_end[sel].max()} end p50/p95/max "
                  f"{int(np.median(en[sel]))}/{int(np.percentile(en[sel], 95))}/{en[sel].max()} "
                  f"rr_batches {rr_n[sel].sum()}")
    print("clock GHz (cycles / life):", round(float(np.median(cyc / np.maximum(life, 1))) / 10, 3))
    print("ticks per block (median life/blocks):", int(np.median(life / np.maximum(nb, 1))))


if __name__ == "__main__":
    main()
