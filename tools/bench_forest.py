"""Forest-builder timing (tree mode's kNN graph + minimum spanning forest) on the bench's
SIFT-like rows, with the reference run.sh parameters by default (nn-fast: NUM_NN=50,
NUM_DIM=3, NUM_BLOCKS=10, OVERLAP=0.01; mst: NUM_NN_TAKE=5, no PQ penalty).

  python tools/bench_forest.py [--n 1000000] [--d 128] [--nn 50] [--splits 3] [--blocks 10]
                               [--overlap 0.01] [--take 5] [--reps 3] [--cpu-sample 20000]

Prints one JSON line: per-stage ms (blocks_info, knn_fast, mst), the kNN's algorithmic
rate (sum over blocks of S^2 d pair-dimensions, 3 fp32 ops each), block-size stats, and --
with --cpu-sample -- the oracle's time for the same pipeline on the first rows (one core
per block query loop, OpenMP threads as available), scaled per row."""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402
import bench  # noqa: E402
from pq_huffman_amd import codec, forest  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=1_000_000)
    ap.add_argument("--d", type=int, default=128)
    ap.add_argument("--nn", type=int, default=50)
    ap.add_argument("--splits", type=int, default=3)
    ap.add_argument("--blocks", type=int, default=10)
    ap.add_argument("--overlap", type=float, default=0.01)
    ap.add_argument("--take", type=int, default=5)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--cpu-sample", type=int, default=0)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    x = bench.make_data(torch, a.n, a.d, 1234, 0, dev)
    ctx = codec.Context(0)
    idx = torch.empty((a.n, a.nn), dtype=torch.int32, device=dev)
    dist = torch.empty((a.n, a.nn), dtype=torch.float32, device=dev)
    t = {"blocks_info": [], "knn_fast": [], "mst": []}
    for r in range(a.reps + 1):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        st, en = forest.blocks_info(ctx, x, a.splits, a.blocks, a.overlap)
        t1 = time.perf_counter()
        _, _, sizes = forest.knn_fast(ctx, x, a.nn, st, en, idx, dist)
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        tg, cn = forest.mst(ctx, idx, dist, a.take)
        t3 = time.perf_counter()
        if r:   # the first pass warms up
            t["blocks_info"].append((t1 - t0) * 1e3)
            t["knn_fast"].append((t2 - t1) * 1e3)
            t["mst"].append((t3 - t2) * 1e3)
    ms = {k: round(min(v), 3) for k, v in t.items()}
    pair_dims = float((sizes.astype(np.float64) ** 2).sum()) * a.d
    out = {"workload": f"forest builder: {a.n} x {a.d} SIFT-like fp32, nn={a.nn}, "
                       f"{a.splits} splits x {a.blocks} blocks, overlap {a.overlap}, take {a.take}",
           "ms": ms, "total_ms": round(sum(ms.values()), 3),
           "rows_per_s_M": round(a.n / (sum(ms.values()) * 1e-3) / 1e6, 3),
           "knn_pair_dims": pair_dims,
           "knn_fp32_tflops_algorithmic": round(3 * pair_dims / (ms["knn_fast"] * 1e-3) / 1e12, 2),
           "blocks": int(len(sizes)), "block_rows_min_median_max":
               [int(sizes.min()), int(np.median(sizes)), int(sizes.max())],
           "pairs": int(sizes.sum()), "forest_edges": int(len(tg)),
           "roots": int(a.n - len(tg) // 2),
           "unfilled": int((idx == -1).sum().item())}
    if a.cpu_sample:
        from oracle import oracle_ctypes as oc
        xs = x[:a.cpu_sample].cpu().numpy()
        c0 = time.perf_counter()
        ost, oen = oc.knn_blocks_info(xs, a.splits, a.blocks, a.overlap)
        oi, od, _ = oc.knn_fast(xs, a.nn, ost, oen)
        if not (oi == 0xFFFFFFFF).any():
            oc.mst(oi, od, a.take)
        c1 = time.perf_counter()
        out["cpu_baseline"] = {"kind": "port", "rows": a.cpu_sample, "ms": round((c1 - c0) * 1e3, 1),
                               "threads": int(os.environ.get("OMP_NUM_THREADS", os.cpu_count())),
                               "note": "oracle pipeline on the first rows (block sizes scale "
                                       "with n, so per-row cost grows with n)"}
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
