"""Tree-mode timing (huffman_encoder/huffman_decoder --tree) at SIFT1M shape: 1M rows, M=8,
K=256, on one GPU.  Prints one JSON line: wall-clock ms per tree_encode / tree_decode call
(DFS order + traverser included, inputs resident in HBM), the host walk alone and the
device order (pqh_tree_order_device, forest already in HBM) alone; run under
`rocprofv3 --kernel-trace --stats` for the per-kernel device times.  Synthetic skewed codes
and a seeded random forest in the mst.tree layout (tests/datagen.py)."""
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import datagen  # noqa: E402
from pq_huffman_amd import codec  # noqa: E402


def main():
    n, m, reps = int(os.environ.get("N", 1_000_000)), 8, 5
    codes = datagen.skewed_codes(n, m, 256, seed=3)
    targets, counts = datagen.random_forest(n, roots=100, seed=3)
    ctx = codec.Context(0)
    d = torch.from_numpy(codes).cuda()
    enc = codec.tree_encode(ctx, d, targets, counts)       # warm-up
    dec = codec.tree_decode(ctx, enc)
    assert torch.equal(dec.cpu(), torch.from_numpy(codes[enc.vertices]))
    t0 = time.perf_counter()
    for _ in range(reps):
        codec.tree_order(targets, counts)
    host_ms = (time.perf_counter() - t0) / reps * 1e3
    dt, dc = torch.from_numpy(targets.view(np.int32)).cuda(), torch.from_numpy(counts).cuda()
    codec.tree_order_device(ctx, dt, dc)
    ctx.sync()
    t0 = time.perf_counter()
    for _ in range(reps):
        codec.tree_order_device(ctx, dt, dc)
    ctx.sync()
    dev_order_ms = (time.perf_counter() - t0) / reps * 1e3
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        enc = codec.tree_encode(ctx, d, targets, counts)
    ctx.sync()
    enc_ms = (time.perf_counter() - t0) / reps * 1e3
    t0 = time.perf_counter()
    for _ in range(reps):
        dec = codec.tree_decode(ctx, enc)
    ctx.sync()
    dec_ms = (time.perf_counter() - t0) / reps * 1e3
    print(json.dumps({"workload": f"tree mode, {n} x {m} u8 codes, K=256, 100-root forest",
                      "encode_ms": round(enc_ms, 3), "decode_ms": round(dec_ms, 3),
                      "host_tree_order_ms": round(host_ms, 3),
                      "device_tree_order_ms": round(dev_order_ms, 3),
                      "bits_per_vector": round(enc.bits / n, 3),
                      "ext_rows": int(enc.ext_rows.shape[0]),
                      "roundtrip_mvec_s": round(n / (enc_ms + dec_ms) / 1e3, 2)}))


if __name__ == "__main__":
    main()
