"""Sort-mode timing (huffman_encoder's default strncmp-key stable sort, pqh_sort_rows) on
M x N skewed codes (env M, N; default 1M x 8), alone on the GPU: ms per call by HIP events over 50 calls.
PQH_SORT_IMPL=rocprim selects the library path."""
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import datagen  # noqa: E402
from pq_huffman_amd import codec  # noqa: E402


def main():
    n, m = int(os.environ.get("N", 1_000_000)), int(os.environ.get("M", 8))
    a = torch.from_numpy(datagen.skewed_codes(n, m, 256, seed=5)).cuda()
    ctx = codec.Context(0)
    d = a.clone()
    for _ in range(5):
        d.copy_(a)
        codec.sort_rows(ctx, d)
    torch.cuda.synchronize()
    t = 0.0
    reps = 50
    for _ in range(reps):
        d.copy_(a)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        codec.sort_rows(ctx, d)
        e1.record()
        e1.synchronize()
        t += e0.elapsed_time(e1)
    print(json.dumps({"impl": os.environ.get("PQH_SORT_IMPL", "radix"), "n": n, "m": m,
                      "ms": round(t / reps, 4)}))


if __name__ == "__main__":
    main()
