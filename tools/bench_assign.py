"""Assignment-only timing (diagnostic): the bench's SIFT-shaped batch and trained
centroids, pq_assign_mfma (+ its re-rank fix-up) launched back to back.  Run under
rocprofv3 for per-kernel statistics and PMC counters."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
import bench  # noqa: E402
from pq_huffman_amd import codec  # noqa: E402


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 20
    dev = torch.device("cuda", 0)
    n, d, m, k = 1_000_000, 128, 8, 256
    x = bench.make_data(torch, n, d, 1234, 0, dev)
    cent = bench.train_centroids(torch, x, m, k)
    ctx = codec.Context(0)
    pq = codec.PQ(ctx, cent)
    codes = torch.empty((n, m), dtype=torch.uint8, device=dev)
    for _ in range(3):
        pq.assign(x, codes)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        pq.assign(x, codes)
    torch.cuda.synchronize()
    ms = (time.perf_counter() - t0) / reps * 1e3
    print(f"assign {ms:.4f} ms/launch  ({n / ms / 1e3:.1f} Mvec/s)  rerank {pq.rerank_count()}",
          flush=True)


if __name__ == "__main__":
    main()
