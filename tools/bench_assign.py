"""Assignment-only timing (diagnostic): the bench's SIFT-shaped batch and trained
centroids, pq_assign_mfma (+ its re-rank fix-up) launched back to back.  Run under
rocprofv3 for per-kernel statistics and PMC counters.

  python tools/bench_assign.py [reps] [config]
  config: sift (1M x 128, M=8, K=256; default), deep (1M x 96, M=16, K=256),
          k4096 (1M x 128, M=8, K=4096), m4 (1M x 128, M=4: dsub 32), all
Prints ms per launch, Mvec/s, the algorithmic MFMA rate (2 K D flop per vector) and the
HBM-read fraction (4 D + M * code bytes per vector at 8 TB/s)."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402
import bench  # noqa: E402
from pq_huffman_amd import codec  # noqa: E402

CONFIGS = {"sift": (128, 8, 256), "deep": (96, 16, 256), "k4096": (128, 8, 4096),
           "m4": (128, 4, 256)}


def centroids_from_rows(x, m, k, seed):
    """K centroids per subspace for K > the trainer's reach: data rows plus small offsets."""
    n, d = x.shape
    g = torch.Generator(device=x.device)
    g.manual_seed(seed)
    rows = x[torch.randint(0, n, (k,), generator=g, device=x.device)]
    rows = rows + 0.25 * torch.randn(rows.shape, generator=g, device=x.device)
    return rows.reshape(k, m, d // m).permute(1, 0, 2).contiguous().cpu().numpy()


def run(reps, name):
    d, m, k = CONFIGS[name]
    dev = torch.device("cuda", 0)
    n = int(os.environ.get("BENCH_ASSIGN_N", 1_000_000))
    x = bench.make_data(torch, n, d, 1234, 0, dev) if name != "deep" else \
        torch.nn.functional.normalize(torch.randn((n, d), device=dev,
                                                  generator=torch.Generator(device=dev).manual_seed(7)), dim=1)
    cent = bench.train_centroids(torch, x, m, k) if k == 256 else centroids_from_rows(x, m, k, 5)
    ctx = codec.Context(0)
    pq = codec.PQ(ctx, np.ascontiguousarray(cent, np.float32))
    parts = os.environ.get("BENCH_ASSIGN_PARTS", "0") == "1"   # part-major codes
    ct = torch.uint8 if k <= 256 else torch.int16
    codes = torch.empty((m, (n + 127) // 128 * 128), dtype=ct, device=dev)[:, :n] if parts else \
        torch.empty((n, m), dtype=ct, device=dev)
    run_assign = (lambda mode: pq.assign_parts(x, codes, mode=mode)) if parts else \
        (lambda mode: pq.assign(x, codes, mode=mode))
    modes = (0, 1) if k > 256 and os.environ.get("BENCH_ASSIGN_EXACT", "1") == "1" else (0,)
    for mode in modes:
        r = reps if mode == 0 else max(2, reps // 10)
        for _ in range(2):
            run_assign(mode)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(r):
            run_assign(mode)
        torch.cuda.synchronize()
        ms = (time.perf_counter() - t0) / r * 1e3
        tf = 2.0 * k * d * n / (ms * 1e-3) / 1e12
        hbm = (4 * d + m * (1 if k <= 256 else 2)) * n / (ms * 1e-3) / 8e12
        print(f"{name} mode={mode} assign {ms:.4f} ms/launch ({n / ms / 1e3:.1f} Mvec/s) "
              f"mfma_tflops_algorithmic {tf:.1f} hbm_frac {hbm:.3f} rerank {pq.rerank_count()}",
              flush=True)


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 20
    name = sys.argv[2] if len(sys.argv) > 2 else "sift"
    for nm in (CONFIGS if name == "all" else [name]):
        run(reps, nm)


if __name__ == "__main__":
    main()
