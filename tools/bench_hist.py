"""Context-histogram timing (diagnostic): codec.histogram (hist_ctx + hist_ctx_reduce) on the
bench's 1M-row codes, HIP events around 50 back-to-back calls.
  python tools/bench_hist.py [sift|deep]     (BENCH_HIST_REP=r: the codes tiled r times)
The kernel form is picked per process: PQH_HIST_IMPL=thread (per-thread row runs) or the
default wave-contiguous form; PQH_HIST_BLOCK=256 the 256-thread per-thread form."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
import bench  # noqa: E402
from pq_huffman_amd import codec  # noqa: E402

name = sys.argv[1] if len(sys.argv) > 1 else "sift"
d, m = {"sift": (128, 8), "deep": (96, 16)}[name]
gen = bench.make_deep if name == "deep" else bench.make_data
dev = torch.device("cuda", 0)
n = 1_000_000
x = gen(torch, n, d, 0x5EED, 0, dev)
cent = bench.train_centroids(torch, gen(torch, 200_000, d, 0x5EED, 0, dev), m, 256)
ctx = codec.Context(0)
pq = codec.PQ(ctx, cent)
codes = torch.empty((n, m), dtype=torch.uint8, device=dev)
pq.assign(x, codes)
rep = int(os.environ.get("BENCH_HIST_REP", "1"))   # the batch's codes tiled rep times
if rep > 1:
    codes = codes.repeat(rep, 1)
counts = torch.empty((m, 65536), dtype=torch.int32, device=dev)
for _ in range(3):
    codec.histogram(ctx, codes, 256, True, counts=counts, accumulate=False)
torch.cuda.synchronize()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record()
for _ in range(50):
    codec.histogram(ctx, codes, 256, True, counts=counts, accumulate=False)
e1.record()
torch.cuda.synchronize()
form = os.environ.get("PQH_HIST_IMPL", "wave") + "/" + os.environ.get("PQH_HIST_BLOCK", "1024")
print(f"hist {name} {form} rows {codes.shape[0]} big_min {os.environ.get('PQH_HIST_BIG_MIN', '4000000')} "
      f"{e0.elapsed_time(e1) / 50:.4f} ms "
      f"checksum {int(counts.to(torch.int64).sum())}", flush=True)
