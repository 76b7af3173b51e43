"""Context-histogram timing (diagnostic): the 1024-thread and 256-thread (PQH_HIST_BLOCK)
variants of hist_ctx on the bench's 1M-row SIFT-shaped codes, then pq_assign_mfma alone."""
import os, sys
sys.path.insert(0, os.getcwd())
import torch
from pq_huffman_amd import codec
import bench
dev = torch.device("cuda", 0)
x = bench.make_data(torch, 1_000_000, 128, 0x5EED, 0, dev)
cent = bench.train_centroids(torch, bench.make_data(torch, 200_000, 128, 0x5EED, 0, dev), 8, 256)
ctx = codec.Context(0)
pq = codec.PQ(ctx, cent)
codes = torch.empty((1_000_000, 8), dtype=torch.uint8, device=dev)
pq.assign(x, codes)
counts = torch.empty((8, 65536), dtype=torch.int32, device=dev)
for impl in ("1024", "256"):
    os.environ["PQH_HIST_BLOCK"] = impl
    for _ in range(3): codec.histogram(ctx, codes, 256, True, counts=counts, accumulate=False)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(50): codec.histogram(ctx, codes, 256, True, counts=counts, accumulate=False)
    e1.record(); torch.cuda.synchronize()
    print("hist", impl, e0.elapsed_time(e1) / 50, "ms", flush=True)
# assign alone
for _ in range(3): pq.assign(x, codes)
torch.cuda.synchronize()
e0.record()
for _ in range(20): pq.assign(x, codes)
e1.record(); torch.cuda.synchronize()
print("assign", e0.elapsed_time(e1) / 20, "ms", flush=True)
