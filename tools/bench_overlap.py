"""Overlap experiment (diagnostic): the code-table build on a CU-limited stream beside the
next batch's assignment on another stream.  Prints standalone and concurrent times."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402
from pq_huffman_amd import codec  # noqa: E402


def timed(fn, reps=10):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / reps * 1e3


def main():
    dev = torch.device("cuda", 0)
    n, d, m, k = 1_000_000, 128, 8, 256
    g = torch.Generator(device=dev)
    g.manual_seed(3)
    x = torch.round(torch.rand((n, d), generator=g, device=dev) * 60 + 
                    torch.randint(0, 4, (n, 1), generator=g, device=dev) * 40)
    cent = x[torch.randperm(n, generator=g, device=dev)[:k]].reshape(k, m, 16).permute(1, 0, 2)
    cent = np.ascontiguousarray(cent.cpu().numpy())
    sA = torch.cuda.Stream()
    ctxA = codec.Context(0, stream=sA)
    pq = codec.PQ(ctxA, cent)
    codes = torch.empty((n, m), dtype=torch.uint8, device=dev)
    with torch.cuda.stream(sA):
        pq.assign(x, codes)
        counts = codec.histogram(ctxA, codes, k, True)
    torch.cuda.synchronize()
    for cus in (0, 32, 64, 128):
        ctxB = codec.Context(0, cus=cus) if cus else codec.Context(0, stream=torch.cuda.Stream())
        tabs = codec.Tables(ctxB, m, k, True)
        a = timed(lambda: pq.assign(x, codes))
        b = timed(lambda: tabs.build(counts))
        c = timed(lambda: (tabs.build(counts), pq.assign(x, codes)))
        print(f"cus={cus or 'all'}: assign {a:.3f} ms, tables {b:.3f} ms, both concurrent "
              f"{c:.3f} ms (serial sum {a + b:.3f})", flush=True)


if __name__ == "__main__":
    main()
