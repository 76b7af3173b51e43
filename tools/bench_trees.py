"""Micro-benchmark of the GPU code-table build (trees + decode tables) on a realistic
context histogram: SIFT-like codes -> histogram -> Tables.build timed with HIP events.
Diagnostic tool (not part of the product path)."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
from pq_huffman_amd import codec  # noqa: E402


def main():
    dev = torch.device("cuda", 0)
    n, m, k = 1_000_000, 8, 256
    g = torch.Generator(device=dev)
    g.manual_seed(1)
    # Markov-ish skewed codes: next code near the previous one with Zipf jumps
    z = torch.distributions.Zipf if hasattr(torch.distributions, "Zipf") else None
    base = torch.randint(0, k, (n, m), generator=g, device=dev)
    skew = (torch.rand((n, m), generator=g, device=dev) ** 3 * k).long()
    codes = ((base // 16) * 16 + skew % 16).clamp(0, k - 1).to(torch.uint8)
    ctx = codec.Context(0)
    if os.environ.get("K") == "4096":   # configs[4]: 8 plain alphabets of 4,096 symbols
        k = 4096
        codes = ((torch.rand((n, m), generator=g, device=dev) ** 4) * k).long().clamp(0, k - 1)
        codes = codes.to(torch.int16)
    for mode in ((False,) if k > 256 else (True, False)):
        items = k * k if mode else k
        counts = torch.zeros((m, items), dtype=torch.int32, device=dev)
        codec.histogram(ctx, codes, k, mode, counts=counts)
        tabs = codec.Tables(ctx, m, k, mode)
        for _ in range(3):
            tabs.build(counts)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        reps = 20
        e0.record()
        for _ in range(reps):
            tabs.build(counts)
        e1.record()
        torch.cuda.synchronize()
        L, out = stamps()
        L.pqh_debug_tree_stamps(ctx.ptr, out)
        st = list(out)
        e2, e3 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e2.record()
        for _ in range(reps):   # the trees alone (build - trees = the decode tables)
            tabs.build_trees(counts)
        e3.record()
        torch.cuda.synchronize()
        print(f"ctx={mode} build_ms={e0.elapsed_time(e1) / reps:.4f} "
              f"trees_ms={e2.elapsed_time(e3) / reps:.4f} "
              f"tree0 cycles: scan={st[1]-st[0]} leaves={st[2]-st[1]} merges={st[3]-st[2]} "
              f"codes={st[4]-st[3]} nz={st[5]} nodes={st[6]}", flush=True)


def stamps():
    """Phase cycle counts of tree 0 (s_memtime) after a ctx build."""
    import ctypes
    from pq_huffman_amd.capi import lib
    L = lib()
    L.pqh_debug_tree_stamps.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
    out = (ctypes.c_ulonglong * 16)()
    return L, out


if __name__ == "__main__":
    main()

