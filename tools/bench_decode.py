"""Decode micro-benchmark with phase stamps of workgroup 0 (diagnostic tool)."""
import ctypes
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
from pq_huffman_amd import codec  # noqa: E402
from pq_huffman_amd.capi import lib  # noqa: E402


def main():
    dev = torch.device("cuda", 0)
    n, m, k = 1_000_000, 8, 256
    g = torch.Generator(device=dev)
    g.manual_seed(1)
    base = torch.randint(0, k, (n, m), generator=g, device=dev)
    skew = (torch.rand((n, m), generator=g, device=dev) ** 3 * k).long()
    codes = ((base // 16) * 16 + skew % 16).clamp(0, k - 1).to(torch.uint8)
    ctx = codec.Context(0)
    L = lib()
    L.pqh_debug_tree_stamps.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
    for mode in (True, False):
        for C in (16, 8):
            items = k * k if mode else k
            counts = torch.zeros((m, items), dtype=torch.int32, device=dev)
            codec.histogram(ctx, codes, k, mode, counts=counts)
            tabs = codec.Tables(ctx, m, k, mode)
            tabs.build(counts)
            enc = codec.encode(ctx, tabs, codes, chunk_vectors=C)
            dec = torch.empty_like(codes)
            for _ in range(3):
                codec.decode(ctx, tabs, enc, out=dec)
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(10):
                codec.decode(ctx, tabs, enc, out=dec)
            e1.record()
            torch.cuda.synchronize()
            assert torch.equal(dec, codes)
            out = (ctypes.c_ulonglong * 16)()
            L.pqh_debug_tree_stamps(ctx.ptr, out)
            st = list(out)
            print(f"ctx={mode} C={C} decode_ms={e0.elapsed_time(e1) / 10:.4f} wg0 cycles: "
                  f"tables={st[9]-st[8]} window={st[10]-st[9]} decode={st[11]-st[10]} "
                  f"in_lds={st[13]} bits/vec={enc.bits / n:.2f}", flush=True)


if __name__ == "__main__":
    main()
