"""Row-sharded multi-GPU protocol of the encode path, one process per GPU.

The path shards by contiguous row ranges; the only data exchanges are small:

  1. context mode: the one-vector halo -- every rank all-gathers each rank's last row so
     rank r > 0 can count the pair (last row of r-1, first row of r) and encode its first
     row with that row as context (huffman_encoder.c:166-205, :220-238);
  2. the symbol histogram all-reduce (sum) that feeds the shared code tables
     (huffman_encoder.c:139-205 over the whole input);
  3. an all-gather of every shard's exact bit length, whose exclusive scan places each
     shard's stream in the global bit stream (the bit cursor of bitstream.c:71-101).

Every rank then builds identical tables (the build is deterministic, so no broadcast) and
writes its shard at bit `offset % 32` of its own word-aligned buffer; `stitch` ORs the
buffers into the single reference stream.  Context mode's raw first row belongs to global
row 0 only (huffman_encoder.c:234).

The functions take a torch.distributed process group (RCCL on the GPU, gloo in the CPU
tests) and torch tensors on the group's device.
"""
from __future__ import annotations

from typing import Iterable, Sequence, Tuple


def row_range(n_total: int, world: int, rank: int) -> Tuple[int, int]:
    """Contiguous shard [begin, end) of rank `rank`: sizes differ by at most one row."""
    base, extra = divmod(n_total, world)
    begin = rank * base + min(rank, extra)
    return begin, begin + base + (1 if rank < extra else 0)


def exchange_halo(last_row, world: int, rank: int, group=None):
    """All-gather every rank's last code row; returns the previous rank's row (the halo of
    this shard's first vector) or None on rank 0.  `last_row` is an (m,) tensor."""
    import torch
    import torch.distributed as dist
    if world == 1:
        return None
    row = last_row.contiguous().reshape(-1)
    gathered = torch.empty(world * row.numel(), dtype=row.dtype, device=row.device)
    dist.all_gather_into_tensor(gathered, row, group=group)
    return gathered.view(world, -1)[rank - 1] if rank > 0 else None


def reduce_counts(counts, world: int, group=None):
    """Global symbol histogram: in-place sum over ranks."""
    import torch.distributed as dist
    if world > 1:
        dist.all_reduce(counts, group=group)
    return counts


def bit_offsets(total_bits, world: int, rank: int, group=None) -> Tuple[int, int]:
    """(global bit offset of this shard, global stream length in bits) from every shard's
    exact bit length.  `total_bits` is a (1,) int64 tensor."""
    import torch
    import torch.distributed as dist
    if world == 1:
        t = int(total_bits.item())
        return 0, t
    everyone = torch.empty(world, dtype=torch.int64, device=total_bits.device)
    dist.all_gather_into_tensor(everyone, total_bits.reshape(1).to(torch.int64), group=group)
    host = [int(v) for v in everyone.cpu().tolist()]
    return sum(host[:rank]), sum(host)


def bit_offsets_device(total_bits, world: int, rank: int, group=None):
    """bit_offsets without a host round trip: (this shard's global bit offset, the global
    length) as (1,) int64 device tensors, from an all-gather of the shards' lengths and a
    prefix sum on the device -- for pqh_encode_write_at."""
    import torch
    import torch.distributed as dist
    t = total_bits.reshape(1).to(torch.int64)
    if world == 1:
        return torch.zeros_like(t), t.clone()
    everyone = torch.empty(world, dtype=torch.int64, device=t.device)
    dist.all_gather_into_tensor(everyone, t, group=group)
    excl = torch.cumsum(everyone, 0) - everyone
    return excl[rank:rank + 1].clone(), everyone.sum().reshape(1)


def local_bit_offset(global_offset: int) -> int:
    """Bit offset inside the shard's own buffer, which starts at global word offset // 32."""
    return global_offset % 32


def buffer_byte_start(global_offset: int) -> int:
    """Byte position of the shard buffer's first byte in the global stream."""
    return (global_offset // 32) * 4


def stitch(shards: Iterable[Tuple[bytes, int, int]], total_bits: int) -> bytes:
    """Concatenate shard buffers into the global stream (huffman_indices.bin payload).

    shards: (buffer, global_bit_offset, bits) per shard, where buffer holds the shard's
    stream starting at bit `global_bit_offset % 32` and is zero elsewhere.  Bit ranges are
    disjoint, so OR-ing the buffers at their word positions yields the reference stream
    (zero padded to a byte, bitstream.c:104-110)."""
    out = bytearray((total_bits + 7) // 8)
    for buf, goff, bits in shards:
        if bits == 0:
            continue
        start = buffer_byte_start(goff)
        end_byte = (goff + bits + 7) // 8            # last global byte holding shard bits
        need = end_byte - start
        if need > len(buf):
            raise ValueError("shard buffer shorter than its bit range")
        for j in range(need):
            out[start + j] |= buf[j]
    return bytes(out)


def stitch_np(shards: Sequence[Tuple["object", int, int]], total_bits: int):
    """numpy version of `stitch` for large streams (buffers are uint8 arrays)."""
    import numpy as np
    out = np.zeros((total_bits + 7) // 8, np.uint8)
    for buf, goff, bits in shards:
        if bits == 0:
            continue
        start = buffer_byte_start(goff)
        need = (goff + bits + 7) // 8 - start
        out[start:start + need] |= np.asarray(buf[:need], np.uint8)
    return out


def raw_first(rank: int) -> int:
    """Context mode writes global row 0 raw; only rank 0 holds it."""
    return 1 if rank == 0 else 0
