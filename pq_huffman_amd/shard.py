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

The protocol itself is the library's (include/pqh.h "multi-GPU row shards"):
pqh_shard_encode runs a rank's whole encode with the caller's collectives as hooks (TorchComm
adapts a torch.distributed process group: RCCL on the GPU, gloo in the rehearsals), and the
host pieces -- row ranges (pqh_shard_block), offsets (pqh_shard_offsets), the stitch
(pqh_shard_stitch), the ragged halo's source (pqh_shard_halo_source) -- are C functions this
module calls.  The remaining helpers issue torch.distributed collectives for the bench's
overlapped schedule (bench.py), which interleaves the same steps across batches and streams.
"""
from __future__ import annotations

import ctypes
from typing import Iterable, Sequence, Tuple


def _lib():
    from .capi import lib
    return lib()


def row_range(n_total: int, world: int, rank: int) -> Tuple[int, int]:
    """Contiguous shard [begin, end) of rank `rank`: sizes differ by at most one row
    (pqh_shard_block, a block_t descriptor)."""
    from .capi import Block, check
    b = Block()
    check(_lib().pqh_shard_block(n_total, world, rank, ctypes.byref(b)), "pqh_shard_block")
    return b.id, b.id + b.size


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


def offsets_of(lengths: Sequence[int], rank: int) -> Tuple[int, int]:
    """(this rank's global bit offset, the global length) from every rank's bit length
    (pqh_shard_offsets)."""
    from .capi import check
    w = len(lengths)
    arr = (ctypes.c_ulonglong * w)(*[int(v) for v in lengths])
    off, tot = ctypes.c_ulonglong(), ctypes.c_ulonglong()
    check(_lib().pqh_shard_offsets(arr, w, rank, ctypes.byref(off), ctypes.byref(tot)),
          "pqh_shard_offsets")
    return off.value, tot.value


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
    return offsets_of(everyone.cpu().tolist(), rank)


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
    """Concatenate shard buffers into the global stream (huffman_indices.bin payload) with
    pqh_shard_stitch.

    shards: (buffer, global_bit_offset, bits) per shard, where buffer holds the shard's
    stream starting at bit `global_bit_offset % 32` and is zero elsewhere.  Bit ranges are
    disjoint, so OR-ing the buffers at their word positions yields the reference stream
    (zero padded to a byte, bitstream.c:104-110)."""
    from .capi import check
    shards = list(shards)
    w = len(shards)
    for buf, goff, bits in shards:
        if bits and (goff + bits + 7) // 8 - buffer_byte_start(goff) > len(buf):
            raise ValueError("shard buffer shorter than its bit range")
    keep = [ctypes.create_string_buffer(bytes(b), max(1, len(b))) for b, _, _ in shards]
    bufs = (ctypes.c_void_p * w)(*[ctypes.addressof(k) for k in keep])
    offs = (ctypes.c_ulonglong * w)(*[int(g) for _, g, _ in shards])
    bits = (ctypes.c_ulonglong * w)(*[int(n) for _, _, n in shards])
    nb = (sum(int(n) for _, _, n in shards) + 7) // 8
    if sum(int(n) for _, _, n in shards) != total_bits:
        raise ValueError("shard lengths do not add up to total_bits")
    out = ctypes.create_string_buffer(max(1, nb))
    check(_lib().pqh_shard_stitch(w, bufs, offs, bits, out, nb), "pqh_shard_stitch")
    return out.raw[:nb]


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


# ---- sort mode across ranks ("sort mode is not embarrassingly parallel") ----
#
# The reference's default mode sorts all rows (huffman_encoder.c:301-317: qsort + strncmp) --
# a stable sort by key(row) = the row with every byte after its first 0 zeroed.  Across
# ranks it is a sample sort: every rank sorts its shard (stable), all-gathers a few sample
# keys, picks world - 1 splitters, and all-to-alls each row to the rank whose key range holds
# it.  A row goes to rank d = #{splitters < key}, so all rows with one key land on one rank;
# they arrive in source-rank order (= global row order) and each source's run is already in
# stable order, so a final stable local sort yields the rank's slice of the global order.
# The slices concatenated in rank order are the reference's sorted rows; some slices may be
# empty (heavy keys), which `halo_ragged` handles.


def sort_key_words(codes):
    """(n, ceil(m/8)) int64 words that order like the strncmp key: the row's bytes with every
    byte after its first 0 zeroed, big-endian, sign bit flipped so that signed int64
    comparison is unsigned comparison."""
    import torch
    n, m = codes.shape
    c = codes.to(torch.int64)
    ones = torch.ones((n, 1), dtype=torch.int64, device=c.device)
    alive = torch.cumprod(torch.cat([ones, (c[:, :-1] != 0).to(torch.int64)], 1), 1)
    kb = c * alive
    w = (m + 7) // 8
    if w * 8 != m:
        kb = torch.cat([kb, torch.zeros((n, w * 8 - m), dtype=torch.int64, device=c.device)], 1)
    shifts = torch.arange(56, -1, -8, dtype=torch.int64, device=c.device)
    words = (kb.view(n, w, 8) << shifts).sum(-1)          # disjoint fields: sum == or
    return words ^ torch.tensor(-(1 << 63), dtype=torch.int64, device=c.device)


def _count_le(words, key):
    """#rows of the lexicographically sorted (n, W) `words` that are <= `key` (W ints)."""
    import torch
    lo, hi = 0, words.shape[0]
    for j, kv in enumerate(key):
        col = words[lo:hi, j].contiguous()
        t = torch.tensor([kv], dtype=torch.int64, device=words.device)
        a = int(torch.searchsorted(col, t).item())
        b = int(torch.searchsorted(col, t, right=True).item())
        if j == len(key) - 1:
            return lo + b
        lo, hi = lo + a, lo + b     # rows before lo are smaller; [lo, hi) tie on word j
        if lo == hi:
            break
    return lo


def sort_rows_distributed(codes, world: int, rank: int, local_sort, group=None,
                          samples: int = 256):
    """This rank's slice of the stable strncmp-key sort of all ranks' rows.

    codes: (n_r, m) uint8 tensor, the rank's contiguous row shard (rank order = row order).
    local_sort(t) -> t sorted (stable, strncmp key): the GPU library's pqh_sort_rows
    (`codec.sort_rows`) on the GPU; the CPU tests pass the oracle's.  Returns a new
    (n'_r, m) tensor on the same device."""
    import torch
    import torch.distributed as dist
    srt = local_sort(codes) if codes.shape[0] else codes
    if world == 1:
        return srt
    n, m = srt.shape
    dev = srt.device
    words = sort_key_words(srt)
    nw = words.shape[1]
    # samples: evenly spaced keys of the sorted shard (an empty shard sends none)
    s = min(samples, n)
    idx = (torch.arange(s, device=dev) * n) // max(s, 1) if s else torch.zeros(0, dtype=torch.long,
                                                                               device=dev)
    mine = torch.full((samples, nw + 1), 0, dtype=torch.int64, device=dev)
    if s:
        mine[:s, :nw] = words[idx]
        mine[:s, nw] = 1                                        # valid flag
    allsamp = torch.empty((world * samples, nw + 1), dtype=torch.int64, device=dev)
    dist.all_gather_into_tensor(allsamp, mine, group=group)
    keys = sorted(tuple(r[:nw]) for r in allsamp.cpu().tolist() if r[nw])
    splitters = [keys[(j + 1) * len(keys) // world - 1] for j in range(world - 1)] if keys else []
    # rows to rank d: #splitters < key, i.e. the boundaries are #rows <= splitter_j
    bounds = [0] + [_count_le(words, sp) for sp in splitters] + [n] * (world - len(splitters))
    send = torch.tensor([bounds[d + 1] - bounds[d] for d in range(world)], dtype=torch.int64)
    recv = torch.empty_like(send)
    sd, rd = send.to(dev), recv.to(dev)
    dist.all_to_all_single(rd, sd, group=group)
    recv = rd.cpu()
    out = torch.empty((int(recv.sum()), m), dtype=srt.dtype, device=dev)
    dist.all_to_all_single(out.view(-1), srt.reshape(-1),
                           output_split_sizes=[int(v) * m for v in recv.tolist()],
                           input_split_sizes=[int(v) * m for v in send.tolist()], group=group)
    return local_sort(out) if out.shape[0] else out


def library_sort(ctx):
    """local_sort for sort_rows_distributed on the GPU: the library's stable radix sort
    (pqh_sort_rows, in place) on the context's stream."""
    from . import codec

    def run(t):
        t = t.contiguous()
        codec.sort_rows(ctx, t)
        return t
    return run


def halo_ragged(last_row, world: int, rank: int, group=None, device=None, dtype=None):
    """exchange_halo for shards that may be empty (sorted slices): `last_row` is the (m,)
    last row or None.  Returns (halo, raw_first): the last row of the nearest non-empty
    predecessor (None if there is none), in last_row's dtype (`dtype` on an empty rank,
    uint8 by default) on the group's device, and whether this rank holds global row 0,
    which context mode writes raw (huffman_encoder.c:234).

    Everything moves as device tensors through all_gather_into_tensor, so the same call runs
    on an RCCL group (device = this rank's GPU) and a gloo one (CPU tensors).  `device` is
    needed only on a rank whose slice is empty; it defaults to the current GPU when the
    group's backend is nccl, else the CPU."""
    import torch
    import torch.distributed as dist
    if world == 1:
        return None, 1
    if last_row is not None:
        dev, dt = last_row.device, last_row.dtype
    else:
        nccl = dist.get_backend(group) == "nccl"
        dev = device if device is not None else (
            torch.device("cuda", torch.cuda.current_device()) if nccl else torch.device("cpu"))
        dt = dtype if dtype is not None else torch.uint8
    # everyone needs m: share it with the non-empty flag
    info = torch.tensor([1 if last_row is not None else 0,
                         last_row.numel() if last_row is not None else 0],
                        dtype=torch.int64, device=dev)
    allinfo = torch.empty(world * 2, dtype=torch.int64, device=dev)
    dist.all_gather_into_tensor(allinfo, info, group=group)
    allinfo = allinfo.view(world, 2).cpu().tolist()
    mm = max(r[1] for r in allinfo)
    row = torch.zeros(mm, dtype=torch.int64, device=dev)
    if last_row is not None:
        row[:last_row.numel()] = last_row.reshape(-1).to(torch.int64)
    rows = torch.empty(world * mm, dtype=torch.int64, device=dev)
    dist.all_gather_into_tensor(rows, row, group=group)
    from .capi import check
    has = (ctypes.c_int * world)(*[int(r[0]) for r in allinfo])
    prev, raw = ctypes.c_int(), ctypes.c_int()
    check(_lib().pqh_shard_halo_source(has, world, rank, ctypes.byref(prev), ctypes.byref(raw)),
          "pqh_shard_halo_source")
    halo = rows.view(world, mm)[prev.value].to(dt).contiguous() if prev.value >= 0 else None
    return halo, raw.value


# ---- the library's whole-shard encode (pqh_shard_encode) with torch.distributed hooks ----

class TorchComm:
    """pqh_shard_comm_t over a torch.distributed process group.  The library hands the hooks
    raw device pointers; they must lie inside tensors registered here (the counts and the
    scratch the encode uses), which the hooks slice and pass to all_reduce /
    all_gather_into_tensor, ordered on the library context's stream."""

    def __init__(self, world: int, rank: int, group=None):
        from .capi import ALL_GATHER, ALL_REDUCE_U32, ShardComm
        self.world, self.rank, self.group = world, rank, group
        self._tensors = []
        self._streams = {}   # the library streams' ExternalStream objects, made once each
        self._reduce = ALL_REDUCE_U32(self._all_reduce)
        self._gather = ALL_GATHER(self._all_gather)
        self.struct = ShardComm(None, world, rank, self._reduce, self._gather)
        self.error = None

    def register(self, *tensors):
        for t in tensors:
            if t is not None:
                self._tensors.append(t)
        return self

    def clear(self):
        """forget the registered tensors (shard_encode registers its buffers per call)"""
        self._tensors = []
        return self

    def _view(self, ptr, nbytes, dtype):
        import torch
        for t in self._tensors:
            base = t.data_ptr()
            size = t.numel() * t.element_size()
            if base <= ptr and ptr + nbytes <= base + size:
                flat = t.view(-1).view(torch.uint8)
                return flat[ptr - base:ptr - base + nbytes].view(dtype)
        raise ValueError(f"device pointer {ptr:#x} is in no registered tensor")

    def _on_stream(self, stream, fn):
        import torch
        try:
            if stream:
                es = self._streams.get(stream)
                if es is None:
                    es = self._streams[stream] = torch.cuda.ExternalStream(stream)
            with torch.cuda.stream(es) if stream else _null():
                fn()
            return 0
        except Exception as e:  # the C caller gets a status; keep the reason
            self.error = e
            return 1

    def _all_reduce(self, user, ptr, count, stream):
        import torch
        import torch.distributed as dist
        return self._on_stream(stream, lambda: dist.all_reduce(
            self._view(ptr, count * 4, torch.int32), group=self.group))

    def _all_gather(self, user, send, recv, nbytes, stream):
        import torch
        import torch.distributed as dist
        return self._on_stream(stream, lambda: dist.all_gather_into_tensor(
            self._view(recv, nbytes * self.world, torch.uint8),
            self._view(send, nbytes, torch.uint8), group=self.group))


class _null:
    def __enter__(self):
        return self

    def __exit__(self, *a):
        return False


def shard_encode(ctx, comm: TorchComm, codes, tables, counts, out, chunk_vectors=0,
                 chunk_offsets=None, chunk_prev=None, first_row=0, raw_first=True, check=False):
    """This rank's encode through pqh_shard_encode (halo, histogram all-reduce, GPU code
    tables, lengths all-gather, device offsets, write) -- asynchronous on ctx's stream.
    codes: (n, m) uint8 cuda tensor (n may be 0); counts: (m, items) int32; out: uint8
    buffer.  Returns (offsets, raw): offsets a (2,) int64 device tensor {global bit offset,
    global length}; raw = whether this shard wrote the raw first row (read back from the
    device when raw_first is True -- the call's one host round trip -- else None).  A failure
    on another rank shows in offsets[1] == -1: check=True synchronises and raises on it here
    (status()); otherwise the caller checks with status()."""
    import torch
    from .capi import Block, check as _check
    n, m = codes.shape
    dev = codes.device
    scratch = torch.empty(int(_lib().pqh_shard_scratch_bytes(comm.world, m)), dtype=torch.uint8,
                          device=dev)
    offsets = torch.zeros(2, dtype=torch.int64, device=dev)
    b = Block()
    b.id, b.size, b.capacity = first_row, n, n
    raw = ctypes.c_int()
    ptr = (lambda t: ctypes.c_void_p(t.data_ptr()) if t is not None else None)
    comm.error = None
    comm.register(counts, scratch)   # the hooks' buffers, for this call only
    try:
        rc = _lib().pqh_shard_encode(ctx.ptr, ctypes.byref(comm.struct), ctypes.byref(b),
                                     ptr(codes) if n else None, m, tables.k, int(tables.context),
                                     tables.ptr, ptr(counts), ptr(out), out.numel(), chunk_vectors,
                                     ptr(chunk_offsets), ptr(chunk_prev), ptr(offsets),
                                     ptr(scratch), ctypes.byref(raw) if raw_first else None)
    finally:
        comm.clear()
    if comm.error is not None:
        raise comm.error
    _check(rc, "pqh_shard_encode")
    if ctx.stream != torch.cuda.current_stream(dev):
        scratch.record_stream(ctx.stream)   # (asynchronous: keep it until the stream is done)
    if check:
        status(ctx, offsets)
    return offsets, (raw.value if raw_first else None)


def status(ctx, offsets):
    """Synchronise; raise if any rank's pqh_shard_encode behind `offsets` failed
    (pqh_shard_status: PQH_ERR_REMOTE)."""
    from .capi import check
    check(_lib().pqh_shard_status(ctx.ptr, ctypes.c_void_p(offsets.data_ptr())),
          "pqh_shard_status")


# ---- the same protocol in two phases (pqh_shard_encode_tables / _write), for a caller that
# pipelines batches: phase 1 on the table lane, phase 2 on the encode stream, other batches'
# collectives between them (bench.py's world > 1 schedule) ----

def scratch_for(comm: TorchComm, m: int, device):
    """the d_scratch of one in-flight batch (halo records, halo row, lengths)"""
    import torch
    return torch.empty(int(_lib().pqh_shard_scratch_bytes(comm.world, m)), dtype=torch.uint8,
                       device=device)


def _block(first_row, n):
    from .capi import Block
    b = Block()
    b.id, b.size, b.capacity = first_row, n, n
    return b


def shard_encode_tables(ctx, comm: TorchComm, codes, tables, counts, scratch, first_row=0,
                        parts_n=None, partials=None) -> int:
    """Phase 1 on ctx's stream: halo, histogram, all-reduce, code tables.  Returns the
    rank's status (0 or a negative pqh status), to be handed to shard_encode_write.
    parts_n: codes are PART-MAJOR (m, >= parts_n) (pqh_shard_encode_tables_parts);
    partials: their partial pair counts, already taken (pqh_histogram_partial_parts)."""
    ptr = (lambda t: ctypes.c_void_p(t.data_ptr()) if t is not None else None)
    comm.error = None
    comm.register(counts, scratch)
    try:
        if parts_n is not None:
            m, n = codes.shape[0], parts_n
            rc = _lib().pqh_shard_encode_tables_parts(
                ctx.ptr, ctypes.byref(comm.struct), ctypes.byref(_block(first_row, n)),
                ptr(codes) if n else None, codes.stride(0), m, tables.k, int(tables.context),
                tables.ptr, ptr(counts), ptr(scratch), ptr(partials))
        else:
            n, m = codes.shape
            rc = _lib().pqh_shard_encode_tables(ctx.ptr, ctypes.byref(comm.struct),
                                                ctypes.byref(_block(first_row, n)),
                                                ptr(codes) if n else None, m, tables.k,
                                                int(tables.context), tables.ptr, ptr(counts),
                                                ptr(scratch))
    finally:
        comm.clear()
    if comm.error is not None:
        raise comm.error
    return rc


def shard_encode_write(ctx, comm: TorchComm, codes, tables, out, chunk_vectors, chunk_offsets,
                       chunk_prev, offsets, scratch, status=0, first_row=0, parts_n=None):
    """Phase 2 on ctx's stream: length, all-gather, device offsets (into `offsets`, a (2,)
    int64 tensor), the write.  Raises on this rank's failure; another rank's shows in
    offsets[1] == -1 (status()).  parts_n: part-major codes (pqh_shard_encode_write_parts)."""
    from .capi import check
    ptr = (lambda t: ctypes.c_void_p(t.data_ptr()) if t is not None else None)
    comm.error = None
    comm.register(scratch)
    try:
        if parts_n is not None:
            m, n = codes.shape[0], parts_n
            rc = _lib().pqh_shard_encode_write_parts(
                ctx.ptr, ctypes.byref(comm.struct), ctypes.byref(_block(first_row, n)),
                ptr(codes) if n else None, codes.stride(0), m, tables.k, int(tables.context),
                tables.ptr, ptr(out), out.numel(), chunk_vectors, ptr(chunk_offsets),
                ptr(chunk_prev), ptr(offsets), ptr(scratch), int(status), None)
        else:
            n, m = codes.shape
            rc = _lib().pqh_shard_encode_write(ctx.ptr, ctypes.byref(comm.struct),
                                               ctypes.byref(_block(first_row, n)),
                                               ptr(codes) if n else None, m, tables.k,
                                               int(tables.context), tables.ptr, ptr(out),
                                               out.numel(), chunk_vectors, ptr(chunk_offsets),
                                               ptr(chunk_prev), ptr(offsets), ptr(scratch),
                                               int(status), None)
    finally:
        comm.clear()
    if comm.error is not None:
        raise comm.error
    check(rc, "pqh_shard_encode_write")


def scratch_shard_bits(scratch, world: int, m: int):
    """this shard's exact length in bits, as phase 2 left it in the scratch (a (1,) int64
    device view)"""
    rec = (16 + m + 15) // 16 * 16
    off = rec * (world + 2)
    return scratch[off:off + 8].view(__import__("torch").int64)
