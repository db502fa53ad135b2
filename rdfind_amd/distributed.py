"""Sharded multi-GPU CIND discovery: one process per GPU, torch.distributed over RCCL.

Each rank holds a slice of the triples (or all of them, and the library takes its row range).  The collectives
the library requests one at a time (``rdf_shard_step``):

  a. all-to-all       unary (key, count) partials of the slices to the key's owner rank, which sums them
                      (FrequentConditionPlanner.scala:293-309)
  a''. all-gather     (world > 1) each owner's hot join value candidates and every rank's slice size: every rank
                      derives the same owner table for the hottest join values (balanced, largest first)
  a'. all-gather      the frequent unary keys of every owner (sorted afterwards: global ranks)
  b. all-to-all       binary (key, count) partials to the key's owner rank, which sums them (:381-393)
  c. all-gather       the frequent binary keys of every owner (sorted afterwards: deterministic ids)
  (c'. all-reduce     --use-ars only: the slices' triple counts of the frequent conditions, for the rules,
                      FrequentConditionPlanner.scala:130-194)
  d. all-to-all       every triple to the ranks owning its join values (RDFind.scala:339-345 groupBy(joinValue)),
                      so rank r builds the capture groups of its join-value hash shard
  1. all-reduce(sum)  capture supports (distinct join values per capture)
  2. all-gather       group-size histograms -> global heavy threshold + this rank's heavy bit base
  3. all-reduce(sum)  heavy-group bitmasks (bits of different ranks are disjoint, so sum == or)
  4. all-reduce(min)  (pivot size, rank) per dependent
  5. all-reduce(sum)  light-group counts, the number of ranks holding light groups per dependent and their
                      rank mask
  6. all-to-all       holder-first light exchange: only the rank holding d's globally smallest group (the pivot
                      holder) draws candidates from it and checks its own light groups; each survivor (dep, ref)
                      goes to the owner (dep_owner(dep), a hash mod R) as the holder's report and to every other rank with a light
                      group of dep for verification
  7. all-to-all       the verified survivors -> the owner, which keeps a ref iff every rank with a light group of
                      dep reported it.  Together this is the reference's combiner-side intersection
                      (AllAtOnceTraversalStrategy.scala:62-65) and the shuffle to the IntersectCindCandidates
                      reducer, with candidate generation done once per dependent instead of once per rank.
  8. all-gather       the final explicit CIND pairs of the unary dependents (R1 / R4 probe the components of
                      binary dependents, which are unary); binary dependents' pairs stay with their owner
  9. all-gather       filtered ref lists of the bitmask classes pivoted on each rank

Each rank then emits the CINDs of its own dependents; the union over ranks is the single-GPU result.

``run_sharded`` drives any object with ``shard_begin/shard_step/shard_export/shard_import`` (the HIP
``Context``); ``run_protocol`` is the backend-neutral loop, also used by the CPU protocol tests.

Failure agreement.  Every collective starts with one small all-gather of a header per rank -- (status, op, count,
send counts) -- which also carries the counts allgatherv / alltoallv need, and the run ends with one more header (op
DONE).  A rank whose library step, export or import fails joins the next header with a failure status and raises; every
other rank sees it there and raises ``PeerFailure`` instead of waiting in a collective the failed rank never enters
(the reference's job fails as a whole on any task's exception, FLK/jobs/AbstractProgram.java:119-126).  A rank that
dies inside a collective is covered by the process group's timeout (``init_process_group(timeout=...)``).
"""
from __future__ import annotations

import torch
import torch.distributed as dist

from . import _lib

_DTYPES = {_lib.X_ALLREDUCE_SUM_U32: torch.int32}


def _dtype(op):
    return _DTYPES.get(op, torch.int64)


_COMPACT_CHUNK_BYTES = 64 << 20  # staging chunk of allgatherv's in-place compaction


def _compact_in_place(buf: torch.Tensor, counts, mx: int) -> int:
    """Move slice r of ``buf`` (at r * mx, counts[r] elements) to the running offset sum(counts[:r]), in place and in
    rank order.  Destinations never pass their sources, so copying each slice front to back in chunks staged through
    one bounded scratch tensor never overwrites data not yet moved.  Returns the total count."""
    chunk = max(_COMPACT_CHUNK_BYTES // buf.element_size(), 1)
    scratch = None
    off = 0
    for r, c in enumerate(counts):
        src = r * mx
        if c and src != off:
            if scratch is None:
                scratch = buf.new_empty(min(chunk, max(counts)))
            for k in range(0, c, chunk):
                m = min(chunk, c - k)
                scratch[:m].copy_(buf[src + k: src + k + m])
                buf[off + k: off + k + m].copy_(scratch[:m])
        off += c
    return off


def allgatherv(send: torch.Tensor, group=None, counts=None) -> torch.Tensor:
    """Variable-length all-gather: concatenation of every rank's ``send`` in rank order.  The counts (from the header
    exchange, or one all-gather of them), then, unless the contributions are very skewed, one all-gather of padded slices
    into a single preallocated tensor (world x the largest slice) that is compacted in place, so the peak is that tensor
    (+ one padded copy of this rank's slice and a 64 MiB staging chunk), not a second result-sized copy.  When padding
    would exceed 4x the payload and 64 MiB, one broadcast per rank into its exact slice of the result instead."""
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    if counts is None:
        n = torch.tensor([send.numel()], dtype=torch.int64, device=send.device)
        counts_t = torch.empty(world, dtype=torch.int64, device=send.device)
        dist.all_gather_into_tensor(counts_t, n, group=group)
        counts = [int(c) for c in counts_t.tolist()]
    mx, tot = max(counts), sum(counts)
    if not tot:
        return send.new_empty(0)
    pad_bytes = (world * mx - tot) * send.element_size()
    if world * mx <= 4 * tot or pad_bytes <= (64 << 20):
        pad = send
        if send.numel() < mx:
            pad = send.new_zeros(mx)
            pad[: send.numel()].copy_(send)
        gathered = send.new_empty(world * mx)
        dist.all_gather_into_tensor(gathered, pad, group=group)
        del pad
        return gathered[: _compact_in_place(gathered, counts, mx)]
    out = send.new_empty(tot)
    off = 0
    for r, c in enumerate(counts):
        if c:
            part = out[off: off + c]
            if r == rank:
                part.copy_(send)
            dist.broadcast(part, src=dist.get_global_rank(group, r) if group is not None else r, group=group)
        off += c
    return out


def alltoallv(send: torch.Tensor, send_counts, group=None, recv_counts=None) -> torch.Tensor:
    """Variable-length all-to-all: ``send`` holds consecutive slices for ranks 0..R-1.  recv_counts: from the header
    exchange (else one all-to-all of the counts)."""
    world = dist.get_world_size(group)
    sc = [int(x) for x in send_counts] + [0] * (world - len(send_counts))
    if recv_counts is None:
        sct = torch.tensor(sc, dtype=torch.int64, device=send.device)
        rc = torch.empty_like(sct)
        dist.all_to_all_single(rc, sct, group=group)
        recv_counts = [int(x) for x in rc.tolist()]
    out = send.new_empty(sum(recv_counts))
    dist.all_to_all_single(out, send, output_split_sizes=list(recv_counts), input_split_sizes=sc, group=group)
    return out


def exchange(req: _lib.ExchangeRequest, send: torch.Tensor, group=None, header=None) -> torch.Tensor:
    """Perform the collective ``req`` describes on ``send`` and return the result tensor.  header: the agreed per-rank
    header rows (``agree``), whose counts replace the count exchanges of allgatherv / alltoallv."""
    op = req.op
    if op in (_lib.X_ALLREDUCE_SUM_U32, _lib.X_ALLREDUCE_SUM_U64):
        dist.all_reduce(send, op=dist.ReduceOp.SUM, group=group)  # two's-complement sums == unsigned sums
        return send
    if op == _lib.X_ALLREDUCE_MIN_U64:
        dist.all_reduce(send, op=dist.ReduceOp.MIN, group=group)  # values < 2^63 by contract
        return send
    if op == _lib.X_ALLGATHERV_U64:
        return allgatherv(send, group, None if header is None else [h[2] for h in header])
    if op == _lib.X_ALLTOALLV_U64:
        me = dist.get_rank(group)
        return alltoallv(send, req.send_counts, group, None if header is None else [h[3 + me] for h in header])
    raise ValueError(f"unknown exchange op {op}")


class PeerFailure(RuntimeError):
    """Another rank of the sharded run failed; this rank stops at the same collective instead of waiting in it."""


_ST_OK, _ST_FAILED = 0, 1
_OP_DONE = -1


def agree(status: int, op: int, count: int, send_counts, group=None, device=None):
    """One all-gather of (status, op, count, send counts[world]) per rank: returns every rank's header row.  Raises
    PeerFailure when another rank reports a failure, RuntimeError when the ranks disagree on the collective (a protocol
    bug: the collective itself would hang or mix data)."""
    world = dist.get_world_size(group)
    me = dist.get_rank(group)
    sc = [int(x) for x in (send_counts or [])][:world]
    row = torch.tensor([status, op, count] + sc + [0] * (world - len(sc)), dtype=torch.int64, device=device)
    allrows = torch.empty(world * (3 + world), dtype=torch.int64, device=device)
    dist.all_gather_into_tensor(allrows, row, group=group)
    rows = [[int(x) for x in allrows[r * (3 + world):(r + 1) * (3 + world)].tolist()] for r in range(world)]
    failed = [r for r in range(world) if rows[r][0] != _ST_OK and r != me]
    if failed:
        raise PeerFailure(f"rank {me}: sharded run stopped, rank(s) {failed} failed")
    if status == _ST_OK and any(rows[r][1] != op for r in range(world)):
        raise RuntimeError(f"rank {me}: ranks disagree on the collective: ops {[rows[r][1] for r in range(world)]}")
    return rows


def exchange_device(group=None) -> torch.device:
    """Where exchange buffers live: HBM for RCCL, host memory for gloo (a CPU-only process group)."""
    if dist.get_backend(group) == "nccl":
        return torch.device("cuda", torch.cuda.current_device())
    return torch.device("cpu")


_BIG_EXCHANGE_BYTES = 1 << 30  # a collective above this (the triples' routing at 10^9-triple scale) is not cached


def _send_buffer(machine, n, dtype, device):
    """The rank's send buffer for one collective: a view of a persistent buffer per (dtype, device), grown by half
    again when a collective needs more (the collectives of a run reuse it instead of allocating each time).  A send of
    more than _BIG_EXCHANGE_BYTES gets a buffer of its own, released after the collective, so the one large exchange of a
    run (the triples to their join owners: ~21 GB per rank for c4 at 10^9 triples over 2 ranks) does not stay allocated
    through the group build that follows it."""
    elem = torch.empty(0, dtype=dtype).element_size()
    if n * elem > _BIG_EXCHANGE_BYTES:
        return torch.empty(n, dtype=dtype, device=device)
    bufs = machine.__dict__.setdefault("_x_send", {})
    key = (dtype, device.type, device.index)
    b = bufs.get(key)
    if b is None or b.numel() < n:
        b = torch.empty(max(n, 1, b.numel() + b.numel() // 2 if b is not None else 0), dtype=dtype, device=device)
        bufs[key] = b
    return b[:n]


def run_protocol(machine, group=None, device=None):
    """Drive a shard machine to completion.  ``machine.shard_step()`` returns an ExchangeRequest;
    ``machine.shard_export(ptr)`` fills ``count`` elements at ``ptr``; ``machine.shard_import(ptr, n)``
    takes the result.  Every collective is preceded by the header agreement (``agree``): a failure of this rank's step,
    export or import is announced in the next header and re-raised here; a peer's failure raises PeerFailure.  Returns
    the number of collectives performed."""
    device = device or exchange_device(group)
    world = dist.get_world_size(group)
    n = 0
    sent = received = 0
    while True:
        try:
            req = machine.shard_step()
            send = None
            if req.op != _lib.X_DONE:
                send = _send_buffer(machine, req.count, _dtype(req.op), device)
                machine.shard_export(send.data_ptr())
        except Exception:
            # this rank failed before its collective: the peers wait in (or are about to start) the next header
            try:
                agree(_ST_FAILED, 0, 0, None, group, device)
            except Exception:
                pass
            raise
        op = _OP_DONE if req.op == _lib.X_DONE else int(req.op)
        sc = list(req.send_counts)[:world] if req.op == _lib.X_ALLTOALLV_U64 else None
        header = agree(_ST_OK, op, int(req.count), sc, group, device)
        if req.op == _lib.X_DONE:
            # this rank's exchange volume (elements x element size), kept on the machine for the bench's work counters
            machine.x_stats = {"collectives": n, "bytes_sent": sent, "bytes_received": received}
            return n
        if req.count == 0 and req.op in (_lib.X_ALLREDUCE_SUM_U32, _lib.X_ALLREDUCE_SUM_U64, _lib.X_ALLREDUCE_MIN_U64):
            recv = send  # an all-reduce has the same count on every rank: all skip it
        else:
            # shard_export returns once the library's stream has written `send`, so the collective (on torch's stream)
            # may start at once; the library reads `recv` on its own stream, so torch's stream must have finished it
            recv = exchange(req, send, group, header).contiguous()
            if device.type == "cuda":
                torch.cuda.current_stream(device).synchronize()
            sent += send.numel() * send.element_size()
            received += recv.numel() * recv.element_size()
        try:
            machine.shard_import(recv.data_ptr(), recv.numel())
        except Exception:
            try:  # the peers are at the next step's header
                agree(_ST_FAILED, 0, 0, None, group, device)
            except Exception:
                pass
            raise
        big = max(send.numel() * send.element_size(), recv.numel() * recv.element_size()) > _BIG_EXCHANGE_BYTES
        del send, recv
        if big and device.type == "cuda":  # give the large exchange's HBM back to the library's allocations
            torch.cuda.empty_cache()
        n += 1


def run_sharded(ctx, min_support: int, projection="spo", clean_implied=True, traversal_strategy=1, group=None,
                device=None, local_slice=False, use_ars=False):
    """Sharded CIND discovery on this rank's context; returns (group_stats, cind_stats) of this rank.
    local_slice: the context's resident triples are this rank's slice of the input.  use_ars: association rules from
    the combined counts (one more all-reduce), applied as on one GPU."""
    rank = dist.get_rank(group)
    world = dist.get_world_size(group)
    ctx.shard_begin(rank, world, min_support, projection, clean_implied, traversal_strategy, local_slice, use_ars)
    try:
        run_protocol(ctx, group, device)
    except _lib.RdfError as e:
        if e.status == _lib.RDF_ERR_OOM:  # sharded runs are not paged (one GPU pages, rdf_discover_cinds_paged)
            raise _lib.RdfError(f"rank {rank} of {world}: its share of the result exceeds the device memory; sharded "
                                f"discovery is not paged, use more ranks ({e})", e.status) from e
        raise
    return ctx.last_stats()


def run_ingest(ctx, data: bytes, tabs=False, group=None, device=None) -> int:
    """Sharded ingest (rdf_shard_parse_begin): this rank parses ``data`` (its part of the input), the dictionary
    exchange assigns global term ids, and the rank's triples become its slice in that id space.  Returns the rank's
    triple count; ``ctx.num_terms`` is the global dictionary size."""
    n = ctx.shard_parse_begin(dist.get_rank(group), dist.get_world_size(group), data, tabs)
    run_protocol(ctx, group, device)
    ctx.num_terms_now()
    return n


def run_dictionary(ctx, group=None, device=None):
    """After a sharded run on sharded-ingest triples: the formatting dictionary of every term an output line can name,
    gathered from the terms' owners (rdf_shard_dictionary_begin)."""
    ctx.shard_dictionary_begin()
    run_protocol(ctx, group, device)
