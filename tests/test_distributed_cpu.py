"""Sharded protocol on the CPU: real gloo collectives, world size 2 (and 3), driven by the same
``rdfind_amd.distributed.run_protocol`` loop as the GPU path, with ``tests/shard_sim.ShardSim`` standing in
for the HIP library.  The union of the ranks' CINDs must equal the single-process oracle result, and the
ranks' outputs must be disjoint (each dependent has exactly one owner)."""
import os
import random
import socket

import numpy as np
import pytest
import torch.distributed as dist
import torch.multiprocessing as mp

from oracle import rdfind_oracle as R


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _worker(rank, world, port, cases, q, local_slice=False):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from rdfind_amd import distributed
    from tests.shard_sim import ShardSim

    try:
        out = []
        for arr, ms, strategy, clean in cases:
            nv = 1 + max((max(t) for t in arr), default=0)  # one dictionary for all ranks
            # local slices: an interleaved partition (slices need not be contiguous row ranges)
            sim = ShardSim(arr[rank::world] if local_slice else arr, nv, local_slice)
            sim.shard_begin(rank, world, ms, "spo", clean, strategy)
            n = distributed.run_protocol(sim)
            out.append((n, sorted(R.cind_set(sim.result))))
        q.put((rank, out))
    finally:
        dist.destroy_process_group()


def _run(world, cases, local_slice=False):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, cases, q, local_slice)) for r in range(world)]
    for p in procs:
        p.start()
    results = dict(q.get(timeout=300) for _ in procs)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    return results


def _cases(seed, count):
    rng = random.Random(seed)
    cases = []
    for i in range(count):
        nv = rng.randrange(4, 30)
        n = rng.randrange(10, 160)
        arr = [(rng.randrange(nv), rng.randrange(nv // 3 + 1), rng.randrange(nv)) for _ in range(n)]
        strategy, clean = [(1, True), (0, True), (0, False), (1, False)][i % 4]
        cases.append((arr, rng.randrange(1, 4), strategy, clean))
    return cases


@pytest.mark.parametrize("world,local_slice", [(2, False), (3, False), (2, True), (3, True)])
def test_sharded_protocol_matches_oracle(world, local_slice):
    cases = _cases(world, 12)
    res = _run(world, cases, local_slice)
    for k, (arr, ms, strategy, clean) in enumerate(cases):
        tr = [tuple(t) for t in arr]
        if strategy == 1 and not clean:
            uf = R.frequent_unary_conditions(tr, ms)
            v = R.all_at_once(R.join_lines(tr, uf, R.frequent_binary_conditions(tr, uf, ms)), ms, False,
                              literal_implies=False)
            expected = R.cind_set(R.s2l_exact_raw(v))
        else:
            expected = R.cind_set(R.rdfind(tr, ms, strategy, clean))
        parts = [set(res[r][k][1]) for r in range(world)]
        assert all(res[r][k][0] == 15 for r in range(world))  # the library's fifteen collectives (world > 1)
        union = set().union(*parts)
        assert sum(len(p) for p in parts) == len(union)      # every dependent has one owner
        assert union == expected, (k, ms, strategy, clean)


def test_exchange_helpers_gloo():
    """allgatherv (padded all-gather for balanced contributions, broadcasts for skewed ones) / alltoallv with ragged
    and empty contributions."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_helpers_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    got = dict(q.get(timeout=120) for _ in procs)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert got[0]["ag"] == [0, 1, 2, 10] and got[1]["ag"] == [0, 1, 2, 10]
    assert got[0]["empty"] == [] and got[1]["empty"] == []
    assert got[0]["skew"] == list(range(10)) + [77] and got[1]["skew"] == got[0]["skew"]
    # rank 0 sends [100] to 0 and [101, 102] to 1; rank 1 sends [] to 0 and [200] to 1
    assert got[0]["a2a"] == [100] and got[1]["a2a"] == [101, 102, 200]


def _helpers_worker(rank, world, port, q):
    import torch

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from rdfind_amd import distributed

    try:
        send = torch.tensor([0, 1, 2] if rank == 0 else [10], dtype=torch.int64)
        ag = distributed.allgatherv(send).tolist()
        empty = distributed.allgatherv(torch.zeros(0, dtype=torch.int64)).tolist()
        skew = distributed.allgatherv(torch.arange(10, dtype=torch.int64) if rank == 0 else  # broadcasts (skewed)
                                      torch.tensor([77], dtype=torch.int64)).tolist()
        if rank == 0:
            a2a = distributed.alltoallv(torch.tensor([100, 101, 102], dtype=torch.int64), [1, 2]).tolist()
        else:
            a2a = distributed.alltoallv(torch.tensor([200], dtype=torch.int64), [0, 1]).tolist()
        q.put((rank, {"ag": ag, "empty": empty, "skew": skew, "a2a": a2a}))
    finally:
        dist.destroy_process_group()


def test_allgatherv_compaction_in_place():
    """allgatherv's in-place compaction of the padded all-gather (no second result-sized copy): random ragged counts,
    gaps of one element between a slice's source and destination, and chunks much smaller than a slice."""
    import torch

    from rdfind_amd import distributed

    rng = random.Random(5)
    old = distributed._COMPACT_CHUNK_BYTES
    try:
        for it in range(300):
            distributed._COMPACT_CHUNK_BYTES = 8 * rng.choice([1, 2, 3, 7, 1000])
            world = rng.randrange(1, 9)
            counts = [rng.choice([0, rng.randrange(1, 20), 19]) for _ in range(world)]
            mx = max(counts + [1])
            buf = torch.full((world * mx,), -1, dtype=torch.int64)
            want = []
            for r, c in enumerate(counts):
                vals = torch.arange(c, dtype=torch.int64) + 1000 * r
                buf[r * mx: r * mx + c] = vals
                want += vals.tolist()
            tot = distributed._compact_in_place(buf, counts, mx)
            assert tot == sum(counts) and buf[:tot].tolist() == want, (counts, it)
    finally:
        distributed._COMPACT_CHUNK_BYTES = old


def _skew_worker(rank, world, port, q):
    import torch

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from rdfind_amd import distributed

    try:
        distributed._COMPACT_CHUNK_BYTES = 16  # 2 elements: many chunks per slice
        sizes = [6, 7, 0, 5][:world]
        send = torch.arange(sizes[rank], dtype=torch.int64) + 100 * rank
        q.put((rank, distributed.allgatherv(send).tolist()))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3, 4])
def test_allgatherv_skewed_contributions_gloo(world):
    """Ragged contributions (one rank empty) through the padded all-gather and its in-place compaction, over gloo."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_skew_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    got = dict(q.get(timeout=120) for _ in procs)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    sizes = [6, 7, 0, 5][:world]
    want = [100 * r + i for r in range(world) for i in range(sizes[r])]
    assert all(got[r] == want for r in range(world))


def _fail_worker(rank, world, port, q, fail_phase, where):
    import time

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from rdfind_amd import distributed
    from tests.shard_sim import ShardSim

    class Failing(ShardSim):  # rank 1 fails in its step, export or import at one phase
        def shard_step(self):
            if rank == 1 and where == "step" and self.phase == fail_phase:
                raise RuntimeError("test: step failed")
            return super().shard_step()

        def shard_import(self, ptr, n):
            if rank == 1 and where == "import" and self.phase == fail_phase:
                raise RuntimeError("test: import failed")
            return super().shard_import(ptr, n)

    t0 = time.perf_counter()
    try:
        arr = _cases(7, 1)[0][0]
        sim = Failing(arr, 1 + max(max(t) for t in arr))
        sim.shard_begin(rank, world, 2, "spo", True, 1)
        distributed.run_protocol(sim)
        q.put((rank, ("ok", time.perf_counter() - t0)))
    except Exception as e:
        q.put((rank, (f"{type(e).__name__}: {e}", time.perf_counter() - t0)))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,fail_phase,where", [(2, 14, "step"), (3, 5, "step"), (2, 6, "import"), (2, 8, "import")])
def test_rank_failure_agreement_gloo(world, fail_phase, where):
    """Cross-rank failure agreement of run_protocol (the header all-gather before each collective and at the end): a
    rank whose step or import raises announces it in the next header; every other rank raises PeerFailure there instead
    of waiting in a collective the failed rank never enters (import at phase 8: the last collective, caught by the final
    DONE header)."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_fail_worker, args=(r, world, port, q, fail_phase, where)) for r in range(world)]
    for p in procs:
        p.start()
    got = dict(q.get(timeout=120) for _ in procs)
    for p in procs:
        p.join(timeout=60)
    assert got[1][0].startswith("RuntimeError: test:"), got
    for r in range(world):
        if r != 1:
            assert got[r][0].startswith("PeerFailure") and "[1]" in got[r][0], got
    assert max(v[1] for v in got.values()) < 60, got
