"""Benchmark: CIND-discovery triples/s on MI355X (BASELINE.json metric), one JSON line on rank 0.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config c2] [--scale 1.0] [--scaling weak|strong]

A *step* is T_disc of SURVEY.md 8(d) / BASELINE.md 2 over one batch: from dictionary-encoded triples resident
in HBM to CIND id-records in host memory.  rdf_run = frequent conditions -> capture groups -> CIND extraction +
--clean-implied minimality (strategy 1, the reference default), then rdf_copy_result_compact hands the
CindSet-shaped result (explicit ref runs + the shared ref lists of the mask classes, ALG/data/CindSet.scala:9-13)
to pinned host memory.  `value` = triples / step time.  Workload at N = 1: BASELINE configs[1] = LUBM-100-shaped
synthetic triples (12.7M), support 10, one MI355X.  `device_resident` repeats the steps without the hand-over.

N > 1: one rank per GPU under torch.distributed.run (started by this script when no launcher is used), RCCL over
xGMI; the workload is sharded (rdfind_amd/distributed.py): each rank holds only its slice of the
triples (synth.config_slice), the condition counts are summed over ranks, every triple travels to the ranks
owning its join values, each rank builds the capture groups of its join-value hash shard and owns the
dependents by hash (dep_owner); the protocol's collectives run inside the timed region and every rank hands over its own
result.  Default weak scaling: N GPUs run the config at N x scale (c2: LUBM-(100 N)), so each GPU holds one
LUBM-100-sized share; `value` = all triples / max-over-ranks step time.  `roofline` is computed for the dominant
kernel family from HIP events recorded on the library's stream; `cpu_baseline` times the C restatement
(oracle/, OpenMP) on rank 0.

`c4_strong` (default with the c2 workload; `--c4-strong off` skips it): BASELINE configs[3], c4 at 10^9 triples,
split over the same N GPUs (strong scaling, the north-star scaling config), after the main leg: each rank draws only
its 1/N of the rows, a rank whose join shard holds >= 2^32/9 triples builds its groups in join ranges, and the step is
the same T_disc with every rank's result handed over.  It reports ms per step, triples/s, the ranks' work balance
(max / mean) and the one-GPU c4 step of round 5 (0.852 s; round 4: 1.616 s) as its reference; `value` stays the c2 leg's.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E peak (MI355X_MICROARCH.md chip-level parameters)
RADIX_MAX_BITS = 9     # widest radix digit of the library's sorts (rdfind_amd/csrc/primitives.hip RS_MAX_BITS)


def sort_passes(bits):
    """Digit passes of a library sort of `bits` key bits (primitives.hip: digits of <= RS_MAX_BITS bits)."""
    return -(-bits // RADIX_MAX_BITS)

# timer family -> its kernels, whose rocprofv3 PMC traffic (profiles/pmc_<config>.json, tools/pmc.sh) is summed
FAMILY_KERNELS = {
    "unary": ["k_u2_part", "k_u2_slices", "k_u2_count", "k_u2_finish", "k_u2_fval"],
    "binary": ["k_b2_part", "k_b2_slices", "k_b2_count", "k_spill_insert", "k_bin_freq_flags", "k_bin_freq_scatter",
               "k_bin_lookup_build"],
    "emit": ["k_emit_records", "k_emit_compact"],
    "support": ["k_fresh_bounds", "k_cstart_fix", "k_run_support", "k_support_flags", "k_compact_captures",
                "k_skip_counts", "k_keep_scatter"],
    "groups": ["k_key_offsets", "k_group_flags", "k_group_build", "k_dgrp"],
    "pivot": ["k_group_info", "k_pivot_nseg", "k_pivot_short", "k_pivot_seg", "k_pivot_final", "k_dup_insert", "k_dup_rep",
              "k_dup_verify", "k_dup_unplan"],
    "light": ["k_light", "k_light_stage", "k_light_plain", "k_light_packed", "k_light_mseg_emit", "k_mseg_chunks", "k_slot_compact"],
    "rules": ["k_rules_explicit", "k_rules_mark", "k_compact_refs"],
    "cemit": ["k_class_emit"],
}
# CPU baseline sample per config: the streamed C restatement runs ~10-30 s on the box's threads at these scales
# (c1/c2: the whole workload; c5 grows super-linearly with its pair explosion)
CPU_SAMPLE_SCALE = {"c1": 1.0, "c2": 1.0, "c3": 0.1, "c4": 0.02, "c5": 0.05}
PMC_STEP_KERNEL = "k_pivot_final"  # launched once per discovery step: the number of steps in the PMC run


def pmc_traffic(config, family):
    """HBM bytes per step of the family's kernels from the committed PMC summary (FETCH_SIZE x2 + WRITE_SIZE,
    corrected as MI355X_MICROARCH.md prescribes; per-launch averages x launches / steps of that run), or None when
    no summary for this config is committed.  The radix sort (shared by several sorts) has no per-family split."""
    path = os.path.join(ROOT, "profiles", f"pmc_{config}.json")
    ks = FAMILY_KERNELS.get(family)
    if not ks or not os.path.exists(path):
        return None
    pmc = json.load(open(path))
    steps = pmc.get(PMC_STEP_KERNEL, {}).get("launches")
    if not steps:
        return None
    tot = sum(pmc[k]["hbm_bytes"] * pmc[k]["launches"] for k in ks if k in pmc)
    return int(tot / steps) if tot else None


def algorithmic_bytes(name, d, fc, gs, cs, counts):
    """Minimal HBM bytes a kernel family must move per step ('Algorithmic bytes'), or None
    for families without a formula (tiny bookkeeping kernels)."""
    n, V = d.n, d.num_terms
    J, Jf = gs["n_records"], gs["n_frequent_records"]
    E = cs["n_explicit_raw"]
    if name == "unary":
        return 12 * n + 12 * V                          # read s, p, o once; write 3 counters per term
    if name == "binary":
        return 12 * n + 12 * fc["n_binary_keys"]        # read the triples; one (8-B key, 4-B count) per distinct key
    if name == "emit":
        return 12 * n + 8 * J                           # read triples, write (join, capture) records
    if name == "sort":
        return 16 * counts["sort_passes_records"]       # read + write each record once per digit pass
    if name == "support":
        Js = gs.get("n_sorted_records", J)              # the sorted records (an emission iteration's repeats dropped)
        return 12 * Js + 16 * Jf                        # read records + write fresh flags; dk + fk per kept record
    if name == "groups":
        return 16 * Jf * counts["group_passes"] + 32 * Jf   # fk sort passes; flags/build/gcap/dgrp gathers
    if name == "pivot":
        return 12 * Jf                                  # per (dependent, group): group id + its bounds
    if name == "light":
        # every candidate (pivot member) and every group entry of a light dependent read once, each explicit pair
        # written to its slot, read and written compacted
        return 4 * cs["n_light_candidates"] + 4 * cs["n_light_entries"] + 24 * E
    if name == "rules":
        return 16 * E                                   # read each explicit pair, keep flag, compacted ref
    if name == "cemit":
        return 4 * cs["n_class_cinds"]                  # 4-B ref per CIND written (dependent-run output); the shared
                                                        # class lists (< 1 MB) are read from L2
    if name == "hcount":
        return 20 * cs["n_heavy_candidates"] + 12 * cs["n_heavy_chunks"]  # candidate id + 16-B info; chunk bits + counts
    if name == "hwrite":
        return 8 * cs["n_heavy_candidates"]             # candidate id read, <= one 4-B output per candidate
    return None


def family_rooflines(d, fc, gs, cs, kt, counts):
    out = {}
    for name, ms in kt.items():
        b = algorithmic_bytes(name, d, fc, gs, cs, counts)
        if b is None or ms <= 0:
            continue
        gbs = b / (ms * 1e-3) / 1e9
        out[name] = {"ms": round(ms, 4), "bytes": int(b), "achieved": round(gbs, 1), "frac": round(gbs / HBM_PEAK_GBS, 4)}
    return out


class CompactSink:
    """Pinned host buffers for the compact CindSet-shaped result (rdf_copy_result_compact): the id-records the
    metric's T_disc ends with.  Sized from the first run's layout, grown if a run needs more.  A result
    with more explicit refs than STREAM_REFS (the pages of c5 at full size: up to 10^10 refs each) streams them through
    one bounded pinned staging buffer (rdf_copy_result_refs), as a sink consuming its input would; page-locking tens of
    GB per page cost more than the copies."""

    STREAM_REFS = 1 << 28  # 1 GiB of u32 refs

    def __init__(self, early=True):
        self.bufs, self.cap, self.pinned, self._keep = None, {}, True, []
        self.early = early  # register the pinned buffers for the library's early hand-over (rdf_set_handover)
        self.heavy, self.heavy_cap, self.heavy_chunks = {}, 0, 0  # the heavy-bits form's chunks (rdf_copy_result_heavy)

    def register(self, ctx):
        """The unpaged discoveries that follow fill the refs and the capture table of these buffers while they still
        compute (rdf_set_handover); copy() then moves only the rest."""
        if self.early and self.pinned and self.bufs is not None:
            ctx.set_handover(self.bufs["refs"], self.cap["refs"], self.bufs["runoff"], self.bufs["rundep"],
                             min(self.cap["runoff"] - 1, self.cap["rundep"]), self.bufs["capture_ids"],
                             self.bufs["supports"], min(self.cap["capture_ids"], self.cap["supports"]))

    def ensure(self, ctx):
        from rdfind_amd import _lib
        L = ctx.result_layout()
        grown = False
        if self.bufs is None:
            self.bufs, self._keep = {}, {}
        for name, dt, count in _lib.COMPACT_PARTS:  # only a part that outgrew its buffer is re-allocated
            need = max(count(L), 1)
            if name == "refs":
                need = min(need, self.STREAM_REFS)
            if name in self.cap and need <= self.cap[name]:
                continue
            if name in self.cap:  # grow with headroom: page-locking is slow
                need = max(need, self.cap[name] + self.cap[name] // 2)
                if name == "refs":
                    need = min(need, self.STREAM_REFS)
            self._keep.pop(name, None)
            try:  # page-locked memory from the library (rdf_host_alloc)
                b = _lib.PinnedBuffer(need, dt)
                self._keep[name] = b
                self.bufs[name] = b.ptr
            except _lib.RdfError:  # no pinned memory: pageable numpy (slower link rate, stated in the line)
                self.pinned = False
                a = np.empty(need, dt)
                self._keep[name] = a
                self.bufs[name] = a.ctypes.data
            self.cap[name] = need
            grown = True
        if grown:
            self.register(ctx)
        return L

    def copy_heavy(self, ctx):
        """The heavy-bits form's part: one (dependent, list position, survivor word) per chunk of 64 class-list
        candidates (rdf_copy_result_heavy), into pinned buffers grown like the others."""
        from rdfind_amd import _lib
        nh = ctx.heavy_chunk_count()
        self.heavy_chunks = nh
        if not nh:
            return
        if nh > self.heavy_cap:
            need = max(nh, self.heavy_cap + self.heavy_cap // 2)
            self.heavy = {}
            for name, dt in (("deps", np.uint32), ("pos", np.uint64), ("bits", np.uint64)):
                self.heavy[name] = _lib.PinnedBuffer(need, dt)
            self.heavy_cap = need
        ctx.copy_result_heavy(self.heavy["deps"].ptr, self.heavy["pos"].ptr, self.heavy["bits"].ptr)

    def copy(self, ctx, overlap=False):
        """overlap (pages): the refs are queued on the library's copy stream (rdf_copy_result_refs_async) and leave
        while the next page computes; the caller ends with ctx.handover_wait()."""
        L = self.ensure(ctx)
        self.copy_heavy(ctx)
        if L["n_refs"] <= self.cap["refs"] and not (overlap and self.pinned):
            ctx.copy_result_compact(self.bufs)
            return L
        ctx.copy_result_compact(dict(self.bufs, refs=0))  # everything but the refs, which stream in chunks
        off = 0
        while off < L["n_refs"]:
            if overlap and self.pinned:
                off += ctx.copy_result_refs_async(off, self.cap["refs"], self.bufs["refs"])
            else:
                off += ctx.copy_result_refs(off, self.cap["refs"], self.bufs["refs"])
        return L


def layout_bytes(L, heavy_chunks=0):
    return (4 * L["n_refs"] + 12 * L["n_runs"] + 8 + 4 * L["n_list_refs"] + 8 * (L["n_lists"] + 1) +
            8 * L["n_members"] + 8 * L["n_captures"] + 20 * heavy_chunks)


def ctx_pages(ctx):
    """Pages of the last paged run (rdf_next_page calls that produced a page)."""
    return getattr(ctx, "_pages", None)


def launch_ranks(nranks, argv):
    """--gpus N without a launcher: one rank per GPU under torch.distributed.run, started as child processes before
    this process touches a GPU (rdfind_amd/program.py launch_ranks); returns their exit status."""
    import socket
    import subprocess
    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={nranks}",
           "--master-addr=127.0.0.1", f"--master-port={port}", os.path.abspath(__file__)] + list(argv)
    return subprocess.run(cmd, env=dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0")).returncode


def per_rank_balance(dist, world, mine):
    """Every rank's work counters (all-gathered) and max / mean over ranks per numeric quantity."""
    allr = [None] * world
    dist.all_gather_object(allr, mine)
    return {"per_rank": allr,
            "max_over_mean": {k: round(max(r[k] for r in allr) / max(sum(r[k] for r in allr) / world, 1e-12), 3)
                              for k in mine if all(isinstance(r.get(k), (int, float)) for r in allr)}}


# the one-GPU c4 step this leg is compared with: round 6 (digit-row scans, K1's radix form, vectorized scans, the wider
# emission grid), the c4_strong leg of profiles/r06_bench_c2.json (earlier in round 6: 819.6 and 789.6 ms, round 5: 830.8, round 4: 1616)
C4_ONE_GPU_MS = 787.9


def c4_golden(scale):
    """The committed golden entry (count, set checksum) of c4 at this scale, strategy 1 --clean-implied, or None."""
    g = json.load(open(os.path.join(ROOT, "tests", "golden", "full_size.json")))
    key = "c4@1.0/s1_clean" if scale == 1.0 else f"c4@{scale}/s1_clean"
    return g.get(key)


def c4_strong_leg(args, dist, rank, world, local_rank, barrier, max_over_ranks):
    """BASELINE configs[3] (c4 at 10^9 triples, support 100) split over the N ranks -- strong scaling, the north-star
    scaling config.  Each rank draws and holds only its 1/N of the rows (synth.config_slice); a rank whose join shard
    holds >= 2^32/9 triples builds its groups in join ranges (N = 1, 2, 4).  Same step as the main leg: T_disc with every
    rank's compact result handed to pinned host memory."""
    from rdfind_amd import _lib, synth

    scale = args.c4_scale
    if dist is not None:
        d, total_n = synth.config_slice("c4", scale, rank, world)
    else:
        d = synth.config("c4", scale)
        total_n = d.n
    ms = d.min_support
    n_local = d.n
    sink = CompactSink()
    with _lib.Context(local_rank) as ctx:
        ctx.set_triples(d.s, d.p, d.o, d.num_terms)
        del d
        if dist is not None:
            from rdfind_amd import distributed

            def step():
                distributed.run_sharded(ctx, ms, local_slice=True)
                sink.copy(ctx)
                return ctx.cinds
        else:
            def step():
                cs = ctx.run(ms)
                sink.copy(ctx)
                return cs
        for _ in range(args.c4_warmup):
            step()
        ctx.sync()
        barrier()
        kt_sum = {}
        t0 = time.perf_counter()
        for _ in range(args.c4_steps):
            cs = step()
            for k, v in ctx.kernel_times().items():
                kt_sum[k] = kt_sum.get(k, 0.0) + v
        ctx.sync()
        barrier()
        elapsed = max_over_ranks(time.perf_counter() - t0)
        steps = max(args.c4_steps, 1)
        checksum = ctx.checksum()  # this rank's set checksum (rdf_cind_checksum; the ranks' sets are disjoint)
        gs = ctx.groups
        kt = {k: v / steps for k, v in kt_sum.items()}
        mine = {"triples": n_local, "records": gs["n_records"], "join_ranges": gs.get("n_join_ranges", 1),
                "ranges_kept": gs.get("n_ranges_kept", 0), "groups": gs["n_groups"], "light_chunks": cs["n_light_chunks"], "explicit_raw": cs["n_explicit_raw"],
                "cinds": cs["n_cinds"], "light_ms": round(kt.get("light", 0.0), 3),
                "kernel_ms": round(sum(kt.values()), 3), "hbm_held_gib": round(ctx.device_bytes() / 2**30, 1),
                **{k: v for k, v in (getattr(ctx, "x_stats", None) or {}).items() if k in ("bytes_sent", "bytes_received")}}
    total_cinds = cs["n_cinds"]
    total_checksum = checksum
    bal = None
    if dist is not None:
        bal = per_rank_balance(dist, world, mine)
        total_cinds = sum(r["cinds"] for r in bal["per_rank"])
        sums = [None] * world
        dist.all_gather_object(sums, checksum)
        total_checksum = sum(sums) % (1 << 64)
    ms_step = elapsed * 1000.0 / steps
    golden = c4_golden(scale)
    return {"workload": f"c4 (Freebase-shaped) scale {scale}: {total_n} triples split over {world} GPU(s), support {ms}, "
                        "strategy 1 --use-fis --clean-implied",
            "scaling": "strong", "n_gpus": world, "steps": args.c4_steps, "warmup": args.c4_warmup,
            "ms_per_step": round(ms_step, 3), "triples_per_s": round(total_n * steps / elapsed, 1), "cinds": total_cinds,
            "checksum": str(total_checksum),
            # the ranks' summed CIND count and set checksum against the committed golden of the streamed C oracle
            # (tests/golden/full_size.json, read as data): the same set at every N
            "matches_golden": None if golden is None else bool(total_cinds == golden["n_cinds"] and
                                                               total_checksum == int(golden["checksum"])),
            "golden": None if golden is None else f"tests/golden/full_size.json c4@{scale}/s1_clean",
            "one_gpu_ms_ref": C4_ONE_GPU_MS if scale == 1.0 else None,
            "speedup_vs_one_gpu_ref": round(C4_ONE_GPU_MS / ms_step, 3) if scale == 1.0 else None,
            "kernel_ms_rank0": {k: round(v, 3) for k, v in kt.items()}, "rank0": mine,
            **({"ranks": bal} if bal else {})}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=None, help="GPUs (ranks); default: WORLD_SIZE or 1.  Without a "
                    "launcher, N > 1 starts N ranks under torch.distributed.run itself")
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--config", default="c2")
    ap.add_argument("--scale", type=float, default=1.0, help="per-GPU scale of the config (weak scaling) or the "
                    "total scale (--scaling strong)")
    ap.add_argument("--scaling", choices=("weak", "strong"), default="weak",
                    help="weak: every GPU holds one config-sized share (N GPUs run the config at N x scale); "
                         "strong: the config at scale is split over the GPUs")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-ingest", action="store_true", help="skip the N-Triples ingest leg (rank 0, N=1)")
    ap.add_argument("--cpu-sample-scale", type=float, default=None,
                    help="scale of the config the CPU baseline runs (default: CPU_SAMPLE_SCALE, ~10-30 s of CPU work)")
    ap.add_argument("--cpu-full-max", type=int, default=20_000_000,
                    help="time the CPU baseline on the benchmarked workload itself up to this many triples")
    ap.add_argument("--backend", default="nccl", help="process-group backend for N > 1 (gloo: host-staged "
                    "exchanges, to rehearse several ranks on one GPU)")
    ap.add_argument("--no-resident", action="store_true", help="skip the device-resident repeat of the steps")
    ap.add_argument("--no-early-handover", action="store_true", help="hand the whole result over after each run "
                    "(no rdf_set_handover: the refs and the capture table are not copied while the run computes)")
    ap.add_argument("--page-log", action="store_true", help="one progress line per page on stderr (paged runs)")
    ap.add_argument("--expanded-heavy", action="store_true", help="hand the heavy-only dependents' CINDs over as one "
                    "u32 ref each (default: RDF_FORM_HEAVY_BITS, a survivor word per 64 class-list candidates)")
    ap.add_argument("--no-page-overlap", action="store_true", help="paged runs: hand each page's refs over before the "
                    "next page starts (default: queued on the copy stream while the next page computes)")
    ap.add_argument("--no-numa-bind", action="store_true", help="leave the process on every CPU (default: bound to the "
                    "GPU's NUMA node before any host buffer is allocated, rdfind_amd/numa.py)")
    ap.add_argument("--c4-strong", choices=("auto", "on", "off"), default="auto",
                    help="also time BASELINE configs[3] (c4, Freebase-shaped, 10^9 triples, support 100) split over the "
                         "N GPUs (strong scaling; the north-star scaling config) and report it as `c4_strong` (auto: "
                         "when N > 1 with the default c2 workload and the nccl backend)")
    ap.add_argument("--c4-scale", type=float, default=1.0, help="scale of the c4_strong leg (1.0 = 10^9 triples)")
    ap.add_argument("--c4-steps", type=int, default=2)
    ap.add_argument("--c4-warmup", type=int, default=1)
    ap.add_argument("--c4-deadline", type=float, default=420.0,
                    help="seconds the c4_strong leg may take; past it rank 0 prints the line with the c2 leg's "
                         "measurement and c4_strong.error, and every rank exits (the line is never lost to a hang)")
    ap.add_argument("--pg-timeout", type=float, default=300.0, help="process-group timeout (seconds) for N > 1")
    ap.add_argument("--page-bytes", type=int, default=None,
                    help="paged discovery (rdf_discover_cinds_paged) with this working memory per page, 0 = "
                         "automatic; every page is handed over in turn.  Default: unpaged, or automatic pages when the "
                         "unpaged run exceeds HBM (RDF_ERR_OOM; c5 beyond scale 0.3)")
    args = ap.parse_args()

    env_world = os.environ.get("WORLD_SIZE")
    if env_world is None and (args.gpus or 1) > 1:  # self-launch before any GPU call
        sys.exit(launch_ranks(args.gpus, sys.argv[1:]))
    world = int(env_world or 1)
    if args.gpus is not None and args.gpus != world:
        print(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world}", file=sys.stderr)
        sys.exit(2)
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    import torch

    local_rank %= max(torch.cuda.device_count(), 1)
    if not args.no_numa_bind:  # host buffers on the GPU's NUMA node (rdfind_amd/numa.py)
        from rdfind_amd import numa

        numa.bind_to_device_node(local_rank)
    if world > 1:
        import torch.distributed as dist

        torch.cuda.set_device(local_rank)
        import datetime
        # a rank lost inside a collective ends the run after this long (gloo raises; RCCL's watchdog aborts the
        # process) instead of leaving its peers waiting; failures outside collectives are agreed on at once
        # (rdfind_amd/distributed.py run_protocol)
        dist.init_process_group(args.backend, timeout=datetime.timedelta(seconds=args.pg_timeout))

    from rdfind_amd import _lib, synth

    total_scale = args.scale * world if args.scaling == "weak" else args.scale
    if dist is not None:  # each rank holds only its slice of the input (sharded input)
        d, total_n = synth.config_slice(args.config, total_scale, rank, world)
    else:
        d = synth.config(args.config, total_scale)
        total_n = d.n
    ms = d.min_support
    ctx = _lib.Context(local_rank)
    ctx.set_triples(d.s, d.p, d.o, d.num_terms)  # inputs resident in HBM before the timed region
    sink = CompactSink(early=not args.no_early_handover)
    # the heavy-only binary dependents' CINDs hand over as survivor words over their class lists (rdf_set_result_form;
    # --expanded-heavy: one u32 ref each)
    ctx.set_result_form(not args.expanded_heavy)

    paged = dist is None and args.page_bytes is not None
    if dist is None and not paged:  # a result larger than HBM: the unpaged run fails with RDF_ERR_OOM -> pages
        try:
            ctx.run(ms)
        except _lib.RdfError as e:
            if e.status != _lib.RDF_ERR_OOM:
                raise
            print("bench.py: the unpaged result exceeds HBM; paged discovery", file=sys.stderr, flush=True)
            ctx.release_scratch()
            paged = True
    if dist is not None:
        from rdfind_amd import distributed

        def discover(hand_over):
            distributed.run_sharded(ctx, ms, local_slice=True)
            if hand_over:
                sink.copy(ctx)
            return ctx.cinds
    elif paged:  # pages of bounded HBM, each handed over before the next (the reference streams to its sink)
        def discover(hand_over):
            ctx.frequent_conditions(ms)
            ctx.build_capture_groups("spo")
            n = 0
            t_page = time.perf_counter()
            for i, _ in enumerate(ctx.pages(True, 1, args.page_bytes or 0)):
                n += ctx.cind_count()
                t_copy = time.perf_counter()
                if hand_over:  # a page's refs leave while the next page computes (--no-page-overlap: in turn)
                    sink.copy(ctx, overlap=not args.no_page_overlap)
                if args.page_log:
                    _, pcs = ctx.last_stats()
                    t_end = time.perf_counter()
                    print(f"page {i}: {n} CINDs so far, explicit raw {pcs['n_explicit_raw']}, "
                          f"HBM held {ctx.device_bytes() / 2**30:.1f} GiB, page {t_copy - t_page:.2f} s, "
                          f"hand-over {t_end - t_copy:.2f} s", file=sys.stderr, flush=True)
                    t_page = time.perf_counter()
            ctx.handover_wait()  # the last page's refs are in host memory
            _, cs = ctx.last_stats()
            return dict(cs, n_cinds=n, pages=ctx_pages(ctx))
    else:
        def discover(hand_over):
            cs = ctx.run(ms)
            if hand_over:
                sink.copy(ctx)
            return cs

    def step():  # T_disc: encoded triples in HBM -> compact CIND id-records in (pinned) host memory
        return discover(True)

    def barrier():
        if dist is not None:
            import torch
            dist.barrier()
            torch.cuda.synchronize()

    def max_over_ranks(x):
        if dist is None:
            return x
        import torch
        dev = f"cuda:{local_rank}" if args.backend == "nccl" else "cpu"
        t = torch.tensor([x], device=dev, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        return float(t.item())

    t_w = time.perf_counter()
    for _ in range(args.warmup):
        step()
    # untimed spin-up beyond W until ~0.25 s of steps have run (a fresh box's first steps run slow: clocks, caches);
    # one GPU only: with several ranks every rank must run the same number of (collective) steps
    for _ in range(50 if args.warmup and dist is None else 0):
        if time.perf_counter() - t_w > 0.25:
            break
        step()
    ctx.sync()
    barrier()
    kt_sum = {}
    t0 = time.perf_counter()
    for _ in range(args.steps):
        cs = step()
        for k, v in ctx.kernel_times().items():
            kt_sum[k] = kt_sum.get(k, 0.0) + v
    ctx.sync()
    barrier()
    elapsed = max_over_ranks(time.perf_counter() - t0)
    L = ctx.result_layout()
    # the same steps without the hand-over (results left in HBM): the device-resident rate
    elapsed_dev = None
    if not args.no_resident:
        ctx.set_handover()  # results stay in HBM: no early copies either
        barrier()
        t1 = time.perf_counter()
        for _ in range(args.steps):
            discover(False)
        ctx.sync()
        barrier()
        elapsed_dev = max_over_ranks(time.perf_counter() - t1)
    if dist is not None:
        import torch
        dev = f"cuda:{local_rank}" if args.backend == "nccl" else "cpu"
        tot = torch.tensor([cs["n_cinds"], layout_bytes(L, sink.heavy_chunks)], device=dev, dtype=torch.int64)
        dist.all_reduce(tot)
        total_cinds, total_bytes = (int(x) for x in tot.tolist())
    else:
        total_cinds, total_bytes = cs["n_cinds"], layout_bytes(L, sink.heavy_chunks)
    steps = max(args.steps, 1)
    ms_per_step = elapsed * 1000.0 / steps
    value = float(total_n) * steps / elapsed

    gs, fc = ctx.groups, ctx.fc
    kt = {k: v / steps for k, v in kt_sum.items()}
    # passes of the record sort (bits = join bits + capture bits, 8 per pass) and of the group sort (join bits)
    V = d.num_terms
    capbits = int(2 * sum(fc["n_frequent_unary"]) + fc["n_frequent_binary"] - 1).bit_length()  # compact capture ids
    joinbits = max(int(V - 1).bit_length(), 1)
    # the first pass reads every emitted record slot, the others only the records it kept (repeats dropped)
    counts = {"sort_passes_records": gs["n_records"] + (sort_passes(capbits + joinbits) - 1) * gs["n_sorted_records"],
              "group_passes": sort_passes(joinbits)}
    fams = family_rooflines(d, fc, gs, cs, kt, counts)
    if total_scale == 1.0 and world == 1:  # HBM bytes per step from the committed PMC summary of this config
        for name, f in fams.items():
            t = pmc_traffic(args.config, name)
            if t is not None:
                f["traffic"] = t
                f["traffic_x"] = round(t / f["bytes"], 2) if f["bytes"] else None
    dominant = max(kt, key=lambda k: kt[k])
    roof = None
    for name in [dominant] + sorted(kt, key=lambda k: -kt[k]):
        if name in fams:
            f = fams[name]
            roof = {"bound": "hbm", "kernel": name, "achieved": f["achieved"], "peak": HBM_PEAK_GBS, "unit": "GB/s",
                    "frac": f["frac"], "traffic": f.get("traffic"), "ms": f["ms"], "bytes_per_launch": f["bytes"],
                    "dominant_kernel": dominant, "dominant_ms": round(kt[dominant], 4)}
            break

    # BASELINE metric also names "% HBM roofline of count kernels": K1 (unary) and K2 (binary condition counts)
    count_roof = {k: dict(fams[k], bound="hbm") for k in ("unary", "binary") if k in fams}

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        from oracle import c_oracle

        # the same workload when the streamed C restatement finishes in ~30 s on the box's threads, else a sample
        cpu_scale = args.cpu_sample_scale or min(total_scale, CPU_SAMPLE_SCALE.get(args.config, 0.3))
        if d.n <= args.cpu_full_max and args.config in ("c1", "c2"):
            cpu_scale = total_scale  # the benchmarked workload itself
        sd = d if cpu_scale == total_scale else synth.config(args.config, cpu_scale)
        t = time.perf_counter()
        r = c_oracle.stream(sd.s, sd.p, sd.o, sd.num_terms, sd.min_support, 1, True)
        ct = time.perf_counter() - t
        nt = c_oracle.threads()
        same = cpu_scale == total_scale
        cpu = {"value": round(sd.n / ct, 1), "unit": "triples/s", "cores": nt, "kind": "port",
               "sample": f"{args.config} scale {cpu_scale} ({sd.n} triples, {r['n_cinds']} CINDs"
                         f"{', the benchmarked workload itself' if same else ''}) through oracle/c/rdfind_oracle.c "
                         f"(streamed count + checksum, same stages incl. minimality) on {nt} OpenMP threads, {ct:.1f}s"}
        if same and not paged:
            parts = ctx.copy_result_compact()  # the hand-over the timed steps copied, expanded by the checker
            n_c, h_c, _ = c_oracle.checksum_compact(parts, d.num_terms)
            cpu["matches_gpu"] = bool(r["n_cinds"] == n_c == cs["n_cinds"] and r["checksum"] == h_c)

    ingest = None
    # one rdf_parse_ntriples call holds < 2^31 term occurrences (its table has 2x as many u32-indexed slots), and the
    # text is built in host memory (~170 B per triple): the ingest leg is for inputs up to 2 * 10^8 triples
    if rank == 0 and world == 1 and not args.no_ingest and d.n > 200_000_000:
        ingest = {"skipped": f"{d.n} triples: beyond one parse call's term table (< 2^31 occurrences) and the text's "
                             "host memory; the ingest leg runs up to 2e8 triples"}
    elif rank == 0 and world == 1 and not args.no_ingest:
        # parse/encode timed separately -- the same triples as N-Triples text through
        # rdf_parse_ntriples (ids/terms are checked by tests/)
        tt = d.terms.term
        strs = np.array([tt(i) + " " for i in range(d.num_terms)], dtype=object)
        text = "".join(map("".join, zip(strs[d.s], strs[d.p], strs[d.o], [".\n"] * d.n))).encode()
        del strs
        pt, wt = [], []
        for _ in range(3):
            t0 = time.perf_counter()
            n_parsed, n_terms, pms = ctx.parse_ntriples(text)
            wt.append((time.perf_counter() - t0) * 1e3)
            pt.append(pms)
        pms, wms = sorted(pt)[1], sorted(wt)[1]
        assert n_parsed == d.n
        ingest = {"ms": round(pms, 3), "text_bytes": len(text), "gbs_text": round(len(text) / pms / 1e6, 1),
                  "triples_per_s": round(d.n / pms * 1e3, 1), "terms": n_terms,
                  "wall_ms_incl_h2d": round(wms, 3), "t_disc_plus_ingest_ms": round(pms + ms_per_step, 3),
                  "note": "ms: rdf_parse_ntriples device time (median of 3), text already in HBM; wall_ms_incl_h2d: "
                          "the same call timed on the host, including the text's upload from pageable memory"}
        del text

    # per-rank work and time (N > 1): the balance of the sharded ownership, max / mean over ranks per quantity
    ranks = None
    if dist is not None:
        mine = {"triples": d.n, "records": gs["n_records"], "groups": gs["n_groups"],
                "light_chunks": cs["n_light_chunks"], "explicit_raw": cs["n_explicit_raw"], "cinds": cs["n_cinds"],
                "light_ms": round(kt.get("light", 0.0), 4), "kernel_ms": round(sum(kt.values()), 4),
                **{k: v for k, v in (getattr(ctx, "x_stats", None) or {}).items() if k in ("bytes_sent", "bytes_received")}}
        ranks = per_rank_balance(dist, world, mine)

    ctx.close()
    line = None
    if rank == 0:
        per = "per GPU" if args.scaling == "weak" else "total"
        wl = {"c2": "LUBM-shaped"}.get(args.config, args.config)
        line = {
            "metric": "CIND-discovery triples/sec", "value": round(value, 1), "unit": "triples/s",
            "n_gpus": world, "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(ms_per_step, 3),
            "higher_is_better": True, "scaling": args.scaling if world > 1 else "weak", "vs_baseline": None,
            "dtype": "u32", "data": "synthetic",
            "config": {"workload": f"{args.config} ({wl}, scale {args.scale} {per}: {total_n} triples over {world} GPU(s), "
                                   f"support {ms}, strategy 1 --use-fis --clean-implied)",
                       "triples": total_n, "triples_rank0": d.n, "cinds": total_cinds, "cinds_rank0": cs["n_cinds"],
                       "parallelism": f"input slices + join-hash shards x{world} (RCCL)" if world > 1 else "single"},
            "step": "T_disc (SURVEY.md 8(d)): dictionary-encoded triples resident in HBM -> compact CindSet-shaped "
                    "id-records (rdf_copy_result_compact) in pinned host memory, every rank" +
                    (" (paged: every page handed over in turn)" if paged else ""),
            "handover": {"bytes_all_ranks": total_bytes, "pinned": sink.pinned, "early": sink.early and sink.pinned,
                         "n_refs": L["n_refs"], "heavy_chunks": sink.heavy_chunks,
                         "n_list_refs": L["n_list_refs"], "n_members": L["n_members"], "n_runs": L["n_runs"]},
            "device_resident": None if elapsed_dev is None else
                               {"ms_per_step": round(elapsed_dev * 1000.0 / steps, 3),
                                "triples_per_s": round(float(total_n) * steps / elapsed_dev, 1),
                                "note": "the same steps with the result left in HBM"},
            "roofline": roof, "count_kernels": count_roof, "families": fams,
            "cpu_baseline": cpu, "ingest": ingest, **({"ranks": ranks} if ranks else {}),
            "kernel_ms": {k: round(v, 4) for k, v in kt.items()},
            "work": {"records": gs["n_records"], "groups": gs["n_groups"], "captures": gs["n_captures"],
                     "join_ranges": gs.get("n_join_ranges", 1), "ranges_kept": gs.get("n_ranges_kept", 0),
                     "heavy_groups": gs["n_heavy_groups"], "light_chunks": cs["n_light_chunks"],
                     "explicit_raw": cs["n_explicit_raw"], "heavy_chunks": cs["n_heavy_chunks"],
                     "heavy_candidates": cs["n_heavy_candidates"], "class_members": cs["n_class_members"],
                     "classes": cs["n_classes"], "class_cinds": cs["n_class_cinds"],
                     **({"exchange_rank0": getattr(ctx, "x_stats", None)} if world > 1 else {})},
        }
    want_c4 = args.c4_strong == "on" or (args.c4_strong == "auto" and args.config == "c2"
                                         and (world == 1 or args.backend == "nccl"))
    if want_c4:
        if line is not None:  # the main leg's measurement, on record before the c4 leg starts (stderr)
            print("bench.py: main leg: " + json.dumps(line), file=sys.stderr, flush=True)
        import threading

        def expire():  # the c4 leg hangs (a rank lost inside a collective): the line goes out without it
            if line is not None:
                line["c4_strong"] = {"error": f"the c4_strong leg exceeded --c4-deadline {args.c4_deadline:.0f} s; "
                                              "every rank stopped"}
                print(json.dumps(line), flush=True)
            sys.stderr.flush()
            os._exit(0)

        timer = threading.Timer(args.c4_deadline, expire)
        timer.daemon = True
        timer.start()
        try:
            c4 = c4_strong_leg(args, dist, rank, world, local_rank, barrier, max_over_ranks)
        except Exception as e:  # reported in the line; the main leg's measurement stands
            c4 = {"error": f"{type(e).__name__}: {e}"[:500]}
        timer.cancel()
        if line is not None:
            line["c4_strong"] = c4
    if line is not None:
        print(json.dumps(line), flush=True)
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
