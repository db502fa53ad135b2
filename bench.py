"""Benchmark: CIND-discovery triples/s on MI355X (BASELINE.json metric), one JSON line on rank 0.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config c2] [--scale 1.0]

A *step* is one pass of the hot path over one batch: rdf_run = frequent conditions -> capture groups
-> CIND extraction + --clean-implied minimality (strategy 1, the reference default), with the
dictionary-encoded triples already resident in HBM and the CIND id-records left in HBM (the
PCIe-inclusive rate is reported separately in DESIGN.md).  Workload: BASELINE configs[1] =
LUBM-100-shaped synthetic triples (~13.4M), support 10, one MI355X.

For N > 1 (launched by torch.distributed.run, one rank per GPU, RCCL over xGMI) the SAME workload is
sharded (rdfind_amd/distributed.py): every rank holds the triples, owns the capture groups
of its join-value hash shard and the dependents d % N, and the eight collectives of the protocol run
inside the timed region.  `value` is the workload's triples divided by the max-over-ranks time per
step (strong scaling).  `roofline` is computed for the dominant kernel family from HIP events recorded on
the library's stream; `cpu_baseline` times the C restatement (oracle/, OpenMP) on a bounded sample on rank 0.
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

# timer family -> the kernel whose rocprofv3 PMC traffic (profiles/pmc_<config>.json, tools/pmc.sh) is reported
FAMILY_KERNEL = {"cemit": "k_class_emit", "light": "k_light", "unary": "k_unary_count", "emit": "k_emit_records",
                 "sort": "k_radix_scatter", "hwrite": "k_heavy", "hcount": "k_heavy"}


def pmc_traffic(config, family):
    """HBM bytes per launch of the family's kernel from the committed PMC summary (FETCH_SIZE x2 + WRITE_SIZE,
    corrected as MI355X_MICROARCH.md prescribes), or None when no summary for this config is committed."""
    path = os.path.join(ROOT, "profiles", f"pmc_{config}.json")
    k = FAMILY_KERNEL.get(family)
    if not k or not os.path.exists(path):
        return None
    ent = json.load(open(path)).get(k)
    return int(ent["hbm_bytes"]) if ent else None


def algorithmic_bytes(name, d, gs, cs, kt_counts):
    """Minimal HBM bytes a kernel family must move per launch (DESIGN.md 'Kernels and rooflines')."""
    n = d.n
    J = gs["n_records"]
    if name == "unary":
        return 12 * n                                   # read s, p, o once
    if name == "emit":
        return 12 * n + 8 * J                           # read triples, write (join, capture) records
    if name == "sort":
        return 16 * kt_counts["sort_passes_records"]    # read + write each record once per 8-bit pass
    if name == "cemit":
        n_out = cs["n_class_cinds"]
        return 4 * n_out                                # 4-B ref per CIND written (dependent-run output); the shared
                                                        # class lists (< 1 MB) are read from L2
    if name in ("hwrite", "hcount"):
        cand = cs["n_heavy_candidates"]
        out = 4 * cs["n_cinds"] if name == "hwrite" else 4 * cs["n_heavy_chunks"]
        return 20 * cand + out                          # candidate ids + 16-B capture info, output records
    return None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--config", default="c2")
    ap.add_argument("--scale", type=float, default=1.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-ingest", action="store_true", help="skip the N-Triples ingest leg (rank 0, N=1)")
    ap.add_argument("--cpu-sample-scale", type=float, default=0.3)
    ap.add_argument("--backend", default="nccl", help="process-group backend for N > 1 (gloo: host-staged "
                    "exchanges, to rehearse several ranks on one GPU)")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    if world > 1:
        import torch
        import torch.distributed as dist

        local_rank %= max(torch.cuda.device_count(), 1)
        torch.cuda.set_device(local_rank)
        dist.init_process_group(args.backend)

    from rdfind_amd import _lib, synth

    d = synth.config(args.config, args.scale)  # same seeded workload on every rank
    ms = d.min_support
    ctx = _lib.Context(local_rank)
    ctx.set_triples(d.s, d.p, d.o, d.num_terms)  # inputs resident in HBM before the timed region

    if dist is not None:
        from rdfind_amd import distributed

        def step():
            distributed.run_sharded(ctx, ms)
            return ctx.cinds
    else:
        def step():
            return ctx.run(ms)

    def barrier():
        if dist is not None:
            import torch
            dist.barrier()
            torch.cuda.synchronize()

    for _ in range(args.warmup):
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
    elapsed = time.perf_counter() - t0
    if dist is not None:
        import torch
        dev = f"cuda:{local_rank}" if args.backend == "nccl" else "cpu"
        t = torch.tensor([elapsed], device=dev, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
        tot = torch.tensor([cs["n_cinds"]], device=dev, dtype=torch.int64)
        dist.all_reduce(tot)
        total_cinds = int(tot.item())
    else:
        total_cinds = cs["n_cinds"]
    total_triples = float(d.n)
    steps = max(args.steps, 1)
    ms_per_step = elapsed * 1000.0 / steps
    value = total_triples * steps / elapsed

    gs, fc = ctx.groups, ctx.fc
    kt = {k: v / steps for k, v in kt_sum.items()}
    counts = {"sort_passes_records": 0}
    # passes of the record sort (bits = join bits + capture bits, 8 per pass)
    V = d.num_terms
    capbits = int(2 * sum(fc["n_frequent_unary"]) + fc["n_frequent_binary"] - 1).bit_length()  # compact capture ids
    joinbits = int(V - 1).bit_length()
    counts["sort_passes_records"] = ((capbits + joinbits + 7) // 8) * gs["n_records"]
    dominant = max(kt, key=lambda k: kt[k])
    roof = None
    for name in [dominant] + sorted(kt, key=lambda k: -kt[k]):
        b = algorithmic_bytes(name, d, gs, cs, counts)
        if b is not None and kt[name] > 0:
            achieved = b / (kt[name] * 1e-3) / 1e9
            roof = {"bound": "hbm", "kernel": name, "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS,
                    "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4),
                    "traffic": pmc_traffic(args.config, name) if args.scale == 1.0 and world == 1 else None,
                    "ms": round(kt[name], 4), "bytes_per_launch": int(b), "dominant_kernel": dominant,
                    "dominant_ms": round(kt[dominant], 4)}
            break

    # BASELINE metric also names "% HBM roofline of count kernels": K1 (unary) and K2 (binary condition counts)
    count_roof = {}
    for name, b in (("unary", 12 * d.n), ("binary", 12 * d.n + 12 * fc["n_binary_keys"])):
        if kt.get(name, 0) > 0:
            gbs = b / (kt[name] * 1e-3) / 1e9
            count_roof[name] = {"bytes": int(b), "ms": round(kt[name], 4), "achieved": round(gbs, 1),
                                "frac": round(gbs / HBM_PEAK_GBS, 4), "bound": "memory-side atomics"}

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        from oracle import c_oracle

        sd = synth.config(args.config, args.cpu_sample_scale)
        t = time.perf_counter()
        _, _, st = c_oracle.run(sd.s, sd.p, sd.o, sd.num_terms, sd.min_support, 1, True)
        ct = time.perf_counter() - t
        nt = c_oracle.threads()
        cpu = {"value": round(sd.n / ct, 1), "unit": "triples/s", "cores": nt, "kind": "port",
               "sample": f"{args.config} scale {args.cpu_sample_scale} ({sd.n} triples, {st['n_cinds']} CINDs) "
                         f"through oracle/c/rdfind_oracle.c on {nt} OpenMP threads, {ct:.1f}s"}

    ingest = None
    if rank == 0 and world == 1 and not args.no_ingest:
        # parse/encode timed separately -- the same triples as N-Triples text through
        # rdf_parse_ntriples (device time, text already uploaded; the ids/terms are checked by tests/)
        import numpy as np

        tt = d.terms.term
        strs = np.array([tt(i) + " " for i in range(d.num_terms)], dtype=object)
        text = "".join(map("".join, zip(strs[d.s], strs[d.p], strs[d.o], [".\n"] * d.n))).encode()
        del strs
        pt = []
        for _ in range(3):
            n_parsed, n_terms, pms = ctx.parse_ntriples(text)
            pt.append(pms)
        pms = sorted(pt)[1]
        assert n_parsed == d.n
        ingest = {"ms": round(pms, 3), "text_bytes": len(text), "gbs_text": round(len(text) / pms / 1e6, 1),
                  "triples_per_s": round(d.n / pms * 1e3, 1), "terms": n_terms,
                  "end_to_end_ms": round(pms + ms_per_step, 3),
                  "note": "rdf_parse_ntriples device time (median of 3), excl. the text's H2D copy; end_to_end = "
                          "ingest + one discovery step, both device-resident"}
        del text

    if rank == 0:
        line = {
            "metric": "CIND-discovery triples/sec", "value": round(value, 1), "unit": "triples/s",
            "n_gpus": world, "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(ms_per_step, 3),
            "higher_is_better": True, "scaling": "strong" if world > 1 else "weak", "vs_baseline": None, "dtype": "u32", "data": "synthetic",
            "config": {"workload": f"{args.config} ({'LUBM-100-shaped' if args.config == 'c2' else args.config}, "
                                   f"scale {args.scale}, support {ms}, strategy 1 --use-fis --clean-implied)",
                       "triples": d.n, "cinds": total_cinds, "cinds_rank0": cs["n_cinds"],
                       "parallelism": f"join-hash shards x{world} (RCCL)" if world > 1 else "single"},
            "roofline": roof, "count_kernels": count_roof, "cpu_baseline": cpu, "ingest": ingest,
            "kernel_ms": {k: round(v, 4) for k, v in kt.items()},
            "work": {"records": gs["n_records"], "groups": gs["n_groups"], "captures": gs["n_captures"],
                     "heavy_groups": gs["n_heavy_groups"], "light_chunks": cs["n_light_chunks"],
                     "explicit_raw": cs["n_explicit_raw"], "heavy_chunks": cs["n_heavy_chunks"],
                     "heavy_candidates": cs["n_heavy_candidates"], "class_members": cs["n_class_members"],
                     "classes": cs["n_classes"], "class_cinds": cs["n_class_cinds"]},
        }
        print(json.dumps(line), flush=True)
    ctx.close()
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
