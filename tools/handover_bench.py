"""Dev tool: time the compact hand-over alone (rdf_copy_result_compact into the bench's pinned sink) on c2."""
import os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
from rdfind_amd import _lib, synth
import bench

d = synth.config("c2", 1.0)
with _lib.Context(0) as ctx:
    ctx.set_triples(d.s, d.p, d.o, d.num_terms)
    ctx.run(d.min_support)
    sink = bench.CompactSink()
    sink.copy(ctx)
    for rep in range(3):
        t = time.perf_counter()
        for _ in range(20):
            sink.copy(ctx)
        dt = (time.perf_counter() - t) / 20
        L = ctx.result_layout()
        print(f"sink.copy {dt * 1e3:.3f} ms for {bench.layout_bytes(L) / 1e6:.1f} MB = {bench.layout_bytes(L) / dt / 1e9:.1f} GB/s",
              flush=True)
    bufs = ctx.copy_result_compact()
    t = time.perf_counter()
    for _ in range(20):
        ctx.copy_result_compact(bufs)
    print(f"pageable numpy {(time.perf_counter() - t) / 20 * 1e3:.3f} ms", flush=True)
    t = time.perf_counter()
    for _ in range(20):
        L = ctx.result_layout()
    print(f"result_layout {(time.perf_counter() - t) / 20 * 1e6:.1f} us", flush=True)
    t = time.perf_counter()
    for _ in range(20):
        kt = ctx.kernel_times()
    print(f"kernel_times {(time.perf_counter() - t) / 20 * 1e3:.3f} ms", flush=True)
    for mode in ("run", "run+copy", "run+copy+kt"):
        t = time.perf_counter()
        for _ in range(10):
            ctx.run(d.min_support)
            if "copy" in mode:
                sink.copy(ctx)
            if "kt" in mode:
                ctx.kernel_times()
        print(f"{mode}: {(time.perf_counter() - t) / 10 * 1e3:.3f} ms", flush=True)
