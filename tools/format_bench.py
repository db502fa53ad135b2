"""Dev tool: throughput of the device formatter (K8) on the c2 result.  python tools/format_bench.py"""
import os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from rdfind_amd import _lib, synth

d = synth.config("c2", 1.0)
terms = ["<http://www.Department%d.University%d.edu/Term%d>" % (i % 15, i % 7, i) for i in range(d.num_terms)]
with _lib.Context(0) as ctx:
    ctx.set_triples(d.s, d.p, d.o, d.num_terms)
    ctx.run(d.min_support)
    ctx.set_dictionary(terms)
    n = ctx.cind_count()
    rows = 1 << 23
    ctx.format_cinds(0, rows)  # warm-up (builds the capture string table)
    t = time.perf_counter()
    tot = 0
    for k in range(4):
        tot += len(ctx.format_array((k + 1) * rows, rows))
    dt = time.perf_counter() - t
    print(f"FORMAT rows={4 * rows} bytes={tot} {dt * 1e3:.1f} ms incl. D2H copy: {4 * rows / dt / 1e6:.1f} M lines/s, "
          f"{tot / dt / 1e9:.2f} GB/s of text; full result {n} rows ~{n * tot / (4 * rows) / 1e9:.0f} GB", flush=True)
