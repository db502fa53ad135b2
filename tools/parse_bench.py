"""Dev tool: device N-Triples ingest (rdf_parse_ntriples) throughput on the c2 triples written as N-Triples
text, vs the host parser on a sample.  python tools/parse_bench.py [scale]"""
import os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
from rdfind_amd import _lib, ntriples, synth

scale = float(sys.argv[1]) if len(sys.argv) > 1 else 1.0
d = synth.config("c2", scale)
t = time.perf_counter()
tt = d.terms.term
strs = np.array([tt(i) + " " for i in range(d.num_terms)], dtype=object)
data = "".join(map("".join, zip(strs[d.s], strs[d.p], strs[d.o], [".\n"] * d.n))).encode()
print(f"text {len(data) / 1e9:.2f} GB, {d.n} lines, {d.num_terms} terms (built in {time.perf_counter() - t:.1f}s)",
      flush=True)
with _lib.Context(0) as ctx:
    times = []
    for _ in range(4):
        n, v, ms = ctx.parse_ntriples(data)
        times.append(ms)
    ms = float(np.median(times[1:]))
    s, p, o = ctx.copy_triples(n)
    used = np.unique(np.concatenate([d.s, d.p, d.o])).shape[0]  # the generator's id space has unused ids
    assert n == d.n and v == used, (n, v, used)
    print(f"PARSE device {ms:.2f} ms (median of {len(times) - 1}, excl. H2D): {len(data) / ms / 1e6:.1f} GB/s of text, "
          f"{n / ms / 1e6:.2f} G triples/s", flush=True)
    k = min(d.n, 200_000)
    sample = b"".join(data.splitlines(keepends=True)[:k])
    import tempfile
    with tempfile.NamedTemporaryFile(suffix=".nt") as f:
        f.write(sample)
        f.flush()
        t = time.perf_counter()
        hs, hp, ho, hd = ntriples.read_triples([f.name])
        dt = time.perf_counter() - t
    print(f"PARSE host parser (1 thread) on {k} lines: {k / dt / 1e6:.3f} M triples/s", flush=True)
