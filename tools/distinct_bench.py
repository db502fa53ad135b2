"""Dev tool: device time of rdf_distinct_triples (--distinct-triples) on the c2 triples with 25% of them
repeated (shuffled in).  Algorithmic bytes per call: 12 B read per input triple + 12 B written per kept one.
python tools/distinct_bench.py"""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
from rdfind_amd import _lib, synth

d = synth.config("c2", 1.0)
rng = np.random.default_rng(0)
dup = rng.integers(0, d.s.shape[0], d.s.shape[0] // 4)
perm = rng.permutation(d.s.shape[0] + dup.shape[0])
s, p, o = (np.concatenate([x, x[dup]])[perm] for x in (d.s, d.p, d.o))
n = s.shape[0]
with _lib.Context(0) as ctx:
    times = []
    for it in range(6):
        ctx.set_triples(s, p, o, d.num_terms)
        kept, ms = ctx.distinct_triples()
        times.append(ms)
    ms = float(np.median(times[1:]))
    gbs = (12 * n + 12 * kept) / ms / 1e6
    print(f"DISTINCT n={n} kept={kept} (c2 distinct {d.s.shape[0]}) {ms:.3f} ms median of {len(times) - 1}: "
          f"{n / ms / 1e6:.2f} G triples/s, {gbs:.0f} GB/s algorithmic ({gbs / 8000:.3f} of 8 TB/s)", flush=True)
    assert kept == d.s.shape[0]
