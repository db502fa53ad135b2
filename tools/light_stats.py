"""Light-intersection work counters on a BASELINE config (dev tool; needs `make stats`)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ["RDFIND_HIP_LIB"] = os.path.join(ROOT, "rdfind_amd", "librdfind_hip_stats.so")
sys.path.insert(0, ROOT)
from rdfind_amd import _lib, synth  # noqa: E402

cfg = sys.argv[1] if len(sys.argv) > 1 else "c2"
scale = float(sys.argv[2]) if len(sys.argv) > 2 else 1.0
d = synth.config(cfg, scale)
with _lib.Context(0) as ctx:
    ctx.set_triples(d.s, d.p, d.o, d.num_terms)
    cs = ctx.run(d.min_support)
    print(cfg, scale, ctx.groups, cs, ctx.kernel_times(), flush=True)
