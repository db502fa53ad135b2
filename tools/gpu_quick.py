"""Quick GPU parity check against the C oracle on random + synthetic inputs (dev tool)."""
import random, sys, time, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
from rdfind_amd import _lib, synth
from oracle import c_oracle as C, rdfind_oracle as R

ctx = _lib.Context(0)
rng = random.Random(3)
bad = 0
t0 = time.time()
for it in range(200):
    n = rng.randrange(1, 200); nv = rng.randrange(2, 30); ms = rng.randrange(1, 5)
    arr = np.array([(rng.randrange(nv), rng.randrange(nv//3+1), rng.randrange(nv)) for _ in range(n)], dtype=np.uint32)
    for strat, clean in ((1, True), (0, True), (0, False), (1, False)):
        exp, _ = C.run_set(arr[:,0], arr[:,1], arr[:,2], nv, ms, strat, clean)
        if strat == 1 and not clean:
            tr = [tuple(x) for x in arr.tolist()]
            uf = R.frequent_unary_conditions(tr, ms); bf = R.frequent_binary_conditions(tr, uf, ms)
            V = R.all_at_once(R.join_lines(tr, uf, bf), ms, False, literal_implies=False)
            exp = R.cind_set(R.s2l_exact_raw(V))
        ctx.set_triples(arr[:,0], arr[:,1], arr[:,2], nv)
        ctx.run(ms, "spo", clean, strat)
        got = _lib.decoded_to_set(ctx.decoded_cinds())
        if got != exp:
            bad += 1
            if bad < 5:
                print("MISMATCH", it, strat, clean, n, nv, ms, len(exp), len(got), sorted(exp-got)[:3], sorted(got-exp)[:3], flush=True)
print("random: bad", bad, "%.1fs" % (time.time()-t0), flush=True)
for name, scale in [("c1", 0.2), ("c2", 0.05), ("c5", 0.01)]:
    d = synth.config(name, scale)
    t = time.time(); exp, st = C.run_set(d.s, d.p, d.o, d.num_terms, d.min_support, 1, True); tc = time.time() - t
    ctx.set_triples(d.s, d.p, d.o, d.num_terms)
    t = time.time(); cs = ctx.run(d.min_support); ctx.sync(); tg = time.time() - t
    got = _lib.decoded_to_set(ctx.decoded_cinds())
    print(name, scale, d.n, "oracle", len(exp), "%.2fs" % tc, "gpu", len(got), "%.3fs" % tg, "OK" if got == exp else "MISMATCH",
          ctx.groups, cs, ctx.stage_times(), flush=True)
