import os, sys, random
sys.path.insert(0, "/root/repo")
import numpy as np
from rdfind_amd import _lib
ctxs = {}
for flag in ("1", "0"):
    os.environ["RDFIND_HCLASS"] = flag
    ctxs[flag] = _lib.Context(0)
rng = random.Random(11)
bad = 0
for it in range(150):
    n = rng.randrange(1, 250); nv = rng.randrange(2, 40); ms = rng.randrange(1, 5)
    arr = np.array([(rng.randrange(nv), rng.randrange(nv // 3 + 1), rng.randrange(nv)) for _ in range(n)], dtype=np.uint32)
    for strategy, clean in [(1, True), (0, True), (0, False), (1, False)]:
        res = {}
        for f, c in ctxs.items():
            c.set_triples(arr[:, 0], arr[:, 1], arr[:, 2], nv)
            cs = c.run(ms, "spo", clean, strategy)
            res[f] = (_lib.decoded_to_set(c.decoded_cinds()), dict(c.groups), cs)
        if res["1"][0] != res["0"][0]:
            bad += 1
            if bad <= 3:
                print("DIFF", it, n, nv, ms, strategy, clean, "extra", sorted(res["1"][0] - res["0"][0])[:4], "missing", sorted(res["0"][0] - res["1"][0])[:4])
                print("   groups", res["1"][1]["n_heavy_groups"], res["1"][1]["heavy_threshold"], {k: res["1"][2][k] for k in ("n_heavy_chunks", "n_class_members", "n_classes")})
print("bad", bad)
