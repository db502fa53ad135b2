import os, random, sys
sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", "."))
os.environ["RDFIND_HEAVY_MIN"] = "64"
import numpy as np
from rdfind_amd import _lib
from oracle import c_oracle as C
from tests.test_gpu import MODES, expected_set
g = _lib.Context(0)
rng = random.Random(564)
for it in range(30):
    n = rng.randrange(20, 400); nv = rng.randrange(4, 40); ms = rng.randrange(1, 4)
    arr = np.array([(rng.randrange(nv), rng.randrange(nv // 4 + 1), rng.randrange(nv)) for _ in range(n)], dtype=np.uint32)
    for strategy, clean in MODES:
        exp = expected_set(arr, nv, ms, strategy, clean)
        g.set_triples(arr[:, 0], arr[:, 1], arr[:, 2], nv)
        g.frequent_conditions(ms); g.build_capture_groups("spo")
        seen, log = {}, []
        print("case", it, strategy, clean, flush=True)
        for (d0, d1) in g.pages(clean, strategy, 1):
            parts = g.copy_result_compact()
            cnt = g.cind_count()
            rows = _lib.decoded_to_set(g.decoded_cinds())
            L = parts["layout"]
            ro = parts["runoff"][: L["n_runs"] + 1]
            lo = parts["list_off"][: L["n_lists"] + 1]
            probs = []
            if len(ro) and (ro[-1] != L["n_refs"] or (np.diff(ro.astype(np.int64)) < 0).any()):
                probs.append(("runoff", ro[:8].tolist(), ro[-3:].tolist(), L))
            if L["n_lists"] and (lo[-1] != L["n_list_refs"] or (np.diff(lo.astype(np.int64)) < 0).any()):
                probs.append(("list_off", lo[:8].tolist(), lo[-3:].tolist(), L))
            mem = parts["members"][: L["n_members"]]
            if L["n_members"] and ((mem >> 32) >= max(L["n_lists"], 1)).any():
                probs.append(("members", (mem >> 32)[:8].tolist(), L))
            if probs:
                print("BAD PARTS case", it, strategy, clean, "page", (d0, d1), probs, flush=True)
                sys.exit(0)
            ck = g.checksum()
            cc = C.checksum_compact(parts, g.num_terms)[:2]
            dup = [r for r in rows if r in seen]
            log.append(((d0, d1), cnt, len(rows), len(dup), sorted({seen[r] for r in dup})[:3], cc == (cnt, ck)))
            for r in rows:
                seen.setdefault(r, (d0, d1))
        miss = exp - set(seen)
        if any(x[3] for x in log) or miss or set(seen) != exp:
            print("FAIL case", it, n, nv, ms, strategy, clean, "exp", len(exp), "got", len(seen), "missing", len(miss),
                  "extra", len(set(seen) - exp))
            for x in log:
                if x[1] or x[3]:
                    print("  ", x)
            sys.exit(0)
print("all ok")
