"""Dev tool: compare the classed and pivot-scan heavy-only binary paths (RDFIND_HCLASS) on c5 shapes and
verify differing CINDs against the triples.  python tools/diff_paths.py <scale>..."""
import os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
from rdfind_amd import _lib, synth

def joins(d, code, v1, v2):
    cols = {1: d.s, 2: d.p, 4: d.o}
    prim, proj = code & 7, (code >> 3) & 7
    first = prim & -prim
    second = prim & ~first
    mask = cols[first] == v1
    if second:
        mask &= cols[second] == v2
    return np.unique(cols[proj][mask])

ctxs = {}
for flag in ("1", "0"):
    os.environ["RDFIND_HCLASS"] = flag
    ctxs[flag] = _lib.Context(0)
for sc in [float(x) for x in sys.argv[1:]]:
    d = synth.config("c5", sc)
    res = {}
    for flag, c in ctxs.items():
        c.set_triples(d.s, d.p, d.o, d.num_terms)
        cs = c.run(d.min_support)
        res[flag] = (c.cind_count(), c.checksum(), cs)
    print("scale", sc, "triples", d.n, {k: v[:2] for k, v in res.items()}, flush=True)
    if res["1"][0] == res["0"][0] or max(res["1"][0], res["0"][0]) > 6e8:
        continue
    rows = {}
    for flag, c in ctxs.items():
        c.set_triples(d.s, d.p, d.o, d.num_terms)
        c.run(d.min_support)
        r = c.copy_cinds()
        rows[flag] = (np.sort((r["dep"].astype(np.uint64) << np.uint64(32)) | r["ref"].astype(np.uint64)), c.binary_keys())
    a, b = rows["1"][0], rows["0"][0]
    only_new = np.setdiff1d(a, b, assume_unique=True)
    only_old = np.setdiff1d(b, a, assume_unique=True)
    print("only classed", len(only_new), "only pivot", len(only_old), flush=True)
    bk = rows["1"][1]
    for name, arr in (("only classed", only_new), ("only pivot", only_old)):
        if not len(arr):
            continue
        deps = np.unique(arr >> np.uint64(32))
        print(name, "distinct deps", len(deps), flush=True)
        pick = arr[np.random.default_rng(0).choice(len(arr), size=min(6, len(arr)), replace=False)]
        rr = np.zeros(len(pick), dtype=_lib.CIND_DTYPE)
        rr["dep"] = (pick >> np.uint64(32)).astype(np.uint32)
        rr["ref"] = (pick & np.uint64(0xFFFFFFFF)).astype(np.uint32)
        dec = _lib.decode_rows(rr, d.num_terms, bk)
        for x in dec.tolist():
            dc, d1, d2, rc, r1, r2, _ = x
            jd, jr = joins(d, dc, d1, d2), joins(d, rc, r1, r2)
            print("  ", name, x[:6], "|jd|", len(jd), "|jr|", len(jr), "valid", bool(np.isin(jd, jr).all()), flush=True)
