"""A/B of light-kernel variants (dev tool): python tools/light_ab.py <cfg:scale>... ; each variant library
(RDFIND_AB_LIBS, comma-separated .so names under rdfind_amd/) runs in its own process."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

if len(sys.argv) > 1 and sys.argv[1] == "--child":
    sys.path.insert(0, ROOT)
    import numpy as np
    from rdfind_amd import _lib, synth
    out = {}
    for spec in sys.argv[2:]:
        cfg, sc = spec.split(":")
        cache = os.path.join(os.environ.get("TMPDIR", "/tmp"), f"ab_{cfg}_{sc}.npz")  # shared by the variants
        if os.path.exists(cache):
            z = np.load(cache)
            ds, dp, do, nv, msup = z["s"], z["p"], z["o"], int(z["nv"]), int(z["ms"])
        else:
            d = synth.config(cfg, float(sc))
            ds, dp, do, nv, msup = d.s, d.p, d.o, d.num_terms, d.min_support
            np.savez(cache, s=ds, p=dp, o=do, nv=nv, ms=msup)
        with _lib.Context(0) as ctx:
            ctx.set_triples(ds, dp, do, nv)
            best = None
            for _ in range(3):
                cs = ctx.run(msup)
                kt = ctx.kernel_times()
                best = kt if best is None or kt["light"] < best["light"] else best
            out[spec] = {"light": round(best["light"], 3), "pivot": round(best["pivot"], 3),
                         "binary": round(best["binary"], 3), "unary": round(best["unary"], 3), "sort": round(best["sort"], 3), "groups": round(best["groups"], 3), "emit": round(best["emit"], 3), "support": round(best["support"], 3),
                         "total": round(sum(best.values()), 3), "n": ctx.cind_count(), "sum": ctx.checksum()}
    print("AB", json.dumps(out), flush=True)
    sys.exit(0)

# a variant is "<lib>[@VAR=value[@VAR=value]]": the library plus environment switches (e.g. RDFIND_SIG=0)
for variant in os.environ.get("RDFIND_AB_LIBS", "librdfind_hip.so").split(","):
    lib, *envs = variant.split("@")
    env = dict(os.environ, RDFIND_HIP_LIB=os.path.join(ROOT, "rdfind_amd", lib))
    env.update(e.split("=", 1) for e in envs)
    r = subprocess.run([sys.executable, __file__, "--child"] + sys.argv[1:], env=env, capture_output=True, text=True,
                       timeout=900)
    line = [ln for ln in r.stdout.splitlines() if ln.startswith("AB")]
    print(variant, line[0][3:] if line else r.stderr[-2000:], flush=True)
    for ln in r.stderr.splitlines():  # library decisions printed under RDFIND_DEBUG_LIGHT
        if ln.startswith(("dense:", "LIGHT weighted")):
            print("  ", ln, flush=True)
