"""Per-work-item profile of k_light on a BASELINE config (dev tool; needs `make -C rdfind_amd/csrc stats`).

Usage: python tools/light_items.py <config> <scale>.  Each k_light work item writes a 16-field record
(kernels.inl, RDF_LIGHT_STATS); this prints where the cycles go."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ["RDFIND_HIP_LIB"] = os.path.join(ROOT, "rdfind_amd", "librdfind_hip_stats.so")
dump = os.path.join(os.environ.get("TMPDIR", "/tmp"), "light_items.bin")  # large: kept out of gpurun_out
os.environ["RDFIND_LIGHT_DUMP"] = dump
sys.path.insert(0, ROOT)
from rdfind_amd import _lib, synth  # noqa: E402

cfg = sys.argv[1] if len(sys.argv) > 1 else "c2"
scale = float(sys.argv[2]) if len(sys.argv) > 2 else 1.0
d = synth.config(cfg, scale)
with _lib.Context(0) as ctx:
    ctx.set_triples(d.s, d.p, d.o, d.num_terms)
    cs = ctx.run(d.min_support)
    print(cfg, scale, ctx.groups, cs, ctx.kernel_times(), flush=True)

r = np.fromfile(dump, dtype=np.uint32).reshape(-1, 24).astype(np.int64)
names = ["dep", "ng", "segg", "nseg", "piv", "alive0", "alive1", "win", "ser", "bat", "depth", "lg", "cyc_lo", "cyc_hi",
         "gsum", "gmax", "t_p2", "t_meta", "t_dense", "t_serial", "t_sweep", "t_batch"]
col = {n: r[:, i] for i, n in enumerate(names)}
for n in names[16:]:
    col[n] = col[n] * 256  # phase cycles are recorded / 256
cyc = col["cyc_lo"] + (col["cyc_hi"] << 32)
col["sweep"] = col["ser"] >> 16  # windows verified by a range sweep (kernels.inl light_sweep)
col["ser"] = col["ser"] & 0xFFFF
tot = cyc.sum()
print(f"items {len(r)}  total cycles {tot:.3e}  mean {cyc.mean():.0f}  max {cyc.max()}")


def share(mask, label):
    print(f"  {label:44s} items {mask.sum():9d} ({mask.mean():6.1%})  cycles {cyc[mask].sum() / tot:6.1%}"
          f"  mean cyc {cyc[mask].mean() if mask.any() else 0:9.0f}")


share(col["alive0"] == 0, "no candidate after the filter")
share((col["alive0"] > 0) & (col["alive1"] == 0), "all candidates killed")
share(col["alive1"] > 0, "survivors")
share(col["nseg"] > 1, "multi-segment dependents")
for lo, hi in [(0, 1), (1, 2), (2, 5), (5, 17), (17, 65), (65, 1 << 30)]:
    share((col["win"] >= lo) & (col["win"] < hi), f"windows in [{lo},{hi})")
for lo, hi in [(0, 1), (1, 4), (4, 16), (16, 64), (64, 256), (256, 1 << 30)]:
    share((col["bat"] >= lo) & (col["bat"] < hi), f"batch rounds in [{lo},{hi})")
s = lambda k: col[k].sum()
for lo, hi in [(0, 1), (1, 4), (4, 16), (16, 1 << 30)]:
    share((col["sweep"] >= lo) & (col["sweep"] < hi), f"swept windows in [{lo},{hi})")
print(f"sums: windows {s('win')}  swept {s('sweep')}  serial groups {s('ser')}  batches {s('bat')}  depth {s('depth')}  light groups {s('lg')}"
      f"  light group members {s('gsum')}  alive0 {s('alive0')}  alive1 {s('alive1')}")
print(f"mean depth per batch {s('depth') / max(s('bat'), 1):.2f}; "
      f"members per light group {s('gsum') / max(s('lg'), 1):.1f}; batches per window {s('bat') / max(s('win'), 1):.2f}")
# a linear model of the cycles: which counter explains them
X = np.stack([np.ones(len(r)), col["win"], col["ser"], col["bat"], col["depth"], col["sweep"]], 1).astype(np.float64)
coef, *_ = np.linalg.lstsq(X, cyc.astype(np.float64), rcond=None)
print("cycles ~ " + " + ".join(f"{c:.0f}*{n}" for c, n in zip(coef, ["1", "win", "ser", "bat", "depth", "sweep"])))
print("phase cycles: " + ", ".join(f"{n[2:]} {col[n].sum() / tot:5.1%}" for n in names[16:]) + "  (of the item cycles)")
top = np.argsort(-cyc)[:12]
print("slowest items:")
for i in top:
    print("  " + " ".join(f"{n}={col[n][i]}" for n in names if not n.startswith("cyc")) + f" sweep={col['sweep'][i]} cyc={cyc[i]}")
# per-dependent totals
deps, inv = np.unique(col["dep"], return_inverse=True)
dc = np.bincount(inv, weights=cyc.astype(np.float64))
o = np.argsort(-dc)[:8]
print("costliest dependents (sum of item cycles):")
for j in o:
    m = inv == j
    print(f"  dep {deps[j]} items {m.sum()} ng {col['ng'][m][0]} piv {col['piv'][m][0]} cycles {dc[j] / tot:6.2%}"
          f" alive0 {col['alive0'][m].sum()} alive1 {col['alive1'][m].sum()}")
print("LIGHT_ITEMS done", flush=True)
