"""Markdown results table from the committed bench lines (dev tool): python tools/results_table.py [round tag]

Reads profiles/<tag>_bench_c2.json and profiles/<tag>_cfg_*.json (one bench.py JSON line each) and prints the rows of
BASELINE.md section 2 / DESIGN.md section 9: T_disc, triples/s, the light family's roofline fraction, the CPU
baseline and what it ran on."""
import glob
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
tag = sys.argv[1] if len(sys.argv) > 1 else "r04"


def line(path):
    for ln in open(path):
        if ln.startswith("{"):
            return json.loads(ln)
    return None


files = [os.path.join(ROOT, "profiles", f"{tag}_bench_c2.json")] + sorted(glob.glob(os.path.join(ROOT, "profiles", f"{tag}_cfg_*.json")))
print("| config | triples | CINDs | GPUs | T_disc ms | resident ms | triples/s | light ms (frac of HBM peak) | CPU baseline triples/s (cores, sample) |")
print("|---|---|---|---|---|---|---|---|---|")
for f in files:
    if not os.path.exists(f):
        continue
    d = line(f)
    if not d:
        continue
    cfg = d["config"]
    fam = d.get("families", {}).get("light", {})
    cpu = d.get("cpu_baseline") or {}
    res = (d.get("device_resident") or {}).get("ms_per_step")
    name = os.path.basename(f)[len(tag) + 1:-5]
    sample = cpu.get("sample", "")
    samp = sample.split(" (")[0] if sample else "—"
    cpu_s = f"{cpu['value']:.3g} ({cpu['cores']}, {samp}{', = GPU' if cpu.get('matches_gpu') else ''})" if cpu else "—"
    print(f"| {name} | {cfg.get('triples')} | {cfg.get('cinds'):.3g} | {d['n_gpus']} | {d['ms_per_step']} | {res} | "
          f"{d['value']:.3g} | {fam.get('ms', '—')} ({fam.get('frac', '—')}) | {cpu_s} |")
