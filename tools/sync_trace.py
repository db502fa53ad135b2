"""Host round trips of one discovery step (dev tool): python tools/sync_trace.py [config] [scale].

Runs the step in a child with RDFIND_SYNC_TRACE=1 (rdfind_hip.hip traced_sync) and lists, for the last of three
runs, every host wait on the stream by source line: how long the host waited for the GPU, and the host time since
the previous wait returned (launch and bookkeeping time, during which the GPU may idle)."""
import collections
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

if len(sys.argv) > 1 and sys.argv[1] == "--child":
    sys.path.insert(0, ROOT)
    from rdfind_amd import _lib, synth
    d = synth.config(sys.argv[2], float(sys.argv[3]))
    with _lib.Context(0) as ctx:
        ctx.set_triples(d.s, d.p, d.o, d.num_terms)
        for i in range(3):
            print(f"RUN {i}", file=sys.stderr, flush=True)
            t = time.perf_counter()
            ctx.run(d.min_support)
            ctx.sync()
            wall = (time.perf_counter() - t) * 1e3
            kt = ctx.kernel_times()
            print(f"WALL {wall:.3f} KSUM {sum(kt.values()):.3f}", file=sys.stderr, flush=True)
    sys.exit(0)

cfg = sys.argv[1] if len(sys.argv) > 1 else "c2"
sc = sys.argv[2] if len(sys.argv) > 2 else "1.0"
r = subprocess.run([sys.executable, __file__, "--child", cfg, sc], env=dict(os.environ, RDFIND_SYNC_TRACE="1"),
                   capture_output=True, text=True, timeout=600)
lines = r.stderr.splitlines()
last = max(i for i, ln in enumerate(lines) if ln.startswith("RUN "))
rows, wall = [], None
for ln in lines[last + 1:]:
    f = ln.split()
    if f and f[0] == "SYNC":
        rows.append((int(f[1]), float(f[2]), float(f[3])))
    elif f and f[0] == "WALL":
        wall, ksum = float(f[1]), float(f[3])
if r.returncode or wall is None:
    print(r.stderr[-3000:])
    sys.exit(1)
print(f"{cfg} {sc}: {len(rows)} host waits in one step; wall {wall:.3f} ms, kernel-family sum {ksum:.3f} ms")
by = collections.OrderedDict()
prev_end = None
for line, t0, w in rows:
    host = 0.0 if prev_end is None else t0 - prev_end
    prev_end = t0 + w
    e = by.setdefault(line, [0, 0.0, 0.0])
    e[0] += 1
    e[1] += w
    e[2] += host
print(f"{'line':>6} {'n':>3} {'wait_us':>9} {'host_us_before':>15}")
for line, (n, w, h) in by.items():
    print(f"{line:6d} {n:3d} {w:9.1f} {h:15.1f}")
print(f"total wait {sum(e[1] for e in by.values()):.1f} us, host time between waits "
      f"{sum(e[2] for e in by.values()):.1f} us")
