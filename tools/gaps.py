"""GPU idle time inside one discovery step (dev tool), from a rocprofv3 kernel + memory-copy trace:

  rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d DIR -o tl -- python3 tools/sync_trace.py --child c2 1.0
  python tools/gaps.py DIR

The child runs three steps; the last one starts at its last k_u2_part launch.  Prints the step's span, the time
covered by kernels and copies, and the largest idle gaps with the operations on either side."""
import csv
import glob
import os
import sys

d = sys.argv[1]


def load(pattern):
    fs = glob.glob(os.path.join(d, "**", pattern), recursive=True)
    return list(csv.DictReader(open(fs[0]))) if fs else []


ops = []
for r in load("*kernel_trace.csv"):
    ops.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"].split("(")[0][:48]))
for r in load("*memory_copy_trace.csv"):
    ops.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), "copy " + r.get("Direction", "")))
ops.sort()
starts = [i for i, o in enumerate(ops) if "k_u2_part" in o[2]]
first = starts[-2] if len(starts) >= 2 else 0  # k_u2_part<false> of the last step (two launches per step)
step = ops[first:]
t0 = step[0][0]
t1 = max(o[1] for o in step)
busy, cur_s, cur_e, gaps = 0, step[0][0], step[0][1], []
prev = step[0]
for o in step[1:]:
    if o[0] > cur_e:
        busy += cur_e - cur_s
        gaps.append((o[0] - cur_e, prev[2], o[2]))
        cur_s, cur_e = o[0], o[1]
    else:
        cur_e = max(cur_e, o[1])
    if o[1] >= cur_e:
        prev = o
busy += cur_e - cur_s
print(f"step span {(t1 - t0) / 1e3:.1f} us, busy {busy / 1e3:.1f} us, idle {(t1 - t0 - busy) / 1e3:.1f} us "
      f"in {len(gaps)} gaps; {len(step)} operations")
gaps.sort(reverse=True)
for g, a, b in gaps[:40]:
    print(f"  {g / 1e3:8.1f} us  after {a:48s} before {b}")
small = sum(g for g, _, _ in gaps if g < 5000)
print(f"gaps < 5 us: {sum(1 for g, _, _ in gaps if g < 5000)} totalling {small / 1e3:.1f} us")
