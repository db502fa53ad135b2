"""Per-kernel durations of the last bench step from a rocprofv3 kernel trace (dev tool).
usage: python tools/trace_step.py gpurun_out/prof_X/run_kernel_trace.csv [first_kernel]"""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
first = sys.argv[2] if len(sys.argv) > 2 else "k_ucount_part"
idx = [i for i, r in enumerate(rows) if first in r["Kernel_Name"]]
last = rows[idx[-1]:]
tot = 0.0
for r in last:
    n = r["Kernel_Name"].split("(")[0].replace("void ", "").replace("rdf::", "")
    d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
    tot += d
    print(f"{n[:44]:44s} {d:9.1f} us  grid={r['Grid_Size_X']}")
print(f"total kernel time {tot:.1f} us; span {(int(last[-1]['End_Timestamp']) - int(last[0]['Start_Timestamp'])) / 1e3:.1f} us")
