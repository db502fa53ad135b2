"""Per-step kernel table from a rocprofv3 kernel_stats.csv: python tools/kstats.py <csv> <steps> [top]"""
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
steps = int(sys.argv[2]) if len(sys.argv) > 2 else 1
top = int(sys.argv[3]) if len(sys.argv) > 3 else 16
tot = sum(int(r["TotalDurationNs"]) for r in rows) / 1e6 / steps
for r in rows[:top]:
    name = r["Name"].replace("rdf::", "").replace("void ", "").split("(")[0]
    print("%-34s %5s calls  %9.3f ms/step" % (name[:34], r["Calls"], int(r["TotalDurationNs"]) / 1e6 / steps))
print("%-34s %9.3f ms/step (all kernels)" % ("total", tot))
