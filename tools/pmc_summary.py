"""Summarise rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes into per-kernel HBM bytes per launch.

Corrections (MI355X_MICROARCH.md, HBM section): counters are in KB (1024 B); on gfx950 FETCH_SIZE
reports half of the bytes of wide coalesced streaming reads, so it is doubled; WRITE_SIZE is exact for
16-B-per-lane streaming stores.  Divergent 4-B gathers are counted in full (tools/micro/gcal.hip,
profiles/r04_fetch_calibration.log: a random 4-B load reads as 64 B, 16 lanes in one 64-B line as 4 B each), so the
gather-bound kernels (GATHER_KERNELS) are not doubled; "fetch_bytes_stream" keeps the doubled figure as their upper
bound.  Output: {kernel: {"launches", "fetch_bytes", "write_bytes", "hbm_bytes"}} averaged per launch, keyed by
the short kernel name (rdf::k_xxx without template args / signature).
"""
import csv
import glob
import json
import os
import re
import sys


def short(name):
    name = re.sub(r"\(.*$", "", name)
    name = re.sub(r"<.*>", "", name)
    return name.split("::")[-1].replace("void ", "").strip()


def load(d, counter):
    per = {}
    files = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
    for f in files:
        with open(f) as fh:
            for row in csv.DictReader(fh):
                if row.get("Counter_Name") != counter:
                    continue
                k = short(row["Kernel_Name"])
                per.setdefault(k, {}).setdefault(row["Dispatch_Id"], 0.0)
                per[k][row["Dispatch_Id"]] += float(row["Counter_Value"])
    return {k: (len(v), sum(v.values()) / max(len(v), 1)) for k, v in per.items()}


# kernels whose reads are mostly divergent 4-B loads (member-list searches, group metadata, dense-bitmap words)
GATHER_KERNELS = {"k_light", "k_light_stage", "k_light_plain", "k_light_plain_hi", "k_light_packed", "k_light_mseg_emit"}


def main():
    fetch = load(sys.argv[1], "FETCH_SIZE")
    write = load(sys.argv[2], "WRITE_SIZE")
    out = {}
    for k in sorted(set(fetch) | set(write)):
        nf, f = fetch.get(k, (0, 0.0))
        nw, w = write.get(k, (0, 0.0))
        gather = k in GATHER_KERNELS
        fb, wb = (1.0 if gather else 2.0) * f * 1024.0, w * 1024.0
        out[k] = {"launches": max(nf, nw), "fetch_bytes": round(fb), "write_bytes": round(wb), "hbm_bytes": round(fb + wb)}
        if gather:
            out[k]["fetch_bytes_stream"] = round(2.0 * f * 1024.0)
    print(json.dumps(out, indent=1, sort_keys=True))


if __name__ == "__main__":
    main()
