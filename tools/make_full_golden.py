"""Full-size golden vectors: (count, checksum) of the CIND result of each BASELINE config at the largest size a
single MI355X holds, computed by the C oracle's streamed mode (oracle/c/rdfind_oracle.c orc_stream) on the seeded
synthetic inputs (rdfind_amd/synth.py).  Output: tests/golden/full_size.json (one entry per config/scale/mode).

    python tools/make_full_golden.py [name ...]      # e.g. c1 c2 (default: all)

The GPU tests regenerate the same seeded input, run the HIP path and compare count, checksum and stage counts
(tests/test_gpu_full.py); a fingerprint of the triples guards against generator drift.
"""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from oracle import c_oracle as C  # noqa: E402
from rdfind_amd import synth  # noqa: E402

OUT = os.path.join(ROOT, "tests", "golden", "full_size.json")

# (config, scale, [(strategy, clean), ...])
CASES = {
    "c1": ("c1", 1.0, [(1, True), (0, True), (0, False), (1, False)]),
    "c2": ("c2", 1.0, [(1, True), (0, True)]),
    "c3": ("c3", 1.0, [(1, True)]),
    "c4": ("c4", 0.05, [(1, True)]),
    "c4_0.1": ("c4", 0.1, [(1, True)]),      # counter-based generator from here on (synth._c4_rows)
    "c4_0.4": ("c4", 0.4, [(1, True)]),
    "c4_1.0": ("c4", 1.0, [(1, True)]),      # the BASELINE size: the oracle's stages 3-4 in join-value ranges
    "c5": ("c5", 0.3, [(1, True), (0, False)]),
    "c5_1.0": ("c5", 1.0, [(1, True)]),      # the BASELINE size (paged discovery on the GPU)
}


def fingerprint(d):
    """Order-independent 64-bit fingerprint of the triples (guards the seeded generator)."""
    m = np.uint64(0x9E3779B97F4A7C15)
    with np.errstate(over="ignore"):
        x = (d.s.astype(np.uint64) * m) ^ (d.p.astype(np.uint64) << np.uint64(21)) ^ (d.o.astype(np.uint64) * np.uint64(0xC2B2AE3D27D4EB4F))
        x ^= x >> np.uint64(29)
        x *= np.uint64(0xBF58476D1CE4E5B9)
        x ^= x >> np.uint64(32)
        return int(x.sum(dtype=np.uint64))


# oracle stages 3-4 in join-value ranges of at most this many records (memory: ~16 B per record of a range)
RANGE_RECORDS = {"c4_1.0": 200_000_000}


def main(names):
    out = json.load(open(OUT)) if os.path.exists(OUT) else {}
    for name in names:
        cfg, scale, modes = CASES[name]
        C.set_range_records(RANGE_RECORDS.get(name, 0))
        t = time.time()
        d = synth.config(cfg, scale)
        gen_s = time.time() - t
        for strategy, clean in modes:
            t = time.time()
            r = C.stream(d.s, d.p, d.o, d.num_terms, d.min_support, strategy, clean)
            key = f"{cfg}@{scale}/s{strategy}{'_clean' if clean else '_raw'}"
            st = r["stats"]
            out[key] = {"config": cfg, "scale": scale, "strategy": strategy, "clean": clean,
                        "min_support": d.min_support, "n_triples": d.n, "num_terms": d.num_terms,
                        "fingerprint": str(fingerprint(d)), "n_cinds": r["n_cinds"], "checksum": str(r["checksum"]),
                        "n_kind": r["n_kind"], "n_raw": r["n_raw"], "n_freq_unary": st["n_freq_unary"],
                        "n_freq_binary": st["n_freq_binary"], "n_records": st["n_records"],
                        "n_freq_captures": st["n_freq_captures"],
                        "oracle_s": round(time.time() - t, 1), "gen_s": round(gen_s, 1), "threads": C.threads()}
            print(key, out[key], flush=True)
            json.dump(out, open(OUT, "w"), indent=1, sort_keys=True)
        del d


if __name__ == "__main__":
    main(sys.argv[1:] or list(CASES))
