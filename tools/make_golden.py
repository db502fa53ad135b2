"""Generate the golden fixtures in tests/golden/ (committed together with this script).

Inputs are small seeded synthetic N-Triples files of the BASELINE config shapes; expected outputs
are the sorted ``Cind.toString`` lines produced by the literal Python restatement of the reference
(oracle/rdfind_oracle.py): S2L (strategy 1, the default) and AllAtOnce (strategy 0), with and without
--clean-implied.  The reference itself cannot run here (no JVM/Flink).
"""
import gzip
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from rdfind_amd import synth, ntriples  # noqa: E402
from oracle import rdfind_oracle as R  # noqa: E402

OUT = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests", "golden")

FIXTURES = {
    # name: (dataset factory, min_support)
    "zipf_small": (lambda: synth.zipf_rdf("zipf_small", 4000, 1500, 30, 1.1, 1.0, 0.15, 12, 1.2, 0.3, 1500, 1.0, 1.0, 3, 11), 3),
    "lubm_small": (lambda: synth.lubm(1, seed=7, min_support=10, max_departments=1), 10),
    "skew_small": (lambda: synth.zipf_rdf("skew_small", 1500, 400, 12, 1.1, 1.0, 0.1, 8, 1.2, 0.2, 300, 1.0, 1.5, 2, 5), 2),
}

MODES = {  # file suffix: (strategy, clean, extra)
    "s1_clean": (1, True),
    "s0_clean": (0, True),
    "s0_raw": (0, False),
}


def expected_lines(triples, ms, strategy, clean):
    return R.format_cinds(R.rdfind(triples, ms, strategy, clean, full_prune=True))


def main():
    os.makedirs(OUT, exist_ok=True)
    for name, (make, ms) in FIXTURES.items():
        d = make()
        path = os.path.join(OUT, f"{name}.nt.gz")
        lines = list(d.lines())
        ntriples.write_ntriples(path, lines)
        # re-read through the parser so the oracle sees exactly what every consumer sees
        s, p, o, dic = ntriples.read_triples([path])
        triples = [(dic.term(a), dic.term(b), dic.term(c)) for a, b, c in zip(s.tolist(), p.tolist(), o.tolist())]
        for mode, (strategy, clean) in MODES.items():
            out = expected_lines(triples, ms, strategy, clean)
            with gzip.open(os.path.join(OUT, f"{name}.{mode}.txt.gz"), "wt", encoding="utf-8") as f:
                f.write(f"# min_support={ms} traversal_strategy={strategy} clean_implied={clean}\n")
                for ln in out:
                    f.write(ln + "\n")
            print(name, mode, len(lines), "triples", len(out), "cinds")


if __name__ == "__main__":
    main()
