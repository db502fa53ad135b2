"""The C restatement (oracle/c/rdfind_oracle.c) against the literal Python restatement and the goldens."""
import random

import numpy as np
import pytest

from oracle import c_oracle as C, rdfind_oracle as R
from rdfind_amd import ntriples
from tests import kats
from tests.test_oracle import golden_triples, read_golden
import os
from tests.conftest import GOLDEN


def _py(tr, ms, strategy, clean):
    if strategy == 1 and not clean:  # the C oracle's strategy-1 raw mode is the full valid set V
        uf = R.frequent_unary_conditions(tr, ms)
        lines = R.join_lines(tr, uf, R.frequent_binary_conditions(tr, uf, ms))
        return R.cind_set(R.all_at_once(lines, ms, False, literal_implies=False))
    return R.cind_set(R.rdfind(tr, ms, strategy, clean))


def test_c_oracle_matches_python_random():
    rng = random.Random(1)
    for _ in range(120):
        n = rng.randrange(1, 120)
        nv = rng.randrange(2, 25)
        ms = rng.randrange(1, 5)
        arr = np.array([(rng.randrange(nv), rng.randrange(nv // 3 + 1), rng.randrange(nv)) for _ in range(n)],
                       dtype=np.uint32)
        tr = [tuple(x) for x in arr.tolist()]
        for strategy in (0, 1):
            for clean in (True, False):
                got, _ = C.run_set(arr[:, 0], arr[:, 1], arr[:, 2], nv, ms, strategy, clean)
                assert got == _py(tr, ms, strategy, clean), (n, nv, ms, strategy, clean)


def test_c_oracle_projection_subsets():
    rng = random.Random(2)
    for _ in range(30):
        arr = np.array([(rng.randrange(9), rng.randrange(4), rng.randrange(9)) for _ in range(40)], dtype=np.uint32)
        tr = [tuple(x) for x in arr.tolist()]
        for proj in ("s", "po", "sp", "o"):
            got, _ = C.run_set(arr[:, 0], arr[:, 1], arr[:, 2], 9, 2, 1, True, proj)
            exp = R.cind_set(R.rdfind(tr, 2, 1, True, projection=proj))
            assert got == exp, proj


def test_c_oracle_empty_input():
    e = np.zeros(0, np.uint32)
    got, st = C.run_set(e, e, e, 1, 1, 1, True)
    assert got == set() and st["n_records"] == 0


@pytest.mark.parametrize("name", ["zipf_small", "lubm_small", "skew_small"])
@pytest.mark.parametrize("mode,strategy,clean", [("s1_clean", 1, True), ("s0_clean", 0, True), ("s0_raw", 0, False)])
def test_c_oracle_reproduces_golden(name, mode, strategy, clean):
    ms, expected = read_golden(name, mode)
    s, p, o, dic = ntriples.read_triples([os.path.join(GOLDEN, f"{name}.nt.gz")])
    got, _ = C.run_set(s, p, o, dic.size, ms, strategy, clean)
    lines = R.format_cinds([R.Cind(*x) for x in got], dic.term)
    assert lines == expected


@pytest.mark.parametrize("kat", kats.RULE_KATS, ids=lambda k: k["name"])
def test_rule_kats_c_oracle(kat):
    """The hand-derived KATs (tests/kats.py) through the C restatement: clean in both strategies, strategy 0 raw, and
    strategy 1 raw (the C oracle's raw strategy-1 mode is the valid set V)."""
    arr, dic = kats.encode(kat)
    ms, proj = kat["support"], kat["projection"]
    run = lambda strategy, clean: kats.lines_of(C.run_set(arr[:, 0], arr[:, 1], arr[:, 2], dic.size, ms, strategy,
                                                          clean, proj)[0], dic.term)
    assert run(1, True) == run(0, True) == kats.expected(kat, "clean")
    assert run(0, False) == kats.expected(kat, "s0_raw")
    assert run(1, False) == sorted(kat["v"])
