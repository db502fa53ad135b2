"""The oracle itself: hand-derived known answers, the S2L == AllAtOnce cross-check, golden fixtures.

There are no golden CIND vectors in the reference; these tests pin the two independent
restatements against each other and against hand-derived results."""
import gzip
import os
import random

import pytest
from hypothesis import given, settings, strategies as st

from oracle import rdfind_oracle as R
from rdfind_amd import ntriples
from tests import kats
from tests.conftest import GOLDEN

# hand-derived: see DESIGN.md "known-answer test" for the derivation
KAT_PEOPLE = [("<a>", "<type>", "<Person>"), ("<b>", "<type>", "<Person>"), ("<a>", "<name>", '"A"'),
              ("<b>", "<name>", '"B"'), ("<c>", "<type>", "<City>")]
KAT_PEOPLE_CLEAN = sorted([
    "p[s=<a>] < p[s=<b>] (support=2)",
    "p[s=<b>] < p[s=<a>] (support=2)",
    "s[o=<Person>] < s[p=<name>] (support=2)",
    "s[p=<name>] < s[p=<type>,o=<Person>] (support=2)",
    "s[o=<Person>] < s[p=<type>,o=<Person>] (support=2)",
])
KAT_PEOPLE_RAW = sorted(KAT_PEOPLE_CLEAN + [
    "s[p=<name>] < s[p=<type>] (support=2)",         # R3 (via s[p=<name>] < s[p=<type>,o=<Person>])
    "s[p=<name>] < s[o=<Person>] (support=2)",       # R3
    "s[o=<Person>] < s[p=<type>] (support=2)",       # R3
    "s[p=<type>,o=<Person>] < s[p=<name>] (support=2)",  # R1 (via s[o=<Person>] < s[p=<name>])
])


def test_kat_people_clean_both_strategies():
    for strategy in (0, 1):
        assert R.format_cinds(R.rdfind(KAT_PEOPLE, 2, strategy, True)) == KAT_PEOPLE_CLEAN


def test_kat_people_raw():
    assert R.format_cinds(R.rdfind(KAT_PEOPLE, 2, 0, False)) == KAT_PEOPLE_RAW


# strategy-0 quirk: Condition.isImpliedBy compares this.v1 with that.v2 for same-type binary captures
KAT_QUIRK = [("<x>", "<P>", "<y>"), ("<y>", "<P>", "<z>")]


def test_kat_literal_implies_quirk():
    lines1 = set(R.format_cinds(R.small_to_large(_lines(KAT_QUIRK, 1), _bfc(KAT_QUIRK, 1), 1, False,
                                                 full_prune=True)))
    lines0 = set(R.format_cinds(R.rdfind(KAT_QUIRK, 1, 0, False)))
    d_lt_x = "p[s=<x>,o=<y>] < p[s=<y>,o=<z>] (support=1)"
    x_lt_d = "p[s=<y>,o=<z>] < p[s=<x>,o=<y>] (support=1)"
    # S2L's raw output keeps no 2/2 CIND here (R4 via p[s=<x>] < p[s=<y>,o=<z>]); V has both
    uf = R.frequent_unary_conditions(KAT_QUIRK, 1)
    v = set(R.format_cinds(R.all_at_once(R.join_lines(KAT_QUIRK, uf, R.frequent_binary_conditions(KAT_QUIRK, uf, 1)),
                                         1, False, literal_implies=False)))
    assert d_lt_x in v and x_lt_d in v
    assert x_lt_d in lines0 and d_lt_x not in lines0  # X.v1 == D.v2 -> dropped by the literal filter
    assert d_lt_x not in lines1


def _lines(triples, ms):
    uf = R.frequent_unary_conditions(triples, ms)
    return R.join_lines(triples, uf, R.frequent_binary_conditions(triples, uf, ms))


def _bfc(triples, ms):
    return R.frequent_binary_conditions(triples, R.frequent_unary_conditions(triples, ms), ms)


triples_st = st.lists(st.tuples(st.integers(0, 9), st.integers(0, 3), st.integers(0, 9)), min_size=1, max_size=60)


@settings(max_examples=60, deadline=None)
@given(triples_st, st.integers(1, 3), st.integers(0, 10**6))
def test_s2l_equals_semantic_all_at_once(triples, ms, seed):
    """S2L + clean-implied == remove_implied(V), independent of candidate Bloom false positives and of
    the order-dependent 2/2 prune (checked rather than assumed)."""
    v = R.all_at_once(_lines(triples, ms), ms, True, literal_implies=False)
    s2l = R.rdfind(triples, ms, 1, True, bloom_fpp=0.25, prune_seed=seed)
    assert R.cind_set(s2l) == R.cind_set(v)


@settings(max_examples=40, deadline=None)
@given(triples_st, st.integers(1, 3))
def test_literal_strategy0_differs_only_by_quirk(triples, ms):
    lines = _lines(triples, ms)
    raw_sem = R.cind_set(R.all_at_once(lines, ms, False, literal_implies=False))
    raw_lit = R.cind_set(R.all_at_once(lines, ms, False, literal_implies=True))
    diff = raw_sem - raw_lit
    assert raw_lit <= raw_sem
    for dt, dv1, dv2, rt, rv1, rv2, _ in diff:
        assert dt == rt and R.is_binary(dt) and rv1 == dv2


@settings(max_examples=40, deadline=None)
@given(triples_st, st.integers(1, 3))
def test_s2l_exact_raw_formula(triples, ms):
    v = R.all_at_once(_lines(triples, ms), ms, False, literal_implies=False)
    assert R.cind_set(R.s2l_exact_raw(v)) == R.cind_set(R.rdfind(triples, ms, 1, False, full_prune=True))


def test_fc_filters_are_inert():
    rng = random.Random(4)
    for _ in range(30):
        tr = [(rng.randrange(8), rng.randrange(3), rng.randrange(8)) for _ in range(rng.randrange(1, 50))]
        ms = rng.randrange(1, 4)
        assert R.cind_set(R.rdfind(tr, ms, 0, True, use_fis=True)) == R.cind_set(R.rdfind(tr, ms, 0, True, use_fis=False))


def read_golden(name, mode):
    with gzip.open(os.path.join(GOLDEN, f"{name}.{mode}.txt.gz"), "rt", encoding="utf-8") as f:
        header = f.readline()
        ms = int(header.split("min_support=")[1].split()[0])
        return ms, [ln.rstrip("\n") for ln in f]


def golden_triples(name):
    s, p, o, dic = ntriples.read_triples([os.path.join(GOLDEN, f"{name}.nt.gz")])
    return [(dic.term(a), dic.term(b), dic.term(c)) for a, b, c in zip(s.tolist(), p.tolist(), o.tolist())]


@pytest.mark.parametrize("name", ["zipf_small", "skew_small"])
@pytest.mark.parametrize("mode,strategy,clean", [("s1_clean", 1, True), ("s0_clean", 0, True), ("s0_raw", 0, False)])
def test_python_oracle_reproduces_golden(name, mode, strategy, clean):
    ms, expected = read_golden(name, mode)
    got = R.format_cinds(R.rdfind(golden_triples(name), ms, strategy, clean, full_prune=True))
    assert got == expected


@pytest.mark.parametrize("kat", kats.RULE_KATS, ids=lambda k: k["name"])
def test_rule_kats_python_oracle(kat):
    """Hand-derived KATs (tests/kats.py) for R1-R4 and the 1/2, 2/1, 2/2 paths: the valid set V, both strategies'
    clean output, S2L's raw output and strategy 0's raw output."""
    tr, ms, proj = kat["triples"], kat["support"], kat["projection"]
    uf = R.frequent_unary_conditions(tr, ms)
    v = R.all_at_once(R.join_lines(tr, uf, R.frequent_binary_conditions(tr, uf, ms), proj), ms, False,
                      literal_implies=False)
    assert R.format_cinds(v) == sorted(kat["v"])
    for strategy in (0, 1):
        assert R.format_cinds(R.rdfind(tr, ms, strategy, True, projection=proj)) == kats.expected(kat, "clean")
    assert R.format_cinds(R.rdfind(tr, ms, 1, False, projection=proj, full_prune=True)) == kats.expected(kat, "s2l_raw")
    # the candidate Bloom filters' false positives and the 2/2 prune's order do not change S2L's clean output
    for seed in range(3):
        assert R.format_cinds(R.rdfind(tr, ms, 1, True, projection=proj, bloom_fpp=0.5, prune_seed=seed)) == \
            kats.expected(kat, "clean")
    assert R.format_cinds(R.rdfind(tr, ms, 0, False, projection=proj)) == kats.expected(kat, "s0_raw")


def test_rule_kats_cover_every_rule_and_path():
    """Every rule removes at least one hand-derived line, and every CIND kind survives in some clean result."""
    removed = {rule for k in kats.RULE_KATS for rule in k["v"].values() if rule}
    assert removed == {"R1", "R2", "R3", "R4"}
    kinds = [set(i for i, part in enumerate(kats.split(kats.expected(k, "clean"))) if part) for k in kats.RULE_KATS]
    assert set().union(*kinds) == {0, 1, 2, 3}  # 1/1, 1/2, 2/1, 2/2 all present in some clean output
