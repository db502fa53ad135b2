"""GPU parity for --use-ars (rdf_association_rules + the AR-aware discovery, rdfind_amd/csrc/ars.inl) against the
oracle: the rules themselves, and the CIND sets in every mode (strategy 0 / S2L x --clean-implied), on random
inputs, with the heavy-group paths forced, and through the RDFind-compatible driver (--use-ars / --ar-output)."""
import random

import numpy as np
import pytest

from oracle import rdfind_oracle as R
from rdfind_amd import _lib, ntriples, program, synth
from tests.test_oracle import KAT_PEOPLE
from tests.test_oracle_ars import KAT_PEOPLE_ARS, KAT_PEOPLE_RULES

pytestmark = pytest.mark.gpu

MODES = [(1, True), (0, True), (0, False), (1, False)]
CODE = {R.S: 1, R.P: 2, R.O: 4}


@pytest.fixture(scope="module")
def ctx():
    c = _lib.Context(0)
    yield c
    c.close()


def expected(tr, ms, strategy, clean):
    if strategy == 0:
        return R.cind_set(R.rdfind(tr, ms, 0, clean, use_ars=True))
    # S2L: the closed form (tests/test_oracle_ars.py checks it against the literal S2L plan)
    uf = R.frequent_unary_conditions(tr, ms)
    bf = R.frequent_binary_conditions(tr, uf, ms)
    rules = R.association_rules(uf, bf)
    lines = R.join_lines(tr, uf, bf, "spo", True, R.ar_implied_conditions(rules))
    v = R.all_at_once(lines, ms, False, literal_implies=False)
    return R.cind_set(R.s2l_ars_closed_form(v, R.ar_implied_cinds(rules), clean))


def gpu_run(g, arr, nv, ms, strategy, clean):
    g.set_triples(arr[:, 0], arr[:, 1], arr[:, 2], nv)
    g.frequent_conditions(ms)
    g.association_rules()
    rules = g.copy_association_rules()
    g.build_capture_groups("spo")
    g.discover_cinds(clean, strategy)
    return _lib.decoded_to_set(g.decoded_cinds()), rules


def _random_case(rng, nmax=250, pdiv=3):
    n = rng.randrange(1, nmax)
    nv = rng.randrange(2, 30)
    ms = rng.randrange(1, 4)
    arr = np.array([(rng.randrange(nv), rng.randrange(nv // pdiv + 1), rng.randrange(nv)) for _ in range(n)],
                   dtype=np.uint32)
    return arr, nv, ms


def test_rules_and_cinds_random(ctx):
    rng = random.Random(21)
    n_rules = 0
    for _ in range(80):
        arr, nv, ms = _random_case(rng)
        tr = [tuple(x) for x in arr.tolist()]
        uf = R.frequent_unary_conditions(tr, ms)
        exp_rules = {(CODE[ta], CODE[tc], va, vc, n)
                     for ta, tc, va, vc, n in R.association_rules(uf, R.frequent_binary_conditions(tr, uf, ms))}
        n_rules += len(exp_rules)
        for strategy, clean in MODES:
            got, rules = gpu_run(ctx, arr, nv, ms, strategy, clean)
            assert {tuple(r) for r in rules.tolist()} == exp_rules
            assert got == expected(tr, ms, strategy, clean), (len(tr), nv, ms, strategy, clean)
    assert n_rules > 50


@pytest.mark.parametrize("heavy_min", [1, 4])
def test_heavy_paths_with_ars(monkeypatch, heavy_min):
    """Heavy groups as bitmask columns: the heavy-only unary dependents then take k_heavy (not the mask classes),
    with the per-dependent AR filter and the R3 mark pass."""
    monkeypatch.setenv("RDFIND_HEAVY_MIN", str(heavy_min))
    g = _lib.Context(0)
    try:
        rng = random.Random(300 + heavy_min)
        for _ in range(40):
            arr, nv, ms = _random_case(rng, 400, 4)
            tr = [tuple(x) for x in arr.tolist()]
            for strategy, clean in MODES:
                got, _ = gpu_run(g, arr, nv, ms, strategy, clean)
                assert got == expected(tr, ms, strategy, clean), (len(tr), nv, ms, strategy, clean, heavy_min)
        assert g.groups["n_heavy_groups"] > 0
    finally:
        g.close()


def test_synthetic_config_with_ars(ctx):
    d = synth.config("c1", 0.003)
    tr = list(zip(d.s.tolist(), d.p.tolist(), d.o.tolist()))
    arr = np.stack([d.s, d.p, d.o], axis=1).astype(np.uint32)
    for strategy, clean in ((1, True), (0, True)):
        got, rules = gpu_run(ctx, arr, d.num_terms, d.min_support, strategy, clean)
        assert len(rules) > 0
        assert got == expected(tr, d.min_support, strategy, clean)


def test_program_use_ars_and_ar_output(tmp_path):
    nt = tmp_path / "people.nt"
    nt.write_text("".join(f"{s} {p} {o} .\n" for s, p, o in KAT_PEOPLE))
    for flags in (["--use-fis"], ["--traversal-strategy", "0", "--use-fis"]):
        out, ars = tmp_path / "cinds.txt", tmp_path / "rules.txt"
        program.RDFind(flags + ["--use-ars", "--clean-implied", "--support", "2", "--output", str(out),
                                "--ar-output", str(ars), str(nt)]).run()
        assert sorted(out.read_text().splitlines()) == KAT_PEOPLE_ARS
        assert ars.read_text().splitlines() == KAT_PEOPLE_RULES
    # --ar-output alone prints the rules and leaves the CINDs as without --use-ars
    out2, ars2 = tmp_path / "c2.txt", tmp_path / "r2.txt"
    program.RDFind(["--use-fis", "--clean-implied", "--support", "2", "--output", str(out2), "--ar-output", str(ars2),
                    str(nt)]).run()
    assert ars2.read_text().splitlines() == KAT_PEOPLE_RULES
    assert sorted(out2.read_text().splitlines()) == R.format_cinds(R.rdfind(KAT_PEOPLE, 2, 1, True))


def test_ars_state_and_errors(ctx):
    arr = np.array([[0, 1, 2], [3, 1, 2], [0, 1, 4]], np.uint32)
    ctx.set_triples(arr[:, 0], arr[:, 1], arr[:, 2], 5)
    with pytest.raises(_lib.RdfError):
        ctx.association_rules()  # before rdf_frequent_conditions
    ctx.frequent_conditions(1)
    ctx.association_rules()
    with pytest.raises(_lib.RdfError):
        ctx.association_rules()  # twice on the same frequent conditions
    ctx.frequent_conditions(1)  # resets: discovery without rules again
    ctx.build_capture_groups("spo")
    ctx.discover_cinds(True, 1)
    tr = [tuple(x) for x in arr.tolist()]
    assert _lib.decoded_to_set(ctx.decoded_cinds()) == R.cind_set(R.rdfind(tr, 1, 1, True))
    with pytest.raises(_lib.RdfError):
        ctx.shard_begin(2, 2, 1, use_ars=True)  # rank outside [0, nranks)
    ctx.shard_begin(0, 1, 1, use_ars=True)  # sharded rules are supported
