"""Full-size parity: the HIP path on BASELINE configs at the largest size one MI355X holds, against the C
oracle's golden vectors (tests/golden/full_size.json, made by tools/make_full_golden.py with the streamed
oracle: count + order-independent checksum of (dep, ref, support) rows + stage counts).

* c1 at full size is also compared row by row with the materializing oracle (set equality);
* c3 at full size additionally verifies sampled CINDs directly against the triples.
"""
import json
import os

import numpy as np
import pytest

from rdfind_amd import _lib
from tests.conftest import GOLDEN
from tests.parity import dataset, dataset_npz

pytestmark = pytest.mark.gpu

GOLD = json.load(open(os.path.join(GOLDEN, "full_size.json")))


@pytest.fixture(scope="module")
def ctx():
    c = _lib.Context(0)
    yield c
    c.close()


def fingerprint(d):
    from tools.make_full_golden import fingerprint as fp
    return fp(d)


# golden entries whose result exceeds one GPU's HBM at once: checked page by page (test_paged_full_size_vs_oracle);
# c4 at 10^9 triples has its own test (test_c4_full_size_one_gpu), which checks the same golden entry
PAGED_ONLY = {"c5@1.0/s1_clean"}
OWN_TEST = {"c4@1.0/s1_clean"}


@pytest.mark.timeout(300)
@pytest.mark.parametrize("key", sorted(set(GOLD) - PAGED_ONLY - OWN_TEST))
def test_full_size_vs_oracle(ctx, key):
    g = GOLD[key]
    d = dataset(g["config"], g["scale"])
    assert d.n == g["n_triples"] and d.num_terms == g["num_terms"]
    assert str(fingerprint(d)) == g["fingerprint"], "synthetic generator drifted from the golden input"
    ctx.set_triples(d.s, d.p, d.o, d.num_terms)
    ctx.run(d.min_support, "spo", g["clean"], g["strategy"])
    assert ctx.fc["n_frequent_unary"] == g["n_freq_unary"]
    assert ctx.fc["n_frequent_binary"] == g["n_freq_binary"]
    assert ctx.groups["n_records"] == g["n_records"]
    assert ctx.groups["n_captures"] == g["n_freq_captures"]
    assert ctx.cind_count() == g["n_cinds"]
    # the compact hand-over (shared lists not expanded), expanded by the checker
    from oracle import c_oracle as C
    n, h, kind = C.checksum_compact(ctx.copy_result_compact(), d.num_terms)
    assert (n, h, kind) == (g["n_cinds"], int(g["checksum"]), g["n_kind"])
    assert ctx.checksum() == int(g["checksum"])  # the device's own expansion


def _packed(dep, ref, sup):
    key = (dep.astype(np.uint64) << np.uint64(32)) | ref.astype(np.uint64)
    order = np.argsort(key)
    return key[order], sup[order]


@pytest.mark.timeout(300)
def test_c1_full_rows_vs_oracle(ctx):
    """c1 (1M triples) at full size: every result row equals the materializing oracle's."""
    from oracle import c_oracle as C
    d = dataset("c1", 1.0)
    for strategy, clean in ((1, True), (0, True), (0, False)):
        rows, _, st = C.run(d.s, d.p, d.o, d.num_terms, d.min_support, strategy, clean)
        ctx.set_triples(d.s, d.p, d.o, d.num_terms)
        ctx.run(d.min_support, "spo", clean, strategy)
        got = ctx.copy_cinds()
        assert got.shape[0] == rows.shape[0] == st["n_cinds"]
        ek, es = _packed(rows["dep"], rows["ref"], rows["support"])
        gk, gs = _packed(got["dep"], got["ref"], got["support"])
        np.testing.assert_array_equal(gk, ek)
        np.testing.assert_array_equal(gs, es)


def _capture_joins(d, code, v1, v2):
    cols = {1: d.s, 2: d.p, 4: d.o}
    prim, proj = code & 7, (code >> 3) & 7
    first = prim & -prim
    second = prim & ~first
    mask = cols[first] == v1
    if second:
        mask &= cols[second] == v2
    return np.unique(cols[proj][mask])


@pytest.mark.timeout(600)
def test_c3_full_sampled_direct_verification(ctx):
    """c3 (100M triples, support 25) at full size: sampled CINDs hold on the triples themselves (every join value
    of the dependent is one of the referenced capture, support = the dependent's distinct join values)."""
    g = GOLD["c3@1.0/s1_clean"]
    d = dataset("c3", 1.0)
    ctx.set_triples(d.s, d.p, d.o, d.num_terms)
    ctx.run(d.min_support)
    n = ctx.cind_count()
    assert n == g["n_cinds"]
    rng = np.random.default_rng(3)
    offs = rng.choice(n, size=min(16, n), replace=False)
    sample = np.concatenate([ctx.copy_cinds_range(int(o), 1) for o in offs])
    dec = _lib.decode_rows(sample, d.num_terms, ctx.binary_keys())
    for dc, d1, d2, rc, r1, r2, sup in dec.tolist():
        jd = _capture_joins(d, dc, d1, d2)
        jr = _capture_joins(d, rc, r1, r2)
        assert len(jd) == sup >= d.min_support
        assert np.isin(jd, jr).all()


@pytest.mark.timeout(600)
def test_join_ranges_full_size_vs_oracle(monkeypatch):
    """c4 at 0.1 (10^8 triples, 5.6·10^8 records) with its capture groups built in join-value ranges of <= 10^8 records
    (RDFIND_GROUP_RANGE; the automatic path of inputs >= 2^32/9 triples) gives the golden vector."""
    g = GOLD["c4@0.1/s1_clean"]
    d = dataset(g["config"], g["scale"])
    monkeypatch.setenv("RDFIND_GROUP_RANGE", str(100_000_000))
    with _lib.Context(0) as c:
        c.set_triples(d.s, d.p, d.o, d.num_terms)
        c.run(d.min_support, "spo", g["clean"], g["strategy"])
        assert c.groups["n_join_ranges"] >= 5
        assert c.groups["n_records"] == g["n_records"] and c.groups["n_captures"] == g["n_freq_captures"]
        assert (c.cind_count(), c.checksum()) == (g["n_cinds"], int(g["checksum"]))


def _sample_verify(ctx, d, k, seed):
    """k sampled CINDs of the current result hold on the triples themselves: every join value of the dependent is one
    of the referenced capture's, and the support is the dependent's number of distinct join values."""
    n = ctx.cind_count()
    rng = np.random.default_rng(seed)
    offs = rng.choice(n, size=min(k, n), replace=False)
    sample = np.concatenate([ctx.copy_cinds_range(int(o), 1) for o in offs])
    dec = _lib.decode_rows(sample, d.num_terms, ctx.binary_keys())
    for dc, d1, d2, rc, r1, r2, sup in dec.tolist():
        jd = _capture_joins(d, dc, d1, d2)
        jr = _capture_joins(d, rc, r1, r2)
        assert len(jd) == sup >= d.min_support
        assert np.isin(jd, jr).all()


@pytest.mark.timeout(300)
def test_c4_full_size_one_gpu(ctx):
    """c4 at its BASELINE size (Freebase-shaped, 10^9 triples, support 100) on one MI355X.  Its ~5.8·10^9 capture
    records exceed one sort's u32 offsets, so the capture groups are built in join-value ranges (the reference's
    sort-based groupBy spills instead, ALG/programs/RDFind.scala:339-345).  One run, checked against the streamed
    oracle's golden vector (stage counts, count, checksum), through the compact hand-over expanded by the checker, and
    by sampled CINDs verified on the triples; then run again in the same context, which must give the same ranges,
    records, count and checksum.  Other range splits are parity-tested at c4 at 0.1
    (test_join_ranges_full_size_vs_oracle) and on random inputs (test_gpu.py::test_join_range_groups_parity)."""
    from oracle import c_oracle as C

    g = GOLD["c4@1.0/s1_clean"]
    d = dataset("c4", 1.0)
    assert d.n == 1_000_000_000 == g["n_triples"]
    assert str(fingerprint(d)) == g["fingerprint"]
    ctx.set_triples(d.s, d.p, d.o, d.num_terms)
    ctx.run(d.min_support)
    assert ctx.groups["n_join_ranges"] > 1
    assert ctx.groups["n_records"] > 2 ** 32  # more records than one pass addresses
    assert ctx.fc["n_frequent_unary"] == g["n_freq_unary"] and ctx.fc["n_frequent_binary"] == g["n_freq_binary"]
    assert ctx.groups["n_records"] == g["n_records"] and ctx.groups["n_captures"] == g["n_freq_captures"]
    assert (ctx.cind_count(), ctx.checksum()) == (g["n_cinds"], int(g["checksum"]))
    n, h, kind = C.checksum_compact(ctx.copy_result_compact(), d.num_terms)
    assert (n, h, kind) == (g["n_cinds"], int(g["checksum"]), g["n_kind"])
    _sample_verify(ctx, d, 10, 4)
    # determinism at the scale where the records exceed 2^32: a second run in the same context (kept-store ranges, the
    # buffers of the first run reused) gives the same ranges, records and result
    first = (ctx.groups["n_join_ranges"], ctx.groups["n_records"], ctx.cind_count(), ctx.checksum())
    ctx.run(d.min_support)
    assert (ctx.groups["n_join_ranges"], ctx.groups["n_records"], ctx.cind_count(), ctx.checksum()) == first


_VARIANT_CHILD = r"""
import json, sys
sys.path.insert(0, sys.argv[1])
from rdfind_amd import _lib
from tests.parity import load_npz
out = []
with _lib.Context(0) as ctx:
    for g, path in json.loads(sys.argv[2]):
        s, p, o, nv, ms = load_npz(path)
        ctx.set_triples(s, p, o, nv)
        ctx.run(ms, "spo", g["clean"], g["strategy"])
        out.append({"n": ctx.cind_count(), "sum": str(ctx.checksum())})
print(json.dumps(out))
"""


@pytest.mark.timeout(300)
@pytest.mark.parametrize("env", [{"RDFIND_STAGE": "0"}, {"RDFIND_STAGE": "1"},
                                 {"RDFIND_SIG": "0", "RDFIND_PIV2": "0"}, {"RDFIND_SIG": "1", "RDFIND_PIV2": "2"},
                                 {"RDFIND_DENSE": "0"}, {"RDFIND_DENSE": "256"}, {"RDFIND_LIGHT2": "1"},
                                 {"RDFIND_LIGHT2": "1", "RDFIND_DENSE": "0"},
                                 {"RDFIND_SWEEP_F": "0"}, {"RDFIND_SWEEP_F": "1000000000"},
                                 {"RDFIND_SWEEP_F": "1000000000", "RDFIND_LIGHT2": "1", "RDFIND_DENSE": "0"},
                                 {"RDFIND_LIGHT_HIOCC": "1"}, {"RDFIND_LIGHT_HIOCC": "0"}, {"RDFIND_PIVX": "0"},
                                 {"RDFIND_LIGHT_DEDUP": "0"}, {"RDFIND_LIGHT_DEDUP": "1"},
                                 {"RDFIND_LIGHT_DEDUP": "1", "RDFIND_DUP_MIN": "1"},
                                 {"RDFIND_PIVX_N": "2"}, {"RDFIND_PIVX_PACKED": "1"}])
def test_light_variants_full_size(ctx, env):
    """The light pass's alternative code paths (LDS-staged small groups or not, signature filter off / on both
    paths, second pivot off / k_light only, dense-group bitmaps off / for groups of >= C/256 members, the filter and
    verify passes forced instead of one light pass (with and without bitmaps), window range sweeps
    never / whenever many candidates are alive, the plain variant at 6 waves per SIMD forced on / off, no extra pivots /
    two, every light dependent verified on its own instead of once per class of equal group lists, or every list of
    any length looking for an equal one) each reproduce the c1 and c2 golden vectors (and c4 at 0.1 for the sweep, two-pass, occupancy and pivot
    switches).  The switches are read
    once per process, so each combination runs in its own child process."""
    import subprocess
    import sys

    ctx.release_scratch()  # the module context's buffers from the full-size runs (c5 at 0.3: ~100 GB) would starve the child
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    keys = ["c1@1.0/s1_clean", "c2@1.0/s1_clean"]
    if {"RDFIND_SWEEP_F", "RDFIND_LIGHT2", "RDFIND_LIGHT_HIOCC", "RDFIND_PIVX", "RDFIND_PIVX_N", "RDFIND_LIGHT_DEDUP",
            "RDFIND_PIVX_PACKED"} & set(env):  # c4 runs these
        keys.append("c4@0.1/s1_clean")
    jobs = [(GOLD[key], dataset_npz(GOLD[key]["config"], GOLD[key]["scale"])) for key in keys]
    r = subprocess.run([sys.executable, "-c", _VARIANT_CHILD, root, json.dumps(jobs)], env=dict(os.environ, **env),
                       capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-2000:]
    for key, got in zip(keys, json.loads(r.stdout.strip().splitlines()[-1])):
        g = GOLD[key]
        assert got["n"] == g["n_cinds"] and got["sum"] == g["checksum"], (key, env, got)


@pytest.mark.timeout(300)
@pytest.mark.parametrize("key,page_bytes", [("c5@0.3/s1_clean", 4 << 30), ("c5@1.0/s1_clean", 0)])
def test_paged_full_size_vs_oracle(ctx, key, page_bytes):
    """Paged discovery (bounded HBM per page) at the pair-explosion config: the pages' counts and checksums (device
    expansion, and the compact hand-over expanded by the checker) sum to the streamed oracle's golden vector.  c5 at
    scale 1.0 is the BASELINE size; its result does not fit in HBM at once."""
    from oracle import c_oracle as C

    if key not in GOLD:
        pytest.skip(f"{key} golden vector not generated")
    g = GOLD[key]
    d = dataset(g["config"], g["scale"])
    assert str(fingerprint(d)) == g["fingerprint"], "synthetic generator drifted from the golden input"
    ctx.set_triples(d.s, d.p, d.o, d.num_terms)
    ctx.frequent_conditions(d.min_support)
    ctx.build_capture_groups("spo")
    n = h = hc = pages = 0
    for _ in ctx.pages(g["clean"], g["strategy"], page_bytes):
        cnt, hh, _ = C.checksum_compact(ctx.copy_result_compact(), d.num_terms)
        assert cnt == ctx.cind_count()
        n += cnt
        hc = (hc + hh) % (1 << 64)
        h = (h + ctx.checksum()) % (1 << 64)
        pages += 1
    assert pages >= 2
    assert n == g["n_cinds"] and h == int(g["checksum"]) and hc == h


_TWO_PASS_CHILD = r"""
import json, random, sys
sys.path.insert(0, sys.argv[1])
import numpy as np
from rdfind_amd import _lib
from oracle import c_oracle as C
rng = random.Random(int(sys.argv[2]))
bad = []
with _lib.Context(0) as g:
    for it in range(40):
        n = rng.randrange(50, 600)
        nv = rng.randrange(4, 40)
        ms = rng.randrange(1, 3)
        arr = np.array([(rng.randrange(nv), rng.randrange(nv // 4 + 1), rng.randrange(nv)) for _ in range(n)],
                       dtype=np.uint32)
        for strategy, clean in ((1, True), (0, True), (0, False)):
            exp, _ = C.run_set(arr[:, 0], arr[:, 1], arr[:, 2], nv, ms, strategy, clean)
            g.set_triples(arr[:, 0], arr[:, 1], arr[:, 2], nv)
            g.run(ms, "spo", clean, strategy)
            if _lib.decoded_to_set(g.decoded_cinds()) != exp:
                bad.append((it, n, nv, ms, strategy, clean))
print(json.dumps({"bad": bad}))
"""


@pytest.mark.timeout(300)
@pytest.mark.parametrize("heavy_min", ["64", "2"])
def test_two_light_passes_random(ctx, heavy_min):
    """The filter + verify light passes forced on random inputs (RDFIND_LIGHT2=1; LIGHT_PRE_MAX defers every chunk of
    a multi-chunk dependent) against the C oracle in three modes, with and without lowered heavy columns.  In its own
    process: the switch is read once per process."""
    import subprocess
    import sys

    ctx.release_scratch()  # the module context's pages of c5 at full size stay allocated otherwise
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, RDFIND_LIGHT2="1", RDFIND_HEAVY_MIN=heavy_min)
    r = subprocess.run([sys.executable, "-c", _TWO_PASS_CHILD, root, "71" + heavy_min], env=env, capture_output=True,
                       text=True, timeout=280)
    assert r.returncode == 0, r.stderr[-2000:]
    assert json.loads(r.stdout.strip().splitlines()[-1])["bad"] == []
