"""GPU parity: the HIP path (through the C ABI) against the oracle.

* bit-exact CIND sets vs the C/Python restatements on random inputs, edge cases and scaled BASELINE
  configs, in every mode (strategy 0/1 x --clean-implied on/off);
* the golden fixtures through the full program (N-Triples -> GPU -> Cind.toString lines);
* at the bench size (c2 = LUBM-100 shape), size-independent properties: determinism, rule
  monotonicity (clean <= S2L-raw <= V), and direct verification of sampled CINDs against the triples.
"""
import os
import random

import numpy as np
import pytest

from oracle import c_oracle as C, rdfind_oracle as R
from rdfind_amd import _lib, ntriples, program, synth
from tests import kats
from tests.conftest import GOLDEN
from tests.parity import assert_rows_equal, assert_stream_matches, dataset, oracle_stream
from tests.test_oracle import KAT_PEOPLE, KAT_PEOPLE_CLEAN, KAT_PEOPLE_RAW, read_golden

pytestmark = pytest.mark.gpu

MODES = [(1, True), (0, True), (0, False), (1, False)]


@pytest.fixture(scope="module")
def ctx():
    c = _lib.Context(0)
    yield c
    c.close()


def expected_set(arr, nv, ms, strategy, clean):
    if strategy == 1 and not clean:  # exact-candidate S2L raw output (oracle.s2l_exact_raw)
        tr = [tuple(x) for x in arr.tolist()]
        uf = R.frequent_unary_conditions(tr, ms)
        v = R.all_at_once(R.join_lines(tr, uf, R.frequent_binary_conditions(tr, uf, ms)), ms, False,
                          literal_implies=False)
        return R.cind_set(R.s2l_exact_raw(v))
    got, _ = C.run_set(arr[:, 0], arr[:, 1], arr[:, 2], nv, ms, strategy, clean)
    return got


def gpu_set(ctx, arr, nv, ms, strategy, clean, projection="spo"):
    ctx.set_triples(arr[:, 0], arr[:, 1], arr[:, 2], nv)
    ctx.run(ms, projection, clean, strategy)
    return _lib.decoded_to_set(ctx.decoded_cinds())


def compact_matches(ctx, nv):
    """The compact hand-over (rdf_copy_result_compact: explicit runs + shared lists) expands to the same rows as the
    device's own expansion: count and order-independent checksum."""
    parts = ctx.copy_result_compact()
    n, h, _ = C.checksum_compact(parts, nv)
    return n == ctx.cind_count() and h == ctx.checksum()


def test_random_parity_all_modes(ctx):
    rng = random.Random(11)
    for _ in range(150):
        n = rng.randrange(1, 250)
        nv = rng.randrange(2, 40)
        ms = rng.randrange(1, 5)
        arr = np.array([(rng.randrange(nv), rng.randrange(nv // 3 + 1), rng.randrange(nv)) for _ in range(n)],
                       dtype=np.uint32)
        for strategy, clean in MODES:
            assert gpu_set(ctx, arr, nv, ms, strategy, clean) == expected_set(arr, nv, ms, strategy, clean), \
                (n, nv, ms, strategy, clean)
            assert compact_matches(ctx, nv)


def test_projection_subsets(ctx):
    rng = random.Random(5)
    for proj in ("s", "p", "o", "sp", "so", "po"):
        arr = np.array([(rng.randrange(12), rng.randrange(4), rng.randrange(12)) for _ in range(200)], dtype=np.uint32)
        exp, _ = C.run_set(arr[:, 0], arr[:, 1], arr[:, 2], 12, 2, 1, True, proj)
        assert gpu_set(ctx, arr, 12, 2, 1, True, proj) == exp, proj


def test_edge_cases(ctx):
    empty = np.zeros((0, 3), np.uint32)
    assert gpu_set(ctx, empty, 1, 1, 1, True) == set()
    one = np.array([[0, 1, 2]], np.uint32)
    assert gpu_set(ctx, one, 3, 1, 1, True) == expected_set(one, 3, 1, 1, True)
    dup = np.array([[0, 1, 2]] * 50, np.uint32)  # duplicates count for conditions, not for support
    for strategy, clean in MODES:
        assert gpu_set(ctx, dup, 3, 2, strategy, clean) == expected_set(dup, 3, 2, strategy, clean)
    same = np.array([[4, 4, 4], [4, 4, 4], [1, 4, 4], [4, 1, 1]], np.uint32)  # equal values across positions
    for strategy, clean in MODES:
        assert gpu_set(ctx, same, 5, 1, strategy, clean) == expected_set(same, 5, 1, strategy, clean)
    big_ms = np.array([[0, 1, 2], [1, 1, 2]], np.uint32)
    assert gpu_set(ctx, big_ms, 3, 1000, 1, True) == set()
    assert gpu_set(ctx, big_ms, 3, 0, 1, True) == expected_set(big_ms, 3, 1, 1, True)  # support 0 == 1


def test_kat_people(ctx):
    dic = ntriples.Dictionary()
    arr = np.array([[dic.encode(a), dic.encode(b), dic.encode(c)] for a, b, c in KAT_PEOPLE], np.uint32)
    for clean, expected in ((True, KAT_PEOPLE_CLEAN), (False, None)):
        ctx.set_triples(arr[:, 0], arr[:, 1], arr[:, 2], dic.size)
        ctx.run(2, "spo", clean, 0)
        lines = sorted(program.format_rows(ctx.decoded_cinds(), dic.term))
        assert lines == (expected if expected is not None else KAT_PEOPLE_RAW)


@pytest.mark.parametrize("kat", kats.RULE_KATS, ids=lambda k: k["name"])
def test_rule_kats(ctx, tmp_path, kat):
    """The hand-derived R1-R4 / 1/2, 2/1, 2/2 KATs (tests/kats.py) on the GPU in all four modes, with the heavy-group
    paths both off and forced (every group a bit column), and through the driver from N-Triples text."""
    arr, dic = kats.encode(kat)
    ms, proj = kat["support"], kat["projection"]
    want = {(1, True): "clean", (0, True): "clean", (0, False): "s0_raw", (1, False): "s2l_raw"}
    for g in (ctx, None):
        own = g is None
        if own:
            os.environ["RDFIND_HEAVY_MIN"] = "1"
            try:
                g = _lib.Context(0)
            finally:
                del os.environ["RDFIND_HEAVY_MIN"]
        try:
            for (strategy, clean), mode in want.items():
                g.set_triples(arr[:, 0], arr[:, 1], arr[:, 2], dic.size)
                g.run(ms, proj, clean, strategy)
                got = kats.lines_of(_lib.decoded_to_set(g.decoded_cinds()), dic.term)
                assert got == kats.expected(kat, mode), (kat["name"], strategy, clean, own)
        finally:
            if own:
                g.close()
    nt = tmp_path / "kat.nt"
    ntriples.write_ntriples(str(nt), (f"{a} {b} {c} ." for a, b, c in kat["triples"]))
    out = tmp_path / "out.txt"
    program.RDFind(["--use-fis", "--clean-implied", "--support", str(ms), "--projection", proj,
                    "--output", f"file://{out}", str(nt)]).run()
    assert sorted(out.read_text().splitlines()) == kats.expected(kat, "clean")


@pytest.mark.parametrize("name", ["zipf_small", "lubm_small", "skew_small"])
@pytest.mark.parametrize("mode,flags", [("s1_clean", ["--use-fis", "--clean-implied"]),
                                        ("s0_clean", ["--traversal-strategy", "0", "--clean-implied"]),
                                        ("s0_raw", ["--traversal-strategy", "0"])])
def test_program_reproduces_golden(tmp_path, name, mode, flags):
    ms, expected = read_golden(name, mode)
    out = tmp_path / "cinds.txt"
    prog = program.RDFind(flags + ["--support", str(ms), "--output", f"file://{out}",
                                   os.path.join(GOLDEN, f"{name}.nt.gz")])
    prog.run()
    assert sorted(out.read_text().splitlines()) == expected


@pytest.mark.parametrize("cfg,scale", [("c1", 0.3), ("c2", 0.05), ("c3", 0.002), ("c4", 0.0003), ("c5", 0.01)])
def test_synthetic_configs_vs_oracle(ctx, cfg, scale):
    """Scaled BASELINE shapes: every result row equals the materializing C oracle's, and the intermediate stage
    counts agree with the restatement too."""
    d = dataset(cfg, scale)
    ctx.set_triples(d.s, d.p, d.o, d.num_terms)
    ctx.run(d.min_support)
    st = assert_rows_equal(ctx, d, 1, True)
    assert ctx.fc["n_frequent_unary"] == st["n_freq_unary"]
    assert ctx.fc["n_frequent_binary"] == st["n_freq_binary"]
    assert ctx.groups["n_records"] == st["n_records"]
    assert ctx.groups["n_captures"] == st["n_freq_captures"]
    assert_stream_matches(ctx, cfg, scale)


def test_global_count_paths(ctx, monkeypatch):
    """The global-atomic unary counting kernel (fallback of the partitioned K1) agrees with the oracle and
    with the partitioned path (condition statistics and the order-independent result checksum)."""
    monkeypatch.setenv("RDFIND_COUNT_PATHS", "atomic")
    g = _lib.Context(0)
    try:
        rng = random.Random(23)
        for _ in range(30):
            n = rng.randrange(1, 250)
            nv = rng.randrange(2, 40)
            ms = rng.randrange(1, 5)
            arr = np.array([(rng.randrange(nv), rng.randrange(nv // 3 + 1), rng.randrange(nv)) for _ in range(n)],
                           dtype=np.uint32)
            for strategy, clean in ((1, True), (0, False)):
                assert gpu_set(g, arr, nv, ms, strategy, clean) == expected_set(arr, nv, ms, strategy, clean)
        for cfg, scale in (("c1", 0.2), ("c5", 0.01)):
            d = dataset(cfg, scale)
            stats = []
            for c in (g, ctx):
                c.set_triples(d.s, d.p, d.o, d.num_terms)
                c.run(d.min_support)
                stats.append((dict(c.fc), c.checksum()))
            assert stats[0] == stats[1], cfg
    finally:
        g.close()


def test_unary_radix_path_parity(ctx, monkeypatch):
    """K1's radix form (u32 keys grouped by bucket with stable radix passes, bucket starts by binary search, the same
    counting blocks; the default from 3n >= 2^27) forced on every input by RDFIND_U1_RADIX_MIN=1: random inputs in two
    modes equal the oracle, and c1 / c5 / c2 samples give the partition passes' condition statistics and checksum."""
    monkeypatch.setenv("RDFIND_U1_RADIX_MIN", "1")
    g = _lib.Context(0)
    try:
        rng = random.Random(61)
        for _ in range(30):
            n = rng.randrange(1, 400)
            nv = rng.randrange(2, 60)
            ms = rng.randrange(1, 5)
            arr = np.array([(rng.randrange(nv), rng.randrange(nv // 3 + 1), rng.randrange(nv)) for _ in range(n)],
                           dtype=np.uint32)
            for strategy, clean in ((1, True), (0, False)):
                assert gpu_set(g, arr, nv, ms, strategy, clean) == expected_set(arr, nv, ms, strategy, clean)
        for cfg, scale in (("c1", 0.2), ("c5", 0.01), ("c2", 0.05)):
            d = dataset(cfg, scale)
            stats = []
            for c in (g, ctx):
                c.set_triples(d.s, d.p, d.o, d.num_terms)
                c.run(d.min_support)
                stats.append((dict(c.fc), c.cind_count(), c.checksum()))
            assert stats[0] == stats[1], cfg
    finally:
        g.close()


def _capture_joins(d, code, v1, v2):
    """Distinct join values of a capture, straight from the triples (the definition of its groups)."""
    cols = {1: d.s, 2: d.p, 4: d.o}
    prim, proj = code & 7, (code >> 3) & 7
    first = prim & -prim
    second = prim & ~first
    mask = cols[first] == v1
    if second:
        mask &= cols[second] == v2
    return np.unique(cols[proj][mask])


def test_bench_size_properties(ctx):
    """c2 at full size (the bench workload): determinism, rule monotonicity, sampled verification."""
    d = dataset("c2", 1.0)
    ctx.set_triples(d.s, d.p, d.o, d.num_terms)
    ctx.run(d.min_support, "spo", True, 1)
    n_clean = ctx.cind_count()
    sum_clean = ctx.checksum()
    rng = np.random.default_rng(0)
    offsets = rng.choice(n_clean, size=min(40, n_clean), replace=False)
    sample = np.concatenate([ctx.copy_cinds_range(int(off), 1) for off in offsets])
    bkeys = ctx.binary_keys()
    ctx.run(d.min_support, "spo", True, 1)
    assert ctx.cind_count() == n_clean and ctx.checksum() == sum_clean  # deterministic set
    ctx.run(d.min_support, "spo", False, 1)
    n_s2l_raw = ctx.cind_count()
    ctx.run(d.min_support, "spo", False, 0)
    n_v_literal = ctx.cind_count()
    assert 0 < n_clean <= n_s2l_raw and n_v_literal > 0
    # verify sampled CINDs directly: every join value of dep is a join value of ref; support = #joins(dep)
    dec = _lib.decode_rows(sample, d.num_terms, bkeys)
    for r in dec.tolist():
        dc, d1, d2, rc, r1, r2, sup = r
        jd = _capture_joins(d, dc, d1, d2)
        jr = _capture_joins(d, rc, r1, r2)
        assert len(jd) == sup
        assert np.isin(jd, jr).all()


@pytest.mark.parametrize("heavy_min", [1, 2, 8])
def test_heavy_paths_parity(monkeypatch, heavy_min):
    """Small inputs with a lowered heavy-group minimum (RDFIND_HEAVY_MIN test hook), so the bitmask columns,
    the mask classes (unary and binary heavy-only dependents) and the mark passes of R2/R3 carry most of the
    result, in every mode."""
    monkeypatch.setenv("RDFIND_HEAVY_MIN", str(heavy_min))
    g = _lib.Context(0)
    try:
        rng = random.Random(100 + heavy_min)
        for _ in range(30):
            n = rng.randrange(20, 400)
            nv = rng.randrange(4, 40)
            ms = rng.randrange(1, 4)
            arr = np.array([(rng.randrange(nv), rng.randrange(nv // 4 + 1), rng.randrange(nv)) for _ in range(n)],
                           dtype=np.uint32)
            for strategy, clean in MODES:
                g.set_triples(arr[:, 0], arr[:, 1], arr[:, 2], nv)
                g.run(ms, "spo", clean, strategy)
                parts = g.copy_result_compact()  # before any row accessor expands the class part
                assert _lib.decoded_to_set(g.decoded_cinds()) == expected_set(arr, nv, ms, strategy, clean), \
                    (n, nv, ms, strategy, clean, heavy_min)
                assert C.checksum_compact(parts, nv)[:2] == (g.cind_count(), g.checksum())
        for cfg, scale in (("c5", 0.01), ("c1", 0.05)):
            d = dataset(cfg, scale)
            g.set_triples(d.s, d.p, d.o, d.num_terms)
            g.run(d.min_support)
            assert_stream_matches(g, cfg, scale, what=heavy_min)
            assert g.groups["n_heavy_groups"] > 0
    finally:
        g.close()


@pytest.mark.parametrize("budget", [None, "384"])
def test_dense_bitmap_paths_parity(monkeypatch, budget):
    """Every light group verified through its exact member bitmap (RDFIND_DENSE / RDFIND_DENSE_MIN test hooks: the
    dense-group path of the light kernels, serial, batched, packed and second-pivot checks), in every mode, and the
    heavy columns lowered too so that bitmaps and heavy masks mix.  With a bitmap budget of 3 rows (RDFIND_DENSE_BYTES)
    the first groups get bitmaps and the rest keep their member lists, mixed within one dependent."""
    monkeypatch.setenv("RDFIND_DENSE", "1000000")
    monkeypatch.setenv("RDFIND_DENSE_MIN", "1")
    if budget:
        monkeypatch.setenv("RDFIND_DENSE_BYTES", budget)
    for heavy_min in (64, 2):
        monkeypatch.setenv("RDFIND_HEAVY_MIN", str(heavy_min))
        g = _lib.Context(0)
        try:
            rng = random.Random(300 + heavy_min)
            for _ in range(30):
                n = rng.randrange(20, 400)
                nv = rng.randrange(4, 40)
                ms = rng.randrange(1, 4)
                arr = np.array([(rng.randrange(nv), rng.randrange(nv // 4 + 1), rng.randrange(nv)) for _ in range(n)],
                               dtype=np.uint32)
                for strategy, clean in MODES:
                    assert gpu_set(g, arr, nv, ms, strategy, clean) == expected_set(arr, nv, ms, strategy, clean), \
                        (n, nv, ms, strategy, clean, heavy_min)
            for cfg, scale in (("c5", 0.01), ("c1", 0.05), ("c4", 0.0003)):
                d = dataset(cfg, scale)
                g.set_triples(d.s, d.p, d.o, d.num_terms)
                g.run(d.min_support)
                assert_stream_matches(g, cfg, scale, what=heavy_min)
        finally:
            g.close()


def _paged(g, ms, strategy, clean, page_bytes, keep_rows=True):
    """Every page of a paged run: (union of decoded rows, total count, sum of page checksums, pages, compact ok).
    Without keep_rows only the counts and checksums are summed (disjointness then follows from count + checksum
    equal to the oracle's)."""
    g.frequent_conditions(ms)
    g.build_capture_groups("spo")
    rows, n, h, pages, compact_ok = set(), 0, 0, 0, True
    for _ in g.pages(clean, strategy, page_bytes):
        parts = g.copy_result_compact()
        cnt = g.cind_count()
        if keep_rows:
            page_rows = _lib.decoded_to_set(g.decoded_cinds())
            assert not (rows & page_rows)  # pages are disjoint
            rows |= page_rows
        n += cnt
        h = (h + g.checksum()) % (1 << 64)
        compact_ok &= C.checksum_compact(parts, g.num_terms)[:2] == (cnt, g.checksum())
        pages += 1
    return rows, n, h, pages, compact_ok


@pytest.mark.parametrize("heavy_min", [64, 2])
def test_heavy_bits_form_parity(monkeypatch, heavy_min):
    """rdf_set_result_form(RDF_FORM_HEAVY_BITS): the heavy-only binary dependents' CINDs leave as survivor words over the
    class lists (rdf_copy_result_heavy) instead of explicit refs.  The compact parts, expanded by the checker, give the
    device's count and checksum and the oracle's, unpaged (random inputs in the classed mode, c5 / c1 / c2 samples) and
    paged (later pages index the first page's lists); the expanded form's explicit refs are the explicit part plus the
    heavy chunks' refs."""
    monkeypatch.setenv("RDFIND_HEAVY_MIN", str(heavy_min))
    g = _lib.Context(0)
    e = _lib.Context(0)
    try:
        g.set_result_form(True)
        rng = random.Random(900 + heavy_min)
        chunks = 0
        for _ in range(12):
            n = rng.randrange(20, 400)
            nv = rng.randrange(4, 40)
            ms = rng.randrange(1, 4)
            arr = np.array([(rng.randrange(nv), rng.randrange(nv // 4 + 1), rng.randrange(nv)) for _ in range(n)],
                           dtype=np.uint32)
            g.set_triples(arr[:, 0], arr[:, 1], arr[:, 2], nv)
            g.run(ms)
            parts = g.copy_result_compact()
            chunks += parts["n_heavy_chunks"]
            assert C.checksum_compact(parts, nv)[:2] == (g.cind_count(), g.checksum()), (n, nv, ms)
        for cfg, scale in (("c5", 0.01), ("c1", 0.05), ("c2", 0.02)):
            d = dataset(cfg, scale)
            exp = oracle_stream(cfg, scale)
            for c in (g, e):
                c.set_triples(d.s, d.p, d.o, d.num_terms)
                c.run(d.min_support)
            parts, full = g.copy_result_compact(), e.copy_result_compact()
            chunks += parts["n_heavy_chunks"]
            assert C.checksum_compact(parts, d.num_terms)[:2] == (exp["n_cinds"], exp["checksum"]), cfg
            assert C.checksum_compact(full, d.num_terms)[:2] == (exp["n_cinds"], exp["checksum"]), cfg
            if parts["n_heavy_chunks"]:
                assert parts["layout"]["n_refs"] < full["layout"]["n_refs"], cfg
            # the device-side result (the heavy refs expanded on first use) equals the expanded form's
            assert (g.cind_count(), g.checksum()) == (e.cind_count(), e.checksum()) == (exp["n_cinds"], exp["checksum"])
            if cfg != "c2":  # every row (external ids) against the materializing C oracle
                assert_rows_equal(g, d)
        assert chunks > 0  # the form was exercised
        # paged: each page's parts (heavy chunks indexing the first page's class lists)
        d = dataset("c5", 0.01)
        exp = oracle_stream("c5", 0.01)
        g.set_triples(d.s, d.p, d.o, d.num_terms)
        g.frequent_conditions(d.min_support)
        g.build_capture_groups("spo")
        n = h = pages = 0
        lists = None
        for _ in g.pages(True, 1, 1 << 16):
            parts = g.copy_result_compact()
            if lists is None:
                lists = parts["list_refs"].copy()
            parts["heavy_lists"] = lists
            cnt, hh, _ = C.checksum_compact(parts, d.num_terms)
            assert (cnt, hh) == (g.cind_count(), g.checksum())
            n += cnt
            h = (h + hh) % (1 << 64)
            pages += 1
        assert (n, h) == (exp["n_cinds"], exp["checksum"]) and pages > 2
    finally:
        g.close()
        e.close()


@pytest.mark.parametrize("heavy_min", [64, 2])
def test_paged_discovery_matches_unpaged(monkeypatch, heavy_min):
    """rdf_discover_cinds_paged with a one-byte page budget (every binary dependent is its own page) partitions the
    unpaged result, in every mode, with and without bitmask columns and classes."""
    monkeypatch.setenv("RDFIND_HEAVY_MIN", str(heavy_min))
    g = _lib.Context(0)
    try:
        rng = random.Random(500 + heavy_min)
        for _ in range(16):
            n = rng.randrange(20, 400)
            nv = rng.randrange(4, 40)
            ms = rng.randrange(1, 4)
            arr = np.array([(rng.randrange(nv), rng.randrange(nv // 4 + 1), rng.randrange(nv)) for _ in range(n)],
                           dtype=np.uint32)
            for strategy, clean in MODES:
                exp = expected_set(arr, nv, ms, strategy, clean)
                g.set_triples(arr[:, 0], arr[:, 1], arr[:, 2], nv)
                rows, cnt, _, pages, ok = _paged(g, ms, strategy, clean, 1)
                assert rows == exp and cnt == len(exp) and ok, (n, nv, ms, strategy, clean, heavy_min)
        for cfg, scale in (("c5", 0.01), ("c1", 0.05)):
            d = dataset(cfg, scale)
            exp = oracle_stream(cfg, scale)
            g.set_triples(d.s, d.p, d.o, d.num_terms)
            _, cnt, h, pages, ok = _paged(g, d.min_support, 1, True, 1 << 16, keep_rows=False)
            assert (cnt, h) == (exp["n_cinds"], exp["checksum"]) and ok and pages > 2, (cfg, heavy_min, pages)
    finally:
        g.close()


def test_paged_async_refs_survive_the_next_page():
    """rdf_copy_result_refs_async: page k's refs are queued on the copy stream into page-locked memory and the next
    page is computed before anyone waits; after rdf_handover_wait each page's refs equal a synchronous copy of the same
    page (the next page's emission waits for the copy on the GPU before it overwrites `out`).  Small pages of c5 and c1
    samples, the two host buffers alternating, one of them in two chunks."""
    g = _lib.Context(0)
    try:
        for cfg, scale, budget in (("c5", 0.01, 1 << 16), ("c1", 0.05, 1 << 14)):
            d = dataset(cfg, scale)
            g.set_triples(d.s, d.p, d.o, d.num_terms)
            g.frequent_conditions(d.min_support)
            g.build_capture_groups("spo")
            bufs = [None, None]
            pending = []  # (buffer, expected refs) of the page whose copy is in flight
            pages = checked = 0
            for k, _ in enumerate(g.pages(True, 1, budget)):
                n = g.result_layout()["n_refs"]
                exp = np.empty(max(n, 1), np.uint32)
                assert g.copy_result_refs(0, n, exp) == n  # (waits for the previous page's queued copy first)
                for buf, want in pending:  # that copy is complete now: its page's refs arrived intact
                    assert np.array_equal(buf.array[:len(want)], want), (cfg, k)
                    checked += 1
                pending = []
                b = bufs[k % 2]
                if b is None or b.array.size < n:
                    b = bufs[k % 2] = _lib.PinnedBuffer(max(n, 1), np.uint32)
                half = n // 2
                q = g.copy_result_refs_async(0, half, b.ptr)
                q += g.copy_result_refs_async(half, n - half, b.ptr + 4 * half)
                assert q == n
                pending.append((b, exp[:n].copy()))
                pages += 1
            g.handover_wait()
            for buf, want in pending:
                assert np.array_equal(buf.array[:len(want)], want), cfg
                checked += 1
            assert pages > 2 and checked == pages, (cfg, pages, checked)
    finally:
        g.close()


@pytest.mark.parametrize("range_records,keep", [(1, 1), (7, 1), (300, 1), (1, 0), (7, 0), (300, 0)])
def test_join_range_groups_parity(monkeypatch, range_records, keep):
    """Capture groups built in join-value ranges (the path of inputs with >= 2^32/9 triples; RDFIND_GROUP_RANGE forces
    ranges of at most that many K3 records, a single join value's records may exceed it): every mode gives the oracle's
    set, and the stage statistics equal the one-pass build's.  RDFIND_RANGE_KEEP=1 (the default, up to 256 ranges):
    every range is emitted at once into its region of the kept store (k_emit_ranges), and the second pass reads the first
    pass's sorted records; RDFIND_RANGE_KEEP=0: every range is emitted twice, the second emission writing at the first's
    cached block offsets (each block bounded by the next offset)."""
    ref = _lib.Context(0)
    monkeypatch.setenv("RDFIND_GROUP_RANGE", str(range_records))
    monkeypatch.setenv("RDFIND_RANGE_KEEP", str(keep))
    g = _lib.Context(0)
    try:
        rng = random.Random(900 + range_records)
        for _ in range(25):
            n = rng.randrange(1, 400)
            nv = rng.randrange(2, 60)
            ms = rng.randrange(1, 4)
            arr = np.array([(rng.randrange(nv), rng.randrange(nv // 3 + 1), rng.randrange(nv)) for _ in range(n)],
                           dtype=np.uint32)
            for strategy, clean in MODES:
                assert gpu_set(g, arr, nv, ms, strategy, clean) == expected_set(arr, nv, ms, strategy, clean), \
                    (n, nv, ms, strategy, clean, range_records)
                assert compact_matches(g, nv)
            gpu_set(ref, arr, nv, ms, 1, True)
            gpu_set(g, arr, nv, ms, 1, True)
            keys = ("n_records", "n_frequent_records", "n_groups", "n_captures", "n_heavy_groups", "n_sorted_records")
            assert {k: g.groups[k] for k in keys} == {k: ref.groups[k] for k in keys}
            assert (g.cind_count(), g.checksum()) == (ref.cind_count(), ref.checksum())
            if range_records == 1 and n > 50:
                assert g.groups["n_join_ranges"] > 1
            nr = g.groups["n_join_ranges"]
            assert g.groups["n_ranges_kept"] == (nr if keep and nr <= 256 else 0)
        for cfg, scale in (("c1", 0.05), ("c5", 0.01), ("c4", 0.0003)):
            d = dataset(cfg, scale)
            g.set_triples(d.s, d.p, d.o, d.num_terms)
            g.run(d.min_support)
            st = assert_stream_matches(g, cfg, scale, what=range_records)["stats"]
            assert g.groups["n_records"] == st["n_records"] and g.groups["n_captures"] == st["n_freq_captures"]
            nr = g.groups["n_join_ranges"]
            assert nr > 1 and g.groups["n_ranges_kept"] == (nr if keep and nr <= 256 else 0)
    finally:
        g.close()
        ref.close()


def test_binary_keys_right_after_frequent_conditions(ctx):
    """rdf_copy_binary_keys straight after rdf_frequent_conditions (whose key sort may still be queued on the context
    stream) returns the sorted keys, the same as after a whole discovery."""
    for cfg, scale in (("c2", 0.05), ("c1", 0.3)):
        d = dataset(cfg, scale)
        ctx.set_triples(d.s, d.p, d.o, d.num_terms)
        ctx.frequent_conditions(d.min_support)
        early = ctx.binary_keys()
        ctx.run(d.min_support)
        late = ctx.binary_keys()
        assert early.shape[0] > 1000
        np.testing.assert_array_equal(early, late)
        assert (early[1:] > early[:-1]).all()  # sorted, unpacked keys


@pytest.mark.parametrize("env", [{"RDFIND_B2_SPLIT": "2"}, {"RDFIND_B2_RADIX_MIN": "1"}], ids=["split", "radix"])
def test_k2_split_forced_small_inputs(monkeypatch, env):
    """The K2 paths of large inputs forced on small ones (read once per process: a child process): the sub-bucket split
    (k_b2_split, RDFIND_B2_SPLIT=2) and the hash-prefix radix grouping of compact records (k_b2_emit +
    radix_partition_hashed, which inputs of 3n >= 2^27 records take: c3, c4; RDFIND_B2_RADIX_MIN=1) give the oracle's
    sets in every mode and c1/c5 samples' checksums."""
    import json
    import subprocess
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    child = r"""
import json, random, sys
sys.path.insert(0, sys.argv[1])
import numpy as np
from rdfind_amd import _lib
from tests.test_gpu import MODES, expected_set
from tests.parity import dataset, oracle_stream
bad = []
rng = random.Random(61)
with _lib.Context(0) as g:
    for it in range(20):
        n = rng.randrange(20, 400); nv = rng.randrange(4, 40); ms = rng.randrange(1, 4)
        arr = np.array([(rng.randrange(nv), rng.randrange(nv // 4 + 1), rng.randrange(nv)) for _ in range(n)], dtype=np.uint32)
        for strategy, clean in MODES:
            g.set_triples(arr[:, 0], arr[:, 1], arr[:, 2], nv)
            g.run(ms, "spo", clean, strategy)
            if _lib.decoded_to_set(g.decoded_cinds()) != expected_set(arr, nv, ms, strategy, clean):
                bad.append((it, strategy, clean))
    for cfg, scale in (("c1", 0.05), ("c5", 0.01)):
        d = dataset(cfg, scale)
        g.set_triples(d.s, d.p, d.o, d.num_terms)
        g.run(d.min_support)
        e = oracle_stream(cfg, scale)
        if (g.cind_count(), g.checksum()) != (e["n_cinds"], e["checksum"]):
            bad.append(cfg)
print(json.dumps({"bad": bad}))
"""
    r = subprocess.run([sys.executable, "-c", child, root], env=dict(os.environ, **env), capture_output=True,
                       text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-2000:]
    assert json.loads(r.stdout.strip().splitlines()[-1])["bad"] == []


def test_failed_split_launch_is_an_error_not_a_fault():
    """A k_b2_split launch that does not run (RDFIND_TEST_FAIL_LAUNCH=k_b2_split: an invalid block size; the split forced
    by RDFIND_B2_SPLIT=2) makes rdf_frequent_conditions fail with RDF_ERR_HIP before any kernel consumes the sub-bucket
    offsets it would have written -- the round-4 aperture violation was a count kernel reading such offsets (DESIGN.md
    section 10).  A context without the hook then runs normally in the same process.  Own process: both switches are
    read once per process or per context."""
    import json
    import subprocess
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    child = r"""
import json, os, sys
sys.path.insert(0, sys.argv[1])
from rdfind_amd import _lib
from tests.parity import dataset, oracle_stream
d = dataset("c1", 0.05)
out = {}
with _lib.Context(0) as g:
    g.set_triples(d.s, d.p, d.o, d.num_terms)
    try:
        g.frequent_conditions(d.min_support)
        out["failed"] = None
    except _lib.RdfError as e:
        out["failed"], out["msg"] = e.status, str(e)
del os.environ["RDFIND_TEST_FAIL_LAUNCH"]
with _lib.Context(0) as h:
    h.set_triples(d.s, d.p, d.o, d.num_terms)
    h.run(d.min_support)
    out["ok"] = (h.cind_count(), h.checksum()) == (oracle_stream("c1", 0.05)["n_cinds"], oracle_stream("c1", 0.05)["checksum"])
print(json.dumps(out))
"""
    env = dict(os.environ, RDFIND_TEST_FAIL_LAUNCH="k_b2_split", RDFIND_B2_SPLIT="2")
    r = subprocess.run([sys.executable, "-c", child, root], env=env, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-2000:]
    got = json.loads(r.stdout.strip().splitlines()[-1])
    assert got["failed"] == -2 and "hipGetLastError" in got["msg"], got  # RDF_ERR_HIP
    assert got["ok"], got


def test_next_page_needs_a_current_paged_run(ctx):
    """rdf_next_page fails with RDF_ERR_STATE (never runs on stale page state) once new triples, new capture groups or
    an unpaged discovery replaced the paged run."""
    rng = random.Random(4)
    arr = np.array([(rng.randrange(30), rng.randrange(6), rng.randrange(30)) for _ in range(300)], dtype=np.uint32)
    for breaker in ("set_triples", "groups", "unpaged"):
        ctx.set_triples(arr[:, 0], arr[:, 1], arr[:, 2], 30)
        ctx.frequent_conditions(2)
        ctx.build_capture_groups("spo")
        ctx.discover_cinds_paged(True, 1, 1)
        assert ctx.next_page() is not None
        if breaker == "set_triples":
            ctx.set_triples(arr[:, 0], arr[:, 1], arr[:, 2], 30)
        elif breaker == "groups":
            ctx.frequent_conditions(2)
            ctx.build_capture_groups("spo")
        else:
            ctx.discover_cinds(True, 1)
        with pytest.raises(_lib.RdfError):
            ctx.next_page()


def test_large_grids_two_paths(monkeypatch):
    """c5 at scale 0.3 (8.7e9 CINDs): the heavy-only binary dependents take > 2^26 work items (a dispatch holds
    < 2^32 work-items, so the kernels loop over virtual blocks).  The classed path and the pivot-scan path
    (RDFIND_HCLASS=0) compute them independently and must agree on the count and the set checksum."""
    d = dataset("c5", 0.3)
    got = []
    for flag in ("1", "0"):
        monkeypatch.setenv("RDFIND_HCLASS", flag)
        g = _lib.Context(0)
        try:
            g.set_triples(d.s, d.p, d.o, d.num_terms)
            cs = g.run(d.min_support)
            got.append((g.cind_count(), g.checksum()))
            if flag == "0":
                assert cs["n_heavy_chunks"] * 64 > 2 ** 32
        finally:
            g.close()
    assert got[0] == got[1] and got[0][0] > 2 ** 32


def test_device_formatting_matches_host(ctx):
    """rdf_format_cinds (K8) writes exactly the host Cind.toString lines (program.format_rows), in result order,
    for any row range; terms with multi-byte UTF-8, empty and long strings."""
    rng = random.Random(7)
    for it in range(20):
        n = rng.randrange(30, 400)
        nv = rng.randrange(4, 40)
        ms = rng.randrange(1, 4)
        arr = np.array([(rng.randrange(nv), rng.randrange(nv // 3 + 1), rng.randrange(nv)) for _ in range(n)],
                       dtype=np.uint32)
        terms = [rng.choice(["<http://ex.org/e%d>" % i, '"l%d"' % i, "été-%d" % i, "", "x" * rng.randrange(1, 300)])
                 for i in range(nv)]
        strategy, clean = MODES[it % 4]
        ctx.set_triples(arr[:, 0], arr[:, 1], arr[:, 2], nv)
        ctx.run(ms, "spo", clean, strategy)
        ctx.set_dictionary(terms)
        rows = ctx.decoded_cinds()
        expected = program.format_rows(rows, terms.__getitem__)
        text = ctx.format_cinds()
        assert text.decode("utf-8").split("\n")[:-1] == expected if expected else text == b""
        total = len(rows)
        if total > 3:
            a, b = total // 3, 2 * total // 3
            parts = ctx.format_cinds(0, a) + ctx.format_cinds(a, b - a) + ctx.format_cinds(b, total)
            assert parts == text
    d = dataset("c2", 0.05)
    ctx.set_triples(d.s, d.p, d.o, d.num_terms)
    ctx.run(d.min_support)
    terms = ["<http://www.Department%d.University%d.edu/t%d>" % (i % 15, i % 7, i) for i in range(d.num_terms)]
    ctx.set_dictionary(terms)
    n = ctx.cind_count()
    rows = ctx.copy_cinds_range(n // 2, 20000)
    dec = _lib.decode_rows(rows, d.num_terms, ctx.binary_keys())
    assert ctx.format_cinds(n // 2, 20000).decode().split("\n")[:-1] == program.format_rows(dec, terms.__getitem__)


@pytest.mark.parametrize("n,nv", [(0, 1), (1, 3), (1000, 4), (200_000, 40), (300_000, 3000), (100_000, 1)])
def test_distinct_triples_kernel(ctx, n, nv):
    """rdf_distinct_triples (RDFind.scala:284-287) keeps exactly the first occurrence of every triple, in
    input order (bit-exact vs the oracle), and the pipeline on the result equals the oracle on it."""
    rng = np.random.default_rng(n + nv)
    arr = rng.integers(0, nv, size=(n, 3), dtype=np.uint32)
    ctx.set_triples(arr[:, 0], arr[:, 1], arr[:, 2], nv)
    kept, ms = ctx.distinct_triples()
    es, ep, eo = R.distinct_triples(arr[:, 0], arr[:, 1], arr[:, 2])
    assert kept == es.shape[0]
    s, p, o = ctx.copy_triples(n)
    assert s.shape[0] == kept
    np.testing.assert_array_equal(s, es)
    np.testing.assert_array_equal(p, ep)
    np.testing.assert_array_equal(o, eo)
    if n <= 1000:
        ctx.run(2)
        exp, _ = C.run_set(es, ep, eo, nv, 2, 1, True)
        assert _lib.decoded_to_set(ctx.decoded_cinds()) == exp
    kept2, _ = ctx.distinct_triples()  # idempotent
    assert kept2 == kept


def test_program_prefixes_and_distinct_triples(tmp_path):
    """--prefixes + --distinct-triples through the program vs the oracle on per-triple shortened, distinct
    string triples (ShortenUrls.map then triples.distinct, RDFind.scala:243-287)."""
    rng = random.Random(17)
    ents = [f"<http://ex.org/{'a/' if i % 3 else ''}e{i}>" for i in range(40)]
    preds = [f"<http://ex.org/p{j}>" for j in range(5)]
    objs = ents + ['"l1"', '"l2"', "ex:e1"]
    tr = [(rng.choice(ents), rng.choice(preds), rng.choice(objs)) for _ in range(600)]
    tr += tr[:200]  # duplicates: they change condition counts unless removed
    (tmp_path / "in.nt").write_text("".join(f"{a} {b} {c} .\n" for a, b, c in tr))
    (tmp_path / "pre.nt").write_text("@prefix ex: <http://ex.org/> .\n@prefix exa: <http://ex.org/a/> .\n")
    prefixes = [("ex", "http://ex.org/"), ("exa", "http://ex.org/a/")]
    short = [tuple(R.shorten_term(x, prefixes) for x in t) for t in tr]
    for distinct in (False, True):
        out = tmp_path / f"out{distinct}.txt"
        argv = ["--use-fis", "--clean-implied", "--support", "3", "--prefixes", str(tmp_path / "pre.nt"),
                "--output", f"file://{out}", str(tmp_path / "in.nt")] + (["--distinct-triples"] if distinct else [])
        program.RDFind(argv).run()
        expected = R.format_cinds(R.rdfind(short, 3, 1, True, distinct_triples=distinct))
        assert sorted(out.read_text().splitlines()) == expected, distinct


_NT_SAMPLE = (
    "# comment line\n"
    "<http://ex.org/a> <http://ex.org/p> \"plain\" .\n"
    "\n   \t \n"
    "<http://ex.org/a> <http://ex.org/p> \"esc \\\" quote\"@en-US .\n"
    "_:b0 <http://ex.org/q> \"5\"^^<http://www.w3.org/2001/XMLSchema#int> .\r\n"
    "<http://ex.org/b>\t<http://ex.org/p>   \"x\"^^xsd:int .\n"
    "  <http://ex.org/a> <http://ex.org/q> _:b0 .\n"
    "<http://ex.org/b> <http://ex.org/p> <http://ex.org/a> <http://ex.org/graph> .\n"
    "#<http://ex.org/c> <http://ex.org/p> <http://ex.org/a> .\n"
    "<http://ex.org/a> <http://ex.org/p> \"plain\" ."  # no final newline
)


def _long_line_text() -> bytes:
    """Lines of 300-2000 B literals, so most 256-line tokenizer blocks exceed the 48 KB LDS tile and parse from
    global memory (NtGlobal), mixed with short-line blocks (LDS), and one single line > 48 KB."""
    rng = np.random.default_rng(7)
    lines = []
    for i in range(3000):
        if (i // 256) % 3 == 2:
            lines.append(f"<s{i % 97}> <p{i % 5}> <o{i % 211}> .")
        else:
            lit = "".join(chr(97 + c) for c in rng.integers(0, 26, int(rng.integers(300, 2000))))
            lines.append(f"<s{i % 97}> <p{i % 5}> \"{lit}\"@en .")
        if i == 1500:
            lines.append("<big> <p0> \"" + "z" * 60000 + "\" .")
    return ("\n".join(lines) + "\n").encode()


def _host_parse(tmp_path, data: bytes, tabs=False):
    f = tmp_path / "host.nt"
    f.write_bytes(data)
    return ntriples.read_triples([str(f)], tabs=tabs)


def _device_parse(ctx, data: bytes, tabs=False):
    n, v, _ = ctx.parse_ntriples(data, tabs=tabs)
    s, p, o = ctx.copy_triples(n)
    return s, p, o, ntriples.HeapDictionary(*ctx.parsed_terms())


@pytest.mark.parametrize("case", ["sample", "empty", "only_comments", "tabs", "long_lines", "cr_nbsp", "golden_lubm", "golden_zipf",
                                  "synthetic_c1"])
def test_device_parser_matches_host(ctx, tmp_path, case):
    """rdf_parse_ntriples gives the host parser's triples and dictionary bit-exactly (same ids, same terms)."""
    import gzip as _gz
    tabs = case == "tabs"
    if case == "sample":
        data = _NT_SAMPLE.encode()
    elif case == "empty":
        data = b""
    elif case == "only_comments":
        data = b"# a\n\n#b\n"
    elif case == "tabs":
        data = b"<a>\t<p>\t\"x y\"\t.\n# c\n<b>\t<p>\t<a>\n\n<a> x\t<q>\t\"z\"\r\n"
    elif case == "long_lines":
        data = _long_line_text()
    elif case == "cr_nbsp":
        # a lone '\r' ends no line; NBSP / U+3000 are term bytes, not separators (ASCII whitespace only)
        data = ("<a> <p> \"x\ry\" .\n<b>\u00a0<c> <p> <d> .\r\n<e> <p> \"s\u3000t\" .\n"
                "<f> <p>\r<g> <h> .\n<i> <p> <j>").encode()
    elif case.startswith("golden"):
        data = _gz.open(os.path.join(GOLDEN, f"{case.split('_')[1]}_small.nt.gz"), "rb").read()
    else:
        data = "".join(ln + "\n" for ln in synth.config("c1", 0.05).lines()).encode()
    hs, hp, ho, hd = _host_parse(tmp_path, data, tabs)
    ds, dp, do, dd = _device_parse(ctx, data, tabs)
    assert dd.size == hd.size
    assert dd.terms == hd.terms
    np.testing.assert_array_equal(ds, hs)
    np.testing.assert_array_equal(dp, hp)
    np.testing.assert_array_equal(do, ho)


def test_device_parser_rejects_malformed_line(ctx):
    with pytest.raises(_lib.RdfError, match="line 2"):
        ctx.parse_ntriples(b"<a> <p> <b> .\n<a> <p> \"unterminated .\n")
    with pytest.raises(_lib.RdfError, match="line 1"):
        ctx.parse_ntriples(b"<a> <p>\n")


def test_parsed_dictionary_formatting(ctx, tmp_path):
    """rdf_set_dictionary_parsed (the parse's dictionary built into the formatter in HBM) formats the same bytes
    as the host-uploaded dictionary; it is refused once triples were set another way."""
    data = "".join(ln + "\n" for ln in synth.config("c1", 0.05).lines()).encode()
    ctx.parse_ntriples(data)
    ctx.run(5)
    heap, offsets = ctx.parsed_terms()
    ctx.set_dictionary_heap(heap, offsets)
    host = ctx.format_array(0, 1 << 20).tobytes()
    ctx.set_dictionary_parsed()
    dev = ctx.format_array(0, 1 << 20).tobytes()
    assert dev == host and len(dev) > 0
    ctx.set_triples(np.zeros(1, np.uint32), np.zeros(1, np.uint32), np.zeros(1, np.uint32), 1)
    with pytest.raises(_lib.RdfError, match="rdf_parse_ntriples"):
        ctx.set_dictionary_parsed()


@pytest.mark.parametrize("name", ["lubm_small", "skew_small"])
def test_program_host_parser_reproduces_golden(tmp_path, name):
    """--host-parser (host tokenizer + dictionary) gives the same output as the default device ingest."""
    ms, expected = read_golden(name, "s1_clean")
    out = tmp_path / "cinds.txt"
    program.RDFind(["--use-fis", "--clean-implied", "--host-parser", "--support", str(ms), "--output", f"file://{out}",
                    os.path.join(GOLDEN, f"{name}.nt.gz")]).run()
    assert sorted(out.read_text().splitlines()) == expected


def test_copy_result_refs_ranges(ctx):
    """rdf_copy_result_refs (the streaming hand-over of the explicit refs) returns the refs part of the compact result
    chunk by chunk, with a short last chunk and nothing past the end."""
    d = dataset("c1", 0.05)
    ctx.set_triples(d.s, d.p, d.o, d.num_terms)
    ctx.run(d.min_support)
    whole = ctx.copy_result_compact()
    nrefs = ctx.result_layout()["n_refs"]
    assert nrefs > 1000
    for chunk in (1, 97, 1 << 12, nrefs, nrefs + 5):
        buf = np.empty(chunk, np.uint32)
        got, off = [], 0
        while off < nrefs:
            k = ctx.copy_result_refs(off, chunk, buf)
            assert 0 < k <= chunk
            got.append(buf[:k].copy())
            off += k
        np.testing.assert_array_equal(np.concatenate(got), whole["refs"][:nrefs])
        assert ctx.copy_result_refs(nrefs, chunk, buf) == 0


def test_copy_cinds_decoded_matches_host_decode(ctx):
    """rdf_copy_cinds_decoded (Cind-shaped rows decoded on the device) equals the host decode of rdf_copy_cinds,
    for the whole result and for ranges, in every mode."""
    rng = random.Random(29)
    for it in range(12):
        n = rng.randrange(30, 400)
        nv = rng.randrange(4, 40)
        arr = np.array([(rng.randrange(nv), rng.randrange(nv // 3 + 1), rng.randrange(nv)) for _ in range(n)],
                       dtype=np.uint32)
        strategy, clean = MODES[it % 4]
        ctx.set_triples(arr[:, 0], arr[:, 1], arr[:, 2], nv)
        ctx.run(rng.randrange(1, 4), "spo", clean, strategy)
        host = ctx.decoded_cinds()
        dev = ctx.copy_cinds_decoded()
        assert dev.shape[0] == host.shape[0]
        for a, b in (("dep_capture_type", "dep_code"), ("dep_value1", "dep_v1"), ("dep_value2", "dep_v2"),
                     ("ref_capture_type", "ref_code"), ("ref_value1", "ref_v1"), ("ref_value2", "ref_v2"),
                     ("support", "support")):
            np.testing.assert_array_equal(dev[a], host[b].astype(np.uint32))
        if host.shape[0] > 5:
            part = ctx.copy_cinds_decoded(2, 3)
            np.testing.assert_array_equal(part, dev[2:5])
    d = dataset("c2", 0.05)
    ctx.set_triples(d.s, d.p, d.o, d.num_terms)
    ctx.run(d.min_support)
    n = ctx.cind_count()
    dev = ctx.copy_cinds_decoded(n // 3, 1 << 21)
    host = _lib.decode_rows(ctx.copy_cinds_range(n // 3, 1 << 21), d.num_terms, ctx.binary_keys())
    np.testing.assert_array_equal(dev["ref_value1"], host["ref_v1"])
    np.testing.assert_array_equal(dev["dep_capture_type"], host["dep_code"].astype(np.uint32))
    np.testing.assert_array_equal(dev["support"], host["support"])


def test_parse_scratch_released(ctx):
    """After rdf_parse_ntriples only the text and the term table stay resident: the parse scratch (~36 B per term
    occurrence + the slot table) is released before discovery (rdf_device_bytes)."""
    c = _lib.Context(0)
    try:
        data = "".join(ln + "\n" for ln in synth.config("c1", 0.2).lines()).encode()
        before = c.device_bytes()
        n, v, _ = c.parse_ntriples(data)
        held = c.device_bytes() - before
        # text + triples (12 B each) + term table (12 B per term) + small scans; the scratch alone would be
        # 3 * 36 B per line plus a 2^k * 8 B slot table
        assert held < len(data) + 16 * n + 16 * v + (1 << 22), (held, len(data), n, v)
        c.run(10)
        assert c.cind_count() > 0
    finally:
        c.close()


def test_early_handover_matches_plain_copy():
    """rdf_set_handover: the explicit refs and the capture table copied into registered page-locked buffers while the
    discovery still computes, the rest by rdf_copy_result_compact, equal the plain hand-over into fresh arrays (random
    inputs in every mode, a refs buffer too small for some results -- those go the plain way --, and re-runs into the
    same buffers), and the checker expands them to the device's own count and checksum."""
    import ctypes

    from bench import CompactSink

    g = _lib.Context(0)
    try:
        sink = CompactSink(early=True)
        rng = random.Random(31)
        seen_early = 0
        for it in range(30):
            n = rng.randrange(1, 500)
            nv = rng.randrange(2, 60)
            ms = rng.randrange(1, 4)
            arr = np.array([(rng.randrange(nv), rng.randrange(nv // 3 + 1), rng.randrange(nv)) for _ in range(n)],
                           dtype=np.uint32)
            for strategy, clean in MODES:
                g.set_triples(arr[:, 0], arr[:, 1], arr[:, 2], nv)
                g.run(ms, "spo", clean, strategy)
                L = sink.copy(g)
                plain = g.copy_result_compact()
                for name, dt, count in _lib.COMPACT_PARTS:
                    k = count(L)
                    got = np.ctypeslib.as_array(ctypes.cast(sink.bufs[name], ctypes.POINTER(
                        ctypes.c_uint32 if dt == np.uint32 else ctypes.c_uint64)), shape=(max(k, 1),))[:k]
                    assert np.array_equal(got, plain[name][:k]), (it, strategy, clean, name)
                cnt, h, _ = C.checksum_compact(plain, nv)
                assert (cnt, h) == (g.cind_count(), g.checksum()), (it, strategy, clean)
                seen_early += L["n_refs"] <= sink.cap["refs"]
        assert seen_early > 0
    finally:
        g.close()


@pytest.mark.parametrize("dedup,dup_min", [("0", "256"), ("1", "1"), ("1", "256")])
def test_light_dedup_parity(monkeypatch, dedup, dup_min):
    """Light dependents with identical group lists verified once per class (RDFIND_LIGHT_DEDUP=1; members take their
    representative's refs minus themselves and their trivially implied components) or each on its own (0): random
    inputs with many equal join sets in every mode, with the heavy columns lowered too, and c1 / c5 samples, equal the
    oracle.  The strategy-0 quirk and --use-ars keep per-dependent verification (the filters are per dependent).
    RDFIND_DUP_MIN=1 lets every light dependent look for an equal list (the default, 256 groups, leaves the random
    inputs' short lists alone)."""
    monkeypatch.setenv("RDFIND_LIGHT_DEDUP", dedup)
    monkeypatch.setenv("RDFIND_DUP_MIN", dup_min)
    for heavy_min in ("64", "2"):
        monkeypatch.setenv("RDFIND_HEAVY_MIN", heavy_min)
        g = _lib.Context(0)
        try:
            rng = random.Random(600 + int(heavy_min))
            for _ in range(30):
                n = rng.randrange(1, 400)
                nv = rng.randrange(2, 40)
                ms = rng.randrange(1, 4)
                arr = np.array([(rng.randrange(nv), rng.randrange(nv // 4 + 1), rng.randrange(nv)) for _ in range(n)],
                               dtype=np.uint32)
                for strategy, clean in MODES:
                    assert gpu_set(g, arr, nv, ms, strategy, clean) == expected_set(arr, nv, ms, strategy, clean), \
                        (n, nv, ms, strategy, clean, dedup, heavy_min)
            for cfg, scale in (("c1", 0.05), ("c5", 0.01), ("c2", 0.02)):
                d = dataset(cfg, scale)
                g.set_triples(d.s, d.p, d.o, d.num_terms)
                g.run(d.min_support)
                assert_stream_matches(g, cfg, scale, what=(dedup, heavy_min))
        finally:
            g.close()
