"""The drop-in driver (python -m rdfind_amd / program.RDFind) on results larger than what one discovery holds: paged
discovery written page by page, and the automatic switch to pages when the unpaged run exceeds the device memory
(the reference streams its result to the sink at any size, ALG/programs/RDFind.scala:507-520)."""
import io
import json
import os

import numpy as np
import pytest

from rdfind_amd import program, synth
from tests.conftest import GOLDEN

pytestmark = pytest.mark.gpu

GOLD = json.load(open(os.path.join(GOLDEN, "full_size.json")))


def write_text(d, path):
    """The dataset as N-Triples text (the device parser assigns its own ids; the CIND lines are the same)."""
    tt = d.terms.term
    strs = np.array([tt(i) + " " for i in range(d.num_terms)], dtype=object)
    with open(path, "w", encoding="utf-8") as f:
        step = 1 << 21
        for b in range(0, d.n, step):
            e = min(b + step, d.n)
            f.write("".join(map("".join, zip(strs[d.s[b:e]], strs[d.p[b:e]], strs[d.o[b:e]], [".\n"] * (e - b)))))


def run_program(args):
    out = io.StringIO()
    prog = program.RDFind(args)
    prog.run(out=out)
    return prog, out.getvalue()


@pytest.mark.timeout(600)
def test_program_small_pages_match_unpaged(tmp_path):
    """c1 at full size through the driver with a 1 MiB page budget (one page per binary dependent range) writes the
    same lines as the unpaged run, and as many as the golden vector's CINDs."""
    g = GOLD["c1@1.0/s1_clean"]
    d = synth.config("c1", 1.0)
    nt = tmp_path / "c1.nt"
    write_text(d, nt)
    common = ["--use-fis", "--clean-implied", "--support", str(d.min_support)]
    a, b = tmp_path / "paged.txt", tmp_path / "unpaged.txt"
    prog, _ = run_program(common + ["--page-bytes", str(1 << 20), "--output", f"file://{a}", str(nt)])
    assert prog.stats["pages"] > 2
    run_program(common + ["--output", f"file://{b}", str(nt)])
    la, lb = a.read_text().splitlines(), b.read_text().splitlines()
    assert len(la) == len(lb) == g["n_cinds"]
    assert sorted(la) == sorted(lb)


@pytest.mark.timeout(900)
def test_program_result_beyond_hbm_switches_to_pages(tmp_path):
    """c5 at its BASELINE size (10^7 triples, support 2: 1.75·10^11 CINDs, far more than HBM holds) through the driver
    without any page option: the unpaged discovery runs out of device memory, the driver continues page by page and
    reports the golden vector's count."""
    g = GOLD["c5@1.0/s1_clean"]
    d = synth.config("c5", 1.0)
    nt = tmp_path / "c5.nt"
    write_text(d, nt)
    del d
    prog, out = run_program(["--use-fis", "--clean-implied", "--support", "2", "--debug-level", "1", str(nt)])
    assert prog.stats["pages"] >= 2
    assert f"Detected {g['n_cinds']} CINDs." in out


@pytest.mark.timeout(900)
def test_program_pages_written_lines_vs_oracle(tmp_path):
    """c5 (support 2, the pair-explosion shape) at 3·10^4 triples: 2.7·10^6 CINDs written through the driver in pages
    of a 4 MiB budget are exactly the C oracle's rows formatted as Cind.toString lines.  (At the BASELINE sizes the
    written text would be 0.5 TB (c5 at 0.3) or more; those runs are checked by count and checksum instead:
    test_program_result_beyond_hbm_switches_to_pages and tests/test_gpu.py::test_paged_full_size_vs_oracle.)"""
    from oracle import c_oracle
    from tests.kats import lines_of

    d = synth.config("c5", 0.003)
    nt = tmp_path / "c5.nt"
    write_text(d, nt)
    out = tmp_path / "cinds.txt"
    prog, _ = run_program(["--use-fis", "--clean-implied", "--support", str(d.min_support), "--page-bytes",
                           str(4 << 20), "--output", f"file://{out}", str(nt)])
    assert prog.stats["pages"] >= 4
    got = out.read_text(encoding="utf-8").splitlines()
    rows, _ = c_oracle.run_set(d.s, d.p, d.o, d.num_terms, d.min_support, 1, True)
    want = lines_of(rows, d.terms.term)
    assert len(got) == len(want) == 2698238
    assert sorted(got) == want


@pytest.mark.timeout(300)
def test_program_oom_fallback_writes_output(tmp_path, monkeypatch):
    """The driver's RDF_ERR_OOM fallback with --output: the unpaged discovery fails (RDFIND_TEST_OOM_DISCOVERY, read when
    the context is created), the driver continues in pages and writes the same lines as a run without the hook.  Only
    the discovery is inside the fallback's try: the output is written once (no truncated-then-rewritten file)."""
    d = synth.config("c1", 0.05)
    nt = tmp_path / "c1.nt"
    write_text(d, nt)
    common = ["--use-fis", "--clean-implied", "--support", str(d.min_support)]
    a, b = tmp_path / "fallback.txt", tmp_path / "plain.txt"
    run_program(common + ["--output", f"file://{b}", str(nt)])
    monkeypatch.setenv("RDFIND_TEST_OOM_DISCOVERY", "1")
    prog, out = run_program(common + ["--debug-level", "1", "--output", f"file://{a}", str(nt)])
    assert prog.stats["pages"] >= 1
    la, lb = a.read_text().splitlines(), b.read_text().splitlines()
    assert len(la) == len(lb) > 1000
    assert sorted(la) == sorted(lb)
