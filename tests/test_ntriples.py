import gzip

import numpy as np
import pytest

from rdfind_amd import ntriples


def test_parse_terms():
    assert ntriples.parse_line('<a> <b> <c> .') == ("<a>", "<b>", "<c>")
    assert ntriples.parse_line('_:x <b> "hello world"@en .') == ("_:x", "<b>", '"hello world"@en')
    assert ntriples.parse_line('<a> <b> "1"^^<http://www.w3.org/2001/XMLSchema#int> .') == \
        ("<a>", "<b>", '"1"^^<http://www.w3.org/2001/XMLSchema#int>')
    assert ntriples.parse_line('<a>\t<b>  "q \\" x" .') == ("<a>", "<b>", '"q \\" x"')
    assert ntriples.parse_line("<a>\t<b>\t<c>\n", tabs=True) == ("<a>", "<b>", "<c>")
    with pytest.raises(ntriples.ParseError):
        ntriples.parse_line("<a> <b>")


def test_read_triples_comments_gz_dictionary(tmp_path):
    p = tmp_path / "x.nt.gz"
    with gzip.open(p, "wt") as f:
        f.write("# comment\n<a> <p> <b> .\n\n<b> <p> <a> .\n")
    s, pp, o, d = ntriples.read_triples([str(p)])
    assert d.terms == ["<a>", "<p>", "<b>"]
    assert s.tolist() == [0, 2] and pp.tolist() == [1, 1] and o.tolist() == [2, 0]


def test_resolve_patterns(tmp_path):
    for n in ("a1.nt", "a2.nt", "b.nt"):
        (tmp_path / n).write_text("<a> <p> <b> .\n")
    got = ntriples.resolve_paths([f"{tmp_path}/a*.nt"])
    assert [x.rsplit("/", 1)[1] for x in got] == ["a1.nt", "a2.nt"]


# --prefixes (ALG/operators/ParseRdfPrefixes.scala, ShortenUrls.scala, util/StringTrie.scala) against the
# oracle's linear-scan restatement
from oracle import rdfind_oracle as R  # noqa: E402


@pytest.mark.parametrize("line", [
    "@prefix foaf: <http://xmlns.com/foaf/0.1/> .", "@prefix  ex:\t<http://ex.org/>.", "@prefix <http://base/> .",
    "@prefix dc: <http://purl.org/dc/elements/1.1/> .\n", "@prefix x: <a>   .",
    "@prefix : <http://empty/> .", "prefix ex: <http://ex.org/> .", "@prefix ex: http://ex.org/ .",
    "@prefix ex: <http://ex.org/>", " @prefix ex: <http://ex.org/> .", "@prefix ex: <http://ex.org/> . #",
])
def test_prefix_line_parsing_matches_oracle(line):
    try:
        exp = R.parse_prefix_line(line)
    except ValueError:
        with pytest.raises(ValueError):
            ntriples.parse_prefix_line(line)
        return
    assert ntriples.parse_prefix_line(line) == exp


def test_shortening_matches_oracle():
    import random
    rng = random.Random(3)
    alphabet = "ab/#:.x"
    for _ in range(300):
        urls = {"http://" + "".join(rng.choice(alphabet) for _ in range(rng.randrange(0, 6)))
                for _ in range(rng.randrange(0, 6))}
        prefixes = [(f"p{i}", u) for i, u in enumerate(sorted(urls))]
        table = ntriples.PrefixTable(prefixes)
        for _ in range(40):
            body = "http://" + "".join(rng.choice(alphabet) for _ in range(rng.randrange(0, 9)))
            term = rng.choice([f"<{body}>", f'"{body}"', f'"v"^^<{body}>', body, f"<{body}"])
            assert table.shorten(term) == R.shorten_term(term, prefixes), (term, prefixes)


def test_shorten_dictionary_equals_per_triple_shortening(tmp_path):
    pref = tmp_path / "prefixes.nt"
    pref.write_text("# comment\n@prefix ex: <http://ex.org/> .\n@prefix exa: <http://ex.org/a/> .\n"
                    "@prefix <http://base.org/> .\n")
    tr = [("<http://ex.org/a/x>", "<http://ex.org/p>", '"lit"'), ("<http://ex.org/b>", "<http://base.org/q>", "<other>"),
          ("<http://ex.org/a/x>", "<http://ex.org/p>", "<http://ex.org/a/x>"), ("ex:b", "<http://base.org/q>", "<other>")]
    d = ntriples.Dictionary()
    arr = np.array([[d.encode(x) for x in t] for t in tr], np.uint32)
    prefixes = ntriples.read_prefixes([str(pref)])
    assert prefixes == [("ex", "http://ex.org/"), ("exa", "http://ex.org/a/"), ("", "http://base.org/")]
    s, p, o, short = ntriples.shorten_dictionary(arr[:, 0], arr[:, 1], arr[:, 2], d, prefixes)
    got = [(short.term(a), short.term(b), short.term(c)) for a, b, c in zip(s, p, o)]
    exp = [tuple(R.shorten_term(x, prefixes) for x in t) for t in tr]
    assert got == exp == [("exa:x", "ex:p", '"lit"'), ("ex:b", ":q", "<other>"), ("exa:x", "ex:p", "exa:x"),
                          ("ex:b", ":q", "<other>")]
    assert short.size == len({x for t in exp for x in t})  # "<http://ex.org/b>" and "ex:b" share one id


def test_duplicate_prefix_key_rejected():
    with pytest.raises(ValueError, match="Key already exists"):
        ntriples.PrefixTable([("a", "http://x/"), ("b", "http://x/")])


def test_prefixes_and_distinct_flags_accepted():
    from rdfind_amd import program
    prog = program.RDFind(["--use-fis", "--prefixes", "a.nt,b.nt", "--prefixes", "c.nt", "--distinct-triples", "x.nt"])
    assert prog.args.prefixes == ["a.nt,b.nt", "c.nt"] and prog.args.distinct_triples


def test_read_byte_range_partitions_lines(tmp_path):
    """The sharded ingest's byte ranges (read_byte_range): the ranks' parts are whole lines and concatenate to the
    input stream (plain files seeked, .gz files decompressed, a line break after a file without one)."""
    import gzip

    a, b, c = tmp_path / "a.nt", tmp_path / "b.nt.gz", tmp_path / "c.nt"
    a.write_bytes(b"".join(b"<s%d> <p> <o%d> .\n" % (i, i) for i in range(100)))
    with gzip.open(b, "wb") as f:
        f.write(b"".join(b'<x%d> <p> "l%d" .\n' % (i, i) for i in range(57)) + b"<last> <p> <o> .")
    c.write_bytes(b"<c1> <p> <o> .\n<c2> <p> <o> .")
    paths = [str(a), str(b), str(c)]
    full = ntriples.read_bytes(paths)
    for nranks in (1, 2, 3, 5, 8, 64):
        parts = [ntriples.read_byte_range(paths, r, nranks) for r in range(nranks)]
        assert b"".join(parts) == full, nranks
        assert all(not p or p.endswith(b"\n") for p in parts)


def test_read_byte_range_small_chunks(tmp_path, monkeypatch):
    """The one-pass range reader across chunk boundaries (chunks of 7 bytes), empty files, long lines and files
    without a final line break: the ranks' parts still partition the stream's lines."""
    import gzip
    import random

    monkeypatch.setattr(ntriples, "_GZ_STEP", 7)
    rng = random.Random(3)
    paths = []
    for k in range(6):
        lines = [b"<s%d> <p> \"%s\" ." % (i, b"x" * rng.randrange(0, 90)) for i in range(rng.randrange(0, 40))]
        data = b"\n".join(lines) + (b"\n" if lines and rng.random() < 0.5 else b"")
        path = tmp_path / (f"f{k}.nt.gz" if k % 2 else f"f{k}.nt")
        if k % 2:
            with gzip.open(path, "wb") as f:
                f.write(data)
        else:
            path.write_bytes(data)
        paths.append(str(path))
    full = ntriples.read_bytes(paths)
    for nranks in (1, 2, 3, 7, 13, 50, 400):
        parts = [ntriples.read_byte_range(paths, r, nranks) for r in range(nranks)]
        assert b"".join(parts) == full, nranks
        assert all(not p or p.endswith(b"\n") for p in parts)
