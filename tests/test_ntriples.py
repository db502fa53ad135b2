import gzip

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
