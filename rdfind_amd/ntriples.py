"""N-Triples ingest: tokenizer + term dictionary (host side of the boundary).

Reference behaviour (ALG/programs/RDFind.scala:196-237): input files are read line by line
(``MultiFileTextInputFormat``, ``.gz`` decompressed), lines *starting with* ``#`` are dropped
(:211-213), and each remaining line is split into three raw terms by rdf-converter's
``NTriplesParser`` (or ``NQuadsParser`` for ``.nq`` inputs, ``--tabs`` for tab separation).  Terms keep
their N-Triples spelling: IRIs with angle brackets, literals with quotes and any language tag or
datatype.  rdf-converter 0.0.2-SNAPSHOT is not available offline, so its handling of exotic escapes
and blank lines is *parity unpinned*; this tokenizer accepts the standard N-Triples term forms and
skips blank lines.

The dictionary assigns one id space to subjects, predicates and objects because join values cross
positions.
"""
from __future__ import annotations

import gzip
import io
import os
import re
from dataclasses import dataclass, field

import numpy as np


class ParseError(ValueError):
    pass


# Term separators: ASCII whitespace only, the device tokenizer's nt_space (kernels.inl).  Python's
# str.isspace would also accept NBSP and the Unicode spaces, which the reference's byte-level line
# records never split on.
_SPACE_CHARS = " \t\n\v\f\r\x1c\x1d\x1e\x1f"
_SPACE = frozenset(_SPACE_CHARS)


def _is_space(ch: str) -> bool:
    return ch in _SPACE


def _strip_terminator(line: str) -> str:
    """Lines end at '\n' only; one '\r' before it belongs to the terminator ("\r\n")."""
    if line.endswith("\n"):
        line = line[:-1]
        if line.endswith("\r"):
            line = line[:-1]
    return line


def _term_end(line: str, i: int, n: int) -> int:
    c = line[i]
    if c == "<":
        j = line.find(">", i + 1)
        if j < 0:
            raise ParseError(f"unterminated IRI: {line!r}")
        return j + 1
    if c == '"':
        j = i + 1
        while j < n:
            ch = line[j]
            if ch == "\\":
                j += 2
                continue
            if ch == '"':
                break
            j += 1
        if j >= n:
            raise ParseError(f"unterminated literal: {line!r}")
        j += 1
        if j < n and line[j] == "@":
            while j < n and not _is_space(line[j]):
                j += 1
        elif j + 1 < n and line[j] == "^" and line[j + 1] == "^":
            j += 2
            if j < n and line[j] == "<":
                j = line.find(">", j) + 1
                if j <= 0:
                    raise ParseError(f"unterminated datatype IRI: {line!r}")
            else:
                while j < n and not _is_space(line[j]):
                    j += 1
        return j
    # blank node or bare token
    j = i
    while j < n and not _is_space(line[j]):
        j += 1
    return j


def parse_line(line: str, tabs: bool = False, quads: bool = False):
    """Split one N-Triples (N-Quads) line into its subject, predicate and object terms."""
    if tabs:
        parts = _strip_terminator(line).split("\t")
        if len(parts) < 3:
            raise ParseError(f"expected 3 tab-separated terms: {line!r}")
        return parts[0], parts[1], parts[2]
    n = len(line)
    terms = []
    i = 0
    need = 4 if quads else 3
    while len(terms) < 3:
        while i < n and _is_space(line[i]):
            i += 1
        if i >= n:
            raise ParseError(f"expected {need} terms: {line!r}")
        j = _term_end(line, i, n)
        terms.append(line[i:j])
        i = j
    return terms[0], terms[1], terms[2]


@dataclass
class Dictionary:
    """term string <-> uint32 id; ids are assigned in order of first appearance."""

    ids: dict = field(default_factory=dict)
    terms: list = field(default_factory=list)

    def encode(self, term: str) -> int:
        tid = self.ids.get(term)
        if tid is None:
            tid = len(self.terms)
            self.ids[term] = tid
            self.terms.append(term)
        return tid

    def term(self, tid: int) -> str:
        return self.terms[tid]

    @property
    def size(self) -> int:
        return len(self.terms)


def _open(path: str):
    if path.startswith("file:"):
        path = path[5:]
        while path.startswith("//"):
            path = path[1:]
    if path.endswith(".gz"):
        return io.TextIOWrapper(gzip.open(path, "rb"), encoding="utf-8", newline="\n")
    return open(path, "r", encoding="utf-8", newline="\n")  # no universal newlines: a lone '\r' ends no line


def resolve_paths(paths):
    """Expand a '*' in the last path segment (RDFind.resolvePathPattern, RDFind.scala:154-191)."""
    import fnmatch

    out = []
    for raw in paths:
        if "*" in raw:
            last = raw.rfind("/")
            if raw.find("*") < last:
                raise ValueError(f"Path expansion is only possible on the last path segment: {raw}")
            parent = raw[:last] if last >= 0 else "."
            pattern = raw[last + 1:]
            local = parent[5:] if parent.startswith("file:") else parent
            for name in sorted(os.listdir(local)):
                if fnmatch.fnmatchcase(name, pattern):
                    out.append(f"{parent}/{name}")
        else:
            out.append(raw)
    return out


def read_triples(paths, tabs: bool = False, dictionary: Dictionary | None = None):
    """Read N-Triples/N-Quads files into (s, p, o) uint32 arrays + the dictionary."""
    d = dictionary if dictionary is not None else Dictionary()
    quads = bool(paths) and paths[0].endswith("nq")
    s, p, o = [], [], []
    enc = d.encode
    for path in paths:
        with _open(path) as f:
            for line in f:
                if line.startswith("#"):
                    continue
                line = _strip_terminator(line)
                if not line.strip(_SPACE_CHARS):
                    continue
                a, b, c = parse_line(line, tabs, quads)
                s.append(enc(a))
                p.append(enc(b))
                o.append(enc(c))
    return (np.array(s, dtype=np.uint32), np.array(p, dtype=np.uint32), np.array(o, dtype=np.uint32), d)


def write_ntriples(path: str, lines):
    opener = gzip.open if path.endswith(".gz") else open
    with opener(path, "wt", encoding="utf-8") as f:
        for ln in lines:
            f.write(ln)
            f.write("\n")


# ------------------------------------------------------------------------------------------------
# --prefixes: URL shortening (ALG/programs/RDFind.scala:243-267, ALG/operators/ShortenUrls.scala:16-61)

_PREFIX_RE = re.compile(r"@prefix\s+(\S+): <(\S+)>\s*\.\n?")
_BASE_RE = re.compile(r"@prefix\s+<(\S+)>\s*\.\n?")

def parse_prefix_line(line: str):
    """ParseRdfPrefixes.map (ALG/operators/ParseRdfPrefixes.scala:14-26): ``@prefix p: <url> .`` gives
    (p, url), ``@prefix <url> .`` gives ("", url); any other line is an error."""
    m = _PREFIX_RE.fullmatch(line)
    if m:
        return m.group(1), m.group(2)
    m = _BASE_RE.fullmatch(line)
    if m:
        return "", m.group(1)
    raise ValueError(f"Could not parse the line {line!r} correctly.")


def read_prefixes(paths):
    """Prefix files -> [(prefix, url)]; lines starting with '#' are comments (RDFind.scala:256-258)."""
    out = []
    for path in resolve_paths(paths):
        with _open(path) as f:
            for line in f.read().splitlines():
                if line.startswith("#"):
                    continue
                out.append(parse_prefix_line(line))
    return out


class PrefixTable:
    """The prefix trie of ShortenUrls.PrefixTrieCreator (ALG/operators/ShortenUrls.scala:55-60):
    key ``<url`` -> value ``prefix:``, longest matching key wins (StringTrie.getKeyAndValue,
    ALG/util/StringTrie.scala:44-54).  Held as one hash set per key length, probed longest first."""

    def __init__(self, prefixes):
        self.by_len = {}
        for prefix, url in prefixes:
            key = "<" + url
            tab = self.by_len.setdefault(len(key), {})
            if key in tab:  # StringTrie.+= (StringTrie.scala:36-38)
                raise ValueError(f"Key already exists: {key}.")
            tab[key] = prefix + ":"
        self.lengths = sorted(self.by_len, reverse=True)

    def shorten(self, term: str) -> str:
        """ShortenUrls.shorten (ShortenUrls.scala:36-44)."""
        if not term.endswith(">"):
            return term
        for n in self.lengths:
            if n <= len(term):
                v = self.by_len[n].get(term[:n])
                if v is not None:
                    if n > len(term) - 1:  # String.substring(n, len-1) with n > len-1 throws in the JVM
                        raise ValueError(f"prefix key {term[:n]!r} covers the whole term {term!r}")
                    return v + term[n:len(term) - 1]
        return term


def shorten_dictionary(s, p, o, dictionary: Dictionary, prefixes):
    """Applies the URL shortening to every distinct term once (not to every triple, as the reference's
    per-triple map does) and re-encodes: terms that shorten to the same string share one id afterwards,
    exactly as they would have after a per-triple map followed by dictionary encoding."""
    table = PrefixTable(prefixes)
    short = Dictionary()
    remap = np.fromiter((short.encode(table.shorten(t)) for t in dictionary.terms), dtype=np.uint32,
                        count=dictionary.size)
    return remap[s], remap[p], remap[o], short


# ------------------------------------------------------------------------------------------------
# Device ingest (rdf_parse_ntriples): the host side only reads (and gunzips) the bytes

def read_bytes(paths) -> bytes:
    """The input files' bytes, concatenated with a line break between files (MultiFileTextInputFormat reads
    every file's lines, FLK/persistence/MultiFileTextInputFormat.java:199-206)."""
    parts = []
    for path in paths:
        if path.startswith("file:"):
            path = path[5:]
            while path.startswith("//"):
                path = path[1:]
        opener = gzip.open if path.endswith(".gz") else open
        with opener(path, "rb") as f:
            data = f.read()
        parts.append(data)
        if data and not data.endswith(b"\n"):
            parts.append(b"\n")
    return b"".join(parts)


def _plain_path(path):
    if path.startswith("file:"):
        path = path[5:]
        while path.startswith("//"):
            path = path[1:]
    return path


_GZ_STEP = 1 << 22


def _gz_size(path):
    """(decompressed size, last byte) of a .gz file, streamed."""
    n, last = 0, b""
    with gzip.open(path, "rb") as f:
        while chunk := f.read(_GZ_STEP):
            n += len(chunk)
            last = chunk[-1:]
    return n, last


def _stream_from(files, start):
    """(absolute offset, chunk) pairs of the concatenated input stream from byte `start` on: plain files are seeked,
    a .gz file is decompressed once from its beginning (the bytes before `start` discarded as they come), and a file
    without a final line break is followed by one."""
    base = 0
    for path, sz, gz in files:
        if base + sz <= start:
            base += sz
            continue
        skip = max(start - base, 0)
        got = 0  # bytes of this file's stream part produced so far (from its byte `skip` on)
        if gz:
            pos = 0
            with gzip.open(path, "rb") as f:
                while chunk := f.read(_GZ_STEP):
                    lo = max(skip - pos, 0)
                    if lo < len(chunk):
                        yield base + pos + lo, chunk[lo:]
                        got += len(chunk) - lo
                    pos += len(chunk)
        else:
            with open(path, "rb") as f:
                f.seek(skip)
                while chunk := f.read(_GZ_STEP):
                    yield base + skip + got, chunk
                    got += len(chunk)
        if skip + got < sz:  # the virtual line break after a file without one
            yield base + skip + got, b"\n"
        base += sz


def read_byte_range(paths, rank: int, nranks: int) -> bytes:
    """This rank's part of the input for the sharded ingest: the bytes of the whole lines that start in
    [T * rank / nranks, T * (rank + 1) / nranks) of the concatenated input of T bytes (read_bytes' stream: a line
    break after a file without one).  A line belongs to the rank its first byte falls to, so the parts partition the
    lines (the reference's input splits, FLK/persistence/MultiFileTextInputFormat.java:49-100).  One forward pass from
    the byte before the range finds its first line start, collects the range and stops at the first line start at or
    after its end: plain files are seeked, a .gz file (which cannot be split) is decompressed once for its size and once
    up to the end of the range, and only the range is kept: no rank holds a whole compressed input."""
    files = []  # (path, size of its stream part, gz)
    for path in paths:
        path = _plain_path(path)
        if path.endswith(".gz"):
            size, last = _gz_size(path)
            files.append((path, size + (0 if last in (b"", b"\n") else 1), True))
        else:
            size = os.path.getsize(path)
            with open(path, "rb") as f:
                if size:
                    f.seek(size - 1)
                    last = f.read(1)
                else:
                    last = b"\n"
            files.append((path, size + (0 if last == b"\n" else 1), False))
    total = sum(sz for _, sz, _ in files)
    lo, hi = total * rank // nranks, total * (rank + 1) // nranks
    if lo >= total:
        return b""
    # a line starts at 0 or right after a "\n": the range's first line start is the first one >= lo, found from the
    # byte before lo on; its end is the first line start >= hi (the total when hi reaches it)
    b0 = 0 if lo == 0 else None
    b1 = total if hi >= total else None
    out = []
    for pos, chunk in _stream_from(files, max(lo - 1, 0)):
        if b0 is None:
            k = chunk.find(b"\n", max(lo - 1 - pos, 0))
            if k < 0:
                continue
            b0 = pos + k + 1
        if b1 is None:
            k = chunk.find(b"\n", max(hi - 1 - pos, 0))
            if k >= 0:
                b1 = pos + k + 1
        end = len(chunk) if b1 is None else min(len(chunk), b1 - pos)
        begin = max(b0 - pos, 0)
        if begin < end:
            out.append(chunk[begin:end])
        if b1 is not None and pos + len(chunk) >= b1:
            break
    if b0 is None or b1 is None or b0 >= b1:
        return b""
    return b"".join(out)


class HeapDictionary:
    """Term id -> string over a (heap, offsets) pair, e.g. the device dictionary of rdf_parse_ntriples."""

    def __init__(self, heap: bytes, offsets):
        self.heap = heap
        self.offsets = offsets
        self._terms = None

    @property
    def size(self) -> int:
        return len(self.offsets) - 1

    def term(self, tid: int) -> str:
        return self.heap[int(self.offsets[tid]):int(self.offsets[tid + 1])].decode("utf-8")

    @property
    def terms(self):
        if self._terms is None:
            self._terms = [self.term(i) for i in range(self.size)]
        return self._terms
