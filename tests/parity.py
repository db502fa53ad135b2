"""Shared checkers for the GPU parity tests (test infrastructure: imports the oracle).

* ``dataset(cfg, scale)``: one synthetic BASELINE-shaped input per (config, scale) per pytest session, kept in a
  size-bounded cache (the 10^9-triple c4 input is 12 GB and is drawn once, not once per test);
* ``oracle_stream(...)``: the streamed C oracle's (count, checksum, per-kind counts) per (config, scale, mode), cached
  for the session, so the hook-variant tests (heavy columns, dense bitmaps, pages, join ranges) that re-run one
  config compare against one oracle run;
* ``assert_rows_equal(ctx, d, ...)``: exact row-by-row parity of the current result with the materializing oracle, as
  sorted packed (dep, ref) keys + supports (vectorized; a Python set of 10^7 tuples took ~40 s per check);
* ``dataset_npz(cfg, scale)``: the same input saved once as .npy files, for child processes that must start fresh
  (switches read once per process) without regenerating it.
"""
from __future__ import annotations

import os
import tempfile
from collections import OrderedDict

import numpy as np

from oracle import c_oracle as C
from rdfind_amd import synth

_CACHE_BYTES = int(os.environ.get("RDFIND_TEST_CACHE_BYTES", str(40 << 30)))
_DATA: "OrderedDict[tuple, synth.Dataset]" = OrderedDict()
_STREAM: dict = {}
_NPZ: dict = {}
_NPZ_DIR = None


def _nbytes(d) -> int:
    return d.s.nbytes + d.p.nbytes + d.o.nbytes


def dataset(cfg: str, scale: float):
    """The seeded synthetic input (synth.config), shared by every test of the session; least recently used inputs are
    dropped once the cache exceeds RDFIND_TEST_CACHE_BYTES (default 40 GiB of host memory)."""
    key = (cfg, float(scale))
    if key in _DATA:
        _DATA.move_to_end(key)
        return _DATA[key]
    d = synth.config(cfg, scale)
    need = _nbytes(d)
    while _DATA and sum(_nbytes(x) for x in _DATA.values()) + need > _CACHE_BYTES:
        _DATA.popitem(last=False)
    _DATA[key] = d
    return d


def oracle_stream(cfg: str, scale: float, strategy: int = 1, clean: bool = True, projection: str = "spo") -> dict:
    """Streamed C oracle on the dataset: dict(n_cinds, checksum, n_kind, n_raw, stats); cached per session."""
    key = (cfg, float(scale), strategy, bool(clean), projection)
    if key not in _STREAM:
        d = dataset(cfg, scale)
        _STREAM[key] = C.stream(d.s, d.p, d.o, d.num_terms, d.min_support, strategy, clean, projection)
    return _STREAM[key]


def assert_stream_matches(ctx, cfg: str, scale: float, strategy: int = 1, clean: bool = True, what=None):
    """The context's current result has the oracle's count and order-independent checksum (rdf_cind_checksum =
    orc_stream's mix over (dep, ref, support) rows)."""
    exp = oracle_stream(cfg, scale, strategy, clean)
    got = (ctx.cind_count(), ctx.checksum())
    assert got == (exp["n_cinds"], exp["checksum"]), (cfg, scale, strategy, clean, what, got, exp["n_cinds"])
    return exp


def packed(rows):
    """(sorted dep<<32|ref keys, supports in that order) of a dep/ref/support row array."""
    key = (rows["dep"].astype(np.uint64) << np.uint64(32)) | rows["ref"].astype(np.uint64)
    order = np.argsort(key, kind="stable")
    return key[order], np.asarray(rows["support"])[order]


def assert_rows_equal(ctx, d, strategy: int = 1, clean: bool = True, projection: str = "spo"):
    """Every row of the context's current result equals the materializing C oracle's (external capture ids: binary
    ids index the sorted frequent binary keys on both sides).  Returns the oracle's stage statistics."""
    rows, _, st = C.run(d.s, d.p, d.o, d.num_terms, d.min_support, strategy, clean, projection)
    got = ctx.copy_cinds()
    assert got.shape[0] == rows.shape[0], (got.shape[0], rows.shape[0])
    ek, es = packed(rows)
    gk, gs = packed(got)
    np.testing.assert_array_equal(gk, ek)
    np.testing.assert_array_equal(gs, es)
    return st


def dataset_npz(cfg: str, scale: float) -> str:
    """Directory holding s.npy, p.npy, o.npy and meta.npy (num_terms, min_support) of the dataset, written once per
    session under the system temp dir (removed at interpreter exit)."""
    global _NPZ_DIR
    key = (cfg, float(scale))
    if key in _NPZ:
        return _NPZ[key]
    if _NPZ_DIR is None:
        _NPZ_DIR = tempfile.TemporaryDirectory(prefix="rdfind_tests_")
    path = os.path.join(_NPZ_DIR.name, f"{cfg}_{scale}")
    os.makedirs(path, exist_ok=True)
    d = dataset(cfg, scale)
    for name in ("s", "p", "o"):
        np.save(os.path.join(path, name + ".npy"), getattr(d, name))
    np.save(os.path.join(path, "meta.npy"), np.array([d.num_terms, d.min_support], np.uint64))
    _NPZ[key] = path
    return path


def load_npz(path: str):
    """(s, p, o, num_terms, min_support) of a dataset_npz directory, memory-mapped."""
    s, p, o = (np.load(os.path.join(path, n + ".npy"), mmap_mode="r") for n in ("s", "p", "o"))
    nv, ms = (int(x) for x in np.load(os.path.join(path, "meta.npy")))
    return s, p, o, nv, ms
