"""ORACLE -- test infrastructure only (ctypes binding of oracle/c/rdfind_oracle.c).

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg may use this.
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "build", "liborc.so")
_lib = None

UNARY_CODES = (10, 12, 17, 20, 33, 34)
BINARY_CODES = (14, 21, 35)


class OrcCind(ctypes.Structure):
    _fields_ = [("dep", ctypes.c_uint32), ("ref", ctypes.c_uint32), ("support", ctypes.c_uint32)]


class OrcStats(ctypes.Structure):
    _fields_ = [("n_freq_unary", ctypes.c_uint64 * 3), ("n_binary_keys", ctypes.c_uint64),
                ("n_freq_binary", ctypes.c_uint64), ("n_records", ctypes.c_uint64),
                ("n_unique", ctypes.c_uint64), ("n_groups", ctypes.c_uint64),
                ("n_freq_captures", ctypes.c_uint64), ("n_raw_cinds", ctypes.c_uint64),
                ("n_cinds", ctypes.c_uint64), ("n_join_ranges", ctypes.c_uint64)]


class OrcStream(ctypes.Structure):
    _fields_ = [("n_cinds", ctypes.c_uint64), ("checksum", ctypes.c_uint64), ("n_kind", ctypes.c_uint64 * 4),
                ("n_raw", ctypes.c_uint64)]


# minimality rules of the streamed mode (oracle/c/rdfind_oracle.c ORC_R*)
R1, R2, R3, R4 = 1, 2, 4, 8


def rules_for(strategy, clean):
    """--clean-implied: R1-R4; strategy-1 raw: the exact-candidate S2L output (R1 and R4); strategy-0 raw: V."""
    if clean:
        return R1 | R2 | R3 | R4
    return R1 | R4 if strategy == 1 else 0


def build():
    subprocess.check_call(["make", "-s", "-C", _HERE])


def _load():
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB_PATH):
            build()
        lib = ctypes.CDLL(_LIB_PATH)
        lib.orc_run.restype = ctypes.c_int
        lib.orc_run.argtypes = [ctypes.c_void_p] * 3 + [ctypes.c_uint64, ctypes.c_uint32, ctypes.c_uint32,
                                                         ctypes.c_int, ctypes.c_int, ctypes.c_char_p,
                                                         ctypes.POINTER(ctypes.POINTER(OrcCind)),
                                                         ctypes.POINTER(ctypes.c_uint64),
                                                         ctypes.POINTER(ctypes.POINTER(ctypes.c_uint64)),
                                                         ctypes.POINTER(ctypes.c_uint64),
                                                         ctypes.POINTER(OrcStats)]
        lib.orc_free.argtypes = [ctypes.c_void_p]
        lib.orc_stream.restype = ctypes.c_int
        lib.orc_stream.argtypes = [ctypes.c_void_p] * 3 + [ctypes.c_uint64, ctypes.c_uint32, ctypes.c_uint32,
                                                            ctypes.c_int, ctypes.c_int, ctypes.c_char_p,
                                                            ctypes.POINTER(OrcStream), ctypes.POINTER(OrcStats)]
        lib.orc_set_range_records.argtypes = [ctypes.c_uint64]
        lib.orc_checksum.restype = ctypes.c_uint64
        lib.orc_checksum.argtypes = [ctypes.c_void_p, ctypes.c_uint64]
        _lib = lib
    return _lib


def decode_capture(cap, num_terms, bin_keys):
    """capture id -> (code, v1, v2|None)"""
    V = num_terms
    if cap < 6 * V:
        return UNARY_CODES[cap // V], cap % V, None
    key = int(bin_keys[cap - 6 * V])
    return BINARY_CODES[key >> 62], (key >> 31) & 0x7FFFFFFF, key & 0x7FFFFFFF


def threads():
    """OpenMP threads the restatement runs on (OMP_NUM_THREADS, else all cores)."""
    lib = _load()
    lib.orc_threads.restype = ctypes.c_int
    return int(lib.orc_threads())


def run(s, p, o, num_terms, min_support, strategy=1, clean=True, projection="spo"):
    """Returns (set of (dt, dv1, dv2, rt, rv1, rv2, support), stats dict, raw arrays)."""
    lib = _load()
    s = np.ascontiguousarray(s, dtype=np.uint32)
    p = np.ascontiguousarray(p, dtype=np.uint32)
    o = np.ascontiguousarray(o, dtype=np.uint32)
    out = ctypes.POINTER(OrcCind)()
    n_out = ctypes.c_uint64()
    bk = ctypes.POINTER(ctypes.c_uint64)()
    nbk = ctypes.c_uint64()
    st = OrcStats()
    rc = lib.orc_run(s.ctypes.data, p.ctypes.data, o.ctypes.data, len(s), num_terms, min_support,
                     strategy, int(clean), projection.encode(), ctypes.byref(out), ctypes.byref(n_out),
                     ctypes.byref(bk), ctypes.byref(nbk), ctypes.byref(st))
    if rc != 0:
        raise RuntimeError(f"orc_run failed with {rc}")
    n = n_out.value
    arr = np.ctypeslib.as_array(out, shape=(n,)).copy() if n else np.zeros(0, dtype=[("dep", "<u4"), ("ref", "<u4"), ("support", "<u4")])
    keys = np.ctypeslib.as_array(bk, shape=(nbk.value,)).copy() if nbk.value else np.zeros(0, np.uint64)
    lib.orc_free(out)
    lib.orc_free(bk)
    stats = {f: (list(getattr(st, f)) if f == "n_freq_unary" else getattr(st, f)) for f, _ in OrcStats._fields_}
    return arr, keys, stats


def set_range_records(n):
    """Stages 3-4 (capture records and groups) in join-value ranges of at most n records each (0: one pass): the
    memory of inputs whose records do not fit at once (c4 at 10^9 triples emits ~5.8·10^9)."""
    _load().orc_set_range_records(int(n))


def stream(s, p, o, num_terms, min_support, strategy=1, clean=True, projection="spo"):
    """Count + order-independent checksum of the result without materializing it (the library's
    rdf_cind_checksum mix).  Returns dict(n_cinds, checksum, n_kind=[11, 12, 21, 22], n_raw, stats)."""
    lib = _load()
    s = np.ascontiguousarray(s, dtype=np.uint32)
    p = np.ascontiguousarray(p, dtype=np.uint32)
    o = np.ascontiguousarray(o, dtype=np.uint32)
    res = OrcStream()
    st = OrcStats()
    rc = lib.orc_stream(s.ctypes.data, p.ctypes.data, o.ctypes.data, len(s), num_terms, min_support, strategy,
                        rules_for(strategy, clean), projection.encode(), ctypes.byref(res), ctypes.byref(st))
    if rc != 0:
        raise RuntimeError(f"orc_stream failed with {rc}")
    stats = {f: (list(getattr(st, f)) if f == "n_freq_unary" else getattr(st, f)) for f, _ in OrcStats._fields_}
    return {"n_cinds": res.n_cinds, "checksum": res.checksum, "n_kind": list(res.n_kind), "n_raw": res.n_raw,
            "stats": stats}


def checksum_rows(arr):
    """The streamed checksum of a materialized result (structured dep/ref/support array)."""
    lib = _load()
    a = np.ascontiguousarray(arr)
    return int(lib.orc_checksum(a.ctypes.data, a.shape[0])) if a.shape[0] else 0


def checksum_compact(parts, num_terms):
    """(count, checksum, n_kind) of a compact result (rdfind_amd._lib Context.copy_result_compact parts, sized by
    ``parts["layout"]``): the expansion a consumer of the compact hand-over would do, counted by the checker."""
    lib = _load()
    lib.orc_checksum_compact.restype = ctypes.c_uint64
    lib.orc_checksum_compact.argtypes = ([ctypes.c_void_p] * 3 + [ctypes.c_uint64] + [ctypes.c_void_p] * 3 +
                                         [ctypes.c_uint64] + [ctypes.c_void_p] * 2 + [ctypes.c_uint32] +
                                         [ctypes.POINTER(ctypes.c_uint64), ctypes.c_void_p])
    L = parts["layout"]
    arr = {k: np.ascontiguousarray(parts[k]) for k in ("refs", "runoff", "rundep", "list_refs", "list_off", "members",
                                                        "capture_ids", "supports")}
    cnt = ctypes.c_uint64()
    kind = np.zeros(4, np.uint64)
    h = lib.orc_checksum_compact(arr["refs"].ctypes.data, arr["runoff"].ctypes.data, arr["rundep"].ctypes.data,
                                 L["n_runs"], arr["list_refs"].ctypes.data, arr["list_off"].ctypes.data,
                                 arr["members"].ctypes.data, L["n_members"], arr["capture_ids"].ctypes.data,
                                 arr["supports"].ctypes.data, num_terms, ctypes.byref(cnt), kind.ctypes.data)
    nh = int(parts.get("n_heavy_chunks", 0) or 0)
    if nh:  # the heavy-bits form (rdf_copy_result_heavy): chunks of class-list candidates as survivor words
        lib.orc_checksum_heavy.restype = ctypes.c_uint64
        lib.orc_checksum_heavy.argtypes = ([ctypes.c_void_p] * 3 + [ctypes.c_uint64] + [ctypes.c_void_p] * 3 +
                                           [ctypes.c_uint32, ctypes.POINTER(ctypes.c_uint64), ctypes.c_void_p])
        lists = np.ascontiguousarray(parts.get("heavy_lists", parts["list_refs"]))  # (a later page: the first page's)
        hv = {k: np.ascontiguousarray(parts[k]) for k in ("heavy_deps", "heavy_pos", "heavy_bits")}
        hc = ctypes.c_uint64()
        hk = np.zeros(4, np.uint64)
        h2 = lib.orc_checksum_heavy(hv["heavy_deps"].ctypes.data, hv["heavy_pos"].ctypes.data,
                                    hv["heavy_bits"].ctypes.data, nh, lists.ctypes.data, arr["capture_ids"].ctypes.data,
                                    arr["supports"].ctypes.data, num_terms, ctypes.byref(hc), hk.ctypes.data)
        h = (int(h) + int(h2)) % (1 << 64)
        cnt.value += hc.value
        kind += hk
    return int(cnt.value), int(h), [int(x) for x in kind]


def run_set(s, p, o, num_terms, min_support, strategy=1, clean=True, projection="spo"):
    arr, keys, stats = run(s, p, o, num_terms, min_support, strategy, clean, projection)
    out = set()
    for dep, ref, sup in zip(arr["dep"].tolist(), arr["ref"].tolist(), arr["support"].tolist()):
        dt, dv1, dv2 = decode_capture(dep, num_terms, keys)
        rt, rv1, rv2 = decode_capture(ref, num_terms, keys)
        out.add((dt, dv1, dv2, rt, rv1, rv2, sup))
    return out, stats
