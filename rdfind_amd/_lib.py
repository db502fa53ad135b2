"""ctypes binding of the C ABI in ``include/rdfind_hip.h`` (``rdfind_amd/librdfind_hip.so``).

This is the product path: there is no CPU fallback.  If the HIP library is missing or no GPU is
visible, :func:`load` / :class:`Context` raise immediately.
"""
from __future__ import annotations

import ctypes
import os

import numpy as np

from . import codes

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("RDFIND_HIP_LIB") or os.path.join(_HERE, "librdfind_hip.so")  # env: dev variants only

RDF_CLEAN_IMPLIED = 1
RDF_STRATEGY_ALL_AT_ONCE = 2
RDF_SHARD_LOCAL_SLICE = 4
RDF_USE_ASSOCIATION_RULES = 8

# every symbol declared in include/rdfind_hip.h
EXPORTED_SYMBOLS = (
    "rdf_ctx_create", "rdf_ctx_destroy", "rdf_last_error", "rdf_version", "rdf_set_triples",
    "rdf_set_triples_device", "rdf_frequent_conditions", "rdf_build_capture_groups", "rdf_discover_cinds",
    "rdf_run", "rdf_cind_count", "rdf_copy_cinds", "rdf_decode_capture", "rdf_binary_key_count",
    "rdf_copy_binary_keys", "rdf_stage_times", "rdf_kernel_times", "rdf_sync",
    "rdf_copy_cinds_range", "rdf_cind_checksum", "rdf_last_stats", "rdf_shard_begin", "rdf_shard_step",
    "rdf_shard_export", "rdf_shard_import", "rdf_set_dictionary", "rdf_format_size", "rdf_format_cinds",
    "rdf_distinct_triples", "rdf_copy_triples", "rdf_parse_ntriples", "rdf_copy_terms",
    "rdf_set_dictionary_parsed", "rdf_device_bytes", "rdf_copy_cinds_decoded", "rdf_result_sizes",
    "rdf_copy_result_raw", "rdf_association_rules", "rdf_copy_association_rules", "rdf_get_result_layout",
    "rdf_copy_result_compact", "rdf_association_rule_count", "rdf_host_alloc", "rdf_host_free",
    "rdf_discover_cinds_paged", "rdf_next_page", "rdf_shard_parse_begin", "rdf_shard_dictionary_begin", "rdf_num_terms",
    "rdf_dictionary_terms", "rdf_copy_result_refs", "rdf_release_scratch", "rdf_set_handover",
    "rdf_copy_result_refs_async", "rdf_handover_wait", "rdf_set_result_form", "rdf_heavy_chunk_count",
    "rdf_copy_result_heavy",
)
RDF_NT_TABS = 1

# rdf_exchange ops (sharded mode, include/rdfind_hip.h)
X_DONE, X_ALLREDUCE_SUM_U32, X_ALLREDUCE_SUM_U64, X_ALLREDUCE_MIN_U64, X_ALLGATHERV_U64, X_ALLTOALLV_U64 = range(6)
MAX_RANKS = 64

# RDF_T_* kernel-family timers (include/rdfind_hip.h)
TIMER_NAMES = ("unary", "binary", "emit", "sort", "support", "groups", "heavymask", "pivot", "light", "esort",
               "hcount", "rules", "hwrite", "class", "cemit")


class FcStats(ctypes.Structure):
    _fields_ = [("min_support", ctypes.c_uint32), ("n_ar_suppressed", ctypes.c_uint32),
                ("n_frequent_unary", ctypes.c_uint64 * 3), ("n_binary_keys", ctypes.c_uint64),
                ("n_frequent_binary", ctypes.c_uint64)]


class GroupStats(ctypes.Structure):
    _fields_ = [("n_records", ctypes.c_uint64), ("n_frequent_records", ctypes.c_uint64),
                ("n_groups", ctypes.c_uint64), ("n_captures", ctypes.c_uint64),
                ("n_unary_captures", ctypes.c_uint64), ("n_heavy_groups", ctypes.c_uint64),
                ("heavy_threshold", ctypes.c_uint64), ("n_sorted_records", ctypes.c_uint64),
                ("n_join_ranges", ctypes.c_uint64), ("n_ranges_kept", ctypes.c_uint64)]


class CindStats(ctypes.Structure):
    _fields_ = [("n_cinds", ctypes.c_uint64), ("n_explicit_raw", ctypes.c_uint64),
                ("n_light_chunks", ctypes.c_uint64), ("n_heavy_chunks", ctypes.c_uint64),
                ("ms_pivot", ctypes.c_float), ("ms_light", ctypes.c_float), ("ms_rules", ctypes.c_float),
                ("ms_heavy", ctypes.c_float), ("n_heavy_candidates", ctypes.c_uint64),
                ("n_class_members", ctypes.c_uint64), ("n_classes", ctypes.c_uint64), ("n_class_cinds", ctypes.c_uint64),
                ("n_light_candidates", ctypes.c_uint64), ("n_light_entries", ctypes.c_uint64)]


class ResultLayout(ctypes.Structure):
    _fields_ = [(k, ctypes.c_uint64) for k in ("n_cinds", "n_refs", "n_runs", "n_lists", "n_list_refs", "n_members",
                                                "n_captures")]


# rdf_copy_result_compact parts: name -> (dtype, element count from the layout)
COMPACT_PARTS = (("refs", np.uint32, lambda L: L["n_refs"]), ("runoff", np.uint64, lambda L: L["n_runs"] + 1),
                 ("rundep", np.uint32, lambda L: L["n_runs"]), ("list_refs", np.uint32, lambda L: L["n_list_refs"]),
                 ("list_off", np.uint64, lambda L: L["n_lists"] + 1), ("members", np.uint64, lambda L: L["n_members"]),
                 ("capture_ids", np.uint32, lambda L: L["n_captures"]), ("supports", np.uint32, lambda L: L["n_captures"]))


class Exchange(ctypes.Structure):
    _fields_ = [("op", ctypes.c_int32), ("elem_bytes", ctypes.c_uint32), ("count", ctypes.c_uint64),
                ("send_counts", ctypes.c_uint64 * MAX_RANKS)]


class ExchangeRequest:
    """A collective the sharded library asks its caller to perform (see rdfind_amd/distributed.py)."""

    def __init__(self, op: int, elem_bytes: int, count: int, send_counts=None):
        self.op, self.elem_bytes, self.count = op, elem_bytes, count
        self.send_counts = list(send_counts or [])

    def __repr__(self):
        return f"ExchangeRequest(op={self.op}, count={self.count}, send_counts={self.send_counts})"


# rdf_assoc_rule (include/rdfind_hip.h): condition codes s = 1, p = 2, o = 4, term ids, support
RULE_DTYPE = np.dtype([("antecedent_type", "<u4"), ("consequent_type", "<u4"), ("antecedent", "<u4"),
                       ("consequent", "<u4"), ("support", "<u4")])
CIND_DTYPE = np.dtype([("dep", "<u4"), ("ref", "<u4"), ("support", "<u4")])
# rdf_cind_row (include/rdfind_hip.h): the reference's Cind shape with term ids
ROW_DTYPE = np.dtype([("dep_capture_type", "<u4"), ("dep_value1", "<u4"), ("dep_value2", "<u4"),
                      ("ref_capture_type", "<u4"), ("ref_value1", "<u4"), ("ref_value2", "<u4"), ("support", "<u4")])

_lib = None


RDF_ERR_OOM = -3  # device memory exhausted (include/rdfind_hip.h)


class RdfError(RuntimeError):
    """A failed library call; ``status`` is its rdf_status (e.g. RDF_ERR_OOM), None for load failures."""

    def __init__(self, msg, status=None):
        super().__init__(msg)
        self.status = status


def load():
    """Load librdfind_hip.so (raises if it is missing: the product has no fallback)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise RdfError(f"{LIB_PATH} not built; run __graft_entry__.build() (HIP extension missing)")
    lib = ctypes.CDLL(LIB_PATH)
    P, u32, u64, i32 = ctypes.c_void_p, ctypes.c_uint32, ctypes.c_uint64, ctypes.c_int32
    sig = {
        "rdf_ctx_create": (i32, [ctypes.c_int, ctypes.POINTER(P)]),
        "rdf_ctx_destroy": (None, [P]),
        "rdf_last_error": (ctypes.c_char_p, [P]),
        "rdf_version": (ctypes.c_char_p, []),
        "rdf_set_triples": (i32, [P, P, P, P, u64, u32]),
        "rdf_set_triples_device": (i32, [P, P, P, P, u64, u32]),
        "rdf_distinct_triples": (i32, [P, ctypes.POINTER(u64), ctypes.POINTER(ctypes.c_float)]),
        "rdf_copy_triples": (i32, [P, P, P, P, u64, ctypes.POINTER(u64)]),
        "rdf_parse_ntriples": (i32, [P, ctypes.c_char_p, u64, u32, ctypes.POINTER(u64), ctypes.POINTER(u32),
                                     ctypes.POINTER(ctypes.c_float)]),
        "rdf_copy_terms": (i32, [P, P, P, u64, ctypes.POINTER(u64)]),
        "rdf_set_dictionary_parsed": (i32, [P]),
        "rdf_frequent_conditions": (i32, [P, u32, ctypes.POINTER(FcStats)]),
        "rdf_build_capture_groups": (i32, [P, ctypes.c_char_p, ctypes.POINTER(GroupStats)]),
        "rdf_discover_cinds": (i32, [P, u32, ctypes.POINTER(CindStats)]),
        "rdf_run": (i32, [P, u32, ctypes.c_char_p, u32, ctypes.POINTER(FcStats), ctypes.POINTER(GroupStats),
                          ctypes.POINTER(CindStats)]),
        "rdf_cind_count": (i32, [P, ctypes.POINTER(u64)]),
        "rdf_copy_cinds": (i32, [P, P, u64, ctypes.POINTER(u64)]),
        "rdf_decode_capture": (i32, [P, u32, ctypes.POINTER(u32), ctypes.POINTER(u32), ctypes.POINTER(u32)]),
        "rdf_binary_key_count": (i32, [P, ctypes.POINTER(u64)]),
        "rdf_copy_binary_keys": (i32, [P, P, u64]),
        "rdf_stage_times": (i32, [P, ctypes.POINTER(ctypes.c_float)]),
        "rdf_kernel_times": (i32, [P, ctypes.POINTER(ctypes.c_float), ctypes.c_int]),
        "rdf_sync": (i32, [P]),
        "rdf_device_bytes": (i32, [P, ctypes.POINTER(u64)]),
        "rdf_release_scratch": (i32, [P]),
        "rdf_copy_cinds_range": (i32, [P, u64, P, u64, ctypes.POINTER(u64)]),
        "rdf_cind_checksum": (i32, [P, ctypes.POINTER(u64)]),
        "rdf_copy_cinds_decoded": (i32, [P, u64, P, u64, ctypes.POINTER(u64)]),
        "rdf_result_sizes": (i32, [P, ctypes.POINTER(u64), ctypes.POINTER(u64), ctypes.POINTER(u64)]),
        "rdf_copy_result_raw": (i32, [P, P, P, P, P, P]),
        "rdf_get_result_layout": (i32, [P, ctypes.POINTER(ResultLayout)]),
        "rdf_copy_result_compact": (i32, [P, P, P, P, P, P, P, P, P]),
        "rdf_copy_result_refs": (i32, [P, u64, u64, P, ctypes.POINTER(u64)]),
        "rdf_copy_result_refs_async": (i32, [P, u64, u64, P, ctypes.POINTER(u64)]),
        "rdf_handover_wait": (i32, [P]),
        "rdf_set_result_form": (i32, [P, u32]),
        "rdf_heavy_chunk_count": (i32, [P, ctypes.POINTER(u64)]),
        "rdf_copy_result_heavy": (i32, [P, P, P, P]),
        "rdf_set_handover": (i32, [P, P, u64, P, P, u64, P, P, u64]),
        "rdf_set_dictionary": (i32, [P, P, u64, P, u64]),
        "rdf_format_size": (i32, [P, u64, u64, ctypes.POINTER(u64)]),
        "rdf_format_cinds": (i32, [P, u64, u64, P, u64, ctypes.POINTER(u64)]),
        "rdf_last_stats": (i32, [P, ctypes.POINTER(FcStats), ctypes.POINTER(GroupStats), ctypes.POINTER(CindStats)]),
        "rdf_association_rules": (i32, [P, ctypes.POINTER(u64)]),
        "rdf_copy_association_rules": (i32, [P, P, u64, ctypes.POINTER(u64)]),
        "rdf_association_rule_count": (i32, [P, ctypes.POINTER(u64)]),
        "rdf_host_alloc": (P, [u64]),
        "rdf_shard_parse_begin": (i32, [P, u32, u32, ctypes.c_char_p, u64, u32, ctypes.POINTER(u64)]),
        "rdf_shard_dictionary_begin": (i32, [P]),
        "rdf_num_terms": (i32, [P, ctypes.POINTER(u32)]),
        "rdf_dictionary_terms": (i32, [P, P, u64, P, u64, P]),
        "rdf_discover_cinds_paged": (i32, [P, u32, u64, ctypes.POINTER(CindStats)]),
        "rdf_next_page": (i32, [P, ctypes.POINTER(u32), ctypes.POINTER(u64), ctypes.POINTER(u64)]),
        "rdf_host_free": (None, [P]),
        "rdf_shard_begin": (i32, [P, u32, u32, u32, ctypes.c_char_p, u32]),
        "rdf_shard_step": (i32, [P, ctypes.POINTER(Exchange)]),
        "rdf_shard_export": (i32, [P, P]),
        "rdf_shard_import": (i32, [P, P, u64]),
    }
    for name, (res, args) in sig.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    _lib = lib
    return lib


class PinnedBuffer:
    """Page-locked host memory from the library (rdf_host_alloc), as a numpy array view; freed with the object."""

    def __init__(self, count: int, dtype):
        self.lib = load()
        self.nbytes = max(int(count), 1) * np.dtype(dtype).itemsize
        self.ptr = self.lib.rdf_host_alloc(self.nbytes)
        if not self.ptr:
            raise RdfError(f"rdf_host_alloc({self.nbytes}) failed")
        self.array = np.ctypeslib.as_array((ctypes.c_uint8 * self.nbytes).from_address(self.ptr)).view(dtype)

    def __del__(self):
        if getattr(self, "ptr", None):
            self.lib.rdf_host_free(self.ptr)
            self.ptr = None


def _struct_dict(st):
    out = {}
    for name, _ in st._fields_:
        val = getattr(st, name)
        out[name] = list(val) if isinstance(val, ctypes.Array) else val
    return out


class Context:
    """One GPU context (one per device / rank), mirroring one Flink task instance."""

    def __init__(self, device: int = 0):
        self.lib = load()
        self.ptr = ctypes.c_void_p()
        rc = self.lib.rdf_ctx_create(device, ctypes.byref(self.ptr))
        if rc != 0:
            raise RdfError(f"rdf_ctx_create(device={device}) failed ({rc}): is a GPU visible?")
        self.num_terms = 0
        self.fc = self.groups = self.cinds = None

    def close(self):
        if self.ptr:
            self.lib.rdf_ctx_destroy(self.ptr)
            self.ptr = ctypes.c_void_p()

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def _check(self, rc, what):
        if rc != 0:
            msg = self.lib.rdf_last_error(self.ptr)
            raise RdfError(f"{what} failed ({rc}): {msg.decode() if msg else ''}", rc)

    # -- stages ------------------------------------------------------------------------------
    def set_triples(self, s, p, o, num_terms: int):
        s = np.ascontiguousarray(s, dtype=np.uint32)
        p = np.ascontiguousarray(p, dtype=np.uint32)
        o = np.ascontiguousarray(o, dtype=np.uint32)
        if not (s.shape == p.shape == o.shape):
            raise ValueError("s, p, o must have the same length")
        self._check(self.lib.rdf_set_triples(self.ptr, s.ctypes.data, p.ctypes.data, o.ctypes.data, s.shape[0],
                                             num_terms), "rdf_set_triples")
        self.num_terms = num_terms

    def set_triples_device(self, s_ptr: int, p_ptr: int, o_ptr: int, n: int, num_terms: int):
        self._check(self.lib.rdf_set_triples_device(self.ptr, s_ptr, p_ptr, o_ptr, n, num_terms),
                    "rdf_set_triples_device")
        self.num_terms = num_terms

    def distinct_triples(self):
        """--distinct-triples on the resident triples (RDFind.scala:284-287); returns (kept, device ms)."""
        n = ctypes.c_uint64()
        ms = ctypes.c_float()
        self._check(self.lib.rdf_distinct_triples(self.ptr, ctypes.byref(n), ctypes.byref(ms)),
                    "rdf_distinct_triples")
        return int(n.value), float(ms.value)

    def parse_ntriples(self, data: bytes, tabs: bool = False):
        """N-Triples text -> resident dictionary-encoded triples, on the device (rdf_parse_ntriples).
        Returns (n_triples, num_terms, device ms) and keeps ``data`` for :meth:`parsed_terms`."""
        n, v, ms = ctypes.c_uint64(), ctypes.c_uint32(), ctypes.c_float()
        self._check(self.lib.rdf_parse_ntriples(self.ptr, data, len(data), RDF_NT_TABS if tabs else 0,
                                                ctypes.byref(n), ctypes.byref(v), ctypes.byref(ms)),
                    "rdf_parse_ntriples")
        self.num_terms = int(v.value)
        self._parsed = data
        return int(n.value), int(v.value), float(ms.value)

    def parsed_terms(self):
        """The device dictionary of the last parse as (heap bytes, uint64 offsets[V + 1]): term i is
        heap[offsets[i]:offsets[i + 1]] (UTF-8)."""
        v = self.num_terms
        off, ln = np.empty(v, np.uint64), np.empty(v, np.uint32)
        got = ctypes.c_uint64()
        self._check(self.lib.rdf_copy_terms(self.ptr, off.ctypes.data, ln.ctypes.data, v, ctypes.byref(got)),
                    "rdf_copy_terms")
        ln64 = ln.astype(np.int64)
        offsets = np.zeros(v + 1, np.uint64)
        np.cumsum(ln64, out=offsets[1:])
        src = np.frombuffer(self._parsed, np.uint8)
        pos = np.arange(int(offsets[-1]), dtype=np.int64) + np.repeat(off.astype(np.int64) - offsets[:-1].astype(np.int64),
                                                                       ln64)
        return src[pos].tobytes(), offsets

    def set_dictionary_parsed(self):
        """The last parse's dictionary becomes the formatting dictionary, in HBM (rdf_set_dictionary_parsed)."""
        self._check(self.lib.rdf_set_dictionary_parsed(self.ptr), "rdf_set_dictionary_parsed")

    def set_dictionary_heap(self, heap: bytes, offsets):
        """rdf_set_dictionary from a ready heap + offsets (e.g. :meth:`parsed_terms`)."""
        offsets = np.ascontiguousarray(offsets, dtype=np.uint64)
        buf = ctypes.create_string_buffer(heap, max(len(heap), 1))
        self._check(self.lib.rdf_set_dictionary(self.ptr, buf, len(heap), offsets.ctypes.data, offsets.shape[0] - 1),
                    "rdf_set_dictionary")

    def copy_triples(self, n: int):
        """The resident triples as three uint32 arrays (the first n of them)."""
        s, p, o = (np.empty(n, np.uint32) for _ in range(3))
        got = ctypes.c_uint64()
        self._check(self.lib.rdf_copy_triples(self.ptr, s.ctypes.data, p.ctypes.data, o.ctypes.data, n,
                                              ctypes.byref(got)), "rdf_copy_triples")
        return s[:got.value], p[:got.value], o[:got.value]

    def frequent_conditions(self, min_support: int):
        st = FcStats()
        self._check(self.lib.rdf_frequent_conditions(self.ptr, min_support, ctypes.byref(st)),
                    "rdf_frequent_conditions")
        self.fc = _struct_dict(st)
        return self.fc

    def association_rules(self) -> int:
        """--use-ars after frequent_conditions (rdf_association_rules); returns the number of rules."""
        n = ctypes.c_uint64()
        self._check(self.lib.rdf_association_rules(self.ptr, ctypes.byref(n)), "rdf_association_rules")
        self.n_rules = int(n.value)
        return self.n_rules

    def copy_association_rules(self) -> np.ndarray:
        """The rules of the last rdf_association_rules (or sharded run with use_ars), RULE_DTYPE rows."""
        n = ctypes.c_uint64()
        self._check(self.lib.rdf_association_rule_count(self.ptr, ctypes.byref(n)), "rdf_association_rule_count")
        self.n_rules = int(n.value)
        out = np.empty(self.n_rules, dtype=RULE_DTYPE)
        got = ctypes.c_uint64()
        self._check(self.lib.rdf_copy_association_rules(self.ptr, out.ctypes.data, len(out), ctypes.byref(got)),
                    "rdf_copy_association_rules")
        return out[:got.value]

    def build_capture_groups(self, projection: str = "spo"):
        st = GroupStats()
        self._check(self.lib.rdf_build_capture_groups(self.ptr, projection.encode(), ctypes.byref(st)),
                    "rdf_build_capture_groups")
        self.groups = _struct_dict(st)
        return self.groups

    def discover_cinds(self, clean_implied: bool = True, traversal_strategy: int = 1):
        flags = (RDF_CLEAN_IMPLIED if clean_implied else 0) | (RDF_STRATEGY_ALL_AT_ONCE if traversal_strategy == 0 else 0)
        st = CindStats()
        self._check(self.lib.rdf_discover_cinds(self.ptr, flags, ctypes.byref(st)), "rdf_discover_cinds")
        self.cinds = _struct_dict(st)
        return self.cinds

    def discover_cinds_paged(self, clean_implied: bool = True, traversal_strategy: int = 1, page_bytes: int = 0):
        """rdf_discover_cinds_paged: prepares a paged run (page_bytes of working memory per page, 0 = automatic)."""
        flags = (RDF_CLEAN_IMPLIED if clean_implied else 0) | (RDF_STRATEGY_ALL_AT_ONCE if traversal_strategy == 0 else 0)
        st = CindStats()
        self._check(self.lib.rdf_discover_cinds_paged(self.ptr, flags, page_bytes, ctypes.byref(st)),
                    "rdf_discover_cinds_paged")
        self.cinds = _struct_dict(st)
        return self.cinds

    def next_page(self):
        """rdf_next_page: the next page becomes the current result; returns (first_dep, end_dep), or None when done."""
        done, d0, d1 = ctypes.c_uint32(), ctypes.c_uint64(), ctypes.c_uint64()
        self._check(self.lib.rdf_next_page(self.ptr, ctypes.byref(done), ctypes.byref(d0), ctypes.byref(d1)),
                    "rdf_next_page")
        return None if done.value else (int(d0.value), int(d1.value))

    def pages(self, clean_implied: bool = True, traversal_strategy: int = 1, page_bytes: int = 0):
        """Iterates a paged run: yields (first_dep, end_dep) with each page as the current result."""
        self.discover_cinds_paged(clean_implied, traversal_strategy, page_bytes)
        self._pages = 0
        while True:
            r = self.next_page()
            if r is None:
                return
            self._pages += 1
            yield r

    def run(self, min_support=10, projection="spo", clean_implied=True, traversal_strategy=1, use_ars=False):
        self.frequent_conditions(min_support)
        if use_ars:
            self.association_rules()
        self.build_capture_groups(projection)
        return self.discover_cinds(clean_implied, traversal_strategy)

    def sync(self):
        self._check(self.lib.rdf_sync(self.ptr), "rdf_sync")

    def device_bytes(self) -> int:
        """HBM bytes the context holds (rdf_device_bytes)."""
        v = ctypes.c_uint64()
        self._check(self.lib.rdf_device_bytes(self.ptr, ctypes.byref(v)), "rdf_device_bytes")
        return int(v.value)

    def release_scratch(self):
        """rdf_release_scratch: frees every per-run buffer (triples and dictionary stay); frequent_conditions next."""
        self._check(self.lib.rdf_release_scratch(self.ptr), "rdf_release_scratch")

    def last_stats(self):
        fc, gs, cs = FcStats(), GroupStats(), CindStats()
        self._check(self.lib.rdf_last_stats(self.ptr, ctypes.byref(fc), ctypes.byref(gs), ctypes.byref(cs)),
                    "rdf_last_stats")
        self.fc, self.groups, self.cinds = _struct_dict(fc), _struct_dict(gs), _struct_dict(cs)
        return self.groups, self.cinds

    # -- sharded mode (driven by rdfind_amd.distributed.run_sharded) ---------------------------
    def shard_begin(self, rank: int, nranks: int, min_support: int, projection="spo", clean_implied=True,
                    traversal_strategy=1, local_slice=False, use_ars=False):
        self.n_rules = 0
        """local_slice: the resident triples are this rank's slice of the input (else every rank holds all of
        them and the library takes its row range).  use_ars: association rules from the combined counts."""
        flags = (RDF_CLEAN_IMPLIED if clean_implied else 0) | (RDF_STRATEGY_ALL_AT_ONCE if traversal_strategy == 0 else 0)
        flags |= RDF_SHARD_LOCAL_SLICE if local_slice else 0
        flags |= RDF_USE_ASSOCIATION_RULES if use_ars else 0
        self._nranks = nranks
        self._check(self.lib.rdf_shard_begin(self.ptr, rank, nranks, min_support, projection.encode(), flags),
                    "rdf_shard_begin")

    def shard_parse_begin(self, rank: int, nranks: int, data: bytes, tabs: bool = False) -> int:
        """Sharded ingest of this rank's part of the input (rdf_shard_parse_begin); drive it with
        distributed.run_protocol.  Returns the rank's triples."""
        n = ctypes.c_uint64()
        self._nranks = nranks
        self._parsed = data
        self._check(self.lib.rdf_shard_parse_begin(self.ptr, rank, nranks, data, len(data), RDF_NT_TABS if tabs else 0,
                                                   ctypes.byref(n)), "rdf_shard_parse_begin")
        return int(n.value)

    def shard_dictionary_begin(self):
        """The formatting dictionary by owner lookup after a sharded run (rdf_shard_dictionary_begin)."""
        self._check(self.lib.rdf_shard_dictionary_begin(self.ptr), "rdf_shard_dictionary_begin")

    def num_terms_now(self) -> int:
        v = ctypes.c_uint32()
        self._check(self.lib.rdf_num_terms(self.ptr, ctypes.byref(v)), "rdf_num_terms")
        self.num_terms = int(v.value)
        return self.num_terms

    def dictionary_terms(self, ids) -> list:
        """Terms of the formatting dictionary (rdf_dictionary_terms), as str."""
        ids = np.ascontiguousarray(ids, dtype=np.uint32)
        off = np.zeros(ids.shape[0] + 1, np.uint64)
        cap = 1 << 20
        while True:
            out = ctypes.create_string_buffer(cap)
            rc = self.lib.rdf_dictionary_terms(self.ptr, ids.ctypes.data, ids.shape[0], out, cap, off.ctypes.data)
            if rc == 0:
                raw = out.raw
                return [raw[int(off[i]):int(off[i + 1])].decode("utf-8") for i in range(ids.shape[0])]
            if int(off[-1]) <= cap:
                self._check(rc, "rdf_dictionary_terms")
            cap = int(off[-1])

    def shard_step(self) -> ExchangeRequest:
        x = Exchange()
        self._check(self.lib.rdf_shard_step(self.ptr, ctypes.byref(x)), "rdf_shard_step")
        return ExchangeRequest(x.op, x.elem_bytes, x.count, list(x.send_counts)[: self._nranks])

    def shard_export(self, dst_ptr: int):
        self._check(self.lib.rdf_shard_export(self.ptr, dst_ptr), "rdf_shard_export")

    def shard_import(self, src_ptr: int, count: int):
        self._check(self.lib.rdf_shard_import(self.ptr, src_ptr, count), "rdf_shard_import")

    def stage_times(self):
        arr = (ctypes.c_float * 3)()
        self._check(self.lib.rdf_stage_times(self.ptr, arr), "rdf_stage_times")
        return list(arr)

    def kernel_times(self):
        arr = (ctypes.c_float * len(TIMER_NAMES))()
        self._check(self.lib.rdf_kernel_times(self.ptr, arr, len(TIMER_NAMES)), "rdf_kernel_times")
        return dict(zip(TIMER_NAMES, list(arr)))

    # -- results -----------------------------------------------------------------------------
    def cind_count(self) -> int:
        n = ctypes.c_uint64()
        self._check(self.lib.rdf_cind_count(self.ptr, ctypes.byref(n)), "rdf_cind_count")
        return n.value

    def copy_cinds(self) -> np.ndarray:
        n = self.cind_count()
        out = np.empty(n, dtype=CIND_DTYPE)
        copied = ctypes.c_uint64()
        self._check(self.lib.rdf_copy_cinds(self.ptr, out.ctypes.data, n, ctypes.byref(copied)), "rdf_copy_cinds")
        return out[: copied.value]

    def copy_cinds_range(self, offset: int, count: int) -> np.ndarray:
        out = np.empty(count, dtype=CIND_DTYPE)
        copied = ctypes.c_uint64()
        self._check(self.lib.rdf_copy_cinds_range(self.ptr, offset, out.ctypes.data, count, ctypes.byref(copied)),
                    "rdf_copy_cinds_range")
        return out[: copied.value]

    def result_sizes(self):
        """(n_refs, n_runs, n_captures) of the CindSet-shaped result (rdf_result_sizes)."""
        a, b, c = ctypes.c_uint64(), ctypes.c_uint64(), ctypes.c_uint64()
        self._check(self.lib.rdf_result_sizes(self.ptr, ctypes.byref(a), ctypes.byref(b), ctypes.byref(c)),
                    "rdf_result_sizes")
        return int(a.value), int(b.value), int(c.value)

    def copy_result_raw(self, refs_ptr=None, runoff=None, rundep=None, capture_ids=None, supports=None):
        """rdf_copy_result_raw into caller buffers (raw pointers or numpy arrays; None skips a part)."""
        def ptr(x):
            return None if x is None else (x if isinstance(x, int) else x.ctypes.data)
        self._check(self.lib.rdf_copy_result_raw(self.ptr, ptr(refs_ptr), ptr(runoff), ptr(rundep), ptr(capture_ids),
                                                 ptr(supports)), "rdf_copy_result_raw")

    def result_layout(self) -> dict:
        """Sizes of the compact CindSet-shaped result (rdf_get_result_layout)."""
        L = ResultLayout()
        self._check(self.lib.rdf_get_result_layout(self.ptr, ctypes.byref(L)), "rdf_get_result_layout")
        return _struct_dict(L)

    def copy_result_compact(self, bufs: dict | None = None) -> dict:
        """rdf_copy_result_compact into ``bufs`` (name -> numpy array or raw pointer, e.g. pinned memory sized from
        :meth:`result_layout`), or into fresh numpy arrays; returns the name -> buffer dict."""
        fresh = bufs is None
        if fresh:
            L = self.result_layout()
            bufs = {name: np.empty(max(count(L), 1), dt) for name, dt, count in COMPACT_PARTS}
            bufs["layout"] = L
        ptrs = [bufs[name] if isinstance(bufs[name], int) else bufs[name].ctypes.data for name, _, _ in COMPACT_PARTS]
        self._check(self.lib.rdf_copy_result_compact(self.ptr, *ptrs), "rdf_copy_result_compact")
        if fresh:  # the heavy-bits form's chunks (rdf_set_result_form), when the result has them
            nh = self.heavy_chunk_count()
            bufs["n_heavy_chunks"] = nh
            if nh:
                bufs["heavy_deps"] = np.empty(nh, np.uint32)
                bufs["heavy_pos"] = np.empty(nh, np.uint64)
                bufs["heavy_bits"] = np.empty(nh, np.uint64)
                self.copy_result_heavy(bufs["heavy_deps"], bufs["heavy_pos"], bufs["heavy_bits"])
        return bufs

    def set_handover(self, refs=None, refs_cap: int = 0, runoff=None, rundep=None, runs_cap: int = 0, capture_ids=None,
                     supports=None, capture_cap: int = 0):
        """rdf_set_handover: page-locked buffers (raw pointers or numpy arrays) the next unpaged discoveries fill early;
        rdf_copy_result_compact with the same buffers then copies only the rest.  No arguments: unregister."""
        p = [None if x is None else (x if isinstance(x, int) else x.ctypes.data)
             for x in (refs, runoff, rundep, capture_ids, supports)]
        self._check(self.lib.rdf_set_handover(self.ptr, p[0] or None, refs_cap, p[1] or None, p[2] or None, runs_cap,
                                              p[3] or None, p[4] or None, capture_cap), "rdf_set_handover")

    def copy_result_refs(self, offset: int, count: int, ptr) -> int:
        """rdf_copy_result_refs: refs[offset, offset + count) of the compact result into ``ptr`` (numpy array or raw
        pointer); returns the refs copied."""
        copied = ctypes.c_uint64()
        p = ptr if isinstance(ptr, int) else ptr.ctypes.data
        self._check(self.lib.rdf_copy_result_refs(self.ptr, offset, count, p, ctypes.byref(copied)), "rdf_copy_result_refs")
        return copied.value

    def copy_result_refs_async(self, offset: int, count: int, ptr: int) -> int:
        """rdf_copy_result_refs_async: the same copy queued on the context's copy stream (``ptr``: page-locked, untouched
        until handover_wait); returns the refs queued."""
        copied = ctypes.c_uint64()
        self._check(self.lib.rdf_copy_result_refs_async(self.ptr, offset, count, ptr, ctypes.byref(copied)),
                    "rdf_copy_result_refs_async")
        return copied.value

    def set_result_form(self, heavy_bits: bool) -> None:
        """rdf_set_result_form: RDF_FORM_HEAVY_BITS (the heavy-only refs as survivor words over the class lists) or
        the expanded form, from the next discovery on."""
        self._check(self.lib.rdf_set_result_form(self.ptr, 1 if heavy_bits else 0), "rdf_set_result_form")

    def heavy_chunk_count(self) -> int:
        n = ctypes.c_uint64()
        self._check(self.lib.rdf_heavy_chunk_count(self.ptr, ctypes.byref(n)), "rdf_heavy_chunk_count")
        return int(n.value)

    def copy_result_heavy(self, deps, pos, bits) -> None:
        """rdf_copy_result_heavy into three buffers (numpy arrays or raw pointers) of heavy_chunk_count() elements."""
        ptrs = [b if isinstance(b, int) else b.ctypes.data for b in (deps, pos, bits)]
        self._check(self.lib.rdf_copy_result_heavy(self.ptr, *ptrs), "rdf_copy_result_heavy")

    def handover_wait(self) -> None:
        """rdf_handover_wait: every queued copy has reached the host."""
        self._check(self.lib.rdf_handover_wait(self.ptr), "rdf_handover_wait")

    def copy_cinds_decoded(self, offset: int = 0, count: int | None = None) -> np.ndarray:
        """Cind-shaped rows decoded on the device (rdf_copy_cinds_decoded), ROW_DTYPE."""
        if count is None:
            count = max(self.cind_count() - offset, 0)
        out = np.empty(count, dtype=ROW_DTYPE)
        copied = ctypes.c_uint64()
        self._check(self.lib.rdf_copy_cinds_decoded(self.ptr, offset, out.ctypes.data, count, ctypes.byref(copied)),
                    "rdf_copy_cinds_decoded")
        return out[: copied.value]

    def checksum(self) -> int:
        v = ctypes.c_uint64()
        self._check(self.lib.rdf_cind_checksum(self.ptr, ctypes.byref(v)), "rdf_cind_checksum")
        return v.value

    def binary_keys(self) -> np.ndarray:
        n = ctypes.c_uint64()
        self._check(self.lib.rdf_binary_key_count(self.ptr, ctypes.byref(n)), "rdf_binary_key_count")
        out = np.empty(n.value, dtype=np.uint64)
        if n.value:
            self._check(self.lib.rdf_copy_binary_keys(self.ptr, out.ctypes.data, n.value), "rdf_copy_binary_keys")
        return out

    def set_dictionary(self, terms):
        """Uploads the dictionary (term id -> string) for device-side formatting."""
        enc = [t.encode("utf-8") for t in terms]
        heap = b"".join(enc)
        offsets = np.zeros(len(enc) + 1, dtype=np.uint64)
        if enc:
            np.cumsum(np.fromiter((len(e) for e in enc), dtype=np.uint64, count=len(enc)), out=offsets[1:])
        buf = ctypes.create_string_buffer(heap, max(len(heap), 1))
        self._check(self.lib.rdf_set_dictionary(self.ptr, buf, len(heap), offsets.ctypes.data, len(enc)),
                    "rdf_set_dictionary")

    def format_array(self, offset=0, count=None) -> np.ndarray:
        """Cind.toString lines ("...\n" each) of result rows [offset, offset + count), formatted on the GPU, as a
        uint8 array (no intermediate copies: write it to a file with ``arr.tofile`` / ``f.write(arr)``)."""
        if count is None:
            count = self.cind_count() - offset
        need = ctypes.c_uint64()
        self._check(self.lib.rdf_format_size(self.ptr, offset, count, ctypes.byref(need)), "rdf_format_size")
        out = np.empty(max(need.value, 1), dtype=np.uint8)
        got = ctypes.c_uint64()
        self._check(self.lib.rdf_format_cinds(self.ptr, offset, count, out.ctypes.data, need.value, ctypes.byref(got)),
                    "rdf_format_cinds")
        return out[: got.value]

    def format_cinds(self, offset=0, count=None) -> bytes:
        """As format_array, as bytes."""
        return self.format_array(offset, count).tobytes()

    def decoded_cinds(self):
        """Structured array with (dep_code, dep_v1, dep_v2, ref_code, ref_v1, ref_v2, support);
        v2 = 0xFFFFFFFF for unary captures."""
        rows = self.copy_cinds()
        return decode_rows(rows, self.num_terms, self.binary_keys())


DECODED_DTYPE = np.dtype([("dep_code", "u1"), ("dep_v1", "<u4"), ("dep_v2", "<u4"), ("ref_code", "u1"),
                          ("ref_v1", "<u4"), ("ref_v2", "<u4"), ("support", "<u4")])


def decode_captures(cap: np.ndarray, num_terms: int, bin_keys: np.ndarray):
    """Vectorised capture id -> (code, v1, v2)."""
    V = np.uint64(max(num_terms, 1))
    cap = cap.astype(np.uint64)
    unary = cap < np.uint64(6) * V
    code = np.empty(cap.shape, np.uint8)
    v1 = np.empty(cap.shape, np.uint32)
    v2 = np.full(cap.shape, 0xFFFFFFFF, np.uint32)
    ucodes = np.array(codes.UNARY_CODES, np.uint8)
    code[unary] = ucodes[(cap[unary] // V).astype(np.int64)]
    v1[unary] = (cap[unary] % V).astype(np.uint32)
    if (~unary).any():
        keys = bin_keys[(cap[~unary] - np.uint64(6) * V).astype(np.int64)]
        bcodes = np.array(codes.BINARY_CODES, np.uint8)
        code[~unary] = bcodes[(keys >> np.uint64(62)).astype(np.int64)]
        v1[~unary] = ((keys >> np.uint64(31)) & np.uint64(0x7FFFFFFF)).astype(np.uint32)
        v2[~unary] = (keys & np.uint64(0x7FFFFFFF)).astype(np.uint32)
    return code, v1, v2


def decode_rows(rows: np.ndarray, num_terms: int, bin_keys: np.ndarray) -> np.ndarray:
    out = np.empty(rows.shape[0], dtype=DECODED_DTYPE)
    out["dep_code"], out["dep_v1"], out["dep_v2"] = decode_captures(rows["dep"], num_terms, bin_keys)
    out["ref_code"], out["ref_v1"], out["ref_v2"] = decode_captures(rows["ref"], num_terms, bin_keys)
    out["support"] = rows["support"]
    return out


def decoded_to_set(dec: np.ndarray):
    """Set of (dt, dv1, dv2|None, rt, rv1, rv2|None, support) -- the oracle's comparison form."""
    none = 0xFFFFFFFF
    out = set()
    for r in dec.tolist():
        dt, dv1, dv2, rt, rv1, rv2, sup = r
        out.add((dt, dv1, None if dv2 == none else dv2, rt, rv1, None if rv2 == none else rv2, sup))
    return out
