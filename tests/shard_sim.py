"""CPU model of the sharded protocol (test infrastructure, built on the oracle).

``ShardSim`` answers the same ``shard_begin / shard_step / shard_export / shard_import`` calls as the HIP
``Context`` in sharded mode, with the same sequence of collectives (rdfind_amd/distributed.py), but
computes each rank's part with the Python oracle: join lines of the join values this rank owns, local
intersections of the light dependents, owner-side multiplicity check, then minimality on the gathered
explicit set.  It treats every group as light (no bitmask columns), so the class exchange is empty.
It lets the CPU suite run the real collectives (gloo, world size 2) and check that the decomposition
-- shard by join hash, intersect locally, route by dependent, count reporters -- reproduces the
single-process oracle result.
"""
from __future__ import annotations

import ctypes

import numpy as np

from oracle import rdfind_oracle as R
from rdfind_amd import _lib


def shard_of(join: int, nranks: int) -> int:
    """Owner of a join value; the same function as common.hpp shard_of."""
    if nranks <= 1:
        return 0
    return (((join * 0x9E3779B97F4A7C15) & 0xFFFFFFFFFFFFFFFF) >> 32) % nranks


def _view(ptr, n, dtype):
    ct = ctypes.c_int32 if dtype == np.int32 else ctypes.c_int64
    return np.ctypeslib.as_array((ct * n).from_address(ptr)) if n else np.zeros(0, dtype)


class ShardSim:
    def __init__(self, triples):
        self.triples = [tuple(int(x) for x in t) for t in triples]
        self.result = None

    def shard_begin(self, rank, nranks, min_support, projection="spo", clean_implied=True, traversal_strategy=1):
        self.rank, self.R, self.ms = rank, nranks, max(min_support, 1)
        self.proj, self.clean, self.strategy = projection, clean_implied, traversal_strategy
        self.phase = 0
        self.pending = None

    # -- machine ----------------------------------------------------------------------------
    def shard_step(self):
        fn = getattr(self, f"_phase{self.phase}")
        return fn()

    def _req(self, op, send, nxt, send_counts=None):
        self.pending = (op, np.ascontiguousarray(send))
        self.phase = nxt
        return _lib.ExchangeRequest(op, 4 if op == _lib.X_ALLREDUCE_SUM_U32 else 8, len(send), send_counts)

    def shard_export(self, ptr):
        op, arr = self.pending
        if len(arr):
            _view(ptr, len(arr), arr.dtype)[:] = arr

    def shard_import(self, ptr, n):
        op, arr = self.pending
        self.recv = _view(ptr, n, arr.dtype).copy()

    def _phase0(self):
        tr = self.triples
        self.uf = R.frequent_unary_conditions(tr, self.ms)
        self.bf = R.frequent_binary_conditions(tr, self.uf, self.ms)
        lines = R.join_lines(tr, self.uf, self.bf, self.proj)
        caps = set()
        self.local = []
        for jv, line in lines.items():
            u, b = R.line_captures(line)
            caps |= u | b
            if shard_of(jv, self.R) == self.rank:
                self.local.append(u | b)
        self.universe = sorted(caps, key=lambda c: c.key())  # identical on every rank (replicated triples)
        self.index = {c: i for i, c in enumerate(self.universe)}
        sup = np.zeros(len(self.universe), np.int32)
        for g in self.local:
            for c in g:
                sup[self.index[c]] += 1
        return self._req(_lib.X_ALLREDUCE_SUM_U32, sup, 1)

    def _phase1(self):
        self.support = self.recv.astype(np.int64)
        self.freq = [c for c in self.universe if self.support[self.index[c]] >= self.ms]
        self.cid = {c: i for i, c in enumerate(self.freq)}
        self.groups = [frozenset(self.cid[c] for c in g if c in self.cid) for g in self.local]
        self.groups = [g for g in self.groups if g]
        return self._req(_lib.X_ALLGATHERV_U64, np.zeros(256, np.int64), 2)  # no bitmask columns

    def _phase2(self):
        assert len(self.recv) == 256 * self.R
        return self._req(_lib.X_ALLREDUCE_SUM_U64, np.zeros(len(self.freq), np.int64), 3)

    def _phase3(self):
        C = len(self.freq)
        self.dep_groups = [[] for _ in range(C)]
        for g in self.groups:
            for d in g:
                self.dep_groups[d].append(g)
        best = np.full(C, np.iinfo(np.int64).max, np.int64)
        for d, gs in enumerate(self.dep_groups):
            if gs:
                best[d] = (min(len(g) for g in gs) << 32) | self.rank
        return self._req(_lib.X_ALLREDUCE_MIN_U64, best, 4)

    def _phase4(self):
        self.gbest = self.recv.copy()
        words = np.array([len(gs) | ((1 if gs else 0) << 40) for gs in self.dep_groups], np.int64)
        return self._req(_lib.X_ALLREDUCE_SUM_U64, words, 5)

    def _excluded(self, d, r):
        dc, rc = self.freq[d], self.freq[r]
        return dc.implies(rc) if self.strategy == 0 else R.trivially_implied(dc, rc)

    def _phase5(self):
        self.nrl = (self.recv >> 40).astype(np.int64)
        out = [[] for _ in range(self.R)]
        for d, gs in enumerate(self.dep_groups):
            if not gs:
                continue
            refs = set.intersection(*(set(g) for g in gs))
            for r in sorted(refs):
                if r != d and not self._excluded(d, r):
                    out[d % self.R].append((d << 32) | r)
        send = np.array([x for part in out for x in part], np.int64)
        return self._req(_lib.X_ALLTOALLV_U64, send, 6, [len(p) for p in out])

    def _phase6(self):
        vals, cnt = np.unique(self.recv, return_counts=True)
        keep = [int(v) for v, c in zip(vals.tolist(), cnt.tolist()) if c == self.nrl[int(v) >> 32]]
        return self._req(_lib.X_ALLGATHERV_U64, np.array(keep, np.int64), 7)

    def _phase7(self):
        self.explicit = sorted(int(x) for x in self.recv)
        return self._req(_lib.X_ALLGATHERV_U64, np.zeros(0, np.int64), 8)

    def _phase8(self):
        assert len(self.recv) == 0
        v = []
        for pr in self.explicit:
            d, r = pr >> 32, pr & 0xFFFFFFFF
            dc, rc = self.freq[d], self.freq[r]
            v.append(R.norm_cind(dc.type, dc.v1, dc.v2, rc.type, rc.v1, rc.v2, int(self.support[self.index[dc]])))
        if self.clean:
            v = R.remove_implied(*R.split_by_arity(v))
        elif self.strategy == 1:
            v = R.s2l_exact_raw(v)
        owned = {self.freq[d].key() for d in range(len(self.freq)) if d % self.R == self.rank}
        self.result = [c for c in v if R.Cond(c.dv1, c.dv2, c.dt).key() in owned]
        self.phase = 9
        return _lib.ExchangeRequest(_lib.X_DONE, 8, 0)
