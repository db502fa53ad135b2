"""CPU model of the sharded protocol (test infrastructure, built on the oracle).

``ShardSim`` answers the same ``shard_begin / shard_step / shard_export / shard_import`` calls as the HIP
``Context`` in sharded mode, with the same sequence of collectives and message layouts
(rdfind_amd/distributed.py, rdfind_hip.hip sh_phase10, 16, 18, 11-14 and 1-8), but computes each rank's part with
the Python oracle: unary and binary (key, count) partials of the rank's slice routed to the key's owner
(all-to-all, same key hash as shard.inl key_owner), the hot join value candidates and slice sizes all-gathered and
turned into the same balanced owner table as sh_phase18 on every rank, the frequent keys all-gathered, every
triple routed to the owners of its join values (all-to-all, two words per copy; join_owner: the hot table, else the
hash), join lines of the join values this rank owns, local intersections, owner-side multiplicity check, then
minimality on the gathered
explicit set (every rank's unary dependents' pairs + its own binary ones).  It treats every group as light (no bitmask columns), so the class exchange is empty.
It lets the CPU suite run the real collectives (gloo, world size 2 and 3) and check that the decomposition
reproduces the single-process oracle result.
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


M64 = 0xFFFFFFFFFFFFFFFF


def mix64(x: int) -> int:
    """common.hpp mix64 (murmur3 finaliser)."""
    x ^= x >> 33
    x = (x * 0xFF51AFD7ED558CCD) & M64
    x ^= x >> 33
    x = (x * 0xC4CEB9FE1A85EC53) & M64
    x ^= x >> 33
    return x


HOT_DIV, HOT_CAP = 4096, 32768  # rdfind_hip.hip sh_phase16 / sh_phase18


def hot_owner_table(words, V: int, nranks: int, nproj: int) -> dict:
    """rdfind_hip.hip sh_phase18: every rank's gathered hot candidates (key << 32 | count, key = pos * V + value) and
    slice-size markers (0xffffffff << 32 | n) -> {join value: owner rank}, identical on every rank: occurrences summed
    per value, values with >= nproj * n_total / (R * HOT_DIV) of them assigned largest first (ties: smaller value) to the
    least loaded rank (ties: lower rank), each rank starting from its share of the hashed rest."""
    n_total, occ = 0, {}
    for w in words:
        w &= M64
        key, cnt = w >> 32, w & 0xFFFFFFFF
        if key == 0xFFFFFFFF:
            n_total += cnt
            continue
        occ[key % V] = occ.get(key % V, 0) + cnt
    total = float(nproj * n_total)
    thr = max(1, int(total / (float(nranks) * HOT_DIV)))
    hot = sorted(((c, v) for v, c in occ.items() if c >= thr), key=lambda x: (-x[0], x[1]))
    if not hot:
        return {}
    hot_total = float(sum(c for c, _ in hot))
    load = [max(0.0, total - hot_total) / nranks] * nranks
    table = {}
    for c, v in hot:
        r = min(range(nranks), key=lambda q: (load[q], q))
        load[r] += c
        table[v] = r
    return table


def key_owner(key: int, nranks: int) -> int:
    """shard.inl key_owner: the rank that sums a binary condition's partial counts."""
    return (mix64(key) & 0xFFFFFFFF) % nranks


def dep_owner(d: int, nranks: int) -> int:
    """common.hpp dep_owner: the rank that finalises a dependent's refs."""
    return 0 if nranks <= 1 else (mix64(d) >> 32) % nranks


# binary condition type (S|P, S|O, P|O) <-> the library's key type bt (o[s,p] 2, p[s,o] 1, s[p,o] 0)
_BT = {3: 2, 5: 1, 6: 0}
_BT_INV = {v: k for k, v in _BT.items()}


def bin_key(t, v1, v2):
    return (_BT[t] << 62) | (v1 << 31) | v2


def _i64(x: int) -> int:
    """unsigned 64-bit word -> the int64 the exchange buffers hold"""
    return x - (1 << 64) if x >= (1 << 63) else x


def _view(ptr, n, dtype):
    ct = ctypes.c_int32 if dtype == np.int32 else ctypes.c_int64
    return np.ctypeslib.as_array((ct * n).from_address(ptr)) if n else np.zeros(0, dtype)


class ShardSim:
    def __init__(self, triples, num_terms=None, local_slice=False):
        self.triples = [tuple(int(x) for x in t) for t in triples]
        self.V = num_terms if num_terms is not None else 1 + max((max(t) for t in self.triples), default=0)
        self.local_slice = local_slice
        self.result = None

    def shard_begin(self, rank, nranks, min_support, projection="spo", clean_implied=True, traversal_strategy=1,
                    local_slice=None):
        self.rank, self.R, self.ms = rank, nranks, max(min_support, 1)
        self.proj, self.clean, self.strategy = projection, clean_implied, traversal_strategy
        if local_slice is not None:
            self.local_slice = local_slice
        n = len(self.triples)
        self.slice = self.triples if self.local_slice else self.triples[n * rank // nranks: n * (rank + 1) // nranks]
        self.phase = 10
        self.pending = None
        self.hot = {}

    def join_owner(self, v: int) -> int:
        """common.hpp join_owner: the hot table's owner, else the hash"""
        return self.hot.get(v, shard_of(v, self.R))

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

    def _phase10(self):  # unary (key << 32 | count) partials of the slice -> the keys' owners
        V = self.V
        cnt = np.zeros(3 * V, np.int64)
        for s, p, o in self.slice:
            cnt[s] += 1
            cnt[V + p] += 1
            cnt[2 * V + o] += 1
        out = [[] for _ in range(self.R)]
        for k in np.nonzero(cnt)[0].tolist():
            out[key_owner(k, self.R)].append((k << 32) | int(cnt[k]))
        send = np.array([x for o in out for x in o], np.int64)
        return self._req(_lib.X_ALLTOALLV_U64, send, 16, [len(o) for o in out])

    def _phase16(self):  # summed partials of the owned unary keys -> hot join value candidates + slice size
        V = self.V
        self.tot = {}
        for w in self.recv.astype(np.int64).tolist():
            self.tot[w >> 32] = self.tot.get(w >> 32, 0) + (w & 0xFFFFFFFF)
        pbits = sum(1 << i for i, c in enumerate("spo") if c in self.proj)
        nproj = bin(pbits).count("1")
        thr = max(1, nproj * len(self.slice) // (3 * HOT_DIV))
        cand = sorted(((c, k) for k, c in self.tot.items() if c >= thr and (pbits >> (k // V)) & 1),
                      key=lambda x: (-x[0], x[1]))[:HOT_CAP]  # the top HOT_CAP by count (ties: smaller key)
        words = [(0xFFFFFFFF << 32) | len(self.slice)] + [(k << 32) | c for c, k in cand]
        return self._req(_lib.X_ALLGATHERV_U64, np.array([_i64(w) for w in words], np.int64), 18)

    def _phase18(self):  # the hot join values' owners (same table on every rank); frequent unary keys -> all-gather
        nproj = sum(1 for c in "spo" if c in self.proj)
        self.hot = hot_owner_table(self.recv.tolist(), self.V, self.R, nproj)
        return self._req(_lib.X_ALLGATHERV_U64,
                         np.array(sorted(k for k, c in self.tot.items() if c >= self.ms), np.int64), 11)

    def _phase11(self):  # frequent unary conditions (every owner's keys); binary partials -> owners
        V = self.V
        keys = sorted(int(k) for k in self.recv.tolist())
        self.uf = {t: {} for t in (R.S, R.P, R.O)}
        for k in keys:
            self.uf[(R.S, R.P, R.O)[k // V]][k % V] = 1  # presence is all the join-line construction reads
        part = R.frequent_binary_conditions(self.slice, self.uf, 1)  # local counts of every key (threshold 1)
        out = [[] for _ in range(self.R)]
        for (t, v1, v2), c in sorted(part.items()):
            k = bin_key(t, v1, v2)
            out[key_owner(k, self.R)] += [_i64(k), c]
        send = np.array([x for o in out for x in o], np.int64)
        return self._req(_lib.X_ALLTOALLV_U64, send, 12, [len(o) for o in out])

    def _phase12(self):  # summed partials of the owned keys -> frequent keys -> all-gather
        tot = {}
        r = self.recv.astype(np.int64)
        for k, c in zip(r[0::2].tolist(), r[1::2].tolist()):
            tot[k] = tot.get(k, 0) + c
        return self._req(_lib.X_ALLGATHERV_U64, np.array(sorted(k for k, c in tot.items() if c >= self.ms), np.int64), 13)

    def _phase13(self):  # every owner's frequent keys; triples -> the owners of their join values
        self.bf = {}
        for k in self.recv.tolist():
            k &= M64
            self.bf[(_BT_INV[k >> 62], (k >> 31) & 0x7FFFFFFF, k & 0x7FFFFFFF)] = 1
        out = [[] for _ in range(self.R)]
        for s, p, o in self.slice:
            dests = []
            for pos, v in (("s", s), ("p", p), ("o", o)):
                if pos in self.proj and self.join_owner(v) not in dests:
                    dests.append(self.join_owner(v))
            for d in dests:
                out[d] += [(s << 32) | p, o]
        send = np.array([x for o in out for x in o], np.int64)
        return self._req(_lib.X_ALLTOALLV_U64, send, 14, [len(o) for o in out])

    def _phase14(self):  # join lines of the owned join values; capture universe from the global conditions
        r = self.recv.astype(np.int64)
        tr = [(int(w0 >> 32), int(w0 & 0xFFFFFFFF), int(w1)) for w0, w1 in zip(r[0::2].tolist(), r[1::2].tolist())]
        lines = R.join_lines(tr, self.uf, self.bf, self.proj)
        self.local = []
        for jv, line in lines.items():
            if self.join_owner(jv) == self.rank:
                u, b = R.line_captures(line)
                self.local.append(u | b)
        caps = set()
        for t, sec in ((R.S, (R.P, R.O)), (R.P, (R.S, R.O)), (R.O, (R.S, R.P))):
            for v in self.uf[t]:
                for q in sec:
                    caps.add(R.Cond(v, None, R.create_code(t, secondary=q)))
        for (t, v1, v2) in self.bf:
            caps.add(R.Cond(v1, v2, R.add_secondary(t)))
        self.universe = sorted(caps, key=lambda c: c.key())  # identical on every rank
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
        words = [len(gs) | ((1 if gs else 0) << 40) for gs in self.dep_groups]
        words += [(1 << self.rank) if gs else 0 for gs in self.dep_groups]
        return self._req(_lib.X_ALLREDUCE_SUM_U64, np.array([_i64(w) for w in words], np.int64), 5)

    def _excluded(self, d, r):
        dc, rc = self.freq[d], self.freq[r]
        return dc.implies(rc) if self.strategy == 0 else R.trivially_implied(dc, rc)

    def _phase5(self):  # holder-first: the pivot holder's survivors -> owner (report) + other light ranks (verify)
        C = len(self.freq)
        self.nrl = (self.recv[:C] >> 40).astype(np.int64)
        lmask = [int(x) & ((1 << 64) - 1) for x in self.recv[C:].tolist()]
        out = [[] for _ in range(self.R)]
        for d, gs in enumerate(self.dep_groups):
            if not gs or (int(self.gbest[d]) & 0xFFFFFFFF) != self.rank:
                continue
            refs = set.intersection(*(set(g) for g in gs))
            for r in sorted(refs):
                if r != d and not self._excluded(d, r):
                    out[dep_owner(d, self.R)].append((0, d, r))
                    for q in range(self.R):
                        if q != self.rank and (lmask[d] >> q) & 1:
                            out[q].append((1, d, r))
        send = np.array([(t << 63) | (d << 32) | r for part in out for t, d, r in part], np.uint64).view(np.int64)
        return self._req(_lib.X_ALLTOALLV_U64, send, 15, [len(p) for p in out])

    def _phase15(self):  # keep the reports; verify the other pairs against the local light groups -> owners
        words = self.recv.view(np.uint64).tolist()
        self.reports = [w for w in words if not w >> 63]
        out = [[] for _ in range(self.R)]
        for w in words:
            if w >> 63:
                d, r = (w >> 32) & 0x7FFFFFFF, w & 0xFFFFFFFF
                if all(r in g for g in self.dep_groups[d]):
                    out[dep_owner(d, self.R)].append((d << 32) | r)
        send = np.array([x for part in out for x in part], np.int64)
        return self._req(_lib.X_ALLTOALLV_U64, send, 6, [len(p) for p in out])

    def _phase6(self):  # owner check; only the unary dependents' pairs go to every rank (R1/R4 probe those)
        allr = np.concatenate([self.recv.astype(np.int64), np.array(self.reports, np.int64)])
        vals, cnt = np.unique(allr, return_counts=True)
        keep = [int(v) for v, c in zip(vals.tolist(), cnt.tolist()) if c == self.nrl[int(v) >> 32]]
        self.own_binary = [k for k in keep if self.freq[k >> 32].v2 is not None]
        unary = [k for k in keep if self.freq[k >> 32].v2 is None]
        return self._req(_lib.X_ALLGATHERV_U64, np.array(unary, np.int64), 7)

    def _phase7(self):  # every rank's unary pairs + this rank's binary pairs: all the rules of owned dependents need
        self.explicit = sorted([int(x) for x in self.recv] + self.own_binary)
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
        owned = {self.freq[d].key() for d in range(len(self.freq)) if dep_owner(d, self.R) == self.rank}
        self.result = [c for c in v if R.Cond(c.dv1, c.dv2, c.dt).key() in owned]
        self.phase = 9
        return _lib.ExchangeRequest(_lib.X_DONE, 8, 0)
