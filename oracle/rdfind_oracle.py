"""ORACLE -- test infrastructure only.  Never imported by the product path.

A pure-Python, literal CPU restatement of RDFind's CIND-discovery hot path
(reference: stratosphere/rdfind @ /root/reference, Scala on Flink 0.9).  It is
used by ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s
``cpu_baseline`` leg as the *checker*; nothing here is ever measured as the
product or shipped.

Abbreviations in citations: ``ALG/`` = ``rdfind-algorithm/src/main/scala/de/hpi/isg/sodap/rdfind/``.

Two independent restatements are provided:

* :func:`all_at_once` -- traversal strategy 0 (``ALG/plan/AllAtOnceTraversalStrategy.scala:33-85``):
  every capture of a capture group is a dependent, its reference candidates are
  all other non-implied captures of the group, and candidate sets are intersected
  per dependent (``IntersectCindCandidates``).
* :func:`small_to_large` -- traversal strategy 1, the default S2L
  (``ALG/plan/SmallToLargeTraversalStrategy.scala:38-634``): 1/1 overlaps,
  Apriori-style 1/2, 2/1, 2/2 candidate generation, candidate filters and exact
  intersection.  Guava Bloom filters are replaced by exact sets; an optional
  deterministic false-positive simulation (``bloom_fpp``) and the reference's
  order-dependent 2/2 prune (``PruneNonMinimalDoubleDoubleCindCandidates.scala:60``,
  only ``buffer(0)`` is checked) are reproduced so tests can show the
  ``--clean-implied`` output does not depend on them.

Finding (checked by ``tests/test_oracle.py``): S2L + ``--clean-implied`` equals
``remove_implied`` applied to the set V of *all* valid CINDs (AllAtOnce with the
semantic triviality test, ``literal_implies=False``) -- independent of candidate
Bloom false positives and of the prune order.  The literal strategy 0 differs:
``Condition.isImpliedBy`` (``ALG/data/Condition.scala:35-43``) compares
``this.v1`` with ``that.v2`` when both are binary captures of the same type, so
``CreateAllCindCandidates`` drops the valid 2/2 refs ``X`` with ``X.v1 == D.v2``.

Parity pinning: the reference cannot be built or run here (no JVM, Flink 0.9,
un-vendored Guava fork).  The only reference tests that pin
this path are ``ConditionCodes$Test`` / ``NullSensitiveOrdered$Test`` (ported in
``tests/test_codes.py``); there are no reference golden CIND vectors.  Beyond
them the oracle is pinned by the cross-check of the two independent
restatements on random inputs and by hand-derived known-answer tests in
``tests/golden`` -- "parity pinned by restatement cross-check, not by reference
runs".

Values are any totally ordered hashables (term ids or strings); ``None`` is the
reference's ``null`` and sorts first (``ALG/util/NullSensitiveOrdered.scala:9-15``).
"""
from __future__ import annotations

import hashlib
import random
from collections import defaultdict
from dataclasses import dataclass

S, P, O = 1, 2, 4
TYPE_MASK = 7


# ---------------------------------------------------------------------------
# ConditionCodes (ALG/util/ConditionCodes.scala:11-130)

def _low(x):
    return x & -x


def prim(code):
    return code & TYPE_MASK


def sec(code):
    return (code >> 3) & TYPE_MASK


def create_code(p1, p2=0, secondary=0):
    return ((p1 | p2) & TYPE_MASK) | ((secondary & TYPE_MASK) << 3)


def add_secondary(code):
    return (code & TYPE_MASK) | ((~code & TYPE_MASK) << 3)


def is_unary(code):
    return bin(code & TYPE_MASK).count("1") == 1


def is_binary(code):
    return bin(code & TYPE_MASK).count("1") == 2


def is_subcode(a, b):
    return (a & b) == a


def first_sub(code):
    return (code & ~TYPE_MASK) | _low(code)


def second_sub(code):
    first = _low(code)
    return (code & ~TYPE_MASK) | _low(code & ~first)


def decode(code):
    first = _low(code)
    second = _low(code & ~first)
    return first, second, ~first & ~second & 7


def _nn(v):
    """conditionValueXNotNull / Funnel's null -> '' coalescing: we normalise '' to None."""
    return None if v == "" else v


# ---------------------------------------------------------------------------
# Records

@dataclass(frozen=True, order=False)
class Cond:
    """``ALG/data/Condition.scala:10`` (v1, v2, type); frozen so it can live in sets."""

    v1: object
    v2: object
    type: int

    def key(self):
        # Condition.compare: type, then v1, then v2, null-first (Condition.scala:55-63)
        return (self.type, (0,) if self.v1 is None else (1, self.v1),
                (0,) if self.v2 is None else (1, self.v2))

    def is_implied_by(self, that: "Cond") -> bool:
        """``Condition.isImpliedBy`` (Condition.scala:35-43)."""
        if self == that:
            return True
        if not is_subcode(self.type, that.type):
            return False
        other = that.v1 if first_sub(that.type) == self.type else that.v2
        return self.v1 == other

    def implies(self, that: "Cond") -> bool:
        return that.is_implied_by(self)


@dataclass(frozen=True)
class Cind:
    """``ALG/data/Cind.scala:12-15``: (dep type, dv1, dv2, ref type, rv1, rv2, support)."""

    dt: int
    dv1: object
    dv2: object
    rt: int
    rv1: object
    rv2: object
    support: int = -1

    def key(self):
        return (self.dt, self.dv1, self.dv2, self.rt, self.rv1, self.rv2)


def norm_cind(dt, dv1, dv2, rt, rv1, rv2, support):
    """Unary captures carry no second value (``Cind`` comment, Cind.scala:7-9)."""
    if is_unary(dt):
        dv2 = None
    if is_unary(rt):
        rv2 = None
    return Cind(dt, _nn(dv1), _nn(dv2), rt, _nn(rv1), _nn(rv2), support)


# ---------------------------------------------------------------------------
# Frequent conditions (ALG/plan/FrequentConditionPlanner.scala)

def frequent_unary_conditions(triples, min_support):
    """``findFrequentSingleConditions`` (FrequentConditionPlanner.scala:291-311 / file lines 488-508).

    Returns {condition type (1,2,4): {value: count}} with count >= min_support.
    Triples are a multiset: duplicates count (RDFind.scala:285-287 without --distinct-triples).
    """
    counts = {S: defaultdict(int), P: defaultdict(int), O: defaultdict(int)}
    for s, p, o in triples:
        counts[S][s] += 1
        counts[P][p] += 1
        counts[O][o] += 1
    return {t: {v: c for v, c in d.items() if c >= min_support} for t, d in counts.items()}


def frequent_binary_conditions(triples, unary_fc, min_support):
    """``CreatedReducedDoubleConditionCounts.flatMap`` (CreatedReducedDoubleConditionCounts.scala:45-86)
    + ``findFrequentDoubleConditions`` (FrequentConditionPlanner.scala:374-394).

    The unary Bloom filters are exact sets here (no false negatives in either).
    Returns {(type, v1, v2): count} for type in {3, 5, 6}.
    """
    counts = defaultdict(int)
    for s0, p0, o0 in triples:
        s = s0 if s0 in unary_fc[S] else None
        p = p0 if p0 in unary_fc[P] else None
        o = o0 if o0 in unary_fc[O] else None
        if (s is not None) + (p is not None) + (o is not None) < 2:
            continue
        if s is not None:
            if p is not None:
                counts[(S | P, s, p)] += 1
            if o is not None:
                counts[(S | O, s, o)] += 1
        if p is not None and o is not None:
            counts[(P | O, p, o)] += 1
    return {k: c for k, c in counts.items() if c >= min_support}


def association_rules(unary_fc, binary_fc):
    """``FrequentConditionPlanner.findAssociationRules`` (FrequentConditionPlanner.scala:130-194, --use-ars):
    a frequent unary condition A and a frequent binary condition {A, B} give the rule A -> B with confidence
    count(A, B) / count(A); only confidence-1 rules are kept (:188-190).  Antecedents on the binary's first
    value give s->p, s->o, p->o (:147-165), on its second value o->s, o->p, p->s (:167-185).

    Returns [(antecedent type, consequent type, antecedent value, consequent value, support)].
    """
    rules = []
    for (t, v1, v2), cb in binary_fc.items():
        t1 = t & -t
        t2 = t & ~t1
        if unary_fc[t1].get(v1) == cb:
            rules.append((t1, t2, v1, v2, cb))
        if unary_fc[t2].get(v2) == cb:
            rules.append((t2, t1, v2, v1, cb))
    return rules


def ar_implied_conditions(rules):
    """``CreateJoinPartners.AssocationRuleBroadcastInitializer`` (CreateJoinPartners.scala:183-196): the binary
    condition of every rule (values ordered by type); its capture equals the antecedent's, so it is not
    emitted as a join partner (:100, :117, :134)."""
    out = set()
    for ta, tc, va, vc, _ in rules:
        out.add((ta | tc, va, vc) if ta < tc else (ta | tc, vc, va))
    return out


def ar_implied_cinds(rules):
    """``FilterAssociationRuleImpliedCinds.AssocationRuleBroadcastInitializer``
    (FilterAssociationRuleImpliedCinds.scala:44-58): rule A -> B at the third position pi gives the 1/1 CIND
    pi[A] < pi[B], which S2L drops before candidate generation (SmallToLargeTraversalStrategy.scala:80-85)."""
    out = set()
    for ta, tc, va, vc, _ in rules:
        cond = ta | tc
        proj = add_secondary(cond) & ~cond
        out.add((ta | proj, va, tc | proj, vc))
    return out


def format_rules(rules, term=lambda v: v):
    """``AssociationRule.toString`` (ALG/data/AssociationRule.scala:15-19), sorted: the --ar-output lines."""
    chars = {S: "s", P: "p", O: "o"}
    return sorted(f"[{chars[ta]}={term(va)}] -> [{chars[tc]}={term(vc)}] (support={n},confidence=100.00%)"
                  for ta, tc, va, vc, n in rules)


# ---------------------------------------------------------------------------
# Join lines (capture groups)

def create_join_partners(triple, unary_fc, binary_fc, projection="spo", use_fis=True, ar_implied=frozenset()):
    """``CreateJoinPartners.flatMap`` (ALG/operators/CreateJoinPartners.scala:86-147).

    Yields (join value, Cond).  With ``use_fis`` the unary/binary FC Bloom filters
    are the exact frequent sets; without it every value passes and every binary
    capture is emitted (``mightBeFrequent`` is true when the filter is off, :78).
    """
    ts, tp, to = triple
    if use_fis:
        s = ts if ts in unary_fc[S] else None
        p = tp if tp in unary_fc[P] else None
        o = to if to in unary_fc[O] else None

        def freq2(v1, v2, t):  # mightBeFrequent && !isAssociationRuleImplied (CreateJoinPartners.scala:100)
            return (t, v1, v2) in binary_fc and (t, v1, v2) not in ar_implied
    else:
        s, p, o = ts, tp, to

        def freq2(v1, v2, t):
            return True
    out = []
    if "o" in projection:
        if s is not None:
            if p is not None and freq2(s, p, S | P):
                out.append((to, Cond(s, p, add_secondary(S | P))))
            elif p is not None:
                out.append((to, Cond(p, None, create_code(P, secondary=O))))
            out.append((to, Cond(s, None, create_code(S, secondary=O))))
        elif p is not None:
            out.append((to, Cond(p, None, create_code(P, secondary=O))))
    if "p" in projection:
        if s is not None:
            if o is not None and freq2(s, o, S | O):
                out.append((tp, Cond(s, o, add_secondary(S | O))))
            elif o is not None:
                out.append((tp, Cond(o, None, create_code(O, secondary=P))))
            out.append((tp, Cond(s, None, create_code(S, secondary=P))))
        elif o is not None:
            out.append((tp, Cond(o, None, create_code(O, secondary=P))))
    if "s" in projection:
        if p is not None:
            if o is not None and freq2(p, o, P | O):
                out.append((ts, Cond(p, o, add_secondary(P | O))))
            elif o is not None:
                out.append((ts, Cond(o, None, create_code(O, secondary=S))))
            out.append((ts, Cond(p, None, create_code(P, secondary=S))))
        elif o is not None:
            out.append((ts, Cond(o, None, create_code(O, secondary=S))))
    return out


def join_lines(triples, unary_fc, binary_fc, projection="spo", use_fis=True, ar_implied=frozenset()):
    """``UnionJoinCandidates`` + ``UnionCombinedJoinCandidates`` (UnionJoinCandidates.scala:27-44,
    UnionCombinedJoinCandidates.scala:21-31): group by join value, distinct conditions.

    Returns {join value: frozenset(Cond)}.
    """
    groups = defaultdict(set)
    for t in triples:
        for jv, cond in create_join_partners(t, unary_fc, binary_fc, projection, use_fis, ar_implied):
            groups[jv].add(cond)
    return {jv: frozenset(c) for jv, c in groups.items()}


def split_binary(cond: Cond):
    """``CreateDependencyCandidates.splitAndCollectUnaryCaptures`` (e.g. ExtractUnaryBinaryCindCandidates.scala:59-65)."""
    c1, c2, free = decode(cond.type)
    return (Cond(cond.v1, None, create_code(c1, secondary=free)),
            Cond(cond.v2, None, create_code(c2, secondary=free)))


def line_captures(line):
    """``CreateDependencyCandidates.flatMap`` gathering (CreateDependencyCandidates.scala:90-105):
    unary captures (direct + split binaries) and binary captures."""
    unary, binary = set(), set()
    for c in line:
        if is_binary(c.type):
            binary.add(c)
            unary.update(split_binary(c))
        else:
            unary.add(c)
    return unary, binary


# ---------------------------------------------------------------------------
# Intersection of CindSets (IntersectCindCandidates.scala:14-51 + BulkMergeDependencies.scala:48-152)

class _Intersector:
    """Per dependent: intersect ref sets over all its evidences, sum depCount."""

    def __init__(self):
        self.refs = {}
        self.count = defaultdict(int)

    def add(self, dep, refs):
        self.count[dep] += 1
        if dep in self.refs:
            self.refs[dep] &= refs
        else:
            self.refs[dep] = set(refs)

    def results(self):
        for dep, refs in self.refs.items():
            yield dep, self.count[dep], refs


def _split(dep: Cond, count, refs):
    """``CindSet.split`` / ``splitAndCleanCindSets`` (TraversalStrategy.scala:49-59)."""
    return [norm_cind(dep.type, dep.v1, dep.v2, r.type, r.v1, r.v2, count) for r in refs]


# ---------------------------------------------------------------------------
# Minimality (TraversalStrategy.removeImpliedCinds, TraversalStrategy.scala:126-168)

def _comp_values(c_type, v1, v2):
    """(first subcapture code, v1), (second subcapture code, v2) of a binary capture."""
    return ((first_sub(c_type), v1), (second_sub(c_type), v2))


def remove_implied(v11, v12, v21, v22):
    """R1-R4 of ``removeImpliedCinds``; each rule is evaluated on the raw input sets.

    R1 RemoveNonMinimalDoubleXxxCinds (2/1 vs 1/1 on ref, RemoveNonMinimalDoubleXxxCinds.scala:19-40)
    R2 RemoveNonMinimalXxxSingleCinds (2/1 vs 2/2 on dep, RemoveNonMinimalXxxSingleCinds.scala:19-41)
    R3 RemoveNonMinimalXxxSingleCinds (1/1 vs 1/2 on dep)
    R4 RemoveNonMinimalDoubleXxxCinds (2/2 vs 1/2 on ref)
    V12 is kept whole.
    """
    # R1: probing table per ref: {dep capture (type, v1)} of 1/1 CINDs
    deps_by_ref11 = defaultdict(set)
    for c in v11:
        deps_by_ref11[(c.rt, c.rv1)].add((c.dt, c.dv1))
    after_r1 = []
    for c in v21:
        table = deps_by_ref11.get((c.rt, c.rv1), set())
        (t1, a), (t2, b) = _comp_values(c.dt, c.dv1, c.dv2)
        if (t1, a) in table or (t2, b) in table:
            continue
        after_r1.append(c)
    # R2: probing table per dep: components of refs of 2/2 CINDs
    comps_by_dep22 = defaultdict(set)
    for c in v22:
        for comp in _comp_values(c.rt, c.rv1, c.rv2):
            comps_by_dep22[(c.dt, c.dv1, c.dv2)].add(comp)
    min21 = [c for c in after_r1 if (c.rt, c.rv1) not in comps_by_dep22.get((c.dt, c.dv1, c.dv2), set())]
    # R3: probing table per dep (unary): components of refs of 1/2 CINDs
    comps_by_dep12 = defaultdict(set)
    for c in v12:
        for comp in _comp_values(c.rt, c.rv1, c.rv2):
            comps_by_dep12[(c.dt, c.dv1)].add(comp)
    min11 = [c for c in v11 if (c.rt, c.rv1) not in comps_by_dep12.get((c.dt, c.dv1), set())]
    # R4: probing table per ref (binary): deps of 1/2 CINDs
    deps_by_ref12 = defaultdict(set)
    for c in v12:
        deps_by_ref12[(c.rt, c.rv1, c.rv2)].add((c.dt, c.dv1))
    min22 = []
    for c in v22:
        table = deps_by_ref12.get((c.rt, c.rv1, c.rv2), set())
        (t1, a), (t2, b) = _comp_values(c.dt, c.dv1, c.dv2)
        if (t1, a) in table or (t2, b) in table:
            continue
        min22.append(c)
    return min11 + list(v12) + min21 + min22


def split_by_arity(cinds):
    v11, v12, v21, v22 = [], [], [], []
    for c in cinds:
        if is_unary(c.dt):
            (v11 if is_unary(c.rt) else v12).append(c)
        else:
            (v21 if is_unary(c.rt) else v22).append(c)
    return v11, v12, v21, v22


# ---------------------------------------------------------------------------
# Traversal strategy 0: AllAtOnce

def trivially_implied(dep: Cond, ref: Cond) -> bool:
    """Semantic triviality: ``ref`` is ``dep`` itself or a unary sub-capture of binary ``dep`` with
    the same value (what S2L excludes: ``dep != ref`` in ExtractBinaryBinaryCindCandidates.scala:67,
    ``!binaryCapture.implies(unaryCapture)`` in CreateBinaryUnaryCindCandidates.scala:76)."""
    if dep == ref:
        return True
    if is_binary(dep.type) and is_unary(ref.type) and is_subcode(ref.type, dep.type):
        return ref.v1 == (dep.v1 if first_sub(dep.type) == ref.type else dep.v2)
    return False


def all_at_once(lines, min_support, clean_implied=True, literal_implies=True, ar_cinds=frozenset()):
    """``AllAtOnceTraversalStrategy.enhanceFlinkPlan`` (AllAtOnceTraversalStrategy.scala:42-84) with
    ``CreateAllCindCandidates`` (CreateAllCindCandidates.scala:71-121).

    ``literal_implies=True`` reproduces the reference's ``!dep.implies(ref)`` filter (:113), whose
    ``Condition.isImpliedBy`` (Condition.scala:35-43) also drops a *binary* ref ``X`` of the same type
    as a binary dep ``D`` whenever ``X.v1 == D.v2`` (it compares ``this.v1`` with ``that.v2``).
    ``literal_implies=False`` uses :func:`trivially_implied` instead: the set of all valid CINDs.
    With --use-ars a unary dep also skips the ref its association rule implies (``findImpliedCondition``,
    CreateDependencyCandidates.scala:125-129, used at CreateAllCindCandidates.scala:108-115): ``ar_cinds``.
    """
    inter = _Intersector()
    excluded = (lambda d, r: d.implies(r)) if literal_implies else trivially_implied
    for line in lines.values():
        unary, binary = line_captures(line)
        allc = unary | binary
        for dep in allc:
            refs = {r for r in allc if not excluded(dep, r)
                    and (dep.type, dep.v1, r.type, r.v1) not in ar_cinds}
            inter.add(dep, refs)
    cinds = []
    for dep, count, refs in inter.results():
        if count >= min_support:
            cinds.extend(_split(dep, count, refs))
    if not clean_implied:
        return cinds
    return remove_implied(*split_by_arity(cinds))


# ---------------------------------------------------------------------------
# Traversal strategy 1: SmallToLarge (S2L)

class _CandidateFilter:
    """Exact replacement of the candidate Bloom filters, with an optional deterministic
    false-positive simulation (any non-member passes with probability ``fpp``)."""

    def __init__(self, members, fpp=0.0, salt=""):
        self.members = set(members)
        self.fpp = fpp
        self.salt = salt

    def might_contain(self, key):
        if key in self.members:
            return True
        if self.fpp <= 0:
            return False
        h = hashlib.blake2b(repr((self.salt, key)).encode(), digest_size=8).digest()
        return int.from_bytes(h, "little") / 2 ** 64 < self.fpp


def _ckey(dt, dv1, dv2, rt, rv1, rv2):
    """``Cind.Funnel`` key (Cind.scala:34-41): null values coalesce with ''."""
    return (dt, _nn(dv1), _nn(dv2), rt, _nn(rv1), _nn(rv2))


def small_to_large(lines, binary_fc, min_support, clean_implied=True, bloom_fpp=0.0, prune_seed=None,
                   full_prune=False, ar_cinds=frozenset()):
    """``SmallToLargeTraversalStrategy.enhanceFlinkPlan`` (SmallToLargeTraversalStrategy.scala:38-171).

    ``binary_fc`` = frequent double conditions {(type, v1, v2): count} (needed by the 2/2 phase,
    :534-548).  ``prune_seed`` shuffles the co-grouped 1/2 CINDs before the buggy prune to mimic
    Flink's unspecified order; ``full_prune`` checks every co-grouped 1/2 CIND instead (the evident intent
    of the operator, making the raw output deterministic).
    """
    ms = min_support
    # -- 1/1 overlaps: CreateUnaryUnaryOverlapCandidates (CreateUnaryUnaryOverlapCandidates.scala:44-74)
    #    + MultiunionOverlapCandidates (MultiunionOverlapCandidates.scala:17-48)
    lhs_count = defaultdict(int)
    overlap = defaultdict(int)
    for line in lines.values():
        unary, _ = line_captures(line)
        ordered = sorted(unary, key=Cond.key)
        for i, lhs in enumerate(ordered):
            lhs_count[lhs] += 1
            for rhs in ordered[i + 1:]:
                overlap[(lhs, rhs)] += 1
    # filter lhsCount >= ms and rhs.count >= ms (:300-305); join distinct values (:334-363)
    distinct = {c: n for c, n in lhs_count.items() if n >= ms}
    pairwise = []
    for (a, b), n in overlap.items():
        if a in distinct and n >= ms and b in distinct:
            pairwise.append((a, distinct[a], b, distinct[b], n))
    v11, proper = [], []
    for a, na, b, nb, n in pairwise:  # :63-105
        (v11 if na == n else proper).append(norm_cind(a.type, a.v1, None, b.type, b.v1, None, n))
        (v11 if nb == n else proper).append(norm_cind(b.type, b.v1, None, a.type, a.v1, None, n))
    if ar_cinds:  # --use-ars: FilterAssociationRuleImpliedCinds on the 1/1 CINDs (:80-85)
        v11 = [c for c in v11 if (c.dt, c.dv1, c.rt, c.rv1) not in ar_cinds]

    # -- 1/2: GenerateUnaryBinaryCindCandidates (GenerateXxxBinaryCindCandidates.scala:26-65,
    #    GenerateUnaryBinaryCindCandidates.scala:16-41)
    by_dep = defaultdict(list)
    for c in v11:
        by_dep[(c.dt, c.dv1)].append(c)
    cand12 = set()
    for group in by_dep.values():
        _gen_xxx_binary(group, cand12)
        for c in group:  # refined: s[p1] < s[o1] -> s[p1] < s[p1,o1]
            pd, pr = prim(c.dt), prim(c.rt)
            if pd != pr and sec(c.dt) == sec(c.rt):
                rt = c.rt | c.dt
                rv = (c.dv1, c.rv1) if pd < pr else (c.rv1, c.dv1)
                cand12.add(_ckey(c.dt, c.dv1, c.dv2, rt, rv[0], rv[1]))
    filt12 = _CandidateFilter(cand12, bloom_fpp, "12")
    inter = _Intersector()
    for line in lines.values():  # ExtractUnaryBinaryCindCandidates.scala:67-83
        unary, binary = line_captures(line)
        for u in unary:
            refs = {b for b in binary if filt12.might_contain(_ckey(u.type, u.v1, u.v2, b.type, b.v1, b.v2))}
            inter.add(u, refs)
    v12 = []
    for dep, count, refs in inter.results():  # :412-422
        if refs and count >= ms:
            v12.extend(_split(dep, count, refs))

    # -- 2/1: GenerateBinaryUnaryCindCandidates over proper overlaps grouped by ref
    #    (GenerateBinaryUnaryCindCandidates.scala:23-57)
    by_ref = defaultdict(list)
    for c in proper:
        by_ref[(c.rt, c.rv1)].append(c)
    cand21 = set()
    for group in by_ref.values():
        if len(group) > 1:
            g = sorted(group, key=lambda c: c.dt)
            for i in range(len(g) - 1):
                for j in range(i + 1, len(g)):
                    o1, o2 = g[i], g[j]
                    if sec(o1.dt) == sec(o2.dt) and prim(o1.dt) != prim(o2.dt):
                        cand21.add(_ckey(o1.dt | o2.dt, o1.dv1, o2.dv1, o1.rt, o1.rv1, o1.rv2))
    filt21 = _CandidateFilter(cand21, bloom_fpp, "21")
    inter = _Intersector()
    for line in lines.values():  # CreateBinaryUnaryCindCandidates.scala:70-87
        unary, binary = line_captures(line)
        for b in binary:
            refs = {u for u in unary
                    if not b.implies(u) and filt21.might_contain(_ckey(b.type, b.v1, b.v2, u.type, u.v1, u.v2))}
            inter.add(b, refs)
    v21 = []
    for dep, count, refs in inter.results():  # :479-489
        if count >= ms and refs:
            v21.extend(_split(dep, count, refs))

    # -- 2/2 (findDoubleDoubleCindSets, :497-634)
    inferred = _infer_double_single(v11, proper)  # InferDoubleSingleCinds.scala:26-54
    freq_caps = {(add_secondary(t), a, b) for (t, a, b) in binary_fc}
    inferred = [c for c in inferred if (c.dt, c.dv1, c.dv2) in freq_caps]  # :534-548
    all21 = v21 + inferred
    by_dep2 = defaultdict(list)
    for c in all21:
        by_dep2[(c.dt, c.dv1, c.dv2)].append(c)
    cand22 = []
    for group in by_dep2.values():  # GenerateBinaryBinaryCindCandidates.scala:20-42
        out = set()
        _gen_xxx_binary(group, out)
        for c in group:
            if is_subcode(c.rt, c.dt):
                if first_sub(c.dt) == c.rt:
                    rv = (c.rv1, c.dv2)
                else:
                    rv = (c.dv1, c.rv1)
                out.add(_ckey(c.dt, c.dv1, c.dv2, c.dt, rv[0], rv[1]))
        cand22.extend(out)
    # PruneNonMinimalDoubleDoubleCindCandidates (:40-66): only the first co-grouped 1/2 CIND is checked.
    v12_by_ref = defaultdict(list)
    for c in v12:
        v12_by_ref[(c.rt, c.rv1, c.rv2)].append(c)
    rng = random.Random(prune_seed) if prune_seed is not None else None
    pruned22 = []
    for cand in cand22:
        dt, dv1, dv2, rt, rv1, rv2 = cand
        buf = list(v12_by_ref.get((rt, rv1, rv2), []))
        if not buf:
            pruned22.append(cand)
            continue
        if rng is not None:
            rng.shuffle(buf)
        minimal = True
        for first in (buf if full_prune else buf[:1]):
            if is_subcode(first.dt, dt):
                c1, _, _ = decode(dt)
                if is_subcode(c1, first.dt):
                    minimal = dv1 != first.dv1
                else:
                    minimal = dv2 != first.dv1
            if not minimal:
                break
        if minimal:
            pruned22.append(cand)
    filt22 = _CandidateFilter(pruned22, bloom_fpp, "22")
    inter = _Intersector()
    for line in lines.values():  # ExtractBinaryBinaryCindCandidates.scala:60-78
        _, binary = line_captures(line)
        for d in binary:
            refs = {r for r in binary
                    if d != r and filt22.might_contain(_ckey(d.type, d.v1, d.v2, r.type, r.v1, r.v2))}
            inter.add(d, refs)
    v22 = []
    for dep, count, refs in inter.results():  # :616-626
        if count >= ms and refs:
            v22.extend(_split(dep, count, refs))

    if clean_implied:
        return remove_implied(v11, v12, v21, v22)
    return v11 + v12 + v21 + v22


def s2l_ars_closed_form(v, ar_cinds, clean_implied=True):
    """S2L's result under --use-ars as a closed form over V (all valid CINDs of the AR-suppressed join lines),
    derived from ``small_to_large`` above and cross-checked against it (tests/test_oracle.py):

    * V11' = V11 minus the AR-implied 1/1 CINDs (FilterAssociationRuleImpliedCinds, :80-85);
    * V12' = A < X in V12 such that every component Xk != A has A < Xk in V11' (1/2 candidates are generated
      from pairs of V11' refs, or one V11' ref and A itself, GenerateUnaryBinaryCindCandidates.scala:16-41);
    * V21s = D < R in V21 with no component c of D such that c < R in V11 (candidates: pairs of proper
      overlaps, GenerateBinaryUnaryCindCandidates.scala:23-57);
    * V22' = D < Y in V22 such that every component Yk of Y that is not a component of D has D < Yk in all21,
      all21(D, R) = no component c of D with c < R in V11 and AR-implied (all21 = V21s plus the 2/1 CINDs
      InferDoubleSingleCinds derives from V11' and proper overlaps, SmallToLargeTraversalStrategy.scala:497-562);
    * --clean-implied: R1-R4 on (V11', V12', V21s, V22'); raw: V22' minus R4 (the full prune).
    """
    v11, v12, v21, v22 = split_by_arity(v)
    s11 = {(c.dt, c.dv1, c.rt, c.rv1) for c in v11}
    bad = ar_cinds & s11
    v11p = [c for c in v11 if (c.dt, c.dv1, c.rt, c.rv1) not in bad]
    v12p = []
    for c in v12:
        ok = True
        for (t, val) in _comp_values(c.rt, c.rv1, c.rv2):
            if (t, val) != (c.dt, c.dv1) and (c.dt, c.dv1, t, val) in bad:
                ok = False
        if ok:
            v12p.append(c)
    v21s = [c for c in v21 if not any((t, val, c.rt, c.rv1) in s11 for (t, val) in _comp_values(c.dt, c.dv1, c.dv2))]

    def all21(dt, dv1, dv2, rt, rv1):
        return not any((t, val, rt, rv1) in bad for (t, val) in _comp_values(dt, dv1, dv2))

    v22p = []
    for c in v22:
        dcomps = set(_comp_values(c.dt, c.dv1, c.dv2))
        if all(all21(c.dt, c.dv1, c.dv2, t, val) for (t, val) in _comp_values(c.rt, c.rv1, c.rv2) if (t, val) not in dcomps):
            v22p.append(c)
    if clean_implied:
        return remove_implied(v11p, v12p, v21s, v22p)
    deps_by_ref12 = defaultdict(set)
    for c in v12p:
        deps_by_ref12[(c.rt, c.rv1, c.rv2)].add((c.dt, c.dv1))
    v22r = [c for c in v22p if not any(comp in deps_by_ref12.get((c.rt, c.rv1, c.rv2), set())
                                       for comp in _comp_values(c.dt, c.dv1, c.dv2))]
    return v11p + v12p + v21s + v22r


def _gen_xxx_binary(group, out):
    """``GenerateXxxBinaryCindCandidates.reduce`` pair loop (GenerateXxxBinaryCindCandidates.scala:26-58)."""
    if len(group) <= 1:
        return
    g = sorted(group, key=lambda c: c.rt)  # stable, like Scala's sortBy
    for i in range(len(g) - 1):
        for j in range(i + 1, len(g)):
            o1, o2 = g[i], g[j]
            if sec(o1.rt) == sec(o2.rt) and prim(o1.rt) != prim(o2.rt):
                out.add(_ckey(o1.dt, o1.dv1, o1.dv2, o1.rt | o2.rt, o1.rv1, o2.rv1))


def _infer_double_single(v11, proper):
    """``InferDoubleSingleCinds.reduce`` (InferDoubleSingleCinds.scala:26-54): grouped by ref; pairs
    where at least one is a 1/1 CIND (support marker 0) with same projection, disjoint conditions."""
    by_ref = defaultdict(list)
    for c in v11:
        by_ref[(c.rt, c.rv1)].append((c, True))
    for c in proper:
        by_ref[(c.rt, c.rv1)].append((c, False))
    out = []
    for group in by_ref.values():
        if len(group) < 2:
            continue
        g = sorted(group, key=lambda x: x[0].dt)
        for i in range(len(g) - 1):
            d1, is1 = g[i]
            for j in range(i + 1, len(g)):
                d2, is2 = g[j]
                if (is1 or is2) and sec(d1.dt) == sec(d2.dt) and (prim(d1.dt) & prim(d2.dt)) == 0:
                    out.append(norm_cind(d1.dt | d2.dt, d1.dv1, d2.dv1, d1.rt, d1.rv1, None, -1))
    return out


# ---------------------------------------------------------------------------
# Whole program (RDFind.createFlinkPlan, ALG/programs/RDFind.scala:196-580, hot-path portion)

def rdfind(triples, min_support=10, traversal_strategy=1, clean_implied=True, use_fis=True,
           projection="spo", bloom_fpp=0.0, prune_seed=None, distinct_triples=False, full_prune=False,
           use_ars=False):
    """Run the reference plan on in-memory triples; returns a list of :class:`Cind`."""
    triples = list(triples)
    if distinct_triples:
        triples = list(dict.fromkeys(triples))
    if traversal_strategy == 1 and not use_fis:
        # frequentDoubleConditions is null without --use-fis (RDFind.scala:290-296) -> NPE at
        # SmallToLargeTraversalStrategy.scala:534 in the reference.
        raise ValueError("S2L traversal requires --use-fis")
    unary_fc = frequent_unary_conditions(triples, min_support)
    binary_fc = frequent_binary_conditions(triples, unary_fc, min_support)
    rules = association_rules(unary_fc, binary_fc) if use_ars else []  # needs --use-fis in the reference
    lines = join_lines(triples, unary_fc, binary_fc, projection, use_fis, ar_implied_conditions(rules))
    if traversal_strategy == 0:
        return all_at_once(lines, min_support, clean_implied, ar_cinds=ar_implied_cinds(rules))
    if traversal_strategy == 1:
        return small_to_large(lines, binary_fc, min_support, clean_implied, bloom_fpp, prune_seed, full_prune,
                              ar_implied_cinds(rules))
    raise ValueError(f"unsupported traversal strategy {traversal_strategy}")


def format_cinds(cinds, term=lambda v: v):
    """Sorted ``Cind.toString`` lines (Cind.scala:29-31 + ConditionCodes.prettyPrint :102-107)."""
    chars = {S: "s", P: "p", O: "o"}

    def pp(code, v1, v2):
        proj = chars.get(sec(code), "")
        c1, c2, _ = decode(prim(code))
        if c2 == 0:
            return f"{proj}[{chars[c1]}={term(v1)}]"
        return f"{proj}[{chars[c1]}={term(v1)},{chars[c2]}={term(v2)}]"

    return sorted(f"{pp(c.dt, c.dv1, c.dv2)} < {pp(c.rt, c.rv1, c.rv2)} (support={c.support})" for c in cinds)


def cind_set(cinds):
    """Comparable set of (dt, dv1, dv2, rt, rv1, rv2, support)."""
    return {(c.dt, c.dv1, c.dv2, c.rt, c.rv1, c.rv2, c.support) for c in cinds}


def s2l_exact_raw(cinds_v):
    """Raw (no --clean-implied) S2L output with exact candidate sets and the full 2/2 prune:
    V11 + V12 + (V21 minus R1) + (V22 minus R4), computed from the set V of all valid CINDs."""
    v11, v12, v21, v22 = split_by_arity(cinds_v)
    deps_by_ref11 = defaultdict(set)
    for c in v11:
        deps_by_ref11[(c.rt, c.rv1)].add((c.dt, c.dv1))
    deps_by_ref12 = defaultdict(set)
    for c in v12:
        deps_by_ref12[(c.rt, c.rv1, c.rv2)].add((c.dt, c.dv1))
    out = list(v11) + list(v12)
    for c in v21:
        t = deps_by_ref11.get((c.rt, c.rv1), set())
        (t1, a), (t2, b) = _comp_values(c.dt, c.dv1, c.dv2)
        if (t1, a) not in t and (t2, b) not in t:
            out.append(c)
    for c in v22:
        t = deps_by_ref12.get((c.rt, c.rv1, c.rv2), set())
        (t1, a), (t2, b) = _comp_values(c.dt, c.dv1, c.dv2)
        if (t1, a) not in t and (t2, b) not in t:
            out.append(c)
    return out


# ------------------------------------------------------------------------------------------------
# Input-side options

def distinct_triples(s, p, o):
    """``triples.distinct`` (ALG/programs/RDFind.scala:284-287): every triple once.  Flink's distinct
    defines a set; this checker keeps first occurrences in input order (the GPU path's documented order)."""
    import numpy as np
    seen = set()
    keep = []
    for i, t in enumerate(zip(s.tolist(), p.tolist(), o.tolist())):
        if t not in seen:
            seen.add(t)
            keep.append(i)
    idx = np.array(keep, dtype=np.int64)
    return s[idx], p[idx], o[idx]


def parse_prefix_line(line):
    """ParseRdfPrefixes.map (ALG/operators/ParseRdfPrefixes.scala:14-26): ``@prefix p: <url> .`` or
    ``@prefix <url> .`` (prefix ""); anything else raises."""
    import re
    m = re.fullmatch(r"@prefix\s+(\S+): <(\S+)>\s*\.\n?", line)
    if m:
        return m.group(1), m.group(2)
    m = re.fullmatch(r"@prefix\s+<(\S+)>\s*\.\n?", line)
    if m:
        return "", m.group(1)
    raise ValueError(f"Could not parse the line {line!r} correctly.")


def shorten_term(term, prefixes):
    """ShortenUrls.shorten (ALG/operators/ShortenUrls.scala:36-44) with the trie of PrefixTrieCreator
    (:55-60): key ``<url``, value ``prefix:``; the LONGEST key that is a prefix of the term wins
    (StringTrie.getKeyAndValue, ALG/util/StringTrie.scala:44-54), by a linear scan here."""
    if not term.endswith(">"):
        return term
    best = None
    for prefix, url in prefixes:
        key = "<" + url
        if term.startswith(key) and (best is None or len(key) > len(best[0])):
            best = (key, prefix + ":")
    if best is None:
        return term
    return best[1] + term[len(best[0]):len(term) - 1]
