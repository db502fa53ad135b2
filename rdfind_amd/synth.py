"""Seeded synthetic RDF generators for the BASELINE.json configurations.

Every generator returns a :class:`Dataset`: dictionary-encoded ``uint32`` columns ``s, p, o``
(one id space shared by all positions, as the reference's join values cross positions,
SURVEY.md Appendix B.3) plus a :class:`TermTable` that maps ids back to N-Triples terms.

* ``zipf_rdf``  -- Zipf-distributed entity/predicate/class/literal graph (c1, c3, c4, c5 shapes).
* ``zipf_rows`` -- the same distributions from a counter-based generator (rdfind_amd/csrc/synth_gen.c): row i
                   depends only on (seed, i), so any row range is drawn on its own (c4 beyond scale 0.05).
* ``lubm``      -- LUBM-schema generator (universities -> departments -> faculty, students,
                   courses, publications; ~18 predicates), the c2 shape.  The official Java UBA
                   is unavailable offline; this follows its published cardinalities.
"""
from __future__ import annotations

import ctypes
import os
from dataclasses import dataclass, field

import numpy as np

RDF_TYPE = "<http://www.w3.org/1999/02/22-rdf-syntax-ns#type>"


@dataclass
class TermTable:
    """id -> term string by contiguous ranges: (start, count, formatter(local_index) -> str)."""

    ranges: list = field(default_factory=list)
    size: int = 0

    def add(self, count: int, fmt) -> int:
        start = self.size
        self.ranges.append((start, count, fmt))
        self.size += count
        return start

    def term(self, tid: int) -> str:
        lo, hi = 0, len(self.ranges)
        while lo < hi:
            mid = (lo + hi) // 2
            if self.ranges[mid][0] <= tid:
                lo = mid + 1
            else:
                hi = mid
        start, count, fmt = self.ranges[lo - 1]
        if not (start <= tid < start + count):
            raise KeyError(tid)
        return fmt(tid - start)


@dataclass
class Dataset:
    name: str
    s: np.ndarray
    p: np.ndarray
    o: np.ndarray
    terms: TermTable
    min_support: int

    @property
    def n(self) -> int:
        return int(self.s.shape[0])

    @property
    def num_terms(self) -> int:
        return self.terms.size

    def lines(self):
        """N-Triples lines (for small datasets / fixtures)."""
        t = self.terms.term
        for a, b, c in zip(self.s.tolist(), self.p.tolist(), self.o.tolist()):
            yield f"{t(a)} {t(b)} {t(c)} ."


def _zipf_ranks(rng: np.random.Generator, n_items: int, alpha: float, size: int) -> np.ndarray:
    """Rank in [0, n_items) with P(rank=k) ~ (k+1)^-alpha (continuous inverse-CDF approximation)."""
    u = rng.random(size)
    if abs(alpha - 1.0) < 1e-9:
        x = np.power(float(n_items + 1), u)
    else:
        a = 1.0 - alpha
        x = np.power((np.power(n_items + 1.0, a) - 1.0) * u + 1.0, 1.0 / a)
    r = np.floor(x).astype(np.int64) - 1
    return np.clip(r, 0, n_items - 1)


def _dedup(s, p, o):
    """Distinct triples in lexicographic (s, p, o) order (== np.unique(axis=0), ~4x faster): one sort of
    (s << 32 | p), then one of (rank of the (s, p) run << 32 | o)."""
    n = s.shape[0]
    if n == 0:
        return s.copy(), p.copy(), o.copy()
    k = (s.astype(np.uint64) << np.uint64(32)) | p.astype(np.uint64)
    i1 = np.argsort(k)
    ks = k[i1]
    del k
    run = np.empty(n, np.uint64)
    run[0] = 0
    np.cumsum(ks[1:] != ks[:-1], out=run[1:])
    del ks
    k2 = (run << np.uint64(32)) | o[i1].astype(np.uint64)
    del run
    i2 = np.argsort(k2)
    order = i1[i2]
    k2s = k2[i2]
    del k2, i1, i2
    keep = np.ones(n, bool)
    keep[1:] = k2s[1:] != k2s[:-1]
    order = order[keep]
    return s[order], p[order], o[order]


def zipf_rdf(name: str, n: int, n_entities: int, n_predicates: int, pred_alpha: float,
             subj_alpha: float, class_frac: float, n_classes: int, class_alpha: float,
             literal_frac: float, n_literals: int, lit_alpha: float, obj_alpha: float,
             min_support: int, seed: int, dedup: bool = True) -> Dataset:
    rng = np.random.default_rng(seed)
    terms = TermTable()
    t_type = terms.add(1, lambda i: RDF_TYPE)
    t_pred = terms.add(n_predicates, lambda i: f"<http://ex.org/p{i}>")
    t_cls = terms.add(n_classes, lambda i: f"<http://ex.org/C{i}>")
    t_ent = terms.add(n_entities, lambda i: f"<http://ex.org/e{i}>")
    t_lit = terms.add(n_literals, lambda i: f'"l{i}"')
    def draw(m):
        s = t_ent + _zipf_ranks(rng, n_entities, subj_alpha, m)
        kind = rng.random(m)
        is_cls = kind < class_frac
        is_lit = (kind >= class_frac) & (kind < class_frac + literal_frac)
        p = t_pred + _zipf_ranks(rng, n_predicates, pred_alpha, m)
        p = np.where(is_cls, t_type, p)
        o_ent = t_ent + _zipf_ranks(rng, n_entities, obj_alpha, m)
        o_cls = t_cls + _zipf_ranks(rng, n_classes, class_alpha, m)
        o_lit = t_lit + _zipf_ranks(rng, n_literals, lit_alpha, m)
        o = np.where(is_cls, o_cls, np.where(is_lit, o_lit, o_ent))
        return s.astype(np.uint32), p.astype(np.uint32), o.astype(np.uint32)

    # oversample a little so that deduplication lands near n; draw more until n distinct triples exist
    m = int(n * 1.08) if dedup else n
    s, p, o = draw(m)
    if dedup:
        s, p, o = _dedup(s, p, o)
        for _ in range(16):
            got = s.shape[0]
            if got >= n or got == 0:
                break
            extra = draw(int((n - got) * (m / got) * 1.25) + 1024)  # distinct yield of the draws so far
            m += extra[0].shape[0]
            s, p, o = _dedup(np.concatenate([s, extra[0]]), np.concatenate([p, extra[1]]),
                             np.concatenate([o, extra[2]]))
            del extra
        if s.shape[0] > n:
            idx = np.sort(rng.choice(s.shape[0], n, replace=False))
            s, p, o = s[idx], p[idx], o[idx]
    return Dataset(name, s, p, o, terms, min_support)


class _SynthParams(ctypes.Structure):
    _fields_ = [("seed", ctypes.c_uint64)] + [(k, ctypes.c_uint32) for k in (
        "t_type", "t_pred", "t_cls", "t_ent", "t_lit", "n_pred", "n_cls", "n_ent", "n_lit")] + [
        (k, ctypes.c_double) for k in ("pred_alpha", "subj_alpha", "class_frac", "class_alpha", "literal_frac",
                                       "lit_alpha", "obj_alpha")]


_SYNTH_LIB = None


def _synth_lib():
    global _SYNTH_LIB
    if _SYNTH_LIB is None:
        path = os.path.join(os.path.dirname(os.path.abspath(__file__)), "libsynth.so")
        if not os.path.exists(path):
            raise RuntimeError(f"{path} not built; run __graft_entry__.build()")
        lib = ctypes.CDLL(path)
        lib.synth_zipf_rows.restype = None
        lib.synth_zipf_rows.argtypes = [ctypes.POINTER(_SynthParams), ctypes.c_uint64, ctypes.c_uint64,
                                        ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]
        _SYNTH_LIB = lib
    return _SYNTH_LIB


def zipf_rows(name: str, n: int, row0: int, nrows: int, n_entities: int, n_predicates: int, pred_alpha: float,
              subj_alpha: float, class_frac: float, n_classes: int, class_alpha: float, literal_frac: float,
              n_literals: int, lit_alpha: float, obj_alpha: float, min_support: int, seed: int) -> Dataset:
    """Rows [row0, row0 + nrows) of an n-row i.i.d. Zipf configuration (no deduplication), drawn by the
    counter-based generator: the same term table and distributions as :func:`zipf_rdf`, and any row range is
    generated independently of the others (sharded inputs: the ranks' slices always form the same input)."""
    terms = TermTable()
    q = _SynthParams(seed=seed)
    q.t_type = terms.add(1, lambda i: RDF_TYPE)
    q.t_pred = terms.add(n_predicates, lambda i: f"<http://ex.org/p{i}>")
    q.t_cls = terms.add(n_classes, lambda i: f"<http://ex.org/C{i}>")
    q.t_ent = terms.add(n_entities, lambda i: f"<http://ex.org/e{i}>")
    q.t_lit = terms.add(n_literals, lambda i: f'"l{i}"')
    q.n_pred, q.n_cls, q.n_ent, q.n_lit = n_predicates, n_classes, n_entities, n_literals
    q.pred_alpha, q.subj_alpha, q.class_frac, q.class_alpha = pred_alpha, subj_alpha, class_frac, class_alpha
    q.literal_frac, q.lit_alpha, q.obj_alpha = literal_frac, lit_alpha, obj_alpha
    if not 0 <= row0 <= row0 + nrows <= n:
        raise ValueError("row range outside the configuration")
    s, p, o = (np.empty(nrows, np.uint32) for _ in range(3))
    if nrows:
        _synth_lib().synth_zipf_rows(ctypes.byref(q), row0, nrows, s.ctypes.data, p.ctypes.data, o.ctypes.data)
    return Dataset(name, s, p, o, terms, min_support)


def _c4_rows(scale: float, lo: int, hi: int) -> Dataset:
    """c4 beyond scale 0.05: rows [lo, hi) of the counter-based Freebase-shaped configuration."""
    n = int(1_000_000_000 * scale)
    return zipf_rows("c4", n, lo, hi - lo, max(int(100_000_000 * scale), 100), max(int(20_000 * scale), 20), 1.2, 1.0,
                     0.10, 2000, 1.2, 0.35, max(int(150_000_000 * scale), 100), 1.0, 1.0, 100, 4)


# ---------------------------------------------------------------------------
# LUBM-shaped generator (c2)

_UB = "http://swat.cse.lehigh.edu/onto/univ-bench.owl#"
_PREDS = ["name", "emailAddress", "telephone", "worksFor", "headOf", "memberOf", "subOrganizationOf",
          "undergraduateDegreeFrom", "mastersDegreeFrom", "doctoralDegreeFrom", "teacherOf", "takesCourse",
          "advisor", "publicationAuthor", "researchInterest", "teachingAssistantOf"]
_CLASSES = ["University", "Department", "FullProfessor", "AssociateProfessor", "AssistantProfessor",
            "Lecturer", "UndergraduateStudent", "GraduateStudent", "Course", "GraduateCourse",
            "ResearchGroup", "Publication", "TeachingAssistant"]
# per-department entity kinds: (label, min, max) counts follow the UBA generator
_FAC = [("FullProfessor", 7, 10, 15, 20), ("AssociateProfessor", 10, 14, 10, 18),
        ("AssistantProfessor", 8, 11, 5, 10), ("Lecturer", 5, 7, 0, 5)]
_N_UNIV_POOL = 1000          # degree-granting universities referenced by degreeFrom
_N_RESEARCH = 30             # researchInterest literal pool "Research{i}"
_NAME_POOL = 2000            # name literals "UndergraduateStudent{i}" etc. repeat across departments


def lubm(n_universities: int = 100, seed: int = 0, min_support: int = 10, max_departments: int | None = None) -> Dataset:
    """LUBM(n)-shaped triples (~133k per university).  Term ids are allocated in ranges so that
    :class:`TermTable` can print them; literals such as names repeat across departments as in UBA."""
    rng = np.random.default_rng(seed)
    terms = TermTable()
    T = {}
    T["type"] = terms.add(1, lambda i: RDF_TYPE)
    T["pred"] = terms.add(len(_PREDS), lambda i: f"<{_UB}{_PREDS[i]}>")
    T["cls"] = terms.add(len(_CLASSES), lambda i: f"<{_UB}{_CLASSES[i]}>")
    T["univ"] = terms.add(_N_UNIV_POOL, lambda i: f"<http://www.University{i}.edu>")
    T["research"] = terms.add(_N_RESEARCH, lambda i: f'"Research{i}"')
    kinds = ["FullProfessor", "AssociateProfessor", "AssistantProfessor", "Lecturer", "UndergraduateStudent",
             "GraduateStudent", "Course", "GraduateCourse", "Publication", "ResearchGroup", "Department"]
    name_base = {}
    for k in kinds:
        name_base[k] = terms.add(_NAME_POOL, (lambda kk: (lambda i: f'"{kk}{i}"'))(k))
    pred = {nm: T["pred"] + i for i, nm in enumerate(_PREDS)}
    cls = {nm: T["cls"] + i for i, nm in enumerate(_CLASSES)}

    # Plan all departments first so that entity id ranges can be allocated contiguously.
    depts = []
    for u in range(n_universities):
        n_dep = int(rng.integers(15, 26))
        if max_departments is not None:
            n_dep = min(n_dep, max_departments)
        for d in range(n_dep):
            fac = [int(rng.integers(lo, hi + 1)) for (_, lo, hi, _, _) in _FAC]
            nf = sum(fac)
            depts.append(dict(u=u, d=d, fac=fac, nf=nf, ug=nf * int(rng.integers(8, 15)),
                              gr=nf * int(rng.integers(3, 5)), rg=int(rng.integers(10, 21))))
    # entity table: for each department a block [dept, faculty..., ug..., grad..., courses..., gcourses...,
    # research groups..., publications...]; emails/phones are per person (faculty+students).
    blocks = []
    total = 0
    for dp in depts:
        nf = dp["nf"]
        n_course = nf * 2                # upper bound: each faculty teaches 1-2 courses
        n_gcourse = nf * 2
        pubs = [int(rng.integers(plo, phi + 1)) for (_, _, _, plo, phi) in _FAC for _ in range(1)]
        # publications per faculty drawn per rank below; reserve an upper bound
        n_pub = sum(c * phi for c, (_, _, _, _, phi) in zip(dp["fac"], _FAC))
        dp.update(n_course=n_course, n_gcourse=n_gcourse, n_pub=n_pub)
        size = 1 + nf + dp["ug"] + dp["gr"] + n_course + n_gcourse + dp["rg"] + n_pub
        dp["base"] = total
        dp["size"] = size
        total += size
        del pubs
    ent_labels = []

    def ent_fmt(i, _depts=depts):
        # binary search department by base
        lo, hi = 0, len(_depts)
        while lo < hi:
            mid = (lo + hi) // 2
            if _depts[mid]["base"] <= i:
                lo = mid + 1
            else:
                hi = mid
        dp = _depts[lo - 1]
        j = i - dp["base"]
        host = f"http://www.Department{dp['d']}.University{dp['u']}.edu"
        if j == 0:
            return f"<{host}>"
        j -= 1
        for (lab, _, _, _, _), c in zip(_FAC, dp["fac"]):
            if j < c:
                return f"<{host}/{lab}{j}>"
            j -= c
        for lab, c in (("UndergraduateStudent", dp["ug"]), ("GraduateStudent", dp["gr"]),
                       ("Course", dp["n_course"]), ("GraduateCourse", dp["n_gcourse"]),
                       ("ResearchGroup", dp["rg"]), ("Publication", dp["n_pub"])):
            if j < c:
                return f"<{host}/{lab}{j}>"
            j -= c
        raise KeyError(i)

    T["ent"] = terms.add(total, ent_fmt)
    n_person_max = total
    T["email"] = terms.add(n_person_max, lambda i: f'"email{i}@lubm.edu"')
    T["phone"] = terms.add(n_person_max, lambda i: f'"xxx-{i // 10000:03d}-{i % 10000:04d}"')
    del ent_labels

    S, Pp, O = [], [], []

    def emit(s, p, o):
        s = np.asarray(s, dtype=np.int64)
        o = np.asarray(o, dtype=np.int64)
        n = max(s.size, o.size)
        S.append(np.broadcast_to(s, (n,)).astype(np.uint32))
        Pp.append(np.full(n, p, dtype=np.uint32))
        O.append(np.broadcast_to(o, (n,)).astype(np.uint32))

    E = T["ent"]
    for dp in depts:
        b = E + dp["base"]
        dept = b
        univ = T["univ"] + dp["u"]
        emit(dept, T["type"], cls["Department"])
        emit(dept, pred["name"], name_base["Department"] + dp["d"] % _NAME_POOL)
        emit(dept, pred["subOrganizationOf"], univ)
        nf = dp["nf"]
        fac = np.arange(b + 1, b + 1 + nf)
        ranks = np.repeat(np.arange(4), dp["fac"])
        rank_local = np.concatenate([np.arange(c) for c in dp["fac"]])
        ug = np.arange(b + 1 + nf, b + 1 + nf + dp["ug"])
        gr = np.arange(ug[-1] + 1, ug[-1] + 1 + dp["gr"])
        c0 = gr[-1] + 1
        courses_all = np.arange(c0, c0 + dp["n_course"])
        gcourses_all = np.arange(c0 + dp["n_course"], c0 + dp["n_course"] + dp["n_gcourse"])
        rg = np.arange(gcourses_all[-1] + 1, gcourses_all[-1] + 1 + dp["rg"])
        pub0 = rg[-1] + 1
        # faculty
        for r, (lab, _, _, _, _) in enumerate(_FAC):
            emit(fac[ranks == r], T["type"], cls[lab])
            emit(fac[ranks == r], pred["name"], name_base[lab] + rank_local[ranks == r] % _NAME_POOL)
        emit(fac, pred["emailAddress"], T["email"] + (fac - E))
        emit(fac, pred["telephone"], T["phone"] + (fac - E))
        emit(fac, pred["researchInterest"], T["research"] + rng.integers(0, _N_RESEARCH, nf))
        emit(fac, pred["undergraduateDegreeFrom"], T["univ"] + rng.integers(0, _N_UNIV_POOL, nf))
        emit(fac, pred["mastersDegreeFrom"], T["univ"] + rng.integers(0, _N_UNIV_POOL, nf))
        emit(fac, pred["doctoralDegreeFrom"], T["univ"] + rng.integers(0, _N_UNIV_POOL, nf))
        emit(fac, pred["worksFor"], dept)
        emit(fac[0], pred["headOf"], dept)
        # courses: each faculty teaches 1-2 courses and 1-2 graduate courses
        nc = rng.integers(1, 3, nf)
        ngc = rng.integers(1, 3, nf)
        teach_c = np.concatenate([np.full(k, f) for f, k in zip(fac, nc)])
        teach_g = np.concatenate([np.full(k, f) for f, k in zip(fac, ngc)])
        courses = courses_all[: teach_c.size]
        gcourses = gcourses_all[: teach_g.size]
        emit(teach_c, pred["teacherOf"], courses)
        emit(teach_g, pred["teacherOf"], gcourses)
        emit(courses, T["type"], cls["Course"])
        emit(courses, pred["name"], name_base["Course"] + np.arange(courses.size) % _NAME_POOL)
        emit(gcourses, T["type"], cls["GraduateCourse"])
        emit(gcourses, pred["name"], name_base["GraduateCourse"] + np.arange(gcourses.size) % _NAME_POOL)
        # research groups
        emit(rg, T["type"], cls["ResearchGroup"])
        emit(rg, pred["subOrganizationOf"], dept)
        # publications
        pub_auth = []
        for r, (_, _, _, plo, phi) in enumerate(_FAC):
            for f in fac[ranks == r]:
                pub_auth.append(np.full(int(rng.integers(plo, phi + 1)), f))
        pub_auth = np.concatenate(pub_auth) if pub_auth else np.zeros(0, np.int64)
        pubs = pub0 + np.arange(pub_auth.size)
        emit(pubs, T["type"], cls["Publication"])
        emit(pubs, pred["name"], name_base["Publication"] + np.arange(pubs.size) % _NAME_POOL)
        emit(pubs, pred["publicationAuthor"], pub_auth)
        # undergraduate students
        nu = ug.size
        emit(ug, T["type"], cls["UndergraduateStudent"])
        emit(ug, pred["name"], name_base["UndergraduateStudent"] + np.arange(nu) % _NAME_POOL)
        emit(ug, pred["emailAddress"], T["email"] + (ug - E))
        emit(ug, pred["telephone"], T["phone"] + (ug - E))
        emit(ug, pred["memberOf"], dept)
        k = rng.integers(2, 5, nu)
        emit(np.repeat(ug, k), pred["takesCourse"], courses[rng.integers(0, courses.size, int(k.sum()))])
        adv = ug[rng.random(nu) < 0.2]
        profs = fac[ranks < 3]
        emit(adv, pred["advisor"], profs[rng.integers(0, profs.size, adv.size)])
        # graduate students
        ng = gr.size
        emit(gr, T["type"], cls["GraduateStudent"])
        emit(gr, pred["name"], name_base["GraduateStudent"] + np.arange(ng) % _NAME_POOL)
        emit(gr, pred["emailAddress"], T["email"] + (gr - E))
        emit(gr, pred["telephone"], T["phone"] + (gr - E))
        emit(gr, pred["memberOf"], dept)
        emit(gr, pred["undergraduateDegreeFrom"], T["univ"] + rng.integers(0, _N_UNIV_POOL, ng))
        k = rng.integers(1, 4, ng)
        emit(np.repeat(gr, k), pred["takesCourse"], gcourses[rng.integers(0, gcourses.size, int(k.sum()))])
        emit(gr, pred["advisor"], profs[rng.integers(0, profs.size, ng)])
        ta = gr[rng.random(ng) < 0.22]
        emit(ta, T["type"], cls["TeachingAssistant"])
        emit(ta, pred["teachingAssistantOf"], courses[rng.integers(0, courses.size, ta.size)])
        # grad students co-author some publications
        if pubs.size:
            co = rng.integers(0, 3, ng)
            emit(pubs[rng.integers(0, pubs.size, int(co.sum()))], pred["publicationAuthor"], np.repeat(gr, co))
    for u in range(min(n_universities, _N_UNIV_POOL)):
        emit(T["univ"] + u, T["type"], cls["University"])
    s = np.concatenate(S)
    p = np.concatenate(Pp)
    o = np.concatenate(O)
    s, p, o = _dedup(s, p, o)  # UBA output is a set of triples
    return Dataset(f"lubm{n_universities}", s, p, o, terms, min_support)


# ---------------------------------------------------------------------------
# BASELINE configs

def config_slice(name: str, scale: float, rank: int, nranks: int) -> tuple:
    """This rank's slice of a BASELINE config for the sharded (multi-GPU) bench: (Dataset of the slice, total
    triples), the contiguous row range [n * rank / nranks, n * (rank + 1) / nranks).  c4 beyond scale 0.05 (1B
    triples at full size: no deduplication, i.i.d. rows) draws only its own rows from the counter-based
    generator, so no rank ever holds the whole input and the slices form the same input as config() for any
    nranks.  Every other config is generated whole (deterministically on every rank) and cut."""
    if name == "c4" and scale > 0.05:
        n = int(1_000_000_000 * scale)
        lo, hi = n * rank // nranks, n * (rank + 1) // nranks
        return _c4_rows(scale, lo, hi), n
    d = config(name, scale)
    n = d.n
    lo, hi = n * rank // nranks, n * (rank + 1) // nranks
    return Dataset(d.name, d.s[lo:hi].copy(), d.p[lo:hi].copy(), d.o[lo:hi].copy(), d.terms, d.min_support), n


def config(name: str, scale: float = 1.0, seed: int | None = None) -> Dataset:
    """c1..c5 of BASELINE.json; ``scale`` shrinks N (and the vocabularies) for tests."""
    if name == "c1":
        n = int(1_000_000 * scale)
        return zipf_rdf("c1", n, max(int(200_000 * scale), 50), 100, 1.1, 1.0, 0.15, 50, 1.2, 0.30,
                        max(int(300_000 * scale), 50), 1.0, 1.0, 10, 1 if seed is None else seed)
    if name == "c2":
        return lubm(max(int(round(100 * scale)), 1), 0 if seed is None else seed, 10)
    if name == "c3":
        n = int(100_000_000 * scale)
        return zipf_rdf("c3", n, max(int(20_000_000 * scale), 100), max(int(50_000 * scale), 20), 1.3, 1.0,
                        0.20, 800, 1.2, 0.45, max(int(30_000_000 * scale), 100), 1.0, 1.0, 25,
                        3 if seed is None else seed)
    if name == "c4":
        n = int(1_000_000_000 * scale)
        if scale > 0.05:  # i.i.d. rows, counter-based (the scales that are also run sharded)
            return _c4_rows(scale, 0, n)
        return zipf_rdf("c4", n, max(int(100_000_000 * scale), 100), max(int(20_000 * scale), 20), 1.2, 1.0,
                        0.10, 2000, 1.2, 0.35, max(int(150_000_000 * scale), 100), 1.0, 1.0, 100,
                        4 if seed is None else seed, dedup=scale <= 0.05)
    if name == "c5":
        n = int(10_000_000 * scale)
        return zipf_rdf("c5", n, max(int(1_000_000 * scale), 50), 50, 1.1, 1.0, 0.10, 30, 1.2, 0.20,
                        max(int(1_000_000 * scale), 50), 1.0, 1.5, 2, 5 if seed is None else seed)
    raise ValueError(name)
