/*
 * ORACLE -- test infrastructure only.  Never linked into the product path.
 *
 * Scalar C restatement of RDFind's CIND discovery on dictionary-encoded
 * triples.  It is the mid-size parity checker for the HIP library (tests/,
 * __graft_entry__.smoke()) and the "port" CPU baseline of bench.py.  Stages 5
 * and 6 (per-dependent intersection, minimality) run on OpenMP threads
 * (OMP_NUM_THREADS); the output order does not depend on the thread count.  Cross-checked against the literal Python restatement
 * (oracle/rdfind_oracle.py) by tests/test_oracle_c.py.
 *
 * Abbreviation: ALG/ = rdfind-algorithm/src/main/scala/de/hpi/isg/sodap/rdfind/
 * Stages (each follows the cited reference code):
 *   1. unary condition counts            ALG/plan/FrequentConditionPlanner.scala:291-311
 *   2. binary condition counts           ALG/operators/candidate_extraction/CreatedReducedDoubleConditionCounts.scala:45-86
 *   3. join partners (capture records)   ALG/operators/CreateJoinPartners.scala:86-147 (+ binary split,
 *                                        CreateDependencyCandidates.scala:90-105)
 *   4. capture groups = distinct (join, capture) grouped by join value
 *                                        ALG/operators/UnionJoinCandidates.scala:27-44, UnionCombinedJoinCandidates.scala:21-31
 *   5. AllAtOnce candidates + intersection per dependent
 *                                        ALG/operators/candidate_extraction/CreateAllCindCandidates.scala:71-121,
 *                                        ALG/operators/candidate_merging/IntersectCindCandidates.scala:14-51
 *   6. minimality R1-R4                  ALG/plan/TraversalStrategy.scala:126-168
 *
 * Capture ids: unary type t (codes 10,12,17,20,33,34) with value v -> t*V+v;
 * binary b (index into the sorted frequent binary keys) -> 6V+b.  Binary key =
 * bt<<62 | v1<<31 | v2, bt = 0 (s[p,o], code 14), 1 (p[s,o], 21), 2 (o[s,p], 35).
 */
#include <omp.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

typedef struct {
    uint32_t dep, ref, support;
} orc_cind;

typedef struct {
    uint64_t n_freq_unary[3];
    uint64_t n_binary_keys;     /* distinct candidate binary conditions counted */
    uint64_t n_freq_binary;
    uint64_t n_records;         /* (join, capture) records emitted */
    uint64_t n_unique;          /* distinct (join, capture) */
    uint64_t n_groups;
    uint64_t n_freq_captures;   /* captures with support >= ms */
    uint64_t n_raw_cinds;       /* |V| before minimality */
    uint64_t n_cinds;
    uint64_t n_join_ranges;     /* join-value ranges stages 3-4 ran in */
} orc_stats;

/* ---------------------------------------------------------------- utils */

static void *xmalloc(size_t n) { return malloc(n ? n : 1); }

/* LSD radix sort, 11-bit digits; each pass: per-thread histograms of contiguous blocks, digit-major
 * offsets, stable scatter (OpenMP threads; same result for any thread count) */
static void radix_sort_u64(uint64_t *a, uint64_t n) {
    if (n < 2) return;
    uint64_t *tmp = (uint64_t *)xmalloc(n * sizeof(uint64_t));
    uint64_t *src = a, *dst = tmp;
    const int nt = n < (1u << 16) ? 1 : omp_get_max_threads();
    uint64_t *cnt = (uint64_t *)xmalloc((size_t)nt * 2048 * sizeof(uint64_t));
    for (int shift = 0; shift < 64; shift += 11) {
        memset(cnt, 0, (size_t)nt * 2048 * sizeof(uint64_t));
#pragma omp parallel num_threads(nt)
        {
            const int t = omp_get_thread_num();
            const uint64_t b0 = n * t / nt, b1 = n * (t + 1) / nt;
            uint64_t *c = cnt + (size_t)t * 2048;
            for (uint64_t i = b0; i < b1; ++i) c[(src[i] >> shift) & 2047]++;
        }
        int trivial = 0;
        for (int d = 0; d < 2048 && !trivial; ++d) {
            uint64_t tot = 0;
            for (int t = 0; t < nt; ++t) tot += cnt[(size_t)t * 2048 + d];
            trivial = tot == n;
        }
        if (trivial) continue;
        uint64_t sum = 0;
        for (int d = 0; d < 2048; ++d)
            for (int t = 0; t < nt; ++t) { uint64_t c = cnt[(size_t)t * 2048 + d]; cnt[(size_t)t * 2048 + d] = sum; sum += c; }
#pragma omp parallel num_threads(nt)
        {
            const int t = omp_get_thread_num();
            const uint64_t b0 = n * t / nt, b1 = n * (t + 1) / nt;
            uint64_t *c = cnt + (size_t)t * 2048;
            for (uint64_t i = b0; i < b1; ++i) dst[c[(src[i] >> shift) & 2047]++] = src[i];
        }
        uint64_t *t = src; src = dst; dst = t;
    }
    if (src != a) memcpy(a, src, n * sizeof(uint64_t));
    free(cnt);
    free(tmp);
}

static uint64_t mix64(uint64_t x) {
    x ^= x >> 33; x *= 0xff51afd7ed558ccdULL; x ^= x >> 33; x *= 0xc4ceb9fe1a85ec53ULL; x ^= x >> 33;
    return x;
}

/* open-addressing u64 -> u32 map (key ~0 = empty) */
typedef struct { uint64_t *keys; uint32_t *vals; uint64_t mask; uint64_t size; } u64map;

static void map_init(u64map *m, uint64_t expected) {
    uint64_t cap = 16;
    while (cap < expected * 2) cap <<= 1;
    m->keys = (uint64_t *)xmalloc(cap * sizeof(uint64_t));
    m->vals = (uint32_t *)xmalloc(cap * sizeof(uint32_t));
    memset(m->keys, 0xff, cap * sizeof(uint64_t));
    memset(m->vals, 0, cap * sizeof(uint32_t));
    m->mask = cap - 1;
    m->size = 0;
}

static uint32_t *map_slot(u64map *m, uint64_t key, int insert) {
    uint64_t h = mix64(key) & m->mask;
    for (;;) {
        if (m->keys[h] == key) return &m->vals[h];
        if (m->keys[h] == ~0ULL) {
            if (!insert) return NULL;
            m->keys[h] = key;
            m->size++;
            return &m->vals[h];
        }
        h = (h + 1) & m->mask;
    }
}

static void map_free(u64map *m) { free(m->keys); free(m->vals); }

static int bsearch_u64(const uint64_t *a, uint64_t n, uint64_t key) {
    uint64_t lo = 0, hi = n;
    while (lo < hi) {
        uint64_t mid = (lo + hi) >> 1;
        if (a[mid] < key) lo = mid + 1; else hi = mid;
    }
    return lo < n && a[lo] == key;
}

/* ---------------------------------------------------------------- codes */

static const int UNARY_CODES[6] = {10, 12, 17, 20, 33, 34};
static const int BINARY_CODES[3] = {14, 21, 35};

static int unary_index(int code) {
    for (int i = 0; i < 6; ++i) if (UNARY_CODES[i] == code) return i;
    return -1;
}

/* components of binary type bt: unary type indices of first (v1) and second (v2) subcapture */
static void binary_components(int bt, int *t1, int *t2) {
    int code = BINARY_CODES[bt];
    int rest = code & ~7;
    int first = code & -code;
    int second = (code & ~first) & -(code & ~first);
    *t1 = unary_index(rest | first);
    *t2 = unary_index(rest | second);
}

/* ---------------------------------------------------------------- stages 1-4 */

/* capture groups + dependent -> groups CSR of one input (stages 1-4) */
typedef struct {
    uint32_t V, ms;
    uint64_t nb;          /* frequent binary conditions (sorted keys) */
    uint64_t *bkeys;
    uint64_t ncap, ng;    /* capture id space 6V + nb; groups */
    uint32_t *fidx;       /* [ncap] index of a frequent capture (support >= ms) among them, ~0 otherwise */
    uint64_t C;           /* frequent captures */
    uint32_t *csup;       /* [C] their supports (distinct join values) */
    uint64_t *cdoff;      /* [C + 1] their groups in dgrp */
    uint64_t *goff;       /* [ng + 1] */
    uint32_t *gcap;       /* group members, ascending capture ids */
    uint32_t *dgrp;
} orc_csr;

#define ORC_NONE 0xffffffffu

static void csr_free(orc_csr *c) {
    free(c->fidx); free(c->csup); free(c->cdoff); free(c->goff); free(c->gcap); free(c->dgrp);
}

/* support[ncap] -> fidx / csup / cdoff (the frequent captures in id order); returns C */
static uint64_t compact_captures(orc_csr *c, const uint32_t *support, uint64_t ncap, uint32_t ms) {
    c->fidx = (uint32_t *)xmalloc(ncap * sizeof(uint32_t));
    uint64_t C = 0;
    for (uint64_t a = 0; a < ncap; ++a) c->fidx[a] = support[a] >= ms ? (uint32_t)C++ : ORC_NONE;
    c->C = C;
    c->csup = (uint32_t *)xmalloc(C * sizeof(uint32_t));
    c->cdoff = (uint64_t *)xmalloc((C + 1) * sizeof(uint64_t));
    uint64_t acc = 0;
    for (uint64_t a = 0; a < ncap; ++a)
        if (c->fidx[a] != ORC_NONE) { c->csup[c->fidx[a]] = support[a]; c->cdoff[c->fidx[a]] = acc; acc += support[a]; }
    c->cdoff[C] = acc;
    return C;
}

static uint64_t g_range_records = 0;  /* orc_set_range_records: join-range size of stages 3-4 (0: one pass) */

void orc_set_range_records(uint64_t r) { g_range_records = r; }

static int prep(const uint32_t *s, const uint32_t *p, const uint32_t *o, uint64_t n, uint32_t V, uint32_t ms,
                const char *projection, orc_csr *c, orc_stats *st) {
    const uint64_t range_records = g_range_records;
    memset(st, 0, sizeof(*st));
    memset(c, 0, sizeof(*c));
    if (V >= (1u << 31)) return -1;
    c->V = V;
    c->ms = ms;
    int proj_s = strchr(projection, 's') != NULL;
    int proj_p = strchr(projection, 'p') != NULL;
    int proj_o = strchr(projection, 'o') != NULL;

    /* 1. unary condition counts (FrequentConditionPlanner.scala:291-311) */
    uint32_t *cnt = (uint32_t *)calloc((size_t)3 * V + 1, sizeof(uint32_t));
    for (uint64_t i = 0; i < n; ++i) { cnt[s[i]]++; cnt[(uint64_t)V + p[i]]++; cnt[2ull * V + o[i]]++; }
    uint8_t *freq = (uint8_t *)calloc((size_t)V + 1, 1); /* bit0 s, bit1 p, bit2 o */
    for (uint32_t v = 0; v < V; ++v) {
        for (int t = 0; t < 3; ++t)
            if (cnt[(uint64_t)t * V + v] >= ms) { freq[v] |= (uint8_t)(1u << t); st->n_freq_unary[t]++; }
    }
    free(cnt);

    /* 2. binary condition counts (CreatedReducedDoubleConditionCounts.scala:45-86): the keys of the triples with two
     *    frequent values, one binary type (key bits 62-63) at a time, sorted and counted per run; the types ascend in
     *    the key's top bits, so the frequent keys of the three passes concatenate sorted (memory ~16 B per key of one
     *    type; chunked passes keep any thread count's result identical) */
    enum { NCH = 4096 };
    uint64_t *chunk = (uint64_t *)calloc(NCH + 1, sizeof(uint64_t));
    uint64_t *bkeys = NULL, nb = 0, ndist = 0;
    for (int bt = 0; bt < 3; ++bt) {
        /* bt 0: s[p,o] (p, o frequent); 1: p[s,o] (s, o); 2: o[s,p] (s, p) */
#define BKEY_OF(i, OK, KEY)                                                                       \
        int fs = freq[s[i]] & 1, fp = (freq[p[i]] >> 1) & 1, fo = (freq[o[i]] >> 2) & 1;           \
        const int OK = bt == 0 ? (fp && fo) : bt == 1 ? (fs && fo) : (fs && fp);                     \
        const uint64_t KEY = bt == 0 ? (((uint64_t)p[i] << 31) | o[i])                             \
                           : bt == 1 ? ((1ull << 62) | ((uint64_t)s[i] << 31) | o[i])                \
                                     : ((2ull << 62) | ((uint64_t)s[i] << 31) | p[i]);
        chunk[0] = 0;
#pragma omp parallel for schedule(dynamic, 1)
        for (int ch = 0; ch < NCH; ++ch) {
            uint64_t k = 0;
            for (uint64_t i = n * ch / NCH; i < n * (ch + 1) / NCH; ++i) {
                BKEY_OF(i, ok, key)
                (void)key;
                k += ok;
            }
            chunk[ch + 1] = k;
        }
        for (int ch = 0; ch < NCH; ++ch) chunk[ch + 1] += chunk[ch];
        const uint64_t nk = chunk[NCH];
        uint64_t *keys = (uint64_t *)xmalloc(nk * sizeof(uint64_t));
#pragma omp parallel for schedule(dynamic, 1)
        for (int ch = 0; ch < NCH; ++ch) {
            uint64_t k = chunk[ch];
            for (uint64_t i = n * ch / NCH; i < n * (ch + 1) / NCH; ++i) {
                BKEY_OF(i, ok, key)
                if (ok) keys[k++] = key;
            }
        }
#undef BKEY_OF
        radix_sort_u64(keys, nk);
        uint64_t nf = 0;
        for (uint64_t i = 0; i < nk;) {
            uint64_t j = i + 1;
            while (j < nk && keys[j] == keys[i]) ++j;
            ndist++;
            if (j - i >= ms) keys[nf++] = keys[i];  /* ascending: the frequent keys come out sorted */
            i = j;
        }
        bkeys = (uint64_t *)realloc(bkeys, (nb + nf + 1) * sizeof(uint64_t));
        memcpy(bkeys + nb, keys, nf * sizeof(uint64_t));
        nb += nf;
        free(keys);
    }
    st->n_binary_keys = ndist;
    st->n_freq_binary = nb;
    u64map bidx;
    map_init(&bidx, nb + 16);
    for (uint64_t b = 0; b < nb; ++b) *map_slot(&bidx, bkeys[b], 1) = (uint32_t)b;

    /* 3. join partners (CreateJoinPartners.scala:86-147), binary captures split into their unary
     *    components as every consumer does (CreateDependencyCandidates.scala:90-105), as records
     *    join << capbits | capture.  Inputs whose records exceed range_records (0: no limit) are processed in ranges
     *    of join values (the reference's sort-based groupBy("joinValue") spills instead, RDFind.scala:339-345): a
     *    join value's records all fall in one range, so each range's groups are whole. */
    const uint64_t capbits = 64 - __builtin_clzll((uint64_t)6 * V + nb + 1);
    const uint64_t ncap = 6ull * V + nb;
    const uint64_t capmask = (1ull << capbits) - 1;
#define EMIT_ALL(EMIT)                                                                            \
    {                                                                                             \
        uint32_t ts = s[i], tp = p[i], to = o[i];                                                 \
        int fs = freq[ts] & 1, fp = (freq[tp] >> 1) & 1, fo = (freq[to] >> 2) & 1;               \
        uint32_t *b;                                                                              \
        if (proj_o) {                                                                             \
            if (fs) EMIT(to, 4ull * V + ts);             /* o[s] */                               \
            if (fp) EMIT(to, 5ull * V + tp);             /* o[p] */                               \
            if (fs && fp && (b = map_slot(&bidx, (2ull << 62) | ((uint64_t)ts << 31) | tp, 0)))   \
                EMIT(to, 6ull * V + *b);                 /* o[s,p] */                             \
        }                                                                                         \
        if (proj_p) {                                                                             \
            if (fs) EMIT(tp, 2ull * V + ts);             /* p[s] */                               \
            if (fo) EMIT(tp, 3ull * V + to);             /* p[o] */                               \
            if (fs && fo && (b = map_slot(&bidx, (1ull << 62) | ((uint64_t)ts << 31) | to, 0)))   \
                EMIT(tp, 6ull * V + *b);                 /* p[s,o] */                             \
        }                                                                                         \
        if (proj_s) {                                                                             \
            if (fp) EMIT(ts, 0ull * V + tp);             /* s[p] */                               \
            if (fo) EMIT(ts, 1ull * V + to);             /* s[o] */                               \
            if (fp && fo && (b = map_slot(&bidx, (0ull << 62) | ((uint64_t)tp << 31) | to, 0)))   \
                EMIT(ts, 6ull * V + *b);                 /* s[p,o] */                             \
        }                                                                                         \
    }
#define IN_RANGE(join) ((uint64_t)(join) >= jlo && (uint64_t)(join) < jhi)
#define COUNT(join, cap) if (IN_RANGE(join)) { (void)(cap); k++; }
#define STORE(join, cap) if (IN_RANGE(join)) rec[k++] = ((uint64_t)(join) << capbits) | (uint64_t)(cap)
#define HIST(join, cap) { (void)(cap); h[(uint64_t)(join) >> jshift]++; }
    /* join ranges: records per join bucket (2^16 buckets), consecutive buckets up to range_records records each */
    enum { NJB = 1 << 16 };
    const int joinbits = V > 1 ? 64 - __builtin_clzll((uint64_t)V - 1) : 1;
    const int jshift = joinbits > 16 ? joinbits - 16 : 0;
    uint64_t *rlo = (uint64_t *)xmalloc((NJB + 2) * sizeof(uint64_t)), nrange = 0;
    if (range_records) {
        const int nt = omp_get_max_threads();
        uint64_t *hist = (uint64_t *)calloc((size_t)nt * NJB, sizeof(uint64_t));
#pragma omp parallel
        {
            uint64_t *h = hist + (size_t)omp_get_thread_num() * NJB;
#pragma omp for schedule(dynamic, 1)
            for (int ch = 0; ch < NCH; ++ch)
                for (uint64_t i = n * ch / NCH; i < n * (ch + 1) / NCH; ++i) EMIT_ALL(HIST)
        }
        uint64_t acc = 0;
        rlo[nrange++] = 0;
        for (uint64_t bk = 0; bk < NJB; ++bk) {
            uint64_t hb = 0;
            for (int t = 0; t < nt; ++t) hb += hist[(size_t)t * NJB + bk];
            if (acc && acc + hb > range_records) { rlo[nrange++] = bk << jshift; acc = 0; }
            acc += hb;
        }
        free(hist);
    } else {
        rlo[nrange++] = 0;
    }
    rlo[nrange] = ~0ull;
    st->n_join_ranges = nrange;

    /* records of join values [jlo, jhi), sorted and made distinct (UnionJoinCandidates / UnionCombinedJoinCandidates) */
    uint64_t *rec = NULL, nu = 0;
#define RANGE_RECORDS(r)                                                                          \
    {                                                                                             \
        const uint64_t jlo = rlo[r], jhi = rlo[(r) + 1];                                          \
        chunk[0] = 0;                                                                             \
        _Pragma("omp parallel for schedule(dynamic, 1)")                                          \
        for (int ch = 0; ch < NCH; ++ch) {                                                        \
            uint64_t k = 0;                                                                       \
            for (uint64_t i = n * ch / NCH; i < n * (ch + 1) / NCH; ++i) EMIT_ALL(COUNT)          \
            chunk[ch + 1] = k;                                                                    \
        }                                                                                         \
        for (int ch = 0; ch < NCH; ++ch) chunk[ch + 1] += chunk[ch];                             \
        const uint64_t nr = chunk[NCH];                                                           \
        free(rec);                                                                                \
        rec = (uint64_t *)xmalloc(nr * sizeof(uint64_t));                                         \
        _Pragma("omp parallel for schedule(dynamic, 1)")                                          \
        for (int ch = 0; ch < NCH; ++ch) {                                                        \
            uint64_t k = chunk[ch];                                                               \
            for (uint64_t i = n * ch / NCH; i < n * (ch + 1) / NCH; ++i) EMIT_ALL(STORE)          \
        }                                                                                         \
        radix_sort_u64(rec, nr);                                                                  \
        nu = 0;                                                                                   \
        for (uint64_t i = 0; i < nr; ++i)                                                         \
            if (nu == 0 || rec[nu - 1] != rec[i]) rec[nu++] = rec[i];                             \
        rec_count = nr;                                                                           \
    }
    /* 4a. supports = distinct join values per capture (BulkMergeDependencies.scala:78), summed over the ranges */
    uint32_t *support = (uint32_t *)calloc(ncap + 1, sizeof(uint32_t));
    for (uint64_t r = 0; r < nrange; ++r) {
        uint64_t rec_count = 0;
        RANGE_RECORDS(r)
        st->n_records += rec_count;
        st->n_unique += nu;
        for (uint64_t i = 0; i < nu; ++i) support[rec[i] & capmask]++;
        if (nrange > 1) { free(rec); rec = NULL; }
    }
    const uint64_t C = compact_captures(c, support, ncap, ms);
    free(support);
    st->n_freq_captures = C;
    /* 4b. groups (join values with a frequent member; a ref is in every group of its dependent, so its support is at
     *     least the dependent's: infrequent captures are no refs), members ascending; dependent -> groups, ascending */
    const uint64_t Jf = c->cdoff[C];
    const uint64_t gmax = Jf < V ? Jf : V;
    uint64_t *goff = (uint64_t *)xmalloc((gmax + 1) * sizeof(uint64_t));
    uint32_t *gcap = (uint32_t *)xmalloc((Jf ? Jf : 1) * sizeof(uint32_t));
    uint32_t *dgrp = (uint32_t *)xmalloc((Jf ? Jf : 1) * sizeof(uint32_t));
    uint64_t *cur = (uint64_t *)xmalloc((C + 1) * sizeof(uint64_t));
    memcpy(cur, c->cdoff, (C + 1) * sizeof(uint64_t));
    uint64_t ng = 0, gpos = 0;
    for (uint64_t r = 0; r < nrange; ++r) {
        if (nrange > 1) {
            uint64_t rec_count = 0;
            RANGE_RECORDS(r)
            (void)rec_count;
        }
        for (uint64_t i = 0; i < nu;) {
            uint64_t j = i;
            const uint64_t gstart = gpos;
            for (; j < nu && (rec[j] >> capbits) == (rec[i] >> capbits); ++j) {
                const uint32_t cap = (uint32_t)(rec[j] & capmask), f = c->fidx[cap];
                if (f == ORC_NONE) continue;
                gcap[gpos++] = cap;
                dgrp[cur[f]++] = (uint32_t)ng;
            }
            if (gpos > gstart) goff[ng++] = gstart;
            i = j;
        }
    }
    goff[ng] = gpos;
    free(rec);
    free(cur);
    free(rlo);
#undef RANGE_RECORDS
#undef IN_RANGE
#undef HIST
#undef COUNT
#undef STORE
#undef EMIT_ALL
    free(chunk);
    map_free(&bidx);
    free(freq);
    st->n_groups = ng;
    c->nb = nb; c->bkeys = bkeys; c->ncap = ncap; c->ng = ng;
    c->goff = goff; c->gcap = gcap; c->dgrp = dgrp;
    return 0;
}

/* ---------------------------------------------------------------- stage 5: raw refs of one dependent */

typedef struct { uint32_t *refs, *tmp; uint64_t cap; } refbuf;

static void refbuf_free(refbuf *b) { free(b->refs); free(b->tmp); b->refs = b->tmp = NULL; b->cap = 0; }

/* unary components (capture ids) of binary capture x >= 6V */
static void comps_of(const orc_csr *c, uint64_t x, uint32_t *c1, uint32_t *c2) {
    uint64_t key = c->bkeys[x - 6ull * c->V];
    int t1, t2;
    binary_components((int)(key >> 62), &t1, &t2);
    *c1 = (uint32_t)((uint64_t)t1 * c->V + ((key >> 31) & 0x7fffffff));
    *c2 = (uint32_t)((uint64_t)t2 * c->V + (key & 0x7fffffff));
}

static uint64_t lower_bound_u32(const uint32_t *a, uint64_t n, uint32_t key) {
    uint64_t lo = 0, hi = n;
    while (lo < hi) {
        uint64_t mid = (lo + hi) >> 1;
        if (a[mid] < key) lo = mid + 1; else hi = mid;
    }
    return lo;
}

/* Raw ref set of dependent a (support >= ms), sorted ascending, in b->refs; returns its size.
 * ref set = intersection over a's groups of (group \ {a} \ implied)
 * (CreateAllCindCandidates.scala:106-121 + IntersectCindCandidates.scala:40-43).  The intersection starts
 * from a's smallest group; a group much larger than the surviving set is probed by binary search, otherwise
 * merged (the set is the same in any order; this only bounds the work by the smallest group). */
static uint64_t raw_refs(const orc_csr *c, uint64_t a, int strategy, refbuf *b) {
    const uint64_t V = c->V;
    /* trivial refs of a binary dep: its two unary components (Condition.isImpliedBy) */
    uint32_t triv1 = ~0u, triv2 = ~0u;
    int dep_bt = -1;
    uint32_t dv2 = 0;
    if (a >= 6ull * V) {
        uint64_t key = c->bkeys[a - 6ull * V];
        dep_bt = (int)(key >> 62);
        dv2 = (uint32_t)(key & 0x7fffffff);
        comps_of(c, a, &triv1, &triv2);
    }
    const uint32_t fa = c->fidx[a];
    const uint64_t j0 = c->cdoff[fa], j1 = c->cdoff[fa + 1];
    if (j0 == j1) return 0;
    uint64_t jp = j0;  /* pivot: smallest group */
    for (uint64_t j = j0 + 1; j < j1; ++j) {
        const uint64_t g = c->dgrp[j], gp = c->dgrp[jp];
        if (c->goff[g + 1] - c->goff[g] < c->goff[gp + 1] - c->goff[gp]) jp = j;
    }
    {
        const uint64_t g = c->dgrp[jp], k = c->goff[g + 1] - c->goff[g];
        const uint32_t *gc = c->gcap + c->goff[g];
        if (k > b->cap) {
            b->cap = k * 2;
            b->refs = (uint32_t *)realloc(b->refs, b->cap * sizeof(uint32_t));
            b->tmp = (uint32_t *)realloc(b->tmp, b->cap * sizeof(uint32_t));
        }
        uint64_t nref = 0;
        for (uint64_t i = 0; i < k; ++i) {
            uint32_t r = gc[i];
            if (r == a || r == triv1 || r == triv2) continue;
            if (strategy == 0 && dep_bt >= 0 && r >= 6ull * V) {
                /* literal Condition.isImpliedBy quirk for same-type binary captures:
                 * ref X is "implied" by dep D when X.v1 == D.v2 (Condition.scala:35-43) */
                uint64_t rk = c->bkeys[r - 6ull * V];
                if ((int)(rk >> 62) == dep_bt && (uint32_t)((rk >> 31) & 0x7fffffff) == dv2) continue;
            }
            b->refs[nref++] = r;
        }
        for (uint64_t j = j0; j < j1 && nref; ++j) {
            if (j == jp) continue;
            const uint64_t gg = c->dgrp[j], kk = c->goff[gg + 1] - c->goff[gg];
            const uint32_t *gm = c->gcap + c->goff[gg];
            uint64_t m = 0;
            if (kk > 16 * nref) {
                uint64_t lo = 0;
                for (uint64_t x = 0; x < nref; ++x) {
                    lo += lower_bound_u32(gm + lo, kk - lo, b->refs[x]);
                    if (lo < kk && gm[lo] == b->refs[x]) b->tmp[m++] = b->refs[x];
                }
            } else {
                uint64_t x = 0, y = 0;
                while (x < nref && y < kk) {
                    if (b->refs[x] < gm[y]) x++;
                    else if (b->refs[x] > gm[y]) y++;
                    else { b->tmp[m++] = b->refs[x]; x++; y++; }
                }
            }
            uint32_t *t = b->refs; b->refs = b->tmp; b->tmp = t;
            nref = m;
        }
        return nref;
    }
}

static int cmp_u32(const void *x, const void *y) {
    const uint32_t a = *(const uint32_t *)x, b = *(const uint32_t *)y;
    return a < b ? -1 : (a > b);
}


/* ---------------------------------------------------------------- materialized result */

int orc_run(const uint32_t *s, const uint32_t *p, const uint32_t *o, uint64_t n, uint32_t V,
            uint32_t ms, int strategy, int clean, const char *projection,
            orc_cind **out, uint64_t *n_out, uint64_t **bin_keys_out, uint64_t *n_bin_out,
            orc_stats *st) {
    orc_csr c;
    if (prep(s, p, o, n, V, ms, projection, &c, st)) return -1;
    const uint64_t ncap = c.ncap;
    const uint64_t *bkeys = c.bkeys;

    /* 5. per dependent: raw ref set.  Dependents are split into chunks processed by OpenMP threads; each
     *    chunk's CINDs go to its own buffer and the buffers are concatenated in chunk (= dependent) order. */
    const uint64_t nchunk = ncap < 4096 ? 1 : 4096;
    orc_cind **cbuf = (orc_cind **)calloc(nchunk, sizeof(orc_cind *));
    uint64_t *ccnt = (uint64_t *)calloc(nchunk + 1, sizeof(uint64_t));
#pragma omp parallel
    {
        refbuf rb = {NULL, NULL, 0};
#pragma omp for schedule(dynamic, 1)
        for (uint64_t ch = 0; ch < nchunk; ++ch) {
            uint64_t ccap = 256, nc = 0;
            orc_cind *cind = (orc_cind *)xmalloc(ccap * sizeof(orc_cind));
            const uint64_t a0 = ncap * ch / nchunk, a1 = ncap * (ch + 1) / nchunk;
            for (uint64_t a = a0; a < a1; ++a) {
                if (c.fidx[a] == ORC_NONE) continue;
                const uint64_t nref = raw_refs(&c, a, strategy, &rb);
                for (uint64_t i = 0; i < nref; ++i) {
                    if (nc == ccap) { ccap *= 2; cind = (orc_cind *)realloc(cind, ccap * sizeof(orc_cind)); }
                    cind[nc].dep = (uint32_t)a;
                    cind[nc].ref = rb.refs[i];
                    cind[nc].support = c.csup[c.fidx[a]];
                    nc++;
                }
            }
            cbuf[ch] = cind;
            ccnt[ch] = nc;
        }
        refbuf_free(&rb);
    }
    uint64_t nc = 0;
    for (uint64_t ch = 0; ch < nchunk; ++ch) { uint64_t cc = ccnt[ch]; ccnt[ch] = nc; nc += cc; }
    ccnt[nchunk] = nc;
    orc_cind *cind = (orc_cind *)xmalloc(nc * sizeof(orc_cind));
#pragma omp parallel for schedule(dynamic, 16)
    for (uint64_t ch = 0; ch < nchunk; ++ch) {
        memcpy(cind + ccnt[ch], cbuf[ch], (ccnt[ch + 1] - ccnt[ch]) * sizeof(orc_cind));
        free(cbuf[ch]);
    }
    free(cbuf); free(ccnt);
    st->n_raw_cinds = nc;

    /* 6. minimality (TraversalStrategy.removeImpliedCinds :126-168), rules on the raw sets */
    if (clean && nc) {
        const uint64_t U = 6ull * V;
        uint64_t *s11 = (uint64_t *)xmalloc(nc * sizeof(uint64_t)), n11 = 0;   /* (dep,ref) of 1/1 */
        uint64_t *s12 = (uint64_t *)xmalloc(nc * sizeof(uint64_t)), n12 = 0;   /* (dep,ref) of 1/2 */
        uint64_t *s12c = (uint64_t *)xmalloc(2 * nc * sizeof(uint64_t)), n12c = 0; /* (dep, comp(ref)) of 1/2 */
        uint64_t *s22c = (uint64_t *)xmalloc(2 * nc * sizeof(uint64_t)), n22c = 0; /* (dep, comp(ref)) of 2/2 */
        for (uint64_t i = 0; i < nc; ++i) {
            uint64_t d = cind[i].dep, r = cind[i].ref;
            int du = d < U, ru = r < U;
            uint64_t pair = (d << 32) | r;
            if (du && ru) s11[n11++] = pair;
            if (du && !ru) s12[n12++] = pair;
            if (!ru) {
                uint32_t c1, c2;
                comps_of(&c, r, &c1, &c2);
                if (du) { s12c[n12c++] = (d << 32) | c1; s12c[n12c++] = (d << 32) | c2; }
                else { s22c[n22c++] = (d << 32) | c1; s22c[n22c++] = (d << 32) | c2; }
            }
        }
        radix_sort_u64(s11, n11); radix_sort_u64(s12, n12);
        radix_sort_u64(s12c, n12c); radix_sort_u64(s22c, n22c);
        uint8_t *keep = (uint8_t *)xmalloc(nc);
#pragma omp parallel for schedule(static)
        for (uint64_t i = 0; i < nc; ++i) {
            uint64_t d = cind[i].dep, r = cind[i].ref;
            int du = d < U, ru = r < U;
            int drop = 0;
            if (du && ru) {
                drop = bsearch_u64(s12c, n12c, (d << 32) | r);                          /* R3 */
            } else if (!du) {
                uint32_t c1, c2;
                comps_of(&c, d, &c1, &c2);
                if (ru) {
                    drop = bsearch_u64(s11, n11, ((uint64_t)c1 << 32) | r) || bsearch_u64(s11, n11, ((uint64_t)c2 << 32) | r)  /* R1 */
                        || bsearch_u64(s22c, n22c, (d << 32) | r);                                      /* R2 */
                } else {
                    drop = bsearch_u64(s12, n12, ((uint64_t)c1 << 32) | r) || bsearch_u64(s12, n12, ((uint64_t)c2 << 32) | r); /* R4 */
                }
            }
            keep[i] = (uint8_t)!drop;
        }
        uint64_t m = 0;
        for (uint64_t i = 0; i < nc; ++i)
            if (keep[i]) cind[m++] = cind[i];
        free(keep);
        nc = m;
        free(s11); free(s12); free(s12c); free(s22c);
    }
    (void)bkeys;
    csr_free(&c);
    st->n_cinds = nc;
    *out = cind;
    *n_out = nc;
    *bin_keys_out = c.bkeys;
    *n_bin_out = c.nb;
    return 0;
}

/* ---------------------------------------------------------------- streamed result */

/* Order-independent checksum term of one result row (the same mix as the library's rdf_cind_checksum):
 * external capture ids (unary t*V+v, binary 6V+b) and the dependent's support. */
static inline uint64_t row_hash(uint32_t dep, uint32_t ref, uint32_t support) {
    return mix64((((uint64_t)dep << 32) | ref) + (uint64_t)support * 0x9E3779B97F4A7C15ULL);
}

#define ORC_R1 1
#define ORC_R2 2
#define ORC_R3 4
#define ORC_R4 8

typedef struct {
    uint64_t n_cinds;
    uint64_t checksum;
    uint64_t n_kind[4];   /* 1/1, 1/2, 2/1, 2/2 after the rules */
    uint64_t n_raw;       /* |V| */
} orc_stream_result;

/* Count + checksum of the result without materializing it: every dependent's raw refs, then R1-R4 per
 * dependent.  R2 and R3 only look at the dependent's own raw refs; R1 and R4 test membership of (comp(D), ref)
 * in V11 / V12, i.e. in the raw refs of the two unary components of a binary dependent D, which are computed
 * here (cached per thread: binary ids follow the sorted keys, so consecutive dependents share comp1).
 * rules: ORC_R* mask (15 = --clean-implied, R1|R4 = strategy-1 raw output, 0 = strategy-0 raw). */
int orc_stream(const uint32_t *s, const uint32_t *p, const uint32_t *o, uint64_t n, uint32_t V, uint32_t ms,
               int strategy, int rules, const char *projection, orc_stream_result *res, orc_stats *st) {
    orc_csr c;
    memset(res, 0, sizeof(*res));
    if (prep(s, p, o, n, V, ms, projection, &c, st)) return -1;
    const uint64_t ncap = c.ncap, U = 6ull * V;
    const uint64_t nchunk = ncap < 4096 ? 1 : 65536;
    uint64_t t_cnt = 0, t_sum = 0, t_raw = 0, t_kind[4] = {0, 0, 0, 0};
#pragma omp parallel reduction(+ : t_cnt, t_sum, t_raw)
    {
        refbuf rb = {NULL, NULL, 0};
        /* per-thread direct-mapped cache of the raw refs of binary dependents' unary components */
        enum { NSLOT = 256 };
        refbuf cache[NSLOT];
        uint64_t ckey[NSLOT], cn[NSLOT];
        memset(cache, 0, sizeof(cache));
        for (int k = 0; k < NSLOT; ++k) ckey[k] = ~0ull, cn[k] = 0;
        uint32_t *comp = NULL;
        uint64_t comp_cap = 0;
        uint64_t kind[4] = {0, 0, 0, 0};
#pragma omp for schedule(dynamic, 1)
        for (uint64_t ch = 0; ch < nchunk; ++ch) {
            const uint64_t a0 = ncap * ch / nchunk, a1 = ncap * (ch + 1) / nchunk;
            for (uint64_t a = a0; a < a1; ++a) {
                if (c.fidx[a] == ORC_NONE) continue;
                const uint64_t nref = raw_refs(&c, a, strategy, &rb);
                if (!nref) continue;
                t_raw += nref;
                const uint32_t sup = c.csup[c.fidx[a]];
                /* first binary ref (refs are sorted: unary ids < 6V first) */
                uint64_t nb0 = 0;
                while (nb0 < nref && rb.refs[nb0] < U) nb0++;
                /* components of the binary raw refs (R2 for binary deps, R3 for unary deps) */
                uint64_t ncomp = 0;
                const int mark = a < U ? (rules & ORC_R3) : (rules & ORC_R2);
                if (mark && nref > nb0) {
                    if (2 * (nref - nb0) > comp_cap) {
                        comp_cap = 4 * (nref - nb0);
                        comp = (uint32_t *)realloc(comp, comp_cap * sizeof(uint32_t));
                    }
                    for (uint64_t i = nb0; i < nref; ++i) comps_of(&c, rb.refs[i], &comp[ncomp], &comp[ncomp + 1]), ncomp += 2;
                    qsort(comp, ncomp, sizeof(uint32_t), cmp_u32);
                }
                const uint32_t *r1 = NULL, *r2 = NULL;
                uint64_t n1 = 0, n2 = 0;
                if (a >= U && (rules & (ORC_R1 | ORC_R4))) {
                    uint32_t cc[2];
                    comps_of(&c, a, &cc[0], &cc[1]);
                    const uint64_t k1 = mix64(cc[0]) % NSLOT;
                    uint64_t k2 = mix64(cc[1]) % NSLOT;
                    if (k2 == k1) k2 = (k2 + 1) % NSLOT;  /* both components stay resident */
                    const uint64_t ks[2] = {k1, k2};
                    for (int q = 0; q < 2; ++q) {
                        const uint64_t k = ks[q];
                        if (ckey[k] != cc[q]) { cn[k] = raw_refs(&c, cc[q], strategy, &cache[k]); ckey[k] = cc[q]; }
                    }
                    r1 = cache[k1].refs; n1 = cn[k1];
                    r2 = cache[k2].refs; n2 = cn[k2];
                }
                /* refs, comp, r1 and r2 are all sorted: membership by forward-moving cursors */
                uint64_t pc = 0, p1 = 0, p2 = 0;
                for (uint64_t i = 0; i < nref; ++i) {
                    const uint32_t r = rb.refs[i];
                    const int ru = r < U;
                    int drop = 0;
                    if (ncomp && ru) {                                                           /* R3 / R2 */
                        while (pc < ncomp && comp[pc] < r) pc++;
                        drop = pc < ncomp && comp[pc] == r;
                    }
                    if (!drop && a >= U) {
                        const int rule = ru ? (rules & ORC_R1) : (rules & ORC_R4);                  /* R1 / R4 */
                        if (rule) {
                            while (p1 < n1 && r1[p1] < r) p1++;
                            while (p2 < n2 && r2[p2] < r) p2++;
                            drop = (p1 < n1 && r1[p1] == r) || (p2 < n2 && r2[p2] == r);
                        }
                    }
                    if (drop) continue;
                    t_cnt++;
                    t_sum += row_hash((uint32_t)a, r, sup);
                    kind[(a >= U) * 2 + !ru]++;
                }
            }
        }
#pragma omp critical
        for (int k = 0; k < 4; ++k) t_kind[k] += kind[k];
        refbuf_free(&rb);
        for (int k = 0; k < NSLOT; ++k) refbuf_free(&cache[k]);
        free(comp);
    }
    res->n_cinds = t_cnt;
    res->checksum = t_sum;
    res->n_raw = t_raw;
    for (int k = 0; k < 4; ++k) res->n_kind[k] = t_kind[k];
    st->n_raw_cinds = t_raw;
    st->n_cinds = t_cnt;
    free(c.bkeys);
    csr_free(&c);
    return 0;
}

/* checksum of a materialized result (same row hash as orc_stream) */
uint64_t orc_checksum(const orc_cind *rows, uint64_t n) {
    uint64_t acc = 0;
#pragma omp parallel for reduction(+ : acc) schedule(static)
    for (uint64_t i = 0; i < n; ++i) acc += row_hash(rows[i].dep, rows[i].ref, rows[i].support);
    return acc;
}

/* Count, per-kind counts and checksum of a compact result (include/rdfind_hip.h rdf_copy_result_compact): the
 * explicit runs plus, for every member of a shared list, the list minus the member itself.  Checker for the
 * device's compact hand-over (the expansion the consumer would do), with external ids via capture_ids. */
uint64_t orc_checksum_compact(const uint32_t *refs, const uint64_t *runoff, const uint32_t *rundep, uint64_t nruns,
                              const uint32_t *list_refs, const uint64_t *list_off, const uint64_t *members,
                              uint64_t nmem, const uint32_t *capture_ids, const uint32_t *supports, uint32_t V,
                              uint64_t *count, uint64_t kind[4]) {
    const uint64_t U = 6ull * V;
    uint64_t acc = 0, cnt = 0, k0 = 0, k1 = 0, k2 = 0, k3 = 0;
#pragma omp parallel for reduction(+ : acc, cnt, k0, k1, k2, k3) schedule(dynamic, 64)
    for (uint64_t r = 0; r < nruns; ++r) {
        const uint32_t d = rundep[r], dx = capture_ids[d], sup = supports[d];
        for (uint64_t i = runoff[r]; i < runoff[r + 1]; ++i) {
            const uint32_t rx = capture_ids[refs[i]];
            acc += row_hash(dx, rx, sup);
            cnt++;
            const int k = (dx >= U) * 2 + (rx >= U);
            k0 += k == 0; k1 += k == 1; k2 += k == 2; k3 += k == 3;
        }
    }
#pragma omp parallel for reduction(+ : acc, cnt, k0, k1, k2, k3) schedule(dynamic, 1)
    for (uint64_t j = 0; j < nmem; ++j) {
        const uint64_t l = members[j] >> 32;
        const uint32_t d = (uint32_t)members[j], dx = capture_ids[d], sup = supports[d];
        for (uint64_t i = list_off[l]; i < list_off[l + 1]; ++i) {
            if (list_refs[i] == d) continue;
            const uint32_t rx = capture_ids[list_refs[i]];
            acc += row_hash(dx, rx, sup);
            cnt++;
            const int k = (dx >= U) * 2 + (rx >= U);
            k0 += k == 0; k1 += k == 1; k2 += k == 2; k3 += k == 3;
        }
    }
    *count = cnt;
    kind[0] = k0; kind[1] = k1; kind[2] = k2; kind[3] = k3;
    return acc;
}

/* The heavy-bits part of a compact result (rdf_copy_result_heavy): chunk w of 64 class-list candidates of dependent
 * deps[w] starting at list position pos[w]; bit b of bits[w] set = the CIND deps[w] < list_refs[pos[w] + b]. */
uint64_t orc_checksum_heavy(const uint32_t *deps, const uint64_t *pos, const uint64_t *bits, uint64_t nchunks,
                            const uint32_t *list_refs, const uint32_t *capture_ids, const uint32_t *supports, uint32_t V,
                            uint64_t *count, uint64_t kind[4]) {
    const uint64_t U = 6ull * V;
    uint64_t acc = 0, cnt = 0, k0 = 0, k1 = 0, k2 = 0, k3 = 0;
#pragma omp parallel for reduction(+ : acc, cnt, k0, k1, k2, k3) schedule(static, 4096)
    for (uint64_t w = 0; w < nchunks; ++w) {
        const uint32_t d = deps[w], dx = capture_ids[d], sup = supports[d];
        for (uint64_t m = bits[w]; m; m &= m - 1) {
            const uint32_t rx = capture_ids[list_refs[pos[w] + (uint64_t)__builtin_ctzll(m)]];
            acc += row_hash(dx, rx, sup);
            cnt++;
            const int k = (dx >= U) * 2 + (rx >= U);
            k0 += k == 0; k1 += k == 1; k2 += k == 2; k3 += k == 3;
        }
    }
    *count = cnt;
    kind[0] = k0; kind[1] = k1; kind[2] = k2; kind[3] = k3;
    return acc;
}

void orc_free(void *ptr) { free(ptr); }

/* threads stages 4-6 use (OMP_NUM_THREADS, else all cores) */
int orc_threads(void) { return omp_get_max_threads(); }
