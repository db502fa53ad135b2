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
 *   1. unary condition counts            ALG/plan/FrequentConditionPlanner.scala:488-508
 *   2. binary condition counts           ALG/operators/candidate_extraction/CreatedReducedDoubleConditionCounts.scala:45-86
 *   3. join partners (capture records)   ALG/operators/CreateJoinPartners.scala:86-147 (+ binary split,
 *                                        CreateDependencyCandidates.scala:157-186)
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

/* ---------------------------------------------------------------- main */

int orc_run(const uint32_t *s, const uint32_t *p, const uint32_t *o, uint64_t n, uint32_t V,
            uint32_t ms, int strategy, int clean, const char *projection,
            orc_cind **out, uint64_t *n_out, uint64_t **bin_keys_out, uint64_t *n_bin_out,
            orc_stats *st) {
    memset(st, 0, sizeof(*st));
    if (V >= (1u << 31)) return -1;
    int proj_s = strchr(projection, 's') != NULL;
    int proj_p = strchr(projection, 'p') != NULL;
    int proj_o = strchr(projection, 'o') != NULL;

    /* 1. unary condition counts (FrequentConditionPlanner.scala:488-508) */
    uint32_t *cnt = (uint32_t *)calloc((size_t)3 * V + 1, sizeof(uint32_t));
    for (uint64_t i = 0; i < n; ++i) { cnt[s[i]]++; cnt[(uint64_t)V + p[i]]++; cnt[2ull * V + o[i]]++; }
    uint8_t *freq = (uint8_t *)calloc((size_t)V + 1, 1); /* bit0 s, bit1 p, bit2 o */
    for (uint32_t v = 0; v < V; ++v) {
        for (int t = 0; t < 3; ++t)
            if (cnt[(uint64_t)t * V + v] >= ms) { freq[v] |= (uint8_t)(1u << t); st->n_freq_unary[t]++; }
    }
    free(cnt);

    /* 2. binary condition counts (CreatedReducedDoubleConditionCounts.scala:45-86) */
    u64map bmap;
    map_init(&bmap, 3 * n + 16);
    for (uint64_t i = 0; i < n; ++i) {
        int fs = freq[s[i]] & 1, fp = (freq[p[i]] >> 1) & 1, fo = (freq[o[i]] >> 2) & 1;
        if (fs + fp + fo < 2) continue;
        if (fs && fp) (*map_slot(&bmap, (2ull << 62) | ((uint64_t)s[i] << 31) | p[i], 1))++;
        if (fs && fo) (*map_slot(&bmap, (1ull << 62) | ((uint64_t)s[i] << 31) | o[i], 1))++;
        if (fp && fo) (*map_slot(&bmap, (0ull << 62) | ((uint64_t)p[i] << 31) | o[i], 1))++;
    }
    st->n_binary_keys = bmap.size;
    uint64_t nb = 0;
    for (uint64_t h = 0; h <= bmap.mask; ++h)
        if (bmap.keys[h] != ~0ULL && bmap.vals[h] >= ms) nb++;
    uint64_t *bkeys = (uint64_t *)xmalloc(nb * sizeof(uint64_t));
    nb = 0;
    for (uint64_t h = 0; h <= bmap.mask; ++h)
        if (bmap.keys[h] != ~0ULL && bmap.vals[h] >= ms) bkeys[nb++] = bmap.keys[h];
    map_free(&bmap);
    radix_sort_u64(bkeys, nb);
    st->n_freq_binary = nb;
    u64map bidx;
    map_init(&bidx, nb + 16);
    for (uint64_t b = 0; b < nb; ++b) *map_slot(&bidx, bkeys[b], 1) = (uint32_t)b;

    /* 3. join partners (CreateJoinPartners.scala:86-147), binary captures split into their unary
     *    components as every consumer does (CreateDependencyCandidates.scala:157-186) */
    const uint64_t capbits = 64 - __builtin_clzll((uint64_t)6 * V + nb + 1);
    uint64_t cap_records = 9 * n;
    uint64_t *rec = (uint64_t *)xmalloc(cap_records * sizeof(uint64_t));
    uint64_t nr = 0;
#define EMIT(join, cap) rec[nr++] = ((uint64_t)(join) << capbits) | (uint64_t)(cap)
    for (uint64_t i = 0; i < n; ++i) {
        uint32_t ts = s[i], tp = p[i], to = o[i];
        int fs = freq[ts] & 1, fp = (freq[tp] >> 1) & 1, fo = (freq[to] >> 2) & 1;
        uint32_t *b;
        if (proj_o) {
            if (fs) EMIT(to, 4ull * V + ts);             /* o[s] */
            if (fp) EMIT(to, 5ull * V + tp);             /* o[p] */
            if (fs && fp && (b = map_slot(&bidx, (2ull << 62) | ((uint64_t)ts << 31) | tp, 0)))
                EMIT(to, 6ull * V + *b);                 /* o[s,p] */
        }
        if (proj_p) {
            if (fs) EMIT(tp, 2ull * V + ts);             /* p[s] */
            if (fo) EMIT(tp, 3ull * V + to);             /* p[o] */
            if (fs && fo && (b = map_slot(&bidx, (1ull << 62) | ((uint64_t)ts << 31) | to, 0)))
                EMIT(tp, 6ull * V + *b);                 /* p[s,o] */
        }
        if (proj_s) {
            if (fp) EMIT(ts, 0ull * V + tp);             /* s[p] */
            if (fo) EMIT(ts, 1ull * V + to);             /* s[o] */
            if (fp && fo && (b = map_slot(&bidx, (0ull << 62) | ((uint64_t)tp << 31) | to, 0)))
                EMIT(ts, 6ull * V + *b);                 /* s[p,o] */
        }
    }
#undef EMIT
    map_free(&bidx);
    free(freq);
    st->n_records = nr;

    /* 4. capture groups: sort + unique (UnionJoinCandidates / UnionCombinedJoinCandidates) */
    radix_sort_u64(rec, nr);
    uint64_t nu = 0;
    for (uint64_t i = 0; i < nr; ++i)
        if (nu == 0 || rec[nu - 1] != rec[i]) rec[nu++] = rec[i];
    st->n_unique = nu;
    const uint64_t capmask = (1ull << capbits) - 1;
    const uint64_t ncap = 6ull * V + nb;
    uint32_t *support = (uint32_t *)calloc(ncap + 1, sizeof(uint32_t));
    uint64_t ng = 0;
    for (uint64_t i = 0; i < nu; ++i) {
        support[rec[i] & capmask]++;
        if (i == 0 || (rec[i] >> capbits) != (rec[i - 1] >> capbits)) ng++;
    }
    st->n_groups = ng;
    uint64_t *goff = (uint64_t *)xmalloc((ng + 1) * sizeof(uint64_t));
    uint32_t *gcap = (uint32_t *)xmalloc(nu * sizeof(uint32_t));
    ng = 0;
    for (uint64_t i = 0; i < nu; ++i) {
        if (i == 0 || (rec[i] >> capbits) != (rec[i - 1] >> capbits)) goff[ng++] = i;
        gcap[i] = (uint32_t)(rec[i] & capmask);
    }
    goff[ng] = nu;
    free(rec);

    /* transposed: capture -> groups (only captures with support >= ms can be dependents) */
    uint64_t *doff = (uint64_t *)xmalloc((ncap + 1) * sizeof(uint64_t));
    uint64_t acc = 0;
    for (uint64_t c = 0; c < ncap; ++c) {
        doff[c] = acc;
        if (support[c] >= ms) { acc += support[c]; st->n_freq_captures++; }
    }
    doff[ncap] = acc;
    uint32_t *dgrp = (uint32_t *)xmalloc(acc * sizeof(uint32_t));
    uint64_t *cur = (uint64_t *)xmalloc((ncap + 1) * sizeof(uint64_t));
    memcpy(cur, doff, (ncap + 1) * sizeof(uint64_t));
    for (uint64_t g = 0; g < ng; ++g)
        for (uint64_t i = goff[g]; i < goff[g + 1]; ++i)
            if (support[gcap[i]] >= ms) dgrp[cur[gcap[i]]++] = (uint32_t)g;
    free(cur);

    /* 5. per dependent: ref set = intersection over its groups of (group \ implied)
     *    (CreateAllCindCandidates.scala:106-121 + IntersectCindCandidates.scala:40-43).
     *    Dependents are split into chunks processed by OpenMP threads; each chunk's CINDs go to its own
     *    buffer and the buffers are concatenated in chunk (= dependent) order. */
    const uint64_t nchunk = ncap < 4096 ? 1 : 4096;
    orc_cind **cbuf = (orc_cind **)calloc(nchunk, sizeof(orc_cind *));
    uint64_t *ccnt = (uint64_t *)calloc(nchunk + 1, sizeof(uint64_t));
#pragma omp parallel
    {
        uint32_t *refs = NULL, *tmp = NULL;
        uint64_t refs_cap = 0;
#pragma omp for schedule(dynamic, 1)
        for (uint64_t ch = 0; ch < nchunk; ++ch) {
            uint64_t ccap = 256, nc = 0;
            orc_cind *cind = (orc_cind *)xmalloc(ccap * sizeof(orc_cind));
            const uint64_t a0 = ncap * ch / nchunk, a1 = ncap * (ch + 1) / nchunk;
            for (uint64_t a = a0; a < a1; ++a) {
                if (support[a] < ms) continue;
                /* trivial refs of a binary dep: its two unary components (Condition.isImpliedBy) */
                uint32_t triv1 = ~0u, triv2 = ~0u;
                int dep_bt = -1;
                uint32_t dv1 = 0, dv2 = 0;
                if (a >= 6ull * V) {
                    uint64_t key = bkeys[a - 6ull * V];
                    dep_bt = (int)(key >> 62);
                    dv1 = (uint32_t)((key >> 31) & 0x7fffffff);
                    dv2 = (uint32_t)(key & 0x7fffffff);
                    int t1, t2;
                    binary_components(dep_bt, &t1, &t2);
                    triv1 = (uint32_t)((uint64_t)t1 * V + dv1);
                    triv2 = (uint32_t)((uint64_t)t2 * V + dv2);
                }
                uint64_t nref = 0;
                for (uint64_t j = doff[a]; j < doff[a + 1]; ++j) {
                    uint64_t g = dgrp[j];
                    uint64_t k = goff[g + 1] - goff[g];
                    const uint32_t *gc = gcap + goff[g];
                    if (j == doff[a]) {
                        if (k > refs_cap) {
                            refs_cap = k * 2;
                            refs = (uint32_t *)realloc(refs, refs_cap * sizeof(uint32_t));
                            tmp = (uint32_t *)realloc(tmp, refs_cap * sizeof(uint32_t));
                        }
                        for (uint64_t i = 0; i < k; ++i) {
                            uint32_t r = gc[i];
                            if (r == a || r == triv1 || r == triv2) continue;
                            if (strategy == 0 && dep_bt >= 0 && r >= 6ull * V) {
                                /* literal Condition.isImpliedBy quirk for same-type binary captures:
                                 * ref X is "implied" by dep D when X.v1 == D.v2 (Condition.scala:35-43) */
                                uint64_t rk = bkeys[r - 6ull * V];
                                if ((int)(rk >> 62) == dep_bt && (uint32_t)((rk >> 31) & 0x7fffffff) == dv2) continue;
                            }
                            refs[nref++] = r;
                        }
                    } else {
                        /* merge-intersect sorted refs with sorted group */
                        uint64_t x = 0, y = 0, m = 0;
                        while (x < nref && y < k) {
                            if (refs[x] < gc[y]) x++;
                            else if (refs[x] > gc[y]) y++;
                            else { tmp[m++] = refs[x]; x++; y++; }
                        }
                        uint32_t *t = refs; refs = tmp; tmp = t;
                        nref = m;
                    }
                    if (nref == 0) break;
                }
                for (uint64_t i = 0; i < nref; ++i) {
                    if (nc == ccap) { ccap *= 2; cind = (orc_cind *)realloc(cind, ccap * sizeof(orc_cind)); }
                    cind[nc].dep = (uint32_t)a;
                    cind[nc].ref = refs[i];
                    cind[nc].support = support[a];
                    nc++;
                }
            }
            cbuf[ch] = cind;
            ccnt[ch] = nc;
        }
        free(refs); free(tmp);
    }
    uint64_t nc = 0;
    for (uint64_t ch = 0; ch < nchunk; ++ch) { uint64_t c = ccnt[ch]; ccnt[ch] = nc; nc += c; }
    ccnt[nchunk] = nc;
    orc_cind *cind = (orc_cind *)xmalloc(nc * sizeof(orc_cind));
#pragma omp parallel for schedule(dynamic, 16)
    for (uint64_t ch = 0; ch < nchunk; ++ch) {
        memcpy(cind + ccnt[ch], cbuf[ch], (ccnt[ch + 1] - ccnt[ch]) * sizeof(orc_cind));
        free(cbuf[ch]);
    }
    free(cbuf); free(ccnt);
    free(dgrp); free(doff); free(goff); free(gcap); free(support);
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
                uint64_t key = bkeys[r - U];
                int t1, t2;
                binary_components((int)(key >> 62), &t1, &t2);
                uint64_t c1 = (uint64_t)t1 * V + ((key >> 31) & 0x7fffffff);
                uint64_t c2 = (uint64_t)t2 * V + (key & 0x7fffffff);
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
                uint64_t key = bkeys[d - U];
                int t1, t2;
                binary_components((int)(key >> 62), &t1, &t2);
                uint64_t c1 = (uint64_t)t1 * V + ((key >> 31) & 0x7fffffff);
                uint64_t c2 = (uint64_t)t2 * V + (key & 0x7fffffff);
                if (ru) {
                    drop = bsearch_u64(s11, n11, (c1 << 32) | r) || bsearch_u64(s11, n11, (c2 << 32) | r)  /* R1 */
                        || bsearch_u64(s22c, n22c, (d << 32) | r);                                      /* R2 */
                } else {
                    drop = bsearch_u64(s12, n12, (c1 << 32) | r) || bsearch_u64(s12, n12, (c2 << 32) | r); /* R4 */
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
    st->n_cinds = nc;
    *out = cind;
    *n_out = nc;
    *bin_keys_out = bkeys;
    *n_bin_out = nb;
    return 0;
}

void orc_free(void *ptr) { free(ptr); }

/* threads stages 4-6 use (OMP_NUM_THREADS, else all cores) */
int orc_threads(void) { return omp_get_max_threads(); }
