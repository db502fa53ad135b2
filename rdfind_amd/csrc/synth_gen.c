/*
 * libsynth.so: counter-based synthetic RDF rows for the large Zipf configurations (bench/test input only).
 *
 * Row i of a configuration depends only on (seed, i): every uniform it needs is a mix64 hash of (seed, i, k).
 * So any row range is generated independently and in parallel, and the union of N ranks' row ranges is the
 * same input whatever N is (rdfind_amd/synth.py zipf_rows).  The distributions are those of synth.zipf_rdf:
 * Zipf ranks by the continuous inverse CDF, rdf:type rows with a class object, literal objects, entity objects.
 */
#include <math.h>
#include <stdint.h>

static inline uint64_t mix64(uint64_t x) {
    x ^= x >> 30;
    x *= 0xBF58476D1CE4E5B9ull;
    x ^= x >> 27;
    x *= 0x94D049BB133111EBull;
    x ^= x >> 31;
    return x;
}

/* uniform in [0, 1) from the top 53 bits */
static inline double unit(uint64_t seed, uint64_t row, uint64_t k) {
    const uint64_t h = mix64(seed ^ mix64(row * 8 + k + 0x9E3779B97F4A7C15ull));
    return (double)(h >> 11) * (1.0 / 9007199254740992.0);
}

/* rank in [0, n) with P(rank = r) ~ (r + 1)^-alpha (synth._zipf_ranks) */
static inline uint64_t zipf(double u, uint64_t n, double alpha) {
    double x;
    if (fabs(alpha - 1.0) < 1e-9) {
        x = pow((double)(n + 1), u);
    } else {
        const double a = 1.0 - alpha;
        x = pow((pow((double)n + 1.0, a) - 1.0) * u + 1.0, 1.0 / a);
    }
    int64_t r = (int64_t)floor(x) - 1;
    if (r < 0) r = 0;
    if ((uint64_t)r >= n) r = (int64_t)n - 1;
    return (uint64_t)r;
}

typedef struct {
    uint64_t seed;
    uint32_t t_type, t_pred, t_cls, t_ent, t_lit;      /* first term id of each range */
    uint32_t n_pred, n_cls, n_ent, n_lit;
    double pred_alpha, subj_alpha, class_frac, class_alpha, literal_frac, lit_alpha, obj_alpha;
} synth_params;

/* rows [row0, row0 + n) -> s, p, o */
void synth_zipf_rows(const synth_params *q, uint64_t row0, uint64_t n, uint32_t *s, uint32_t *p, uint32_t *o) {
#pragma omp parallel for schedule(static)
    for (int64_t j = 0; j < (int64_t)n; ++j) {
        const uint64_t i = row0 + (uint64_t)j;
        const double kind = unit(q->seed, i, 1);
        const int is_cls = kind < q->class_frac;
        const int is_lit = !is_cls && kind < q->class_frac + q->literal_frac;
        s[j] = q->t_ent + (uint32_t)zipf(unit(q->seed, i, 0), q->n_ent, q->subj_alpha);
        p[j] = is_cls ? q->t_type : q->t_pred + (uint32_t)zipf(unit(q->seed, i, 2), q->n_pred, q->pred_alpha);
        if (is_cls) o[j] = q->t_cls + (uint32_t)zipf(unit(q->seed, i, 3), q->n_cls, q->class_alpha);
        else if (is_lit) o[j] = q->t_lit + (uint32_t)zipf(unit(q->seed, i, 3), q->n_lit, q->lit_alpha);
        else o[j] = q->t_ent + (uint32_t)zipf(unit(q->seed, i, 3), q->n_ent, q->obj_alpha);
    }
}
