/*
 * rdfind_hip.h -- C ABI of the MI355X-native RDFind CIND-discovery hot path (librdfind_hip.so).
 *
 * Plain C types only.  Each entry point replaces one operator boundary of the reference
 * (stratosphere/rdfind; ALG/ = rdfind-algorithm/src/main/scala/de/hpi/isg/sodap/rdfind/):
 *
 *   rdf_set_triples            the DataSet[RDFTriple] handed to the plan
 *                              (ALG/programs/RDFind.scala:220-237, RDFTriple ALG/data/RDFTriple.scala:7),
 *                              dictionary-encoded: one uint32 id space for s, p and o.
 *   rdf_frequent_conditions    FrequentConditionPlanner.constructFrequentConditionPlan
 *                              (ALG/plan/FrequentConditionPlanner.scala:33-122), called at
 *                              ALG/programs/RDFind.scala:290-296 (--use-fis).
 *   rdf_build_capture_groups   CreateJoinPartners (RichFlatMapFunction, ALG/operators/CreateJoinPartners.scala:23-147)
 *                              -> UnionJoinCandidates (ALG/operators/UnionJoinCandidates.scala:19-44)
 *                              -> UnionCombinedJoinCandidates (ALG/operators/UnionCombinedJoinCandidates.scala:17-31),
 *                              wired at ALG/programs/RDFind.scala:310-346.
 *   rdf_discover_cinds         TraversalStrategy.enhanceFlinkPlan (ALG/plan/TraversalStrategy.scala:28-33),
 *                              selected at ALG/programs/RDFind.scala:50-56 and called at :459, including
 *                              splitAndCleanCindSets / removeImpliedCinds (ALG/plan/TraversalStrategy.scala:45-168).
 *   rdf_copy_cinds             the DataSet[Cind] result (ALG/data/Cind.scala:12-31) before Cind.toString.
 *
 * Conventions (mirroring the reference's one-UDF-instance-per-task model):
 *   - inputs are borrowed and copied to HBM before the call returns (rdf_set_triples), or borrowed
 *     device pointers that must stay valid until the next rdf_set_triples* call;
 *   - results are library-owned and device-resident until copied out or the next call.  In HBM the
 *     result is CindSet-shaped (ALG/data/CindSet.scala:9-13): one u32 ref per CIND, grouped in runs that
 *     share a dependent (run table: start offset + dependent), 4 B per CIND; rdf_copy_cinds* expand it;
 *   - no exceptions cross the ABI: every call returns rdf_status (0 = OK, < 0 = error) and
 *     rdf_last_error() describes the last failure; errors are sticky per call, not per context;
 *   - a context is not thread-safe; different contexts (one per GPU) may run concurrently.
 */
#ifndef RDFIND_HIP_H
#define RDFIND_HIP_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef int32_t rdf_status;
#define RDF_OK 0
#define RDF_ERR_ARG (-1)      /* invalid argument (IllegalArgumentException in the reference) */
#define RDF_ERR_HIP (-2)      /* HIP runtime / device error */
#define RDF_ERR_OOM (-3)      /* device memory exhausted */
#define RDF_ERR_STATE (-4)    /* stage called out of order (IllegalStateException) */
#define RDF_ERR_LIMIT (-5)    /* input exceeds an implementation limit (e.g. >= 2^30 terms) */

/* rdf_discover_cinds flags */
#define RDF_CLEAN_IMPLIED 1u          /* --clean-implied: R1-R4 minimality (TraversalStrategy.scala:126-168) */
#define RDF_STRATEGY_ALL_AT_ONCE 2u   /* --traversal-strategy 0 semantics (literal Condition.isImpliedBy);
                                         default is strategy 1 (S2L) */
#define RDF_USE_ASSOCIATION_RULES 8u  /* rdf_run: --use-ars, rdf_association_rules between the first two stages */

typedef struct rdf_ctx rdf_ctx;

typedef struct {
    uint32_t min_support;
    uint32_t n_ar_suppressed;       /* --use-ars: frequent binary conditions whose captures the rules suppress */
    uint64_t n_frequent_unary[3];   /* frequent s / p / o conditions */
    uint64_t n_binary_keys;         /* distinct candidate binary conditions counted */
    uint64_t n_frequent_binary;     /* frequent binary conditions */
} rdf_fc_stats;

typedef struct {
    uint64_t n_records;             /* (join value, capture) join partners emitted */
    uint64_t n_frequent_records;    /* distinct records of captures with support >= min_support */
    uint64_t n_groups;              /* capture groups (join values) */
    uint64_t n_captures;            /* captures with support >= min_support (dependent candidates) */
    uint64_t n_unary_captures;
    uint64_t n_heavy_groups;        /* groups tracked as bitmask columns */
    uint64_t heavy_threshold;       /* minimum size of a heavy group */
    uint64_t n_sorted_records;      /* records the join-partner sort keeps after its first pass (an emission iteration's
                                       repeats dropped) */
    uint64_t n_join_ranges;         /* join-value ranges the groups were built in (1; more for inputs of >= 2^32/9
                                       triples, whose records exceed one sort: Flink's spilling groupBy, RDFind.scala:339-345) */
    uint64_t n_ranges_kept;         /* join ranges whose sorted records the second pass read back instead of emitting
                                       and sorting them again (0: none kept) */
} rdf_group_stats;

typedef struct {
    uint64_t n_cinds;               /* CINDs in the result */
    uint64_t n_explicit_raw;        /* raw CINDs of dependents with a light group */
    uint64_t n_light_chunks;
    uint64_t n_heavy_chunks;
    float ms_pivot, ms_light, ms_rules, ms_heavy;  /* device time per K6/K7 kernel family */
    uint64_t n_heavy_candidates;    /* pivot members scanned for binary dependents whose groups are all heavy */
    uint64_t n_class_members;       /* unary dependents whose groups are all heavy (emitted per mask class) */
    uint64_t n_classes;             /* distinct heavy bitmasks among them */
    uint64_t n_class_cinds;         /* CINDs emitted by the class path */
    uint64_t n_light_candidates;    /* pivot members of dependents with light groups (intersection candidates) */
    uint64_t n_light_entries;       /* (dependent, group) entries of those dependents */
} rdf_cind_stats;

/* Kernel-family device timers (HIP events on the context stream), see rdf_kernel_times. */
enum {
    RDF_T_UNARY = 0,    /* K1 unary condition counts (+ frequent-value count) */
    RDF_T_BINARY,       /* K2 binary condition counts + frequent-key extraction */
    RDF_T_EMIT,         /* K3 join-partner emission */
    RDF_T_SORT,         /* K4 radix sort of (join, capture) records */
    RDF_T_SUPPORT,      /* K5 distinct records, supports, frequent-capture compaction */
    RDF_T_GROUPS,       /* capture-group CSR + dependent -> group CSR */
    RDF_T_HEAVYMASK,    /* heavy-group selection, bitmask columns, binary components/parents */
    RDF_T_PIVOT,        /* K6 pivot selection */
    RDF_T_LIGHT,        /* K6 light-dependent intersection */
    RDF_T_ESORT,        /* sort of explicit pairs + CSR offsets */
    RDF_T_HCOUNT,       /* K6 heavy-only count pass (minimality fused) */
    RDF_T_RULES,        /* K7 minimality on explicit pairs */
    RDF_T_HWRITE,       /* K6 heavy-only write pass (minimality fused) */
    RDF_T_CLASS,        /* K6c mask classes of unary heavy-only dependents + filtered shared ref lists */
    RDF_T_CEMIT,        /* K6c streaming emission of the class ref lists */
    RDF_NUM_TIMERS
};

/* One result row: capture ids (see rdf_decode_capture) and the support of the dependent. */
typedef struct {
    uint32_t dep;
    uint32_t ref;
    uint32_t support;
} rdf_cind;

rdf_status rdf_ctx_create(int device, rdf_ctx** out);
void rdf_ctx_destroy(rdf_ctx* ctx);
const char* rdf_last_error(const rdf_ctx* ctx);
const char* rdf_version(void);

rdf_status rdf_set_triples(rdf_ctx* ctx, const uint32_t* s, const uint32_t* p, const uint32_t* o,
                           uint64_t n, uint32_t num_terms);
rdf_status rdf_set_triples_device(rdf_ctx* ctx, const uint32_t* d_s, const uint32_t* d_p, const uint32_t* d_o,
                                  uint64_t n, uint32_t num_terms);

/* --distinct-triples: `triples.distinct` (ALG/programs/RDFind.scala:284-287) on the resident triples, in HBM.
 * Keeps the first occurrence of every triple in input order; *n_distinct receives the new count and *ms
 * (optional) the device time.  The compacted triples are context-owned from then on. */
rdf_status rdf_distinct_triples(rdf_ctx* ctx, uint64_t* n_distinct, float* ms);

/* N-Triples ingest on the device: the `Parse triples` map (ALG/programs/RDFind.scala:196-237, rdf-converter's
 * NTriplesParser) plus dictionary encoding, replacing the host parser (rdfind_amd/ntriples.py, same rules).
 * text: the raw (decompressed) file bytes, '\n'-terminated lines; lines starting with '#' and blank lines are
 * skipped.  Term ids follow first appearance (line-major, then s, p, o).  The parsed triples become the resident
 * input; a malformed line fails with RDF_ERR_ARG naming it. */
#define RDF_NT_TABS 1u                 /* --tabs: tab-separated terms */
rdf_status rdf_parse_ntriples(rdf_ctx* ctx, const char* text, uint64_t nbytes, uint32_t flags, uint64_t* n_triples,
                              uint32_t* num_terms, float* ms);
/* Uses the dictionary of the last rdf_parse_ntriples as the formatting dictionary (rdf_set_dictionary without a
 * host round trip); RDF_ERR_STATE if triples were set another way since. */
rdf_status rdf_set_dictionary_parsed(rdf_ctx* ctx);
/* The dictionary of the last rdf_parse_ntriples: term id i is text[offsets[i] .. offsets[i] + lengths[i]). */
rdf_status rdf_copy_terms(rdf_ctx* ctx, uint64_t* offsets, uint32_t* lengths, uint64_t cap, uint64_t* n_copied);

/* Copies min(cap, n) resident triples to host arrays (e.g. after rdf_distinct_triples). */
rdf_status rdf_copy_triples(rdf_ctx* ctx, uint32_t* s, uint32_t* p, uint32_t* o, uint64_t cap, uint64_t* n_copied);

rdf_status rdf_frequent_conditions(rdf_ctx* ctx, uint32_t min_support, rdf_fc_stats* stats);
/* --use-ars: exact association rules between frequent conditions (FrequentConditionPlanner.findAssociationRules,
 * ALG/plan/FrequentConditionPlanner.scala:130-194).  Call between rdf_frequent_conditions and
 * rdf_build_capture_groups: the AR-implied binary conditions then produce no captures (CreateJoinPartners.scala:
 * 99-141), and rdf_discover_cinds leaves out the CINDs the reference does not produce with the rules
 * (CreateAllCindCandidates.scala:108-115 for strategy 0; SmallToLargeTraversalStrategy.scala:80-85 and the
 * candidate generation built on it for S2L). */
rdf_status rdf_association_rules(rdf_ctx* ctx, uint64_t* n_rules);
/* Sharded mode takes RDF_USE_ASSOCIATION_RULES in rdf_shard_begin: the rules come from the summed counts of every
 * rank's slice (one all-reduce), are identical on every rank, and rdf_copy_association_rules returns them there. */
/* One rule (AssociationRule, ALG/data/AssociationRule.scala:9-19; confidence is always 1): condition codes
 * s = 1, p = 2, o = 4 and term ids; support = the triple count of the binary condition. */
typedef struct {
    uint32_t antecedent_type;
    uint32_t consequent_type;
    uint32_t antecedent;
    uint32_t consequent;
    uint32_t support;
} rdf_assoc_rule;
rdf_status rdf_copy_association_rules(rdf_ctx* ctx, rdf_assoc_rule* out, uint64_t cap, uint64_t* n_copied);
rdf_status rdf_association_rule_count(rdf_ctx* ctx, uint64_t* n);
/* projection: any combination of 's', 'p', 'o' (--projection, default "spo"). */
rdf_status rdf_build_capture_groups(rdf_ctx* ctx, const char* projection, rdf_group_stats* stats);
rdf_status rdf_discover_cinds(rdf_ctx* ctx, uint32_t flags, rdf_cind_stats* stats);

/* Paged discovery, for results larger than HBM (the reference streams its output to the sink, ALG/programs/RDFind.scala:
 * 507-520): after rdf_build_capture_groups, rdf_discover_cinds_paged prepares the run with a working-memory budget per
 * page (page_bytes; 0 = a quarter of the free HBM) and every rdf_next_page makes the next page the current result
 * (rdf_get_result_layout, rdf_copy_result_compact, rdf_cind_checksum, the row accessors).  Page 0 holds the unary
 * dependents, each later page a range [*first_dep, *end_dep) of binary dependents (compact capture ids); *done = 1 once
 * the pages are exhausted (the current result is then empty).  The pages partition rdf_discover_cinds's result.
 * Single GPU. */
rdf_status rdf_discover_cinds_paged(rdf_ctx* ctx, uint32_t flags, uint64_t page_bytes, rdf_cind_stats* stats);
rdf_status rdf_next_page(rdf_ctx* ctx, uint32_t* done, uint64_t* first_dep, uint64_t* end_dep);

/* Whole pipeline on the current triples (the three stages above). */
rdf_status rdf_run(rdf_ctx* ctx, uint32_t min_support, const char* projection, uint32_t flags,
                   rdf_fc_stats* fc, rdf_group_stats* gs, rdf_cind_stats* cs);

rdf_status rdf_cind_count(rdf_ctx* ctx, uint64_t* n);
/* Copies min(cap, count) rows to host memory; *n_copied receives the number copied. */
rdf_status rdf_copy_cinds(rdf_ctx* ctx, rdf_cind* out, uint64_t cap, uint64_t* n_copied);

/* The result as CindSet-shaped id-records (4 B per CIND): refs[n_refs] (compact capture ids), the run table
 * (run r holds refs [runoff[r], runoff[r+1]) of dependent rundep[r]; runoff has n_runs + 1 entries) and, per
 * compact capture id, its external capture id (see rdf_decode_capture) and support.  Null pointers skip a part;
 * pinned host memory lets the copies run at the link rate. */
rdf_status rdf_result_sizes(rdf_ctx* ctx, uint64_t* n_refs, uint64_t* n_runs, uint64_t* n_captures);
rdf_status rdf_copy_result_raw(rdf_ctx* ctx, uint32_t* refs, uint64_t* runoff, uint32_t* rundep, uint32_t* capture_ids,
                               uint32_t* supports);

/* The compact result: what rdf_discover_cinds leaves in HBM, without expanding shared ref lists.  A CindSet
 * (ALG/data/CindSet.scala:9-13: one dependent, its support, its ref conditions) per dependent, in two forms:
 *   - explicit runs: refs[runoff[r] .. runoff[r+1]) are the refs of dependent rundep[r] (n_runs runs, n_refs refs);
 *   - shared lists: members[i] = list << 32 | dependent; that dependent's refs are list_refs[list_off[list] ..
 *     list_off[list+1]) except itself (n_members members of n_lists lists; dependents whose capture groups all
 *     have the same heavy-group bitmask share one filtered list).
 * Every id is a compact capture id: capture_ids[id] is its capture id (rdf_decode_capture) and supports[id] the
 * dependent's support.  n_cinds = n_refs + sum over members of the list length minus the member itself.  This
 * is the id-record hand-over the metric's T_disc ends with; the row accessors below expand it. */
typedef struct {
    uint64_t n_cinds;
    uint64_t n_refs;
    uint64_t n_runs;
    uint64_t n_lists;
    uint64_t n_list_refs;
    uint64_t n_members;
    uint64_t n_captures;
} rdf_result_layout;
rdf_status rdf_get_result_layout(rdf_ctx* ctx, rdf_result_layout* layout);
/* Null pointers skip a part.  Sizes: refs n_refs, runoff n_runs + 1, rundep n_runs, list_refs n_list_refs,
 * list_off n_lists + 1, members n_members, capture_ids and supports n_captures. */
rdf_status rdf_copy_result_compact(rdf_ctx* ctx, uint32_t* refs, uint64_t* runoff, uint32_t* rundep, uint32_t* list_refs,
                                   uint64_t* list_off, uint64_t* members, uint32_t* capture_ids, uint32_t* supports);

/* Early hand-over (optional; pipelining of the sink with the computation).  Registers page-locked host buffers that
 * every later unpaged single-GPU rdf_discover_cinds / rdf_run may fill on a copy stream while it still computes: the
 * capture table (capture_ids, supports: up to capture_cap entries) when the discovery starts, the explicit refs (up to
 * refs_cap) and the explicit dependents' runs (runoff / rundep [0, n_captures), runs_cap >= n_captures) once their
 * minimality rules have run, before the class stage.  A later rdf_copy_result_compact given the
 * same pointers copies only what is left and returns when everything has arrived; the buffers must not be read before
 * it returns.  Parts that do not fit are copied by rdf_copy_result_compact as before.  Null pointers / zero capacities
 * unregister.  The reference's sink likewise consumes results while the job still runs (ALG/programs/RDFind.scala:507-520). */
rdf_status rdf_set_handover(rdf_ctx* ctx, uint32_t* refs, uint64_t refs_cap, uint64_t* runoff, uint32_t* rundep,
                            uint64_t runs_cap, uint32_t* capture_ids, uint32_t* supports, uint64_t capture_cap);

/* refs[offset, offset + count) of the compact result (the explicit ref part, n_refs in all) -> refs; *n_copied = the
 * refs copied (fewer at the end).  A streaming sink hands a large page over through one bounded staging buffer
 * (the reference's sink consumes its output as it comes, ALG/programs/RDFind.scala:507-520). */
rdf_status rdf_copy_result_refs(rdf_ctx* ctx, uint64_t offset, uint64_t count, uint32_t* refs, uint64_t* n_copied);

/* The same copy, queued on the context's copy stream instead of waiting for it: the refs of a page leave while the
 * next rdf_next_page computes (its emission waits on the GPU for the copy before it overwrites them; only a page that
 * needs a larger output buffer waits on the host).  `refs` must be page-locked (rdf_host_alloc) and stay untouched
 * until rdf_handover_wait, or until another copy call, returns.  Copies queued this way into one buffer complete in
 * order.  Replaces the page-by-page synchronous sink of ALG/programs/RDFind.scala:507-520 with an overlapped one. */
rdf_status rdf_copy_result_refs_async(rdf_ctx* ctx, uint64_t offset, uint64_t count, uint32_t* refs, uint64_t* n_copied);

/* Wait until every queued asynchronous copy (rdf_copy_result_refs_async, the early hand-over) has reached the host. */
rdf_status rdf_handover_wait(rdf_ctx* ctx);

/* Result form of the compact hand-over, from the next discovery on.  RDF_FORM_EXPANDED (default): every non-class ref
 * is an explicit ref.  RDF_FORM_HEAVY_BITS: the refs of the heavy-only binary dependents (checked against their mask
 * class's shared list, K6d) leave as one 64-bit survivor word per chunk of 64 list candidates instead of one u32 per
 * CIND: rdf_get_result_layout then counts only the explicit refs and runs, and rdf_copy_result_heavy hands over the
 * chunks (dependent, position in the class lists `list_refs`, bits: bit b set = the CIND dependent ⊆ list_refs[pos + b]).
 * Paged results send the class lists with the first page only; the later pages' chunks index them.  The device-side
 * result (row accessors, checksums, formatting) is unchanged.  A CindSet per dependent either way
 * (ALG/data/CindSet.scala:9-13). */
#define RDF_FORM_EXPANDED 0u
#define RDF_FORM_HEAVY_BITS 1u
rdf_status rdf_set_result_form(rdf_ctx* ctx, uint32_t form);
rdf_status rdf_heavy_chunk_count(rdf_ctx* ctx, uint64_t* n_chunks);
rdf_status rdf_copy_result_heavy(rdf_ctx* ctx, uint32_t* deps, uint64_t* pos, uint64_t* bits);

/* Page-locked host memory (hipHostMalloc) for hand-over buffers: the copies above then run at the link rate.
 * Returns null on failure; free with rdf_host_free. */
void* rdf_host_alloc(uint64_t bytes);
void rdf_host_free(void* ptr);

/* One result row in the reference's Cind shape (ALG/data/Cind.scala:12-15: depCaptureType, depConditionValue1/2,
 * refCaptureType, refConditionValue1/2, support), with term ids for the condition values; value2 = UINT32_MAX
 * stands for the reference's null (unary capture).  Seven uint32 fields, no padding. */
typedef struct {
    uint32_t dep_capture_type;
    uint32_t dep_value1;
    uint32_t dep_value2;
    uint32_t ref_capture_type;
    uint32_t ref_value1;
    uint32_t ref_value2;
    uint32_t support;
} rdf_cind_row;
/* Decoded rows [offset, offset+count) of the result (clipped), decoded on the device; *n_copied receives the number
 * copied.  This is what a JNI/FFI caller turns into Cind objects (no capture-id arithmetic on the caller side). */
rdf_status rdf_copy_cinds_decoded(rdf_ctx* ctx, uint64_t offset, rdf_cind_row* out, uint64_t count, uint64_t* n_copied);

/* Copies rows [offset, offset+count) of the result (clipped); *n_copied receives the number copied. */
rdf_status rdf_copy_cinds_range(rdf_ctx* ctx, uint64_t offset, rdf_cind* out, uint64_t count, uint64_t* n_copied);
/* Order-independent checksum of the result set: sum over rows of mix64(((dep << 32) | ref) + support * 0x9E3779B97F4A7C15)
 * (external capture ids; the C oracle's streamed mode computes the same sum without materializing rows). */
rdf_status rdf_cind_checksum(rdf_ctx* ctx, uint64_t* checksum);

/* Capture ids: unary type t (codes 10,12,17,20,33,34) with value v -> t*V + v; binary capture b
 * (codes 14,21,35) -> 6V + b.  Decodes to the capture code and its condition values
 * (value2 = UINT32_MAX for unary captures). */
rdf_status rdf_decode_capture(rdf_ctx* ctx, uint32_t capture, uint32_t* code, uint32_t* value1, uint32_t* value2);
/* Frequent binary condition keys (bt << 62 | v1 << 31 | v2), indexed by b. */
rdf_status rdf_binary_key_count(rdf_ctx* ctx, uint64_t* n);
rdf_status rdf_copy_binary_keys(rdf_ctx* ctx, uint64_t* out, uint64_t cap);

/*
 * Output formatting on the device (replaces the host-side Cind.toString / TextOutputFormat write,
 * ALG/data/Cind.scala:29-31 and ALG/programs/RDFind.scala:507-520).  The caller uploads its dictionary once:
 * term t is heap[offsets[t], offsets[t+1]) (UTF-8 bytes, offsets[n_terms] == heap_bytes).  Lines are
 * "<dep> < <ref> (support=<n>)\n" with ConditionCodes.prettyPrint captures ("s[p=<term>]",
 * "o[s=<term>,p=<term>]"), for result rows [offset, offset+count) in result order.
 */
rdf_status rdf_set_dictionary(rdf_ctx* ctx, const char* heap, uint64_t heap_bytes, const uint64_t* offsets,
                              uint64_t n_terms);
/* Bytes the lines of rows [offset, offset+count) take. */
rdf_status rdf_format_size(rdf_ctx* ctx, uint64_t offset, uint64_t count, uint64_t* bytes);
/* Writes those lines to out (host memory, cap bytes); *bytes receives their size.  RDF_ERR_ARG if cap is
 * smaller (nothing written). */
rdf_status rdf_format_cinds(rdf_ctx* ctx, uint64_t offset, uint64_t count, char* out, uint64_t cap, uint64_t* bytes);

/* Statistics of the last completed run (single-GPU or sharded). */
rdf_status rdf_last_stats(rdf_ctx* ctx, rdf_fc_stats* fc, rdf_group_stats* gs, rdf_cind_stats* cs);

/*
 * Sharded multi-GPU mode (the reference's --dop parallelism over Flink task slots).
 * With RDF_SHARD_LOCAL_SLICE the resident triples are this rank's slice of the input (any partition of the
 * triples over the ranks, one dictionary); without it every rank holds all triples and takes rows
 * [n * rank / nranks, n * (rank + 1) / nranks).  Condition counts are summed over ranks (unary and binary: the
 * slice's nonzero (key, count) partials all-to-all'd to the key's owner, frequent keys all-gathered), then
 * each triple travels to the ranks owning its join values (hash(join) % nranks), so rank r builds the capture
 * groups of its join values and owns the dependents d with dep_owner(d) == r (a hash).  The library stops at every
 * collective and describes it in an rdf_exchange; the caller performs it (torch.distributed over RCCL,
 * see rdfind_amd/distributed.py) and hands the result back:
 *
 *     rdf_shard_begin(ctx, rank, nranks, min_support, projection, flags);
 *     for (;;) {
 *         rdf_shard_step(ctx, &x);               // runs device work up to the next collective
 *         if (x.op == RDF_X_DONE) break;
 *         rdf_shard_export(ctx, send);           // x.count elements of x.elem_bytes (device or host memory)
 *         ... collective(send -> recv) ...
 *         rdf_shard_import(ctx, recv, n_recv);   // all-reduce: x.count; all-gather: concatenation in rank
 *     }                                          // order; all-to-all: concatenation of what each rank sent here
 *
 * Afterwards rdf_cind_count / rdf_copy_cinds* return this rank's CINDs (those of its own dependents);
 * the union over ranks equals the single-GPU result.  Replaces the reference's hash-partitioned
 * shuffles between the capture-group, candidate-merging and minimality operators
 * (ALG/plan/AllAtOnceTraversalStrategy.scala:62-65 combine, ALG/plan/TraversalStrategy.scala:126-168).
 */
#define RDF_MAX_RANKS 64
#define RDF_SHARD_LOCAL_SLICE 4u   /* rdf_shard_begin flags: the resident triples are this rank's input slice */
enum {
    RDF_X_DONE = 0,
    RDF_X_ALLREDUCE_SUM_U32 = 1,   /* element-wise sum, uint32 */
    RDF_X_ALLREDUCE_SUM_U64 = 2,   /* element-wise sum, uint64 */
    RDF_X_ALLREDUCE_MIN_U64 = 3,   /* element-wise minimum, values < 2^63 */
    RDF_X_ALLGATHERV_U64 = 4,      /* variable-length all-gather, uint64 */
    RDF_X_ALLTOALLV_U64 = 5        /* variable-length all-to-all, uint64; send_counts per destination */
};
typedef struct {
    int32_t op;
    uint32_t elem_bytes;
    uint64_t count;                          /* elements this rank contributes */
    uint64_t send_counts[RDF_MAX_RANKS];     /* RDF_X_ALLTOALLV_U64: elements for rank r, consecutive */
} rdf_exchange;

rdf_status rdf_shard_begin(rdf_ctx* ctx, uint32_t rank, uint32_t nranks, uint32_t min_support, const char* projection,
                           uint32_t flags);
rdf_status rdf_shard_step(rdf_ctx* ctx, rdf_exchange* x);
rdf_status rdf_shard_export(rdf_ctx* ctx, void* dst);
rdf_status rdf_shard_import(rdf_ctx* ctx, const void* src, uint64_t count);

/*
 * Sharded ingest (-dop N; the reference splits its input per task, FLK/persistence/MultiFileTextInputFormat.java:49-100,
 * and parses in parallel, ALG/programs/RDFind.scala:196-237): rdf_shard_parse_begin parses this rank's part of the
 * input (whole lines) into a local dictionary, then the same rdf_shard_step / export / import loop as above runs
 * the dictionary exchange: every local term goes to the rank owning its hash, which deduplicates the terms it
 * receives (byte-verified) and assigns global ids (owner base + first-arrival rank), and the ids come back.  At
 * RDF_X_DONE the resident triples are this rank's slice in the global id space (rdf_num_terms = all distinct terms),
 * ready for rdf_shard_begin with RDF_SHARD_LOCAL_SLICE.  After that run, rdf_shard_dictionary_begin + the loop give
 * every rank the formatting dictionary of the terms its output lines can name (the values of the frequent
 * conditions, gathered from their owners); rdf_dictionary_terms reads terms of it back.
 */
rdf_status rdf_shard_parse_begin(rdf_ctx* ctx, uint32_t rank, uint32_t nranks, const char* text, uint64_t nbytes,
                                 uint32_t flags, uint64_t* n_triples);
rdf_status rdf_shard_dictionary_begin(rdf_ctx* ctx);
rdf_status rdf_num_terms(rdf_ctx* ctx, uint32_t* n);
/* offsets[n + 1]: term ids[i] is out[offsets[i], offsets[i+1]); RDF_ERR_ARG (offsets filled) if cap is too small. */
rdf_status rdf_dictionary_terms(rdf_ctx* ctx, const uint32_t* ids, uint64_t n, char* out, uint64_t cap, uint64_t* offsets);

/* Device time (ms) of the last call of each stage: [0] fc, [1] groups, [2] cinds. */
rdf_status rdf_stage_times(rdf_ctx* ctx, float* ms3);
/* Device time (ms) of each kernel family (RDF_T_*) in the last calls; count <= RDF_NUM_TIMERS. */
rdf_status rdf_kernel_times(rdf_ctx* ctx, float* ms, int count);
/* Synchronise the context stream. */
rdf_status rdf_sync(rdf_ctx* ctx);
/* Device memory (bytes) the context holds right now (its HBM buffers and scratch). */
rdf_status rdf_device_bytes(rdf_ctx* ctx, uint64_t* bytes);
/* Releases every per-run device buffer, keeping only the resident triples and the formatting dictionary (e.g. after
 * rdf_discover_cinds failed with RDF_ERR_OOM, before a paged run).  The context is back at the "triples set" stage:
 * rdf_frequent_conditions comes next. */
rdf_status rdf_release_scratch(rdf_ctx* ctx);

#ifdef __cplusplus
}
#endif
#endif /* RDFIND_HIP_H */
