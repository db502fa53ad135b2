// librdfind_hip.so: C-ABI host orchestration of the MI355X CIND-discovery pipeline.
// See include/rdfind_hip.h for the boundary and DESIGN.md for the data layout in HBM.
#include <algorithm>
#include <cstdio>
#include <cstring>
#include <cstdlib>
#include <string>
#include <chrono>
#include <vector>
#include <utility>
#include <initializer_list>
#include <unordered_map>

#include "../../include/rdfind_hip.h"
#include "primitives.hpp"
#include "kernels.inl"

using namespace rdf;

#define RDF_VERSION "rdfind_amd 0.1 (gfx950)"

struct rdf_ctx {
    int device = 0;
    hipStream_t stream = nullptr;
    std::string err;
    Workspace ws;

    // device scalars + pinned host mirror
    DevBuf scal;
    u64* hscal = nullptr;
    u64* hread = nullptr;   // pinned, device-mapped: k_gather_scalars writes the read-back scalars here directly
    u64* hread_d = nullptr; // its device address

    // triples
    DevBuf ts, tp, to;
    DevBuf dtab, dkeep, dpos, xs, xp, xo;  // --distinct-triples: slot table, keep flags, positions, compacted copy
    // N-Triples ingest: text, line/term arrays, dictionary table, term table
    DevBuf ntext, ncnt, ncoff, nlstart, ntstart, ntlen, nvalid, nlpos, nhv, nslot, ntab, nrep, nfirst, nfid, nterm_off, nterm_len;
    u64 n_terms_parsed = 0;  // rows of nterm_off/nterm_len (rdf_copy_terms)
    bool parsed_dict = false;  // the resident triples' ids are the last parse's dictionary
    const u32 *s = nullptr, *p = nullptr, *o = nullptr;
    u64 n = 0;
    u32 V = 0;
    int stage = 0;  // 0 none, 1 triples, 2 fc, 3 groups, 4 cinds

    // frequent conditions
    u32 ms = 1;
    DevBuf frank, fval, fext;
    u32 U = 0, Us = 0, Up = 0;
    DevBuf cnt, tkeys, tcnt, bkeys, bkeys_tmp, lkeys, lvals, flags, pos;
    u64 B = 0, lcap = 0;
    std::vector<u64> h_bkeys;
    bool h_bkeys_valid = false;
    bool force_global_counts = false;
    bool allow_hclass = true;
    u64 heavy_min = 64;  // smaller groups are cheaper to verify by binary search than as bit columns
    // --use-ars (rdf_association_rules): rules (5 u32 each), per-condition counts, unary dependent -> implied ref
    bool ar_on = false;
    u64 n_rules = 0;
    DevBuf arcnt, ar_bits, ar_rules, arref;  // arcnt: triple counts of the frequent unary | binary conditions

    // capture groups
    DevBuf rec, rec_tmp, support, fidx, fcap, info, fk, fk_tmp, fpos, cstart, skip, gflag, gexcl, goff, gcap, gmap, csup, doff, dcur, dgrp;
    DevBuf hist, heavy_list, hbit, bcomp, bkeyc, pcnt, poff, pcur, plist;
    DevBuf jhist, rsup, offp;  // capture groups built in join-value ranges (g_build_ranges)
    DevBuf jbh;                // ... the emission blocks' join-bucket histograms (k_emit_join_bhist)
    DevBuf lsup;               // sharded join ranges: this rank's supports (the all-reduce replaces c->support)
    struct JoinRange { u32 lo, hi; u64 recs; };
    std::vector<JoinRange> jranges;  // the current build's join ranges (pass 1 -> pass 2)
    u64 jr_cap_rec = 1;              // records of the largest range (the range scratch's size)
    // pass 1's sorted records of every range, kept for pass 2 when they fit next to the range scratch (pass 2 then
    // neither re-emits nor re-sorts a range); RDFIND_RANGE_KEEP=0: always re-emit
    DevBuf rstore;
    std::vector<u64> jr_seg, jr_J;   // range k's slots in rstore start at jr_seg[k]; its sorted records
    bool jr_keep = false, range_keep = true;
    u64 peak_bytes = 0;              // RDFIND_MEM_REPORT: the largest sum of the buffers' sizes so far
    DevBuf jrmap;                    // the kept range build: the ranges' first join values and first join buckets
    // light dependents with identical group lists (d_light_dedup): keys, key table, class representatives, counts
    DevBuf ukey, utab, urep, ucnt, unoff, uebin, umem;
    u32 dup_min = 256;               // RDFIND_DUP_MIN: the shortest group list that looks for an equal one
    u64 u1_radix_min = 0;            // RDFIND_U1_RADIX_MIN: 3n from which K1 takes its radix form (0: the rule)
    int light_dedup = -1;            // RDFIND_LIGHT_DEDUP: 0 every light dependent verified on its own, 1 once per class
                                     // of equal group lists, unset: classes where the light pass stages (c2-like inputs)
    u64 n_dedup_members = 0;         // light dependents that took their representative's refs (last discovery)
    bool dedup_pending = false;      // d_light_dedup ran: d_dedup_expand reads the member count
    bool sh_ranged = false;          // the sharded build of this run goes in join ranges (sh_phase14 -> sh_phase1)
    u64 sh_m = 0;                    // sharded: triples received for this rank's join shard (wts / wtp / wto)
    std::string test_fail_launch;    // RDFIND_TEST_FAIL_LAUNCH: a kernel launched with an invalid configuration (test hook)
    bool test_oom_discovery = false; // RDFIND_TEST_OOM_DISCOVERY: rdf_discover_cinds fails with RDF_ERR_OOM (test hook)
    int test_fail_rank = -1, test_fail_phase = -1;  // RDFIND_TEST_FAIL_SHARD=rank:phase: that rank's rdf_shard_step fails
                                                    // with RDF_ERR_OOM at that phase (test hook: cross-rank failure agreement)
    int holder_qbits = 2;            // RDFIND_HOLDER_Q: pivot-holder election on log-size buckets (holder_key; 0: exact)
    bool hot_balance = true;         // RDFIND_HOT_BALANCE=0: every join value's owner by hash (no hot table)
    DevBuf hot, hotc;                // hot join values' owners (open-addressing table), this owner's candidates
    u32 hot_mask = 0;                // table slots - 1 (0 with hot_n == 0: no table)
    u64 hot_n = 0, sh_Bu = 0;        // hot values in the table; this owner's frequent unary keys (phase 16 -> 18)
    u64 group_range_records = 0;  // RDFIND_GROUP_RANGE test hook: records per join range (0: automatic)
    u64 n_group_ranges = 1;
    u64 J = 0, Jf = 0, G = 0, J_emit = 0;  // J: distinct-within-iteration records sorted; J_emit: records emitted
    u32 C = 0, Cu = 0, nheavy = 0;
    u64 heavy_threshold = 0;
    int capbits = 0, joinbits = 0;
    u64 *rec_sorted = nullptr;

    // cinds
    DevBuf pivot, nchl, nchh, choffl, choffh, epairs, epairs_tmp, eoff, hcounts, hoff, hbits, cbits, hown, cown, sbase, dcls, crep, out, stage_rows;
    DevBuf dheap, dtoff, cslen, csoff, cstr, flen, floff, fbuf;  // output formatting (K8)
    u64 dict_terms = 0, run_id = 0, capstr_run = ~0ull;
    DevBuf drows;           // decoded Cind-shaped rows (rdf_copy_cinds_decoded)
    DevBuf ppart;           // per-block partial sums of the pivot statistics
    DevBuf runoff, rundep;  // output run table: run r holds refs [runoff[r], runoff[r+1]) of dependent rundep[r]
    DevBuf nitl, itoffl, dead, ebin, pseg, psegoff, pbest, pnl;
    DevBuf lsig;          // light-group signatures (SIG_W words per compact capture), computed by the pivot pass
    DevBuf brkeys2, bstart2;  // K2 records re-partitioned into sub-buckets (k_b2_split) and their starts
    DevBuf ginfo;  // group -> size | heavy bit (k_group_info)
    DevBuf gsums;  // sum of light group sizes, of their squares (k_group_info)
    bool light_stage = false;  // k_light_stage: stage small light groups in LDS rows (chosen per run)
    bool light_hiocc = false;  // k_light_plain_hi: the plain variant at 6 waves per SIMD (LIGHT_HIOCC_*)
    u64 light_wmean = 0;       // member-weighted mean light group size of the run (k_group_info sums)
    DevBuf piv2;   // dependent -> second pivot (smallest light group after the pivot)
    DevBuf pivx;   // dependent -> the next PIV_EXTRA light groups after the second pivot (k_light plain only)
    bool pivx_on = false;
    int pivx_kept = 0;  // extra pivots the pivot pass computed this run (PIV_EXTRA_PLAIN or PIV_EXTRA)
    int light_npx = 0;  // ... and how many k_light checks
    DevBuf gdrow, dlist, dbits;  // dense light groups: group -> bitmap row, row -> group, the bitmaps
    u32* dbits_p = nullptr;      // the bitmaps in use (dbits)
    DevBuf iflag, iexcl, iorder; // k_light's issue order (k_light_long_flags / k_light_order)
    hipStream_t side = nullptr;  // k_light_packed beside k_light (their slots are disjoint), joined before the compaction
    hipEvent_t ev_fork = nullptr, ev_join = nullptr;
    // early hand-over (rdf_set_handover): pinned host buffers the unpaged discovery fills on a copy stream while it still
    // computes -- the capture table as the discovery starts, the explicit refs once the rules have run (before the
    // class stage); rdf_copy_result_compact then copies only the rest
    hipStream_t hstream = nullptr;
    hipEvent_t hv_ev = nullptr;
    uint32_t *hv_refs = nullptr, *hv_capid = nullptr, *hv_sup = nullptr, *hv_rundep = nullptr;
    uint64_t* hv_runoff = nullptr;
    u64 hv_refs_cap = 0, hv_cap_cap = 0, hv_runs_cap = 0;
    u64 hv_runs_n = ~0ull;       // explicit runs [0, hv_runs_n) copied early (runoff and rundep; ~0: none)
    u64 hv_refs_n = ~0ull;       // refs copied early by the current result (~0: none)
    bool hv_caps_done = false;   // capture ids and supports copied early
    bool hv_pending = false;     // copies queued on hstream not yet waited for
    // paged hand-over (rdf_copy_result_refs_async): a page's refs leave on hstream while the next page computes; the
    // next page's emission waits for hv_done on the GPU before it writes `out` (a growing `out` waits on the host)
    hipEvent_t hv_done = nullptr;
    bool hv_gpu_wait = false;
    bool dense_on = false;
    u64 dwords = 0, n_dense = 0;
    int dense_div = -1;                   // RDFIND_DENSE (0: no bitmaps; -1: by input, d_dense_flags)
    bool dense_flagged = false;           // d_dense_flags numbered rows this run (d_dense_build fills them)
    u64 dense_min = LIGHT_DENSE_MIN;      // RDFIND_DENSE_MIN (test hook: bitmaps for small groups too)
    bool sig_on = false;  // lsig holds this run's signatures (RDFIND_SIG=0 turns the filter off)
    bool sig_packed = false;  // the packed light path tests them too (RDFIND_SIG=1; default 2: k_light only)
    bool piv2_on = false;     // piv2 holds this run's second pivots
    bool piv2_packed = true;  // ... and the packed light path checks them first too (RDFIND_PIV2=2: k_light only)
    DevBuf ctab, cflag, ccid, ckeys, ckeys_tmp, coff, cmask, cpiv, cnch, cchoff, ccnt, lwoff, clists, cself, cmcnt, cobase,
        ctiles, ctoff;
    u64 n_class_members = 0, n_classes = 0, n_class_out = 0;
    // compact result: the class part (members x shared lists) is expanded into `out` only on demand
    bool class_pending = false;
    u64 pend_NT = 0, pend_base = 0, n_lists = 0, n_list_refs = 0, n_runs_explicit = 0;
    // compact form of the heavy-only refs (rdf_set_result_form(RDF_FORM_HEAVY_BITS)): the current result's K explicit
    // refs, its explicit runs [0, res_nx) and heavy work items (chunks of 64 class-list candidates) [0, res_wh) of the
    // work-item range starting at res_h0; res_bits: the form applies to this result (classed heavy-only dependents)
    u32 result_form = 0;
    u64 res_K = 0, res_nx = 0, res_wh = 0, res_h0 = 0;
    bool res_bits = false;
    DevBuf hpos;
    // ... and their expansion into `out` (k_heavy_write) deferred to the first row accessor, like the class part:
    // work items [hp_h0, hp_h0 + hp_W) at output offset hp_K
    bool heavy_pending = false;
    u64 hp_W = 0, hp_h0 = 0, hp_K = 0;
    DevBuf loff;  // list offsets of the shared (class) ref lists
    // paged discovery (rdf_discover_cinds_paged / rdf_next_page): dependents in ranges, one page at a time
    bool paged = false, pg_unary_done = false;
    u32 pg_flags = 0, pg_next = 0;
    u64 pg_budget = 0, pg_Eu = 0, pg_HC = 0, pg_NT = 0, pg_WM = 0, pg_pages = 0;
    std::vector<u64> h_choffl, h_choffh, h_eoffu;
    bool hclassed = false;  // binary heavy-only dependents emitted from class lists (single GPU, S2L semantics)
    DevBuf pedges, pedges_tmp;
    u64 ncap = 0;
    u64 n_explicit_raw = 0, n_light_chunks = 0, n_light_survivors = 0, n_multi_items = 0;
    rdf_fc_stats fstats = {};
    rdf_group_stats gstats = {};
    rdf_cind_stats cstats = {};

    // sharded mode: this rank's share of the join values, and the pending exchange
    u32 rank = 0, nranks = 1;
    u32 sh_rank = 0, sh_nranks = 1, sh_ms = 1, sh_flags = 0;
    u64 sh_nfreq[3] = {0, 0, 0}, sh_nkeys = 0;
    DevBuf wts, wtp, wto;  // sharded input: the triples received for this rank's join shard
    int sh_proj = 7, sh_phase = -1;
    u64 sh_WH = 0, sh_H = 0, sh_E = 0, sh_tcapc = 0;
    u32 h_hist_local[256] = {};
    int x_op = RDF_X_DONE;
    const void* x_src = nullptr;
    u64 x_count = 0, x_recv_count = 0;
    u32 x_bytes = 8;
    bool x_imported = true;
    DevBuf item_dep, eblk, lslot, npk, pkoff, pk_dep, nmch, mchoff, mch_dep;
    DevBuf uhist, urecs, usl, cntg, fstage, bfreq, boff, fbits, brkeys;  // partitioned K1 / K2 (counts.inl)
    DevBuf xsend, xrecv, gbest, nrl, smask, smask_tmp, cpairs, cpairs_tmp, obounds;
    DevBuf lmask, hrep, vpairs, vcoff, vpiv;  // holder-first light exchange (sh_phase5 / sh_phase15)
    DevBuf ebown, segb, sege, seglen;         // this rank's binary dependents' final pairs; dependent segments
    DevBuf bslots, bcounts;                   // light pass B's output slots (pass A's stay in epairs_tmp / lslot)
    DevBuf ukeys, ukeys_tmp;                  // sharded: frequent unary keys (owned, then every rank's, sorted)
    // sharded ingest (rdf_shard_parse_begin): local terms routed to their owners, the owner's dictionary, global ids
    DevBuf ithv, ikeys, ikeys_tmp, iwords, iwoff, ihdr, ipay, ibnd, iwb, rhdr, rlen, rwords, rwoff, rts, rhv, rvalid, rtab,
        rslot, rrep, rfirst, rfid, rhist, rreply, own_text, own_off, own_len, gmapv;
    DevBuf dneed, dnpos, dwn, dwo, dhdr, dlen, dlwords, dwoff, tids, tlenv, toffv, tout;  // dictionary by owner lookup
    bool ingest_sharded = false;              // the resident ids are global ids of a sharded ingest
    u32 own_n = 0, own_base = 0;
    u64 ing_Vl = 0, ing_m = 0;
    std::vector<u64> ing_pay_counts, ing_src_counts;
    u64 sh_Eb = 0;
    u64 n_hrep = 0;
    u64 n_out = 0, n_runs = 0;
    u32* out_ptr = nullptr;
    bool h_runs_valid = false;  // host mirror of the run table (filled on the first copy)
    std::vector<u64> h_runoff;
    std::vector<u32> h_rundep;
    std::vector<u32> h_fcap;
    std::vector<u32> h_csup;

    hipEvent_t ev[8] = {};
    float stage_ms[3] = {0, 0, 0};
    // stage timings whose end events are recorded but not yet read (read at the run's final wait, or on demand):
    // the stage boundaries do not drain the stream
    bool pend_fc = false, pend_groups = false;
    bool pend_heavy = false;
    bool spare_fc = false, spare_groups = false;  // reclaim_spare may release these stages' scratch
    bool spare_x = false;  // ... and the exchange buffers, from the routing of the triples to the end of the group build
    DevBuf ecache;                   // join ranges: each range's scanned K3 block offsets from its first emission
    std::vector<u64> ecache_je;      // ... and its record-slot count  // heavy threshold / count of the last group build still on the device (hist + 256, + 258)
    // per kernel-family device timers (events on the context stream)
    static constexpr int kTSeg = 32;  // segments per timer (a kernel family may run in several places: the two light
                                      // passes record ~14 light segments)
    hipEvent_t tev[2 * RDF_NUM_TIMERS * kTSeg] = {};
    int tn[RDF_NUM_TIMERS] = {};
    float tms[RDF_NUM_TIMERS] = {};
    u64 sort_passes_records = 0, sort_passes_pairs = 0;
    u64 heavy_candidates = 0;
    u64 light_candidates = 0, light_entries = 0;  // pivot members / group entries of dependents with light groups
};

static void tbegin(rdf_ctx* c, int id) {
    if (c->tn[id] < rdf_ctx::kTSeg) (void)hipEventRecord(c->tev[2 * (id * rdf_ctx::kTSeg + c->tn[id])], c->stream);
}
static void tend(rdf_ctx* c, int id) {
    if (c->tn[id] < rdf_ctx::kTSeg) (void)hipEventRecord(c->tev[2 * (id * rdf_ctx::kTSeg + c->tn[id]) + 1], c->stream);
    c->tn[id]++;
}
// call after a stream sync: fold the recorded segments of timers [lo, hi) into tms (add: onto the previous value)
static void tcollect(rdf_ctx* c, int lo, int hi, bool add = false) {
    for (int i = lo; i < hi; ++i) {
        float total = 0;
        for (int k = 0; k < std::min(c->tn[i], rdf_ctx::kTSeg); ++k) {
            float ms = 0;
            const int e = 2 * (i * rdf_ctx::kTSeg + k);
            if (hipEventElapsedTime(&ms, c->tev[e], c->tev[e + 1]) == hipSuccess) total += ms;
        }
        c->tms[i] = add ? c->tms[i] + total : total;
        c->tn[i] = 0;
    }
}

static rdf_status fail(rdf_ctx* c, rdf_status code, const std::string& msg) {
    if (c) c->err = msg;
    return code;
}

#define HIP_TRY(ctx, expr)                                                                          \
    do {                                                                                            \
        hipError_t _e = (expr);                                                                     \
        if (_e != hipSuccess)                                                                       \
            return fail(ctx, _e == hipErrorOutOfMemory ? RDF_ERR_OOM : RDF_ERR_HIP,                 \
                        std::string(#expr) + ": " + hipGetErrorString(_e));                        \
    } while (0)

#define TRY(expr)                    \
    do {                             \
        rdf_status _r = (expr);      \
        if (_r != RDF_OK) return _r; \
    } while (0)

// Spare buffers: the frequent-condition stage's record scratch after that stage, and the group build's record and
// sort buffers after it (up to ~120 GB at 10^9 triples).  They stay allocated across runs (re-allocating tens of GB
// every step cost seconds: c4 at 10^9 triples spent 4.3 of 6.4 s per step outside its kernels) and are released
// only when an allocation of a later stage would otherwise fail.
static bool reclaim_spare(rdf_ctx* c, const DevBuf* keep) {
    const std::vector<DevBuf*> fc_scratch = {&c->brkeys, &c->brkeys2, &c->tkeys, &c->urecs};
    const std::vector<DevBuf*> grp_scratch = {&c->rec, &c->rec_tmp, &c->fk, &c->fk_tmp, &c->rstore};
    const std::vector<DevBuf*> x_scratch = {&c->xsend, &c->xrecv};
    bool any = false;
    for (int k = 0; k < 3; ++k) {
        if (!(k == 0 ? c->spare_fc : k == 1 ? c->spare_groups : c->spare_x)) continue;
        for (DevBuf* b : (k == 0 ? fc_scratch : k == 1 ? grp_scratch : x_scratch)) {
            if (b == keep || !b->p) continue;
            if (!any) (void)hipStreamSynchronize(c->stream);  // queued kernels may still read them
            b->release();
            any = true;
        }
    }
    (void)hipGetLastError();
    return any;
}
static void mem_track(rdf_ctx* c);
static rdf_status ensure_buf(rdf_ctx* c, DevBuf* b, size_t bytes, const char* what) {
    const size_t cap0 = b->cap;
    hipError_t e = b->ensure(bytes);
    if (e == hipErrorOutOfMemory && reclaim_spare(c, b)) e = b->ensure(bytes);
    if (e == hipSuccess && b->cap != cap0) mem_track(c);
    if (e != hipSuccess)
        return fail(c, e == hipErrorOutOfMemory ? RDF_ERR_OOM : RDF_ERR_HIP, std::string(what) + ": " + hipGetErrorString(e));
    return RDF_OK;
}
#define ENSURE(ctx, buf, bytes) TRY(ensure_buf(ctx, &(ctx)->buf, (size_t)(bytes), "allocating " #buf))
// the early hand-over's copies (rdf_set_handover) must finish before the device buffers they read are rewritten or
// freed by the next stage, and before the caller reads its host buffers; a new result forgets them
static rdf_status hv_wait(rdf_ctx* c, bool forget) {
    if (c->hv_pending) {
        c->hv_pending = false;
        c->hv_gpu_wait = false;
        HIP_TRY(c, hipStreamSynchronize(c->hstream));
    }
    if (forget) {
        c->hv_refs_n = ~0ull;
        c->hv_runs_n = ~0ull;
        c->hv_caps_done = false;
    }
    return RDF_OK;
}
#define ENSURE_KEEP(ctx, buf, bytes) HIP_TRY(ctx, (ctx)->buf.grow_keep((size_t)(bytes), (ctx)->stream))

static int bits_for(u64 maxval) {  // bits needed to represent values in [0, maxval]
    int b = 0;
    while (b < 64 && (maxval >> b)) ++b;
    return b < 1 ? 1 : b;
}

static u64 next_pow2(u64 x) {
    u64 p = 1;
    while (p < x) p <<= 1;
    return p;
}

// Host waits on the stream.  Each read-back of a device size drains the stream: the GPU idles from the end of the
// read until the host has launched the next kernel (~25-40 us per read on c2, tools/gaps.py), so the reads are one
// kernel that stores the scalars straight into pinned host memory (no separate copy).  RDFIND_SPIN=1 polls the stream
// instead of blocking in hipStreamSynchronize (measured: no gain on c2, 10.27 vs 10.23 ms, profiles/r04_sync_trace_*).
// RDFIND_SYNC_TRACE=1: every wait prints "SYNC <line> <t_us> <wait_us>" to stderr (tools/sync_trace.py).
static hipError_t stream_wait(hipStream_t s, int line) {
    static const bool trace = getenv("RDFIND_SYNC_TRACE") != nullptr;
    static const bool spin = getenv("RDFIND_SPIN") && atoi(getenv("RDFIND_SPIN")) != 0;
    using clk = std::chrono::steady_clock;
    static const clk::time_point t00 = clk::now();
    const clk::time_point t0 = trace ? clk::now() : clk::time_point();
    hipError_t e;
    if (spin) {
        while ((e = hipStreamQuery(s)) == hipErrorNotReady) {
        }
    } else {
        e = hipStreamSynchronize(s);
    }
    if (trace) {
        const clk::time_point t1 = clk::now();
        fprintf(stderr, "SYNC %d %.1f %.1f\n", line, std::chrono::duration<double, std::micro>(t0 - t00).count(),
                std::chrono::duration<double, std::micro>(t1 - t0).count());
    }
    return e;
}
#define hipStreamSynchronize(s) stream_wait((s), __LINE__)

// Host <-> device copies of a context's buffers are ordered on the context's stream and wait for it.  The context
// stream is non-blocking, so the null stream a plain hipMemcpy runs on would not wait for kernels still queued there
// (e.g. rdf_copy_binary_keys right after rdf_frequent_conditions, whose key sort may still be running).
static hipError_t ctx_copy_(hipStream_t s, void* dst, const void* src, size_t bytes, hipMemcpyKind kind, int line) {
    const hipError_t e = hipMemcpyAsync(dst, src, bytes, kind, s);
    return e != hipSuccess ? e : stream_wait(s, line);
}
#define ctx_copy(c, dst, src, bytes, kind) ctx_copy_((c)->stream, (dst), (src), (bytes), (kind), __LINE__)

// Several device scalars with ONE host round trip: a one-thread kernel gathers them into the mapped host buffer.
struct ScalarGather {
    const void* p[8];
    int bytes[8];
    int n;
};

__global__ void k_gather_scalars(ScalarGather g, u64* dst) {
    for (int i = 0; i < g.n; ++i) dst[i] = g.bytes[i] == 8 ? *(const u64*)g.p[i] : (u64) * (const u32*)g.p[i];
}

static u64* dscal(rdf_ctx* c, int i) { return c->scal.as<u64>() + i; }

static rdf_status gather_read(rdf_ctx* c, const ScalarGather& g, u64* out) {
    hipLaunchKernelGGL(k_gather_scalars, dim3(1), dim3(1), 0, c->stream, g, c->hread_d);
    HIP_TRY(c, hipGetLastError());
    HIP_TRY(c, hipStreamSynchronize(c->stream));
    const volatile u64* h = c->hread;
    for (int i = 0; i < g.n; ++i) out[i] = h[i];
    return RDF_OK;
}

// scal[0, count) -> hscal[0, count)
static rdf_status read_scalars(rdf_ctx* c, int count) {
    ScalarGather g = {};
    for (int i = 0; i < count; ++i) {
        g.p[i] = dscal(c, i);
        g.bytes[i] = 8;
    }
    g.n = count;
    return gather_read(c, g, c->hscal);
}

static rdf_status read_u64(rdf_ctx* c, const void* dptr, u64* out) {
    ScalarGather g = {};
    g.p[0] = dptr;
    g.bytes[0] = 8;
    g.n = 1;
    return gather_read(c, g, out);
}

static rdf_status read_u32(rdf_ctx* c, const void* dptr, u32* out) {
    ScalarGather g = {};
    g.p[0] = dptr;
    g.bytes[0] = 4;
    g.n = 1;
    u64 v = 0;
    TRY(gather_read(c, g, &v));
    *out = (u32)v;
    return RDF_OK;
}

static rdf_status read_multi(rdf_ctx* c, std::initializer_list<std::pair<const void*, int>> refs, u64* out) {
    ScalarGather g = {};
    for (const auto& r : refs) {
        g.p[g.n] = r.first;
        g.bytes[g.n] = r.second;
        ++g.n;
    }
    return gather_read(c, g, out);
}

static rdf_status load_bkeys(rdf_ctx* c) {
    if (c->h_bkeys_valid) return RDF_OK;
    c->h_bkeys.resize(c->B);
    if (c->B) HIP_TRY(c, ctx_copy(c, c->h_bkeys.data(), c->bkeys.p, c->B * 8, hipMemcpyDeviceToHost));
    c->h_bkeys_valid = true;
    return RDF_OK;
}

#ifndef RDF_KGRID
#define RDF_KGRID 2048
#endif
static const unsigned kGrid = RDF_KGRID;  // grid-stride kernels: 8 blocks of 256 threads per CU
// work-item kernels loop over virtual blocks: a dispatch holds < 2^32 work-items in x, so grids are capped
static const u64 kMaxBlocks = 1ull << 20;
static inline unsigned vgrid(u64 blocks) { return (unsigned)std::min<u64>(std::max<u64>(blocks, 1), kMaxBlocks); }
static inline u64 wave_blocks(u64 waves) { return (waves + RDF_WAVES_PER_BLOCK - 1) / RDF_WAVES_PER_BLOCK; }
static inline u64 thread_blocks(u64 threads) { return (threads + RDF_BLOCK - 1) / RDF_BLOCK; }

// every device buffer a context owns (release on destroy; rdf_device_bytes)
static std::vector<DevBuf*> ctx_buffers(rdf_ctx* c) {
    return {&c->scal, &c->ts, &c->tp, &c->to, &c->cnt, &c->tkeys, &c->tcnt, &c->bkeys, &c->bkeys_tmp,
                      &c->lkeys, &c->lvals, &c->flags, &c->pos, &c->rec, &c->rec_tmp, &c->support, &c->fidx,
                      &c->fcap, &c->frank, &c->fval, &c->fext, &c->info, &c->fk, &c->fk_tmp, &c->fpos, &c->cstart, &c->skip, &c->gflag, &c->gexcl, &c->goff,
                      &c->gcap, &c->gmap, &c->csup,
                      &c->doff, &c->dcur, &c->dgrp, &c->jhist, &c->rsup, &c->lsup, &c->hot, &c->hotc, &c->jrmap, &c->offp, &c->hist, &c->heavy_list, &c->hbit, &c->bcomp, &c->bkeyc,
                      &c->pcnt, &c->poff, &c->pcur, &c->plist, &c->pivot, &c->nchl, &c->nchh, &c->choffl,
                      &c->choffh, &c->epairs, &c->epairs_tmp, &c->eoff, &c->hcounts, &c->hoff, &c->hbits, &c->cbits, &c->hown, &c->cown, &c->sbase, &c->dcls, &c->crep, &c->out,
                      &c->stage_rows, &c->nitl, &c->itoffl, &c->dead, &c->ebin,
                      &c->pseg, &c->psegoff, &c->pbest, &c->pnl, &c->lsig, &c->brkeys2, &c->bstart2, &c->ginfo, &c->gsums, &c->piv2, &c->pivx, &c->ecache, &c->ctab, &c->cflag, &c->ccid, &c->ckeys,
                      &c->ckeys_tmp, &c->coff, &c->cmask, &c->cpiv, &c->cnch, &c->cchoff, &c->ccnt, &c->lwoff,
                      &c->clists, &c->cself, &c->cmcnt, &c->cobase, &c->ctiles, &c->ctoff, &c->pedges, &c->pedges_tmp,
                      &c->item_dep, &c->eblk, &c->lslot, &c->npk, &c->pkoff, &c->pk_dep, &c->nmch, &c->mchoff, &c->mch_dep, &c->uhist, &c->urecs, &c->usl, &c->cntg, &c->fstage, &c->bfreq, &c->boff,
                      &c->fbits, &c->brkeys, &c->xsend, &c->xrecv, &c->gbest, &c->nrl, &c->smask, &c->smask_tmp, &c->cpairs, &c->cpairs_tmp,
                      &c->obounds, &c->lmask, &c->hrep, &c->vpairs, &c->vcoff, &c->vpiv, &c->runoff, &c->rundep, &c->dheap, &c->dtoff, &c->cslen, &c->csoff,
                      &c->cstr, &c->flen, &c->floff, &c->fbuf, &c->drows, &c->ppart, &c->wts, &c->wtp,
            &c->wto, &c->arcnt, &c->ar_bits, &c->ar_rules, &c->arref, &c->loff, &c->gdrow, &c->dlist, &c->dbits, &c->ebown, &c->bslots, &c->bcounts, &c->segb, &c->sege, &c->seglen, &c->ukeys,
            &c->ukeys_tmp, &c->ithv, &c->ikeys, &c->ikeys_tmp, &c->iwords, &c->iwoff, &c->ihdr, &c->ipay, &c->ibnd, &c->iwb,
            &c->rhdr, &c->rlen, &c->rwords, &c->rwoff, &c->rts, &c->rhv, &c->rvalid, &c->rtab, &c->rslot, &c->rrep, &c->rfirst,
            &c->rfid, &c->rhist, &c->rreply, &c->own_text, &c->own_off, &c->own_len, &c->gmapv, &c->dneed, &c->dnpos, &c->dwn,
            &c->dwo, &c->dhdr, &c->dlen, &c->dlwords, &c->dwoff, &c->tids, &c->tlenv, &c->toffv, &c->tout, &c->rstore, &c->jbh, &c->iflag, &c->iexcl, &c->iorder, &c->ukey, &c->utab, &c->urep, &c->ucnt, &c->unoff, &c->uebin, &c->umem, &c->hpos};
}

// RDFIND_MEM_REPORT=1: after each rdf_run, the context's buffers of >= 256 MiB (name, GiB) on stderr, largest first
static const char* const kBufNames[] = {"scal", "ts", "tp", "to", "cnt", "tkeys", "tcnt", "bkeys", "bkeys_tmp", "lkeys", "lvals", "flags", "pos", "rec", "rec_tmp", "support", "fidx", "fcap", "frank", "fval", "fext", "info", "fk", "fk_tmp", "fpos", "cstart", "skip", "gflag", "gexcl", "goff", "gcap", "gmap", "csup", "doff", "dcur", "dgrp", "jhist", "rsup", "lsup", "hot", "hotc", "jrmap", "offp", "hist", "heavy_list", "hbit", "bcomp", "bkeyc", "pcnt", "poff", "pcur", "plist", "pivot", "nchl", "nchh", "choffl", "choffh", "epairs", "epairs_tmp", "eoff", "hcounts", "hoff", "hbits", "cbits", "hown", "cown", "sbase", "dcls", "crep", "out", "stage_rows", "nitl", "itoffl", "dead", "ebin", "pseg", "psegoff", "pbest", "pnl", "lsig", "brkeys2", "bstart2", "ginfo", "gsums", "piv2", "pivx", "ecache", "ctab", "cflag", "ccid", "ckeys", "ckeys_tmp", "coff", "cmask", "cpiv", "cnch", "cchoff", "ccnt", "lwoff", "clists", "cself", "cmcnt", "cobase", "ctiles", "ctoff", "pedges", "pedges_tmp", "item_dep", "eblk", "lslot", "npk", "pkoff", "pk_dep", "nmch", "mchoff", "mch_dep", "uhist", "urecs", "usl", "cntg", "fstage", "bfreq", "boff", "fbits", "brkeys", "xsend", "xrecv", "gbest", "nrl", "smask", "smask_tmp", "cpairs", "cpairs_tmp", "obounds", "lmask", "hrep", "vpairs", "vcoff", "vpiv", "runoff", "rundep", "dheap", "dtoff", "cslen", "csoff", "cstr", "flen", "floff", "fbuf", "drows", "ppart", "wts", "wtp", "wto", "arcnt", "ar_bits", "ar_rules", "arref", "loff", "gdrow", "dlist", "dbits", "ebown", "bslots", "bcounts", "segb", "sege", "seglen", "ukeys", "ukeys_tmp", "ithv", "ikeys", "ikeys_tmp", "iwords", "iwoff", "ihdr", "ipay", "ibnd", "iwb", "rhdr", "rlen", "rwords", "rwoff", "rts", "rhv", "rvalid", "rtab", "rslot", "rrep", "rfirst", "rfid", "rhist", "rreply", "own_text", "own_off", "own_len", "gmapv", "dneed", "dnpos", "dwn", "dwo", "dhdr", "dlen", "dlwords", "dwoff", "tids", "tlenv", "toffv", "tout", "rstore", "jbh", "iflag", "iexcl", "iorder", "ukey", "utab", "urep", "ucnt", "unoff", "uebin", "umem", "hpos"};
static bool mem_report_on() {
    static const bool on = getenv("RDFIND_MEM_REPORT") && atoi(getenv("RDFIND_MEM_REPORT")) != 0;
    return on;
}
// the context's peak of buffer bytes (RDFIND_MEM_REPORT only: summed at every allocation that changes a buffer)
static void mem_track(rdf_ctx* c) {
    if (!mem_report_on()) return;
    size_t total = c->ws.bytes();
    for (DevBuf* b : ctx_buffers(c)) total += b->cap;
    c->peak_bytes = std::max<u64>(c->peak_bytes, total);
}
static void mem_report(rdf_ctx* c) {
    if (!mem_report_on()) return;
    std::vector<DevBuf*> bufs = ctx_buffers(c);
    std::vector<std::pair<size_t, const char*>> big;
    size_t total = 0;
    for (size_t i = 0; i < bufs.size(); ++i) {
        total += bufs[i]->cap;
        if (bufs[i]->cap >= (256ull << 20)) big.push_back({bufs[i]->cap, i < sizeof(kBufNames) / sizeof(kBufNames[0]) ? kBufNames[i] : "?"});
    }
    std::sort(big.begin(), big.end(), [](const std::pair<size_t, const char*>& x, const std::pair<size_t, const char*>& y) {
        return x.first > y.first;
    });
    fprintf(stderr, "MEM total %.2f GiB, peak %.2f GiB (workspace %.2f GiB):", total / 1073741824.0,
            std::max<u64>(c->peak_bytes, total) / 1073741824.0, c->ws.bytes() / 1073741824.0);
    for (const auto& b : big) fprintf(stderr, " %s=%.2f", b.second, b.first / 1073741824.0);
    fprintf(stderr, "\n");
}

extern "C" {

const char* rdf_version(void) { return RDF_VERSION; }

rdf_status rdf_ctx_create(int device, rdf_ctx** out) {
    if (!out) return RDF_ERR_ARG;
    *out = nullptr;
    rdf_ctx* c = new rdf_ctx();
    c->device = device;
    // test hook: RDFIND_COUNT_PATHS=atomic selects the global-atomic unary counting kernel (the fallback of
    // the partitioned K1 for |V| > 2^26 / 3), so the parity tests cover both paths
    const char* paths = getenv("RDFIND_COUNT_PATHS");
    c->force_global_counts = paths && !strcmp(paths, "atomic");
    // test hook: RDFIND_HEAVY_MIN=<power of two> lowers the minimum heavy-group size (default 64), so small
    // parity inputs exercise the bitmask / class / heavy-only paths
    const char* hcl = getenv("RDFIND_HCLASS");
    c->allow_hclass = !(hcl && !strcmp(hcl, "0"));
    const char* hmin = getenv("RDFIND_HEAVY_MIN");
    if (hmin && atoll(hmin) > 0) c->heavy_min = (u64)atoll(hmin);
    // dense light-group bitmaps: RDFIND_DENSE=<divisor> (groups of >= C / divisor members; 0 = off) and the test hook
    // RDFIND_DENSE_MIN=<members> (absolute minimum, default LIGHT_DENSE_MIN)
    if (const char* dd = getenv("RDFIND_DENSE")) c->dense_div = atoi(dd);
    // test hook: RDFIND_GROUP_RANGE=<records> builds the capture groups in join-value ranges of at most that many
    // K3 records (the path inputs of >= 2^32 / 9 triples take), so small parity inputs run it
    if (const char* gr = getenv("RDFIND_GROUP_RANGE"))
        if (atoll(gr) > 0) c->group_range_records = (u64)atoll(gr);
    if (const char* dm = getenv("RDFIND_DENSE_MIN"))
        if (atoll(dm) > 0) c->dense_min = (u64)atoll(dm);
    if (const char* hq = getenv("RDFIND_HOLDER_Q")) c->holder_qbits = std::max(0, std::min(atoi(hq), 8));
    if (const char* tf = getenv("RDFIND_TEST_FAIL_LAUNCH")) c->test_fail_launch = tf;
    if (const char* to = getenv("RDFIND_TEST_OOM_DISCOVERY")) c->test_oom_discovery = atoi(to) != 0;
    if (const char* tf = getenv("RDFIND_TEST_FAIL_SHARD")) {
        if (sscanf(tf, "%d:%d", &c->test_fail_rank, &c->test_fail_phase) != 2) c->test_fail_rank = c->test_fail_phase = -1;
    }
    if (const char* hb = getenv("RDFIND_HOT_BALANCE")) c->hot_balance = atoi(hb) != 0;
    if (const char* rk = getenv("RDFIND_RANGE_KEEP")) c->range_keep = atoi(rk) != 0;
    if (const char* ld = getenv("RDFIND_LIGHT_DEDUP")) c->light_dedup = atoi(ld) != 0 ? 1 : 0;
    if (const char* dm = getenv("RDFIND_DUP_MIN")) c->dup_min = (u32)std::max(1, atoi(dm));
    if (const char* um = getenv("RDFIND_U1_RADIX_MIN")) c->u1_radix_min = strtoull(um, nullptr, 10);
    hipError_t e = hipSetDevice(device);
    if (e == hipSuccess) e = hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking);
    if (e == hipSuccess) e = hipStreamCreateWithFlags(&c->side, hipStreamNonBlocking);
    if (e == hipSuccess) e = hipEventCreateWithFlags(&c->ev_fork, hipEventDisableTiming);
    if (e == hipSuccess) e = hipStreamCreateWithFlags(&c->hstream, hipStreamNonBlocking);
    if (e == hipSuccess) e = hipEventCreateWithFlags(&c->hv_ev, hipEventDisableTiming);
    if (e == hipSuccess) e = hipEventCreateWithFlags(&c->hv_done, hipEventDisableTiming);
    if (e == hipSuccess) e = hipEventCreateWithFlags(&c->ev_join, hipEventDisableTiming);
    if (e == hipSuccess) e = c->scal.ensure(16 * sizeof(u64));
    if (e == hipSuccess) e = hipHostMalloc((void**)&c->hscal, 16 * sizeof(u64), hipHostMallocDefault);
    if (e == hipSuccess) e = hipHostMalloc((void**)&c->hread, 16 * sizeof(u64), hipHostMallocMapped | hipHostMallocCoherent);
    if (e == hipSuccess) e = hipHostGetDevicePointer((void**)&c->hread_d, c->hread, 0);
    for (int i = 0; i < 8 && e == hipSuccess; ++i) e = hipEventCreate(&c->ev[i]);
    for (int i = 0; i < 2 * RDF_NUM_TIMERS * rdf_ctx::kTSeg && e == hipSuccess; ++i) e = hipEventCreate(&c->tev[i]);
    if (e != hipSuccess) {
        rdf_ctx_destroy(c);
        return RDF_ERR_HIP;
    }
    *out = c;
    return RDF_OK;
}

void rdf_ctx_destroy(rdf_ctx* c) {
    if (!c) return;
    (void)hipSetDevice(c->device);
    if (c->stream) (void)hipStreamSynchronize(c->stream);
    if (c->side) (void)hipStreamSynchronize(c->side);
    if (c->hstream) (void)hipStreamSynchronize(c->hstream);
    for (DevBuf* b : ctx_buffers(c)) b->release();
    c->ws.release();
    if (c->hscal) (void)hipHostFree(c->hscal);
    if (c->hread) (void)hipHostFree(c->hread);
    for (auto& e : c->ev)
        if (e) (void)hipEventDestroy(e);
    for (auto& e : c->tev)
        if (e) (void)hipEventDestroy(e);
    if (c->ev_fork) (void)hipEventDestroy(c->ev_fork);
    if (c->hstream) (void)hipStreamDestroy(c->hstream);
    if (c->hv_ev) (void)hipEventDestroy(c->hv_ev);
    if (c->ev_join) (void)hipEventDestroy(c->ev_join);
    if (c->side) (void)hipStreamDestroy(c->side);
    if (c->stream) (void)hipStreamDestroy(c->stream);
    delete c;
}

const char* rdf_last_error(const rdf_ctx* c) { return c ? c->err.c_str() : "null context"; }

rdf_status rdf_sync(rdf_ctx* c) {
    if (!c) return RDF_ERR_ARG;
    HIP_TRY(c, hipStreamSynchronize(c->stream));
    return hv_wait(c, false);  // (and the copies queued on the copy stream)
}

rdf_status rdf_device_bytes(rdf_ctx* c, uint64_t* bytes) {
    if (!c || !bytes) return RDF_ERR_ARG;
    u64 t = c->ws.bytes();
    for (DevBuf* b : ctx_buffers(c)) t += b->cap;
    *bytes = t;
    return RDF_OK;
}

// Per-context input limits: term ids < 2^30 (binary keys, K2's count bits); 3n K1/K2 records addressed by u32 offsets.
// Inputs of >= 2^32 / 9 triples build their capture groups in join-value ranges (g_build_ranges).
static rdf_status check_terms(rdf_ctx* c, u64 n, u32 num_terms) {
    if (num_terms >= (1u << 30)) return fail(c, RDF_ERR_LIMIT, "num_terms must be < 2^30");
    if (n >= (1ull << 32) / 3) return fail(c, RDF_ERR_LIMIT, "n must be < 2^32/3 triples per GPU (shard larger inputs)");
    return RDF_OK;
}

// Per-run buffers only grow, so a context that ran a large input keeps its buffers.  When a new input arrives and
// what the context holds beyond the input and the uploaded dictionary exceeds max(4 GB, 1 KB per new triple), it is
// released first: a test sequence c4 at 0.4 (400M triples) -> c5 at 0.3 (3M triples, 10^10 CINDs) must not carry
// the first run's buffers into the second run's growth.
static void release_run_buffers(rdf_ctx* c, u64 n_next, bool always = false) {
    const DevBuf* keep[] = {&c->scal, &c->ts, &c->tp, &c->to, &c->dheap, &c->dtoff, &c->own_text, &c->own_off, &c->own_len};
    auto kept = [&](const DevBuf* b) {
        for (const DevBuf* k : keep)
            if (k == b) return true;
        return false;
    };
    u64 held = c->ws.bytes();
    for (DevBuf* b : ctx_buffers(c))
        if (!kept(b)) held += b->cap;
    if (!always && held <= std::max<u64>(4ull << 30, n_next << 10)) return;
    (void)hipStreamSynchronize(c->stream);
    c->paged = false;
    for (DevBuf* b : ctx_buffers(c))
        if (!kept(b)) b->release();
    c->ws.release();
    c->dense_on = false;
    c->class_pending = false;
    c->h_runs_valid = false;
    c->h_bkeys_valid = false;
    c->capstr_run = ~0ull;
}

rdf_status rdf_release_scratch(rdf_ctx* c) {
    if (!c) return RDF_ERR_ARG;
    HIP_TRY(c, hipSetDevice(c->device));
    TRY(hv_wait(c, true));
    release_run_buffers(c, 0, true);
    (void)hipGetLastError();  // an out-of-memory failure before this call is not the next call's error
    c->paged = false;
    c->stage = std::min(c->stage, 1);
    return RDF_OK;
}

rdf_status rdf_set_triples(rdf_ctx* c, const uint32_t* s, const uint32_t* p, const uint32_t* o, uint64_t n,
                           uint32_t num_terms) {
    if (!c || (n && (!s || !p || !o))) return fail(c, RDF_ERR_ARG, "null triple arrays");
    rdf_status st = check_terms(c, n, num_terms);
    if (st) return st;
    HIP_TRY(c, hipSetDevice(c->device));
    TRY(hv_wait(c, true));
    release_run_buffers(c, n);
    ENSURE(c, ts, n * 4);
    ENSURE(c, tp, n * 4);
    ENSURE(c, to, n * 4);
    if (n) {
        HIP_TRY(c, hipMemcpyAsync(c->ts.p, s, n * 4, hipMemcpyHostToDevice, c->stream));
        HIP_TRY(c, hipMemcpyAsync(c->tp.p, p, n * 4, hipMemcpyHostToDevice, c->stream));
        HIP_TRY(c, hipMemcpyAsync(c->to.p, o, n * 4, hipMemcpyHostToDevice, c->stream));
    }
    HIP_TRY(c, hipStreamSynchronize(c->stream));
    c->s = c->ts.as<u32>();
    c->p = c->tp.as<u32>();
    c->o = c->to.as<u32>();
    c->n = n;
    c->V = num_terms;
    c->stage = 1;
    c->paged = false;  // a paged run's state belongs to the previous input
    c->parsed_dict = false;
    c->ingest_sharded = false;
    return RDF_OK;
}

rdf_status rdf_set_triples_device(rdf_ctx* c, const uint32_t* s, const uint32_t* p, const uint32_t* o, uint64_t n,
                                  uint32_t num_terms) {
    if (!c || (n && (!s || !p || !o))) return fail(c, RDF_ERR_ARG, "null triple arrays");
    if (c) TRY(hv_wait(c, true));
    rdf_status st = check_terms(c, n, num_terms);
    if (st) return st;
    c->s = s;
    c->p = p;
    c->o = o;
    c->n = n;
    c->V = num_terms;
    c->stage = 1;
    c->paged = false;  // a paged run's state belongs to the previous input
    c->parsed_dict = false;
    c->ingest_sharded = false;
    return RDF_OK;
}

// --distinct-triples (`triples.distinct`, ALG/programs/RDFind.scala:284-287): removes duplicate triples
// from the resident input in HBM (first occurrences kept, input order preserved).  The compacted triples
// are context-owned afterwards, also after rdf_set_triples_device.
rdf_status rdf_distinct_triples(rdf_ctx* c, uint64_t* n_distinct, float* ms) {
    if (!c) return RDF_ERR_ARG;
    if (c->stage < 1) return fail(c, RDF_ERR_STATE, "rdf_set_triples must be called first");
    HIP_TRY(c, hipSetDevice(c->device));
    TRY(hv_wait(c, true));
    hipStream_t st = c->stream;
    const u64 n = c->n;
    HIP_TRY(c, hipEventRecord(c->ev[6], st));
    u64 kept = 0;
    if (n) {
        const u64 T = next_pow2(2 * n);
        ENSURE(c, dtab, T * 8);
        ENSURE(c, dkeep, n * 4);
        ENSURE(c, dpos, n * 4);
        ENSURE(c, xs, n * 4);
        ENSURE(c, xp, n * 4);
        ENSURE(c, xo, n * 4);
        HIP_TRY(c, hipMemsetAsync(c->dtab.p, 0xff, T * 8, st));
        const unsigned g = grid_for(n, RDF_BLOCK, kGrid);
        hipLaunchKernelGGL(k_distinct_insert, dim3(g), dim3(RDF_BLOCK), 0, st, c->s, c->p, c->o, n, c->dtab.as<u64>(), T - 1);
        hipLaunchKernelGGL(k_distinct_keep, dim3(g), dim3(RDF_BLOCK), 0, st, c->s, c->p, c->o, n, c->dtab.as<u64>(), T - 1,
                           c->dkeep.as<u32>());
        HIP_TRY(c, exclusive_scan_u32(c->ws, c->dkeep.as<u32>(), c->dpos.as<u32>(), n, (u32*)dscal(c, 7), st));
        hipLaunchKernelGGL(k_distinct_scatter, dim3(g), dim3(RDF_BLOCK), 0, st, c->s, c->p, c->o, n, c->dkeep.as<u32>(),
                           c->dpos.as<u32>(), c->xs.as<u32>(), c->xp.as<u32>(), c->xo.as<u32>());
        HIP_TRY(c, hipGetLastError());
        HIP_TRY(c, hipMemsetAsync((char*)dscal(c, 7) + 4, 0, 4, st));
        HIP_TRY(c, hipEventRecord(c->ev[7], st));
        rdf_status rs = read_u64(c, dscal(c, 7), &kept);
        if (rs) return rs;
        std::swap(c->ts, c->xs);
        std::swap(c->tp, c->xp);
        std::swap(c->to, c->xo);
        c->s = c->ts.as<u32>();
        c->p = c->tp.as<u32>();
        c->o = c->to.as<u32>();
    } else {
        HIP_TRY(c, hipEventRecord(c->ev[7], st));
        HIP_TRY(c, hipStreamSynchronize(st));
    }
    if (ms) HIP_TRY(c, hipEventElapsedTime(ms, c->ev[6], c->ev[7]));
    c->n = kept;
    c->stage = 1;
    c->paged = false;  // a paged run's state belongs to the previous input
    if (n_distinct) *n_distinct = kept;
    return RDF_OK;
}

// Copies the resident triples (after rdf_distinct_triples: the compacted ones) to host arrays.
rdf_status rdf_copy_triples(rdf_ctx* c, uint32_t* s, uint32_t* p, uint32_t* o, uint64_t cap, uint64_t* n_copied) {
    if (!c) return RDF_ERR_ARG;
    if (c->stage < 1) return fail(c, RDF_ERR_STATE, "rdf_set_triples must be called first");
    const u64 n = std::min<u64>(cap, c->n);
    if (n && (!s || !p || !o)) return fail(c, RDF_ERR_ARG, "null triple arrays");
    HIP_TRY(c, hipSetDevice(c->device));
    if (n) {
        HIP_TRY(c, hipMemcpyAsync(s, c->s, n * 4, hipMemcpyDeviceToHost, c->stream));
        HIP_TRY(c, hipMemcpyAsync(p, c->p, n * 4, hipMemcpyDeviceToHost, c->stream));
        HIP_TRY(c, hipMemcpyAsync(o, c->o, n * 4, hipMemcpyDeviceToHost, c->stream));
    }
    HIP_TRY(c, hipStreamSynchronize(c->stream));
    if (n_copied) *n_copied = n;
    return RDF_OK;
}

// N-Triples ingest on the device (the `Parse triples` map of ALG/programs/RDFind.scala:196-237
// plus dictionary encoding).  The parsed triples become the resident input (as after rdf_set_triples).
rdf_status rdf_parse_ntriples(rdf_ctx* c, const char* text, uint64_t nbytes, uint32_t flags, uint64_t* n_triples,
                              uint32_t* num_terms, float* ms) {
    if (!c || (nbytes && !text)) return fail(c, RDF_ERR_ARG, "null text");
    HIP_TRY(c, hipSetDevice(c->device));
    TRY(hv_wait(c, true));
    hipStream_t st = c->stream;
    const unsigned char* dtext = nullptr;
    ENSURE(c, ntext, nbytes + 16);  // 16-B loads of the last tile stay inside the buffer
    if (nbytes) HIP_TRY(c, hipMemcpyAsync(c->ntext.p, text, nbytes, hipMemcpyHostToDevice, st));
    dtext = (const unsigned char*)c->ntext.p;
    HIP_TRY(c, hipEventRecord(c->ev[6], st));
    const u64 nchunks = std::max<u64>((nbytes + NT_CHUNK - 1) / NT_CHUNK, 1);
    ENSURE(c, ncnt, nchunks * 4);
    ENSURE(c, ncoff, nchunks * 8);
    const unsigned gc = (unsigned)std::min<u64>(nchunks, kGrid);  // one block per tile
    hipLaunchKernelGGL(k_nt_count_lines, dim3(gc), dim3(RDF_BLOCK), 0, st, dtext, nbytes, nchunks, c->ncnt.as<u32>());
    HIP_TRY(c, exclusive_scan_u32_u64(c->ws, c->ncnt.as<u32>(), c->ncoff.as<u64>(), nchunks, dscal(c, 0), st));
    u64 newlines = 0;
    rdf_status rs = read_u64(c, dscal(c, 0), &newlines);
    if (rs) return rs;
    const u64 nlines = newlines + 1, nocc = 3 * nlines;
    if (nocc >= 0xffffffffull) return fail(c, RDF_ERR_LIMIT, "too many lines (3 * lines must be < 2^32)");
    ENSURE(c, nlstart, nlines * 8);
    hipLaunchKernelGGL(k_nt_line_starts, dim3(gc), dim3(RDF_BLOCK), 0, st, dtext, nbytes, nchunks, c->ncoff.as<u64>(),
                       c->nlstart.as<u64>());
    ENSURE(c, ntstart, nocc * 8);
    ENSURE(c, nhv, nocc * 8);
    ENSURE(c, ntlen, nocc * 4);
    ENSURE(c, nvalid, nlines * 4);
    ENSURE(c, nlpos, nlines * 4);
    HIP_TRY(c, hipMemsetAsync(dscal(c, 1), 0xff, 8, st));
    const unsigned gl = grid_for(nlines, RDF_BLOCK, kGrid), go = grid_for(nocc, RDF_BLOCK, kGrid);
    hipLaunchKernelGGL(k_nt_tokenize, dim3(gl), dim3(RDF_BLOCK), 0, st, dtext, nbytes, c->nlstart.as<u64>(), nlines,
                       (int)(flags & RDF_NT_TABS), c->ntstart.as<u64>(), c->ntlen.as<u32>(), c->nhv.as<u64>(),
                       c->nvalid.as<u32>(), dscal(c, 1));
    HIP_TRY(c, hipMemsetAsync(dscal(c, 2), 0, 8, st));
    HIP_TRY(c, exclusive_scan_u32(c->ws, c->nvalid.as<u32>(), c->nlpos.as<u32>(), nlines, (u32*)dscal(c, 2), st));
    const u64 T = next_pow2(2 * nocc);
    if (T > (1ull << 32)) return fail(c, RDF_ERR_LIMIT, "too many terms per parse call (split the input)");
    ENSURE(c, ntab, T * 8);
    ENSURE(c, nslot, nocc * 4);
    ENSURE(c, nrep, nocc * 4);
    ENSURE(c, nfirst, nocc * 4);
    ENSURE(c, nfid, nocc * 4);
    HIP_TRY(c, hipMemsetAsync(c->ntab.p, 0xff, T * 8, st));
    hipLaunchKernelGGL(k_nt_dict_insert, dim3(go), dim3(RDF_BLOCK), 0, st, dtext, c->ntstart.as<u64>(), c->ntlen.as<u32>(),
                       c->nvalid.as<u32>(), nocc, c->nhv.as<u64>(), c->ntab.as<u64>(), T - 1, c->nslot.as<u32>());
    hipLaunchKernelGGL(k_nt_dict_rep, dim3(go), dim3(RDF_BLOCK), 0, st, c->nvalid.as<u32>(), nocc, c->nslot.as<u32>(),
                       c->ntab.as<u64>(), c->nrep.as<u32>(), c->nfirst.as<u32>());
    HIP_TRY(c, hipMemsetAsync(dscal(c, 3), 0, 8, st));
    HIP_TRY(c, exclusive_scan_u32(c->ws, c->nfirst.as<u32>(), c->nfid.as<u32>(), nocc, (u32*)dscal(c, 3), st));
    u64 sc[3];
    rs = read_multi(c, {{dscal(c, 1), 8}, {dscal(c, 2), 8}, {dscal(c, 3), 8}}, sc);
    if (rs) return rs;
    if (sc[0] != ~0ull) return fail(c, RDF_ERR_ARG, "malformed N-Triples line " + std::to_string(sc[0] + 1));
    const u64 n = sc[1], V = sc[2];
    rs = check_terms(c, n, (u32)std::min<u64>(V, 0xffffffffull));
    if (rs) return rs;
    ENSURE(c, ts, n * 4);
    ENSURE(c, tp, n * 4);
    ENSURE(c, to, n * 4);
    ENSURE(c, nterm_off, V * 8);
    ENSURE(c, nterm_len, V * 4);
    hipLaunchKernelGGL(k_nt_assign, dim3(go), dim3(RDF_BLOCK), 0, st, c->ntstart.as<u64>(), c->ntlen.as<u32>(),
                       c->nvalid.as<u32>(), c->nlpos.as<u32>(), nocc, c->nrep.as<u32>(), c->nfirst.as<u32>(),
                       c->nfid.as<u32>(), c->ts.as<u32>(), c->tp.as<u32>(), c->to.as<u32>(), c->nterm_off.as<u64>(),
                       c->nterm_len.as<u32>());
    HIP_TRY(c, hipGetLastError());
    HIP_TRY(c, hipEventRecord(c->ev[7], st));
    HIP_TRY(c, hipStreamSynchronize(st));
    if (ms) HIP_TRY(c, hipEventElapsedTime(ms, c->ev[6], c->ev[7]));
    // parse-only scratch (~36 B per term occurrence + the slot table): only the text and the term table stay,
    // which rdf_set_dictionary_parsed needs, so discovery gets the HBM back
    for (DevBuf* b : {&c->ncnt, &c->ncoff, &c->nlstart, &c->ntstart, &c->ntlen, &c->nvalid, &c->nlpos, &c->nhv,
                      &c->nslot, &c->ntab, &c->nrep, &c->nfirst, &c->nfid})
        b->release();
    c->s = c->ts.as<u32>();
    c->p = c->tp.as<u32>();
    c->o = c->to.as<u32>();
    c->n = n;
    c->V = (u32)V;
    c->stage = 1;
    c->paged = false;  // a paged run's state belongs to the previous input
    c->n_terms_parsed = V;
    c->parsed_dict = true;
    c->ingest_sharded = false;
    if (n_triples) *n_triples = n;
    if (num_terms) *num_terms = (u32)V;
    return RDF_OK;
}

// Term table of the last rdf_parse_ntriples: byte offset (into the parsed text) and length of term id i.
rdf_status rdf_copy_terms(rdf_ctx* c, uint64_t* offsets, uint32_t* lengths, uint64_t cap, uint64_t* n_copied) {
    if (!c) return RDF_ERR_ARG;
    const u64 n = std::min<u64>(cap, c->n_terms_parsed);
    if (n && (!offsets || !lengths)) return fail(c, RDF_ERR_ARG, "null term arrays");
    HIP_TRY(c, hipSetDevice(c->device));
    if (n) {
        HIP_TRY(c, hipMemcpyAsync(offsets, c->nterm_off.p, n * 8, hipMemcpyDeviceToHost, c->stream));
        HIP_TRY(c, hipMemcpyAsync(lengths, c->nterm_len.p, n * 4, hipMemcpyDeviceToHost, c->stream));
    }
    HIP_TRY(c, hipStreamSynchronize(c->stream));
    if (n_copied) *n_copied = n;
    return RDF_OK;
}

// ------------------------------------------------------------------------------------------------
// Stage 1: frequent conditions (FrequentConditionPlanner.constructFrequentConditionPlan)

// K1 partitioned over (s, p, o, n): bucket histogram, scatter of the low key bits, per-bucket LDS counting.
// counts_only: the dense counts land in cntg (sharded input: their nonzero entries go to the keys' owners);
// otherwise ranks, fbits and the rank-block totals bfreq are written (fc_unary_finish makes them global).
static rdf_status fc_unary_part(rdf_ctx* c, const u32* s, const u32* p, const u32* o, u64 n, int ubits, u64 NB,
                                bool counts_only) {
    hipStream_t st = c->stream;
    const u32 V = c->V ? c->V : 1;
    const u64 K = 3ull * V;
    ENSURE(c, usl, (NB + 1) * 4);
    // large inputs whose bucket counters leave one partition block per CU (NB x 4 B of LDS > 80 KB): the keys as u32,
    // grouped by bucket with two stable radix passes over the bucket bits, bucket starts by binary search (G = 1); the
    // keys live in K2's record buffers, which the next stage needs anyway.  c4 at 10^9 triples (22,891 buckets of 2^15
    // keys): K1 53.1 -> 42.9 ms; c4 at 0.4 (18,313 buckets, two blocks per CU) 14.1 -> 16.8 and c3 2.4 -> 4.6 lose, so
    // they keep the partition passes (profiles/r06_k1_radix_ab.log).  RDFIND_U1_RADIX_MIN=<3n> replaces the rule
    const bool radix_rule = c->u1_radix_min ? 3 * n >= c->u1_radix_min : 3 * n >= U1_RADIX_MIN && NB * 4 > U1_RADIX_LDS;
    const bool radix = radix_rule && 3 * n < (1ull << 32) && K <= 0xffffffffull;
    const void* recs = nullptr;
    unsigned G = 1;
    if (radix) {
        const u64 m = 3 * n;
        ENSURE(c, brkeys, m * 4);
        ENSURE(c, brkeys2, m * 4);
        ENSURE(c, uhist, (NB + 1) * 4);
        u32* keys = c->brkeys.as<u32>();
        u32* tmp = c->brkeys2.as<u32>();
        hipLaunchKernelGGL(k_u1_keys, dim3(grid_for(n, RDF_BLOCK, 8 * kGrid)), dim3(RDF_BLOCK), 0, st, s, p, o, n, V, keys);
        HIP_TRY(c, radix_partition_u32(c->ws, keys, tmp, m, ubits, ubits + bits_for(NB - 1), st));
        hipLaunchKernelGGL(k_u1_bucket_starts, dim3(grid_for(NB + 1, RDF_BLOCK, kGrid)), dim3(RDF_BLOCK), 0, st, keys, m,
                           ubits, (u32)NB, c->uhist.as<u32>());
        recs = keys;
    } else {
        G = (unsigned)std::max<u64>(1, std::min<u64>({1024, (n + 2047) / 2048, (1ull << 25) / NB}));
        const u64 nh = NB * G;
        ENSURE(c, uhist, (nh + 1) * 4);
        ENSURE(c, urecs, 3 * n * 2 + 16);
        const size_t lds = NB * 4;
        hipLaunchKernelGGL((k_u2_part<false>), dim3(G), dim3(RDF_BLOCK), lds, st, s, p, o, n, V, (u32)NB, ubits,
                           c->uhist.as<u32>(), (uint16_t*)nullptr);
        HIP_TRY(c, exclusive_scan_u32(c->ws, c->uhist.as<u32>(), c->uhist.as<u32>(), nh, c->uhist.as<u32>() + nh, st));
        hipLaunchKernelGGL((k_u2_part<true>), dim3(G), dim3(RDF_BLOCK), lds, st, s, p, o, n, V, (u32)NB, ubits,
                           c->uhist.as<u32>(), c->urecs.as<uint16_t>());
        recs = c->urecs.p;
    }
    HIP_TRY(c, hipGetLastError());
    hipLaunchKernelGGL(k_u2_slices, dim3((unsigned)NB), dim3(RDF_BLOCK), 0, st, c->uhist.as<u32>(), (u32)NB, G, ubits, K,
                       c->usl.as<u32>(), c->cntg.as<u32>());
    HIP_TRY(c, exclusive_scan_u32(c->ws, c->usl.as<u32>(), c->usl.as<u32>(), NB, c->usl.as<u32>() + NB, st));
    const u64 max_slices = NB + 3 * n / U2_SLICE + 1;  // >= sum over buckets of max(1, ceil(len / U2_SLICE))
    const int co = counts_only ? 1 : 0;
#define RDF_U2_COUNT(BITS, RT)                                                                                           \
    hipLaunchKernelGGL((k_u2_count<BITS, RT>), dim3((unsigned)max_slices), dim3(U2_CBLOCK), 0, st, (const RT*)recs,     \
                       c->uhist.as<u32>(), c->usl.as<u32>(), (u32)NB, G, K, V, c->ms, c->frank.as<u32>(),                \
                       c->bfreq.as<u32>(), c->fstage.as<u32>(), c->fbits.as<u64>(), dscal(c, 0), c->cntg.as<u32>(), co)
    if (ubits == 14) {
        if (radix) RDF_U2_COUNT(14, u32);
        else RDF_U2_COUNT(14, uint16_t);
        if (!counts_only)
            hipLaunchKernelGGL(k_u2_finish<14>, dim3((unsigned)NB), dim3(U2_CBLOCK), 0, st, c->usl.as<u32>(), (u32)NB, K, V,
                               c->ms, c->cntg.as<u32>(), c->frank.as<u32>(), c->bfreq.as<u32>(), c->fstage.as<u32>(),
                               c->fbits.as<u64>(), dscal(c, 0));
    } else {
        if (radix) RDF_U2_COUNT(15, u32);
        else RDF_U2_COUNT(15, uint16_t);
        if (!counts_only)
            hipLaunchKernelGGL(k_u2_finish<15>, dim3((unsigned)NB), dim3(U2_CBLOCK), 0, st, c->usl.as<u32>(), (u32)NB, K, V,
                               c->ms, c->cntg.as<u32>(), c->frank.as<u32>(), c->bfreq.as<u32>(), c->fstage.as<u32>(),
                               c->fbits.as<u64>(), dscal(c, 0));
    }
#undef RDF_U2_COUNT
    HIP_TRY(c, hipGetLastError());
    return RDF_OK;
}

// rank-block totals -> boff, U, the s / p / o split (frequent keys below V and 2V = boff of their rank block +
// the part below), fval, and global ranks in frank
static rdf_status fc_unary_finish(rdf_ctx* c, u64 nfreq[3]) {
    hipStream_t st = c->stream;
    const u32 V = c->V ? c->V : 1;
    const u64 K = 3ull * V;
    const u64 NR = (K + FR_R - 1) / FR_R;
    HIP_TRY(c, exclusive_scan_u32(c->ws, c->bfreq.as<u32>(), c->boff.as<u32>(), NR, c->boff.as<u32>() + NR, st));
    u64 sc[5];
    TRY(read_multi(c, {{c->boff.as<u32>() + NR, 4}, {c->boff.as<u32>() + (V >> FR_BITS), 4}, {dscal(c, 1), 8},
                       {c->boff.as<u32>() + ((2ull * V) >> FR_BITS), 4}, {dscal(c, 2), 8}}, sc));
    c->U = (u32)sc[0];
    const u64 b1 = sc[1] + sc[2], b2 = sc[3] + sc[4];
    nfreq[0] = b1;
    nfreq[1] = b2 - b1;
    nfreq[2] = sc[0] - b2;
    ENSURE(c, fval, std::max<u64>(c->U, 1) * 4);
    if (c->U)
        hipLaunchKernelGGL(k_u2_fval, dim3(grid_for(c->U, RDF_BLOCK, kGrid)), dim3(RDF_BLOCK), 0, st, c->boff.as<u32>(),
                           (u32)NR, c->fstage.as<u32>(), V, c->fval.as<u32>(), c->frank.as<u32>());
    HIP_TRY(c, hipMemsetAsync(c->boff.p, 0, (NR + 2) * 4, st));  // frank holds global ranks now
    return RDF_OK;
}

static rdf_status fc_unary_alloc(rdf_ctx* c) {
    const u32 V = c->V ? c->V : 1;
    const u64 K = 3ull * V;
    const u64 NR = (K + FR_R - 1) / FR_R;
    ENSURE(c, frank, K * 4);
    ENSURE(c, boff, (NR + 2) * 4);
    ENSURE(c, fbits, ((K + 63) / 64 + 1) * 8);
    ENSURE(c, cntg, K * 4);
    ENSURE(c, fstage, K * 4);
    ENSURE(c, bfreq, (NR + 2) * 4);
    HIP_TRY(c, hipMemsetAsync(dscal(c, 0), 0, 3 * 8, c->stream));
    return RDF_OK;
}

static int fc_ubits(u64 K) { return (K + (1ull << 14) - 1) >> 14 <= U2_MAXB ? 14 : 15; }

// K1 on the resident triples: frank (global ranks), fval, fbits, U; nfreq = frequent s / p / o conditions
static rdf_status fc_unary(rdf_ctx* c, u64 nfreq[3]) {
    hipStream_t st = c->stream;
    const u64 n = c->n;
    const u32 V = c->V ? c->V : 1;
    const u64 K = 3ull * V;
    const u64 NR = (K + FR_R - 1) / FR_R;
    TRY(fc_unary_alloc(c));
    const int ubits = fc_ubits(K);
    const u64 NB = (K + (1ull << ubits) - 1) >> ubits;
    if (n && NB <= U2_MAXB && !c->force_global_counts) {
        TRY(fc_unary_part(c, c->s, c->p, c->o, n, ubits, NB, false));
        return fc_unary_finish(c, nfreq);
    }
    // fallback (|V| beyond the partitioned range; RDFIND_COUNT_PATHS=atomic test hook): global-atomic counts,
    // then global ranks by one scan (boff = 0)
    ENSURE(c, cnt, K * 4);
    HIP_TRY(c, hipMemsetAsync(c->cnt.p, 0, K * 4, st));
    HIP_TRY(c, hipMemsetAsync(c->boff.p, 0, (NR + 2) * 4, st));
    if (n)
        hipLaunchKernelGGL(k_unary_count, dim3(std::min<unsigned>(grid_for(n, RDF_BLOCK * 4), 1024)), dim3(RDF_BLOCK), 0,
                           st, c->s, c->p, c->o, n, V, c->cnt.as<u32>());
    ENSURE(c, flags, K * 4);
    hipLaunchKernelGGL(k_frank_flags, dim3(grid_for(K, RDF_BLOCK, kGrid)), dim3(RDF_BLOCK), 0, st, c->cnt.as<u32>(), K,
                       c->ms, c->flags.as<u32>());
    hipLaunchKernelGGL(k_fbits_from_counts, dim3(grid_for(K, RDF_BLOCK, kGrid)), dim3(RDF_BLOCK), 0, st,
                       c->cnt.as<u32>(), K, c->ms, c->fbits.as<u64>());
    HIP_TRY(c, exclusive_scan_u32(c->ws, c->flags.as<u32>(), c->frank.as<u32>(), K, (u32*)dscal(c, 6), st));
    hipLaunchKernelGGL(k_count_frequent, dim3(grid_for(V, RDF_BLOCK, kGrid)), dim3(RDF_BLOCK), 0, st,
                       c->cnt.as<u32>(), V, c->ms, dscal(c, 0));
    TRY(read_scalars(c, 7));
    for (int t = 0; t < 3; ++t) nfreq[t] = c->hscal[t];
    c->U = (u32)c->hscal[6];
    ENSURE(c, fval, std::max<u64>(c->U, 1) * 4);
    hipLaunchKernelGGL(k_frank_final, dim3(grid_for(V, RDF_BLOCK, kGrid)), dim3(RDF_BLOCK), 0, st, c->cnt.as<u32>(), V,
                       c->ms, c->frank.as<u32>(), c->fval.as<u32>());
    return RDF_OK;
}

// sum (key, count) pairs in one global table (2x the pairs) and append the frequent keys at bkeys + *B; the pairs
// are either two arrays (keys, cnt) or interleaved words (cnt == nullptr).  *nkeys += distinct keys.
static rdf_status fc_sum_pairs(rdf_ctx* c, const u64* keys, const u32* cnt, u64 m, u64* B, u64* nkeys,
                               bool packed = false, DevBuf* outbuf = nullptr) {
    hipStream_t st = c->stream;
    DevBuf& out = outbuf ? *outbuf : c->bkeys;
    const u64 tcap = next_pow2(std::max<u64>(1024, 2 * m));
    ENSURE(c, lkeys, tcap * 8);  // lkeys / lvals are rebuilt afterwards (frequent-key lookup)
    ENSURE(c, lvals, tcap * 4);
    HIP_TRY(c, hipMemsetAsync(c->lkeys.p, 0xff, tcap * 8, st));
    HIP_TRY(c, hipMemsetAsync(c->lvals.p, 0, tcap * 4, st));
    if (m) {
        if (packed)
            hipLaunchKernelGGL(k_packed_insert, dim3(grid_for(m, RDF_BLOCK, kGrid)), dim3(RDF_BLOCK), 0, st, keys, m,
                               c->lkeys.as<u64>(), c->lvals.as<u32>(), tcap - 1);
        else if (cnt)
            hipLaunchKernelGGL(k_spill_insert, dim3(grid_for(m, RDF_BLOCK, kGrid)), dim3(RDF_BLOCK), 0, st, keys, cnt, m,
                               c->lkeys.as<u64>(), c->lvals.as<u32>(), tcap - 1);
        else
            hipLaunchKernelGGL(k_pairs_insert, dim3(grid_for(m, RDF_BLOCK, kGrid)), dim3(RDF_BLOCK), 0, st, keys, m,
                               c->lkeys.as<u64>(), c->lvals.as<u32>(), tcap - 1);
    }
    ENSURE(c, flags, tcap * 4);
    ENSURE(c, fpos, tcap * 8);
    HIP_TRY(c, hipMemsetAsync(dscal(c, 6), 0, 16, st));
    hipLaunchKernelGGL(k_bin_freq_flags, dim3(grid_for(tcap, RDF_BLOCK, kGrid)), dim3(RDF_BLOCK), 0, st, c->lkeys.as<u64>(),
                       c->lvals.as<u32>(), tcap, c->ms, c->flags.as<u32>(), dscal(c, 6));
    HIP_TRY(c, exclusive_scan_u32_u64(c->ws, c->flags.as<u32>(), c->fpos.as<u64>(), tcap, dscal(c, 7), st));
    TRY(read_scalars(c, 8));
    const u64 nf = c->hscal[7];
    HIP_TRY(c, out.grow_keep((size_t)(*B + nf + 1) * 8, st));
    hipLaunchKernelGGL(k_bin_freq_scatter, dim3(grid_for(tcap, RDF_BLOCK, kGrid)), dim3(RDF_BLOCK), 0, st, c->lkeys.as<u64>(),
                       c->flags.as<u32>(), c->fpos.as<u64>(), tcap, out.as<u64>() + *B);
    *nkeys += c->hscal[6];
    *B += nf;
    return RDF_OK;
}

// K2 partitioned over (s, p, o, n): (key, run count) records by key-hash bucket, LDS hash count per bucket slice.
// partials = false: frequent keys -> bkeys[0, *B), distinct count -> *nkeys (multi-slice buckets summed by
// fc_sum_pairs).  partials = true (sharded input): every local (key, count) partial -> the spill list
// (c->tkeys keys, c->pos counts), *S entries.
static rdf_status fc_binary_count(rdf_ctx* c, const u64* recs, const u32* bstart, u32 NBc, u32 Gc, bool partials, u64* B,
                                  u64* nkeys, u64* S);
static rdf_status fc_binary_part(rdf_ctx* c, const u32* s, const u32* p, const u32* o, u64 n, bool partials, u64* B,
                                 u64* nkeys, u64* S) {
    hipStream_t st = c->stream;
    const u32 V = c->V ? c->V : 1;
    // 2^13 buckets up to 3n = 64M keys (c2: 0.97 ms; 2^14: 1.16, 2^15: 1.46), then one bit per doubling up to
    // 2^15 (c3 at half scale, 132M keys: 7.6 ms at 2^13, 3.9 ms at 2^15: its buckets no longer spill)
    int bits = 1;
    while (bits < 13 && (1ull << bits) * 1024 < 3 * n) ++bits;
    while (bits >= 13 && bits < B2_MAXBITS && 3 * n > (B2_BIG << (bits - 13))) ++bits;
    const u32 NB2 = 1u << bits;
    const unsigned G2 = (unsigned)std::max<u64>(1, std::min<u64>({512, (n + 4095) / 4096, (1ull << 24) / NB2}));
    const u64 nh = (u64)NB2 * G2;
    const u64 maxrec = std::max<u64>(3 * n, 1);
    ENSURE(c, uhist, (nh + 1) * 4);
    ENSURE(c, brkeys, maxrec * 8);
    ENSURE(c, usl, (NB2 + 1) * 4);
    ENSURE(c, tkeys, maxrec * 8);  // spill list: keys
    ENSURE(c, pos, maxrec * 4);    // spill list: counts
    const u64 bmax = maxrec / std::max<u32>(c->ms, 1) + 1;  // frequent keys: each counts >= ms of <= 3n records
    ENSURE(c, bkeys, bmax * 8);
    static const int split_mode = getenv("RDFIND_B2_SPLIT") ? atoi(getenv("RDFIND_B2_SPLIT")) : 1;
    // large inputs: compact records grouped by hash prefix with the radix passes (k_b2_emit, radix_partition_hashed)
    static const u64 radix_min = getenv("RDFIND_B2_RADIX_MIN") ? strtoull(getenv("RDFIND_B2_RADIX_MIN"), nullptr, 10)
                                                               : B2_RADIX_MIN;
    if (split_mode != 0 && 3 * n >= radix_min && maxrec < (1ull << 32)) {
        ENSURE(c, brkeys2, maxrec * 8);
        HIP_TRY(c, hipMemsetAsync(dscal(c, 2), 0, 8, st));
        hipLaunchKernelGGL(k_b2_emit, dim3(grid_for(n, RDF_BLOCK * PART_U, kGrid)), dim3(RDF_BLOCK), 0, st, s, p, o, n, V,
                           c->fbits.as<u64>(), c->brkeys.as<u64>(), dscal(c, 2));
        HIP_TRY(c, hipGetLastError());
        TRY(read_scalars(c, 3));
        const u64 R = c->hscal[2];
        int T = 1;  // hash-prefix buckets of about 0.9 counting slice each
        while (T < 20 && R > ((u64)1 << T) * (B2_SLICE * 9 / 10)) ++T;
        u64* keys = c->brkeys.as<u64>();
        u64* tmp = c->brkeys2.as<u64>();
        HIP_TRY(c, radix_partition_hashed(c->ws, keys, tmp, R, T, ~B2_CBITS, st));
        const u32 NBh = 1u << T;
        ENSURE(c, bstart2, ((u64)NBh + 1) * 4);
        hipLaunchKernelGGL(k_b2_hbounds, dim3(grid_for(R + 1, RDF_BLOCK, kGrid)), dim3(RDF_BLOCK), 0, st, keys, R, T,
                           c->bstart2.as<u32>());
        HIP_TRY(c, hipGetLastError());
        return fc_binary_count(c, keys, c->bstart2.as<u32>(), NBh, 1, partials, B, nkeys, S);
    }
    const size_t lds = (size_t)NB2 * 4;
    hipLaunchKernelGGL((k_b2_part<false>), dim3(G2), dim3(B2_PBLOCK), lds, st, s, p, o, n, V, c->fbits.as<u64>(), bits,
                       c->uhist.as<u32>(), (u64*)nullptr);
    HIP_TRY(c, exclusive_scan_u32(c->ws, c->uhist.as<u32>(), c->uhist.as<u32>(), nh, c->uhist.as<u32>() + nh, st));
    hipLaunchKernelGGL((k_b2_part<true>), dim3(G2), dim3(B2_PBLOCK), lds, st, s, p, o, n, V, c->fbits.as<u64>(), bits,
                       c->uhist.as<u32>(), c->brkeys.as<u64>());
    // buckets that outgrow a counting slice are split by the next hash bits (RDFIND_B2_SPLIT=0: never)
    // into sub-buckets of about 0.9 slice each (smaller ones pay the counting block's per-slice table setup for
    // nothing); decided on the actual record count, read back only when the 3n bound says it may be needed
    // (RDFIND_B2_SPLIT=2: at least one split bit whatever the size, a test hook for the split path on small inputs)
    // a failed launch would leave uhist stale for the scan and the split below: caught here, not as a fault in a
    // consumer of garbage offsets
    HIP_TRY(c, hipGetLastError());
    int sub = 0;
    if (split_mode && 3 * n > (u64)NB2 * B2_SLICE) {
        u32 R = 0;
        TRY(read_u32(c, c->uhist.as<u32>() + nh, &R));
        while (sub < B2_SUB_MAX && (u64)R > ((u64)NB2 << sub) * (B2_SLICE * 9 / 10)) ++sub;
    }
    if (split_mode == 2 && n) sub = std::max(sub, 1);
    const u64* recs = c->brkeys.as<u64>();
    const u32* bstart = c->uhist.as<u32>();
    u32 NBc = NB2, Gc = G2;
    if (sub) {
        NBc = NB2 << sub;
        Gc = 1;
        ENSURE(c, brkeys2, maxrec * 8);
        ENSURE(c, bstart2, ((u64)NBc + 1) * 4);
        // RDFIND_TEST_FAIL_LAUNCH=k_b2_split (test hook): launched with an invalid block size, so the launch fails
        const unsigned sblock = c->test_fail_launch == "k_b2_split" ? 4 * 1024 : RDF_BLOCK;
        hipLaunchKernelGGL(k_b2_split, dim3(std::min<u32>(NB2, B2_SPLIT_GRID)), dim3(sblock), 0, st, c->brkeys.as<u64>(),
                           c->uhist.as<u32>(), NB2, G2, bits, sub, c->brkeys2.as<u64>(), c->bstart2.as<u32>());
        // bstart2 (the sub-bucket starts) is consumed as record offsets by k_b2_slices and k_b2_count: a launch that
        // did not run must stop here (the round-4 aperture violation in rdf_frequent_conditions was a count kernel
        // reading offsets no kernel had written)
        HIP_TRY(c, hipGetLastError());
        recs = c->brkeys2.as<u64>();
        bstart = c->bstart2.as<u32>();
    }
    return fc_binary_count(c, recs, bstart, NBc, Gc, partials, B, nkeys, S);
}

// K2 counting of bucketed records (bucket b = recs[bstart[b * G], bstart[(b + 1) * G])): (bucket, slice) list, LDS
// hash aggregation per slice, spill list summed in one global table
static rdf_status fc_binary_count(rdf_ctx* c, const u64* recs, const u32* bstart, u32 NBc, u32 Gc, bool partials, u64* B,
                                  u64* nkeys, u64* S) {
    hipStream_t st = c->stream;
    ENSURE(c, usl, ((u64)NBc + 1) * 4);
    hipLaunchKernelGGL(k_b2_slices, dim3(grid_for(NBc, RDF_BLOCK, kGrid)), dim3(RDF_BLOCK), 0, st, bstart, NBc, Gc,
                       c->usl.as<u32>());
    HIP_TRY(c, exclusive_scan_u32(c->ws, c->usl.as<u32>(), c->usl.as<u32>(), NBc, c->usl.as<u32>() + NBc, st));
    HIP_TRY(c, hipMemsetAsync(dscal(c, 3), 0, 3 * 8, st));
    hipLaunchKernelGGL(k_b2_count, dim3(256 * 3), dim3(RDF_BLOCK), 0, st, recs, bstart, c->usl.as<u32>(), NBc, Gc, c->ms, c->bkeys.as<u64>(), c->tkeys.as<u64>(),
                       (u32*)c->pos.p, dscal(c, 3), partials ? 1 : 0);
    TRY(read_scalars(c, 6));
    *B = c->hscal[3];
    *nkeys = c->hscal[4];
    *S = c->hscal[5];
    if (!partials && *S) TRY(fc_sum_pairs(c, c->tkeys.as<u64>(), (const u32*)c->pos.p, *S, B, nkeys));
    return RDF_OK;
}

// K2 fallback: one global open-addressing table sized from the emitted keys
static rdf_status fc_binary_global(rdf_ctx* c, u64* B, u64* nkeys) {
    hipStream_t st = c->stream;
    const u64 n = c->n;
    const u32 V = c->V ? c->V : 1;
    const u32* boff = c->boff.as<u32>();
    HIP_TRY(c, hipMemsetAsync(dscal(c, 3), 0, 8, st));
    hipLaunchKernelGGL(k_binary_emit_count, dim3(grid_for(n, RDF_BLOCK, kGrid)), dim3(RDF_BLOCK), 0, st, c->s, c->p, c->o,
                       n, V, c->frank.as<u32>(), boff, dscal(c, 3));
    TRY(read_scalars(c, 4));
    const u64 E = c->hscal[3];
    const u64 tcap = next_pow2(std::max<u64>(1024, E + E / 2 + 1));
    ENSURE(c, tkeys, tcap * 8);
    ENSURE(c, tcnt, tcap * 4);
    HIP_TRY(c, hipMemsetAsync(c->tkeys.p, 0xff, tcap * 8, st));
    HIP_TRY(c, hipMemsetAsync(c->tcnt.p, 0, tcap * 4, st));
    if (E)
        hipLaunchKernelGGL(k_binary_count, dim3(std::min<unsigned>(grid_for(n, RDF_BLOCK * 4), 1024)), dim3(RDF_BLOCK), 0, st,
                           c->s, c->p, c->o, n, V, c->frank.as<u32>(), boff, c->tkeys.as<u64>(), c->tcnt.as<u32>(), tcap - 1);
    ENSURE(c, flags, tcap * 4);
    ENSURE(c, pos, tcap * 8);
    HIP_TRY(c, hipMemsetAsync(dscal(c, 4), 0, 16, st));
    hipLaunchKernelGGL(k_bin_freq_flags, dim3(grid_for(tcap, RDF_BLOCK, kGrid)), dim3(RDF_BLOCK), 0, st, c->tkeys.as<u64>(),
                       c->tcnt.as<u32>(), tcap, c->ms, c->flags.as<u32>(), dscal(c, 4));
    HIP_TRY(c, exclusive_scan_u32_u64(c->ws, c->flags.as<u32>(), c->pos.as<u64>(), tcap, dscal(c, 5), st));
    TRY(read_scalars(c, 6));
    *nkeys = c->hscal[4];
    *B = c->hscal[5];
    ENSURE(c, bkeys, std::max<u64>(*B, 1) * 8);
    hipLaunchKernelGGL(k_bin_freq_scatter, dim3(grid_for(tcap, RDF_BLOCK, kGrid)), dim3(RDF_BLOCK), 0, st, c->tkeys.as<u64>(),
                       c->flags.as<u32>(), c->pos.as<u64>(), tcap, c->bkeys.as<u64>());
    return RDF_OK;
}

// frequent binary keys bkeys[0, B) -> sorted (deterministic binary ids) + the key -> id lookup table
static rdf_status fc_binary_index(rdf_ctx* c, u64 B) {
    hipStream_t st = c->stream;
    c->B = B;
    ENSURE_KEEP(c, bkeys, std::max<u64>(B, 1) * 8);
    ENSURE(c, bkeys_tmp, std::max<u64>(B, 1) * 8);
    {
        u64* k = c->bkeys.as<u64>();
        u64* t = c->bkeys_tmp.as<u64>();
        const int jb = c->V ? bits_for(c->V - 1) : 31;
        const bool dense = B && jb < 31;
        // one GPU: the keys by their conditions' global ranks when that saves a radix pass (frank / fval are final)
        const int rb = c->U ? bits_for(c->U - 1) : 31;
        const bool ranked = dense && c->nranks == 1 && radix_sort_passes(2 + 2 * rb) < radix_sort_passes(2 + 2 * jb);
        const dim3 g(grid_for(B, RDF_BLOCK, kGrid));
        if (ranked)
            hipLaunchKernelGGL(k_bkey_rank_repack, g, dim3(RDF_BLOCK), 0, st, k, B, rb, c->V, c->frank.as<u32>(),
                               c->fval.as<u32>(), 0);
        else if (dense)
            hipLaunchKernelGGL(k_bkey_repack, g, dim3(RDF_BLOCK), 0, st, k, B, jb, 0);
        HIP_TRY(c, radix_sort_u64(c->ws, k, t, B, ranked ? 2 + 2 * rb : dense ? 2 + 2 * jb : 64, st));
        if (k != c->bkeys.as<u64>()) std::swap(c->bkeys, c->bkeys_tmp);
        if (ranked)
            hipLaunchKernelGGL(k_bkey_rank_repack, g, dim3(RDF_BLOCK), 0, st, c->bkeys.as<u64>(), B, rb, c->V,
                               c->frank.as<u32>(), c->fval.as<u32>(), 1);
        else if (dense)
            hipLaunchKernelGGL(k_bkey_repack, g, dim3(RDF_BLOCK), 0, st, c->bkeys.as<u64>(), B, jb, 1);
    }
// lookup slots per key, in quarters: 16 = a table at most a quarter full.  Most K3 probes of a triple's pairs miss
// (the pair is not frequent), and a linear-probing miss at load 1/2 reads ~2.5 slots: at most 1/4 full, c2 emit 0.63 ->
// 0.58 ms, c3 5.90 -> 5.66, c4 at 0.4 36.5 -> 34.1 (at most 1/2: the old size; profiles/r06_lookup_load_ab.log).  Tables
// past 2 GB keep the half-full size
#ifndef RDF_LCAP_QUARTERS
#define RDF_LCAP_QUARTERS 16
#endif
    c->lcap = next_pow2(RDF_LCAP_QUARTERS * B / 4 + 16);
    if (c->lcap * 16 > (2ull << 30)) c->lcap = next_pow2(2 * B + 16);
    ENSURE(c, lkeys, c->lcap * (RDF_LOOKUP_SLOT16 ? 16 : 8));
    ENSURE(c, lvals, RDF_LOOKUP_SLOT16 ? 4 : c->lcap * 4);
    HIP_TRY(c, hipMemsetAsync(c->lkeys.p, 0xff, c->lcap * (RDF_LOOKUP_SLOT16 ? 16 : 8), st));
    if (B)
        hipLaunchKernelGGL(k_bin_lookup_build, dim3(grid_for(B, RDF_BLOCK, kGrid)), dim3(RDF_BLOCK), 0, st,
                           c->bkeys.as<u64>(), B, c->lkeys.as<u64>(), c->lvals.as<u32>(), c->lcap - 1);
    c->h_bkeys_valid = false;  // host copy made on first use (decode / copy-out)
    return RDF_OK;
}

static void fc_stats(rdf_ctx* c, const u64 nfreq[3], u64 nkeys, u64 B) {
    c->Us = (u32)nfreq[0];
    c->Up = (u32)nfreq[1];
    memset(&c->fstats, 0, sizeof(c->fstats));
    c->fstats.min_support = c->ms;
    for (int i = 0; i < 3; ++i) c->fstats.n_frequent_unary[i] = nfreq[i];
    c->fstats.n_binary_keys = nkeys;
    c->fstats.n_frequent_binary = B;
}

static rdf_status fc_begin(rdf_ctx* c, uint32_t min_support) {
    c->ms = min_support ? min_support : 1;  // a support of 0 admits exactly the captures that exist
    c->ar_on = false;
    c->n_rules = 0;
    c->class_pending = false;
    c->paged = false;
    for (int i = 0; i < RDF_NUM_TIMERS; ++i) c->tn[i] = 0;  // a failed run may have left segments behind
    c->pend_fc = c->pend_groups = c->pend_heavy = false;
    c->spare_fc = false;  // this stage's scratch is in use again
    HIP_TRY(c, hipEventRecord(c->ev[0], c->stream));
    HIP_TRY(c, hipMemsetAsync(c->scal.p, 0, 16 * sizeof(u64), c->stream));
    return RDF_OK;
}

static rdf_status fc_end(rdf_ctx* c) {
    HIP_TRY(c, hipEventRecord(c->ev[1], c->stream));
    c->pend_fc = true;
    c->spare_fc = true;
    c->stage = 2;
    return RDF_OK;
}

// read the pending stage timings (waits for their end events; free after the run's final stream wait)
static void settle_timings(rdf_ctx* c) {
    if (c->pend_fc && hipEventSynchronize(c->ev[1]) == hipSuccess) {
        (void)hipEventElapsedTime(&c->stage_ms[0], c->ev[0], c->ev[1]);
        tcollect(c, RDF_T_UNARY, RDF_T_BINARY + 1);
    }
    c->pend_fc = false;
    if (c->pend_groups && hipEventSynchronize(c->ev[3]) == hipSuccess) {
        (void)hipEventElapsedTime(&c->stage_ms[1], c->ev[2], c->ev[3]);
        tcollect(c, RDF_T_EMIT, RDF_T_HEAVYMASK + 1);
    }
    c->pend_groups = false;
}

rdf_status rdf_frequent_conditions(rdf_ctx* c, uint32_t min_support, rdf_fc_stats* stats) {
    if (!c) return RDF_ERR_ARG;
    if (c->stage < 1) return fail(c, RDF_ERR_STATE, "rdf_set_triples must be called first");
    HIP_TRY(c, hipSetDevice(c->device));
    TRY(hv_wait(c, true));
    TRY(fc_begin(c, min_support));
    u64 nfreq[3] = {0, 0, 0};
    tbegin(c, RDF_T_UNARY);
    TRY(fc_unary(c, nfreq));
    tend(c, RDF_T_UNARY);
    tbegin(c, RDF_T_BINARY);
    u64 B = 0, nkeys = 0, S = 0;
    if (c->n && !c->force_global_counts) TRY(fc_binary_part(c, c->s, c->p, c->o, c->n, false, &B, &nkeys, &S));
    else if (c->n) TRY(fc_binary_global(c, &B, &nkeys));
    TRY(fc_binary_index(c, B));
    tend(c, RDF_T_BINARY);
    TRY(fc_end(c));
    fc_stats(c, nfreq, nkeys, B);
    if (stats) *stats = c->fstats;
    return RDF_OK;
}

// Association rules (--use-ars, FrequentConditionPlanner.findAssociationRules, ALG/plan/FrequentConditionPlanner.scala:
// 129-193): triple counts of the frequent conditions (k_ar_count), rule bits per frequent binary key, the rules, and
// the frequent binary keys without the AR-implied ones (CreateJoinPartners.scala:99-141 never emits those captures).
// ar_counts: the counts of these triples into arcnt = [unary (U) | binary (B)] (sharded input: the slice's partial
// counts, summed over the ranks before ar_apply).
static rdf_status ar_counts(rdf_ctx* c, const u32* s, const u32* p, const u32* o, u64 n) {
    hipStream_t st = c->stream;
    const u32 V = c->V ? c->V : 1;
    const u64 B = c->B, U = c->U;
    ENSURE(c, arcnt, (U + B + 1) * 4);
    HIP_TRY(c, hipMemsetAsync(c->arcnt.p, 0, (U + B + 1) * 4, st));
    if (n && B)
        hipLaunchKernelGGL(k_ar_count, dim3(grid_for(n, RDF_BLOCK * 4, kGrid)), dim3(RDF_BLOCK), 0, st, s, p, o, n, V,
                           c->frank.as<u32>(), c->lkeys.as<u64>(), c->lvals.as<u32>(), c->lcap - 1, c->arcnt.as<u32>(),
                           c->arcnt.as<u32>() + U);
    return RDF_OK;
}

// the rules from the (global) counts in arcnt; the frequent binary keys become the kept ones
static rdf_status ar_apply(rdf_ctx* c) {
    hipStream_t st = c->stream;
    const u32 V = c->V ? c->V : 1;
    const u64 B = c->B, U = c->U;
    const u32* ucnt = c->arcnt.as<u32>();
    const u32* bcnt = c->arcnt.as<u32>() + U;
    ENSURE(c, ar_bits, std::max<u64>(B, 1) * 4);
    ENSURE(c, flags, (B + 1) * 4);
    ENSURE(c, fpos, (B + 1) * 4);
    ENSURE(c, pos, (B + 1) * 4);
    ENSURE(c, bkeys_tmp, std::max<u64>(B, 1) * 8);
    if (B)
        hipLaunchKernelGGL(k_ar_flags, dim3(grid_for(B, RDF_BLOCK, kGrid)), dim3(RDF_BLOCK), 0, st, c->bkeys.as<u64>(), B, V,
                           c->frank.as<u32>(), ucnt, bcnt, c->ar_bits.as<u32>(), c->flags.as<u32>(), (u32*)c->pos.p);
    // rule slots (flags) and kept keys (pos) -> exclusive offsets fpos / pos (in place)
    HIP_TRY(c, exclusive_scan_u32(c->ws, c->flags.as<u32>(), c->fpos.as<u32>(), B, c->fpos.as<u32>() + B, st));
    HIP_TRY(c, exclusive_scan_u32(c->ws, (u32*)c->pos.p, (u32*)c->pos.p, B, (u32*)c->pos.p + B, st));
    u64 v[2];
    TRY(read_multi(c, {{c->fpos.as<u32>() + B, 4}, {(u32*)c->pos.p + B, 4}}, v));
    const u64 NR = v[0], Bk = v[1];
    ENSURE(c, ar_rules, std::max<u64>(NR, 1) * 5 * 4);
    if (B)
        hipLaunchKernelGGL(k_ar_emit, dim3(grid_for(B, RDF_BLOCK, kGrid)), dim3(RDF_BLOCK), 0, st, c->bkeys.as<u64>(), B,
                           c->ar_bits.as<u32>(), bcnt, c->fpos.as<u32>(), (const u32*)c->pos.p, c->ar_rules.as<u32>(),
                           c->bkeys_tmp.as<u64>());
    std::swap(c->bkeys, c->bkeys_tmp);
    TRY(fc_binary_index(c, Bk));  // already sorted: the radix passes keep the order
    HIP_TRY(c, hipStreamSynchronize(st));
    c->n_rules = NR;
    c->ar_on = true;
    // n_frequent_binary stays the frequent-condition count of the reference's planner; the keys whose captures the
    // rules suppress are counted apart
    c->fstats.n_ar_suppressed = (u32)(B - Bk);
    return RDF_OK;
}

rdf_status rdf_association_rules(rdf_ctx* c, uint64_t* n_rules) {
    if (!c) return RDF_ERR_ARG;
    if (c->stage != 2) return fail(c, RDF_ERR_STATE, "rdf_association_rules follows rdf_frequent_conditions");
    if (c->ar_on) return fail(c, RDF_ERR_STATE, "association rules already applied to these frequent conditions");
    HIP_TRY(c, hipSetDevice(c->device));
    TRY(ar_counts(c, c->s, c->p, c->o, c->n));
    TRY(ar_apply(c));
    if (n_rules) *n_rules = c->n_rules;
    return RDF_OK;
}

rdf_status rdf_association_rule_count(rdf_ctx* c, uint64_t* n) {
    if (!c || !n) return RDF_ERR_ARG;
    if (!c->ar_on) return fail(c, RDF_ERR_STATE, "rdf_association_rules must be called first");
    *n = c->n_rules;
    return RDF_OK;
}

// rules as rdf_assoc_rule rows (antecedent type, consequent type, antecedent, consequent, support)
rdf_status rdf_copy_association_rules(rdf_ctx* c, rdf_assoc_rule* out, uint64_t cap, uint64_t* n_copied) {
    if (!c || (!out && cap)) return RDF_ERR_ARG;
    if (!c->ar_on) return fail(c, RDF_ERR_STATE, "rdf_association_rules must be called first");
    const u64 m = std::min<u64>(cap, c->n_rules);
    if (m) HIP_TRY(c, ctx_copy(c, out, c->ar_rules.p, m * sizeof(rdf_assoc_rule), hipMemcpyDeviceToHost));
    if (n_copied) *n_copied = m;
    return RDF_OK;
}

// unary compact dependent -> its AR-implied ref (after the capture compaction)
static rdf_status g_ar_refs(rdf_ctx* c) {
    hipStream_t st = c->stream;
    ENSURE(c, arref, std::max<u64>(c->Cu, 1) * 4);
    HIP_TRY(c, hipMemsetAsync(c->arref.p, 0xff, std::max<u64>(c->Cu, 1) * 4, st));
    if (c->n_rules)
        hipLaunchKernelGGL(k_ar_refs, dim3(grid_for(c->n_rules, RDF_BLOCK, kGrid)), dim3(RDF_BLOCK), 0, st,
                           c->ar_rules.as<u32>(), c->n_rules, c->V ? c->V : 1, c->frank.as<u32>(), c->support.as<u32>(),
                           c->fidx.as<u32>(), c->ms, c->arref.as<u32>());
    return RDF_OK;
}

// ------------------------------------------------------------------------------------------------
// Stage 2: capture groups (CreateJoinPartners -> UnionJoinCandidates -> UnionCombinedJoinCandidates)

static int heavy_threshold_from_hist(const u32* hist, u64 min_size) {
    // smallest bucket such that all groups in buckets >= it number at most HMAX
    u64 cum = 0;
    int best = -1;
    for (int b = 255; b >= 0; --b) {
        cum += hist[b];
        if (cum > (u64)HMAX) break;
        if (hist[b]) best = b;
    }
    (void)min_size;
    return best;
}

static u64 bucket_min_size(int b) {
    for (u64 s = 1; s < 64; ++s)
        if (size_bucket(s) == b) return s;
    int msb = b / 4, frac = b % 4;
    return (u64)(4 + frac) << (msb - 2);
}

static rdf_status parse_projection(rdf_ctx* c, const char* projection, int* proj) {
    const char* pr = projection ? projection : "spo";
    int m = 0;
    for (const char* q = pr; *q; ++q) {
        if (*q == 's') m |= 1;
        else if (*q == 'p') m |= 2;
        else if (*q == 'o') m |= 4;
        else return fail(c, RDF_ERR_ARG, std::string("invalid projection attribute in '") + pr + "'");
    }
    *proj = m;
    return RDF_OK;
}


// record key layout of this run's K3 records: capture << joinbits | join
static rdf_status g_record_bits(rdf_ctx* c) {
    c->spare_groups = false;  // a group build starts: its record buffers are in use
    c->jr_keep = false;
    c->dense_on = false;
    const u32 V = c->V ? c->V : 1;
    const u64 ncap = 2ull * c->U + c->B;  // compact candidate captures (k_frank_final)
    const int capbits = bits_for(ncap ? ncap - 1 : 0);
    const int joinbits = bits_for(V - 1);
    if (capbits + joinbits > 64) return fail(c, RDF_ERR_LIMIT, "join+capture bits exceed 64");
    if (6ull * V + c->B >= (1ull << 32)) return fail(c, RDF_ERR_LIMIT, "capture id space exceeds 2^32");
    c->capbits = capbits;
    c->joinbits = joinbits;
    c->ncap = ncap;
    return RDF_OK;
}

// this rank's join shard (sharded build; one GPU: every join value): the hash owner, or the hot table's
static JoinSel shard_sel(const rdf_ctx* c) {
    JoinSel js{c->rank, c->nranks, 0u, JOIN_ALL_HI};
    if (c->nranks > 1 && c->hot_n) {
        js.hot = c->hot.as<u64>();
        js.hmask = c->hot_mask;
    }
    return js;
}

// K3 emission of the selected join values (record buffers of cap_rec slots), K4 sort by (capture, join), K5 run
// bounds (cstart), fresh-record scan (fpos) and the records' supports -> sup[ncap].  The sorted records are left in
// c->rec_sorted; *Jout = their number.  Adds to c->J_emit and c->sort_passes_records.
// Join ranges (g_build_ranges) emit every range twice with the same selection: the first emission (cache = +1 + k,
// range k) keeps the scanned per-block offsets and the slot count, the second (cache = -1 - k) reuses them instead of
// re-running the count pass and its scan and read-back.  cache = 0: no reuse.
// a range's cached block offsets: one fixed-size slot per range (the grid follows a range's entry count, <= kGrid)
// the emission kernels' grid (K3): 8192 blocks, 4x the grid-stride kernels' (c2 emit 0.72 -> 0.63 ms, c4 at 0.4
// 40.8 -> 37.0 ms; a larger grid for every kernel cost K2 and the heavy mask as much; profiles/r06_emit_grid_ab.log)
#ifndef RDF_EMIT_GRID
#define RDF_EMIT_GRID 8192
#endif
static const unsigned kEmitGrid = RDF_EMIT_GRID;
// the join-range emission's grid (k_emit_join_bhist + k_emit_ranges): each block keeps a JH_BUCKETS row of the
// histogram (64 KB), so its grid stays at the grid-stride cap unless measured otherwise
#ifndef RDF_RANGE_EMIT_GRID
#define RDF_RANGE_EMIT_GRID 2048
#endif
static const unsigned kRangeEmitGrid = RDF_RANGE_EMIT_GRID;
static constexpr u64 ECACHE_STRIDE = RDF_EMIT_GRID + 1ull;
static rdf_status g_sort_support(rdf_ctx* c, u64* keys, u64* tmp, u64 Je, u32* sup, u64* Jout, u64* keep_out);
static rdf_status g_emit_range(rdf_ctx* c, int proj, JoinSel js, u64 cap_rec, u32* sup, u64* Jout, int cache = 0) {
    hipStream_t st = c->stream;
    const u64 n = c->n;
    const u32 V = c->V ? c->V : 1;
    const int capbits = c->capbits, joinbits = c->joinbits;
    HIP_TRY(c, hipMemsetAsync(c->scal.p, 0, 16 * sizeof(u64), st));
    ENSURE(c, rec, std::max<u64>(cap_rec, 1) * 8);
    ENSURE(c, rec_tmp, std::max<u64>(cap_rec, 1) * 8);
    u64* ebuf = c->rec.as<u64>();
    const u64 slot_cap = cap_rec;
    tbegin(c, RDF_T_EMIT);
    const int slot = cache > 0 ? cache - 1 : cache < 0 ? -cache - 1 : -1;
    // the selection takes a part of the join values (a join range, or a rank's shard): lazy condition-rank loads
    const bool lazy = js.nranks > 1 || js.lo != 0u || js.hi != JOIN_ALL_HI;
    const unsigned eg = grid_for(n, RDF_BLOCK, kEmitGrid);
    const u64 per = n ? (n + eg - 1) / eg : 0;
    ENSURE(c, eblk, 2 * (eg + 1ull) * 8);
    const bool reuse = cache < 0 && slot < (int)c->ecache_je.size();
    u64* overflow = (u64*)dscal(c, 8);  // the write pass's overflow word (zeroed above)
    // one pass (no count pass) when the record buffers hold 9 records per triple: every block writes its kept records
    // into its own region of rec_tmp (9 x per slots), then k_emit_compact packs the regions into rec by the scanned
    // block counts; no padding reaches the sort.  c2 emit 0.86 -> 0.73 ms, sort 1.79 -> 1.71, c3 step 72.4 -> 69.9 ms
    // (profiles/r05_emit_onepass_ab.log).  RDFIND_EMIT_ONEPASS=0: the count pass + write pass with padding
    static const bool onepass_env = !getenv("RDFIND_EMIT_ONEPASS") || atoi(getenv("RDFIND_EMIT_ONEPASS")) != 0;
    const bool onepass = onepass_env && cache == 0 && slot_cap >= 9 * n;
    if (onepass && n) {
        u64* eoff = c->eblk.as<u64>() + (eg + 1ull);
        HIP_TRY(c, hipMemsetAsync(c->eblk.as<u64>() + eg, 0, 8, st));  // records emitted, repeats included
        if (lazy)
            hipLaunchKernelGGL((k_emit_records<true, true>), dim3(eg), dim3(RDF_BLOCK), 0, st, c->s, c->p, c->o, n, per, V,
                               2u * c->U, c->frank.as<u32>(), c->lkeys.as<u64>(), c->lvals.as<u32>(), c->lcap - 1, proj,
                               joinbits, js, c->eblk.as<u64>(), (const u64*)nullptr, c->rec_tmp.as<u64>(), capbits + joinbits);
        else
            hipLaunchKernelGGL((k_emit_records<true, false>), dim3(eg), dim3(RDF_BLOCK), 0, st, c->s, c->p, c->o, n, per, V,
                               2u * c->U, c->frank.as<u32>(), c->lkeys.as<u64>(), c->lvals.as<u32>(), c->lcap - 1, proj,
                               joinbits, js, c->eblk.as<u64>(), (const u64*)nullptr, c->rec_tmp.as<u64>(), capbits + joinbits);
        HIP_TRY(c, hipGetLastError());
        HIP_TRY(c, exclusive_scan_u64(c->ws, c->eblk.as<u64>(), eoff, eg, dscal(c, 0), st));
        hipLaunchKernelGGL(k_emit_compact, dim3(eg), dim3(RDF_BLOCK), 0, st, c->rec_tmp.as<u64>(), 9 * per,
                           c->eblk.as<u64>(), eoff, ebuf);
        HIP_TRY(c, hipGetLastError());
        HIP_TRY(c, hipMemcpyAsync(dscal(c, 3), c->eblk.as<u64>() + eg, 8, hipMemcpyDeviceToDevice, st));
    }
    u64 je_early = ~0ull;  // the slot count, when read before the write pass
    if (cache > 0) {
        if ((int)c->ecache_je.size() <= slot) c->ecache_je.resize(slot + 1);
        HIP_TRY(c, c->ecache.grow_keep((size_t)(slot + 1) * ECACHE_STRIDE * 8, st));
    }
    if (n && !onepass) {
        // the write pass's block offsets: eg + 1 entries (the last one the slot count), each block bounded by the next
        if (reuse) {
            HIP_TRY(c, hipMemcpyAsync(c->eblk.p, c->ecache.as<u64>() + (u64)slot * ECACHE_STRIDE, (eg + 1ull) * 8ull,
                                      hipMemcpyDeviceToDevice, st));
        } else {
            if (lazy)
                hipLaunchKernelGGL((k_emit_records<false, true>), dim3(eg), dim3(RDF_BLOCK), 0, st, c->s, c->p, c->o, n, per, V,
                                   2u * c->U, c->frank.as<u32>(), c->lkeys.as<u64>(), c->lvals.as<u32>(), c->lcap - 1, proj,
                                   joinbits, js, c->eblk.as<u64>(), (const u64*)nullptr, (u64*)nullptr, capbits + joinbits);
            else
                hipLaunchKernelGGL((k_emit_records<false, false>), dim3(eg), dim3(RDF_BLOCK), 0, st, c->s, c->p, c->o, n, per, V,
                                   2u * c->U, c->frank.as<u32>(), c->lkeys.as<u64>(), c->lvals.as<u32>(), c->lcap - 1, proj,
                                   joinbits, js, c->eblk.as<u64>(), (const u64*)nullptr, (u64*)nullptr, capbits + joinbits);
            HIP_TRY(c, hipGetLastError());
            HIP_TRY(c, exclusive_scan_u64(c->ws, c->eblk.as<u64>(), c->eblk.as<u64>(), eg, c->eblk.as<u64>() + eg, st));
            HIP_TRY(c, hipMemcpyAsync(dscal(c, 0), c->eblk.as<u64>() + eg, 8, hipMemcpyDeviceToDevice, st));
            if (cache > 0)
                HIP_TRY(c, hipMemcpyAsync(c->ecache.as<u64>() + (u64)slot * ECACHE_STRIDE, c->eblk.p, (eg + 1ull) * 8ull,
                                          hipMemcpyDeviceToDevice, st));
            if (slot_cap < 9 * n) {  // a join range's buffers: the slot count is checked before the write pass
                TRY(read_scalars(c, 1));
                je_early = c->hscal[0];
                if (je_early > slot_cap)
                    return fail(c, RDF_ERR_LIMIT, "K3 emitted more records than the join range was sized for");
            }
        }
        if (lazy)
            hipLaunchKernelGGL((k_emit_records<true, true>), dim3(eg), dim3(RDF_BLOCK), 0, st, c->s, c->p, c->o, n, per, V,
                               2u * c->U, c->frank.as<u32>(), c->lkeys.as<u64>(), c->lvals.as<u32>(), c->lcap - 1, proj,
                               joinbits, js, overflow, c->eblk.as<u64>(), ebuf, capbits + joinbits);
        else
            hipLaunchKernelGGL((k_emit_records<true, false>), dim3(eg), dim3(RDF_BLOCK), 0, st, c->s, c->p, c->o, n, per, V,
                               2u * c->U, c->frank.as<u32>(), c->lkeys.as<u64>(), c->lvals.as<u32>(), c->lcap - 1, proj,
                               joinbits, js, overflow, c->eblk.as<u64>(), ebuf, capbits + joinbits);
        HIP_TRY(c, hipGetLastError());
    }
    tend(c, RDF_T_EMIT);
    u64 Je = 0;  // emitted record slots (repeats within an emission iteration are padding)
    if (n && !onepass) {
        // every block of the write pass stayed inside its region [off[b], off[b + 1]) (k_emit_records bounds it); the
        // overflow word says whether a block had more records than its region (a join range's second emission reusing
        // its first's offsets, if the two ever differed): an error, never a write past the buffer
        TRY(read_u64(c, overflow, &c->hscal[8]));
        if (c->hscal[8])
            return fail(c, RDF_ERR_LIMIT, "K3: a block emitted more records than its scanned region (records past it "
                                          "were not written)");
    }
    if (reuse) {
        Je = c->ecache_je[slot];
    } else {
        if (je_early == ~0ull) {
            TRY(read_scalars(c, onepass ? 4 : 1));
            je_early = c->hscal[0];
            // one pass: the kept records are sorted, the emitted ones (repeats included) count as n_records
            if (onepass && n && c->hscal[3] >= je_early) c->J_emit += c->hscal[3] - je_early;
        }
        Je = je_early;
        if (cache > 0) c->ecache_je[slot] = Je;
    }
    if (Je > slot_cap) return fail(c, RDF_ERR_LIMIT, "K3 emitted more records than the join range was sized for");
    return g_sort_support(c, ebuf, c->rec_tmp.as<u64>(), Je, sup, Jout, nullptr);
}

// fresh-record flags (c->flags) and capture run starts (c->cstart[0, ncap]) of J sorted records
static rdf_status g_fresh_bounds(rdf_ctx* c, const u64* keys, u64 J) {
    hipStream_t st = c->stream;
    HIP_TRY(c, hipMemsetAsync(c->cstart.p, 0xff, (c->ncap + 1) * 4, st));
    hipLaunchKernelGGL(k_fresh_bounds, dim3(grid_for(J + 1, RDF_BLOCK, kGrid)), dim3(RDF_BLOCK), 0, st, keys, J, c->ncap,
                       c->joinbits, c->flags.as<u32>(), c->cstart.as<u32>());
    hipLaunchKernelGGL(k_cstart_fix, dim3(grid_for(c->ncap + 1, RDF_BLOCK, kGrid)), dim3(RDF_BLOCK), 0, st, keys, J, c->ncap,
                       c->joinbits, c->cstart.as<u32>());
    return RDF_OK;
}

// K4 sort of Je emitted record slots (keys, with tmp as the other buffer; padding dropped) and K5 supports -> sup.
// keep_out: the sorted records must end there (keys == keep_out: a range of rstore, copied back after an odd number of
// passes).  Sets c->rec_sorted, *Jout.
static rdf_status g_sort_support(rdf_ctx* c, u64* keys, u64* tmp, u64 Je, u32* sup, u64* Jout, u64* keep_out) {
    hipStream_t st = c->stream;
    const u64 ncap = c->ncap;
    const int capbits = c->capbits, joinbits = c->joinbits;
    c->J_emit += Je;
    u64 J = 0;
    tbegin(c, RDF_T_SORT);
    HIP_TRY(c, radix_sort_u64_drop(c->ws, keys, tmp, Je, capbits + joinbits, (u32*)dscal(c, 1), &J, st));
    if (keep_out && keys != keep_out) {  // an odd number of passes ended in tmp
        if (J) HIP_TRY(c, hipMemcpyAsync(keep_out, keys, J * 8, hipMemcpyDeviceToDevice, st));
        keys = keep_out;
    }
    tend(c, RDF_T_SORT);
    *Jout = J;
    c->rec_sorted = keys;
    c->sort_passes_records += Je + (u64)(radix_sort_passes(capbits + joinbits) - 1) * J;
    // supports = distinct join values per capture: fresh (capture, join) records counted per key run
    ENSURE(c, flags, std::max<u64>(J, 1) * 4);
    ENSURE(c, fpos, (J + 1) * 4);
    ENSURE(c, cstart, (ncap + 1) * 4);
    tbegin(c, RDF_T_SUPPORT);
    TRY(g_fresh_bounds(c, keys, J));
    HIP_TRY(c, exclusive_scan_u32(c->ws, c->flags.as<u32>(), c->fpos.as<u32>(), J, c->fpos.as<u32>() + J, st));
    if (ncap)
        hipLaunchKernelGGL(k_run_support, dim3(grid_for(ncap, RDF_BLOCK, kGrid)), dim3(RDF_BLOCK), 0, st, c->cstart.as<u32>(),
                           ncap, c->fpos.as<u32>(), sup);
    tend(c, RDF_T_SUPPORT);
    return RDF_OK;
}

// K3 emission of this rank's join shard, K4 sort by (capture, join), K5 local supports -> c->support[ncap]
static rdf_status g_emit_sort_support(rdf_ctx* c, int proj) {
    TRY(g_record_bits(c));
    HIP_TRY(c, hipEventRecord(c->ev[2], c->stream));
    c->J_emit = 0;
    c->sort_passes_records = 0;
    ENSURE(c, support, std::max<u64>(c->ncap, 1) * 4);
    u64 J = 0;
    TRY(g_emit_range(c, proj, shard_sel(c), 9 * c->n, c->support.as<u32>(), &J));
    c->J = J;
    return RDF_OK;
}

// frequent-capture compaction (c->support = global supports): C, Cu, fidx, fcap, info, fext
static rdf_status g_compact_captures(rdf_ctx* c) {
    hipStream_t st = c->stream;
    const u32 V = c->V ? c->V : 1;
    const u64 ncap = c->ncap;
    ENSURE(c, flags, std::max<u64>(ncap, 1) * 4);
    ENSURE(c, fidx, (ncap + 1) * 4);
    hipLaunchKernelGGL(k_support_flags, dim3(grid_for(ncap, RDF_BLOCK, kGrid)), dim3(RDF_BLOCK), 0, st,
                       c->support.as<u32>(), ncap, c->ms, c->flags.as<u32>());
    HIP_TRY(c, exclusive_scan_u32(c->ws, c->flags.as<u32>(), c->fidx.as<u32>(), ncap, c->fidx.as<u32>() + ncap, st));
    u32 C = 0, Cu = 0;
    {
        u64 v[2];
        TRY(read_multi(c, {{c->fidx.as<u32>() + ncap, 4}, {c->fidx.as<u32>() + 2ull * c->U, 4}}, v));
        C = (u32)v[0];
        Cu = (u32)v[1];
    }
    c->C = C;
    c->Cu = Cu;
    ENSURE(c, fcap, std::max<u64>(C, 1) * 4);
    ENSURE(c, info, std::max<u64>(C, 1) * sizeof(CapInfo));
    hipLaunchKernelGGL(k_compact_captures, dim3(grid_for(ncap, RDF_BLOCK, kGrid)), dim3(RDF_BLOCK), 0, st,
                       c->support.as<u32>(), c->fidx.as<u32>(), ncap, c->ms, c->fcap.as<u32>(), c->info.as<CapInfo>());
    ENSURE(c, fext, std::max<u64>(C, 1) * 4);
    if (C)
        hipLaunchKernelGGL(k_external_ids, dim3(grid_for(C, RDF_BLOCK, kGrid)), dim3(RDF_BLOCK), 0, st, c->fcap.as<u32>(), C,
                           2u * c->U, V, c->fval.as<u32>(), c->Us, c->Up, c->fext.as<u32>());
    return RDF_OK;
}

// frequent-capture compaction (c->support = global supports), capture groups, dependent -> groups CSR
static rdf_status g_compact_groups(rdf_ctx* c) {
    hipStream_t st = c->stream;
    const u32 V = c->V ? c->V : 1;
    const u64 ncap = c->ncap, J = c->J;
    const int joinbits = c->joinbits;
    u64* keys = c->rec_sorted;
    tbegin(c, RDF_T_SUPPORT);
    ENSURE(c, flags, std::max(J, ncap) * 4);
    TRY(g_compact_captures(c));
    const u32 C = c->C;
    // distinct records of frequent captures -> dk = (compact capture << 32 | join) in (capture, join) order,
    // written to the record buffer that does not hold the sorted keys
    ENSURE(c, skip, (ncap + 1) * 4);
    if (ncap)
        hipLaunchKernelGGL(k_skip_counts, dim3(grid_for(ncap, RDF_BLOCK, kGrid)), dim3(RDF_BLOCK), 0, st, c->cstart.as<u32>(),
                           c->fpos.as<u32>(), c->support.as<u32>(), ncap, c->ms, c->flags.as<u32>());
    HIP_TRY(c, exclusive_scan_u32(c->ws, c->flags.as<u32>(), c->skip.as<u32>(), ncap, c->skip.as<u32>() + ncap, st));
    u64 fs[2];
    TRY(read_multi(c, {{c->fpos.as<u32>() + J, 4}, {c->skip.as<u32>() + ncap, 4}}, fs));
    const u64 Jf = fs[0] - fs[1];
    c->Jf = Jf;
    u64* dk = keys == c->rec.as<u64>() ? c->rec_tmp.as<u64>() : c->rec.as<u64>();
    ENSURE(c, fk, std::max<u64>(Jf, 1) * 8);
    ENSURE(c, fk_tmp, std::max<u64>(Jf, 1) * 8);
    if (J)
        hipLaunchKernelGGL(k_keep_scatter, dim3(grid_for(J, RDF_BLOCK, kGrid)), dim3(RDF_BLOCK), 0, st, keys, J, joinbits,
                           c->fpos.as<u32>(), c->skip.as<u32>(), c->support.as<u32>(), c->ms, c->fidx.as<u32>(), dk,
                           c->fk.as<u64>());
    tend(c, RDF_T_SUPPORT);
    tbegin(c, RDF_T_GROUPS);
    // dependent -> join offsets straight from dk; groups need the (join, capture) order: a stable sort of
    // fk = (join << 32 | capture) on the join bits keeps each group's captures ascending
    ENSURE(c, csup, std::max<u64>(C, 1) * 4);
    ENSURE(c, doff, (C + 1ull) * 8);
    ENSURE(c, dgrp, std::max<u64>(Jf, 1) * 4);
    if (C)
        hipLaunchKernelGGL(k_info_support_u32, dim3(grid_for(C, RDF_BLOCK, kGrid)), dim3(RDF_BLOCK), 0, st,
                           c->info.as<CapInfo>(), C, c->csup.as<u32>());
    if (Jf) {
        hipLaunchKernelGGL(k_key_offsets, dim3(grid_for(C + 1ull, RDF_BLOCK, kGrid)), dim3(RDF_BLOCK), 0, st, dk, Jf, C,
                           c->doff.as<u64>());
        u64* tk = c->fk.as<u64>();
        u64* tt = c->fk_tmp.as<u64>();
        HIP_TRY(c, radix_sort_u64_bits(c->ws, tk, tt, Jf, 32, 32 + joinbits, st));
        if (tk != c->fk.as<u64>()) std::swap(c->fk, c->fk_tmp);
    } else {
        HIP_TRY(c, hipMemsetAsync(c->doff.p, 0, (C + 1ull) * 8, st));
    }
    ENSURE(c, gflag, std::max<u64>(Jf, 1) * 4);
    ENSURE(c, gexcl, (Jf + 1) * 4);
    if (Jf)
        hipLaunchKernelGGL(k_group_flags, dim3(grid_for(Jf, RDF_BLOCK, kGrid)), dim3(RDF_BLOCK), 0, st, c->fk.as<u64>(), Jf,
                           c->gflag.as<u32>());
    HIP_TRY(c, exclusive_scan_u32(c->ws, c->gflag.as<u32>(), c->gexcl.as<u32>(), Jf, c->gexcl.as<u32>() + Jf, st));
    u32 G32 = 0;
    TRY(read_u32(c, c->gexcl.as<u32>() + Jf, &G32));
    const u64 G = G32;
    c->G = G;
    ENSURE(c, goff, (G + 1) * 8);
    ENSURE(c, gcap, std::max<u64>(Jf, 1) * 4 + 16);  // + 16 B: the light pass reads whole aligned quads
    ENSURE(c, gmap, (u64)V * 4);
    if (Jf) {
        hipLaunchKernelGGL(k_group_build, dim3(grid_for(Jf, RDF_BLOCK, kGrid)), dim3(RDF_BLOCK), 0, st, c->fk.as<u64>(), Jf,
                           c->gflag.as<u32>(), c->gexcl.as<u32>(), c->goff.as<u64>(), c->gcap.as<u32>(), c->gmap.as<u32>());
        hipLaunchKernelGGL(k_dgrp, dim3(grid_for(Jf, RDF_BLOCK, kGrid)), dim3(RDF_BLOCK), 0, st, dk, Jf, c->gmap.as<u32>(),
                           c->dgrp.as<u32>());
    }
    c->hscal[14] = Jf;
    HIP_TRY(c, hipMemcpyAsync(c->goff.as<u64>() + G, c->hscal + 14, 8, hipMemcpyHostToDevice, st));
    tend(c, RDF_T_GROUPS);
    return RDF_OK;
}

// Capture groups in ranges of join values, for inputs whose K3 records exceed what one sort holds (the u32 record
// offsets of K4/K5: n >= 2^32 / 9 triples; c4 at full size emits ~5.8·10^9 records) or the memory of one pass.  The
// reference has no such ceiling: Flink's sort-based groupBy("joinValue") spills (ALG/programs/RDFind.scala:339-345).
// Pass 1 (g_ranges_supports):
//  1. records per join bucket (k_emit_join_bhist) -> consecutive bucket ranges of at most max_range records each;
//  2. per range: K3-K5 (g_emit_range), its supports summed into c->support (a join value's records are all in one
//     range, so the ranges' distinct (capture, join) counts add up).
// Pass 2 (g_ranges_groups):
//  3. capture compaction; doff = scan of the frequent captures' record counts (a frequent capture keeps one record per
//     join value: its support on one GPU, its local support `lsup` on a rank of a sharded run);
//  4. per range again: K3-K5, the kept records -> that range's groups appended at (G0, Jf0) and its dependent ->
//     group entries placed behind the earlier ranges' (dcur).  Ranges ascend in join value and groups are numbered in
//     join order, so goff / gcap / gmap / dgrp are exactly the one-pass build's.
// One GPU runs the passes back to back (g_build_ranges).  A rank of a sharded run (own = its join shard) runs pass 1
// on the triples it received, all-reduces the supports, and runs pass 2 (sh_phase14 -> sh_phase1).
// Keep pass 1's sorted records of every range (rstore: the ranges' record counts, 8 B each) when they fit beside the
// range scratch and the build's global arrays (the bound of auto_range_records): pass 2 then reads them instead of
// emitting and sorting every range a second time (c4 at 10^9 triples: 47 GB kept, one emission and one sort saved
// per range).  Otherwise, or when the allocation fails, pass 2 re-emits.
static rdf_status g_range_keep_plan(rdf_ctx* c) {
    const std::vector<rdf_ctx::JoinRange>& ranges = c->jranges;
    c->jr_keep = false;
    if (!c->range_keep || ranges.empty() || ranges.size() > EMIT_MAX_RANGES) return RDF_OK;
    u64 total = 0;
    c->jr_seg.assign(ranges.size() + 1, 0);
    c->jr_J.assign(ranges.size(), 0);
    for (size_t k = 0; k < ranges.size(); ++k) {
        c->jr_seg[k] = total;
        total += ranges[k].recs;
    }
    c->jr_seg[ranges.size()] = total;
    size_t free_b = 0, total_b = 0;
    if (hipMemGetInfo(&free_b, &total_b) != hipSuccess) return RDF_OK;
    // held by this context and reusable here: the spare stages' scratch and the range buffers of an earlier build
    const u64 held = (u64)c->brkeys.cap + c->brkeys2.cap + c->tkeys.cap + c->urecs.cap +
                     (c->spare_x ? (u64)c->xsend.cap + c->xrecv.cap : 0ull) + c->rec.cap + c->rec_tmp.cap + c->fk.cap +
                     c->fk_tmp.cap + c->rstore.cap;
    const u64 global = 8 * 9 * c->n / 2 + 16ull * (c->V ? c->V : 1) + (4ull << 30);
    const u64 need = 8 * total + 40 * c->jr_cap_rec + global;  // rec_tmp (8 B per record) is not used when keeping
    if ((u64)free_b + held < need) {
        (void)hipStreamSynchronize(c->stream);
        c->rstore.release();  // an earlier build's: the range buffers may need the room
        return RDF_OK;
    }
    (void)hipStreamSynchronize(c->stream);
    c->rec_tmp.release();  // not used by a kept build (an earlier build's)
    hipError_t e = c->rstore.ensure(std::max<u64>(total, 1) * 8);
    if (e == hipErrorOutOfMemory && reclaim_spare(c, &c->rstore)) e = c->rstore.ensure(std::max<u64>(total, 1) * 8);
    (void)hipGetLastError();
    c->jr_keep = e == hipSuccess;
    return RDF_OK;
}

// K3 of every range in one emission into its rstore region (k_emit_ranges: a count pass per (range, block), one scan,
// the write pass): each triple is read twice for all ranges instead of twice per range.  The regions' sizes are the
// join histogram's range counts; the scanned counts must agree with them.
static rdf_status g_emit_all_ranges(rdf_ctx* c, int proj, JoinSel own) {
    hipStream_t st = c->stream;
    const u64 n = c->n;
    const u32 V = c->V ? c->V : 1;
    const std::vector<rdf_ctx::JoinRange>& ranges = c->jranges;
    const u32 nr = (u32)ranges.size();
    ENSURE(c, rec, std::max<u64>(c->jr_cap_rec, 1) * 8);  // the ranges' sort buffer
    // the ranges' first join values, then their first join buckets (+ the end)
    const int jshift = c->joinbits > JH_BITS ? c->joinbits - JH_BITS : 0;
    std::vector<u32> lo(2 * nr + 1);
    for (u32 k = 0; k < nr; ++k) {
        lo[k] = ranges[k].lo;
        lo[nr + k] = ranges[k].lo >> jshift;
    }
    lo[2 * nr] = JH_BUCKETS;
    ENSURE(c, jrmap, (2 * nr + 1) * 4ull);
    HIP_TRY(c, ctx_copy(c, c->jrmap.p, lo.data(), (2 * nr + 1) * 4ull, hipMemcpyHostToDevice));
    const unsigned eg = grid_for(n, RDF_BLOCK, kRangeEmitGrid);
    const u64 per = n ? (n + eg - 1) / eg : 0;
    const u64 nb = (u64)nr * eg;
    ENSURE(c, eblk, (nb + 1) * 8);
    HIP_TRY(c, hipMemsetAsync(c->scal.p, 0, 16 * sizeof(u64), st));
    const bool lazy = own.nranks > 1;
    const int recbits = c->capbits + c->joinbits;
    const u32 twoU = 2u * c->U;
    tbegin(c, RDF_T_EMIT);
    if (n) {  // per (range, block) counts from the histogram pass's block rows
        hipLaunchKernelGGL(k_range_block_counts, dim3(grid_for(nb * RDF_WAVE, RDF_BLOCK, 1u << 30)), dim3(RDF_BLOCK), 0, st,
                           c->jbh.as<u32>(), eg, c->jrmap.as<u32>() + nr, nr, c->eblk.as<u64>());
        HIP_TRY(c, hipGetLastError());
        HIP_TRY(c, exclusive_scan_u64(c->ws, c->eblk.as<u64>(), c->eblk.as<u64>(), nb, c->eblk.as<u64>() + nb, st));
    }
    // the regions must be the histogram's: each range's first block offset = its rstore offset
    std::vector<u64> off(nb + 1, 0);
    if (n) HIP_TRY(c, ctx_copy(c, off.data(), c->eblk.p, (nb + 1) * 8, hipMemcpyDeviceToHost));
    for (u32 k = 0; k <= nr; ++k)
        if ((n ? off[(u64)k * eg] : 0) != c->jr_seg[k])
            return fail(c, RDF_ERR_LIMIT, "K3 records per join range disagree with the join histogram");
    if (n) {
        u64* overflow = (u64*)dscal(c, 8);  // zeroed above
        if (lazy)
            hipLaunchKernelGGL((k_emit_ranges<true>), dim3(eg), dim3(RDF_BLOCK), 0, st, c->s, c->p, c->o, n, per, V, twoU,
                               c->frank.as<u32>(), c->lkeys.as<u64>(), c->lvals.as<u32>(), c->lcap - 1, proj, c->joinbits, own,
                               c->jrmap.as<u32>(), nr, overflow, c->eblk.as<u64>(), c->rstore.as<u64>(), recbits);
        else
            hipLaunchKernelGGL((k_emit_ranges<false>), dim3(eg), dim3(RDF_BLOCK), 0, st, c->s, c->p, c->o, n, per, V, twoU,
                               c->frank.as<u32>(), c->lkeys.as<u64>(), c->lvals.as<u32>(), c->lcap - 1, proj, c->joinbits, own,
                               c->jrmap.as<u32>(), nr, overflow, c->eblk.as<u64>(), c->rstore.as<u64>(), recbits);
        HIP_TRY(c, hipGetLastError());
        // every (range, block) region ends at the next offset; records past it were not written
        TRY(read_u64(c, overflow, &c->hscal[8]));
        if (c->hscal[8])
            return fail(c, RDF_ERR_LIMIT, "K3 records per (join range, block) disagree with the join histogram");
    }
    tend(c, RDF_T_EMIT);
    return RDF_OK;
}

static rdf_status g_ranges_supports(rdf_ctx* c, int proj, u64 max_range, JoinSel own) {
    hipStream_t st = c->stream;
    const u64 n = c->n;
    const u32 V = c->V ? c->V : 1;
    TRY(g_record_bits(c));
    const u64 ncap = c->ncap;
    const int joinbits = c->joinbits;
    HIP_TRY(c, hipEventRecord(c->ev[2], st));
    c->J_emit = 0;
    c->sort_passes_records = 0;
    // the frequent-condition stage's record scratch (up to 84 GB at 10^9 triples) is spare from here on: reclaimed
    // by the range buffers' allocation if they need the room
    // 1. ranges
    const int jshift = joinbits > JH_BITS ? joinbits - JH_BITS : 0;
    ENSURE(c, jhist, JH_BUCKETS * 8);
    HIP_TRY(c, hipMemsetAsync(c->jhist.p, 0, JH_BUCKETS * 8, st));
    // the blocks of the emission (g_emit_all_ranges): their bucket histograms give its per-range block offsets
    const unsigned eg = grid_for(n, RDF_BLOCK, kRangeEmitGrid);
    const u64 per = n ? (n + eg - 1) / eg : 0;
    ENSURE(c, jbh, (u64)eg * JH_BUCKETS * 4);
    tbegin(c, RDF_T_EMIT);
    if (n) {
        if (own.nranks > 1)
            hipLaunchKernelGGL(k_emit_join_bhist<true>, dim3(eg), dim3(JH_BLOCK), 0, st, c->s, c->p, c->o, n, per, V, 2u * c->U,
                               c->frank.as<u32>(), c->lkeys.as<u64>(), c->lvals.as<u32>(), c->lcap - 1, proj, joinbits, own,
                               jshift, c->jbh.as<u32>(), c->jhist.as<u64>());
        else
            hipLaunchKernelGGL(k_emit_join_bhist<false>, dim3(eg), dim3(JH_BLOCK), 0, st, c->s, c->p, c->o, n, per, V, 2u * c->U,
                               c->frank.as<u32>(), c->lkeys.as<u64>(), c->lvals.as<u32>(), c->lcap - 1, proj, joinbits, own,
                               jshift, c->jbh.as<u32>(), c->jhist.as<u64>());
        HIP_TRY(c, hipGetLastError());
    }
    tend(c, RDF_T_EMIT);
    std::vector<u64> h(JH_BUCKETS);
    HIP_TRY(c, hipMemcpyAsync(h.data(), c->jhist.p, JH_BUCKETS * 8, hipMemcpyDeviceToHost, st));
    HIP_TRY(c, hipStreamSynchronize(st));
    std::vector<rdf_ctx::JoinRange>& ranges = c->jranges;
    ranges.clear();
    u64 acc = 0, cap_rec = 1;
    u32 lo = 0;
    for (u32 b = 0; b < JH_BUCKETS; ++b) {
        if (acc && acc + h[b] > max_range) {
            ranges.push_back({lo, b << jshift, acc});
            lo = b << jshift;
            acc = 0;
        }
        acc += h[b];
    }
    ranges.push_back({lo, JOIN_ALL_HI, acc});
    for (const rdf_ctx::JoinRange& r : ranges) cap_rec = std::max(cap_rec, r.recs);
    if (cap_rec >= (1ull << 32) - 1)
        return fail(c, RDF_ERR_LIMIT, "one join bucket holds >= 2^32 capture records");
    c->jr_cap_rec = cap_rec;
    c->n_group_ranges = ranges.size();
    TRY(g_range_keep_plan(c));
    // 2. supports
    ENSURE(c, support, std::max<u64>(ncap, 1) * 4);
    ENSURE(c, rsup, std::max<u64>(ncap, 1) * 4);
    HIP_TRY(c, hipMemsetAsync(c->support.p, 0, std::max<u64>(ncap, 1) * 4, st));
    u64 Jtot = 0;
    c->ecache_je.clear();
    if (c->jr_keep) TRY(g_emit_all_ranges(c, proj, own));
    for (size_t k = 0; k < ranges.size(); ++k) {
        const rdf_ctx::JoinRange& r = ranges[k];
        u64 J = 0;
        JoinSel js = own;
        js.lo = r.lo;
        js.hi = r.hi;
        if (c->jr_keep) {  // range k's records are emitted (g_emit_all_ranges): its sort in place
            u64* seg = c->rstore.as<u64>() + c->jr_seg[k];
            TRY(g_sort_support(c, seg, c->rec.as<u64>(), c->jr_seg[k + 1] - c->jr_seg[k], c->rsup.as<u32>(), &J, seg));
            c->jr_J[k] = J;
        } else {
            TRY(g_emit_range(c, proj, js, cap_rec, c->rsup.as<u32>(), &J, 1 + (int)k));
        }
        Jtot += J;
        if (ncap)
            hipLaunchKernelGGL(k_add_u32, dim3(grid_for(ncap, RDF_BLOCK, kGrid)), dim3(RDF_BLOCK), 0, st, c->support.as<u32>(),
                               c->rsup.as<u32>(), ncap);
    }
    c->J = Jtot;
    return RDF_OK;
}

// pass 2 of a kept range: its sorted records from rstore, their run bounds (cstart) and fresh-record scan (fpos)
static rdf_status g_restore_range(rdf_ctx* c, size_t k, u64* Jout) {
    hipStream_t st = c->stream;
    const u64 J = c->jr_J[k], ncap = c->ncap;
    u64* keys = c->rstore.as<u64>() + c->jr_seg[k];
    ENSURE(c, flags, std::max<u64>(J, 1) * 4);
    ENSURE(c, fpos, (J + 1) * 4);
    ENSURE(c, cstart, (ncap + 1) * 4);
    ENSURE(c, rec, std::max<u64>(c->jr_cap_rec, 1) * 8);  // the kept records' destination (dk) in pass 2
    tbegin(c, RDF_T_SUPPORT);
    TRY(g_fresh_bounds(c, keys, J));
    HIP_TRY(c, exclusive_scan_u32(c->ws, c->flags.as<u32>(), c->fpos.as<u32>(), J, c->fpos.as<u32>() + J, st));
    tend(c, RDF_T_SUPPORT);
    c->rec_sorted = keys;
    *Jout = J;
    return RDF_OK;
}

// pass 2 (above): c->support holds the global supports; local_sup (sharded: this rank's supports from pass 1) gives
// each frequent capture's record count here, nullptr = its global support (one GPU)
static rdf_status g_ranges_groups(rdf_ctx* c, int proj, JoinSel own, const u32* local_sup) {
    hipStream_t st = c->stream;
    const u32 V = c->V ? c->V : 1;
    const u64 ncap = c->ncap;
    const int joinbits = c->joinbits;
    const std::vector<rdf_ctx::JoinRange>& ranges = c->jranges;
    const u64 cap_rec = c->jr_cap_rec;
    const u64 J_emit = c->J_emit, Jtot = c->J;
    // 3. compaction; each frequent capture's dependent -> group list has one entry per (local) join value
    tbegin(c, RDF_T_SUPPORT);
    TRY(g_compact_captures(c));
    const u32 C = c->C;
    ENSURE(c, csup, std::max<u64>(C, 1) * 4);
    ENSURE(c, doff, (C + 1ull) * 8);
    ENSURE(c, dcur, std::max<u64>(C, 1) * 4);
    if (C)
        hipLaunchKernelGGL(k_info_support_u32, dim3(grid_for(C, RDF_BLOCK, kGrid)), dim3(RDF_BLOCK), 0, st,
                           c->info.as<CapInfo>(), C, c->csup.as<u32>());
    const u32* nrec = c->csup.as<u32>();
    if (local_sup) {  // records per frequent capture on this rank: its local support (dcur is scratch until zeroed)
        if (C)
            hipLaunchKernelGGL(k_gather_u32, dim3(grid_for(C, RDF_BLOCK, kGrid)), dim3(RDF_BLOCK), 0, st, local_sup,
                               c->fcap.as<u32>(), (u64)C, c->dcur.as<u32>());
        nrec = c->dcur.as<u32>();
    }
    HIP_TRY(c, exclusive_scan_u32_u64(c->ws, nrec, c->doff.as<u64>(), C, c->doff.as<u64>() + C, st));
    tend(c, RDF_T_SUPPORT);
    u64 Jf = 0;
    TRY(read_u64(c, c->doff.as<u64>() + C, &Jf));
    c->Jf = Jf;
    const u64 Gmax = std::min<u64>(V, Jf);
    ENSURE(c, goff, (Gmax + 1) * 8);
    ENSURE(c, gcap, std::max<u64>(Jf, 1) * 4 + 16);  // + 16 B: the light pass reads whole aligned quads
    ENSURE(c, gmap, (u64)V * 4);
    ENSURE(c, dgrp, std::max<u64>(Jf, 1) * 4);
    ENSURE(c, offp, (C + 1ull) * 8);
    ENSURE(c, skip, (ncap + 1) * 4);
    HIP_TRY(c, hipMemsetAsync(c->dcur.p, 0, std::max<u64>(C, 1) * 4, st));
    // 4. groups, range by range
    u64 Jf0 = 0, G0 = 0;
    for (size_t k = 0; k < ranges.size(); ++k) {
        const rdf_ctx::JoinRange& r = ranges[k];
        u64 J = 0;
        JoinSel js = own;
        js.lo = r.lo;
        js.hi = r.hi;
        if (c->jr_keep) TRY(g_restore_range(c, k, &J));
        else TRY(g_emit_range(c, proj, js, cap_rec, c->rsup.as<u32>(), &J, -1 - (int)k));
        u64* keys = c->rec_sorted;
        tbegin(c, RDF_T_SUPPORT);
        ENSURE(c, flags, std::max<u64>(std::max<u64>(J, ncap), 1) * 4);
        if (ncap)
            hipLaunchKernelGGL(k_skip_counts, dim3(grid_for(ncap, RDF_BLOCK, kGrid)), dim3(RDF_BLOCK), 0, st, c->cstart.as<u32>(),
                               c->fpos.as<u32>(), c->support.as<u32>(), ncap, c->ms, c->flags.as<u32>());
        HIP_TRY(c, exclusive_scan_u32(c->ws, c->flags.as<u32>(), c->skip.as<u32>(), ncap, c->skip.as<u32>() + ncap, st));
        u64 fs[2];
        TRY(read_multi(c, {{c->fpos.as<u32>() + J, 4}, {c->skip.as<u32>() + ncap, 4}}, fs));
        const u64 Jr = fs[0] - fs[1];  // this range's kept records
        u64* dk = keys == c->rec.as<u64>() ? c->rec_tmp.as<u64>() : c->rec.as<u64>();
        ENSURE(c, fk, std::max<u64>(Jr, 1) * 8);
        ENSURE(c, fk_tmp, std::max<u64>(Jr, 1) * 8);
        if (J)
            hipLaunchKernelGGL(k_keep_scatter, dim3(grid_for(J, RDF_BLOCK, kGrid)), dim3(RDF_BLOCK), 0, st, keys, J, joinbits,
                               c->fpos.as<u32>(), c->skip.as<u32>(), c->support.as<u32>(), c->ms, c->fidx.as<u32>(), dk,
                               c->fk.as<u64>());
        tend(c, RDF_T_SUPPORT);
        tbegin(c, RDF_T_GROUPS);
        if (Jr) {
            u64* tk = c->fk.as<u64>();
            u64* tt = c->fk_tmp.as<u64>();
            HIP_TRY(c, radix_sort_u64_bits(c->ws, tk, tt, Jr, 32, 32 + joinbits, st));
            if (tk != c->fk.as<u64>()) std::swap(c->fk, c->fk_tmp);
        }
        ENSURE(c, gflag, std::max<u64>(Jr, 1) * 4);
        ENSURE(c, gexcl, (Jr + 1) * 4);
        if (Jr)
            hipLaunchKernelGGL(k_group_flags, dim3(grid_for(Jr, RDF_BLOCK, kGrid)), dim3(RDF_BLOCK), 0, st, c->fk.as<u64>(), Jr,
                               c->gflag.as<u32>());
        HIP_TRY(c, exclusive_scan_u32(c->ws, c->gflag.as<u32>(), c->gexcl.as<u32>(), Jr, c->gexcl.as<u32>() + Jr, st));
        u32 Gr = 0;
        TRY(read_u32(c, c->gexcl.as<u32>() + Jr, &Gr));
        if (G0 + Gr > Gmax || Jf0 + Jr > Jf) return fail(c, RDF_ERR_LIMIT, "join ranges disagree on the kept records");
        if (Jr) {
            hipLaunchKernelGGL(k_group_build_at, dim3(grid_for(Jr, RDF_BLOCK, kGrid)), dim3(RDF_BLOCK), 0, st, c->fk.as<u64>(), Jr,
                               c->gflag.as<u32>(), c->gexcl.as<u32>(), Jf0, (u32)G0, c->goff.as<u64>(), c->gcap.as<u32>(),
                               c->gmap.as<u32>());
            hipLaunchKernelGGL(k_key_offsets, dim3(grid_for(C + 1ull, RDF_BLOCK, kGrid)), dim3(RDF_BLOCK), 0, st, dk, Jr, C,
                               c->offp.as<u64>());
            hipLaunchKernelGGL(k_dgrp_range, dim3(grid_for(Jr, RDF_BLOCK, kGrid)), dim3(RDF_BLOCK), 0, st, dk, Jr,
                               c->offp.as<u64>(), c->doff.as<u64>(), c->dcur.as<u32>(), c->gmap.as<u32>(), c->dgrp.as<u32>());
            if (C)
                hipLaunchKernelGGL(k_dcur_add, dim3(grid_for(C, RDF_BLOCK, kGrid)), dim3(RDF_BLOCK), 0, st, c->offp.as<u64>(), C,
                                   c->dcur.as<u32>());
        }
        tend(c, RDF_T_GROUPS);
        Jf0 += Jr;
        G0 += Gr;
    }
    if (Jf0 != Jf) return fail(c, RDF_ERR_LIMIT, "join ranges disagree on the kept records");
    c->G = G0;
    c->J = Jtot;
    c->J_emit = J_emit;  // every range was emitted twice: the first pass's count
    c->hscal[14] = Jf;
    HIP_TRY(c, hipMemcpyAsync(c->goff.as<u64>() + G0, c->hscal + 14, 8, hipMemcpyHostToDevice, st));
    HIP_TRY(c, hipStreamSynchronize(st));
    // the range scratch is sized by the largest range: spare for the discovery stage (g_finish marks it)
    c->rec_sorted = nullptr;
    return RDF_OK;
}

static rdf_status g_build_ranges(rdf_ctx* c, int proj, u64 max_range) {
    const JoinSel all = {0u, 1u, 0u, JOIN_ALL_HI};
    TRY(g_ranges_supports(c, proj, max_range, all));
    return g_ranges_groups(c, proj, all, nullptr);
}

// records per join range of the automatic g_build_ranges: the range scratch (two record buffers, fresh flags + scan,
// kept keys and their sort buffer, group flags + scan: <= 48 B per record) in the free HBM left after the stage's
// global arrays (gcap + dgrp, <= 8 B per record overall), at most 2^31.  This sizes the ranges only: a range is
// consecutive 2^(joinbits-14)-value join buckets, so one bucket larger than this (hot join values) makes a larger
// range; the hard bound is the u32 record offsets inside a range (cstart, fpos: < 2^32 - 1 records, checked with
// RDF_ERR_LIMIT), and a range's buffers are sized by the largest range (an allocation failure is RDF_ERR_OOM)
static u64 auto_range_records(rdf_ctx* c) {
    size_t free_b = 0, total_b = 0;
    if (hipMemGetInfo(&free_b, &total_b) != hipSuccess) return 1ull << 30;
    // spare buffers an allocation of the build may release (reclaim_spare)
    const u64 held = (u64)c->brkeys.cap + c->brkeys2.cap + c->tkeys.cap + c->urecs.cap +
                     (c->spare_x ? (u64)c->xsend.cap + c->xrecv.cap : 0ull) + c->rstore.cap;
    const u64 avail = (u64)free_b + held;
    // ~4.5 records per triple kept
    const u64 global = 8 * 9 * c->n / 2 + 16ull * (c->V ? c->V : 1) + (4ull << 30);
    const u64 r = avail > global ? (avail - global) / 48 : 0;
    return std::max<u64>(std::min<u64>(r, 1ull << 31), 1ull << 24);
}

// local group-size histogram (quarter-octave buckets) -> h_hist (host; nullptr: left on the device for
// k_heavy_threshold)
static rdf_status g_size_hist(rdf_ctx* c, u32* h_hist) {
    hipStream_t st = c->stream;
    tbegin(c, RDF_T_HEAVYMASK);
    ENSURE(c, hist, 256 * 4 + 64);
    HIP_TRY(c, hipMemsetAsync(c->hist.p, 0, 256 * 4 + 64, st));
    if (c->G)
        hipLaunchKernelGGL(k_group_size_hist, dim3(grid_for(c->G, RDF_BLOCK, kGrid)), dim3(RDF_BLOCK), 0, st,
                           c->goff.as<u64>(), c->G, c->hist.as<u32>());
    tend(c, RDF_T_HEAVYMASK);
    if (!h_hist) return RDF_OK;
    HIP_TRY(c, hipMemcpyAsync(h_hist, c->hist.p, 256 * 4, hipMemcpyDeviceToHost, st));
    HIP_TRY(c, hipStreamSynchronize(st));
    return RDF_OK;
}

// heavy threshold from the (global) histogram; 0 = no heavy groups
static u64 heavy_threshold(const rdf_ctx* c, const u32* hist) {
    int tb = heavy_threshold_from_hist(hist, c->heavy_min);
    return tb >= 0 ? std::max<u64>(bucket_min_size(tb), c->heavy_min) : 0;
}

// groups of a histogram at or above the threshold (exact: a power-of-two heavy_min starts a bucket)
static u64 heavy_count(const u32* hist, u64 thr) {
    if (!thr) return 0;
    u64 n = 0;
    for (int b = size_bucket(thr); b < 256; ++b) n += hist[b];
    return n;
}

// heavy groups -> bitmask columns base.. (this rank's), binary components and parents CSR.  dev_thr: the threshold
// comes from the device histogram (k_heavy_threshold) and the heavy count stays on the device until the run's stats
// are read (settle_group_stats); otherwise thr is the host's (sharded: from the all-gathered histogram).
static rdf_status g_heavy_binary(rdf_ctx* c, u64 thr, u32 base, bool dev_thr = false) {
    hipStream_t st = c->stream;
    const u64 G = c->G;
    const u32 C = c->C, Cu = c->Cu;
    const u32 V = c->V ? c->V : 1;
    tbegin(c, RDF_T_HEAVYMASK);
    c->heavy_threshold = thr;
    ENSURE(c, heavy_list, HMAX * 4);
    ENSURE(c, hbit, std::max<u64>(G, 1));
    u32* d_nheavy = c->hist.as<u32>() + 256;
    u64* d_thr = reinterpret_cast<u64*>(c->hist.as<u32>() + 258);
    HIP_TRY(c, hipMemsetAsync(d_nheavy, 0, 4, st));
    if (dev_thr) hipLaunchKernelGGL(k_heavy_threshold, dim3(1), dim3(1), 0, st, c->hist.as<u32>(), c->heavy_min, d_thr);
    if (G)
        hipLaunchKernelGGL(k_heavy_select, dim3(grid_for(G, RDF_BLOCK, kGrid)), dim3(RDF_BLOCK), 0, st, c->goff.as<u64>(), G,
                           thr, dev_thr ? d_thr : nullptr, base, d_nheavy, c->heavy_list.as<u32>(), c->hbit.as<uint8_t>());
    if (dev_thr) {
        // k_heavy_select numbers at most HMAX - base columns (base = 0 here)
        c->pend_heavy = true;
        if (G)
            hipLaunchKernelGGL(k_heavy_mask, dim3(64, HMAX), dim3(RDF_BLOCK), 0, st, c->goff.as<u64>(), c->gcap.as<u32>(),
                               c->heavy_list.as<u32>(), 0u, c->info.as<CapInfo>(), (const u32*)d_nheavy);
    } else {
        u32 nh = 0;
        TRY(read_u32(c, d_nheavy, &nh));
        nh = base >= (u32)HMAX ? 0 : std::min<u32>(nh, HMAX - base);
        c->nheavy = nh;
        if (nh)
            hipLaunchKernelGGL(k_heavy_mask, dim3(64, nh), dim3(RDF_BLOCK), 0, st, c->goff.as<u64>(), c->gcap.as<u32>(),
                               c->heavy_list.as<u32>(), base, c->info.as<CapInfo>(), (const u32*)nullptr);
    }
    const u32 Cb = C - Cu;
    ENSURE(c, bcomp, std::max<u64>(2ull * Cb, 1) * 4);
    ENSURE(c, bkeyc, std::max<u64>(Cb, 1) * 8);
    ENSURE(c, poff, (Cu + 1ull) * 8);
    ENSURE(c, plist, std::max<u64>(2ull * Cb, 1) * 4);
    ENSURE(c, pedges, std::max<u64>(2ull * Cb, 1) * 8);
    ENSURE(c, pedges_tmp, std::max<u64>(2ull * Cb, 1) * 8);
    if (Cb) {
        hipLaunchKernelGGL(k_binary_info, dim3(grid_for(Cb, RDF_BLOCK, kGrid)), dim3(RDF_BLOCK), 0, st, c->fcap.as<u32>(),
                           c->fidx.as<u32>(), c->bkeys.as<u64>(), c->frank.as<u32>(), C, Cu, V, 2u * c->U,
                           c->bcomp.as<u32>(), c->bkeyc.as<u64>(), c->pedges.as<u64>(), c->info.as<CapInfo>());
        u64* k = c->pedges.as<u64>();
        u64* t = c->pedges_tmp.as<u64>();
        HIP_TRY(c, radix_sort_u64_bits(c->ws, k, t, 2ull * Cb, 32, 32 + bits_for(Cu ? Cu - 1 : 0), st));  // edges in binary order
        if (k != c->pedges.as<u64>()) std::swap(c->pedges, c->pedges_tmp);
    }
    hipLaunchKernelGGL(k_parents_csr, dim3(grid_for(std::max<u64>(2ull * Cb, Cu + 1ull), RDF_BLOCK, kGrid)), dim3(RDF_BLOCK), 0,
                       st, c->pedges.as<u64>(), 2ull * Cb, Cu, c->poff.as<u64>(), c->plist.as<u32>(), c->info.as<CapInfo>());
    HIP_TRY(c, hipGetLastError());
    tend(c, RDF_T_HEAVYMASK);
    return RDF_OK;
}

static void fill_group_stats(rdf_ctx* c) {
    rdf_group_stats& s = c->gstats;
    memset(&s, 0, sizeof(s));
    s.n_records = c->J_emit;
    s.n_sorted_records = c->J;
    s.n_frequent_records = c->Jf;
    s.n_groups = c->G;
    s.n_captures = c->C;
    s.n_unary_captures = c->Cu;
    s.n_heavy_groups = c->nheavy;
    s.heavy_threshold = c->heavy_threshold;
    s.n_join_ranges = c->n_group_ranges;
    s.n_ranges_kept = c->jr_keep ? c->n_group_ranges : 0;
}

// the heavy threshold and count of a device-threshold build -> gstats (one host read; at the run's end for rdf_run)
static rdf_status settle_group_stats(rdf_ctx* c) {
    if (c->pend_heavy) {
        u64 v[2];
        TRY(read_multi(c, {{c->hist.as<u32>() + 258, 8}, {c->hist.as<u32>() + 256, 4}}, v));
        c->heavy_threshold = v[0];
        c->nheavy = (u32)std::min<u64>(v[1], HMAX);
        c->pend_heavy = false;
        fill_group_stats(c);
    }
    return RDF_OK;
}

static rdf_status g_finish(rdf_ctx* c, rdf_group_stats* stats) {
    HIP_TRY(c, hipEventRecord(c->ev[3], c->stream));
    c->spare_groups = true;  // the records and their sort buffers are not read after the group build
    c->rec_sorted = nullptr;
    c->pend_groups = true;
    fill_group_stats(c);
    if (stats) {
        TRY(settle_group_stats(c));
        *stats = c->gstats;
    }
    c->stage = 3;
    return RDF_OK;
}

rdf_status rdf_build_capture_groups(rdf_ctx* c, const char* projection, rdf_group_stats* stats) {
    if (!c) return RDF_ERR_ARG;
    if (c->stage < 2) return fail(c, RDF_ERR_STATE, "rdf_frequent_conditions must be called first");
    HIP_TRY(c, hipSetDevice(c->device));
    TRY(hv_wait(c, true));
    int proj = 0;
    TRY(parse_projection(c, projection, &proj));
    c->rank = 0;
    c->nranks = 1;
    c->paged = false;
    c->n_group_ranges = 1;
    if (c->group_range_records || 9 * c->n >= (1ull << 32)) {
        TRY(g_build_ranges(c, proj, c->group_range_records ? c->group_range_records : auto_range_records(c)));
    } else {
        TRY(g_emit_sort_support(c, proj));
        TRY(g_compact_groups(c));
    }
    if (c->ar_on) TRY(g_ar_refs(c));
    TRY(g_size_hist(c, nullptr));
    TRY(g_heavy_binary(c, 0, 0, true));
    return g_finish(c, stats);
}

// ------------------------------------------------------------------------------------------------
// Stage 3: CIND extraction + minimality (TraversalStrategy.enhanceFlinkPlan)

static CindView make_view(rdf_ctx* c, uint32_t flags) {
    CindView v;
    v.C = c->C;
    v.Cu = c->Cu;
    v.info = c->info.as<CapInfo>();
    v.gcap = c->gcap.as<u32>();
    v.goff = c->goff.as<u64>();
    v.hbit = c->hbit.as<uint8_t>();
    v.doff = c->doff.as<u64>();
    v.dgrp = c->dgrp.as<u32>();
    v.bcomp = c->bcomp.as<u32>();
    v.bkeyc = c->bkeyc.as<u64>();
    v.poff = c->poff.as<u64>();
    v.plist = c->plist.as<u32>();
    v.eoff = nullptr;
    v.epairs = nullptr;
    v.ebin = nullptr;
    v.literal = (flags & RDF_STRATEGY_ALL_AT_ONCE) ? 1 : 0;
    v.mode = (flags & RDF_CLEAN_IMPLIED) ? RULES_CLEAN : (v.literal ? RULES_NONE : RULES_S2L_RAW);
    v.vcoff = nullptr;
    v.vpairs = nullptr;
    v.ar = c->ar_on ? (v.literal ? AR_S0 : AR_S2L) : AR_NONE;
    v.arref = c->arref.as<u32>();
    v.sig = c->sig_on ? c->lsig.as<u64>() : nullptr;
    v.ginfo = c->ginfo.as<u32>();
    v.piv2 = c->piv2_on ? c->piv2.as<u32>() : nullptr;
    v.pivx = c->pivx_on ? c->pivx.as<u32>() : nullptr;
    v.npx = 0;  // set per k_light launch (d_light_kernels)
    v.gdrow = c->dense_on ? c->gdrow.as<u32>() : nullptr;
    v.dbits = c->dense_on ? c->dbits_p : nullptr;
    v.dwords = c->dwords;
    v.prefilter = 0;
    v.p2done = 0;
    static const int sweep_f = getenv("RDFIND_SWEEP_F") ? atoi(getenv("RDFIND_SWEEP_F")) : LIGHT_SWEEP_F;
    v.sweep_f = sweep_f;
    return v;
}

// exact member bitmaps of the dense light groups (a row of C bits each; thresholds in kernels.hpp, DENSE_MIN_ABS;
// RDFIND_DENSE=<div> sets C / div for every input, 0 turns them off).  Two steps around the pivot pass's one
// read-back: d_dense_flags numbers the rows on the device, d_dense_build (after the read, which carries the row count)
// sizes the bitmap for the rows that exist, capped at DENSE_BYTES and half the free HBM (rows past the cap stay member
// lists), and fills it.
static rdf_status d_dense_flags(rdf_ctx* c) {
    hipStream_t st = c->stream;
    const u64 G = c->G, C = c->C;
    c->dense_on = false;
    c->dense_flagged = false;
    const int div = c->dense_div >= 0 ? c->dense_div : DENSE_DIV_STAGE;  // RDFIND_DENSE: one divisor for every input
    if (div <= 0 || !G || !C) return RDF_OK;
    auto clampd = [&](u64 m) { return (u32)std::min<u64>(std::max<u64>(m, c->dense_min), 0x7fffffffu); };
    const u32 dmin_stage = clampd((C + div - 1) / div);
    const u32 dmin_other = c->dense_div >= 0 ? dmin_stage : clampd(std::min<u64>((C + 31) / 32, DENSE_MIN_ABS));
    tbegin(c, RDF_T_LIGHT);
    ENSURE(c, gflag, G * 4);
    ENSURE(c, gexcl, (G + 1) * 4);
    ENSURE(c, gdrow, G * 4);
    hipLaunchKernelGGL(k_dense_flags, dim3(grid_for(G, RDF_BLOCK, kGrid)), dim3(RDF_BLOCK), 0, st, c->ginfo.as<u32>(), G,
                       c->gsums.as<u64>(), dmin_stage, dmin_other, c->gflag.as<u32>());
    HIP_TRY(c, exclusive_scan_u32(c->ws, c->gflag.as<u32>(), c->gexcl.as<u32>(), G, c->gexcl.as<u32>() + G, st));
    tend(c, RDF_T_LIGHT);
    c->dense_flagged = true;
    return RDF_OK;
}

static rdf_status d_dense_build(rdf_ctx* c, CindView& v, u64 nrows) {
    hipStream_t st = c->stream;
    v.gdrow = nullptr;
    v.dbits = nullptr;
    if (!c->dense_flagged || !nrows) return RDF_OK;
    const u64 G = c->G, C = c->C;
    const u64 dwords = ((C + 31) / 32 + 31) & ~31ull;  // rows start on 128-B lines
    u64 budget = getenv("RDFIND_DENSE_BYTES") ? (u64)atoll(getenv("RDFIND_DENSE_BYTES")) : DENSE_BYTES;
    size_t hfree = 0, htotal = 0;
    if (hipMemGetInfo(&hfree, &htotal) == hipSuccess) budget = std::min<u64>(budget, std::max<u64>(c->dbits.cap, hfree / 2));
    (void)hipGetLastError();
    const u64 rows = std::min<u64>(nrows, budget / (dwords * 4));
    if (getenv("RDFIND_DEBUG_LIGHT"))
        fprintf(stderr, "dense: C %llu G %llu rows %llu of %llu, %.1f MB\n", (unsigned long long)C, (unsigned long long)G,
                (unsigned long long)rows, (unsigned long long)nrows, rows * dwords * 4 / 1e6);
    if (!rows) return RDF_OK;
    ENSURE(c, dlist, rows * 4);
    // the bitmaps only speed the light pass up: without the memory for them the member lists serve (no reclaim of the
    // spare scratch for them either: the next run would allocate that again)
    if (c->dbits.ensure(rows * dwords * 4) != hipSuccess) {
        (void)hipGetLastError();
        return RDF_OK;
    }
    c->dbits_p = c->dbits.as<u32>();
    tbegin(c, RDF_T_LIGHT);
    hipLaunchKernelGGL(k_dense_rows, dim3(grid_for(G, RDF_BLOCK, kGrid)), dim3(RDF_BLOCK), 0, st, c->gflag.as<u32>(),
                       c->gexcl.as<u32>(), G, (u32)rows, c->gdrow.as<u32>(), c->dlist.as<u32>());
    hipLaunchKernelGGL(k_dense_build, dim3((unsigned)std::min<u64>(rows, 4096)), dim3(RDF_BLOCK), 0, st,
                       c->dlist.as<u32>(), c->gexcl.as<u32>() + G, rows, c->goff.as<u64>(), c->gcap.as<u32>(),
                       dwords, c->dbits_p);
    tend(c, RDF_T_LIGHT);
    c->dense_on = true;
    c->dwords = dwords;
    v.gdrow = c->gdrow.as<u32>();
    v.dbits = c->dbits_p;
    v.dwords = dwords;
    return RDF_OK;
}

// local pivot statistics: pbest[d] = (size << 32 | group) of d's smallest local group, pnl[d] = local light groups
static rdf_status d_pivot_local(rdf_ctx* c, CindView& v) {
    hipStream_t st = c->stream;
    const u32 C = c->C;
    HIP_TRY(c, hipEventRecord(c->ev[4], st));
    HIP_TRY(c, hipMemsetAsync(c->scal.p, 0, 16 * sizeof(u64), st));
    ENSURE(c, pivot, std::max<u64>(C, 1) * 4);
    ENSURE(c, nchl, std::max<u64>(C, 1) * 4);
    ENSURE(c, nchh, std::max<u64>(C, 1) * 4);
    ENSURE(c, choffl, (C + 1ull) * 8);
    ENSURE(c, choffh, (C + 1ull) * 8);
    ENSURE(c, nitl, std::max<u64>(C, 1) * 4);
    ENSURE(c, itoffl, (C + 1ull) * 8);
    ENSURE(c, npk, std::max<u64>(C, 1) * 4);
    ENSURE(c, pkoff, (C + 1ull) * 8);
    ENSURE(c, pseg, std::max<u64>(C, 1) * 4);
    ENSURE(c, psegoff, (C + 1ull) * 8);
    ENSURE(c, pbest, std::max<u64>(C, 1) * 8);
    ENSURE(c, pnl, std::max<u64>(C, 1) * 4);
    // signature test in k_light only by default (mode 2): on the packed path (few groups per dependent) the extra
    // line per candidate cost more than it saved (c5 at 0.1: 20.8 vs 17.6 ms light); mode 1 tests it in both
    static const int sig_mode = getenv("RDFIND_SIG") ? atoi(getenv("RDFIND_SIG")) : 2;
    const bool sig_enabled = sig_mode != 0;
    c->sig_on = sig_enabled;
    c->sig_packed = sig_mode != 2;
    u64* sig = nullptr;
    if (sig_enabled) {
        ENSURE(c, lsig, std::max<u64>(C, 1) * 8 * SIG_W);
        sig = c->lsig.as<u64>();
    }
    const u64 G = c->G;
    ENSURE(c, ginfo, std::max<u64>(G, 1) * 4);
    v.ginfo = c->ginfo.as<u32>();
    const unsigned gi_grid = grid_for(std::max<u64>(G, 1), RDF_BLOCK, kGrid);
    ENSURE(c, ppart, 3ull * gi_grid * 8);
    ENSURE(c, gsums, 3 * 8);
    tbegin(c, RDF_T_PIVOT);
    HIP_TRY(c, hipMemsetAsync(c->gsums.p, 0, 3 * 8, st));
    if (G) {
        hipLaunchKernelGGL(k_group_info, dim3(gi_grid), dim3(RDF_BLOCK), 0, st, c->goff.as<u64>(), c->hbit.as<uint8_t>(), G,
                           c->ginfo.as<u32>(), c->ppart.as<u64>());
        hipLaunchKernelGGL(k_sum_partials3, dim3(1), dim3(RDF_BLOCK), 0, st, c->ppart.as<u64>(), gi_grid, c->gsums.as<u64>());
    }
    tend(c, RDF_T_PIVOT);
    TRY(d_dense_flags(c));
    static const int piv2_mode = getenv("RDFIND_PIV2") ? atoi(getenv("RDFIND_PIV2")) : 1;  // 2: k_light only
    const bool piv2_enabled = piv2_mode != 0;
    c->piv2_packed = piv2_mode != 2;
    u32* piv2 = nullptr;
    if (piv2_enabled) {
        ENSURE(c, piv2, std::max<u64>(C, 1) * 4);
        piv2 = c->piv2.as<u32>();
    }
    c->piv2_on = piv2_enabled;
    static const bool pivx_enabled = piv2_enabled && (!getenv("RDFIND_PIVX") || atoi(getenv("RDFIND_PIVX")) != 0);
    u32* pivx = nullptr;
    if (pivx_enabled) {
        ENSURE(c, pivx, std::max<u64>(C, 1) * 4 * PIV_EXTRA);
        pivx = c->pivx.as<u32>();
    }
    c->pivx_on = pivx_enabled;
    tbegin(c, RDF_T_PIVOT);
    if (piv2 && C) HIP_TRY(c, hipMemsetAsync(piv2, 0xff, (u64)C * 4, st));  // multi-segment dependents: none
    if (pivx && C) HIP_TRY(c, hipMemsetAsync(pivx, 0xff, (u64)C * 4 * PIV_EXTRA, st));
    if (sig && C) HIP_TRY(c, hipMemsetAsync(sig, 0, (u64)C * 8 * SIG_W, st));
    if (C) {
        hipLaunchKernelGGL(k_pivot_nseg, dim3(grid_for(C, RDF_BLOCK, kGrid)), dim3(RDF_BLOCK), 0, st, c->doff.as<u64>(), C,
                           c->pseg.as<u32>());
        HIP_TRY(c, exclusive_scan_u32_u64(c->ws, c->pseg.as<u32>(), c->psegoff.as<u64>(), C, c->psegoff.as<u64>() + C, st));
        HIP_TRY(c, hipMemsetAsync(c->pbest.p, 0xff, (u64)C * 8, st));
        HIP_TRY(c, hipMemsetAsync(c->pnl.p, 0, (u64)C * 4, st));
    }
    tend(c, RDF_T_PIVOT);
    u64 WS = 0;
    c->light_stage = false;
    c->light_wmean = 0;
    if (C) {
        u64 r[4] = {0, 0, 0, 0};
        if (c->dense_flagged)
            TRY(read_multi(c, {{c->psegoff.as<u64>() + C, 8}, {c->gsums.as<u64>(), 8}, {c->gsums.as<u64>() + 1, 8},
                               {c->gexcl.as<u32>() + c->G, 4}}, r));
        else
            TRY(read_multi(c, {{c->psegoff.as<u64>() + C, 8}, {c->gsums.as<u64>(), 8}, {c->gsums.as<u64>() + 1, 8}}, r));
        TRY(d_dense_build(c, v, r[3]));
        WS = r[0];
        // member-weighted mean light group size sum(n^2) / sum(n): small groups -> the LDS-staging light variant
        c->light_stage = r[2] <= (u64)LIGHT_STAGE_AVG * r[1];
        c->light_wmean = r[1] ? r[2] / r[1] : 0;
        static const char* force = getenv("RDFIND_STAGE");  // A/B and test hook: 0 / 1 forces the variant
        if (force) c->light_stage = atoi(force) != 0;
    }
    // extra pivots: all PIV_EXTRA where the high-occupancy light variant may run (large groups), one elsewhere
    c->pivx_kept = !pivx ? 0
                   : (!c->light_stage && c->light_wmean >= PIVX_WMEAN && G >= PIVX_GPC * (u64)C) ? PIV_EXTRA
                                                                                                 : PIV_EXTRA_PLAIN;
    tbegin(c, RDF_T_PIVOT);
    if (C) {
        if (c->pivx_kept == PIV_EXTRA)
            hipLaunchKernelGGL(k_pivot_short<PIV_EXTRA>, dim3(grid_for(C, RDF_BLOCK, kGrid)), dim3(RDF_BLOCK), 0, st, v,
                               c->dgrp.as<u32>(), c->pbest.as<u64>(), c->pnl.as<u32>(), sig, piv2, pivx);
        else
            hipLaunchKernelGGL(k_pivot_short<PIV_EXTRA_PLAIN>, dim3(grid_for(C, RDF_BLOCK, kGrid)), dim3(RDF_BLOCK), 0, st, v,
                               c->dgrp.as<u32>(), c->pbest.as<u64>(), c->pnl.as<u32>(), sig, piv2, pivx);
    }
    if (WS) {
        const dim3 g(vgrid(wave_blocks(WS)));
        if (c->pivx_kept == PIV_EXTRA)
            hipLaunchKernelGGL(k_pivot_seg<PIV_EXTRA>, g, dim3(RDF_BLOCK), 0, st, (u64)wave_blocks(WS), v, c->dgrp.as<u32>(),
                               c->psegoff.as<u64>(), WS, c->pbest.as<u64>(), c->pnl.as<u32>(), sig, piv2, pivx);
        else
            hipLaunchKernelGGL(k_pivot_seg<PIV_EXTRA_PLAIN>, g, dim3(RDF_BLOCK), 0, st, (u64)wave_blocks(WS), v,
                               c->dgrp.as<u32>(), c->psegoff.as<u64>(), WS, c->pbest.as<u64>(), c->pnl.as<u32>(), sig, piv2,
                               pivx);
    }
    tend(c, RDF_T_PIVOT);
    v.sig = sig;  // the candidate passes of this run test the signatures
    v.piv2 = piv2;
    v.pivx = pivx;
    return RDF_OK;
}

// work-chunk offsets after the pivot final pass
static rdf_status d_chunks(rdf_ctx* c, u64* WL, u64* WH, u64* WI, u64* WP) {
    hipStream_t st = c->stream;
    const u32 C = c->C;
    {
        const u32* in[4] = {c->nchl.as<u32>(), c->nitl.as<u32>(), c->nchh.as<u32>(), c->npk.as<u32>()};
        u64* out[4] = {c->choffl.as<u64>(), c->itoffl.as<u64>(), c->choffh.as<u64>(), c->pkoff.as<u64>()};
        HIP_TRY(c, exclusive_scan_u32_u64_batch(c->ws, in, out, 4, C, st));
    }
    u64 v[8];  // [7]: k_multi_items' sum when rdf_discover_cinds launched it (else stale, unused)
    TRY(read_multi(c, {{c->choffl.as<u64>() + C, 8}, {c->pkoff.as<u64>() + C, 8}, {c->choffh.as<u64>() + C, 8},
                       {dscal(c, 2), 8}, {c->itoffl.as<u64>() + C, 8}, {dscal(c, 3), 8}, {dscal(c, 4), 8},
                       {dscal(c, 5), 8}}, v));
    c->n_multi_items = v[7];
    *WL = v[0];
    c->light_hiocc = !c->light_stage && c->light_wmean >= LIGHT_HIOCC_AVG && v[0] >= LIGHT_HIOCC_OCT * (u64)C;
    static const char* hi = getenv("RDFIND_LIGHT_HIOCC");  // A/B and test hook: 0 / 1 forces the occupancy
    if (hi) c->light_hiocc = !c->light_stage && atoi(hi) != 0;
    c->light_npx = std::min(c->pivx_kept, c->light_hiocc ? PIV_EXTRA : PIV_EXTRA_PLAIN);
    static const char* npx = getenv("RDFIND_PIVX_N");  // A/B and test hook: how many extra pivots k_light checks
    if (npx) c->light_npx = std::min(c->pivx_kept, atoi(npx));
    if (getenv("RDFIND_DEBUG_LIGHT"))
        fprintf(stderr, "LIGHT weighted mean light group %llu, octets per capture %.1f (stage %d, hiocc %d, extra pivots %d of %d)\n",
                (unsigned long long)c->light_wmean, C ? (double)v[0] / C : 0.0, (int)c->light_stage, (int)c->light_hiocc,
                c->light_npx, c->pivx_kept);
    *WP = v[1];
    *WH = v[2];
    c->heavy_candidates = v[3];
    *WI = v[4];
    c->light_candidates = v[5];
    c->light_entries = v[6];
    return RDF_OK;
}

// owner tables of the light work (all dependents): item_dep over the k_light items, pk_dep over the packed octets,
// the multi-segment chunks (mchoff, mch_dep); *WM = their number
static rdf_status d_light_owners(rdf_ctx* c, u64 WI, u64 WP, u64* WM) {
    hipStream_t st = c->stream;
    ENSURE(c, item_dep, std::max<u64>(WI, 1) * 4);
    ENSURE(c, pk_dep, std::max<u64>(WP, 1) * 4);
    *WM = 0;
    tbegin(c, RDF_T_LIGHT);
    if (WI)
        hipLaunchKernelGGL(k_expand_owner, dim3(grid_for(c->C, RDF_BLOCK, kGrid)), dim3(RDF_BLOCK), 0, st, c->itoffl.as<u64>(),
                           c->C, c->item_dep.as<u32>());
    if (WP)
        hipLaunchKernelGGL(k_expand_owner, dim3(grid_for(c->C, RDF_BLOCK, kGrid)), dim3(RDF_BLOCK), 0, st, c->pkoff.as<u64>(),
                           c->C, c->pk_dep.as<u32>());
    // chunks of dependents whose groups span several segments: emitted once all their segments are done
    if (WI) {
        ENSURE(c, nmch, std::max<u64>(c->C, 1) * 4);
        ENSURE(c, mchoff, (c->C + 1ull) * 8);
        hipLaunchKernelGGL(k_mseg_chunks, dim3(grid_for(c->C, RDF_BLOCK, kGrid)), dim3(RDF_BLOCK), 0, st, c->doff.as<u64>(),
                           c->nitl.as<u32>(), c->C, c->nmch.as<u32>());
        HIP_TRY(c, exclusive_scan_u32_u64(c->ws, c->nmch.as<u32>(), c->mchoff.as<u64>(), c->C, c->mchoff.as<u64>() + c->C, st));
        TRY(read_u64(c, c->mchoff.as<u64>() + c->C, WM));
    }
    if (*WM) {
        ENSURE(c, mch_dep, *WM * 4);
        hipLaunchKernelGGL(k_expand_owner, dim3(grid_for(c->C, RDF_BLOCK, kGrid)), dim3(RDF_BLOCK), 0, st, c->mchoff.as<u64>(),
                           c->C, c->mch_dep.as<u32>());
    }
    tend(c, RDF_T_LIGHT);
    return RDF_OK;
}

// Work of the light dependents [d0, d1): k_light items [i0, i1), packed octets [q0, q1), multi-segment chunks [m0, m1)
// and output octets [o0, o1) (the scans itoffl, pkoff, mchoff, choffl at d0 and d1).
struct LightRange {
    u64 i0, i1, q0, q1, m0, m1, o0, o1;
};

static rdf_status light_range(rdf_ctx* c, u32 d0, u32 d1, bool mseg, LightRange* r) {
    u64 v[8];
    const u64* mo = mseg ? c->mchoff.as<u64>() : c->itoffl.as<u64>();  // no multi-segment items: any zero-width pair
    TRY(read_multi(c, {{c->itoffl.as<u64>() + d0, 8}, {c->itoffl.as<u64>() + d1, 8}, {c->pkoff.as<u64>() + d0, 8},
                       {c->pkoff.as<u64>() + d1, 8}, {mo + d0, 8}, {mo + d1, 8}, {c->choffl.as<u64>() + d0, 8},
                       {c->choffl.as<u64>() + d1, 8}}, v));
    *r = {v[0], v[1], v[2], v[3], mseg ? v[4] : 0, mseg ? v[5] : 0, v[6], v[7]};
    return RDF_OK;
}

// light kernels of dependent range r: survivor slots (8 per output octet, relative to r.o0) and per-octet counts
static rdf_status d_light_kernels(rdf_ctx* c, const CindView& v, const u32* pivot, const LightRange& r, DevBuf& slots,
                                  DevBuf& counts) {
    hipStream_t st = c->stream;
    const u64 WL = r.o1 - r.o0, WI = r.i1 - r.i0, WP = r.q1 - r.q0, WM = r.m1 - r.m0, ob = r.o0;
    const u64 nslot = std::max<u64>(WL, 1);
    HIP_TRY(c, slots.ensure(nslot * 8 * 8));
    ENSURE(c, dead, nslot * 8);  // kill masks of multi-segment chunks, keyed by the chunk's first octet
    HIP_TRY(c, hipMemsetAsync(c->dead.p, 0, nslot * 8, st));
    HIP_TRY(c, counts.ensure(nslot * 4));
    HIP_TRY(c, hipMemsetAsync(counts.p, 0, nslot * 4, st));
#ifdef RDF_LIGHT_STATS
    u32* lrec = nullptr;
    if (WI && getenv("RDFIND_LIGHT_DUMP")) {
        HIP_TRY(c, hipMalloc(&lrec, r.i1 * 96));
        HIP_TRY(c, hipMemset(lrec, 0, r.i1 * 96));
        HIP_TRY(c, hipMemcpyToSymbol(HIP_SYMBOL(g_item_rec), &lrec, sizeof(lrec)));
    }
#endif
    tbegin(c, RDF_T_LIGHT);
    CindView vp = v;
    if (!c->sig_packed) vp.sig = nullptr;
    if (!c->piv2_packed) vp.piv2 = nullptr;
    // the packed path checks the first extra pivot after the second one on large-group inputs (c3 full: packed + plain
    // light 27.5 -> 26.8 ms; c2, c5 lose 1-2 %: profiles/r04_light_ab_pivx_packed.log).  RDFIND_PIVX_PACKED=0/1 forces
    static const char* pxp = getenv("RDFIND_PIVX_PACKED");
    const bool pivx_packed = pxp ? atoi(pxp) != 0 : !c->light_stage && c->light_wmean >= PIVX_WMEAN;
    vp.npx = pivx_packed && c->pivx_kept ? 1 : 0;
    if (!vp.npx) vp.pivx = nullptr;
    // the packed dependents on the side stream, beside k_light (disjoint output octets): their blocks fill the SIMDs
    // k_light's long items leave idle (RDFIND_LIGHT_SIDE=0: one stream)
    static const bool side_ok = !(getenv("RDFIND_LIGHT_SIDE") && atoi(getenv("RDFIND_LIGHT_SIDE")) == 0);
    const bool side = side_ok && WP && WI;
    if (side) {
        HIP_TRY(c, hipEventRecord(c->ev_fork, st));
        HIP_TRY(c, hipStreamWaitEvent(c->side, c->ev_fork, 0));
    }
    if (WP)
        hipLaunchKernelGGL(k_light_packed, dim3(vgrid(thread_blocks(WP * 8))), dim3(RDF_BLOCK), 0, side ? c->side : st,
                           (u64)thread_blocks(WP * 8), vp, pivot, c->pkoff.as<u64>(), c->pk_dep.as<u32>(), r.q0, WP,
                           c->choffl.as<u64>(), ob, slots.as<u64>(), counts.as<u32>());
    if (side) HIP_TRY(c, hipEventRecord(c->ev_join, c->side));
    if (WI) {
        auto kl = c->light_stage ? k_light_stage : c->light_hiocc ? k_light_plain_hi : k_light_plain;
        CindView vl = v;
        vl.npx = c->light_npx;
        // issue order: the items of dependents with many light-group entries first (RDFIND_LIGHT_ORDER=<entries>, 0: off).
        // By default for the staging variant only: c2 light 2.22 -> 2.03 ms, while the plain variant's inputs lose a
        // little (c3 17.0 -> 17.2, c4 at 0.4 60.4 -> 61.1; profiles/r05_light_order_ab.log).  The partition is stable:
        // an octave-class order whose slots came from atomics measured 2.23 ms on c2 (consecutive items of one
        // dependent share its groups in L2; profiles/r05_light_order_classes_ab.log)
        static const char* oenv = getenv("RDFIND_LIGHT_ORDER");
        const u64 order_thr = oenv ? strtoull(oenv, nullptr, 10) : c->light_stage ? LIGHT_ORDER_MIN : 0;
        const u32* order = nullptr;
        if (order_thr && WI < (1ull << 32)) {
            ENSURE(c, iflag, WI * 4);
            ENSURE(c, iexcl, (WI + 1) * 4);
            ENSURE(c, iorder, WI * 4);
            hipLaunchKernelGGL(k_light_long_flags, dim3(grid_for(WI, RDF_BLOCK, kGrid)), dim3(RDF_BLOCK), 0, st,
                               c->item_dep.as<u32>(), v.doff, r.i0, WI, order_thr, c->iflag.as<u32>());
            HIP_TRY(c, exclusive_scan_u32(c->ws, c->iflag.as<u32>(), c->iexcl.as<u32>(), WI, c->iexcl.as<u32>() + WI, st));
            hipLaunchKernelGGL(k_light_order, dim3(grid_for(WI, RDF_BLOCK, kGrid)), dim3(RDF_BLOCK), 0, st, c->iflag.as<u32>(),
                               c->iexcl.as<u32>(), WI, c->iorder.as<u32>());
            order = c->iorder.as<u32>();
        }
        hipLaunchKernelGGL(kl, dim3(vgrid(wave_blocks(WI))), dim3(RDF_BLOCK),
                           0, st, (u64)wave_blocks(WI), vl, pivot, c->itoffl.as<u64>(), c->item_dep.as<u32>(), c->choffl.as<u64>(),
                           r.i0, WI, ob, c->dead.as<u64>(), slots.as<u64>(), counts.as<u32>(), order);
    }
    if (side) HIP_TRY(c, hipStreamWaitEvent(st, c->ev_join, 0));
    if (WM)
        hipLaunchKernelGGL(k_light_mseg_emit, dim3(vgrid(wave_blocks(WM))),
                           dim3(RDF_BLOCK), 0, st, (u64)wave_blocks(WM), v, pivot, c->mchoff.as<u64>(), c->mch_dep.as<u32>(), r.m0,
                           WM, c->choffl.as<u64>(), ob, c->dead.as<u64>(), slots.as<u64>(), counts.as<u32>());
    tend(c, RDF_T_LIGHT);
#ifdef RDF_LIGHT_STATS
    if (lrec) {  // per-item records -> $RDFIND_LIGHT_DUMP (raw u32 x 24 per item)
        std::vector<u32> h(r.i1 * 24);
        HIP_TRY(c, ctx_copy(c, h.data(), lrec, r.i1 * 96, hipMemcpyDeviceToHost));
        if (FILE* f = fopen(getenv("RDFIND_LIGHT_DUMP"), "wb")) {
            fwrite(h.data(), 96, r.i1, f);
            fclose(f);
        }
        u32* z = nullptr;
        HIP_TRY(c, hipMemcpyToSymbol(HIP_SYMBOL(g_item_rec), &z, sizeof(z)));
        HIP_TRY(c, hipFree(lrec));
    }
    fprintf(stderr, "LIGHT_STATS WI=%llu WL=%llu WP=%llu\n", (unsigned long long)WI, (unsigned long long)WL,
            (unsigned long long)WP);
#endif
    return RDF_OK;
}

// the WL octets' survivor slots, in octet (= (dep, ref)) order, -> out[ebase, ebase + *E)
static rdf_status d_light_compact(rdf_ctx* c, u64 WL, const DevBuf& slots, const DevBuf& counts, DevBuf& out, u64 ebase,
                                  u64* E) {
    hipStream_t st = c->stream;
    tbegin(c, RDF_T_LIGHT);
    ENSURE(c, pos, (WL + 1) * 8);
    HIP_TRY(c, exclusive_scan_u32_u64(c->ws, counts.as<u32>(), c->pos.as<u64>(), WL, c->pos.as<u64>() + WL, st));
    tend(c, RDF_T_LIGHT);
    TRY(read_u64(c, c->pos.as<u64>() + WL, E));
    size_t need = (size_t)std::max<u64>(ebase + *E, 1) * 8;
    if (ebase && need > out.cap) need = std::max<size_t>(need, out.cap + out.cap / 4);  // appends (paged): grow by >= 1/4
    HIP_TRY(c, out.grow_keep(need, st));
    tbegin(c, RDF_T_LIGHT);
    if (WL)
        hipLaunchKernelGGL(k_slot_compact, dim3(vgrid(thread_blocks(WL * 8))), dim3(RDF_BLOCK), 0, st, (u64)thread_blocks(WL * 8),
                           slots.as<u64>(), counts.as<u32>(), c->pos.as<u64>(), WL, out.as<u64>() + ebase);
    tend(c, RDF_T_LIGHT);
    return RDF_OK;
}

// light dependents of range r -> explicit raw (dep << 32 | ref) pairs at epairs + ebase, in (dep, ref) order;
// *E = their count.  Output slots are octets (8 pivot candidates each), relative to r.o0.
static rdf_status d_light_run(rdf_ctx* c, const CindView& v, const u32* pivot, const LightRange& r, u64 ebase, u64* E) {
    TRY(d_light_kernels(c, v, pivot, r, c->epairs_tmp, c->lslot));
    return d_light_compact(c, r.o1 - r.o0, c->epairs_tmp, c->lslot, c->epairs, ebase, E);
}

// every light dependent at once: explicit raw pairs in epairs[0, *E) (WI k_light items, WL octets, WP packed octets)
static rdf_status d_light(rdf_ctx* c, const CindView& v, u64 WI, u64 WL, u64 WP, u64* E, const u32* pivot) {
    u64 WM = 0;
    TRY(d_light_owners(c, WI, WP, &WM));
    const LightRange r = {0, WI, 0, WP, 0, WM, 0, WL};
    return d_light_run(c, v, pivot, r, 0, E);
}

// The two light passes pay ~5 host round trips and a dozen launches more than one pass; they are taken when the
// multi-chunk dependents hold at least LIGHT2_MIN_ITEMS k_light items, the work whose repeated group reads the second
// pass removes.  Measured by the device-resident step (profiles/r03_light_two_pass_steps.log), multi-chunk items ->
// ms one / two passes: c4 at 0.05 1.21M -> 40.4 / 39.3; c3 at 0.5 441k -> 42.7 / 42.8; c5 at 0.1 91k -> 60.2 / 62.7;
// c1 45k -> 3.37 / 3.73; c2 123 (of 256k items) -> nothing to gain.  RDFIND_LIGHT2=0 / 1 forces one / two passes.
static constexpr u64 LIGHT2_MIN_ITEMS = 1ull << 20;
// the multi-chunk dependents' k_light items -> dscal(c, 5), read back by d_chunks (c->n_multi_items)
static rdf_status d_multi_items(rdf_ctx* c) {
    hipStream_t st = c->stream;
    const unsigned gp = grid_for(std::max<u32>(c->C, 1), RDF_BLOCK, kGrid);
    ENSURE(c, ppart, 3ull * gp * 8);
    hipLaunchKernelGGL(k_multi_items, dim3(gp), dim3(RDF_BLOCK), 0, st, c->doff.as<u64>(), c->nitl.as<u32>(), c->C,
                       c->ppart.as<u64>());
    hipLaunchKernelGGL(k_sum_partials3, dim3(1), dim3(RDF_BLOCK), 0, st, c->ppart.as<u64>(), gp, dscal(c, 5));
    return RDF_OK;
}
// With the window range sweeps (light_sweep) one pass is faster on every measured shape (light ms, one / two passes:
// c4 at 0.4 181.8 / 197.9, c4 at 0.05 11.2 / 12.5, c3 at 0.5 10.6 / 10.9, c5 at 0.1 17.9 / 20.4, c2 2.60 / 2.92), so the
// two passes only run on request (RDFIND_LIGHT2=1, which the parity tests use) or with the sweeps off.
static bool use_two_pass(const rdf_ctx* c, u64 WI) {
    static const char* force = getenv("RDFIND_LIGHT2");
    if (!WI) return false;
    if (force) return atoi(force) != 0;
    return LIGHT_SWEEP_F == 0 && c->n_multi_items >= LIGHT2_MIN_ITEMS;
}

// Two light passes (single GPU).  A k_light work item verifies 64 pivot candidates of one dependent against a segment of
// its groups, so every chunk of a dependent re-reads the same groups, although the cheap filters (support, heavy mask,
// signature, second pivot) often leave few candidates per chunk.  Pass A verifies the packed dependents and those of one
// chunk as before; the chunks of the other dependents (at most LIGHT_PRE_MAX candidates left, by default all) only
// filter, and their survivors stay in their output slots tagged (PRE_TAG).  Pass B verifies the tagged survivors 64 to a
// chunk, as the sharded verify pass does (candidates given by vcoff / vpairs; the pivot group is still skipped, the
// second pivot not checked again); a fix-up drops the tagged slots pass B killed, and one compaction writes the
// (dep, ref)-ordered result, so pass A's verified pairs are never moved.  RDFIND_LIGHT2=0 keeps the single pass.
static rdf_status d_light_two_pass(rdf_ctx* c, const CindView& v, u64 WI, u64 WL, u64 WP, u64* E, const u32* pivot) {
    hipStream_t st = c->stream;
    const u32 C = c->C;
    CindView va = v;
    va.prefilter = 1;
    u64 WM = 0;
    TRY(d_light_owners(c, WI, WP, &WM));
    TRY(d_light_kernels(c, va, pivot, {0, WI, 0, WP, 0, WM, 0, WL}, c->epairs_tmp, c->lslot));
    // the tagged octets' survivors -> vpairs (octet order keeps (dep, ref) order)
    tbegin(c, RDF_T_LIGHT);
    ENSURE(c, flags, std::max<u64>(WL, 1) * 4);
    ENSURE(c, vcoff, (std::max<u64>(WL, C) + 1ull) * 8);  // tagged octet offsets first, then pass B's dependent offsets
    if (WL)
        hipLaunchKernelGGL(k_tag_octets, dim3(grid_for(WL, RDF_BLOCK, kGrid)), dim3(RDF_BLOCK), 0, st, c->epairs_tmp.as<u64>(),
                           c->lslot.as<u32>(), WL, c->flags.as<u32>());
    HIP_TRY(c, exclusive_scan_u32_u64(c->ws, c->flags.as<u32>(), c->vcoff.as<u64>(), WL, c->vcoff.as<u64>() + WL, st));
    tend(c, RDF_T_LIGHT);
    u64 T = 0;
    TRY(read_u64(c, c->vcoff.as<u64>() + WL, &T));
    c->n_light_survivors = T;
    if (T) {
        tbegin(c, RDF_T_LIGHT);
        ENSURE(c, vpairs, T * 8);
        hipLaunchKernelGGL(k_tag_gather, dim3(grid_for(WL, RDF_BLOCK, kGrid)), dim3(RDF_BLOCK), 0, st, c->epairs_tmp.as<u64>(),
                           c->flags.as<u32>(), c->vcoff.as<u64>(), WL, c->vpairs.as<u64>());
        ENSURE(c, ebin, std::max<u64>(C, 1) * 8);
        hipLaunchKernelGGL(k_pair_offsets, dim3(grid_for(C + 1ull, RDF_BLOCK, kGrid)), dim3(RDF_BLOCK), 0, st,
                           c->vpairs.as<u64>(), T, C, c->Cu, c->vcoff.as<u64>(), c->ebin.as<u64>());
        CindView vb = v;
        vb.vcoff = c->vcoff.as<u64>();
        vb.vpairs = c->vpairs.as<u64>();
        vb.p2done = 1;
        if (C)
            hipLaunchKernelGGL(k_verify_plan, dim3(grid_for(C, RDF_BLOCK, kGrid)), dim3(RDF_BLOCK), 0, st, vb, c->pnl.as<u32>(),
                               c->nchl.as<u32>(), c->nitl.as<u32>(), c->npk.as<u32>());
        tend(c, RDF_T_LIGHT);
        const u64 hc = c->heavy_candidates, lc = c->light_candidates, le = c->light_entries;
        u64 WL2 = 0, WH2 = 0, WI2 = 0, WP2 = 0, WM2 = 0, EB = 0;
        TRY(d_chunks(c, &WL2, &WH2, &WI2, &WP2));
        c->heavy_candidates = hc;
        c->light_candidates = lc;
        c->light_entries = le;
        TRY(d_light_owners(c, WI2, WP2, &WM2));
        TRY(d_light_kernels(c, vb, pivot, {0, WI2, 0, WP2, 0, WM2, 0, WL2}, c->bslots, c->bcounts));
        TRY(d_light_compact(c, WL2, c->bslots, c->bcounts, c->cpairs, 0, &EB));
        // pass B's verdicts back into pass A's tagged slots
        tbegin(c, RDF_T_LIGHT);
        hipLaunchKernelGGL(k_pair_offsets, dim3(grid_for(C + 1ull, RDF_BLOCK, kGrid)), dim3(RDF_BLOCK), 0, st,
                           c->cpairs.as<u64>(), EB, C, c->Cu, c->vcoff.as<u64>(), c->ebin.as<u64>());
        hipLaunchKernelGGL(k_tag_fix, dim3(grid_for(WL, RDF_BLOCK, kGrid)), dim3(RDF_BLOCK), 0, st, c->epairs_tmp.as<u64>(),
                               c->lslot.as<u32>(), c->flags.as<u32>(), WL, c->cpairs.as<u64>(), c->vcoff.as<u64>());
        tend(c, RDF_T_LIGHT);
    }
    return d_light_compact(c, WL, c->epairs_tmp, c->lslot, c->epairs, 0, E);
}

// sort the explicit pairs (epairs[0, E)) and index them: v.eoff / v.ebin / v.epairs
// (presorted: the single-GPU light pass already emits them in (dep, ref) order, chunk by chunk; indexed: eoff / ebin
// are already those of epairs[0, E), d_dedup_expand)
static rdf_status d_explicit_index(rdf_ctx* c, CindView& v, u64 E, bool presorted, bool indexed = false) {
    hipStream_t st = c->stream;
    const u32 C = c->C;
    if (!presorted) ENSURE(c, epairs_tmp, std::max<u64>(E, 1) * 8);
    tbegin(c, RDF_T_ESORT);
    if (!presorted) {
        u64* k = c->epairs.as<u64>();
        u64* t = c->epairs_tmp.as<u64>();
        HIP_TRY(c, radix_sort_u64(c->ws, k, t, E, 32 + bits_for(C ? C - 1 : 0), st));
        if (k != c->epairs.as<u64>()) std::swap(c->epairs, c->epairs_tmp);
    }
    ENSURE(c, eoff, (C + 1ull) * 8);
    ENSURE(c, ebin, std::max<u64>(C, 1) * 8);
    if (!indexed)
        hipLaunchKernelGGL(k_pair_offsets, dim3(grid_for(C + 1ull, RDF_BLOCK, kGrid)), dim3(RDF_BLOCK), 0, st,
                           c->epairs.as<u64>(), E, C, c->Cu, c->eoff.as<u64>(), c->ebin.as<u64>());
    tend(c, RDF_T_ESORT);
    c->sort_passes_pairs = presorted ? 0 : (u64)radix_sort_passes(32 + bits_for(C ? C - 1 : 0)) * E;
    v.eoff = c->eoff.as<u64>();
    v.epairs = c->epairs.as<u64>();
    v.ebin = c->ebin.as<u64>();
    return RDF_OK;
}

// heavy-only binary dependents: count pass -> hoff, *H
// (classed: the work items are chunks of class lists, sbase/dcls from d_class_bin; else chunks of pivot groups)
static rdf_status d_heavy_count(rdf_ctx* c, const CindView& v, u64 WH, u64* H) {
    hipStream_t st = c->stream;
    ENSURE(c, hcounts, std::max<u64>(WH, 1) * 4);
    ENSURE(c, hoff, (WH + 1) * 8);
    ENSURE(c, hbits, std::max<u64>(WH, 1) * 8);
    ENSURE(c, hown, std::max<u64>(WH, 1) * 4);
    tbegin(c, RDF_T_HCOUNT);
    if (WH) {
        hipLaunchKernelGGL(k_expand_owner, dim3(grid_for(c->C, RDF_BLOCK, kGrid)), dim3(RDF_BLOCK), 0, st, c->choffh.as<u64>(),
                           c->C, c->hown.as<u32>());
        const u64 nvb = wave_blocks(WH);
        const dim3 grid(vgrid(nvb));
        if (c->hclassed)
            hipLaunchKernelGGL(k_class_bin_eval, grid, dim3(RDF_BLOCK), 0, st, nvb, v, c->choffh.as<u64>(), c->hown.as<u32>(), 0ull, WH,
                               c->sbase.as<u64>(), c->dcls.as<u32>(), c->cchoff.as<u64>(), c->lwoff.as<u64>(),
                               c->clists.as<u32>(), c->hbits.as<u64>());
        else
            hipLaunchKernelGGL(k_heavy_eval, grid, dim3(RDF_BLOCK), 0, st, nvb, v, c->pivot.as<u32>(), c->choffh.as<u64>(),
                               c->hown.as<u32>(), 0ull, WH, c->hbits.as<u64>());
        if (v.mode == RULES_CLEAN && !c->hclassed)
            hipLaunchKernelGGL(k_heavy_mark, grid, dim3(RDF_BLOCK), 0, st, nvb, v, c->pivot.as<u32>(), c->choffh.as<u64>(), c->hown.as<u32>(), 0ull, WH,
                               c->hbits.as<u64>());
        hipLaunchKernelGGL(k_popc_counts, dim3(grid_for(WH, RDF_BLOCK, kGrid)), dim3(RDF_BLOCK), 0, st, c->hbits.as<u64>(),
                           WH, c->hcounts.as<u32>());
    }
    tend(c, RDF_T_HCOUNT);
    HIP_TRY(c, exclusive_scan_u32_u64(c->ws, c->hcounts.as<u32>(), c->hoff.as<u64>(), WH, c->hoff.as<u64>() + WH, st));
    TRY(read_u64(c, c->hoff.as<u64>() + WH, H));
    return RDF_OK;
}

// mask-class hash table of the unary heavy-only dependents; *nmem members, *ncls classes, *tcapc table size
// (cmax = C also classes the binary heavy-only dependents; *nmem counts the unary members only)
static rdf_status d_class_table(rdf_ctx* c, const CindView& v, u32 cmax, u64* nmem, u32* ncls, u64* tcapc_out) {
    hipStream_t st = c->stream;
    const u64 tcapc = next_pow2(2ull * cmax + 16);
    *tcapc_out = tcapc;
    ENSURE(c, ctab, tcapc * 8);
    ENSURE(c, cflag, tcapc * 4);
    ENSURE(c, ccid, (tcapc + 1) * 4);
    HIP_TRY(c, hipMemsetAsync(c->ctab.p, 0, tcapc * 8, st));
    HIP_TRY(c, hipMemsetAsync(dscal(c, 3), 0, 2 * 8, st));
    if (cmax)
        hipLaunchKernelGGL(k_class_insert, dim3(grid_for(cmax, RDF_BLOCK, kGrid)), dim3(RDF_BLOCK), 0, st, v, cmax,
                           c->ctab.as<u64>(), tcapc - 1, dscal(c, 3));
    hipLaunchKernelGGL(k_nonzero_flags, dim3(grid_for(tcapc, RDF_BLOCK, kGrid)), dim3(RDF_BLOCK), 0, st, c->ctab.as<u64>(),
                       tcapc, c->cflag.as<u32>());
    HIP_TRY(c, exclusive_scan_u32(c->ws, c->cflag.as<u32>(), c->ccid.as<u32>(), tcapc, c->ccid.as<u32>() + tcapc, st));
    u64 rv[2];
    TRY(read_multi(c, {{dscal(c, 3), 8}, {c->ccid.as<u32>() + tcapc, 4}}, rv));
    *nmem = rv[0];
    *ncls = (u32)rv[1];
    return RDF_OK;
}

// class emission tiles (members -> selfpos / output bases; per-class tile offsets); lists at
// lwoff[cchoff[m]] .. lwoff[cchoff[m+1]]
static rdf_status d_class_tiles(rdf_ctx* c, u64 nmem, u32 ncls, u64* HC, u64* NT) {
    hipStream_t st = c->stream;
    *HC = 0;
    *NT = 0;
    if (!nmem) return RDF_OK;
    ENSURE(c, cself, nmem * 4);
    ENSURE(c, cmcnt, nmem * 4);
    ENSURE(c, cobase, (nmem + 1) * 8);
    hipLaunchKernelGGL(k_class_members, dim3(grid_for(nmem, RDF_BLOCK, kGrid)), dim3(RDF_BLOCK), 0, st, c->ckeys.as<u64>(),
                       nmem, c->cchoff.as<u64>(), c->lwoff.as<u64>(), c->clists.as<u32>(), c->cself.as<u32>(),
                       c->cmcnt.as<u32>());
    HIP_TRY(c, exclusive_scan_u32_u64(c->ws, c->cmcnt.as<u32>(), c->cobase.as<u64>(), nmem, c->cobase.as<u64>() + nmem, st));
    ENSURE(c, ctiles, std::max<u64>(ncls, 1) * 4);
    ENSURE(c, ctoff, (ncls + 1ull) * 8);
    hipLaunchKernelGGL(k_class_tiles, dim3(grid_for(std::max<u32>(ncls, 1), RDF_BLOCK, kGrid)), dim3(RDF_BLOCK), 0, st,
                       c->coff.as<u64>(), c->cchoff.as<u64>(), c->lwoff.as<u64>(), ncls, c->ctiles.as<u32>());
    HIP_TRY(c, exclusive_scan_u32_u64(c->ws, c->ctiles.as<u32>(), c->ctoff.as<u64>(), ncls, c->ctoff.as<u64>() + ncls, st));
    u64 v[2];
    TRY(read_multi(c, {{c->cobase.as<u64>() + nmem, 8}, {c->ctoff.as<u64>() + ncls, 8}}, v));
    *HC = v[0];
    *NT = v[1];
    return RDF_OK;
}

// single-rank class path: table -> keys -> per-class pivot -> filtered lists -> tiles.  With c->hclassed the
// binary heavy-only dependents are classed too (their lists are filtered per dependent by d_class_bin).
static rdf_status d_classes_single(rdf_ctx* c, const CindView& v, u64* HC, u64* NT) {
    hipStream_t st = c->stream;
    tbegin(c, RDF_T_CLASS);
    u64 nmem = 0, tcapc = 0;
    u32 ncls = 0;
    TRY(d_class_table(c, v, v.ar ? 0u : (c->hclassed ? c->C : c->Cu), &nmem, &ncls, &tcapc));
    *HC = 0;
    *NT = 0;
    if (ncls) {
        ENSURE(c, ckeys, std::max<u64>(nmem, 1) * 8);
        ENSURE(c, ckeys_tmp, std::max<u64>(nmem, 1) * 8);
        if (nmem) {
            hipLaunchKernelGGL(k_class_keys, dim3(grid_for(c->Cu, RDF_BLOCK, kGrid)), dim3(RDF_BLOCK), 0, st, v,
                               c->ctab.as<u64>(), c->ccid.as<u32>(), tcapc - 1, 0u, 1u, c->ckeys.as<u64>(), dscal(c, 4));
            u64* k = c->ckeys.as<u64>();
            u64* t = c->ckeys_tmp.as<u64>();
            HIP_TRY(c, radix_sort_u64(c->ws, k, t, nmem, 32 + bits_for(ncls ? ncls - 1 : 0), st));
            if (k != c->ckeys.as<u64>()) std::swap(c->ckeys, c->ckeys_tmp);
        }
        const u32* crep = nullptr;
        if (c->hclassed) {
            ENSURE(c, crep, (u64)ncls * 4);
            ENSURE(c, dcls, std::max<u64>(c->C - c->Cu, 1) * 4);
            HIP_TRY(c, hipMemsetAsync(c->crep.p, 0xff, (u64)ncls * 4, st));
            if (c->C)
                hipLaunchKernelGGL(k_class_of, dim3(grid_for(c->C, RDF_BLOCK, kGrid)), dim3(RDF_BLOCK), 0, st, v,
                                   c->ctab.as<u64>(), c->ccid.as<u32>(), tcapc - 1, c->dcls.as<u32>(), c->crep.as<u32>());
            crep = c->crep.as<u32>();
        }
        ENSURE(c, coff, (ncls + 1ull) * 8);
        ENSURE(c, cmask, std::max<u64>(ncls, 1) * 8);
        ENSURE(c, cpiv, std::max<u64>(ncls, 1) * 4);
        ENSURE(c, cnch, std::max<u64>(ncls, 1) * 4);
        ENSURE(c, cchoff, (ncls + 1ull) * 8);
        hipLaunchKernelGGL(k_class_info, dim3(grid_for(ncls + 1ull, RDF_BLOCK, kGrid)), dim3(RDF_BLOCK), 0, st, v,
                           c->ckeys.as<u64>(), nmem, ncls, c->pivot.as<u32>(), crep, c->coff.as<u64>(), c->cmask.as<u64>(),
                           c->cpiv.as<u32>(), c->cnch.as<u32>());
        HIP_TRY(c, exclusive_scan_u32_u64(c->ws, c->cnch.as<u32>(), c->cchoff.as<u64>(), ncls, c->cchoff.as<u64>() + ncls, st));
        u64 WC = 0;
        TRY(read_u64(c, c->cchoff.as<u64>() + ncls, &WC));
        ENSURE(c, ccnt, std::max<u64>(WC, 1) * 4);
        ENSURE(c, cbits, std::max<u64>(WC, 1) * 8);
        ENSURE(c, cown, std::max<u64>(WC, 1) * 4);
        ENSURE(c, lwoff, (WC + 1) * 8);
        if (WC) {
            hipLaunchKernelGGL(k_expand_owner, dim3(grid_for(ncls, RDF_BLOCK, kGrid)), dim3(RDF_BLOCK), 0, st,
                               c->cchoff.as<u64>(), ncls, c->cown.as<u32>());
            const u64 nvb = wave_blocks(WC);
            const dim3 grid(vgrid(nvb));
            hipLaunchKernelGGL(k_class_eval, grid, dim3(RDF_BLOCK), 0, st, nvb, v, c->cchoff.as<u64>(), c->cown.as<u32>(), WC,
                               c->cmask.as<u64>(), c->cpiv.as<u32>(), c->cbits.as<u64>());
            if (v.mode == RULES_CLEAN)
                hipLaunchKernelGGL(k_class_mark, grid, dim3(RDF_BLOCK), 0, st, nvb, v, c->cchoff.as<u64>(), c->cown.as<u32>(), WC,
                                   c->cmask.as<u64>(), c->cpiv.as<u32>(), c->cbits.as<u64>());
            hipLaunchKernelGGL(k_popc_counts, dim3(grid_for(WC, RDF_BLOCK, kGrid)), dim3(RDF_BLOCK), 0, st, c->cbits.as<u64>(),
                               WC, c->ccnt.as<u32>());
        }
        HIP_TRY(c, exclusive_scan_u32_u64(c->ws, c->ccnt.as<u32>(), c->lwoff.as<u64>(), WC, c->lwoff.as<u64>() + WC, st));
        u64 LT = 0;
        TRY(read_u64(c, c->lwoff.as<u64>() + WC, &LT));
        ENSURE(c, clists, std::max<u64>(LT, 1) * 4);
        if (WC)
            hipLaunchKernelGGL(k_class_write, dim3(vgrid(wave_blocks(WC))),
                               dim3(RDF_BLOCK), 0, st, (u64)wave_blocks(WC), v, c->cchoff.as<u64>(), c->cown.as<u32>(), WC, c->cpiv.as<u32>(),
                               c->cbits.as<u64>(), c->lwoff.as<u64>(), c->clists.as<u32>(), (u64*)nullptr);
        TRY(d_class_tiles(c, nmem, ncls, HC, NT));
    }
    tend(c, RDF_T_CLASS);
    c->n_class_members = nmem;
    c->n_classes = ncls;
    return RDF_OK;
}

// classed binary heavy-only dependents: work items = chunks of their class lists -> choffh, *WH
static rdf_status d_class_bin(rdf_ctx* c, const CindView& v, u64* WH) {
    hipStream_t st = c->stream;
    const u32 C = c->C;
    ENSURE(c, sbase, std::max<u64>(C, 1) * 8);
    tbegin(c, RDF_T_HCOUNT);
    if (c->n_classes && C)
        hipLaunchKernelGGL(k_class_bin_chunks, dim3(grid_for(C, RDF_BLOCK, kGrid)), dim3(RDF_BLOCK), 0, st, v,
                           c->dcls.as<u32>(), c->cchoff.as<u64>(), c->lwoff.as<u64>(), c->nchh.as<u32>(), c->sbase.as<u64>());
    else
        HIP_TRY(c, hipMemsetAsync(c->nchh.p, 0, std::max<u64>(C, 1) * 4, st));
    tend(c, RDF_T_HCOUNT);
    HIP_TRY(c, exclusive_scan_u32_u64(c->ws, c->nchh.as<u32>(), c->choffh.as<u64>(), C, c->choffh.as<u64>() + C, st));
    TRY(read_u64(c, c->choffh.as<u64>() + C, WH));
    c->heavy_candidates = *WH * RDF_WAVE;  // class-list entries scanned (upper bound)
    return RDF_OK;
}

// K7 minimality on the (owned) explicit pairs, heavy-only binary write pass, class emission -> out
// minimality rules on the explicit pairs and their kept refs compacted into out[0, *K) (out sized for E refs + `extra`)
static rdf_status d_emit_rules(rdf_ctx* c, const CindView& v, u64 E, u64 extra, u64* Kout) {
    hipStream_t st = c->stream;
    ENSURE(c, out, std::max<u64>(E + extra, 1) * 4);  // the class part is expanded behind it on demand (materialize)
    ENSURE(c, flags, std::max<u64>(E, 1) * 4);
    ENSURE(c, pos, (E + 1) * 8);
    tbegin(c, RDF_T_RULES);
    if (E)
        hipLaunchKernelGGL(k_rules_explicit, dim3(grid_for(E, RDF_BLOCK, kGrid)), dim3(RDF_BLOCK), 0, st, v,
                           c->epairs.as<u64>(), E, c->rank, c->nranks, c->flags.as<u32>());
    if (E && v.mode == RULES_CLEAN)
        hipLaunchKernelGGL(k_rules_mark, dim3(grid_for(E, RDF_BLOCK, kGrid)), dim3(RDF_BLOCK), 0, st, v, c->epairs.as<u64>(),
                           0ull, E, c->rank, c->nranks, c->flags.as<u32>());
    HIP_TRY(c, exclusive_scan_u32_u64(c->ws, c->flags.as<u32>(), c->pos.as<u64>(), E, c->pos.as<u64>() + E, st));
    if (E)
        hipLaunchKernelGGL(k_compact_refs, dim3(grid_for(E, RDF_BLOCK, kGrid)), dim3(RDF_BLOCK), 0, st, c->epairs.as<u64>(), E,
                           c->flags.as<u32>(), c->pos.as<u64>(), c->out.as<u32>());
    tend(c, RDF_T_RULES);
    return read_u64(c, c->pos.as<u64>() + E, Kout);
}

static rdf_status d_emit_rest(rdf_ctx* c, const CindView& v, u64 E, u64 K, u64 WH, u64 H, u64 HC, u64 NT, u64 runs0);
static rdf_status d_emit(rdf_ctx* c, const CindView& v, u64 E, u64 WH, u64 H, u64 HC, u64 NT) {
    u64 K = 0;
    TRY(d_emit_rules(c, v, E, H, &K));
    return d_emit_rest(c, v, E, K, WH, H, HC, NT, 0);
}

// the heavy-only refs behind the K explicit ones, the class lists' offsets, the run table from run runs0 on (the
// explicit runs [0, runs0) were written early), the stage's statistics
static rdf_status d_emit_rest(rdf_ctx* c, const CindView& v, u64 E, u64 K, u64 WH, u64 H, u64 HC, u64 NT, u64 runs0) {
    hipStream_t st = c->stream;
    (void)E;
    if ((u64)c->out.cap < std::max<u64>(K + H, 1) * 4) {  // the early rules sized `out` before H was known
        TRY(hv_wait(c, false));
        HIP_TRY(c, c->out.grow_keep(std::max<u64>(K + H, 1) * 4, st));
    }
    c->res_bits = c->result_form == RDF_FORM_HEAVY_BITS && c->hclassed && WH;
    c->heavy_pending = false;
    tbegin(c, RDF_T_HWRITE);
    if (WH && c->res_bits) {  // (handed over as bits; expanded in `out` only when a row accessor needs it)
        c->heavy_pending = true;
        c->hp_W = WH;
        c->hp_h0 = 0;
        c->hp_K = K;
    } else if (WH) {
        hipLaunchKernelGGL(k_heavy_write, dim3(vgrid(wave_blocks(WH))),
                           dim3(RDF_BLOCK), 0, st, (u64)wave_blocks(WH), v, c->pivot.as<u32>(), c->choffh.as<u64>(), c->hown.as<u32>(), 0ull, WH,
                           c->hbits.as<u64>(), c->hclassed ? c->clists.as<u32>() : c->gcap.as<u32>(),
                           c->hclassed ? c->sbase.as<u64>() : (const u64*)nullptr, c->hoff.as<u64>(), K, c->out.as<u32>());
    }
    tend(c, RDF_T_HWRITE);
    // The class part stays compact: each member's refs are its class's shared list minus itself (a CindSet whose
    // ref list is shared, ALG/data/CindSet.scala:9-13).  rdf_copy_result_compact hands it over as is; the expanded
    // per-dependent runs (k_class_emit) are written only when a caller asks for rows (materialize).
    c->class_pending = NT > 0;
    c->pend_NT = NT;
    c->pend_base = K + H;
    c->res_K = K;
    c->res_nx = c->C;
    c->res_wh = WH;
    c->res_h0 = 0;
    const u32 ncls = (u32)c->n_classes;
    c->n_lists = HC || c->res_bits ? ncls : 0;  // (the heavy bits index the class lists)
    c->n_list_refs = 0;
    if (c->n_lists) {
        ENSURE(c, loff, (ncls + 1ull) * 8);
        hipLaunchKernelGGL(k_list_offsets, dim3(grid_for(ncls + 1ull, RDF_BLOCK, kGrid)), dim3(RDF_BLOCK), 0, st,
                           c->cchoff.as<u64>(), c->lwoff.as<u64>(), ncls, c->loff.as<u64>());
    }
    // run table: the dependent of every output ref (CindSet-shaped result, ALG/data/CindSet.scala:9-13)
    const u64 nmem = HC ? c->n_class_members : 0;
    const u64 R = (u64)c->C + WH + nmem;
    if (runs0) {  // the explicit runs are in place (and may be on their way to the host): grow keeping them
        if ((u64)c->runoff.cap < (R + 1) * 8 || (u64)c->rundep.cap < std::max<u64>(R, 1) * 4) {
            TRY(hv_wait(c, false));
            HIP_TRY(c, c->runoff.grow_keep((R + 1) * 8, st));
            HIP_TRY(c, c->rundep.grow_keep(std::max<u64>(R, 1) * 4, st));
        }
    } else {
        ENSURE(c, runoff, (R + 1) * 8);
        ENSURE(c, rundep, std::max<u64>(R, 1) * 4);
    }
    hipLaunchKernelGGL(k_output_runs, dim3(grid_for(R + 1 - runs0, RDF_BLOCK, kGrid)), dim3(RDF_BLOCK), 0, st, c->C, v.eoff,
                       c->pos.as<u64>(), WH, c->choffh.as<u64>(), c->hoff.as<u64>(), K, nmem, c->ckeys.as<u64>(),
                       c->cobase.as<u64>(), H, K + H + HC, c->runoff.as<u64>(), c->rundep.as<u32>(), runs0, R);
    c->n_runs = R;
    c->n_runs_explicit = (u64)c->C + WH;
    c->h_runs_valid = false;
    ++c->run_id;
    HIP_TRY(c, hipEventRecord(c->ev[5], st));
    HIP_TRY(c, hipGetLastError());
    HIP_TRY(c, hipStreamSynchronize(st));
    if (c->n_lists) TRY(read_u64(c, c->loff.as<u64>() + ncls, &c->n_list_refs));
    HIP_TRY(c, hipEventElapsedTime(&c->stage_ms[2], c->ev[4], c->ev[5]));
    settle_timings(c);
    tcollect(c, RDF_T_PIVOT, RDF_NUM_TIMERS);
    c->n_out = K + H + HC;
    c->n_class_out = HC;
    c->out_ptr = c->out.as<u32>();
    rdf_cind_stats& s = c->cstats;
    memset(&s, 0, sizeof(s));
    s.n_cinds = c->n_out;
    s.n_explicit_raw = c->n_explicit_raw;
    s.n_light_chunks = c->n_light_chunks;
    s.n_heavy_chunks = WH;
    s.ms_pivot = c->tms[RDF_T_PIVOT];
    s.ms_light = c->tms[RDF_T_LIGHT];
    s.ms_rules = c->tms[RDF_T_RULES];
    s.ms_heavy = c->tms[RDF_T_HCOUNT] + c->tms[RDF_T_HWRITE];
    s.n_heavy_candidates = c->heavy_candidates;
    s.n_class_members = c->n_class_members;
    s.n_classes = c->n_classes;
    s.n_class_cinds = c->n_class_out;
    s.n_light_candidates = c->light_candidates;
    s.n_light_entries = c->light_entries;
    c->stage = 4;
    return RDF_OK;
}

// Light dependents with identical group lists (k_dup_*, kernels.inl): after the pivot pass the members of every class
// lose their light items (only the representative, the class's smallest compact id, is verified); after the light pass
// their explicit pairs are derived from the representative's (d_dedup_expand).  Strategy 1 without association rules
// (the strategy-0 quirk and the rules' per-pair drop are per dependent), one GPU, unpaged.
static rdf_status d_light_dedup(rdf_ctx* c, const CindView& v) {
    c->n_dedup_members = 0;
    c->dedup_pending = false;
    const u32 C = c->C;
    // automatic: only inputs whose light pass takes the LDS-staging variant (small light groups) have enough such
    // classes to pay for finding them (c2: 22 % of the light group entries, light 2.02 -> 1.80 ms, step -0.08 ms; c3
    // and c4 at 0.4: ~2.5 %, no gain; profiles/r06_light_dedup_ab.log).  The member count waits in scalar slot 9
    // (which no light-pass stage uses) until d_dedup_expand reads it with the pair count
    const bool on = c->light_dedup < 0 ? c->light_stage : c->light_dedup != 0;
    if (!on || v.literal || v.ar || c->nranks != 1 || !C) return RDF_OK;
    hipStream_t st = c->stream;
    const u64 tcap = next_pow2(2ull * C + 16);
    ENSURE(c, ukey, (u64)C * 8);
    ENSURE(c, utab, tcap * 8);
    ENSURE(c, urep, (u64)C * 4);
    tbegin(c, RDF_T_PIVOT);
    HIP_TRY(c, hipMemsetAsync(c->utab.p, 0xff, tcap * 8, st));
    HIP_TRY(c, hipMemsetAsync(dscal(c, 9), 0, 8, st));
    const dim3 g(grid_for(C, RDF_BLOCK, kGrid));
    hipLaunchKernelGGL(k_dup_insert, g, dim3(RDF_BLOCK), 0, st, v, c->nchl.as<u32>(), c->ukey.as<u64>(), c->utab.as<u64>(),
                       tcap - 1, (u64)c->dup_min);
    ENSURE(c, ucnt, (u64)C * 4);
    ENSURE(c, unoff, (C + 1ull) * 8);
    ENSURE(c, eoff, (C + 1ull) * 8);  // (scratch here: the members' chunk offsets; the explicit index rewrites it)
    hipLaunchKernelGGL(k_dup_rep, g, dim3(RDF_BLOCK), 0, st, v, c->ukey.as<u64>(), c->utab.as<u64>(), tcap - 1,
                       c->urep.as<u32>(), c->ucnt.as<u32>(), (u32*)c->unoff.p);
    HIP_TRY(c, exclusive_scan_u32_u64(c->ws, c->ucnt.as<u32>(), c->eoff.as<u64>(), C, c->eoff.as<u64>() + C, st));
    // (the chunk count stays on the device: a grid-stride verify pass instead of a read-back)
    hipLaunchKernelGGL(k_dup_verify, dim3(kGrid), dim3(RDF_BLOCK), 0, st, v, c->urep.as<u32>(), c->eoff.as<u64>(),
                       (u32*)c->unoff.p);
    ENSURE(c, umem, (u64)C * 4);
    hipLaunchKernelGGL(k_dup_unplan, g, dim3(RDF_BLOCK), 0, st, c->urep.as<u32>(), (const u32*)c->unoff.p, C,
                       c->nchl.as<u32>(), c->nitl.as<u32>(), c->npk.as<u32>(), (u32*)dscal(c, 9), c->umem.as<u32>());
    HIP_TRY(c, hipGetLastError());
    tend(c, RDF_T_PIVOT);
    c->dedup_pending = true;  // the member count is read with the expansion's pair count (d_dedup_expand)
    return RDF_OK;
}

// the members' explicit pairs from their representatives' (V(r) minus the member and its components), every pair in
// (dependent, ref) order again; *E grows by the members' pairs.  The new index (eoff = the scanned counts, ebin shifted
// by the same offsets) is written here, so d_explicit_index need not search the pairs again (*indexed)
static rdf_status d_dedup_expand(rdf_ctx* c, const CindView& v, u64* E, bool* indexed) {
    *indexed = false;
    if (!c->dedup_pending) return RDF_OK;
    c->dedup_pending = false;
    hipStream_t st = c->stream;
    const u32 C = c->C;
    const u64 E0 = *E;
    ENSURE(c, eoff, (C + 1ull) * 8);
    ENSURE(c, ebin, std::max<u64>(C, 1) * 8);
    ENSURE(c, ucnt, (u64)C * 4);
    ENSURE(c, unoff, (C + 1ull) * 8);
    ENSURE(c, uebin, std::max<u64>(C, 1) * 8);
    tbegin(c, RDF_T_ESORT);
    hipLaunchKernelGGL(k_pair_offsets, dim3(grid_for(C + 1ull, RDF_BLOCK, kGrid)), dim3(RDF_BLOCK), 0, st,
                       c->epairs.as<u64>(), E0, C, c->Cu, c->eoff.as<u64>(), c->ebin.as<u64>());
    hipLaunchKernelGGL(k_dup_counts, dim3(grid_for(C, RDF_BLOCK, kGrid)), dim3(RDF_BLOCK), 0, st, v, c->urep.as<u32>(),
                       c->eoff.as<u64>(), c->ucnt.as<u32>());
    HIP_TRY(c, exclusive_scan_u32_u64(c->ws, c->ucnt.as<u32>(), c->unoff.as<u64>(), C, c->unoff.as<u64>() + C, st));
    tend(c, RDF_T_ESORT);
    ScalarGather sg = {};  // one read-back: the expanded pair count and the member count
    sg.p[0] = c->unoff.as<u64>() + C;
    sg.bytes[0] = 8;
    sg.p[1] = dscal(c, 9);
    sg.bytes[1] = 4;
    sg.n = 2;
    u64 rb[2] = {0, 0};
    TRY(gather_read(c, sg, rb));
    const u64 E1 = rb[0];
    c->n_dedup_members = rb[1];
    if (!c->n_dedup_members) return RDF_OK;  // (E1 == E0: nothing moves)
    ENSURE(c, epairs_tmp, std::max<u64>(E1, 1) * 8);
    tbegin(c, RDF_T_ESORT);
    hipLaunchKernelGGL(k_dup_move, dim3(grid_for(std::max<u64>(E0, C), RDF_BLOCK, kGrid)), dim3(RDF_BLOCK), 0, st,
                       c->epairs.as<u64>(), E0, C, c->urep.as<u32>(), c->eoff.as<u64>(), c->ebin.as<u64>(),
                       c->unoff.as<u64>(), c->epairs_tmp.as<u64>(), c->uebin.as<u64>());
    const u64 nm = c->n_dedup_members;
    const unsigned eg = grid_for(nm, RDF_WAVES_PER_BLOCK, 4 * kGrid);
    hipLaunchKernelGGL(k_dup_expand, dim3(eg), dim3(RDF_BLOCK), 0, st, (u64)eg * RDF_WAVES_PER_BLOCK, nm, v,
                       c->umem.as<u32>(), c->urep.as<u32>(), c->epairs.as<u64>(), c->eoff.as<u64>(), c->ebin.as<u64>(),
                       c->unoff.as<u64>(), c->epairs_tmp.as<u64>(), c->uebin.as<u64>());
    HIP_TRY(c, hipGetLastError());
    tend(c, RDF_T_ESORT);
    std::swap(c->epairs, c->epairs_tmp);
    std::swap(c->eoff, c->unoff);
    std::swap(c->ebin, c->uebin);
    *E = E1;
    *indexed = true;
    return RDF_OK;
}

rdf_status rdf_discover_cinds(rdf_ctx* c, uint32_t flags, rdf_cind_stats* stats) {
    if (!c) return RDF_ERR_ARG;
    if (c->stage < 3) return fail(c, RDF_ERR_STATE, "rdf_build_capture_groups must be called first");
    if (c->nranks != 1) return fail(c, RDF_ERR_STATE, "capture groups were built in sharded mode");
    HIP_TRY(c, hipSetDevice(c->device));
    TRY(hv_wait(c, true));
    c->res_bits = c->heavy_pending = false;  // (the heavy-bits form: results of d_emit_rest / d_page_emit only)
    c->paged = false;
    // test hook (RDFIND_TEST_OOM_DISCOVERY=1): the unpaged discovery reports RDF_ERR_OOM at once, so a caller's
    // fallback to pages runs on small inputs
    if (c->test_oom_discovery) return fail(c, RDF_ERR_OOM, "test hook: the unpaged discovery runs out of memory");
    hipStream_t st = c->stream;
    if (c->hv_capid && c->hv_sup && c->C && (u64)c->C <= c->hv_cap_cap) {  // the capture table is final: early copy
        HIP_TRY(c, hipEventRecord(c->hv_ev, st));
        HIP_TRY(c, hipStreamWaitEvent(c->hstream, c->hv_ev, 0));
        HIP_TRY(c, hipMemcpyAsync(c->hv_capid, c->fext.p, (u64)c->C * 4, hipMemcpyDeviceToHost, c->hstream));
        HIP_TRY(c, hipMemcpyAsync(c->hv_sup, c->csup.p, (u64)c->C * 4, hipMemcpyDeviceToHost, c->hstream));
        c->hv_caps_done = true;
        c->hv_pending = true;
    }
    CindView v = make_view(c, flags);
    TRY(d_pivot_local(c, v));
    tbegin(c, RDF_T_PIVOT);
    if (c->C) {
        const unsigned gp = grid_for(c->C, RDF_BLOCK, kGrid);
        ENSURE(c, ppart, 3ull * gp * 8);
        hipLaunchKernelGGL(k_pivot_final, dim3(gp), dim3(RDF_BLOCK), 0, st, v, c->pbest.as<u64>(),
                           c->pnl.as<u32>(), c->pivot.as<u32>(), c->nchl.as<u32>(), c->nitl.as<u32>(), c->npk.as<u32>(),
                           c->nchh.as<u32>(), c->info.as<CapInfo>(), c->ppart.as<u64>());
        hipLaunchKernelGGL(k_sum_partials3, dim3(1), dim3(RDF_BLOCK), 0, st, c->ppart.as<u64>(), gp, dscal(c, 2));
    }
    tend(c, RDF_T_PIVOT);
    TRY(d_light_dedup(c, v));
    u64 WL = 0, WH = 0, WI = 0, WP = 0, E = 0, H = 0, HC = 0, NT = 0;
    TRY(d_multi_items(c));
    TRY(d_chunks(c, &WL, &WH, &WI, &WP));
    c->n_light_survivors = 0;
    const bool two = use_two_pass(c, WI);
    if (two) TRY(d_light_two_pass(c, v, WI, WL, WP, &E, c->pivot.as<u32>()));
    else TRY(d_light(c, v, WI, WL, WP, &E, c->pivot.as<u32>()));
    bool indexed = false;
    TRY(d_dedup_expand(c, v, &E, &indexed));
    if (getenv("RDFIND_LIGHT2_LOG"))
        fprintf(stderr, "LIGHT2 two=%d items=%llu multi_chunk_items=%llu survivors=%llu explicit=%llu\n",
                (int)two, (unsigned long long)WI, (unsigned long long)c->n_multi_items,
                (unsigned long long)c->n_light_survivors, (unsigned long long)E);
    c->n_explicit_raw = E;
    c->n_light_chunks = WL;
    TRY(d_explicit_index(c, v, E, true, indexed));
    // the explicit pairs' rules first: their refs are final before the class stage, so an early hand-over copies them
    // while the classes and the heavy-only dependents are computed
    u64 K = 0;
    TRY(d_emit_rules(c, v, E, 0, &K));
    u64 runs0 = 0;  // explicit runs written early
    if (c->hv_runoff && c->hv_rundep && (u64)c->C <= c->hv_runs_cap) {
        ENSURE(c, runoff, (c->C + 1ull) * 8);
        ENSURE(c, rundep, std::max<u64>(c->C, 1) * 4);
        if (c->C)
            hipLaunchKernelGGL(k_output_runs, dim3(grid_for(c->C, RDF_BLOCK, kGrid)), dim3(RDF_BLOCK), 0, st, c->C, v.eoff,
                               c->pos.as<u64>(), 0ull, c->choffh.as<u64>(), c->hoff.as<u64>(), K, 0ull, c->ckeys.as<u64>(),
                               c->cobase.as<u64>(), 0ull, K, c->runoff.as<u64>(), c->rundep.as<u32>(), 0ull,
                               (u64)c->C - 1);
        runs0 = c->C;
    }
    if ((c->hv_refs && K <= c->hv_refs_cap) || runs0) {
        HIP_TRY(c, hipEventRecord(c->hv_ev, st));
        HIP_TRY(c, hipStreamWaitEvent(c->hstream, c->hv_ev, 0));
        if (c->hv_refs && K <= c->hv_refs_cap) {
            if (K) HIP_TRY(c, hipMemcpyAsync(c->hv_refs, c->out.p, K * 4, hipMemcpyDeviceToHost, c->hstream));
            c->hv_refs_n = K;
        }
        if (runs0) {
            HIP_TRY(c, hipMemcpyAsync(c->hv_runoff, c->runoff.p, runs0 * 8, hipMemcpyDeviceToHost, c->hstream));
            HIP_TRY(c, hipMemcpyAsync(c->hv_rundep, c->rundep.p, runs0 * 4, hipMemcpyDeviceToHost, c->hstream));
            c->hv_runs_n = runs0;
        }
        c->hv_pending = true;
    }
    // strategy 0's quirk filter is per dependent: keep the pivot scan there (RDFIND_HCLASS=0: test hook)
    c->hclassed = !v.literal && c->allow_hclass && !v.ar;
    TRY(d_classes_single(c, v, &HC, &NT));
    if (c->hclassed) TRY(d_class_bin(c, v, &WH));
    TRY(d_heavy_count(c, v, WH, &H));
    TRY(d_emit_rest(c, v, E, K, WH, H, HC, NT, runs0));
    if (stats) *stats = c->cstats;
    mem_report(c);
    return RDF_OK;
}

// ------------------------------------------------------------------------------------------------
// Paged discovery: the result of a dependent range at a time, in bounded HBM (the reference streams its output to
// the sink, ALG/programs/RDFind.scala:507-520).  The minimality rules probe other dependents only through the unary
// components of binary dependents (R1 / R4), so the unary dependents' explicit pairs are computed first and stay
// resident; every later page takes a range of binary dependents: its light pass, its explicit index on top of the
// unary pairs, its rules, its heavy-only dependents.  Page 0 holds the unary dependents (explicit runs, the shared
// class lists, heavy-path ones), pages 1.. the binary ones.  Each page is the context's current result (compact
// hand-over, checksum, row accessors); the pages partition the result of rdf_discover_cinds.

// result of dependents [d0, d1): explicit pairs epairs[e0, e1) (their rules), heavy-only work items [h0, h1), and on
// page 0 the class part (pending expansion)
static rdf_status d_page_emit(rdf_ctx* c, const CindView& v, u32 d0, u32 d1, u64 e0, u64 e1, u64 h0, u64 h1, u64 HC,
                              u64 NT) {
    hipStream_t st = c->stream;
    const u64 E = e1 - e0, WHr = h1 - h0, nd = d1 - d0;
    // heavy-only dependents of the range: survivor bits, counts, offsets
    ENSURE(c, hcounts, std::max<u64>(WHr, 1) * 4);
    ENSURE(c, hoff, (WHr + 1) * 8);
    ENSURE(c, hbits, std::max<u64>(WHr, 1) * 8);
    ENSURE(c, hown, std::max<u64>(WHr, 1) * 4);
    tbegin(c, RDF_T_HCOUNT);
    if (WHr) {
        hipLaunchKernelGGL(k_expand_owner_range, dim3(grid_for(nd, RDF_BLOCK, kGrid)), dim3(RDF_BLOCK), 0, st,
                           c->choffh.as<u64>(), d0, d1, c->hown.as<u32>());
        const u64 nvb = wave_blocks(WHr);
        const dim3 grid(vgrid(nvb));
        if (c->hclassed)
            hipLaunchKernelGGL(k_class_bin_eval, grid, dim3(RDF_BLOCK), 0, st, nvb, v, c->choffh.as<u64>(), c->hown.as<u32>(),
                               h0, WHr, c->sbase.as<u64>(), c->dcls.as<u32>(), c->cchoff.as<u64>(), c->lwoff.as<u64>(),
                               c->clists.as<u32>(), c->hbits.as<u64>());
        else
            hipLaunchKernelGGL(k_heavy_eval, grid, dim3(RDF_BLOCK), 0, st, nvb, v, c->pivot.as<u32>(), c->choffh.as<u64>(),
                               c->hown.as<u32>(), h0, WHr, c->hbits.as<u64>());
        if (v.mode == RULES_CLEAN && !c->hclassed)
            hipLaunchKernelGGL(k_heavy_mark, grid, dim3(RDF_BLOCK), 0, st, nvb, v, c->pivot.as<u32>(), c->choffh.as<u64>(),
                               c->hown.as<u32>(), h0, WHr, c->hbits.as<u64>());
        hipLaunchKernelGGL(k_popc_counts, dim3(grid_for(WHr, RDF_BLOCK, kGrid)), dim3(RDF_BLOCK), 0, st, c->hbits.as<u64>(),
                           WHr, c->hcounts.as<u32>());
    }
    tend(c, RDF_T_HCOUNT);
    HIP_TRY(c, exclusive_scan_u32_u64(c->ws, c->hcounts.as<u32>(), c->hoff.as<u64>(), WHr, c->hoff.as<u64>() + WHr, st));
    // minimality on the range's explicit pairs
    ENSURE(c, flags, std::max<u64>(E, 1) * 4);
    ENSURE(c, pos, (E + 1) * 8);
    tbegin(c, RDF_T_RULES);
    if (E)
        hipLaunchKernelGGL(k_rules_explicit, dim3(grid_for(E, RDF_BLOCK, kGrid)), dim3(RDF_BLOCK), 0, st, v,
                           c->epairs.as<u64>() + e0, E, 0u, 1u, c->flags.as<u32>());
    if (E && v.mode == RULES_CLEAN)
        hipLaunchKernelGGL(k_rules_mark, dim3(grid_for(E, RDF_BLOCK, kGrid)), dim3(RDF_BLOCK), 0, st, v, c->epairs.as<u64>(),
                           e0, E, 0u, 1u, c->flags.as<u32>());
    HIP_TRY(c, exclusive_scan_u32_u64(c->ws, c->flags.as<u32>(), c->pos.as<u64>(), E, c->pos.as<u64>() + E, st));
    tend(c, RDF_T_RULES);
    u64 kh[2];
    TRY(read_multi(c, {{c->pos.as<u64>() + E, 8}, {c->hoff.as<u64>() + WHr, 8}}, kh));
    const u64 K = kh[0], H = kh[1];
    if (c->hv_gpu_wait) {  // the previous page's refs may still be on their way to the host (rdf_copy_result_refs_async)
        if (c->out.cap < std::max<u64>(K + H, 1) * 4) TRY(hv_wait(c, false));  // (growing frees what the copy reads)
        else HIP_TRY(c, hipStreamWaitEvent(c->stream, c->hv_done, 0));
    }
    ENSURE(c, out, std::max<u64>(K + H, 1) * 4);
    if (E)
        hipLaunchKernelGGL(k_compact_refs, dim3(grid_for(E, RDF_BLOCK, kGrid)), dim3(RDF_BLOCK), 0, st,
                           c->epairs.as<u64>() + e0, E, c->flags.as<u32>(), c->pos.as<u64>(), c->out.as<u32>());
    c->res_bits = c->result_form == RDF_FORM_HEAVY_BITS && c->hclassed && c->n_classes;
    c->heavy_pending = false;  // (the previous page's, if nobody asked for its rows)
    tbegin(c, RDF_T_HWRITE);
    if (WHr && c->res_bits) {  // (handed over as bits; expanded in `out` only when a row accessor needs it)
        c->heavy_pending = true;
        c->hp_W = WHr;
        c->hp_h0 = h0;
        c->hp_K = K;
    } else if (WHr) {
        hipLaunchKernelGGL(k_heavy_write, dim3(vgrid(wave_blocks(WHr))), dim3(RDF_BLOCK), 0, st, (u64)wave_blocks(WHr), v,
                           c->pivot.as<u32>(), c->choffh.as<u64>(), c->hown.as<u32>(), h0, WHr, c->hbits.as<u64>(),
                           c->hclassed ? c->clists.as<u32>() : c->gcap.as<u32>(),
                           c->hclassed ? c->sbase.as<u64>() : (const u64*)nullptr, c->hoff.as<u64>(), K, c->out.as<u32>());
    }
    tend(c, RDF_T_HWRITE);
    c->class_pending = NT > 0;
    c->pend_NT = NT;
    c->pend_base = K + H;
    c->res_K = K;
    c->res_nx = nd;
    c->res_wh = WHr;
    c->res_h0 = h0;
    const u32 ncls = (u32)c->n_classes;
    // the class lists go with the first page (the class part; in the heavy-bits form also the lists every later page's
    // heavy bits index: a consumer keeps them)
    c->n_lists = HC || (c->res_bits && d0 == 0) ? ncls : 0;
    c->n_list_refs = 0;
    if (c->n_lists) {
        ENSURE(c, loff, (ncls + 1ull) * 8);
        hipLaunchKernelGGL(k_list_offsets, dim3(grid_for(ncls + 1ull, RDF_BLOCK, kGrid)), dim3(RDF_BLOCK), 0, st,
                           c->cchoff.as<u64>(), c->lwoff.as<u64>(), ncls, c->loff.as<u64>());
    }
    const u64 nmem = HC ? c->n_class_members : 0;
    const u64 R = nd + WHr + nmem;
    ENSURE(c, runoff, (R + 1) * 8);
    ENSURE(c, rundep, std::max<u64>(R, 1) * 4);
    hipLaunchKernelGGL(k_output_runs_range, dim3(grid_for(R + 1, RDF_BLOCK, kGrid)), dim3(RDF_BLOCK), 0, st, c->C, d0, d1,
                       v.eoff, e0, c->pos.as<u64>(), h0, WHr, c->choffh.as<u64>(), c->hoff.as<u64>(), K, nmem,
                       c->ckeys.as<u64>(), c->cobase.as<u64>(), H, K + H + HC, c->runoff.as<u64>(), c->rundep.as<u32>());
    HIP_TRY(c, hipGetLastError());
    HIP_TRY(c, hipStreamSynchronize(st));
    if (c->n_lists) TRY(read_u64(c, c->loff.as<u64>() + ncls, &c->n_list_refs));
    c->n_runs = R;
    c->n_runs_explicit = nd + WHr;
    c->h_runs_valid = false;
    ++c->run_id;
    c->n_out = K + H + HC;
    c->n_class_out = HC;
    c->out_ptr = c->out.as<u32>();
    c->cstats.n_cinds = c->n_out;
    c->stage = 4;
    return RDF_OK;
}

// greedy dependent range from d0 whose light octets and heavy work items fit the page budget (at least one dependent)
static constexpr u64 PAGE_PER_OCT = 8 * 8 + 8 + 12 + 8 * 4 + 8 + 4;  // slots, kill mask, counts, pairs, flags / positions, refs
static constexpr u64 PAGE_PER_CHUNK = 8 + 4 + 8 + 4 + RDF_WAVE * 4;   // bits, counts, offsets, owner, refs
static u32 page_end(const rdf_ctx* c, u32 d0, u32 dmax) {
    u32 d1 = d0 + 1;
    while (d1 < dmax) {
        const u64 oct = c->h_choffl[d1 + 1] - c->h_choffl[d0], ch = c->h_choffh[d1 + 1] - c->h_choffh[d0];
        if (oct * PAGE_PER_OCT + ch * PAGE_PER_CHUNK > c->pg_budget) break;
        ++d1;
    }
    return d1;
}
// the same for the unary dependents' output pages, whose explicit pairs are resident: the emission's per-pair scratch
// (rule flags, positions, output refs) and the heavy work items of the range must fit the budget
static u32 unary_page_end(const rdf_ctx* c, u32 d0) {
    const u64 per_pair = 4 + 8 + 4;
    if (d0 >= c->Cu) return c->Cu;
    u32 d1 = d0 + 1;
    while (d1 < c->Cu) {
        const u64 np = c->h_eoffu[d1 + 1] - c->h_eoffu[d0], ch = c->h_choffh[d1 + 1] - c->h_choffh[d0];
        if (np * per_pair + ch * PAGE_PER_CHUNK > c->pg_budget) break;
        ++d1;
    }
    return d1;
}

rdf_status rdf_discover_cinds_paged(rdf_ctx* c, uint32_t flags, uint64_t page_bytes, rdf_cind_stats* stats) {
    if (!c) return RDF_ERR_ARG;
    if (c->stage < 3) return fail(c, RDF_ERR_STATE, "rdf_build_capture_groups must be called first");
    if (c->nranks != 1) return fail(c, RDF_ERR_STATE, "capture groups were built in sharded mode");
    HIP_TRY(c, hipSetDevice(c->device));
    TRY(hv_wait(c, true));
    c->res_bits = c->heavy_pending = false;  // (the heavy-bits form: results of d_emit_rest / d_page_emit only)
    hipStream_t st = c->stream;
    if (!page_bytes) {  // an eighth of the free HBM, at most 32 GB: the resident unary pairs need the rest
        size_t fr = 0, tot = 0;
        HIP_TRY(c, hipMemGetInfo(&fr, &tot));
        page_bytes = std::max<u64>(std::min<u64>(fr / 8, 32ull << 30), 1ull << 26);
    }
    CindView v = make_view(c, flags);
    TRY(d_pivot_local(c, v));
    tbegin(c, RDF_T_PIVOT);
    if (c->C) {
        const unsigned gp = grid_for(c->C, RDF_BLOCK, kGrid);
        ENSURE(c, ppart, 3ull * gp * 8);
        hipLaunchKernelGGL(k_pivot_final, dim3(gp), dim3(RDF_BLOCK), 0, st, v, c->pbest.as<u64>(),
                           c->pnl.as<u32>(), c->pivot.as<u32>(), c->nchl.as<u32>(), c->nitl.as<u32>(), c->npk.as<u32>(),
                           c->nchh.as<u32>(), c->info.as<CapInfo>(), c->ppart.as<u64>());
        hipLaunchKernelGGL(k_sum_partials3, dim3(1), dim3(RDF_BLOCK), 0, st, c->ppart.as<u64>(), gp, dscal(c, 2));
    }
    tend(c, RDF_T_PIVOT);
    u64 WL = 0, WH = 0, WI = 0, WP = 0, WM = 0, HC = 0, NT = 0;
    TRY(d_chunks(c, &WL, &WH, &WI, &WP));
    TRY(d_light_owners(c, WI, WP, &WM));
    c->pg_budget = page_bytes;
    c->pg_WM = WM;
    c->h_choffl.resize(c->C + 1ull);
    HIP_TRY(c, ctx_copy(c, c->h_choffl.data(), c->choffl.p, (c->C + 1ull) * 8, hipMemcpyDeviceToHost));
    c->h_choffh.assign(c->C + 1ull, 0);  // no heavy work while the unary light pass is batched
    // the unary dependents' explicit pairs, in budgeted batches, resident for the rest of the run
    u64 Eu = 0;
    for (u32 d0 = 0; d0 < c->Cu;) {
        const u32 d1 = page_end(c, d0, c->Cu);
        LightRange r;
        TRY(light_range(c, d0, d1, WM > 0, &r));
        u64 E = 0;
        TRY(d_light_run(c, v, c->pivot.as<u32>(), r, Eu, &E));
        Eu += E;
        d0 = d1;
    }
    c->n_explicit_raw = Eu;
    c->n_light_chunks = WL;
    // room behind the resident unary pairs for the largest binary page (<= 8 pairs per light octet of the budget), so
    // the pages append without re-copying the resident pairs
    HIP_TRY(c, c->epairs.grow_keep((size_t)(Eu + c->pg_budget / PAGE_PER_OCT * 8 + 1) * 8, st));
    TRY(d_explicit_index(c, v, Eu, true));
    c->h_eoffu.resize(c->Cu + 1ull);  // on the context stream: hipMemcpy would not wait for k_pair_offsets there
    HIP_TRY(c, hipMemcpyAsync(c->h_eoffu.data(), c->eoff.p, (c->Cu + 1ull) * 8, hipMemcpyDeviceToHost, st));
    HIP_TRY(c, hipStreamSynchronize(st));
    c->hclassed = !v.literal && c->allow_hclass && !v.ar;
    TRY(d_classes_single(c, v, &HC, &NT));
    if (c->hclassed) TRY(d_class_bin(c, v, &WH));
    HIP_TRY(c, ctx_copy(c, c->h_choffh.data(), c->choffh.p, (c->C + 1ull) * 8, hipMemcpyDeviceToHost));
    c->pg_Eu = Eu;
    c->pg_HC = HC;
    c->pg_NT = NT;
    c->pg_flags = flags;
    c->pg_next = 0;
    c->pg_pages = 0;
    c->pg_unary_done = false;
    c->paged = true;
    HIP_TRY(c, hipEventRecord(c->ev[5], st));
    HIP_TRY(c, hipStreamSynchronize(st));
    HIP_TRY(c, hipEventElapsedTime(&c->stage_ms[2], c->ev[4], c->ev[5]));
    settle_timings(c);
    tcollect(c, RDF_T_PIVOT, RDF_NUM_TIMERS);
    rdf_cind_stats& cs = c->cstats;
    memset(&cs, 0, sizeof(cs));
    cs.n_light_chunks = WL;
    cs.n_heavy_chunks = WH;
    cs.n_class_members = c->n_class_members;
    cs.n_classes = c->n_classes;
    cs.n_class_cinds = HC;
    cs.n_light_candidates = c->light_candidates;
    cs.n_light_entries = c->light_entries;
    cs.n_heavy_candidates = c->heavy_candidates;
    if (stats) *stats = cs;
    c->stage = 3;  // no current result until rdf_next_page
    return RDF_OK;
}

rdf_status rdf_next_page(rdf_ctx* c, uint32_t* done, uint64_t* first_dep, uint64_t* end_dep) {
    if (!c || !done) return RDF_ERR_ARG;
    if (!c->paged || c->stage < 3) return fail(c, RDF_ERR_STATE, "rdf_discover_cinds_paged must be called first");
    HIP_TRY(c, hipSetDevice(c->device));
    CindView v = make_view(c, c->pg_flags);
    v.eoff = c->eoff.as<u64>();
    v.epairs = c->epairs.as<u64>();
    v.ebin = c->ebin.as<u64>();
    u32 d0 = 0, d1 = 0;
    *done = 0;
    if (!c->pg_unary_done) {  // the unary dependents (their pairs resident), in ranges; the first holds the class part
        d0 = c->pg_next;
        d1 = unary_page_end(c, d0);
        const bool first = d0 == 0;
        TRY(d_page_emit(c, v, d0, d1, c->h_eoffu[d0], c->h_eoffu[d1], c->h_choffh[d0], c->h_choffh[d1],
                        first ? c->pg_HC : 0, first ? c->pg_NT : 0));
        c->pg_unary_done = d1 >= c->Cu;
        c->pg_next = d1;
    } else if (c->pg_next < c->C) {  // a range of binary dependents on top of the resident unary pairs
        d0 = c->pg_next;
        d1 = page_end(c, d0, c->C);
        LightRange r;
        TRY(light_range(c, d0, d1, c->pg_WM > 0, &r));
        u64 Eb = 0;
        TRY(d_light_run(c, v, c->pivot.as<u32>(), r, c->pg_Eu, &Eb));
        c->n_explicit_raw += Eb;
        TRY(d_explicit_index(c, v, c->pg_Eu + Eb, true));
        TRY(d_page_emit(c, v, d0, d1, c->pg_Eu, c->pg_Eu + Eb, c->h_choffh[d0], c->h_choffh[d1], 0, 0));
        c->pg_next = d1;
    } else {
        *done = 1;
        c->n_out = c->n_class_out = c->n_runs = c->n_runs_explicit = c->n_lists = c->n_list_refs = 0;
        c->res_bits = c->heavy_pending = false;
        c->class_pending = false;
        HIP_TRY(c, c->runoff.ensure(8));
        HIP_TRY(c, hipMemsetAsync(c->runoff.p, 0, 8, c->stream));
        HIP_TRY(c, hipStreamSynchronize(c->stream));
        c->stage = 4;
        return RDF_OK;
    }
    ++c->pg_pages;
    tcollect(c, RDF_T_PIVOT, RDF_NUM_TIMERS, true);  // kernel-family times add up over the pages
    c->cstats.n_explicit_raw = c->n_explicit_raw;
    if (first_dep) *first_dep = d0;
    if (end_dep) *end_dep = d1;
    return RDF_OK;
}

rdf_status rdf_run(rdf_ctx* c, uint32_t min_support, const char* projection, uint32_t flags, rdf_fc_stats* fc,
                   rdf_group_stats* gs, rdf_cind_stats* cs) {
    rdf_status r = rdf_frequent_conditions(c, min_support, fc);
    if (r) return r;
    if (flags & RDF_USE_ASSOCIATION_RULES) {
        r = rdf_association_rules(c, nullptr);
        if (r) return r;
    }
    r = rdf_build_capture_groups(c, projection, nullptr);  // its stats are read after the discovery (no extra wait)
    if (r) return r;
    r = rdf_discover_cinds(c, flags, cs);
    if (r) return r;
    TRY(settle_group_stats(c));
    if (gs) *gs = c->gstats;
    return RDF_OK;
}

// ------------------------------------------------------------------------------------------------
// Sharded mode: a state machine that stops at every collective; the caller performs it
// (torch.distributed over RCCL, rdfind_amd/distributed.py) and hands the result back.

static rdf_status x_request(rdf_ctx* c, rdf_exchange* req, int op, const void* src, u64 count, int next_phase) {
    memset(req, 0, sizeof(*req));
    req->op = op;
    req->elem_bytes = op == RDF_X_ALLREDUCE_SUM_U32 ? 4 : 8;
    req->count = count;
    c->x_op = op;
    c->x_src = src;
    c->x_count = count;
    c->x_bytes = req->elem_bytes;
    c->x_imported = false;
    c->sh_phase = next_phase;
    return RDF_OK;
}

// ---- sharded input: condition counts as partial sums, then triples routed to their join owners ----

// this rank's input slice: the resident triples (RDF_SHARD_LOCAL_SLICE), or its row range of replicated triples
static void sh_slice(rdf_ctx* c, const u32** s, const u32** p, const u32** o, u64* n) {
    u64 b = 0, e = c->n;
    if (!(c->sh_flags & RDF_SHARD_LOCAL_SLICE)) {
        b = c->n * c->sh_rank / c->sh_nranks;
        e = c->n * (c->sh_rank + 1) / c->sh_nranks;
    }
    *s = c->s + b;
    *p = c->p + b;
    *o = c->o + b;
    *n = e - b;
}

// local dense unary counts -> nonzero (key, count) words to the keys' owners (all-to-all)
static rdf_status sh_phase10(rdf_ctx* c, rdf_exchange* req) {
    hipStream_t st = c->stream;
    TRY(fc_begin(c, c->sh_ms));
    TRY(fc_unary_alloc(c));
    const u32 V = c->V ? c->V : 1;
    const u64 K = 3ull * V;
    const u32 *s, *p, *o;
    u64 n;
    sh_slice(c, &s, &p, &o, &n);
    const int ubits = fc_ubits(K);
    const u64 NB = (K + (1ull << ubits) - 1) >> ubits;
    tbegin(c, RDF_T_UNARY);
    if (n && NB <= U2_MAXB && !c->force_global_counts) {
        TRY(fc_unary_part(c, s, p, o, n, ubits, NB, true));
    } else {
        HIP_TRY(c, hipMemsetAsync(c->cntg.p, 0, K * 4, st));
        if (n)
            hipLaunchKernelGGL(k_unary_count, dim3(std::min<unsigned>(grid_for(n, RDF_BLOCK * 4), 1024)), dim3(RDF_BLOCK), 0,
                               st, s, p, o, n, V, c->cntg.as<u32>());
    }
    const u32 R = c->sh_nranks;
    const unsigned G = (unsigned)std::max<u64>(1, std::min<u64>(1024, (K + 65535) / 65536));
    ENSURE(c, uhist, ((u64)R * G + 1) * 4);
    ENSURE(c, xsend, std::max<u64>(std::min<u64>(K, 3 * n), 1) * 8);
    hipLaunchKernelGGL((k_unary_route<false>), dim3(G), dim3(RDF_BLOCK), 0, st, c->cntg.as<u32>(), K, R, c->uhist.as<u32>(),
                       (u64*)nullptr);
    HIP_TRY(c, exclusive_scan_u32(c->ws, c->uhist.as<u32>(), c->uhist.as<u32>(), (u64)R * G, c->uhist.as<u32>() + (u64)R * G, st));
    hipLaunchKernelGGL((k_unary_route<true>), dim3(G), dim3(RDF_BLOCK), 0, st, c->cntg.as<u32>(), K, R, c->uhist.as<u32>(),
                       c->xsend.as<u64>());
    tend(c, RDF_T_UNARY);
    std::vector<u32> h((u64)R * G + 1);
    HIP_TRY(c, hipMemcpyAsync(h.data(), c->uhist.p, h.size() * 4, hipMemcpyDeviceToHost, st));
    HIP_TRY(c, hipStreamSynchronize(st));
    TRY(x_request(c, req, RDF_X_ALLTOALLV_U64, c->xsend.p, h[(u64)R * G], 16));
    for (u32 r = 0; r < R; ++r) req->send_counts[r] = h[(u64)(r + 1) * G] - h[(u64)r * G];
    return RDF_OK;
}

// received unary partials of this rank's keys -> summed -> frequent keys -> all-gather
// hot join values (sharded): a value is hot with >= 1 / HOT_DIV of a rank's expected occurrences (so at most
// HOT_DIV * N of them); an owner submits at most HOT_CAP candidate keys
static constexpr u64 HOT_DIV = 4096;
static constexpr u64 HOT_CAP = 32768;

static rdf_status sh_phase16(rdf_ctx* c, rdf_exchange* req) {
    hipStream_t st = c->stream;
    tbegin(c, RDF_T_UNARY);
    u64 Bu = 0, nk = 0;
    const u64 m = c->x_recv_count;
    TRY(fc_sum_pairs(c, c->xrecv.as<u64>(), nullptr, m, &Bu, &nk, true, &c->ukeys));
    tend(c, RDF_T_UNARY);
    c->sh_Bu = Bu;
    c->hot_n = 0;
    c->hot_mask = 0;
    // (hot balancing packs a key as key << 32 | count with 0xffffffff as the slice-size marker: dictionaries whose 3V
    // keys reach it keep the hash owners)
    if (!c->hot_balance || c->sh_nranks <= 1 || 3ull * (c->V ? c->V : 1) >= 0xffffffffull) {
        HIP_TRY(c, hipStreamSynchronize(st));
        return x_request(c, req, RDF_X_ALLGATHERV_U64, c->ukeys.p, Bu, 11);
    }
    // hot join value candidates: this owner's summed keys of projected positions with >= |proj| n_local / HOT_DIV
    // occurrences (a rank's share of the load is ~|proj| n_local), then all-gathered with every rank's slice size
    // (phase 18 builds the same owner table on every rank from the same gathered words)
    const u32 *s, *p, *o;
    u64 n;
    sh_slice(c, &s, &p, &o, &n);
    const int np = __builtin_popcount((unsigned)c->sh_proj & 7u);
    const u64 thr = std::max<u64>(1, (u64)np * n / (3 * HOT_DIV));  // a hot value may spread over 3 positions
    const u64 tcap = next_pow2(std::max<u64>(1024, 2 * m));  // fc_sum_pairs' table (lkeys / lvals)
    ENSURE(c, hotc, (HOT_CAP + 2) * 8);
    HIP_TRY(c, hipMemsetAsync(c->hotc.as<u64>() + HOT_CAP + 1, 0, 8, st));
    hipLaunchKernelGGL(k_hot_candidates, dim3(grid_for(tcap, RDF_BLOCK, kGrid)), dim3(RDF_BLOCK), 0, st, c->lkeys.as<u64>(),
                       c->lvals.as<u32>(), tcap, c->V ? c->V : 1u, c->sh_proj, (u32)std::min<u64>(thr, 0xffffffffu),
                       (u32)HOT_CAP, c->hotc.as<u64>() + 1, (u32*)(c->hotc.as<u64>() + HOT_CAP + 1));
    HIP_TRY(c, hipGetLastError());
    u32 k = 0;
    TRY(read_u32(c, c->hotc.as<u64>() + HOT_CAP + 1, &k));
    if (k > HOT_CAP) {
        // more candidates than the cap (an owner whose slice is small against the summed counts it owns): all of them
        // again, and the HOT_CAP largest by (count desc, key asc), so the submitted set does not depend on the order of
        // the device's atomics and keeps the hottest values
        const u64 kk = k;
        ENSURE(c, hotc, (kk + 2) * 8);
        HIP_TRY(c, hipMemsetAsync(c->hotc.as<u64>() + kk + 1, 0, 8, st));
        hipLaunchKernelGGL(k_hot_candidates, dim3(grid_for(tcap, RDF_BLOCK, kGrid)), dim3(RDF_BLOCK), 0, st,
                           c->lkeys.as<u64>(), c->lvals.as<u32>(), tcap, c->V ? c->V : 1u, c->sh_proj,
                           (u32)std::min<u64>(thr, 0xffffffffu), (u32)kk, c->hotc.as<u64>() + 1,
                           (u32*)(c->hotc.as<u64>() + kk + 1));
        HIP_TRY(c, hipGetLastError());
        std::vector<u64> cand(kk);
        HIP_TRY(c, ctx_copy(c, cand.data(), c->hotc.as<u64>() + 1, kk * 8, hipMemcpyDeviceToHost));
        std::partial_sort(cand.begin(), cand.begin() + HOT_CAP, cand.end(), [](u64 a, u64 b) {
            return (u32)a != (u32)b ? (u32)a > (u32)b : (a >> 32) < (b >> 32);
        });
        HIP_TRY(c, ctx_copy(c, c->hotc.as<u64>() + 1, cand.data(), HOT_CAP * 8, hipMemcpyHostToDevice));
    }
    k = std::min<u32>(k, HOT_CAP);
    c->hscal[14] = (0xffffffffull << 32) | n;  // marker word: this rank's slice size
    HIP_TRY(c, ctx_copy(c, c->hotc.p, c->hscal + 14, 8, hipMemcpyHostToDevice));
    return x_request(c, req, RDF_X_ALLGATHERV_U64, c->hotc.p, 1ull + k, 18);
}

// every rank's hot candidates -> the hot join values' owners, identical on every rank: occurrences per value summed over
// its positions, values with >= |proj| n_total / (N HOT_DIV) occurrences assigned largest first to the least loaded
// rank (each rank starting from its expected share of the hashed rest; ties to the lower rank) -> c->hot; then the
// frequent unary keys are all-gathered as before (phase 11)
static rdf_status sh_phase18(rdf_ctx* c, rdf_exchange* req) {
    const u64 cnt = c->x_recv_count;
    const u32 V = c->V ? c->V : 1;
    const u32 R = c->sh_nranks;
    std::vector<u64> w(cnt);
    if (cnt) HIP_TRY(c, ctx_copy(c, w.data(), c->xrecv.p, cnt * 8, hipMemcpyDeviceToHost));
    u64 n_total = 0;
    std::unordered_map<u32, u64> occ;
    for (u64 x : w) {
        const u64 key = x >> 32;
        if (key == 0xffffffffull) {
            n_total += (u32)x;
            continue;
        }
        occ[(u32)(key % V)] += (u32)x;
    }
    const int np = __builtin_popcount((unsigned)c->sh_proj & 7u);
    const double total = (double)np * (double)n_total;
    const u64 thr = std::max<u64>(1, (u64)(total / ((double)R * HOT_DIV)));
    std::vector<std::pair<u64, u32>> hot;  // (occurrences, value)
    for (const auto& kv : occ)
        if (kv.second >= thr) hot.push_back({kv.second, kv.first});
    std::sort(hot.begin(), hot.end(), [](const std::pair<u64, u32>& a, const std::pair<u64, u32>& b) {
        return a.first != b.first ? a.first > b.first : a.second < b.second;
    });
    c->hot_n = hot.size();
    if (!hot.empty()) {
        double hot_total = 0;
        for (const auto& h : hot) hot_total += (double)h.first;
        std::vector<double> load(R, std::max(0.0, total - hot_total) / R);
        const u64 slots = next_pow2(std::max<u64>(64, 2 * hot.size()));
        std::vector<u64> table(slots, EMPTY64);
        for (const auto& h : hot) {
            u32 r = 0;
            for (u32 q = 1; q < R; ++q)
                if (load[q] < load[r]) r = q;
            load[r] += (double)h.first;
            u32 slot = hot_slot(h.second, (u32)(slots - 1));
            while (table[slot] != EMPTY64) slot = (slot + 1) & (u32)(slots - 1);
            table[slot] = ((u64)h.second << 32) | r;
        }
        ENSURE(c, hot, slots * 8);
        HIP_TRY(c, ctx_copy(c, c->hot.p, table.data(), slots * 8, hipMemcpyHostToDevice));
        c->hot_mask = (u32)(slots - 1);
    }
    return x_request(c, req, RDF_X_ALLGATHERV_U64, c->ukeys.p, c->sh_Bu, 11);
}

// every owner's frequent unary keys -> global ranks; local binary (key, count) partials -> all-to-all to the keys' owners
static rdf_status sh_phase11(rdf_ctx* c, rdf_exchange* req) {
    hipStream_t st = c->stream;
    const u32 V = c->V ? c->V : 1;
    const u64 K = 3ull * V, NR = (K + FR_R - 1) / FR_R;
    const u64 U = c->x_recv_count;
    tbegin(c, RDF_T_UNARY);
    ENSURE(c, ukeys, std::max<u64>(U, 1) * 8);
    ENSURE(c, ukeys_tmp, std::max<u64>(U, 1) * 8);
    if (U) HIP_TRY(c, hipMemcpyAsync(c->ukeys.p, c->xrecv.p, U * 8, hipMemcpyDeviceToDevice, st));
    {
        u64* k = c->ukeys.as<u64>();
        u64* t = c->ukeys_tmp.as<u64>();
        HIP_TRY(c, radix_sort_u64(c->ws, k, t, U, bits_for(K - 1), st));
        if (k != c->ukeys.as<u64>()) std::swap(c->ukeys, c->ukeys_tmp);
    }
    HIP_TRY(c, hipMemsetAsync(c->frank.p, 0xff, K * 4, st));
    HIP_TRY(c, hipMemsetAsync(c->fbits.p, 0, ((K + 63) / 64 + 1) * 8, st));
    HIP_TRY(c, hipMemsetAsync(c->boff.p, 0, (NR + 2) * 4, st));  // frank holds global ranks
    ENSURE(c, fval, std::max<u64>(U, 1) * 4);
    if (U)
        hipLaunchKernelGGL(k_ranks_from_keys, dim3(grid_for(U, RDF_BLOCK, kGrid)), dim3(RDF_BLOCK), 0, st, c->ukeys.as<u64>(), U,
                           V, c->frank.as<u32>(), c->fval.as<u32>(), c->fbits.as<u64>());
    hipLaunchKernelGGL(k_lower_bound1, dim3(1), dim3(1), 0, st, c->ukeys.as<u64>(), U, (u64)V, dscal(c, 5));
    hipLaunchKernelGGL(k_lower_bound1, dim3(1), dim3(1), 0, st, c->ukeys.as<u64>(), U, 2ull * V, dscal(c, 6));
    u64 lb[2];
    TRY(read_multi(c, {{dscal(c, 5), 8}, {dscal(c, 6), 8}}, lb));
    tend(c, RDF_T_UNARY);
    c->U = (u32)U;
    c->sh_nfreq[0] = lb[0];
    c->sh_nfreq[1] = lb[1] - lb[0];
    c->sh_nfreq[2] = U - lb[1];
    const u32 *s, *p, *o;
    u64 n;
    sh_slice(c, &s, &p, &o, &n);
    tbegin(c, RDF_T_BINARY);
    u64 B = 0, nkeys = 0, S = 0;
    if (n) TRY(fc_binary_part(c, s, p, o, n, true, &B, &nkeys, &S));
    const u32 R = c->sh_nranks;
    const unsigned G = (unsigned)std::max<u64>(1, std::min<u64>(1024, (S + 4095) / 4096));
    ENSURE(c, uhist, ((u64)R * G + 1) * 4);
    ENSURE(c, xsend, std::max<u64>(2 * S, 1) * 8);
    hipLaunchKernelGGL((k_route_pairs<false>), dim3(G), dim3(RDF_BLOCK), 0, st, c->tkeys.as<u64>(), (const u32*)c->pos.p, S,
                       R, c->uhist.as<u32>(), (u64*)nullptr);
    HIP_TRY(c, exclusive_scan_u32(c->ws, c->uhist.as<u32>(), c->uhist.as<u32>(), (u64)R * G, c->uhist.as<u32>() + (u64)R * G, st));
    hipLaunchKernelGGL((k_route_pairs<true>), dim3(G), dim3(RDF_BLOCK), 0, st, c->tkeys.as<u64>(), (const u32*)c->pos.p, S,
                       R, c->uhist.as<u32>(), c->xsend.as<u64>());
    tend(c, RDF_T_BINARY);
    std::vector<u32> h((u64)R * G + 1);
    HIP_TRY(c, hipMemcpyAsync(h.data(), c->uhist.p, h.size() * 4, hipMemcpyDeviceToHost, st));
    HIP_TRY(c, hipStreamSynchronize(st));
    TRY(x_request(c, req, RDF_X_ALLTOALLV_U64, c->xsend.p, 2 * S, 12));
    for (u32 r = 0; r < R; ++r) req->send_counts[r] = 2ull * (h[(u64)(r + 1) * G] - h[(u64)r * G]);
    return RDF_OK;
}

// received partials of this rank's keys -> summed -> frequent keys -> all-gather
static rdf_status sh_phase12(rdf_ctx* c, rdf_exchange* req) {
    tbegin(c, RDF_T_BINARY);
    u64 B = 0, nkeys = 0;
    ENSURE(c, bkeys, 8);
    TRY(fc_sum_pairs(c, c->xrecv.as<u64>(), nullptr, c->x_recv_count / 2, &B, &nkeys));
    tend(c, RDF_T_BINARY);
    c->sh_nkeys = nkeys;
    HIP_TRY(c, hipStreamSynchronize(c->stream));
    return x_request(c, req, RDF_X_ALLGATHERV_U64, c->bkeys.p, B, 13);
}

// the local triples -> the ranks owning their join values (all-to-all, then phase 14)
static rdf_status sh_route_triples(rdf_ctx* c, rdf_exchange* req) {
    hipStream_t st = c->stream;
    const u32 *s, *p, *o;
    u64 n;
    sh_slice(c, &s, &p, &o, &n);
    const u32 R = c->sh_nranks;
    const unsigned G = (unsigned)std::max<u64>(1, std::min<u64>(1024, (n + 4095) / 4096));
    ENSURE(c, uhist, ((u64)R * G + 1) * 4);
    ENSURE(c, xsend, std::max<u64>(6 * n, 1) * 8);  // <= 3 copies of 2 words
    tbegin(c, RDF_T_EMIT);
    const u64* hot = c->hot_n ? c->hot.as<u64>() : nullptr;
    hipLaunchKernelGGL((k_route_triples<false>), dim3(G), dim3(RDF_BLOCK), 0, st, s, p, o, n, c->sh_proj, R, hot, c->hot_mask,
                       c->uhist.as<u32>(), (u64*)nullptr);
    HIP_TRY(c, exclusive_scan_u32(c->ws, c->uhist.as<u32>(), c->uhist.as<u32>(), (u64)R * G, c->uhist.as<u32>() + (u64)R * G, st));
    hipLaunchKernelGGL((k_route_triples<true>), dim3(G), dim3(RDF_BLOCK), 0, st, s, p, o, n, c->sh_proj, R, hot, c->hot_mask,
                       c->uhist.as<u32>(), c->xsend.as<u64>());
    tend(c, RDF_T_EMIT);
    std::vector<u32> h((u64)R * G + 1);
    HIP_TRY(c, hipMemcpyAsync(h.data(), c->uhist.p, h.size() * 4, hipMemcpyDeviceToHost, st));
    HIP_TRY(c, hipStreamSynchronize(st));
    const u64 copies = h[(u64)R * G];
    TRY(x_request(c, req, RDF_X_ALLTOALLV_U64, c->xsend.p, 2 * copies, 14));
    for (u32 r = 0; r < R; ++r) req->send_counts[r] = 2ull * (h[(u64)(r + 1) * G] - h[(u64)r * G]);
    return RDF_OK;
}

// every rank's frequent keys -> sorted binary ids; then (--use-ars) the slice's triple counts of the frequent
// conditions -> all-reduce (phase 17), or the triples -> their join owners
static rdf_status sh_phase13(rdf_ctx* c, rdf_exchange* req) {
    hipStream_t st = c->stream;
    const u64 B = c->x_recv_count;
    tbegin(c, RDF_T_BINARY);
    ENSURE(c, bkeys, std::max<u64>(B, 1) * 8);
    if (B) HIP_TRY(c, hipMemcpyAsync(c->bkeys.p, c->xrecv.p, B * 8, hipMemcpyDeviceToDevice, st));
    TRY(fc_binary_index(c, B));
    tend(c, RDF_T_BINARY);
    TRY(fc_end(c));
    fc_stats(c, c->sh_nfreq, c->sh_nkeys, B);  // n_binary_keys: the distinct keys owned by this rank
    if (!(c->sh_flags & RDF_USE_ASSOCIATION_RULES)) return sh_route_triples(c, req);
    const u32 *s, *p, *o;
    u64 n;
    sh_slice(c, &s, &p, &o, &n);
    TRY(ar_counts(c, s, p, o, n));  // FrequentConditionPlanner.findAssociationRules on the combined counts
    HIP_TRY(c, hipStreamSynchronize(st));
    return x_request(c, req, RDF_X_ALLREDUCE_SUM_U32, c->arcnt.p, (u64)c->U + c->B, 17);
}

// --use-ars: the summed counts -> the rules (identical on every rank) and the kept binary keys; then the triples
static rdf_status sh_phase17(rdf_ctx* c, rdf_exchange* req) {
    const u64 m = (u64)c->U + c->B;
    if (m) HIP_TRY(c, hipMemcpyAsync(c->arcnt.p, c->xrecv.p, m * 4, hipMemcpyDeviceToDevice, c->stream));
    TRY(ar_apply(c));
    return sh_route_triples(c, req);
}

// the triples this rank received for its join shard (wts/wtp/wto, sh_m of them) stand in for the resident input while
// in scope; the resident slice is restored on every exit path (it is the input of the next run)
struct ReceivedTriples {
    rdf_ctx* c;
    const u32 *s0, *p0, *o0;
    u64 n0;
    explicit ReceivedTriples(rdf_ctx* ctx) : c(ctx), s0(ctx->s), p0(ctx->p), o0(ctx->o), n0(ctx->n) {
        c->s = c->wts.as<u32>();
        c->p = c->wtp.as<u32>();
        c->o = c->wto.as<u32>();
        c->n = c->sh_m;
    }
    ~ReceivedTriples() {
        c->s = s0;
        c->p = p0;
        c->o = o0;
        c->n = n0;
    }
};

// received triples (every triple with a join value owned here) -> join partners of this rank's shard, sort,
// local supports -> all-reduce(sum) (then phases 1-8)
static rdf_status sh_phase14(rdf_ctx* c, rdf_exchange* req) {
    hipStream_t st = c->stream;
    const u64 m = c->x_recv_count / 2;
    ENSURE(c, wts, std::max<u64>(m, 1) * 4);
    ENSURE(c, wtp, std::max<u64>(m, 1) * 4);
    ENSURE(c, wto, std::max<u64>(m, 1) * 4);
    if (m)
        hipLaunchKernelGGL(k_unpack_triples, dim3(grid_for(m, RDF_BLOCK, kGrid)), dim3(RDF_BLOCK), 0, st, c->xrecv.as<u64>(), m,
                           c->wts.as<u32>(), c->wtp.as<u32>(), c->wto.as<u32>());
    // the routing's exchange buffers (16 B per received copy, 48 B per slice triple: ~45 GB per rank for c4 at 10^9
    // triples over 2 ranks) hold nothing the group build reads: spare until the build ends (phase 1), released only
    // if one of its allocations would fail (re-allocating them every step would cost more than keeping them)
    c->spare_x = true;
    c->rank = c->sh_rank;
    c->nranks = c->sh_nranks;
    c->sh_m = m;
    // a join shard whose K3 records exceed one sort's u32 offsets (>= 2^32/9 received triples, e.g. c4 at 10^9 triples
    // over 2 or 4 ranks) builds its groups in join ranges, as one GPU does: pass 1 here, pass 2 after the all-reduce
    c->sh_ranged = c->group_range_records || 9 * m >= (1ull << 32);
    c->n_group_ranges = 1;
    {
        ReceivedTriples rt(c);  // K3 reads the received triples; the resident input stays this rank's slice
        if (c->sh_ranged) {
            TRY(g_ranges_supports(c, c->sh_proj, c->group_range_records ? c->group_range_records : auto_range_records(c),
                                  shard_sel(c)));
            // this rank's supports, kept for pass 2 (the all-reduce brings the global ones)
            ENSURE(c, lsup, std::max<u64>(c->ncap, 1) * 4);
            HIP_TRY(c, hipMemcpyAsync(c->lsup.p, c->support.p, std::max<u64>(c->ncap, 1) * 4, hipMemcpyDeviceToDevice, st));
        } else {
            TRY(g_emit_sort_support(c, c->sh_proj));
        }
    }
    HIP_TRY(c, hipStreamSynchronize(st));
    return x_request(c, req, RDF_X_ALLREDUCE_SUM_U32, c->support.p, c->ncap, 1);
}

static rdf_status sh_phase1(rdf_ctx* c, rdf_exchange* req) {
    HIP_TRY(c, hipMemcpyAsync(c->support.p, c->xrecv.p, c->ncap * 4, hipMemcpyDeviceToDevice, c->stream));
    if (c->sh_ranged) {  // pass 2 of the join-range build, on the received triples again
        ReceivedTriples rt(c);
        TRY(g_ranges_groups(c, c->sh_proj, shard_sel(c), c->lsup.as<u32>()));
    } else {
        TRY(g_compact_groups(c));
    }
    c->spare_x = false;  // the exchange buffers carry the collectives again
    if (c->ar_on) TRY(g_ar_refs(c));
    TRY(g_size_hist(c, c->h_hist_local));
    ENSURE(c, xsend, 256 * 8);
    std::vector<u64> w(256);
    for (int i = 0; i < 256; ++i) w[i] = c->h_hist_local[i];
    HIP_TRY(c, ctx_copy(c, c->xsend.p, w.data(), 256 * 8, hipMemcpyHostToDevice));
    return x_request(c, req, RDF_X_ALLGATHERV_U64, c->xsend.p, 256, 2);
}

static rdf_status sh_phase2(rdf_ctx* c, rdf_exchange* req) {
    const u32 R = c->nranks;
    if (c->x_recv_count != 256ull * R) return fail(c, RDF_ERR_ARG, "histogram all-gather: wrong element count");
    std::vector<u64> all(256ull * R);
    HIP_TRY(c, ctx_copy(c, all.data(), c->xrecv.p, all.size() * 8, hipMemcpyDeviceToHost));
    u32 gh[256] = {};
    for (u32 r = 0; r < R; ++r)
        for (int b = 0; b < 256; ++b) gh[b] += (u32)all[256ull * r + b];
    const u64 thr = heavy_threshold(c, gh);
    u32 base = 0;
    for (u32 r = 0; r < c->rank; ++r) {
        u32 lh[256];
        for (int b = 0; b < 256; ++b) lh[b] = (u32)all[256ull * r + b];
        base += (u32)heavy_count(lh, thr);
    }
    TRY(g_heavy_binary(c, thr, base));
    TRY(g_finish(c, nullptr));
    c->gstats.n_heavy_groups = heavy_count(gh, thr);
    ENSURE(c, xsend, std::max<u64>(c->C, 1) * 8);
    if (c->C)
        hipLaunchKernelGGL(k_extract_hmask, dim3(grid_for(c->C, RDF_BLOCK, kGrid)), dim3(RDF_BLOCK), 0, c->stream,
                           c->info.as<CapInfo>(), c->C, c->xsend.as<u64>());
    HIP_TRY(c, hipStreamSynchronize(c->stream));
    return x_request(c, req, RDF_X_ALLREDUCE_SUM_U64, c->xsend.p, c->C, 3);  // heavy bits are disjoint: sum == or
}

static rdf_status sh_phase3(rdf_ctx* c, rdf_exchange* req) {
    if (c->C)
        hipLaunchKernelGGL(k_set_hmask, dim3(grid_for(c->C, RDF_BLOCK, kGrid)), dim3(RDF_BLOCK), 0, c->stream,
                           c->xrecv.as<u64>(), c->C, c->info.as<CapInfo>());
    CindView v = make_view(c, c->sh_flags);
    TRY(d_pivot_local(c, v));
    ENSURE(c, xsend, std::max<u64>(c->C, 1) * 8);
    if (c->C)
        hipLaunchKernelGGL(k_shard_best_keys, dim3(grid_for(c->C, RDF_BLOCK, kGrid)), dim3(RDF_BLOCK), 0, c->stream,
                           c->pbest.as<u64>(), c->info.as<CapInfo>(), c->C, c->rank, c->holder_qbits, c->xsend.as<u64>());
    HIP_TRY(c, hipStreamSynchronize(c->stream));
    return x_request(c, req, RDF_X_ALLREDUCE_MIN_U64, c->xsend.p, c->C, 4);
}

static rdf_status sh_phase4(rdf_ctx* c, rdf_exchange* req) {
    ENSURE(c, gbest, std::max<u64>(c->C, 1) * 8);
    HIP_TRY(c, hipMemcpyAsync(c->gbest.p, c->xrecv.p, (u64)c->C * 8, hipMemcpyDeviceToDevice, c->stream));
    ENSURE(c, xsend, std::max<u64>(2ull * c->C, 1) * 8);
    if (c->C)
        hipLaunchKernelGGL(k_shard_light_words, dim3(grid_for(c->C, RDF_BLOCK, kGrid)), dim3(RDF_BLOCK), 0, c->stream,
                           c->pnl.as<u32>(), c->C, c->rank, c->xsend.as<u64>());
    HIP_TRY(c, hipStreamSynchronize(c->stream));
    return x_request(c, req, RDF_X_ALLREDUCE_SUM_U64, c->xsend.p, 2ull * c->C, 5);
}

static rdf_status sh_phase5(rdf_ctx* c, rdf_exchange* req) {
    hipStream_t st = c->stream;
    const u32 C = c->C, R = c->nranks;
    CindView v = make_view(c, c->sh_flags);
    ENSURE(c, nrl, std::max<u64>(C, 1) * 4);
    tbegin(c, RDF_T_PIVOT);
    if (C) {
        const unsigned gp = grid_for(C, RDF_BLOCK, kGrid);
        ENSURE(c, ppart, 3ull * gp * 8);
        hipLaunchKernelGGL(k_pivot_final_shard, dim3(gp), dim3(RDF_BLOCK), 0, st, v,
                           c->pbest.as<u64>(), c->pnl.as<u32>(), c->gbest.as<u64>(), c->xrecv.as<u64>(), c->rank,
                           c->pivot.as<u32>(), c->nchl.as<u32>(), c->nitl.as<u32>(), c->npk.as<u32>(), c->nchh.as<u32>(),
                           c->nrl.as<u32>(),
                           c->info.as<CapInfo>(), c->ppart.as<u64>());
        hipLaunchKernelGGL(k_sum_partials3, dim3(1), dim3(RDF_BLOCK), 0, st, c->ppart.as<u64>(), gp, dscal(c, 2));
    }
    tend(c, RDF_T_PIVOT);
    u64 WL = 0, WH = 0, WI = 0, WP = 0, E = 0;
    TRY(d_chunks(c, &WL, &WH, &WI, &WP));
    c->sh_WH = WH;
    TRY(d_light(c, v, WI, WL, WP, &E, c->pivot.as<u32>()));
    c->n_explicit_raw = E;  // the holder's survivors until the owners have the verified pairs (sh_phase6)
    c->n_light_chunks = WL;
    // holder-first exchange: every survivor to d's owner (report) and to the other ranks holding light groups of d
    // (verify), grouped by destination
    const int cb = bits_for(C ? C - 1 : 0);
    if (33 + cb > 58) return fail(c, RDF_ERR_LIMIT, "sharded mode: too many captures for the routing key");
    ENSURE(c, lmask, std::max<u64>(C, 1) * 8);
    HIP_TRY(c, hipMemcpyAsync(c->lmask.p, c->xrecv.as<u64>() + C, (u64)C * 8, hipMemcpyDeviceToDevice, st));
    ENSURE(c, flags, std::max<u64>(E, 1) * 4);
    ENSURE(c, pos, (E + 1) * 8);
    tbegin(c, RDF_T_ESORT);
    if (E)
        hipLaunchKernelGGL((k_route_survivors<false>), dim3(grid_for(E, RDF_BLOCK, kGrid)), dim3(RDF_BLOCK), 0, st,
                           c->epairs.as<u64>(), E, c->lmask.as<u64>(), c->rank, R, cb, c->flags.as<u32>(), (const u64*)nullptr,
                           (u64*)nullptr);
    HIP_TRY(c, exclusive_scan_u32_u64(c->ws, c->flags.as<u32>(), c->pos.as<u64>(), E, c->pos.as<u64>() + E, st));
    u64 T = 0;
    TRY(read_u64(c, c->pos.as<u64>() + E, &T));
    ENSURE(c, cpairs, std::max<u64>(T, 1) * 8);
    ENSURE(c, cpairs_tmp, std::max<u64>(T, 1) * 8);
    if (E)
        hipLaunchKernelGGL((k_route_survivors<true>), dim3(grid_for(E, RDF_BLOCK, kGrid)), dim3(RDF_BLOCK), 0, st,
                           c->epairs.as<u64>(), E, c->lmask.as<u64>(), c->rank, R, cb, (u32*)nullptr, c->pos.as<u64>(),
                           c->cpairs.as<u64>());
    if (T) {
        u64* k = c->cpairs.as<u64>();
        u64* t = c->cpairs_tmp.as<u64>();
        HIP_TRY(c, radix_sort_u64_bits(c->ws, k, t, T, 58, 64, st));
        if (k != c->cpairs.as<u64>()) std::swap(c->cpairs, c->cpairs_tmp);
    }
    ENSURE(c, obounds, (RDF_MAX_RANKS + 1) * 8);
    hipLaunchKernelGGL(k_dest_bounds, dim3(1), dim3(RDF_BLOCK), 0, st, c->cpairs.as<u64>(), T, R, c->obounds.as<u64>());
    if (T)
        hipLaunchKernelGGL(k_clear_bits, dim3(grid_for(T, RDF_BLOCK, kGrid)), dim3(RDF_BLOCK), 0, st, c->cpairs.as<u64>(), T,
                           63ull << 58);
    tend(c, RDF_T_ESORT);
    std::vector<u64> bounds(R + 1);
    HIP_TRY(c, hipMemcpyAsync(bounds.data(), c->obounds.p, (R + 1) * 8, hipMemcpyDeviceToHost, st));
    HIP_TRY(c, hipStreamSynchronize(st));
    TRY(x_request(c, req, RDF_X_ALLTOALLV_U64, c->cpairs.p, T, 15));
    for (u32 r = 0; r < R; ++r) req->send_counts[r] = bounds[r + 1] - bounds[r];
    return RDF_OK;
}

// (dep << 32 | ref) pairs epairs[0, E) -> grouped by owner rank (dep_owner) for an all-to-all to next_phase
static rdf_status sh_to_owners(rdf_ctx* c, rdf_exchange* req, u64 E, int next_phase) {
    hipStream_t st = c->stream;
    const u32 C = c->C, R = c->nranks;
    const int cb = bits_for(C ? C - 1 : 0);
    const int ob = bits_for(R);
    if (2 * cb + ob > 64) return fail(c, RDF_ERR_LIMIT, "sharded mode: too many captures for the owner sort key");
    ENSURE(c, epairs_tmp, std::max<u64>(E, 1) * 8);
    ENSURE(c, obounds, (RDF_MAX_RANKS + 1) * 8);
    tbegin(c, RDF_T_ESORT);
    if (E) {
        hipLaunchKernelGGL(k_owner_pack, dim3(grid_for(E, RDF_BLOCK, kGrid)), dim3(RDF_BLOCK), 0, st, c->epairs.as<u64>(), E, R, cb);
        u64* k = c->epairs.as<u64>();
        u64* t = c->epairs_tmp.as<u64>();
        HIP_TRY(c, radix_sort_u64(c->ws, k, t, E, 2 * cb + ob, st));
        if (k != c->epairs.as<u64>()) std::swap(c->epairs, c->epairs_tmp);
    }
    hipLaunchKernelGGL(k_owner_bounds, dim3(1), dim3(RDF_BLOCK), 0, st, c->epairs.as<u64>(), E, cb, R, c->obounds.as<u64>());
    if (E) hipLaunchKernelGGL(k_owner_strip, dim3(grid_for(E, RDF_BLOCK, kGrid)), dim3(RDF_BLOCK), 0, st, c->epairs.as<u64>(), E, cb);
    tend(c, RDF_T_ESORT);
    std::vector<u64> bounds(R + 1);
    HIP_TRY(c, hipMemcpyAsync(bounds.data(), c->obounds.p, (R + 1) * 8, hipMemcpyDeviceToHost, st));
    HIP_TRY(c, hipStreamSynchronize(st));
    TRY(x_request(c, req, RDF_X_ALLTOALLV_U64, c->epairs.p, E, next_phase));
    for (u32 r = 0; r < R; ++r) req->send_counts[r] = bounds[r + 1] - bounds[r];
    return RDF_OK;
}

// received holder words: reports for the dependents this rank owns (kept for phase 6) and verify pairs, checked
// against this rank's light groups of the dependent (the light kernels with the given candidates and no pivot);
// the survivors go to the owners as this rank's reports
static rdf_status sh_phase15(rdf_ctx* c, rdf_exchange* req) {
    hipStream_t st = c->stream;
    const u64 n = c->x_recv_count;
    const u32 C = c->C;
    const int cb = bits_for(C ? C - 1 : 0);
    ENSURE(c, cpairs, std::max<u64>(n, 1) * 8);
    ENSURE(c, cpairs_tmp, std::max<u64>(n, 1) * 8);
    HIP_TRY(c, hipMemcpyAsync(c->cpairs.p, c->xrecv.p, n * 8, hipMemcpyDeviceToDevice, st));
    tbegin(c, RDF_T_ESORT);
    if (n) {
        u64* k = c->cpairs.as<u64>();
        u64* t = c->cpairs_tmp.as<u64>();
        HIP_TRY(c, radix_sort_u64(c->ws, k, t, n, 33 + cb, st));
        if (k != c->cpairs.as<u64>()) std::swap(c->cpairs, c->cpairs_tmp);
    }
    ENSURE(c, obounds, (RDF_MAX_RANKS + 1) * 8);
    // split point = first word with the verify tag: k_dest_bounds on the words shifted ... one lower bound
    hipLaunchKernelGGL(k_lower_bound1, dim3(1), dim3(1), 0, st, c->cpairs.as<u64>(), n, 1ull << (32 + cb),
                       c->obounds.as<u64>());
    u64 nh = 0;
    TRY(read_u64(c, c->obounds.as<u64>(), &nh));
    const u64 nv = n - nh;
    c->n_hrep = nh;
    ENSURE(c, hrep, std::max<u64>(nh, 1) * 8);
    ENSURE(c, vpairs, std::max<u64>(nv, 1) * 8);
    if (nh) HIP_TRY(c, hipMemcpyAsync(c->hrep.p, c->cpairs.p, nh * 8, hipMemcpyDeviceToDevice, st));
    if (nv) {
        HIP_TRY(c, hipMemcpyAsync(c->vpairs.p, c->cpairs.as<u64>() + nh, nv * 8, hipMemcpyDeviceToDevice, st));
        hipLaunchKernelGGL(k_clear_bits, dim3(grid_for(nv, RDF_BLOCK, kGrid)), dim3(RDF_BLOCK), 0, st, c->vpairs.as<u64>(), nv,
                           1ull << (32 + cb));
    }
    ENSURE(c, vcoff, (C + 1ull) * 8);
    ENSURE(c, ebin, std::max<u64>(C, 1) * 8);
    hipLaunchKernelGGL(k_pair_offsets, dim3(grid_for(C + 1ull, RDF_BLOCK, kGrid)), dim3(RDF_BLOCK), 0, st,
                       c->vpairs.as<u64>(), nv, C, c->Cu, c->vcoff.as<u64>(), c->ebin.as<u64>());
    tend(c, RDF_T_ESORT);
    CindView v = make_view(c, c->sh_flags);
    v.vcoff = c->vcoff.as<u64>();
    v.vpairs = c->vpairs.as<u64>();
    ENSURE(c, vpiv, std::max<u64>(C, 1) * 4);
    HIP_TRY(c, hipMemsetAsync(c->vpiv.p, 0xff, std::max<u64>(C, 1) * 4, st));  // no pivot group to skip
    tbegin(c, RDF_T_LIGHT);
    if (C)
        hipLaunchKernelGGL(k_verify_plan, dim3(grid_for(C, RDF_BLOCK, kGrid)), dim3(RDF_BLOCK), 0, st, v, c->pnl.as<u32>(),
                           c->nchl.as<u32>(), c->nitl.as<u32>(), c->npk.as<u32>());
    tend(c, RDF_T_LIGHT);
    const u64 hc = c->heavy_candidates, lc = c->light_candidates, le = c->light_entries;
    u64 WL = 0, WH = 0, WI = 0, WP = 0, E = 0;
    TRY(d_chunks(c, &WL, &WH, &WI, &WP));
    c->heavy_candidates = hc;
    c->light_candidates = lc;
    c->light_entries = le;
    TRY(d_light(c, v, WI, WL, WP, &E, c->vpiv.as<u32>()));
    c->n_light_chunks += WL;
    return sh_to_owners(c, req, E, 6);
}

static rdf_status sh_phase6(rdf_ctx* c, rdf_exchange* req) {
    hipStream_t st = c->stream;
    const u64 n6 = c->x_recv_count, nh = c->n_hrep, n = n6 + nh;  // verifiers' reports + the holders' reports
    const u32 C = c->C;
    ENSURE(c, epairs, std::max<u64>(n, 1) * 8);
    ENSURE(c, epairs_tmp, std::max<u64>(n, 1) * 8);
    if (n6) HIP_TRY(c, hipMemcpyAsync(c->epairs.p, c->xrecv.p, n6 * 8, hipMemcpyDeviceToDevice, st));
    if (nh) HIP_TRY(c, hipMemcpyAsync(c->epairs.as<u64>() + n6, c->hrep.p, nh * 8, hipMemcpyDeviceToDevice, st));
    tbegin(c, RDF_T_ESORT);
    {
        u64* k = c->epairs.as<u64>();
        u64* t = c->epairs_tmp.as<u64>();
        HIP_TRY(c, radix_sort_u64(c->ws, k, t, n, 32 + bits_for(C ? C - 1 : 0), st));
        if (k != c->epairs.as<u64>()) std::swap(c->epairs, c->epairs_tmp);
    }
    ENSURE(c, flags, std::max<u64>(n, 1) * 4);
    ENSURE(c, pos, (n + 1) * 8);
    if (n)
        hipLaunchKernelGGL(k_mult_flags, dim3(grid_for(n, RDF_BLOCK, kGrid)), dim3(RDF_BLOCK), 0, st, c->epairs.as<u64>(), n,
                           c->nrl.as<u32>(), c->flags.as<u32>());
    HIP_TRY(c, exclusive_scan_u32_u64(c->ws, c->flags.as<u32>(), c->pos.as<u64>(), n, c->pos.as<u64>() + n, st));
    u64 E = 0;
    TRY(read_u64(c, c->pos.as<u64>() + n, &E));
    c->n_explicit_raw = E;  // the verified raw pairs this rank owns (the ranks' sum is the single-GPU count)
    ENSURE(c, xsend, std::max<u64>(E, 1) * 8);
    if (n)
        hipLaunchKernelGGL(k_compact_u64, dim3(grid_for(n, RDF_BLOCK, kGrid)), dim3(RDF_BLOCK), 0, st, c->epairs.as<u64>(), n,
                           c->flags.as<u32>(), c->pos.as<u64>(), c->xsend.as<u64>());
    // The minimality rules probe other dependents only through the unary components of binary dependents
    // (R1 / R4, rule_keep -> member(comp, ref)), so only the unary dependents' pairs -- a prefix of the sorted final
    // pairs -- go to every rank; the binary dependents' pairs stay with their owner (this rank).
    ENSURE(c, obounds, (RDF_MAX_RANKS + 1) * 8);
    hipLaunchKernelGGL(k_lower_bound1, dim3(1), dim3(1), 0, st, c->xsend.as<u64>(), E, (u64)c->Cu << 32,
                       c->obounds.as<u64>());
    u64 Eu = 0;
    TRY(read_u64(c, c->obounds.as<u64>(), &Eu));
    c->sh_Eb = E - Eu;
    ENSURE(c, ebown, std::max<u64>(E - Eu, 1) * 8);
    if (E > Eu) HIP_TRY(c, hipMemcpyAsync(c->ebown.p, c->xsend.as<u64>() + Eu, (E - Eu) * 8, hipMemcpyDeviceToDevice, st));
    tend(c, RDF_T_ESORT);
    HIP_TRY(c, hipStreamSynchronize(st));
    return x_request(c, req, RDF_X_ALLGATHERV_U64, c->xsend.p, Eu, 7);
}

// Pairs of several (dep, ref)-sorted runs whose dependents are disjoint (each rank's unary pairs, this rank's binary
// pairs) -> one (dep, ref)-sorted array, by dependent segments (no sort): out[eoff[d] + i - head(d)] = in[i].
static rdf_status merge_dep_runs(rdf_ctx* c, const u64* in, u64 n, u64* out) {
    hipStream_t st = c->stream;
    const u32 C = c->C;
    ENSURE(c, segb, std::max<u64>(C, 1) * 8);
    ENSURE(c, sege, std::max<u64>(C, 1) * 8);
    ENSURE(c, seglen, std::max<u64>(C, 1) * 4);
    ENSURE(c, eoff, (C + 1ull) * 8);
    if (!C) return RDF_OK;
    HIP_TRY(c, hipMemsetAsync(c->segb.p, 0, (u64)C * 8, st));
    HIP_TRY(c, hipMemsetAsync(c->sege.p, 0, (u64)C * 8, st));
    if (n)
        hipLaunchKernelGGL(k_seg_bounds, dim3(grid_for(n, RDF_BLOCK, kGrid)), dim3(RDF_BLOCK), 0, st, in, n, c->segb.as<u64>(),
                           c->sege.as<u64>());
    hipLaunchKernelGGL(k_seg_lengths, dim3(grid_for(C, RDF_BLOCK, kGrid)), dim3(RDF_BLOCK), 0, st, c->segb.as<u64>(),
                       c->sege.as<u64>(), C, c->seglen.as<u32>());
    HIP_TRY(c, exclusive_scan_u32_u64(c->ws, c->seglen.as<u32>(), c->eoff.as<u64>(), C, c->eoff.as<u64>() + C, st));
    if (n)
        hipLaunchKernelGGL(k_seg_scatter, dim3(grid_for(n, RDF_BLOCK, kGrid)), dim3(RDF_BLOCK), 0, st, in, n, c->segb.as<u64>(),
                           c->eoff.as<u64>(), out);
    return RDF_OK;
}

static rdf_status sh_phase7(rdf_ctx* c, rdf_exchange* req) {
    hipStream_t st = c->stream;
    const u64 Eu = c->x_recv_count, Eb = c->sh_Eb;  // every rank's unary pairs + this rank's binary pairs
    const u64 E = Eu + Eb;
    ENSURE(c, epairs_tmp, std::max<u64>(E, 1) * 8);
    ENSURE(c, epairs, std::max<u64>(E, 1) * 8);
    if (Eu) HIP_TRY(c, hipMemcpyAsync(c->epairs_tmp.p, c->xrecv.p, Eu * 8, hipMemcpyDeviceToDevice, st));
    if (Eb) HIP_TRY(c, hipMemcpyAsync(c->epairs_tmp.as<u64>() + Eu, c->ebown.p, Eb * 8, hipMemcpyDeviceToDevice, st));
    c->sh_E = E;
    tbegin(c, RDF_T_ESORT);
    TRY(merge_dep_runs(c, c->epairs_tmp.as<u64>(), E, c->epairs.as<u64>()));
    tend(c, RDF_T_ESORT);
    CindView v = make_view(c, c->sh_flags);
    TRY(d_explicit_index(c, v, E, true));
    u64 H = 0;
    TRY(d_heavy_count(c, v, c->sh_WH, &H));
    c->sh_H = H;
    // classes: deterministic ids (sorted masks), owned members, lists of the classes pivoted here
    tbegin(c, RDF_T_CLASS);
    u64 nmem_all = 0, tcapc = 0;
    u32 ncls = 0;
    TRY(d_class_table(c, v, v.ar ? 0u : c->Cu, &nmem_all, &ncls, &tcapc));  // --use-ars: per-dependent heavy path
    c->sh_tcapc = tcapc;
    c->n_classes = ncls;
    ENSURE(c, smask, std::max<u64>(ncls, 1) * 8);
    ENSURE(c, smask_tmp, std::max<u64>(ncls, 1) * 8);
    ENSURE(c, pos, (tcapc + 1) * 8);
    HIP_TRY(c, exclusive_scan_u32_u64(c->ws, c->cflag.as<u32>(), c->pos.as<u64>(), tcapc, c->pos.as<u64>() + tcapc, st));
    hipLaunchKernelGGL(k_compact_u64, dim3(grid_for(tcapc, RDF_BLOCK, kGrid)), dim3(RDF_BLOCK), 0, st, c->ctab.as<u64>(), tcapc,
                       c->cflag.as<u32>(), c->pos.as<u64>(), c->smask.as<u64>());
    {
        u64* k = c->smask.as<u64>();
        u64* t = c->smask_tmp.as<u64>();
        HIP_TRY(c, radix_sort_u64(c->ws, k, t, ncls, 64, st));
        if (k != c->smask.as<u64>()) std::swap(c->smask, c->smask_tmp);
    }
    if (ncls)
        hipLaunchKernelGGL(k_class_rank, dim3(grid_for(ncls, RDF_BLOCK, kGrid)), dim3(RDF_BLOCK), 0, st, c->ctab.as<u64>(),
                           tcapc - 1, c->smask.as<u64>(), ncls, c->ccid.as<u32>());
    // owned members
    ENSURE(c, ckeys, std::max<u64>(nmem_all, 1) * 8);
    ENSURE(c, ckeys_tmp, std::max<u64>(nmem_all, 1) * 8);
    HIP_TRY(c, hipMemsetAsync(dscal(c, 4), 0, 8, st));
    if (c->Cu && ncls)  // (--use-ars: no classes, every heavy-only dependent takes the heavy path)
        hipLaunchKernelGGL(k_class_keys, dim3(grid_for(c->Cu, RDF_BLOCK, kGrid)), dim3(RDF_BLOCK), 0, st, v, c->ctab.as<u64>(),
                           c->ccid.as<u32>(), tcapc - 1, c->rank, c->nranks, c->ckeys.as<u64>(), dscal(c, 4));
    u64 nmem = 0;
    TRY(read_u64(c, dscal(c, 4), &nmem));
    {
        u64* k = c->ckeys.as<u64>();
        u64* t = c->ckeys_tmp.as<u64>();
        HIP_TRY(c, radix_sort_u64(c->ws, k, t, nmem, 32 + bits_for(ncls ? ncls - 1 : 0), st));
        if (k != c->ckeys.as<u64>()) std::swap(c->ckeys, c->ckeys_tmp);
    }
    c->n_class_members = nmem;
    ENSURE(c, coff, (ncls + 1ull) * 8);
    ENSURE(c, cmask, std::max<u64>(ncls, 1) * 8);
    ENSURE(c, cpiv, std::max<u64>(ncls, 1) * 4);
    ENSURE(c, cnch, std::max<u64>(ncls, 1) * 4);
    ENSURE(c, cchoff, (ncls + 1ull) * 8);
    hipLaunchKernelGGL(k_class_info_shard, dim3(grid_for(ncls + 1ull, RDF_BLOCK, kGrid)), dim3(RDF_BLOCK), 0, st,
                       c->ckeys.as<u64>(), nmem, ncls, c->smask.as<u64>(), c->coff.as<u64>(), c->cmask.as<u64>());
    HIP_TRY(c, hipMemsetAsync(c->cnch.p, 0, std::max<u64>(ncls, 1) * 4, st));
    if (c->Cu && ncls)
        hipLaunchKernelGGL(k_class_pivot_shard, dim3(grid_for(c->Cu, RDF_BLOCK, kGrid)), dim3(RDF_BLOCK), 0, st, v,
                           c->ctab.as<u64>(), tcapc - 1, c->ccid.as<u32>(), c->pivot.as<u32>(), c->gbest.as<u64>(), c->rank,
                           c->cpiv.as<u32>(), c->cnch.as<u32>());
    HIP_TRY(c, exclusive_scan_u32_u64(c->ws, c->cnch.as<u32>(), c->cchoff.as<u64>(), ncls, c->cchoff.as<u64>() + ncls, st));
    u64 WC = 0;
    TRY(read_u64(c, c->cchoff.as<u64>() + ncls, &WC));
    ENSURE(c, ccnt, std::max<u64>(WC, 1) * 4);
    ENSURE(c, cbits, std::max<u64>(WC, 1) * 8);
    ENSURE(c, cown, std::max<u64>(WC, 1) * 4);
    if (WC)
        hipLaunchKernelGGL(k_expand_owner, dim3(grid_for(std::max<u32>(ncls, 1), RDF_BLOCK, kGrid)), dim3(RDF_BLOCK), 0, st,
                           c->cchoff.as<u64>(), ncls, c->cown.as<u32>());
    ENSURE(c, lwoff, (WC + 1) * 8);
    if (WC) {
        const u64 nvb = wave_blocks(WC);
        const dim3 grid(vgrid(nvb));
        hipLaunchKernelGGL(k_class_eval, grid, dim3(RDF_BLOCK), 0, st, nvb, v, c->cchoff.as<u64>(), c->cown.as<u32>(), WC, c->cmask.as<u64>(),
                           c->cpiv.as<u32>(), c->cbits.as<u64>());
        if (v.mode == RULES_CLEAN)
            hipLaunchKernelGGL(k_class_mark, grid, dim3(RDF_BLOCK), 0, st, nvb, v, c->cchoff.as<u64>(), c->cown.as<u32>(), WC,
                               c->cmask.as<u64>(), c->cpiv.as<u32>(), c->cbits.as<u64>());
        hipLaunchKernelGGL(k_popc_counts, dim3(grid_for(WC, RDF_BLOCK, kGrid)), dim3(RDF_BLOCK), 0, st, c->cbits.as<u64>(),
                           WC, c->ccnt.as<u32>());
    }
    HIP_TRY(c, exclusive_scan_u32_u64(c->ws, c->ccnt.as<u32>(), c->lwoff.as<u64>(), WC, c->lwoff.as<u64>() + WC, st));
    u64 LT = 0;
    TRY(read_u64(c, c->lwoff.as<u64>() + WC, &LT));
    ENSURE(c, xsend, std::max<u64>(LT, 1) * 8);
    if (WC)
        hipLaunchKernelGGL(k_class_write, dim3(vgrid(wave_blocks(WC))),
                           dim3(RDF_BLOCK), 0, st, (u64)wave_blocks(WC), v, c->cchoff.as<u64>(), c->cown.as<u32>(), WC, c->cpiv.as<u32>(), c->cbits.as<u64>(),
                           c->lwoff.as<u64>(), (u32*)nullptr, c->xsend.as<u64>());
    tend(c, RDF_T_CLASS);
    HIP_TRY(c, hipStreamSynchronize(st));
    return x_request(c, req, RDF_X_ALLGATHERV_U64, c->xsend.p, LT, 8);
}

static rdf_status sh_phase8(rdf_ctx* c, rdf_exchange* req) {
    hipStream_t st = c->stream;
    const u64 n = c->x_recv_count;  // (class << 32 | ref) pairs of every class
    const u32 ncls = (u32)c->n_classes;
    ENSURE(c, cpairs, std::max<u64>(n, 1) * 8);
    ENSURE(c, cpairs_tmp, std::max<u64>(n, 1) * 8);
    HIP_TRY(c, hipMemcpyAsync(c->cpairs.p, c->xrecv.p, n * 8, hipMemcpyDeviceToDevice, st));
    tbegin(c, RDF_T_CLASS);
    {
        u64* k = c->cpairs.as<u64>();
        u64* t = c->cpairs_tmp.as<u64>();
        HIP_TRY(c, radix_sort_u64(c->ws, k, t, n, 32 + bits_for(ncls ? ncls - 1 : 0), st));
        if (k != c->cpairs.as<u64>()) std::swap(c->cpairs, c->cpairs_tmp);
    }
    ENSURE(c, clists, std::max<u64>(n, 1) * 4);
    ENSURE(c, lwoff, (ncls + 1ull) * 8);
    ENSURE(c, cchoff, (ncls + 1ull) * 8);
    hipLaunchKernelGGL(k_class_lists, dim3(grid_for(std::max<u64>(n, ncls + 1ull), RDF_BLOCK, kGrid)), dim3(RDF_BLOCK), 0, st,
                       c->cpairs.as<u64>(), n, ncls, c->clists.as<u32>(), c->lwoff.as<u64>(), c->cchoff.as<u64>());
    u64 HC = 0, NT = 0;
    TRY(d_class_tiles(c, c->n_class_members, ncls, &HC, &NT));
    tend(c, RDF_T_CLASS);
    CindView v = make_view(c, c->sh_flags);
    v.eoff = c->eoff.as<u64>();
    v.epairs = c->epairs.as<u64>();
    v.ebin = c->ebin.as<u64>();
    TRY(d_emit(c, v, c->sh_E, c->sh_WH, c->sh_H, HC, NT));
    memset(req, 0, sizeof(*req));
    req->op = RDF_X_DONE;
    c->sh_phase = 9;
    mem_report(c);
    return RDF_OK;
}

// ---- sharded ingest (SURVEY.md 8f row 1 at -dop N; FLK/persistence/MultiFileTextInputFormat.java:49-100 splits the
// input per task): every rank parses its own byte range into a local dictionary; each local term goes to the
// rank owning its hash, which deduplicates the terms it receives (byte-verified) and assigns global ids; the ids go
// back and the rank's triples are rewritten.  Global id = the owner's base (an exclusive scan of the owners' term
// counts) + the term's rank among the owner's distinct terms in arrival order: deterministic for any thread count.

// local terms -> owners: headers (hash, src << 58 | len << 32 | local id) to the owners (all-to-all)
static rdf_status sh_phase20(rdf_ctx* c, rdf_exchange* req) {
    hipStream_t st = c->stream;
    const u64 V = c->ing_Vl;
    const u32 R = c->sh_nranks;
    const unsigned char* text = (const unsigned char*)c->ntext.p;
    ENSURE(c, ithv, std::max<u64>(V, 1) * 8);
    ENSURE(c, ikeys, std::max<u64>(V, 1) * 8);
    ENSURE(c, ikeys_tmp, std::max<u64>(V, 1) * 8);
    ENSURE(c, iwords, std::max<u64>(V, 1) * 4);
    ENSURE(c, iwoff, (V + 1) * 8);
    ENSURE(c, ibnd, (RDF_MAX_RANKS + 1) * 8);
    ENSURE(c, iwb, (RDF_MAX_RANKS + 1) * 8);
    if (V)
        hipLaunchKernelGGL(k_term_route_keys, dim3(grid_for(V, RDF_BLOCK, kGrid)), dim3(RDF_BLOCK), 0, st, text,
                           c->nterm_off.as<u64>(), c->nterm_len.as<u32>(), V, R, c->ithv.as<u64>(), c->ikeys.as<u64>());
    {
        u64* k = c->ikeys.as<u64>();
        u64* t = c->ikeys_tmp.as<u64>();
        HIP_TRY(c, radix_sort_u64(c->ws, k, t, V, 32 + bits_for(R), st));
        if (k != c->ikeys.as<u64>()) std::swap(c->ikeys, c->ikeys_tmp);
    }
    if (V)
        hipLaunchKernelGGL(k_term_words, dim3(grid_for(V, RDF_BLOCK, kGrid)), dim3(RDF_BLOCK), 0, st, c->ikeys.as<u64>(), V,
                           c->nterm_len.as<u32>(), c->iwords.as<u32>());
    HIP_TRY(c, exclusive_scan_u32_u64(c->ws, c->iwords.as<u32>(), c->iwoff.as<u64>(), V, c->iwoff.as<u64>() + V, st));
    hipLaunchKernelGGL(k_owner_bounds, dim3(1), dim3(RDF_BLOCK), 0, st, c->ikeys.as<u64>(), V, 16, R, c->ibnd.as<u64>());
    hipLaunchKernelGGL(k_gather_u64_at, dim3(1), dim3(RDF_BLOCK), 0, st, c->iwoff.as<u64>(), c->ibnd.as<u64>(), R + 1,
                       c->iwb.as<u64>());
    std::vector<u64> bnd(R + 1), wb(R + 1);
    HIP_TRY(c, hipMemcpyAsync(bnd.data(), c->ibnd.p, (R + 1) * 8, hipMemcpyDeviceToHost, st));
    HIP_TRY(c, hipMemcpyAsync(wb.data(), c->iwb.p, (R + 1) * 8, hipMemcpyDeviceToHost, st));
    HIP_TRY(c, hipStreamSynchronize(st));
    const u64 W = wb[R];
    ENSURE(c, ihdr, std::max<u64>(2 * V, 1) * 8);
    ENSURE(c, ipay, std::max<u64>(W, 1) * 8);
    if (V)
        hipLaunchKernelGGL(k_term_pack, dim3(grid_for(V, RDF_BLOCK, kGrid)), dim3(RDF_BLOCK), 0, st, text, c->ikeys.as<u64>(), V,
                           c->nterm_off.as<u64>(), c->nterm_len.as<u32>(), c->ithv.as<u64>(), c->iwoff.as<u64>(), c->sh_rank,
                           c->ihdr.as<u64>(), c->ipay.as<u64>());
    HIP_TRY(c, hipStreamSynchronize(st));
    c->ing_pay_counts.assign(R, 0);
    TRY(x_request(c, req, RDF_X_ALLTOALLV_U64, c->ihdr.p, 2 * V, 21));
    for (u32 r = 0; r < R; ++r) {
        req->send_counts[r] = 2 * (bnd[r + 1] - bnd[r]);
        c->ing_pay_counts[r] = wb[r + 1] - wb[r];
    }
    return RDF_OK;
}

// received headers -> kept; the payload words follow (all-to-all, same grouping)
static rdf_status sh_phase21(rdf_ctx* c, rdf_exchange* req) {
    const u64 n = c->x_recv_count;
    ENSURE(c, rhdr, std::max<u64>(n, 1) * 8);
    if (n) HIP_TRY(c, hipMemcpyAsync(c->rhdr.p, c->xrecv.p, n * 8, hipMemcpyDeviceToDevice, c->stream));
    HIP_TRY(c, hipStreamSynchronize(c->stream));
    c->ing_m = n / 2;
    u64 W = 0;
    for (u64 w : c->ing_pay_counts) W += w;
    TRY(x_request(c, req, RDF_X_ALLTOALLV_U64, c->ipay.p, W, 22));
    for (u32 r = 0; r < c->sh_nranks; ++r) req->send_counts[r] = c->ing_pay_counts[r];
    return RDF_OK;
}

// owner: the received terms deduplicated (hash table of the parser, byte-verified), ids by first arrival; the count of
// distinct owned terms -> all-gather
static rdf_status sh_phase22(rdf_ctx* c, rdf_exchange* req) {
    hipStream_t st = c->stream;
    const u64 m = c->ing_m, W = c->x_recv_count;
    if (m >= 0xffffffffull) return fail(c, RDF_ERR_LIMIT, "sharded ingest: too many terms at one owner");
    ENSURE(c, own_text, W * 8 + 16);
    if (W) HIP_TRY(c, hipMemcpyAsync(c->own_text.p, c->xrecv.p, W * 8, hipMemcpyDeviceToDevice, st));
    ENSURE(c, rlen, std::max<u64>(m, 1) * 4);
    ENSURE(c, rwords, std::max<u64>(m, 1) * 4);
    ENSURE(c, rwoff, (m + 1) * 8);
    ENSURE(c, rts, std::max<u64>(m, 1) * 8);
    ENSURE(c, rhv, std::max<u64>(m, 1) * 8);
    ENSURE(c, rhist, RDF_MAX_RANKS * 4);
    const u64 nv = (m + 2) / 3;
    ENSURE(c, rvalid, std::max<u64>(nv, 1) * 4);
    HIP_TRY(c, hipMemsetAsync(c->rhist.p, 0, RDF_MAX_RANKS * 4, st));
    if (m)
        hipLaunchKernelGGL(k_term_records, dim3(grid_for(m, RDF_BLOCK, kGrid)), dim3(RDF_BLOCK), 0, st, c->rhdr.as<u64>(), m,
                           c->rwords.as<u32>(), c->rlen.as<u32>(), c->rhv.as<u64>(), c->rhist.as<u32>());
    HIP_TRY(c, exclusive_scan_u32_u64(c->ws, c->rwords.as<u32>(), c->rwoff.as<u64>(), m, c->rwoff.as<u64>() + m, st));
    if (m) {
        hipLaunchKernelGGL(k_words_to_bytes, dim3(grid_for(m, RDF_BLOCK, kGrid)), dim3(RDF_BLOCK), 0, st, c->rwoff.as<u64>(), m,
                           c->rts.as<u64>());
        hipLaunchKernelGGL(k_fill_u32, dim3(grid_for(nv, RDF_BLOCK, kGrid)), dim3(RDF_BLOCK), 0, st, c->rvalid.as<u32>(), nv, 1u);
    }
    const u64 T = next_pow2(2 * std::max<u64>(m, 1));
    ENSURE(c, rtab, T * 8);
    ENSURE(c, rslot, std::max<u64>(m, 1) * 4);
    ENSURE(c, rrep, std::max<u64>(m, 1) * 4);
    ENSURE(c, rfirst, std::max<u64>(m, 1) * 4);
    ENSURE(c, rfid, (m + 1) * 4);
    HIP_TRY(c, hipMemsetAsync(c->rtab.p, 0xff, T * 8, st));
    const unsigned g = grid_for(std::max<u64>(m, 1), RDF_BLOCK, kGrid);
    if (m) {
        hipLaunchKernelGGL(k_nt_dict_insert, dim3(g), dim3(RDF_BLOCK), 0, st, (const unsigned char*)c->own_text.p,
                           c->rts.as<u64>(), c->rlen.as<u32>(), c->rvalid.as<u32>(), m, c->rhv.as<u64>(), c->rtab.as<u64>(),
                           T - 1, c->rslot.as<u32>());
        hipLaunchKernelGGL(k_nt_dict_rep, dim3(g), dim3(RDF_BLOCK), 0, st, c->rvalid.as<u32>(), m, c->rslot.as<u32>(),
                           c->rtab.as<u64>(), c->rrep.as<u32>(), c->rfirst.as<u32>());
    }
    HIP_TRY(c, exclusive_scan_u32(c->ws, c->rfirst.as<u32>(), c->rfid.as<u32>(), m, c->rfid.as<u32>() + m, st));
    u32 nown = 0;
    TRY(read_u32(c, c->rfid.as<u32>() + m, &nown));
    c->own_n = nown;
    c->ing_src_counts.assign(RDF_MAX_RANKS, 0);
    std::vector<u32> hh(RDF_MAX_RANKS);
    HIP_TRY(c, ctx_copy(c, hh.data(), c->rhist.p, RDF_MAX_RANKS * 4, hipMemcpyDeviceToHost));
    for (int r = 0; r < RDF_MAX_RANKS; ++r) c->ing_src_counts[r] = hh[r];
    ENSURE(c, xsend, 8);
    c->hscal[14] = nown;
    HIP_TRY(c, ctx_copy(c, c->xsend.p, c->hscal + 14, 8, hipMemcpyHostToDevice));
    return x_request(c, req, RDF_X_ALLGATHERV_U64, c->xsend.p, 1, 23);
}

// owners' term counts -> bases; each received term's global id back to its sender (all-to-all)
static rdf_status sh_phase23(rdf_ctx* c, rdf_exchange* req) {
    hipStream_t st = c->stream;
    const u32 R = c->sh_nranks;
    if (c->x_recv_count != R) return fail(c, RDF_ERR_ARG, "term-count all-gather: wrong element count");
    std::vector<u64> cnt(R);
    HIP_TRY(c, ctx_copy(c, cnt.data(), c->xrecv.p, R * 8, hipMemcpyDeviceToHost));
    u64 base = 0, tot = 0;
    for (u32 r = 0; r < R; ++r) {
        if (r < c->sh_rank) base += cnt[r];
        tot += cnt[r];
    }
    if (tot >= (1ull << 30)) return fail(c, RDF_ERR_LIMIT, "num_terms must be < 2^30");
    c->own_base = (u32)base;
    const u64 m = c->ing_m;
    ENSURE(c, rreply, std::max<u64>(m, 1) * 8);
    ENSURE(c, own_off, std::max<u64>(c->own_n, 1) * 8);
    ENSURE(c, own_len, std::max<u64>(c->own_n, 1) * 4);
    if (m)
        hipLaunchKernelGGL(k_term_reply, dim3(grid_for(m, RDF_BLOCK, kGrid)), dim3(RDF_BLOCK), 0, st, c->rhdr.as<u64>(), m,
                           c->rrep.as<u32>(), c->rfirst.as<u32>(), c->rfid.as<u32>(), (u32)base, c->rts.as<u64>(),
                           c->rlen.as<u32>(), c->rreply.as<u64>(), c->own_off.as<u64>(), c->own_len.as<u32>());
    HIP_TRY(c, hipStreamSynchronize(st));
    c->V = (u32)tot;
    TRY(x_request(c, req, RDF_X_ALLTOALLV_U64, c->rreply.p, m, 24));
    for (u32 r = 0; r < R; ++r) req->send_counts[r] = c->ing_src_counts[r];
    return RDF_OK;
}

// every local term's global id -> the rank's triples rewritten in the global id space
static rdf_status sh_phase24(rdf_ctx* c, rdf_exchange* req) {
    hipStream_t st = c->stream;
    const u64 m = c->x_recv_count, Vl = c->ing_Vl;
    if (m != Vl) return fail(c, RDF_ERR_ARG, "sharded ingest: a local term got no global id");
    ENSURE(c, gmapv, std::max<u64>(Vl, 1) * 4);
    if (m)
        hipLaunchKernelGGL(k_term_gmap, dim3(grid_for(m, RDF_BLOCK, kGrid)), dim3(RDF_BLOCK), 0, st, c->xrecv.as<u64>(), m,
                           c->gmapv.as<u32>());
    if (c->n)
        hipLaunchKernelGGL(k_remap3, dim3(grid_for(c->n, RDF_BLOCK, kGrid)), dim3(RDF_BLOCK), 0, st, c->ts.as<u32>(),
                           c->tp.as<u32>(), c->to.as<u32>(), c->n, c->gmapv.as<u32>());
    HIP_TRY(c, hipGetLastError());
    HIP_TRY(c, hipStreamSynchronize(st));
    c->parsed_dict = false;
    c->ingest_sharded = true;
    c->stage = 1;
    c->paged = false;  // a paged run's state belongs to the previous input
    memset(req, 0, sizeof(*req));
    req->op = RDF_X_DONE;
    c->sh_phase = 9;
    return RDF_OK;
}

// ---- formatting dictionary by owner lookup: the values of the frequent conditions (the only terms an output line
// can name) from their owners to every rank (two all-gathers: headers, then the bytes)
static rdf_status sh_phase30(rdf_ctx* c, rdf_exchange* req) {
    hipStream_t st = c->stream;
    const u32 nown = c->own_n;
    ENSURE(c, dneed, std::max<u64>(nown, 1) * 4);
    ENSURE(c, dnpos, (nown + 1ull) * 4);
    ENSURE(c, dwn, std::max<u64>(nown, 1) * 4);
    ENSURE(c, dwo, (nown + 1ull) * 8);
    HIP_TRY(c, hipMemsetAsync(c->dneed.p, 0, std::max<u64>(nown, 1) * 4, st));
    if ((u64)c->U + c->B)
        hipLaunchKernelGGL(k_mark_needed, dim3(grid_for((u64)c->U + c->B, RDF_BLOCK, kGrid)), dim3(RDF_BLOCK), 0, st,
                           c->fval.as<u32>(), (u64)c->U, c->bkeys.as<u64>(), c->B, c->own_base, nown, c->dneed.as<u32>());
    HIP_TRY(c, exclusive_scan_u32(c->ws, c->dneed.as<u32>(), c->dnpos.as<u32>(), nown, c->dnpos.as<u32>() + nown, st));
    if (nown)
        hipLaunchKernelGGL(k_needed_words, dim3(grid_for(nown, RDF_BLOCK, kGrid)), dim3(RDF_BLOCK), 0, st, c->dneed.as<u32>(),
                           c->own_len.as<u32>(), nown, c->dwn.as<u32>());
    HIP_TRY(c, exclusive_scan_u32_u64(c->ws, c->dwn.as<u32>(), c->dwo.as<u64>(), nown, c->dwo.as<u64>() + nown, st));
    u64 v[2];
    TRY(read_multi(c, {{c->dnpos.as<u32>() + nown, 4}, {c->dwo.as<u64>() + nown, 8}}, v));
    const u64 nneed = v[0], W = v[1];
    ENSURE(c, ihdr, std::max<u64>(nneed, 1) * 8);
    ENSURE(c, ipay, std::max<u64>(W, 1) * 8);
    if (nown)
        hipLaunchKernelGGL(k_dict_pack, dim3(grid_for(nown, RDF_BLOCK, kGrid)), dim3(RDF_BLOCK), 0, st, c->dneed.as<u32>(),
                           c->dnpos.as<u32>(), nown, c->own_base, c->own_off.as<u64>(), c->own_len.as<u32>(),
                           (const unsigned char*)c->own_text.p, c->dwo.as<u64>(), c->ihdr.as<u64>(), c->ipay.as<u64>());
    HIP_TRY(c, hipStreamSynchronize(st));
    c->ing_pay_counts.assign(1, W);
    return x_request(c, req, RDF_X_ALLGATHERV_U64, c->ihdr.p, nneed, 31);
}

static rdf_status sh_phase31(rdf_ctx* c, rdf_exchange* req) {
    const u64 M = c->x_recv_count;
    ENSURE(c, dhdr, std::max<u64>(M, 1) * 8);
    if (M) HIP_TRY(c, hipMemcpyAsync(c->dhdr.p, c->xrecv.p, M * 8, hipMemcpyDeviceToDevice, c->stream));
    HIP_TRY(c, hipStreamSynchronize(c->stream));
    c->ing_m = M;
    return x_request(c, req, RDF_X_ALLGATHERV_U64, c->ipay.p, c->ing_pay_counts[0], 32);
}

static rdf_status sh_phase32(rdf_ctx* c, rdf_exchange* req) {
    hipStream_t st = c->stream;
    const u64 M = c->ing_m, V = c->V;
    ENSURE(c, dlen, std::max<u64>(V, 1) * 4);
    ENSURE(c, dlwords, std::max<u64>(M, 1) * 4);
    ENSURE(c, dwoff, (M + 1) * 8);
    ENSURE(c, dtoff, (V + 1) * 8);
    HIP_TRY(c, hipMemsetAsync(c->dlen.p, 0, std::max<u64>(V, 1) * 4, st));
    if (M)
        hipLaunchKernelGGL(k_dict_lengths, dim3(grid_for(M, RDF_BLOCK, kGrid)), dim3(RDF_BLOCK), 0, st, c->dhdr.as<u64>(), M,
                           c->dlen.as<u32>(), c->dlwords.as<u32>());
    HIP_TRY(c, exclusive_scan_u32_u64(c->ws, c->dlwords.as<u32>(), c->dwoff.as<u64>(), M, c->dwoff.as<u64>() + M, st));
    HIP_TRY(c, exclusive_scan_u32_u64(c->ws, c->dlen.as<u32>(), c->dtoff.as<u64>(), V, c->dtoff.as<u64>() + V, st));
    u64 heap = 0;
    TRY(read_u64(c, c->dtoff.as<u64>() + V, &heap));
    ENSURE(c, dheap, std::max<u64>(heap, 1));
    if (M)
        hipLaunchKernelGGL(k_dict_fill, dim3(grid_for(M, RDF_BLOCK, kGrid)), dim3(RDF_BLOCK), 0, st, c->dhdr.as<u64>(), M,
                           c->dwoff.as<u64>(), c->xrecv.as<u64>(), c->dtoff.as<u64>(), c->dheap.as<char>());
    HIP_TRY(c, hipGetLastError());
    HIP_TRY(c, hipStreamSynchronize(st));
    c->dict_terms = V;
    c->capstr_run = ~0ull;
    memset(req, 0, sizeof(*req));
    req->op = RDF_X_DONE;
    c->sh_phase = 9;
    return RDF_OK;
}

// phases: 10, 16, 11-14 (condition counts, routing of the triples), then 1-8 (15 between 5 and 6); pending = a
// phase that follows a collective
static bool sh_phase_valid(int ph, bool pending) {
    if (ph >= 1 && ph <= 8) return true;
    if (ph >= 11 && ph <= 18) return true;
    if (ph >= 21 && ph <= 24) return true;
    if (ph >= 31 && ph <= 32) return true;
    return !pending && (ph == 10 || ph == 20 || ph == 30);
}

rdf_status rdf_shard_begin(rdf_ctx* c, uint32_t rank, uint32_t nranks, uint32_t min_support, const char* projection,
                           uint32_t flags) {
    if (!c) return RDF_ERR_ARG;
    if (c) TRY(hv_wait(c, true));
    c->res_bits = c->heavy_pending = false;  // (the heavy-bits form: results of d_emit_rest / d_page_emit only)
    if (nranks < 1 || nranks > RDF_MAX_RANKS || rank >= nranks) return fail(c, RDF_ERR_ARG, "invalid rank / nranks");
    if (c->stage < 1) return fail(c, RDF_ERR_STATE, "rdf_set_triples must be called first");
    c->hclassed = false;
    int proj = 0;
    TRY(parse_projection(c, projection, &proj));
    c->sh_rank = rank;
    c->sh_nranks = nranks;
    c->sh_ms = min_support;
    c->sh_proj = proj;
    c->sh_flags = flags;
    c->sh_phase = 10;
    c->x_imported = true;
    c->spare_x = false;  // (a run that failed between phases 14 and 1 left them marked)
    c->stage = std::min(c->stage, 1);
    c->paged = false;
    return RDF_OK;
}

rdf_status rdf_shard_parse_begin(rdf_ctx* c, uint32_t rank, uint32_t nranks, const char* text, uint64_t nbytes,
                                 uint32_t flags, uint64_t* n_triples) {
    if (!c) return RDF_ERR_ARG;
    if (c) TRY(hv_wait(c, true));
    if (nranks < 1 || nranks > RDF_MAX_RANKS || rank >= nranks) return fail(c, RDF_ERR_ARG, "invalid rank / nranks");
    uint64_t n = 0;
    u32 Vl = 0;
    TRY(rdf_parse_ntriples(c, text, nbytes, flags, &n, &Vl, nullptr));
    c->ing_Vl = Vl;
    c->ingest_sharded = false;
    c->sh_rank = rank;
    c->sh_nranks = nranks;
    c->sh_phase = 20;
    c->x_imported = true;
    c->stage = 0;  // no usable triples until the global ids arrive
    c->paged = false;
    if (n_triples) *n_triples = n;
    return RDF_OK;
}

rdf_status rdf_shard_dictionary_begin(rdf_ctx* c) {
    if (!c) return RDF_ERR_ARG;
    if (!c->ingest_sharded) return fail(c, RDF_ERR_STATE, "the triples do not come from rdf_shard_parse_begin");
    if (c->stage < 2) return fail(c, RDF_ERR_STATE, "a (sharded) run must come first: the frequent conditions name the terms");
    c->sh_phase = 30;
    c->x_imported = true;
    return RDF_OK;
}

rdf_status rdf_num_terms(rdf_ctx* c, uint32_t* n) {
    if (!c || !n) return RDF_ERR_ARG;
    *n = c->V;
    return RDF_OK;
}

// terms of ids[0, n) from the formatting dictionary: offsets[n + 1] and their bytes (cap bytes; RDF_ERR_ARG if short)
rdf_status rdf_dictionary_terms(rdf_ctx* c, const uint32_t* ids, uint64_t n, char* out, uint64_t cap, uint64_t* offsets) {
    if (!c || (n && (!ids || !offsets))) return RDF_ERR_ARG;
    if (c->dict_terms < c->V) return fail(c, RDF_ERR_STATE, "no formatting dictionary covers the term ids");
    HIP_TRY(c, hipSetDevice(c->device));
    hipStream_t st = c->stream;
    ENSURE(c, tids, std::max<u64>(n, 1) * 4);
    ENSURE(c, tlenv, std::max<u64>(n, 1) * 4);
    ENSURE(c, toffv, (n + 1) * 8);
    if (n) HIP_TRY(c, hipMemcpyAsync(c->tids.p, ids, n * 4, hipMemcpyHostToDevice, st));
    if (n)
        hipLaunchKernelGGL(k_dict_term_len, dim3(grid_for(n, RDF_BLOCK, kGrid)), dim3(RDF_BLOCK), 0, st, c->tids.as<u32>(), n,
                           c->dtoff.as<u64>(), c->tlenv.as<u32>());
    HIP_TRY(c, exclusive_scan_u32_u64(c->ws, c->tlenv.as<u32>(), c->toffv.as<u64>(), n, c->toffv.as<u64>() + n, st));
    HIP_TRY(c, hipMemcpyAsync(offsets, c->toffv.p, (n + 1) * 8, hipMemcpyDeviceToHost, st));
    HIP_TRY(c, hipStreamSynchronize(st));
    const u64 total = offsets[n];
    if (total > cap) return fail(c, RDF_ERR_ARG, "term buffer too small (see offsets[n])");
    ENSURE(c, tout, std::max<u64>(total, 1));
    if (n)
        hipLaunchKernelGGL(k_dict_term_copy, dim3(grid_for(n, RDF_BLOCK, kGrid)), dim3(RDF_BLOCK), 0, st, c->tids.as<u32>(), n,
                           c->dtoff.as<u64>(), c->dheap.as<char>(), c->toffv.as<u64>(), c->tout.as<char>());
    if (total) HIP_TRY(c, hipMemcpyAsync(out, c->tout.p, total, hipMemcpyDeviceToHost, st));
    HIP_TRY(c, hipStreamSynchronize(st));
    return RDF_OK;
}

rdf_status rdf_shard_step(rdf_ctx* c, rdf_exchange* req) {
    if (!c || !req) return RDF_ERR_ARG;
    if (!sh_phase_valid(c->sh_phase, false)) return fail(c, RDF_ERR_STATE, "rdf_shard_begin must be called first");
    if (!c->x_imported) return fail(c, RDF_ERR_STATE, "rdf_shard_import must supply the pending exchange first");
    HIP_TRY(c, hipSetDevice(c->device));
    if ((int)c->sh_rank == c->test_fail_rank && c->sh_phase == c->test_fail_phase)
        return fail(c, RDF_ERR_OOM, "RDFIND_TEST_FAIL_SHARD: this rank fails at phase " + std::to_string(c->sh_phase));
    rdf_status r = RDF_OK;
    switch (c->sh_phase) {
        case 1: r = sh_phase1(c, req); break;
        case 2: r = sh_phase2(c, req); break;
        case 3: r = sh_phase3(c, req); break;
        case 4: r = sh_phase4(c, req); break;
        case 5: r = sh_phase5(c, req); break;
        case 15: r = sh_phase15(c, req); break;
        case 16: r = sh_phase16(c, req); break;
        case 17: r = sh_phase17(c, req); break;
        case 18: r = sh_phase18(c, req); break;
        case 20: r = sh_phase20(c, req); break;
        case 21: r = sh_phase21(c, req); break;
        case 22: r = sh_phase22(c, req); break;
        case 23: r = sh_phase23(c, req); break;
        case 24: r = sh_phase24(c, req); break;
        case 30: r = sh_phase30(c, req); break;
        case 31: r = sh_phase31(c, req); break;
        case 32: r = sh_phase32(c, req); break;
        case 6: r = sh_phase6(c, req); break;
        case 7: r = sh_phase7(c, req); break;
        case 8: r = sh_phase8(c, req); break;
        case 10: r = sh_phase10(c, req); break;
        case 11: r = sh_phase11(c, req); break;
        case 12: r = sh_phase12(c, req); break;
        case 13: r = sh_phase13(c, req); break;
        case 14: r = sh_phase14(c, req); break;
    }
    if (r != RDF_OK) c->sh_phase = -1;  // a failed machine must be restarted with rdf_shard_begin
    return r;
}

rdf_status rdf_shard_export(rdf_ctx* c, void* dst) {
    if (!c) return RDF_ERR_ARG;
    if (c->x_imported || !sh_phase_valid(c->sh_phase, true)) return fail(c, RDF_ERR_STATE, "no pending exchange");
    if (c->x_count && !dst) return fail(c, RDF_ERR_ARG, "null exchange buffer");
    HIP_TRY(c, hipSetDevice(c->device));
    if (c->x_count)
        HIP_TRY(c, hipMemcpyAsync(dst, c->x_src, c->x_count * c->x_bytes, hipMemcpyDefault, c->stream));
    HIP_TRY(c, hipStreamSynchronize(c->stream));
    return RDF_OK;
}

rdf_status rdf_shard_import(rdf_ctx* c, const void* src, uint64_t count) {
    if (!c) return RDF_ERR_ARG;
    if (c->x_imported || !sh_phase_valid(c->sh_phase, true)) return fail(c, RDF_ERR_STATE, "no pending exchange");
    if (count && !src) return fail(c, RDF_ERR_ARG, "null exchange buffer");
    const bool reduce = c->x_op == RDF_X_ALLREDUCE_SUM_U32 || c->x_op == RDF_X_ALLREDUCE_SUM_U64 ||
                        c->x_op == RDF_X_ALLREDUCE_MIN_U64;
    if (reduce && count != c->x_count) return fail(c, RDF_ERR_ARG, "all-reduce result has the wrong element count");
    HIP_TRY(c, hipSetDevice(c->device));
    ENSURE(c, xrecv, std::max<u64>(count, 1) * c->x_bytes);
    if (count) HIP_TRY(c, hipMemcpyAsync(c->xrecv.p, src, count * c->x_bytes, hipMemcpyDefault, c->stream));
    HIP_TRY(c, hipStreamSynchronize(c->stream));
    c->x_recv_count = count;
    c->x_imported = true;
    return RDF_OK;
}

// Expands the class part of the result (members x shared lists) into per-dependent runs behind the explicit refs:
// needed by every row-level accessor (copy, decode, checksum, formatting), not by rdf_copy_result_compact.
// the heavy-bits form's refs written into `out` behind the explicit ones (k_heavy_write, deferred by d_emit_rest /
// d_page_emit): row accessors and the device checksum read them there
static rdf_status materialize_heavy(rdf_ctx* c) {
    if (!c->heavy_pending) return RDF_OK;
    hipStream_t st = c->stream;
    HIP_TRY(c, hipSetDevice(c->device));
    TRY(hv_wait(c, false));
    CindView v = {};  // (the classed write reads only the class lists through sbase)
    hipLaunchKernelGGL(k_heavy_write, dim3(vgrid(wave_blocks(c->hp_W))), dim3(RDF_BLOCK), 0, st, (u64)wave_blocks(c->hp_W),
                       v, c->pivot.as<u32>(), c->choffh.as<u64>(), c->hown.as<u32>(), c->hp_h0, c->hp_W, c->hbits.as<u64>(),
                       c->clists.as<u32>(), c->sbase.as<u64>(), c->hoff.as<u64>(), c->hp_K, c->out.as<u32>());
    HIP_TRY(c, hipGetLastError());
    HIP_TRY(c, hipStreamSynchronize(st));
    c->heavy_pending = false;
    return RDF_OK;
}

static rdf_status materialize(rdf_ctx* c) {
    TRY(materialize_heavy(c));
    if (!c->class_pending) return RDF_OK;
    hipStream_t st = c->stream;
    HIP_TRY(c, hipSetDevice(c->device));
    TRY(hv_wait(c, false));  // an early refs copy may still read `out`
    HIP_TRY(c, c->out.grow_keep((size_t)std::max<u64>(c->n_out, 1) * 4, st));
    c->tn[RDF_T_CEMIT] = 0;
    tbegin(c, RDF_T_CEMIT);
    hipLaunchKernelGGL(k_class_emit, dim3(vgrid(c->pend_NT)), dim3(RDF_BLOCK), 0, st, c->pend_NT, c->coff.as<u64>(),
                       c->cchoff.as<u64>(), c->lwoff.as<u64>(), c->clists.as<u32>(), c->ctoff.as<u64>(),
                       (u32)c->n_classes, c->cself.as<u32>(), c->cobase.as<u64>(), c->pend_base, c->out.as<u32>());
    tend(c, RDF_T_CEMIT);
    HIP_TRY(c, hipGetLastError());
    HIP_TRY(c, hipStreamSynchronize(st));
    tcollect(c, RDF_T_CEMIT, RDF_T_CEMIT + 1);
    c->out_ptr = c->out.as<u32>();
    c->class_pending = false;
    return RDF_OK;
}

// page-locked host memory for the result hand-over (the copies then run at the link rate)
void* rdf_host_alloc(uint64_t bytes) {
    void* p = nullptr;
    return hipHostMalloc(&p, bytes ? bytes : 1, hipHostMallocDefault) == hipSuccess ? p : nullptr;
}
void rdf_host_free(void* p) {
    if (p) (void)hipHostFree(p);
}

// explicit refs and runs of the compact result: all of the non-class refs, or (heavy-bits form) the explicit ones only,
// the heavy-only ones leaving as bits (rdf_copy_result_heavy)
static u64 compact_refs(const rdf_ctx* c) { return c->res_bits ? c->res_K : c->n_out - c->n_class_out; }
static u64 compact_runs(const rdf_ctx* c) { return c->res_bits ? c->res_nx : c->n_runs_explicit; }

rdf_status rdf_get_result_layout(rdf_ctx* c, rdf_result_layout* L) {
    if (!c || !L) return RDF_ERR_ARG;
    if (c->stage < 4) return fail(c, RDF_ERR_STATE, "rdf_discover_cinds must be called first");
    L->n_cinds = c->n_out;
    L->n_refs = compact_refs(c);
    L->n_runs = compact_runs(c);
    L->n_lists = c->n_lists;
    L->n_list_refs = c->n_list_refs;
    L->n_members = c->n_class_out ? c->n_class_members : 0;
    L->n_captures = c->C;
    return RDF_OK;
}

// The compact CindSet-shaped result (SURVEY.md 8(d) "CIND id-records in host memory"): explicit refs in runs of one
// dependent, the shared lists and their member dependents, the capture table.  Plain async copies on the context
// stream (pinned caller memory lets them run at the link rate); nothing is expanded.
rdf_status rdf_copy_result_compact(rdf_ctx* c, uint32_t* refs, uint64_t* runoff, uint32_t* rundep, uint32_t* list_refs,
                                   uint64_t* list_off, uint64_t* members, uint32_t* capture_ids, uint32_t* supports) {
    if (!c) return RDF_ERR_ARG;
    if (c->stage < 4) return fail(c, RDF_ERR_STATE, "rdf_discover_cinds must be called first");
    HIP_TRY(c, hipSetDevice(c->device));
    hipStream_t st = c->stream;
    const u64 nrefs = compact_refs(c), R = compact_runs(c);
    const u64 nmem = c->n_class_out ? c->n_class_members : 0;
    // parts the early hand-over already copied into these same buffers: only their tails (heavy-only refs behind the
    // explicit ones) or nothing
    const u64 r0 = refs && refs == c->hv_refs && c->hv_refs_n != ~0ull ? std::min<u64>(c->hv_refs_n, nrefs) : 0;
    const bool caps_done = c->hv_caps_done && capture_ids == c->hv_capid && supports == c->hv_sup;
    if (refs && nrefs > r0)
        HIP_TRY(c, hipMemcpyAsync(refs + r0, c->out_ptr + r0, (nrefs - r0) * 4, hipMemcpyDeviceToHost, st));
    const u64 q0 = runoff && rundep && runoff == c->hv_runoff && rundep == c->hv_rundep && c->hv_runs_n != ~0ull
                       ? std::min<u64>(c->hv_runs_n, R) : 0;
    if (runoff)
        HIP_TRY(c, hipMemcpyAsync(runoff + q0, c->runoff.as<u64>() + q0, (R + 1 - q0) * 8, hipMemcpyDeviceToHost, st));
    if (rundep && R > q0)
        HIP_TRY(c, hipMemcpyAsync(rundep + q0, c->rundep.as<u32>() + q0, (R - q0) * 4, hipMemcpyDeviceToHost, st));
    if (c->n_lists) {
        if (list_refs && c->n_list_refs)
            HIP_TRY(c, hipMemcpyAsync(list_refs, c->clists.p, c->n_list_refs * 4, hipMemcpyDeviceToHost, st));
        if (list_off) HIP_TRY(c, hipMemcpyAsync(list_off, c->loff.p, (c->n_lists + 1) * 8, hipMemcpyDeviceToHost, st));
    } else if (list_off) {
        list_off[0] = 0;
    }
    if (members && nmem) HIP_TRY(c, hipMemcpyAsync(members, c->ckeys.p, nmem * 8, hipMemcpyDeviceToHost, st));
    if (capture_ids && c->C && !caps_done)
        HIP_TRY(c, hipMemcpyAsync(capture_ids, c->fext.p, (u64)c->C * 4, hipMemcpyDeviceToHost, st));
    if (supports && c->C && !caps_done)
        HIP_TRY(c, hipMemcpyAsync(supports, c->csup.p, (u64)c->C * 4, hipMemcpyDeviceToHost, st));
    HIP_TRY(c, hipStreamSynchronize(st));
    TRY(hv_wait(c, false));
    return RDF_OK;
}

rdf_status rdf_set_handover(rdf_ctx* c, uint32_t* refs, uint64_t refs_cap, uint64_t* runoff, uint32_t* rundep,
                            uint64_t runs_cap, uint32_t* capture_ids, uint32_t* supports, uint64_t capture_cap) {
    if (!c) return RDF_ERR_ARG;
    HIP_TRY(c, hipSetDevice(c->device));
    TRY(hv_wait(c, true));
    c->hv_refs = refs_cap ? refs : nullptr;
    c->hv_refs_cap = refs ? refs_cap : 0;
    c->hv_runoff = runs_cap && rundep ? runoff : nullptr;
    c->hv_rundep = runs_cap && runoff ? rundep : nullptr;
    c->hv_runs_cap = runoff && rundep ? runs_cap : 0;
    c->hv_capid = capture_cap ? capture_ids : nullptr;
    c->hv_sup = capture_cap ? supports : nullptr;
    c->hv_cap_cap = capture_ids && supports ? capture_cap : 0;
    return RDF_OK;
}

rdf_status rdf_copy_result_refs(rdf_ctx* c, uint64_t offset, uint64_t count, uint32_t* refs, uint64_t* n_copied) {
    if (!c || (count && !refs)) return RDF_ERR_ARG;
    if (c->stage < 4) return fail(c, RDF_ERR_STATE, "rdf_discover_cinds must be called first");
    HIP_TRY(c, hipSetDevice(c->device));
    TRY(hv_wait(c, false));  // (an asynchronous copy may still write the same host buffer)
    const u64 nrefs = compact_refs(c);
    const u64 n = offset < nrefs ? std::min<u64>(count, nrefs - offset) : 0;
    if (n) HIP_TRY(c, hipMemcpyAsync(refs, c->out_ptr + offset, n * 4, hipMemcpyDeviceToHost, c->stream));
    HIP_TRY(c, hipStreamSynchronize(c->stream));
    if (n_copied) *n_copied = n;
    return RDF_OK;
}

rdf_status rdf_copy_result_refs_async(rdf_ctx* c, uint64_t offset, uint64_t count, uint32_t* refs, uint64_t* n_copied) {
    if (!c || (count && !refs)) return RDF_ERR_ARG;
    if (c->stage < 4) return fail(c, RDF_ERR_STATE, "rdf_discover_cinds must be called first");
    HIP_TRY(c, hipSetDevice(c->device));
    const u64 nrefs = compact_refs(c);
    const u64 n = offset < nrefs ? std::min<u64>(count, nrefs - offset) : 0;
    if (n) {  // after everything queued so far on the compute stream, on the copy stream
        HIP_TRY(c, hipEventRecord(c->hv_ev, c->stream));
        HIP_TRY(c, hipStreamWaitEvent(c->hstream, c->hv_ev, 0));
        HIP_TRY(c, hipMemcpyAsync(refs, c->out_ptr + offset, n * 4, hipMemcpyDeviceToHost, c->hstream));
        HIP_TRY(c, hipEventRecord(c->hv_done, c->hstream));
        c->hv_pending = true;
        c->hv_gpu_wait = true;
    }
    if (n_copied) *n_copied = n;
    return RDF_OK;
}

rdf_status rdf_handover_wait(rdf_ctx* c) {
    if (!c) return RDF_ERR_ARG;
    HIP_TRY(c, hipSetDevice(c->device));
    return hv_wait(c, false);
}

rdf_status rdf_set_result_form(rdf_ctx* c, uint32_t form) {
    if (!c || form > RDF_FORM_HEAVY_BITS) return RDF_ERR_ARG;
    c->result_form = form;  // (from the next discovery on)
    return RDF_OK;
}

rdf_status rdf_heavy_chunk_count(rdf_ctx* c, uint64_t* n) {
    if (!c || !n) return RDF_ERR_ARG;
    if (c->stage < 4) return fail(c, RDF_ERR_STATE, "rdf_discover_cinds must be called first");
    *n = c->res_bits ? c->res_wh : 0;
    return RDF_OK;
}

rdf_status rdf_copy_result_heavy(rdf_ctx* c, uint32_t* deps, uint64_t* pos, uint64_t* bits) {
    if (!c) return RDF_ERR_ARG;
    if (c->stage < 4) return fail(c, RDF_ERR_STATE, "rdf_discover_cinds must be called first");
    HIP_TRY(c, hipSetDevice(c->device));
    const u64 W = c->res_bits ? c->res_wh : 0;
    if (!W) return RDF_OK;
    if (!deps || !pos || !bits) return RDF_ERR_ARG;
    hipStream_t st = c->stream;
    ENSURE(c, hpos, W * 8);
    hipLaunchKernelGGL(k_heavy_pos, dim3(grid_for(W, RDF_BLOCK, kGrid)), dim3(RDF_BLOCK), 0, st, c->C, c->res_h0, W,
                       c->choffh.as<u64>(), c->rundep.as<u32>() + c->res_nx, c->sbase.as<u64>(), c->hpos.as<u64>());
    HIP_TRY(c, hipGetLastError());
    HIP_TRY(c, hipMemcpyAsync(deps, c->rundep.as<u32>() + c->res_nx, W * 4, hipMemcpyDeviceToHost, st));
    HIP_TRY(c, hipMemcpyAsync(pos, c->hpos.p, W * 8, hipMemcpyDeviceToHost, st));
    HIP_TRY(c, hipMemcpyAsync(bits, c->hbits.p, W * 8, hipMemcpyDeviceToHost, st));
    HIP_TRY(c, hipStreamSynchronize(st));
    return RDF_OK;
}

rdf_status rdf_last_stats(rdf_ctx* c, rdf_fc_stats* fc, rdf_group_stats* gs, rdf_cind_stats* cs) {
    if (!c) return RDF_ERR_ARG;
    if (c->stage < 4) return fail(c, RDF_ERR_STATE, "no completed run");
    if (fc) *fc = c->fstats;
    if (gs) {
        TRY(settle_group_stats(c));
        *gs = c->gstats;
    }
    if (cs) *cs = c->cstats;
    return RDF_OK;
}

rdf_status rdf_cind_count(rdf_ctx* c, uint64_t* n) {
    if (!c || !n) return RDF_ERR_ARG;
    if (c->stage < 4) return fail(c, RDF_ERR_STATE, "rdf_discover_cinds must be called first");
    *n = c->n_out;
    return RDF_OK;
}

// host mirrors for copy-out (run table, external capture ids, supports): filled on the first copy after a
// run, so a run whose results stay in HBM pays no device -> host traffic
static rdf_status load_runs(rdf_ctx* c) {
    if (c->h_runs_valid) return RDF_OK;
    c->h_runoff.resize(c->n_runs + 1);
    c->h_rundep.resize(c->n_runs);
    HIP_TRY(c, ctx_copy(c, c->h_runoff.data(), c->runoff.p, (c->n_runs + 1) * 8, hipMemcpyDeviceToHost));
    if (c->n_runs) HIP_TRY(c, ctx_copy(c, c->h_rundep.data(), c->rundep.p, c->n_runs * 4, hipMemcpyDeviceToHost));
    const u32 C = c->C;
    c->h_fcap.resize(C);
    c->h_csup.resize(C);
    if (C) {
        HIP_TRY(c, ctx_copy(c, c->h_fcap.data(), c->fext.p, (u64)C * 4, hipMemcpyDeviceToHost));
        HIP_TRY(c, ctx_copy(c, c->h_csup.data(), c->csup.p, (u64)C * 4, hipMemcpyDeviceToHost));
    }
    c->h_runs_valid = true;
    return RDF_OK;
}

// decode output elements [offset, offset + m) to caller records (external ids + dependent support)
static rdf_status copy_decoded(rdf_ctx* c, u64 offset, u64 m, rdf_cind* out) {
    TRY(load_runs(c));
    const u64 chunk = 1ull << 24;
    std::vector<u32> buf(std::min<u64>(chunk, std::max<u64>(m, 1)));
    // first run holding element offset (largest r with runoff[r] <= offset)
    u64 r = (u64)(std::upper_bound(c->h_runoff.begin(), c->h_runoff.begin() + c->n_runs, offset) - c->h_runoff.begin());
    r = r ? r - 1 : 0;
    for (u64 b = 0; b < m; b += chunk) {
        const u64 k = std::min(chunk, m - b);
        HIP_TRY(c, ctx_copy(c, buf.data(), c->out_ptr + offset + b, k * 4, hipMemcpyDeviceToHost));
        for (u64 i = 0; i < k; ++i) {
            const u64 e = offset + b + i;
            while (c->h_runoff[r + 1] <= e) ++r;
            const u32 d = c->h_rundep[r];
            out[b + i].dep = c->h_fcap[d];
            out[b + i].ref = c->h_fcap[buf[i]];
            out[b + i].support = c->h_csup[d];
        }
    }
    return RDF_OK;
}

rdf_status rdf_copy_cinds(rdf_ctx* c, rdf_cind* out, uint64_t cap, uint64_t* n_copied) {
    if (!c || (cap && !out)) return RDF_ERR_ARG;
    if (c->stage < 4) return fail(c, RDF_ERR_STATE, "rdf_discover_cinds must be called first");
    HIP_TRY(c, hipSetDevice(c->device));
    TRY(materialize(c));
    const u64 total = std::min<u64>(cap, c->n_out);
    if (total) TRY(copy_decoded(c, 0, total, out));
    if (n_copied) *n_copied = total;
    return RDF_OK;
}

rdf_status rdf_copy_cinds_range(rdf_ctx* c, uint64_t offset, rdf_cind* out, uint64_t count, uint64_t* n_copied) {
    if (!c || (count && !out)) return RDF_ERR_ARG;
    if (c->stage < 4) return fail(c, RDF_ERR_STATE, "rdf_discover_cinds must be called first");
    HIP_TRY(c, hipSetDevice(c->device));
    TRY(materialize(c));
    const u64 m = offset >= c->n_out ? 0 : std::min<u64>(count, c->n_out - offset);
    if (m) TRY(copy_decoded(c, offset, m, out));
    if (n_copied) *n_copied = m;
    return RDF_OK;
}

// The CindSet-shaped result as id-records ("CIND id-records in host memory"): refs + run table +
// the compact -> external capture ids and supports.  Plain async copies on the context stream (pinned caller
// memory makes them DMA at the link rate).
rdf_status rdf_result_sizes(rdf_ctx* c, uint64_t* n_refs, uint64_t* n_runs, uint64_t* n_captures) {
    if (!c) return RDF_ERR_ARG;
    if (c->stage < 4) return fail(c, RDF_ERR_STATE, "rdf_discover_cinds must be called first");
    if (n_refs) *n_refs = c->n_out;
    if (n_runs) *n_runs = c->n_runs;
    if (n_captures) *n_captures = c->C;
    return RDF_OK;
}

rdf_status rdf_copy_result_raw(rdf_ctx* c, uint32_t* refs, uint64_t* runoff, uint32_t* rundep, uint32_t* capture_ids,
                               uint32_t* supports) {
    if (!c) return RDF_ERR_ARG;
    if (c->stage < 4) return fail(c, RDF_ERR_STATE, "rdf_discover_cinds must be called first");
    HIP_TRY(c, hipSetDevice(c->device));
    TRY(materialize(c));
    hipStream_t st = c->stream;
    if (refs && c->n_out) HIP_TRY(c, hipMemcpyAsync(refs, c->out_ptr, c->n_out * 4, hipMemcpyDeviceToHost, st));
    if (runoff) HIP_TRY(c, hipMemcpyAsync(runoff, c->runoff.p, (c->n_runs + 1) * 8, hipMemcpyDeviceToHost, st));
    if (rundep && c->n_runs) HIP_TRY(c, hipMemcpyAsync(rundep, c->rundep.p, c->n_runs * 4, hipMemcpyDeviceToHost, st));
    if (capture_ids && c->C) HIP_TRY(c, hipMemcpyAsync(capture_ids, c->fext.p, (u64)c->C * 4, hipMemcpyDeviceToHost, st));
    if (supports && c->C) HIP_TRY(c, hipMemcpyAsync(supports, c->csup.p, (u64)c->C * 4, hipMemcpyDeviceToHost, st));
    HIP_TRY(c, hipStreamSynchronize(st));
    return RDF_OK;
}

// Cind-shaped rows on the device (decode kernel), copied to the caller in chunks
rdf_status rdf_copy_cinds_decoded(rdf_ctx* c, uint64_t offset, rdf_cind_row* out, uint64_t count, uint64_t* n_copied) {
    if (!c || (count && !out)) return RDF_ERR_ARG;
    if (c->stage < 4) return fail(c, RDF_ERR_STATE, "rdf_discover_cinds must be called first");
    HIP_TRY(c, hipSetDevice(c->device));
    TRY(materialize(c));
    const u64 m = offset >= c->n_out ? 0 : std::min<u64>(count, c->n_out - offset);
    const u64 kChunk = 1ull << 22;
    if (m) ENSURE(c, drows, std::min<u64>(m, kChunk) * sizeof(rdf_cind_row));
    for (u64 b = 0; b < m; b += kChunk) {
        const u64 k = std::min(kChunk, m - b);
        hipLaunchKernelGGL(k_decode_rows, dim3(grid_for(k, RDF_BLOCK, kGrid)), dim3(RDF_BLOCK), 0, c->stream, c->out_ptr,
                           offset + b, k, c->runoff.as<u64>(), c->rundep.as<u32>(), c->n_runs, c->fext.as<u32>(),
                           c->csup.as<u32>(), c->V ? c->V : 1u, c->bkeys.as<u64>(), c->drows.as<u32>());
        HIP_TRY(c, hipGetLastError());
        HIP_TRY(c, hipMemcpyAsync(out + b, c->drows.p, k * sizeof(rdf_cind_row), hipMemcpyDeviceToHost, c->stream));
        HIP_TRY(c, hipStreamSynchronize(c->stream));  // drows is reused by the next chunk
    }
    if (n_copied) *n_copied = m;
    return RDF_OK;
}

rdf_status rdf_cind_checksum(rdf_ctx* c, uint64_t* checksum) {
    if (!c || !checksum) return RDF_ERR_ARG;
    if (c->stage < 4) return fail(c, RDF_ERR_STATE, "rdf_discover_cinds must be called first");
    HIP_TRY(c, hipSetDevice(c->device));
    TRY(materialize_heavy(c));
    HIP_TRY(c, hipMemsetAsync(dscal(c, 7), 0, 8, c->stream));
    // a pending class part is summed from the compact form (no expansion: 4 B per row of HBM it would need)
    const u64 nrows = c->class_pending ? c->n_out - c->n_class_out : c->n_out;
    if (nrows)
        hipLaunchKernelGGL(k_checksum, dim3(grid_for(nrows, RDF_BLOCK, kGrid)), dim3(RDF_BLOCK), 0, c->stream,
                           c->out_ptr, nrows, c->runoff.as<u64>(), c->rundep.as<u32>(), c->n_runs, c->fext.as<u32>(),
                           c->csup.as<u32>(), dscal(c, 7));
    if (c->class_pending && c->pend_NT)
        hipLaunchKernelGGL(k_class_checksum, dim3(vgrid(c->pend_NT)), dim3(RDF_BLOCK), 0, c->stream, c->pend_NT,
                           c->coff.as<u64>(), c->cchoff.as<u64>(), c->lwoff.as<u64>(), c->clists.as<u32>(),
                           c->ctoff.as<u64>(), (u32)c->n_classes, c->ckeys.as<u64>(), c->fext.as<u32>(),
                           c->csup.as<u32>(), dscal(c, 7));
    HIP_TRY(c, hipGetLastError());
    u64 v = 0;
    rdf_status rs = read_u64(c, dscal(c, 7), &v);
    *checksum = v;
    return rs;
}

// ------------------------------------------------------------------------------------------------
// Output formatting (K8): Cind.toString lines on the device from the caller's dictionary

rdf_status rdf_set_dictionary(rdf_ctx* c, const char* heap, uint64_t heap_bytes, const uint64_t* offsets,
                              uint64_t n_terms) {
    if (!c || (heap_bytes && !heap) || !offsets) return RDF_ERR_ARG;
    if (offsets[n_terms] != heap_bytes) return fail(c, RDF_ERR_ARG, "offsets[n_terms] must equal heap_bytes");
    HIP_TRY(c, hipSetDevice(c->device));
    ENSURE(c, dheap, std::max<u64>(heap_bytes, 1));
    ENSURE(c, dtoff, (n_terms + 1) * 8);
    if (heap_bytes) HIP_TRY(c, ctx_copy(c, c->dheap.p, heap, heap_bytes, hipMemcpyHostToDevice));
    HIP_TRY(c, ctx_copy(c, c->dtoff.p, offsets, (n_terms + 1) * 8, hipMemcpyHostToDevice));
    c->dict_terms = n_terms;
    c->capstr_run = ~0ull;
    return RDF_OK;
}

// The dictionary of the last rdf_parse_ntriples as the formatting dictionary, built in HBM (no host copy).
rdf_status rdf_set_dictionary_parsed(rdf_ctx* c) {
    if (!c) return RDF_ERR_ARG;
    if (!c->parsed_dict) return fail(c, RDF_ERR_STATE, "the resident triples do not come from rdf_parse_ntriples");
    HIP_TRY(c, hipSetDevice(c->device));
    hipStream_t st = c->stream;
    const u64 V = c->n_terms_parsed;
    ENSURE(c, dtoff, (V + 1) * 8);
    HIP_TRY(c, exclusive_scan_u32_u64(c->ws, c->nterm_len.as<u32>(), c->dtoff.as<u64>(), V, c->dtoff.as<u64>() + V, st));
    u64 total = 0;
    TRY(read_u64(c, c->dtoff.as<u64>() + V, &total));
    ENSURE(c, dheap, std::max<u64>(total, 1));
    if (V)
        hipLaunchKernelGGL(k_nt_dict_gather, dim3(grid_for(V, RDF_BLOCK, kGrid)), dim3(RDF_BLOCK), 0, st,
                           (const unsigned char*)c->ntext.p, c->nterm_off.as<u64>(), c->dtoff.as<u64>(), V,
                           c->dheap.as<char>());
    HIP_TRY(c, hipGetLastError());
    HIP_TRY(c, hipStreamSynchronize(st));
    c->dict_terms = V;
    c->capstr_run = ~0ull;
    return RDF_OK;
}

// pretty strings of the run's compact captures (built once per run)
static rdf_status ensure_capstr(rdf_ctx* c) {
    if (c->stage < 4) return fail(c, RDF_ERR_STATE, "rdf_discover_cinds must be called first");
    if (c->dict_terms < c->V) return fail(c, RDF_ERR_STATE, "rdf_set_dictionary must cover every term id");
    if (c->capstr_run == c->run_id) return RDF_OK;
    hipStream_t st = c->stream;
    const u32 C = c->C;
    ENSURE(c, cslen, std::max<u64>(C, 1) * 4);
    ENSURE(c, csoff, (C + 1ull) * 8);
    if (C)
        hipLaunchKernelGGL(k_capstr_len, dim3(grid_for(C, RDF_BLOCK, kGrid)), dim3(RDF_BLOCK), 0, st, c->fext.as<u32>(), C,
                           c->V, c->bkeys.as<u64>(), c->dtoff.as<u64>(), c->cslen.as<u32>());
    HIP_TRY(c, exclusive_scan_u32_u64(c->ws, c->cslen.as<u32>(), c->csoff.as<u64>(), C, c->csoff.as<u64>() + C, st));
    u64 total = 0;
    TRY(read_u64(c, c->csoff.as<u64>() + C, &total));
    ENSURE(c, cstr, std::max<u64>(total, 1));
    if (C)
        hipLaunchKernelGGL(k_capstr_write, dim3(grid_for(C, RDF_WAVES_PER_BLOCK, kGrid)), dim3(RDF_BLOCK), 0, st,
                           c->fext.as<u32>(), C, c->V, c->bkeys.as<u64>(), c->dtoff.as<u64>(), c->dheap.as<char>(),
                           c->csoff.as<u64>(), c->cstr.as<char>());
    c->capstr_run = c->run_id;
    return RDF_OK;
}

// line offsets of result rows [offset, offset + m) -> floff, *bytes
static rdf_status fmt_prepare(rdf_ctx* c, u64 offset, u64 m, u64* bytes) {
    hipStream_t st = c->stream;
    TRY(materialize(c));
    TRY(ensure_capstr(c));
    ENSURE(c, flen, std::max<u64>(m, 1) * 4);
    ENSURE(c, floff, (m + 1) * 8);
    if (m)
        hipLaunchKernelGGL(k_fmt_len, dim3(grid_for(m, RDF_BLOCK, kGrid)), dim3(RDF_BLOCK), 0, st, c->out_ptr, offset, m,
                           c->runoff.as<u64>(), c->rundep.as<u32>(), c->n_runs, c->csoff.as<u64>(), c->csup.as<u32>(),
                           c->flen.as<u32>());
    HIP_TRY(c, exclusive_scan_u32_u64(c->ws, c->flen.as<u32>(), c->floff.as<u64>(), m, c->floff.as<u64>() + m, st));
    return read_u64(c, c->floff.as<u64>() + m, bytes);
}

rdf_status rdf_format_size(rdf_ctx* c, uint64_t offset, uint64_t count, uint64_t* bytes) {
    if (!c || !bytes) return RDF_ERR_ARG;
    if (c->stage < 4) return fail(c, RDF_ERR_STATE, "rdf_discover_cinds must be called first");
    HIP_TRY(c, hipSetDevice(c->device));
    const u64 m = offset >= c->n_out ? 0 : std::min<u64>(count, c->n_out - offset);
    return fmt_prepare(c, offset, m, (u64*)bytes);
}

rdf_status rdf_format_cinds(rdf_ctx* c, uint64_t offset, uint64_t count, char* out, uint64_t cap, uint64_t* bytes) {
    if (!c || !bytes || (cap && !out)) return RDF_ERR_ARG;
    if (c->stage < 4) return fail(c, RDF_ERR_STATE, "rdf_discover_cinds must be called first");
    HIP_TRY(c, hipSetDevice(c->device));
    const u64 m = offset >= c->n_out ? 0 : std::min<u64>(count, c->n_out - offset);
    u64 total = 0;
    TRY(fmt_prepare(c, offset, m, &total));
    *bytes = total;
    if (total > cap) return fail(c, RDF_ERR_ARG, "output buffer too small (see *bytes)");
    ENSURE(c, fbuf, std::max<u64>(total, 1));
    if (m)
        hipLaunchKernelGGL(k_fmt_write, dim3(grid_for((m + RDF_WAVE - 1) / RDF_WAVE, RDF_WAVES_PER_BLOCK, kGrid)),
                           dim3(RDF_BLOCK), 0, c->stream, c->out_ptr, offset, m, c->runoff.as<u64>(), c->rundep.as<u32>(),
                           c->n_runs, c->csoff.as<u64>(), c->cstr.as<char>(), c->csup.as<u32>(), c->floff.as<u64>(),
                           c->fbuf.as<char>());
    HIP_TRY(c, hipGetLastError());
    if (total) HIP_TRY(c, hipMemcpyAsync(out, c->fbuf.p, total, hipMemcpyDeviceToHost, c->stream));
    HIP_TRY(c, hipStreamSynchronize(c->stream));
    return RDF_OK;
}

rdf_status rdf_decode_capture(rdf_ctx* c, uint32_t capture, uint32_t* code, uint32_t* value1, uint32_t* value2) {
    if (!c || !code || !value1 || !value2) return RDF_ERR_ARG;
    static const uint32_t UN[6] = {10, 12, 17, 20, 33, 34}, BI[3] = {14, 21, 35};
    const u64 V = c->V ? c->V : 1;
    if (capture < 6 * V) {
        *code = UN[capture / V];
        *value1 = (u32)(capture % V);
        *value2 = 0xffffffffu;
        return RDF_OK;
    }
    const u64 b = capture - 6 * V;
    TRY(load_bkeys(c));
    if (b >= c->h_bkeys.size()) return fail(c, RDF_ERR_ARG, "capture id out of range");
    const u64 k = c->h_bkeys[b];
    *code = BI[bin_key_type(k)];
    *value1 = bin_key_v1(k);
    *value2 = bin_key_v2(k);
    return RDF_OK;
}

rdf_status rdf_binary_key_count(rdf_ctx* c, uint64_t* n) {
    if (!c || !n) return RDF_ERR_ARG;
    *n = c->B;
    return RDF_OK;
}

rdf_status rdf_copy_binary_keys(rdf_ctx* c, uint64_t* out, uint64_t cap) {
    if (!c || (cap && !out)) return RDF_ERR_ARG;
    TRY(load_bkeys(c));
    const u64 m = std::min<u64>(cap, c->h_bkeys.size());
    if (m) memcpy(out, c->h_bkeys.data(), m * 8);
    return RDF_OK;
}

rdf_status rdf_kernel_times(rdf_ctx* c, float* ms, int count) {
    if (!c || !ms || count < 0) return RDF_ERR_ARG;
    settle_timings(c);
    for (int i = 0; i < count; ++i) ms[i] = i < RDF_NUM_TIMERS ? c->tms[i] : 0.f;
    return RDF_OK;
}

rdf_status rdf_stage_times(rdf_ctx* c, float* ms3) {
    if (!c || !ms3) return RDF_ERR_ARG;
    settle_timings(c);
    for (int i = 0; i < 3; ++i) ms3[i] = c->stage_ms[i];
    return RDF_OK;
}

}  // extern "C"
