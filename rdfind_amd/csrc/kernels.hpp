// Kernel declarations for the CIND-discovery pipeline.
#pragma once
#include "common.hpp"

namespace rdf {

static constexpr int LH_SLOTS = 4096;     // LDS hash slots (u32 keys) for unary counting
static constexpr int LB_SLOTS = 2048;     // LDS hash slots (u64 keys) for binary counting
static constexpr int HMAX = 64;           // heavy groups tracked as bit columns (one u64 per capture)
static constexpr uint8_t LIGHT = 0xff;
static constexpr u32 DGRP_HEAVY = 0x80000000u;
static constexpr u32 GINFO_HEAVY = 0x80000000u;  // ginfo[g] = member count | this bit for heavy groups  // tag of a dependent -> group entry whose group is heavy
#ifndef RDF_LIGHT_SEG
#define RDF_LIGHT_SEG 2048
#endif
static constexpr u64 LIGHT_SEG = RDF_LIGHT_SEG;  // groups of one dependent verified by one light work item
#ifndef RDF_LIGHT_IT
#define RDF_LIGHT_IT 4
#endif
static constexpr int LIGHT_IT = RDF_LIGHT_IT;  // groups per lane whose metadata is loaded together
#ifndef RDF_SIG_W
#define RDF_SIG_W 8
#endif
// Light-group signatures: bit h(g) of a 64*SIG_W-bit word set for every light group g of a capture.  G(d) <= G(c)
// implies sig(d) <= sig(c), so a candidate whose signature misses a bit of the dependent's is not a ref; this kills
// most doomed candidates before any group search (the heavy groups are exact bits of hmask already).
static constexpr int SIG_W = RDF_SIG_W;
static constexpr int SIG_LOG = SIG_W == 16 ? 10 : SIG_W == 8 ? 9 : SIG_W == 4 ? 8 : SIG_W == 2 ? 7 : 6;
static_assert((1 << (SIG_LOG - 6)) == SIG_W, "SIG_W must be 1, 2, 4, 8 or 16");
// Light groups checked one at a time (lanes over candidates) after the second pivot and before the windows: the
// pivot pass stores PIV_EXTRA of them per dependent (the next smallest), the plain light variant checks v.npx of them.
// One on the plain variant's inputs, all four on the high-occupancy ones (large groups, long items: c4), whose pivot
// pass keeps them; measured in profiles/r04_light_ab_pivots.log (c4 at 0.4 light 157.5 -> 121.3 ms with one, 98.9 with
// four; c3 full 29.7 -> 27.2 with one but 31.5 with four; c2, which runs the staging variant, none)
static constexpr int PIV_EXTRA = 4;
static constexpr int PIV_EXTRA_PLAIN = 1;
// the pivot pass keeps PIV_EXTRA (else PIV_EXTRA_PLAIN) from this weighted mean light group up on inputs with at
// least PIVX_GPC groups per capture (the light variant's choice comes later; these predict it: c4 45-51, c3 15)
static constexpr u64 PIVX_WMEAN = 2048;
static constexpr u64 PIVX_GPC = 32;
static constexpr u64 LIGHT_PACK_MAXG = 32;  // dependents with at most this many groups take the packed light path
#ifndef RDF_PACK_MAXG2
#define RDF_PACK_MAXG2 512
#endif
#ifndef RDF_PACK_NL
#define RDF_PACK_NL 16
#endif
static constexpr u64 LIGHT_PACK_MAXG2 = RDF_PACK_MAXG2;  // ... and those with at most this many groups of
static constexpr u32 LIGHT_PACK_NL = RDF_PACK_NL;        // which at most this many are light
#ifndef RDF_LIGHT_BATCH
#define RDF_LIGHT_BATCH 4  // 8 before round 5: c2 light 2.52 -> 2.21 ms, c3 at 0.5 7.33 -> 7.12, c4 at 0.4 64.2 -> 60.1 (profiles/r05_light_ab_batch.log)
#endif
static constexpr int LIGHT_BATCH = RDF_LIGHT_BATCH;  // candidates searched together in k_light
#ifndef RDF_LIGHT_ORDER_MIN
#define RDF_LIGHT_ORDER_MIN 128
#endif
static constexpr u64 LIGHT_ORDER_MIN = RDF_LIGHT_ORDER_MIN;  // light-group entries from which a dependent's items go first
#ifndef RDF_LIGHT_DENSE_BATCH
#define RDF_LIGHT_DENSE_BATCH 8
#endif
static constexpr int LIGHT_DENSE_BATCH = RDF_LIGHT_DENSE_BATCH;  // dense groups' bitmap words in flight per lane (k_light)
#ifndef RDF_LIGHT_SERIAL
#define RDF_LIGHT_SERIAL 4
#endif
static constexpr int LIGHT_SERIAL = RDF_LIGHT_SERIAL;  // windows with at most this many light groups: lanes over candidates
static constexpr u32 LIGHT_LDS = 512;
// Dense light groups also get an exact bitmap over the compact capture space (C bits): a (candidate, group) test is one
// 4-B load instead of a ~log2(n)-level divergent search.  Threshold (d_dense_flags): C / DENSE_DIV_STAGE members for the
// staging light variant (c2: a row no larger than its member list), else min(C / 32, DENSE_MIN_ABS) members (a row up
// to C / (4 DENSE_MIN_ABS) times its list); at least LIGHT_DENSE_MIN; at most DENSE_BYTES of rows and half the free
// HBM.  Measured light ms at thresholds of C / 32 | C / 128 | C / 512 | C / 1024 members: c3 26.8 | 21.8 | 18.1 | 17.7
// (C / 1024 = 1,452), c4 at 0.4 101 | 80.3 | 64.1 (C / 512 = 2,036) | -, c4 at 0.05 10.8 | 7.7 (1,293) | - | 12.0 (256),
// c5 at 0.1 18.2 | 15.3 | 15.1 | 15.1 (profiles/r04_dense_ab.log, r04_dense_div_ab.log): ~2k members is near the best
// everywhere.
static constexpr u64 LIGHT_DENSE_MIN = 256;
static constexpr int DENSE_DIV_STAGE = 32;
static constexpr u64 DENSE_MIN_ABS = 2048;
static constexpr u64 DENSE_BYTES = 8ull << 30;
#ifndef RDF_DENSE_SER
#define RDF_DENSE_SER 8
#endif
static constexpr int LIGHT_DENSE_SER = RDF_DENSE_SER;  // alive candidates from which dense groups go lanes-over-candidates
#ifndef RDF_LIGHT_SMALL
#define RDF_LIGHT_SMALL 31
#endif
#ifndef RDF_STAGE_MIN
#define RDF_STAGE_MIN 3
#endif
// windows whose light groups all have <= LIGHT_SMALL members are staged into per-lane LDS rows once at least
// LIGHT_STAGE_MIN candidates are alive (LIGHT_STAGE_MIN > 64 turns it off)
static constexpr u32 LIGHT_SMALL = RDF_LIGHT_SMALL;  // odd: also the row stride (conflict-free banks)
static_assert(LIGHT_SMALL % 2 == 1, "LIGHT_SMALL is the LDS row stride and must be odd");
static constexpr u32 LIGHT_BUF = LIGHT_LDS > 64 * LIGHT_SMALL ? LIGHT_LDS : 64 * LIGHT_SMALL;  // u32 per wave
static constexpr int LIGHT_STAGE_MIN = RDF_STAGE_MIN;
#ifndef RDF_STAGE_AVG
#define RDF_STAGE_AVG 48
#endif
// k_light_plain_hi (6 waves per SIMD) when the member-weighted mean light group has >= LIGHT_HIOCC_AVG members AND
// the light work has >= LIGHT_HIOCC_OCT output octets per capture (long, latency-bound items: many candidates per
// dependent searched in large groups).  Measured (profiles/r04_light_ab_hiocc.log): c4 at 0.05 (2,674 / 59) light
// 11.2 -> 10.5 ms, c4 at 0.4 (13,560 / 55) 182 -> 160 ms; c3 at 0.5 (4,719 / 9.7) 10.6 -> 11.5 and c1 (412 / 68)
// 0.96 -> 1.10 lose, c5 at 0.1 (1,291 / 232) is flat, so both conditions must hold.
static constexpr u64 LIGHT_HIOCC_AVG = 2048;
static constexpr u64 LIGHT_HIOCC_OCT = 32;
static constexpr u64 LIGHT_STAGE_AVG = RDF_STAGE_AVG;  // staging variant when the weighted mean light group is smaller
                  // groups up to this size are searched in LDS (2 KiB per wave)

#ifndef RDF_SWEEP_F
#define RDF_SWEEP_F 32
#endif
#ifndef RDF_SWEEP_MIN
#define RDF_SWEEP_MIN 16
#endif
static constexpr int LIGHT_SWEEP_F = RDF_SWEEP_F;      // default of CindView::sweep_f (RDFIND_SWEEP_F)
static constexpr int LIGHT_SWEEP_MIN = RDF_SWEEP_MIN;  // alive candidates from which a window may be swept

#ifndef RDF_EMIT_DEDUP_SLOTS
#define RDF_EMIT_DEDUP_SLOTS 2048  // 4096: c2 emit 1.05 ms, 2048: 0.93 (more blocks per CU)
#endif
static constexpr int EMIT_DEDUP_SLOTS = RDF_EMIT_DEDUP_SLOTS;  // K3 write pass: LDS hash of one iteration's repeating
                                                               // records (<= 4 x 256)
static constexpr u64 EMIT_PAD = ~0ull;         // K3 padding of removed duplicates (no record has all bits set)
static constexpr u32 PRE_TAG = 0x80000000u;  // light pass A: an unverified survivor (ref bit 31; compact ids < 2^31)
#ifndef RDF_PRE_MAX
#define RDF_PRE_MAX 64
#endif
static constexpr int LIGHT_PRE_MAX = RDF_PRE_MAX;  // pass A defers chunks with at most this many candidates left (64: all)

// per frequent capture (compact id) metadata, 16 bytes, one dwordx4 load
struct __align__(16) CapInfo {
    u64 hmask;     // bit j set <=> capture is in heavy group j
    u32 support;   // number of capture groups containing it (distinct join values)
    u32 meta;      // bit0 binary, bit1 has parents, bit2 heavy-only
};
static constexpr u32 META_BIN = 1u, META_PARENTS = 2u, META_HEAVY_ONLY = 4u;

// Rule modes for K7 (TraversalStrategy.removeImpliedCinds, TraversalStrategy.scala:126-168)
enum RuleMode : int { RULES_NONE = 0, RULES_S2L_RAW = 1, RULES_CLEAN = 2 };
// --use-ars on the discovery side (ars.inl ar_drop): strategy 0 drops the AR-implied 1/1 CINDs, S2L also the larger
// CINDs its candidate generation cannot reach without them
enum ArMode : int { AR_NONE = 0, AR_S0 = 1, AR_S2L = 2 };

struct CindView {
    // compact capture space [0, C); unary compact ids are [0, Cu), binary [Cu, C)
    u32 C, Cu;
    const CapInfo* info;
    const u32* gcap;      // group members (compact ids), sorted within a group
    const u64* goff;      // group offsets [G+1]
    const uint8_t* hbit;  // heavy bit of a group or LIGHT
    const u64* doff;      // dependent -> groups offsets [C+1]
    const u32* dgrp;      // dependent -> group ids
    const u32* bcomp;     // binary compact id b: components at [2*(b-Cu)], [2*(b-Cu)+1]
    const u64* bkeyc;     // binary compact id b: bin key (bt, v1, v2)
    const u64* poff;      // unary compact id -> parents offsets [Cu+1]
    const u32* plist;     // parents (binary compact ids)
    const u64* eoff;      // explicit CSR: dep -> refs [C+1]
    const u64* epairs;    // explicit (dep << 32 | ref) pairs, sorted
    const u64* ebin;      // first explicit pair of a dep whose ref is binary
    int literal;          // strategy-0 Condition.isImpliedBy quirk
    int mode;             // RuleMode
    const u64* vcoff;     // sharded verify pass: dependent -> offsets [C+1] into vpairs (null: pivot candidates)
    const u64* vpairs;    // (dep << 32 | candidate) pairs sorted, the global pivot holder's survivors to verify
    int ar;               // ArMode (--use-ars)
    const u32* arref;     // unary compact id -> the ref its association rule implies, or NONE32 [Cu]
    const u64* sig;       // light-group signature of each capture, SIG_W words (null: no signature test)
    const u32* ginfo;     // group -> member count | GINFO_HEAVY (k_group_info)
    const u32* piv2;      // dependent -> its smallest light group other than the pivot (NONE32: none / not computed)
    const u32* pivx;      // ... the next smallest, [d * PIV_EXTRA + k] (k_light plain only; NONE32: none)
    int npx;              // how many of them k_light checks (<= PIV_EXTRA)
    const u32* gdrow;     // group -> row of its exact member bitmap (dense light groups), NONE32 (null: no bitmaps)
    const u32* dbits;     // dense-group bitmaps: row r at dbits + r * dwords, bit x set iff capture x is a member
    u64 dwords;
    int prefilter;        // light pass A: dependents of several chunks only filtered (survivors tagged PRE_TAG)
    int p2done;           // light pass B: the given candidates already passed the second pivot
    int sweep_f;          // k_light range sweep: a window's groups are swept when their members in the alive candidates'
                          // value range number <= sweep_f x alive x log2(mean group size) (0: never)
};

}  // namespace rdf
