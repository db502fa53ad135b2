// CIND-discovery kernels (included by rdfind_hip.hip).
//
// Abbreviation: ALG/ = rdfind-algorithm/src/main/scala/de/hpi/isg/sodap/rdfind/ in the reference.
// Each kernel names the reference operator whose semantics it implements.
#include "kernels.hpp"

namespace rdf {

// ================================================================================================
// K1: unary condition counts  (FrequentConditionPlanner.findFrequentSingleConditions,
//     ALG/plan/FrequentConditionPlanner.scala:488-508: flatMap 3 x (type, value, 1) -> groupBy.sum)
// Keys are type*V + value.  Per-block LDS hash table pre-aggregates hot keys (Zipf predicates /
// classes) so only one global atomic per distinct key per block remains; table misses go global.

__device__ inline void lds_count_u32(u32* lkey, u32* lcnt, u32 key, u32* gcnt) {
    u32 h = hash32(key) & (LH_SLOTS - 1);
#pragma unroll 1
    for (int probe = 0; probe < 8; ++probe) {
        u32 k = lkey[h];
        if (k == key) {
            atomicAdd(&lcnt[h], 1u);
            return;
        }
        if (k == EMPTY32) {
            u32 prev = atomicCAS(&lkey[h], EMPTY32, key);
            if (prev == EMPTY32 || prev == key) {
                atomicAdd(&lcnt[h], 1u);
                return;
            }
        }
        h = (h + 1) & (LH_SLOTS - 1);
    }
    atomicAdd(&gcnt[key], 1u);
}

__global__ __launch_bounds__(RDF_BLOCK) void k_unary_count(const u32* __restrict__ s, const u32* __restrict__ p,
                                                           const u32* __restrict__ o, u64 n, u32 V, u32* cnt) {
    __shared__ u32 lkey[LH_SLOTS];
    __shared__ u32 lcnt[LH_SLOTS];
    for (int i = threadIdx.x; i < LH_SLOTS; i += RDF_BLOCK) {
        lkey[i] = EMPTY32;
        lcnt[i] = 0;
    }
    __syncthreads();
    const u64 stride = (u64)gridDim.x * RDF_BLOCK;
    for (u64 i = (u64)blockIdx.x * RDF_BLOCK + threadIdx.x; i < n; i += stride) {
        lds_count_u32(lkey, lcnt, s[i], cnt);
        lds_count_u32(lkey, lcnt, V + p[i], cnt);
        lds_count_u32(lkey, lcnt, 2u * V + o[i], cnt);
    }
    __syncthreads();
    for (int i = threadIdx.x; i < LH_SLOTS; i += RDF_BLOCK)
        if (lkey[i] != EMPTY32) atomicAdd(&cnt[lkey[i]], lcnt[i]);
}

// number of frequent values per condition type (for stats)
__global__ __launch_bounds__(RDF_BLOCK) void k_count_frequent(const u32* __restrict__ cnt, u32 V, u32 ms, u64* out3) {
    const u64 total = 3ull * V;
    u32 c[3] = {0, 0, 0};
    for (u64 i = (u64)blockIdx.x * RDF_BLOCK + threadIdx.x; i < total; i += (u64)gridDim.x * RDF_BLOCK)
        if (cnt[i] >= ms) c[i / V]++;
    for (int t = 0; t < 3; ++t) {
        u32 w = wave_sum(c[t]);
        if (lane_id() == 0 && w) atomicAdd(&out3[t], (u64)w);
    }
}

// ================================================================================================
// K2: binary condition counts  (CreatedReducedDoubleConditionCounts.flatMap,
//     ALG/operators/candidate_extraction/CreatedReducedDoubleConditionCounts.scala:45-86, + groupBy.sum
//     FrequentConditionPlanner.scala:571-591).  Only triples with >= 2 frequent values emit sp/so/po.

__device__ inline void freq_flags(const u32* cnt, u32 V, u32 ms, u32 s, u32 p, u32 o, bool& fs, bool& fp, bool& fo) {
    fs = cnt[s] >= ms;
    fp = cnt[V + p] >= ms;
    fo = cnt[2u * V + o] >= ms;
}

__global__ __launch_bounds__(RDF_BLOCK) void k_binary_emit_count(const u32* __restrict__ s, const u32* __restrict__ p,
                                                                 const u32* __restrict__ o, u64 n, u32 V, u32 ms,
                                                                 const u32* __restrict__ cnt, u64* total) {
    u32 c = 0;
    for (u64 i = (u64)blockIdx.x * RDF_BLOCK + threadIdx.x; i < n; i += (u64)gridDim.x * RDF_BLOCK) {
        bool fs, fp, fo;
        freq_flags(cnt, V, ms, s[i], p[i], o[i], fs, fp, fo);
        c += (fs && fp) + (fs && fo) + (fp && fo);
    }
    c = wave_sum(c);
    if (lane_id() == 0 && c) atomicAdd(total, (u64)c);
}

__device__ inline void global_hash_add(u64* tkeys, u32* tcnt, u64 mask, u64 key, u32 c) {
    u64 h = mix64(key) & mask;
    for (;;) {
        u64 k = tkeys[h];
        if (k == key) {
            atomicAdd(&tcnt[h], c);
            return;
        }
        if (k == EMPTY64) {
            u64 prev = atomicCAS(&tkeys[h], EMPTY64, key);
            if (prev == EMPTY64 || prev == key) {
                atomicAdd(&tcnt[h], c);
                return;
            }
        }
        h = (h + 1) & mask;
    }
}

__device__ inline void lds_count_u64(u64* lkey, u32* lcnt, u64 key, u64* tkeys, u32* tcnt, u64 tmask) {
    u32 h = (u32)mix64(key) & (LB_SLOTS - 1);
#pragma unroll 1
    for (int probe = 0; probe < 8; ++probe) {
        u64 k = lkey[h];
        if (k == key) {
            atomicAdd(&lcnt[h], 1u);
            return;
        }
        if (k == EMPTY64) {
            u64 prev = atomicCAS(&lkey[h], EMPTY64, key);
            if (prev == EMPTY64 || prev == key) {
                atomicAdd(&lcnt[h], 1u);
                return;
            }
        }
        h = (h + 1) & (LB_SLOTS - 1);
    }
    global_hash_add(tkeys, tcnt, tmask, key, 1u);
}

__global__ __launch_bounds__(RDF_BLOCK) void k_binary_count(const u32* __restrict__ s, const u32* __restrict__ p,
                                                            const u32* __restrict__ o, u64 n, u32 V, u32 ms,
                                                            const u32* __restrict__ cnt, u64* tkeys, u32* tcnt,
                                                            u64 tmask) {
    __shared__ u64 lkey[LB_SLOTS];
    __shared__ u32 lcnt[LB_SLOTS];
    for (int i = threadIdx.x; i < LB_SLOTS; i += RDF_BLOCK) {
        lkey[i] = EMPTY64;
        lcnt[i] = 0;
    }
    __syncthreads();
    const u64 stride = (u64)gridDim.x * RDF_BLOCK;
    for (u64 i = (u64)blockIdx.x * RDF_BLOCK + threadIdx.x; i < n; i += stride) {
        u32 ts = s[i], tp = p[i], to = o[i];
        bool fs, fp, fo;
        freq_flags(cnt, V, ms, ts, tp, to, fs, fp, fo);
        if (fs && fp) lds_count_u64(lkey, lcnt, bin_key(2, ts, tp), tkeys, tcnt, tmask);   // o[s,p] (35)
        if (fs && fo) lds_count_u64(lkey, lcnt, bin_key(1, ts, to), tkeys, tcnt, tmask);   // p[s,o] (21)
        if (fp && fo) lds_count_u64(lkey, lcnt, bin_key(0, tp, to), tkeys, tcnt, tmask);   // s[p,o] (14)
    }
    __syncthreads();
    for (int i = threadIdx.x; i < LB_SLOTS; i += RDF_BLOCK)
        if (lkey[i] != EMPTY64) global_hash_add(tkeys, tcnt, tmask, lkey[i], lcnt[i]);
}

// frequent binary conditions: filter >= minSupport (FrequentConditionPlanner.scala:587-589)
__global__ __launch_bounds__(RDF_BLOCK) void k_bin_freq_flags(const u64* __restrict__ tkeys, const u32* __restrict__ tcnt,
                                                              u64 cap, u32 ms, u32* flags) {
    for (u64 i = (u64)blockIdx.x * RDF_BLOCK + threadIdx.x; i < cap; i += (u64)gridDim.x * RDF_BLOCK)
        flags[i] = (tkeys[i] != EMPTY64 && tcnt[i] >= ms) ? 1u : 0u;
}

__global__ __launch_bounds__(RDF_BLOCK) void k_bin_freq_scatter(const u64* __restrict__ tkeys, const u32* __restrict__ flags,
                                                                const u64* __restrict__ pos, u64 cap, u64* out) {
    for (u64 i = (u64)blockIdx.x * RDF_BLOCK + threadIdx.x; i < cap; i += (u64)gridDim.x * RDF_BLOCK)
        if (flags[i]) out[pos[i]] = tkeys[i];
}

__global__ __launch_bounds__(RDF_BLOCK) void k_count_nonempty(const u64* __restrict__ tkeys, u64 cap, u64* total) {
    u32 c = 0;
    for (u64 i = (u64)blockIdx.x * RDF_BLOCK + threadIdx.x; i < cap; i += (u64)gridDim.x * RDF_BLOCK)
        c += tkeys[i] != EMPTY64;
    c = wave_sum(c);
    if (lane_id() == 0 && c) atomicAdd(total, (u64)c);
}

// lookup table of frequent binary keys -> index b (keys sorted, so b is deterministic)
__global__ __launch_bounds__(RDF_BLOCK) void k_bin_lookup_build(const u64* __restrict__ bkeys, u64 B, u64* lkeys, u32* lvals,
                                                                u64 mask) {
    for (u64 b = (u64)blockIdx.x * RDF_BLOCK + threadIdx.x; b < B; b += (u64)gridDim.x * RDF_BLOCK) {
        u64 key = bkeys[b];
        u64 h = mix64(key) & mask;
        for (;;) {
            u64 prev = atomicCAS(&lkeys[h], EMPTY64, key);
            if (prev == EMPTY64) {
                lvals[h] = (u32)b;
                break;
            }
            h = (h + 1) & mask;
        }
    }
}

__device__ inline u32 bin_lookup(const u64* lkeys, const u32* lvals, u64 mask, u64 key) {
    u64 h = mix64(key) & mask;
    for (;;) {
        u64 k = lkeys[h];
        if (k == key) return lvals[h];
        if (k == EMPTY64) return NONE32;
        h = (h + 1) & mask;
    }
}

// ================================================================================================
// K3: join partners  (CreateJoinPartners.flatMap, ALG/operators/CreateJoinPartners.scala:86-147)
// Per triple and projection: unary captures of the frequent condition values and, when the binary
// condition is frequent, the binary capture.  Binary captures are emitted together with both unary
// components, which is what every consumer reconstructs (CreateDependencyCandidates.scala:157-186,
// splitAndCollectUnaryCaptures).  Record = join << capbits | capture id.

__global__ __launch_bounds__(RDF_BLOCK) void k_emit_records(const u32* __restrict__ s, const u32* __restrict__ p,
                                                            const u32* __restrict__ o, u64 n, u32 V, u32 ms,
                                                            const u32* __restrict__ cnt, const u64* __restrict__ lkeys,
                                                            const u32* __restrict__ lvals, u64 lmask, int proj,
                                                            int capbits, u64* out, u64* counter) {
    const u64 stride = (u64)gridDim.x * RDF_BLOCK;
    const u64 n_round = (n + RDF_WAVE - 1) / RDF_WAVE * RDF_WAVE;  // all lanes of a wave iterate together
    const u64 B6 = 6ull * V;
    for (u64 i = (u64)blockIdx.x * RDF_BLOCK + threadIdx.x; i < n_round; i += stride) {
        u64 rec[9];
        u32 c = 0;
        if (i < n) {
            const u32 ts = s[i], tp = p[i], to = o[i];
            bool fs, fp, fo;
            freq_flags(cnt, V, ms, ts, tp, to, fs, fp, fo);
            if (proj & 4) {  // project objects: o[s], o[p], o[s,p]
                const u64 j = (u64)to << capbits;
                if (fs) rec[c++] = j | (4ull * V + ts);
                if (fp) rec[c++] = j | (5ull * V + tp);
                if (fs && fp) {
                    u32 b = bin_lookup(lkeys, lvals, lmask, bin_key(2, ts, tp));
                    if (b != NONE32) rec[c++] = j | (B6 + b);
                }
            }
            if (proj & 2) {  // project predicates: p[s], p[o], p[s,o]
                const u64 j = (u64)tp << capbits;
                if (fs) rec[c++] = j | (2ull * V + ts);
                if (fo) rec[c++] = j | (3ull * V + to);
                if (fs && fo) {
                    u32 b = bin_lookup(lkeys, lvals, lmask, bin_key(1, ts, to));
                    if (b != NONE32) rec[c++] = j | (B6 + b);
                }
            }
            if (proj & 1) {  // project subjects: s[p], s[o], s[p,o]
                const u64 j = (u64)ts << capbits;
                if (fp) rec[c++] = j | (0ull * V + tp);
                if (fo) rec[c++] = j | (1ull * V + to);
                if (fp && fo) {
                    u32 b = bin_lookup(lkeys, lvals, lmask, bin_key(0, tp, to));
                    if (b != NONE32) rec[c++] = j | (B6 + b);
                }
            }
        }
        u64 base = wave_append(counter, c);
        for (u32 k = 0; k < c; ++k) out[base + k] = rec[k];
    }
}

// ================================================================================================
// K4/K5: capture groups  (UnionJoinCandidates.combine / UnionCombinedJoinCandidates.reduce,
//     ALG/operators/UnionJoinCandidates.scala:27-44, UnionCombinedJoinCandidates.scala:21-31: distinct
//     captures per join value) and capture supports (depCount summed per group,
//     ALG/operators/candidate_merging/BulkMergeDependencies.scala:78-84)

__global__ __launch_bounds__(RDF_BLOCK) void k_unique_support(const u64* __restrict__ keys, u64 n, u64 capmask,
                                                              u32* support) {
    for (u64 i = (u64)blockIdx.x * RDF_BLOCK + threadIdx.x; i < n; i += (u64)gridDim.x * RDF_BLOCK) {
        u64 k = keys[i];
        if (i == 0 || keys[i - 1] != k) atomicAdd(&support[k & capmask], 1u);
    }
}

__global__ __launch_bounds__(RDF_BLOCK) void k_support_flags(const u32* __restrict__ support, u64 ncap, u32 ms, u32* flags) {
    for (u64 i = (u64)blockIdx.x * RDF_BLOCK + threadIdx.x; i < ncap; i += (u64)gridDim.x * RDF_BLOCK)
        flags[i] = support[i] >= ms;
}

// fidx is the exclusive scan of the support flags: compact id of a frequent capture
__global__ __launch_bounds__(RDF_BLOCK) void k_compact_captures(const u32* __restrict__ support, const u32* __restrict__ fidx,
                                                                u64 ncap, u32 ms, u32* fcap, CapInfo* info) {
    for (u64 i = (u64)blockIdx.x * RDF_BLOCK + threadIdx.x; i < ncap; i += (u64)gridDim.x * RDF_BLOCK) {
        u32 sup = support[i];
        if (sup >= ms) {
            u32 c = fidx[i];
            fcap[c] = (u32)i;
            CapInfo ci;
            ci.hmask = 0;
            ci.support = sup;
            ci.meta = 0;
            info[c] = ci;
        }
    }
}

// keep distinct records of frequent captures
__global__ __launch_bounds__(RDF_BLOCK) void k_keep_flags(const u64* __restrict__ keys, u64 n, u64 capmask,
                                                          const u32* __restrict__ support, u32 ms, u32* flags) {
    for (u64 i = (u64)blockIdx.x * RDF_BLOCK + threadIdx.x; i < n; i += (u64)gridDim.x * RDF_BLOCK) {
        u64 k = keys[i];
        flags[i] = ((i == 0 || keys[i - 1] != k) && support[k & capmask] >= ms) ? 1u : 0u;
    }
}

__global__ __launch_bounds__(RDF_BLOCK) void k_keep_scatter(const u64* __restrict__ keys, u64 n, int capbits, u64 capmask,
                                                            const u32* __restrict__ flags, const u64* __restrict__ pos,
                                                            const u32* __restrict__ fidx, u64* out) {
    for (u64 i = (u64)blockIdx.x * RDF_BLOCK + threadIdx.x; i < n; i += (u64)gridDim.x * RDF_BLOCK) {
        if (flags[i]) {
            u64 k = keys[i];
            out[pos[i]] = ((k >> capbits) << 32) | fidx[k & capmask];
        }
    }
}

__global__ __launch_bounds__(RDF_BLOCK) void k_group_flags(const u64* __restrict__ fk, u64 n, u32* flags) {
    for (u64 i = (u64)blockIdx.x * RDF_BLOCK + threadIdx.x; i < n; i += (u64)gridDim.x * RDF_BLOCK)
        flags[i] = (i == 0 || (fk[i - 1] >> 32) != (fk[i] >> 32)) ? 1u : 0u;
}

// groups: goff[g] = first record; gcap[i] = compact capture id; gid[i] = group of record i
__global__ __launch_bounds__(RDF_BLOCK) void k_group_build(const u64* __restrict__ fk, u64 n, const u32* __restrict__ gflag,
                                                           const u32* __restrict__ gexcl, u64* goff, u32* gcap, u32* gid) {
    for (u64 i = (u64)blockIdx.x * RDF_BLOCK + threadIdx.x; i < n; i += (u64)gridDim.x * RDF_BLOCK) {
        u32 g = gexcl[i] + gflag[i] - 1;
        if (gflag[i]) goff[g] = i;
        gcap[i] = (u32)(fk[i] & 0xffffffffu);
        gid[i] = g;
    }
}

__global__ __launch_bounds__(RDF_BLOCK) void k_info_support_u32(const CapInfo* __restrict__ info, u32 C, u32* out) {
    for (u64 i = (u64)blockIdx.x * RDF_BLOCK + threadIdx.x; i < C; i += (u64)gridDim.x * RDF_BLOCK) out[i] = info[i].support;
}

// dependent -> groups (transposed CSR); order inside a list is irrelevant
__global__ __launch_bounds__(RDF_BLOCK) void k_dep_scatter(const u32* __restrict__ gcap, const u32* __restrict__ gid, u64 n,
                                                           u64* cursor, u32* dgrp) {
    for (u64 i = (u64)blockIdx.x * RDF_BLOCK + threadIdx.x; i < n; i += (u64)gridDim.x * RDF_BLOCK) {
        u64 pos = atomicAdd(&cursor[gcap[i]], 1ull);
        dgrp[pos] = gid[i];
    }
}

// ---- heavy groups: quarter-octave size buckets, then the top groups become bit columns
__device__ __host__ inline int size_bucket(u64 size) {
    if (size == 0) return 0;
    int msb = 63 - __builtin_clzll(size);
    int frac = msb >= 2 ? (int)((size >> (msb - 2)) & 3) : (int)((size << (2 - msb)) & 3);
    return 4 * msb + frac;
}

__global__ __launch_bounds__(RDF_BLOCK) void k_group_size_hist(const u64* __restrict__ goff, u64 G, u32* hist) {
    for (u64 g = (u64)blockIdx.x * RDF_BLOCK + threadIdx.x; g < G; g += (u64)gridDim.x * RDF_BLOCK)
        atomicAdd(&hist[size_bucket(goff[g + 1] - goff[g])], 1u);
}

__global__ __launch_bounds__(RDF_BLOCK) void k_heavy_select(const u64* __restrict__ goff, u64 G, u64 threshold, u32* nheavy,
                                                            u32* heavy_list, uint8_t* hbit) {
    for (u64 g = (u64)blockIdx.x * RDF_BLOCK + threadIdx.x; g < G; g += (u64)gridDim.x * RDF_BLOCK) {
        u64 sz = goff[g + 1] - goff[g];
        uint8_t b = LIGHT;
        if (threshold && sz >= threshold) {
            u32 j = atomicAdd(nheavy, 1u);
            if (j < (u32)HMAX) {
                b = (uint8_t)j;
                heavy_list[j] = (u32)g;
            }
        }
        hbit[g] = b;
    }
}

__global__ __launch_bounds__(RDF_BLOCK) void k_heavy_mask(const u64* __restrict__ goff, const u32* __restrict__ gcap,
                                                          const u32* __restrict__ heavy_list, CapInfo* info) {
    const u32 h = blockIdx.y;
    const u32 g = heavy_list[h];
    const u64 b = goff[g], e = goff[g + 1];
    for (u64 i = b + (u64)blockIdx.x * RDF_BLOCK + threadIdx.x; i < e; i += (u64)gridDim.x * RDF_BLOCK)
        atomicOr(&info[gcap[i]].hmask, 1ull << h);
}

// binary captures: components (unary compact ids) and keys; unary captures: parent counts
__global__ __launch_bounds__(RDF_BLOCK) void k_binary_info(const u32* __restrict__ fcap, const u32* __restrict__ fidx,
                                                           const u64* __restrict__ bkeys, u32 C, u32 Cu, u32 V,
                                                           u32* bcomp, u64* bkeyc, u32* pcnt, CapInfo* info) {
    for (u64 c = Cu + (u64)blockIdx.x * RDF_BLOCK + threadIdx.x; c < C; c += (u64)gridDim.x * RDF_BLOCK) {
        u64 key = bkeys[fcap[c] - 6ull * V];
        int bt = bin_key_type(key);
        u32 c1 = fidx[(u64)bin_comp1(bt) * V + bin_key_v1(key)];
        u32 c2 = fidx[(u64)bin_comp2(bt) * V + bin_key_v2(key)];
        bcomp[2 * (c - Cu)] = c1;
        bcomp[2 * (c - Cu) + 1] = c2;
        bkeyc[c - Cu] = key;
        atomicAdd(&pcnt[c1], 1u);
        atomicAdd(&pcnt[c2], 1u);
        info[c].meta |= META_BIN;
    }
}

__global__ __launch_bounds__(RDF_BLOCK) void k_parents_scatter(const u32* __restrict__ bcomp, u32 C, u32 Cu,
                                                               u64* cursor, u32* plist) {
    for (u64 c = Cu + (u64)blockIdx.x * RDF_BLOCK + threadIdx.x; c < C; c += (u64)gridDim.x * RDF_BLOCK) {
        plist[atomicAdd(&cursor[bcomp[2 * (c - Cu)]], 1ull)] = (u32)c;
        plist[atomicAdd(&cursor[bcomp[2 * (c - Cu) + 1]], 1ull)] = (u32)c;
    }
}

__global__ __launch_bounds__(RDF_BLOCK) void k_parent_meta(const u32* __restrict__ pcnt, u32 Cu, CapInfo* info) {
    for (u64 c = (u64)blockIdx.x * RDF_BLOCK + threadIdx.x; c < Cu; c += (u64)gridDim.x * RDF_BLOCK)
        if (pcnt[c]) info[c].meta |= META_PARENTS;
}

// ================================================================================================
// K6: CIND extraction by intersection  (CreateAllCindCandidates.scala:71-121 + IntersectCindCandidates
//     .scala:14-51: the refs of a dependent A are the captures present in every group of A, i.e.
//     count(A,B) == support(A)).  A's smallest group (its pivot) bounds the candidates; the heavy-group
//     bitmask test (hmask(B) covers hmask(A)) verifies every heavy group at once, and the remaining light
//     groups are verified by binary search with one lane per group.  Deps whose groups are all heavy
//     ("heavy-only") need no verification: their refs are the pivot members passing the mask test.

// pivot pass: one wave per dependent
__global__ __launch_bounds__(RDF_BLOCK) void k_pivot(CindView v, u32* pivot, u32* nchunk_light, u32* nchunk_heavy,
                                                     CapInfo* info, u64* heavy_candidates) {
    const int lane = lane_id();
    const u64 d = (u64)blockIdx.x * RDF_WAVES_PER_BLOCK + threadIdx.x / RDF_WAVE;
    if (d >= v.C) return;
    const u64 b = v.doff[d], e = v.doff[d + 1];
    u64 best = ~0ull;  // (size << 32 | group)
    u32 nlight = 0;
    for (u64 j = b + lane; j < e; j += RDF_WAVE) {
        u32 g = v.dgrp[j];
        u64 sz = v.goff[g + 1] - v.goff[g];
        u64 key = (sz << 32) | g;
        best = key < best ? key : best;
        nlight += v.hbit[g] == LIGHT;
    }
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) {
        u64 o = __shfl_xor(best, off, RDF_WAVE);
        best = o < best ? o : best;
    }
    nlight = wave_sum(nlight);
    if (lane == 0) {
        u32 g = (u32)(best & 0xffffffffu);
        u64 sz = best >> 32;
        u32 nch = (u32)((sz + RDF_WAVE - 1) / RDF_WAVE);
        pivot[d] = g;
        nchunk_light[d] = nlight ? nch : 0;
        nchunk_heavy[d] = nlight ? 0 : nch;
        if (!nlight) {
            info[d].meta |= META_HEAVY_ONLY;
            atomicAdd(heavy_candidates, sz);
        }
    }
}

__device__ inline bool bsearch_u32(const u32* a, u64 n, u32 key) {
    u64 lo = 0, hi = n;
    while (lo < hi) {
        u64 mid = (lo + hi) >> 1;
        u32 x = a[mid];
        if (x < key) lo = mid + 1;
        else hi = mid;
    }
    return lo < n && a[lo] == key;
}

__device__ inline bool bsearch_u64(const u64* a, u64 n, u64 key) {
    u64 lo = 0, hi = n;
    while (lo < hi) {
        u64 mid = (lo + hi) >> 1;
        u64 x = a[mid];
        if (x < key) lo = mid + 1;
        else hi = mid;
    }
    return lo < n && a[lo] == key;
}

// ref is trivially implied by dep: a unary component of a binary dep (Condition.isImpliedBy,
// ALG/data/Condition.scala:35-43; excluded by CreateBinaryUnaryCindCandidates.scala:76)
__device__ inline bool is_trivial(const CindView& v, u32 dep, u32 ref) {
    if (dep < v.Cu) return false;
    const u32* bc = v.bcomp + 2ull * (dep - v.Cu);
    return ref == bc[0] || ref == bc[1];
}

// literal strategy-0 quirk: Condition.isImpliedBy compares this.v1 with that.v2 for two binary
// captures of the same type, so CreateAllCindCandidates.scala:113 drops X from D's refs when X.v1 == D.v2
__device__ inline bool is_quirk(const CindView& v, u32 dep, u32 ref) {
    if (!v.literal || dep < v.Cu || ref < v.Cu) return false;
    u64 kd = v.bkeyc[dep - v.Cu], kr = v.bkeyc[ref - v.Cu];
    return bin_key_type(kd) == bin_key_type(kr) && bin_key_v1(kr) == bin_key_v2(kd);
}

// X < Y is a (raw) CIND
__device__ inline bool member(const CindView& v, u32 x, u32 y) {
    if (x == y) return false;
    const CapInfo ix = v.info[x];
    const u64 my = v.info[y].hmask;
    if ((ix.hmask & my) != ix.hmask) return false;
    if (is_trivial(v, x, y) || is_quirk(v, x, y)) return false;
    if (ix.meta & META_HEAVY_ONLY) return true;
    const u64 b = v.eoff[x], e = v.eoff[x + 1];
    return bsearch_u64(v.epairs + b, e - b, ((u64)x << 32) | y);
}

// TraversalStrategy.removeImpliedCinds (TraversalStrategy.scala:126-168):
//   R1 drop 2/1 D<R if comp(D)<R in V11          RemoveNonMinimalDoubleXxxCinds.scala:19-40
//   R2 drop 2/1 D<R if D<X in V22, R in comp(X)  RemoveNonMinimalXxxSingleCinds.scala:19-41
//   R3 drop 1/1 A<R if A<X in V12, R in comp(X)
//   R4 drop 2/2 D<X if comp(D)<X in V12
// RULES_S2L_RAW applies only R1 and R4: the exact-candidate S2L output without --clean-implied.
__device__ inline bool rule_keep(const CindView& v, u32 a, u32 r) {
    if (v.mode == RULES_NONE) return true;
    const bool ab = a >= v.Cu, rb = r >= v.Cu;
    if (!ab && rb) return true;
    if (!ab && !rb) {
        if (v.mode != RULES_CLEAN) return true;
        if (!(v.info[r].meta & META_PARENTS)) return true;
        for (u64 j = v.poff[r]; j < v.poff[r + 1]; ++j)
            if (member(v, a, v.plist[j])) return false;
        return true;
    }
    const u32* bc = v.bcomp + 2ull * (a - v.Cu);
    if (member(v, bc[0], r) || member(v, bc[1], r)) return false;  // R1 / R4
    if (rb || v.mode != RULES_CLEAN) return true;
    if (!(v.info[r].meta & META_PARENTS)) return true;
    for (u64 j = v.poff[r]; j < v.poff[r + 1]; ++j)  // R2
        if (member(v, a, v.plist[j])) return false;
    return true;
}

__device__ inline u32 find_dep(const u64* chunk_off, u32 C, u64 w) {
    // largest d with chunk_off[d] <= w
    u32 lo = 0, hi = C;
    while (lo < hi) {
        u32 mid = (lo + hi + 1) >> 1;
        if (chunk_off[mid] <= w) lo = mid;
        else hi = mid - 1;
    }
    return lo;
}

// candidate filter for a chunk of the pivot group: returns this lane's candidate (or NONE)
__device__ inline u32 chunk_candidate(const CindView& v, u32 d, const CapInfo& id, u32 piv, u64 chunk) {
    const u64 gb = v.goff[piv], ge = v.goff[piv + 1];
    const u64 idx = gb + chunk * RDF_WAVE + lane_id();
    if (idx >= ge) return NONE32;
    const u32 r = v.gcap[idx];
    if (r == d) return NONE32;
    const CapInfo ir = v.info[r];
    if (ir.support < id.support) return NONE32;
    if ((ir.hmask & id.hmask) != id.hmask) return NONE32;
    if (is_trivial(v, d, r) || is_quirk(v, d, r)) return NONE32;
    return r;
}

// light dependents: verify light groups, write explicit (dep << 32 | ref) pairs
__global__ __launch_bounds__(RDF_BLOCK) void k_light(CindView v, const u32* __restrict__ pivot, const u64* __restrict__ choff,
                                                     u64 W, u64* pairs, u64* npairs) {
    const u64 w = (u64)blockIdx.x * RDF_WAVES_PER_BLOCK + threadIdx.x / RDF_WAVE;
    if (w >= W) return;
    const int lane = lane_id();
    const u32 d = find_dep(choff, v.C, w);
    const u64 chunk = w - choff[d];
    const u32 piv = pivot[d];
    const CapInfo id = v.info[d];
    const u32 cand = chunk_candidate(v, d, id, piv, chunk);
    u64 alive = __ballot(cand != NONE32);
    const u64 b = v.doff[d], e = v.doff[d + 1];
    for (u64 j0 = b; j0 < e && alive; j0 += RDF_WAVE) {
        const u64 j = j0 + lane;
        u32 g = NONE32;
        if (j < e) {
            g = v.dgrp[j];
            if (g == piv || v.hbit[g] != LIGHT) g = NONE32;
        }
        const u32* gm = nullptr;
        u64 gsz = 0;
        if (g != NONE32) {
            gm = v.gcap + v.goff[g];
            gsz = v.goff[g + 1] - v.goff[g];
        }
        u64 todo = alive;
        while (todo) {
            const int bit = __ffsll((long long)todo) - 1;
            todo &= todo - 1;
            const u32 c = __shfl(cand, bit, RDF_WAVE);
            const bool ok = (g == NONE32) || bsearch_u32(gm, gsz, c);
            if (!__all(ok)) alive &= ~(1ull << bit);
        }
    }
    if (!alive) return;
    const u32 cnt = (u32)__popcll(alive);
    u64 base = 0;
    if (lane == 0) base = atomicAdd(npairs, (u64)cnt);
    base = __shfl(base, 0, RDF_WAVE);
    if ((alive >> lane) & 1ull) pairs[base + __popcll(alive & lanemask_lt())] = ((u64)d << 32) | cand;
}

// explicit CSR offsets: eoff[d] = first pair with dep >= d
__global__ __launch_bounds__(RDF_BLOCK) void k_pair_offsets(const u64* __restrict__ pairs, u64 E, u32 C, u64* eoff) {
    for (u64 d = (u64)blockIdx.x * RDF_BLOCK + threadIdx.x; d <= C; d += (u64)gridDim.x * RDF_BLOCK) {
        u64 key = d << 32, lo = 0, hi = E;
        while (lo < hi) {
            u64 mid = (lo + hi) >> 1;
            if (pairs[mid] < key) lo = mid + 1;
            else hi = mid;
        }
        eoff[d] = lo;
    }
}

// minimality on explicit pairs -> output
__global__ __launch_bounds__(RDF_BLOCK) void k_rules_explicit(CindView v, const u64* __restrict__ pairs, u64 E, u64* out,
                                                              u64* nout) {
    const u64 n_round = (E + RDF_WAVE - 1) / RDF_WAVE * RDF_WAVE;
    for (u64 i = (u64)blockIdx.x * RDF_BLOCK + threadIdx.x; i < n_round; i += (u64)gridDim.x * RDF_BLOCK) {
        u32 keep = 0;
        u64 pr = 0;
        if (i < E) {
            pr = pairs[i];
            keep = rule_keep(v, (u32)(pr >> 32), (u32)pr) ? 1u : 0u;
        }
        u64 pos = wave_append(nout, keep);
        if (keep) out[pos] = pr;
    }
}

// heavy-only dependents: refs = pivot members passing the mask test; minimality fused.
// WRITE=false: count per work item; WRITE=true: write at the scanned offsets.
template <bool WRITE>
__global__ __launch_bounds__(RDF_BLOCK) void k_heavy(CindView v, const u32* __restrict__ pivot, const u64* __restrict__ choff,
                                                     u64 W, u32* counts, const u64* __restrict__ woff, u64 out_base,
                                                     u64* out) {
    const u64 w = (u64)blockIdx.x * RDF_WAVES_PER_BLOCK + threadIdx.x / RDF_WAVE;
    if (w >= W) return;
    const int lane = lane_id();
    const u32 d = find_dep(choff, v.C, w);
    const u64 chunk = w - choff[d];
    const CapInfo id = v.info[d];
    const u32 cand = chunk_candidate(v, d, id, pivot[d], chunk);
    const bool keep = cand != NONE32 && rule_keep(v, d, cand);
    const u64 kept = __ballot(keep);
    if (!WRITE) {
        if (lane == 0) counts[w] = (u32)__popcll(kept);
    } else if (keep) {
        out[out_base + woff[w] + __popcll(kept & lanemask_lt())] = ((u64)d << 32) | cand;
    }
}

}  // namespace rdf

namespace rdf {
// order-independent checksum of the result set (capture ids, so it is comparable across runs)
__global__ __launch_bounds__(RDF_BLOCK) void k_checksum(const u64* __restrict__ pairs, u64 n, const u32* __restrict__ fcap,
                                                        u64* sum) {
    u64 acc = 0;
    for (u64 i = (u64)blockIdx.x * RDF_BLOCK + threadIdx.x; i < n; i += (u64)gridDim.x * RDF_BLOCK) {
        const u64 pr = pairs[i];
        acc += mix64(((u64)fcap[pr >> 32] << 32) | fcap[(u32)pr]);
    }
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) acc += __shfl_xor(acc, off, RDF_WAVE);
    if (lane_id() == 0 && acc) atomicAdd(sum, acc);
}
}  // namespace rdf
