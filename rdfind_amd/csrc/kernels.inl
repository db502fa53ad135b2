// CIND-discovery kernels (included by rdfind_hip.hip).
//
// Abbreviation: ALG/ = rdfind-algorithm/src/main/scala/de/hpi/isg/sodap/rdfind/ in the reference.
// Each kernel names the reference operator whose semantics it implements.
#include "kernels.hpp"

namespace rdf {

__device__ inline u64 lower_bound_u64(const u64* a, u64 n, u64 key) {
    u64 lo = 0, hi = n;
    while (lo < hi) {
        u64 mid = (lo + hi) >> 1;
        if (a[mid] < key) lo = mid + 1;
        else hi = mid;
    }
    return lo;
}

// ================================================================================================
// K1: unary condition counts  (FrequentConditionPlanner.findFrequentSingleConditions,
//     ALG/plan/FrequentConditionPlanner.scala:291-311: flatMap 3 x (type, value, 1) -> groupBy.sum)
// Keys are type*V + value.  Per-block LDS hash table pre-aggregates hot keys (Zipf predicates /
// classes) so only one global atomic per distinct key per block remains; table misses go global.

// Wave-level merge of equal keys before counting (all lanes call it): runs of equal keys in adjacent lanes
// collapse into their first lane (subject-ordered input, sorted records), then up to ROUNDS keys repeated
// across the remaining run heads collapse into one lane each (hot predicates/classes).  Returns the count
// this lane adds: 0 when inactive or merged into another lane.
template <typename T, int ROUNDS>
__device__ inline u32 wave_merge(T key, bool active) {
    const int lane = lane_id();
    const u64 A = __ballot(active);
    const T prev = __shfl_up(key, 1, RDF_WAVE);
    const bool head = active && (lane == 0 || !((A >> (lane - 1)) & 1ull) || prev != key);
    const u64 H = __ballot(head);
    const u64 stop = H | ~A;  // a run ends at the next head or inactive lane
    u32 cnt = 0;
    if (head) {
        const u64 above = lane == RDF_WAVE - 1 ? 0ull : stop & (~0ull << (lane + 1));
        cnt = (u32)((above ? __ffsll((long long)above) - 1 : RDF_WAVE) - lane);
    }
    u64 todo = H;
#pragma unroll
    for (int r = 0; r < ROUNDS; ++r) {
        if (__popcll(todo) <= 1) break;
        const int l = __ffsll((long long)todo) - 1;
        const T kl = __shfl(key, l, RDF_WAVE);
        const bool mine = ((todo >> lane) & 1ull) && key == kl;
        const u64 m = __ballot(mine);
        todo &= ~m;
        if (__popcll(m) > 1) {
            const u32 tot = wave_sum(mine ? cnt : 0u);
            if (mine) cnt = lane == l ? tot : 0u;
        }
    }
    return cnt;
}

// LDS hash add with LDS_PROBES probes, then the global counter.  Few probes: once the table is full of
// cold keys, probing further only delays the global atomic; hot keys claim their slots early.
static constexpr int LDS_PROBES = 2;

__device__ inline void lds_count_u32(u32* lkey, u32* lcnt, u32 key, u32 c, u32* gcnt) {
    u32 h = hash32(key) & (LH_SLOTS - 1);
#pragma unroll
    for (int probe = 0; probe < LDS_PROBES; ++probe) {
        u32 k = lkey[h];
        if (k == EMPTY32) {
            const u32 prev = atomicCAS(&lkey[h], EMPTY32, key);
            k = prev == EMPTY32 ? key : prev;
        }
        if (k == key) {
            atomicAdd(&lcnt[h], c);
            return;
        }
        h = (h + 1) & (LH_SLOTS - 1);
    }
    atomicAdd(&gcnt[key], c);
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
    // one contiguous chunk per block so that runs of equal values (e.g. subjects) aggregate in LDS
    const u64 per = (n + gridDim.x - 1) / gridDim.x;
    const u64 b = (u64)blockIdx.x * per, e = b + per < n ? b + per : n;
    for (u64 i0 = b; i0 < e; i0 += RDF_BLOCK) {
        const u64 i = i0 + threadIdx.x;
        const bool act = i < e;
        const u32 ks = act ? s[i] : 0u, kp = act ? V + p[i] : 0u, ko = act ? 2u * V + o[i] : 0u;
        const u32 cs = wave_merge<u32, 2>(ks, act);
        const u32 cp = wave_merge<u32, 4>(kp, act);
        const u32 co = wave_merge<u32, 4>(ko, act);
        if (cs) lds_count_u32(lkey, lcnt, ks, cs, cnt);
        if (cp) lds_count_u32(lkey, lcnt, kp, cp, cnt);
        if (co) lds_count_u32(lkey, lcnt, ko, co, cnt);
    }
    __syncthreads();
    for (int i = threadIdx.x; i < LH_SLOTS; i += RDF_BLOCK)
        if (lkey[i] != EMPTY32) atomicAdd(&cnt[lkey[i]], lcnt[i]);
}

// Weighted variant of the leader rounds of wave_merge: lanes holding the same key (anywhere in the wave)
// collapse into one lane carrying the summed weight.
template <typename T, int ROUNDS>
__device__ inline u32 wave_merge_weighted(T key, bool active, u32 w) {
    const int lane = lane_id();
    u32 cnt = active ? w : 0u;
    u64 todo = __ballot(active);
#pragma unroll
    for (int r = 0; r < ROUNDS; ++r) {
        if (__popcll(todo) <= 1) break;
        const int l = __ffsll((long long)todo) - 1;
        const T kl = __shfl(key, l, RDF_WAVE);
        const bool mine = ((todo >> lane) & 1ull) && key == kl;
        const u64 m = __ballot(mine);
        todo &= ~m;
        if (__popcll(m) > 1) {
            const u32 tot = wave_sum(mine ? cnt : 0u);
            if (mine) cnt = lane == l ? tot : 0u;
        }
    }
    return cnt;
}

#include "counts.inl"

// Block-reduced counter add (all threads of the block call it): device-scope atomics execute at the
// memory side, ~11 ns apart on one address, so one per block instead of one per wave.
__device__ inline void block_counter_add(u64* counter, u32 v) {
    __shared__ u32 s_part[RDF_WAVES_PER_BLOCK];
    v = wave_sum(v);
    if (lane_id() == 0) s_part[threadIdx.x / RDF_WAVE] = v;
    __syncthreads();
    if (threadIdx.x == 0) {
        u64 t = 0;
#pragma unroll
        for (int w = 0; w < RDF_WAVES_PER_BLOCK; ++w) t += s_part[w];
        if (t) atomicAdd(counter, t);
    }
    __syncthreads();
}

// block-wide exclusive scan of one u32 per thread; *total = block sum (all threads must call it)
__device__ inline u32 block_exclusive_scan_u32(u32 v, u32* lds_wave, u32* total) {
    const int wave = threadIdx.x / RDF_WAVE;
    const u32 incl = wave_inclusive_scan(v);
    if (lane_id() == RDF_WAVE - 1) lds_wave[wave] = incl;
    __syncthreads();
    u32 woff = 0, sum = 0;
#pragma unroll
    for (int w = 0; w < RDF_WAVES_PER_BLOCK; ++w) {
        const u32 x = lds_wave[w];
        woff += w < wave ? x : 0u;
        sum += x;
    }
    *total = sum;
    __syncthreads();  // lds_wave is reused by the next call
    return woff + incl - v;
}

// number of frequent values per condition type (for stats)
__global__ __launch_bounds__(RDF_BLOCK) void k_count_frequent(const u32* __restrict__ cnt, u32 V, u32 ms, u64* out3) {
    for (int t = 0; t < 3; ++t) {
        const u32* ct = cnt + (u64)t * V;
        u32 c = 0;
        for (u64 i = (u64)blockIdx.x * RDF_BLOCK + threadIdx.x; i < V; i += (u64)gridDim.x * RDF_BLOCK) c += ct[i] >= ms;
        block_counter_add(&out3[t], c);
    }
}

// frequent-condition ranks: frank[i] (i = pos * V + value, pos 0 s / 1 p / 2 o) = index of the condition
// among all frequent conditions, NONE if infrequent; fval[index] = value.  They give the compact candidate
// capture space: unary capture (type t, value v) -> 2 * frank[cap_pos(t) * V + v] + (t >= 3), binary
// capture b -> 2U + b (U = frequent conditions), so sort keys and support arrays scale with U, not |V|.
__global__ __launch_bounds__(RDF_BLOCK) void k_frank_flags(const u32* __restrict__ cnt, u64 n3, u32 ms, u32* flags) {
    for (u64 i = (u64)blockIdx.x * RDF_BLOCK + threadIdx.x; i < n3; i += (u64)gridDim.x * RDF_BLOCK) flags[i] = cnt[i] >= ms;
}

__global__ __launch_bounds__(RDF_BLOCK) void k_frank_final(const u32* __restrict__ cnt, u32 V, u32 ms, u32* frank,
                                                           u32* fval) {
    for (int t = 0; t < 3; ++t)
        for (u64 v = (u64)blockIdx.x * RDF_BLOCK + threadIdx.x; v < V; v += (u64)gridDim.x * RDF_BLOCK) {
            const u64 i = (u64)t * V + v;
            if (cnt[i] >= ms) fval[frank[i]] = (u32)v;
            else frank[i] = NONE32;
        }
}

// condition position (0 s, 1 p, 2 o) of unary capture type t (0 s[p], 1 s[o], 2 p[s], 3 p[o], 4 o[s], 5 o[p])
__host__ __device__ inline int cap_pos(int t) { return (t == 2 || t == 4) ? 0 : ((t == 0 || t == 5) ? 1 : 2); }

// candidate capture id of unary capture (t, v); NONE if its condition is infrequent
__device__ inline u32 ucap(const u32* frank, u32 V, int t, u32 v) {
    const u32 r = frank[(u64)cap_pos(t) * V + v];
    return r == NONE32 ? NONE32 : 2u * r + (t >= 3 ? 1u : 0u);
}

// external capture id (t * V + v for unary, 6V + b for binary) of a candidate id
__global__ __launch_bounds__(RDF_BLOCK) void k_external_ids(const u32* __restrict__ fcap, u32 C, u32 twoU, u32 V,
                                                            const u32* __restrict__ fval, u32 Us, u32 Up, u32* ext) {
    for (u64 c = (u64)blockIdx.x * RDF_BLOCK + threadIdx.x; c < C; c += (u64)gridDim.x * RDF_BLOCK) {
        const u32 id = fcap[c];
        if (id < twoU) {
            const u32 u = id >> 1, j = id & 1u;
            const int pos = u < Us ? 0 : (u < Us + Up ? 1 : 2);
            const u32 t = pos == 0 ? (j ? 4u : 2u) : (pos == 1 ? (j ? 5u : 0u) : (j ? 3u : 1u));
            ext[c] = t * V + fval[u];
        } else {
            ext[c] = 6u * V + (id - twoU);
        }
    }
}

// ================================================================================================
// K2: binary condition counts  (CreatedReducedDoubleConditionCounts.flatMap,
//     ALG/operators/candidate_extraction/CreatedReducedDoubleConditionCounts.scala:45-86, + groupBy.sum
//     FrequentConditionPlanner.scala:374-394).  Only triples with >= 2 frequent values emit sp/so/po.

__device__ inline void freq_flags(const u32* frank, const u32* boff, u32 V, u32 s, u32 p, u32 o, bool& fs, bool& fp,
                                  bool& fo) {
    fs = frank_at(frank, boff, s) != NONE32;
    fp = frank_at(frank, boff, (u64)V + p) != NONE32;
    fo = frank_at(frank, boff, 2ull * V + o) != NONE32;
}

__global__ __launch_bounds__(RDF_BLOCK) void k_binary_emit_count(const u32* __restrict__ s, const u32* __restrict__ p,
                                                                 const u32* __restrict__ o, u64 n, u32 V,
                                                                 const u32* __restrict__ frank, const u32* __restrict__ boff,
                                                                 u64* total) {
    u32 c = 0;
    for (u64 i = (u64)blockIdx.x * RDF_BLOCK + threadIdx.x; i < n; i += (u64)gridDim.x * RDF_BLOCK) {
        bool fs, fp, fo;
        freq_flags(frank, boff, V, s[i], p[i], o[i], fs, fp, fo);
        c += (fs && fp) + (fs && fo) + (fp && fo);
    }
    block_counter_add(total, c);
}

// u32 count that saturates at 2^32 - 1 instead of wrapping (a condition summed over the ranks' slices can reach 2^32
// occurrences; saturation keeps every `count >= min_support` test right).  Any add that wraps sets the maximum, which
// no later add can lower: the final value is exact below 2^32 and 2^32 - 1 otherwise.
__device__ inline void sat_add_u32(u32* p, u32 c) {
    const u32 old = atomicAdd(p, c);
    if (old + c < old) atomicMax(p, 0xffffffffu);
}

__device__ inline void global_hash_add(u64* tkeys, u32* tcnt, u64 mask, u64 key, u32 c) {
    u64 h = mix64(key) & mask;
    for (;;) {
        u64 k = tkeys[h];
        if (k == key) {
            sat_add_u32(&tcnt[h], c);
            return;
        }
        if (k == EMPTY64) {
            u64 prev = atomicCAS(&tkeys[h], EMPTY64, key);
            if (prev == EMPTY64 || prev == key) {
                sat_add_u32(&tcnt[h], c);
                return;
            }
        }
        h = (h + 1) & mask;
    }
}

__global__ __launch_bounds__(RDF_BLOCK) void k_spill_insert(const u64* __restrict__ keys, const u32* __restrict__ cnt, u64 n,
                                                            u64* tkeys, u32* tcnt, u64 tmask) {
    for (u64 i = (u64)blockIdx.x * RDF_BLOCK + threadIdx.x; i < n; i += (u64)gridDim.x * RDF_BLOCK)
        global_hash_add(tkeys, tcnt, tmask, keys[i], cnt[i]);
}

__device__ inline void lds_count_u64(u64* lkey, u32* lcnt, u64 key, u32 c, u64* tkeys, u32* tcnt, u64 tmask) {
    u32 h = (u32)mix64(key) & (LB_SLOTS - 1);
#pragma unroll
    for (int probe = 0; probe < LDS_PROBES; ++probe) {
        u64 k = lkey[h];
        if (k == EMPTY64) {
            const u64 prev = atomicCAS(&lkey[h], EMPTY64, key);
            k = prev == EMPTY64 ? key : prev;
        }
        if (k == key) {
            atomicAdd(&lcnt[h], c);
            return;
        }
        h = (h + 1) & (LB_SLOTS - 1);
    }
    global_hash_add(tkeys, tcnt, tmask, key, c);
}

__global__ __launch_bounds__(RDF_BLOCK) void k_binary_count(const u32* __restrict__ s, const u32* __restrict__ p,
                                                            const u32* __restrict__ o, u64 n, u32 V,
                                                            const u32* __restrict__ frank, const u32* __restrict__ boff,
                                                            u64* tkeys, u32* tcnt, u64 tmask) {
    __shared__ u64 lkey[LB_SLOTS];
    __shared__ u32 lcnt[LB_SLOTS];
    for (int i = threadIdx.x; i < LB_SLOTS; i += RDF_BLOCK) {
        lkey[i] = EMPTY64;
        lcnt[i] = 0;
    }
    __syncthreads();
    // one contiguous chunk per block (subject runs stay together for the wave merge)
    const u64 per = (n + gridDim.x - 1) / gridDim.x;
    const u64 b = (u64)blockIdx.x * per, e = b + per < n ? b + per : n;
    for (u64 i0 = b; i0 < e; i0 += RDF_BLOCK) {
        const u64 i = i0 + threadIdx.x;
        const bool act = i < e;
        u32 ts = 0, tp = 0, to = 0;
        bool fs = false, fp = false, fo = false;
        if (act) {
            ts = s[i];
            tp = p[i];
            to = o[i];
            freq_flags(frank, boff, V, ts, tp, to, fs, fp, fo);
        }
        const u64 k_sp = bin_key(2, ts, tp), k_so = bin_key(1, ts, to), k_po = bin_key(0, tp, to);
        const u32 c_sp = wave_merge<u64, 2>(k_sp, fs && fp);  // o[s,p] (35)
        const u32 c_so = wave_merge<u64, 2>(k_so, fs && fo);  // p[s,o] (21)
        const u32 c_po = wave_merge<u64, 4>(k_po, fp && fo);  // s[p,o] (14)
        if (c_sp) lds_count_u64(lkey, lcnt, k_sp, c_sp, tkeys, tcnt, tmask);
        if (c_so) lds_count_u64(lkey, lcnt, k_so, c_so, tkeys, tcnt, tmask);
        if (c_po) lds_count_u64(lkey, lcnt, k_po, c_po, tkeys, tcnt, tmask);
    }
    __syncthreads();
    for (int i = threadIdx.x; i < LB_SLOTS; i += RDF_BLOCK)
        if (lkey[i] != EMPTY64) global_hash_add(tkeys, tcnt, tmask, lkey[i], lcnt[i]);
}

// frequent binary conditions: filter >= minSupport (FrequentConditionPlanner.scala:390-392); *nonempty =
// number of distinct binary keys (stats)
__global__ __launch_bounds__(RDF_BLOCK) void k_bin_freq_flags(const u64* __restrict__ tkeys, const u32* __restrict__ tcnt,
                                                              u64 cap, u32 ms, u32* flags, u64* nonempty) {
    u32 c = 0;
    for (u64 i = (u64)blockIdx.x * RDF_BLOCK + threadIdx.x; i < cap; i += (u64)gridDim.x * RDF_BLOCK) {
        const bool used = tkeys[i] != EMPTY64;
        c += used;
        flags[i] = (used && tcnt[i] >= ms) ? 1u : 0u;
    }
    block_counter_add(nonempty, c);
}

__global__ __launch_bounds__(RDF_BLOCK) void k_bin_freq_scatter(const u64* __restrict__ tkeys, const u32* __restrict__ flags,
                                                                const u64* __restrict__ pos, u64 cap, u64* out) {
    for (u64 i = (u64)blockIdx.x * RDF_BLOCK + threadIdx.x; i < cap; i += (u64)gridDim.x * RDF_BLOCK)
        if (flags[i]) out[pos[i]] = tkeys[i];
}

// lookup table of frequent binary keys -> index b (keys sorted, so b is deterministic)
// binary keys (bt << 62 | v1 << 31 | v2) <-> (bt << 2jb | v1 << jb | v2), values < 2^jb: the dense form keeps the
// order and needs 2 + 2jb radix bits instead of 64
__global__ __launch_bounds__(RDF_BLOCK) void k_bkey_repack(u64* __restrict__ keys, u64 B, int jb, int unpack) {
    const u64 m = (1ull << jb) - 1;
    for (u64 b = (u64)blockIdx.x * RDF_BLOCK + threadIdx.x; b < B; b += (u64)gridDim.x * RDF_BLOCK) {
        const u64 k = keys[b];
        keys[b] = unpack ? bin_key(k >> (2 * jb), (k >> jb) & m, k & m)
                         : ((u64)bin_key_type(k) << (2 * jb)) | ((u64)bin_key_v1(k) << jb) | bin_key_v2(k);
    }
}

// the same keys packed by the global ranks of their two frequent unary conditions (strictly increasing in the value for
// a fixed position, and the positions are fixed per key type), so the order is the same in fewer bits: c2's keys
// 2 + 2 x 23 -> 2 + 2 x 19 bits, five radix passes instead of six.  bt 0: (p, o), 1: (s, o), 2: (s, p)
__global__ __launch_bounds__(RDF_BLOCK) void k_bkey_rank_repack(u64* __restrict__ keys, u64 B, int rb, u32 V,
                                                                const u32* __restrict__ frank, const u32* __restrict__ fval,
                                                                int unpack) {
    const u64 m = (1ull << rb) - 1;
    for (u64 b = (u64)blockIdx.x * RDF_BLOCK + threadIdx.x; b < B; b += (u64)gridDim.x * RDF_BLOCK) {
        const u64 k = keys[b];
        if (unpack) {
            keys[b] = bin_key(k >> (2 * rb), fval[(k >> rb) & m], fval[k & m]);
        } else {
            const int bt = bin_key_type(k);
            const u64 pa = bt == 0 ? 1 : 0, pb = bt == 2 ? 1 : 2;
            const u64 r1 = frank[pa * V + bin_key_v1(k)], r2 = frank[pb * V + bin_key_v2(k)];
            keys[b] = ((u64)bt << (2 * rb)) | (r1 << rb) | r2;
        }
    }
}

// binary-condition lookup table (open addressing, at most half full).  SLOT16: key and value side by side in one
// 16-byte slot, so a probe is one load; 0: separate key / value arrays (the value a second, dependent load)
#ifndef RDF_LOOKUP_SLOT16
#define RDF_LOOKUP_SLOT16 1
#endif
__global__ __launch_bounds__(RDF_BLOCK) void k_bin_lookup_build(const u64* __restrict__ bkeys, u64 B, u64* lkeys, u32* lvals,
                                                                u64 mask) {
    for (u64 b = (u64)blockIdx.x * RDF_BLOCK + threadIdx.x; b < B; b += (u64)gridDim.x * RDF_BLOCK) {
        u64 key = bkeys[b];
        u64 h = mix64(key) & mask;
        for (;;) {
            u64 prev = atomicCAS(&lkeys[RDF_LOOKUP_SLOT16 ? 2 * h : h], EMPTY64, key);
            if (prev == EMPTY64) {
                if (RDF_LOOKUP_SLOT16)
                    lkeys[2 * h + 1] = b;
                else
                    lvals[h] = (u32)b;
                break;
            }
            h = (h + 1) & mask;
        }
    }
}

struct alignas(16) LookupSlot {
    u64 key, val;
};
__device__ inline u32 bin_lookup_from(const u64* lkeys, const u32* lvals, u64 mask, u64 key, u64 h) {
    for (;;) {
        if (RDF_LOOKUP_SLOT16) {
            const LookupSlot sl = ((const LookupSlot*)lkeys)[h];
            if (sl.key == key) return (u32)sl.val;
            if (sl.key == EMPTY64) return NONE32;
        } else {
            u64 k = lkeys[h];
            if (k == key) return lvals[h];
            if (k == EMPTY64) return NONE32;
        }
        h = (h + 1) & mask;
    }
}
__device__ inline u32 bin_lookup(const u64* lkeys, const u32* lvals, u64 mask, u64 key) {
    return bin_lookup_from(lkeys, lvals, mask, key, mix64(key) & mask);
}

// a triple's (up to) three binary lookups together: the three first probes' key loads are issued at once, then the
// hits' value loads at once; a probe that meets another key continues alone (rare: the table is at most half full).
// One lookup after the other made K3 wait for up to six dependent round trips per triple.
__device__ inline void bin_lookup3(const u64* __restrict__ lkeys, const u32* __restrict__ lvals, u64 mask,
                                   const u64 (&key)[3], const bool (&need)[3], u32 (&out)[3]) {
    u64 h[3], k[3];
#pragma unroll
    for (int t = 0; t < 3; ++t) {
        h[t] = mix64(key[t]) & mask;
        k[t] = need[t] ? lkeys[RDF_LOOKUP_SLOT16 ? 2 * h[t] : h[t]] : EMPTY64;
    }
#pragma unroll
    for (int t = 0; t < 3; ++t)
        out[t] = need[t] && k[t] == key[t] ? (RDF_LOOKUP_SLOT16 ? (u32)lkeys[2 * h[t] + 1] : lvals[h[t]]) : NONE32;
#pragma unroll
    for (int t = 0; t < 3; ++t)
        if (need[t] && k[t] != key[t] && k[t] != EMPTY64) out[t] = bin_lookup_from(lkeys, lvals, mask, key[t], (h[t] + 1) & mask);
}

#include "ars.inl"


// ================================================================================================
// K3: join partners  (CreateJoinPartners.flatMap, ALG/operators/CreateJoinPartners.scala:86-147)
// Per triple and projection: unary captures of the frequent condition values and, when the binary
// condition is frequent, the binary capture.  Binary captures are emitted together with both unary
// components, which is what every consumer reconstructs (CreateDependencyCandidates.scala:90-105,
// splitAndCollectUnaryCaptures).  Record = capture << joinbits | join: sorted, a capture's records are
// contiguous, so its support is a run length (no atomics) and its join list is the dependent -> groups CSR.

// records of triple i (at most 9); returns the count.  LAZY: load only the condition ranks the taken join values'
// records need (join ranges, shards: a selection takes a fraction of the join values, and the random rank loads bound
// the emission: c4 at 10^9 triples 457 -> 401 ms); without it all three are loaded up front (one GPU, one pass: the
// lazy form cost c2's emission 0.80 -> 0.91 ms)
// rep (optional): bit k set for the records that repeat across triples of one subject or one (predicate, object) pair
// (p[s], s[p], o[p], p[o]: the same predicate twice for a subject, the same typed object for many subjects); the others
// (o[s], s[o] and the binary captures) practically never repeat within an emission iteration
template <bool LAZY>
__device__ inline u32 triple_records(u64 i, const u32* __restrict__ s, const u32* __restrict__ p, const u32* __restrict__ o,
                                     u32 V, u32 twoU, const u32* __restrict__ frank, const u64* __restrict__ lkeys,
                                     const u32* __restrict__ lvals, u64 lmask, int proj, int joinbits, JoinSel js,
                                     u64 (&rec)[9], u32* rep = nullptr, u32* grp = nullptr) {
    u32 c = 0, rp_mask = 0;
    const u32 ts = s[i], tp = p[i], to = o[i];
    const bool jo = (proj & 4) && js.take(to), jp = (proj & 2) && js.take(tp), js_ = (proj & 1) && js.take(ts);
    u32 rs, rp, ro;  // global condition ranks (or NONE)
    if (LAZY) {
        rs = jo || jp ? frank[ts] : NONE32;
        rp = jo || js_ ? frank[(u64)V + tp] : NONE32;
        ro = jp || js_ ? frank[2ull * V + to] : NONE32;
    } else {
        rs = frank[ts];
        rp = frank[(u64)V + tp];
        ro = frank[2ull * V + to];
    }
    const bool fs = rs != NONE32, fp = rp != NONE32, fo = ro != NONE32;
    // the binary captures o[s,p], p[s,o], s[p,o]: their lookups in flight together (bin_lookup3)
    const u64 bkey[3] = {bin_key(2, ts, tp), bin_key(1, ts, to), bin_key(0, tp, to)};
    const bool bneed[3] = {jo && fs && fp, jp && fs && fo, js_ && fp && fo};
    u32 bval[3];
#ifndef RDF_K3_LOOKUP3  // 1: bin_lookup3 (measured slower: c4 at 0.4 emit 54.1 -> 57.8 ms, c3 8.44 -> 8.88; its registers
#define RDF_K3_LOOKUP3 0   // cost the write pass an occupancy step; profiles/r05_k3_lookup3_ab.log)
#endif
    if (RDF_K3_LOOKUP3) {
        bin_lookup3(lkeys, lvals, lmask, bkey, bneed, bval);
    } else {  // one lookup after the other (A/B switch)
#pragma unroll
        for (int t = 0; t < 3; ++t) bval[t] = bneed[t] ? bin_lookup(lkeys, lvals, lmask, bkey[t]) : NONE32;
    }
    if (jo) {  // project objects: o[s] (t4), o[p] (t5), o[s,p]
        if (fs) rec[c++] = ((2ull * rs + 1) << joinbits) | to;
        if (fp) { rp_mask |= 1u << c; rec[c++] = ((2ull * rp + 1) << joinbits) | to; }
        if (bval[0] != NONE32) rec[c++] = (((u64)twoU + bval[0]) << joinbits) | to;
    }
    const u32 co = c;
    if (jp) {  // project predicates: p[s] (t2), p[o] (t3), p[s,o]
        if (fs) { rp_mask |= 1u << c; rec[c++] = ((2ull * rs) << joinbits) | tp; }
        if (fo) { rp_mask |= 1u << c; rec[c++] = ((2ull * ro + 1) << joinbits) | tp; }
        if (bval[1] != NONE32) rec[c++] = (((u64)twoU + bval[1]) << joinbits) | tp;
    }
    if (grp) *grp = co | ((c - co) << 2);  // records joined on the object, on the predicate (the rest: the subject)
    if (js_) {  // project subjects: s[p] (t0), s[o] (t1), s[p,o]
        if (fp) { rp_mask |= 1u << c; rec[c++] = ((2ull * rp) << joinbits) | ts; }
        if (fo) rec[c++] = ((2ull * ro) << joinbits) | ts;
        if (bval[2] != NONE32) rec[c++] = (((u64)twoU + bval[2]) << joinbits) | ts;
    }
    if (rep) *rep = rp_mask;
    return c;
}

// two passes over contiguous per-block chunks of triples: COUNT writes each block's record count, the
// write pass places records at the scanned block offset + block-local prefix (no shared counter, and the
// record order is deterministic).  The write pass is bounded by construction: block b writes only below
// block_offsets[b + 1] (the scan's eg + 1 entries, the last one the total), so offsets that do not match this
// emission (a join range's second emission reusing its first's scanned offsets) cannot write past the buffer; a record
// that does not fit sets *block_counts (the overflow word of the write pass) and the host fails the build with
// RDF_ERR_LIMIT (g_emit_range)
template <bool WRITE, bool LAZY>
__global__ __launch_bounds__(RDF_BLOCK) void k_emit_records(const u32* __restrict__ s, const u32* __restrict__ p,
                                                            const u32* __restrict__ o, u64 n, u64 per, u32 V, u32 twoU,
                                                            const u32* __restrict__ frank, const u64* __restrict__ lkeys,
                                                            const u32* __restrict__ lvals, u64 lmask, int proj,
                                                            int joinbits, JoinSel js, u64* block_counts,
                                                            const u64* __restrict__ block_offsets, u64* out, int recbits) {
    __shared__ u32 lds_wave[RDF_WAVES_PER_BLOCK];
    __shared__ u64 htab[WRITE ? EMIT_DEDUP_SLOTS : 1];  // the iteration's distinct records (write pass)
    const u64 b = (u64)blockIdx.x * per;
    const u64 e = b + per < n ? b + per : n;
    if (!WRITE) {  // the block's record count: per-thread sums, one block reduction at the end
        u32 mine = 0;
        for (u64 i = b + threadIdx.x; i < e; i += RDF_BLOCK) {
            u64 rec[9];
            mine += triple_records<LAZY>(i, s, p, o, V, twoU, frank, lkeys, lvals, lmask, proj, joinbits, js, rec);
        }
        u32 total;
        block_exclusive_scan_u32(mine, lds_wave, &total);
        if (threadIdx.x == 0) block_counts[blockIdx.x] = total;
        return;
    }
    // region mode (block_offsets == nullptr, k_emit_compact after it): no count pass; the block writes its kept records
    // from 9 x per x block on and its kept count to block_counts, no padding
    const bool region = block_offsets == nullptr;
    const u64 rbase = region ? 9ull * per * blockIdx.x : 0ull;
    u64 run = region ? rbase : block_offsets[blockIdx.x];
    const u64 lim = region ? rbase + 9ull * per : block_offsets[blockIdx.x + 1];
    bool over = false;
    u64 emitted = 0;  // region mode: records emitted, repeats included (the run's n_records)
#ifndef RDF_EMIT_DEDUP
#define RDF_EMIT_DEDUP 1
#endif
    const bool dedup = RDF_EMIT_DEDUP && recbits <= 48;
    u32 tag = 0;
    if (dedup) {
        for (u32 k = threadIdx.x; k < (u32)EMIT_DEDUP_SLOTS; k += RDF_BLOCK) htab[k] = 0;  // tag 0: empty
        __syncthreads();
    }
    for (u64 i0 = b; i0 < e; i0 += RDF_BLOCK) {
        const u64 i = i0 + threadIdx.x;
        u64 rec[9];
        u32 c = 0, rep = 0;
        if (i < e) c = triple_records<LAZY>(i, s, p, o, V, twoU, frank, lkeys, lvals, lmask, proj, joinbits, js, rec, &rep);
        // Records repeated within the iteration's 256 triples (the same subject's predicate, the same (predicate,
        // object) pair: ~23 % of c2's records; only the kinds flagged by triple_records are looked up) are written
        // once; the count pass's region stays as it is and its tail is padded with EMIT_PAD, which the record sort's
        // first pass drops.  The LDS table slots carry the iteration's tag in bits 48.. (records have <= 48 bits
        // here), so it is cleared only when the tag wraps; the previous iteration's insertions finished before its
        // scan's barriers.
        u32 keep = (1u << c) - 1u;
        if (dedup) {
            ++tag;
            if (tag == (1u << 15)) {  // tags wrap: clear the table once
                __syncthreads();
                for (u32 k = threadIdx.x; k < (u32)EMIT_DEDUP_SLOTS; k += RDF_BLOCK) htab[k] = 0;
                __syncthreads();
                tag = 1;
            }
            keep = ((1u << c) - 1u) & ~rep;  // only the repeating kinds go through the table
            for (int k = 0; k < 9; ++k) {
                if ((u32)k >= c) break;
                if (!((rep >> k) & 1u)) continue;
                const u64 want = rec[k] | ((u64)tag << 48);
                u32 h = (u32)(mix64(rec[k]) >> 40) & (EMIT_DEDUP_SLOTS - 1);
                u64 cur = htab[h];
                while (true) {
                    if ((u32)(cur >> 48) != tag) {  // a slot of an earlier iteration: free
                        const u64 prev = atomicCAS((unsigned long long*)&htab[h], (unsigned long long)cur,
                                                   (unsigned long long)want);
                        if (prev == cur) {  // the first copy of the record: kept
                            keep |= 1u << k;
                            break;
                        }
                        cur = prev;
                        continue;
                    }
                    if (cur == want) break;  // a copy is kept by another record
                    h = (h + 1) & (EMIT_DEDUP_SLOTS - 1);
                    cur = htab[h];
                }
            }
        }
        // one scan of (kept, emitted) packed in 16-bit halves (each <= 9 x 256): this thread's kept records go to the
        // front of the iteration's region, its dropped ones become padding behind all kept records
        const u32 nk = (u32)__popc(keep);
        u32 tot;
        const u32 off = block_exclusive_scan_u32(nk | (c << 16), lds_wave, &tot);
        const u32 kept = tot & 0xffffu, total = tot >> 16;
        u64 q = run + (off & 0xffffu);
#pragma unroll
        for (int k = 0; k < 9; ++k)
            if ((keep >> k) & 1u) {
                if (q < lim) out[q] = rec[k];
                else over = true;
                ++q;
            }
        if (region) {
            run += kept;
            emitted += total;
            continue;
        }
        u64 pq = run + kept + ((off >> 16) - (off & 0xffffu));
        for (u32 k = nk; k < c; ++k, ++pq) {
            if (pq < lim) out[pq] = EMIT_PAD;
            else over = true;
        }
        run += total;
    }
    if (region && threadIdx.x == 0) {
        block_counts[blockIdx.x] = run - rbase;
        atomicAdd((unsigned long long*)(block_counts + gridDim.x), (unsigned long long)emitted);
    }
    if (!region && over) atomicOr((unsigned long long*)block_counts, 1ull);
}

// region mode's compaction: block b's kept records [9 x per x b, + cnt[b]) -> dst[off[b], + cnt[b]) (coalesced, 4 loads
// in flight per lane)
__global__ __launch_bounds__(RDF_BLOCK) void k_emit_compact(const u64* __restrict__ src, u64 region,
                                                            const u64* __restrict__ cnt, const u64* __restrict__ off,
                                                            u64* __restrict__ dst) {
    const u64 b = blockIdx.x, m = cnt[b];
    const u64* sp = src + b * region;
    u64* dp = dst + off[b];
    for (u64 i0 = threadIdx.x; i0 < m; i0 += 4ull * RDF_BLOCK) {
        u64 v[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) v[u] = i0 + (u64)u * RDF_BLOCK < m ? sp[i0 + (u64)u * RDF_BLOCK] : 0ull;
#pragma unroll
        for (int u = 0; u < 4; ++u)
            if (i0 + (u64)u * RDF_BLOCK < m) dp[i0 + (u64)u * RDF_BLOCK] = v[u];
    }
}

// K3 of every join range at once (the kept range build, g_emit_all_ranges): the records go to their range's region of
// rstore.  The per (range, block) counts come from the join histogram pass's block rows (k_range_block_counts), scanned
// into block_offsets (nr x gridDim.x + 1 entries, the last the total); a triple's records joined on one attribute (one
// join value, so one range) go to that range's block offset + an LDS cursor.  The order inside a block's region is free
// (every range is sorted afterwards), so the cursors need no scan.  A (range, block) region ends at the next offset:
// records past it are not written and set *overflow (the host fails the build: the histogram and this emission
// disagree).  Ranges: nr <= EMIT_MAX_RANGES ascending first join values rlo[0..nr), rlo[0] = 0.
static constexpr u32 EMIT_MAX_RANGES = 256;
__device__ inline u32 range_of(const u32* rlo, u32 nr, u32 j) {  // last k with rlo[k] <= j
    u32 a = 0, b = nr - 1;
    while (a < b) {
        const u32 m = (a + b + 1) >> 1;
        if (rlo[m] <= j) a = m;
        else b = m - 1;
    }
    return a;
}
template <bool LAZY>
__global__ __launch_bounds__(RDF_BLOCK) void k_emit_ranges(const u32* __restrict__ s, const u32* __restrict__ p,
                                                           const u32* __restrict__ o, u64 n, u64 per, u32 V, u32 twoU,
                                                           const u32* __restrict__ frank, const u64* __restrict__ lkeys,
                                                           const u32* __restrict__ lvals, u64 lmask, int proj,
                                                           int joinbits, JoinSel js, const u32* __restrict__ rlo_g, u32 nr,
                                                           u64* overflow, const u64* __restrict__ block_offsets,
                                                           u64* out, int recbits) {
    __shared__ u32 rlo[EMIT_MAX_RANGES];
    __shared__ u32 cur[EMIT_MAX_RANGES];
    __shared__ u64 base[EMIT_MAX_RANGES];
    __shared__ u64 lim[EMIT_MAX_RANGES];
    __shared__ u64 htab[EMIT_DEDUP_SLOTS];  // the iteration's distinct records
    for (u32 k = threadIdx.x; k < nr; k += RDF_BLOCK) {
        rlo[k] = rlo_g[k];
        cur[k] = 0;
        base[k] = block_offsets[(u64)k * gridDim.x + blockIdx.x];
        lim[k] = block_offsets[(u64)k * gridDim.x + blockIdx.x + 1];
    }
    const bool dedup = RDF_EMIT_DEDUP && recbits <= 48;
    if (dedup)
        for (u32 k = threadIdx.x; k < (u32)EMIT_DEDUP_SLOTS; k += RDF_BLOCK) htab[k] = 0;  // tag 0: empty
    __syncthreads();
    const u64 b = (u64)blockIdx.x * per;
    const u64 e = b + per < n ? b + per : n;
    u32 tag = 0;
    bool over = false;
    for (u64 i0 = b; i0 < e; i0 += RDF_BLOCK) {
        const u64 i = i0 + threadIdx.x;
        u64 rec[9];
        u32 c = 0, rep = 0, grp = 0;
        if (i < e) c = triple_records<LAZY>(i, s, p, o, V, twoU, frank, lkeys, lvals, lmask, proj, joinbits, js, rec, &rep, &grp);
        const u32 co = grp & 3u, cp = (grp >> 2) & 3u, cs = c - co - cp;
        u32 keep = (1u << c) - 1u;
        if (dedup) {  // as k_emit_records: the repeating kinds through the iteration's LDS table, the others kept
            ++tag;
            if (tag == (1u << 15)) {
                for (u32 k = threadIdx.x; k < (u32)EMIT_DEDUP_SLOTS; k += RDF_BLOCK) htab[k] = 0;
                __syncthreads();
                tag = 1;
            }
            keep = ((1u << c) - 1u) & ~rep;
            for (int k = 0; k < 9; ++k) {
                if ((u32)k >= c) break;
                if (!((rep >> k) & 1u)) continue;
                const u64 want = rec[k] | ((u64)tag << 48);
                u32 h = (u32)(mix64(rec[k]) >> 40) & (EMIT_DEDUP_SLOTS - 1);
                u64 cur_h = htab[h];
                while (true) {
                    if ((u32)(cur_h >> 48) != tag) {
                        const u64 prev = atomicCAS((unsigned long long*)&htab[h], (unsigned long long)cur_h,
                                                   (unsigned long long)want);
                        if (prev == cur_h) {
                            keep |= 1u << k;
                            break;
                        }
                        cur_h = prev;
                        continue;
                    }
                    if (cur_h == want) break;
                    h = (h + 1) & (EMIT_DEDUP_SLOTS - 1);
                    cur_h = htab[h];
                }
            }
        }
        // one LDS cursor claim per attribute group (its join value: o, p or s of the triple)
        u32 ro = 0, rp = 0, rs = 0;
        u64 qo = 0, qp = 0, qs = 0;
        if (co) ro = range_of(rlo, nr, o[i]);
        if (cp) rp = range_of(rlo, nr, p[i]);
        if (cs) rs = range_of(rlo, nr, s[i]);
        if (co) qo = base[ro] + atomicAdd(&cur[ro], co);
        if (cp) qp = base[rp] + atomicAdd(&cur[rp], cp) - co;
        if (cs) qs = base[rs] + atomicAdd(&cur[rs], cs) - co - cp;
#pragma unroll
        for (int k = 0; k < 9; ++k) {
            if ((u32)k >= c) break;
            const bool ko = (u32)k < co, kp = !ko && (u32)k < co + cp;
            const u64 q = (ko ? qo : kp ? qp : qs) + k;
            if (q < lim[ko ? ro : kp ? rp : rs]) out[q] = ((keep >> k) & 1u) ? rec[k] : EMIT_PAD;
            else over = true;
        }
        if (dedup) __syncthreads();  // the next iteration's tag reuses the table's slots
    }
    if (over) atomicOr((unsigned long long*)overflow, 1ull);
}

#ifndef RDF_JH_BITS
#define RDF_JH_BITS 14
#endif
static constexpr int JH_BITS = RDF_JH_BITS;
static constexpr u32 JH_BUCKETS = 1u << JH_BITS;  // join buckets of the join-range build (join >> jshift)
// ================================================================================================
// K4/K5: capture groups  (UnionJoinCandidates.combine / UnionCombinedJoinCandidates.reduce,
//     ALG/operators/UnionJoinCandidates.scala:27-44, UnionCombinedJoinCandidates.scala:21-31: distinct
//     captures per join value) and capture supports (depCount summed per group,
//     ALG/operators/candidate_merging/BulkMergeDependencies.scala:78-84)

// Sorted (capture << joinbits | join) records: fresh[i] = keys[i] differs from keys[i - 1] (a distinct
// (capture, join) pair), and the capture runs' bounds: cstart[c] = first record of capture c, for every
// c in [0, ncap] (captures without records get the next run's start; cstart[ncap] = n).
// Streaming kernels over the sorted records take STREAM_U elements per thread per step, their loads issued together
// (element step * U * T + u * T + thread: every load instruction stays coalesced).  One element per thread per step
// kept ~16 KB in flight per CU, which at 10^9-triple sizes (arrays far beyond the MALL) held these kernels near
// 1.5-2 TB/s.
#ifndef RDF_STREAM_U
#define RDF_STREAM_U 4
#endif
static constexpr int STREAM_U = RDF_STREAM_U;

static constexpr u64 CSTART_GAP = 64;  // run starts a k_fresh_bounds thread writes per gap of absent captures
__global__ __launch_bounds__(RDF_BLOCK) void k_fresh_bounds(const u64* __restrict__ keys, u64 n, u64 ncap, int joinbits,
                                                            u32* fresh, u32* cstart) {
    const u64 T = (u64)gridDim.x * RDF_BLOCK;
    for (u64 i0 = (u64)blockIdx.x * RDF_BLOCK + threadIdx.x; i0 <= n; i0 += T * STREAM_U) {
        u64 k[STREAM_U], kp[STREAM_U];
#pragma unroll
        for (int u = 0; u < STREAM_U; ++u) {
            const u64 i = i0 + (u64)u * T;
            k[u] = i < n ? keys[i] : 0ull;
            kp[u] = i && i <= n ? keys[i - 1] : 0ull;
        }
#pragma unroll
        for (int u = 0; u < STREAM_U; ++u) {
            const u64 i = i0 + (u64)u * T;
            if (i > n) break;
            if (i < n) fresh[i] = (i == 0 || kp[u] != k[u]) ? 1u : 0u;
            const u64 c = i < n ? k[u] >> joinbits : ncap;
            const u64 cp = i ? (kp[u] >> joinbits) + 1 : 0;
            // the captures in (previous record's, this record's]: at most CSTART_GAP of them here (the gap's end);
            // the rest of a longer gap keeps the caller's fill and k_cstart_fix finds it (a thread looping over a
            // gap of millions of absent captures -- a join range holding only high capture ids -- took 20 ms)
            for (u64 x = c + 1 > cp + CSTART_GAP ? c + 1 - CSTART_GAP : cp; x <= c; ++x) cstart[x] = (u32)i;
        }
    }
}

// run starts k_fresh_bounds left unwritten (cstart filled with ~0 before it): the first record of capture >= x
__global__ __launch_bounds__(RDF_BLOCK) void k_cstart_fix(const u64* __restrict__ keys, u64 n, u64 ncap, int joinbits,
                                                          u32* cstart) {
    for (u64 x = (u64)blockIdx.x * RDF_BLOCK + threadIdx.x; x <= ncap; x += (u64)gridDim.x * RDF_BLOCK)
        if (cstart[x] == ~0u) cstart[x] = (u32)(x == ncap ? n : lower_bound_u64(keys, n, x << joinbits));
}

// support of capture c = distinct join values among its records = fresh records of its run; fpos = exclusive
// scan of the fresh flags (fpos[n] = their total).  No atomics: a hot capture (s[p=rdf:type], in ~every
// group) is one subtraction.
__global__ __launch_bounds__(RDF_BLOCK) void k_run_support(const u32* __restrict__ cstart, u64 ncap,
                                                           const u32* __restrict__ fpos, u32* support) {
    for (u64 c = (u64)blockIdx.x * RDF_BLOCK + threadIdx.x; c < ncap; c += (u64)gridDim.x * RDF_BLOCK)
        support[c] = fpos[cstart[c + 1]] - fpos[cstart[c]];
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
// Fresh records of an infrequent capture are dropped; in (capture, join) order the kept ones of a capture
// stay contiguous, so a kept record's position is its fresh rank minus the fresh records of the infrequent
// captures before it.  skipv[c] = this rank's fresh records of c when c is infrequent (global support).
__global__ __launch_bounds__(RDF_BLOCK) void k_skip_counts(const u32* __restrict__ cstart, const u32* __restrict__ fpos,
                                                           const u32* __restrict__ support, u64 ncap, u32 ms, u32* skipv) {
    for (u64 c = (u64)blockIdx.x * RDF_BLOCK + threadIdx.x; c < ncap; c += (u64)gridDim.x * RDF_BLOCK)
        skipv[c] = support[c] >= ms ? 0u : fpos[cstart[c + 1]] - fpos[cstart[c]];
}

// kept records -> dk = (compact capture << 32 | join) in (capture, join) order (the dependent -> join CSR)
// and fk = (join << 32 | compact capture) at the same position (sorted by join next, for the groups)
__global__ __launch_bounds__(RDF_BLOCK) void k_keep_scatter(const u64* __restrict__ keys, u64 n, int joinbits,
                                                            const u32* __restrict__ fpos, const u32* __restrict__ skip,
                                                            const u32* __restrict__ support, u32 ms,
                                                            const u32* __restrict__ fidx, u64* dk, u64* fk) {
    const u64 jmask = (1ull << joinbits) - 1;
    const u64 T = (u64)gridDim.x * RDF_BLOCK;
    for (u64 i0 = (u64)blockIdx.x * RDF_BLOCK + threadIdx.x; i0 < n; i0 += T * STREAM_U) {
        u64 k[STREAM_U], kp[STREAM_U];
#pragma unroll
        for (int u = 0; u < STREAM_U; ++u) {
            const u64 i = i0 + (u64)u * T;
            k[u] = i < n ? keys[i] : 0ull;
            kp[u] = i && i < n ? keys[i - 1] : ~k[u];
        }
#pragma unroll
        for (int u = 0; u < STREAM_U; ++u) {
            const u64 i = i0 + (u64)u * T;
            if (i >= n || kp[u] == k[u]) continue;
            const u64 cap = k[u] >> joinbits;
            if (support[cap] < ms) continue;
            const u64 p = fpos[i] - skip[cap];
            const u64 c = fidx[cap], j = k[u] & jmask;
            dk[p] = (c << 32) | j;
            fk[p] = (j << 32) | c;
        }
    }
}

__global__ __launch_bounds__(RDF_BLOCK) void k_group_flags(const u64* __restrict__ fk, u64 n, u32* flags) {
    const u64 T = (u64)gridDim.x * RDF_BLOCK;
    for (u64 i0 = (u64)blockIdx.x * RDF_BLOCK + threadIdx.x; i0 < n; i0 += T * STREAM_U) {
        u64 a[STREAM_U], b[STREAM_U];
#pragma unroll
        for (int u = 0; u < STREAM_U; ++u) {
            const u64 i = i0 + (u64)u * T;
            a[u] = i < n ? fk[i] >> 32 : 0ull;
            b[u] = i && i < n ? fk[i - 1] >> 32 : ~a[u];
        }
#pragma unroll
        for (int u = 0; u < STREAM_U; ++u) {
            const u64 i = i0 + (u64)u * T;
            if (i < n) flags[i] = a[u] != b[u] ? 1u : 0u;
        }
    }
}

// groups: goff[g] = first record; gcap[i] = compact capture id; gmap[join] = g (fk = join << 32 | capture)
// STREAM_U elements per thread with their loads in flight together (a one-element grid-stride loop keeps one load per
// lane in flight and is latency-bound at ~2 TB/s)
__device__ inline void group_build_body(const u64* __restrict__ fk, u64 n, const u32* __restrict__ gflag,
                                        const u32* __restrict__ gexcl, u64 rbase, u32 gbase, u64* goff, u32* gcap,
                                        u32* gmap) {
    const u64 T = (u64)gridDim.x * RDF_BLOCK;
    for (u64 i0 = (u64)blockIdx.x * RDF_BLOCK + threadIdx.x; i0 < n; i0 += T * STREAM_U) {
        u64 k[STREAM_U];
        u32 f[STREAM_U], x[STREAM_U];
#pragma unroll
        for (int u = 0; u < STREAM_U; ++u) {
            const u64 i = i0 + (u64)u * T;
            k[u] = i < n ? fk[i] : 0ull;
            f[u] = i < n ? gflag[i] : 0u;
            x[u] = i < n ? gexcl[i] : 0u;
        }
#pragma unroll
        for (int u = 0; u < STREAM_U; ++u) {
            const u64 i = i0 + (u64)u * T;
            if (i >= n) break;
            gcap[rbase + i] = (u32)(k[u] & 0xffffffffu);
            if (f[u]) {
                const u32 g = gbase + x[u];
                goff[g] = rbase + i;
                gmap[k[u] >> 32] = g;
            }
        }
    }
}
__global__ __launch_bounds__(RDF_BLOCK) void k_group_build(const u64* __restrict__ fk, u64 n, const u32* __restrict__ gflag,
                                                           const u32* __restrict__ gexcl, u64* goff, u32* gcap, u32* gmap) {
    group_build_body(fk, n, gflag, gexcl, 0, 0u, goff, gcap, gmap);
}

// dependent -> groups: dgrp[i] = group of the join value of dk[i].  A capture's joins ascend and group ids
// are assigned in join order, so every dependent's group list comes out sorted.
__global__ __launch_bounds__(RDF_BLOCK) void k_dgrp(const u64* __restrict__ dk, u64 n, const u32* __restrict__ gmap, u32* dgrp) {
    const u64 T = (u64)gridDim.x * RDF_BLOCK;
    for (u64 i0 = (u64)blockIdx.x * RDF_BLOCK + threadIdx.x; i0 < n; i0 += T * STREAM_U) {
        u32 j[STREAM_U], g[STREAM_U];
#pragma unroll
        for (int u = 0; u < STREAM_U; ++u) j[u] = i0 + (u64)u * T < n ? (u32)dk[i0 + (u64)u * T] : 0u;
#pragma unroll
        for (int u = 0; u < STREAM_U; ++u) g[u] = i0 + (u64)u * T < n ? gmap[j[u]] : 0u;
#pragma unroll
        for (int u = 0; u < STREAM_U; ++u)
            if (i0 + (u64)u * T < n) dgrp[i0 + (u64)u * T] = g[u];
    }
}

__global__ __launch_bounds__(RDF_BLOCK) void k_info_support_u32(const CapInfo* __restrict__ info, u32 C, u32* out) {
    for (u64 i = (u64)blockIdx.x * RDF_BLOCK + threadIdx.x; i < C; i += (u64)gridDim.x * RDF_BLOCK) out[i] = info[i].support;
}

// offsets of a sorted (id << 32 | x) key array: off[d] = first key with id >= d, d in [0, C]
__global__ __launch_bounds__(RDF_BLOCK) void k_key_offsets(const u64* __restrict__ keys, u64 n, u32 C, u64* off) {
    for (u64 d = (u64)blockIdx.x * RDF_BLOCK + threadIdx.x; d <= C; d += (u64)gridDim.x * RDF_BLOCK)
        off[d] = lower_bound_u64(keys, n, d << 32);
}

// ---- capture groups built in join-value ranges (one GPU, more records than one sort pass holds) -----------------
// Records of join value j all lie in one range, so a range's groups are whole; ranges ascend, so group ids, the
// members of each group and every dependent's group list come out exactly as the one-pass build makes them.

// records per join bucket (join >> jshift, JH_BUCKETS buckets): the K3 count pass's per-triple record counts split by
// their join value (o, p or s of the triple), LDS-privatised per block of contiguous triples (the blocks of
// k_emit_ranges: per = ceil(n / gridDim.x)): the block's bucket counts -> bh[block * JH_BUCKETS + bucket], the totals
// -> hist.  A triple's records joined on one attribute share a join value: one LDS atomic per attribute
// (triple_records' group counts).
// 1024 threads per block: the 64-KB LDS histogram allows two blocks per CU, so the block is what sets the waves in
// flight for the gathers (256 threads: 2 waves per SIMD)
static constexpr int JH_BLOCK = 1024;
template <bool LAZY>
__global__ __launch_bounds__(JH_BLOCK) void k_emit_join_bhist(const u32* __restrict__ s, const u32* __restrict__ p,
                                                               const u32* __restrict__ o, u64 n, u64 per, u32 V, u32 twoU,
                                                               const u32* __restrict__ frank, const u64* __restrict__ lkeys,
                                                               const u32* __restrict__ lvals, u64 lmask, int proj,
                                                               int joinbits, JoinSel own, int jshift, u32* bh, u64* hist) {
    __shared__ u32 lh[JH_BUCKETS];
    for (u32 k = threadIdx.x; k < JH_BUCKETS; k += JH_BLOCK) lh[k] = 0;
    __syncthreads();
    JoinSel all = own;  // this rank's join values (sharded: hash or hot-table owner), every range
    all.lo = 0u;
    all.hi = JOIN_ALL_HI;
    const u64 b = (u64)blockIdx.x * per;
    const u64 e = b + per < n ? b + per : n;
    for (u64 i = b + threadIdx.x; i < e; i += JH_BLOCK) {
        u64 rec[9];
        u32 grp = 0;
        const u32 c = triple_records<LAZY>(i, s, p, o, V, twoU, frank, lkeys, lvals, lmask, proj, joinbits, all, rec,
                                           nullptr, &grp);
        const u32 co = grp & 3u, cp = (grp >> 2) & 3u, cs = c - co - cp;
        if (co) atomicAdd(&lh[o[i] >> jshift], co);
        if (cp) atomicAdd(&lh[p[i] >> jshift], cp);
        if (cs) atomicAdd(&lh[s[i] >> jshift], cs);
    }
    __syncthreads();
    u32* row = bh + (u64)blockIdx.x * JH_BUCKETS;
    for (u32 k = threadIdx.x; k < JH_BUCKETS; k += JH_BLOCK) {
        const u32 x = lh[k];
        row[k] = x;
        if (x) atomicAdd(&hist[k], (u64)x);
    }
}

// per (range, block) record counts from the blocks' bucket histograms: one wave per pair sums the range's buckets
// [blo[r], blo[r + 1]) of the block's row -> counts[r * nblk + block] (the layout k_emit_ranges' count pass writes)
__global__ __launch_bounds__(RDF_BLOCK) void k_range_block_counts(const u32* __restrict__ bh, u32 nblk,
                                                                  const u32* __restrict__ blo, u32 nr, u64* counts) {
    const u64 wv = ((u64)blockIdx.x * RDF_BLOCK + threadIdx.x) / RDF_WAVE;
    if (wv >= (u64)nr * nblk) return;
    const u32 r = (u32)(wv / nblk), blk = (u32)(wv % nblk);
    const u32* row = bh + (u64)blk * JH_BUCKETS;
    u32 acc = 0;  // a block's records: <= 9 per triple of its chunk, far below 2^32
    for (u32 k = blo[r] + lane_id(); k < blo[r + 1]; k += RDF_WAVE) acc += row[k];
    acc = wave_sum(acc);
    if (lane_id() == 0) counts[wv] = acc;
}

// a range's groups: goff[gbase + g] = rbase + first member, gcap[rbase + i], gmap[join] = gbase + g
__global__ __launch_bounds__(RDF_BLOCK) void k_group_build_at(const u64* __restrict__ fk, u64 n, const u32* __restrict__ gflag,
                                                              const u32* __restrict__ gexcl, u64 rbase, u32 gbase, u64* goff,
                                                              u32* gcap, u32* gmap) {
    group_build_body(fk, n, gflag, gexcl, rbase, gbase, goff, gcap, gmap);
}

// a range's dependent -> group entries: dk (compact capture << 32 | join, (capture, join) order) with this range's
// per-dependent offsets offp; dependent d's entries go behind the dcur[d] entries of earlier ranges
__global__ __launch_bounds__(RDF_BLOCK) void k_dgrp_range(const u64* __restrict__ dk, u64 n, const u64* __restrict__ offp,
                                                          const u64* __restrict__ doff, const u32* __restrict__ dcur,
                                                          const u32* __restrict__ gmap, u32* dgrp) {
    const u64 T = (u64)gridDim.x * RDF_BLOCK;
    for (u64 i0 = (u64)blockIdx.x * RDF_BLOCK + threadIdx.x; i0 < n; i0 += T * STREAM_U) {
        u64 k[STREAM_U];
#pragma unroll
        for (int u = 0; u < STREAM_U; ++u) k[u] = i0 + (u64)u * T < n ? dk[i0 + (u64)u * T] : 0ull;
        u32 g[STREAM_U];
        u64 at[STREAM_U];
#pragma unroll
        for (int u = 0; u < STREAM_U; ++u) {
            const u64 i = i0 + (u64)u * T;
            const u32 d = (u32)(k[u] >> 32);
            g[u] = i < n ? gmap[(u32)k[u]] : 0u;
            at[u] = i < n ? doff[d] + dcur[d] + (i - offp[d]) : 0ull;
        }
#pragma unroll
        for (int u = 0; u < STREAM_U; ++u)
            if (i0 + (u64)u * T < n) dgrp[at[u]] = g[u];
    }
}

__global__ __launch_bounds__(RDF_BLOCK) void k_dcur_add(const u64* __restrict__ offp, u32 C, u32* dcur) {
    for (u64 d = (u64)blockIdx.x * RDF_BLOCK + threadIdx.x; d < C; d += (u64)gridDim.x * RDF_BLOCK)
        dcur[d] += (u32)(offp[d + 1] - offp[d]);
}

__global__ __launch_bounds__(RDF_BLOCK) void k_add_u32(u32* a, const u32* __restrict__ b, u64 n) {
    for (u64 i = (u64)blockIdx.x * RDF_BLOCK + threadIdx.x; i < n; i += (u64)gridDim.x * RDF_BLOCK) a[i] += b[i];
}

// out[i] = v[idx[i]] (a frequent capture's local support, sharded join ranges)
__global__ __launch_bounds__(RDF_BLOCK) void k_gather_u32(const u32* __restrict__ v, const u32* __restrict__ idx, u64 n,
                                                          u32* out) {
    for (u64 i = (u64)blockIdx.x * RDF_BLOCK + threadIdx.x; i < n; i += (u64)gridDim.x * RDF_BLOCK) out[i] = v[idx[i]];
}


// ---- heavy groups: quarter-octave size buckets, then the top groups become bit columns
__device__ __host__ inline int size_bucket(u64 size) {
    if (size == 0) return 0;
    int msb = 63 - __builtin_clzll(size);
    int frac = msb >= 2 ? (int)((size >> (msb - 2)) & 3) : (int)((size << (2 - msb)) & 3);
    return 4 * msb + frac;
}

__global__ __launch_bounds__(RDF_BLOCK) void k_group_size_hist(const u64* __restrict__ goff, u64 G, u32* hist) {
    __shared__ u32 lh[256];
    lh[threadIdx.x] = 0;
    __syncthreads();
    for (u64 g = (u64)blockIdx.x * RDF_BLOCK + threadIdx.x; g < G; g += (u64)gridDim.x * RDF_BLOCK)
        atomicAdd(&lh[size_bucket(goff[g + 1] - goff[g])], 1u);
    __syncthreads();
    if (lh[threadIdx.x]) atomicAdd(&hist[threadIdx.x], lh[threadIdx.x]);
}

// heavy threshold on the device (single GPU: no host round trip between the histogram and the selection): the
// smallest size bucket such that the groups in it and above number at most HMAX, its smallest size, at least min_size;
// 0 = no heavy groups.  The same rule as the host's heavy_threshold (rdfind_hip.hip), which sharded runs use on the
// all-gathered histogram.
__global__ void k_heavy_threshold(const u32* __restrict__ hist, u64 min_size, u64* thr) {
    u64 cum = 0;
    int best = -1;
    for (int b = 255; b >= 0; --b) {
        cum += hist[b];
        if (cum > (u64)HMAX) break;
        if (hist[b]) best = b;
    }
    u64 t = 0;
    if (best >= 0) {
        t = 0;
        for (u64 sz = 1; sz < 64 && !t; ++sz)
            if (size_bucket(sz) == best) t = sz;
        if (!t) t = (u64)(4 + best % 4) << (best / 4 - 2);
        t = t > min_size ? t : min_size;
    }
    *thr = t;
}

__global__ __launch_bounds__(RDF_BLOCK) void k_heavy_select(const u64* __restrict__ goff, u64 G, u64 threshold_h,
                                                            const u64* __restrict__ threshold_d, u32 base,
                                                            u32* nheavy, u32* heavy_list, uint8_t* hbit) {
    const u64 threshold = threshold_d ? *threshold_d : threshold_h;
    for (u64 g = (u64)blockIdx.x * RDF_BLOCK + threadIdx.x; g < G; g += (u64)gridDim.x * RDF_BLOCK) {
        u64 sz = goff[g + 1] - goff[g];
        uint8_t b = LIGHT;
        if (threshold && sz >= threshold) {
            u32 j = atomicAdd(nheavy, 1u);
            if (base + j < (u32)HMAX) {
                b = (uint8_t)(base + j);
                heavy_list[j] = (u32)g;
            }
        }
        hbit[g] = b;
    }
}

// one block row per heavy column; with nheavy (device count) the grid has HMAX - base rows and the rows beyond the
// count exit
__global__ __launch_bounds__(RDF_BLOCK) void k_heavy_mask(const u64* __restrict__ goff, const u32* __restrict__ gcap,
                                                          const u32* __restrict__ heavy_list, u32 base, CapInfo* info,
                                                          const u32* __restrict__ nheavy) {
    const u32 h = blockIdx.y;
    if (nheavy && h >= *nheavy) return;
    const u32 g = heavy_list[h];
    const u64 b = goff[g], e = goff[g + 1];
    for (u64 i = b + (u64)blockIdx.x * RDF_BLOCK + threadIdx.x; i < e; i += (u64)gridDim.x * RDF_BLOCK)
        atomicOr(&info[gcap[i]].hmask, 1ull << (base + h));
}

// binary captures: components (unary compact ids) and keys; unary captures: parent counts
// binary captures: components (unary compact ids) and keys; parent edges (component << 32 | binary)
// are radix-sorted into the parents CSR (no per-unary cursor atomics: s[p=name] has thousands of parents)
__global__ __launch_bounds__(RDF_BLOCK) void k_binary_info(const u32* __restrict__ fcap, const u32* __restrict__ fidx,
                                                           const u64* __restrict__ bkeys, const u32* __restrict__ frank,
                                                           u32 C, u32 Cu, u32 V, u32 twoU, u32* bcomp, u64* bkeyc,
                                                           u64* pedges, CapInfo* info) {
    for (u64 c = Cu + (u64)blockIdx.x * RDF_BLOCK + threadIdx.x; c < C; c += (u64)gridDim.x * RDF_BLOCK) {
        u64 key = bkeys[fcap[c] - twoU];
        int bt = bin_key_type(key);
        // a frequent binary condition has frequent unary conditions, and its captures' components are
        // in every group the binary capture is in, so they are frequent captures too
        u32 c1 = fidx[ucap(frank, V, bin_comp1(bt), bin_key_v1(key))];
        u32 c2 = fidx[ucap(frank, V, bin_comp2(bt), bin_key_v2(key))];
        bcomp[2 * (c - Cu)] = c1;
        bcomp[2 * (c - Cu) + 1] = c2;
        bkeyc[c - Cu] = key;
        pedges[2 * (c - Cu)] = ((u64)c1 << 32) | c;
        pedges[2 * (c - Cu) + 1] = ((u64)c2 << 32) | c;
        info[c].meta |= META_BIN;
    }
}

// poff[u] = first edge of unary u; plist = low words; META_PARENTS for unary captures with parents
__global__ __launch_bounds__(RDF_BLOCK) void k_parents_csr(const u64* __restrict__ pedges, u64 npe, u32 Cu, u64* poff,
                                                           u32* plist, CapInfo* info) {
    for (u64 i = (u64)blockIdx.x * RDF_BLOCK + threadIdx.x; i < npe; i += (u64)gridDim.x * RDF_BLOCK)
        plist[i] = (u32)pedges[i];
    for (u64 u = (u64)blockIdx.x * RDF_BLOCK + threadIdx.x; u <= Cu; u += (u64)gridDim.x * RDF_BLOCK) {
        const u64 lo = lower_bound_u64(pedges, npe, u << 32);
        poff[u] = lo;
        if (u < Cu && lo < npe && (u32)(pedges[lo] >> 32) == u) info[u].meta |= META_PARENTS;
    }
}

// ================================================================================================
// K6: CIND extraction by intersection  (CreateAllCindCandidates.scala:71-121 + IntersectCindCandidates
//     .scala:14-51: the refs of a dependent A are the captures present in every group of A, i.e.
//     count(A,B) == support(A)).  A's smallest group (its pivot) bounds the candidates; the heavy-group
//     bitmask test (hmask(B) covers hmask(A)) verifies every heavy group at once, and the remaining light
//     groups are verified by binary search with one lane per group.  Deps whose groups are all heavy
//     ("heavy-only") need no verification: their refs are the pivot members passing the mask test.

// pivot pass, itemised: a work item is (dependent, segment of PIVOT_SEG of its groups), one wave each, so a
// dependent in ~every group (s[p=rdf:type]) is spread over many waves.  Items of a multi-segment dependent
// combine with atomicMin/atomicAdd; k_pivot_final derives the chunk counts.
// per-block partial sums of three counters -> part[3 * blockIdx.x + k] (reduced by k_sum_partials: one atomic per
// block on one address would serialise at the memory side, ~11 ns each)
__device__ inline void block_partials3(const u64 (&acc)[3], u64* part) {
    __shared__ u64 s_acc[3][RDF_WAVES_PER_BLOCK];
    for (int k = 0; k < 3; ++k) {
        u64 v = acc[k];
#pragma unroll
        for (int off = 32; off >= 1; off >>= 1) v += __shfl_xor(v, off, RDF_WAVE);
        if (lane_id() == 0) s_acc[k][threadIdx.x / RDF_WAVE] = v;
    }
    __syncthreads();
    if (threadIdx.x < 3) {
        u64 t = 0;
        for (int w = 0; w < RDF_WAVES_PER_BLOCK; ++w) t += s_acc[threadIdx.x][w];
        part[3ull * blockIdx.x + threadIdx.x] = t;
    }
}

// out[k] = sum over blocks of part[3 * b + k] (one block)
__global__ __launch_bounds__(RDF_BLOCK) void k_sum_partials3(const u64* __restrict__ part, u32 nblocks, u64* out) {
    __shared__ u64 s_acc[3][RDF_WAVES_PER_BLOCK];
    for (int k = 0; k < 3; ++k) {
        u64 v = 0;
        for (u32 b = threadIdx.x; b < nblocks; b += RDF_BLOCK) v += part[3ull * b + k];
#pragma unroll
        for (int off = 32; off >= 1; off >>= 1) v += __shfl_xor(v, off, RDF_WAVE);
        if (lane_id() == 0) s_acc[k][threadIdx.x / RDF_WAVE] = v;
    }
    __syncthreads();
    if (threadIdx.x < 3) {
        u64 t = 0;
        for (int w = 0; w < RDF_WAVES_PER_BLOCK; ++w) t += s_acc[threadIdx.x][w];
        out[threadIdx.x] = t;
    }
}

static constexpr u64 PIVOT_SEG = 4096;

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

static constexpr u64 PIVOT_SHORT = 32;  // dependents with at most this many groups: one lane each

__device__ inline u32 sig_bit(u32 g) { return (g * 0x9E3779B1u) >> (32 - SIG_LOG); }
__device__ inline void sig_add(u64 (&sg)[SIG_W], u32 g) {
    const u32 h = sig_bit(g);
#pragma unroll
    for (int k = 0; k < SIG_W; ++k) sg[k] |= (h >> 6) == (u32)k ? 1ull << (h & 63) : 0ull;
}

// segments of the long dependents (the short ones are done lane-per-dependent by k_pivot_short)
// owner[w] = d for every work item w in [off[d], off[d+1]) (replaces a binary search per work item)
__global__ __launch_bounds__(RDF_BLOCK) void k_expand_owner(const u64* __restrict__ off, u32 C, u32* owner) {
    for (u64 d = (u64)blockIdx.x * RDF_BLOCK + threadIdx.x; d < C; d += (u64)gridDim.x * RDF_BLOCK)
        for (u64 w = off[d]; w < off[d + 1]; ++w) owner[w] = (u32)d;
}
// the same for dependents [d0, d1), owner relative to off[d0]
__global__ __launch_bounds__(RDF_BLOCK) void k_expand_owner_range(const u64* __restrict__ off, u32 d0, u32 d1, u32* owner) {
    const u64 w0 = off[d0];
    for (u64 d = d0 + (u64)blockIdx.x * RDF_BLOCK + threadIdx.x; d < d1; d += (u64)gridDim.x * RDF_BLOCK)
        for (u64 w = off[d]; w < off[d + 1]; ++w) owner[w - w0] = (u32)d;
}

__global__ __launch_bounds__(RDF_BLOCK) void k_pivot_nseg(const u64* __restrict__ doff, u32 C, u32* nseg) {
    for (u64 d = (u64)blockIdx.x * RDF_BLOCK + threadIdx.x; d < C; d += (u64)gridDim.x * RDF_BLOCK) {
        const u64 len = doff[d + 1] - doff[d];
        nseg[d] = len > PIVOT_SHORT ? (u32)((len + PIVOT_SEG - 1) / PIVOT_SEG) : 0u;
    }
}

// The pivot pass visits every (dependent, group) entry once and tags the entries of heavy groups in place
// (DGRP_HEAVY): the light kernels then skip them without a per-group gather of hbit.
// the smallest light group other than the pivot, from the pivot key and the two smallest light keys
__device__ inline u32 second_pivot(u64 best, u64 l1, u64 l2) {
    const u64 k = (u32)l1 == (u32)best ? l2 : l1;
    return k == ~0ull ? NONE32 : (u32)k;
}
// the NP smallest light keys l[0..NP) of a dependent (ascending; distinct: one entry per group).  NP = EX + 2: the
// pivot may be l[0], then the second pivot, then EX extra pivots
template <int NP>
__device__ inline void smallest_k(u64 (&l)[NP], u64 key) {
    if (key >= l[NP - 1]) return;
    l[NP - 1] = key;
#pragma unroll
    for (int i = NP - 1; i > 0; --i)
        if (l[i] < l[i - 1]) {
            const u64 t = l[i - 1];
            l[i - 1] = l[i];
            l[i] = t;
        }
}
// the light groups after the second pivot: pivx[d * PIV_EXTRA + k] (NONE32 where there is none / k >= EX)
template <int NP>
__device__ inline void extra_pivots(u64 best, const u64 (&l)[NP], u32* pivx, u64 d) {
    const int s = (u32)l[0] == (u32)best ? 2 : 1;  // skip the pivot (if light) and the second pivot
#pragma unroll
    for (int k = 0; k < PIV_EXTRA; ++k) {
        const u64 x = s + k < NP ? l[s + k] : ~0ull;
        pivx[d * PIV_EXTRA + k] = x == ~0ull ? NONE32 : (u32)x;
    }
}

#ifndef RDF_PIVOT_U
#define RDF_PIVOT_U 4
#endif
static constexpr int PIVOT_U = RDF_PIVOT_U;  // group entries per lane whose loads are in flight together (pivot pass)
template <int EX>
__global__ __launch_bounds__(RDF_BLOCK) void k_pivot_short(CindView v, u32* dgrp_tag, u64* best_out, u32* nlight_out,
                                                           u64* sig, u32* piv2, u32* pivx) {
    constexpr int NPIV = EX + 2;
    for (u64 d = (u64)blockIdx.x * RDF_BLOCK + threadIdx.x; d < v.C; d += (u64)gridDim.x * RDF_BLOCK) {
        const u64 b = v.doff[d], e = v.doff[d + 1];
        if (e - b > PIVOT_SHORT) continue;
        u64 best = ~0ull;  // smallest group; the NPIV smallest light groups
        u64 l[NPIV];
#pragma unroll
        for (int k = 0; k < NPIV; ++k) l[k] = ~0ull;
        u32 nlight = 0;
        u64 sg[SIG_W] = {};
        for (u64 j0 = b; j0 < e; j0 += PIVOT_U) {  // PIVOT_U entries' loads, then their gathers, in flight together
            u32 raw[PIVOT_U], gi[PIVOT_U];
#pragma unroll
            for (int u = 0; u < PIVOT_U; ++u) raw[u] = j0 + u < e ? v.dgrp[j0 + u] : 0u;
#pragma unroll
            for (int u = 0; u < PIVOT_U; ++u) gi[u] = j0 + u < e ? v.ginfo[raw[u] & ~DGRP_HEAVY] : 0u;
#pragma unroll
            for (int u = 0; u < PIVOT_U; ++u) {
                const u64 j = j0 + u;
                if (j >= e) break;
                const u32 g = raw[u] & ~DGRP_HEAVY;
                const u64 key = ((u64)(gi[u] & ~GINFO_HEAVY) << 32) | g;
                best = key < best ? key : best;
                const bool light = !(gi[u] & GINFO_HEAVY);
                nlight += light;
                if (light) {
                    sig_add(sg, g);
                    smallest_k(l, key);
                }
                const u32 tagged = light ? g : (g | DGRP_HEAVY);
                if (tagged != raw[u]) dgrp_tag[j] = tagged;  // in place: light entries stay as they are (no rewrite)
            }
        }
        best_out[d] = best;
        nlight_out[d] = nlight;
        if (piv2) piv2[d] = second_pivot(best, l[0], l[1]);
        if (pivx) extra_pivots(best, l, pivx, d);
        if (sig)
#pragma unroll
            for (int k = 0; k < SIG_W; ++k) sig[d * SIG_W + k] = sg[k];
    }
}

template <int EX>
__device__ inline void k_pivot_seg_body(u64 vblk, CindView v, u32* dgrp_tag, const u64* __restrict__ segoff, u64 W,
                                        u64* best_out, u32* nlight_out, u64* sig, u32* piv2, u32* pivx) {
    constexpr int NPIV = EX + 2;
    const u64 w = (u64)vblk * RDF_WAVES_PER_BLOCK + threadIdx.x / RDF_WAVE;
    if (w >= W) return;
    const int lane = lane_id();
    const u32 d = find_dep(segoff, v.C, w);
    const u64 b0 = v.doff[d], e0 = v.doff[d + 1];
    const u64 b = b0 + (w - segoff[d]) * PIVOT_SEG;
    const u64 e = b + PIVOT_SEG < e0 ? b + PIVOT_SEG : e0;
    u64 best = ~0ull;  // (size << 32 | group): smallest; the NPIV smallest light
    u64 l[NPIV];
#pragma unroll
    for (int k = 0; k < NPIV; ++k) l[k] = ~0ull;
    u32 nlight = 0;
    u64 sg[SIG_W] = {};
    // PIVOT_U entries per lane at a time: their dgrp loads, then their ginfo gathers, each batch in flight together
    for (u64 j0 = b + lane; j0 < e; j0 += (u64)RDF_WAVE * PIVOT_U) {
        u32 raw[PIVOT_U], gi[PIVOT_U];
#pragma unroll
        for (int u = 0; u < PIVOT_U; ++u) {
            const u64 j = j0 + (u64)u * RDF_WAVE;
            raw[u] = j < e ? v.dgrp[j] : 0u;
        }
#pragma unroll
        for (int u = 0; u < PIVOT_U; ++u) gi[u] = j0 + (u64)u * RDF_WAVE < e ? v.ginfo[raw[u] & ~DGRP_HEAVY] : 0u;
#pragma unroll
        for (int u = 0; u < PIVOT_U; ++u) {
            const u64 j = j0 + (u64)u * RDF_WAVE;
            if (j >= e) break;
            const u32 g = raw[u] & ~DGRP_HEAVY;
            const u64 key = ((u64)(gi[u] & ~GINFO_HEAVY) << 32) | g;
            best = key < best ? key : best;
            const bool light = !(gi[u] & GINFO_HEAVY);
            nlight += light;
            if (light) {
                sig_add(sg, g);
                smallest_k(l, key);
            }
            const u32 tagged = light ? g : (g | DGRP_HEAVY);
            if (tagged != raw[u]) dgrp_tag[j] = tagged;
        }
    }
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) {
        u64 o = __shfl_xor(best, off, RDF_WAVE);
        best = o < best ? o : best;
        u64 ol[NPIV];
#pragma unroll
        for (int k = 0; k < NPIV; ++k) ol[k] = __shfl_xor(l[k], off, RDF_WAVE);
#pragma unroll
        for (int k = 0; k < NPIV; ++k) smallest_k(l, ol[k]);  // the lanes' keys are distinct (one entry per group)
#pragma unroll
        for (int k = 0; k < SIG_W; ++k) sg[k] |= __shfl_xor(sg[k], off, RDF_WAVE);
    }
    nlight = wave_sum(nlight);
    const bool single = e0 - b0 <= PIVOT_SEG;
    if (lane == 0) {
        if (single) {
            best_out[d] = best;
            nlight_out[d] = nlight;
            if (piv2) piv2[d] = second_pivot(best, l[0], l[1]);  // multi-segment dependents keep NONE32
            if (pivx) extra_pivots(best, l, pivx, d);
        } else {
            atomicMin(&best_out[d], best);
            atomicAdd(&nlight_out[d], nlight);
        }
    }
    if (sig && lane < SIG_W) {  // lane k writes word k (zeroed beforehand for the multi-segment dependents)
        u64 x = 0;
#pragma unroll
        for (int k = 0; k < SIG_W; ++k) x = lane == k ? sg[k] : x;
        if (single) sig[(u64)d * SIG_W + lane] = x;
        else if (x) atomicOr((unsigned long long*)&sig[(u64)d * SIG_W + lane], (unsigned long long)x);
    }
}
template <int EX>
__global__ __launch_bounds__(RDF_BLOCK) void k_pivot_seg(u64 nvblk, CindView v, u32* dgrp_tag,
                                                         const u64* __restrict__ segoff, u64 W, u64* best_out,
                                                         u32* nlight_out, u64* sig, u32* piv2, u32* pivx) {
    for (u64 vb = blockIdx.x; vb < nvblk; vb += gridDim.x) {
        k_pivot_seg_body<EX>(vb, v, dgrp_tag, segoff, W, best_out, nlight_out, sig, piv2, pivx);
    }
}


// Light work plan of dependent d (nlight light groups, pivot of sz captures).  Output slots are octets (8
// candidates of the pivot); noct[d] of them.  A dependent with few groups is "packed": one lane per
// candidate in k_light_packed, with candidates of many dependents sharing a wave.  The others get
// nitem[d] work items of k_light (chunk of 64 candidates x segment of LIGHT_SEG groups, one wave each).
__device__ inline void light_plan(const CindView& v, u32 d, u32 nlight, u64 sz, u32* noct, u32* nitem, u32* npacked) {
    if (!nlight) {
        noct[d] = nitem[d] = npacked[d] = 0;
        return;
    }
    const u64 ng = v.doff[d + 1] - v.doff[d];
    const u32 oc = (u32)((sz + 7) / 8);
    // packed: each lane walks all ng group entries (heavy ones are skipped by their tag) and searches the
    // light ones, so it pays when the groups are few or almost all heavy
    const bool packed = (ng <= LIGHT_PACK_MAXG && ng <= (sz > 4 ? sz : 4)) || (ng <= LIGHT_PACK_MAXG2 && nlight <= LIGHT_PACK_NL);
    noct[d] = oc;
    nitem[d] = packed ? 0u : (u32)((sz + RDF_WAVE - 1) / RDF_WAVE) * (u32)((ng + LIGHT_SEG - 1) / LIGHT_SEG);
    npacked[d] = packed ? oc : 0u;
}

__global__ __launch_bounds__(RDF_BLOCK) void k_pivot_final(CindView v, const u64* __restrict__ best_in,
                                                           const u32* __restrict__ nlight_in, u32* pivot, u32* nchunk_light,
                                                           u32* nitem_light, u32* npacked, u32* nchunk_heavy, CapInfo* info,
                                                           u64* heavy_candidates /* [3 * gridDim.x] partials */) {
    u64 acc[3] = {0, 0, 0};  // heavy candidates, light candidates, light entries
    for (u64 d = (u64)blockIdx.x * RDF_BLOCK + threadIdx.x; d < v.C; d += (u64)gridDim.x * RDF_BLOCK) {
        u32 hc = 0, lc = 0, le = 0;
        if (d < v.C) {
            const u64 best = best_in[d];
            const u32 nlight = nlight_in[d];
            const u64 sz = best >> 32;
            const u32 nch = (u32)((sz + RDF_WAVE - 1) / RDF_WAVE);
            pivot[d] = (u32)(best & 0xffffffffu);
            light_plan(v, (u32)d, nlight, sz, nchunk_light, nitem_light, npacked);
            if (nlight && nchunk_light[d]) {
                lc = (u32)sz;
                le = (u32)(v.doff[d + 1] - v.doff[d]);
            }
            // unary heavy-only dependents are emitted per bitmask class (k_class_*), binary ones by k_heavy; with
            // --use-ars every heavy-only dependent takes k_heavy (a class list is not per-dependent)
            const bool classed = d < v.Cu && !v.ar;
            nchunk_heavy[d] = (nlight || classed) ? 0 : nch;
            if (!nlight) {
                info[d].meta |= META_HEAVY_ONLY;
                if (!classed) hc = (u32)sz;
            }
        }
        acc[0] += hc;
        acc[1] += lc;
        acc[2] += le;
    }
    block_partials3(acc, heavy_candidates);
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

// K keys searched in one sorted array of n (> 0) distinct values; the K loads of a level are independent
template <int K>
__device__ inline void search_batch(const u32* __restrict__ a, u64 n, const u32 (&key)[K], bool (&found)[K]) {
    u64 base[K];
#pragma unroll
    for (int k = 0; k < K; ++k) base[k] = 0;
    if (!a) {
#pragma unroll
        for (int k = 0; k < K; ++k) found[k] = false;
        return;
    }
    while (n > 1) {
        const u64 half = n >> 1;
#pragma unroll
        for (int k = 0; k < K; ++k) base[k] = a[base[k] + half] <= key[k] ? base[k] + half : base[k];
        n -= half;
    }
#pragma unroll
    for (int k = 0; k < K; ++k) found[k] = a[base[k]] == key[k];
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
    if (is_trivial(v, x, y) || is_quirk(v, x, y) || ar_drop(v, x, y)) return false;
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
// rule_keep tests R1/R4 per pair.  R2/R3 are applied by "mark" passes instead (k_rules_mark,
// k_heavy_mark, k_class_mark): if a < X (raw) then joins(a) <= joins(X) <= joins(comp(X)), so every
// component of a raw binary ref X of a is itself a raw ref of a (or trivial).  The unary refs R2/R3 drop
// are therefore exactly the components of a's raw binary refs: each binary ref clears its (<= 2)
// components in a's own sorted ref list -- O(binary refs x log) instead of a scan of parents(R) per pair.
__device__ inline bool rule_keep(const CindView& v, u32 a, u32 r) {
    if (v.mode == RULES_NONE || a < v.Cu) return true;
    const u32* bc = v.bcomp + 2ull * (a - v.Cu);
    if (v.ar == AR_S2L && r < v.Cu)  // S2L's 2/1 candidates avoid every 1/1 CIND, AR-implied ones included (R1)
        return !(member(v, bc[0], r) || v.arref[bc[0]] == r || member(v, bc[1], r) || v.arref[bc[1]] == r);
    return !(member(v, bc[0], r) || member(v, bc[1], r));                               // R1 / R4
}

// position of capture x in the (ascending) member list of group g, or NONE
__device__ inline u64 group_pos(const CindView& v, u32 g, u32 x) {
    const u64 b = v.goff[g], n = v.goff[g + 1] - b;
    const u32* a = v.gcap + b;
    u64 lo = 0, hi = n;
    while (lo < hi) {
        const u64 mid = (lo + hi) >> 1;
        if (a[mid] < x) lo = mid + 1;
        else hi = mid;
    }
    return (lo < n && a[lo] == x) ? lo : ~0ull;
}


// exact member bitmap of a dense light group (null: g has none; search its member list)
__device__ inline const u32* dense_row(const CindView& v, u32 g) {
    if (!v.gdrow) return nullptr;
    const u32 r = v.gdrow[g];
    return r == NONE32 ? nullptr : v.dbits + (u64)r * v.dwords;
}
__device__ inline bool dense_has(const u32* row, u32 x) { return (row[x >> 5] >> (x & 31)) & 1u; }

// dense light groups: flags (light, >= dmin members) for the row numbering scan
// dmin = dmin_stage where the light pass will take the staging variant (member-weighted mean light group <=
// LIGHT_STAGE_AVG, from gsums = (sum n, sum n^2) of k_group_info: the same test the host makes after its read-back),
// else dmin_other
__global__ __launch_bounds__(RDF_BLOCK) void k_dense_flags(const u32* __restrict__ ginfo, u64 G, const u64* __restrict__ gsums,
                                                           u32 dmin_stage, u32 dmin_other, u32* flags) {
    const u32 dmin = gsums[1] <= (u64)LIGHT_STAGE_AVG * gsums[0] ? dmin_stage : dmin_other;
    for (u64 g = (u64)blockIdx.x * RDF_BLOCK + threadIdx.x; g < G; g += (u64)gridDim.x * RDF_BLOCK) {
        const u32 gi = ginfo[g];
        flags[g] = !(gi & GINFO_HEAVY) && gi >= dmin ? 1u : 0u;
    }
}
// rows >= cap (past the bitmap budget) stay member lists
__global__ __launch_bounds__(RDF_BLOCK) void k_dense_rows(const u32* __restrict__ flags, const u32* __restrict__ pos, u64 G,
                                                          u32 cap, u32* gdrow, u32* dlist) {
    for (u64 g = (u64)blockIdx.x * RDF_BLOCK + threadIdx.x; g < G; g += (u64)gridDim.x * RDF_BLOCK) {
        if (flags[g] && pos[g] < cap) {
            gdrow[g] = pos[g];
            dlist[pos[g]] = (u32)g;
        } else {
            gdrow[g] = NONE32;
        }
    }
}
// one block per dense row: zero it, then OR in the members (sorted, so a wave's lanes that hit the same word are
// merged by a segmented scan and only the segment's last lane issues the atomic)
__global__ __launch_bounds__(RDF_BLOCK) void k_dense_build(const u32* __restrict__ dlist, const u32* __restrict__ nrows,
                                                           u64 rows_max, const u64* __restrict__ goff,
                                                           const u32* __restrict__ gcap, u64 dwords, u32* dbits) {
    const u64 nr = *nrows;
    const int lane = lane_id();
    for (u64 r = blockIdx.x; r < nr && r < rows_max; r += gridDim.x) {
        u32* row = dbits + r * dwords;
        for (u64 w = threadIdx.x; w < dwords; w += RDF_BLOCK) row[w] = 0;
        __threadfence();
        __syncthreads();
        const u32 g = dlist[r];
        const u64 b = goff[g], e = goff[g + 1];
        for (u64 j0 = b; j0 < e; j0 += RDF_BLOCK) {
            const u64 j = j0 + threadIdx.x;
            const u32 x = j < e ? gcap[j] : NONE32;
            const u32 w = x == NONE32 ? NONE32 : x >> 5;
            u32 acc = x == NONE32 ? 0u : 1u << (x & 31);
#pragma unroll
            for (int off = 1; off < RDF_WAVE; off <<= 1) {
                const u32 ow = __shfl_up(w, off, RDF_WAVE), ob = __shfl_up(acc, off, RDF_WAVE);
                if (lane >= off && ow == w) acc |= ob;
            }
            const u32 nw = __shfl_down(w, 1, RDF_WAVE);
            if (w != NONE32 && (lane == RDF_WAVE - 1 || nw != w)) atomicOr(&row[w], acc);
        }
        __syncthreads();
    }
}

// ---- light dependents with identical group lists -------------------------------------------------------------
// Two captures that occur with exactly the same join values (LUBM: s[o=X] and s[p=P,o=X] when X only occurs as the
// object of P; 22 % of c2's light group entries belong to such dependents) have the same groups, support, heavy mask
// and light-group signature, so the light pass would verify the same candidates against the same groups twice.  The
// smallest compact id of such a class (its representative) is verified; every other member m takes the
// representative r's verified refs V(r) = out(r) + {r} + triv(r) (r itself and r's trivially implied components pass
// every test for m: their join sets contain r's), minus m and m's own trivially implied components, which are in V(r)
// for the same reason (IntersectCindCandidates.scala:40-43 intersects the same groups for both).
// key of a light dependent (its support, heavy mask, signature words and group count; 0: not a light dependent) -> key,
// and an open-addressing table (slots 2^k >= 2 C, EMPTY64 = free) of tag << 32 | the smallest dependent of the key: the
// slot comes from the low bits of the key's hash and the tag from its high 32, so one atomic claims or lowers a slot
// (two keys sharing a slot and a tag merge; k_dup_verify then finds their lists differ).  Members are often
// consecutive ids (the same join value under consecutive capture codes): a dependent whose predecessor in the wave has
// its key leaves the table alone (the predecessor is smaller), which keeps a large class off one slot.
__device__ inline u64 dup_key(const CindView& v, u32 d) {
    const CapInfo id = v.info[d];
    u64 h = mix64(((u64)id.support << 32) ^ (v.doff[d + 1] - v.doff[d])) ^ mix64(id.hmask + 0x9E3779B97F4A7C15ull);
    if (v.sig) {
        const u64* sd = v.sig + (u64)d * SIG_W;
#pragma unroll
        for (int k = 0; k < SIG_W; ++k) h = mix64(h ^ (sd[k] + (u64)k));
    }
    return h ? h : 1;
}
__device__ inline u64 dup_tag(u64 hk) {
    const u64 t = hk >> 32;
    return (t == 0xffffffffull ? 0xfffffffeull : t) << 32;
}
__global__ __launch_bounds__(RDF_BLOCK) void k_dup_insert(CindView v, const u32* __restrict__ nchunk_light, u64* key,
                                                          u64* tab, u64 tmask, u64 min_entries) {
    const u64 stride = (u64)gridDim.x * RDF_BLOCK;
    for (u64 d0 = (u64)blockIdx.x * RDF_BLOCK + (threadIdx.x & ~(RDF_WAVE - 1)); d0 < v.C; d0 += stride) {
        const u64 d = d0 + lane_id();
        // (only lists of >= min_entries groups, 256 by default: c2's classes average ~2,200 entries per member, and
        // the short lists' atomics cost more than their light work)
        const u64 k = d < v.C && nchunk_light[d] && v.doff[d + 1] - v.doff[d] >= min_entries ? dup_key(v, (u32)d) : 0;
        if (d < v.C) key[d] = k;
        const u64 kp = __shfl_up(k, 1, RDF_WAVE);
        if (!k || (lane_id() && kp == k)) continue;
        const u64 hk = mix64(k), tag = dup_tag(hk), want = tag | d;
        u64 h = hk & tmask;
        for (;;) {
            u64 cur = tab[h];  // a smaller id already there needs no atomic
            if (cur == EMPTY64)
                cur = atomicCAS((unsigned long long*)&tab[h], (unsigned long long)EMPTY64, (unsigned long long)want);
            if (cur == EMPTY64) break;
            if ((cur & 0xffffffff00000000ull) == tag) {
                if (want < cur) atomicMin((unsigned long long*)&tab[h], (unsigned long long)want);
                break;
            }
            h = (h + 1) & tmask;
        }
    }
}
// every light dependent's candidate representative (the smallest id of its key; crep[d] = d when none is smaller) and
// the 4096-entry chunks of its group list to compare with the representative's (0: nothing to compare)
static constexpr u64 DUP_CHUNK = 4096;
__global__ __launch_bounds__(RDF_BLOCK) void k_dup_rep(CindView v, const u64* __restrict__ key, const u64* __restrict__ tab,
                                                       u64 tmask, u32* crep, u32* nchunk, u32* bad) {
    for (u64 d = (u64)blockIdx.x * RDF_BLOCK + threadIdx.x; d < v.C; d += (u64)gridDim.x * RDF_BLOCK) {
        const u64 k = key[d];
        u32 r = (u32)d;
        if (k) {
            const u64 hk = mix64(k), tag = dup_tag(hk);
            u64 h = hk & tmask;
            while ((tab[h] & 0xffffffff00000000ull) != tag) h = (h + 1) & tmask;
            r = (u32)tab[h];
        }
        const u64 n = v.doff[d + 1] - v.doff[d];
        if (r != (u32)d && v.doff[r + 1] - v.doff[r] != n) r = (u32)d;  // (the key covers the length; a collision)
        crep[d] = r;
        nchunk[d] = r != (u32)d ? (u32)((n + DUP_CHUNK - 1) / DUP_CHUNK) : 0u;
        bad[d] = 0;
    }
}
// one wave per chunk of a candidate member's group list: any entry that differs from the representative's -> bad[d]
// (the lists are equal entry for entry exactly when the two captures have the same join values)
__global__ __launch_bounds__(RDF_BLOCK) void k_dup_verify(CindView v, const u32* __restrict__ crep,
                                                          const u64* __restrict__ ckoff, u32* bad) {
    const u64 W = ckoff[v.C];
    const u64 nw = (u64)gridDim.x * RDF_WAVES_PER_BLOCK;
    for (u64 w = (u64)blockIdx.x * RDF_WAVES_PER_BLOCK + threadIdx.x / RDF_WAVE; w < W; w += nw) {
        u32 lo = 0, hi = v.C;  // the member: last d with ckoff[d] <= w
        while (lo < hi) {
            const u32 mid = (lo + hi + 1) >> 1;
            if (ckoff[mid] <= w) lo = mid;
            else hi = mid - 1;
        }
        const u32 d = lo, r = crep[d];
        const u64 n = v.doff[d + 1] - v.doff[d];
        const u64 j0 = (w - ckoff[d]) * DUP_CHUNK, j1 = j0 + DUP_CHUNK < n ? j0 + DUP_CHUNK : n;
        const u32* a = v.dgrp + v.doff[d];
        const u32* b = v.dgrp + v.doff[r];
        bool diff = false;
        for (u64 j = j0 + lane_id(); j < j1; j += 8 * RDF_WAVE) {
            u32 x[8], y[8];
#pragma unroll
            for (int u = 0; u < 8; ++u) {
                const u64 jj = j + (u64)u * RDF_WAVE;
                x[u] = jj < j1 ? a[jj] : 0u;
                y[u] = jj < j1 ? b[jj] : 0u;
            }
#pragma unroll
            for (int u = 0; u < 8; ++u) diff |= x[u] != y[u];
        }
        if (__any(diff) && lane_id() == 0) bad[d] = 1;
    }
}
// verified members do no light work of their own (a member with a differing list is its own representative); the
// members are listed in `members` (in any order: their output offsets come from a scan) and counted in *nmembers
__global__ __launch_bounds__(RDF_BLOCK) void k_dup_unplan(u32* crep, const u32* __restrict__ bad, u32 C, u32* nchunk_light,
                                                          u32* nitem_light, u32* npacked, u32* nmembers, u32* members) {
    const u64 stride = (u64)gridDim.x * RDF_BLOCK;
    for (u64 d0 = (u64)blockIdx.x * RDF_BLOCK + (threadIdx.x & ~(RDF_WAVE - 1)); d0 < C; d0 += stride) {
        const u64 d = d0 + lane_id();
        bool mem = false;
        if (d < C) {
            const u32 r = crep[d];
            if (r != (u32)d && bad[d]) crep[d] = (u32)d;
            mem = r != (u32)d && !bad[d];
            if (mem) nchunk_light[d] = nitem_light[d] = npacked[d] = 0;
        }
        const u64 mask = __ballot(mem);
        if (!mask) continue;
        u32 base = 0;
        if (lane_id() == 0) base = atomicAdd(nmembers, (u32)__popcll(mask));
        base = __shfl(base, 0, RDF_WAVE);
        if (mem) members[base + __popcll(mask & ((1ull << lane_id()) - 1))] = (u32)d;
    }
}
__device__ inline u32 ntriv(const CindView& v, u32 x) { return x >= v.Cu ? 2u : 0u; }
// explicit pairs per dependent after the expansion: its own (eoff) or its representative's + 1 + triv(r) - 1 - triv(m)
__global__ __launch_bounds__(RDF_BLOCK) void k_dup_counts(CindView v, const u32* __restrict__ crep, const u64* __restrict__ eoff,
                                                          u32* cnt) {
    for (u64 d = (u64)blockIdx.x * RDF_BLOCK + threadIdx.x; d < v.C; d += (u64)gridDim.x * RDF_BLOCK) {
        const u32 r = crep[d];
        cnt[d] = (u32)(eoff[r + 1] - eoff[r]) + (r != (u32)d ? ntriv(v, r) - ntriv(v, (u32)d) : 0u);
    }
}
// non-members' pairs moved to their new offsets, and their ebin shifted by the same amount
__global__ __launch_bounds__(RDF_BLOCK) void k_dup_move(const u64* __restrict__ pairs, u64 E, u32 C, const u32* __restrict__ crep,
                                                        const u64* __restrict__ eoff, const u64* __restrict__ ebin,
                                                        const u64* __restrict__ noff, u64* out, u64* nbin) {
    for (u64 j = (u64)blockIdx.x * RDF_BLOCK + threadIdx.x; j < E || j < C; j += (u64)gridDim.x * RDF_BLOCK) {
        if (j < E) {
            const u64 x = pairs[j];
            const u32 d = (u32)(x >> 32);
            out[noff[d] + (j - eoff[d])] = x;
        }
        if (j < C && crep[j] == (u32)j) nbin[j] = noff[j] + (ebin[j] - eoff[j]);
    }
}
// one wave per member m (representative r): V(r) = out(r) + {r} + triv(r), ascending, without m and triv(m), written at
// noff[m]; nbin[m] = noff[m] + #{refs < Cu}
__global__ __launch_bounds__(RDF_BLOCK) void k_dup_expand(u64 nwaves, u64 nm, CindView v, const u32* __restrict__ members,
                                                          const u32* __restrict__ crep, const u64* __restrict__ pairs,
                                                          const u64* __restrict__ eoff, const u64* __restrict__ ebin,
                                                          const u64* __restrict__ noff, u64* out, u64* nbin) {
    const u64 w0 = (u64)blockIdx.x * RDF_WAVES_PER_BLOCK + threadIdx.x / RDF_WAVE;
    for (u64 w = w0; w < nm; w += nwaves) {
        const u64 m = members[w];
        const u32 r = crep[m];
        // the extras (r and its components) and the exclusions (m and its components): at most 3 each
        u32 ex[3], ne = 0, xs[3], nx = 0;
        ex[ne++] = r;
        if (r >= v.Cu) {
            ex[ne++] = v.bcomp[2ull * (r - v.Cu)];
            ex[ne++] = v.bcomp[2ull * (r - v.Cu) + 1];
        }
        xs[nx++] = (u32)m;
        if (m >= v.Cu) {
            xs[nx++] = v.bcomp[2ull * (m - v.Cu)];
            xs[nx++] = v.bcomp[2ull * (m - v.Cu) + 1];
        }
        const u64 b = eoff[r], n = eoff[r + 1] - b;
        const u64 base = noff[m];
        const u64 hi = m << 32;
        // a ref x of V(r) goes to rank(x) = #{V(r) < x} - #{exclusions < x}
        for (u64 i = lane_id(); i < n; i += RDF_WAVE) {
            const u32 x = (u32)pairs[b + i];
            bool drop = false;
            u32 below = (u32)i;
            for (u32 k = 0; k < ne; ++k) below += ex[k] < x;
            for (u32 k = 0; k < nx; ++k) {
                below -= xs[k] < x;
                drop |= xs[k] == x;
            }
            if (!drop) out[base + below] = hi | x;
        }
        if (lane_id() < ne) {
            const u32 x = ex[lane_id()];
            bool drop = false;
            u32 lo = 0, h2 = (u32)n;  // #out(r) < x
            while (lo < h2) {
                const u32 mid = (lo + h2) >> 1;
                if ((u32)pairs[b + mid] < x) lo = mid + 1;
                else h2 = mid;
            }
            u32 below = lo;
            for (u32 k = 0; k < ne; ++k) below += ex[k] < x;
            for (u32 k = 0; k < nx; ++k) {
                below -= xs[k] < x;
                drop |= xs[k] == x;
            }
            if (!drop) out[base + below] = hi | x;
        }
        if (lane_id() == 0) {  // refs below Cu: V(r)'s minus the exclusions'
            u32 below = (u32)(ebin[r] - b);
            for (u32 k = 0; k < ne; ++k) below += ex[k] < v.Cu;
            for (u32 k = 0; k < nx; ++k) below -= xs[k] < v.Cu;
            nbin[m] = base + below;
        }
    }
}

// candidate filter: the i-th member of the pivot group (or NONE)
__device__ inline u32 pivot_candidate(const CindView& v, u32 d, const CapInfo& id, u32 piv, u64 i) {
    if (v.vcoff) {  // sharded verify pass: the candidates are given (already filtered by the pivot holder)
        const u64 idx = v.vcoff[d] + i;
        return idx < v.vcoff[d + 1] ? (u32)v.vpairs[idx] : NONE32;
    }
    const u64 gb = v.goff[piv], ge = v.goff[piv + 1];
    const u64 idx = gb + i;
    if (idx >= ge) return NONE32;
    const u32 r = v.gcap[idx];
    if (r == d) return NONE32;
    const CapInfo ir = v.info[r];
    if (ir.support < id.support) return NONE32;
    if ((ir.hmask & id.hmask) != id.hmask) return NONE32;
    if (v.sig && !(id.meta & META_HEAVY_ONLY)) {  // light-group signature containment (dependent's words: uniform loads)
        const u64* sd = v.sig + (u64)d * SIG_W;
        const u64* sr = v.sig + (u64)r * SIG_W;
        u64 miss = 0;
#pragma unroll
        for (int k = 0; k < SIG_W; ++k) miss |= sd[k] & ~sr[k];
        if (miss) return NONE32;
    }
    if (is_trivial(v, d, r) || is_quirk(v, d, r) || ar_drop(v, d, r)) return NONE32;
    return r;
}

// candidate filter for a chunk of 64 pivot members: returns this lane's candidate (or NONE)
__device__ inline u32 chunk_candidate(const CindView& v, u32 d, const CapInfo& id, u32 piv, u64 chunk) {
    return pivot_candidate(v, d, id, piv, chunk * RDF_WAVE + lane_id());
}

// per group: ginfo = size | heavy << 31 (one 4-B gather for the pivot pass instead of two offsets + the heavy byte)
// part: per-block partials of (sum of light group sizes n, sum of n^2): the member-weighted mean light group size
// picks the light kernel's variant (k_light<STAGE>)
__global__ __launch_bounds__(RDF_BLOCK) void k_group_info(const u64* __restrict__ goff, const uint8_t* __restrict__ hbit,
                                                          u64 G, u32* ginfo, u64* part) {
    u64 acc[3] = {0, 0, 0};
    for (u64 g = (u64)blockIdx.x * RDF_BLOCK + threadIdx.x; g < G; g += (u64)gridDim.x * RDF_BLOCK) {
        const u64 n = goff[g + 1] - goff[g];
        const bool light = hbit[g] == LIGHT;
        ginfo[g] = (u32)n | (light ? 0u : GINFO_HEAVY);
        if (light) {
            acc[0] += n;
            acc[1] += n * n;
        }
    }
    block_partials3(acc, part);
}

// One group (members [gb, gb+gs)) checked for every alive candidate of the wave (lanes over candidates): a group of
// at most LIGHT_LDS members is staged into the wave's LDS slice by one coalesced load, so each search is LDS probes;
// a larger one is searched in place (the lanes share its top levels).  Returns the candidates still alive.
__device__ inline u64 check_group(const CindView& v, u64 gb, u32 gs, u32 cand, u64 alive, u32* buf, const u32* drow) {
    const int lane = lane_id();
    const bool mine = (alive >> lane) & 1ull;
    bool found = true;
    if (drow) {  // dense group: one bitmap word per candidate
        if (mine) found = dense_has(drow, cand);
    } else if (gs <= LIGHT_LDS) {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");  // earlier reads of buf precede the refill
        __builtin_amdgcn_wave_barrier();
        for (u32 k = lane; k < gs; k += RDF_WAVE) buf[k] = v.gcap[gb + k];
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        if (mine) {
            u32 lo = 0, hi = gs;
            while (lo < hi) {
                const u32 mid = (lo + hi) >> 1;
                if (buf[mid] < cand) lo = mid + 1;
                else hi = mid;
            }
            found = lo < gs && buf[lo] == cand;
        }
    } else if (mine) {
        found = bsearch_u32(v.gcap + gb, gs, cand);
    }
    return alive & __ballot(found);
}

// Survivors go to per-octet slots (8 candidates of a pivot each; no shared counter: a single global append
// counter serialises at the memory side); k_slot_compact packs the slots afterwards in slot order, which
// is (dependent, ref) order.  Lanes [8o, 8o+8) of the wave own octet oct0 + o; octets >= nvalid belong to
// the next dependent and are not touched.
__device__ inline void slot_emit(u64 oct0, u32 nvalid, u32 d, u32 cand, u64 alive, u64* slots, u32* counts) {
    const int lane = lane_id(), o = lane >> 3, j = lane & 7;
    if ((u32)o >= nvalid) return;
    const u32 om = (u32)(alive >> (o * 8)) & 0xffu;
    if (j == 0) counts[oct0 + o] = (u32)__popc(om);
    if ((om >> j) & 1u) slots[(oct0 + o) * 8 + __popc(om & ((1u << j) - 1u))] = ((u64)d << 32) | cand;
}

__device__ inline void k_slot_compact_body(u64 vblk, const u64* __restrict__ slots, const u32* __restrict__ counts,
                                           const u64* __restrict__ pos, u64 W, u64* out) {
    const u64 g = (u64)vblk * RDF_BLOCK + threadIdx.x;
    const u64 o = g >> 3;
    if (o >= W) return;
    const u32 j = (u32)(g & 7);
    if (j < counts[o]) out[pos[o] + j] = slots[g];
}
__global__ __launch_bounds__(RDF_BLOCK) void k_slot_compact(u64 nvblk, const u64* __restrict__ slots,
                                                            const u32* __restrict__ counts, const u64* __restrict__ pos,
                                                            u64 W, u64* out) {
    for (u64 vb = blockIdx.x; vb < nvblk; vb += gridDim.x) {
        k_slot_compact_body(vb, slots, counts, pos, W, out);
    }
}


// one key searched in K sorted arrays at once (n[k] == 0: no array); the loads of a level are independent
#ifndef RDF_PACK_STEP
#define RDF_PACK_STEP 4
#endif
static constexpr int PACK_STEP = RDF_PACK_STEP;  // group entries per step of the packed path
template <int K>
__device__ inline void multi_search(const u32* const (&a)[K], const u64 (&n)[K], u32 key, bool (&found)[K]) {
    u64 base[K], m[K];
    bool more = false;
#pragma unroll
    for (int k = 0; k < K; ++k) {
        base[k] = 0;
        m[k] = n[k];
        more |= m[k] > 1;
    }
    while (more) {
        more = false;
#pragma unroll
        for (int k = 0; k < K; ++k) {
            if (m[k] > 1) {
                const u64 half = m[k] >> 1;
                base[k] = a[k][base[k] + half] <= key ? base[k] + half : base[k];
                m[k] -= half;
            }
            more |= m[k] > 1;
        }
    }
#pragma unroll
    for (int k = 0; k < K; ++k) found[k] = n[k] && a[k][base[k]] == key;
}

// packed light dependents (few groups): one lane per pivot candidate, 8-lane octets, candidates of many
// dependents per wave.  Each lane walks its dependent's groups and binary-searches its candidate in every
// light one (the same test as k_light's few-groups path, without a mostly idle wave per dependent).
__device__ inline void k_light_packed_body(u64 vblk, CindView v, const u32* __restrict__ pivot,
                                           const u64* __restrict__ pkoff, const u32* __restrict__ pk_dep, u64 q0, u64 WP,
                                           const u64* __restrict__ choff, u64 ob, u64* slots, u32* counts) {
    const u64 g = (u64)vblk * RDF_BLOCK + threadIdx.x;
    if ((g >> 3) >= WP) return;  // whole octets only, so the octet ballots below see complete octets
    const u64 q = q0 + (g >> 3);  // packed octets [q0, q0 + WP); output octets relative to ob (paged runs)
    const u32 d = pk_dep[q];
    const u64 k = q - pkoff[d];
    const u32 piv = pivot[d];
    const CapInfo id = v.info[d];
    const u32 cand = pivot_candidate(v, d, id, piv, k * 8 + (g & 7));
    bool ok = cand != NONE32;
    const u32 p2 = v.piv2 ? v.piv2[d] : NONE32;  // the smallest light group after the pivot first (most kills)
    if (ok && p2 != NONE32 && !v.p2done) {
        const u32* dr2 = dense_row(v, p2);
        ok = dr2 ? dense_has(dr2, cand) : bsearch_u32(v.gcap + v.goff[p2], v.goff[p2 + 1] - v.goff[p2], cand);
    }
    const u32 p3 = v.pivx && v.npx ? v.pivx[(u64)d * PIV_EXTRA] : NONE32;  // ... then the next one
    if (ok && p3 != NONE32 && !v.p2done) {
        const u32* dr3 = dense_row(v, p3);
        ok = dr3 ? dense_has(dr3, cand) : bsearch_u32(v.gcap + v.goff[p3], v.goff[p3 + 1] - v.goff[p3], cand);
    }
    const u64 b = v.doff[d], e = v.doff[d + 1];
    // PACK_STEP group entries at a time: their ids, bounds and searches are independent loads (one round trip per
    // level for all of them instead of one chain per group)
    for (u64 j0 = b; ok && j0 < e; j0 += PACK_STEP) {
        u32 gr[PACK_STEP];
        const u32* ga[PACK_STEP];
        const u32* dr[PACK_STEP];
        u64 gn[PACK_STEP];
#pragma unroll
        for (int i = 0; i < PACK_STEP; ++i) gr[i] = j0 + i < e ? v.dgrp[j0 + i] : NONE32;  // heavy entries: DGRP_HEAVY
#pragma unroll
        for (int i = 0; i < PACK_STEP; ++i) {
            const bool lt = !(gr[i] == piv || gr[i] == p2 || gr[i] == p3 || (gr[i] & DGRP_HEAVY));
            dr[i] = lt ? dense_row(v, gr[i]) : nullptr;
            const u64 gb = lt ? v.goff[gr[i]] : 0;
            gn[i] = lt && !dr[i] ? v.goff[gr[i] + 1] - gb : 0;  // dense groups: a bitmap word instead of a search
            ga[i] = v.gcap + gb;
        }
        bool f[PACK_STEP];
        u32 dw[PACK_STEP];  // the dense groups' bitmap words, loaded together (not behind each other's test)
#pragma unroll
        for (int i = 0; i < PACK_STEP; ++i) dw[i] = dr[i] ? dr[i][cand >> 5] : ~0u;
        multi_search<PACK_STEP>(ga, gn, cand, f);
#pragma unroll
        for (int i = 0; i < PACK_STEP; ++i) ok = ok && (dr[i] ? ((dw[i] >> (cand & 31)) & 1u) != 0 : (gn[i] == 0 || f[i]));
    }
    const u64 alive = __ballot(ok);
    const int lane = lane_id(), o = lane >> 3, jj = lane & 7;
    const u32 om = (u32)(alive >> (o * 8)) & 0xffu;
    const u64 oct = choff[d] + k - ob;
    if (jj == 0) counts[oct] = (u32)__popc(om);
    if (ok) slots[oct * 8 + __popc(om & ((1u << jj) - 1u))] = ((u64)d << 32) | cand;
}
__global__ __launch_bounds__(RDF_BLOCK) void k_light_packed(u64 nvblk, CindView v, const u32* __restrict__ pivot,
                                                            const u64* __restrict__ pkoff,
                                                            const u32* __restrict__ pk_dep, u64 q0, u64 WP,
                                                            const u64* __restrict__ choff, u64 ob, u64* slots,
                                                            u32* counts) {
    for (u64 vb = blockIdx.x; vb < nvblk; vb += gridDim.x) {
        k_light_packed_body(vb, v, pivot, pkoff, pk_dep, q0, WP, choff, ob, slots, counts);
    }
}


#ifdef RDF_LIGHT_STATS
// dev instrumentation (make stats): one 16 x u32 record per k_light work item, written by lane 0 without atomics:
// [0] dep [1] groups of the dependent [2] groups of this segment [3] nseg [4] pivot size [5] alive0 [6] alive at exit
// [7] 64-group windows visited [8] groups taken by the serial path [9] batch rounds [10] sum of batch search depths
// [11] light groups in visited windows [12..13] clock64 cycles [14] sum of visited light group sizes [15] largest
__device__ u32* g_item_rec;
#define LSTAT_T0 const unsigned long long lstat_t0 = clock64(); u32 ls_win = 0, ls_ser = 0, ls_bat = 0, ls_dep = 0, ls_lg = 0, ls_gs = 0, ls_gmax = 0; \
    unsigned long long ls_ph[6] = {0, 0, 0, 0, 0, 0}, ls_tic = 0
// phase timers (cycles): [0] second pivot, [1] window metadata loads, [2] dense groups, [3] serial groups, [4] sweeps,
// [5] batches
#define LSTAT_TIC() (ls_tic = clock64())
#define LSTAT_TOC(k) (ls_ph[k] += clock64() - ls_tic)
#define LSTAT_WIN(lmask, gsz) do { ++ls_win; ls_lg += __popcll(lmask); ls_gs += wave_sum((u32)(gsz)); \
    u32 m_ = (u32)(gsz); for (int o_ = 32; o_ >= 1; o_ >>= 1) { u32 t_ = __shfl_xor(m_, o_, RDF_WAVE); m_ = t_ > m_ ? t_ : m_; } \
    ls_gmax = m_ > ls_gmax ? m_ : ls_gmax; } while (0)
#define LSTAT_SER(k) (ls_ser += (k))
#define LSTAT_BAT(depth) do { ++ls_bat; ls_dep += (depth); } while (0)
#else
#define LSTAT_T0 do { } while (0)
#define LSTAT_TIC() do { } while (0)
#define LSTAT_TOC(k) do { } while (0)
#define LSTAT_WIN(lmask, gsz) do { } while (0)
#define LSTAT_SER(k) do { } while (0)
#define LSTAT_BAT(depth) do { } while (0)
#endif

// one batch of the group-parallel window: the next K alive candidates (taken from todo) searched in every lane's
// group gm (g == NONE32: no group in this lane); a candidate missing from any lane's group dies
template <int K>
__device__ inline void light_batch(const u32* gm, u64 gsz, const u32* drow, u32 g, u32 cand, u64& todo, u64& alive) {
    int bit[K];
    u32 key[K];
#pragma unroll
    for (int k = 0; k < K; ++k) {
        bit[k] = todo ? __ffsll((long long)todo) - 1 : -1;
        todo &= todo - 1;
        key[k] = __shfl(cand, bit[k] < 0 ? bit[0] : bit[k], RDF_WAVE);
    }
    bool ok[K];
    if (drow) {  // dense group: K independent bitmap words
#pragma unroll
        for (int k = 0; k < K; ++k) ok[k] = dense_has(drow, key[k]);
    } else {
        search_batch<K>(gm, gsz, key, ok);
    }
#pragma unroll
    for (int k = 0; k < K; ++k)
        if (bit[k] >= 0 && !__all(g == NONE32 || ok[k])) alive &= ~(1ull << bit[k]);
}

// Range sweep of a window (lanes over its groups, many candidates alive).  A candidate-major batch searches every alive
// candidate in every lane's group: per (candidate, group) a ~log2(n)-level chain of divergent loads.  The alive
// candidates of a chunk are consecutive pivot members, so they span a narrow slice of the capture-id space: each lane
// bounds its group's members to [min, max] of the alive candidates (two searches in flight), and when those members are
// few against the searches they replace, the wave reads them all instead -- coalesced, SWEEP_U loads in flight per lane, the
// window's ranges concatenated so every lane stays busy -- and marks the candidates each group holds.  Returns false
// (nothing done) when the slices are too large for that to pay; the caller then batches as before.
// LDS per wave (the light pass's 2 KB slice): member starts (u64) and range prefix (u32) per lane, the lanes' candidates,
// the per-group found masks (u64).
#ifndef RDF_SWEEP_U
#define RDF_SWEEP_U 8
#endif
static constexpr int SWEEP_U = RDF_SWEEP_U;
__device__ inline bool light_sweep(const CindView& v, const u32* gm, u64 gsz, u32 g, u32 cand, u64& alive, u32* buf) {
    const int lane = lane_id();
    const bool mine = (alive >> lane) & 1ull;
    u32 cmn = mine ? cand : 0xffffffffu, cmx = mine ? cand : 0u;
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) {
        const u32 a = __shfl_xor(cmn, off, RDF_WAVE), b = __shfl_xor(cmx, off, RDF_WAVE);
        cmn = a < cmn ? a : cmn;
        cmx = b > cmx ? b : cmx;
    }
    u64 lo = 0, hi = 0;
    if (g != NONE32 && gsz) {  // lower_bound(cmn), upper_bound(cmx): two independent chains
        u64 b0 = 0, n0 = gsz, b1 = 0, n1 = gsz;
        while (n0 > 0 || n1 > 0) {
            if (n0 > 0) {
                const u64 h = n0 >> 1;
                if (gm[b0 + h] < cmn) { b0 += h + 1; n0 -= h + 1; } else n0 = h;
            }
            if (n1 > 0) {
                const u64 h = n1 >> 1;
                if (gm[b1 + h] <= cmx) { b1 += h + 1; n1 -= h + 1; } else n1 = h;
            }
        }
        lo = b0;
        hi = b1 > b0 ? b1 : b0;
    }
    const u32 r = (u32)(hi - lo);
    const u32 incl = wave_inclusive_scan(r);
    const u32 R = __shfl(incl, RDF_WAVE - 1, RDF_WAVE);
    // cost model: a batch round searches 8 alive candidates in every lane's group, ~L = log2(mean group size) levels of
    // divergent loads; the sweep reads R members, SWEEP_U x 64 per round plus LDS lookups.  Sweep when
    // R <= sweep_f x alive x L (measured: sweep_f 16 beat 64 and 256 on c4, whose wide slices made 64 ~2x slower)
    u32 lv = g != NONE32 && gsz > 1 ? 64 - __clzll(gsz - 1) : 0;
    const u32 nl = (u32)__popcll(__ballot(g != NONE32));
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) lv += __shfl_xor(lv, off, RDF_WAVE);
    const u64 L = nl ? (lv + nl - 1) / nl : 1;
    if ((u64)R > (u64)v.sweep_f * (u64)__popcll(alive) * L) return false;
    u64* s_start = (u64*)buf;                 // [64] first member of each lane's slice (global index into gcap)
    u32* s_pre = buf + 2 * RDF_WAVE;          // [65] exclusive prefix of the slice lengths
    u32* s_cand = s_pre + RDF_WAVE + 1;       // [64] the lanes' candidates (ascending)
    u64* s_found = (u64*)(buf + 4 * RDF_WAVE + 2);  // [64] candidates found in lane l's group (8-B aligned: 258 words)
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");  // earlier reads of buf precede the refill
    __builtin_amdgcn_wave_barrier();
    s_start[lane] = (u64)(gm - v.gcap) + lo;
    s_pre[lane] = incl - r;
    if (lane == 0) s_pre[RDF_WAVE] = R;
    // the lanes' candidates, ascending: a lane without an alive candidate repeats the nearest alive one below it, so a
    // lower bound lands on the alive lane (pivot members ascend by lane; filtered lanes hold NONE32)
    u32 cv = mine ? cand : 0u;
#pragma unroll
    for (int off = 1; off < RDF_WAVE; off <<= 1) {
        const u32 t = __shfl_up(cv, off, RDF_WAVE);
        if (lane >= off) cv = t > cv ? t : cv;
    }
    s_cand[lane] = cv;
    s_found[lane] = 0;
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    for (u32 base = 0; base < R; base += SWEEP_U * RDF_WAVE) {
        u32 x[SWEEP_U];
        int owner[SWEEP_U];
#pragma unroll
        for (int u = 0; u < SWEEP_U; ++u) {
            const u32 f = base + (u32)u * RDF_WAVE + (u32)lane;
            owner[u] = -1;
            x[u] = 0;
            if (f < R) {
                int a = 0, b = RDF_WAVE - 1;  // last lane whose slice starts at or before f
                while (a < b) {
                    const int m = (a + b + 1) >> 1;
                    if (s_pre[m] <= f) a = m;
                    else b = m - 1;
                }
                owner[u] = a;
                x[u] = v.gcap[s_start[a] + (f - s_pre[a])];
            }
        }
#pragma unroll
        for (int u = 0; u < SWEEP_U; ++u) {
            if (owner[u] < 0) continue;
            int a = 0, b = RDF_WAVE;  // lower_bound of the member among the 64 candidates
            while (a < b) {
                const int m = (a + b) >> 1;
                if (s_cand[m] < x[u]) a = m + 1;
                else b = m;
            }
            if (a < RDF_WAVE && s_cand[a] == x[u]) atomicOr((unsigned long long*)&s_found[owner[u]], 1ull << a);
        }
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    u64 keep = g != NONE32 ? s_found[lane] : ~0ull;
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) keep &= __shfl_xor(keep, off, RDF_WAVE);
    alive &= keep;
    return true;
}

// light dependents: a work item is (dependent, chunk of 64 pivot candidates, segment of LIGHT_SEG of the
// dependent's groups).  Single-segment dependents emit their explicit (dep << 32 | ref) pairs directly;
// multi-segment ones publish the candidates they kill with atomicOr, and the last segment to finish emits.
template <bool STAGE>
__device__ inline void k_light_body(u64 vblk, CindView v, const u32* __restrict__ pivot,
                                    const u64* __restrict__ itemoff, const u32* __restrict__ item_dep,
                                    const u64* __restrict__ choff, u64 w0, u64 W, u64 ob, u64* dead, u64* slots,
                                    u32* counts, const u32* __restrict__ order) {
    // a staged group, or (STAGE) the lanes' small-group rows.  The larger buffer is only allocated by the variant
    // that uses it: on c3 (large light groups) 31.7 KB per block cost 30 % of the kernel even with the path unused
    __shared__ u32 s_light[RDF_WAVES_PER_BLOCK][STAGE ? LIGHT_BUF : LIGHT_LDS];
    const u64 wq = (u64)vblk * RDF_WAVES_PER_BLOCK + threadIdx.x / RDF_WAVE;
    if (wq >= W) return;
    const u64 wl = order ? order[wq] : wq;  // the long items first (k_light_order), so none starts last
    const u64 w = w0 + wl;  // work items [w0, w0 + W); octets relative to ob (paged runs)
    const int lane = lane_id();
    const u32 d = item_dep[w];
    const u64 b0 = v.doff[d], e0 = v.doff[d + 1];
    const u64 nseg = (e0 - b0 + LIGHT_SEG - 1) / LIGHT_SEG;
    const u64 item = w - itemoff[d];
    const u64 chunk = item / nseg, seg = item % nseg;
    const u32 piv = pivot[d];
    const CapInfo id = v.info[d];
    const u64 b = b0 + seg * LIGHT_SEG;
    const u64 e = b + LIGHT_SEG < e0 ? b + LIGHT_SEG : e0;
    // The dependent's smallest light groups after the pivot first, lanes over candidates: they kill most doomed
    // candidates with one (often LDS-staged) search each before the group-parallel windows below.  (Issuing the first
    // window's metadata loads before the candidate filter's was measured: c2 -0.8 %, c4 +19 %: the items whose
    // candidates all fail the filter paid for loads they never use.)
    const u32 p2 = v.piv2 ? v.piv2[d] : NONE32;
    // the extra pivots (plain variant only: the staging variant's inputs, c2, lose with them); read in a rolled loop
    // below, not held in registers (four unrolled checks cost the plain variant an occupancy step: 130 VGPRs)
    const u32* pxs = !STAGE && v.pivx && v.npx ? v.pivx + (u64)d * PIV_EXTRA : nullptr;
    u32 gg[LIGHT_IT];
    u64 gbv[LIGHT_IT];
    u32 gszv[LIGHT_IT];
    const u32* gdr[LIGHT_IT];
    const u32 cand = chunk_candidate(v, d, id, piv, chunk);
    const u64 alive0 = __ballot(cand != NONE32);
    u64 alive = alive0;
    LSTAT_T0;
    // pass A (prefilter): a chunk of a dependent of several chunks with few candidates left after the filters and the
    // second pivot is not verified here; its survivors go out tagged (item seg 0) and pass B verifies them compacted
    const bool multi = v.prefilter && itemoff[d + 1] - itemoff[d] > nseg;
    LSTAT_TIC();
    if (p2 != NONE32 && alive && !v.p2done) {
        const u64 gb2 = v.goff[p2];
        alive = check_group(v, gb2, (u32)(v.goff[p2 + 1] - gb2), cand, alive, s_light[threadIdx.x / RDF_WAVE],
                            dense_row(v, p2));
    }
    // the next smallest light groups too: the candidates that survive the second pivot mostly die in the first
    // window's searches (c3: half of the light cycles), one targeted check each (lanes over candidates) before it
    if (pxs && !v.p2done) {
#pragma unroll 1
        for (int k = 0; k < v.npx && alive; ++k) {
            const u32 pk = pxs[k];
            if (pk == NONE32) break;  // ascending: no more light groups
            const u64 gb3 = v.goff[pk];
            alive = check_group(v, gb3, (u32)(v.goff[pk + 1] - gb3), cand, alive, s_light[threadIdx.x / RDF_WAVE],
                                dense_row(v, pk));
        }
    }
    LSTAT_TOC(0);
    if (multi && __popcll(alive) <= LIGHT_PRE_MAX) {  // every segment item of the chunk reaches the same decision
        if (seg == 0) {
            const u64 oct0 = choff[d] + chunk * 8 - ob;
            const u64 noct = choff[d + 1] - ob - oct0;
            slot_emit(oct0, noct < 8 ? (u32)noct : 8u, d, cand | PRE_TAG, alive, slots, counts);
            if (nseg > 1 && lane == 0) dead[oct0] = ~0ull;  // k_light_mseg_emit leaves the chunk alone
        }
        return;
    }
    // Lanes take one group each (LIGHT_IT per lane); dependents with few groups went to k_light_packed, so
    // here groups outnumber candidates.  The segment's group metadata is loaded up front, LIGHT_IT
    // independent gathers per level, so the serial chain is three round trips per segment, not per 64 groups.
    for (u64 s0 = b; s0 < e && alive; s0 += (u64)LIGHT_IT * RDF_WAVE) {
        LSTAT_TIC();
#pragma unroll
        for (int it = 0; it < LIGHT_IT; ++it) {
            const u64 j = s0 + (u64)it * RDF_WAVE + lane;
            gg[it] = j < e ? v.dgrp[j] : NONE32;
        }
#pragma unroll
        for (int it = 0; it < LIGHT_IT; ++it)
            if (gg[it] == piv || gg[it] == p2 || (gg[it] & DGRP_HEAVY))  // the extra pivots stay (their re-check is
                gg[it] = NONE32;  // one group of a window); NONE32 carries DGRP_HEAVY
#pragma unroll
        for (int it = 0; it < LIGHT_IT; ++it) {
            gbv[it] = 0;
            gszv[it] = 0;
            gdr[it] = nullptr;
            if (gg[it] != NONE32) {
                gbv[it] = v.goff[gg[it]];
                gszv[it] = (u32)(v.goff[gg[it] + 1] - gbv[it]);
                gdr[it] = dense_row(v, gg[it]);
            }
        }
#ifdef RDF_LIGHT_STATS
        { u32 x = gszv[0] + (u32)gbv[0]; asm volatile("" : : "v"(x)); }  // stats: the metadata loads have arrived
#endif
        LSTAT_TOC(1);
#pragma unroll
        for (int it = 0; it < LIGHT_IT; ++it) {
            if (s0 + (u64)it * RDF_WAVE >= e) break;
            // a multi-segment item drops the candidates other segments have already killed
            if (nseg > 1 && (it || s0 != b)) alive &= ~__hip_atomic_load(&dead[choff[d] + chunk * 8 - ob], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            if (!alive) break;
            u32 g = gg[it];
            u64 lm = __ballot(g != NONE32);  // light groups of this window
            LSTAT_WIN(lm, gszv[it]);
            const u64 dm = __ballot(gdr[it] != nullptr);  // ... of which dense (member bitmaps)
            LSTAT_TIC();
            if (dm && __popcll(alive) >= LIGHT_DENSE_SER) {
                // many candidates alive: the dense groups one at a time with the lanes over the candidates.  The
                // candidates are ascending pivot members, so a group's 64 tests hit a few lines of its bitmap row
                // (lanes over groups would touch 64 rows per candidate).  LIGHT_DENSE_BATCH groups' bitmap words are
                // loaded unconditionally before any is tested, so they are in flight together (a short-circuit test
                // per group would make each load wait for the previous one's result)
                u64 t = dm;
                while (t && alive) {
                    const bool mine = (alive >> lane) & 1ull;
                    u32 wv[LIGHT_DENSE_BATCH];
#pragma unroll
                    for (int k = 0; k < LIGHT_DENSE_BATCH; ++k) {
                        const int l = t ? __ffsll((long long)t) - 1 : -1;
                        t &= t - 1;
                        const u32* dr = l < 0 ? nullptr : (const u32*)__shfl((unsigned long long)gdr[it], l, RDF_WAVE);
                        wv[k] = mine && dr ? dr[cand >> 5] : ~0u;
                    }
                    u32 all = ~0u;
#pragma unroll
                    for (int k = 0; k < LIGHT_DENSE_BATCH; ++k) all &= wv[k];
                    alive &= __ballot(!mine || ((all >> (cand & 31)) & 1u));
                }
                if (gdr[it]) g = NONE32;  // what is left: the sparse light groups of the window
                lm = __ballot(g != NONE32);
                LSTAT_TOC(2);
                if (!lm || !alive) continue;
            }
            if (__popcll(lm) <= LIGHT_SERIAL) {
                // few light groups (the common case: most groups of a dependent are heavy and verified by the
                // mask test): take them one at a time with the lanes over the candidates.  A group of at most
                // LIGHT_LDS captures is staged into the wave's LDS slice by one coalesced load, so each
                // candidate's search is one global round trip plus LDS probes.
                LSTAT_TIC();
                u32* buf = s_light[threadIdx.x / RDF_WAVE];
                u64 tg = lm;
                while (tg && alive) {
                    const int l = __ffsll((long long)tg) - 1;
                    tg &= tg - 1;
                    LSTAT_SER(1);
                    const u64 gb = __shfl(gbv[it], l, RDF_WAVE);
                    const u32 gs = __shfl(gszv[it], l, RDF_WAVE);
                    const u32* dr = (const u32*)__shfl((unsigned long long)gdr[it], l, RDF_WAVE);
                    alive = check_group(v, gb, gs, cand, alive, buf, dr);
                }
                LSTAT_TOC(3);
                continue;
            }
            const u32* gm = g != NONE32 ? v.gcap + gbv[it] : nullptr;
            const u64 gsz = gszv[it];
            LSTAT_TIC();
            if (v.sweep_f && __popcll(alive) >= LIGHT_SWEEP_MIN && !__any(gdr[it] != nullptr && g != NONE32) &&
                light_sweep(v, gm, gsz, g, cand, alive, s_light[threadIdx.x / RDF_WAVE])) {
                LSTAT_SER(1u << 16);  // stats records: swept windows in the serial counter's high half
                LSTAT_TOC(4);
                continue;
            }
            LSTAT_TOC(4);
            LSTAT_TIC();
            if (STAGE && __popcll(alive) >= LIGHT_STAGE_MIN && __all(g == NONE32 || gsz <= LIGHT_SMALL)) {
                // every light group of the window is small: each lane copies its group into its own LDS row with
                // <= 9 aligned 16-B loads, then the alive candidates are searched in LDS (instead of A x log2 n
                // divergent global loads)
                u32* row = s_light[threadIdx.x / RDF_WAVE] + lane * LIGHT_SMALL;  // odd stride: rows spread over banks
                __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");  // earlier reads of the rows precede the refill
                __builtin_amdgcn_wave_barrier();
                if (g != NONE32) {
                    const u64 gb = gbv[it], a0 = gb & ~3ull;
                    const int lead = (int)(gb - a0), n = (int)gsz;
                    const int nq = (lead + n + 3) >> 2;
                    for (int q = 0; q < nq; ++q) {
                        const uint4 w4 = *(const uint4*)(v.gcap + a0 + 4 * q);  // gcap is padded by 16 B
                        const u32 wv[4] = {w4.x, w4.y, w4.z, w4.w};
#pragma unroll
                        for (int t = 0; t < 4; ++t) {
                            const int ei = 4 * q + t - lead;
                            if (ei >= 0 && ei < n) row[ei] = wv[t];
                        }
                    }
                }
                __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
                __builtin_amdgcn_wave_barrier();
                __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
                u64 todo = alive;
                while (todo) {
                    const int l = __ffsll((long long)todo) - 1;
                    todo &= todo - 1;
                    const u32 key = __shfl(cand, l, RDF_WAVE);
                    bool found = true;
                    if (g != NONE32) {
                        u32 lo = 0, hi = (u32)gsz;
                        while (lo < hi) {
                            const u32 mid = (lo + hi) >> 1;
                            if (row[mid] < key) lo = mid + 1;
                            else hi = mid;
                        }
                        found = lo < gsz && row[lo] == key;
                    }
                    if (!__all(found)) alive &= ~(1ull << l);
                }
                continue;
            }
            // up to LIGHT_BATCH alive candidates are searched at once: their loads at one level of the
            // search are independent, so the serial chain is one search, not one per candidate
            // the batch width follows the alive count: a key slot without its own candidate would repeat another
            // slot's loads (each a divergent wave-wide load over 64 groups)
            u64 todo = alive;
            while (todo) {
                LSTAT_BAT(gsz ? 64 - __clzll(gsz) : 0);
                const int na = __popcll(todo);
                const u32* dr = g == NONE32 ? nullptr : gdr[it];
                if (na <= 2) light_batch<2>(gm, gsz, dr, g, cand, todo, alive);
                else if (na <= 4) light_batch<4>(gm, gsz, dr, g, cand, todo, alive);
                else light_batch<LIGHT_BATCH>(gm, gsz, dr, g, cand, todo, alive);
            }
            LSTAT_TOC(5);
        }
    }
#ifdef RDF_LIGHT_STATS
    if (lane == 0 && g_item_rec) {
        const unsigned long long dt = clock64() - lstat_t0;
        u32* r = g_item_rec + 24 * w;
        const u32 rec[16] = {d, (u32)(e0 - b0), (u32)(e - b), (u32)nseg, (u32)(v.goff[piv + 1] - v.goff[piv]),
                             (u32)__popcll(alive0), (u32)__popcll(alive), ls_win, ls_ser, ls_bat, ls_dep, ls_lg,
                             (u32)dt, (u32)(dt >> 32), ls_gs, ls_gmax};
        for (int k = 0; k < 16; ++k) r[k] = rec[k];
        for (int k = 0; k < 6; ++k) r[16 + k] = (u32)(ls_ph[k] >> 8);  // phase cycles / 256
        r[22] = r[23] = 0;
    }
#endif
    const u64 oct0 = choff[d] + chunk * 8 - ob;  // first octet slot of this chunk
    const u64 noct = choff[d + 1] - ob - oct0;
    const u32 nvalid = noct < 8 ? (u32)noct : 8u;
    if (nseg == 1) {
        slot_emit(oct0, nvalid, d, cand, alive, slots, counts);
        return;
    }
    // several segments: publish the killed candidates (a device-scope atomic, executed at the memory side);
    // k_light_mseg_emit emits the survivors once this kernel has finished.  No fence and no arrival
    // counter: an agent-scope release fence writes back the whole L2 of the XCD, per work item.
    if (lane == 0 && (alive0 & ~alive)) atomicOr(&dead[oct0], alive0 & ~alive);
}
// Occupancy per variant (waves per SIMD; the register budget follows): the staging variant (small groups, c2) is
// fastest unconstrained (122 VGPRs, 4 waves; 5 waves with spills measured no better: profiles/r05_light_ab_occupancy.log);
// the plain variant (large groups, c4) at RDF_LIGHT_PLAIN_WAVES (profiles/r04_light_ab_occupancy.log)
#ifdef RDF_LIGHT_STAGE_WAVES
#define RDF_LIGHT_STAGE_ATTR __attribute__((amdgpu_waves_per_eu(RDF_LIGHT_STAGE_WAVES)))
#else
#define RDF_LIGHT_STAGE_ATTR
#endif
#ifdef RDF_LIGHT_PLAIN_WAVES
#define RDF_LIGHT_PLAIN_ATTR __attribute__((amdgpu_waves_per_eu(RDF_LIGHT_PLAIN_WAVES)))
#else
#define RDF_LIGHT_PLAIN_ATTR
#endif
#define RDF_LIGHT_ARGS                                                                                                     \
    u64 nvblk, CindView v, const u32 *__restrict__ pivot, const u64 *__restrict__ itemoff,                               \
        const u32 *__restrict__ item_dep, const u64 *__restrict__ choff, u64 w0, u64 W, u64 ob, u64 *dead, u64 *slots,  \
        u32 *counts, const u32 *__restrict__ order
__global__ __launch_bounds__(RDF_BLOCK) RDF_LIGHT_STAGE_ATTR void k_light_stage(RDF_LIGHT_ARGS) {
    for (u64 vb = blockIdx.x; vb < nvblk; vb += gridDim.x)
        k_light_body<true>(vb, v, pivot, itemoff, item_dep, choff, w0, W, ob, dead, slots, counts, order);
}
__global__ __launch_bounds__(RDF_BLOCK) RDF_LIGHT_PLAIN_ATTR void k_light_plain(RDF_LIGHT_ARGS) {
    for (u64 vb = blockIdx.x; vb < nvblk; vb += gridDim.x)
        k_light_body<false>(vb, v, pivot, itemoff, item_dep, choff, w0, W, ob, dead, slots, counts, order);
}
// Work items in issue order, the items of dependents with >= thr light-group entries (many windows: c2's 6 % of
// items that hold 45 % of the cycles) first: blocks are dispatched in index order, and a 10^6-cycle item issued near
// the end set the kernel's tail.  flags -> excl (exclusive scan) -> order (a stable two-way partition).
__global__ __launch_bounds__(RDF_BLOCK) void k_light_long_flags(const u32* __restrict__ item_dep, const u64* __restrict__ doff,
                                                                u64 w0, u64 W, u64 thr, u32* flags) {
    for (u64 i = (u64)blockIdx.x * RDF_BLOCK + threadIdx.x; i < W; i += (u64)gridDim.x * RDF_BLOCK) {
        const u32 d = item_dep[w0 + i];
        flags[i] = doff[d + 1] - doff[d] >= thr ? 1u : 0u;
    }
}
__global__ __launch_bounds__(RDF_BLOCK) void k_light_order(const u32* __restrict__ flags, const u32* __restrict__ excl, u64 W,
                                                           u32* order) {
    const u32 nlong = excl[W];
    for (u64 i = (u64)blockIdx.x * RDF_BLOCK + threadIdx.x; i < W; i += (u64)gridDim.x * RDF_BLOCK)
        order[flags[i] ? excl[i] : nlong + (u32)i - excl[i]] = (u32)i;
}

// the plain variant at 6 waves per SIMD (84 VGPRs, some spills): inputs whose light groups are very large (c4: the
// searches and sweeps are latency-bound, more waves hide more of it), chosen by LIGHT_HIOCC_AVG
__global__ __launch_bounds__(RDF_BLOCK) __attribute__((amdgpu_waves_per_eu(6))) void k_light_plain_hi(RDF_LIGHT_ARGS) {
    for (u64 vb = blockIdx.x; vb < nvblk; vb += gridDim.x)
        k_light_body<false>(vb, v, pivot, itemoff, item_dep, choff, w0, W, ob, dead, slots, counts, order);
}


// chunks verified by several segments: survivors = candidates minus the union of the segments' kills
// (launched after k_light; the kernel boundary orders the kills before these reads)
__device__ inline void k_light_mseg_emit_body(u64 vblk, CindView v, const u32* __restrict__ pivot,
                                              const u64* __restrict__ mchoff, const u32* __restrict__ mch_dep, u64 m0,
                                              u64 WM, const u64* __restrict__ choff, u64 ob, const u64* __restrict__ dead,
                                              u64* slots, u32* counts) {
    const u64 wl = (u64)vblk * RDF_WAVES_PER_BLOCK + threadIdx.x / RDF_WAVE;
    if (wl >= WM) return;
    const u64 w = m0 + wl;
    const u32 d = mch_dep[w];
    const u64 chunk = w - mchoff[d];
    const u32 cand = chunk_candidate(v, d, v.info[d], pivot[d], chunk);
    const u64 alive0 = __ballot(cand != NONE32);
    const u64 oct0 = choff[d] + chunk * 8 - ob;
    const u64 noct = choff[d + 1] - ob - oct0;
    if (v.prefilter && dead[oct0] == ~0ull) return;  // pass A: a tagged chunk, emitted by its first segment item
    slot_emit(oct0, noct < 8 ? (u32)noct : 8u, d, cand, alive0 & ~dead[oct0], slots, counts);
}
__global__ __launch_bounds__(RDF_BLOCK) void k_light_mseg_emit(u64 nvblk, CindView v, const u32* __restrict__ pivot,
                                                               const u64* __restrict__ mchoff,
                                                               const u32* __restrict__ mch_dep, u64 m0, u64 WM,
                                                               const u64* __restrict__ choff, u64 ob,
                                                               const u64* __restrict__ dead, u64* slots, u32* counts) {
    for (u64 vb = blockIdx.x; vb < nvblk; vb += gridDim.x) {
        k_light_mseg_emit_body(vb, v, pivot, mchoff, mch_dep, m0, WM, choff, ob, dead, slots, counts);
    }
}


// multi-segment chunks per dependent: nitem / nseg when the dependent's groups span several segments
__global__ __launch_bounds__(RDF_BLOCK) void k_mseg_chunks(const u64* __restrict__ doff, const u32* __restrict__ nitem, u32 C,
                                                           u32* nmch) {
    for (u64 d = (u64)blockIdx.x * RDF_BLOCK + threadIdx.x; d < C; d += (u64)gridDim.x * RDF_BLOCK) {
        const u64 nseg = (doff[d + 1] - doff[d] + LIGHT_SEG - 1) / LIGHT_SEG;
        nmch[d] = nseg > 1 ? (u32)(nitem[d] / nseg) : 0u;
    }
}

// the k_light items of dependents with several candidate chunks (what the two light passes compact), as per-block
// partials [0] = such items, [1] = all items, [2] = unused
__global__ __launch_bounds__(RDF_BLOCK) void k_multi_items(const u64* __restrict__ doff, const u32* __restrict__ nitem, u32 C,
                                                           u64* part) {
    u64 acc[3] = {0, 0, 0};
    for (u64 d = (u64)blockIdx.x * RDF_BLOCK + threadIdx.x; d < C; d += (u64)gridDim.x * RDF_BLOCK) {
        const u64 nseg = (doff[d + 1] - doff[d] + LIGHT_SEG - 1) / LIGHT_SEG;
        acc[0] += nitem[d] > nseg ? nitem[d] : 0u;
        acc[1] += nitem[d];
    }
    block_partials3(acc, part);
}

// explicit CSR offsets: eoff[d] = first pair with dep >= d
// ebin[d] = first explicit pair of d with a binary ref (ref >= Cu)
__global__ __launch_bounds__(RDF_BLOCK) void k_pair_offsets(const u64* __restrict__ pairs, u64 E, u32 C, u32 Cu, u64* eoff,
                                                            u64* ebin) {
    for (u64 d = (u64)blockIdx.x * RDF_BLOCK + threadIdx.x; d <= C; d += (u64)gridDim.x * RDF_BLOCK) {
        eoff[d] = lower_bound_u64(pairs, E, d << 32);
        if (d < C) ebin[d] = lower_bound_u64(pairs, E, (d << 32) | Cu);
    }
}

// two light passes: the octets whose slots hold tagged survivors (flags = their counts, else 0), their survivors
// gathered in octet order (tag cleared), and pass B's verdicts applied back: a tagged slot stays iff pass B kept its
// pair (bpairs sorted, boff = its lower bounds per dependent)
__global__ __launch_bounds__(RDF_BLOCK) void k_tag_octets(const u64* __restrict__ slots, const u32* __restrict__ counts,
                                                          u64 W, u32* flags) {
    for (u64 o = (u64)blockIdx.x * RDF_BLOCK + threadIdx.x; o < W; o += (u64)gridDim.x * RDF_BLOCK) {
        const u32 n = counts[o];
        flags[o] = n && ((u32)slots[o * 8] & PRE_TAG) ? n : 0u;
    }
}
__global__ __launch_bounds__(RDF_BLOCK) void k_tag_gather(const u64* __restrict__ slots, const u32* __restrict__ flags,
                                                          const u64* __restrict__ pos, u64 W, u64* out) {
    for (u64 o = (u64)blockIdx.x * RDF_BLOCK + threadIdx.x; o < W; o += (u64)gridDim.x * RDF_BLOCK)
        for (u32 j = 0; j < flags[o]; ++j) out[pos[o] + j] = slots[o * 8 + j] & ~(u64)PRE_TAG;
}
__global__ __launch_bounds__(RDF_BLOCK) void k_tag_fix(u64* slots, u32* counts, const u32* __restrict__ flags, u64 W,
                                                       const u64* __restrict__ bpairs, const u64* __restrict__ boff) {
    for (u64 o = (u64)blockIdx.x * RDF_BLOCK + threadIdx.x; o < W; o += (u64)gridDim.x * RDF_BLOCK) {
        const u32 n = flags[o];
        if (!n) continue;
        u32 k = 0;
        for (u32 j = 0; j < n; ++j) {
            const u64 x = slots[o * 8 + j] & ~(u64)PRE_TAG;
            const u64 d = x >> 32;
            if (bsearch_u64(bpairs + boff[d], boff[d + 1] - boff[d], x)) slots[o * 8 + k++] = x;
        }
        counts[o] = k;
    }
}

// minimality on explicit pairs -> output (R1/R4; R2/R3 by k_rules_mark afterwards)
__global__ __launch_bounds__(RDF_BLOCK) void k_rules_explicit(CindView v, const u64* __restrict__ pairs, u64 E, u32 rank,
                                                              u32 nranks, u32* keep) {
    for (u64 i = (u64)blockIdx.x * RDF_BLOCK + threadIdx.x; i < E; i += (u64)gridDim.x * RDF_BLOCK) {
        const u64 pr = pairs[i];
        const u32 d = (u32)(pr >> 32);
        keep[i] = (dep_owner(d, nranks) == rank && rule_keep(v, d, (u32)pr)) ? 1u : 0u;
    }
}

// R2/R3 (--clean-implied) on explicit dependents: every binary raw pair (a, X) clears the components of X
// in a's unary refs [eoff[a], ebin[a]).  Plain stores of 0 (idempotent; k_rules_explicit has finished).
// (pairs [e0, e0 + E) of v.epairs; keep is relative to e0, and every pair of a dependent lies in the range)
__global__ __launch_bounds__(RDF_BLOCK) void k_rules_mark(CindView v, const u64* __restrict__ pairs, u64 e0, u64 E,
                                                          u32 rank, u32 nranks, u32* keep) {
    for (u64 i = (u64)blockIdx.x * RDF_BLOCK + threadIdx.x; i < E; i += (u64)gridDim.x * RDF_BLOCK) {
        const u64 pr = pairs[e0 + i];
        const u32 a = (u32)(pr >> 32), x = (u32)pr;
        if (x < v.Cu || dep_owner(a, nranks) != rank) continue;
        const u64 b = v.eoff[a], n = v.ebin[a] - b;
        const u32* bc = v.bcomp + 2ull * (x - v.Cu);
#pragma unroll
        for (int k = 0; k < 2; ++k) {
            const u64 key = ((u64)a << 32) | bc[k];
            const u64 j = lower_bound_u64(pairs + b, n, key);
            if (j < n && pairs[b + j] == key) keep[b + j - e0] = 0u;
        }
    }
}

__global__ __launch_bounds__(RDF_BLOCK) void k_popc_counts(const u64* __restrict__ bits, u64 W, u32* counts) {
    for (u64 w = (u64)blockIdx.x * RDF_BLOCK + threadIdx.x; w < W; w += (u64)gridDim.x * RDF_BLOCK)
        counts[w] = (u32)__popcll(bits[w]);
}

// heavy-only binary dependents: refs = pivot members passing the mask test.  One wave per work item (chunk of
// 64 pivot members); bits[w] holds the surviving lanes: k_heavy_eval (candidate filter + R1/R4), then
// k_heavy_mark (R2: the components of every raw binary ref are cleared, they sit in the same pivot group),
// then k_heavy_write streams the survivors at the scanned offsets (popcounts of bits).
// Work items [w0, w0 + W) (a paged run takes a dependent range at a time); owner / bits / woff are indexed
// relative to w0.
__device__ inline void k_heavy_eval_body(u64 vblk, CindView v, const u32* __restrict__ pivot,
                                         const u64* __restrict__ choff, const u32* __restrict__ owner, u64 w0, u64 W,
                                         u64* bits) {
    const u64 wl = (u64)vblk * RDF_WAVES_PER_BLOCK + threadIdx.x / RDF_WAVE;
    if (wl >= W) return;
    const u64 w = w0 + wl;
    const u32 d = owner[wl];
    const CapInfo id = v.info[d];
    const u32 piv = pivot[d];
    const u64 chunk = w - choff[d];
    const u32 cand = chunk_candidate(v, d, id, piv, chunk);
    const bool keep = cand != NONE32 && rule_keep(v, d, cand);
    const u64 kept = __ballot(keep);
    if (lane_id() == 0) bits[wl] = kept;
}
__global__ __launch_bounds__(RDF_BLOCK) void k_heavy_eval(u64 nvblk, CindView v, const u32* __restrict__ pivot,
                                                          const u64* __restrict__ choff, const u32* __restrict__ owner,
                                                          u64 w0, u64 W, u64* bits) {
    for (u64 vb = blockIdx.x; vb < nvblk; vb += gridDim.x) {
        k_heavy_eval_body(vb, v, pivot, choff, owner, w0, W, bits);
    }
}


// clear bit p of a per-chunk survivor bitmap (all lanes call it).  Many binary refs share a component
// (s[p=P,o=*] -> s[p=P]), so equal targets of a wave merge first and a target already cleared by another
// wave is skipped by a plain load: only the first clear of a bit goes to the memory-side atomic.
__device__ inline void mark_clear(u64* bits, u64 p, bool active) {
    if (!wave_merge<u64, 4>(active ? p : ~0ull, active)) return;
    u64* word = bits + p / RDF_WAVE;
    const u64 m = 1ull << (p % RDF_WAVE);
    if (!(*word & m)) return;
    atomicAnd((unsigned long long*)word, ~m);
}

__device__ inline void k_heavy_mark_body(u64 vblk, CindView v, const u32* __restrict__ pivot,
                                         const u64* __restrict__ choff, const u32* __restrict__ owner, u64 w0, u64 W,
                                         u64* bits) {
    const u64 wl = (u64)vblk * RDF_WAVES_PER_BLOCK + threadIdx.x / RDF_WAVE;
    if (wl >= W) return;
    const u64 w = w0 + wl;
    const u32 d = owner[wl];
    const CapInfo id = v.info[d];
    const u32 piv = pivot[d];
    const u32 x = chunk_candidate(v, d, id, piv, w - choff[d]);
    const bool bin = x != NONE32 && x >= v.Cu;
    if (!__ballot(bin)) return;
    const u64 base = (choff[d] - w0) * RDF_WAVE;  // bit index of pivot position 0 (all of d's chunks are in range)
#pragma unroll
    for (int k = 0; k < 2; ++k) {
        const u32 t = bin ? v.bcomp[2ull * (x - v.Cu) + k] : NONE32;
        const u32 tprev = __shfl_up(t, 1, RDF_WAVE);
        const bool head = bin && (lane_id() == 0 || tprev != t);  // consecutive refs share component 0
        const u64 p = head ? group_pos(v, piv, t) : ~0ull;
        mark_clear(bits, base + p, p != ~0ull);
    }
}
__global__ __launch_bounds__(RDF_BLOCK) void k_heavy_mark(u64 nvblk, CindView v, const u32* __restrict__ pivot,
                                                          const u64* __restrict__ choff, const u32* __restrict__ owner,
                                                          u64 w0, u64 W, u64* bits) {
    for (u64 vb = blockIdx.x; vb < nvblk; vb += gridDim.x) {
        k_heavy_mark_body(vb, v, pivot, choff, owner, w0, W, bits);
    }
}


// survivors of a heavy work item -> output run of its dependent; src[sbase[d] + i] is candidate i of d
// (classed binary dependents: their class list; otherwise sbase = null and the pivot group is the source)
__device__ inline void k_heavy_write_body(u64 vblk, CindView v, const u32* __restrict__ pivot,
                                          const u64* __restrict__ choff, const u32* __restrict__ owner, u64 w0, u64 W,
                                          const u64* __restrict__ bits, const u32* __restrict__ src,
                                          const u64* __restrict__ sbase, const u64* __restrict__ woff, u64 out_base,
                                          u32* out) {
    const u64 wl = (u64)vblk * RDF_WAVES_PER_BLOCK + threadIdx.x / RDF_WAVE;
    if (wl >= W) return;
    const u64 w = w0 + wl;
    const u64 kept = bits[wl];
    const int lane = lane_id();
    if (!((kept >> lane) & 1ull)) return;
    const u32 d = owner[wl];
    const u64 base = sbase ? sbase[d] : v.goff[pivot[d]];
    out[out_base + woff[wl] + __popcll(kept & lanemask_lt())] = src[base + (w - choff[d]) * RDF_WAVE + lane];
}
__global__ __launch_bounds__(RDF_BLOCK) void k_heavy_write(u64 nvblk, CindView v, const u32* __restrict__ pivot,
                                                           const u64* __restrict__ choff, const u32* __restrict__ owner,
                                                           u64 w0, u64 W, const u64* __restrict__ bits,
                                                           const u32* __restrict__ src, const u64* __restrict__ sbase,
                                                           const u64* __restrict__ woff, u64 out_base, u32* out) {
    for (u64 vb = blockIdx.x; vb < nvblk; vb += gridDim.x) {
        k_heavy_write_body(vb, v, pivot, choff, owner, w0, W, bits, src, sbase, woff, out_base, out);
    }
}



// ================================================================================================
// K6c: unary heavy-only dependents by bitmask class.  A dependent A whose groups are all heavy has
// support(A) = popcount(hmask(A)) and refs(A) = {B : hmask(B) covers hmask(A)} \ {A}; every dependent with
// the same mask shares the pivot group and therefore the ref list L(m).  Under --clean-implied, R3 removes
// from a unary A's 1/1 refs every R that is a component of a binary ref X of A -- for heavy-only A that is
// "R has a parent binary whose mask covers m", again a class property.  So L'(m) is built once per class
// and each dependent's output is L'(m) minus itself: a streaming copy bound by the HBM write rate.

// masks of the heavy-only dependents [0, cmax): cmax = Cu (unary only) or C (binary ones classed too)
// slot of mask m in the class table (bounded probe: a mask that is not there gives ~0 instead of a spinning wave)
__device__ inline u64 class_slot(const u64* __restrict__ tkeys, u64 tmask, u64 m) {
    u64 h = mix64(m) & tmask;
    for (u64 probe = 0; probe <= tmask; ++probe, h = (h + 1) & tmask) {
        const u64 k = tkeys[h];
        if (k == m) return h;
        if (k == 0) return ~0ull;
    }
    return ~0ull;
}

__global__ __launch_bounds__(RDF_BLOCK) void k_class_insert(CindView v, u32 cmax, u64* tkeys, u64 tmask, u64* nmembers) {
    u32 cnt = 0;
    const u64 n_round = ((u64)cmax + RDF_WAVE - 1) / RDF_WAVE * RDF_WAVE;
    for (u64 d = (u64)blockIdx.x * RDF_BLOCK + threadIdx.x; d < n_round; d += (u64)gridDim.x * RDF_BLOCK) {
        const bool member = d < cmax && (v.info[d].meta & META_HEAVY_ONLY);
        const u64 m = member ? v.info[d].hmask : 0ull;  // never 0 for a heavy-only dependent
        cnt += member && d < v.Cu;
        // few classes, many members: one lane per distinct mask of the wave inserts (one CAS per address)
        if (wave_merge<u64, 4>(m, member)) {
            u64 h = mix64(m) & tmask;
            for (;;) {
                u64 k = tkeys[h];
                if (k == m) break;
                if (k == 0) {
                    u64 prev = atomicCAS(&tkeys[h], 0ull, m);
                    if (prev == 0 || prev == m) break;
                }
                h = (h + 1) & tmask;
            }
        }
    }
    block_counter_add(nmembers, cnt);
}

__global__ __launch_bounds__(RDF_BLOCK) void k_nonzero_flags(const u64* __restrict__ a, u64 n, u32* flags) {
    for (u64 i = (u64)blockIdx.x * RDF_BLOCK + threadIdx.x; i < n; i += (u64)gridDim.x * RDF_BLOCK) flags[i] = a[i] != 0;
}

// (class << 32 | dep) keys for all unary heavy-only dependents
__global__ __launch_bounds__(RDF_BLOCK) void k_class_keys(CindView v, const u64* __restrict__ tkeys, const u32* __restrict__ cid,
                                                          u64 tmask, u32 rank, u32 nranks, u64* out, u64* counter) {
    const u64 n_round = ((u64)v.Cu + RDF_WAVE - 1) / RDF_WAVE * RDF_WAVE;
    for (u64 d = (u64)blockIdx.x * RDF_BLOCK + threadIdx.x; d < n_round; d += (u64)gridDim.x * RDF_BLOCK) {
        u32 want = 0;
        u64 key = 0;
        if (d < v.Cu && (v.info[d].meta & META_HEAVY_ONLY) && dep_owner((u32)d, nranks) == rank) {
            const u64 h = class_slot(tkeys, tmask, v.info[d].hmask);
            if (h != ~0ull) {
                key = ((u64)cid[h] << 32) | d;
                want = 1;
            }
        }
        u64 pos = wave_append(counter, want);
        if (want) out[pos] = key;
    }
}

// binary heavy-only dependents join the mask classes (single GPU, S2L semantics): class id per dependent and
// a representative member of every class (members of a class share the pivot group)
__global__ __launch_bounds__(RDF_BLOCK) void k_class_of(CindView v, const u64* __restrict__ tkeys, const u32* __restrict__ cid,
                                                        u64 tmask, u32* dcls, u32* crep) {
    for (u64 d = (u64)blockIdx.x * RDF_BLOCK + threadIdx.x; d < v.C; d += (u64)gridDim.x * RDF_BLOCK) {
        u32 m = NONE32;
        if (v.info[d].meta & META_HEAVY_ONLY) {
            const u64 h = class_slot(tkeys, tmask, v.info[d].hmask);
            if (h != ~0ull) {
                m = cid[h];
                // any member represents its class (same groups, same pivot): a plain store once the slot is seen
                // taken is skipped (thousands of members per class would otherwise serialise on one address)
                if (crep[m] == NONE32) crep[m] = (u32)d;
            }
        }
        if (d >= v.Cu) dcls[d - v.Cu] = m;
    }
}

// work items of a classed binary dependent: chunks of 64 of its class list L'(m); sbase = list start
__global__ __launch_bounds__(RDF_BLOCK) void k_class_bin_chunks(CindView v, const u32* __restrict__ dcls,
                                                                const u64* __restrict__ cchoff, const u64* __restrict__ lwoff,
                                                                u32* nchunk, u64* sbase) {
    for (u64 d = (u64)blockIdx.x * RDF_BLOCK + threadIdx.x; d < v.C; d += (u64)gridDim.x * RDF_BLOCK) {
        u32 n = 0;
        if (d >= v.Cu && dcls[d - v.Cu] != NONE32) {
            const u32 m = dcls[d - v.Cu];
            const u64 b = lwoff[cchoff[m]], e = lwoff[cchoff[m + 1]];
            sbase[d] = b;
            n = (u32)((e - b + RDF_WAVE - 1) / RDF_WAVE);
        }
        nchunk[d] = n;
    }
}

// classed binary dependent D: refs = L'(m) minus D, its components (trivial) and R1/R4 (comp(D) < R).
// R2 is already in L'(m): D's binary raw refs are the binary members of L(m), the class marks cleared their
// components.  Survivor bits per chunk, as k_heavy_eval.
__device__ inline void k_class_bin_eval_body(u64 vblk, CindView v, const u64* __restrict__ choff,
                                             const u32* __restrict__ owner, u64 w0, u64 W, const u64* __restrict__ sbase,
                                             const u32* __restrict__ dcls, const u64* __restrict__ cchoff,
                                             const u64* __restrict__ lwoff, const u32* __restrict__ lists, u64* bits) {
    const u64 wl = (u64)vblk * RDF_WAVES_PER_BLOCK + threadIdx.x / RDF_WAVE;
    if (wl >= W) return;
    const u64 w = w0 + wl;
    const u32 d = owner[wl];
    const u32 m = dcls[d - v.Cu];
    const u64 i = sbase[d] + (w - choff[d]) * RDF_WAVE + lane_id();
    bool keep = i < lwoff[cchoff[m + 1]];
    const u32 r = keep ? lists[i] : 0u;
    keep = keep && r != d && !is_trivial(v, d, r) && rule_keep(v, d, r);
    const u64 kept = __ballot(keep);
    if (lane_id() == 0) bits[wl] = kept;
}
__global__ __launch_bounds__(RDF_BLOCK) void k_class_bin_eval(u64 nvblk, CindView v, const u64* __restrict__ choff,
                                                              const u32* __restrict__ owner, u64 w0, u64 W,
                                                              const u64* __restrict__ sbase,
                                                              const u32* __restrict__ dcls,
                                                              const u64* __restrict__ cchoff,
                                                              const u64* __restrict__ lwoff,
                                                              const u32* __restrict__ lists, u64* bits) {
    for (u64 vb = blockIdx.x; vb < nvblk; vb += gridDim.x) {
        k_class_bin_eval_body(vb, v, choff, owner, w0, W, sbase, dcls, cchoff, lwoff, lists, bits);
    }
}


// per class: member offsets, mask, pivot, pivot-chunk count
__global__ __launch_bounds__(RDF_BLOCK) void k_class_info(CindView v, const u64* __restrict__ keys, u64 nkeys, u32 ncls,
                                                          const u32* __restrict__ pivot, const u32* __restrict__ crep,
                                                          u64* coff, u64* cmask, u32* cpiv, u32* cnch) {
    for (u64 m = (u64)blockIdx.x * RDF_BLOCK + threadIdx.x; m <= ncls; m += (u64)gridDim.x * RDF_BLOCK) {
        u64 lo = lower_bound_u64(keys, nkeys, m << 32);
        coff[m] = lo;
        if (m < ncls) {
            const u32 rep = crep ? crep[m] : (u32)keys[lo];
            const u32 g = pivot[rep];
            cmask[m] = v.info[rep].hmask;
            cpiv[m] = g;
            cnch[m] = (u32)((v.goff[g + 1] - v.goff[g] + RDF_WAVE - 1) / RDF_WAVE);
        }
    }
}

// R3 for a unary ref with few parents is a scan of parents(r) in the eval pass (cheap, no atomics); the
// components with long parent lists (s[p=P] under every s[p=P,o=*]) are cleared by the mark pass instead
static constexpr u64 PARENT_SCAN_MAX = 32;
__device__ inline bool short_parents(const CindView& v, u32 r) {
    return !(v.info[r].meta & META_PARENTS) || v.poff[r + 1] - v.poff[r] <= PARENT_SCAN_MAX;
}

// L'(m): the class pivot group filtered by the mask test (bits per chunk of 64 members), then, under
// --clean-implied, R3: the components of the binary members of L(m) are dropped (a binary X with
// hmask(X) >= m is a raw ref of every member; its components sit in the same pivot group) -- by a scan of
// parents(r) in the eval pass when that list is short, by k_class_mark otherwise.
__device__ inline void k_class_eval_body(u64 vblk, CindView v, const u64* __restrict__ cchoff,
                                         const u32* __restrict__ owner, u64 W, const u64* __restrict__ cmask,
                                         const u32* __restrict__ cpiv, u64* bits) {
    const u64 w = (u64)vblk * RDF_WAVES_PER_BLOCK + threadIdx.x / RDF_WAVE;
    if (w >= W) return;
    const u32 m = owner[w];
    const u32 g = cpiv[m];
    const u64 mask = cmask[m];
    const u64 idx = v.goff[g] + (w - cchoff[m]) * RDF_WAVE + lane_id();
    const u32 r = idx < v.goff[g + 1] ? v.gcap[idx] : 0u;
    bool keep = idx < v.goff[g + 1] && (v.info[r].hmask & mask) == mask;
    if (keep && v.mode == RULES_CLEAN && r < v.Cu && short_parents(v, r))  // R3 here; long lists: k_class_mark
        for (u64 j = v.poff[r]; j < v.poff[r + 1] && keep; ++j) keep = (v.info[v.plist[j]].hmask & mask) != mask;
    const u64 kept = __ballot(keep);
    if (lane_id() == 0) bits[w] = kept;
}
__global__ __launch_bounds__(RDF_BLOCK) void k_class_eval(u64 nvblk, CindView v, const u64* __restrict__ cchoff,
                                                          const u32* __restrict__ owner, u64 W,
                                                          const u64* __restrict__ cmask, const u32* __restrict__ cpiv,
                                                          u64* bits) {
    for (u64 vb = blockIdx.x; vb < nvblk; vb += gridDim.x) {
        k_class_eval_body(vb, v, cchoff, owner, W, cmask, cpiv, bits);
    }
}


__device__ inline void k_class_mark_body(u64 vblk, CindView v, const u64* __restrict__ cchoff,
                                         const u32* __restrict__ owner, u64 W, const u64* __restrict__ cmask,
                                         const u32* __restrict__ cpiv, u64* bits) {
    const u64 w = (u64)vblk * RDF_WAVES_PER_BLOCK + threadIdx.x / RDF_WAVE;
    if (w >= W) return;
    const u32 m = owner[w];
    const u32 g = cpiv[m];
    const u64 mask = cmask[m];
    const u64 idx = v.goff[g] + (w - cchoff[m]) * RDF_WAVE + lane_id();
    const u32 x = idx < v.goff[g + 1] ? v.gcap[idx] : 0u;
    const bool bin = x >= v.Cu && (v.info[x].hmask & mask) == mask;
    if (!__ballot(bin)) return;
    const u64 base = cchoff[m] * RDF_WAVE;
#pragma unroll
    for (int k = 0; k < 2; ++k) {
        const u32 t = bin ? v.bcomp[2ull * (x - v.Cu) + k] : NONE32;
        const u32 tprev = __shfl_up(t, 1, RDF_WAVE);
        const bool head = bin && (lane_id() == 0 || tprev != t) && !short_parents(v, t);  // consecutive refs share comp 0
        const u64 p = head ? group_pos(v, g, t) : ~0ull;
        mark_clear(bits, base + p, p != ~0ull);
    }
}
__global__ __launch_bounds__(RDF_BLOCK) void k_class_mark(u64 nvblk, CindView v, const u64* __restrict__ cchoff,
                                                          const u32* __restrict__ owner, u64 W,
                                                          const u64* __restrict__ cmask, const u32* __restrict__ cpiv,
                                                          u64* bits) {
    for (u64 vb = blockIdx.x; vb < nvblk; vb += gridDim.x) {
        k_class_mark_body(vb, v, cchoff, owner, W, cmask, cpiv, bits);
    }
}


__device__ inline void k_class_write_body(u64 vblk, CindView v, const u64* __restrict__ cchoff,
                                          const u32* __restrict__ owner, u64 W, const u32* __restrict__ cpiv,
                                          const u64* __restrict__ bits, const u64* __restrict__ woff, u32* lists,
                                          u64* cpairs) {
    const u64 w = (u64)vblk * RDF_WAVES_PER_BLOCK + threadIdx.x / RDF_WAVE;
    if (w >= W) return;
    const u64 kept = bits[w];
    const int lane = lane_id();
    if (!((kept >> lane) & 1ull)) return;
    const u32 m = owner[w];
    const u32 r = v.gcap[v.goff[cpiv[m]] + (w - cchoff[m]) * RDF_WAVE + lane];
    const u64 o = woff[w] + __popcll(kept & lanemask_lt());
    if (cpairs) cpairs[o] = ((u64)m << 32) | r;  // sharded mode: (class, ref) pairs for the all-gather
    else lists[o] = r;
}
__global__ __launch_bounds__(RDF_BLOCK) void k_class_write(u64 nvblk, CindView v, const u64* __restrict__ cchoff,
                                                           const u32* __restrict__ owner, u64 W,
                                                           const u32* __restrict__ cpiv, const u64* __restrict__ bits,
                                                           const u64* __restrict__ woff, u32* lists, u64* cpairs) {
    for (u64 vb = blockIdx.x; vb < nvblk; vb += gridDim.x) {
        k_class_write_body(vb, v, cchoff, owner, W, cpiv, bits, woff, lists, cpairs);
    }
}


// per member dependent: position of itself in L'(m) (or NONE) and its output count
__global__ __launch_bounds__(RDF_BLOCK) void k_class_members(const u64* __restrict__ keys, u64 nkeys,
                                                             const u64* __restrict__ cchoff, const u64* __restrict__ lwoff,
                                                             const u32* __restrict__ lists, u32* selfpos, u32* cnt) {
    for (u64 i = (u64)blockIdx.x * RDF_BLOCK + threadIdx.x; i < nkeys; i += (u64)gridDim.x * RDF_BLOCK) {
        const u32 m = (u32)(keys[i] >> 32), d = (u32)keys[i];
        const u64 b = lwoff[cchoff[m]], e = lwoff[cchoff[m + 1]];
        u64 lo = b, hi = e;
        while (lo < hi) {
            u64 mid = (lo + hi) >> 1;
            if (lists[mid] < d) lo = mid + 1;
            else hi = mid;
        }
        const bool self = lo < e && lists[lo] == d;
        selfpos[i] = self ? (u32)(lo - b) : NONE32;
        cnt[i] = (u32)(e - b) - (self ? 1u : 0u);
    }
}

// per class: number of emission tiles = ceil(members / CLS_DT) * ceil(|L'| / CLS_LS)
typedef u32 u32x4 __attribute__((ext_vector_type(4)));
#ifndef RDF_CLS_DT
#define RDF_CLS_DT 8
#endif
#ifndef RDF_CLS_LS
#define RDF_CLS_LS 16384
#endif
static constexpr u32 CLS_DT = RDF_CLS_DT;            // dependents per tile
static constexpr u32 CLS_LS = RDF_CLS_LS;            // list elements per tile (staged in LDS; power of two)

__global__ __launch_bounds__(RDF_BLOCK) void k_class_tiles(const u64* __restrict__ coff, const u64* __restrict__ cchoff,
                                                           const u64* __restrict__ lwoff, u32 ncls, u32* ntiles) {
    for (u64 m = (u64)blockIdx.x * RDF_BLOCK + threadIdx.x; m < ncls; m += (u64)gridDim.x * RDF_BLOCK) {
        const u64 k = coff[m + 1] - coff[m];
        const u64 len = lwoff[cchoff[m + 1]] - lwoff[cchoff[m]];
        ntiles[m] = (u32)(((k + CLS_DT - 1) / CLS_DT) * ((len + CLS_LS - 1) / CLS_LS));
    }
}

// streaming emission into the dependent-run output (refs only; the run table names the dependent): each
// block stages one list segment in LDS once and writes it for CLS_DT dependents.  HBM writes run at full
// rate only for whole 128-B lines, so (1) a dependent's run is cut into segments at 128-B boundaries of the
// OUTPUT (not of the list), so that no line is shared by two blocks, and (2) lanes own 16-B quads counted
// from the 256-B boundary below the segment start, so every wave-wide store covers whole lines.  Segment s
// of a run needs list entries [s*CLS_LS - 31, (s+1)*CLS_LS + 1), hence the staged halo.
__device__ inline void k_class_emit_body(u64 vblk, const u64* __restrict__ coff, const u64* __restrict__ cchoff,
                                         const u64* __restrict__ lwoff, const u32* __restrict__ lists,
                                         const u64* __restrict__ toff, u32 ncls, const u32* __restrict__ selfpos,
                                         const u64* __restrict__ obase, u64 out_base, u32* out) {
    __shared__ u32 sl[CLS_LS + 64];
    __shared__ u32 s_sp[CLS_DT];
    __shared__ u64 s_base[CLS_DT];
    __shared__ u32 s_m;
    if (threadIdx.x == 0) s_m = find_dep(toff, ncls, vblk);
    __syncthreads();
    const u32 m = s_m;
    const u64 lb = lwoff[cchoff[m]], len = lwoff[cchoff[m + 1]] - lb;
    const u64 nseg = (len + CLS_LS - 1) / CLS_LS;
    const u64 t = vblk - toff[m];
    const u64 dt = t / nseg, seg = t % nseg;
    const u64 k0 = coff[m] + dt * CLS_DT, k1 = k0 + CLS_DT < coff[m + 1] ? k0 + CLS_DT : coff[m + 1];
    const u64 p0 = seg * CLS_LS;
    const u64 sb = p0 >= 32 ? p0 - 32 : 0;                                   // staged list range [sb, se)
    const u64 se = p0 + CLS_LS + 1 < len ? p0 + CLS_LS + 1 : len;
    for (u64 i = threadIdx.x; i < se - sb; i += RDF_BLOCK) sl[i] = lists[lb + sb + i];
    if (threadIdx.x < k1 - k0) {  // the tile's dependents, loaded once instead of one dependent load chain each
        const u64 i = k0 + threadIdx.x;
        s_sp[threadIdx.x] = selfpos[i];
        s_base[threadIdx.x] = obase[i];
    }
    __syncthreads();
    for (u64 i = 0; i < k1 - k0; ++i) {
        const u32 sp = s_sp[i];
        const u64 n_run = len - (sp != NONE32 ? 1 : 0);
        const u64 r0 = out_base + s_base[i];
        // run element where segment s starts: the first 128-B boundary of the output at or below r0 + s*CLS_LS
        auto bound = [&](u64 s) -> u64 {
            if (s == 0) return 0;
            if (s >= nseg) return n_run;
            const u64 x = (r0 + s * CLS_LS) & ~31ull;
            return x <= r0 ? 0 : (x - r0 < n_run ? x - r0 : n_run);
        };
        const u64 kb = bound(seg), ke = bound(seg + 1);
        if (kb >= ke) continue;
        const u64 ob = r0 + kb;
        const int n = (int)(ke - kb);
        const int lead = (int)(ob & 63);
        const int nq = (lead + n + 3) >> 2;
        u32* q_out = out + (ob - lead);                                       // 256-B aligned quad base
        const int skip = sp != NONE32 ? (int)((u64)sp - kb) : 0x7fffffff;    // run element >= skip reads one further
        const int base = (int)(kb - sb);                                     // run element kb at sl[base]
        for (int t = threadIdx.x; t < nq; t += RDF_BLOCK) {
            const int q0 = 4 * t - lead;                                      // segment element of the quad's first slot
            u32 val[4];
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const int q = q0 + j;
                const int li = base + q + (q >= skip ? 1 : 0);
                val[j] = sl[li < 0 ? 0 : (li > (int)(CLS_LS + 63) ? (int)(CLS_LS + 63) : li)];
            }
            if (q0 >= 0 && q0 + 3 < n) {  // one 16-B store (the builtin keeps it from being split)
                const u32x4 w = {val[0], val[1], val[2], val[3]};
                __builtin_nontemporal_store(w, (u32x4*)(q_out + 4 * t));
            } else {
#pragma unroll
                for (int j = 0; j < 4; ++j)
                    if (q0 + j >= 0 && q0 + j < n) q_out[4 * t + j] = val[j];
            }
        }
    }
}
__global__ __launch_bounds__(RDF_BLOCK) void k_class_emit(u64 nvblk, const u64* __restrict__ coff,
                                                          const u64* __restrict__ cchoff, const u64* __restrict__ lwoff,
                                                          const u32* __restrict__ lists, const u64* __restrict__ toff,
                                                          u32 ncls, const u32* __restrict__ selfpos,
                                                          const u64* __restrict__ obase, u64 out_base, u32* out) {
    for (u64 vb = blockIdx.x; vb < nvblk; vb += gridDim.x) {
        k_class_emit_body(vb, coff, cchoff, lwoff, lists, toff, ncls, selfpos, obase, out_base, out);
        __syncthreads();  // shared staging is reused by the next virtual block
    }
}


// first ref of each shared (class) list: class m's list is lists[lwoff[cchoff[m]], lwoff[cchoff[m + 1]])
__global__ __launch_bounds__(RDF_BLOCK) void k_list_offsets(const u64* __restrict__ cchoff, const u64* __restrict__ lwoff,
                                                            u32 ncls, u64* loff) {
    for (u64 m = (u64)blockIdx.x * RDF_BLOCK + threadIdx.x; m <= ncls; m += (u64)gridDim.x * RDF_BLOCK)
        loff[m] = lwoff[cchoff[m]];
}

// output run table (dependent runs in output order): runs [0, C) are the explicit pairs of dependent d
// (start pos[eoff[d]]), [C, C+WH) the heavy-only binary chunks, [C+WH, C+WH+nmem) the class members
__global__ __launch_bounds__(RDF_BLOCK) void k_output_runs(u32 C, const u64* __restrict__ eoff, const u64* __restrict__ epos,
                                                           u64 WH, const u64* __restrict__ choffh, const u64* __restrict__ hoff,
                                                           u64 K, u64 nmem, const u64* __restrict__ ckeys,
                                                           const u64* __restrict__ cobase, u64 H, u64 n_out, u64* runoff,
                                                           u32* rundep, u64 i0, u64 i1) {
    // runs [i0, i1] of the table (the explicit runs [0, C) are final once the rules have run: the early hand-over
    // writes and copies them before the class stage, the rest at the end)
    const u64 R = (u64)C + WH + nmem;
    for (u64 i = i0 + (u64)blockIdx.x * RDF_BLOCK + threadIdx.x; i <= i1 && i <= R; i += (u64)gridDim.x * RDF_BLOCK) {
        if (i == R) {
            runoff[i] = n_out;
        } else if (i < C) {
            runoff[i] = epos[eoff[i]];
            rundep[i] = (u32)i;
        } else if (i < C + WH) {
            const u64 w = i - C;
            runoff[i] = K + hoff[w];
            rundep[i] = find_dep(choffh, C, w);
        } else {
            const u64 j = i - C - WH;
            runoff[i] = K + H + cobase[j];
            rundep[i] = (u32)ckeys[j];
        }
    }
}

// heavy-bits form (rdf_copy_result_heavy): the class-list position of the first candidate of heavy work items
// [h0, h0 + W) (dependent deps[w] from the run table; its chunks are consecutive from choffh[dep])
__global__ __launch_bounds__(RDF_BLOCK) void k_heavy_pos(u32 C, u64 h0, u64 W, const u64* __restrict__ choffh,
                                                         const u32* __restrict__ deps, const u64* __restrict__ sbase,
                                                         u64* pos) {
    for (u64 w = (u64)blockIdx.x * RDF_BLOCK + threadIdx.x; w < W; w += (u64)gridDim.x * RDF_BLOCK) {
        const u32 d = deps[w];
        pos[w] = sbase[d] + (h0 + w - choffh[d]) * RDF_WAVE;
    }
}

// run table of one page of a paged run: explicit runs of dependents [d0, d1) (their pairs start at e0 of the explicit
// array; epos = the page's compaction offsets), heavy work items [h0, h0 + WH), then the class members (page 0)
__global__ __launch_bounds__(RDF_BLOCK) void k_output_runs_range(u32 C, u32 d0, u32 d1, const u64* __restrict__ eoff, u64 e0,
                                                                 const u64* __restrict__ epos, u64 h0, u64 WH,
                                                                 const u64* __restrict__ choffh, const u64* __restrict__ hoff,
                                                                 u64 K, u64 nmem, const u64* __restrict__ ckeys,
                                                                 const u64* __restrict__ cobase, u64 H, u64 n_out,
                                                                 u64* runoff, u32* rundep) {
    const u64 nd = d1 - d0, R = nd + WH + nmem;
    for (u64 i = (u64)blockIdx.x * RDF_BLOCK + threadIdx.x; i <= R; i += (u64)gridDim.x * RDF_BLOCK) {
        if (i == R) {
            runoff[i] = n_out;
        } else if (i < nd) {
            const u32 d = (u32)(d0 + i);
            runoff[i] = epos[eoff[d] - e0];
            rundep[i] = d;
        } else if (i < nd + WH) {
            const u64 w = i - nd;
            runoff[i] = K + hoff[w];
            rundep[i] = find_dep(choffh, C, h0 + w);
        } else {
            const u64 j = i - nd - WH;
            runoff[i] = K + H + cobase[j];
            rundep[i] = (u32)ckeys[j];
        }
    }
}

__global__ __launch_bounds__(RDF_BLOCK) void k_compact_refs(const u64* __restrict__ a, u64 n, const u32* __restrict__ flags,
                                                            const u64* __restrict__ pos, u32* out) {
    for (u64 i = (u64)blockIdx.x * RDF_BLOCK + threadIdx.x; i < n; i += (u64)gridDim.x * RDF_BLOCK)
        if (flags[i]) out[pos[i]] = (u32)a[i];
}

// run containing output element i: largest r with runoff[r] <= i, searched in [lo, hi]
__device__ inline u64 run_of(const u64* __restrict__ runoff, u64 lo, u64 hi, u64 i) {
    while (lo < hi) {
        const u64 mid = (lo + hi + 1) >> 1;
        if (runoff[mid] <= i) lo = mid;
        else hi = mid - 1;
    }
    return lo;
}

// checksum term of one result row (external capture ids + the dependent's support); the C oracle's streamed
// mode (oracle/c/rdfind_oracle.c row_hash) sums the same terms
__device__ inline u64 row_hash(u32 dep, u32 ref, u32 support) {
    return mix64((((u64)dep << 32) | ref) + (u64)support * 0x9E3779B97F4A7C15ull);
}

// order-independent checksum of the result set (external capture ids, so it is comparable across runs and
// layouts).  Each block looks up the runs of its first and last element once; lanes search inside that range.
__global__ __launch_bounds__(RDF_BLOCK) void k_checksum(const u32* __restrict__ refs, u64 n, const u64* __restrict__ runoff,
                                                        const u32* __restrict__ rundep, u64 R, const u32* __restrict__ fcap,
                                                        const u32* __restrict__ csup, u64* sum) {
    __shared__ u64 s_lo, s_hi;
    u64 acc = 0;
    for (u64 b = (u64)blockIdx.x * RDF_BLOCK; b < n; b += (u64)gridDim.x * RDF_BLOCK) {
        __syncthreads();
        if (threadIdx.x == 0) {
            const u64 last = b + RDF_BLOCK - 1 < n ? b + RDF_BLOCK - 1 : n - 1;
            s_lo = run_of(runoff, 0, R - 1, b);
            s_hi = run_of(runoff, s_lo, R - 1, last);
        }
        __syncthreads();
        const u64 i = b + threadIdx.x;
        if (i < n) {
            const u32 d = rundep[run_of(runoff, s_lo, s_hi, i)];
            acc += row_hash(fcap[d], fcap[refs[i]], csup[d]);
        }
    }
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) acc += __shfl_xor(acc, off, RDF_WAVE);
    if (lane_id() == 0 && acc) atomicAdd(sum, acc);
}

// checksum of the class part straight from the compact form (members x shared lists, self excluded), so a
// checksum never needs the expanded rows: same tiles as k_class_emit, list segment staged in LDS once per tile
__global__ __launch_bounds__(RDF_BLOCK) void k_class_checksum(u64 nvblk, const u64* __restrict__ coff,
                                                              const u64* __restrict__ cchoff, const u64* __restrict__ lwoff,
                                                              const u32* __restrict__ lists, const u64* __restrict__ toff,
                                                              u32 ncls, const u64* __restrict__ ckeys,
                                                              const u32* __restrict__ fcap, const u32* __restrict__ csup,
                                                              u64* sum) {
    __shared__ u32 sl[CLS_LS];
    __shared__ u32 s_m;
    u64 acc = 0;
    for (u64 vb = blockIdx.x; vb < nvblk; vb += gridDim.x) {
        __syncthreads();
        if (threadIdx.x == 0) s_m = find_dep(toff, ncls, vb);
        __syncthreads();
        const u32 m = s_m;
        const u64 lb = lwoff[cchoff[m]], len = lwoff[cchoff[m + 1]] - lb;
        const u64 nseg = (len + CLS_LS - 1) / CLS_LS;
        const u64 t = vb - toff[m];
        const u64 dt = t / nseg, seg = t % nseg;
        const u64 k0 = coff[m] + dt * CLS_DT, k1 = k0 + CLS_DT < coff[m + 1] ? k0 + CLS_DT : coff[m + 1];
        const u64 p0 = seg * CLS_LS, p1 = p0 + CLS_LS < len ? p0 + CLS_LS : len;
        for (u64 i = threadIdx.x; i < p1 - p0; i += RDF_BLOCK) sl[i] = fcap[lists[lb + p0 + i]];
        __syncthreads();
        for (u64 k = k0; k < k1; ++k) {
            const u32 d = (u32)ckeys[k], de = fcap[d], sup = csup[d];
            for (u64 i = threadIdx.x; i < p1 - p0; i += RDF_BLOCK)
                if (sl[i] != de) acc += row_hash(de, sl[i], sup);  // fcap is injective: the self entry only
        }
    }
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) acc += __shfl_xor(acc, off, RDF_WAVE);
    if (lane_id() == 0 && acc) atomicAdd(sum, acc);
}
// Cind-shaped rows (ALG/data/Cind.scala:12-15) of output elements [first, first + n): capture code and condition
// values of dependent and referenced capture (value2 = NONE for unary captures) plus the support.
__device__ inline void decode_capture(u32 ext, u32 V, const u64* __restrict__ bkeys, u32* code, u32* v1, u32* v2) {
    const u64 six = 6ull * V;
    if (ext < six) {
        const u32 t = ext / V;
        *code = t == 0 ? 10u : t == 1 ? 12u : t == 2 ? 17u : t == 3 ? 20u : t == 4 ? 33u : 34u;
        *v1 = ext - t * V;
        *v2 = NONE32;
    } else {
        const u64 k = bkeys[ext - six];
        const int bt = bin_key_type(k);
        *code = bt == 0 ? 14u : bt == 1 ? 21u : 35u;
        *v1 = bin_key_v1(k);
        *v2 = bin_key_v2(k);
    }
}

__global__ __launch_bounds__(RDF_BLOCK) void k_decode_rows(const u32* __restrict__ refs, u64 first, u64 n,
                                                           const u64* __restrict__ runoff, const u32* __restrict__ rundep,
                                                           u64 R, const u32* __restrict__ fext, const u32* __restrict__ csup,
                                                           u32 V, const u64* __restrict__ bkeys, u32* __restrict__ rows) {
    __shared__ u64 s_lo, s_hi;
    for (u64 b = (u64)blockIdx.x * RDF_BLOCK; b < n; b += (u64)gridDim.x * RDF_BLOCK) {
        __syncthreads();
        if (threadIdx.x == 0) {
            const u64 last = b + RDF_BLOCK - 1 < n ? b + RDF_BLOCK - 1 : n - 1;
            s_lo = run_of(runoff, 0, R - 1, first + b);
            s_hi = run_of(runoff, s_lo, R - 1, first + last);
        }
        __syncthreads();
        const u64 i = b + threadIdx.x;
        if (i < n) {
            const u32 d = rundep[run_of(runoff, s_lo, s_hi, first + i)];
            u32* row = rows + 7 * i;
            decode_capture(fext[d], V, bkeys, &row[0], &row[1], &row[2]);
            decode_capture(fext[refs[first + i]], V, bkeys, &row[3], &row[4], &row[5]);
            row[6] = csup[d];
        }
    }
}

// ================================================================================================
// Sharded mode: capture groups partitioned by join-value hash over R ranks.  Global
// quantities (supports, group-size histogram, heavy masks, pivot sizes, light-group counts) are combined
// by the caller's collectives; light dependents' local survivors are routed to the dependent's owner
// (dep_owner), which keeps a ref iff every rank holding a light group of the dependent reported it.

// MIN-allreduce keys of the local pivot, INT64_MAX where the rank has no group:
// (smallest local group size, tie-break, rank) of each dependent for the MIN all-reduce that elects the pivot holder.
// Ties between ranks (common: many dependents have equal smallest groups on several ranks) go to a pseudo-random rank,
// not to the lowest rank, so the holders' work (light candidates, verify traffic) spreads evenly.  The tie-break is
// salted by the heavy-group mask when there is one: the members of a mask class have the same groups and must elect
// the same holder (k_class_pivot_shard builds each class's list on its members' holder).
#ifndef RDF_HOLDER_TIEBREAK
#define RDF_HOLDER_TIEBREAK 1
#endif
// Load-aware election (qbits > 0): the size enters as a log-scale bucket with qbits mantissa bits (2^qbits buckets per
// octave), so ranks whose smallest groups are within ~2^(1/2^qbits) of each other tie and the hash spreads them.  A rank
// whose groups are all a little smaller (it holds fewer records) then no longer wins every dependent; the holder's
// pivot grows by at most that factor.  Members of one mask class still agree (same groups on every rank).
__device__ __host__ inline u64 size_bucket_q(u64 size, int qbits) {
    if (!qbits || !size) return size;
    const int lz = 63 - __builtin_clzll(size);
    const u64 m = lz >= qbits ? (size >> (lz - qbits)) : (size << (qbits - lz));
    return ((u64)lz << qbits) | (m & ((1ull << qbits) - 1));
}
__device__ __host__ inline u64 holder_key(u64 size, u64 hmask, u32 d, u32 rank, int qbits) {
    const u64 salt = hmask ? hmask : ((u64)d | (1ull << 63));
    const u64 tie = RDF_HOLDER_TIEBREAK ? mix64(salt ^ ((u64)(rank + 1) * 0x9E3779B97F4A7C15ull)) >> 40 : 0ull;
    return (size_bucket_q(size, qbits) << 32) | (tie << 8) | rank;
}
__device__ __host__ inline u32 holder_rank(u64 key) { return (u32)(key & 0xffu); }

__global__ __launch_bounds__(RDF_BLOCK) void k_shard_best_keys(const u64* __restrict__ best, const CapInfo* __restrict__ info,
                                                               u32 C, u32 rank, int qbits, u64* out) {
    for (u64 d = (u64)blockIdx.x * RDF_BLOCK + threadIdx.x; d < C; d += (u64)gridDim.x * RDF_BLOCK) {
        const u64 b = best[d];
        out[d] = b == ~0ull ? 0x7fffffffffffffffull : holder_key(b >> 32, info[d].hmask, (u32)d, rank, qbits);
    }
}

// SUM-allreduce words of the local light groups: [d] = nlight | (nlight > 0) << 40, [C + d] = this rank's bit when
// it holds a light group of d (bits of different ranks are disjoint: the sum is the rank mask)
__global__ __launch_bounds__(RDF_BLOCK) void k_shard_light_words(const u32* __restrict__ nl, u32 C, u32 rank, u64* out) {
    for (u64 d = (u64)blockIdx.x * RDF_BLOCK + threadIdx.x; d < C; d += (u64)gridDim.x * RDF_BLOCK) {
        out[d] = (u64)nl[d] | ((u64)(nl[d] != 0) << 40);
        out[C + d] = nl[d] ? 1ull << rank : 0ull;
    }
}

// Holder-first light exchange (sharded): the rank holding d's globally smallest group (the pivot holder) checks
// its candidates against its own light groups; each survivor goes to d's owner as the holder's report (tag 0)
// and to every other rank holding a light group of d for verification (tag 1).  Output word:
// dest << 58 | tag << (32 + cb) | dep << 32 | ref, so one 8-bit radix pass on bits 58.. groups by destination and
// a sort on the low 33 + cb bits puts the reports before the (dep, ref)-ordered verify pairs.
template <bool WRITE>
__global__ __launch_bounds__(RDF_BLOCK) void k_route_survivors(const u64* __restrict__ pairs, u64 n,
                                                               const u64* __restrict__ lmask, u32 rank, u32 nranks, int cb,
                                                               u32* cnt, const u64* __restrict__ pos, u64* out) {
    for (u64 i = (u64)blockIdx.x * RDF_BLOCK + threadIdx.x; i < n; i += (u64)gridDim.x * RDF_BLOCK) {
        const u64 pr = pairs[i];
        const u32 d = (u32)(pr >> 32);
        const u64 others = lmask[d] & ~(1ull << rank);
        if (!WRITE) {
            cnt[i] = 1u + (u32)__popcll(others);
            continue;
        }
        u64 o = pos[i];
        out[o++] = ((u64)dep_owner((u32)d, nranks) << 58) | pr;
        for (u64 m = others; m; m &= m - 1) {
            const u64 r = (u64)(__ffsll((long long)m) - 1);
            out[o++] = (r << 58) | (1ull << (32 + cb)) | pr;
        }
    }
}

// destination bounds of the dest-sorted words (dest in bits 58..63), then the destination bits cleared
__global__ __launch_bounds__(RDF_BLOCK) void k_dest_bounds(const u64* __restrict__ words, u64 n, u32 nranks, u64* bounds) {
    for (u64 r = (u64)blockIdx.x * RDF_BLOCK + threadIdx.x; r <= nranks; r += (u64)gridDim.x * RDF_BLOCK)
        bounds[r] = r == nranks ? n : lower_bound_u64(words, n, r << 58);  // r = 64 would wrap the shift
}
__global__ void k_lower_bound1(const u64* __restrict__ words, u64 n, u64 key, u64* out) { *out = lower_bound_u64(words, n, key); }
__global__ __launch_bounds__(RDF_BLOCK) void k_clear_bits(u64* words, u64 n, u64 mask) {
    for (u64 i = (u64)blockIdx.x * RDF_BLOCK + threadIdx.x; i < n; i += (u64)gridDim.x * RDF_BLOCK) words[i] &= ~mask;
}

// verify pass plan: candidates = the verify pairs of d, groups = all local light groups of d (no pivot skipped)

__global__ __launch_bounds__(RDF_BLOCK) void k_verify_plan(CindView v, const u32* __restrict__ nlight_in, u32* nchunk_light,
                                                           u32* nitem_light, u32* npacked) {
    for (u64 d = (u64)blockIdx.x * RDF_BLOCK + threadIdx.x; d < v.C; d += (u64)gridDim.x * RDF_BLOCK) {
        const u64 sz = v.vcoff[d + 1] - v.vcoff[d];
        light_plan(v, (u32)d, sz ? nlight_in[d] : 0u, sz, nchunk_light, nitem_light, npacked);
    }
}

// pivot final, sharded: the rank holding d's globally smallest group (the holder) takes its candidates from that
// group and checks its own light groups; the other ranks with light groups of d verify the holder's survivors
// (k_route_survivors, then a verify pass); a heavy-only dependent (no light group on any rank) is handled by the
// holder alone.  nrl[d] = ranks holding a light group of d.
__global__ __launch_bounds__(RDF_BLOCK) void k_pivot_final_shard(CindView v, const u64* __restrict__ best_in,
                                                                 const u32* __restrict__ nlight_in,
                                                                 const u64* __restrict__ gbest, const u64* __restrict__ glight,
                                                                 u32 rank, u32* pivot, u32* nchunk_light, u32* nitem_light,
                                                                 u32* npacked, u32* nchunk_heavy, u32* nrl, CapInfo* info,
                                                                 u64* heavy_candidates /* [3 * gridDim.x] partials */) {
    u64 acc[3] = {0, 0, 0};  // heavy candidates, light candidates, light entries
    for (u64 d = (u64)blockIdx.x * RDF_BLOCK + threadIdx.x; d < v.C; d += (u64)gridDim.x * RDF_BLOCK) {
        u32 hc = 0, lc = 0, le = 0;
        if (d < v.C) {
            const u64 best = best_in[d];
            const u32 nlight = nlight_in[d];
            const u64 gl = glight[d];
            const bool heavy_only = (gl & ((1ull << 40) - 1)) == 0;
            const bool holder = holder_rank(gbest[d]) == rank && best != ~0ull;
            const u64 sz = best == ~0ull ? 0 : best >> 32;
            const u32 nch = (u32)((sz + RDF_WAVE - 1) / RDF_WAVE);
            pivot[d] = (u32)(best & 0xffffffffu);
            // only the pivot holder generates light candidates (holder-first exchange, k_route_survivors)
            light_plan(v, (u32)d, holder ? nlight : 0u, sz, nchunk_light, nitem_light, npacked);
            if (holder && nlight && nchunk_light[d]) {
                lc = (u32)sz;
                le = (u32)(v.doff[d + 1] - v.doff[d]);
            }
            // unary heavy-only dependents are emitted per bitmask class, except with --use-ars (a class list is not
            // per dependent): then they take the heavy path like the binary ones
            const bool heavy_path = d >= v.Cu || v.ar;
            nchunk_heavy[d] = (heavy_only && heavy_path && holder) ? nch : 0;
            nrl[d] = (u32)(gl >> 40);
            if (heavy_only) {
                info[d].meta |= META_HEAVY_ONLY;
                if (heavy_path && holder) hc = (u32)sz;
            }
        }
        acc[0] += hc;
        acc[1] += lc;
        acc[2] += le;
    }
    block_partials3(acc, heavy_candidates);
}

// dependent segments of concatenated (dep, ref)-sorted runs with disjoint dependents: [segb[d], sege[d]) in the input
__global__ __launch_bounds__(RDF_BLOCK) void k_seg_bounds(const u64* __restrict__ a, u64 n, u64* segb, u64* sege) {
    for (u64 i = (u64)blockIdx.x * RDF_BLOCK + threadIdx.x; i < n; i += (u64)gridDim.x * RDF_BLOCK) {
        const u64 d = a[i] >> 32;
        if (i == 0 || (a[i - 1] >> 32) != d) segb[d] = i;
        if (i + 1 == n || (a[i + 1] >> 32) != d) sege[d] = i + 1;
    }
}
__global__ __launch_bounds__(RDF_BLOCK) void k_seg_lengths(const u64* __restrict__ segb, const u64* __restrict__ sege, u32 C,
                                                           u32* len) {
    for (u64 d = (u64)blockIdx.x * RDF_BLOCK + threadIdx.x; d < C; d += (u64)gridDim.x * RDF_BLOCK)
        len[d] = (u32)(sege[d] - segb[d]);
}
__global__ __launch_bounds__(RDF_BLOCK) void k_seg_scatter(const u64* __restrict__ a, u64 n, const u64* __restrict__ segb,
                                                           const u64* __restrict__ eoff, u64* out) {
    for (u64 i = (u64)blockIdx.x * RDF_BLOCK + threadIdx.x; i < n; i += (u64)gridDim.x * RDF_BLOCK) {
        const u64 d = a[i] >> 32;
        out[eoff[d] + (i - segb[d])] = a[i];
    }
}

// (dep << 32 | ref) -> (owner << 2cb | dep << cb | ref), so one radix sort groups the pairs by owner
__global__ __launch_bounds__(RDF_BLOCK) void k_owner_pack(u64* pairs, u64 n, u32 nranks, int cb) {
    for (u64 i = (u64)blockIdx.x * RDF_BLOCK + threadIdx.x; i < n; i += (u64)gridDim.x * RDF_BLOCK) {
        const u64 pr = pairs[i];
        const u64 d = pr >> 32, r = pr & 0xffffffffull;
        pairs[i] = ((u64)dep_owner((u32)d, nranks) << (2 * cb)) | (d << cb) | r;
    }
}

// first packed pair of each owner (bounds[R] = n)
__global__ __launch_bounds__(RDF_BLOCK) void k_owner_bounds(const u64* __restrict__ pairs, u64 n, int cb, u32 nranks,
                                                            u64* bounds) {
    for (u64 i = (u64)blockIdx.x * RDF_BLOCK + threadIdx.x; i <= nranks; i += (u64)gridDim.x * RDF_BLOCK)
        bounds[i] = lower_bound_u64(pairs, n, (u64)i << (2 * cb));
}

__global__ __launch_bounds__(RDF_BLOCK) void k_owner_strip(u64* pairs, u64 n, int cb) {
    const u64 m = (1ull << cb) - 1;
    for (u64 i = (u64)blockIdx.x * RDF_BLOCK + threadIdx.x; i < n; i += (u64)gridDim.x * RDF_BLOCK) {
        const u64 k = pairs[i];
        pairs[i] = (((k >> cb) & m) << 32) | (k & m);
    }
}

// owner side: sorted reported pairs; keep the first of each run whose length equals the number of
// ranks that hold a light group of the dependent (each rank reports a pair at most once)
__global__ __launch_bounds__(RDF_BLOCK) void k_mult_flags(const u64* __restrict__ a, u64 n, const u32* __restrict__ nrl,
                                                          u32* flags) {
    for (u64 i = (u64)blockIdx.x * RDF_BLOCK + threadIdx.x; i < n; i += (u64)gridDim.x * RDF_BLOCK) {
        const u64 k = a[i];
        u32 f = 0;
        if (i == 0 || a[i - 1] != k) {
            const u32 need = nrl[k >> 32];
            f = (need >= 1 && i + need - 1 < n && a[i + need - 1] == k) ? 1u : 0u;
        }
        flags[i] = f;
    }
}

__global__ __launch_bounds__(RDF_BLOCK) void k_compact_u64(const u64* __restrict__ a, u64 n, const u32* __restrict__ flags,
                                                           const u64* __restrict__ pos, u64* out) {
    for (u64 i = (u64)blockIdx.x * RDF_BLOCK + threadIdx.x; i < n; i += (u64)gridDim.x * RDF_BLOCK)
        if (flags[i]) out[pos[i]] = a[i];
}

// mask classes with deterministic ids: masks sorted ascending, id = rank in that order
__global__ __launch_bounds__(RDF_BLOCK) void k_class_rank(const u64* __restrict__ tkeys, u64 tmask,
                                                          const u64* __restrict__ smask, u32 ncls, u32* cid) {
    for (u64 i = (u64)blockIdx.x * RDF_BLOCK + threadIdx.x; i < ncls; i += (u64)gridDim.x * RDF_BLOCK) {
        const u64 h = class_slot(tkeys, tmask, smask[i]);
        if (h != ~0ull) cid[h] = (u32)i;
    }
}

// per class: owned-member offsets and mask
__global__ __launch_bounds__(RDF_BLOCK) void k_class_info_shard(const u64* __restrict__ keys, u64 nkeys, u32 ncls,
                                                                const u64* __restrict__ smask, u64* coff, u64* cmask) {
    for (u64 m = (u64)blockIdx.x * RDF_BLOCK + threadIdx.x; m <= ncls; m += (u64)gridDim.x * RDF_BLOCK) {
        coff[m] = lower_bound_u64(keys, nkeys, m << 32);
        if (m < ncls) cmask[m] = smask[m];
    }
}

// classes whose pivot group (the globally smallest group of every member) lives on this rank
__global__ __launch_bounds__(RDF_BLOCK) void k_class_pivot_shard(CindView v, const u64* __restrict__ tkeys, u64 tmask,
                                                                 const u32* __restrict__ cid, const u32* __restrict__ pivot,
                                                                 const u64* __restrict__ gbest, u32 rank, u32* cpiv,
                                                                 u32* cnch) {
    for (u64 d = (u64)blockIdx.x * RDF_BLOCK + threadIdx.x; d < v.Cu; d += (u64)gridDim.x * RDF_BLOCK) {
        if (!(v.info[d].meta & META_HEAVY_ONLY) || holder_rank(gbest[d]) != rank) continue;
        const u64 h = class_slot(tkeys, tmask, v.info[d].hmask);
        if (h == ~0ull) continue;
        const u32 c = cid[h];
        const u32 g = pivot[d];  // members of a class have the same groups, hence the same pivot
        cpiv[c] = g;
        cnch[c] = (u32)((v.goff[g + 1] - v.goff[g] + RDF_WAVE - 1) / RDF_WAVE);
    }
}

// gathered (class << 32 | ref) pairs, sorted -> per-class lists; cchoff becomes the identity map
__global__ __launch_bounds__(RDF_BLOCK) void k_class_lists(const u64* __restrict__ pairs, u64 n, u32 ncls, u32* lists,
                                                           u64* loff, u64* ident) {
    for (u64 i = (u64)blockIdx.x * RDF_BLOCK + threadIdx.x; i < n; i += (u64)gridDim.x * RDF_BLOCK) lists[i] = (u32)pairs[i];
    for (u64 m = (u64)blockIdx.x * RDF_BLOCK + threadIdx.x; m <= ncls; m += (u64)gridDim.x * RDF_BLOCK) {
        loff[m] = lower_bound_u64(pairs, n, m << 32);
        ident[m] = m;
    }
}

__global__ __launch_bounds__(RDF_BLOCK) void k_extract_hmask(const CapInfo* __restrict__ info, u32 C, u64* out) {
    for (u64 d = (u64)blockIdx.x * RDF_BLOCK + threadIdx.x; d < C; d += (u64)gridDim.x * RDF_BLOCK) out[d] = info[d].hmask;
}

__global__ __launch_bounds__(RDF_BLOCK) void k_set_hmask(const u64* __restrict__ in, u32 C, CapInfo* info) {
    for (u64 d = (u64)blockIdx.x * RDF_BLOCK + threadIdx.x; d < C; d += (u64)gridDim.x * RDF_BLOCK) info[d].hmask = in[d];
}
// ================================================================================================
// K8: Cind.toString output (ALG/data/Cind.scala:29-31, ConditionCodes.prettyPrint ALG/util/ConditionCodes.scala:102-107)
// Byte work: every capture's pretty string ("s[p=<term>]", "o[s=<a>,p=<b>]") is built once per run into a
// string table (the terms come from the caller's dictionary, uploaded by rdf_set_dictionary); each output
// line "<dep> < <ref> (support=<n>)\n" is then assembled by one wave per 64 lines, the lanes copying 64 bytes
// of a line per step (coalesced stores).

// "s[p=" etc.: projection char, '[', first condition char, '=' -- per unary type t (UNARY_CODES order) and
// binary type bt (BINARY_CODES order); the binary second part is ",o=" / ",o=" / ",p="
__device__ __constant__ char kUnaryHead[6][4] = {{'s', '[', 'p', '='}, {'s', '[', 'o', '='}, {'p', '[', 's', '='},
                                                {'p', '[', 'o', '='}, {'o', '[', 's', '='}, {'o', '[', 'p', '='}};
__device__ __constant__ char kBinaryHead[3][4] = {{'s', '[', 'p', '='}, {'p', '[', 's', '='}, {'o', '[', 's', '='}};
__device__ __constant__ char kBinaryMid[3][3] = {{',', 'o', '='}, {',', 'o', '='}, {',', 'p', '='}};

struct CapStr {
    const char* head;  // 4 chars
    const char* mid;   // 3 chars or null (unary)
    u32 v1, v2;
};

__device__ inline CapStr cap_str(u32 ext, u32 V, const u64* __restrict__ bkeys) {
    CapStr c;
    if (ext < 6u * V) {
        const u32 t = ext / V;
        c.head = kUnaryHead[t];
        c.mid = nullptr;
        c.v1 = ext - t * V;
        c.v2 = 0;
    } else {
        const u64 k = bkeys[ext - 6u * V];
        const u32 bt = bin_key_type(k);
        c.head = kBinaryHead[bt];
        c.mid = kBinaryMid[bt];
        c.v1 = bin_key_v1(k);
        c.v2 = bin_key_v2(k);
    }
    return c;
}

// length of the pretty string of every compact capture
__global__ __launch_bounds__(RDF_BLOCK) void k_capstr_len(const u32* __restrict__ fext, u32 C, u32 V,
                                                          const u64* __restrict__ bkeys, const u64* __restrict__ toff,
                                                          u32* len) {
    for (u64 c = (u64)blockIdx.x * RDF_BLOCK + threadIdx.x; c < C; c += (u64)gridDim.x * RDF_BLOCK) {
        const CapStr s = cap_str(fext[c], V, bkeys);
        u64 n = 4 + (toff[s.v1 + 1] - toff[s.v1]) + 1;
        if (s.mid) n += 3 + (toff[s.v2 + 1] - toff[s.v2]);
        len[c] = (u32)n;
    }
}

// one wave per capture string
__global__ __launch_bounds__(RDF_BLOCK) void k_capstr_write(const u32* __restrict__ fext, u32 C, u32 V,
                                                            const u64* __restrict__ bkeys, const u64* __restrict__ toff,
                                                            const char* __restrict__ heap, const u64* __restrict__ soff,
                                                            char* str) {
    for (u64 c = (u64)blockIdx.x * RDF_WAVES_PER_BLOCK + threadIdx.x / RDF_WAVE; c < C;
         c += (u64)gridDim.x * RDF_WAVES_PER_BLOCK) {
        const CapStr s = cap_str(fext[c], V, bkeys);
        const u64 a1 = toff[s.v1], n1 = toff[s.v1 + 1] - a1;
        const u64 a2 = s.mid ? toff[s.v2] : 0, n2 = s.mid ? toff[s.v2 + 1] - a2 : 0;
        const u64 n = soff[c + 1] - soff[c];
        char* o = str + soff[c];
        for (u64 j = lane_id(); j < n; j += RDF_WAVE) {
            char ch;
            if (j < 4) ch = s.head[j];
            else if (j < 4 + n1) ch = heap[a1 + j - 4];
            else if (!s.mid) ch = ']';
            else if (j < 7 + n1) ch = s.mid[j - 4 - n1];
            else if (j < 7 + n1 + n2) ch = heap[a2 + j - 7 - n1];
            else ch = ']';
            o[j] = ch;
        }
    }
}

__device__ inline u32 dec_digits(u32 x) {
    u32 n = 1;
    while (x >= 10) {
        x /= 10;
        ++n;
    }
    return n;
}

// line length of every CIND in [first, first + n)
__global__ __launch_bounds__(RDF_BLOCK) void k_fmt_len(const u32* __restrict__ refs, u64 first, u64 n,
                                                       const u64* __restrict__ runoff, const u32* __restrict__ rundep,
                                                       u64 R, const u64* __restrict__ soff,
                                                       const u32* __restrict__ csup, u32* len) {
    for (u64 k = (u64)blockIdx.x * RDF_BLOCK + threadIdx.x; k < n; k += (u64)gridDim.x * RDF_BLOCK) {
        const u64 i = first + k;
        const u32 d = rundep[run_of(runoff, 0, R - 1, i)], r = refs[i];
        // "<dep> < <ref> (support=<n>)\n"
        len[k] = (u32)((soff[d + 1] - soff[d]) + 3 + (soff[r + 1] - soff[r]) + 10 + dec_digits(csup[d]) + 2);
    }
}

// lines at loff (exclusive scan of k_fmt_len); one wave per 64 consecutive lines
__global__ __launch_bounds__(RDF_BLOCK) void k_fmt_write(const u32* __restrict__ refs, u64 first, u64 n,
                                                         const u64* __restrict__ runoff, const u32* __restrict__ rundep,
                                                         u64 R, const u64* __restrict__ soff, const char* __restrict__ str,
                                                         const u32* __restrict__ csup, const u64* __restrict__ loff,
                                                         char* out) {
    const int lane = lane_id();
    for (u64 base = ((u64)blockIdx.x * RDF_WAVES_PER_BLOCK + threadIdx.x / RDF_WAVE) * RDF_WAVE; base < n;
         base += (u64)gridDim.x * RDF_WAVES_PER_BLOCK * RDF_WAVE) {
        // lane j looks up line base + j, then the wave writes the lines one after another
        u32 my_d = 0, my_r = 0;
        if (base + lane < n) {
            const u64 i = first + base + lane;
            my_d = rundep[run_of(runoff, 0, R - 1, i)];
            my_r = refs[i];
        }
        const u64 lines = n - base < RDF_WAVE ? n - base : RDF_WAVE;
        for (u64 l = 0; l < lines; ++l) {
            const u32 d = __shfl(my_d, (int)l, RDF_WAVE), r = __shfl(my_r, (int)l, RDF_WAVE);
            const u64 da = soff[d], dn = soff[d + 1] - da, ra = soff[r], rn = soff[r + 1] - ra;
            const u32 sup = csup[d], nd = dec_digits(sup);
            const u64 o0 = loff[base + l], len = dn + 3 + rn + 10 + nd + 2;
            for (u64 j = lane; j < len; j += RDF_WAVE) {
                char ch;
                if (j < dn) ch = str[da + j];
                else if (j < dn + 3) ch = " < "[j - dn];
                else if (j < dn + 3 + rn) ch = str[ra + j - dn - 3];
                else if (j < dn + 13 + rn) ch = " (support="[j - dn - 3 - rn];
                else if (j < dn + 13 + rn + nd) {
                    u32 x = sup;
                    for (u64 q = dn + 13 + rn + nd - 1 - j; q > 0; --q) x /= 10;  // digit j of sup
                    ch = (char)('0' + x % 10);
                } else if (j == len - 2) ch = ')';
                else ch = '\n';
                out[o0 + j] = ch;
            }
        }
    }
}

}  // namespace rdf

namespace rdf {

// ================================================================================================
// Distinct triples (--distinct-triples: `triples.distinct`, ALG/programs/RDFind.scala:284-287).
// One open-addressing table (load <= 1/2) of 64-bit entries: a 32-bit fingerprint of the triple above the
// triple's index.  A slot is claimed once by CAS and only ever lowered afterwards (atomicMin) to an entry
// of an equal triple -- same fingerprint, smaller index -- so it ends holding the FIRST occurrence; the keep
// pass marks exactly the triples that are their slot's index.  Triples are gathered for comparison only on
// a fingerprint match, i.e. for duplicates and rare fingerprint collisions: a unique triple costs one
// random table access per pass.  Survivors keep their input order (the reference's distinct defines a set).

__device__ inline u64 triple_hash(u32 a, u32 b, u32 c) {
    return mix64((((u64)a << 32) | b) ^ mix64((u64)c + 0x9E3779B97F4A7C15ull));
}

__global__ __launch_bounds__(RDF_BLOCK) void k_distinct_insert(const u32* __restrict__ s, const u32* __restrict__ p,
                                                               const u32* __restrict__ o, u64 n, u64* table, u64 mask) {
    for (u64 i = (u64)blockIdx.x * RDF_BLOCK + threadIdx.x; i < n; i += (u64)gridDim.x * RDF_BLOCK) {
        const u32 a = s[i], b = p[i], c = o[i];
        const u64 hv = triple_hash(a, b, c);
        const u64 e = (hv & 0xffffffff00000000ull) | i;  // entries never equal EMPTY64: i < 2^32 - 1
        u64 h = hv & mask;
        for (u64 probe = 0; probe <= mask; ++probe, h = (h + 1) & mask) {
            u64 cur = __hip_atomic_load(&table[h], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            if (cur == EMPTY64) {
                cur = atomicCAS(&table[h], EMPTY64, e);
                if (cur == EMPTY64) break;
            }
            if ((cur >> 32) == (e >> 32)) {
                const u32 j = (u32)cur;
                if (s[j] == a && p[j] == b && o[j] == c) {
                    if (cur > e) atomicMin(&table[h], e);
                    break;
                }
            }
        }
    }
}

__global__ __launch_bounds__(RDF_BLOCK) void k_distinct_keep(const u32* __restrict__ s, const u32* __restrict__ p,
                                                             const u32* __restrict__ o, u64 n,
                                                             const u64* __restrict__ table, u64 mask, u32* keep) {
    for (u64 i = (u64)blockIdx.x * RDF_BLOCK + threadIdx.x; i < n; i += (u64)gridDim.x * RDF_BLOCK) {
        const u32 a = s[i], b = p[i], c = o[i];
        const u64 hv = triple_hash(a, b, c);
        u64 h = hv & mask;
        u32 k = 1;
        for (u64 probe = 0; probe <= mask; ++probe, h = (h + 1) & mask) {
            const u64 cur = table[h];
            if (cur == EMPTY64) break;  // unreachable: every triple's chain ends at its own slot
            if ((cur >> 32) == (hv >> 32)) {
                const u32 j = (u32)cur;
                if (j == (u32)i) break;  // this triple is its slot's first occurrence
                if (s[j] == a && p[j] == b && o[j] == c) {
                    k = 0;
                    break;
                }
            }
        }
        keep[i] = k;
    }
}

__global__ __launch_bounds__(RDF_BLOCK) void k_distinct_scatter(const u32* __restrict__ s, const u32* __restrict__ p,
                                                                const u32* __restrict__ o, u64 n,
                                                                const u32* __restrict__ keep,
                                                                const u32* __restrict__ pos, u32* ds, u32* dp, u32* dq) {
    for (u64 i = (u64)blockIdx.x * RDF_BLOCK + threadIdx.x; i < n; i += (u64)gridDim.x * RDF_BLOCK) {
        if (keep[i]) {
            const u32 j = pos[i];
            ds[j] = s[i];
            dp[j] = p[i];
            dq[j] = o[i];
        }
    }
}

}  // namespace rdf

namespace rdf {

// ================================================================================================
// N-Triples ingest: the `Parse triples` map (ALG/programs/RDFind.scala:196-237) and the
// dictionary encoding that the build puts in its place (one u32 id space for s, p, o; ids in order of first
// appearance, line-major then s, p, o -- the host Dictionary's order, rdfind_amd/ntriples.py).
//   lines    : '\n'-terminated; lines starting with '#' and all-whitespace lines are skipped;
//   terms    : <IRI>, "literal" with \-escapes and an optional @lang / ^^<type> / ^^bare suffix, or a bare
//              token up to whitespace; --tabs: the first three '\t'-separated fields.
// Whitespace is ASCII (" \t\n\v\f\r" and 0x1c-0x1f, the ASCII part of Python's str.isspace).

static constexpr u32 NT_CHUNK = RDF_BLOCK * 16;  // bytes per block tile in the line-start passes (16 per thread)
static constexpr u32 NT_TILE = 49152;           // LDS bytes for one block's lines in the tokenizer (3 blocks per CU)

__device__ inline bool nt_space(unsigned char ch) {
    return ch == ' ' || (ch >= 9 && ch <= 13) || (ch >= 0x1c && ch <= 0x1f);
}

// newline bit mask of this thread's 16 bytes of tile c (one 16-B load; bytes past nbytes never count)
__device__ inline u32 nt_newline_mask(const unsigned char* __restrict__ text, u64 nbytes, u64 c) {
    const u64 b = c * NT_CHUNK + threadIdx.x * 16;
    if (b >= nbytes) return 0;
    const uint4 w = *(const uint4*)(text + b);
    const u32 wd[4] = {w.x, w.y, w.z, w.w};
    u32 m = 0;
#pragma unroll
    for (int k = 0; k < 16; ++k) m |= (u32)(((wd[k >> 2] >> (8 * (k & 3))) & 0xff) == '\n') << k;
    if (nbytes - b < 16) m &= (1u << (nbytes - b)) - 1u;
    return m;
}

// pass 1: newlines per tile
__global__ __launch_bounds__(RDF_BLOCK) void k_nt_count_lines(const unsigned char* __restrict__ text, u64 nbytes,
                                                              u64 nchunks, u32* cnt) {
    __shared__ u32 lds_wave[RDF_WAVES_PER_BLOCK];
    for (u64 c = blockIdx.x; c < nchunks; c += gridDim.x) {
        u32 total;
        (void)block_exclusive_scan_u32(__popc(nt_newline_mask(text, nbytes, c)), lds_wave, &total);
        if (threadIdx.x == 0) cnt[c] = total;
    }
}

// pass 2: line start offsets (line 0 starts at 0; line j+1 starts after the j-th newline)
__global__ __launch_bounds__(RDF_BLOCK) void k_nt_line_starts(const unsigned char* __restrict__ text, u64 nbytes,
                                                              u64 nchunks, const u64* __restrict__ coff, u64* lstart) {
    __shared__ u32 lds_wave[RDF_WAVES_PER_BLOCK];
    if (blockIdx.x == 0 && threadIdx.x == 0) lstart[0] = 0;
    for (u64 c = blockIdx.x; c < nchunks; c += gridDim.x) {
        u32 m = nt_newline_mask(text, nbytes, c), total;
        u64 j = coff[c] + block_exclusive_scan_u32(__popc(m), lds_wave, &total);
        const u64 b = c * NT_CHUNK + threadIdx.x * 16;
        while (m) {
            const int k = __ffs(m) - 1;
            m &= m - 1;
            lstart[++j] = b + k + 1;
        }
    }
}

struct NtGlobal {
    const unsigned char* t;
    __device__ unsigned char operator[](u64 i) const { return t[i]; }
};
struct NtLds {
    const unsigned char* tile;
    u64 base;
    __device__ unsigned char operator[](u64 i) const { return tile[i - base]; }
};

// one line [b, e): its three terms, or false (malformed)
template <typename Src>
__device__ inline bool nt_parse_line(Src text, u64 b, u64 e, int tabs, u64* ts, u64* te) {
    int nt = 0;
    if (tabs) {
        u64 f = b;
        for (u64 i = b; i <= e && nt < 3; ++i)
            if (i == e || text[i] == '\t') {
                ts[nt] = f;
                te[nt] = i;
                ++nt;
                f = i + 1;
            }
        return nt == 3;
    }
    u64 i = b;
    while (nt < 3) {
        while (i < e && nt_space(text[i])) ++i;
        if (i >= e) return false;
        u64 j;
        const unsigned char ch = text[i];
        if (ch == '<') {
            j = i + 1;
            while (j < e && text[j] != '>') ++j;
            if (j >= e) return false;
            ++j;
        } else if (ch == '"') {
            j = i + 1;
            while (j < e && text[j] != '"') j += text[j] == '\\' ? 2 : 1;
            if (j >= e) return false;
            ++j;
            if (j < e && text[j] == '@') {
                while (j < e && !nt_space(text[j])) ++j;
            } else if (j + 1 < e && text[j] == '^' && text[j + 1] == '^') {
                j += 2;
                if (j < e && text[j] == '<') {
                    while (j < e && text[j] != '>') ++j;
                    if (j >= e) return false;
                    ++j;
                } else {
                    while (j < e && !nt_space(text[j])) ++j;
                }
            }
        } else {
            j = i;
            while (j < e && !nt_space(text[j])) ++j;
        }
        ts[nt] = i;
        te[nt] = j;
        ++nt;
        i = j;
    }
    return true;
}

template <typename Src>
__device__ inline u64 nt_hash(Src s, u64 a, u32 n) {
    u64 h = 0x243F6A8885A308D3ull ^ n;
    u32 i = 0;
    for (; i + 8 <= n; i += 8) {
        u64 w = 0;
        for (int k = 0; k < 8; ++k) w |= (u64)s[a + i + k] << (8 * k);
        h = mix64(h ^ w);
    }
    u64 w = 0;
    for (int k = 0; i + k < n; ++k) w |= (u64)s[a + i + k] << (8 * k);
    return mix64(h ^ w ^ 0x9E3779B97F4A7C15ull);
}

template <typename Src>
__device__ inline u32 nt_line(Src text, u64 b, u64 e, u64 l, int tabs, u64* tstart, u32* tlen, u64* hv, u64* bad_line) {
    bool blank = true;
    for (u64 i = b; i < e && blank; ++i) blank = nt_space(text[i]);
    if ((b < e && text[b] == '#') || blank) return 0;
    u64 ts[3], te[3];
    if (!nt_parse_line(text, b, e, tabs, ts, te)) {
        atomicMin(bad_line, l);
        return 0;
    }
    for (int t = 0; t < 3; ++t) {
        tstart[3 * l + t] = ts[t];
        tlen[3 * l + t] = (u32)(te[t] - ts[t]);
        hv[3 * l + t] = nt_hash(text, ts[t], (u32)(te[t] - ts[t]));
    }
    return 1;
}

// per line: the three terms (tstart/tlen per occurrence 3*line+t), valid flag, first malformed line.  A block's
// RDF_BLOCK consecutive lines are one contiguous byte span: it is copied into LDS with coalesced 4-B loads and
// each lane parses its line from there (spans over NT_TILE bytes parse from global memory).
__global__ __launch_bounds__(RDF_BLOCK) void k_nt_tokenize(const unsigned char* __restrict__ text, u64 nbytes,
                                                           const u64* __restrict__ lstart, u64 nlines, int tabs,
                                                           u64* tstart, u32* tlen, u64* hv, u32* valid, u64* bad_line) {
    __shared__ u32 tile[NT_TILE / 4 + 2];
    for (u64 l0 = (u64)blockIdx.x * RDF_BLOCK; l0 < nlines; l0 += (u64)gridDim.x * RDF_BLOCK) {
        const u64 l1 = l0 + RDF_BLOCK < nlines ? l0 + RDF_BLOCK : nlines;
        const u64 b0 = lstart[l0], b1 = l1 < nlines ? lstart[l1] : nbytes;
        const u64 w0 = b0 & ~3ull, nw = (b1 - w0 + 3) / 4;
        const bool in_lds = nw <= NT_TILE / 4;
        __syncthreads();
        if (in_lds)
            for (u64 w = threadIdx.x; w < nw; w += RDF_BLOCK) tile[w] = *(const u32*)(text + w0 + 4 * w);
        __syncthreads();
        const u64 l = l0 + threadIdx.x;
        if (l < l1) {
            const u64 b = lstart[l];
            u64 e = l + 1 < nlines ? lstart[l + 1] - 1 : nbytes;  // excludes the '\n'
            u32 ok;
            if (in_lds) {
                NtLds src{(const unsigned char*)tile, w0};
                if (l + 1 < nlines && e > b && src[e - 1] == '\r') --e;  // "\r\n" ends a line as one terminator
                ok = nt_line(src, b, e, l, tabs, tstart, tlen, hv, bad_line);
            } else {
                NtGlobal src{text};
                if (l + 1 < nlines && e > b && src[e - 1] == '\r') --e;
                ok = nt_line(src, b, e, l, tabs, tstart, tlen, hv, bad_line);
            }
            valid[l] = ok;
        }
    }
}

// 4 text bytes starting at byte offset a, from aligned 4-B loads (the buffer is padded by 16 bytes)
__device__ inline u32 nt_word(const u32* __restrict__ w, u64 a) {
    const u64 i = a >> 2;
    const u32 sh = (u32)(a & 3) * 8;
    const u32 lo = w[i];
    return sh ? (u32)((((u64)w[i + 1] << 32) | lo) >> sh) : lo;
}

// byte equality of text[a, a+n) and text[b, b+n), four bytes per step
__device__ inline bool nt_equal(const unsigned char* __restrict__ text, u64 a, u64 b, u32 n) {
    const u32* w = (const u32*)text;
    u32 i = 0;
    for (; i + 4 <= n; i += 4)
        if (nt_word(w, a + i) != nt_word(w, b + i)) return false;
    if (i < n) {
        const u32 m = (1u << (8 * (n - i))) - 1u;
        if ((nt_word(w, a + i) ^ nt_word(w, b + i)) & m) return false;
    }
    return true;
}

// dictionary table: entries fingerprint<<32 | occurrence; the slot of a term ends holding its first occurrence
__global__ __launch_bounds__(RDF_BLOCK) void k_nt_dict_insert(const unsigned char* __restrict__ text,
                                                              const u64* __restrict__ tstart, const u32* __restrict__ tlen,
                                                              const u32* __restrict__ valid, u64 nocc,
                                                              const u64* __restrict__ hv, u64* table, u64 mask, u32* slot) {
    for (u64 k = (u64)blockIdx.x * RDF_BLOCK + threadIdx.x; k < nocc; k += (u64)gridDim.x * RDF_BLOCK) {
        if (!valid[k / 3]) continue;
        const u64 a = tstart[k];
        const u32 n = tlen[k];
        const u64 h0 = hv[k];
        const u64 e = (h0 & 0xffffffff00000000ull) | k;
        u64 h = h0 & mask;
        for (u64 probe = 0; probe <= mask; ++probe, h = (h + 1) & mask) {
            u64 cur = __hip_atomic_load(&table[h], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            if (cur == EMPTY64) {
                cur = atomicCAS(&table[h], EMPTY64, e);
                if (cur == EMPTY64) break;
            }
            if ((cur >> 32) == (e >> 32)) {
                const u32 j = (u32)cur;
                if (tlen[j] == n && nt_equal(text, tstart[j], a, n)) {
                    if (cur > e) atomicMin(&table[h], e);
                    break;
                }
            }
        }
        slot[k] = (u32)h;  // the term's slot: after the pass it holds the term's first occurrence
    }
}

// per occurrence: its term's first occurrence (rep) and whether it is that first occurrence
__global__ __launch_bounds__(RDF_BLOCK) void k_nt_dict_rep(const u32* __restrict__ valid, u64 nocc,
                                                           const u32* __restrict__ slot, const u64* __restrict__ table,
                                                           u32* rep, u32* first) {
    for (u64 k = (u64)blockIdx.x * RDF_BLOCK + threadIdx.x; k < nocc; k += (u64)gridDim.x * RDF_BLOCK) {
        u32 r = (u32)k, f = 0;
        if (valid[k / 3]) {
            r = (u32)table[slot[k]];
            f = r == (u32)k;
        }
        rep[k] = r;
        first[k] = f;
    }
}

// term ids (scan of `first` = id of each first occurrence) -> triples at their compacted line positions;
// term table (first occurrence's offset and length per id)
__global__ __launch_bounds__(RDF_BLOCK) void k_nt_assign(const u64* __restrict__ tstart, const u32* __restrict__ tlen,
                                                         const u32* __restrict__ valid, const u32* __restrict__ lpos,
                                                         u64 nocc, const u32* __restrict__ rep,
                                                         const u32* __restrict__ first, const u32* __restrict__ fid,
                                                         u32* s, u32* p, u32* o, u64* term_off, u32* term_len) {
    for (u64 k = (u64)blockIdx.x * RDF_BLOCK + threadIdx.x; k < nocc; k += (u64)gridDim.x * RDF_BLOCK) {
        const u64 l = k / 3;
        if (!valid[l]) continue;
        const u32 id = fid[rep[k]];
        const u32 t = (u32)(k - 3 * l), row = lpos[l];
        (t == 0 ? s : t == 1 ? p : o)[row] = id;
        if (first[k]) {
            term_off[id] = tstart[k];
            term_len[id] = tlen[k];
        }
    }
}

}  // namespace rdf

namespace rdf {

// ---- sharded ingest: a global dictionary from every rank's local one (term owner = hash of the term bytes) ----

// per local term: hash of its bytes, owner rank, sort key (owner << 32 | term), payload words (8 B each)
__global__ __launch_bounds__(RDF_BLOCK) void k_term_route_keys(const unsigned char* __restrict__ text,
                                                               const u64* __restrict__ toff, const u32* __restrict__ tlen,
                                                               u64 V, u32 nranks, u64* hv, u64* keys) {
    for (u64 t = (u64)blockIdx.x * RDF_BLOCK + threadIdx.x; t < V; t += (u64)gridDim.x * RDF_BLOCK) {
        const u64 h = nt_hash(text, toff[t], tlen[t]);
        hv[t] = h;
        keys[t] = ((h >> 40) % nranks) << 32 | t;
    }
}
__global__ __launch_bounds__(RDF_BLOCK) void k_term_words(const u64* __restrict__ keys, u64 V, const u32* __restrict__ tlen,
                                                          u32* words) {
    for (u64 i = (u64)blockIdx.x * RDF_BLOCK + threadIdx.x; i < V; i += (u64)gridDim.x * RDF_BLOCK)
        words[i] = (tlen[(u32)keys[i]] + 7) / 8;
}
// headers (hash, src << 58 | len << 32 | local id) and the payload words, in owner-sorted order
__global__ __launch_bounds__(RDF_BLOCK) void k_term_pack(const unsigned char* __restrict__ text, const u64* __restrict__ keys,
                                                         u64 V, const u64* __restrict__ toff, const u32* __restrict__ tlen,
                                                         const u64* __restrict__ hv, const u64* __restrict__ woff, u32 src,
                                                         u64* hdr, u64* payload) {
    for (u64 i = (u64)blockIdx.x * RDF_BLOCK + threadIdx.x; i < V; i += (u64)gridDim.x * RDF_BLOCK) {
        const u32 t = (u32)keys[i];
        const u32 n = tlen[t];
        hdr[2 * i] = hv[t];
        hdr[2 * i + 1] = ((u64)src << 58) | ((u64)n << 32) | t;
        const u64 a = toff[t], w0 = woff[i];
        for (u32 w = 0; w < (n + 7) / 8; ++w) {
            u64 x = 0;
            for (u32 k = 0; k < 8 && 8 * w + k < n; ++k) x |= (u64)text[a + 8 * w + k] << (8 * k);
            payload[w0 + w] = x;
        }
    }
}
// owner side: the received records as "occurrences" of the dictionary kernels (text = payload bytes)
__global__ __launch_bounds__(RDF_BLOCK) void k_term_records(const u64* __restrict__ hdr, u64 m, u32* words, u32* tlen,
                                                            u64* hv, u32* src_hist) {
    __shared__ u32 lh[RDF_MAX_RANKS];
    for (u32 i = threadIdx.x; i < RDF_MAX_RANKS; i += RDF_BLOCK) lh[i] = 0;
    __syncthreads();
    for (u64 i = (u64)blockIdx.x * RDF_BLOCK + threadIdx.x; i < m; i += (u64)gridDim.x * RDF_BLOCK) {
        const u64 w = hdr[2 * i + 1];
        const u32 n = (u32)((w >> 32) & ((1u << 26) - 1));
        tlen[i] = n;
        words[i] = (n + 7) / 8;
        hv[i] = hdr[2 * i];
        atomicAdd(&lh[w >> 58], 1u);
    }
    __syncthreads();
    for (u32 i = threadIdx.x; i < RDF_MAX_RANKS; i += RDF_BLOCK)
        if (lh[i]) atomicAdd(&src_hist[i], lh[i]);
}
__global__ __launch_bounds__(RDF_BLOCK) void k_needed_words(const u32* __restrict__ flags, const u32* __restrict__ len,
                                                            u32 n, u32* words) {
    for (u64 i = (u64)blockIdx.x * RDF_BLOCK + threadIdx.x; i < n; i += (u64)gridDim.x * RDF_BLOCK)
        words[i] = flags[i] ? (len[i] + 7) / 8 : 0u;
}
__global__ void k_gather_u64_at(const u64* __restrict__ a, const u64* __restrict__ idx, u32 n, u64* out) {
    for (u32 i = threadIdx.x; i < n; i += blockDim.x) out[i] = a[idx[i]];
}
__global__ __launch_bounds__(RDF_BLOCK) void k_words_to_bytes(const u64* __restrict__ woff, u64 m, u64* tstart) {
    for (u64 i = (u64)blockIdx.x * RDF_BLOCK + threadIdx.x; i < m; i += (u64)gridDim.x * RDF_BLOCK) tstart[i] = 8 * woff[i];
}
__global__ __launch_bounds__(RDF_BLOCK) void k_fill_u32(u32* a, u64 n, u32 v) {
    for (u64 i = (u64)blockIdx.x * RDF_BLOCK + threadIdx.x; i < n; i += (u64)gridDim.x * RDF_BLOCK) a[i] = v;
}
// owner's global ids: reply word (sender's local id << 32 | global id) per record (records arrive grouped by sender)
// and the owner's term table (first occurrence's byte offset and length in the payload)
__global__ __launch_bounds__(RDF_BLOCK) void k_term_reply(const u64* __restrict__ hdr, u64 m, const u32* __restrict__ rep,
                                                          const u32* __restrict__ first, const u32* __restrict__ fid, u32 base,
                                                          const u64* __restrict__ tstart, const u32* __restrict__ tlen,
                                                          u64* reply, u64* own_off, u32* own_len) {
    for (u64 i = (u64)blockIdx.x * RDF_BLOCK + threadIdx.x; i < m; i += (u64)gridDim.x * RDF_BLOCK) {
        const u32 id = fid[rep[i]];
        reply[i] = ((u64)(u32)hdr[2 * i + 1] << 32) | (base + id);
        if (first[i]) {
            own_off[id] = tstart[i];
            own_len[id] = tlen[i];
        }
    }
}
__global__ __launch_bounds__(RDF_BLOCK) void k_term_gmap(const u64* __restrict__ reply, u64 m, u32* gmapv) {
    for (u64 i = (u64)blockIdx.x * RDF_BLOCK + threadIdx.x; i < m; i += (u64)gridDim.x * RDF_BLOCK)
        gmapv[reply[i] >> 32] = (u32)reply[i];
}
__global__ __launch_bounds__(RDF_BLOCK) void k_remap3(u32* s, u32* p, u32* o, u64 n, const u32* __restrict__ gmapv) {
    for (u64 i = (u64)blockIdx.x * RDF_BLOCK + threadIdx.x; i < n; i += (u64)gridDim.x * RDF_BLOCK) {
        s[i] = gmapv[s[i]];
        p[i] = gmapv[p[i]];
        o[i] = gmapv[o[i]];
    }
}

// formatting dictionary by owner lookup: the terms every rank's output may name are the values of the frequent
// conditions (unary fval, binary keys); each owner marks its own among them
__global__ __launch_bounds__(RDF_BLOCK) void k_mark_needed(const u32* __restrict__ fval, u64 U, const u64* __restrict__ bkeys,
                                                           u64 B, u32 base, u32 nown, u32* flags) {
    for (u64 i = (u64)blockIdx.x * RDF_BLOCK + threadIdx.x; i < U + B; i += (u64)gridDim.x * RDF_BLOCK) {
        u32 v[2] = {NONE32, NONE32};
        if (i < U) {
            v[0] = fval[i];
        } else {
            const u64 k = bkeys[i - U];
            v[0] = bin_key_v1(k);
            v[1] = bin_key_v2(k);
        }
        for (int j = 0; j < 2; ++j)
            if (v[j] != NONE32 && v[j] >= base && v[j] - base < nown) flags[v[j] - base] = 1u;
    }
}
// the owner's needed terms: header (global id << 32 | len) at pos[i], payload words at woff[i]
__global__ __launch_bounds__(RDF_BLOCK) void k_dict_pack(const u32* __restrict__ flags, const u32* __restrict__ pos, u32 nown,
                                                         u32 base, const u64* __restrict__ own_off,
                                                         const u32* __restrict__ own_len,
                                                         const unsigned char* __restrict__ text, const u64* __restrict__ woff,
                                                         u64* hdr, u64* payload) {
    for (u64 i = (u64)blockIdx.x * RDF_BLOCK + threadIdx.x; i < nown; i += (u64)gridDim.x * RDF_BLOCK) {
        if (!flags[i]) continue;
        const u32 j = pos[i], n = own_len[i];
        hdr[j] = ((u64)(base + i) << 32) | n;
        const u64 a = own_off[i], w0 = woff[i];
        for (u32 w = 0; w < (n + 7) / 8; ++w) {
            u64 x = 0;
            for (u32 k = 0; k < 8 && 8 * w + k < n; ++k) x |= (u64)text[a + 8 * w + k] << (8 * k);
            payload[w0 + w] = x;
        }
    }
}
__global__ __launch_bounds__(RDF_BLOCK) void k_dict_lengths(const u64* __restrict__ hdr, u64 m, u32* len, u32* words) {
    for (u64 i = (u64)blockIdx.x * RDF_BLOCK + threadIdx.x; i < m; i += (u64)gridDim.x * RDF_BLOCK) {
        len[hdr[i] >> 32] = (u32)hdr[i];
        words[i] = ((u32)hdr[i] + 7) / 8;
    }
}
__global__ __launch_bounds__(RDF_BLOCK) void k_dict_fill(const u64* __restrict__ hdr, u64 m, const u64* __restrict__ woff,
                                                         const u64* __restrict__ payload, const u64* __restrict__ dtoff,
                                                         char* heap) {
    for (u64 i = (u64)blockIdx.x * RDF_BLOCK + threadIdx.x; i < m; i += (u64)gridDim.x * RDF_BLOCK) {
        const u32 g = (u32)(hdr[i] >> 32), n = (u32)hdr[i];
        const unsigned char* src = (const unsigned char*)(payload + woff[i]);
        for (u32 k = 0; k < n; ++k) heap[dtoff[g] + k] = (char)src[k];
    }
}
// terms of the given ids from the formatting dictionary: lengths, then bytes at the scanned offsets
__global__ __launch_bounds__(RDF_BLOCK) void k_dict_term_len(const u32* __restrict__ ids, u64 n, const u64* __restrict__ dtoff,
                                                             u32* len) {
    for (u64 i = (u64)blockIdx.x * RDF_BLOCK + threadIdx.x; i < n; i += (u64)gridDim.x * RDF_BLOCK)
        len[i] = (u32)(dtoff[ids[i] + 1] - dtoff[ids[i]]);
}
__global__ __launch_bounds__(RDF_BLOCK) void k_dict_term_copy(const u32* __restrict__ ids, u64 n, const u64* __restrict__ dtoff,
                                                              const char* __restrict__ heap, const u64* __restrict__ off,
                                                              char* out) {
    for (u64 i = (u64)blockIdx.x * RDF_BLOCK + threadIdx.x; i < n; i += (u64)gridDim.x * RDF_BLOCK) {
        const u64 a = dtoff[ids[i]], m = dtoff[ids[i] + 1] - a;
        for (u64 k = 0; k < m; ++k) out[off[i] + k] = heap[a + k];
    }
}

// parsed dictionary -> the formatter's contiguous term heap (term i at heap[off[i], off[i+1]))
__global__ __launch_bounds__(RDF_BLOCK) void k_nt_dict_gather(const unsigned char* __restrict__ text,
                                                              const u64* __restrict__ term_off,
                                                              const u64* __restrict__ hoff, u64 V, char* heap) {
    for (u64 i = (u64)blockIdx.x * RDF_BLOCK + threadIdx.x; i < V; i += (u64)gridDim.x * RDF_BLOCK) {
        const u64 a = term_off[i], b = hoff[i], n = hoff[i + 1] - b;
        for (u64 k = 0; k < n; ++k) heap[b + k] = (char)text[a + k];
    }
}

#include "shard.inl"

}  // namespace rdf
