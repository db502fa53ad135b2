// Partitioned condition counting: K1 (unary) and K2 (binary) without per-key global atomics.
// Included by kernels.inl after the wave-merge helpers.
//
// Both counts follow one shape: pass A histograms the keys of each block's contiguous chunk of triples over
// key buckets (LDS counters), an exclusive scan turns the bucket-major histogram into write offsets, pass B
// re-reads the chunk and scatters compact bucket-relative records, and one block per bucket (slice) counts
// them in LDS and keeps what reaches the support.
//
//   K1 (FrequentConditionPlanner.findFrequentSingleConditions, ALG/plan/FrequentConditionPlanner.scala:291-311):
//      key = pos * V + value, bucket = key >> bits (bits = 14, or 15 for a large |V|), record = the low key bits
//      (u16).  The count block holds the bucket's counters in LDS and writes frank = the key's rank among the
//      frequent keys of its 2^14-key rank block (or NONE), the block's frequent count (scanned into boff, so
//      frank_at gives global ranks) and the frequency bitmap fbits (1 bit per key: 2.75 MB on LUBM-100, read
//      from L2 by K2).
//   K2 (CreatedReducedDoubleConditionCounts.scala:45-86 + groupBy(type, v1, v2).sum,
//      FrequentConditionPlanner.scala:374-394): key = bt << 62 | v1 << 31 | v2 of triples whose two values are
//      frequent (fbits), merged across the wave first (wave_merge, so a record counts <= 64 occurrences);
//      bucket = hash(key) >> (64 - bits), record = (u64 key, u8 count).  The count blocks aggregate each bucket
//      in an LDS hash table sized to the bucket and append the frequent keys.

static constexpr int FR_BITS = 14;             // rank blocks: frank_at adds boff[key >> FR_BITS]
static constexpr u32 FR_R = 1u << FR_BITS;
static constexpr u32 U2_MAXB = 32768;          // K1 buckets (128 KB of LDS in the histogram passes)
#ifndef RDF_U2_SLICE_LOG
#define RDF_U2_SLICE_LOG 15
#endif
static constexpr u64 U2_SLICE = 1ull << RDF_U2_SLICE_LOG;  // K1 records per counting block
static constexpr int U2_CBLOCK = 1024;         // threads of a counting block
#ifndef RDF_B2_MAXBITS
#define RDF_B2_MAXBITS 15
#endif
static constexpr int B2_MAXBITS = RDF_B2_MAXBITS;  // K2 buckets <= 2^B2_MAXBITS (4 B of LDS each in the histogram passes)
static constexpr int B2_SLOTS = 4096;          // LDS hash slots of a K2 counting block (48 KB: 3 blocks per CU)
static constexpr u64 B2_BIG = 64ull << 20;     // above 3n = 64M keys, one more bucket bit per doubling (fewer
                                               // multi-slice buckets, which go to the spill table)
static constexpr int B2_PBLOCK = 1024;         // threads of a K2 histogram / scatter block
static constexpr u64 U1_RADIX_MIN = 1ull << 27;  // K1 groups u32 keys with radix passes (k_u1_keys) from 3n keys
static constexpr u64 U1_RADIX_LDS = 80u << 10;   // ... when the partition passes' bucket counters exceed this LDS
static constexpr u64 B2_RADIX_MIN = 1ull << 27;  // 3n from which K2 groups compact records with the radix passes
                                                 // (k_b2_emit; RDFIND_B2_RADIX_MIN overrides)

// global rank of unary condition i (= pos * V + value) among all frequent conditions, or NONE
__device__ inline u32 frank_at(const u32* __restrict__ frank, const u32* __restrict__ boff, u64 i) {
    const u32 r = frank[i];
    return r == NONE32 ? NONE32 : r + boff[i >> FR_BITS];
}

__device__ inline bool fbit(const u64* __restrict__ fbits, u64 i) { return (fbits[i >> 6] >> (i & 63)) & 1ull; }

// Leader rounds of wave merging on a bucket index: in each round, the lanes whose bucket equals the first
// remaining lane's take consecutive positions from one LDS atomic (hot buckets: predicates, Zipf objects); lanes
// left after ROUNDS take one atomic each.  Returns this lane's slot (SCATTER pass) or adds to the histogram.
// A bucket's records are counted in any order.  One round measured fastest on c2 (4 rounds: K1 passes +20 %).
template <int ROUNDS = 1>
__device__ inline u32 bucket_slot(u32* lh, u32 bk, bool active) {
    u64 todo = __ballot(active);
    u32 pos = 0;
    bool done = !active;
#pragma unroll
    for (int r = 0; r < ROUNDS; ++r) {
        if (!todo) break;
        const int l = __ffsll((long long)todo) - 1;
        const u32 bl = __shfl(bk, l, RDF_WAVE);
        const bool mine = !done && bk == bl;
        const u64 m = __ballot(mine);
        u32 base = 0;
        if (lane_id() == l) base = atomicAdd(&lh[bl], (u32)__popcll(m));
        base = __shfl(base, l, RDF_WAVE);
        if (mine) {
            pos = base + (u32)__popcll(m & lanemask_lt());
            done = true;
        }
        todo &= ~m;
        if (__popcll(m) == 1) break;  // no repeats at the head of the wave: the rest take one atomic each
    }
    if (!done) pos = atomicAdd(&lh[bk], 1u);
    return pos;
}

// ---- K1 ----------------------------------------------------------------------------------------

#ifndef RDF_PART_U
#define RDF_PART_U 4
#endif
static constexpr int PART_U = RDF_PART_U;  // triples per thread whose loads are in flight together (partition passes)
// RDF_PART_XCD=1: the K1/K2 partition passes number their blocks with xcd_block (a block's run per bucket is a few
// records: neighbouring blocks' runs share lines)
#ifndef RDF_PART_XCD
#define RDF_PART_XCD 1
#endif
__device__ inline u32 part_block() { return RDF_PART_XCD ? xcd_block() : blockIdx.x; }

template <bool SCATTER>
__global__ __launch_bounds__(RDF_BLOCK) void k_u2_part(const u32* __restrict__ s, const u32* __restrict__ p,
                                                       const u32* __restrict__ o, u64 n, u32 V, u32 NB, int bits,
                                                       u32* ghist, uint16_t* __restrict__ recs) {
    extern __shared__ u32 lh[];
    for (u32 i = threadIdx.x; i < NB; i += RDF_BLOCK) lh[i] = SCATTER ? ghist[(u64)i * gridDim.x + part_block()] : 0u;
    __syncthreads();
    const u64 per = (n + gridDim.x - 1) / gridDim.x;
    const u64 b = (u64)part_block() * per, e = b + per < n ? b + per : n;
    const u64 lmask = (1ull << bits) - 1;
    // PART_U rows per thread loaded before any is used: the chunk is read with PART_U x 3 loads in flight per lane
    // instead of one round trip per 256 rows (the slot reservations below are LDS work)
    for (u64 i0 = b; i0 < e; i0 += (u64)RDF_BLOCK * PART_U) {
        u32 ts[PART_U], tp[PART_U], to[PART_U];
#pragma unroll
        for (int u = 0; u < PART_U; ++u) {
            const u64 i = i0 + (u64)u * RDF_BLOCK + threadIdx.x;
            ts[u] = i < e ? s[i] : 0u;
            tp[u] = i < e ? p[i] : 0u;
            to[u] = i < e ? o[i] : 0u;
        }
#pragma unroll
        for (int u = 0; u < PART_U; ++u) {
            const bool act = i0 + (u64)u * RDF_BLOCK + threadIdx.x < e;
            const u64 key[3] = {(u64)ts[u], (u64)V + tp[u], 2ull * V + to[u]};
#pragma unroll
            for (int t = 0; t < 3; ++t) {
                const u32 pos = bucket_slot(lh, (u32)(key[t] >> bits), act);
                if (SCATTER && act) recs[pos] = (uint16_t)(key[t] & lmask);
            }
        }
    }
    if (!SCATTER) {
        __syncthreads();
        for (u32 i = threadIdx.x; i < NB; i += RDF_BLOCK) ghist[(u64)i * gridDim.x + part_block()] = lh[i];
    }
}

// slices per bucket (>= 1 so every bucket's ranks are written); multi-slice buckets get their global counter
// range zeroed here (their slices add into it)
__global__ __launch_bounds__(RDF_BLOCK) void k_u2_slices(const u32* __restrict__ ghist, u32 NB, u32 G, int bits, u64 K,
                                                         u32* nsl, u32* cntg) {
    const u32 b = blockIdx.x;
    if (b >= NB) return;
    const u64 len = ghist[(u64)(b + 1) * G] - ghist[(u64)b * G];
    const u64 k = (len + U2_SLICE - 1) / U2_SLICE;
    if (threadIdx.x == 0) nsl[b] = k < 1 ? 1u : (u32)k;
    if (k > 1) {
        const u64 base = (u64)b << bits, R = 1ull << bits;
        const u32 lim = (u32)(K - base < R ? K - base : R);
        for (u32 i = threadIdx.x; i < lim; i += RDF_BLOCK) cntg[base + i] = 0;
    }
}

// counts of a bucket -> ranks.  Per 2^14-key rank block r: frank[key] = rank among r's keys with count >= ms
// (NONE otherwise), bfreq[r] = their number, fstage[r * FR_R + rank] = key offset in r (for fval), fbits = the
// flags.  nbound[t] (t = 1, 2) = frequent keys of the rank block holding t * V that lie below t * V.
// Wave w owns keys [w * PER, (w + 1) * PER) of the bucket; two sweeps of 64-key ballots.
template <int BITS>
__device__ inline void u2_ranks(const u32* lc, u32 lim, u32 ms, u64 base, u64 V, u32* frank, u32* bfreq, u32* fstage,
                                u64* fbits, u64* nbound) {
    __shared__ u32 s_wtot[U2_CBLOCK / RDF_WAVE];
    constexpr u32 NW = U2_CBLOCK / RDF_WAVE, PER = (1u << BITS) / NW, WPR = FR_R / PER;  // waves per rank block
    const u32 w = threadIdx.x / RDF_WAVE, lane = lane_id();
    u32 tot = 0;
    for (u32 it = 0; it < PER; it += RDF_WAVE) {
        const u32 k = w * PER + it + lane;
        tot += (u32)__popcll(__ballot(k < lim && lc[k] >= ms));
    }
    if (lane == 0) s_wtot[w] = tot;
    __syncthreads();
    const u32 w0 = w / WPR * WPR;  // first wave of this rank block
    u32 off = 0, all = 0;
    for (u32 j = w0; j < w0 + WPR; ++j) {
        off += j < w ? s_wtot[j] : 0u;
        all += s_wtot[j];
    }
    const u64 rb = (base >> FR_BITS) + w / WPR;  // rank block index
    for (u32 it = 0; it < PER; it += RDF_WAVE) {
        const u32 k = w * PER + it + lane;
        const bool f = k < lim && lc[k] >= ms;
        const u64 m = __ballot(f);
        if (k < lim) {
            const u32 r = off + (u32)__popcll(m & lanemask_lt());
            frank[base + k] = f ? r : NONE32;
            if (f) fstage[(rb << FR_BITS) + r] = (u32)((base + k) & (FR_R - 1));
        }
        const u64 kb = base + w * PER + it;  // first key of this 64-key window (64-aligned)
        if (lane == 0 && w * PER + it < lim) {
            fbits[kb >> 6] = m;
            for (int t = 1; t <= 2; ++t) {  // t * V inside the window: frequent keys of the rank block below it
                const u64 bnd = (u64)t * V;
                if (bnd >= kb && bnd < kb + RDF_WAVE) {
                    const u32 below = (u32)(bnd - kb);
                    nbound[t] = off + (u32)__popcll(m & ((1ull << below) - 1));
                }
            }
        }
        off += (u32)__popcll(m);
    }
    if (lane == 0 && w == w0) bfreq[rb] = all;
}

// one block per (bucket, slice) of the compact slice list soff (exclusive scan of nsl); ghist = scanned
// bucket-major histogram (G blocks per bucket).  Records: the u16 low key bits of the partition passes, or (RT = u32,
// large inputs, fc_unary_part's radix form) whole keys grouped by bucket, G = 1
template <int BITS, typename RT = uint16_t>
__global__ __launch_bounds__(U2_CBLOCK) void k_u2_count(const RT* __restrict__ recs, const u32* __restrict__ ghist,
                                                        const u32* __restrict__ soff, u32 NB, u32 G, u64 K, u32 V, u32 ms,
                                                        u32* frank, u32* bfreq, u32* fstage, u64* fbits, u64* nbound,
                                                        u32* cntg, int counts_only) {
    constexpr u32 R = 1u << BITS;
    __shared__ u32 lc[R];
    const u32 x = blockIdx.x;
    if (x >= soff[NB]) return;
    u32 lo = 0, hi = NB;  // last bucket with soff[b] <= x
    while (hi - lo > 1) {
        const u32 mid = (lo + hi) >> 1;
        if (soff[mid] <= x) lo = mid;
        else hi = mid;
    }
    const u32 bk = lo, j = x - soff[bk];
    const u64 nsl = soff[bk + 1] - soff[bk];
    const u64 start = ghist[(u64)bk * G], end = ghist[(u64)(bk + 1) * G];
    const u64 len = end - start;
    const u64 s0 = start + len * j / nsl, s1 = start + len * (j + 1) / nsl;
    for (u32 i = threadIdx.x; i < R; i += U2_CBLOCK) lc[i] = 0;
    __syncthreads();
    // records in 16-B vectors (8 or 4 per lane) between the unaligned head and tail
    constexpr u64 PV = 16 / sizeof(RT);
    const u64 a0 = (s0 + PV - 1) & ~(PV - 1), a1 = s1 & ~(PV - 1);
    if (a0 < a1) {
        for (u64 i = s0 + threadIdx.x; i < a0; i += U2_CBLOCK) atomicAdd(&lc[recs[i] & (R - 1)], 1u);
        const uint4* v = (const uint4*)(recs + a0);
        const u64 nq = (a1 - a0) / PV;
        for (u64 q = threadIdx.x; q < nq; q += U2_CBLOCK) {
            const uint4 w = v[q];
            const u32 ww[4] = {w.x, w.y, w.z, w.w};
#pragma unroll
            for (int h = 0; h < 4; ++h) {
                if (sizeof(RT) == 2) {
                    atomicAdd(&lc[ww[h] & 0xffffu], 1u);
                    atomicAdd(&lc[ww[h] >> 16], 1u);
                } else {
                    atomicAdd(&lc[ww[h] & (R - 1)], 1u);
                }
            }
        }
        for (u64 i = a1 + threadIdx.x; i < s1; i += U2_CBLOCK) atomicAdd(&lc[recs[i] & (R - 1)], 1u);
    } else {
        for (u64 i = s0 + threadIdx.x; i < s1; i += U2_CBLOCK) atomicAdd(&lc[recs[i] & (R - 1)], 1u);
    }
    __syncthreads();
    const u64 base = (u64)bk << BITS;
    const u32 lim = (u32)(K - base < R ? K - base : R);
    if (nsl == 1 && counts_only) {  // sharded input: the dense local counts, summed over ranks before ranking
        for (u32 i = threadIdx.x; i < lim; i += U2_CBLOCK) cntg[base + i] = lc[i];
    } else if (nsl == 1) {
        u2_ranks<BITS>(lc, lim, ms, base, V, frank, bfreq, fstage, fbits, nbound);
    } else {  // several slices share the bucket: sum into its zeroed global counters, ranked by k_u2_finish
        for (u32 i = threadIdx.x; i < lim; i += U2_CBLOCK)
            if (lc[i]) atomicAdd(&cntg[base + i], lc[i]);
    }
}

// K1 of large inputs (fc_unary_part, 3n >= U1_RADIX_MIN): the keys pos * V + value of every triple as u32, one
// position after the other (coalesced), for the radix partition by bucket; instead of the partition passes' scatter
// of 2-B records into 2^15 open buckets per block (c4 at 10^9 triples: 28 ms for 6 GB of partial-line writes)
__global__ __launch_bounds__(RDF_BLOCK) void k_u1_keys(const u32* __restrict__ s, const u32* __restrict__ p,
                                                       const u32* __restrict__ o, u64 n, u32 V, u32* keys) {
    for (u64 i = (u64)blockIdx.x * RDF_BLOCK + threadIdx.x; i < n; i += (u64)gridDim.x * RDF_BLOCK) {
        keys[i] = s[i];
        keys[n + i] = V + p[i];
        keys[2 * n + i] = 2 * V + o[i];
    }
}
// bucket starts of keys grouped by bucket (key >> bits): ghist[b] = first key of bucket >= b, b in [0, NB]
__global__ __launch_bounds__(RDF_BLOCK) void k_u1_bucket_starts(const u32* __restrict__ keys, u64 m, int bits, u32 NB,
                                                                u32* ghist) {
    for (u64 b = (u64)blockIdx.x * RDF_BLOCK + threadIdx.x; b <= NB; b += (u64)gridDim.x * RDF_BLOCK) {
        u64 lo = 0, hi = m;
        while (lo < hi) {
            const u64 mid = (lo + hi) >> 1;
            if (((u64)keys[mid] >> bits) < b) lo = mid + 1;
            else hi = mid;
        }
        ghist[b] = (u32)lo;
    }
}

// ranks of the multi-slice buckets (one block each; single-slice buckets exit)
template <int BITS>
__global__ __launch_bounds__(U2_CBLOCK) void k_u2_finish(const u32* __restrict__ soff, u32 NB, u64 K, u32 V, u32 ms,
                                                         const u32* __restrict__ cntg, u32* frank, u32* bfreq, u32* fstage,
                                                         u64* fbits, u64* nbound) {
    constexpr u32 R = 1u << BITS;
    __shared__ u32 lc[R];
    const u32 bk = blockIdx.x;
    if (bk >= NB || soff[bk + 1] - soff[bk] <= 1) return;
    const u64 base = (u64)bk << BITS;
    const u32 lim = (u32)(K - base < R ? K - base : R);
    for (u32 i = threadIdx.x; i < R; i += U2_CBLOCK) lc[i] = i < lim ? cntg[base + i] : 0u;
    __syncthreads();
    u2_ranks<BITS>(lc, lim, ms, base, V, frank, bfreq, fstage, fbits, nbound);
}

// fval[u] = value of the frequent condition with global rank u (boff = scanned rank-block totals, NR blocks), and
// frank[key] = u: the block-local ranks become global, so later stages read frank directly
__global__ __launch_bounds__(RDF_BLOCK) void k_u2_fval(const u32* __restrict__ boff, u32 NR, const u32* __restrict__ fstage,
                                                       u32 V, u32* fval, u32* frank) {
    const u32 U = boff[NR];
    for (u64 u = (u64)blockIdx.x * RDF_BLOCK + threadIdx.x; u < U; u += (u64)gridDim.x * RDF_BLOCK) {
        u32 lo = 0, hi = NR;  // last rank block with boff[r] <= u
        while (hi - lo > 1) {
            const u32 mid = (lo + hi) >> 1;
            if (boff[mid] <= u) lo = mid;
            else hi = mid;
        }
        const u64 key = ((u64)lo << FR_BITS) + fstage[((u64)lo << FR_BITS) + (u - boff[lo])];
        fval[u] = (u32)(key % V);
        frank[key] = (u32)u;
    }
}

// fallback path (global-atomic counts): frequency bitmap from the counters
__global__ __launch_bounds__(RDF_BLOCK) void k_fbits_from_counts(const u32* __restrict__ cnt, u64 K, u32 ms, u64* fbits) {
    const u64 n_round = (K + RDF_WAVE - 1) / RDF_WAVE * RDF_WAVE;
    for (u64 i = (u64)blockIdx.x * RDF_BLOCK + threadIdx.x; i < n_round; i += (u64)gridDim.x * RDF_BLOCK) {
        const u64 m = __ballot(i < K && cnt[i] >= ms);
        if (lane_id() == 0) fbits[i >> 6] = m;
    }
}

// ---- K2 ----------------------------------------------------------------------------------------

static constexpr u64 B2_SLICE = 2560;          // K2 records per counting slice (table: next power of two >= 2x, <= B2_SLOTS)
#ifndef RDF_B2_CR
#define RDF_B2_CR 10
#endif
static constexpr int B2_CR = RDF_B2_CR;        // slice records per counting thread loaded together (10 x 256 = a slice)

__device__ inline u32 b2_bucket(u64 key, int bits) { return (u32)(mix64(key) >> (64 - bits)); }

// K2 records carry their count (1..4) in the two key bits that are zero for every term id < 2^30 (bit 30 of v2,
// bit 31 + 30 of v1): no separate count stream to scatter
static constexpr u64 B2_CBITS = (1ull << 30) | (1ull << 61);
__device__ inline u64 b2_pack(u64 key, u32 c) { return key | ((u64)((c - 1) & 1u) << 30) | ((u64)((c - 1) >> 1) << 61); }
__device__ inline u32 b2_count_of(u64 rec) { return 1u + (u32)((rec >> 30) & 1ull) + 2u * (u32)((rec >> 61) & 1ull); }

// runs of equal keys in adjacent active lanes, cut every 4 lanes: returns this lane's record count (0 if it is
// inside a piece, else 1..4)
__device__ inline u32 wave_runs4(u64 key, bool active) {
    const int lane = lane_id();
    const u64 A = __ballot(active);
    const u64 prev = __shfl_up(key, 1, RDF_WAVE);
    const bool head = active && (lane == 0 || !((A >> (lane - 1)) & 1ull) || prev != key);
    const u64 H = __ballot(head);
    if (!active) return 0;
    const u64 le = lane == RDF_WAVE - 1 ? ~0ull : ((1ull << (lane + 1)) - 1);
    const int start = 63 - __clzll((long long)(H & le));  // this lane's run head
    if ((lane - start) & 3) return 0;
    const u64 stop = (H | ~A) & ~le;  // next head or inactive lane above
    const int end = stop ? __ffsll((long long)stop) - 1 : RDF_WAVE;
    return (u32)min(4, end - lane);
}

// the binary keys of one triple window with runs of equal keys in adjacent lanes merged (the same merge in both
// passes, so the histogram pass and the scatter pass agree; a record counts <= 4 occurrences)
__device__ inline void b2_keys(u32 ts, u32 tp, u32 to, bool fs, bool fp, bool fo, u64 (&key)[3], u32 (&cnt)[3]) {
    key[0] = bin_key(2, ts, tp);  // o[s,p] (35)
    key[1] = bin_key(1, ts, to);  // p[s,o] (21)
    key[2] = bin_key(0, tp, to);  // s[p,o] (14)
    cnt[0] = wave_runs4(key[0], fs && fp);
    cnt[1] = wave_runs4(key[1], fs && fo);
    cnt[2] = wave_runs4(key[2], fp && fo);
}

template <bool SCATTER>
__global__ __launch_bounds__(B2_PBLOCK) void k_b2_part(const u32* __restrict__ s, const u32* __restrict__ p,
                                                       const u32* __restrict__ o, u64 n, u32 V, const u64* __restrict__ fbits,
                                                       int bits, u32* ghist, u64* __restrict__ rkeys) {
    extern __shared__ u32 lh[];
    const u32 NB = 1u << bits;
    for (u32 i = threadIdx.x; i < NB; i += B2_PBLOCK) lh[i] = SCATTER ? ghist[(u64)i * gridDim.x + part_block()] : 0u;
    __syncthreads();
    const u64 per = (n + gridDim.x - 1) / gridDim.x;
    const u64 b = (u64)part_block() * per, e = b + per < n ? b + per : n;
    // PART_U rows per thread: their triple loads, then their frequency-bit loads, each batch in flight together
    for (u64 i0 = b; i0 < e; i0 += (u64)B2_PBLOCK * PART_U) {
        u32 ts[PART_U], tp[PART_U], to[PART_U];
#pragma unroll
        for (int u = 0; u < PART_U; ++u) {
            const u64 i = i0 + (u64)u * B2_PBLOCK + threadIdx.x;
            ts[u] = i < e ? s[i] : 0u;
            tp[u] = i < e ? p[i] : 0u;
            to[u] = i < e ? o[i] : 0u;
        }
        bool fs[PART_U], fp[PART_U], fo[PART_U];
#pragma unroll
        for (int u = 0; u < PART_U; ++u) {
            const bool act = i0 + (u64)u * B2_PBLOCK + threadIdx.x < e;
            fs[u] = act && fbit(fbits, ts[u]);
            fp[u] = act && fbit(fbits, (u64)V + tp[u]);
            fo[u] = act && fbit(fbits, 2ull * V + to[u]);
        }
#pragma unroll
        for (int u = 0; u < PART_U; ++u) {
            u64 key[3];
            u32 cnt[3];
            b2_keys(ts[u], tp[u], to[u], fs[u], fp[u], fo[u], key, cnt);
#pragma unroll
            for (int t = 0; t < 3; ++t) {
                const bool a = cnt[t] != 0;
                const u32 pos = bucket_slot(lh, a ? b2_bucket(key[t], bits) : 0u, a);
                if (SCATTER && a) rkeys[pos] = b2_pack(key[t], cnt[t]);
            }
        }
    }
    if (!SCATTER) {
        __syncthreads();
        for (u32 i = threadIdx.x; i < NB; i += B2_PBLOCK) ghist[(u64)i * gridDim.x + part_block()] = lh[i];
    }
}

// Second-level split for inputs whose hash buckets outgrow a counting slice (c3 at full size: 2^15 buckets of ~9k
// records would all spill to the global table): one block per bucket re-partitions its records by the next `sub`
// hash bits into S = 2^sub sub-buckets and writes their starts to bstart[b * S + j].  Counts and scatter slots come
// from per-wave ballots over the S sub-buckets (one LDS atomic per wave and sub-bucket, never one per record: with
// S <= 16 counters, per-record LDS atomics serialise).
static constexpr int B2_SUB_MAX = 4;
__device__ inline u32 b2_sub(u64 rec, int bits, int sub) {
    return (u32)(mix64(rec & ~B2_CBITS) >> (64 - bits - sub)) & ((1u << sub) - 1);
}
#ifndef RDF_B2_SPLIT_R
#define RDF_B2_SPLIT_R 8
#endif
static constexpr int B2_SPLIT_R = RDF_B2_SPLIT_R;  // records per lane in flight in k_b2_split
#ifndef RDF_B2_SPLIT_GRID
#define RDF_B2_SPLIT_GRID 4096
#endif
static constexpr unsigned B2_SPLIT_GRID = RDF_B2_SPLIT_GRID;  // k_b2_split blocks (each loops over buckets)

// lanes of the wave with the same sub-bucket j (j < 2^sub; inactive lanes pass j = 1 << sub and get 0)
__device__ inline u64 sub_peers(u32 j, int sub) {
    const bool act = j < (1u << sub);
    u64 peers = __ballot(act);
    for (int b = 0; b < sub; ++b) {
        const u64 bb = __ballot((j >> b) & 1);
        peers &= ((j >> b) & 1) ? bb : ~bb;
    }
    return act ? peers : 0ull;
}

__global__ __launch_bounds__(RDF_BLOCK) void k_b2_split(const u64* __restrict__ rin, const u32* __restrict__ ghist, u32 NB,
                                                        u32 G, int bits, int sub, u64* __restrict__ rout, u32* bstart) {
    __shared__ u32 cnt[1 << B2_SUB_MAX];
    const u32 S = 1u << sub;
    const int lane = lane_id();
    const u64 lt = lanemask_lt();
    const u64 wave0 = (threadIdx.x / RDF_WAVE) * (u64)(RDF_WAVE * B2_SPLIT_R);
    constexpr u64 STEP = (u64)RDF_BLOCK * B2_SPLIT_R;
    for (u32 b = blockIdx.x; b < NB; b += gridDim.x) {
        const u64 start = ghist[(u64)b * G], end = ghist[(u64)(b + 1) * G];
        if (threadIdx.x < S) cnt[threadIdx.x] = 0;
        __syncthreads();
        for (u64 i0 = start + wave0; i0 < end; i0 += STEP) {  // B2_SPLIT_R coalesced loads per lane in flight
            u32 j[B2_SPLIT_R];
#pragma unroll
            for (int k = 0; k < B2_SPLIT_R; ++k) {
                const u64 i = i0 + (u64)k * RDF_WAVE + lane;
                j[k] = i < end ? b2_sub(rin[i], bits, sub) : S;
            }
#pragma unroll
            for (int k = 0; k < B2_SPLIT_R; ++k) {
                const u64 peers = sub_peers(j[k], sub);
                if (peers && ((peers >> lane) >> 1) == 0) atomicAdd(&cnt[j[k]], (u32)__popcll(peers));  // top peer
            }
        }
        __syncthreads();
        if (threadIdx.x == 0) {
            u32 run = 0;
            for (u32 k = 0; k < S; ++k) {
                const u32 c = cnt[k];
                cnt[k] = run;
                bstart[(u64)b * S + k] = (u32)start + run;
                run += c;
            }
            if (b == NB - 1) bstart[(u64)NB * S] = (u32)end;
        }
        __syncthreads();
        for (u64 i0 = start + wave0; i0 < end; i0 += STEP) {
            u64 r[B2_SPLIT_R];
#pragma unroll
            for (int k = 0; k < B2_SPLIT_R; ++k) {
                const u64 i = i0 + (u64)k * RDF_WAVE + lane;
                r[k] = i < end ? rin[i] : 0;
            }
#pragma unroll
            for (int k = 0; k < B2_SPLIT_R; ++k) {
                const u64 i = i0 + (u64)k * RDF_WAVE + lane;
                const u32 jj = i < end ? b2_sub(r[k], bits, sub) : S;
                const u64 peers = sub_peers(jj, sub);
                const int top = peers ? 63 - __clzll((long long)peers) : lane;
                u32 base = 0;
                if (peers && lane == top) base = atomicAdd(&cnt[jj], (u32)__popcll(peers));
                base = __shfl(base, top, RDF_WAVE);  // each lane reads its own group's top peer
                if (i < end) rout[start + base + (u32)__popcll(peers & lt)] = r[k];
            }
        }
        __syncthreads();  // cnt is reused by the next bucket
    }
}

// K2 for large inputs (fc_binary_part, 3n >= B2_RADIX_MIN): the records written compactly, then grouped by the top
// bits of their key hash with the tile-staged radix passes (radix_partition_hashed) instead of k_b2_part's scatter into
// 2^15 buckets and k_b2_split's second level (at c4 scale both write 8-B records to tens of thousands of open buckets
// per block: partial-line writes).  k_b2_emit: PART_U triples per thread, their merged records (b2_keys) at one
// claim per block iteration (the order of the records is free: the counting slices aggregate in hash tables).
__global__ __launch_bounds__(RDF_BLOCK) void k_b2_emit(const u32* __restrict__ s, const u32* __restrict__ p,
                                                       const u32* __restrict__ o, u64 n, u32 V, const u64* __restrict__ fbits,
                                                       u64* __restrict__ out, u64* counter) {
    __shared__ u32 s_wave[RDF_WAVES_PER_BLOCK];
    __shared__ u64 s_base;
    const int lane = lane_id(), wave = threadIdx.x / RDF_WAVE;
    constexpr u64 TILE = (u64)RDF_BLOCK * PART_U;
    for (u64 i0 = (u64)blockIdx.x * TILE; i0 < n; i0 += (u64)gridDim.x * TILE) {  // block-uniform trip count
        u32 ts[PART_U], tp[PART_U], to[PART_U];
#pragma unroll
        for (int u = 0; u < PART_U; ++u) {
            const u64 i = i0 + (u64)u * RDF_BLOCK + threadIdx.x;
            ts[u] = i < n ? s[i] : 0u;
            tp[u] = i < n ? p[i] : 0u;
            to[u] = i < n ? o[i] : 0u;
        }
        bool fs[PART_U], fp[PART_U], fo[PART_U];
#pragma unroll
        for (int u = 0; u < PART_U; ++u) {
            const bool act = i0 + (u64)u * RDF_BLOCK + threadIdx.x < n;
            fs[u] = act && fbit(fbits, ts[u]);
            fp[u] = act && fbit(fbits, (u64)V + tp[u]);
            fo[u] = act && fbit(fbits, 2ull * V + to[u]);
        }
        u64 key[PART_U][3];
        u32 cnt[PART_U][3];
        u32 mine = 0;
#pragma unroll
        for (int u = 0; u < PART_U; ++u) {
            b2_keys(ts[u], tp[u], to[u], fs[u], fp[u], fo[u], key[u], cnt[u]);
#pragma unroll
            for (int t = 0; t < 3; ++t) mine += cnt[u][t] != 0;
        }
        const u32 incl = wave_inclusive_scan(mine);
        if (lane == RDF_WAVE - 1) s_wave[wave] = incl;
        __syncthreads();
        u32 woff = 0, tot = 0;
#pragma unroll
        for (int w = 0; w < RDF_WAVES_PER_BLOCK; ++w) {
            woff += w < wave ? s_wave[w] : 0u;
            tot += s_wave[w];
        }
        if (threadIdx.x == 0) s_base = tot ? atomicAdd((unsigned long long*)counter, (unsigned long long)tot) : 0ull;
        __syncthreads();
        u64 q = s_base + woff + incl - mine;
#pragma unroll
        for (int u = 0; u < PART_U; ++u)
#pragma unroll
            for (int t = 0; t < 3; ++t)
                if (cnt[u][t]) out[q++] = b2_pack(key[u][t], cnt[u][t]);
        __syncthreads();  // s_wave / s_base are reused by the next iteration
    }
}

// bucket starts of hash-grouped records: bstart[b] = first record whose bucket (top `bits` of the key hash) is >= b,
// b in [0, 2^bits]
__global__ __launch_bounds__(RDF_BLOCK) void k_b2_hbounds(const u64* __restrict__ rec, u64 n, int bits, u32* bstart) {
    const u64 NB = 1ull << bits;
    for (u64 i = (u64)blockIdx.x * RDF_BLOCK + threadIdx.x; i <= n; i += (u64)gridDim.x * RDF_BLOCK) {
        const u64 b = i < n ? b2_bucket(rec[i] & ~B2_CBITS, bits) : NB;
        const u64 bp = i ? (u64)b2_bucket(rec[i - 1] & ~B2_CBITS, bits) + 1 : 0;
        for (u64 x = bp; x <= b; ++x) bstart[x] = (u32)i;
    }
}

__global__ __launch_bounds__(RDF_BLOCK) void k_b2_slices(const u32* __restrict__ ghist, u32 NB, u32 G, u32* nsl) {
    for (u32 b = blockIdx.x * RDF_BLOCK + threadIdx.x; b < NB; b += gridDim.x * RDF_BLOCK) {
        const u64 len = ghist[(u64)(b + 1) * G] - ghist[(u64)b * G];
        const u64 k = (len + B2_SLICE - 1) / B2_SLICE;
        nsl[b] = k < 1 ? 1u : (u32)k;
    }
}

// Blocks loop over the (bucket, slice) list soff: LDS hash aggregation of a slice's (key, count) records in a table
// of 2x the slice (<= B2_SLOTS).  A bucket held by one slice appends its frequent keys (count >= ms) to out and
// counts its distinct keys; the slices of a larger bucket (hot keys) append all their (key, count) partials to the
// spill list instead, which one global table then sums (as do records a crowded table refused).
// counters: [0] frequent keys in out, [1] distinct keys, [2] spill entries.
__global__ __launch_bounds__(RDF_BLOCK) void k_b2_count(const u64* __restrict__ rkeys, const u32* __restrict__ ghist, const u32* __restrict__ soff, u32 NB,
                                                        u32 G, u32 ms, u64* out, u64* spill_keys, u32* spill_cnt,
                                                        u64* counters, int all_to_spill) {
    __shared__ u64 tk[B2_SLOTS];
    __shared__ u32 tc[B2_SLOTS];
    __shared__ u32 s_part[RDF_WAVES_PER_BLOCK];
    __shared__ u64 s_base;
    const u32 nslices = soff[NB];
    u32 nd_acc = 0;
    for (u32 x = blockIdx.x; x < nslices; x += gridDim.x) {
        u32 lo = 0, hi = NB;  // last bucket with soff[b] <= x
        while (hi - lo > 1) {
            const u32 mid = (lo + hi) >> 1;
            if (soff[mid] <= x) lo = mid;
            else hi = mid;
        }
        const u32 bk = lo, j = x - soff[bk];
        const u64 nsl = soff[bk + 1] - soff[bk];
        const u64 start = ghist[(u64)bk * G], end = ghist[(u64)(bk + 1) * G];
        const u64 len = end - start;
        const u64 s0 = start + len * j / nsl, s1 = start + len * (j + 1) / nsl;
        u32 T = 64;
        while (T < B2_SLOTS && T < 2 * (s1 - s0)) T <<= 1;
        for (u32 i = threadIdx.x; i < T; i += RDF_BLOCK) {
            tk[i] = EMPTY64;
            tc[i] = 0;
        }
        __syncthreads();
        // the slice's records (<= B2_CR per thread) are loaded up front: one round trip, not one per record
        u64 rr[B2_CR];
#pragma unroll
        for (int q = 0; q < B2_CR; ++q) {
            const u64 i = s0 + (u64)q * RDF_BLOCK + threadIdx.x;
            rr[q] = i < s1 ? rkeys[i] : 0;
        }
        for (u64 i0 = s0; i0 < s1; i0 += (u64)RDF_BLOCK * B2_CR) {
          if (i0 != s0) {  // slices longer than B2_CR x RDF_BLOCK (only with RDF_B2_CR below the default)
#pragma unroll
            for (int q = 0; q < B2_CR; ++q) {
                const u64 i = i0 + (u64)q * RDF_BLOCK + threadIdx.x;
                rr[q] = i < s1 ? rkeys[i] : 0;
            }
          }
#pragma unroll
          for (int q = 0; q < B2_CR; ++q) {
            if (i0 + (u64)q * RDF_BLOCK + threadIdx.x >= s1) continue;
            const u64 rec = rr[q];
            const u64 key = rec & ~B2_CBITS;
            const u32 c = b2_count_of(rec);
            u32 h = (u32)mix64(key) & (T - 1);  // low hash bits (the bucket used the high ones)
            bool done = false;
            for (u32 probe = 0; probe < 32 && !done; ++probe) {
                u64 k = tk[h];
                if (k == EMPTY64) {
                    const u64 prev = atomicCAS(&tk[h], EMPTY64, key);
                    k = prev == EMPTY64 ? key : prev;
                }
                if (k == key) {
                    atomicAdd(&tc[h], c);
                    done = true;
                }
                h = (h + 1) & (T - 1);
            }
            if (!done) {  // a crowded table: the record goes to the spill list
                const u64 at = atomicAdd(&counters[2], 1ull);
                spill_keys[at] = key;
                spill_cnt[at] = c;
            }
          }
        }
        __syncthreads();
        const u32 per = (T + RDF_BLOCK - 1) / RDF_BLOCK;  // consecutive slots per thread
        const bool single = nsl == 1 && !all_to_spill;  // all_to_spill: local partials for the sharded exchange
        u32 nsel = 0, nd = 0;
        for (u32 q = 0; q < per; ++q) {
            const u32 slot = threadIdx.x * per + q;
            if (slot < T && tk[slot] != EMPTY64) {
                ++nd;
                nsel += single ? (tc[slot] >= ms) : 1u;
            }
        }
        if (single) nd_acc += nd;
        // one reservation per slice
        const u32 w = threadIdx.x / RDF_WAVE;
        const u32 incl = wave_inclusive_scan(nsel);
        if (lane_id() == RDF_WAVE - 1) s_part[w] = incl;
        __syncthreads();
        u32 woff = 0, tot = 0;
        for (u32 k = 0; k < RDF_WAVES_PER_BLOCK; ++k) {
            woff += k < w ? s_part[k] : 0u;
            tot += s_part[k];
        }
        if (threadIdx.x == 0) s_base = tot ? atomicAdd(single ? &counters[0] : &counters[2], (u64)tot) : 0;
        __syncthreads();
        u64 pos = s_base + woff + incl - nsel;
        for (u32 q = 0; q < per; ++q) {
            const u32 slot = threadIdx.x * per + q;
            if (slot >= T || tk[slot] == EMPTY64) continue;
            if (single) {
                if (tc[slot] >= ms) out[pos++] = tk[slot];
            } else {
                spill_keys[pos] = tk[slot];
                spill_cnt[pos] = tc[slot];
                ++pos;
            }
        }
        __syncthreads();  // the table is reused by the next slice
    }
    nd_acc = wave_sum(nd_acc);
    __shared__ u32 s_nd[RDF_WAVES_PER_BLOCK];
    if (lane_id() == 0) s_nd[threadIdx.x / RDF_WAVE] = nd_acc;
    __syncthreads();
    if (threadIdx.x == 0) {
        u64 t = 0;
        for (int k = 0; k < RDF_WAVES_PER_BLOCK; ++k) t += s_nd[k];
        if (t) atomicAdd(&counters[1], t);
    }
}

// spill entries -> one global open-addressing table (summed counts), then k_bin_freq_flags / k_bin_freq_scatter
__global__ __launch_bounds__(RDF_BLOCK) void k_spill_insert(const u64* __restrict__ keys, const u32* __restrict__ cnt, u64 n,
                                                            u64* tkeys, u32* tcnt, u64 tmask);
