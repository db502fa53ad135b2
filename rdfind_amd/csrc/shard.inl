// Sharded input (SURVEY.md 8e with the input itself partitioned): every rank holds only its slice of the
// triples.  The condition counts are combined as partial sums (FrequentConditionPlanner.scala:293-309 and
// :381-393 groupBy(...).sum): unary and binary (key, count) partials by an all-to-all to the key's owner, which
// sums them and contributes its frequent keys to an all-gather.  Then each triple travels to the ranks owning its join values
// (ALG/programs/RDFind.scala:339-345 groupBy(joinValue)), so capture groups stay local to their join shard.
// Included by kernels.inl.

// owner rank of a binary condition key (its partial counts are summed there)
__device__ inline u32 key_owner(u64 key, u32 nranks) { return (u32)((mix64(key) & 0xffffffffull) % nranks); }

// destinations of a triple: the distinct owners of its projected join values (at most 3)
__device__ inline int triple_dests(u32 ts, u32 tp, u32 to, int proj, u32 nranks, const u64* hot, u32 hmask, u32 (&d)[3]) {
    int k = 0;
    const u32 v[3] = {ts, tp, to};
#pragma unroll
    for (int t = 0; t < 3; ++t) {
        if (!(proj & (1 << t))) continue;
        const u32 r = join_owner(v[t], nranks, hot, hmask);
        bool seen = false;
        for (int j = 0; j < k; ++j) seen |= d[j] == r;
        if (!seen) d[k++] = r;
    }
    return k;
}

// route the local triples: pass 1 counts copies per (destination, block), pass 2 writes each copy as two words
// (s << 32 | p, o) at the scanned destination-major offsets (ghist[d * G + block])
template <bool SCATTER>
__global__ __launch_bounds__(RDF_BLOCK) void k_route_triples(const u32* __restrict__ s, const u32* __restrict__ p,
                                                             const u32* __restrict__ o, u64 n, int proj, u32 nranks,
                                                             const u64* __restrict__ hot, u32 hmask, u32* ghist,
                                                             u64* __restrict__ out) {
    __shared__ u32 lh[RDF_MAX_RANKS];
    for (u32 i = threadIdx.x; i < nranks; i += RDF_BLOCK) lh[i] = SCATTER ? ghist[(u64)i * gridDim.x + blockIdx.x] : 0u;
    __syncthreads();
    const u64 per = (n + gridDim.x - 1) / gridDim.x;
    const u64 b = (u64)blockIdx.x * per, e = b + per < n ? b + per : n;
    for (u64 i = b + threadIdx.x; i < e; i += RDF_BLOCK) {
        const u32 ts = s[i], tp = p[i], to = o[i];
        u32 d[3];
        const int k = triple_dests(ts, tp, to, proj, nranks, hot, hmask, d);
        for (int j = 0; j < k; ++j) {
            const u32 pos = atomicAdd(&lh[d[j]], 1u);
            if (SCATTER) {
                out[2ull * pos] = ((u64)ts << 32) | tp;
                out[2ull * pos + 1] = to;
            }
        }
    }
    if (!SCATTER) {
        __syncthreads();
        for (u32 i = threadIdx.x; i < nranks; i += RDF_BLOCK) ghist[(u64)i * gridDim.x + blockIdx.x] = lh[i];
    }
}

__global__ __launch_bounds__(RDF_BLOCK) void k_unpack_triples(const u64* __restrict__ in, u64 m, u32* s, u32* p, u32* o) {
    for (u64 i = (u64)blockIdx.x * RDF_BLOCK + threadIdx.x; i < m; i += (u64)gridDim.x * RDF_BLOCK) {
        const u64 w0 = in[2 * i], w1 = in[2 * i + 1];
        s[i] = (u32)(w0 >> 32);
        p[i] = (u32)w0;
        o[i] = (u32)w1;
    }
}

// binary (key, count) partials grouped by the key's owner, two words each
template <bool SCATTER>
__global__ __launch_bounds__(RDF_BLOCK) void k_route_pairs(const u64* __restrict__ keys, const u32* __restrict__ cnt, u64 m,
                                                           u32 nranks, u32* ghist, u64* __restrict__ out) {
    __shared__ u32 lh[RDF_MAX_RANKS];
    for (u32 i = threadIdx.x; i < nranks; i += RDF_BLOCK) lh[i] = SCATTER ? ghist[(u64)i * gridDim.x + blockIdx.x] : 0u;
    __syncthreads();
    const u64 per = (m + gridDim.x - 1) / gridDim.x;
    const u64 b = (u64)blockIdx.x * per, e = b + per < m ? b + per : m;
    for (u64 i = b + threadIdx.x; i < e; i += RDF_BLOCK) {
        const u64 key = keys[i];
        const u32 pos = atomicAdd(&lh[key_owner(key, nranks)], 1u);
        if (SCATTER) {
            out[2ull * pos] = key;
            out[2ull * pos + 1] = cnt[i];
        }
    }
    if (!SCATTER) {
        __syncthreads();
        for (u32 i = threadIdx.x; i < nranks; i += RDF_BLOCK) ghist[(u64)i * gridDim.x + blockIdx.x] = lh[i];
    }
}

// received (key, count) word pairs -> the global summing table
__global__ __launch_bounds__(RDF_BLOCK) void k_pairs_insert(const u64* __restrict__ in, u64 m, u64* tkeys, u32* tcnt,
                                                            u64 tmask) {
    for (u64 i = (u64)blockIdx.x * RDF_BLOCK + threadIdx.x; i < m; i += (u64)gridDim.x * RDF_BLOCK)
        global_hash_add(tkeys, tcnt, tmask, in[2 * i], (u32)in[2 * i + 1]);
}

// Sparse unary exchange: the slice's nonzero unary counts as (key << 32 | count) words (key = pos * V + value < 2^32),
// grouped by the key's owner rank, which sums them; no rank ever moves the dense 3V counter array.
template <bool SCATTER>
__global__ __launch_bounds__(RDF_BLOCK) void k_unary_route(const u32* __restrict__ cnt, u64 K, u32 nranks, u32* ghist,
                                                           u64* __restrict__ out) {
    __shared__ u32 lh[RDF_MAX_RANKS];
    for (u32 i = threadIdx.x; i < nranks; i += RDF_BLOCK) lh[i] = SCATTER ? ghist[(u64)i * gridDim.x + blockIdx.x] : 0u;
    __syncthreads();
    const u64 per = (K + gridDim.x - 1) / gridDim.x;
    const u64 b = (u64)blockIdx.x * per, e = b + per < K ? b + per : K;
    for (u64 i = b + threadIdx.x; i < e; i += RDF_BLOCK) {
        const u32 c = cnt[i];
        if (!c) continue;
        const u32 pos = atomicAdd(&lh[key_owner(i, nranks)], 1u);
        if (SCATTER) out[pos] = (i << 32) | c;
    }
    if (!SCATTER) {
        __syncthreads();
        for (u32 i = threadIdx.x; i < nranks; i += RDF_BLOCK) ghist[(u64)i * gridDim.x + blockIdx.x] = lh[i];
    }
}

// received (key << 32 | count) words -> the global summing table
__global__ __launch_bounds__(RDF_BLOCK) void k_packed_insert(const u64* __restrict__ in, u64 m, u64* tkeys, u32* tcnt,
                                                             u64 tmask) {
    for (u64 i = (u64)blockIdx.x * RDF_BLOCK + threadIdx.x; i < m; i += (u64)gridDim.x * RDF_BLOCK)
        global_hash_add(tkeys, tcnt, tmask, in[i] >> 32, (u32)in[i]);
}

// every owner's frequent unary keys, sorted: global rank u of key k = its index (frank[k] = u with boff = 0),
// fval[u] = the condition value, fbits = the frequency bitmap (zeroed before)
__global__ __launch_bounds__(RDF_BLOCK) void k_ranks_from_keys(const u64* __restrict__ keys, u64 U, u32 V, u32* frank,
                                                               u32* fval, u64* fbits) {
    for (u64 u = (u64)blockIdx.x * RDF_BLOCK + threadIdx.x; u < U; u += (u64)gridDim.x * RDF_BLOCK) {
        const u64 k = keys[u];
        frank[k] = (u32)u;
        fval[u] = (u32)(k % V);
        atomicOr((unsigned long long*)&fbits[k >> 6], 1ull << (k & 63));
    }
}


// Hot join value candidates of this owner rank: its summed unary (key, count) table entries (key = pos * V + value)
// whose position is projected and whose count reaches thr, as key << 32 | count (at most cap; *n counts them all)
__global__ __launch_bounds__(RDF_BLOCK) void k_hot_candidates(const u64* __restrict__ tkeys, const u32* __restrict__ tcnt,
                                                              u64 tcap, u32 V, int proj, u32 thr, u32 cap, u64* out, u32* n) {
    for (u64 i = (u64)blockIdx.x * RDF_BLOCK + threadIdx.x; i < tcap; i += (u64)gridDim.x * RDF_BLOCK) {
        const u64 k = tkeys[i];
        if (k == EMPTY64) continue;
        const u32 c = tcnt[i];
        if (c < thr || !((proj >> (int)(k / V)) & 1)) continue;
        const u32 slot = atomicAdd(n, 1u);
        if (slot < cap) out[slot] = (k << 32) | c;
    }
}
