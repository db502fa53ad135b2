// Common definitions for the rdfind_amd HIP library (gfx950 / CDNA4, wave64).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stddef.h>

#define RDF_WAVE 64
#define RDF_BLOCK 256
#define RDF_WAVES_PER_BLOCK (RDF_BLOCK / RDF_WAVE)

typedef unsigned long long u64;
typedef uint32_t u32;

static constexpr u64 EMPTY64 = ~0ull;
static constexpr u32 EMPTY32 = 0xffffffffu;
static constexpr u32 NONE32 = 0xffffffffu;

// Unary capture type index t in [0,6): codes 10 s[p], 12 s[o], 17 p[s], 20 p[o], 33 o[s], 34 o[p]
// (ConditionCodes.scala:11-130; pinned by ConditionCodes$Test.scala:28-33).
// Binary type index bt in [0,3): 14 s[p,o], 21 p[s,o], 35 o[s,p].
// Components of binary bt: first (v1) / second (v2) unary type index.
__host__ __device__ inline int bin_comp1(int bt) { return bt == 0 ? 0 : (bt == 1 ? 2 : 4); }
__host__ __device__ inline int bin_comp2(int bt) { return bt == 0 ? 1 : (bt == 1 ? 3 : 5); }

// Binary condition key: bt<<62 | v1<<31 | v2  (requires term ids < 2^31)
__host__ __device__ inline u64 bin_key(u64 bt, u64 v1, u64 v2) { return (bt << 62) | (v1 << 31) | v2; }
__host__ __device__ inline int bin_key_type(u64 k) { return (int)(k >> 62); }
__host__ __device__ inline u32 bin_key_v1(u64 k) { return (u32)((k >> 31) & 0x7fffffffu); }
__host__ __device__ inline u32 bin_key_v2(u64 k) { return (u32)(k & 0x7fffffffu); }

__host__ __device__ inline u64 mix64(u64 x) {
    x ^= x >> 33;
    x *= 0xff51afd7ed558ccdULL;
    x ^= x >> 33;
    x *= 0xc4ceb9fe1a85ec53ULL;
    x ^= x >> 33;
    return x;
}

// owner rank of a join value (capture groups are sharded by join-value hash)
__host__ __device__ inline u32 shard_of(u32 join, u32 nranks) {
    return nranks <= 1 ? 0u : (u32)((((u64)join * 0x9E3779B97F4A7C15ull) >> 32) % nranks);
}

// owner rank of a dependent (compact capture id): it finalises the dependent's refs in sharded mode.  Hashed, not
// d % N: compact ids are 2 rank(cond) + (t >= 3), so id parity follows the projection and d % 2 gave one rank 64 % of
// the CINDs at two ranks
__host__ __device__ inline u32 dep_owner(u32 d, u32 nranks) {
    return nranks <= 1 ? 0u : (u32)((mix64(d) >> 32) % nranks);
}

// Hot join values (sharded): a small open-addressing table of (join << 32 | owner rank) entries, load <= 1/2, probed
// linearly from mix64(join) & mask.  The values whose occurrences are a visible share of a rank's load get owners
// from a balanced (largest-first) assignment instead of the hash (sh_phase18); every other value keeps shard_of.
__host__ __device__ inline u32 hot_slot(u32 join, u32 mask) { return (u32)(mix64(join) & mask); }
__device__ inline u32 join_owner(u32 join, u32 nranks, const u64* __restrict__ hot, u32 hmask) {
    if (nranks <= 1) return 0u;
    if (hot) {
        for (u32 h = hot_slot(join, hmask);; h = (h + 1) & hmask) {
            const u64 e = hot[h];
            if (e == EMPTY64) break;
            if ((u32)(e >> 32) == join) return (u32)e;
        }
    }
    return shard_of(join, nranks);
}

// join values whose capture records a K3 emission writes: this rank's shard (hash, or the hot table's owner) and, when
// the capture groups are built in join-value ranges (inputs whose records exceed one pass), the range [lo, hi)
struct JoinSel {
    u32 rank, nranks, lo, hi;
    const u64* hot = nullptr;  // sharded: the hot join values' owners (nullptr: hash only)
    u32 hmask = 0;
    __device__ inline bool take(u32 join) const {
        return join >= lo && join < hi && join_owner(join, nranks, hot, hmask) == rank;
    }
};
static constexpr u32 JOIN_ALL_HI = 0xffffffffu;

__device__ inline u32 hash32(u32 x) {
    x ^= x >> 16;
    x *= 0x7feb352dU;
    x ^= x >> 15;
    x *= 0x846ca68bU;
    x ^= x >> 16;
    return x;
}

__device__ inline int lane_id() { return (int)(threadIdx.x & (RDF_WAVE - 1)); }
__device__ inline u64 lanemask_lt() { return (1ull << lane_id()) - 1ull; }

// blockIdx.x renumbered so that consecutive numbers share an XCD (blocks are dealt round-robin over the 8 XCDs,
// MI355X_MICROARCH.md "Workgroup dispatch"): XCD x runs numbers [x q + min(x, r), + q + (x < r)), q = n / 8, r = n % 8.
// For kernels whose neighbouring blocks write neighbouring bytes (per-(bin, block) runs of a partition pass, their
// histogram columns): the partial lines the neighbours share meet in one L2.
__device__ inline u32 xcd_block() {
    const u32 b = blockIdx.x, n = gridDim.x, x = b % 8u, q = n / 8u, r = n % 8u;
    return x * q + (x < r ? x : r) + b / 8u;
}

// Wave-wide inclusive scan (u32) with DPP-free shuffles.
__device__ inline u32 wave_inclusive_scan(u32 v) {
    const int lane = lane_id();
#pragma unroll
    for (int off = 1; off < RDF_WAVE; off <<= 1) {
        u32 t = __shfl_up(v, off, RDF_WAVE);
        if (lane >= off) v += t;
    }
    return v;
}

__device__ inline u64 wave_inclusive_scan64(u64 v) {
    const int lane = lane_id();
#pragma unroll
    for (int off = 1; off < RDF_WAVE; off <<= 1) {
        u64 t = __shfl_up(v, off, RDF_WAVE);
        if (lane >= off) v += t;
    }
    return v;
}

__device__ inline u32 wave_sum(u32 v) {
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) v += __shfl_xor(v, off, RDF_WAVE);
    return v;
}

// Wave-aggregated append: every lane with `want` slots reserves them in one atomic per wave.
// Returns this lane's first index.
__device__ inline u64 wave_append(u64* counter, u32 want) {
    u32 incl = wave_inclusive_scan(want);
    u32 total = __shfl(incl, RDF_WAVE - 1, RDF_WAVE);
    u64 base = 0;
    if (lane_id() == RDF_WAVE - 1 && total) base = atomicAdd(counter, (u64)total);
    base = __shfl(base, RDF_WAVE - 1, RDF_WAVE);
    return base + incl - want;
}

inline unsigned grid_for(u64 n, unsigned block, unsigned cap = 65535u * 8u) {
    u64 g = (n + block - 1) / block;
    if (g < 1) g = 1;
    if (g > cap) g = cap;
    return (unsigned)g;
}
