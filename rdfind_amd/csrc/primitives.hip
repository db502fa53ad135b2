// Device-wide primitives: exclusive scan and LSD radix sort of 64-bit keys (gfx950, wave64).
//
// The radix sort is the grouping engine that replaces Flink's sort-based groupBy on the join value
// (ALG/programs/RDFind.scala:339-345 groupBy("joinValue") -> combineGroup -> reduceGroup): records are
// packed as (capture << joinbits | join) and sorted on exactly the needed bits, in as few passes of <= 10-bit
// digits as cover them (43 bits: 9+9+9+8+8).  Per pass: (1) per-tile digit histogram in LDS, (2) device exclusive
// scan of the digit-major histogram, (3) stable scatter where each key's in-tile rank comes from wave ballots (one
// ballot per digit bit gives the peer mask of lanes with the same digit) plus per-wave running digit counters in LDS.
#include <cstdint>
#include <cstdlib>
#include <type_traits>

#include "primitives.hpp"

namespace rdf {

// ------------------------------------------------------------------------------------------------
// Block-level helpers

typedef unsigned int u32x4_t __attribute__((ext_vector_type(4)));
typedef unsigned long long u64x2_t __attribute__((ext_vector_type(2)));

template <typename T>
__device__ inline T block_exclusive_scan(T v, T* lds_wave, T* total) {
    const int lane = lane_id();
    const int wave = threadIdx.x / RDF_WAVE;
    T incl = v;
#pragma unroll
    for (int off = 1; off < RDF_WAVE; off <<= 1) {
        T t = __shfl_up(incl, off, RDF_WAVE);
        if (lane >= off) incl += t;
    }
    if (lane == RDF_WAVE - 1) lds_wave[wave] = incl;
    __syncthreads();
    T wave_off = 0, sum = 0;
#pragma unroll
    for (int w = 0; w < RDF_WAVES_PER_BLOCK; ++w) {
        T x = lds_wave[w];
        if (w < wave) wave_off += x;
        sum += x;
    }
    *total = sum;
    __syncthreads();
    return wave_off + incl - v;
}

// ------------------------------------------------------------------------------------------------
// Exclusive scan: out[i] = sum_{j<i} in[j]   (reduce-then-scan, tile = 256 threads x 16 items)

static constexpr int SCAN_ITEMS = 16;
static constexpr int SCAN_TILE = RDF_BLOCK * SCAN_ITEMS;

template <typename TI, typename TO>
__global__ __launch_bounds__(RDF_BLOCK) void k_scan_reduce(const TI* __restrict__ in, u64 n, TO* __restrict__ tile_sums) {
    __shared__ TO lds_wave[RDF_WAVES_PER_BLOCK];
    const u64 base = (u64)blockIdx.x * SCAN_TILE;
    TO acc = 0;
#pragma unroll
    for (int i = 0; i < SCAN_ITEMS; ++i) {
        u64 idx = base + (u64)i * RDF_BLOCK + threadIdx.x;
        if (idx < n) acc += (TO)in[idx];
    }
    TO total;
    block_exclusive_scan<TO>(acc, lds_wave, &total);
    if (threadIdx.x == 0) tile_sums[blockIdx.x] = total;
}

template <typename TO>
__global__ __launch_bounds__(RDF_BLOCK) void k_scan_single(TO* __restrict__ a, u64 n, TO* __restrict__ grand_total) {
    __shared__ TO lds_wave[RDF_WAVES_PER_BLOCK];
    TO carry = 0;
    for (u64 base = 0; base < n; base += SCAN_TILE) {
        TO v[SCAN_ITEMS];
        TO local = 0;
        const u64 tb = base + (u64)threadIdx.x * SCAN_ITEMS;
#pragma unroll
        for (int i = 0; i < SCAN_ITEMS; ++i) {
            v[i] = (tb + i < n) ? a[tb + i] : (TO)0;
            local += v[i];
        }
        TO total;
        TO off = block_exclusive_scan<TO>(local, lds_wave, &total) + carry;
#pragma unroll
        for (int i = 0; i < SCAN_ITEMS; ++i) {
            if (tb + i < n) a[tb + i] = off;
            off += v[i];
        }
        carry += total;
    }
    if (threadIdx.x == 0 && grand_total) *grand_total = carry;
}

template <typename TI, typename TO>
__global__ __launch_bounds__(RDF_BLOCK) void k_scan_apply(const TI* in, TO* out, u64 n,
                                                          const TO* __restrict__ tile_offsets) {
    __shared__ TO lds[SCAN_TILE];
    __shared__ TO lds_wave[RDF_WAVES_PER_BLOCK];
    const u64 base = (u64)blockIdx.x * SCAN_TILE;
#pragma unroll
    for (int i = 0; i < SCAN_ITEMS; ++i) {
        u64 idx = base + (u64)i * RDF_BLOCK + threadIdx.x;
        lds[i * RDF_BLOCK + threadIdx.x] = (idx < n) ? (TO)in[idx] : (TO)0;
    }
    __syncthreads();
    TO v[SCAN_ITEMS];
    TO local = 0;
#pragma unroll
    for (int i = 0; i < SCAN_ITEMS; ++i) {
        v[i] = lds[threadIdx.x * SCAN_ITEMS + i];
        local += v[i];
    }
    TO total;
    TO off = block_exclusive_scan<TO>(local, lds_wave, &total) + tile_offsets[blockIdx.x];
#pragma unroll
    for (int i = 0; i < SCAN_ITEMS; ++i) {
        lds[threadIdx.x * SCAN_ITEMS + i] = off;
        off += v[i];
    }
    __syncthreads();
#pragma unroll
    for (int i = 0; i < SCAN_ITEMS; ++i) {
        u64 idx = base + (u64)i * RDF_BLOCK + threadIdx.x;
        if (idx < n) out[idx] = lds[i * RDF_BLOCK + threadIdx.x];
    }
}

// up to SCAN_FOLD_TILES tiles: each apply block sums the tile totals before it itself (<= 1024 L2 loads shared by the
// block) instead of a k_scan_single launch between reduce and apply; the last block writes the grand total
static constexpr u64 SCAN_FOLD_TILES = 1024;
template <typename TI, typename TO>
__global__ __launch_bounds__(RDF_BLOCK) void k_scan_apply_fold(const TI* in, TO* out, u64 n, const TO* __restrict__ tile_sums,
                                                               TO* __restrict__ grand_total) {
    __shared__ TO lds[SCAN_TILE];
    __shared__ TO lds_wave[RDF_WAVES_PER_BLOCK];
    const u64 base = (u64)blockIdx.x * SCAN_TILE;
#pragma unroll
    for (int i = 0; i < SCAN_ITEMS; ++i) {
        u64 idx = base + (u64)i * RDF_BLOCK + threadIdx.x;
        lds[i * RDF_BLOCK + threadIdx.x] = (idx < n) ? (TO)in[idx] : (TO)0;
    }
    TO before = 0;
    for (u32 t = threadIdx.x; t < blockIdx.x; t += RDF_BLOCK) before += tile_sums[t];
    TO prior;
    block_exclusive_scan<TO>(before, lds_wave, &prior);  // (the block's sum of the earlier tiles' totals)
    TO v[SCAN_ITEMS];
    TO local = 0;
#pragma unroll
    for (int i = 0; i < SCAN_ITEMS; ++i) {
        v[i] = lds[threadIdx.x * SCAN_ITEMS + i];
        local += v[i];
    }
    TO total;
    TO off = block_exclusive_scan<TO>(local, lds_wave, &total) + prior;
#pragma unroll
    for (int i = 0; i < SCAN_ITEMS; ++i) {
        lds[threadIdx.x * SCAN_ITEMS + i] = off;
        off += v[i];
    }
    if (grand_total && blockIdx.x == gridDim.x - 1 && threadIdx.x == 0) *grand_total = prior + total;
    __syncthreads();
#pragma unroll
    for (int i = 0; i < SCAN_ITEMS; ++i) {
        u64 idx = base + (u64)i * RDF_BLOCK + threadIdx.x;
        if (idx < n) out[idx] = lds[i * RDF_BLOCK + threadIdx.x];
    }
}

// small inputs (a few tiles): one block scans in -> out with a running carry (one launch instead of three)
template <typename TI, typename TO>
__global__ __launch_bounds__(RDF_BLOCK) void k_scan_small(const TI* in, TO* out, u64 n,
                                                          TO* __restrict__ grand_total) {
    __shared__ TO lds_wave[RDF_WAVES_PER_BLOCK];
    TO carry = 0;
    for (u64 base = 0; base < n; base += SCAN_TILE) {
        TO v[SCAN_ITEMS];
        TO local = 0;
        const u64 tb = base + (u64)threadIdx.x * SCAN_ITEMS;
#pragma unroll
        for (int i = 0; i < SCAN_ITEMS; ++i) {
            v[i] = (tb + i < n) ? (TO)in[tb + i] : (TO)0;
            local += v[i];
        }
        TO total;
        TO off = block_exclusive_scan<TO>(local, lds_wave, &total) + carry;
#pragma unroll
        for (int i = 0; i < SCAN_ITEMS; ++i) {
            if (tb + i < n) out[tb + i] = off;
            off += v[i];
        }
        carry += total;
    }
    if (threadIdx.x == 0 && grand_total) *grand_total = carry;
}

// u32 inputs, 16-B aligned in and out: each lane scans 16 consecutive items it loads and stores as 16-B vectors, so the
// tile needs no LDS transposition (the strided LDS reads of k_scan_apply conflict) and a wave's accesses are 4x fewer
#ifndef RDF_SCAN_VEC
#define RDF_SCAN_VEC 1
#endif
__device__ inline void scan_load16(const u32* __restrict__ in, u64 n, u64 tb, u32 (&v)[SCAN_ITEMS]) {
#pragma unroll
    for (int i = 0; i < SCAN_ITEMS; i += 4) {
        if (tb + i + 4 <= n) {
            const u32x4_t x = *(const u32x4_t*)(in + tb + i);
            v[i] = x.x;
            v[i + 1] = x.y;
            v[i + 2] = x.z;
            v[i + 3] = x.w;
        } else {
#pragma unroll
            for (int j = 0; j < 4; ++j) v[i + j] = tb + i + j < n ? in[tb + i + j] : 0u;
        }
    }
}
// out[tb + i] = off + (v[0] + .. + v[i-1])
__device__ inline void scan_store16(u32* __restrict__ out, u64 n, u64 tb, const u32 (&v)[SCAN_ITEMS], u32 off) {
#pragma unroll
    for (int i = 0; i < SCAN_ITEMS; i += 4) {
        u32x4_t x;
        x.x = off;
        x.y = x.x + v[i];
        x.z = x.y + v[i + 1];
        x.w = x.z + v[i + 2];
        off = x.w + v[i + 3];
        if (tb + i + 4 <= n) {
            *(u32x4_t*)(out + tb + i) = x;
        } else {
            if (tb + i < n) out[tb + i] = x.x;
            if (tb + i + 1 < n) out[tb + i + 1] = x.y;
            if (tb + i + 2 < n) out[tb + i + 2] = x.z;
        }
    }
}
__device__ inline void scan_store16(u64* __restrict__ out, u64 n, u64 tb, const u32 (&v)[SCAN_ITEMS], u64 off) {
#pragma unroll
    for (int i = 0; i < SCAN_ITEMS; i += 2) {
        u64x2_t x;
        x.x = off;
        x.y = off + v[i];
        off = x.y + v[i + 1];
        if (tb + i + 2 <= n) *(u64x2_t*)(out + tb + i) = x;
        else if (tb + i < n) out[tb + i] = x.x;
    }
}

template <typename TO>
__global__ __launch_bounds__(RDF_BLOCK) void k_scan_reduce_v(const u32* __restrict__ in, u64 n, TO* __restrict__ tile_sums) {
    __shared__ TO lds_wave[RDF_WAVES_PER_BLOCK];
    u32 v[SCAN_ITEMS];
    scan_load16(in, n, (u64)blockIdx.x * SCAN_TILE + (u64)threadIdx.x * SCAN_ITEMS, v);
    TO acc = 0;
#pragma unroll
    for (int i = 0; i < SCAN_ITEMS; ++i) acc += v[i];
    TO total;
    block_exclusive_scan<TO>(acc, lds_wave, &total);
    if (threadIdx.x == 0) tile_sums[blockIdx.x] = total;
}

// FOLD: tile_sums are the tiles' totals (each block adds the ones before it; the last writes the grand total);
// otherwise they are the tiles' offsets
template <typename TO, bool FOLD>
__global__ __launch_bounds__(RDF_BLOCK) void k_scan_apply_v(const u32* in, TO* out, u64 n, const TO* __restrict__ tile_sums,
                                                            TO* __restrict__ grand_total) {
    __shared__ TO lds_wave[RDF_WAVES_PER_BLOCK];
    const u64 tb = (u64)blockIdx.x * SCAN_TILE + (u64)threadIdx.x * SCAN_ITEMS;
    u32 v[SCAN_ITEMS];
    scan_load16(in, n, tb, v);
    TO prior;
    if (FOLD) {
        TO before = 0;
        for (u32 t = threadIdx.x; t < blockIdx.x; t += RDF_BLOCK) before += tile_sums[t];
        block_exclusive_scan<TO>(before, lds_wave, &prior);
    } else {
        prior = tile_sums[blockIdx.x];
    }
    TO local = 0;
#pragma unroll
    for (int i = 0; i < SCAN_ITEMS; ++i) local += v[i];
    TO total;
    const TO off = block_exclusive_scan<TO>(local, lds_wave, &total) + prior;
    if (FOLD && grand_total && blockIdx.x == gridDim.x - 1 && threadIdx.x == 0) *grand_total = prior + total;
    scan_store16(out, n, tb, v, off);
}

static constexpr u64 SCAN_SMALL_TILES = 4;  // one 1024-thread block up to 8 or 32 tiles measured no faster (c1 groups 0.23 -> 0.39 ms at 32;
                                           // profiles/r05_scan_small_ab.log)

template <typename TI, typename TO>
static hipError_t exclusive_scan_impl(Workspace& ws, const TI* in, TO* out, u64 n, TO* d_total, hipStream_t st) {
    if (n == 0) {
        if (d_total) return hipMemsetAsync(d_total, 0, sizeof(TO), st);
        return hipSuccess;
    }
    u64 tiles = (n + SCAN_TILE - 1) / SCAN_TILE;
    if (tiles <= SCAN_SMALL_TILES) {
        hipLaunchKernelGGL((k_scan_small<TI, TO>), dim3(1), dim3(RDF_BLOCK), 0, st, in, out, n, d_total);
        return hipGetLastError();
    }
    TO* sums = (TO*)ws.scratch(tiles * sizeof(TO), 0);
    if (!sums) return hipErrorOutOfMemory;
    if constexpr (std::is_same<TI, u32>::value) {
        if (RDF_SCAN_VEC && (((uintptr_t)in | (uintptr_t)out) & 15) == 0) {
            hipLaunchKernelGGL((k_scan_reduce_v<TO>), dim3((unsigned)tiles), dim3(RDF_BLOCK), 0, st, in, n, sums);
            if (tiles <= SCAN_FOLD_TILES) {
                hipLaunchKernelGGL((k_scan_apply_v<TO, true>), dim3((unsigned)tiles), dim3(RDF_BLOCK), 0, st, in, out, n, sums,
                                   d_total);
                return hipGetLastError();
            }
            hipLaunchKernelGGL((k_scan_single<TO>), dim3(1), dim3(RDF_BLOCK), 0, st, sums, tiles, d_total);
            hipLaunchKernelGGL((k_scan_apply_v<TO, false>), dim3((unsigned)tiles), dim3(RDF_BLOCK), 0, st, in, out, n, sums,
                               (TO*)nullptr);
            return hipGetLastError();
        }
    }
    hipLaunchKernelGGL((k_scan_reduce<TI, TO>), dim3((unsigned)tiles), dim3(RDF_BLOCK), 0, st, in, n, sums);
    if (tiles <= SCAN_FOLD_TILES) {
        hipLaunchKernelGGL((k_scan_apply_fold<TI, TO>), dim3((unsigned)tiles), dim3(RDF_BLOCK), 0, st, in, out, n, sums,
                           d_total);
        return hipGetLastError();
    }
    hipLaunchKernelGGL((k_scan_single<TO>), dim3(1), dim3(RDF_BLOCK), 0, st, sums, tiles, d_total);
    hipLaunchKernelGGL((k_scan_apply<TI, TO>), dim3((unsigned)tiles), dim3(RDF_BLOCK), 0, st, in, out, n, sums);
    return hipGetLastError();
}

// k scans of equal length in one pass (blockIdx.y = the array): d_chunks' four per-dependent counts on c2 took eight
// launches, now two
struct ScanBatch {
    const u32* in[SCAN_BATCH_MAX];
    u64* out[SCAN_BATCH_MAX];
};
template <bool VEC>
__global__ __launch_bounds__(RDF_BLOCK) void k_scan_reduce_batch(ScanBatch b, u64 n, u64* __restrict__ tile_sums) {
    __shared__ u64 lds_wave[RDF_WAVES_PER_BLOCK];
    const u32* in = b.in[blockIdx.y];
    const u64 base = (u64)blockIdx.x * SCAN_TILE;
    u64 acc = 0;
    if (VEC) {
        u32 v[SCAN_ITEMS];
        scan_load16(in, n, base + (u64)threadIdx.x * SCAN_ITEMS, v);
#pragma unroll
        for (int i = 0; i < SCAN_ITEMS; ++i) acc += v[i];
    } else {
#pragma unroll
        for (int i = 0; i < SCAN_ITEMS; ++i) {
            u64 idx = base + (u64)i * RDF_BLOCK + threadIdx.x;
            if (idx < n) acc += in[idx];
        }
    }
    u64 total;
    block_exclusive_scan<u64>(acc, lds_wave, &total);
    if (threadIdx.x == 0) tile_sums[(u64)blockIdx.y * gridDim.x + blockIdx.x] = total;
}
template <bool VEC>
__global__ __launch_bounds__(RDF_BLOCK) void k_scan_apply_fold_batch(ScanBatch b, u64 n, const u64* __restrict__ tile_sums) {
    __shared__ u64 lds[VEC ? 1 : SCAN_TILE];
    __shared__ u64 lds_wave[RDF_WAVES_PER_BLOCK];
    const u32* in = b.in[blockIdx.y];
    u64* out = b.out[blockIdx.y];
    const u64* sums = tile_sums + (u64)blockIdx.y * gridDim.x;
    const u64 base = (u64)blockIdx.x * SCAN_TILE;
    const u64 tb = base + (u64)threadIdx.x * SCAN_ITEMS;
    u32 vv[SCAN_ITEMS];
    if (VEC) {
        scan_load16(in, n, tb, vv);
    } else {
#pragma unroll
        for (int i = 0; i < SCAN_ITEMS; ++i) {
            u64 idx = base + (u64)i * RDF_BLOCK + threadIdx.x;
            lds[i * RDF_BLOCK + threadIdx.x] = idx < n ? (u64)in[idx] : 0ull;
        }
    }
    u64 before = 0;
    for (u32 t = threadIdx.x; t < blockIdx.x; t += RDF_BLOCK) before += sums[t];
    u64 prior;
    block_exclusive_scan<u64>(before, lds_wave, &prior);  // (its barriers also order the LDS tile's stores)
    u64 v[SCAN_ITEMS];
    u64 local = 0;
#pragma unroll
    for (int i = 0; i < SCAN_ITEMS; ++i) {
        v[i] = VEC ? (u64)vv[i] : lds[threadIdx.x * SCAN_ITEMS + i];
        local += v[i];
    }
    u64 total;
    u64 off = block_exclusive_scan<u64>(local, lds_wave, &total) + prior;
    if (blockIdx.x == gridDim.x - 1 && threadIdx.x == 0) out[n] = prior + total;
    if (VEC) {
        scan_store16(out, n, tb, vv, off);
        return;
    }
#pragma unroll
    for (int i = 0; i < SCAN_ITEMS; ++i) {
        lds[threadIdx.x * SCAN_ITEMS + i] = off;
        off += v[i];
    }
    __syncthreads();
#pragma unroll
    for (int i = 0; i < SCAN_ITEMS; ++i) {
        u64 idx = base + (u64)i * RDF_BLOCK + threadIdx.x;
        if (idx < n) out[idx] = lds[i * RDF_BLOCK + threadIdx.x];
    }
}

hipError_t exclusive_scan_u32_u64_batch(Workspace& ws, const u32* const* in, u64* const* out, int k, u64 n,
                                        hipStream_t st) {
    const u64 tiles = (n + SCAN_TILE - 1) / SCAN_TILE;
    if (k < 1 || k > SCAN_BATCH_MAX) return hipErrorInvalidValue;
    if (n == 0 || tiles <= SCAN_SMALL_TILES || tiles > SCAN_FOLD_TILES) {  // (one launch each already, or large)
        for (int j = 0; j < k; ++j) {
            hipError_t e = exclusive_scan_u32_u64(ws, in[j], out[j], n, out[j] + n, st);
            if (e != hipSuccess) return e;
        }
        return hipSuccess;
    }
    ScanBatch b = {};
    for (int j = 0; j < k; ++j) {
        b.in[j] = in[j];
        b.out[j] = out[j];
    }
    u64* sums = (u64*)ws.scratch(tiles * k * sizeof(u64), 0);
    if (!sums) return hipErrorOutOfMemory;
    uintptr_t align = 0;
    for (int j = 0; j < k; ++j) align |= (uintptr_t)in[j] | (uintptr_t)out[j];
    if (RDF_SCAN_VEC && (align & 15) == 0) {
        hipLaunchKernelGGL(k_scan_reduce_batch<true>, dim3((unsigned)tiles, (unsigned)k), dim3(RDF_BLOCK), 0, st, b, n, sums);
        hipLaunchKernelGGL(k_scan_apply_fold_batch<true>, dim3((unsigned)tiles, (unsigned)k), dim3(RDF_BLOCK), 0, st, b, n, sums);
        return hipGetLastError();
    }
    hipLaunchKernelGGL(k_scan_reduce_batch<false>, dim3((unsigned)tiles, (unsigned)k), dim3(RDF_BLOCK), 0, st, b, n, sums);
    hipLaunchKernelGGL(k_scan_apply_fold_batch<false>, dim3((unsigned)tiles, (unsigned)k), dim3(RDF_BLOCK), 0, st, b, n, sums);
    return hipGetLastError();
}

hipError_t exclusive_scan_u32_u64(Workspace& ws, const u32* in, u64* out, u64 n, u64* d_total, hipStream_t st) {
    return exclusive_scan_impl<u32, u64>(ws, in, out, n, d_total, st);
}
hipError_t exclusive_scan_u64(Workspace& ws, const u64* in, u64* out, u64 n, u64* d_total, hipStream_t st) {
    return exclusive_scan_impl<u64, u64>(ws, in, out, n, d_total, st);
}
hipError_t exclusive_scan_u32(Workspace& ws, const u32* in, u32* out, u64 n, u32* d_total, hipStream_t st) {
    return exclusive_scan_impl<u32, u32>(ws, in, out, n, d_total, st);
}

// ------------------------------------------------------------------------------------------------
// LSD radix sort of u64 keys, 8-bit digits, reduce-then-scan per pass:
//   count:   per-tile digit histogram (wave ballots give each lane its same-digit peers; one leader lane
//            per digit adds the peer count -- no LDS atomics, so a skewed digit costs nothing extra)
//   scan:    device exclusive scan of the digit-major [256][tiles] histogram
//   scatter: stable in-tile ranks (peers + per-wave running counters), the tile is reordered by digit in
//            LDS, then written out as contiguous per-digit runs (coalesced stores instead of 8-byte
//            scattered ones).

#ifndef RDF_RS_ITEMS
#define RDF_RS_ITEMS 16
#endif
static constexpr int RS_ITEMS = RDF_RS_ITEMS;                    // keys per lane per tile
static constexpr int RS_TILE = RDF_BLOCK * RS_ITEMS;             // 4096 keys per tile
static constexpr int RS_WAVE_KEYS = RDF_WAVE * RS_ITEMS;         // 1024 keys per wave


// Tile of a radix block.  RDF_RS_XCD=1: consecutive tiles on one XCD (xcd_block): tile t's digit runs end where tile
// t+1's begin (a 4096-key tile averages 8 keys = 64 B per digit at 9 bits), and the (digit, tile) histogram words of
// neighbouring tiles share lines (c2 sort 1.90 -> 1.78 ms, c3 19.1 -> 17.4; profiles/r05_rs_xcd_ab.log)
#ifndef RDF_RS_XCD
#define RDF_RS_XCD 1
#endif
__device__ inline u32 rs_tile() { return RDF_RS_XCD ? xcd_block() : blockIdx.x; }

// lanes of the wave whose key is valid and has the same DB-bit digit as this lane (0 for invalid lanes)
template <int DB>
__device__ inline u64 digit_peers(u32 d, bool valid) {
    u64 peers = __ballot(valid);
#pragma unroll
    for (int b = 0; b < DB; ++b) {
        const u64 bb = __ballot((d >> b) & 1);
        peers &= ((d >> b) & 1) ? bb : ~bb;
    }
    return valid ? peers : 0ull;
}

typedef unsigned long long u64x2_t __attribute__((ext_vector_type(2)));
typedef unsigned int u32x2_t __attribute__((ext_vector_type(2)));
template <typename KT> struct KeyPair;
template <> struct KeyPair<u64> { typedef u64x2_t type; };
template <> struct KeyPair<u32> { typedef u32x2_t type; };

// 16-byte (u64 keys) or 8-byte (u32 keys, K1's partition) loads of a tile: two consecutive keys per lane and row;
// out-of-range keys read as 0
template <typename KT>
__device__ inline void load_tile_pairs(const KT* __restrict__ keys, u64 n, u64 tbase, KT (&k)[RS_ITEMS]) {
    typedef typename KeyPair<KT>::type KT2;
#pragma unroll
    for (int r = 0; r < RS_ITEMS / 2; ++r) {
        const u64 idx = tbase + 2ull * ((u64)r * RDF_BLOCK + threadIdx.x);
        if (idx + 1 < n) {
            const KT2 v = *(const KT2*)(keys + idx);
            k[2 * r] = v.x;
            k[2 * r + 1] = v.y;
        } else {
            k[2 * r] = idx < n ? keys[idx] : 0;
            k[2 * r + 1] = 0;
        }
    }
}

// Digits of DB bits (the pass's width w <= DB is masked at run time: DB only sizes the LDS counters)
// drop: keys equal to ~0 (padding) are left out of the histogram and of the scattered output (first pass of a sort
// whose input carries padding; the output then holds only the other keys)
// HASH: the digits are those of mix64(key & hmask) (a hash partition: K2's records grouped by the top bits of their
// key hash, radix_partition_hashed); the keys themselves are moved unchanged
template <bool HASH>
__device__ inline u32 radix_digit(u64 k, int shift, u32 dmask, u64 hmask) {
    return (u32)((HASH ? mix64(k & hmask) : k) >> shift) & dmask;
}
template <int DB, bool HASH = false, typename KT = u64>
__global__ __launch_bounds__(RDF_BLOCK) void k_radix_count(const KT* __restrict__ keys, u64 n, int shift, int w,
                                                           u32* __restrict__ hist, u32 num_tiles, int drop, u64 hmask) {
    constexpr u32 NBIN = 1u << DB;
    __shared__ u32 wcnt[RDF_WAVES_PER_BLOCK][NBIN];
    const int lane = lane_id();
    const int wave = threadIdx.x / RDF_WAVE;
    const u32 dmask = (1u << w) - 1u;
    for (u32 i = threadIdx.x; i < RDF_WAVES_PER_BLOCK * NBIN; i += RDF_BLOCK) (&wcnt[0][0])[i] = 0;
    __syncthreads();
    const u32 tile = rs_tile();
    const u64 tbase = (u64)tile * RS_TILE;
    KT k[RS_ITEMS];
    load_tile_pairs<KT>(keys, n, tbase, k);  // counting is order-free: any assignment of keys to lanes works
#pragma unroll
    for (int r = 0; r < RS_ITEMS; ++r) {
        const u64 idx = tbase + 2ull * ((u64)(r / 2) * RDF_BLOCK + threadIdx.x) + (r & 1);
        const bool valid = idx < n && !(drop && k[r] == (KT)~0ull);
        const u32 d = radix_digit<HASH>(k[r], shift, dmask, hmask);
        const u64 peers = digit_peers<DB>(d, valid);
        if (valid && ((peers >> lane) >> 1) == 0) wcnt[wave][d] += (u32)__popcll(peers);
    }
    __syncthreads();
    for (u32 b = threadIdx.x; b <= dmask; b += RDF_BLOCK) {
        u32 sum = 0;
#pragma unroll
        for (int ww = 0; ww < RDF_WAVES_PER_BLOCK; ++ww) sum += wcnt[ww][b];
        hist[(u64)b * num_tiles + tile] = sum;
    }
}

template <int DB, bool HASH = false, typename KT = u64>
__global__ __launch_bounds__(RDF_BLOCK) void k_radix_scatter(const KT* __restrict__ keys, KT* __restrict__ out, u64 n,
                                                             int shift, int w, const u32* __restrict__ offs,
                                                             const u32* __restrict__ rowtot, u32 num_tiles, int drop,
                                                             u64 hmask, u32* d_kept) {
    constexpr u32 NBIN = 1u << DB;
    constexpr u32 PER = NBIN / RDF_BLOCK;  // digits per thread in the tile scan (1, 2 or 4)
    static_assert(NBIN % RDF_BLOCK == 0, "digit bins must be a multiple of the block");
    __shared__ __align__(16) KT skeys[RS_TILE];
    __shared__ u32 wcount[RDF_WAVES_PER_BLOCK][NBIN];
    __shared__ u32 tstart[NBIN];
    __shared__ u32 gbase[NBIN];
    __shared__ u32 lds_wave[RDF_WAVES_PER_BLOCK];
    __shared__ u32 s_tvalid;
    const int lane = lane_id();
    const int wave = threadIdx.x / RDF_WAVE;
    const u32 nbin = 1u << w, dmask = nbin - 1u;
    for (u32 i = threadIdx.x; i < RDF_WAVES_PER_BLOCK * NBIN; i += RDF_BLOCK) (&wcount[0][0])[i] = 0;
    const u32 tile = rs_tile();
    const u64 tbase = (u64)tile * RS_TILE;
    const u64 tn = n - tbase < (u64)RS_TILE ? n - tbase : (u64)RS_TILE;
    {   // stage the tile through LDS: 16-byte global loads, then each wave reads its contiguous sub-range; while they
        // are in flight, the digits' bases (exclusive scan of the row totals, PER digits a thread) + the row prefixes
        KT kin[RS_ITEMS];
        load_tile_pairs<KT>(keys, n, tbase, kin);
        u32 rt[PER], ro[PER], local = 0;
#pragma unroll
        for (u32 q = 0; q < PER; ++q) {
            const u32 dg = threadIdx.x * PER + q;
            rt[q] = dg < nbin ? rowtot[dg] : 0u;
            ro[q] = dg < nbin ? offs[(u64)dg * num_tiles + tile] : 0u;
            local += rt[q];
        }
        u32 total;
        u32 off = block_exclusive_scan<u32>(local, lds_wave, &total);
#pragma unroll
        for (u32 q = 0; q < PER; ++q) {
            gbase[threadIdx.x * PER + q] = off + ro[q];
            off += rt[q];
        }
        if (d_kept && tile == 0 && threadIdx.x == 0) *d_kept = total;
#pragma unroll
        for (int r = 0; r < RS_ITEMS / 2; ++r) {
            const u32 p = 2u * ((u32)r * RDF_BLOCK + threadIdx.x);
            *(typename KeyPair<KT>::type*)(skeys + p) = typename KeyPair<KT>::type{kin[2 * r], kin[2 * r + 1]};
        }
    }
    __syncthreads();
    KT k[RS_ITEMS];
    u32 rank[RS_ITEMS];
    const u64 lt = lanemask_lt();
    const u32 wofs = (u32)wave * RS_WAVE_KEYS;
#pragma unroll
    for (int r = 0; r < RS_ITEMS; ++r) k[r] = skeys[wofs + (u32)r * RDF_WAVE + lane];
#pragma unroll
    for (int r = 0; r < RS_ITEMS; ++r) {
        const bool valid = wofs + (u32)r * RDF_WAVE + lane < tn && !(drop && k[r] == (KT)~0ull);
        const u32 d = radix_digit<HASH>(k[r], shift, dmask, hmask);
        const u64 peers = digit_peers<DB>(d, valid);
        const u32 before = (u32)__popcll(peers & lt);
        const u32 old = valid ? wcount[wave][d] : 0;
        // the highest peer lane publishes the new running count (reads above precede this write)
        if (valid && ((peers >> lane) >> 1) == 0) wcount[wave][d] = old + before + 1;
        rank[r] = old + before;
    }
    __syncthreads();
    {   // exclusive prefix over waves per digit, then over digits for the tile (PER consecutive digits a thread)
        u32 run[PER], local = 0;
#pragma unroll
        for (u32 q = 0; q < PER; ++q) {
            const u32 dg = threadIdx.x * PER + q;
            u32 acc = 0;
#pragma unroll
            for (int ww = 0; ww < RDF_WAVES_PER_BLOCK; ++ww) {
                const u32 c = wcount[ww][dg];
                wcount[ww][dg] = acc;
                acc += c;
            }
            run[q] = acc;
            local += acc;
        }
        u32 total;
        u32 off = block_exclusive_scan<u32>(local, lds_wave, &total);
#pragma unroll
        for (u32 q = 0; q < PER; ++q) {
            tstart[threadIdx.x * PER + q] = off;
            off += run[q];
        }
        if (threadIdx.x == 0) s_tvalid = total;  // the tile's kept keys (all of them unless padding is dropped)
    }
    __syncthreads();
#pragma unroll
    for (int r = 0; r < RS_ITEMS; ++r) {
        if (wofs + (u32)r * RDF_WAVE + lane < tn && !(drop && k[r] == (KT)~0ull)) {
            const u32 d = radix_digit<HASH>(k[r], shift, dmask, hmask);
            skeys[tstart[d] + wcount[wave][d] + rank[r]] = k[r];
        }
    }
    __syncthreads();
    const u32 tv = s_tvalid;
#pragma unroll
    for (int i = 0; i < RS_ITEMS; ++i) {
        const u32 p = (u32)i * RDF_BLOCK + threadIdx.x;
        if (p < tv) {
            const KT key = skeys[p];
            const u32 d = radix_digit<HASH>(key, shift, dmask, hmask);
            out[(u64)gbase[d] + (p - tstart[d])] = key;
        }
    }
}

// The digit-major histogram's rows scanned in place, one 1024-thread block per digit (exclusive within the row: the
// digit's keys in earlier tiles; c2's rows of 14.4k tiles in one step), each row's total to rowtot[digit].  The scatter
// blocks scan the totals into the digits' bases themselves (a few hundred L2 loads, issued behind the tile's key
// loads), so a pass is three launches instead of the five of a device-wide scan (c2: 21 passes per step spent ~35 us
// each in reduce / single / apply)
static constexpr int RS_SCAN_THREADS = 1024;
static constexpr int RS_SCAN_ITEMS = 16;
__global__ __launch_bounds__(RS_SCAN_THREADS) void k_radix_rowscan(u32* __restrict__ hist, u32 row_stride, u32 num_tiles,
                                                                   u32* rowtot) {
    constexpr int NW = RS_SCAN_THREADS / RDF_WAVE;
    constexpr u32 STEP = RS_SCAN_THREADS * RS_SCAN_ITEMS;
    __shared__ u32 lds_wave[NW];
    const int lane = lane_id(), wave = threadIdx.x / RDF_WAVE;
    u32* row = hist + (u64)blockIdx.x * row_stride;  // (rows 16-B aligned: the stride is a multiple of 4)
    u32 carry = 0;
    for (u32 b0 = 0; b0 < num_tiles; b0 += STEP) {
        u32 v[RS_SCAN_ITEMS];
        u32 local = 0;
        const u32 tb = b0 + threadIdx.x * RS_SCAN_ITEMS;
#pragma unroll
        for (int i = 0; i < RS_SCAN_ITEMS; i += 4) {
            u32x4_t x = tb + i < row_stride ? *(const u32x4_t*)(row + tb + i) : u32x4_t{0u, 0u, 0u, 0u};
            v[i] = tb + i < num_tiles ? x.x : 0u;  // (the padding past num_tiles reads as 0)
            v[i + 1] = tb + i + 1 < num_tiles ? x.y : 0u;
            v[i + 2] = tb + i + 2 < num_tiles ? x.z : 0u;
            v[i + 3] = tb + i + 3 < num_tiles ? x.w : 0u;
        }
#pragma unroll
        for (int i = 0; i < RS_SCAN_ITEMS; ++i) local += v[i];
        u32 incl = local;
#pragma unroll
        for (int off = 1; off < RDF_WAVE; off <<= 1) {
            const u32 t = __shfl_up(incl, off, RDF_WAVE);
            if (lane >= off) incl += t;
        }
        if (lane == RDF_WAVE - 1) lds_wave[wave] = incl;
        __syncthreads();
        u32 woff = 0, total = 0;
#pragma unroll
        for (int w = 0; w < NW; ++w) {
            const u32 x = lds_wave[w];
            woff += w < wave ? x : 0u;
            total += x;
        }
        __syncthreads();
        u32 off = carry + woff + incl - local;
#pragma unroll
        for (int i = 0; i < RS_SCAN_ITEMS; i += 4) {
            u32x4_t x;
            x.x = off;
            x.y = off + v[i];
            x.z = x.y + v[i + 1];
            x.w = x.z + v[i + 2];
            off = x.w + v[i + 3];
            if (tb + i < row_stride) *(u32x4_t*)(row + tb + i) = x;
        }
        carry += total;
    }
    if (threadIdx.x == 0) rowtot[blockIdx.x] = carry;
}

static inline u32 hist_stride(u32 tiles) { return (tiles + 3u) & ~3u; }
template <int DB, bool HASH = false, typename KT = u64>
static hipError_t radix_pass(Workspace& ws, const KT* keys, KT* tmp, u64 n, int shift, int w, u32* hist, u32 tiles,
                             hipStream_t st, u32* d_kept = nullptr, u64 hmask = 0) {
    const int drop = d_kept ? 1 : 0;
    u32* rowtot = (u32*)ws.scratch(1024 * sizeof(u32), 2);
    if (!rowtot) return hipErrorOutOfMemory;
    const u32 rs = hist_stride(tiles);  // the histogram's digit rows, 16-B aligned
    hipLaunchKernelGGL((k_radix_count<DB, HASH, KT>), dim3(tiles), dim3(RDF_BLOCK), 0, st, keys, n, shift, w, hist, rs, drop,
                       hmask);
    hipLaunchKernelGGL(k_radix_rowscan, dim3(1u << w), dim3(RS_SCAN_THREADS), 0, st, hist, rs, tiles, rowtot);
    hipLaunchKernelGGL((k_radix_scatter<DB, HASH, KT>), dim3(tiles), dim3(RDF_BLOCK), 0, st, keys, tmp, n, shift, w, hist, rowtot,
                       rs, drop, hmask, d_kept);
    return hipGetLastError();
}

// Widest digit of a sort: RS_MAX_BITS (9).  10-bit digits saving a pass measured slower (c4 at 10^9 triples sorts its
// 50-bit records in 5 passes of 10 bits in 362 ms against 234 ms for 6 passes of <= 9 bits, c3 21.8 vs 19.0 ms: 1,024
// bins leave ~4 keys per bin of a 4096-key tile; profiles/r05_sort10_ab.log)
static hipError_t radix_sort_dmax(Workspace& ws, u64*& keys, u64*& tmp, u64 n, int lo, int hi, int dmax, hipStream_t st);
static int sort_digit_bits(int) { return RS_MAX_BITS; }

int radix_sort_passes(int bits) {
    const int d = sort_digit_bits(bits);
    return bits > 0 ? (bits + d - 1) / d : 0;
}

// Sort of keys some of which are padding (~0): the first pass drops them, *n_out (host) = the other keys, which the
// remaining passes sort.  One host read-back between the first and the second pass.
hipError_t radix_sort_u64_drop(Workspace& ws, u64*& keys, u64*& tmp, u64 n, int bits, u32* d_kept, u64* n_out,
                               hipStream_t st) {
    *n_out = 0;
    if (n == 0 || bits <= 0) return hipSuccess;
    if (n >= (1ull << 32)) return hipErrorInvalidValue;
    const int dmax = sort_digit_bits(bits);
    const int passes = (bits + dmax - 1) / dmax;
    const int w0 = bits / passes + (0 < bits % passes ? 1 : 0);
    const u32 tiles = (u32)((n + RS_TILE - 1) / RS_TILE);
    u32* hist = (u32*)ws.scratch(((u64)hist_stride(tiles) << dmax) * sizeof(u32), 1);
    if (!hist) return hipErrorOutOfMemory;
    hipError_t e = w0 <= 8 ? radix_pass<8>(ws, keys, tmp, n, 0, w0, hist, tiles, st, d_kept)
                 : w0 == 9 ? radix_pass<9>(ws, keys, tmp, n, 0, w0, hist, tiles, st, d_kept)
                           : radix_pass<10>(ws, keys, tmp, n, 0, w0, hist, tiles, st, d_kept);
    if (e != hipSuccess) return e;
    u32 kept = 0;
    e = hipMemcpyAsync(&kept, d_kept, 4, hipMemcpyDeviceToHost, st);
    if (e == hipSuccess) e = hipStreamSynchronize(st);
    if (e != hipSuccess) return e;
    std::swap(keys, tmp);
    *n_out = kept;
    return radix_sort_dmax(ws, keys, tmp, kept, w0, bits, dmax, st);
}

// Passes of at most RS_MAX_BITS bits (10 when that saves a pass), as even as possible (43 bits: 9+9+9+8+8 instead of
// six 8-bit passes)
hipError_t radix_sort_u64_bits(Workspace& ws, u64*& keys, u64*& tmp, u64 n, int lo, int hi, hipStream_t st) {
    return radix_sort_dmax(ws, keys, tmp, n, lo, hi, sort_digit_bits(hi - lo), st);
}

static hipError_t radix_sort_dmax(Workspace& ws, u64*& keys, u64*& tmp, u64 n, int lo, int hi, int dmax, hipStream_t st) {
    if (n < 2 || hi <= lo) return hipSuccess;
    if (n >= (1ull << 32)) return hipErrorInvalidValue;
    const u32 tiles = (u32)((n + RS_TILE - 1) / RS_TILE);
    const int bits = hi - lo;
    const int passes = (bits + dmax - 1) / dmax;
    u32* hist = (u32*)ws.scratch(((u64)hist_stride(tiles) << dmax) * sizeof(u32), 1);
    if (!hist) return hipErrorOutOfMemory;
    int shift = lo;
    for (int p = 0; p < passes; ++p) {
        const int w = bits / passes + (p < bits % passes ? 1 : 0);  // the wider digits first
        hipError_t e = w <= 8 ? radix_pass<8>(ws, keys, tmp, n, shift, w, hist, tiles, st)
                     : w == 9 ? radix_pass<9>(ws, keys, tmp, n, shift, w, hist, tiles, st)
                              : radix_pass<10>(ws, keys, tmp, n, shift, w, hist, tiles, st);
        if (e != hipSuccess) return e;
        u64* t = keys;
        keys = tmp;
        tmp = t;
        shift += w;
    }
    return hipGetLastError();
}

hipError_t radix_sort_u64(Workspace& ws, u64*& keys, u64*& tmp, u64 n, int bits, hipStream_t st) {
    return radix_sort_u64_bits(ws, keys, tmp, n, 0, bits, st);
}

// Keys grouped by bits [64 - bits, 64) of mix64(key & hmask), ascending (LSD passes of <= 9 bits over those hash bits;
// within a group the order is the passes' stable order).  keys / tmp swap like radix_sort_u64_bits.
hipError_t radix_partition_hashed(Workspace& ws, u64*& keys, u64*& tmp, u64 n, int bits, u64 hmask, hipStream_t st) {
    if (n < 2 || bits <= 0) return hipSuccess;
    if (n >= (1ull << 32) || bits > 30) return hipErrorInvalidValue;
    const u32 tiles = (u32)((n + RS_TILE - 1) / RS_TILE);
    // digits of <= 9 bits (c4 at 10^9 triples: 20 bits in 3 passes 89.6 ms of K2, in 2 passes of 10 bits 96.0 ms: a
    // 1,024-bin digit leaves ~4 keys per bin of a tile; RDFIND_PART_DIGIT overrides, 8..10)
    static const int pdig = getenv("RDFIND_PART_DIGIT") ? std::max(8, std::min(10, atoi(getenv("RDFIND_PART_DIGIT")))) : 9;
    const int passes = (bits + pdig - 1) / pdig;
    u32* hist = (u32*)ws.scratch(((u64)hist_stride(tiles) << 10) * sizeof(u32), 1);
    if (!hist) return hipErrorOutOfMemory;
    int shift = 64 - bits;
    for (int p = 0; p < passes; ++p) {
        const int w = bits / passes + (p < bits % passes ? 1 : 0);
        hipError_t e = w <= 8 ? radix_pass<8, true>(ws, keys, tmp, n, shift, w, hist, tiles, st, nullptr, hmask)
                     : w == 9 ? radix_pass<9, true>(ws, keys, tmp, n, shift, w, hist, tiles, st, nullptr, hmask)
                              : radix_pass<10, true>(ws, keys, tmp, n, shift, w, hist, tiles, st, nullptr, hmask);
        if (e != hipSuccess) return e;
        std::swap(keys, tmp);
        shift += w;
    }
    return hipGetLastError();
}

// u32 keys ordered by bits [lo, hi) (LSD passes of <= 8 bits, stable; bits below lo keep the input's order): K1's
// records of large inputs grouped by their 2^14 / 2^15-key bucket (fc_unary_radix).  keys / tmp swap like
// radix_sort_u64_bits.
hipError_t radix_partition_u32(Workspace& ws, u32*& keys, u32*& tmp, u64 n, int lo, int hi, hipStream_t st) {
    if (n < 2 || hi <= lo) return hipSuccess;
    if (n >= (1ull << 32) || hi > 32) return hipErrorInvalidValue;
    const u32 tiles = (u32)((n + RS_TILE - 1) / RS_TILE);
    const int bits = hi - lo, passes = (bits + 7) / 8;
    u32* hist = (u32*)ws.scratch(((u64)hist_stride(tiles) << 8) * sizeof(u32), 1);
    if (!hist) return hipErrorOutOfMemory;
    int shift = lo;
    for (int p = 0; p < passes; ++p) {
        const int w = bits / passes + (p < bits % passes ? 1 : 0);
        hipError_t e = radix_pass<8, false, u32>(ws, keys, tmp, n, shift, w, hist, tiles, st);
        if (e != hipSuccess) return e;
        std::swap(keys, tmp);
        shift += w;
    }
    return hipGetLastError();
}

}  // namespace rdf
