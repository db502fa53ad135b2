// Device memory + primitive declarations.
#pragma once
#include "common.hpp"

namespace rdf {

// Grow-only device buffer.  Re-allocation only happens when a call needs more than before, so a
// steady-state pipeline (the bench's repeated steps) allocates nothing.
struct DevBuf {
    void* p = nullptr;
    size_t cap = 0;
    hipError_t ensure(size_t bytes) {
        if (bytes <= cap && p) return hipSuccess;
        if (p) {
            hipError_t e = hipFree(p);
            if (e != hipSuccess) return e;
            p = nullptr;
            cap = 0;
        }
        size_t want = bytes < 256 ? 256 : bytes;
        hipError_t e = hipMalloc(&p, want);
        if (e != hipSuccess) {
            p = nullptr;
            (void)hipGetLastError();  // the failure is returned here; later hipGetLastError checks must not see it again
            return e;
        }
        cap = want;
        return hipSuccess;
    }
    void release() {
        if (p) (void)hipFree(p);
        p = nullptr;
        cap = 0;
    }
    // grow to at least bytes, keeping the contents (stream-ordered copy, then the old buffer is freed)
    hipError_t grow_keep(size_t bytes, hipStream_t st) {
        if (bytes <= cap && p) return hipSuccess;
        void* q = nullptr;
        size_t want = bytes < 256 ? 256 : bytes;
        hipError_t e = hipMalloc(&q, want);
        if (e != hipSuccess) {
            (void)hipGetLastError();
            return e;
        }
        if (p && cap) {
            e = hipMemcpyAsync(q, p, cap, hipMemcpyDeviceToDevice, st);
            if (e == hipSuccess) e = hipStreamSynchronize(st);
            if (e != hipSuccess) {
                (void)hipFree(q);
                return e;
            }
            (void)hipFree(p);
        }
        p = q;
        cap = want;
        return hipSuccess;
    }
    template <typename T>
    T* as() const { return (T*)p; }
};

struct Workspace {
    static constexpr int kSlots = 8;
    DevBuf slot[kSlots];
    void* scratch(size_t bytes, int s) {
        if (s < 0 || s >= kSlots) return nullptr;
        if (slot[s].ensure(bytes) != hipSuccess) return nullptr;
        return slot[s].p;
    }
    void release() {
        for (auto& b : slot) b.release();
    }
    size_t bytes() const {
        size_t t = 0;
        for (const auto& b : slot) t += b.cap;
        return t;
    }
};

// out[i] = sum_{j<i} in[j]; *d_total (device, optional) = sum of all.  In-place allowed.
hipError_t exclusive_scan_u32_u64(Workspace& ws, const u32* in, u64* out, u64 n, u64* d_total, hipStream_t st);
// k <= SCAN_BATCH_MAX scans of n elements each in one pass; out[j][n] = the total of in[j]
static constexpr int SCAN_BATCH_MAX = 4;
hipError_t exclusive_scan_u32_u64_batch(Workspace& ws, const u32* const* in, u64* const* out, int k, u64 n,
                                        hipStream_t st);
hipError_t exclusive_scan_u64(Workspace& ws, const u64* in, u64* out, u64 n, u64* d_total, hipStream_t st);
hipError_t exclusive_scan_u32(Workspace& ws, const u32* in, u32* out, u64 n, u32* d_total, hipStream_t st);

// LSD radix sort on the low `bits` bits; keys/tmp are swapped so that `keys` holds the result.
// Uses workspace slots 0 and 1.  Requires n < 2^32.
hipError_t radix_sort_u64(Workspace& ws, u64*& keys, u64*& tmp, u64 n, int bits, hipStream_t st);
// Stable sort on bits [lo, hi) only (8 bits per pass from lo; bits at or above the last pass's top must be
// zero or already ordered).  Keys that arrive ordered by their low bits stay so within equal [lo, hi).
#ifndef RDF_RS_MAX_BITS
#define RDF_RS_MAX_BITS 9
#endif
static constexpr int RS_MAX_BITS = RDF_RS_MAX_BITS;  // widest radix digit (8: the old 8-bit passes)
static_assert(RS_MAX_BITS >= 8 && RS_MAX_BITS <= 10, "digit kernels exist for 8, 9 and 10 bits");
hipError_t radix_sort_u64_drop(Workspace& ws, u64*& keys, u64*& tmp, u64 n, int bits, u32* d_kept, u64* n_out,
                               hipStream_t st);
hipError_t radix_sort_u64_bits(Workspace& ws, u64*& keys, u64*& tmp, u64 n, int lo, int hi, hipStream_t st);
int radix_sort_passes(int bits);  // passes of a sort of `bits` key bits
hipError_t radix_partition_hashed(Workspace& ws, u64*& keys, u64*& tmp, u64 n, int bits, u64 hmask, hipStream_t st);
// u32 keys ordered by bits [lo, hi) (stable LSD passes of <= 8 bits); keys / tmp swap so that `keys` holds the result
hipError_t radix_partition_u32(Workspace& ws, u32*& keys, u32*& tmp, u64 n, int lo, int hi, hipStream_t st);

}  // namespace rdf
