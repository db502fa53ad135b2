// Dev micro-benchmark: the library's LSD radix sort (primitives.hip) vs rocPRIM's device radix sort on the same
// (capture << joinbits | join)-shaped u64 keys, sorted on the low `bits` bits.  Build:
//   hipcc -O3 --offload-arch=gfx950 -I rdfind_amd/csrc tools/micro/sortbench.hip rdfind_amd/csrc/primitives.hip -o tools/micro/sortbench
#include <hip/hip_runtime.h>
#include <cstring>
#include <rocprim/device/device_radix_sort.hpp>
#include <cstdio>
#include <cstdlib>
#include <vector>
#include <algorithm>
#include "primitives.hpp"

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s at %d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)

__global__ void gen(unsigned long long* k, size_t n, int capbits, int joinbits, unsigned long long seed) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
        unsigned long long x = (i + 1) * 0x9E3779B97F4A7C15ull ^ seed;
        x ^= x >> 31; x *= 0xBF58476D1CE4E5B9ull; x ^= x >> 29;
        // skewed captures (squares of uniforms), uniform joins
        const unsigned long long c = ((x & 0xffffffffull) * (x & 0xffffffffull)) >> (64 - capbits);
        const unsigned long long j = (x >> 32) % (1ull << joinbits);
        k[i] = c << joinbits | j;
    }
}

int main(int argc, char** argv) {
    const size_t n = argc > 1 ? strtoull(argv[1], 0, 10) : 59067574ull;
    const int capbits = argc > 2 ? atoi(argv[2]) : 20, joinbits = argc > 3 ? atoi(argv[3]) : 23;
    const int bits = capbits + joinbits;
    unsigned long long *a, *b, *c0;
    CK(hipMalloc(&a, n * 8)); CK(hipMalloc(&b, n * 8)); CK(hipMalloc(&c0, n * 8));
    gen<<<4096, 256>>>(c0, n, capbits, joinbits, 12345);
    CK(hipDeviceSynchronize());
    hipStream_t st; CK(hipStreamCreate(&st));
    hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
    rdf::Workspace ws;
    float best = 1e9;
    unsigned long long* res = nullptr;
    for (int it = 0; it < 5; ++it) {
        CK(hipMemcpyAsync(a, c0, n * 8, hipMemcpyDeviceToDevice, st));
        unsigned long long *k = a, *t = b;
        CK(hipEventRecord(e0, st));
        CK(rdf::radix_sort_u64(ws, k, t, n, bits, st));
        CK(hipEventRecord(e1, st));
        CK(hipEventSynchronize(e1));
        float ms; CK(hipEventElapsedTime(&ms, e0, e1)); best = std::min(best, ms);
        res = k;
    }
    std::vector<unsigned long long> h1(n), h2(n);
    CK(hipMemcpy(h1.data(), res, n * 8, hipMemcpyDeviceToHost));
    printf("rdf radix %zu keys %d bits: %.3f ms\n", n, bits, best);
    // rocPRIM
    size_t tb = 0;
    CK(rocprim::radix_sort_keys(nullptr, tb, a, b, n, 0, bits, st));
    void* tmp; CK(hipMalloc(&tmp, tb));
    float best2 = 1e9;
    for (int it = 0; it < 5; ++it) {
        CK(hipMemcpyAsync(a, c0, n * 8, hipMemcpyDeviceToDevice, st));
        CK(hipEventRecord(e0, st));
        CK(rocprim::radix_sort_keys(tmp, tb, a, b, n, 0, bits, st));
        CK(hipEventRecord(e1, st));
        CK(hipEventSynchronize(e1));
        float ms; CK(hipEventElapsedTime(&ms, e0, e1)); best2 = std::min(best2, ms);
    }
    CK(hipMemcpy(h2.data(), b, n * 8, hipMemcpyDeviceToHost));
    printf("rocprim radix %zu keys %d bits: %.3f ms (temp %zu MB) same=%d\n", n, bits, best2, tb >> 20, (int)(h1 == h2));
    return 0;
}
