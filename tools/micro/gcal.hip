// FETCH_SIZE calibration for the access widths of the light pass (dev tool; MI355X_MICROARCH.md: "other access
// widths are uncalibrated: calibrate on a known byte count in your own access pattern").
//   hipcc -O3 --offload-arch=gfx950 -o tools/micro/gcal tools/micro/gcal.hip
//   rocprofv3 --pmc FETCH_SIZE --kernel-trace -d DIR -o run --output-format csv -- tools/micro/gcal
// k_stream16: coalesced 16-B loads over 1 GiB (2^26 lane loads); k_gather4: 2^26 random 4-B loads from a 4 GiB
// table (distinct lines with high probability, far beyond L2 and the Infinity Cache); k_gather4_line: 2^26 4-B loads,
// 16 consecutive lanes in one 64-B line (the member-list searches of adjacent lanes).
// FETCH_SIZE (KB) / loads gives the reported bytes per load of each pattern.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

__device__ inline uint64_t mix(uint64_t x) {
    x ^= x >> 33;
    x *= 0xff51afd7ed558ccdull;
    x ^= x >> 33;
    x *= 0xc4ceb9fe1a85ec53ull;
    x ^= x >> 33;
    return x;
}

__global__ void k_stream16(const uint4* __restrict__ a, uint64_t n, uint32_t* out) {
    uint32_t acc = 0;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
        const uint4 v = a[i];
        acc ^= v.x ^ v.y ^ v.z ^ v.w;
    }
    if (acc == 0x12345678u) out[0] = acc;
}

__global__ void k_gather4(const uint32_t* __restrict__ t, uint64_t words, uint64_t n, uint32_t* out) {
    uint32_t acc = 0;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
        acc ^= t[mix(i) % words];
    if (acc == 0x12345678u) out[0] = acc;
}

__global__ void k_gather4_line(const uint32_t* __restrict__ t, uint64_t words, uint64_t n, uint32_t* out) {
    uint32_t acc = 0;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
        const uint64_t line = mix(i >> 4) % (words / 16);
        acc ^= t[line * 16 + (i & 15)];
    }
    if (acc == 0x12345678u) out[0] = acc;
}

int main() {
    const uint64_t tbytes = 4ull << 30, sbytes = 1ull << 30, n = 1ull << 26;
    void *t = nullptr, *s = nullptr;
    uint32_t* out = nullptr;
    if (hipMalloc(&t, tbytes) != hipSuccess || hipMalloc(&s, sbytes) != hipSuccess || hipMalloc(&out, 4) != hipSuccess) {
        fprintf(stderr, "alloc failed\n");
        return 1;
    }
    (void)hipMemset(t, 1, tbytes);
    (void)hipMemset(s, 1, sbytes);
    for (int rep = 0; rep < 2; ++rep) {
        hipLaunchKernelGGL(k_stream16, dim3(4096), dim3(256), 0, 0, (const uint4*)s, sbytes / 16, out);
        hipLaunchKernelGGL(k_gather4, dim3(4096), dim3(256), 0, 0, (const uint32_t*)t, tbytes / 4, n, out);
        hipLaunchKernelGGL(k_gather4_line, dim3(4096), dim3(256), 0, 0, (const uint32_t*)t, tbytes / 4, n, out);
    }
    if (hipDeviceSynchronize() != hipSuccess) {
        fprintf(stderr, "kernel failed\n");
        return 1;
    }
    printf("GCAL stream16 bytes %llu; gather4 loads %llu (random lines); gather4_line loads %llu (16 per 64-B line)\n",
           (unsigned long long)sbytes, (unsigned long long)n, (unsigned long long)n);
    (void)hipFree(t);
    (void)hipFree(s);
    (void)hipFree(out);
    return 0;
}
