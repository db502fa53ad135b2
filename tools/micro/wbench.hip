// Write-rate microbenchmark (dev tool): how fast can gfx950 stream 16-B stores under the access shapes the
// class emission uses?  Build: hipcc -O3 --offload-arch=gfx950 wbench.hip -o wbench
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

typedef unsigned long long u64;

// contiguous: block b writes [b*T, (b+1)*T) quads
__global__ __launch_bounds__(256) void k_seq(uint4* out, u64 nq, u64 T) {
    const u64 b0 = (u64)blockIdx.x * T;
    for (u64 i = threadIdx.x; i < T && b0 + i < nq; i += 256) out[b0 + i] = make_uint4((unsigned)i, 1, 2, 3);
}
// grid-stride
__global__ __launch_bounds__(256) void k_gs(uint4* out, u64 nq) {
    for (u64 i = (u64)blockIdx.x * 256 + threadIdx.x; i < nq; i += (u64)gridDim.x * 256) out[i] = make_uint4((unsigned)i, 1, 2, 3);
}
// runs: block writes R runs of L quads each, run r of tile t at (r * RS + t * L) (RS = run stride)
__global__ __launch_bounds__(256) void k_runs(uint4* out, u64 R, u64 L, u64 RS, u64 ntile_per_run) {
    const u64 t = blockIdx.x % ntile_per_run, rg = blockIdx.x / ntile_per_run;
    for (u64 r = rg * R; r < rg * R + R; ++r)
        for (u64 i = threadIdx.x; i < L; i += 256) out[r * RS + t * L + i] = make_uint4((unsigned)i, 1, 2, 3);
}

int main() {
    const u64 bytes = 20ull << 30, nq = bytes / 16;
    uint4* out;
    if (hipMalloc(&out, bytes) != hipSuccess) return 1;
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    float ms;
    auto run = [&](const char* name, auto fn) {
        fn();
        hipDeviceSynchronize();
        hipEventRecord(a);
        for (int k = 0; k < 3; ++k) fn();
        hipEventRecord(b);
        hipEventSynchronize(b);
        hipEventElapsedTime(&ms, a, b);
        printf("%-40s %.2f TB/s\n", name, 3.0 * bytes / (ms * 1e-3) / 1e12);
    };
    for (u64 T : {1024ull, 4096ull, 16384ull, 65536ull}) {
        char nm[64];
        snprintf(nm, 64, "seq tile %llu KB", T * 16 / 1024);
        run(nm, [&] { hipLaunchKernelGGL(k_seq, dim3((unsigned)((nq + T - 1) / T)), dim3(256), 0, 0, out, nq, T); });
    }
    for (unsigned g : {2048u, 8192u, 65536u}) {
        char nm[64];
        snprintf(nm, 64, "grid-stride %u blocks", g);
        run(nm, [&] { hipLaunchKernelGGL(k_gs, dim3(g), dim3(256), 0, 0, out, nq); });
    }
    // class shape: runs of 71k u32 = 17.8k quads; per tile R runs x L quads
    const u64 RS = 17792;
    const u64 nruns = nq / RS;
    for (u64 R : {16ull, 64ull})
        for (u64 L : {512ull, 1024ull, 4096ull}) {
            const u64 ntpr = RS / L;
            char nm[64];
            snprintf(nm, 64, "runs R=%llu L=%llu quads", R, L);
            run(nm, [&] { hipLaunchKernelGGL(k_runs, dim3((unsigned)((nruns / R) * ntpr)), dim3(256), 0, 0, out, R, L, RS, ntpr); });
        }
    return 0;
}
