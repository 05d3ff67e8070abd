// FP64 VALU dependent-chain latency and issue cost on gfx950 (one wave per
// SIMD): a chain of N dependent v_fma_f64, then 2 / 4 / 8 independent chains
// interleaved; cycles from s_memtime (the shader clock), per instruction.
// hipcc --offload-arch=gfx950 -O3 -o f64lat f64lat.hip && ./f64lat
#include <hip/hip_runtime.h>
#include <stdio.h>

template <int C>
__global__ void chains(double* out, long long* cyc, double a, double b, int n) {
    double x[C];
    for (int c = 0; c < C; ++c) x[c] = threadIdx.x * 1e-3 + c;
    __syncthreads();
    long long t0 = __builtin_amdgcn_s_memtime();
    for (int i = 0; i < n; ++i) {
#pragma unroll
        for (int k = 0; k < 16; ++k)
#pragma unroll
            for (int c = 0; c < C; ++c) x[c] = fma(x[c], a, b);
    }
    long long t1 = __builtin_amdgcn_s_memtime();
    double s = 0;
    for (int c = 0; c < C; ++c) s += x[c];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
    if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

__global__ void rcp_chain(double* out, long long* cyc, int n) {
    double x = 1.5 + threadIdx.x * 1e-6;
    long long t0 = __builtin_amdgcn_s_memtime();
    for (int i = 0; i < n; ++i) {
#pragma unroll
        for (int k = 0; k < 16; ++k) x = __builtin_amdgcn_rcp(x) + 1.0;
    }
    long long t1 = __builtin_amdgcn_s_memtime();
    out[threadIdx.x] = x;
    if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

template <int C>
static void run(int blocks, const char* what) {
    double* out; long long* cyc;
    hipMalloc(&out, sizeof(double) * 64 * blocks);
    hipMalloc(&cyc, sizeof(long long) * blocks);
    const int n = 256;
    hipLaunchKernelGGL(chains<C>, dim3(blocks), dim3(64), 0, 0, out, cyc, 0.999, 1e-3, n);
    hipLaunchKernelGGL(chains<C>, dim3(blocks), dim3(64), 0, 0, out, cyc, 0.999, 1e-3, n);
    hipDeviceSynchronize();
    long long h[4096];
    hipMemcpy(h, cyc, sizeof(long long) * blocks, hipMemcpyDeviceToHost);
    double avg = 0;
    for (int b = 0; b < blocks; ++b) avg += h[b];
    avg /= blocks;
    printf("%-28s waves %5d: %.2f cycles per fma (per chain step %.2f)\n", what, blocks, avg / (n * 16.0 * C),
           avg / (n * 16.0));
    hipFree(out); hipFree(cyc);
}

int main() {
    for (int blocks : {1, 1024, 2048, 4096}) {
        run<1>(blocks, "1 chain (dependent)");
        run<2>(blocks, "2 chains");
        run<4>(blocks, "4 chains");
        run<8>(blocks, "8 chains");
    }
    double* out; long long* cyc; long long h;
    hipMalloc(&out, sizeof(double) * 64);
    hipMalloc(&cyc, sizeof(long long));
    hipLaunchKernelGGL(rcp_chain, dim3(1), dim3(64), 0, 0, out, cyc, 256);
    hipLaunchKernelGGL(rcp_chain, dim3(1), dim3(64), 0, 0, out, cyc, 256);
    hipDeviceSynchronize();
    hipMemcpy(&h, cyc, sizeof(long long), hipMemcpyDeviceToHost);
    printf("rcp_f64 + add chain: %.2f cycles per step\n", h / (256 * 16.0));
    return 0;
}
