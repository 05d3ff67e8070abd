// Micro-benchmark: GPU-side gap between back-to-back kernels with various
// stream operations in between (event records, D2H copies, mapped writes).
#include <hip/hip_runtime.h>
#include <chrono>
#include <cstdio>

__global__ void k_a(double* p, int n) {
    int t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t < n) p[t] += 1.0;
}
__global__ void k_map(double* p, int n, volatile int* host_flag, int seq) {
    int t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t < n) p[t] += 1.0;
    if (t == 0) { __threadfence_system(); *host_flag = seq; }
}

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("err %s line %d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)

int main() {
    const int n = 1 << 16, R = 200;
    double* d; CK(hipMalloc(&d, n * 8)); CK(hipMemset(d, 0, n * 8));
    int* hp; CK(hipHostMalloc(&hp, 64, hipHostMallocMapped | hipHostMallocCoherent));
    int* hd; CK(hipHostGetDevicePointer((void**)&hd, hp, 0));
    int* pin; CK(hipHostMalloc(&pin, 64, 0));
    hipStream_t st; CK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
    hipEvent_t et, en; CK(hipEventCreate(&et)); CK(hipEventCreateWithFlags(&en, hipEventDisableTiming));
    auto run = [&](const char* name, int mode) -> int {
        CK(hipStreamSynchronize(st));
        auto t0 = std::chrono::high_resolution_clock::now();
        for (int r = 0; r < R; ++r) {
            if (mode == 5) hipLaunchKernelGGL(k_map, dim3(n / 256), dim3(256), 0, st, d, n, (volatile int*)hd, r + 1);
            else hipLaunchKernelGGL(k_a, dim3(n / 256), dim3(256), 0, st, d, n);
            if (mode == 1) CK(hipEventRecord(et, st));
            if (mode == 2) CK(hipEventRecord(en, st));
            if (mode == 3) CK(hipMemcpyAsync(pin, d, 8, hipMemcpyDeviceToHost, st));
            if (mode == 4) { CK(hipEventRecord(et, st)); CK(hipEventSynchronize(et)); }
            if (mode == 5) { while (__atomic_load_n(&hp[0], __ATOMIC_ACQUIRE) != r + 1) {} }
            if (mode == 6) { CK(hipMemcpyAsync(pin, d, 8, hipMemcpyDeviceToHost, st)); CK(hipStreamSynchronize(st)); }
            if (mode == 7) { CK(hipEventRecord(en, st)); CK(hipEventSynchronize(en)); }
        }
        CK(hipStreamSynchronize(st));
        auto t1 = std::chrono::high_resolution_clock::now();
        printf("%-40s %8.2f us/iter\n", name, std::chrono::duration<double, std::micro>(t1 - t0).count() / R);
        return 0;
    };
    for (int rep = 0; rep < 2; ++rep) {
        run("kernel only", 0);
        run("kernel + event(timing)", 1);
        run("kernel + event(no timing)", 2);
        run("kernel + D2H 8B memcpyAsync", 3);
        run("kernel + event(timing) + sync (roundtrip)", 4);
        run("kernel(mapped flag) + host spin (roundtrip)", 5);
        run("kernel + D2H + streamsync (roundtrip)", 6);
        run("kernel + event(no timing) + sync (roundtrip)", 7);
    }
    return 0;
}
