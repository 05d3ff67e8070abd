// Accuracy of the gfx950 hardware reciprocal / reciprocal square root (f64)
// and of one / two Newton steps on them, over log-uniform operands in
// [1e-12, 1e12]: max relative error against the correctly rounded quotient.
// hipcc --offload-arch=gfx950 -O3 -o rcp_acc rcp_acc.hip && ./rcp_acc
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdio>
#include <vector>

__global__ void k_rcp(const double* d, double* out, int n) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const double x = d[i];
    const double r0 = __builtin_amdgcn_rcp(x);
    const double r1 = fma(r0, fma(-x, r0, 1.0), r0);
    const double r2 = fma(r1, fma(-x, r1, 1.0), r1);
    const double q = 1.0 / x;
    const double s0 = __builtin_amdgcn_rsq(x);
    const double s1 = s0 * fma(-0.5 * x * s0, s0, 1.5);
    const double sq = 1.0 / sqrt(x);
    out[6 * i + 0] = fabs(r0 - q) / q;
    out[6 * i + 1] = fabs(r1 - q) / q;
    out[6 * i + 2] = fabs(r2 - q) / q;
    out[6 * i + 3] = fabs(s0 - sq) / sq;
    out[6 * i + 4] = fabs(s1 - sq) / sq;
    out[6 * i + 5] = 0.0;
}

int main() {
    const int n = 1 << 20;
    std::vector<double> h(n);
    unsigned long long s = 88172645463325252ull;
    for (int i = 0; i < n; ++i) {
        s ^= s << 13; s ^= s >> 7; s ^= s << 17;
        const double u = (double)(s >> 11) / 9007199254740992.0;
        h[i] = std::pow(10.0, -12.0 + 24.0 * u);
    }
    double *d = nullptr, *o = nullptr;
    if (hipMalloc(&d, n * sizeof(double)) != hipSuccess || hipMalloc(&o, 6 * n * sizeof(double)) != hipSuccess) return 1;
    if (hipMemcpy(d, h.data(), n * sizeof(double), hipMemcpyHostToDevice) != hipSuccess) return 1;
    hipLaunchKernelGGL(k_rcp, dim3(n / 256), dim3(256), 0, 0, d, o, n);
    std::vector<double> r(6 * (size_t)n);
    if (hipMemcpy(r.data(), o, r.size() * sizeof(double), hipMemcpyDeviceToHost) != hipSuccess) return 1;
    const char* names[] = {"rcp", "rcp+1 Newton", "rcp+2 Newton", "rsq", "rsq+1 Newton"};
    for (int k = 0; k < 5; ++k) {
        double mx = 0.0;
        for (int i = 0; i < n; ++i) mx = std::fmax(mx, r[6 * (size_t)i + k]);
        printf("%-14s max rel. error %.3e (%.1f bits)\n", names[k], mx, mx > 0 ? -std::log2(mx) : 99.0);
    }
    return 0;
}
