// Micro-benchmark of the PH reduction kernels (k_xbar, k_update_w_seg) at
// farmer 100k: full kernels and stripped variants, timed with HIP events.
#include "../../mpi-sppy_amd/csrc/phx_kernels.hip"
#include <cstdio>

// variant: tile partials only (no ticket, no finish)
__global__ __launch_bounds__(RED_NT) void v_tiles(int S, const int32_t* tile_s0, const int32_t* tile_s1,
    const int32_t* tile_slot, const int32_t* tile_nlen, const int32_t* tile_out, const int32_t* slot_col,
    const double* x, const double* pc, double* partial) {
    __shared__ double sh[RED_NT / 64 * 2 * XB_CH];
    xbar_tile(blockIdx.x, S, tile_s0, tile_s1, tile_slot, tile_nlen, tile_out, slot_col, x, pc, partial, sh);
}
// variant: loads only, one store per thread
__global__ __launch_bounds__(RED_NT) void v_loads(int S, const int32_t* slot_col, const double* x, const double* pc,
                                                  double* out) {
    const int s = blockIdx.x * RED_NT + threadIdx.x;
    if (s >= S) return;
    double a = 0;
    for (int j = 0; j < 3; ++j) a += pc[ix(j, s, S)] * x[ix(slot_col[j], s, S)];
    out[s] = a;
}
// variant: 1 scenario per thread, 391 blocks, block_sum_multi of 6 values, partial per block
__global__ __launch_bounds__(256) void v_tiles256(int S, const int32_t* slot_col, const double* x, const double* pc,
                                                  double* partial) {
    __shared__ double sh[4 * 8];
    const int s = blockIdx.x * 256 + threadIdx.x;
    double acc[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) acc[k] = 0.0;
    if (s < S) {
#pragma unroll
        for (int j = 0; j < 3; ++j) {
            const double xv = x[ix(slot_col[j], s, S)];
            const double v = pc[ix(j, s, S)] * xv;
            acc[j] = v; acc[4 + j] = v * xv;
        }
    }
    block_sum_multi<256, 8>(acc, sh);
    if (threadIdx.x == 0) for (int k = 0; k < 8; ++k) partial[blockIdx.x * 8 + k] = acc[k];
}
// variant: 4 scen/thread, no block reduction (thread partials written)
__global__ __launch_bounds__(256) void v_noreduce(int S, const int32_t* slot_col, const double* x, const double* pc,
                                                  double* out) {
    double acc[6] = {0, 0, 0, 0, 0, 0};
    for (int u = 0; u < 4; ++u) {
        const int s = blockIdx.x * 1024 + threadIdx.x + u * 256;
        if (s < S)
#pragma unroll
            for (int j = 0; j < 3; ++j) {
                const double xv = x[ix(slot_col[j], s, S)];
                const double v = pc[ix(j, s, S)] * xv;
                acc[j] += v; acc[3 + j] += v * xv;
            }
    }
    const int t = blockIdx.x * 256 + threadIdx.x;
    if (acc[0] + acc[1] + acc[2] + acc[3] + acc[4] + acc[5] == 12345.0) out[t] = 0.0;
}
__global__ void v_empty(int S, double* out) {
    const int s = blockIdx.x * blockDim.x + threadIdx.x;
    if (s < 0) out[s] = 0;
}

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("err %s line %d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)

int main() {
    const int S = 100000, n = 12, N = 3, CH = 256;
    std::vector<int32_t> slot_col = {0, 1, 2};
    double *x, *pc, *partial, *node, *W, *rho, *seg, *out;
    int32_t *sc, *xi;
    CK(hipMalloc(&x, sizeof(double) * n * S));
    CK(hipMalloc(&pc, sizeof(double) * N * S));
    CK(hipMalloc(&W, sizeof(double) * N * S));
    CK(hipMalloc(&rho, sizeof(double) * N * S));
    CK(hipMalloc(&out, sizeof(double) * S));
    CK(hipMalloc(&partial, sizeof(double) * 4096));
    CK(hipMalloc(&node, sizeof(double) * 64));
    CK(hipMalloc(&seg, sizeof(double) * 64));
    CK(hipMalloc(&sc, sizeof(int32_t) * N));
    CK(hipMalloc(&xi, sizeof(int32_t) * N * S));
    std::vector<double> h(n * S);
    for (int i = 0; i < n * S; ++i) h[i] = (i % 97) * 0.5;
    CK(hipMemcpy(x, h.data(), sizeof(double) * n * S, hipMemcpyHostToDevice));
    CK(hipMemcpy(pc, h.data(), sizeof(double) * N * S, hipMemcpyHostToDevice));
    CK(hipMemcpy(W, h.data(), sizeof(double) * N * S, hipMemcpyHostToDevice));
    CK(hipMemcpy(rho, h.data(), sizeof(double) * N * S, hipMemcpyHostToDevice));
    CK(hipMemcpy(sc, slot_col.data(), sizeof(int32_t) * N, hipMemcpyHostToDevice));
    std::vector<int32_t> hx(N * S);
    for (int j = 0; j < N; ++j) for (int s = 0; s < S; ++s) hx[j * S + s] = j;
    CK(hipMemcpy(xi, hx.data(), sizeof(int32_t) * N * S, hipMemcpyHostToDevice));
    // tiles
    std::vector<int32_t> t0, t1, tsl, tnl, tout, nptr = {0}, noff = {0}, nnl = {3};
    for (int s = 0; s < S; s += CH) { t0.push_back(s); t1.push_back(std::min(S, s + CH)); tsl.push_back(0); tnl.push_back(3); tout.push_back(6 * (int)tout.size()); }
    const int nt = (int)t0.size();
    nptr.push_back(nt);
    auto up = [&](std::vector<int32_t>& v) { int32_t* d; (void)hipMalloc(&d, 4 * v.size()); (void)hipMemcpy(d, v.data(), 4 * v.size(), hipMemcpyHostToDevice); return d; };
    int32_t *d0 = up(t0), *d1 = up(t1), *dsl = up(tsl), *dnl = up(tnl), *dout = up(tout), *dptr = up(nptr), *doff = up(noff), *dnnl = up(nnl);
    std::vector<int32_t> sp = {0, nt};
    int32_t* dsp = up(sp);
    unsigned int* tick; CK(hipMalloc(&tick, 8 * TICKET_SET)); CK(hipMemset(tick, 0, 8 * TICKET_SET));
    hipStream_t st; CK(hipStreamCreate(&st));
    hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
    auto timeit = [&](const char* name, auto launch) {
        for (int r = 0; r < 20; ++r) launch();
        (void)hipStreamSynchronize(st);
        const int R = 200;
        (void)hipEventRecord(e0, st);
        for (int r = 0; r < R; ++r) launch();
        (void)hipEventRecord(e1, st);
        (void)hipEventSynchronize(e1);
        float ms; (void)hipEventElapsedTime(&ms, e0, e1);
        printf("%-44s %8.2f us/launch\n", name, ms * 1000.f / R);
    };
    timeit("empty (391 blocks x 256)", [&] { hipLaunchKernelGGL(v_empty, dim3(391), dim3(256), 0, st, S, out); });
    timeit("loads only (391 x 256, 1 scen/thread)", [&] { hipLaunchKernelGGL(v_loads, dim3(391), dim3(256), 0, st, S, sc, x, pc, out); });
    timeit("xbar 1 scen/thread + block_sum_multi (391 x 256)", [&] { hipLaunchKernelGGL(v_tiles256, dim3(391), dim3(256), 0, st, S, sc, x, pc, partial); });
    timeit("xbar 4 scen/thread, no block reduce (98 x 256)", [&] { hipLaunchKernelGGL(v_noreduce, dim3(98), dim3(256), 0, st, S, sc, x, pc, out); });
    timeit("xbar tiles only (98 x 256)", [&] { hipLaunchKernelGGL(v_tiles, dim3(nt), dim3(RED_NT), 0, st, S, d0, d1, dsl, dnl, dout, sc, x, pc, partial); });
    timeit("k_xbar full", [&] { hipLaunchKernelGGL(k_xbar, dim3(nt), dim3(RED_NT), 0, st, S, nt, d0, d1, dsl, dnl, dout, sc, x, pc, partial, 1, dptr, doff, dnnl, 3, node, tick, (const int32_t*)nullptr, (const int32_t*)nullptr, 1); });
    timeit("k_update_w_seg full", [&] { hipLaunchKernelGGL(k_update_w_seg, dim3(nt), dim3(RED_NT), 0, st, N, S, sc, x, (const double*)node, xi, rho, (const double*)W, W, 1, (double*)nullptr, d0, d1, partial, 1, dsp, seg, tick + TICKET_SET, IterkCtl{}); });
    timeit("k_update_w_seg no W update", [&] { hipLaunchKernelGGL(k_update_w_seg, dim3(nt), dim3(RED_NT), 0, st, N, S, sc, x, (const double*)node, xi, rho, (const double*)W, W, 0, (double*)nullptr, d0, d1, partial, 1, dsp, seg, tick + TICKET_SET, IterkCtl{}); });
    return 0;
}
