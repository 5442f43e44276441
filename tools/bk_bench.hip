// Microbenchmark: cycles per 9 x 9 stage-block factorisation for one wavefront (C2 chain blocks that need 2x2
// pivots, and blocks that factor in natural order), register Bunch-Kaufman vs the LDS routine.
//   hipcc -O3 --offload-arch=gfx950 -mllvm -disable-promote-alloca-to-lds tools/bk_bench.hip -o tools/bk_bench.bin
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#include "../mpc_fatigue_amd/csrc/bk_wave.hpp"
using namespace mf;

constexpr int M = 9, LD = 10, REP = 200;

template <int V>
__global__ __launch_bounds__(64) void kbench(const double *K, unsigned long long *cyc, double *sink) {
    __shared__ double A[M * LD];
    __shared__ int perm[M], piv[M];
    const int lane = threadIdx.x;
    double acc = 0.0;
    unsigned long long t0 = 0;
    for (int r = 0; r < REP + 1; r++) {
        if (r == 1) t0 = __builtin_amdgcn_s_memtime();
        for (int e = lane; e < M * LD; e += 64) A[e] = K[blockIdx.x * M * LD + e];
        wave_lds_sync();
        BKInertia in;
        if constexpr (V == 0) in = bk_factor_regs_piv<LD, M>(A, perm, piv);
        if constexpr (V == 1) in = bk_factor_wave<LD>(A, M, perm, piv);
        if constexpr (V == 2) {
            if (!bk_factor_regs<LD, M>(A, perm, piv, in)) in = bk_factor_wave<LD>(A, M, perm, piv);
        }
        if constexpr (V == 3) in = bk_factor_fixed<LD, M>(A, perm, piv);
        if constexpr (V == 5) in = bk_factor_regs_loop<LD, M>(A, perm, piv);
        if constexpr (V == 6) {
            if (!bk_factor_regs<LD, M>(A, perm, piv, in)) in = bk_factor_regs_loop<LD, M>(A, perm, piv);
        }
        if constexpr (V == 4) {
            if (!bk_factor_regs<LD, M>(A, perm, piv, in)) in = bk_factor_fixed<LD, M>(A, perm, piv);
        }
        acc += A[(lane % M) * LD + lane % M] + in.pos;
        wave_lds_sync();
    }
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    if (lane == 0) cyc[blockIdx.x] = (t1 - t0) / REP;
    sink[blockIdx.x * 64 + lane] = acc;
}

int main() {
    const int nb = 2;
    std::vector<double> K(nb * M * LD, 0.0);
    srand(3);
    auto rnd = [] { return (double)rand() / RAND_MAX - 0.5; };
    for (int b = 0; b < nb; b++) {
        double *k = &K[b * M * LD];
        for (int i = 0; i < 7; i++)
            for (int j = 0; j <= i; j++) {
                double v = 1e-3 * rnd();
                if (i == j) v = (b == 0 ? 1e-4 : 10.0) + fabs(v);
                k[i * LD + j] = k[j * LD + i] = v;
            }
        for (int e = 0; e < 2; e++)
            for (int j = 0; j < 6; j++) k[(7 + e) * LD + j] = k[j * LD + 7 + e] = 0.05 * rnd();
    }
    double *dK, *ds;
    unsigned long long *dc;
    hipMalloc(&dK, K.size() * 8);
    hipMalloc(&ds, nb * 64 * 8);
    hipMalloc(&dc, nb * 8);
    hipMemcpy(dK, K.data(), K.size() * 8, hipMemcpyHostToDevice);
    const char *names[7] = {"regs_piv", "lds_wave", "regs_natural+wave", "lds_fixed", "regs_natural+fixed", "regs_loop",
                            "regs_natural+loop"};
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    for (int v = 0; v < 7; v++) {
        for (int rep = 0; rep < 2; rep++) {
            if (v == 0) hipLaunchKernelGGL(kbench<0>, dim3(nb), dim3(64), 0, 0, dK, dc, ds);
            if (v == 1) hipLaunchKernelGGL(kbench<1>, dim3(nb), dim3(64), 0, 0, dK, dc, ds);
            if (v == 2) hipLaunchKernelGGL(kbench<2>, dim3(nb), dim3(64), 0, 0, dK, dc, ds);
            if (v == 3) hipLaunchKernelGGL(kbench<3>, dim3(nb), dim3(64), 0, 0, dK, dc, ds);
            if (v == 4) hipLaunchKernelGGL(kbench<4>, dim3(nb), dim3(64), 0, 0, dK, dc, ds);
            if (v == 5) hipLaunchKernelGGL(kbench<5>, dim3(nb), dim3(64), 0, 0, dK, dc, ds);
            if (v == 6) hipLaunchKernelGGL(kbench<6>, dim3(nb), dim3(64), 0, 0, dK, dc, ds);
        }
        // clock calibration: the same launch timed by events (REP + 1 factorisations plus loads per wave)
        hipEventRecord(e0, 0);
        if (v == 1) hipLaunchKernelGGL(kbench<1>, dim3(nb), dim3(64), 0, 0, dK, dc, ds);
        hipEventRecord(e1, 0);
        hipEventSynchronize(e1);
        float ms = 0;
        hipEventElapsedTime(&ms, e0, e1);
        if (v == 1) printf("calibration: lds_wave launch %.1f us for %d factorisations per wave\n", ms * 1e3, REP + 1);
        unsigned long long c[nb];
        hipMemcpy(c, dc, sizeof c, hipMemcpyDeviceToHost);
        printf("%-24s pivoting block %llu cycles, natural-order block %llu cycles\n", names[v], c[0], c[1]);
    }
    return 0;
}
