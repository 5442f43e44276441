// Probe (not product code): one wavefront forms C = A B for the generic solver's stage-product shapes
// (M x K times K x N, FP64, operands in LDS) repeatedly, (a) the product's tile_gemm (bk_wave.hpp: each
// lane a register tile of outputs, the operands of one inner index read once per tile) and
// (b) with v_mfma_f64_16x16x4_f64 on zero-padded 16 x 16 output tiles and 4-deep K steps; prints cycles per
// product (s_memtime) and the largest difference of the two results.  DESIGN.md s.9 records the outcome.
//
//   hipcc -O3 --offload-arch=gfx950 tools/mfma_probe.hip -o /tmp/mfma_probe && /tmp/mfma_probe
#include <hip/hip_runtime.h>

#include "../mpc_fatigue_amd/csrc/bk_wave.hpp"

#include <cmath>
#include <cstdio>
#include <vector>

typedef double v4d __attribute__((ext_vector_type(4)));

template <int M, int N, int K>
__global__ __launch_bounds__(64) void k_probe(const double *A, const double *B, double *Cv, double *Cm, long long *cyc,
                                             int reps) {
    __shared__ double As[M * K], Bs[K * N], Cs[M * N];
    const int lane = threadIdx.x;
    for (int e = lane; e < M * K; e += 64) As[e] = A[e];
    for (int e = lane; e < K * N; e += 64) Bs[e] = B[e];
    __syncthreads();
    // (a) VALU: the product's tile_gemm
    long long t0 = __builtin_amdgcn_s_memtime();
    for (int r = 0; r < reps; r++) {
        mf::tile_gemm<M, N, K>(
            lane, [&](int, int) { return 1e-300 * r; }, [&](int l, int i) { return As[i * K + l]; },
            [&](int l, int j) { return Bs[l * N + j]; }, [&](int i, int j, double v) { Cs[i * N + j] = v; });
        __syncthreads();
    }
    long long t1 = __builtin_amdgcn_s_memtime();
    for (int e = lane; e < M * N; e += 64) Cv[e] = Cs[e];
    __syncthreads();
    // (b) MFMA 16x16x4 f64: A operand lane l -> (row l%16, k l/16), B operand (k l/16, col l%16),
    // result lane l, register q -> (row l/16 + 4 q, col l%16)
    constexpr int TM = (M + 15) / 16, TN = (N + 15) / 16, TK = (K + 3) / 4;
    const int i16 = lane % 16, k4 = lane / 16;
    __syncthreads();
    long long t2 = __builtin_amdgcn_s_memtime();
    for (int r = 0; r < reps; r++) {
        // all TM x TN accumulators live at once; per K step the fragments are loaded once and the
        // TM x TN independent MFMAs issue back to back (no dependent chain between neighbours)
        v4d c[TM][TN];
#pragma unroll
        for (int tm = 0; tm < TM; tm++)
#pragma unroll
            for (int tn = 0; tn < TN; tn++) c[tm][tn] = v4d{0.0, 0.0, 0.0, 0.0};
#pragma unroll
        for (int tk = 0; tk < TK; tk++) {
            const int ak = tk * 4 + k4;
            double a[TM], b[TN];
#pragma unroll
            for (int tm = 0; tm < TM; tm++) {
                const int ai = tm * 16 + i16;
                a[tm] = (ai < M && ak < K) ? As[ai * K + ak] : 0.0;
            }
#pragma unroll
            for (int tn = 0; tn < TN; tn++) {
                const int bj = tn * 16 + i16;
                b[tn] = (ak < K && bj < N) ? Bs[ak * N + bj] : 0.0;
            }
#pragma unroll
            for (int tm = 0; tm < TM; tm++)
#pragma unroll
                for (int tn = 0; tn < TN; tn++) c[tm][tn] = __builtin_amdgcn_mfma_f64_16x16x4f64(a[tm], b[tn], c[tm][tn], 0, 0, 0);
        }
#pragma unroll
        for (int tm = 0; tm < TM; tm++)
#pragma unroll
            for (int tn = 0; tn < TN; tn++)
#pragma unroll
                for (int q = 0; q < 4; q++) {
                    const int ci = tm * 16 + k4 + 4 * q, cj = tn * 16 + i16;
                    if (ci < M && cj < N) Cs[ci * N + cj] = c[tm][tn][q] + 1e-300 * r;
                }
        __syncthreads();
    }
    long long t3 = __builtin_amdgcn_s_memtime();
    for (int e = lane; e < M * N; e += 64) Cm[e] = Cs[e];
    if (lane == 0) {
        cyc[0] = (t1 - t0) / reps;
        cyc[1] = (t3 - t2) / reps;
    }
}

template <int M, int N, int K> static void run(const char *what) {
    std::vector<double> A(M * K), B(K * N);
    for (int i = 0; i < M * K; i++) A[i] = std::sin(0.37 * i + 0.1);
    for (int i = 0; i < K * N; i++) B[i] = std::cos(0.23 * i - 0.4);
    double *dA, *dB, *dCv, *dCm;
    long long *dc;
    hipMalloc(&dA, sizeof(double) * A.size());
    hipMalloc(&dB, sizeof(double) * B.size());
    hipMalloc(&dCv, sizeof(double) * M * N);
    hipMalloc(&dCm, sizeof(double) * M * N);
    hipMalloc(&dc, sizeof(long long) * 2);
    hipMemcpy(dA, A.data(), sizeof(double) * A.size(), hipMemcpyHostToDevice);
    hipMemcpy(dB, B.data(), sizeof(double) * B.size(), hipMemcpyHostToDevice);
    hipLaunchKernelGGL((k_probe<M, N, K>), dim3(1), dim3(64), 0, 0, dA, dB, dCv, dCm, dc, 200);
    hipDeviceSynchronize();
    std::vector<double> Cv(M * N), Cm(M * N);
    long long c[2];
    hipMemcpy(Cv.data(), dCv, sizeof(double) * M * N, hipMemcpyDeviceToHost);
    hipMemcpy(Cm.data(), dCm, sizeof(double) * M * N, hipMemcpyDeviceToHost);
    hipMemcpy(c, dc, sizeof c, hipMemcpyDeviceToHost);
    double diff = 0.0, ref = 0.0;
    for (int i = 0; i < M; i++)
        for (int j = 0; j < N; j++) {
            double s = 0.0;
            for (int k = 0; k < K; k++) s += A[i * K + k] * B[k * N + j];
            diff = std::fmax(diff, std::fabs(Cm[i * N + j] - Cv[i * N + j]));
            ref = std::fmax(ref, std::fabs(Cv[i * N + j] - s));
        }
    printf("%-28s M=%2d N=%2d K=%2d  VALU %6lld cycles  MFMA %6lld cycles  |MFMA-VALU| %.2e  |VALU-host| %.2e\n", what,
           M, N, K, c[0], c[1], diff, ref);
    hipFree(dA); hipFree(dB); hipFree(dCv); hipFree(dCm); hipFree(dc);
}

int main() {
    run<12, 7, 12>("C1/C5: P B (nx x nu)");
    run<12, 12, 12>("C1/C5: P A (nx x nx)");
    run<7, 7, 12>("C1/C5: B^T (P B)");
    run<24, 18, 24>("C3: P B (nx x nu)");
    run<24, 24, 24>("C3: P A (nx x nx)");
    run<18, 18, 24>("C3: B^T (P B) (nu x nu)");
    run<42, 42, 19>("C3: J_I^T D J_I (nv x nv)");
    run<28, 20, 28>("C4: P B");
    run<48, 48, 14>("C4: J_I^T D J_I");
    return 0;
}
