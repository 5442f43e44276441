// Microbenchmark: single-wavefront latencies (cycles, s_memtime = shader clock) of the operations the chain kernel's
// serial stage work is made of: a dependent FP64 FMA, a dependent FP64 division, readlane + dependent use, an LDS
// round trip, ds_bpermute, a full wave shuffle reduction.
//   hipcc -O3 --offload-arch=gfx950 tools/lat_bench.hip -o tools/lat_bench.bin
#include <hip/hip_runtime.h>

#include <cstdio>

constexpr int R = 1000;

__global__ __launch_bounds__(64) void klat(double x0, unsigned long long *cyc, double *sink) {
    __shared__ double L[64];
    const int lane = threadIdx.x;
    double x = x0 + lane * 1e-3, acc = 0;
    L[lane] = x;
    __syncthreads();
    unsigned long long t0, t1;
    // 0: dependent fma
    t0 = __builtin_amdgcn_s_memtime();
    for (int r = 0; r < R; r++) x = fma(x, 1.0000001, 1e-9);
    t1 = __builtin_amdgcn_s_memtime();
    if (lane == 0) cyc[0] = t1 - t0;
    acc += x;
    // 1: dependent division
    t0 = __builtin_amdgcn_s_memtime();
    for (int r = 0; r < R; r++) x = 1.0 / (x + 1.0);
    t1 = __builtin_amdgcn_s_memtime();
    if (lane == 0) cyc[1] = t1 - t0;
    acc += x;
    // 2: readlane -> dependent VALU use -> readlane
    t0 = __builtin_amdgcn_s_memtime();
    for (int r = 0; r < R; r++) {
        int lo = __builtin_amdgcn_readlane(__double2loint(x), r & 63);
        int hi = __builtin_amdgcn_readlane(__double2hiint(x), r & 63);
        x = fma(__hiloint2double(hi, lo), 0.5, x * 0.5);
    }
    t1 = __builtin_amdgcn_s_memtime();
    if (lane == 0) cyc[2] = t1 - t0;
    acc += x;
    // 3: LDS round trip (dependent address)
    int idx = lane;
    t0 = __builtin_amdgcn_s_memtime();
    for (int r = 0; r < R; r++) {
        double v = L[idx];
        idx = ((int)v + lane) & 63;
    }
    t1 = __builtin_amdgcn_s_memtime();
    if (lane == 0) cyc[3] = t1 - t0;
    acc += idx;
    // 4: shuffle (ds_bpermute) dependent
    t0 = __builtin_amdgcn_s_memtime();
    for (int r = 0; r < R; r++) x = __shfl_xor(x, 1, 64) * 0.5 + 0.25;
    t1 = __builtin_amdgcn_s_memtime();
    if (lane == 0) cyc[4] = t1 - t0;
    acc += x;
    // 5: LDS store + s_waitcnt + dependent load
    t0 = __builtin_amdgcn_s_memtime();
    for (int r = 0; r < R; r++) {
        L[lane] = x;
        __asm__ volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        x = L[lane ^ 1] * 0.5 + 0.25;
    }
    t1 = __builtin_amdgcn_s_memtime();
    if (lane == 0) cyc[5] = t1 - t0;
    acc += x;
    // 6: dependent sqrt
    t0 = __builtin_amdgcn_s_memtime();
    for (int r = 0; r < R; r++) x = sqrt(x + 1.0);
    t1 = __builtin_amdgcn_s_memtime();
    if (lane == 0) cyc[6] = t1 - t0;
    acc += x;
    // 7: dependent fabs/compare/select chain (argmax step)
    double m = 0;
    int im = 0;
    t0 = __builtin_amdgcn_s_memtime();
    for (int r = 0; r < R; r++) {
        const double v = fabs(x - r * 1e-6);
        if (v > m) { m = v; im = r; }
        x = x + m * 1e-12;
    }
    t1 = __builtin_amdgcn_s_memtime();
    if (lane == 0) cyc[7] = t1 - t0;
    acc += x + im;
    sink[lane] = acc;
}

int main() {
    unsigned long long *dc;
    double *ds;
    hipMalloc(&dc, 16 * 8);
    hipMalloc(&ds, 64 * 8);
    for (int rep = 0; rep < 2; rep++) hipLaunchKernelGGL(klat, dim3(1), dim3(64), 0, 0, 0.3, dc, ds);
    unsigned long long c[8];
    hipMemcpy(c, dc, sizeof c, hipMemcpyDeviceToHost);
    const char *nm[8] = {"fma f64", "div f64", "readlane+use", "lds round trip", "shfl_xor", "lds store+load",
                         "sqrt f64", "argmax step"};
    for (int i = 0; i < 8; i++) printf("%-16s %.1f cycles\n", nm[i], (double)c[i] / R);
    return 0;
}
