// Check: 16-byte LDS-DMA (global_load_lds_dwordx4) from 8-byte-aligned global addresses into an LDS destination that
// is only 8-byte aligned, against plain copies.  hipcc -O3 --offload-arch=gfx950 tools/glds16_check.hip -o tools/glds16_check.bin
#include <hip/hip_runtime.h>

#include <cstdio>
#include <vector>

__global__ __launch_bounds__(64) void kcopy(const double *src, double *out, int soff, int loff, int nd) {
    __shared__ double L[1024 + 8];
    const int lane = threadIdx.x;
    for (int e = lane; e < 1032; e += 64) L[e] = -1.0;
    __syncthreads();
    const double *s = src + soff;
    double *d = L + loff;
    const int n2 = nd & ~1;
    for (int t = 0; t < n2; t += 128)
        if (t + 2 * lane < n2)
            __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void *)(s + t + 2 * lane),
                                             (__attribute__((address_space(3))) void *)(d + t), 16, 0, 0);
    if (nd & 1) {
        const unsigned *s4 = reinterpret_cast<const unsigned *>(s + n2);
        unsigned *d4 = reinterpret_cast<unsigned *>(d + n2);
        if (lane < 2)
            __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void *)(s4 + lane),
                                             (__attribute__((address_space(3))) void *)d4, 4, 0, 0);
    }
    __asm__ volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    for (int e = lane; e < 1032; e += 64) out[e] = L[e];
}

int main() {
    std::vector<double> h(2048);
    for (int i = 0; i < 2048; i++) h[i] = 1000.0 + i;
    double *ds, *dout;
    hipMalloc(&ds, 2048 * 8);
    hipMalloc(&dout, 1032 * 8);
    hipMemcpy(ds, h.data(), 2048 * 8, hipMemcpyHostToDevice);
    int bad_total = 0;
    for (int soff : {0, 1, 3})
        for (int loff : {0, 1, 5})
            for (int nd : {1, 2, 7, 13, 128, 169, 300, 331}) {
                hipLaunchKernelGGL(kcopy, dim3(1), dim3(64), 0, 0, ds, dout, soff, loff, nd);
                std::vector<double> o(1032);
                hipMemcpy(o.data(), dout, 1032 * 8, hipMemcpyDeviceToHost);
                int bad = 0;
                for (int e = 0; e < 1032; e++) {
                    const double want = (e >= loff && e < loff + nd) ? h[soff + e - loff] : -1.0;
                    if (o[e] != want) bad++;
                }
                if (bad) printf("soff %d loff %d nd %d: %d wrong\n", soff, loff, nd, bad);
                bad_total += bad;
            }
    printf("glds16 check: %s (%d wrong entries)\n", bad_total ? "FAILED" : "ok", bad_total);
    return bad_total ? 1 : 0;
}
