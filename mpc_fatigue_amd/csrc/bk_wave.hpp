// One-wavefront (64-lane) symmetric-indefinite LDL^T with Bunch-Kaufman
// pivoting on a small dense matrix held in LDS, plus a multi-RHS solve.
//
// Pivoting rule: LAPACK dsytf2 (alpha = (1+sqrt 17)/8), applied with full
// symmetric row/column swaps so that P A P^T = L D L^T with one permutation;
// the oracle (oracle/mf_oracle.c bk_factor/bk_solve) implements the same rule
// sequentially.  The inertia of A is read off the 1x1 / 2x2 pivots
// (Sylvester), which is how the interior-point solver checks that its KKT
// matrix has the inertia (n_primal, n_dual, 0).
//
// Layout: A row-major with leading dimension LD (LDS); every phase is
// lane-parallel over matrix entries, pivot searches are wave shuffles; the
// wave is the whole workgroup, so __syncthreads() only orders LDS traffic.
#pragma once
#include <hip/hip_runtime.h>

namespace mf {

__device__ __forceinline__ double wave_sum(double x) {
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) x += __shfl_xor(x, off, 64);
    return x;
}
__device__ __forceinline__ double wave_max(double x) {
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) x = fmax(x, __shfl_xor(x, off, 64));
    return x;
}
__device__ __forceinline__ double wave_min(double x) {
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) x = fmin(x, __shfl_xor(x, off, 64));
    return x;
}
__device__ __forceinline__ int wave_sum_i(int x) {
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) x += __shfl_xor(x, off, 64);
    return x;
}
// max |value| with the smallest index among ties (matches a sequential strict-> scan)
__device__ __forceinline__ void wave_argmax(double &v, int &idx) {
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) {
        double ov = __shfl_xor(v, off, 64);
        int oi = __shfl_xor(idx, off, 64);
        if (ov > v || (ov == v && oi < idx)) { v = ov; idx = oi; }
    }
}

struct BKInertia {
    int pos, neg, zero;
};

// perm/piv: LDS int arrays of length >= m.
template <int LD>
__device__ BKInertia bk_factor_wave(double *A, int m, int *perm, int *piv) {
    const int lane = threadIdx.x;
    const double alpha = (1.0 + sqrt(17.0)) / 8.0;
    BKInertia in{0, 0, 0};
    for (int i = lane; i < m; i += 64) perm[i] = i;
    __syncthreads();
    int k = 0;
    while (k < m) {
        double v = 0.0;
        int idx = m;  // sentinel: no candidate
        for (int i = k + 1 + lane; i < m; i += 64) {
            double a = fabs(A[i * LD + k]);
            if (a > v || (a == v && idx == m)) { v = a; idx = i; }
        }
        wave_argmax(v, idx);
        double colmax = v;
        int imax = (idx == m) ? k : idx;
        double absakk = fabs(A[k * LD + k]);
        int kstep = 1, kp = k;
        if (fmax(absakk, colmax) == 0.0) {
            in.zero++;
            if (lane == 0) piv[k] = 1;
            k++;
            __syncthreads();
            continue;
        }
        if (absakk >= alpha * colmax) {
            kp = k;
        } else {
            double rv = 0.0;
            for (int j = k + lane; j < m; j += 64)
                if (j != imax) rv = fmax(rv, fabs(A[imax * LD + j]));
            double rowmax = wave_max(rv);
            if (absakk >= alpha * colmax * (colmax / rowmax)) kp = k;
            else if (fabs(A[imax * LD + imax]) >= alpha * rowmax) kp = imax;
            else { kp = imax; kstep = 2; }
        }
        int kk = k + kstep - 1;
        if (kp != kk) {
            __syncthreads();  // previous pivot's L-column writes must land before rows move
            for (int j = lane; j < m; j += 64) {
                double t = A[kk * LD + j]; A[kk * LD + j] = A[kp * LD + j]; A[kp * LD + j] = t;
            }
            __syncthreads();
            for (int i = lane; i < m; i += 64) {
                double t = A[i * LD + kk]; A[i * LD + kk] = A[i * LD + kp]; A[i * LD + kp] = t;
            }
            if (lane == 0) { int t = perm[kk]; perm[kk] = perm[kp]; perm[kp] = t; }
            __syncthreads();
        }
        if (kstep == 1) {
            double d = A[k * LD + k];
            if (d > 0) in.pos++; else if (d < 0) in.neg++; else in.zero++;
            double inv = 1.0 / d;
            // trailing update reads the (unmodified) pivot column directly
            int t = m - k - 1;
            for (int e = lane; e < t * t; e += 64) {
                int i = k + 1 + e / t, j = k + 1 + e % t;
                if (j <= i) {
                    double ci = A[i * LD + k], cj = A[j * LD + k];
                    double val = A[i * LD + j] - (ci * inv) * cj;
                    A[i * LD + j] = val;
                    A[j * LD + i] = val;
                }
            }
            __syncthreads();
            for (int i = k + 1 + lane; i < m; i += 64) {
                double l = A[i * LD + k] * inv;
                A[i * LD + k] = l;
                A[k * LD + i] = l;
            }
            if (lane == 0) piv[k] = 1;
        } else {
            double a = A[k * LD + k], b = A[(k + 1) * LD + k], c = A[(k + 1) * LD + k + 1];
            double det = a * c - b * b;
            if (det < 0) { in.pos++; in.neg++; }
            else if (det > 0) { if (a + c > 0) in.pos += 2; else in.neg += 2; }
            else in.zero += 2;
            double ia = c / det, ib = -b / det, ic = a / det;
            int t = m - k - 2;
            for (int e = lane; e < t * t; e += 64) {
                int i = k + 2 + e / t, j = k + 2 + e % t;
                if (j <= i) {
                    double c0i = A[i * LD + k], c1i = A[i * LD + k + 1];
                    double c0j = A[j * LD + k], c1j = A[j * LD + k + 1];
                    double l0 = c0i * ia + c1i * ib, l1 = c0i * ib + c1i * ic;
                    double val = A[i * LD + j] - (l0 * c0j + l1 * c1j);
                    A[i * LD + j] = val;
                    A[j * LD + i] = val;
                }
            }
            __syncthreads();
            for (int i = k + 2 + lane; i < m; i += 64) {
                double c0i = A[i * LD + k], c1i = A[i * LD + k + 1];
                double l0 = c0i * ia + c1i * ib, l1 = c0i * ib + c1i * ic;
                A[i * LD + k] = l0;
                A[i * LD + k + 1] = l1;
            }
            if (lane == 0) { piv[k] = 2; piv[k + 1] = 0; }
        }
        k += kstep;
    }
    __syncthreads();
    return in;
}

// Solve A X = B for nr right-hand sides; B is m x NR (row-major, LD NR) in LDS.
// Y: LDS scratch m x NR.
template <int LD, int NR>
__device__ void bk_solve_wave(const double *A, int m, const int *perm, const int *piv, double *B, int nr, double *Y) {
    const int lane = threadIdx.x;
    for (int e = lane; e < m * nr; e += 64) {
        int i = e / nr, c = e % nr;
        Y[i * NR + c] = B[perm[i] * NR + c];
    }
    __syncthreads();
    for (int k = 0; k < m;) {
        int s = piv[k] == 2 ? 2 : 1;
        int rows = m - k - s;
        for (int e = lane; e < rows * nr; e += 64) {
            int i = k + s + e / nr, c = e % nr;
            double y = Y[i * NR + c];
            for (int t = 0; t < s; t++) y -= A[i * LD + k + t] * Y[(k + t) * NR + c];
            Y[i * NR + c] = y;
        }
        __syncthreads();
        k += s;
    }
    for (int e = lane; e < m * nr; e += 64) {
        int i = e / nr, c = e % nr;
        if (piv[i] == 2) {
            double a = A[i * LD + i], bb = A[(i + 1) * LD + i], cc = A[(i + 1) * LD + i + 1];
            double det = a * cc - bb * bb;
            double y0 = Y[i * NR + c], y1 = Y[(i + 1) * NR + c];
            Y[i * NR + c] = (cc * y0 - bb * y1) / det;
            Y[(i + 1) * NR + c] = (a * y1 - bb * y0) / det;
        } else if (piv[i] == 1) {
            Y[i * NR + c] = Y[i * NR + c] / A[i * LD + i];
        }
    }
    __syncthreads();
    for (int k = m - 1; k >= 0;) {
        int k0 = (k > 0 && piv[k] == 0) ? k - 1 : k;
        int s = k - k0 + 1;
        for (int e = lane; e < s * nr; e += 64) {
            int t = e / nr, c = e % nr;
            double acc = Y[(k0 + t) * NR + c];
            for (int i = k0 + s; i < m; i++) acc -= A[i * LD + k0 + t] * Y[i * NR + c];
            Y[(k0 + t) * NR + c] = acc;
        }
        __syncthreads();
        k = k0 - 1;
    }
    for (int e = lane; e < m * nr; e += 64) {
        int i = e / nr, c = e % nr;
        B[perm[i] * NR + c] = Y[i * NR + c];
    }
    __syncthreads();
}

}  // namespace mf
