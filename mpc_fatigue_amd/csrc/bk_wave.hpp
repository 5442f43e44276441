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
// reductions over aligned W-lane segments of the wave (W = 64: the whole wave); kernels that
// give each horizon half a wave reduce with W = 32 and never mix the two halves
template <int W> __device__ __forceinline__ double hw_sum(double x) {
#pragma unroll
    for (int off = W / 2; off > 0; off >>= 1) x += __shfl_xor(x, off, W);
    return x;
}
template <int W> __device__ __forceinline__ double hw_max(double x) {
#pragma unroll
    for (int off = W / 2; off > 0; off >>= 1) x = fmax(x, __shfl_xor(x, off, W));
    return x;
}
template <int W> __device__ __forceinline__ double hw_min(double x) {
#pragma unroll
    for (int off = W / 2; off > 0; off >>= 1) x = fmin(x, __shfl_xor(x, off, W));
    return x;
}
template <int W> __device__ __forceinline__ int hw_sumi(int x) {
#pragma unroll
    for (int off = W / 2; off > 0; off >>= 1) x += __shfl_xor(x, off, W);
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

// The workgroups that use these routines are exactly one wavefront (64 lanes in lockstep),
// so ordering LDS traffic only needs the wave's own LDS operations to have completed:
// s_waitcnt lgkmcnt(0) plus a compiler memory barrier.  __syncthreads() is a workgroup
// release fence and also waits for vmcnt(0) while global stores are outstanding -- and vmcnt
// retires in order, so it would drain every register prefetch in flight as well.
// The lane index as a value the compiler cannot prove loop-invariant: index arithmetic derived
// from it is recomputed where it is used instead of being hoisted out of the serial stage loops
// and held in registers across them (occupancy of the Riccati kernels).
__device__ __forceinline__ int lane_opaque() {
    int l = threadIdx.x;
    __asm__ volatile("" : "+v"(l));
    return l;
}
__device__ __forceinline__ void wave_lds_sync() { __asm__ volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); }
// all of the wave's memory operations (global stores read back by other lanes, LDS) complete
__device__ __forceinline__ void wave_mem_sync() { __asm__ volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory"); }

struct BKInertia {
    int pos, neg, zero;
};

// max of M values as a tree of fmax (log2 M dependent steps)
template <int M>
__device__ __forceinline__ double tree_max(const double (&v)[M]) {
    double t[M];
#pragma unroll
    for (int i = 0; i < M; i++) t[i] = v[i];
#pragma unroll
    for (int st = 1; st < M; st *= 2)
#pragma unroll
        for (int i = 0; i + st < M; i += 2 * st) t[i] = fmax(t[i], t[i + st]);
    return t[0];
}

// perm/piv: LDS int arrays of length >= m.
template <int LD>
__device__ __forceinline__ BKInertia bk_factor_wave(double *A, int m, int *perm, int *piv, int k0 = 0,
                                                     BKInertia in0 = BKInertia{0, 0, 0}) {
    // k0 > 0: columns 0..k0-1 were already eliminated with 1x1 pivots in natural order (bk_factor_regs<.., K0>),
    // their inertia is in0 and perm / piv of those rows are set; the factorisation continues at column k0
    const int lane = lane_opaque();
    const double alpha = (1.0 + sqrt(17.0)) / 8.0;
    BKInertia in = in0;
    for (int i = lane + k0; i < m; i += 64) perm[i] = i;
    __syncthreads();
    int k = k0;
    while (k < m) {
        // pivot search: every lane scans the (<= m) candidates itself from LDS broadcast reads --
        // a serial scan of a short column is far cheaper than a 64-lane shuffle reduction
        // (ds_bpermute round trips); ties keep the smallest index, like a sequential idamax
        double colmax = 0.0;
        int imax = k;
        if (m <= 64) {
            // lane i holds |A_ik| of its row; the wave argmax keeps the smallest index among ties and
            // index k when the column is zero: the result of the sequential strict-> scan below
            colmax = (lane > k && lane < m) ? fabs(A[lane * LD + k]) : 0.0;
            imax = (lane > k && lane < m) ? lane : k;
            wave_argmax(colmax, imax);
        } else {
            for (int i = k + 1; i < m; i++) {
                double a = fabs(A[i * LD + k]);
                if (a > colmax) { colmax = a; imax = i; }
            }
        }
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
            double rowmax = 0.0;
            if (m <= 64) {
                rowmax = (lane >= k && lane < m && lane != imax) ? fabs(A[imax * LD + lane]) : 0.0;
                rowmax = wave_max(rowmax);
            } else {
                for (int j = k; j < m; j++)
                    if (j != imax) rowmax = fmax(rowmax, fabs(A[imax * LD + j]));
            }
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
                    double val = fma(-(ci * inv), cj, A[i * LD + j]);
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
            double det = fma(a, c, -(b * b));
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
                    double l0 = fma(c0i, ia, c1i * ib), l1 = fma(c0i, ib, c1i * ic);
                    double val = A[i * LD + j] - fma(l0, c0j, l1 * c1j);
                    A[i * LD + j] = val;
                    A[j * LD + i] = val;
                }
            }
            __syncthreads();
            for (int i = k + 2 + lane; i < m; i += 64) {
                double c0i = A[i * LD + k], c1i = A[i * LD + k + 1];
                double l0 = fma(c0i, ia, c1i * ib), l1 = fma(c0i, ib, c1i * ic);
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

// Same factorisation with a compile-time size M <= 64: the pivot scans are unrolled, so their
// LDS reads issue back to back instead of one dependent round trip per candidate.
template <int LD, int M>
__device__ __forceinline__ BKInertia bk_factor_fixed(double *A, int *perm, int *piv) {
    const int lane = lane_opaque();
    const double alpha = (1.0 + sqrt(17.0)) / 8.0;
    BKInertia in{0, 0, 0};
    if (lane < M) perm[lane] = lane;
    wave_lds_sync();
    int k = 0;
    while (k < M) {
        double cv[M];
#pragma unroll
        for (int i = 0; i < M; i++) cv[i] = A[i * LD + k];
        // the first row attaining the column maximum (the wave's argmax; k when the column is zero), by a tree of
        // fmax and one mask instead of a dependent compare-and-select chain
        double av[M];
        double absakk = 0.0;
#pragma unroll
        for (int i = 0; i < M; i++) {
            av[i] = (i > k) ? fabs(cv[i]) : 0.0;
            if (i == k) absakk = fabs(cv[i]);
        }
        const double colmax = tree_max(av);
        unsigned hit = 0;
#pragma unroll
        for (int i = 1; i < M; i++) hit |= (i > k && av[i] == colmax) ? 1u << i : 0u;
        const int imax = colmax > 0.0 ? __builtin_ctz(hit) : k;
        int kstep = 1, kp = k;
        if (fmax(absakk, colmax) == 0.0) {
            in.zero++;
            if (lane == 0) piv[k] = 1;
            k++;
            wave_lds_sync();
            continue;
        }
        if (absakk >= alpha * colmax) {
            kp = k;
        } else {
            double rv[M], ra[M];
#pragma unroll
            for (int j = 0; j < M; j++) rv[j] = A[imax * LD + j];
            double aii = 0.0;
#pragma unroll
            for (int j = 0; j < M; j++) {
                ra[j] = (j >= k && j != imax) ? fabs(rv[j]) : 0.0;
                if (j == imax) aii = fabs(rv[j]);
            }
            const double rowmax = tree_max(ra);
            if (absakk >= alpha * colmax * (colmax / rowmax)) kp = k;
            else if (aii >= alpha * rowmax) kp = imax;
            else { kp = imax; kstep = 2; }
        }
        int kk = k + kstep - 1;
        if (kp != kk) {
            wave_lds_sync();
            for (int j = lane; j < M; j += 64) {
                double t = A[kk * LD + j]; A[kk * LD + j] = A[kp * LD + j]; A[kp * LD + j] = t;
            }
            wave_lds_sync();
            for (int i = lane; i < M; i += 64) {
                double t = A[i * LD + kk]; A[i * LD + kk] = A[i * LD + kp]; A[i * LD + kp] = t;
            }
            if (lane == 0) { int t = perm[kk]; perm[kk] = perm[kp]; perm[kp] = t; }
            wave_lds_sync();
        }
        if (kstep == 1) {
            const double d = A[k * LD + k];
            if (d > 0) in.pos++; else if (d < 0) in.neg++; else in.zero++;
            const double inv = 1.0 / d;
            const int t = M - k - 1;
            for (int e = lane; e < t * t; e += 64) {
                const int i = k + 1 + e / t, j = k + 1 + e % t;
                if (j <= i) {
                    const double ci = A[i * LD + k], cj = A[j * LD + k];
                    const double val = fma(-(ci * inv), cj, A[i * LD + j]);
                    A[i * LD + j] = val;
                    A[j * LD + i] = val;
                }
            }
            wave_lds_sync();
            for (int i = k + 1 + lane; i < M; i += 64) {
                const double l = A[i * LD + k] * inv;
                A[i * LD + k] = l;
                A[k * LD + i] = l;
            }
            if (lane == 0) piv[k] = 1;
        } else {
            const double a = A[k * LD + k], bb = A[(k + 1) * LD + k], c = A[(k + 1) * LD + k + 1];
            const double det = fma(a, c, -(bb * bb));
            if (det < 0) { in.pos++; in.neg++; }
            else if (det > 0) { if (a + c > 0) in.pos += 2; else in.neg += 2; }
            else in.zero += 2;
            const double ia = c / det, ib = -bb / det, ic = a / det;
            const int t = M - k - 2;
            for (int e = lane; e < t * t; e += 64) {
                const int i = k + 2 + e / t, j = k + 2 + e % t;
                if (j <= i) {
                    const double c0i = A[i * LD + k], c1i = A[i * LD + k + 1];
                    const double c0j = A[j * LD + k], c1j = A[j * LD + k + 1];
                    const double l0 = fma(c0i, ia, c1i * ib), l1 = fma(c0i, ib, c1i * ic);
                    const double val = A[i * LD + j] - fma(l0, c0j, l1 * c1j);
                    A[i * LD + j] = val;
                    A[j * LD + i] = val;
                }
            }
            wave_lds_sync();
            for (int i = k + 2 + lane; i < M; i += 64) {
                const double c0i = A[i * LD + k], c1i = A[i * LD + k + 1];
                A[i * LD + k] = fma(c0i, ia, c1i * ib);
                A[i * LD + k + 1] = fma(c0i, ib, c1i * ic);
            }
            if (lane == 0) { piv[k] = 2; piv[k + 1] = 0; }
        }
        wave_lds_sync();
        k += kstep;
    }
    return in;
}

__device__ __forceinline__ double readlane_d(double v, int l) {
    const int lo = __builtin_amdgcn_readlane(__double2loint(v), l);
    const int hi = __builtin_amdgcn_readlane(__double2hiint(v), l);
    return __hiloint2double(hi, lo);
}

// Fast path for the stage block K = [[Q, D^T], [D, -dc]] (M = MU + ML, ML <= 2) in registers.
// Lane i keeps row i of K (symmetric) and row i of the right-hand sides B (M x NR in LDS,
// nr <= NR columns).  Q is eliminated by LDL^T with 1x1 pivots in natural order, each pivot
// accepted by the Bunch-Kaufman test |q_kk| >= alpha * max_{i>k} |q_ik| taken within Q; the
// pivot row is read with v_readlane and the forward substitution is fused into the
// elimination.  What is left in rows MU.. is the Schur complement S = -dc - D Q^{-1} D^T,
// solved as one (ML x ML) block.  By Haynsworth additivity inertia(K) = inertia(Q) +
// inertia(S), so the inertia test is the same exact test as a pivoted factorisation of K.
// On success the solution overwrites B; if a pivot fails the test (or S is singular) it
// returns false with A and B untouched and the caller runs the pivoted LDS path.
template <int LD, int NR, int MU, int ML>
__device__ bool ldl_schur_regs(const double *A, double *B, int nr, BKInertia &in) {
    constexpr int M = MU + ML;
    static_assert(ML <= 2, "Schur block of at most 2 rows");
    const int lane = lane_opaque();
    const double alpha = (1.0 + sqrt(17.0)) / 8.0;
    double a[M], y[NR];
#pragma unroll
    for (int j = 0; j < M; j++) a[j] = (lane < M) ? A[lane * LD + j] : 0.0;
#pragma unroll
    for (int c = 0; c < NR; c++) y[c] = (lane < M && c < nr) ? B[lane * NR + c] : 0.0;
    int pos = 0, neg = 0;
    bool ok = true;
#pragma unroll
    for (int k = 0; k < MU; k++) {
        if (ok) {
            double colmax = 0.0;
#pragma unroll
            for (int i = k + 1; i < MU; i++) colmax = fmax(colmax, fabs(readlane_d(a[k], i)));
            const double d = readlane_d(a[k], k);
            if (!(fabs(d) >= alpha * colmax) || d == 0.0) {
                ok = false;
            } else {
                if (d > 0) pos++; else neg++;
                const double inv = 1.0 / d;
                double r[M], yk[NR];
#pragma unroll
                for (int j = k + 1; j < M; j++) r[j] = readlane_d(a[j], k);
#pragma unroll
                for (int c = 0; c < NR; c++) yk[c] = readlane_d(y[c], k);
                if (lane > k && lane < M) {
                    const double l = a[k] * inv;
#pragma unroll
                    for (int j = k + 1; j < M; j++) a[j] = a[j] - l * r[j];
                    a[k] = l;
#pragma unroll
                    for (int c = 0; c < NR; c++) y[c] -= l * yk[c];
                }
            }
        }
    }
    if (!ok) return false;
    // Schur block: inertia and x_S = S^{-1} y_S (rows MU..M-1)
    if (ML == 1) {
        const double s00 = readlane_d(a[MU], MU);
        if (s00 == 0.0) return false;
        if (s00 > 0) pos++; else neg++;
        if (lane == MU)
#pragma unroll
            for (int c = 0; c < NR; c++) y[c] = y[c] / s00;
    } else if (ML == 2) {
        const double s00 = readlane_d(a[MU], MU), s01 = readlane_d(a[MU + 1], MU), s11 = readlane_d(a[M - 1], M - 1);
        const double det = s00 * s11 - s01 * s01;
        if (det == 0.0) return false;
        if (det < 0) { pos++; neg++; }
        else if (s00 + s11 > 0) pos += 2;
        else neg += 2;
        double y0[NR], y1[NR];
#pragma unroll
        for (int c = 0; c < NR; c++) { y0[c] = readlane_d(y[c], MU); y1[c] = readlane_d(y[c], M - 1); }
        if (lane == MU)
#pragma unroll
            for (int c = 0; c < NR; c++) y[c] = (s11 * y0[c] - s01 * y1[c]) / det;
        if (lane == M - 1)
#pragma unroll
            for (int c = 0; c < NR; c++) y[c] = (s00 * y1[c] - s01 * y0[c]) / det;
    }
    // D^{-1} on the Q rows, then L^T x = y from the last row up; lane t (< MU) keeps the unscaled
    // column t of the eliminated matrix in a[t+1..], so L_it = a[i] / d_t
    double dinv = 0.0;
#pragma unroll
    for (int j = 0; j < MU; j++)
        if (j == lane) dinv = 1.0 / a[j];
    if (lane < MU)
#pragma unroll
        for (int c = 0; c < NR; c++) y[c] *= dinv;
#pragma unroll
    for (int i = M - 1; i > 0; i--) {
        double xi[NR];
#pragma unroll
        for (int c = 0; c < NR; c++) xi[c] = readlane_d(y[c], i);
        if (lane < i && lane < MU) {
            const double lit = a[i] * dinv;
#pragma unroll
            for (int c = 0; c < NR; c++) y[c] -= lit * xi[c];
        }
    }
    if (lane < M)
#pragma unroll
        for (int c = 0; c < NR; c++)
            if (c < nr) B[lane * NR + c] = y[c];
    wave_lds_sync();
    in.pos = pos;
    in.neg = neg;
    in.zero = 0;
    return true;
}

// Solve A X = B for nr <= 64 right-hand sides with a compile-time size M: lane c owns column c
// of B (m x NR row-major in LDS) in registers and runs both triangular sweeps itself, reading
// the factor by LDS broadcast; no cross-lane traffic and a single barrier.  The L column t
// acts on rows >= t + 1, or >= t + 2 when t opens a 2x2 pivot (its partner row belongs to D).
template <int LD, int NR, int M>
__device__ __forceinline__ void bk_solve_cols(const double *A, const int *perm, const int *piv, double *B, int nr) {
    const int c = lane_opaque();
    double y[M];
    int pv[M];
    if (c < nr) {
#pragma unroll
        for (int i = 0; i < M; i++) {
            pv[i] = piv[i];
            y[i] = B[perm[i] * NR + c];
        }
#pragma unroll
        for (int t = 0; t < M; t++) {
            const int start = t + 1 + (pv[t] == 2 ? 1 : 0);
#pragma unroll
            for (int i = t + 1; i < M; i++)
                if (i >= start) y[i] -= A[i * LD + t] * y[t];
        }
#pragma unroll
        for (int i = 0; i < M; i++) {
            if (pv[i] == 1) {
                y[i] = y[i] / A[i * LD + i];
            } else if (pv[i] == 2 && i + 1 < M) {
                const double a = A[i * LD + i], bb = A[(i + 1) * LD + i], cc = A[(i + 1) * LD + i + 1];
                const double det = a * cc - bb * bb;
                const double y0 = y[i], y1 = y[i + 1];
                y[i] = (cc * y0 - bb * y1) / det;
                y[i + 1] = (a * y1 - bb * y0) / det;
            }
        }
#pragma unroll
        for (int t = M - 1; t >= 0; t--) {
            const int start = t + 1 + (pv[t] == 2 ? 1 : 0);
            double acc = y[t];
#pragma unroll
            for (int i = t + 1; i < M; i++)
                if (i >= start) acc -= A[i * LD + t] * y[i];
            y[t] = acc;
        }
    }
    wave_lds_sync();  // every lane has read the factor and B before B is overwritten
    if (c < nr) {
#pragma unroll
        for (int i = 0; i < M; i++) B[perm[i] * NR + c] = y[i];
    }
    wave_lds_sync();
}

// LU factorisation with partial pivoting of an n x n matrix in LDS (n <= 64, one row per lane), the order of
// oracle/mf_ocp.c lu_factor (LAPACK getf2): at column c the row of largest |M_rc|, r >= c (the smallest index
// among ties), is swapped in whole, then rows r > c take the multiplier M_rc / M_cc and the update of their
// columns > c.  pi[i] = the original row now at row i (the product of the interchanges).  Returns 1 when a pivot
// column is exactly zero (M is then partly factored).
template <int LD>
__device__ __forceinline__ int lu_factor_wave(double *M, int n, int *pi) {
    const int lane = lane_opaque();
    if (lane < n) pi[lane] = lane;
    __syncthreads();
    for (int c = 0; c < n; c++) {
        double v = (lane >= c && lane < n) ? fabs(M[lane * LD + c]) : -1.0;
        int idx = (lane >= c && lane < n) ? lane : 64;
        wave_argmax(v, idx);
        const int pr = idx;
        if (M[pr * LD + c] == 0.0) return 1;
        if (pr != c) {
            for (int j = lane; j < n; j += 64) {
                const double t = M[c * LD + j];
                M[c * LD + j] = M[pr * LD + j];
                M[pr * LD + j] = t;
            }
            if (lane == 0) { const int t = pi[c]; pi[c] = pi[pr]; pi[pr] = t; }
            __syncthreads();
        }
        if (lane > c && lane < n) {
            const double f = M[lane * LD + c] / M[c * LD + c];
            M[lane * LD + c] = f;
            for (int j = c + 1; j < n; j++) M[lane * LD + j] -= f * M[c * LD + j];
        }
        __syncthreads();
    }
    return 0;
}

// lu_factor_wave with the matrix in registers (compile-time M <= 64): lane r keeps original row r for the whole
// factorisation and `at` = the position it has reached (the oracle swaps whole rows; here only positions move).  At
// column c the pivot is the row of largest |value| among positions >= c, the smallest position among ties (the
// sequential scan's choice); its values reach the other lanes by v_readlane, and the rows at positions > c take the
// multiplier and the update in the same order as lu_factor_wave.  Writes the factor to M (row `at` of lane r) and pi
// (pi[at] = r); returns 1 on an exactly zero pivot column (M, pi then unwritten).
template <int LD, int M>
__device__ __forceinline__ int lu_factor_regs(double *Mat, int *pi) {
    static_assert(M <= 64, "one row per lane");
    const int lane = lane_opaque();
    const bool act = lane < M;
    double a[M];
#pragma unroll
    for (int j = 0; j < M; j++) a[j] = Mat[min(lane, M - 1) * LD + j];
    int at = lane;
    int sing = 0;
#pragma unroll
    for (int c = 0; c < M; c++) {
        double v = (act && at >= c) ? fabs(a[c]) : -1.0;
        int idx = (act && at >= c) ? at : 64;
        wave_argmax(v, idx);  // idx: the pivot row's position
        const unsigned long long bal = __ballot(act && at == idx);
        const int pl = __builtin_ffsll((long long)bal) - 1;  // its lane
        const double p = readlane_d(a[c], pl);
        if (p == 0.0) sing = 1;
        if (sing) break;
        // the rows at positions c and idx trade places
        if (act && at == c) at = idx;
        else if (act && lane == pl) at = c;
        double pr[M];  // the pivot row, broadcast (wave-uniform)
#pragma unroll
        for (int j = c + 1; j < M; j++) pr[j] = readlane_d(a[j], pl);
        if (act && at > c) {
            const double f = a[c] / p;
            a[c] = f;
#pragma unroll
            for (int j = c + 1; j < M; j++) a[j] -= f * pr[j];
        }
    }
    if (sing) return 1;
    if (act) {
#pragma unroll
        for (int j = 0; j < M; j++) Mat[at * LD + j] = a[j];
        pi[at] = lane;
    }
    wave_lds_sync();
    return 0;
}

// y = (LU)^-1 b for the calling lane's right-hand side, b_i = b[pi[i] * bs] (the interchanges applied), in
// registers: the unit-lower sweep by columns, then the upper one (oracle/mf_ocp.c lu_solve, same order)
template <int LD, int M>
__device__ __forceinline__ void lu_solve_lane(const double *LU, const int *pi, const double *b, int bs, double *y) {
#pragma unroll
    for (int i = 0; i < M; i++) y[i] = b[pi[i] * bs];
#pragma unroll
    for (int c = 0; c < M; c++)
#pragma unroll
        for (int r = c + 1; r < M; r++) y[r] -= LU[r * LD + c] * y[c];
#pragma unroll
    for (int c = M - 1; c >= 0; c--) {
        double acc = y[c];
#pragma unroll
        for (int j = c + 1; j < M; j++) acc -= LU[c * LD + j] * y[j];
        y[c] = acc / LU[c * LD + c];
    }
}

// bk_factor_wave with the matrix in registers (lane i holds row i, M <= 64) for the common case
// where Bunch-Kaufman keeps the natural order: every pivot passes the first test
// |a_kk| >= alpha max_{i>k} |a_ik| and is non-zero.  The column of step k is broadcast with
// v_readlane and every lane updates the lower part of its own row, A_ij -= (A_ik / d_k) A_jk for
// k < j <= i, the same arithmetic in the same order as bk_factor_wave, so the factor (L below
// the diagonal, D on it; perm = identity, piv = 1) and the inertia are identical.  Returns false,
// with A, perm and piv untouched, as soon as a pivot would need the pivoted path.
// K0 < M: only columns 0..K0-1 are eliminated (the caller continues with bk_factor_wave from column K0): rows >= K0
// are written back with their multipliers and the Schur-updated trailing block in both triangles.
template <int LD, int M, int K0 = M>
__device__ __forceinline__ bool bk_factor_regs(double *A, int *perm, int *piv, BKInertia &in, int *fail_col = nullptr) {
    static_assert(K0 <= M, "K0 <= M");
    static_assert(M <= 64, "one row per lane");
    const int lane = lane_opaque();
    const double alpha = (1.0 + sqrt(17.0)) / 8.0;
    double a[M];
#pragma unroll
    for (int j = 0; j < M; j++) a[j] = A[min(lane, M - 1) * LD + j];
    int pos = 0, neg = 0;
    bool ok = true;
#pragma unroll
    for (int k = 0; k < K0; k++) {
        if (ok) {
            double r[M];
            double colmax = 0.0;
#pragma unroll
            for (int i = k + 1; i < M; i++) {
                r[i] = readlane_d(a[k], i);
                colmax = fmax(colmax, fabs(r[i]));
            }
            const double d = readlane_d(a[k], k);
            const double absakk = fabs(d);
            const bool keep = absakk >= alpha * colmax;
            if (fmax(absakk, colmax) == 0.0 || !keep) {
                ok = false;
                if (fail_col) *fail_col = k;
            } else {
                if (d > 0) pos++; else neg++;
                const double inv = 1.0 / d;
                if (lane > k && lane < M) {
                    const double ci = a[k];
#pragma unroll
                    for (int j = k + 1; j < M; j++)
                        if (j <= lane) a[j] = fma(-(ci * inv), r[j], a[j]);
                    a[k] = ci * inv;
                }
            }
        }
    }
    if (!ok) return false;
    if (lane < M) {
#pragma unroll
        for (int j = 0; j < M; j++) {
            if (j <= lane) A[lane * LD + j] = a[j];
            if (K0 < M && j >= K0 && j < lane) A[j * LD + lane] = a[j];  // trailing block: upper mirror
        }
        if (lane < K0) {
            perm[lane] = lane;
            piv[lane] = 1;
        }
    }
    wave_lds_sync();
    in.pos = pos;
    in.neg = neg;
    in.zero = 0;
    return true;
}

// bk_factor_wave in registers with its pivoting (1x1 / 2x2 pivots, symmetric row and column swaps), for M <= 64:
// lane i keeps row i of the whole matrix, the pivot searches are readlane scans (the first maximum, like the wave's
// argmax), swaps exchange two lanes' rows and two register columns, and every arithmetic operation is the wave's in
// the wave's order, so the lower triangle (L and D), perm, piv and the inertia are bit-identical to bk_factor_wave's.
// The updates are written with explicit fma in both routines: left to contraction, an update under a per-lane select
// (lower entry or mirrored one) is compiled as a select of two products and an unfused subtraction.
// The wave routine keeps both triangles: an update writes the value it computes for (i, j), i >= j, to (j, i) as
// well.  Lane i computes the upper entries of its row with the mirror's operands ((c_j / d) c_i for the 1x1 update,
// from the mirror's own l_j for the 2x2), which gives the same bits once the block is symmetric.  The block as built
// need not be symmetric to the last bit, and the first step reads it as the wave does (row imax's upper part in the
// pivot test, upper entries moved below the diagonal by a swap); after that step the trailing block is made
// symmetric by copying its lower triangle up, as the wave's first update does.
template <int M>
__device__ __forceinline__ double reg_sel(const double (&a)[M], int idx) {
    double r = a[0];
#pragma unroll
    for (int j = 1; j < M; j++) r = (idx == j) ? a[j] : r;
    return r;
}
template <int LD, int M>
__device__ __forceinline__ BKInertia bk_factor_regs_piv(double *A, int *perm, int *piv) {
    static_assert(M >= 2 && M <= 64, "one row per lane");
    const int lane = lane_opaque();
    const double alpha = (1.0 + sqrt(17.0)) / 8.0;
    double a[M];
#pragma unroll
    for (int j = 0; j < M; j++) a[j] = A[min(lane, M - 1) * LD + j];
    int pm = lane, pv = 1;
    BKInertia in{0, 0, 0};
    bool skip = false;
#pragma unroll
    for (int k = 0; k < M; k++) {
        if (skip) {
            skip = false;
            continue;
        }
        const int k1 = k + 1 < M ? k + 1 : M - 1;  // (the second column of a 2x2 pivot; never k = M - 1)
        // pivot search without a dependent compare-and-select chain: the column maximum by a tree of fmax, then the
        // first row that attains it (the wave's argmax: smallest index among ties, k when the column is zero)
        double cv[M];
#pragma unroll
        for (int i = 0; i < M; i++) cv[i] = i > k ? fabs(readlane_d(a[k], i)) : 0.0;
        const double colmax = tree_max(cv);
        unsigned hit = 0;
#pragma unroll
        for (int i = k + 1; i < M; i++) hit |= (cv[i] == colmax) ? 1u << i : 0u;
        const int imax = colmax > 0.0 ? __builtin_ctz(hit) : k;
        const double absakk = fabs(readlane_d(a[k], k));
        int kstep = 1, kp = k;
        const bool zero = fmax(absakk, colmax) == 0.0;
        if (zero) {
            in.zero++;
        } else {
            if (!(absakk >= alpha * colmax)) {
                // (the row index through an empty asm: the compiler would otherwise speculate these readlanes and the
                // division below out of the branch and pay for them at every step)
                int ir = imax;
                __asm__ volatile("" : "+s"(ir));
                double rv[M], dmax = 0.0;
#pragma unroll
                for (int j = 0; j < M; j++) {
                    const double v = j >= k ? readlane_d(a[j], ir) : 0.0;
                    rv[j] = (j >= k && j != imax) ? fabs(v) : 0.0;
                    dmax = j == imax ? v : dmax;
                }
                const double rowmax = tree_max(rv);
                if (absakk >= alpha * colmax * (colmax / rowmax)) kp = k;
                else if (fabs(dmax) >= alpha * rowmax) kp = imax;
                else { kp = imax; kstep = 2; }
            }
            int kk = k + kstep - 1;
            if (kp != kk) {
                // rows kk <-> kp (two lanes), then columns kk <-> kp (every lane), then perm
                __asm__ volatile("" : "+s"(kk), "+s"(kp));
#pragma unroll
                for (int j = 0; j < M; j++) {
                    const double vkk = readlane_d(a[j], kk), vkp = readlane_d(a[j], kp);
                    a[j] = lane == kk ? vkp : (lane == kp ? vkk : a[j]);
                }
                const double tk = reg_sel(a, kk), tp = reg_sel(a, kp);
#pragma unroll
                for (int j = 0; j < M; j++) a[j] = j == kk ? tp : (j == kp ? tk : a[j]);
                const int pk = __builtin_amdgcn_readlane(pm, kk), pp = __builtin_amdgcn_readlane(pm, kp);
                pm = lane == kk ? pp : (lane == kp ? pk : pm);
            }
            if (kstep == 1) {
                double d = readlane_d(a[k], k);
                __asm__ volatile("" : "+s"(d));  // (not speculated into the 2x2 path)
                if (d > 0) in.pos++;
                else if (d < 0) in.neg++;
                else in.zero++;
                const double inv = 1.0 / d;
                double c[M];
#pragma unroll
                for (int i = k + 1; i < M; i++) c[i] = readlane_d(a[k], i);
                if (lane > k && lane < M) {
                    const double ci = a[k];
#pragma unroll
                    for (int j = k + 1; j < M; j++) {
                        if (j <= lane) a[j] = fma(-(ci * inv), c[j], a[j]);
                        else if (k > 0) a[j] = fma(-(c[j] * inv), ci, a[j]);  // (j, lane)'s value
                    }
                    a[k] = ci * inv;
                } else if (lane == k) {
#pragma unroll
                    for (int i = k + 1; i < M; i++) a[i] = c[i] * inv;  // row k: the L column mirrored
                }
                if (lane == k) pv = 1;
            } else {
                double a2 = readlane_d(a[k], k), b = readlane_d(a[k], k1), c2 = readlane_d(a[k1], k1);
                __asm__ volatile("" : "+s"(a2), "+s"(b), "+s"(c2));  // (not speculated into the 1x1 path)
                const double det = fma(a2, c2, -(b * b));
                if (det < 0) { in.pos++; in.neg++; }
                else if (det > 0) { if (a2 + c2 > 0) in.pos += 2; else in.neg += 2; }
                else in.zero += 2;
                const double ia = c2 / det, ib = -b / det, ic = a2 / det;
                double c0[M], c1[M];
#pragma unroll
                for (int i = k + 2; i < M; i++) {
                    c0[i] = readlane_d(a[k], i);
                    c1[i] = readlane_d(a[k1], i);
                }
                if (lane >= k + 2 && lane < M) {
                    const double c0i = a[k], c1i = a[k1];
                    const double l0 = fma(c0i, ia, c1i * ib), l1 = fma(c0i, ib, c1i * ic);
#pragma unroll
                    for (int j = k + 2; j < M; j++) {
                        if (j <= lane) {
                            a[j] = a[j] - fma(l0, c0[j], l1 * c1[j]);
                        } else if (k > 0) {
                            const double l0j = fma(c0[j], ia, c1[j] * ib), l1j = fma(c0[j], ib, c1[j] * ic);
                            a[j] = a[j] - fma(l0j, c0i, l1j * c1i);  // (j, lane)'s value
                        }
                    }
                    a[k] = l0;
                    a[k1] = l1;
                }
                if (lane == k) pv = 2;
                if (lane == k1) pv = 0;
                skip = true;
            }
        }
        if (k == 0) {
            // the trailing block symmetric from its lower triangle (the wave's first update wrote both triangles),
            // through LDS: rows out, the upper part of each row back in from the columns below the diagonal
            const int t0 = 1 + (kstep == 2 ? 1 : 0);
            if (lane < M) {
#pragma unroll
                for (int j = 0; j < M; j++)
                    if (j <= lane) A[lane * LD + j] = a[j];
            }
            wave_lds_sync();
            if (lane >= t0 && lane < M) {
#pragma unroll
                for (int j = 1; j < M; j++)
                    if (j > lane) a[j] = A[j * LD + lane];
            }
            wave_lds_sync();
        }
    }
    if (lane < M) {
#pragma unroll
        for (int j = 0; j < M; j++) A[lane * LD + j] = a[j];
        perm[lane] = pm;
        piv[lane] = pv;
    }
    wave_lds_sync();
    return in;
}

// bk_factor_regs_piv with a runtime step loop: the column of step k is picked from the registers by a select chain,
// so the step body exists once (about a tenth of the unrolled routine's code).  Same operations, same bits.
template <int M>
__device__ __forceinline__ void reg_put(double (&a)[M], int idx, double v, bool on) {
#pragma unroll
    for (int j = 0; j < M; j++) a[j] = (on && idx == j) ? v : a[j];
}
template <int LD, int M>
__device__ __forceinline__ BKInertia bk_factor_regs_loop(double *A, int *perm, int *piv) {
    static_assert(M >= 2 && M <= 64, "one row per lane");
    const int lane = lane_opaque();
    const double alpha = (1.0 + sqrt(17.0)) / 8.0;
    double a[M];
#pragma unroll
    for (int j = 0; j < M; j++) a[j] = A[min(lane, M - 1) * LD + j];
    int pm = lane, pv = 1;
    BKInertia in{0, 0, 0};
    bool first = true;
    int k = 0;
#pragma unroll 1
    while (k < M) {
        double ck = reg_sel(a, k);
        double cv[M];
#pragma unroll
        for (int i = 0; i < M; i++) cv[i] = i > k ? fabs(readlane_d(ck, i)) : 0.0;
        const double colmax = tree_max(cv);
        unsigned hit = 0;
#pragma unroll
        for (int i = 1; i < M; i++) hit |= (i > k && cv[i] == colmax) ? 1u << i : 0u;
        const int imax = colmax > 0.0 ? __builtin_ctz(hit) : k;
        const double absakk = fabs(readlane_d(ck, k));
        int kstep = 1, kp = k;
        if (fmax(absakk, colmax) == 0.0) {
            in.zero++;
        } else {
            if (!(absakk >= alpha * colmax)) {
                double rv[M], dmax = 0.0;
#pragma unroll
                for (int j = 0; j < M; j++) {
                    const double v = readlane_d(a[j], imax);
                    rv[j] = (j >= k && j != imax) ? fabs(v) : 0.0;
                    dmax = j == imax ? v : dmax;
                }
                const double rowmax = tree_max(rv);
                if (absakk >= alpha * colmax * (colmax / rowmax)) kp = k;
                else if (fabs(dmax) >= alpha * rowmax) kp = imax;
                else { kp = imax; kstep = 2; }
            }
            const int kk = k + kstep - 1;
            if (kp != kk) {
#pragma unroll
                for (int j = 0; j < M; j++) {
                    const double vkk = readlane_d(a[j], kk), vkp = readlane_d(a[j], kp);
                    a[j] = lane == kk ? vkp : (lane == kp ? vkk : a[j]);
                }
                const double tk = reg_sel(a, kk), tp = reg_sel(a, kp);
#pragma unroll
                for (int j = 0; j < M; j++) a[j] = j == kk ? tp : (j == kp ? tk : a[j]);
                const int pk = __builtin_amdgcn_readlane(pm, kk), pp = __builtin_amdgcn_readlane(pm, kp);
                pm = lane == kk ? pp : (lane == kp ? pk : pm);
            }
            const bool below = lane > k + kstep - 1 && lane < M;  // rows of the trailing block
            if (kstep == 1) {
                ck = reg_sel(a, k);
                const double d = readlane_d(ck, k);
                if (d > 0) in.pos++;
                else if (d < 0) in.neg++;
                else in.zero++;
                const double inv = 1.0 / d;
#pragma unroll
                for (int j = 0; j < M; j++) {
                    const double cj = readlane_d(ck, j);
                    if (below && j > k) {
                        if (j <= lane) a[j] = fma(-(ck * inv), cj, a[j]);
                        else if (!first) a[j] = fma(-(cj * inv), ck, a[j]);
                    }
                    if (lane == k && j > k) a[j] = cj * inv;  // row k: the L column mirrored
                }
                reg_put(a, k, ck * inv, below);
                if (lane == k) pv = 1;
            } else {
                const double c0 = reg_sel(a, k), c1 = reg_sel(a, k + 1);
                const double a2 = readlane_d(c0, k), b = readlane_d(c0, k + 1), c2 = readlane_d(c1, k + 1);
                const double det = fma(a2, c2, -(b * b));
                if (det < 0) { in.pos++; in.neg++; }
                else if (det > 0) { if (a2 + c2 > 0) in.pos += 2; else in.neg += 2; }
                else in.zero += 2;
                const double ia = c2 / det, ib = -b / det, ic = a2 / det;
                const double l0 = fma(c0, ia, c1 * ib), l1 = fma(c0, ib, c1 * ic);
#pragma unroll
                for (int j = 0; j < M; j++) {
                    const double c0j = readlane_d(c0, j), c1j = readlane_d(c1, j);
                    if (below && j >= k + 2) {
                        if (j <= lane) {
                            a[j] = a[j] - fma(l0, c0j, l1 * c1j);
                        } else if (!first) {
                            const double l0j = fma(c0j, ia, c1j * ib), l1j = fma(c0j, ib, c1j * ic);
                            a[j] = a[j] - fma(l0j, c0, l1j * c1);
                        }
                    }
                }
                reg_put(a, k, l0, below);
                reg_put(a, k + 1, l1, below);
                if (lane == k) pv = 2;
                if (lane == k + 1) pv = 0;
            }
        }
        if (first) {
            // the trailing block symmetric from its lower triangle (as in bk_factor_regs_piv)
            const int t0 = 1 + (kstep == 2 ? 1 : 0);
            if (lane < M) {
#pragma unroll
                for (int j = 0; j < M; j++)
                    if (j <= lane) A[lane * LD + j] = a[j];
            }
            wave_lds_sync();
            if (lane >= t0 && lane < M) {
#pragma unroll
                for (int j = 1; j < M; j++)
                    if (j > lane) a[j] = A[j * LD + lane];
            }
            wave_lds_sync();
            first = false;
        }
        k += kstep;
    }
    if (lane < M) {
#pragma unroll
        for (int j = 0; j < M; j++) A[lane * LD + j] = a[j];
        perm[lane] = pm;
        piv[lane] = pv;
    }
    wave_lds_sync();
    return in;
}

// Solve A X = B for nr right-hand sides; B is m x NR (row-major, LD NR) in LDS.
// Y: LDS scratch m x NR.
template <int LD, int NR>
__device__ __forceinline__ void bk_solve_wave(const double *A, int m, const int *perm, const int *piv, double *B, int nr, double *Y) {
    const int lane = lane_opaque();
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


// The same solve with one lane per right-hand-side column (nr <= 64): each lane runs the forward
// substitution, the D solve and the back substitution of its own column in the order of
// bk_solve_wave (so the results are identical), with no wave barrier between the pivot steps.
// B and Y: row-major with leading dimension NR; lane c touches column c only.
template <int LD, int NR>
__device__ void bk_solve_cols_lane(const double *A, int m, const int *perm, const int *piv, double *B, int nr,
                                   double *Y) {
    const int c = lane_opaque();
    if (c < nr) {
        for (int i = 0; i < m; i++) Y[i * NR + c] = B[perm[i] * NR + c];
        for (int k = 0; k < m;) {
            const int s = piv[k] == 2 ? 2 : 1;
            for (int i = k + s; i < m; i++) {
                double y = Y[i * NR + c];
                for (int t = 0; t < s; t++) y -= A[i * LD + k + t] * Y[(k + t) * NR + c];
                Y[i * NR + c] = y;
            }
            k += s;
        }
        for (int i = 0; i < m; i++) {
            if (piv[i] == 2) {
                const double a = A[i * LD + i], bb = A[(i + 1) * LD + i], cc = A[(i + 1) * LD + i + 1];
                const double det = a * cc - bb * bb;
                const double y0 = Y[i * NR + c], y1 = Y[(i + 1) * NR + c];
                Y[i * NR + c] = (cc * y0 - bb * y1) / det;
                Y[(i + 1) * NR + c] = (a * y1 - bb * y0) / det;
            } else if (piv[i] == 1) {
                Y[i * NR + c] = Y[i * NR + c] / A[i * LD + i];
            }
        }
        for (int k = m - 1; k >= 0;) {
            const int k0 = (k > 0 && piv[k] == 0) ? k - 1 : k;
            const int s = k - k0 + 1;
            for (int t = 0; t < s; t++) {
                double acc = Y[(k0 + t) * NR + c];
                for (int i = k0 + s; i < m; i++) acc -= A[i * LD + k0 + t] * Y[i * NR + c];
                Y[(k0 + t) * NR + c] = acc;
            }
            k = k0 - 1;
        }
        for (int i = 0; i < m; i++) B[perm[i] * NR + c] = Y[i * NR + c];
    }
    __syncthreads();
}

// C(i, j) = init(i, j) + sum_{l < KK} fa(l, i) fb(l, j) for i < M, j < NN from LDS operands: each lane
// a TR x TC register tile, the operands of one l loaded once per tile.  Per entry the sum runs over l in
// order from init, the arithmetic of the per-entry loop `v = init; for l: v += fa * fb` it replaces.
template <int M, int NN, int KK, class Init, class FA, class FB, class Out>
__device__ __forceinline__ void tile_gemm(int lane, Init init, FA fa, FB fb, Out out) {
    constexpr int TR = (M + 7) / 8, TC = (NN + 7) / 8;
    constexpr int BR = (M + TR - 1) / TR, BC = (NN + TC - 1) / TC;
    static_assert(BR * BC <= 64, "tile grid larger than a wavefront");
    if (lane < BR * BC) {
        const int r0 = (lane / BC) * TR, c0 = (lane % BC) * TC;
        double acc[TR][TC];
#pragma unroll
        for (int i = 0; i < TR; i++)
#pragma unroll
            for (int j = 0; j < TC; j++) acc[i][j] = init(min(r0 + i, M - 1), min(c0 + j, NN - 1));
#pragma unroll 2
        for (int l = 0; l < KK; l++) {
            double av[TR], bv[TC];
#pragma unroll
            for (int i = 0; i < TR; i++) av[i] = fa(l, min(r0 + i, M - 1));
#pragma unroll
            for (int j = 0; j < TC; j++) bv[j] = fb(l, min(c0 + j, NN - 1));
#pragma unroll
            for (int i = 0; i < TR; i++)
#pragma unroll
                for (int j = 0; j < TC; j++) acc[i][j] += av[i] * bv[j];
        }
#pragma unroll
        for (int i = 0; i < TR; i++)
#pragma unroll
            for (int j = 0; j < TC; j++)
                if (r0 + i < M && c0 + j < NN) out(r0 + i, c0 + j, acc[i][j]);
    }
}

}  // namespace mf
