// Null-space solve of one Riccati stage block.
//
// Stage k of the backward recursion solves
//     [ Q  D^T ] [u]   [b_u]        Q = Q_uu (NU x NU), controls u = (qd_0..qd_{NJ-1}, F_0..),
//     [ D   0  ] [l] = [b_l]        D = h Jl_{k+1} on the qd columns, 0 on the force columns,
// for NJ + 1 right-hand sides (the NJ columns of -[Q_ux; Jl_{k+1}] and -[q_u; e_k]), and
// must report whether the block has inertia (NU, 2).  The pivoted Bunch-Kaufman path
// (bk_wave.hpp) does this with nine dependent pivot steps, each a cross-lane exchange.
// Here the two constraint rows are eliminated first, through a 2 x 2 block D_J of D
// picked by partial pivoting (columns j1, j2 of the joint velocities):
//     Z = [ -D_J^{-1} D_R ; I ]  (NU x NR, NR = NU - 2, R = the other controls)
// spans null(D).  With the block pivot [[Q_JJ, D_J^T], [D_J, 0]] (inertia (2, 2) for any
// invertible D_J) Haynsworth additivity gives
//     inertia(K) = (2, 2) + inertia(Z^T Q Z),
// so K has inertia (NU, 2) exactly when the reduced Hessian S = Z^T Q Z (NR x NR) is
// positive definite, i.e. when its LDL^T without pivoting has positive pivots.  That is
// the same exact test as the pivoted factorisation of K, with a fixed elimination order:
//   * one lane per entry forms the lane-uniform tables Z_JR, Q_JR, Q_JJ in LDS, then 25 lanes form
//     S entry-wise from them (the stage solve is FP64-issue bound: shared quantities are formed once);
//   * every lane factors S redundantly in registers (no cross-lane traffic);
//   * lane c solves right-hand side c:  u_p = D_J^{-1} b_l on J, u_R = S^{-1} Z^T (b_u - Q u_p),
//     u_J = u_p,J + Z_JR u_R,  l = D_J^{-T} (b_u,J - (Q u)_J).
// Degenerate constraint blocks (D_J numerically singular) and dc > 0 stay with the pivoted
// path (the caller decides).  The result lands in Rk in the pivoted path's block-row order
// (force rows first, then joint velocities, then the two multipliers).
#pragma once
#include <hip/hip_runtime.h>

namespace mf {

// 1/d to about one ulp: v_rcp_f64 and two Newton steps (a handful of FP64 instructions where a
// correctly rounded division takes about ten; the stage solve is FP64-issue bound)
__device__ __forceinline__ double rcp_nr(double d) {
    double r = __builtin_amdgcn_rcp(d);
    double e = fma(-d, r, 1.0);
    r = fma(r, e, r);
    e = fma(-d, r, 1.0);
    return fma(r, e, r);
}

// returns 1: solved, inertia (NU, 2); 0: wrong inertia; -1: degenerate (use the pivoted path).
// Ss5: LDS scratch of NR * NR + 4 * NR + 3 doubles (reduced Hessian, then the Z / Q tables).
template <int NJ, int NF, int NV, int NRK>
__device__ __forceinline__ int stage_nullspace(const double *Hs, const double *Ps, const double *ss, const double *Gl,
                                               const double *gsk, const double *elk, double h, double *Ss5,
                                               double *Rk) {
    constexpr int NU = NJ + NF, NR = NU - 2;
    const int lane = lane_opaque();
    const double hh = h * h;
    // Q entry (controls x, y; x, y < NJ are joint velocities)
    auto Qe = [&](int x, int y) {
        double v = Hs[(NJ + x) * NV + NJ + y];
        if (x < NJ && y < NJ) v += hh * Ps[x * NJ + y];
        return v;
    };
    auto Dc = [&](int l, int x) { return x < NJ ? h * Gl[l * NJ + x] : 0.0; };
    // ---- pivot columns of D (partial pivoting; ties keep the smallest index).  D = h Jl on the
    // joint velocities: the pivot order depends on Jl alone (h > 0), and the second pivot compares
    // |Jl1_j Jl0_j1 - Jl1_j1 Jl0_j| = |Jl0_j1| |(D_1j - f D_0j) / h| without the division by Jl0_j1.
    int j1 = 0;
    double m1 = fabs(Gl[0]);
#pragma unroll
    for (int j = 1; j < NJ; j++) {
        const double a = fabs(Gl[j]);
        if (a > m1) { m1 = a; j1 = j; }
    }
    const double g0 = Gl[j1], g1 = Gl[NJ + j1];
    int j2 = -1;
    double m2 = 0.0;
    if (m1 > 0.0) {
#pragma unroll
        for (int j = 0; j < NJ; j++) {
            if (j == j1) continue;
            const double a = fabs(Gl[NJ + j] * g0 - g1 * Gl[j]);
            if (a > m2) { m2 = a; j2 = j; }
        }
    }
    if (!(m1 > 0.0) || j2 < 0 || !(m2 > 1e-10 * m1 * m1)) return -1;
    const int J0 = j1, J1 = j2;
    const double d0j1 = h * g0, d1j1 = h * g1;
    const double a00 = d0j1, a01 = h * Gl[J1], a10 = d1j1, a11 = h * Gl[NJ + J1];
    const double det = a00 * a11 - a01 * a10;
    const double rdet = 1.0 / det;
    const double i00 = a11 * rdet, i01 = -a01 * rdet, i10 = -a10 * rdet, i11 = a00 * rdet;  // D_J^{-1}
    const int lo = J0 < J1 ? J0 : J1, hi = J0 < J1 ? J1 : J0;
    auto Ridx = [&](int m) {
        if (m >= NJ - 2) return NJ + (m - (NJ - 2));  // force controls
        int x = m;
        if (x >= lo) x++;
        if (x >= hi) x++;
        return x;
    };
    // ---- lane-uniform tables, one entry per lane (every stage quantity the right-hand sides share is
    // formed once, not per lane and per use): Z_JR = -D_J^{-1} D[:, R] (2 x NR), Q_JR (2 x NR),
    // Q_JJ (q00, q01, q11).  Each lane evaluates both candidate forms and keeps its own.
    double *Zt = Ss5 + NR * NR, *QJ = Zt + 2 * NR, *QJJ = QJ + 2 * NR;
    if (lane < 4 * NR + 3) {
        const int t = lane < 2 * NR ? lane : (lane < 4 * NR ? lane - 2 * NR : 0);
        const int r = t / NR, m = t % NR;
        const int x = Ridx(m);
        const double e0 = Dc(0, x), e1 = Dc(1, x);
        const double zv = -((r == 0 ? i00 : i10) * e0 + (r == 0 ? i01 : i11) * e1);
        // Q entry: (J_r, R_m) for the Q_JR lanes, (J0,J0), (J0,J1), (J1,J1) for the last three
        const int u = lane - 4 * NR;
        const int qa = lane < 4 * NR ? (r == 0 ? J0 : J1) : (u < 2 ? J0 : J1);
        const int qb = lane < 4 * NR ? x : (u == 0 ? J0 : J1);
        const double qv = Qe(qa, qb);
        Ss5[NR * NR + lane] = lane < 2 * NR ? zv : qv;
    }
    wave_lds_sync();
    const double q00 = QJJ[0], q01 = QJJ[1], q11 = QJJ[2];
    // ---- reduced Hessian S = Z^T Q Z, one entry per lane (Q symmetric: Q_{R,J} = Q_{J,R})
    if (lane < NR * NR) {
        const int a = lane / NR, b = lane % NR;
        const double za0 = Zt[a], za1 = Zt[NR + a], zb0 = Zt[b], zb1 = Zt[NR + b];
        double s = Qe(Ridx(a), Ridx(b));
        s += za0 * QJ[b] + za1 * QJ[NR + b];
        s += QJ[a] * zb0 + QJ[NR + a] * zb1;
        s += za0 * (q00 * zb0 + q01 * zb1) + za1 * (q01 * zb0 + q11 * zb1);
        Ss5[lane] = s;
    }
    wave_lds_sync();
    // ---- LDL^T of S, redundantly in every lane (lower triangle of S is read)
    // LD[i][j] = L[i][j] d_j is the unscaled column entry itself: one FMA per update term
    double L[NR][NR], LD[NR][NR], di[NR];
    bool pd = true;
#pragma unroll
    for (int j = 0; j < NR; j++) {
        double dj = Ss5[j * NR + j];
#pragma unroll
        for (int k = 0; k < j; k++) dj -= L[j][k] * LD[j][k];
        pd = pd && (dj > 0.0);
        di[j] = rcp_nr(dj);
#pragma unroll
        for (int i = j + 1; i < NR; i++) {
            double v = Ss5[i * NR + j];
#pragma unroll
            for (int k = 0; k < j; k++) v -= L[i][k] * LD[j][k];
            LD[i][j] = v;
            L[i][j] = v * di[j];
        }
    }
    if (!pd) return 0;
    // ---- right-hand side c per lane
    auto brow = [&](int x) { return x < NJ ? x + NF : x - NJ; };  // control -> block row of Rk
    if (lane < NRK) {
        const int c = lane;
        // right-hand side columns: -[Q_ux | q_u] (c < NJ: column c of Q_ux, c = NJ: q_u), the same
        // instructions for every lane through per-lane base pointers and strides
        const bool cq = c < NJ;
        const double *hb = cq ? Hs + NJ * NV + c : gsk + NJ, *pb = cq ? Ps + c : ss, *gb = cq ? Gl + c : elk;
        const int hst = cq ? NV : 1, pst = cq ? NJ : 1, gst = cq ? NJ : 1;
        auto bu = [&](int x) { return -(hb[x * hst] + (x < NJ ? h * pb[x * pst] : 0.0)); };
        const double bl0 = -gb[0];
        const double bl1 = -gb[gst];
        const double up0 = i00 * bl0 + i01 * bl1, up1 = i10 * bl0 + i11 * bl1;
        const double bJ0 = bu(J0), bJ1 = bu(J1);
        const double rJ0 = bJ0 - q00 * up0 - q01 * up1;
        const double rJ1 = bJ1 - q01 * up0 - q11 * up1;
        double y[NR];
#pragma unroll
        for (int m = 0; m < NR; m++)
            y[m] = bu(Ridx(m)) - QJ[m] * up0 - QJ[NR + m] * up1 + Zt[m] * rJ0 + Zt[NR + m] * rJ1;
#pragma unroll
        for (int i = 0; i < NR; i++)
#pragma unroll
            for (int k = 0; k < i; k++) y[i] -= L[i][k] * y[k];
#pragma unroll
        for (int i = 0; i < NR; i++) y[i] *= di[i];
#pragma unroll
        for (int i = NR - 1; i >= 0; i--)
#pragma unroll
            for (int k = i + 1; k < NR; k++) y[i] -= L[k][i] * y[k];
        double uJ0 = up0, uJ1 = up1, sJ0 = 0.0, sJ1 = 0.0;
#pragma unroll
        for (int m = 0; m < NR; m++) {
            uJ0 += Zt[m] * y[m];
            uJ1 += Zt[NR + m] * y[m];
            sJ0 += QJ[m] * y[m];
            sJ1 += QJ[NR + m] * y[m];
        }
        const double t0 = bJ0 - q00 * uJ0 - q01 * uJ1 - sJ0, t1 = bJ1 - q01 * uJ0 - q11 * uJ1 - sJ1;
        // D_J^T l = t  ->  l = D_J^{-T} t
        const double l0 = i00 * t0 + i10 * t1, l1 = i01 * t0 + i11 * t1;
#pragma unroll
        for (int m = 0; m < NR; m++) Rk[brow(Ridx(m)) * NRK + c] = y[m];
        Rk[brow(J0) * NRK + c] = uJ0;
        Rk[brow(J1) * NRK + c] = uJ1;
        Rk[NU * NRK + c] = l0;
        Rk[(NU + 1) * NRK + c] = l1;
    }
    wave_lds_sync();
    return 1;
}

}  // namespace mf
