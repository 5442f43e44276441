// Forward-over-reverse derivatives of one shooting node.
//
// phi(q, qd, Fw) = sum_j c_j tau_j(q, qd, Fw) + yl . p_f(q)
//   tau = RNEA(q, qd, 0) - J_f(q)^T [Fw; 0]     (force_optimization_pilz_6DOF.py:129-135)
//   p_f = frame point (the line constraint, L150-156)
//
// node_fwd_rev<T> evaluates tau, p_f and the full gradient (d phi/dq, d phi/dqd,
// d phi/dFw) in O(n): a forward Newton-Euler sweep (world frame, as dyn.hpp), then
// a reverse sweep that
//   * rebuilds the forward state of joint i-1 from joint i (R_{i-1} = R_i E_i^T RX_i^T,
//     w_{i-1} = w_i - z_i qd_i, ...), so no tape is kept;
//   * accumulates the suffix wrench (Mt, Ft) -> tau_j = z_j.Mt_j + (o_j x z_j).Ft_j;
//   * back-propagates the adjoints of the velocity / acceleration recurrences
//     (w_bar, dw_bar, a_bar) and of each link's wrench;
//   * turns the adjoints of the geometric quantities of link i (axis z_i, points
//     o_i, com c_i, frame point p_f, world inertia I_i) into q-gradients with the
//     rigid-rotation rule: a change of q_k rotates everything outboard of joint k
//     about (z_k, o_k), so
//        d phi / d q_k = z_k . (Gamma_k - o_k x Obar_k),
//        Gamma_k = sum_{i>=k} [z_i x z_bar_i + sum_points p x p_bar + rho_I,i],
//        Obar_k  = sum_{i>=k} sum_points p_bar,
//     with rho_I = (I dw) x M_bar + (I M_bar) x dw + (I w) x v_bar + (I v_bar) x w,
//     v_bar = M_bar x w, for M = ... + I dw + w x I w.
// Run with T = Dual whose tangent is the unit direction e_v, the .d parts of the
// gradient are column v of the Hessian of phi and tau.d is column v of d tau / dw:
// 13 lanes per node give tau, the Jacobian and the exact Hessian (the hyper-dual
// alternative needs 91 lanes of a 3x costlier scalar type).
//
// Register economy (one lane holds the whole sweep): inputs are produced on use by
// the In functor, results leave through the Emit visitor as soon as they exist,
// rotations are updated row by row with the Rodrigues identities
//   row_a(A [u]x) = A_a x u,   row_a(A [u]x^2) = u (u . A_a) - A_a   (|u| = 1).
#pragma once
#include "dyn.hpp"

namespace mf {

// world inertia (about the com) applied to v: R Ic R^T v
template <class TO, class TR, class TV> MF_HD void inertia_apply(TO *o, const TR *R, const double *Ic, const TV *v) {
    TO l[3], t[3];
    matT_vec(l, R, v);
    cmat_vec(t, Ic, l);
    mat_vec(o, R, t);
}

// rows of R <- rows of A (I + s K + omc K^2)   (sg = +1), or A (I - s K + omc K^2) (sg = -1)
template <class T> MF_HD void rodrigues_rows(T *R, const T *A, const double *ax, T s, T omc) {
#pragma unroll
    for (int r = 0; r < 3; r++) {
        const T *Ar = A + 3 * r;
        T t[3];
        t[0] = Ar[1] * ax[2] - Ar[2] * ax[1];
        t[1] = Ar[2] * ax[0] - Ar[0] * ax[2];
        t[2] = Ar[0] * ax[1] - Ar[1] * ax[0];
        T ad = Ar[0] * ax[0] + Ar[1] * ax[1] + Ar[2] * ax[2];
        T n0 = Ar[0] + s * t[0] + omc * (ad * ax[0] - Ar[0]);
        T n1 = Ar[1] + s * t[1] + omc * (ad * ax[1] - Ar[1]);
        T n2 = Ar[2] + s * t[2] + omc * (ad * ax[2] - Ar[2]);
        R[3 * r] = n0; R[3 * r + 1] = n1; R[3 * r + 2] = n2;
    }
}

// Two scalar types: TP for the pose quantities (functions of q only: rotations, joint origins
// and axes, com and frame points, the c-weighted axis prefix sums) and TV for everything that
// also depends on qd (twists, accelerations, wrenches, torques, all adjoints).  A lane whose
// tangent direction is a joint velocity runs TP = double, TV = Dual: the pose tangent is
// identically zero there, and its arithmetic drops to plain FP64.  TP = TV = Dual for the q
// directions, TP = TV = double for values only.
// fp: frame parent joint (-1: no frame point / external force).
// in.q(i), in.sincos(i, s, c) as TP, in.qd(i) as TV.  Fw: world force applied at p_f (zeros
// without force; a constant: the force column of the derivatives needs no tangent, k_eval_node).
// c: torque weights (NJ; indexed by the running joint, so keep it in memory, not registers),
// yl: frame-point weights (3, zero padded).  The joint loops are deliberately not
// unrolled: one iteration's working set fits in registers, six interleaved do not.
// em.frame(pf) and em.force(gFw) at the frame parent, and
// em.joint(i, tau_i, dphi/dq_i, dphi/dqd_i) during the reverse sweep (i = NJ-1 .. 0).
// ADJ = false: values only (tau, p_f), the same arithmetic without the adjoint
// statements (used by the line search and the initial slacks).
// GQ = false: no q-gradient (em.joint gets gq = 0, em.force is not called).  The gradient in qd
// needs only the adjoints of the velocity / acceleration recurrences (w_bar, dw_bar, a_bar) and
// of the wrench (M_bar = Lz, f_bar = Loz); the geometric adjoints (z_bar, o_bar, the com and
// frame-point adjoints, Gamma, Obar) feed d phi / dq alone.  A lane of a qd direction whose
// caller needs only the qd rows of its Hessian column (the q rows follow from the q lanes by
// symmetry; the force row is identically zero: d phi / dF does not depend on qd) runs GQ = false.
template <class TP, class TV> struct SweepState {
    TP R[9], o[3], Lz[3], Loz[3];                                  // pose, c-weighted axis prefix sums
    TV w[3], dw[3], a[3];                                          // twist, acceleration
    TV Mt[3], Ft[3], wb[3], dwb[3], ab[3], G[3], Ob[3];            // reverse sweep
};

// TV value of an input that may carry a tangent (a plain-double sweep takes its value)
template <class TV, class T> MF_HD TV as_tv(const T &x) {
    if constexpr (sizeof(TV) == sizeof(double)) return val(x);
    else return TV(x);
}

// forward sweep over joints i0 .. i1-1: pose, twist, acceleration; prefix Lambda
template <class TP, class TV, int NJ, bool ADJ, class In>
MF_HD void fwd_range(const DevModel &M, int i0, int i1, const In &in, const double *c, SweepState<TP, TV> &S) {
    TP(&R)[9] = S.R; TP(&o)[3] = S.o; TP(&Lz)[3] = S.Lz; TP(&Loz)[3] = S.Loz;
    TV(&w)[3] = S.w; TV(&dw)[3] = S.dw; TV(&a)[3] = S.a;
#pragma unroll 1
    for (int i = i0; i < i1; i++) {
        const DevJoint &J = joint_at(M, i);
        TP A[9], on[3], z[3];
        if (i == 0) {
#pragma unroll
            for (int k = 0; k < 9; k++) A[k] = TP(J.RX[k]);
#pragma unroll
            for (int k = 0; k < 3; k++) on[k] = TP(J.tX[k]);
        } else {
            matc_mul(A, R, J.RX);
            matc_vec(on, R, J.tX);
#pragma unroll
            for (int k = 0; k < 3; k++) on[k] = on[k] + o[k];
            TP d[3];
            TV t1[3], t2[3];
#pragma unroll
            for (int k = 0; k < 3; k++) d[k] = on[k] - o[k];
            cross3(t1, dw, d);
            cross3(t2, w, d);
            cross3(t2, w, t2);
#pragma unroll
            for (int k = 0; k < 3; k++) a[k] = a[k] + t1[k] + t2[k];
        }
        matc_vec(z, A, J.axis);
        TP s, cq;
        in.sincos(i, s, cq);
        rodrigues_rows(R, A, J.axis, s, TP(1.0) - cq);
        TV zq[3], t[3];
        const TV qdi = as_tv<TV>(in.qd(i));
#pragma unroll
        for (int k = 0; k < 3; k++) zq[k] = z[k] * qdi;
        cross3(t, w, zq);
#pragma unroll
        for (int k = 0; k < 3; k++) { dw[k] = dw[k] + t[k]; w[k] = w[k] + zq[k]; o[k] = on[k]; }
        if constexpr (ADJ) {
            TP oz[3];
            cross3(oz, o, z);
#pragma unroll
            for (int k = 0; k < 3; k++) { Lz[k] += z[k] * c[i]; Loz[k] += oz[k] * c[i]; }
        }
    }
}

// reverse sweep over joints i_hi .. i_lo (descending); the state holds joint i_hi's forward
// quantities on entry and joint i_lo - 1's on exit
template <class TP, class TV, int NJ, bool ADJ, bool GQ, class In, class Emit>
MF_HD void rev_range(const DevModel &M, const DevFrame &F, int fp, int i_hi, int i_lo, const In &in, const double *Fw,
                     const double *c, const double *yl, Emit &em, SweepState<TP, TV> &S) {
    TP(&R)[9] = S.R; TP(&o)[3] = S.o; TP(&Lz)[3] = S.Lz; TP(&Loz)[3] = S.Loz;
    TV(&w)[3] = S.w; TV(&dw)[3] = S.dw; TV(&a)[3] = S.a;
    TV(&Mt)[3] = S.Mt; TV(&Ft)[3] = S.Ft; TV(&wb)[3] = S.wb; TV(&dwb)[3] = S.dwb; TV(&ab)[3] = S.ab;
    TV(&G)[3] = S.G; TV(&Ob)[3] = S.Ob;
#pragma unroll 1
    for (int i = i_hi; i >= i_lo; i--) {
        const DevJoint &J = joint_at(M, i);
        const double m = J.m;
        const TV qdi = as_tv<TV>(in.qd(i));
        TP z[3];
        matc_vec(z, R, J.axis);  // z_i = A_i axis = R_i axis (E_i leaves the axis fixed)
        TV zq[3], wp[3], dwp[3];
        {
            TV t[3];
#pragma unroll
            for (int k = 0; k < 3; k++) { zq[k] = z[k] * qdi; wp[k] = w[k] - zq[k]; }
            cross3(t, wp, zq);
#pragma unroll
            for (int k = 0; k < 3; k++) dwp[k] = dw[k] - t[k];
        }
        TP s(0.0), omc(0.0), d[3];
        if (i > 0) {
            TP cq;
            in.sincos(i, s, cq);
            omc = TP(1.0) - cq;
            // d = R_{i-1} tX = A_i uX = R_i (E_i^T uX),  E^T u = u - s (a x u) + omc (a (a.u) - u)
            const double *ax = J.axis, *u = J.uX;
            const double axu0 = ax[1] * u[2] - ax[2] * u[1], axu1 = ax[2] * u[0] - ax[0] * u[2],
                         axu2 = ax[0] * u[1] - ax[1] * u[0];
            const double au = ax[0] * u[0] + ax[1] * u[1] + ax[2] * u[2];
            TP eu[3];
            eu[0] = TP(u[0]) - s * axu0 + omc * (au * ax[0] - u[0]);
            eu[1] = TP(u[1]) - s * axu1 + omc * (au * ax[1] - u[1]);
            eu[2] = TP(u[2]) - s * axu2 + omc * (au * ax[2] - u[2]);
            mat_vec(d, R, eu);
        }
        // link wrench about the world origin
        TP r[3], cw[3];
        TV f[3];
        matc_vec(r, R, J.c);
        {
            TV t1[3], t2[3];
            cross3(t1, dw, r);
            cross3(t2, w, r);
            cross3(t2, w, t2);
#pragma unroll
            for (int k = 0; k < 3; k++) { cw[k] = o[k] + r[k]; f[k] = (a[k] + t1[k] + t2[k]) * m; }
        }
        TV v1[3], v2[3];
        inertia_apply(v1, R, J.Ic, dw);
        inertia_apply(v2, R, J.Ic, w);
        {
            TV t1[3], t2[3];
            cross3(t1, cw, f);
            cross3(t2, w, v2);
#pragma unroll
            for (int k = 0; k < 3; k++) { Mt[k] += t1[k] + v1[k] + t2[k]; Ft[k] += f[k]; }
        }
        TP pf[3];
        if (i == fp) {
            frame_point(F, o, R, pf);
            em.frame(pf);
            TP pxF[3];
            cross3(pxF, pf, Fw);
#pragma unroll
            for (int k = 0; k < 3; k++) { Mt[k] = Mt[k] - pxF[k]; Ft[k] = Ft[k] - Fw[k]; }
        }
        TP oz[3];
        cross3(oz, o, z);
        const TV taui = dot3(z, Mt) + dot3(oz, Ft);

        TV gqi(0.0), gqdi(0.0), db[3];  // db: adjoint of d_i = o_i - o_{i-1}; o_{i-1} receives -db
        if constexpr (ADJ) {
        // ---- adjoints of link i's quantities (M_bar = Lz, f_bar = Loz)
        TV zb[3], ob[3], cwb[3];
        if constexpr (GQ) {
            TV FxO[3], ZxF[3];
            cross3(FxO, Ft, o);
            cross3(ZxF, z, Ft);
#pragma unroll
            for (int k = 0; k < 3; k++) { zb[k] = (Mt[k] + FxO[k]) * c[i]; ob[k] = ZxF[k] * c[i]; }
        }
        if (GQ && i == fp) {
            TP pfb[3], g1[3], t1[3];
            cross3(pfb, Lz, Fw);
#pragma unroll
            for (int k = 0; k < 3; k++) pfb[k] = pfb[k] + yl[k];
            cross3(g1, pf, Lz);
#pragma unroll
            for (int k = 0; k < 3; k++) g1[k] = g1[k] - Loz[k];
            em.force(g1);
            cross3(t1, pf, pfb);
#pragma unroll
            for (int k = 0; k < 3; k++) { G[k] += t1[k]; Ob[k] += pfb[k]; }
        }
        if constexpr (GQ) cross3(cwb, f, Lz);
        TP ft[3];
        {
            TP t1[3];
            cross3(t1, Lz, cw);
#pragma unroll
            for (int k = 0; k < 3; k++) ft[k] = Loz[k] + t1[k];
        }
        {
            TP u1[3], rxf[3];
            TV mw[3], u2[3], vxl[3];
            inertia_apply(u1, R, J.Ic, Lz);
            cross3(mw, Lz, w);
            inertia_apply(u2, R, J.Ic, mw);
            const TV wr = dot3(w, r), fw = dot3(ft, w), ww = dot3(w, w);
            const TP fr = dot3(ft, r);
            cross3(rxf, r, ft);
            cross3(vxl, v2, Lz);
#pragma unroll
            for (int k = 0; k < 3; k++) {
                dwb[k] += u1[k] + rxf[k] * m;
                wb[k] += vxl[k] + u2[k] + (ft[k] * wr + r[k] * fw - 2.0 * fr * w[k]) * m;
                ab[k] += ft[k] * m;
            }
            if constexpr (GQ) {
            TV r1[3], r2[3], r3[3], r4[3], fxd[3];
            cross3(r1, v1, Lz);
            cross3(r2, u1, dw);
            cross3(r3, v2, mw);
            cross3(r4, u2, w);
            cross3(fxd, ft, dw);
#pragma unroll
            for (int k = 0; k < 3; k++) {
                G[k] += r1[k] + r2[k] + r3[k] + r4[k];
                TV rb = (fxd[k] + w[k] * fw - ww * ft[k]) * m;
                cwb[k] += rb;
                ob[k] -= rb;
            }
            }  // GQ
        }
        // ---- recurrences of joint i: w_i = w_p + zq, dw_i = dw_p + w_p x zq, a_i = a_p + dw_p x d + w_p x (w_p x d)
        TV zqb[3], wpb[3];
        {
            TV t1[3], t2[3];
            cross3(t1, dwb, wp);
            cross3(t2, zq, dwb);
#pragma unroll
            for (int k = 0; k < 3; k++) { zqb[k] = wb[k] + t1[k]; wpb[k] = wb[k] + t2[k]; }
        }
        if constexpr (GQ)
#pragma unroll
            for (int k = 0; k < 3; k++) zb[k] = zb[k] + zqb[k] * qdi;
        gqdi = dot3(z, zqb);
        if (i > 0) {
            TV dxa[3], axd[3];
            cross3(dxa, d, ab);
            cross3(axd, ab, dwp);
            const TV wa = dot3(wp, ab), ww = dot3(wp, wp), wd = dot3(wp, d), ad = dot3(ab, d);
#pragma unroll
            for (int k = 0; k < 3; k++) {
                dwb[k] += dxa[k];
                if constexpr (GQ) db[k] = axd[k] + wp[k] * wa - ww * ab[k];
                wpb[k] = wpb[k] + ab[k] * wd + d[k] * wa - 2.0 * ad * wp[k];
                if constexpr (GQ) ob[k] += db[k];
            }
        }
        // ---- geometric adjoints -> q_i
        if constexpr (GQ) {
            TV t1[3], t2[3], t3[3];
            cross3(t1, z, zb);
            cross3(t2, o, ob);
            cross3(t3, cw, cwb);
#pragma unroll
            for (int k = 0; k < 3; k++) {
                G[k] += t1[k] + t2[k] + t3[k];
                Ob[k] += ob[k] + cwb[k];
            }
            TV oxO[3];
            cross3(oxO, o, Ob);
            gqi = z[0] * (G[0] - oxO[0]) + z[1] * (G[1] - oxO[1]) + z[2] * (G[2] - oxO[2]);
        }
#pragma unroll
        for (int k = 0; k < 3; k++) {
            Lz[k] -= z[k] * c[i];
            Loz[k] -= oz[k] * c[i];
            wb[k] = wpb[k];
        }
        }  // ADJ
        em.joint(i, taui, gqi, gqdi);
        if (i > 0) {
            // a_{i-1}; o_{i-1} = o_i - d (a point of link i-2) receives -db in Gamma / Obar of q_{<i}
            TV t1[3], t2[3];
            cross3(t1, dwp, d);
            cross3(t2, wp, d);
            cross3(t2, wp, t2);
#pragma unroll
            for (int k = 0; k < 3; k++) { a[k] = a[k] - t1[k] - t2[k]; o[k] = o[k] - d[k]; }
            if constexpr (ADJ && GQ) {
                TV opxd[3];
                cross3(opxd, o, db);
#pragma unroll
                for (int k = 0; k < 3; k++) { G[k] -= opxd[k]; Ob[k] -= db[k]; }
            }
        }
#pragma unroll
        for (int k = 0; k < 3; k++) { w[k] = wp[k]; dw[k] = dwp[k]; }
        if (i > 0) {
            // R_{i-1} = (R_i E_i^T) RX_i^T, row by row in place; o_{i-1} = o_i - d
            TP A[9];
            rodrigues_rows(A, R, J.axis, TP(0.0) - s, omc);
#pragma unroll
            for (int rr = 0; rr < 3; rr++)
#pragma unroll
                for (int cc = 0; cc < 3; cc++)
                    R[3 * rr + cc] = A[3 * rr] * J.RX[3 * cc] + A[3 * rr + 1] * J.RX[3 * cc + 1] + A[3 * rr + 2] * J.RX[3 * cc + 2];
        }
    }
}

template <class TP, class TV> MF_HD void sweep_init(const DevModel &M, SweepState<TP, TV> &S) {
#pragma unroll
    for (int k = 0; k < 3; k++) {
        S.w[k] = TV(0.0); S.dw[k] = TV(0.0); S.a[k] = TV(-M.g[k]);
        S.Lz[k] = TP(0.0); S.Loz[k] = TP(0.0);
        S.Mt[k] = TV(0.0); S.Ft[k] = TV(0.0); S.wb[k] = TV(0.0); S.dwb[k] = TV(0.0);
        S.ab[k] = TV(0.0); S.G[k] = TV(0.0); S.Ob[k] = TV(0.0);
    }
}


template <class TP, class TV, int NJ, bool ADJ = true, bool GQ = true, class In, class Emit>
MF_HD void node_fwd_rev(const DevModel &M, const DevFrame &F, int fp, const In &in, const double *Fw, const double *c,
                        const double *yl, Emit &em) {
    SweepState<TP, TV> S;
    sweep_init(M, S);
    fwd_range<TP, TV, NJ, ADJ>(M, 0, NJ, in, c, S);
    rev_range<TP, TV, NJ, ADJ, GQ>(M, F, fp, NJ - 1, 0, in, Fw, c, yl, em, S);
}

// The sweep of a q direction v, split where its tangents vanish.  Every pose and velocity
// quantity of joints i < v is a function of q_0..q_i and qd_0..qd_i only, so its q_v tangent is
// identically zero: the forward sweep runs plain FP64 over joints 0..v-1 and switches to Dual at
// joint v (whose angle carries the tangent); the reverse sweep runs Dual over joints NJ-1..v and
// then, with the pose tangents dropped (exactly zero), over joints v-1..0 as a qd-class sweep
// (TP = double, TV = Dual: the adjoints' tangents are not zero) without the q-gradient (GQ = false:
// its rows i < v are the Hessian's upper triangle, which no caller reads).  em.force is not called
// when the frame parent is below v (that Hessian entry is exactly zero then).  The caller's In
// functor provides sincos / qd for both scalar types (template members).
template <int NJ, class In, class Emit>
MF_HD void node_fwd_rev_split(const DevModel &M, const DevFrame &F, int fp, int v, const In &in, const double *Fw,
                              const double *c, const double *yl, Emit &em) {
    SweepState<double, double> S0;
    sweep_init(M, S0);
    fwd_range<double, double, NJ, true>(M, 0, v, in, c, S0);
    SweepState<Dual, Dual> S1;
#pragma unroll
    for (int k = 0; k < 9; k++) S1.R[k] = Dual(S0.R[k]);
#pragma unroll
    for (int k = 0; k < 3; k++) {
        S1.o[k] = Dual(S0.o[k]); S1.Lz[k] = Dual(S0.Lz[k]); S1.Loz[k] = Dual(S0.Loz[k]);
        S1.w[k] = Dual(S0.w[k]); S1.dw[k] = Dual(S0.dw[k]); S1.a[k] = Dual(S0.a[k]);
        S1.Mt[k] = Dual(0.0); S1.Ft[k] = Dual(0.0); S1.wb[k] = Dual(0.0); S1.dwb[k] = Dual(0.0);
        S1.ab[k] = Dual(0.0); S1.G[k] = Dual(0.0); S1.Ob[k] = Dual(0.0);
    }
    fwd_range<Dual, Dual, NJ, true>(M, v, NJ, in, c, S1);
    rev_range<Dual, Dual, NJ, true, true>(M, F, fp, NJ - 1, v, in, Fw, c, yl, em, S1);
    if (v > 0) {
        SweepState<double, Dual> S2;
#pragma unroll
        for (int k = 0; k < 9; k++) S2.R[k] = S1.R[k].v;
#pragma unroll
        for (int k = 0; k < 3; k++) {
            S2.o[k] = S1.o[k].v; S2.Lz[k] = S1.Lz[k].v; S2.Loz[k] = S1.Loz[k].v;
            S2.w[k] = S1.w[k]; S2.dw[k] = S1.dw[k]; S2.a[k] = S1.a[k];
            S2.Mt[k] = S1.Mt[k]; S2.Ft[k] = S1.Ft[k]; S2.wb[k] = S1.wb[k]; S2.dwb[k] = S1.dwb[k];
            S2.ab[k] = S1.ab[k]; S2.G[k] = S1.G[k]; S2.Ob[k] = S1.Ob[k];
        }
        rev_range<double, Dual, NJ, true, false>(M, F, fp, v - 1, 0, in, Fw, c, yl, em, S2);
    }
}

// ---------------------------------------------------------------- values only
// tau (emitted per joint, em.joint(i, tau_i, 0, 0)) and p_f (em.frame) at
// (q, qd, Fw) given by the In functor: node_fwd_rev without its adjoint statements.
template <int NJ, class In, class Emit>
MF_HD void node_values(const DevModel &M, const DevFrame &F, int fp, const In &in, const double *Fw, Emit &em) {
    node_fwd_rev<double, double, NJ, false>(M, F, fp, in, Fw, nullptr, nullptr, em);
}

template <int NJ> struct ArrIn {  // inputs from plain arrays (global memory or LDS)
    const double *xq, *xqd;
    MF_HD double q(int i) const { return xq[i]; }
    MF_HD double qd(int i) const { return xqd[i]; }
    MF_HD void sincos(int i, double &s, double &c) const { sincos_t(xq[i], s, c); }
};

}  // namespace mf
