// Device dynamics for the MI355X hot path: FP64 scalars, dual numbers (exact
// first derivatives, one direction per lane) and hyper-dual numbers (exact
// second derivatives, one (u,v) pair per lane), run through one world-frame
// Newton-Euler pass over a serial chain.
//
// What it computes is pinocchio::rnea (src/casadi_pinocchio_bridge.hpp:76),
// framesForwardKinematics (L106) and the LOCAL_WORLD_ALIGNED frame Jacobian
// (L141-144), restated in the world frame so that a lane keeps only the
// running pose / twist / acceleration of the current joint in registers:
//
//   per joint i (parent i-1):   A = R_p RX_i,  o_i = o_p + R_p tX_i,  z_i = A axis_i
//                               R_i = A (I + s [a]x + (1-c) [a]x^2)
//   a_i  = a_p + dw_p x d + w_p x (w_p x d)      (joint-origin acceleration, d = o_i - o_p)
//   dw_i = dw_p + z_i qdd_i + w_p x z_i qd_i,    w_i = w_p + z_i qd_i
//   f_i  = m_i (a_i + dw_i x r_i + w_i x (w_i x r_i)),   r_i = R_i c_i
//   M_i  = (o_i + r_i) x f_i + I_w dw_i + w_i x I_w w_i  (moment about the world origin)
//   tau_j = S_j . sum_{i >= j} (M_i, f_i),  S_j = (z_j, o_j x z_j)
//
// The contraction phi = sum_j cw_j tau_j used for Hessian lanes is evaluated in
// the SAME single forward pass via the prefix Lambda_i = sum_{j<=i} cw_j S_j:
// phi = sum_i Lambda_i . (M_i, f_i) - Lambda_fp . W_ext  (no per-joint storage).
#pragma once
#include <hip/hip_runtime.h>

#include <cmath>

#include "model.hpp"

#define MF_HD __host__ __device__ __forceinline__

// Joint i of a model as a pointer of its own.  A descending joint loop otherwise lets the compiler strength-
// reduce &M.j[i] to a base of &M.j[NJ-1] - 400 (NJ-1-i) bytes and fold the constant into the instruction's
// offset.  For a model image in LDS read through a generic pointer (the phase kernels' images, gipm.hip), that
// base register then lies below the start of the LDS aperture whenever the image sits within a few joint
// records of LDS offset 0, and the flat load raises MEMORY_APERTURE_VIOLATION: the aperture of a flat access
// is decided on its base register, not on base + offset (tools/gchk_run.py).
// Only a translation unit whose kernels read model images through generic pointers (gipm.hip: the images are
// selected per arm, MArr) defines MF_GENERIC_MODEL_PTR; elsewhere the images are plain __shared__ objects, the
// loads are LDS instructions, and the pointer stays transparent.
template <class M_> MF_HD const auto &joint_at(const M_ &M, int i) {
    const auto *p = &M.j[i];
#if defined(__HIP_DEVICE_COMPILE__) && defined(MF_GENERIC_MODEL_PTR)
    __asm__ volatile("" : "+v"(p));
#endif
    return *p;
}

namespace mf {

// ---------------------------------------------------------------- scalars
struct Dual {
    double v, d;
    MF_HD Dual() : v(0), d(0) {}
    MF_HD Dual(double x) : v(x), d(0) {}
    MF_HD Dual(double x, double y) : v(x), d(y) {}
};
MF_HD Dual operator+(Dual a, Dual b) { return Dual(a.v + b.v, a.d + b.d); }
MF_HD Dual operator-(Dual a, Dual b) { return Dual(a.v - b.v, a.d - b.d); }
MF_HD Dual operator-(Dual a) { return Dual(-a.v, -a.d); }
MF_HD Dual operator*(Dual a, Dual b) { return Dual(a.v * b.v, fma(a.v, b.d, a.d * b.v)); }
MF_HD Dual operator*(Dual a, double s) { return Dual(a.v * s, a.d * s); }
MF_HD Dual operator*(double s, Dual a) { return Dual(a.v * s, a.d * s); }
MF_HD Dual &operator+=(Dual &a, Dual b) { a = a + b; return a; }
MF_HD Dual &operator-=(Dual &a, Dual b) { a = a - b; return a; }
// mixed with a constant-tangent (plain double) operand: no work on the zero tangent
MF_HD Dual operator+(Dual a, double b) { return Dual(a.v + b, a.d); }
MF_HD Dual operator+(double a, Dual b) { return Dual(a + b.v, b.d); }
MF_HD Dual operator-(Dual a, double b) { return Dual(a.v - b, a.d); }
MF_HD Dual operator-(double a, Dual b) { return Dual(a - b.v, -b.d); }
MF_HD Dual &operator+=(Dual &a, double b) { a.v += b; return a; }
MF_HD Dual &operator-=(Dual &a, double b) { a.v -= b; return a; }

struct HDual {  // a + b e1 + c e2 + d e1 e2
    double a, b, c, d;
    MF_HD HDual() : a(0), b(0), c(0), d(0) {}
    MF_HD HDual(double x) : a(x), b(0), c(0), d(0) {}
    MF_HD HDual(double x, double y, double z, double w) : a(x), b(y), c(z), d(w) {}
};
MF_HD HDual operator+(HDual x, HDual y) { return HDual(x.a + y.a, x.b + y.b, x.c + y.c, x.d + y.d); }
MF_HD HDual operator-(HDual x, HDual y) { return HDual(x.a - y.a, x.b - y.b, x.c - y.c, x.d - y.d); }
MF_HD HDual operator-(HDual x) { return HDual(-x.a, -x.b, -x.c, -x.d); }
MF_HD HDual operator*(HDual x, HDual y) {
    return HDual(x.a * y.a, fma(x.a, y.b, x.b * y.a), fma(x.a, y.c, x.c * y.a),
                 fma(x.a, y.d, fma(x.b, y.c, fma(x.c, y.b, x.d * y.a))));
}
MF_HD HDual operator*(HDual x, double s) { return HDual(x.a * s, x.b * s, x.c * s, x.d * s); }
MF_HD HDual operator*(double s, HDual x) { return HDual(x.a * s, x.b * s, x.c * s, x.d * s); }
MF_HD HDual &operator+=(HDual &x, HDual y) { x = x + y; return x; }
MF_HD HDual &operator-=(HDual &x, HDual y) { x = x - y; return x; }

MF_HD void sincos_t(double x, double &s, double &c) { s = sin(x); c = cos(x); }
MF_HD void sincos_t(Dual x, Dual &s, Dual &c) {
    double sv = sin(x.v), cv = cos(x.v);
    s = Dual(sv, cv * x.d);
    c = Dual(cv, -sv * x.d);
}
MF_HD void sincos_t(HDual x, HDual &s, HDual &c) {
    double sv = sin(x.a), cv = cos(x.a);
    s = HDual(sv, cv * x.b, cv * x.c, cv * x.d - sv * x.b * x.c);
    c = HDual(cv, -sv * x.b, -sv * x.c, -sv * x.d - cv * x.b * x.c);
}
MF_HD double val(double x) { return x; }
MF_HD double val(Dual x) { return x.v; }
MF_HD double val(HDual x) { return x.a; }
MF_HD double dtan(double) { return 0.0; }  // tangent part (0 for a plain double)
MF_HD double dtan(Dual x) { return x.d; }

// ---------------------------------------------------------------- 3-vectors
// Operand types may differ (a Dual with a plain-double pose quantity, adj.hpp): the result
// type TO is the caller's.
template <class TO, class TA, class TB> MF_HD void cross3(TO *o, const TA *a, const TB *b) {
    TO t0 = a[1] * b[2] - a[2] * b[1];
    TO t1 = a[2] * b[0] - a[0] * b[2];
    TO t2 = a[0] * b[1] - a[1] * b[0];
    o[0] = t0; o[1] = t1; o[2] = t2;
}
template <class TA, class TB> MF_HD auto dot3(const TA *a, const TB *b) { return a[0] * b[0] + a[1] * b[1] + a[2] * b[2]; }
template <class TO, class TA> MF_HD void matc_mul(TO *O, const TA *A, const double *B) {
#pragma unroll
    for (int r = 0; r < 3; r++)
#pragma unroll
        for (int c = 0; c < 3; c++) O[3 * r + c] = A[3 * r] * B[c] + A[3 * r + 1] * B[3 + c] + A[3 * r + 2] * B[6 + c];
}
template <class TO, class TA> MF_HD void matc_vec(TO *o, const TA *A, const double *v) {
#pragma unroll
    for (int r = 0; r < 3; r++) o[r] = A[3 * r] * v[0] + A[3 * r + 1] * v[1] + A[3 * r + 2] * v[2];
}
template <class TO, class TA, class TB> MF_HD void mat_vec(TO *o, const TA *A, const TB *v) {
    TO t[3];
#pragma unroll
    for (int r = 0; r < 3; r++) t[r] = A[3 * r] * v[0] + A[3 * r + 1] * v[1] + A[3 * r + 2] * v[2];
    o[0] = t[0]; o[1] = t[1]; o[2] = t[2];
}
template <class TO, class TA, class TB> MF_HD void matT_vec(TO *o, const TA *A, const TB *v) {
    TO t[3];
#pragma unroll
    for (int r = 0; r < 3; r++) t[r] = A[r] * v[0] + A[3 + r] * v[1] + A[6 + r] * v[2];
    o[0] = t[0]; o[1] = t[1]; o[2] = t[2];
}
template <class TO, class TB> MF_HD void cmat_vec(TO *o, const double *C, const TB *v) {  // constant C times v
#pragma unroll
    for (int r = 0; r < 3; r++) o[r] = v[0] * C[3 * r] + v[1] * C[3 * r + 1] + v[2] * C[3 * r + 2];
}

// ---------------------------------------------------------------- joint pose
// (R_p, o_p) -> (R, o, z) of joint J at angle q.  root: parent is the universe.
template <class T>
MF_HD void joint_pose(const DevJoint &J, const T *Rp, const T *op, bool root, T q, T *R, T *o, T *z) {
    T A[9];
    if (root) {
#pragma unroll
        for (int k = 0; k < 9; k++) A[k] = T(J.RX[k]);
#pragma unroll
        for (int k = 0; k < 3; k++) o[k] = T(J.tX[k]);
    } else {
        matc_mul(A, Rp, J.RX);
        matc_vec(o, Rp, J.tX);
#pragma unroll
        for (int k = 0; k < 3; k++) o[k] += op[k];
    }
    matc_vec(z, A, J.axis);
    T AK[9], AK2[9];
    matc_mul(AK, A, J.K);
    matc_mul(AK2, A, J.K2);
    T s, c;
    sincos_t(q, s, c);
    T omc = T(1.0) - c;
#pragma unroll
    for (int k = 0; k < 9; k++) R[k] = A[k] + s * AK[k] + omc * AK2[k];
}

// ---------------------------------------------------------------- Newton-Euler pass
// Serial chain (parent i-1).  For each joint the visitor receives the world axis
// z, origin o, rotation R, and the link wrench about the world origin (Mo, f).
// qdd may be nullptr (q'' = 0, every call site of the reference).
template <class T, class Vis>
MF_HD void ne_pass(const DevModel &M, int n, const T *q, const T *qd, const T *qdd, Vis &vis) {
    T R[9], o[3], w[3], dw[3], a[3];
#pragma unroll
    for (int k = 0; k < 3; k++) { w[k] = T(0.0); dw[k] = T(0.0); a[k] = T(-M.g[k]); o[k] = T(0.0); }
#pragma unroll
    for (int k = 0; k < 9; k++) R[k] = T((k % 4) == 0 ? 1.0 : 0.0);
#pragma unroll
    for (int i = 0; i < n; i++) {
        const DevJoint &J = joint_at(M, i);
        T Rn[9], on[3], z[3];
        joint_pose<T>(J, R, o, i == 0, q[i], Rn, on, z);
        if (i > 0) {
            T d[3], t1[3], t2[3];
#pragma unroll
            for (int k = 0; k < 3; k++) d[k] = on[k] - o[k];
            cross3(t1, dw, d);
            cross3(t2, w, d);
            cross3(t2, w, t2);
#pragma unroll
            for (int k = 0; k < 3; k++) a[k] = a[k] + t1[k] + t2[k];
        }
        T zq[3], t[3];
#pragma unroll
        for (int k = 0; k < 3; k++) zq[k] = z[k] * qd[i];
        cross3(t, w, zq);
#pragma unroll
        for (int k = 0; k < 3; k++) {
            dw[k] = dw[k] + t[k];
            if (qdd) dw[k] += z[k] * qdd[i];
            w[k] = w[k] + zq[k];
        }
#pragma unroll
        for (int k = 0; k < 9; k++) R[k] = Rn[k];
#pragma unroll
        for (int k = 0; k < 3; k++) o[k] = on[k];
        // link wrench
        T r[3], t1[3], t2[3], f[3];
        matc_vec(r, R, J.c);
        cross3(t1, dw, r);
        cross3(t2, w, r);
        cross3(t2, w, t2);
#pragma unroll
        for (int k = 0; k < 3; k++) f[k] = (a[k] + t1[k] + t2[k]) * J.m;
        T lb[3], Ib[3], Idw[3], Iw[3], g[3];
        matT_vec(lb, R, dw);
        cmat_vec(Ib, J.Ic, lb);
        mat_vec(Idw, R, Ib);
        matT_vec(lb, R, w);
        cmat_vec(Ib, J.Ic, lb);
        mat_vec(Iw, R, Ib);
        cross3(g, w, Iw);
        T cpos[3], Mo[3];
#pragma unroll
        for (int k = 0; k < 3; k++) cpos[k] = o[k] + r[k];
        cross3(Mo, cpos, f);
#pragma unroll
        for (int k = 0; k < 3; k++) Mo[k] = Mo[k] + Idw[k] + g[k];
        vis.joint(i, z, o, R, Mo, f);
    }
}

// frame position p = o + R t
template <class T> MF_HD void frame_point(const DevFrame &F, const T *o, const T *R, T *p) {
    matc_vec(p, R, F.t);
#pragma unroll
    for (int k = 0; k < 3; k++) p[k] = p[k] + o[k];
}

// ---------------------------------------------------------------- visitors
// phi = sum_j cw_j tau_j + yl . pf[0:nl],   tau = RNEA(q,qd,0) - J_f^T [Fw; 0]
template <class T, int NJ> struct PhiVis {
    const DevFrame *F;
    const double *cw;  // NJ
    const double *yl;  // nl
    int nl;
    T Fw[3];
    T Lz[3], Loz[3], phi;
    T pf[3];
    MF_HD void init() {
#pragma unroll
        for (int k = 0; k < 3; k++) { Lz[k] = T(0.0); Loz[k] = T(0.0); pf[k] = T(0.0); }
        phi = T(0.0);
    }
    MF_HD void joint(int i, const T *z, const T *o, const T *R, const T *Mo, const T *f) {
        T oz[3];
        cross3(oz, o, z);
#pragma unroll
        for (int k = 0; k < 3; k++) { Lz[k] += z[k] * cw[i]; Loz[k] += oz[k] * cw[i]; }
        phi += dot3(Lz, Mo) + dot3(Loz, f);
        if (i == F->parent) {
            frame_point(*F, o, R, pf);
            T pxF[3];
            cross3(pxF, pf, Fw);
            phi -= dot3(Lz, pxF) + dot3(Loz, Fw);
            for (int l = 0; l < nl; l++) phi += pf[l] * yl[l];
        }
    }
};

// pass 1: total wrench and frame point
template <class T> struct TotVis {
    const DevFrame *F;
    T Mt[3], Ft[3], pf[3];
    MF_HD void init() {
#pragma unroll
        for (int k = 0; k < 3; k++) { Mt[k] = T(0.0); Ft[k] = T(0.0); pf[k] = T(0.0); }
    }
    MF_HD void joint(int i, const T *z, const T *o, const T *R, const T *Mo, const T *f) {
#pragma unroll
        for (int k = 0; k < 3; k++) { Mt[k] += Mo[k]; Ft[k] += f[k]; }
        if (F && i == F->parent) frame_point(*F, o, R, pf);
    }
};

// pass 2: tau_j = S_j . (W_tot - sum_{i<j} W_i) - [j <= fp] S_j . W_ext
template <class T, int NJ> struct EmitVis {
    const TotVis<T> *tot;
    int fp;        // frame parent joint (-1: no external force)
    T Fw[3];
    T PM[3], PF[3];
    T tau[NJ];
    T Mext[3];
    MF_HD void init() {
#pragma unroll
        for (int k = 0; k < 3; k++) { PM[k] = T(0.0); PF[k] = T(0.0); }
        if (fp >= 0) cross3(Mext, tot->pf, Fw);
    }
    MF_HD void joint(int i, const T *z, const T *o, const T *R, const T *Mo, const T *f) {
        T oz[3], dM[3], dF[3];
        cross3(oz, o, z);
#pragma unroll
        for (int k = 0; k < 3; k++) { dM[k] = tot->Mt[k] - PM[k]; dF[k] = tot->Ft[k] - PF[k]; }
        T t = dot3(z, dM) + dot3(oz, dF);
        if (i <= fp) t -= dot3(z, Mext) + dot3(oz, Fw);
        tau[i] = t;
#pragma unroll
        for (int k = 0; k < 3; k++) { PM[k] += Mo[k]; PF[k] += f[k]; }
    }
};

// frame Jacobian (LOCAL_WORLD_ALIGNED) and pose: records z_j, o_j of the chain
template <class T, int NJ> struct JacVis {
    const DevFrame *F;
    T z[NJ][3], o[NJ][3];
    T pf[3], Rf[9];
    MF_HD void joint(int i, const T *zz, const T *oo, const T *R, const T *Mo, const T *f) {
#pragma unroll
        for (int k = 0; k < 3; k++) { z[i][k] = zz[k]; o[i][k] = oo[k]; }
        if (i == F->parent) {
            frame_point(*F, oo, R, pf);
            matc_mul(Rf, R, F->R);
        }
    }
};

// Node values: tau (NJ) and frame point pf (3) at (q, qd, F), q'' = 0.
template <class T, int NJ>
MF_HD void node_tau(const DevModel &M, const DevFrame &F, int nf, const double *fdir, const T *q, const T *qd,
                    const T *Fv, T *tau, T *pf) {
    TotVis<T> tv;
    tv.F = &F;
    tv.init();
    ne_pass<T>(M, NJ, q, qd, (const T *)nullptr, tv);
    EmitVis<T, NJ> ev;
    ev.tot = &tv;
    ev.fp = nf > 0 ? F.parent : -1;
#pragma unroll
    for (int k = 0; k < 3; k++) {
        T acc = T(0.0);
        for (int a = 0; a < nf; a++) acc += Fv[a] * fdir[3 * a + k];
        ev.Fw[k] = acc;
    }
    ev.init();
    ne_pass<T>(M, NJ, q, qd, (const T *)nullptr, ev);
#pragma unroll
    for (int j = 0; j < NJ; j++) tau[j] = ev.tau[j];
#pragma unroll
    for (int k = 0; k < 3; k++) pf[k] = tv.pf[k];
}

}  // namespace mf
