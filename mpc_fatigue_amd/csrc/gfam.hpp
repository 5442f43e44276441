// Node functions of the generic stage-structured OCP (gipm.hip), host + device.
//
// Every reference transcription is, per shooting node k,
//   variables x_k (NX), u_k (NU);  cost l(x, u);  dynamics x_{k+1} = f(x, u);
//   slack rows c_lo <= c_in(x, u) <= c_hi (NI);  state equalities c_eq(x) = 0 (NE)
// and the solver needs, per node, the "node record"
//   [ l | grad l (NV) | c_in (NI) | d c_in (NI x NV) | c_eq (NE) | d c_eq / dx (NE x NX) | f (NX) |
//     A = df/dx (NX x NX) | B = df/du (NX x NU) | W = grad^2 (l + yi.c_in + ye.c_eq + lam.f) (NV x NV) ]
// (row-major blocks, NV = NX + NU).  Families:
//   BoxFam    two 6-DOF Pilz arms holding a box, python/2_pilz_6_DOF/Box_Pilz_6DOF.py:219-456 (C3)
//             x = [q_L, q_R], u = [qd_L, qd_R, F_L, F_R]; c_in = [force equilibrium (3), moment
//             equilibrium (3), tau_L (6), tau_R (6)]; c_eq = |E1 - E2|^2 - L; cost 100|p_box - p_des|^2
//             + qd^T qd.
//   ChainFam  one serial arm (Pilz 3/6-DOF, C1 / C2), optionally with the motor-winding temperature
//             T as state (Tmodel_library.py:9-41, RepeatedMPCwithThermal.py:371-376):
//             x = [q, (T)], u = [qd, F]; c_in = tau; c_eq = p_f[0:2] - line_ref;
//             cost wF|F|^2 + wqd|qd|^2 + wtau|tau|^2 (+ wT|T|^2).
// Derivatives: each arm runs the forward-over-reverse sweep of adj.hpp once per tangent direction
// (q_j or qd_j of that arm; one GPU lane each) on phi_arm = c.tau_arm + seed.p_frame with the
// torque weights c and the frame-point seed chosen so that, together with the closed-form second
// derivatives of the algebraic part (the box cost, distance, equilibrium rows; the thermal
// recursion), the assembled W is the exact Lagrangian Hessian.  The record entries are pure
// functions of a per-node scratch (the lanes' columns) so a block of threads assembles them in
// parallel (device) or a loop does (host test harness, tests/native/famcheck.cpp).
#pragma once
#include "adj.hpp"

namespace mf {

constexpr int GX_MAX = 32;

// Problem constants of a generic family (kernel argument, POD).
struct GParams {
    int N;
    double h;
    int eq_from;
    // ChainFam
    int nf, use_line, thermal;
    double fdir[9];
    double wF, wqd, wtau, wT;
    double th_a, th_b, Ra, Rh;
    double ktau[MF_MAX_JOINTS];
    // BoxFam
    double box_mg, box_L, box_pdes[3], w_box, w_qdb;
    // state bounds (k >= 1)
    double x_lo[GX_MAX], x_hi[GX_MAX];
    // solver options
    double tol, constr_viol_tol, mu_init, F_init;
    int max_iter, max_soc, init_zero, has_u_init;
    double u_init[GX_MAX];
    int force_from, tier1_from, tier1_to;  // first force control; u range regularised first (concave cost)
};

template <int NX_, int NU_, int NI_, int NE_> struct GDims {
    static constexpr int NX = NX_, NU = NU_, NI = NI_, NE = NE_, NV = NX_ + NU_;
    static constexpr int NIA = NI_ > 0 ? NI_ : 1, NEA = NE_ > 0 ? NE_ : 1;
    static constexpr int O_L = 0, O_GL = 1, O_CI = O_GL + NV, O_JI = O_CI + NI, O_CE = O_JI + NI * NV,
                         O_JE = O_CE + NE, O_F = O_JE + NE * NX, O_A = O_F + NX, O_B = O_A + NX * NX,
                         O_W = O_B + NX * NU, REC = O_W + NV * NV;
};

// ---------------------------------------------------------------- lanes (adj.hpp)
// Tangent direction v of an NJ-joint arm: v < NJ -> q_v (TP = Dual, the pose carries the tangent),
// v >= NJ -> qd_{v-NJ} (TP = double: plain-FP64 pose).
template <int NJ, class TP> struct GLaneIn {
    const double *xq, *xqd;
    int v;
    MF_HD Dual qd(int i) const { return Dual(xqd[i], v == NJ + i ? 1.0 : 0.0); }
    MF_HD void sincos(int i, TP &s, TP &c) const {
        if constexpr (sizeof(TP) == sizeof(Dual)) {
            sincos_t(Dual(xq[i], v == i ? 1.0 : 0.0), s, c);
        } else {
            sincos_t(xq[i], s, c);
        }
    }
};
// Lane column layout (LCOL doubles): jt (NJ) | hq (NJ) | hqd (NJ) | hF (3) | pfd (3)
template <int NJ> struct GLaneOut {
    static constexpr int JT = 0, HQ = NJ, HQD = 2 * NJ, HF = 3 * NJ, PFD = 3 * NJ + 3, LCOL = 3 * NJ + 6;
    double *col;
    template <class TP> MF_HD void frame(const TP *p) {
#pragma unroll
        for (int k = 0; k < 3; k++) col[PFD + k] = dtan(p[k]);
    }
    template <class TP> MF_HD void force(const TP *g) {
#pragma unroll
        for (int k = 0; k < 3; k++) col[HF + k] = dtan(g[k]);
    }
    MF_HD void joint(int i, const Dual &t, const Dual &gq, const Dual &gqd) {
        col[JT + i] = t.d;
        col[HQ + i] = gq.d;
        col[HQD + i] = gqd.d;
    }
};
// values only: tau and the frame point
template <int NJ> struct GValOut {
    double *tau, *pf;
    MF_HD void frame(const double *p) {
        for (int k = 0; k < 3; k++) pf[k] = p[k];
    }
    MF_HD void force(const double *) {}
    MF_HD void joint(int i, double t, double, double) { tau[i] = t; }
};

template <int NJ>
MF_HD void arm_values(const DevModel &M, const DevFrame &F, const double *q, const double *qd, const double *Fw,
                      double *tau, double *pf) {
    GValOut<NJ> o{tau, pf};
    ArrIn<NJ> in{q, qd};
    node_values<NJ>(M, F, F.parent, in, Fw, o);
}

template <int NJ>
MF_HD void arm_lane(const DevModel &M, const DevFrame &F, const double *q, const double *qd, const double *Fw,
                    const double *c, const double *seed, int v, double *col) {
    GLaneOut<NJ> o{col};
    if (v < NJ) {
        GLaneIn<NJ, Dual> in{q, qd, v};
        node_fwd_rev<Dual, Dual, NJ>(M, F, F.parent, in, Fw, c, seed, o);
    } else {
        GLaneIn<NJ, double> in{q, qd, v};
        node_fwd_rev<double, Dual, NJ>(M, F, F.parent, in, Fw, c, seed, o);
    }
}

MF_HD double skew_el(const double *y, int r, int c) {  // [y]x (r, c)
    if (r == c) return 0.0;
    if (r == 0) return c == 1 ? -y[2] : y[1];
    if (r == 1) return c == 0 ? y[2] : -y[0];
    return c == 0 ? -y[1] : y[0];
}

// ================================================================ BoxFam (C3)
struct BoxFam {
    static constexpr int NJ = 6, NARM = 2, NDIR = 2 * NJ, NM = 2;
    using D = GDims<12, 18, 18, 1>;
    static constexpr int LANES = NARM * NDIR;  // derivative lanes per node
    static constexpr int LCOL = GLaneOut<NJ>::LCOL;
    // per-node scratch
    struct Scratch {
        double E[NARM][3], tau[NARM][NJ], seed[NARM][3], d[3], dF[3], eb[3];
        double col[NARM][NDIR][LCOL];
    };
    // variables: q_L 0-5, q_R 6-11 | qd_L 12-17, qd_R 18-23, F_L 24-26, F_R 27-29
    // kind: 0 q, 1 qd, 2 F; arm; local index
    MF_HD static void var(int v, int &kind, int &arm, int &loc) {
        if (v < 12) { kind = 0; arm = v / 6; loc = v % 6; }
        else if (v < 24) { kind = 1; arm = (v - 12) / 6; loc = (v - 12) % 6; }
        else { kind = 2; arm = (v - 24) / 3; loc = (v - 24) % 3; }
    }

    // values at (x, u): l, ci, ce, f (line search / slacks).  E: frame points out (may be null)
    template <class MA, class FA> MF_HD static void values(MA M, FA F, const GParams &P, const double *x, const double *u,
                             const double *, double &l, double *ci, double *ce, double *f) {
        double tL[NJ], tR[NJ], E1[3], E2[3];
        arm_values<NJ>(M[0], F[0], x, u, u + 12, tL, E1);
        arm_values<NJ>(M[1], F[1], x + 6, u + 6, u + 15, tR, E2);
        const double *FL = u + 12, *FR = u + 15;
        double d[3], dF[3], m[3];
        for (int r = 0; r < 3; r++) { d[r] = E1[r] - E2[r]; dF[r] = FL[r] - FR[r]; }
        cross3(m, d, dF);
        ci[0] = FL[2] + FR[2] - P.box_mg;
        ci[1] = FL[0] + FR[0];
        ci[2] = FL[1] + FR[1];
        for (int r = 0; r < 3; r++) ci[3 + r] = m[r];
        for (int j = 0; j < NJ; j++) { ci[6 + j] = tL[j]; ci[12 + j] = tR[j]; }
        ce[0] = d[0] * d[0] + d[1] * d[1] + d[2] * d[2] - P.box_L;
        double c = 0.0;
        for (int r = 0; r < 3; r++) {
            const double e = 0.5 * (E1[r] + E2[r]) - P.box_pdes[r];
            c += P.w_box * e * e;
        }
        for (int j = 0; j < 12; j++) {
            c += P.w_qdb * u[j] * u[j];
            f[j] = x[j] + P.h * u[j];
        }
        l = c;
    }

    static constexpr int PRE = NARM;  // pre-pass lanes per node
    // pre-pass lane a: frame point E_a and tau_a at the node
    template <class MA, class FA> MF_HD static void prepass(MA M, FA F, const GParams &, const double *x, const double *u,
                              int a, Scratch &S) {
        arm_values<NJ>(M[a], F[a], x + 6 * a, u + 6 * a, u + 12 + 3 * a, S.tau[a], S.E[a]);
    }
    // seeds of both arms from the pre-pass: lambda_E = d g / d E_a of the algebraic part
    //   g = w_box |(E1+E2)/2 - p|^2 + ye (|d|^2 - L) + y_m . (d x dF),  d = E1 - E2, dF = F_L - F_R
    MF_HD static void seeds(const GParams &P, const double *u, const double *yi, const double *ye, const double *,
                            bool eqon, Scratch &S) {
        const double yev = eqon ? ye[0] : 0.0;
        const double *ym = yi + 3;
        double dFxy[3];
        for (int r = 0; r < 3; r++) {
            S.d[r] = S.E[0][r] - S.E[1][r];
            S.dF[r] = u[12 + r] - u[15 + r];
            S.eb[r] = P.w_box * (0.5 * (S.E[0][r] + S.E[1][r]) - P.box_pdes[r]);
        }
        cross3(dFxy, S.dF, ym);
        for (int r = 0; r < 3; r++) {
            S.seed[0][r] = S.eb[r] + 2.0 * yev * S.d[r] + dFxy[r];
            S.seed[1][r] = S.eb[r] - 2.0 * yev * S.d[r] - dFxy[r];
        }
    }
    // derivative lane t in [0, LANES): arm t / NDIR, direction t % NDIR
    template <class MA, class FA> MF_HD static void lane(MA M, FA F, const double *x, const double *u, const double *yi,
                           int t, Scratch &S) {
        const int a = t / NDIR, v = t % NDIR;
        arm_lane<NJ>(M[a], F[a], x + 6 * a, u + 6 * a, u + 12 + 3 * a, yi + 6 + 6 * a, S.seed[a], v, S.col[a][v]);
    }
    // dE_a[c] / d(var) (frame-point Jacobian; zero unless var is a q of arm a)
    MF_HD static double JE(const Scratch &S, int a, int c, int v) {
        int kind, arm, loc;
        var(v, kind, arm, loc);
        return (kind == 0 && arm == a) ? S.col[a][loc][GLaneOut<NJ>::PFD + c] : 0.0;
    }
    // W(r, c) of the Lagrangian Hessian
    MF_HD static double Wel(const GParams &P, const double *yi, const double *ye, bool eqon, const Scratch &S, int r,
                            int c) {
        int kr, ar, lr, kc, ac, lc;
        var(r, kr, ar, lr);
        var(c, kc, ac, lc);
        using L = GLaneOut<NJ>;
        double w = 0.0;
        // arm sweeps (phi_a = c.tau_a + seed_a . E_a)
        if (ar == ac && !(kr == 2 && kc == 2)) {
            auto colent = [&](int vdir, int kind, int loc) {  // column vdir of arm ar, row (kind, loc)
                const double *cl = S.col[ar][vdir];
                return kind == 0 ? cl[L::HQ + loc] : (kind == 1 ? cl[L::HQD + loc] : cl[L::HF + loc]);
            };
            const int dr = kr == 0 ? lr : NJ + lr, dc = kc == 0 ? lc : NJ + lc;
            if (kr == 2) w = colent(dc, kr, lr);
            else if (kc == 2) w = colent(dr, kc, lc);
            else w = 0.5 * (colent(dc, kr, lr) + colent(dr, kc, lc));
        }
        // algebraic part: J_E^T (d^2 g / dE dE) J_E and the E-F cross terms of the moment rows
        const double yev = eqon ? ye[0] : 0.0;
        if (kr == 0 && kc == 0) {
            const double g = 0.5 * P.w_box + (ar == ac ? 2.0 : -2.0) * yev;
            double acc = 0.0;
            for (int k = 0; k < 3; k++) acc += JE(S, ar, k, r) * JE(S, ac, k, c);
            w += g * acc;
        } else if ((kr == 0 && kc == 2) || (kr == 2 && kc == 0)) {
            const int vq = kr == 0 ? r : c, aq = kr == 0 ? ar : ac, af = kr == 2 ? ar : ac, lf = kr == 2 ? lr : lc;
            const double sgn = (aq == af) ? -1.0 : 1.0;  // d^2 g / dE_aq dF_af = sgn [y_m]x
            double acc = 0.0;
            for (int k = 0; k < 3; k++) acc += JE(S, aq, k, vq) * skew_el(yi + 3, k, lf);
            w += sgn * acc;
        }
        if (r == c && kr == 1) w += 2.0 * P.w_qdb;
        return w;
    }
    // record entry e (D offsets)
    MF_HD static double rec(const GParams &P, const double *x, const double *u, const double *yi, const double *ye,
                            const double *, bool eqon, const Scratch &S, int e, const double *) {
        using L = GLaneOut<NJ>;
        if (e >= D::O_W) {
            const int i = e - D::O_W;
            return Wel(P, yi, ye, eqon, S, i / D::NV, i % D::NV);
        }
        if (e == D::O_L) {
            double c = 0.0;
            for (int r = 0; r < 3; r++) {
                const double v = 0.5 * (S.E[0][r] + S.E[1][r]) - P.box_pdes[r];
                c += P.w_box * v * v;
            }
            for (int j = 0; j < 12; j++) c += P.w_qdb * u[j] * u[j];
            return c;
        }
        if (e < D::O_CI) {  // grad l
            const int v = e - D::O_GL;
            int k, a, l;
            var(v, k, a, l);
            if (k == 0) {
                double acc = 0.0;
                for (int c = 0; c < 3; c++) acc += JE(S, a, c, v) * S.eb[c];
                return acc;
            }
            return k == 1 ? 2.0 * P.w_qdb * u[v - 12] : 0.0;
        }
        if (e < D::O_JI) {  // c_in values
            const int r = e - D::O_CI;
            if (r == 0) return u[14] + u[17] - P.box_mg;
            if (r == 1) return u[12] + u[15];
            if (r == 2) return u[13] + u[16];
            if (r < 6) {
                double m[3];
                cross3(m, S.d, S.dF);
                return m[r - 3];
            }
            return r < 12 ? S.tau[0][r - 6] : S.tau[1][r - 12];
        }
        if (e < D::O_CE) {  // d c_in
            const int i = e - D::O_JI, r = i / D::NV, v = i % D::NV;
            int k, a, l;
            var(v, k, a, l);
            if (r < 3) {  // F_L + F_R - (0, 0, m g), rows (z, x, y)
                const int comp = r == 0 ? 2 : r - 1;
                return (k == 2 && l == comp) ? 1.0 : 0.0;
            }
            if (r < 6) {  // m = d x dF
                const int mr = r - 3;
                if (k == 0) {  // dm/dE_a = -+[dF]x
                    double acc = 0.0;
                    for (int c = 0; c < 3; c++) acc += skew_el(S.dF, mr, c) * JE(S, a, c, v);
                    return a == 0 ? -acc : acc;
                }
                if (k == 2) return (a == 0 ? 1.0 : -1.0) * skew_el(S.d, mr, l);  // dm/dF_L = [d]x, dm/dF_R = -[d]x
                return 0.0;
            }
            const int ta = r < 12 ? 0 : 1, ti = (r - 6) % 6;
            if (a != ta) return 0.0;
            if (k == 2) return -S.col[ta][ti][L::PFD + l];  // d tau_i / d F_c = -dE_c / dq_i
            return S.col[ta][k == 0 ? l : NJ + l][L::JT + ti];
        }
        if (e < D::O_JE) {  // c_eq
            return S.d[0] * S.d[0] + S.d[1] * S.d[1] + S.d[2] * S.d[2] - P.box_L;
        }
        if (e < D::O_F) {  // d c_eq / dx
            const int v = e - D::O_JE;
            double acc = 0.0;
            for (int c = 0; c < 3; c++) acc += 2.0 * S.d[c] * (JE(S, 0, c, v) - JE(S, 1, c, v));
            return acc;
        }
        if (e < D::O_A) {  // f = q + h qd
            const int j = e - D::O_F;
            return x[j] + P.h * u[j];
        }
        if (e < D::O_B) {
            const int i = e - D::O_A;
            return (i / D::NX == i % D::NX) ? 1.0 : 0.0;
        }
        const int i = e - D::O_B, r = i / D::NU, c = i % D::NU;
        return (c == r) ? P.h : 0.0;
    }
};

// ================================================================ ChainFam (C1, C2, thermal)
template <int NJ_, int NF_, int NE_, bool THERMAL_> struct ChainFam {
    static constexpr int NJ = NJ_, NF = NF_, NDIR = 2 * NJ_, NM = 1;
    static constexpr bool TH = THERMAL_;
    using D = GDims<(THERMAL_ ? 2 : 1) * NJ_, NJ_ + NF_, NJ_, NE_>;
    static constexpr int LANES = NDIR;
    static constexpr int LCOL = GLaneOut<NJ>::LCOL;
    struct Scratch {
        double E[1][3], tau[1][NJ], pf[3], cw[NJ], om[NJ], seed[3], Fw[3];
        double col[1][NDIR][LCOL];
    };
    // variables: q 0..NJ-1, (T NJ..2NJ-1) | qd, F
    MF_HD static void var(int v, int &kind, int &loc) {
        constexpr int nx = D::NX;
        if (v < NJ) { kind = 0; loc = v; }
        else if (v < nx) { kind = 3; loc = v - NJ; }
        else if (v < nx + NJ) { kind = 1; loc = v - nx; }
        else { kind = 2; loc = v - nx - NJ; }
    }
    MF_HD static void world_force(const GParams &P, const double *u, double *Fw) {
        for (int r = 0; r < 3; r++) {
            double acc = 0.0;
            for (int a = 0; a < NF; a++) acc += u[NJ + a] * P.fdir[3 * a + r];
            Fw[r] = acc;
        }
    }
    MF_HD static double ploss(const GParams &P, int j, double tau, double qd) {
        const double ia = tau / P.ktau[j];
        return P.Ra * ia * ia + qd * qd / P.Rh;
    }
    template <class MA, class FA> MF_HD static void values(MA M, FA F, const GParams &P, const double *x, const double *u,
                             const double *lref, double &l, double *ci, double *ce, double *f) {
        double tau[NJ], pf[3], Fw[3];
        world_force(P, u, Fw);
        arm_values<NJ>(M[0], F[0], x, u, Fw, tau, pf);
        double c = 0.0;
        for (int a = 0; a < NF; a++) c += P.wF * u[NJ + a] * u[NJ + a];
        for (int j = 0; j < NJ; j++) {
            c += P.wqd * u[j] * u[j] + P.wtau * tau[j] * tau[j];
            ci[j] = tau[j];
            f[j] = x[j] + P.h * u[j];
            if constexpr (TH) {
                f[NJ + j] = P.th_a * x[NJ + j] + P.th_b * ploss(P, j, tau[j], u[j]);
                c += P.wT * x[NJ + j] * x[NJ + j];
            }
        }
        for (int i = 0; i < NE_; i++) ce[i] = pf[i] - lref[i];
        l = c;
    }
    static constexpr int PRE = 1;
    template <class MA, class FA> MF_HD static void prepass(MA M, FA F, const GParams &P, const double *x, const double *u,
                              int, Scratch &S) {
        world_force(P, u, S.Fw);
        arm_values<NJ>(M[0], F[0], x, u, S.Fw, S.tau[0], S.pf);
    }
    // torque weights c_j = yi_j + 2 tau_j (wtau + lam_T,j b Ra / ktau_j^2), Gauss-Newton weights
    // om_j = 2 (wtau + lam_T,j b Ra / ktau_j^2), frame seed = (ye, 0)
    MF_HD static void seeds(const GParams &P, const double *, const double *yi, const double *ye, const double *lam,
                            bool eqon, Scratch &S) {
        for (int j = 0; j < NJ; j++) {
            double w = P.wtau;
            if constexpr (TH) w += lam[NJ + j] * P.th_b * P.Ra / (P.ktau[j] * P.ktau[j]);
            S.om[j] = 2.0 * w;
            S.cw[j] = yi[j] + 2.0 * w * S.tau[0][j];
        }
        for (int r = 0; r < 3; r++) S.seed[r] = (eqon && r < NE_) ? ye[r] : 0.0;
    }
    template <class MA, class FA> MF_HD static void lane(MA M, FA F, const double *x, const double *u, const double *, int v,
                           Scratch &S) {
        arm_lane<NJ>(M[0], F[0], x, u, S.Fw, S.cw, S.seed, v, S.col[0][v]);
    }
    // d tau_j / d(var)
    MF_HD static double dtau(const GParams &P, const Scratch &S, int j, int v) {
        using L = GLaneOut<NJ>;
        int k, l;
        var(v, k, l);
        if (k == 0) return S.col[0][l][L::JT + j];
        if (k == 1) return S.col[0][NJ + l][L::JT + j];
        if (k == 2) {  // -fdir_a . dp_f / dq_j
            const double *pd = S.col[0][j] + L::PFD;
            return -(P.fdir[3 * l] * pd[0] + P.fdir[3 * l + 1] * pd[1] + P.fdir[3 * l + 2] * pd[2]);
        }
        return 0.0;
    }
    MF_HD static double Wel(const GParams &P, const double *u, const double *lam, const Scratch &S, int r, int c) {
        using L = GLaneOut<NJ>;
        int kr, lr, kc, lc;
        var(r, kr, lr);
        var(c, kc, lc);
        double w = 0.0;
        if (kr != 3 && kc != 3 && !(kr == 2 && kc == 2)) {
            auto colent = [&](int vdir, int kind, int loc) {
                const double *cl = S.col[0][vdir];
                if (kind == 0) return cl[L::HQ + loc];
                if (kind == 1) return cl[L::HQD + loc];
                const double *h = cl + L::HF;
                return P.fdir[3 * loc] * h[0] + P.fdir[3 * loc + 1] * h[1] + P.fdir[3 * loc + 2] * h[2];
            };
            const int dr = kr == 0 ? lr : NJ + lr, dc = kc == 0 ? lc : NJ + lc;
            if (kr == 2) w = colent(dc, kr, lr);
            else if (kc == 2) w = colent(dr, kc, lc);
            else w = 0.5 * (colent(dc, kr, lr) + colent(dr, kc, lc));
        }
        if (kr != 3 && kc != 3) {
            double acc = 0.0;
            for (int j = 0; j < NJ; j++) acc += S.om[j] * dtau(P, S, j, r) * dtau(P, S, j, c);
            w += acc;
        }
        if (r == c) {
            if (kr == 1) {
                w += 2.0 * P.wqd;
                if constexpr (TH) w += lam[NJ + lr] * P.th_b * 2.0 / P.Rh;
            }
            if (kr == 2) w += 2.0 * P.wF;
            if (kr == 3) w += 2.0 * P.wT;
        }
        return w;
    }
    MF_HD static double rec(const GParams &P, const double *x, const double *u, const double *yi, const double *ye,
                            const double *lam, bool eqon, const Scratch &S, int e, const double *lref) {
        if (e >= D::O_W) {
            const int i = e - D::O_W;
            return Wel(P, u, lam, S, i / D::NV, i % D::NV);
        }
        if (e == D::O_L) {
            double c = 0.0;
            for (int a = 0; a < NF; a++) c += P.wF * u[NJ + a] * u[NJ + a];
            for (int j = 0; j < NJ; j++) {
                c += P.wqd * u[j] * u[j] + P.wtau * S.tau[0][j] * S.tau[0][j];
                if constexpr (TH) c += P.wT * x[NJ + j] * x[NJ + j];
            }
            return c;
        }
        if (e < D::O_CI) {
            const int v = e - D::O_GL;
            int k, l;
            var(v, k, l);
            double g = 0.0;
            if (k != 3)
                for (int j = 0; j < NJ; j++) g += 2.0 * P.wtau * S.tau[0][j] * dtau(P, S, j, v);
            if (k == 1) g += 2.0 * P.wqd * u[l];
            if (k == 2) g += 2.0 * P.wF * u[NJ + l];
            if (k == 3) g += 2.0 * P.wT * x[NJ + l];
            return g;
        }
        if (e < D::O_JI) return S.tau[0][e - D::O_CI];
        if (e < D::O_CE) {
            const int i = e - D::O_JI;
            return dtau(P, S, i / D::NV, i % D::NV);
        }
        if (e < D::O_JE) return S.pf[e - D::O_CE] - lref[e - D::O_CE];
        if (e < D::O_F) {
            const int i = e - D::O_JE, l = i / D::NX, v = i % D::NX;
            return v < NJ ? S.col[0][v][GLaneOut<NJ>::PFD + l] : 0.0;
        }
        if (e < D::O_A) {
            const int j = e - D::O_F;
            if (j < NJ) return x[j] + P.h * u[j];
            const int t = j - NJ;
            return P.th_a * x[j] + P.th_b * ploss(P, t, S.tau[0][t], u[t]);
        }
        if (e < D::O_B) {
            const int i = e - D::O_A, r = i / D::NX, c = i % D::NX;
            if (r < NJ) return r == c ? 1.0 : 0.0;
            const int t = r - NJ;  // thermal row: a e_T + b 2 Ra tau_t / ktau^2 d tau_t / dq
            if (c >= NJ) return c == r ? P.th_a : 0.0;
            return P.th_b * 2.0 * P.Ra * S.tau[0][t] / (P.ktau[t] * P.ktau[t]) * dtau(P, S, t, c);
        }
        const int i = e - D::O_B, r = i / D::NU, c = i % D::NU;
        if (r < NJ) return c == r ? P.h : 0.0;
        const int t = r - NJ, v = D::NX + c;
        double a = P.th_b * 2.0 * P.Ra * S.tau[0][t] / (P.ktau[t] * P.ktau[t]) * dtau(P, S, t, v);
        if (c == t) a += P.th_b * 2.0 * u[t] / P.Rh;
        return a;
    }
};

}  // namespace mf
