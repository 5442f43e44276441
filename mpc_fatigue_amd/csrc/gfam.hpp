// Node functions of the generic stage-structured OCP (gipm.hip), host + device.
//
// Every reference transcription is, per shooting node k,
//   variables x_k (NX), u_k (NU);  cost l(x, u);  dynamics x_{k+1} = f(x, u);
//   slack rows c_lo <= c_in(x, u) <= c_hi (NI);  state equalities c_eq(x) = 0 (NE, eq_from <= k < N);
//   mixed equalities c_m(x, u) = 0 (NM, every k < N)
// and the solver needs, per node, the "node record"
//   [ l | grad l (NV) | c_in (NI) | d c_in (NI x NV) | c_eq (NE) | d c_eq / dx (NE x NX) | c_m (NM) |
//     d c_m (NM x NV) | f (NX) | A = df/dx (NX x NX) | B = df/du (NX x NU) |
//     W = grad^2 (l + yi.c_in + ye.c_eq + ym.c_m + lam.f) (NV x NV) ]
// (row-major blocks, NV = NX + NU).  Per node the equality multipliers are [ye (NEA) | ym (NM)].
// Families:
//   BoxFam    two 6-DOF Pilz arms holding a box, python/2_pilz_6_DOF/Box_Pilz_6DOF.py:219-456 (C3)
//             x = [q_L, q_R], u = [qd_L, qd_R, F_L, F_R]; c_in = [force equilibrium (3), moment
//             equilibrium (3), tau_L (6), tau_R (6)]; c_eq = |E1 - E2|^2 - L; cost 100|p_box - p_des|^2
//             + qd^T qd.
//   ChainFam  one serial arm (Pilz 3/6-DOF, C1 / C2), optionally with the motor-winding temperature
//             T as state (Tmodel_library.py:9-41, RepeatedMPCwithThermal.py:371-376):
//             x = [q, (T)], u = [qd, F]; c_in = tau; c_eq = p_f[0:2] - line_ref;
//             cost wF|F|^2 + wqd|qd|^2 + wtau|tau|^2 (+ wT|T|^2).
//   CentauroFam  two 7-DOF arms lifting a box with the winding temperatures as state (C4,
//             python/Centauro_script/RepeatedMPCwithThermal.py:154-402): x = [q (14), T (14)],
//             u = [qd (14), F_L, F_R]; c_in = tau = ID + J^T [F; 0] of both arms; c_eq = relative
//             position / orientation of the hands minus their x_0 values; c_m = force and moment
//             equilibrium; cost 100 |p_box - B|^2 + 100 |qd|^2 + 10 |F|^2.
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
    int warm_start, pad_ws;  // IPOPT warm_start_init_point constants for a w0 start (k_ginit)
    double u_init[GX_MAX];
    int force_from, tier1_from, tier1_to;  // first force control; u range regularised first (concave cost)
    int target_decimals;                   // CentauroFam: round the relative-pose targets (-1: exact)
    int dc_always;                         // delta_c from the first factorisation (rank-deficient rows)
    int filter;                            // IPOPT's globalisation (filter, watchdog, restoration; gipm.hip)
    int dbg;                               // trace horizon 0 (diagnostics, gipm.hip mf_gdebug_trace)
    int resto_hard_dyn;                    // restoration phase without elastic variables on the dynamics rows
};

template <int NX_, int NU_, int NI_, int NE_, int NM_ = 0> struct GDims {
    static constexpr int NX = NX_, NU = NU_, NI = NI_, NE = NE_, NM = NM_, NV = NX_ + NU_;
    static constexpr int NIA = NI_ > 0 ? NI_ : 1, NEA = NE_ > 0 ? NE_ : 1, NET = NEA + NM_;
    static constexpr int O_L = 0, O_GL = 1, O_CI = O_GL + NV, O_JI = O_CI + NI, O_CE = O_JI + NI * NV,
                         O_JE = O_CE + NE, O_CM = O_JE + NE * NX, O_JM = O_CM + NM, O_F = O_JM + NM * NV,
                         O_A = O_F + NX, O_B = O_A + NX * NX, O_W = O_B + NX * NU, REC = O_W + NV * NV;
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

// q direction v by the split sweep (adj.hpp node_fwd_rev_split): plain FP64 over the joints below v, Dual from v on
template <int NJ> struct GLaneInSplit {
    const double *xq, *xqd;
    int v;
    MF_HD Dual qd(int i) const { return Dual(xqd[i], 0.0); }
    MF_HD void sincos(int i, double &s, double &c) const { sincos_t(xq[i], s, c); }
    MF_HD void sincos(int i, Dual &s, Dual &c) const { sincos_t(Dual(xq[i], v == i ? 1.0 : 0.0), s, c); }
};
// C2's chain lanes (the specialised solver's eval arithmetic, csrc/ipm_kernels.hip k_eval_q / k_eval_node<..,1>):
// q direction v by the split sweep -- its column is valid in the rows >= v of the q-q block (the rows above are
// never read) -- and qd directions without the q-gradient adjoint (GQ = false: the q-qd block is read from the q
// lanes' qd-gradient).  The force row is zeroed first: the split sweep does not emit it when the frame's parent
// lies below v (the entry is exactly zero then).
template <int NJ>
MF_HD void arm_lane_split(const DevModel &M, const DevFrame &F, const double *q, const double *qd, const double *Fw,
                          const double *c, const double *seed, int v, double *col) {
    GLaneOut<NJ> o{col};
#pragma unroll
    for (int k = 0; k < 3; k++) col[GLaneOut<NJ>::HF + k] = 0.0;
    if (v < NJ) {
        GLaneInSplit<NJ> in{q, qd, v};
        node_fwd_rev_split<NJ>(M, F, F.parent, v, in, Fw, c, seed, o);
    } else {
        GLaneIn<NJ, double> in{q, qd, v};
        node_fwd_rev<double, Dual, NJ, true, false>(M, F, F.parent, in, Fw, c, seed, o);
    }
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

// ================================================================ BoxFam (C3) / shared fatigue budget (N2)
// TH: the winding temperatures of the 12 joints as state, x = [q_L, q_R, T (12)], the thermal recursion of
// Tmodel_library.py:9-41 per joint with that joint's arm torque, and one more slack row: the shared
// fatigue budget sum_j T_j <= c_hi (build-defined extension of C3; parity unpinned).
template <bool TH> struct BoxFamT {
    static constexpr int NJ = 6, NARM = 2, NDIR = 2 * NJ, NM = 2, NQ = 12;
    static constexpr bool SPLIT = false;
    using D = GDims<TH ? 2 * NQ : NQ, 18, TH ? 19 : 18, 1>;
    static constexpr int NX = D::NX;
    static constexpr int LANES = NARM * NDIR;  // derivative lanes per node
    static constexpr int LCOL = GLaneOut<NJ>::LCOL;
    static constexpr int LREF = 2;             // per-problem data (unused)
    // per-node scratch
    struct Scratch {
        double E[NARM][3], tau[NARM][NJ], seed[NARM][3], d[3], dF[3], eb[3];
        double cw[NARM][NJ], om[NARM][NJ];     // torque weights of the sweeps, thermal Gauss-Newton weights
        double ow;                             // objective weight of the derivatives (0: restoration phase)
        double col[NARM][NDIR][LCOL];
    };
    // variables: q_L 0-5, q_R 6-11, (T 12-23) | qd_L, qd_R (NX..NX+11), F_L, F_R (NX+12..NX+17)
    // kind: 0 q, 1 qd, 2 F, 3 T; arm; local index
    MF_HD static void var(int v, int &kind, int &arm, int &loc) {
        if (v < NQ) { kind = 0; arm = v / 6; loc = v % 6; }
        else if (v < NX) { kind = 3; arm = (v - NQ) / 6; loc = (v - NQ) % 6; }
        else if (v < NX + NQ) { kind = 1; arm = (v - NX) / 6; loc = (v - NX) % 6; }
        else { kind = 2; arm = (v - NX - NQ) / 3; loc = (v - NX - NQ) % 3; }
    }
    MF_HD static double ploss(const GParams &P, int j, double tau, double qd) {
        const double ia = tau / P.ktau[j];
        return P.Ra * ia * ia + qd * qd / P.Rh;
    }
    template <class MA, class FA> MF_HD static void targets(MA, FA, const GParams &, const double *, double *) {}

    // values at (x, u): l, ci, ce, f (line search / slacks)
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
        for (int j = 0; j < NQ; j++) {
            c += P.w_qdb * u[j] * u[j];
            f[j] = x[j] + P.h * u[j];
        }
        if constexpr (TH) {
            double sum = 0.0;
            for (int j = 0; j < NQ; j++) {
                const double t = j < NJ ? tL[j] : tR[j - NJ];
                f[NQ + j] = P.th_a * x[NQ + j] + P.th_b * ploss(P, j, t, u[j]);
                c += P.wT * x[NQ + j] * x[NQ + j];
                sum += x[NQ + j];
            }
            ci[18] = sum;
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
    // and the torque weights c = y_tau (+ 2 tau lam_T b Ra / ktau^2 with the thermal state)
    MF_HD static void seeds(const GParams &P, const double *u, const double *yi, const double *ye, const double *lam,
                            bool eqon, double ow, Scratch &S) {
        const double yev = eqon ? ye[0] : 0.0;
        const double *ym = yi + 3;
        double dFxy[3];
        S.ow = ow;
        for (int r = 0; r < 3; r++) {
            S.d[r] = S.E[0][r] - S.E[1][r];
            S.dF[r] = u[12 + r] - u[15 + r];
            S.eb[r] = ow * P.w_box * (0.5 * (S.E[0][r] + S.E[1][r]) - P.box_pdes[r]);
        }
        cross3(dFxy, S.dF, ym);
        for (int r = 0; r < 3; r++) {
            S.seed[0][r] = S.eb[r] + 2.0 * yev * S.d[r] + dFxy[r];
            S.seed[1][r] = S.eb[r] - 2.0 * yev * S.d[r] - dFxy[r];
        }
        for (int a = 0; a < NARM; a++)
            for (int j = 0; j < NJ; j++) {
                double w = 0.0;
                if constexpr (TH) {
                    const int i = NJ * a + j;
                    w = lam[NQ + i] * P.th_b * P.Ra / (P.ktau[i] * P.ktau[i]);
                }
                S.om[a][j] = 2.0 * w;
                S.cw[a][j] = yi[6 + NJ * a + j] + 2.0 * w * S.tau[a][j];
            }
    }
    // derivative lane t in [0, LANES): arm t / NDIR, direction t % NDIR
    template <class MA, class FA> MF_HD static void lane(MA M, FA F, const double *x, const double *u, const double *,
                           int t, Scratch &S) {
        const int a = t / NDIR, v = t % NDIR;
        arm_lane<NJ>(M[a], F[a], x + 6 * a, u + 6 * a, u + 12 + 3 * a, S.cw[a], S.seed[a], v, S.col[a][v]);
    }
    // dE_a[c] / d(var) (frame-point Jacobian; zero unless var is a q of arm a)
    MF_HD static double JE(const Scratch &S, int a, int c, int v) {
        int kind, arm, loc;
        var(v, kind, arm, loc);
        return (kind == 0 && arm == a) ? S.col[a][loc][GLaneOut<NJ>::PFD + c] : 0.0;
    }
    // d tau_(a, i) / d(var)
    MF_HD static double dtau(const Scratch &S, int a, int i, int v) {
        using L = GLaneOut<NJ>;
        int k, b, l;
        var(v, k, b, l);
        if (b != a || k == 3) return 0.0;
        if (k == 0) return S.col[a][l][L::JT + i];
        if (k == 1) return S.col[a][NJ + l][L::JT + i];
        return -S.col[a][i][L::PFD + l];  // d tau_i / d F_c = -dE_c / dq_i
    }
    // W(r, c) of the Lagrangian Hessian
    MF_HD static double Wel(const GParams &P, const double *yi, const double *ye, const double *lam, bool eqon,
                            const Scratch &S, int r, int c) {
        int kr, ar, lr, kc, ac, lc;
        var(r, kr, ar, lr);
        var(c, kc, ac, lc);
        using L = GLaneOut<NJ>;
        double w = 0.0;
        if (kr == 3 || kc == 3) return (r == c) ? 2.0 * S.ow * P.wT : 0.0;  // T enters linearly (plus wT |T|^2)
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
        if constexpr (TH) {  // thermal Gauss-Newton: sum_i om_i dtau_i/dr dtau_i/dc (same arm)
            if (ar == ac) {
                double acc = 0.0;
                for (int i = 0; i < NJ; i++) acc += S.om[ar][i] * dtau(S, ar, i, r) * dtau(S, ar, i, c);
                w += acc;
            }
        }
        // algebraic part: J_E^T (d^2 g / dE dE) J_E and the E-F cross terms of the moment rows
        const double yev = eqon ? ye[0] : 0.0;
        if (kr == 0 && kc == 0) {
            const double g = 0.5 * S.ow * P.w_box + (ar == ac ? 2.0 : -2.0) * yev;
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
        if (r == c && kr == 1) {
            w += 2.0 * S.ow * P.w_qdb;
            if constexpr (TH) w += lam[NQ + NJ * ar + lr] * P.th_b * 2.0 / P.Rh;
        }
        return w;
    }
    // record entry e (D offsets)
    MF_HD static double rec(const GParams &P, const double *x, const double *u, const double *yi, const double *ye,
                            const double *lam, bool eqon, const Scratch &S, int e, const double *) {
        if (e >= D::O_W) {
            const int i = e - D::O_W;
            return Wel(P, yi, ye, lam, eqon, S, i / D::NV, i % D::NV);
        }
        if (e == D::O_L) {
            double c = 0.0;
            for (int r = 0; r < 3; r++) {
                const double v = 0.5 * (S.E[0][r] + S.E[1][r]) - P.box_pdes[r];
                c += P.w_box * v * v;
            }
            for (int j = 0; j < NQ; j++) {
                c += P.w_qdb * u[j] * u[j];
                if constexpr (TH) c += P.wT * x[NQ + j] * x[NQ + j];
            }
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
            if (k == 3) return 2.0 * S.ow * P.wT * x[v];
            return k == 1 ? 2.0 * S.ow * P.w_qdb * u[v - NX] : 0.0;
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
            if (r < 18) return r < 12 ? S.tau[0][r - 6] : S.tau[1][r - 12];
            double sum = 0.0;  // shared fatigue budget
            for (int j = 0; j < NQ; j++) sum += x[NQ + j];
            return sum;
        }
        if (e < D::O_CE) {  // d c_in
            const int i = e - D::O_JI, r = i / D::NV, v = i % D::NV;
            int k, a, l;
            var(v, k, a, l);
            if (r == 18) return k == 3 ? 1.0 : 0.0;
            if (k == 3) return 0.0;
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
            return dtau(S, ta, ti, v);
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
        if (e < D::O_A) {  // f = [q + h qd, a T + b Ploss]
            const int j = e - D::O_F;
            if (j < NQ) return x[j] + P.h * u[j];
            const int t = j - NQ;
            return P.th_a * x[j] + P.th_b * ploss(P, t, S.tau[t / NJ][t % NJ], u[t]);
        }
        if (e < D::O_B) {
            const int i = e - D::O_A, r = i / NX, c = i % NX;
            if (r < NQ) return r == c ? 1.0 : 0.0;
            const int t = r - NQ;
            if (c >= NQ) return c == r ? P.th_a : 0.0;
            return P.th_b * 2.0 * P.Ra * S.tau[t / NJ][t % NJ] / (P.ktau[t] * P.ktau[t]) * dtau(S, t / NJ, t % NJ, c);
        }
        const int i = e - D::O_B, r = i / D::NU, c = i % D::NU;
        if (r < NQ) return (c == r) ? P.h : 0.0;
        const int t = r - NQ;
        double a = P.th_b * 2.0 * P.Ra * S.tau[t / NJ][t % NJ] / (P.ktau[t] * P.ktau[t]) * dtau(S, t / NJ, t % NJ, NX + c);
        if (c == t) a += P.th_b * 2.0 * u[t] / P.Rh;
        return a;
    }
};
using BoxFam = BoxFamT<false>;
using BoxThermFam = BoxFamT<true>;

// ================================================================ ChainFam (C1, C2, thermal)
template <int NJ_, int NF_, int NE_, bool THERMAL_> struct ChainFam {
    static constexpr int NJ = NJ_, NF = NF_, NDIR = 2 * NJ_, NM = 1;
    static constexpr bool TH = THERMAL_;
    // C2 (6 joints, one force, the line rows, no thermal state): the split lanes (arm_lane_split), evaluated
    // direction-major by k_geval_chain (csrc/gkkt_chain.hpp)
    static constexpr bool SPLIT = NJ_ == 6 && NF_ == 1 && NE_ == 2 && !THERMAL_;
    using D = GDims<(THERMAL_ ? 2 : 1) * NJ_, NJ_ + NF_, NJ_, NE_>;
    static constexpr int LANES = NDIR;
    static constexpr int LCOL = GLaneOut<NJ>::LCOL;
    struct Scratch {
        double E[1][3], tau[1][NJ], pf[3], cw[NJ], om[NJ], seed[3], Fw[3];
        double ow;  // objective weight of the derivatives (0: restoration phase)
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
    static constexpr int LREF = 2;    // per-problem data: the line reference
    template <class MA, class FA> MF_HD static void targets(MA, FA, const GParams &, const double *, double *) {}
    template <class MA, class FA> MF_HD static void prepass(MA M, FA F, const GParams &P, const double *x, const double *u,
                              int, Scratch &S) {
        world_force(P, u, S.Fw);
        arm_values<NJ>(M[0], F[0], x, u, S.Fw, S.tau[0], S.pf);
    }
    // torque weights c_j = yi_j + 2 tau_j (wtau + lam_T,j b Ra / ktau_j^2), Gauss-Newton weights
    // om_j = 2 (wtau + lam_T,j b Ra / ktau_j^2), frame seed = (ye, 0)
    MF_HD static void seeds(const GParams &P, const double *, const double *yi, const double *ye, const double *lam,
                            bool eqon, double ow, Scratch &S) {
        S.ow = ow;
        for (int j = 0; j < NJ; j++) {
            double w = ow * P.wtau;
            if constexpr (TH) w += lam[NJ + j] * P.th_b * P.Ra / (P.ktau[j] * P.ktau[j]);
            S.om[j] = 2.0 * w;
            S.cw[j] = yi[j] + 2.0 * w * S.tau[0][j];
        }
        for (int r = 0; r < 3; r++) S.seed[r] = (eqon && r < NE_) ? ye[r] : 0.0;
    }
    template <class MA, class FA> MF_HD static void lane(MA M, FA F, const double *x, const double *u, const double *, int v,
                           Scratch &S) {
        if constexpr (SPLIT) arm_lane_split<NJ>(M[0], F[0], x, u, S.Fw, S.cw, S.seed, v, S.col[0][v]);
        else arm_lane<NJ>(M[0], F[0], x, u, S.Fw, S.cw, S.seed, v, S.col[0][v]);
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
            else if (SPLIT && kr == 0 && kc == 0) w = lr >= lc ? colent(lc, 0, lr) : colent(lr, 0, lc);  // lower triangle
            else if (SPLIT && kr == 0) w = colent(lr, 1, lc);  // the q_lr lane's qd-gradient
            else if (SPLIT && kc == 0) w = colent(lc, 1, lr);
            else w = 0.5 * (colent(dc, kr, lr) + colent(dr, kc, lc));
        }
        if (kr != 3 && kc != 3) {
            double acc = 0.0;
            for (int j = 0; j < NJ; j++) acc += S.om[j] * dtau(P, S, j, r) * dtau(P, S, j, c);
            w += acc;
        }
        if (r == c) {
            if (kr == 1) {
                w += 2.0 * S.ow * P.wqd;
                if constexpr (TH) w += lam[NJ + lr] * P.th_b * 2.0 / P.Rh;
            }
            if (kr == 2) w += 2.0 * S.ow * P.wF;
            if (kr == 3) w += 2.0 * S.ow * P.wT;
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
            return S.ow * g;
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

// ================================================================ CentauroFam (C4)
// World pose of an arm's frame and the world axes / origins of its joints (q'' = qd = 0 sweep).
template <int NJ> struct ArmPose {
    double z[NJ][3], o[NJ][3], p[3], R[9];
};
template <int NJ> MF_HD void arm_pose(const DevModel &M, const DevFrame &F, const double *q, ArmPose<NJ> &P) {
    JacVis<double, NJ> jv;
    jv.F = &F;
    double zero[NJ];
    for (int i = 0; i < NJ; i++) zero[i] = 0.0;
    ne_pass<double>(M, NJ, q, zero, (const double *)nullptr, jv);
    for (int i = 0; i < NJ; i++)
        for (int k = 0; k < 3; k++) { P.z[i][k] = jv.z[i][k]; P.o[i][k] = jv.o[i][k]; }
    for (int k = 0; k < 3; k++) P.p[k] = jv.pf[k];
    for (int k = 0; k < 9; k++) P.R[k] = jv.Rf[k];
}

// skew part of M (row-major) in the reference's component order: (M21 - M12, M20 - M02, M10 - M01) / 2
// (RepeatedMPCwithThermal.py:276-284: ex = R_skew[2,1], ey = R_skew[2,0], ez = R_skew[1,0])
MF_HD void skew_ext(const double *M, double *e) {
    e[0] = 0.5 * (M[7] - M[5]);
    e[1] = 0.5 * (M[6] - M[2]);
    e[2] = 0.5 * (M[3] - M[1]);
}
// A B^T (row-major 3x3)
MF_HD void mul_abt(const double *A, const double *B, double *C) {
    for (int m = 0; m < 3; m++)
        for (int n = 0; n < 3; n++) C[3 * m + n] = A[3 * m] * B[3 * n] + A[3 * m + 1] * B[3 * n + 1] + A[3 * m + 2] * B[3 * n + 2];
}

struct CentauroFam {
    static constexpr int NJ = 7, NARM = 2, NDIR = 2 * NJ, NM = 2, NQ = 2 * NJ;
    static constexpr bool SPLIT = false;
    using D = GDims<2 * NQ, NQ + 6, NQ, 6, 6>;
    static constexpr int LANES = NARM * NDIR;  // derivative lanes per node
    static constexpr int PRE = NARM;
    static constexpr int LREF = 6;             // per-problem targets: relative position (3), orientation (3)
    static constexpr int LCOL = GLaneOut<NJ>::LCOL;
    struct Scratch {
        double tau[NARM][NJ], c[NARM][NJ], om[NARM][NJ];
        ArmPose<NJ> P[NARM];
        double eb[3], dF[3], yr[3], yo[3], ym[3];
        double ow;  // objective weight of the derivatives (0: restoration phase)
        double col[NARM][NDIR][LCOL];
    };
    // variables: q 0..13 (arm v / 7), T 14..27 | qd 28..41, F_L 42..44, F_R 45..47
    // kind: 0 q, 1 T, 2 qd, 3 F; arm; local index
    MF_HD static void var(int v, int &kind, int &arm, int &loc) {
        if (v < NQ) { kind = 0; arm = v / NJ; loc = v % NJ; }
        else if (v < 2 * NQ) { kind = 1; arm = (v - NQ) / NJ; loc = (v - NQ) % NJ; }
        else if (v < 3 * NQ) { kind = 2; arm = (v - 2 * NQ) / NJ; loc = (v - 2 * NQ) % NJ; }
        else { kind = 3; arm = (v - 3 * NQ) / 3; loc = (v - 3 * NQ) % 3; }
    }
    MF_HD static void neg_force(const double *u, int a, double *Fw) {  // tau = ID + J^T F: Fw = -F
        for (int r = 0; r < 3; r++) Fw[r] = -u[NQ + 3 * a + r];
    }
    MF_HD static double ploss(const GParams &P, int j, double tau, double qd) {
        const double ia = tau / P.ktau[j];
        return P.Ra * ia * ia + qd * qd / P.Rh;
    }
    // relative position R_L^T (p_R - p_L) and orientation error of R_L R_R^T
    MF_HD static void relpose(const ArmPose<NJ> &L, const ArmPose<NJ> &Rr, double *r6) {
        double d[3], Ro[9];
        for (int k = 0; k < 3; k++) d[k] = Rr.p[k] - L.p[k];
        for (int b = 0; b < 3; b++) r6[b] = L.R[b] * d[0] + L.R[3 + b] * d[1] + L.R[6 + b] * d[2];
        mul_abt(L.R, Rr.R, Ro);
        skew_ext(Ro, r6 + 3);
    }
    template <class MA, class FA> MF_HD static void targets(MA M, FA F, const GParams &P, const double *x0, double *t) {
        ArmPose<NJ> A0, A1;
        arm_pose<NJ>(M[0], F[0], x0, A0);
        arm_pose<NJ>(M[1], F[1], x0 + NJ, A1);
        relpose(A0, A1, t);
        // the orientation target is rounded as the MPC restart rounds RelativeOrientation_0
        // (RepeatedMPCwithThermal.py:485-486); the position rows chain node k to node k-1 (L255-272), so
        // for k >= 1 they hold the exact relative position of x_0
        if (P.target_decimals >= 0) {
            const double sc = pow(10.0, (double)P.target_decimals);
            for (int i = 3; i < 6; i++) t[i] = rint(t[i] * sc) / sc;
        }
    }
    template <class MA, class FA> MF_HD static void values(MA M, FA F, const GParams &P, const double *x, const double *u,
                             const double *tg, double &l, double *ci, double *ce, double *f) {
        double tau[NQ];
        ArmPose<NJ> A[NARM];
        for (int a = 0; a < NARM; a++) {
            double Fw[3], pf[3];
            neg_force(u, a, Fw);
            arm_values<NJ>(M[a], F[a], x + NJ * a, u + NJ * a, Fw, tau + NJ * a, pf);
            arm_pose<NJ>(M[a], F[a], x + NJ * a, A[a]);
        }
        double r6[6];
        relpose(A[0], A[1], r6);
        for (int i = 0; i < 6; i++) ce[i] = r6[i] - tg[i];
        const double *FL = u + NQ, *FR = u + NQ + 3;
        double dd[3], dF[3], m[3];
        for (int r = 0; r < 3; r++) { dd[r] = A[0].p[r] - A[1].p[r]; dF[r] = FL[r] - FR[r]; }
        cross3(m, dd, dF);
        ce[6] = FL[2] + FR[2] - P.box_mg;
        ce[7] = FL[0] + FR[0];
        ce[8] = FL[1] + FR[1];
        for (int r = 0; r < 3; r++) ce[9 + r] = m[r];
        double c = 0.0;
        for (int r = 0; r < 3; r++) {
            const double e = 0.5 * (A[0].p[r] + A[1].p[r]) - P.box_pdes[r];
            c += P.w_box * e * e + P.wF * (FL[r] * FL[r] + FR[r] * FR[r]);
        }
        for (int j = 0; j < NQ; j++) {
            ci[j] = tau[j];
            c += P.w_qdb * u[j] * u[j] + P.wT * x[NQ + j] * x[NQ + j];
            f[j] = x[j] + P.h * u[j];
            f[NQ + j] = P.th_a * x[NQ + j] + P.th_b * ploss(P, j, tau[j], u[j]);
        }
        l = c;
    }
    // pre-pass lane a: torques and pose of arm a
    template <class MA, class FA> MF_HD static void prepass(MA M, FA F, const GParams &, const double *x, const double *u,
                              int a, Scratch &S) {
        double Fw[3], pf[3];
        neg_force(u, a, Fw);
        arm_values<NJ>(M[a], F[a], x + NJ * a, u + NJ * a, Fw, S.tau[a], pf);
        arm_pose<NJ>(M[a], F[a], x + NJ * a, S.P[a]);
    }
    // torque weights c = yi + 2 tau lam_T b Ra / ktau^2 (the arm sweeps), Gauss-Newton weights om, and the
    // multipliers of the pose functions (closed form)
    MF_HD static void seeds(const GParams &P, const double *u, const double *yi, const double *ye, const double *lam,
                            bool eqon, double ow, Scratch &S) {
        S.ow = ow;
        for (int a = 0; a < NARM; a++)
            for (int j = 0; j < NJ; j++) {
                const int i = NJ * a + j;
                const double w = lam[NQ + i] * P.th_b * P.Ra / (P.ktau[i] * P.ktau[i]);
                S.om[a][j] = 2.0 * w;
                S.c[a][j] = yi[i] + 2.0 * w * S.tau[a][j];
            }
        for (int r = 0; r < 3; r++) {
            S.eb[r] = ow * P.w_box * (0.5 * (S.P[0].p[r] + S.P[1].p[r]) - P.box_pdes[r]);
            S.dF[r] = u[NQ + r] - u[NQ + 3 + r];
            S.yr[r] = eqon ? ye[r] : 0.0;
            S.yo[r] = eqon ? ye[3 + r] : 0.0;
            S.ym[r] = ye[D::NEA + 3 + r];  // moment rows (mixed rows 3..5)
        }
    }
    template <class MA, class FA> MF_HD static void lane(MA M, FA F, const double *x, const double *u, const double *,
                           int t, Scratch &S) {
        const int a = t / NDIR, v = t % NDIR;
        double Fw[3];
        neg_force(u, a, Fw);
        const double zero3[3] = {0.0, 0.0, 0.0};
        arm_lane<NJ>(M[a], F[a], x + NJ * a, u + NJ * a, Fw, S.c[a], zero3, v, S.col[a][v]);
    }

    // ---- pose variations (closed form, rigid-rotation rule) -------------------------------------
    struct PV {
        double dp[NARM][3], dR[NARM][9];
    };
    // first-order variation of joint j of arm a: dp = z x (p - o_j), dR = [z]x R
    MF_HD static void var1(const Scratch &S, int a, int j, PV &V) {
        for (int b = 0; b < NARM; b++) {
            for (int k = 0; k < 3; k++) V.dp[b][k] = 0.0;
            for (int k = 0; k < 9; k++) V.dR[b][k] = 0.0;
        }
        const ArmPose<NJ> &A = S.P[a];
        const double *z = A.z[j];
        double r[3];
        for (int k = 0; k < 3; k++) r[k] = A.p[k] - A.o[j][k];
        cross3(V.dp[a], z, r);
        for (int c = 0; c < 3; c++) {
            const double col[3] = {A.R[c], A.R[3 + c], A.R[6 + c]};
            double t[3];
            cross3(t, z, col);
            for (int k = 0; k < 3; k++) V.dR[a][3 * k + c] = t[k];
        }
    }
    // second-order variation of joints j, k of arm a (i = min, m = max):
    // d2p = z_i x (z_m x (p - o_m)), d2R = [z_i]x [z_m]x R
    MF_HD static void var2(const Scratch &S, int a, int j, int k, PV &V) {
        for (int b = 0; b < NARM; b++) {
            for (int c = 0; c < 3; c++) V.dp[b][c] = 0.0;
            for (int c = 0; c < 9; c++) V.dR[b][c] = 0.0;
        }
        const int i = j < k ? j : k, m = j < k ? k : j;
        const ArmPose<NJ> &A = S.P[a];
        double r[3], t[3];
        for (int c = 0; c < 3; c++) r[c] = A.p[c] - A.o[m][c];
        cross3(t, A.z[m], r);
        cross3(V.dp[a], A.z[i], t);
        for (int c = 0; c < 3; c++) {
            const double col[3] = {A.R[c], A.R[3 + c], A.R[6 + c]};
            double t1[3], t2[3];
            cross3(t1, A.z[m], col);
            cross3(t2, A.z[i], t1);
            for (int q = 0; q < 3; q++) V.dR[a][3 * q + c] = t2[q];
        }
    }
    // directional derivative of the pose functions along a variation, weighted:
    //   eb . (dp_L + dp_R)                               (cost: w_box |p_box - B|^2)
    // + yr . (dR_L^T (p_R - p_L) + R_L^T (dp_R - dp_L))  (relative position rows)
    // + yo . ext(dR_L R_R^T + R_L dR_R^T)                 (orientation rows)
    // + ym . ((dp_L - dp_R) x dF)                         (moment rows)
    MF_HD static double D1(const Scratch &S, const double *eb, const double *yr, const double *yo, const double *ym,
                           const PV &V) {
        const ArmPose<NJ> &L = S.P[0], &Rr = S.P[1];
        double acc = 0.0, d[3], dd[3], m[3];
        for (int k = 0; k < 3; k++) {
            d[k] = Rr.p[k] - L.p[k];
            dd[k] = V.dp[1][k] - V.dp[0][k];
            acc += eb[k] * (V.dp[0][k] + V.dp[1][k]);
        }
        for (int b = 0; b < 3; b++) {
            const double t = V.dR[0][b] * d[0] + V.dR[0][3 + b] * d[1] + V.dR[0][6 + b] * d[2] +
                             L.R[b] * dd[0] + L.R[3 + b] * dd[1] + L.R[6 + b] * dd[2];
            acc += yr[b] * t;
        }
        double M1[9], M2[9], e1[3], e2[3];
        mul_abt(V.dR[0], Rr.R, M1);
        mul_abt(L.R, V.dR[1], M2);
        skew_ext(M1, e1);
        skew_ext(M2, e2);
        for (int b = 0; b < 3; b++) acc += yo[b] * (e1[b] + e2[b]);
        const double ndd[3] = {-dd[0], -dd[1], -dd[2]};  // dp_L - dp_R
        cross3(m, ndd, S.dF);
        for (int b = 0; b < 3; b++) acc += ym[b] * m[b];
        return acc;
    }
    // the bilinear (second-order) part of the weighted pose functions on two variations
    MF_HD static double D2(const GParams &P, const Scratch &S, const PV &V, const PV &W) {
        const ArmPose<NJ> &L = S.P[0], &Rr = S.P[1];
        double acc = 0.0;
        for (int k = 0; k < 3; k++) acc += 0.5 * S.ow * P.w_box * (V.dp[0][k] + V.dp[1][k]) * (W.dp[0][k] + W.dp[1][k]);
        for (int b = 0; b < 3; b++) {
            double t = 0.0;
            for (int k = 0; k < 3; k++)
                t += V.dR[0][3 * k + b] * (W.dp[1][k] - W.dp[0][k]) + W.dR[0][3 * k + b] * (V.dp[1][k] - V.dp[0][k]);
            acc += S.yr[b] * t;
        }
        double M1[9], M2[9], e1[3], e2[3];
        mul_abt(V.dR[0], W.dR[1], M1);
        mul_abt(W.dR[0], V.dR[1], M2);
        skew_ext(M1, e1);
        skew_ext(M2, e2);
        for (int b = 0; b < 3; b++) acc += S.yo[b] * (e1[b] + e2[b]);
        (void)L; (void)Rr;
        return acc;
    }
    // d tau_(a, i) / d(var)
    MF_HD static double dtau(const Scratch &S, int a, int i, int v) {
        using L = GLaneOut<NJ>;
        int k, b, l;
        var(v, k, b, l);
        if (b != a) return 0.0;
        if (k == 0) return S.col[a][l][L::JT + i];
        if (k == 2) return S.col[a][NJ + l][L::JT + i];
        if (k == 3) return S.col[a][i][L::PFD + l];  // + J_lin[l][i] = d p_l / d q_i
        return 0.0;
    }
    MF_HD static double Wel(const GParams &P, const double *u, const double *lam, const Scratch &S, int r, int c) {
        using L = GLaneOut<NJ>;
        int kr, ar, lr, kc, ac, lc;
        var(r, kr, ar, lr);
        var(c, kc, ac, lc);
        double w = 0.0;
        // arm sweeps: phi_a = c_a . tau_a(q, qd, Fw = -F_a)
        if (ar == ac && kr != 1 && kc != 1 && !(kr == 3 && kc == 3)) {
            auto colent = [&](int vdir, int kind, int loc) {
                const double *cl = S.col[ar][vdir];
                return kind == 0 ? cl[L::HQ + loc] : (kind == 2 ? cl[L::HQD + loc] : -cl[L::HF + loc]);
            };
            const int dr = kr == 0 ? lr : NJ + lr, dc = kc == 0 ? lc : NJ + lc;
            if (kr == 3) w = colent(dc, kr, lr);
            else if (kc == 3) w = colent(dr, kc, lc);
            else w = 0.5 * (colent(dc, kr, lr) + colent(dr, kc, lc));
        }
        // thermal Gauss-Newton: sum_i om_i dtau_i/dr dtau_i/dc (same arm)
        if (ar == ac && kr != 1 && kc != 1) {
            double acc = 0.0;
            for (int i = 0; i < NJ; i++) acc += S.om[ar][i] * dtau(S, ar, i, r) * dtau(S, ar, i, c);
            w += acc;
        }
        // pose functions
        if (kr == 0 && kc == 0) {
            PV V, Wv;
            var1(S, ar, lr, V);
            var1(S, ac, lc, Wv);
            w += D2(P, S, V, Wv);
            if (ar == ac) {
                PV V2;
                var2(S, ar, lr, lc, V2);
                w += D1(S, S.eb, S.yr, S.yo, S.ym, V2);
            }
        } else if ((kr == 0 && kc == 3) || (kr == 3 && kc == 0)) {
            // moment rows: ym . ((dp_L - dp_R) x dF), dF = F_L - F_R
            const int aq = kr == 0 ? ar : ac, jq = kr == 0 ? lr : lc, af = kr == 3 ? ar : ac, lf = kr == 3 ? lr : lc;
            PV V;
            var1(S, aq, jq, V);
            double ddp[3], e[3] = {0.0, 0.0, 0.0}, m[3];
            for (int k = 0; k < 3; k++) ddp[k] = V.dp[0][k] - V.dp[1][k];
            e[lf] = af == 0 ? 1.0 : -1.0;
            cross3(m, ddp, e);
            w += S.ym[0] * m[0] + S.ym[1] * m[1] + S.ym[2] * m[2];
        }
        if (r == c) {
            if (kr == 2) w += 2.0 * S.ow * P.w_qdb + lam[NQ + NJ * ar + lr] * P.th_b * 2.0 / P.Rh;
            if (kr == 3) w += 2.0 * S.ow * P.wF;
            if (kr == 1) w += 2.0 * S.ow * P.wT;
        }
        return w;
    }
    MF_HD static double rec(const GParams &P, const double *x, const double *u, const double *yi, const double *ye,
                            const double *lam, bool eqon, const Scratch &S, int e, const double *tg) {
        if (e >= D::O_W) {
            const int i = e - D::O_W;
            return Wel(P, u, lam, S, i / D::NV, i % D::NV);
        }
        const double *FL = u + NQ, *FR = u + NQ + 3;
        if (e == D::O_L) {
            double c = 0.0;
            for (int r = 0; r < 3; r++) {
                const double v = 0.5 * (S.P[0].p[r] + S.P[1].p[r]) - P.box_pdes[r];
                c += P.w_box * v * v + P.wF * (FL[r] * FL[r] + FR[r] * FR[r]);
            }
            for (int j = 0; j < NQ; j++) c += P.w_qdb * u[j] * u[j] + P.wT * x[NQ + j] * x[NQ + j];
            return c;
        }
        const double z3[3] = {0.0, 0.0, 0.0};
        if (e < D::O_CI) {  // grad l
            const int v = e - D::O_GL;
            int k, a, l;
            var(v, k, a, l);
            if (k == 0) {
                PV V;
                var1(S, a, l, V);
                return D1(S, S.eb, z3, z3, z3, V);
            }
            if (k == 1) return 2.0 * S.ow * P.wT * x[v];
            if (k == 2) return 2.0 * S.ow * P.w_qdb * u[v - D::NX];
            return 2.0 * S.ow * P.wF * u[v - D::NX];
        }
        if (e < D::O_JI) {
            const int r = e - D::O_CI;
            return S.tau[r / NJ][r % NJ];
        }
        if (e < D::O_CE) {
            const int i = e - D::O_JI, r = i / D::NV, v = i % D::NV;
            return dtau(S, r / NJ, r % NJ, v);
        }
        if (e < D::O_JE) {  // relative pose rows
            double r6[6];
            relpose(S.P[0], S.P[1], r6);
            return r6[e - D::O_CE] - tg[e - D::O_CE];
        }
        if (e < D::O_CM) {  // d (relative pose) / dx
            const int i = e - D::O_JE, row = i / D::NX, v = i % D::NX;
            if (v >= NQ) return 0.0;
            double y[3] = {0.0, 0.0, 0.0};
            y[row % 3] = 1.0;
            PV V;
            var1(S, v / NJ, v % NJ, V);
            return row < 3 ? D1(S, z3, y, z3, z3, V) : D1(S, z3, z3, y, z3, V);
        }
        if (e < D::O_JM) {  // equilibrium rows
            const int r = e - D::O_CM;
            if (r == 0) return FL[2] + FR[2] - P.box_mg;
            if (r == 1) return FL[0] + FR[0];
            if (r == 2) return FL[1] + FR[1];
            double dd[3], m[3];
            for (int k = 0; k < 3; k++) dd[k] = S.P[0].p[k] - S.P[1].p[k];
            cross3(m, dd, S.dF);
            return m[r - 3];
        }
        if (e < D::O_F) {  // d (equilibrium) / d(x, u)
            const int i = e - D::O_JM, row = i / D::NV, v = i % D::NV;
            int k, a, l;
            var(v, k, a, l);
            if (row < 3) {
                const int comp = row == 0 ? 2 : row - 1;
                return (k == 3 && l == comp) ? 1.0 : 0.0;
            }
            const int mr = row - 3;
            if (k == 0) {
                double y[3] = {0.0, 0.0, 0.0};
                y[mr] = 1.0;
                PV V;
                var1(S, a, l, V);
                return D1(S, z3, z3, z3, y, V);
            }
            if (k == 3) {  // d/dF_(a, l) of (p_L - p_R) x (F_L - F_R)
                double dd[3];
                for (int q = 0; q < 3; q++) dd[q] = S.P[0].p[q] - S.P[1].p[q];
                return (a == 0 ? 1.0 : -1.0) * skew_el(dd, mr, l);
            }
            return 0.0;
        }
        if (e < D::O_A) {
            const int j = e - D::O_F;
            if (j < NQ) return x[j] + P.h * u[j];
            const int t = j - NQ;
            return P.th_a * x[j] + P.th_b * ploss(P, t, S.tau[t / NJ][t % NJ], u[t]);
        }
        if (e < D::O_B) {
            const int i = e - D::O_A, r = i / D::NX, c = i % D::NX;
            if (r < NQ) return r == c ? 1.0 : 0.0;
            const int t = r - NQ;
            if (c >= NQ) return c == r ? P.th_a : 0.0;
            const double tt = S.tau[t / NJ][t % NJ];
            return P.th_b * 2.0 * P.Ra * tt / (P.ktau[t] * P.ktau[t]) * dtau(S, t / NJ, t % NJ, c);
        }
        const int i = e - D::O_B, r = i / D::NU, c = i % D::NU;
        if (r < NQ) return c == r ? P.h : 0.0;
        const int t = r - NQ, v = D::NX + c;
        const double tt = S.tau[t / NJ][t % NJ];
        double a = P.th_b * 2.0 * P.Ra * tt / (P.ktau[t] * P.ktau[t]) * dtau(S, t / NJ, t % NJ, v);
        if (c == t) a += P.th_b * 2.0 * u[t] / P.Rh;
        return a;
    }
};

}  // namespace mf
