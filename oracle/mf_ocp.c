/*
 * ORACLE — test infrastructure only.  Generic stage-structured CPU restatement
 * (plain C99, FP64) of the reference's OCP solves.  Only tests/,
 * __graft_entry__.smoke() and bench.py's cpu_baseline leg may load it, and only
 * as the checker / timed CPU baseline; libmpcfatigue.so never links it.
 *
 * NLP (one horizon; every reference transcription has this shape):
 *   w = [x_0 | (u_k, x_{k+1}) for k < N]          (force_optimization_pilz_6DOF.py:103-172,
 *                                                  Box_Pilz_6DOF.py:213-436,
 *                                                  RepeatedMPCwithThermal.py:183-402)
 *   min  sum_k l(x_k, u_k)
 *   s.t. x_{k+1} = f(x_k, u_k)                    explicit Euler (+ thermal recursion)
 *        c_lo[k] <= c_in(x_k, u_k) <= c_hi[k]     torques, equilibrium rows (slack rows)
 *        c_eq(x_k) = 0,  eq_from <= k < N         state-only equalities (line, distance, relative pose)
 *        c_m(x_k, u_k) = 0,  k < N                 mixed equalities (Centauro equilibrium rows)
 *        x_lo <= x_k <= x_hi (k >= 1), u_lo[k] <= u_k <= u_hi[k]  (lo == hi: fixed)
 * Families (node functions, hyper-dual so every derivative is exact):
 *   MFG_CHAIN  one serial arm: Pilz 3/6-DOF (C1, C2), optionally with the motor-winding
 *              thermal state T (Tmodel_library.py:9-41, RepeatedMPCwithThermal.py:371-376)
 *   MFG_BOX    two arms holding a box (C3, Box_Pilz_6DOF.py:219-456)
 *   MFG_CENT   the Centauro thermal box lift (C4, RepeatedMPCwithThermal.py:154-402) on two 7-DOF
 *              substitute arms: tau = ID + J^T W, relative pose, equilibrium, thermal state
 * Solver: the IPOPT-style primal-dual interior point of DESIGN.md section 4 (the same
 * iteration mf_oracle.c runs for the Pilz family), with a block-tridiagonal KKT over
 * shooting nodes factorised block by block with Bunch-Kaufman (inertia = sum over
 * blocks, Sylvester) -- an algorithm independent of the device's Riccati recursion.
 */
#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

#include "hd_kin.h"

/* Where the host IPM's time goes (bench.py cpu_baseline split): seconds summed over every solve since
 * the last mfg_time_reset, per phase: 0 node derivatives, 1 KKT factorisation (every inertia try),
 * 2 Newton directions (incl. second-order corrections), 3 line-search merit evaluations, 4 total. */
#include <time.h>
static double g_tsplit[5];
static double wall_s(void) {
    struct timespec t;
    clock_gettime(CLOCK_MONOTONIC, &t);
    return t.tv_sec + 1e-9 * t.tv_nsec;
}
void mfg_time_reset(void) { memset(g_tsplit, 0, sizeof g_tsplit); }
void mfg_time_get(double *out5) { memcpy(out5, g_tsplit, sizeof g_tsplit); }

#define GX 32              /* max state size */
#define GU 32              /* max control size */
#define GV (GX + GU)       /* max node variables */
#define GI 48              /* max slack (inequality) rows */
#define GE 16              /* max equality rows (state + mixed) */
#define GB (2 * GX + GU + GE)

enum { MFG_CHAIN = 0, MFG_BOX = 1, MFG_CENT = 2 };

typedef struct {
    int family;
    int N;
    double h;
    int nx, nu, ni, ne;
    int force_from;                 /* u index of the first force component (F_init / warm start) */
    int tier1_from, tier1_to;       /* u range regularised first (concave cost block), empty if equal */
    /* MFG_CHAIN */
    double frame[2][13];            /* frame records (parent, R row-major, t) of chain 0 / 1 */
    int nf;
    double fdir[9];
    int use_line;
    double line_ref[2];
    double wF, wqd, wtau;
    int thermal;
    double th_a, th_b, Ra, Rh;      /* T' = th_a T + th_b (Ra (tau/ktau)^2 + qd^2 / Rh) */
    double ktau[MJ];
    double wT;                      /* optional thermal stage cost wT |T|^2 (0 in the reference) */
    /* MFG_BOX */
    double box_mg, box_L, box_pdes[3], w_box, w_qd;
    /* bounds / data */
    double x0[GX];
    double x_lo[GX], x_hi[GX];      /* states k >= 1 */
    const double *u_lo, *u_hi;      /* N x nu */
    const double *c_lo, *c_hi;      /* N x ni */
    int eq_from;
    /* MFG_CENT (box_mg, box_pdes, w_box, w_qd, wF and the thermal fields above are shared) */
    int nem;                        /* mixed equality rows c_m(x, u) after the ne state rows */
    double relpos0[3], orient0[3];  /* relative-pose targets (set by the solver from x_0) */
    int target_decimals;            /* round the targets (mpc_principal.py:371-373), -1: exact */
    int dc_always;                  /* structurally rank-deficient equality rows: delta_c from the start */
} mfg_ocp;

typedef struct {
    double tol, constr_viol_tol;
    int max_iter;
    double mu_init;
    int init_zero;                  /* 1: IPOPT's x0 = 0 for every free variable; 0: hold x_0 */
    int verbose;
    double F_init;
    const double *w0;               /* warm start (w layout) or NULL */
    double bound_relax;             /* IPOPT bound_relax_factor (0 = off) */
    const double *u_init;           /* initial control (nu) for every node, or NULL (0 / F_init) */
    int max_soc;                    /* IPOPT max_soc (second-order corrections per iteration; 0 = off) */
    double *dual_out;               /* diagnostics: [lam | yi | ye | zxL | zxU | zuL | zuU | vL | vU | mu] or NULL */
    /* optional node-record provider (CPU baseline: the product's forward-over-reverse node functions
     * compiled for the host, oracle/cpu_fast.cpp); NULL = the hyper-dual restatement below.  Record layout
     * [l | grad l | c_in | d c_in | c_eq | d c_eq/dx | f | A | B | W] as csrc/gfam.hpp. */
    int (*node_cb)(void *ctx, const double *xu, const double *yi, const double *ye, const double *lam,
                   const double *lref, int eqon, double *rec);
    void *node_ctx;
    /* optional value provider of the same library (l, c_in, c_eq, f at one node); NULL = hyper-dual */
    int (*val_cb)(void *ctx, const double *x, const double *u, const double *lref, double *l, double *ci,
                  double *ce, double *f);
    /* IPOPT warm_start_init_point = yes (RepeatedMPCwithThermal.py:445-446, mpc_principal.py:349-351): the
     * primal point of w0 pushed by warm_start_bound_push / _frac = 1e-3 (slacks: warm_start_slack_bound_*
     * = 1e-3), bound multipliers max(given, warm_start_mult_bound_push = 1e-3), constraint multipliers as
     * given (CasADi's lam_g0 defaults to 0).  dual_in: optional multipliers in the dual_out layout. */
    int warm_start;
    const double *dual_in;
    /* 1: factor the KKT by the Riccati recursion the device solver runs (csrc/gipm.hip: stage blocks
     * [[Q_uu, D_u^T], [D_u, -dc]], Sylvester inertia per stage) instead of the block-tridiagonal
     * Bunch-Kaufman factorisation; the same Newton direction up to round-off (the CPU baseline);
     * 2: the same in the restoration phase too (elastic dynamics rows through the relaxed recursion of
     * ric_relax; 1 falls back to the block-tridiagonal factorisation there); 3: test mode, both factorisations
     * in the restoration phase compared step by step (mfg_ric_check_max) */
    int riccati;
    /* 1: IPOPT's own globalisation instead of the l1-merit search (IpFilterLSAcceptor.cpp and
     * IpBacktrackingLineSearch.cpp at their defaults): the (theta, phi) filter with the switching
     * condition, Armijo on the barrier objective for f-type steps, second-order corrections, the filter
     * reset on every barrier update, the watchdog (10 shortened iterations -> 3 full trial steps), IPOPT's
     * inertia-correction sequence (IpPDPerturbationHandler.cpp: delta_w = 0 first, 1e-4 / last/3, x100 /
     * x8), the linear damping kappa_d = 1e-5 of single-bounded variables and mu_min = tol / 11.  Where
     * IPOPT would enter its restoration phase the iteration takes the shortest trial step instead
     * (counted in mfg_result.n_ls_fail). */
    int filter;
    /* 1: delta_c = 1e-8 mu^(1/4) on every constraint row, the dynamics rows included, from the first
     * factorisation: IPOPT after it has declared the Jacobian degenerate (the reference transcriptions
     * keep rows that depend only on the fixed x_0, which makes MUMPS report the KKT singular at every
     * iteration).  Block-tridiagonal factorisation only. */
    int dc_all;
    /* 1: the restoration problem keeps the dynamics rows exact (elastic p, n only on the slack and
     * equality rows): the variant the device solver's stage-wise Riccati factorisation runs */
    int resto_hard_dyn;
    /* 1: no solve -- the KKT measures of the given primal-dual point (tests: the oracle's own check of a device
     * solution).  x, u from w0 exactly (no bound push), slacks from s_in (N x ni), multipliers from dual_in
     * exactly (dual_out layout); kkt_out = [E_0 (mu = 0), dual inf., primal inf., complementarity, s_d, s_c,
     * objective]; the problem as solved (bound_relax applies) */
    int kkt_at;
    const double *s_in;
    double *kkt_out;
    double *s_out;  /* diagnostics: the slack rows at the end (N x ni) or NULL */
} mfg_opts;

typedef struct {
    int status, iter;
    double kkt, cviol, obj, mu;
    int n_ls_fail, n_inertia_fix;
} mfg_result;

typedef struct {
    mfo_model M[2];
    mfo_frame F[2];
} models_t;

static int hasb(double b) { return isfinite(b); }
#define KAPPA_D 1e-5  /* IPOPT kappa_d: linear damping of variables with one finite bound (filter mode) */

/* ------------------------------------------------------------------ node functions */
static void chain_tau(const mfo_model *M, const mfo_frame *Fr, const hd *q, const hd *qd, const hd *Fw, int with_force,
                      hd *tau, hd *pf) {
    kin_t Kn;
    hd zero[MJ], R[9];
    kinematics(M, q, &Kn);
    for (int i = 0; i < M->n; i++) zero[i] = K(0);
    rnea(M, &Kn, qd, zero, tau);
    frame_pose(&Kn, Fr, pf, R);
    if (with_force) sub_external(M, &Kn, Fr, pf, Fw, tau);
}

/* l, c_in (ni), c_eq (ne), f (nx) at the node variables xu = [x | u] */
static void node_hd(const mfg_ocp *P, const models_t *MM, const hd *xu, hd *l, hd *ci, hd *ce, hd *f) {
    const int nx = P->nx;
    const hd *u = xu + nx;
    if (P->family == MFG_CHAIN) {
        const int n = MM->M[0].n, nf = P->nf;
        const hd *q = xu, *qd = u, *F = u + n;
        hd tau[MJ], pf[3], Fw[3] = {K(0), K(0), K(0)};
        for (int a = 0; a < nf; a++)
            for (int r = 0; r < 3; r++) Fw[r] = add(Fw[r], muls(F[a], P->fdir[3 * a + r]));
        chain_tau(&MM->M[0], &MM->F[0], q, qd, Fw, nf > 0, tau, pf);
        hd c = K(0);
        for (int a = 0; a < nf; a++) c = add(c, muls(mul(F[a], F[a]), P->wF));
        for (int j = 0; j < n; j++) {
            c = add(c, muls(mul(qd[j], qd[j]), P->wqd));
            c = add(c, muls(mul(tau[j], tau[j]), P->wtau));
            ci[j] = tau[j];
            f[j] = add(q[j], muls(qd[j], P->h));
        }
        if (P->use_line)
            for (int i = 0; i < 2; i++) ce[i] = sub(pf[i], K(P->line_ref[i]));
        if (P->thermal) {
            const hd *T = xu + n;
            for (int j = 0; j < n; j++) {
                hd ia = muls(tau[j], 1.0 / P->ktau[j]);
                hd pl = add(muls(mul(ia, ia), P->Ra), muls(mul(qd[j], qd[j]), 1.0 / P->Rh));
                f[n + j] = add(muls(T[j], P->th_a), muls(pl, P->th_b));
                if (P->wT != 0.0) c = add(c, muls(mul(T[j], T[j]), P->wT));
            }
        }
        *l = c;
        return;
    }
    if (P->family == MFG_CENT) {
        /* x = [q1(7) q2(7) T(14)], u = [qd(14) FL(3) FR(3)]  (RepeatedMPCwithThermal.py:183-402) */
        const int na = MM->M[0].n, n2 = 2 * na;
        const hd *T = xu + n2, *FL = u + n2, *FR = u + n2 + 3;
        hd tau[2 * MJ], pL[3], pR[3], RL[9], RR[9], mF[3];
        kin_t Kn;
        hd zero[MJ];
        for (int i = 0; i < na; i++) zero[i] = K(0);
        /* tau_arm = ID(q, qd, 0) + J^T [F; 0]  (L341-345: the '+' sign; sub_external subtracts J^T Fw) */
        for (int r = 0; r < 3; r++) mF[r] = muls(FL[r], -1.0);
        kinematics(&MM->M[0], xu, &Kn);
        rnea(&MM->M[0], &Kn, u, zero, tau);
        frame_pose(&Kn, &MM->F[0], pL, RL);
        sub_external(&MM->M[0], &Kn, &MM->F[0], pL, mF, tau);
        for (int r = 0; r < 3; r++) mF[r] = muls(FR[r], -1.0);
        kinematics(&MM->M[1], xu + na, &Kn);
        rnea(&MM->M[1], &Kn, u + na, zero, tau + na);
        frame_pose(&Kn, &MM->F[1], pR, RR);
        sub_external(&MM->M[1], &Kn, &MM->F[1], pR, mF, tau + na);
        for (int j = 0; j < n2; j++) ci[j] = tau[j];
        /* state rows: relative position R_L^T (p_R - p_L) (L263-272) and orientation error of
         * R_L R_R^T (L274-292, appended twice in the reference; once here) minus the targets */
        hd d[3];
        for (int r = 0; r < 3; r++) d[r] = sub(pR[r], pL[r]);
        for (int b = 0; b < 3; b++)
            ce[b] = sub(add(add(mul(RL[b], d[0]), mul(RL[3 + b], d[1])), mul(RL[6 + b], d[2])), K(P->relpos0[b]));
        hd Ro[9];
        for (int m = 0; m < 3; m++)
            for (int nn = 0; nn < 3; nn++)
                Ro[3 * m + nn] = add(add(mul(RL[3 * m], RR[3 * nn]), mul(RL[3 * m + 1], RR[3 * nn + 1])),
                                     mul(RL[3 * m + 2], RR[3 * nn + 2]));
        ce[3] = sub(muls(sub(Ro[7], Ro[5]), 0.5), K(P->orient0[0]));  /* ex = skew[2,1] */
        ce[4] = sub(muls(sub(Ro[6], Ro[2]), 0.5), K(P->orient0[1]));  /* ey = skew[2,0] */
        ce[5] = sub(muls(sub(Ro[3], Ro[1]), 0.5), K(P->orient0[2]));  /* ez = skew[1,0] */
        /* mixed rows: force and moment equilibrium (L238-253) */
        const int ne = P->ne;
        ce[ne] = sub(add(FL[2], FR[2]), K(P->box_mg));
        ce[ne + 1] = add(FL[0], FR[0]);
        ce[ne + 2] = add(FL[1], FR[1]);
        hd dd[3], dF[3], mom[3];
        for (int r = 0; r < 3; r++) { dd[r] = sub(pL[r], pR[r]); dF[r] = sub(FL[r], FR[r]); }
        cross3(mom, dd, dF);
        for (int r = 0; r < 3; r++) ce[ne + 3 + r] = mom[r];
        /* cost (L353-356): 100 |p_box - B|^2 + 100 qd^T qd + 10 |F_L|^2 + 10 |F_R|^2 (the thermal term of
         * L357-359 is a constant: it reads the numeric T_0) */
        hd c = K(0);
        for (int r = 0; r < 3; r++) {
            hd e = sub(muls(add(pL[r], pR[r]), 0.5), K(P->box_pdes[r]));
            c = add(c, muls(mul(e, e), P->w_box));
            c = add(c, muls(add(mul(FL[r], FL[r]), mul(FR[r], FR[r])), P->wF));
        }
        for (int j = 0; j < n2; j++) {
            c = add(c, muls(mul(u[j], u[j]), P->w_qd));
            f[j] = add(xu[j], muls(u[j], P->h));
            hd ia = muls(tau[j], 1.0 / P->ktau[j]);
            hd pl = add(muls(mul(ia, ia), P->Ra), muls(mul(u[j], u[j]), 1.0 / P->Rh));
            f[n2 + j] = add(muls(T[j], P->th_a), muls(pl, P->th_b));
            if (P->wT != 0.0) c = add(c, muls(mul(T[j], T[j]), P->wT));
        }
        *l = c;
        return;
    }
    /* MFG_BOX: x = [qL(6) qR(6)], u = [qdL(6) qdR(6) FL(3) FR(3)] */
    const int na = MM->M[0].n;
    const hd *qL = xu, *qR = xu + na, *qdL = u, *qdR = u + na, *FL = u + 2 * na, *FR = u + 2 * na + 3;
    hd tL[MJ], tR[MJ], E1[3], E2[3];
    chain_tau(&MM->M[0], &MM->F[0], qL, qdL, FL, 1, tL, E1);
    chain_tau(&MM->M[1], &MM->F[1], qR, qdR, FR, 1, tR, E2);
    hd d[3], dF[3], mom[3];
    for (int r = 0; r < 3; r++) { d[r] = sub(E1[r], E2[r]); dF[r] = sub(FL[r], FR[r]); }
    cross3(mom, d, dF);   /* cross(E1-E2, F_L) + cross(E2-E1, F_R)  (Box_Pilz_6DOF.py:274) */
    ci[0] = sub(add(FL[2], FR[2]), K(P->box_mg));   /* Box_Pilz_6DOF.py:269 */
    ci[1] = add(FL[0], FR[0]);
    ci[2] = add(FL[1], FR[1]);
    for (int r = 0; r < 3; r++) ci[3 + r] = mom[r];
    for (int j = 0; j < na; j++) { ci[6 + j] = tL[j]; ci[6 + na + j] = tR[j]; }
    ce[0] = sub(dot3(d, d), K(P->box_L));          /* Box_Pilz_6DOF.py:280 */
    hd c = K(0);
    for (int r = 0; r < 3; r++) {                   /* 100 |p_box - p_des|^2 + qd^T qd (L415-416) */
        hd e = sub(muls(add(E1[r], E2[r]), 0.5), K(P->box_pdes[r]));
        c = add(c, muls(mul(e, e), P->w_box));
    }
    for (int j = 0; j < 2 * na; j++) {
        c = add(c, muls(mul(u[j], u[j]), P->w_qd));
        f[j] = add(xu[j], muls(u[j], P->h));
    }
    if (P->thermal) {
        /* shared fatigue budget (build-defined extension of C3): the winding temperature of
         * each of the 12 joints as state (Tmodel_library.py:9-41 with that joint's arm torque) and one slack
         * row sum_j T_j <= budget */
        const hd *T = xu + 2 * na;
        hd sum = K(0);
        for (int j = 0; j < 2 * na; j++) {
            hd t = j < na ? tL[j] : tR[j - na];
            hd ia = muls(t, 1.0 / P->ktau[j]);
            hd pl = add(muls(mul(ia, ia), P->Ra), muls(mul(u[j], u[j]), 1.0 / P->Rh));
            f[2 * na + j] = add(muls(T[j], P->th_a), muls(pl, P->th_b));
            if (P->wT != 0.0) c = add(c, muls(mul(T[j], T[j]), P->wT));
            sum = add(sum, T[j]);
        }
        ci[6 + 2 * na] = sum;
    }
    *l = c;
}

/* ------------------------------------------------------------------ workspace */
typedef struct {
    const mfg_ocp *P;
    const mfg_opts *O;
    const models_t *MM;
    int N, nx, nu, nv, ni, ne, mb;
    int nes;                         /* the first nes of the ne equality rows are state rows */
    /* per-variable masks (after relaxation) */
    double *ulo, *uhi, *clo, *chi;   /* N x nu, N x ni */
    double xlo[GX], xhi[GX];
    unsigned char *ufix;             /* N x nu */
    /* iterate */
    double *x, *u, *s, *lam, *ye, *yi;
    double *zxL, *zxU, *zuL, *zuU, *vL, *vU;
    /* trial */
    double *tx, *tu, *ts;
    /* eval cache (per node) */
    double *l, *gl, *ci, *Ji, *ce, *Je, *f, *Af, *Bf, *W;
    /* step */
    double *dx, *du, *ds, *dlam, *dye, *dyi, *dzxL, *dzxU, *dzuL, *dzuU, *dvL, *dvU;
    /* barrier */
    double *Sx, *gx, *Su, *gu, *Ss, *gs;
    /* kkt */
    double *wv, *G, *Dsave;
    int *perm, *piv;
    double dw, dc, d1;               /* regularisation of the current factorisation */
    /* constraint residuals: current point, trial point, second-order correction */
    double *rdyn, *rin, *req, *trdyn, *trin, *treq, *sdyn, *sin_, *seq;
    double *bk;                      /* saved direction (second-order corrections) */
    /* Riccati factorisation (mfg_opts.riccati): P_{k+1} per stage, stage block factors, gains, and the
     * vector pass's p_{k+1} / k_k */
    int ric, nk;
    double *Pg, *Kst, *Fg, *pvg, *kvg;
    int *Kpp;
    /* relaxed dynamics rows (restoration with elastic dynamics, or dc_all): their diagonal D_r per stage and
     * the state-equality rows of node k+1 seen through the relaxed dynamics, J~ = J_e,k+1 (I + D_r P)^-1 */
    double *Drg, *Jtg, *LUg;
    int *LUp;
    /* IPOPT's restoration phase (filter mode, IpRestoIpoptNLP.cpp): the same variables plus elastic
     * p, n >= 0 on every constraint row, row r in the order [dynamics (N nx) | slack rows (N ni) |
     * equality rows (N ne)], objective rho sum(p + n) + zeta/2 |D_R (w - w_R)|^2, zeta = sqrt(mu).
     * p and n are condensed out of the KKT: row r gains the diagonal 1/Sp + 1/Sn and its residual the
     * term rowr = r_p / Sp - r_n / Sn (the p / n stationarity residuals). */
    int resto, NR;
    double objw;                     /* weight of the original objective in node evaluations (0 in resto) */
    double zeta, rho_r;
    double *wR, *dR;                 /* reference point and D_R^2 over [x ((N+1) nx) | u (N nu)] */
    double *pr, *nr, *zp, *zn, *dpr, *dnr, *dzp, *dzn, *tpr, *tnr, *Sp, *Sn, *gp, *gn, *rowr;
} ws_t;

/* row r of the restoration layout: active, its multiplier */
static int row_on(const ws_t *S, int r);
static double *row_y(ws_t *S, int r);

/* per-problem data handed to the node callbacks: the line reference, or the Centauro pose targets
 * (relpos0 and orient0 are adjacent: 6 values) */
#define AUX(P) ((P)->family == MFG_CENT ? (P)->relpos0 : (P)->line_ref)
static double *dal(size_t n) { return (double *)calloc(n ? n : 1, sizeof(double)); }

/* equality row e of node k active: state rows for eq_from <= k < N, mixed rows for k < N */
#define EQ_ON(S, k, e) ((k) < (S)->N && ((e) >= (S)->nes || (k) >= (S)->P->eq_from))
#define CACT(S, k, r) (hasb((S)->clo[(k) * (S)->ni + (r)]) || hasb((S)->chi[(k) * (S)->ni + (r)]))
/* free variable a (0..nv) of node k */
static int vfree(const ws_t *S, int k, int a) {
    if (a < S->nx) return k > 0;
    return !S->ufix[k * S->nu + a - S->nx];
}
static int row_on(const ws_t *S, int r) {
    const int nd = S->N * S->nx, nI = S->N * S->ni;
    if (r < nd) return 1;
    if (r < nd + nI) { r -= nd; return CACT(S, r / S->ni, r % S->ni); }
    r -= nd + nI;
    return EQ_ON(S, r / S->ne, r % S->ne);
}
static double *row_y(ws_t *S, int r) {
    const int nd = S->N * S->nx, nI = S->N * S->ni;
    if (r < nd) return S->lam + r;
    if (r < nd + nI) return S->yi + (r - nd);
    return S->ye + (r - nd - nI);
}
/* row r carries elastic variables in the restoration problem */
static int row_el(const ws_t *S, int r) {
    if (S->O->resto_hard_dyn && r < S->N * S->nx) return 0;
    return row_on(S, r);
}
/* resto: extra row diagonal and residual correction of row r (0 outside the restoration phase; Sp = Sn =
 * inf on rows without elastic variables) */
#define RDIAG(S, r) ((S)->resto ? 1.0 / (S)->Sp[r] + 1.0 / (S)->Sn[r] : 0.0)
#define RCORR(S, r) ((S)->resto ? (S)->rowr[r] : 0.0)

static void eval_values(const ws_t *S, int k, const double *x, const double *u, double *l, double *ci, double *ce,
                        double *f) {
    if (S->O && S->O->val_cb) {
        S->O->val_cb(S->O->node_ctx, x, u, AUX(S->P), l, ci, ce, f);
        return;
    }
    hd xu[GV], hl, hci[GI], hce[GE], hf[GX];
    for (int a = 0; a < S->nx; a++) xu[a] = K(x[a]);
    for (int a = 0; a < S->nu; a++) xu[S->nx + a] = K(u[a]);
    node_hd(S->P, S->MM, xu, &hl, hci, hce, hf);
    *l = hl.a;
    for (int r = 0; r < S->ni; r++) ci[r] = hci[r].a;
    for (int e = 0; e < S->ne; e++) ce[e] = hce[e].a;
    for (int j = 0; j < S->nx; j++) f[j] = hf[j].a;
}

static void eval_derivs(ws_t *S, int k) {
    const int nx = S->nx, nu = S->nu, nv = S->nv, ni = S->ni, ne = S->ne;
    const double *x = S->x + k * nx, *u = S->u + k * nu;
    double *gl = S->gl + k * nv, *Ji = S->Ji + (size_t)k * ni * nv, *Je = S->Je + (size_t)k * ne * nv;
    double *Af = S->Af + k * nx * nx, *Bf = S->Bf + k * nx * nu, *W = S->W + (size_t)k * nv * nv;
    const double *lam = S->lam + k * nx, *yi = S->yi + k * ni, *ye = S->ye + k * ne;
    const int eqon = EQ_ON(S, k, 0), nes = S->nes, nem = ne - nes;
    if (S->O && S->O->node_cb) {
        /* record: ... | c_eq (nes) | d c_eq/dx (nes x nx) | c_m (nem) | d c_m (nem x nv) | f | A | B | W */
        const int oGL = 1, oCI = oGL + nv, oJI = oCI + ni, oCE = oJI + ni * nv, oJE = oCE + nes, oCM = oJE + nes * nx,
                  oJM = oCM + nem, oF = oJM + nem * nv, oA = oF + nx, oB = oA + nx * nx, oW = oB + nx * nu,
                  REC = oW + nv * nv;
        double xu[GV], rec[2 * GV * GV + GV * GI + GX * GX + 512];
        memcpy(xu, x, nx * sizeof(double));
        memcpy(xu + nx, u, nu * sizeof(double));
        S->O->node_cb(S->O->node_ctx, xu, yi, ye, lam, AUX(S->P), eqon, rec);
        (void)REC;
        if (S->objw != 1.0) {  /* restoration: W without (1 - objw) of the objective's Hessian */
            double rec0[2 * GV * GV + GV * GI + GX * GX + 512], z[GI + GE + GX];
            memset(z, 0, sizeof z);
            S->O->node_cb(S->O->node_ctx, xu, z, z, z, AUX(S->P), eqon, rec0);
            for (int i = 0; i < nv * nv; i++) rec[oW + i] -= (1.0 - S->objw) * rec0[oW + i];
            for (int a = 0; a < nv; a++) rec[oGL + a] *= S->objw;
        }
        S->l[k] = rec[0];
        memcpy(gl, rec + oGL, nv * sizeof(double));
        memcpy(S->ci + k * ni, rec + oCI, ni * sizeof(double));
        memcpy(Ji, rec + oJI, (size_t)ni * nv * sizeof(double));
        memcpy(S->ce + k * ne, rec + oCE, nes * sizeof(double));
        memcpy(S->ce + k * ne + nes, rec + oCM, nem * sizeof(double));
        memset(Je, 0, (size_t)ne * nv * sizeof(double));
        for (int e = 0; e < nes; e++) memcpy(Je + e * nv, rec + oJE + e * nx, nx * sizeof(double));
        memcpy(Je + nes * nv, rec + oJM, (size_t)nem * nv * sizeof(double));
        memcpy(S->f + k * nx, rec + oF, nx * sizeof(double));
        memcpy(Af, rec + oA, (size_t)nx * nx * sizeof(double));
        memcpy(Bf, rec + oB, (size_t)nx * nu * sizeof(double));
        memcpy(W, rec + oW, (size_t)nv * nv * sizeof(double));
        /* fixed variables carry no derivatives (their rows are identities in the KKT) */
        for (int a = 0; a < nv; a++)
            if (!vfree(S, k, a)) {
                gl[a] = 0;
                for (int r = 0; r < ni; r++) Ji[r * nv + a] = 0;
                for (int e = 0; e < ne; e++) Je[e * nv + a] = 0;
                if (a < nx) { for (int j = 0; j < nx; j++) Af[j * nx + a] = 0; }
                else for (int j = 0; j < nx; j++) Bf[j * nu + a - nx] = 0;
                for (int b = 0; b < nv; b++) W[a * nv + b] = W[b * nv + a] = 0;
            }
        return;
    }
    eval_values(S, k, x, u, S->l + k, S->ci + k * ni, S->ce + k * ne, S->f + k * nx);
    memset(gl, 0, sizeof(double) * nv);
    memset(Ji, 0, sizeof(double) * ni * nv);
    memset(Je, 0, sizeof(double) * ne * nv);
    memset(Af, 0, sizeof(double) * nx * nx);
    memset(Bf, 0, sizeof(double) * nx * nu);
    memset(W, 0, sizeof(double) * nv * nv);
    int fv[GV], nfv = 0;
    for (int a = 0; a < nv; a++)
        if (vfree(S, k, a)) fv[nfv++] = a;
    double xu[GV];
    memcpy(xu, x, nx * sizeof(double));
    memcpy(xu + nx, u, nu * sizeof(double));
    for (int ia = 0; ia < nfv; ia++)
        for (int ib = ia; ib < nfv; ib++) {
            const int a = fv[ia], b = fv[ib];
            hd hx[GV], hl, hci[GI], hce[GE], hf[GX];
            for (int i = 0; i < nv; i++) hx[i] = K(xu[i]);
            hx[a].b = 1.0;
            hx[b].c = 1.0;
            node_hd(S->P, S->MM, hx, &hl, hci, hce, hf);
            double h2 = S->objw * hl.d;
            for (int r = 0; r < ni; r++) h2 += yi[r] * hci[r].d;
            for (int e = 0; e < ne; e++)
                if (EQ_ON(S, k, e)) h2 += ye[e] * hce[e].d;
            for (int j = 0; j < nx; j++) h2 += lam[j] * hf[j].d;
            W[a * nv + b] = W[b * nv + a] = h2;
            if (a == b) {
                gl[a] = S->objw * hl.b;
                for (int r = 0; r < ni; r++) Ji[r * nv + a] = hci[r].b;
                for (int e = 0; e < ne; e++) Je[e * nv + a] = hce[e].b;
                if (a < nx) {
                    for (int j = 0; j < nx; j++) Af[j * nx + a] = hf[j].b;
                } else {
                    for (int j = 0; j < nx; j++) Bf[j * nu + a - nx] = hf[j].b;
                }
            }
        }
}

/* IPOPT bound_push / bound_frac (1e-2 cold; warm_start_bound_push / _frac = 1e-3 warm) */
static double push_into_k(double x, double lo, double hi, double k1, double k2) {
    int hl = hasb(lo), hh = hasb(hi);
    if (hl && hh) {
        double pl = fmin(k1 * fmax(1.0, fabs(lo)), k2 * (hi - lo));
        double pu = fmin(k1 * fmax(1.0, fabs(hi)), k2 * (hi - lo));
        x = fmax(x, lo + pl);
        x = fmin(x, hi - pu);
    } else if (hl) {
        x = fmax(x, lo + k1 * fmax(1.0, fabs(lo)));
    } else if (hh) {
        x = fmin(x, hi - k1 * fmax(1.0, fabs(hi)));
    }
    return x;
}
static double push_into(double x, double lo, double hi) { return push_into_k(x, lo, hi, 1e-2, 1e-2); }

/* barrier objective and l1 constraint violation at (x, u, s); optionally the residual vectors.
 * pp, nn: the restoration problem's elastic variables at this point (NULL: the original problem). */
#define merit_parts(S, x, u, s, mu, phi, theta, ok, rdyn, rin, req) \
    merit_parts_e(S, x, u, s, NULL, NULL, mu, phi, theta, ok, rdyn, rin, req)
static void merit_parts_e(const ws_t *S, const double *x, const double *u, const double *s, const double *pp,
                          const double *nn, double mu, double *phi, double *theta, int *ok, double *rdyn, double *rin,
                          double *req) {
    const int N = S->N, nx = S->nx, nu = S->nu, ni = S->ni, ne = S->ne;
    const int oI = N * nx, oE = N * nx + N * ni;
    double fsum = 0, bar = 0, th = 0;
    int good = 1;
#define EL(r) (pp ? nn[r] - pp[r] : 0.0)
#ifdef _OPENMP
#pragma omp parallel for reduction(+ : fsum, th) schedule(static)
#endif
    for (int k = 0; k < N; k++) {
        double l, ci[GI], ce[GE], f[GX];
        eval_values(S, k, x + k * nx, u + k * nu, &l, ci, ce, f);
        if (!pp) fsum += l;
        for (int j = 0; j < nx; j++) {
            const double r = f[j] - x[(k + 1) * nx + j] + EL(k * nx + j);
            th += fabs(r);
            if (rdyn) rdyn[k * nx + j] = r;
        }
        for (int q = 0; q < ni; q++) {
            const double r = CACT(S, k, q) ? ci[q] - s[k * ni + q] + EL(oI + k * ni + q) : 0.0;
            th += fabs(r);
            if (rin) rin[k * ni + q] = r;
        }
        for (int e = 0; e < ne; e++) {
            const double r = EQ_ON(S, k, e) ? ce[e] + EL(oE + k * ne + e) : 0.0;
            th += fabs(r);
            if (req) req[k * ne + e] = r;
        }
    }
#undef EL
    if (pp) {  /* restoration objective: rho sum(p + n) + zeta/2 |D_R (w - w_R)|^2, barrier on p, n */
        double pn = 0, prox = 0, lbar = 0;
        for (int r = 0; r < S->NR; r++)
            if (row_el(S, r)) {
                pn += pp[r] + nn[r];
                if (pp[r] <= 0 || nn[r] <= 0) good = 0;
                else lbar -= log(pp[r]) + log(nn[r]);
            }
        for (int k = 1; k <= N; k++)
            for (int j = 0; j < nx; j++) {
                const int i = k * nx + j;
                prox += S->dR[i] * (x[i] - S->wR[i]) * (x[i] - S->wR[i]);
            }
        for (int i = 0; i < N * nu; i++)
            if (!S->ufix[i]) {
                const int o = (N + 1) * nx + i;
                prox += S->dR[o] * (u[i] - S->wR[o]) * (u[i] - S->wR[o]);
            }
        fsum = S->rho_r * pn + 0.5 * S->zeta * prox + mu * lbar + KAPPA_D * mu * pn;
    }
    double lin = 0;  /* IPOPT kappa_d damping of single-bounded variables (filter mode) */
#define BAR(v, lo, hi)                                              \
    do {                                                            \
        if (hasb(lo)) { if ((v) - (lo) <= 0) good = 0; else bar -= log((v) - (lo)); } \
        if (hasb(hi)) { if ((hi) - (v) <= 0) good = 0; else bar -= log((hi) - (v)); } \
        if (hasb(lo) && !hasb(hi)) lin += (v) - (lo);               \
        if (hasb(hi) && !hasb(lo)) lin += (hi) - (v);               \
    } while (0)
    for (int k = 1; k <= N; k++)
        for (int j = 0; j < nx; j++) BAR(x[k * nx + j], S->xlo[j], S->xhi[j]);
    for (int k = 0; k < N; k++)
        for (int j = 0; j < nu; j++)
            if (!S->ufix[k * nu + j]) BAR(u[k * nu + j], S->ulo[k * nu + j], S->uhi[k * nu + j]);
    for (int k = 0; k < N; k++)
        for (int r = 0; r < ni; r++) BAR(s[k * ni + r], S->clo[k * ni + r], S->chi[k * ni + r]);
#undef BAR
    *phi = fsum + mu * bar + (S->O->filter ? KAPPA_D * mu * lin : 0.0);
    *theta = th;
    *ok = good;
}

static void residuals_cached(const ws_t *S, double *rdyn, double *rin, double *req) {
    const int N = S->N, nx = S->nx, ni = S->ni, ne = S->ne;
    for (int k = 0; k < N; k++) {
        for (int j = 0; j < nx; j++) rdyn[k * nx + j] = S->f[k * nx + j] - S->x[(k + 1) * nx + j];
        for (int q = 0; q < ni; q++) rin[k * ni + q] = CACT(S, k, q) ? S->ci[k * ni + q] - S->s[k * ni + q] : 0.0;
        for (int e = 0; e < ne; e++) req[k * ne + e] = EQ_ON(S, k, e) ? S->ce[k * ne + e] : 0.0;
    }
    if (S->resto) {  /* the restoration rows g - p + n */
        const int oI = N * nx, oE = N * nx + N * ni;
        for (int r = 0; r < S->NR; r++) {
            if (!row_el(S, r)) continue;
            const double el = S->nr[r] - S->pr[r];
            if (r < oI) rdyn[r] += el;
            else if (r < oE) rin[r - oI] += el;
            else req[r - oE] += el;
        }
    }
}

/* Block-tridiagonal KKT over shooting nodes, block k < N: [lam_{k-1} (nx) | x_k (nx) | u_k (nu) | ye_k (ne)],
 * block N: [lam_{N-1} | x_N].  lam_k's row lives in block k+1 and couples to block k through
 * C_k = [0 | A_k | B_k | 0].  Slack rows are condensed: D_s = (Sigma_s + dw) / (1 + dc (Sigma_s + dw)).
 * Factorises block by block (Bunch-Kaufman, D_{k+1}[lam,lam] -= C_k D_k^-1 C_k^T) and stores the factors.
 * Returns 0 if the inertia is (n_primal, n_dual, 0), 1 if it is wrong, 2 on a zero pivot.          */
static int kkt_factor(ws_t *S, double dw, double dc, double d1) {
    const mfg_ocp *P = S->P;
    const int N = S->N, nx = S->nx, nu = S->nu, nv = S->nv, ni = S->ni, ne = S->ne, mb = S->mb;
    const int ol = 0, ox = nx, ou = 2 * nx, oe = 2 * nx + nu;
    int npos_t = 0, nneg_t = 0, nzero_t = 0;
    S->dw = dw; S->dc = dc; S->d1 = d1;
    for (int k = 0; k <= N; k++) {
        const int m = (k < N) ? mb : 2 * nx;
        double *Dm = S->Dsave + (size_t)k * mb * mb;
        memset(Dm, 0, sizeof(double) * mb * mb);
#define D_(i, j) Dm[(i) * m + (j)]
        for (int j = 0; j < nx; j++) {
            if (k > 0) {  /* dynamics rows stay unregularised unless dc_all (delta_c acts on c_eq and slack rows) */
                D_(ol + j, ox + j) = D_(ox + j, ol + j) = -1.0;
                if (S->O->dc_all || S->resto) D_(ol + j, ol + j) = -(S->O->dc_all ? dc : 0.0) - RDIAG(S, (k - 1) * nx + j);
            } else {
                D_(ol + j, ol + j) = -1.0; /* lam_{-1}: dummy */
            }
        }
        if (k < N) {
            const double *W = S->W + (size_t)k * nv * nv, *Ji = S->Ji + (size_t)k * ni * nv;
            const double *Je = S->Je + (size_t)k * ne * nv;
            double Dd[GI];
            for (int q = 0; q < ni; q++) {
                const double sg = S->Ss[k * ni + q] + dw;
                Dd[q] = CACT(S, k, q) ? sg / (1.0 + (dc + RDIAG(S, N * nx + k * ni + q)) * sg) : 0.0;
            }
            for (int a = 0; a < nv; a++)
                for (int b = 0; b < nv; b++) {
                    double v = W[a * nv + b];
                    for (int q = 0; q < ni; q++) v += Ji[q * nv + a] * Dd[q] * Ji[q * nv + b];
                    D_(ox + a, ox + b) = v;
                }
            for (int a = 0; a < nv; a++) {
                double dd = dw;
                if (a < nx) dd += S->Sx[k * nx + a];
                else {
                    dd += S->Su[k * nu + a - nx];
                    if (a - nx >= P->tier1_from && a - nx < P->tier1_to) dd += d1;
                }
                D_(ox + a, ox + a) += dd;
            }
            for (int e = 0; e < ne; e++) {
                if (EQ_ON(S, k, e)) {
                    for (int j = 0; j < nv; j++) D_(oe + e, ox + j) = D_(ox + j, oe + e) = Je[e * nv + j];
                    D_(oe + e, oe + e) = -dc - RDIAG(S, N * nx + N * ni + k * ne + e);
                } else {
                    D_(oe + e, oe + e) = -1.0;
                }
            }
            for (int a = 0; a < nv; a++)
                if (!vfree(S, k, a)) {
                    for (int v = 0; v < m; v++) { D_(ox + a, v) = 0; D_(v, ox + a) = 0; }
                    D_(ox + a, ox + a) = 1.0;
                }
        } else {
            for (int j = 0; j < nx; j++) D_(ox + j, ox + j) = S->Sx[N * nx + j] + dw;
        }
        if (k > 0) {
            const double *Gp = S->G + (size_t)(k - 1) * mb * nx;
            const double *A = S->Af + (k - 1) * nx * nx, *B = S->Bf + (k - 1) * nx * nu;
            for (int c = 0; c < nx; c++)
                for (int c2 = 0; c2 < nx; c2++) {
                    double a = 0;
                    for (int j = 0; j < nx; j++)
                        if (vfree(S, k - 1, j)) a += A[c * nx + j] * Gp[(ox + j) * nx + c2];
                    for (int j = 0; j < nu; j++)
                        if (vfree(S, k - 1, nx + j)) a += B[c * nu + j] * Gp[(ou + j) * nx + c2];
                    D_(ol + c, ol + c2) -= a;
                }
        }
#undef D_
        int np, nn, nz;
        bk_factor(Dm, m, S->perm + k * mb, S->piv + k * mb, &np, &nn, &nz);
        npos_t += np; nneg_t += nn; nzero_t += nz;
        if (nz) return 2;
        if (k < N) {
            const double *A = S->Af + k * nx * nx, *B = S->Bf + k * nx * nu;
            double *Gk = S->G + (size_t)k * mb * nx;
            for (int c = 0; c < nx; c++) {
                double e[BKMAX];
                memset(e, 0, sizeof e);
                for (int j = 0; j < nx; j++)
                    if (vfree(S, k, j)) e[ox + j] = A[c * nx + j];
                for (int j = 0; j < nu; j++)
                    if (vfree(S, k, nx + j)) e[ou + j] = B[c * nu + j];
                bk_solve(Dm, m, S->perm + k * mb, S->piv + k * mb, e);
                for (int i = 0; i < m; i++) Gk[i * nx + c] = e[i];
            }
        }
    }
    const int want_pos = N * nv + nx, want_neg = (N + 1) * nx + N * ne;
    return (npos_t == want_pos && nneg_t == want_neg) ? 0 : 1;
}

/* the slack-row steps (dyi, ds) and the bound-multiplier steps of a primal-dual direction */
static void slack_and_bound_steps(ws_t *S, double mu, const double *rin) {
    const int N = S->N, nx = S->nx, nu = S->nu, nv = S->nv, ni = S->ni;
    const double dw = S->dw, dc = S->dc;
    for (int k = 0; k < N; k++) {
        const double *Ji = S->Ji + (size_t)k * ni * nv;
        for (int q = 0; q < ni; q++) {
            const int i = k * ni + q;
            if (!CACT(S, k, q)) { S->dyi[i] = 0; S->ds[i] = 0; continue; }
            double jd = 0;
            for (int a = 0; a < nx; a++) jd += Ji[q * nv + a] * S->dx[k * nx + a];
            for (int a = 0; a < nu; a++) jd += Ji[q * nv + nx + a] * S->du[k * nu + a];
            const int rr = N * nx + i;
            const double sg = S->Ss[i] + dw, Dd = sg / (1.0 + (dc + RDIAG(S, rr)) * sg);
            const double rs = S->gs[i] - S->yi[i];
            S->dyi[i] = Dd * (jd + rin[i] + RCORR(S, rr) + rs / sg);
            S->ds[i] = (S->dyi[i] - rs) / sg;
        }
    }
#define DZ(dzl, dzu, zl, zu, v, dv, lo, hi)                                              \
    do {                                                                                 \
        dzl = dzu = 0;                                                                   \
        if (hasb(lo)) dzl = mu / ((v) - (lo)) - (zl) - (zl) / ((v) - (lo)) * (dv);       \
        if (hasb(hi)) dzu = mu / ((hi) - (v)) - (zu) + (zu) / ((hi) - (v)) * (dv);       \
    } while (0)
    for (int k = 0; k <= N; k++)
        for (int j = 0; j < nx; j++) {
            const int i = k * nx + j;
            if (k == 0) { S->dzxL[i] = S->dzxU[i] = 0; continue; }
            DZ(S->dzxL[i], S->dzxU[i], S->zxL[i], S->zxU[i], S->x[i], S->dx[i], S->xlo[j], S->xhi[j]);
        }
    for (int i = 0; i < N * nu; i++) {
        if (S->ufix[i]) { S->dzuL[i] = S->dzuU[i] = 0; continue; }
        DZ(S->dzuL[i], S->dzuU[i], S->zuL[i], S->zuU[i], S->u[i], S->du[i], S->ulo[i], S->uhi[i]);
    }
    for (int i = 0; i < N * ni; i++)
        DZ(S->dvL[i], S->dvU[i], S->vL[i], S->vU[i], S->s[i], S->ds[i], S->clo[i], S->chi[i]);
#undef DZ
    if (S->resto) /* the elastic variables: Sp dp = dy - r_p, Sn dn = -dy - r_n, and their bound multipliers */
        for (int r = 0; r < S->NR; r++) {
            if (!row_el(S, r)) { S->dpr[r] = S->dnr[r] = S->dzp[r] = S->dzn[r] = 0.0; continue; }
            const int nd = N * nx, nI = N * ni;
            const double dy = r < nd ? S->dlam[r] : (r < nd + nI ? S->dyi[r - nd] : S->dye[r - nd - nI]);
            const double y = *row_y(S, r);
            const double rp = S->rho_r + S->gp[r] - y, rn = S->rho_r + S->gn[r] + y;
            S->dpr[r] = (dy - rp) / S->Sp[r];
            S->dnr[r] = (-dy - rn) / S->Sn[r];
            S->dzp[r] = mu / S->pr[r] - S->zp[r] - S->zp[r] / S->pr[r] * S->dpr[r];
            S->dzn[r] = mu / S->nr[r] - S->zn[r] - S->zn[r] / S->nr[r] * S->dnr[r];
        }
}

/* Newton direction with the stored factorisation for constraint residuals (rdyn, rin, req): the
 * primal-dual step (dx, du, dlam, dye), the slack-row steps (dyi, ds) and the bound-multiplier steps. */
static void kkt_direction(ws_t *S, double mu, const double *rdyn, const double *rin, const double *req) {
    const int N = S->N, nx = S->nx, nu = S->nu, nv = S->nv, ni = S->ni, ne = S->ne, mb = S->mb;
    const int ol = 0, ox = nx, ou = 2 * nx, oe = 2 * nx + nu;
    const double dw = S->dw, dc = S->dc;
    for (int k = 0; k <= N; k++) {
        const int m = (k < N) ? mb : 2 * nx;
        double *r = S->wv + (size_t)k * mb;
        memset(r, 0, sizeof(double) * mb);
        if (k > 0)
            for (int j = 0; j < nx; j++) r[ol + j] = -(rdyn[(k - 1) * nx + j] + RCORR(S, (k - 1) * nx + j));
        if (k < N) {
            const double *Ji = S->Ji + (size_t)k * ni * nv, *Je = S->Je + (size_t)k * ne * nv;
            double Dd[GI], rdd[GI];
            for (int q = 0; q < ni; q++) {
                const int i = k * ni + q;
                if (CACT(S, k, q)) {
                    const double sg = S->Ss[i] + dw;
                    Dd[q] = sg / (1.0 + (dc + RDIAG(S, N * nx + i)) * sg);
                    rdd[q] = rin[i] + RCORR(S, N * nx + i) + (S->gs[i] - S->yi[i]) / sg;
                } else { Dd[q] = 0; rdd[q] = 0; }
            }
            for (int e = 0; e < ne; e++)
                r[oe + e] = EQ_ON(S, k, e) ? -(req[k * ne + e] + RCORR(S, N * nx + N * ni + k * ne + e)) : 0.0;
            for (int a = 0; a < nv; a++) {
                if (!vfree(S, k, a)) { r[ox + a] = 0; continue; }
                double g = S->gl[k * nv + a];
                for (int q = 0; q < ni; q++) g += Ji[q * nv + a] * (S->yi[k * ni + q] + Dd[q] * rdd[q]);
                if (a < nx) {
                    g += S->gx[k * nx + a] - (k > 0 ? S->lam[(k - 1) * nx + a] : 0.0);
                    for (int jj = 0; jj < nx; jj++) g += S->Af[(k * nx + jj) * nx + a] * S->lam[k * nx + jj];
                } else {
                    g += S->gu[k * nu + a - nx];
                    for (int jj = 0; jj < nx; jj++) g += S->Bf[(k * nx + jj) * nu + a - nx] * S->lam[k * nx + jj];
                }
                for (int e = 0; e < ne; e++)
                    if (EQ_ON(S, k, e)) g += Je[e * nv + a] * S->ye[k * ne + e];
                r[ox + a] = -g;
            }
        } else {
            for (int j = 0; j < nx; j++) r[ox + j] = -(S->gx[N * nx + j] - S->lam[(N - 1) * nx + j]);
        }
        if (k > 0) {
            const double *wp = S->wv + (size_t)(k - 1) * mb;
            const double *A = S->Af + (k - 1) * nx * nx, *B = S->Bf + (k - 1) * nx * nu;
            for (int c = 0; c < nx; c++) {
                double a = 0;
                for (int j = 0; j < nx; j++)
                    if (vfree(S, k - 1, j)) a += A[c * nx + j] * wp[ox + j];
                for (int j = 0; j < nu; j++)
                    if (vfree(S, k - 1, nx + j)) a += B[c * nu + j] * wp[ou + j];
                r[ol + c] -= a;
            }
        }
        bk_solve(S->Dsave + (size_t)k * mb * mb, m, S->perm + k * mb, S->piv + k * mb, r);
    }
    /* back substitution: y_N = w_N, y_k = w_k - G_k y_{k+1}[lam_k] */
    {
        double ynext[BKMAX], y[BKMAX];
        const double *yN = S->wv + (size_t)N * mb;
        for (int j = 0; j < nx; j++) { S->dx[N * nx + j] = yN[ox + j]; S->dlam[(N - 1) * nx + j] = yN[ol + j]; }
        memcpy(ynext, yN, sizeof(double) * 2 * nx);
        for (int k = N - 1; k >= 0; k--) {
            const double *wk = S->wv + (size_t)k * mb, *Gk = S->G + (size_t)k * mb * nx;
            for (int i = 0; i < mb; i++) {
                double a = wk[i];
                for (int c = 0; c < nx; c++) a -= Gk[i * nx + c] * ynext[ol + c];
                y[i] = a;
            }
            for (int j = 0; j < nx; j++) {
                S->dx[k * nx + j] = (k > 0) ? y[ox + j] : 0.0;
                if (k > 0) S->dlam[(k - 1) * nx + j] = y[ol + j];
            }
            for (int j = 0; j < nu; j++) S->du[k * nu + j] = S->ufix[k * nu + j] ? 0.0 : y[ou + j];
            for (int e = 0; e < ne; e++) S->dye[k * ne + e] = EQ_ON(S, k, e) ? y[oe + e] : 0.0;
            memcpy(ynext, y, sizeof(double) * mb);
        }
    }
    slack_and_bound_steps(S, mu, rin);
}


/* ---- Riccati factorisation and direction (mfg_opts.riccati; the device's csrc/gipm.hip recursion) ----
 * Stage k eliminates u_k and the equality rows attached to it -- the state rows of node k+1 through the
 * dynamics (J_e,k+1 [A_k | B_k]) and the mixed rows of stage k (J_m,k) -- with the stage block
 *   K_k = [[Q_uu, D_u^T], [D_u, -dc]],  Q_uu = H_uu + B^T P_{k+1} B,
 * and carries the value function P_k = Q_xx + R^T K_k^{-1}... (R = [Q_ux; D_x]).  The KKT matrix has the
 * inertia (n_primal, n_dual, 0) iff every K_k has inertia (nu, rows) (Sylvester). */
/* Relaxed dynamics rows (the restoration phase's elastic p, n on the dynamics rows, or dc_all): the row
 * reads dx_{k+1} = A dx_k + B du_k + r - D_r dlam_k with D_r >= 0 diagonal.  With dlam_k = P dx_{k+1} + p +
 * J_n^T dy_s (P, p the value function of node k+1, J_n its state-equality rows) the elimination of dx_{k+1}
 * leaves the hard recursion with, for L = I + P D_r (LU with partial pivoting, kept per stage),
 *   P~ = L^-1 P = P (I + D_r P)^-1,   J~^T = L^-1 J_n^T,   p~ = L^-1 p,
 *   the state-equality block -dc - J~ D_r J_n^T,   tv = p~ + P~ r,   z_s = req + J~ r - J_n D_r p~
 * in place of P, J_n, -dc, p + P r, req + J_n r.  (Solves, not the Woodbury difference P - P S G^-1 S P,
 * which cancels to a few digits once P >> 1 / D_r.)  G = I + S P S, S = D_r^(1/2), must have the inertia
 * (nx, 0, 0) for the eliminated (x_{k+1}, lam_k) pair to contribute (nx, nx, 0).  The forward pass recovers
 * dx_{k+1} = z - D_r dlam_k. */
static int lu_factor(double *M, int n, int *pv) {
    for (int c = 0; c < n; c++) {
        int pr = c;
        for (int r = c + 1; r < n; r++)
            if (fabs(M[r * n + c]) > fabs(M[pr * n + c])) pr = r;
        pv[c] = pr;
        if (M[pr * n + c] == 0.0) return 1;
        if (pr != c)
            for (int j = 0; j < n; j++) { const double t = M[c * n + j]; M[c * n + j] = M[pr * n + j]; M[pr * n + j] = t; }
        for (int r = c + 1; r < n; r++) {
            const double f = M[r * n + c] / M[c * n + c];
            M[r * n + c] = f;
            for (int j = c + 1; j < n; j++) M[r * n + j] -= f * M[c * n + j];
        }
    }
    return 0;
}
static void lu_solve(const double *M, int n, const int *pv, double *b) {
    for (int c = 0; c < n; c++)  /* the row interchanges first: they also moved the stored multipliers */
        if (pv[c] != c) { const double t = b[c]; b[c] = b[pv[c]]; b[pv[c]] = t; }
    for (int c = 0; c < n; c++)
        for (int r = c + 1; r < n; r++) b[r] -= M[r * n + c] * b[c];
    for (int c = n - 1; c >= 0; c--) {
        for (int j = c + 1; j < n; j++) b[c] -= M[c * n + j] * b[j];
        b[c] /= M[c * n + c];
    }
}
static int ric_relax(ws_t *S, int k, const double *Pn, double dc, double *Pt, int en) {
    const int nx = S->nx, nes = S->nes, nv = S->nv;
    double *Dr = S->Drg + (size_t)k * nx, *Jt = S->Jtg + (size_t)k * S->ne * nx, *L = S->LUg + (size_t)k * nx * nx;
    int *pv = S->LUp + (size_t)k * nx;
    const double *Jn = S->Je + (size_t)(k + 1) * S->ne * nv;
    int any = 0;
    for (int j = 0; j < nx; j++) {
        Dr[j] = (S->O->dc_all ? dc : 0.0) + RDIAG(S, k * nx + j);
        any |= Dr[j] > 0.0;
    }
    memcpy(Pt, Pn, sizeof(double) * nx * nx);
    if (en)
        for (int e = 0; e < nes; e++)
            for (int j = 0; j < nx; j++) Jt[e * nx + j] = Jn[e * nv + j];
    if (!any) { pv[0] = -1; return 0; }  /* hard rows: L = I */
    double G[GX * GX], sq[GX];
    int gp[2 * GX], np, nn, nz;
    for (int j = 0; j < nx; j++) sq[j] = sqrt(Dr[j]);
    for (int i = 0; i < nx; i++)
        for (int j = 0; j < nx; j++) G[i * nx + j] = (i == j ? 1.0 : 0.0) + sq[i] * Pn[i * nx + j] * sq[j];
    bk_factor(G, nx, gp, gp + nx, &np, &nn, &nz);
    if (nz || nn) return 1;
    for (int i = 0; i < nx; i++)
        for (int j = 0; j < nx; j++) L[i * nx + j] = (i == j ? 1.0 : 0.0) + Pn[i * nx + j] * Dr[j];
    if (lu_factor(L, nx, pv)) return 1;
    for (int j = 0; j < nx; j++) { /* P~ column j */
        double col[GX];
        for (int i = 0; i < nx; i++) col[i] = Pn[i * nx + j];
        lu_solve(L, nx, pv, col);
        for (int i = 0; i < nx; i++) Pt[i * nx + j] = col[i];
    }
    for (int i = 0; i < nx; i++)
        for (int j = 0; j < i; j++) Pt[i * nx + j] = Pt[j * nx + i] = 0.5 * (Pt[i * nx + j] + Pt[j * nx + i]);
    if (en)
        for (int e = 0; e < nes; e++) lu_solve(L, nx, pv, Jt + e * nx);
    return 0;
}
/* p~ = L^-1 p of stage k (identity on hard rows) */
static void ric_ptilde(const ws_t *S, int k, const double *p, double *pt) {
    const int nx = S->nx;
    memcpy(pt, p, sizeof(double) * nx);
    if (S->LUp[(size_t)k * nx] >= 0) lu_solve(S->LUg + (size_t)k * nx * nx, nx, S->LUp + (size_t)k * nx, pt);
}

/* state-equality block of stage k under relaxed dynamics: E = J~ D_r J_n^T */
static double ric_eblock(const ws_t *S, int k, int e1, int e2) {
    const int nx = S->nx, nv = S->nv;
    const double *Dr = S->Drg + (size_t)k * nx, *Jt = S->Jtg + (size_t)k * S->ne * nx;
    const double *Jn = S->Je + (size_t)(k + 1) * S->ne * nv;
    double acc = 0.0;
    for (int l = 0; l < nx; l++) acc += Jt[e1 * nx + l] * Dr[l] * Jn[e2 * nv + l];
    return acc;
}

static int kkt_factor_ric(ws_t *S, double dw, double dc, double d1) {
    const mfg_ocp *P = S->P;
    const int N = S->N, nx = S->nx, nu = S->nu, nv = S->nv, ni = S->ni, ne = S->ne, nes = S->nes, nk = S->nk;
    S->dw = dw; S->dc = dc; S->d1 = d1;
    double Pn[GX * GX], H[GV * GV], T1[GX * GU], T2[GX * GX], K[BKMAX * BKMAX], Rh[BKMAX * GX], Qxx[GX * GX];
    double Dd[GI], Pt[GX * GX];
    const int oE = N * nx + N * ni;
    for (int i = 0; i < nx; i++)
        for (int j = 0; j < nx; j++) Pn[i * nx + j] = (i == j) ? S->Sx[N * nx + i] + dw : 0.0;
    for (int k = N - 1; k >= 0; k--) {
        const double *A = S->Af + (size_t)k * nx * nx, *B = S->Bf + (size_t)k * nx * nu;
        const double *W = S->W + (size_t)k * nv * nv, *Ji = S->Ji + (size_t)k * ni * nv;
        const double *Je = S->Je + (size_t)k * ne * nv, *Jn = S->Jtg + (size_t)k * ne * nx;
        const int en = (k + 1 < N) && EQ_ON(S, k + 1, 0) && nes > 0;
        if (ric_relax(S, k, Pn, dc, Pt, en)) return 1;
        memcpy(Pn, Pt, sizeof(double) * nx * nx);
        memcpy(S->Pg + (size_t)k * nx * nx, Pn, sizeof(double) * nx * nx);
        for (int q = 0; q < ni; q++) {
            const double sg = S->Ss[k * ni + q] + dw;
            Dd[q] = CACT(S, k, q) ? sg / (1.0 + (dc + RDIAG(S, N * nx + k * ni + q)) * sg) : 0.0;
        }
        for (int a = 0; a < nv; a++)
            for (int c = 0; c < nv; c++) {
                double v;
                if (!vfree(S, k, a) || !vfree(S, k, c)) {
                    v = (a == c) ? 1.0 : 0.0;
                } else {
                    v = W[a * nv + c];
                    for (int q = 0; q < ni; q++) v += Ji[q * nv + a] * Dd[q] * Ji[q * nv + c];
                    if (a == c) {
                        v += dw;
                        if (a < nx) v += S->Sx[k * nx + a];
                        else {
                            v += S->Su[k * nu + a - nx];
                            if (a - nx >= P->tier1_from && a - nx < P->tier1_to) v += d1;
                        }
                    }
                }
                H[a * nv + c] = v;
            }
        for (int i = 0; i < nx; i++) {
            for (int c = 0; c < nu; c++) {
                double acc = 0.0;
                for (int l = 0; l < nx; l++) acc += Pn[i * nx + l] * B[l * nu + c];
                T1[i * nu + c] = acc;
            }
            for (int j = 0; j < nx; j++) {
                double acc = 0.0;
                for (int l = 0; l < nx; l++) acc += Pn[i * nx + l] * A[l * nx + j];
                T2[i * nx + j] = acc;
            }
        }
        for (int a = 0; a < nk; a++)
            for (int c = 0; c < nk; c++) {
                double v = 0.0;
                if (a < nu && c < nu) {
                    if (S->ufix[k * nu + a] || S->ufix[k * nu + c]) v = (a == c) ? 1.0 : 0.0;
                    else {
                        v = H[(nx + a) * nv + nx + c];
                        for (int l = 0; l < nx; l++) v += B[l * nu + a] * T1[l * nu + c];
                    }
                } else if (a >= nu && c >= nu) {
                    const int ee = a - nu, e2 = c - nu;
                    if (ee >= nes) /* mixed row of stage k */
                        v = (a == c) ? -dc - RDIAG(S, oE + k * ne + ee) : 0.0;
                    else if (en && e2 < nes) /* state row of node k+1 */
                        v = ((a == c) ? -dc - RDIAG(S, oE + (k + 1) * ne + ee) : 0.0) - ric_eblock(S, k, ee, e2);
                    else
                        v = (a == c) ? (en ? -dc : -1.0) : 0.0;
                } else {
                    const int ee = (a >= nu ? a : c) - nu, uu = a >= nu ? c : a;
                    if (S->ufix[k * nu + uu]) v = 0.0;
                    else if (ee >= nes) v = Je[ee * nv + nx + uu];  /* mixed row of stage k */
                    else if (en)
                        for (int l = 0; l < nx; l++) v += Jn[ee * nx + l] * B[l * nu + uu];
                }
                K[a * nk + c] = v;
            }
        for (int a = 0; a < nk; a++)
            for (int j = 0; j < nx; j++) {
                double v = 0.0;
                if (k > 0) {
                    if (a < nu) {
                        if (!S->ufix[k * nu + a]) {
                            v = H[(nx + a) * nv + j];
                            for (int l = 0; l < nx; l++) v += B[l * nu + a] * T2[l * nx + j];
                        }
                    } else if (a - nu >= nes) {
                        v = Je[(a - nu) * nv + j];
                    } else if (en) {
                        for (int l = 0; l < nx; l++) v += Jn[(a - nu) * nx + l] * A[l * nx + j];
                    }
                }
                Rh[a * nx + j] = v;
            }
        for (int i = 0; i < nx; i++)
            for (int j = 0; j < nx; j++) {
                double v = H[i * nv + j];
                for (int l = 0; l < nx; l++) v += A[l * nx + i] * T2[l * nx + j];
                Qxx[i * nx + j] = v;
            }
        double *Kk = S->Kst + (size_t)k * nk * nk;
        int *pp = S->Kpp + (size_t)k * 2 * nk;
        memcpy(Kk, K, sizeof(double) * nk * nk);
        int np, nn, nz;
        bk_factor(Kk, nk, pp, pp + nk, &np, &nn, &nz);
        if (nz) return 2;
        if (np != nu || nn != ne) return 1;
        double *Fk = S->Fg + (size_t)k * nk * nx;
        for (int j = 0; j < nx; j++) {
            double col[BKMAX];
            for (int a = 0; a < nk; a++) col[a] = -Rh[a * nx + j];
            bk_solve(Kk, nk, pp, pp + nk, col);
            for (int a = 0; a < nk; a++) Fk[a * nx + j] = col[a];
        }
        if (k > 0) {
            double Pt[GX * GX];
            for (int i = 0; i < nx; i++)
                for (int j = 0; j < nx; j++) {
                    double acc = Qxx[i * nx + j];
                    for (int a = 0; a < nk; a++) acc += Rh[a * nx + i] * Fk[a * nx + j];
                    Pt[i * nx + j] = acc;
                }
            for (int i = 0; i < nx; i++)
                for (int j = 0; j < nx; j++) Pn[i * nx + j] = 0.5 * (Pt[i * nx + j] + Pt[j * nx + i]);
        }
    }
    return 0;
}

static void kkt_direction_ric(ws_t *S, double mu, const double *rdyn, const double *rin, const double *req) {
    const int N = S->N, nx = S->nx, nu = S->nu, nv = S->nv, ni = S->ni, ne = S->ne, nes = S->nes, nk = S->nk;
    const double dw = S->dw, dc = S->dc;
    const int oE = N * nx + N * ni;
    double pvs[GX], vx[GV], tv[GX], zv[BKMAX], dxs[GX], dxn[GX], duv[BKMAX], rh[GX];
    for (int j = 0; j < nx; j++) pvs[j] = S->gx[N * nx + j] - S->lam[(N - 1) * nx + j];
    for (int k = N - 1; k >= 0; k--) {
        const double *A = S->Af + (size_t)k * nx * nx, *B = S->Bf + (size_t)k * nx * nu;
        const double *Ji = S->Ji + (size_t)k * ni * nv, *Je = S->Je + (size_t)k * ne * nv;
        const double *Jn = S->Jtg + (size_t)k * ne * nx, *Pk = S->Pg + (size_t)k * nx * nx;
        const double *Dr = S->Drg + (size_t)k * nx;
        const int en = (k + 1 < N) && EQ_ON(S, k + 1, 0) && nes > 0;
        memcpy(S->pvg + (size_t)k * nx, pvs, sizeof(double) * nx);
        double pt[GX];
        ric_ptilde(S, k, pvs, pt);
        for (int j = 0; j < nx; j++) rh[j] = rdyn[k * nx + j] + RCORR(S, k * nx + j);
        for (int a = 0; a < nv; a++) {
            double g = 0.0;
            if (vfree(S, k, a)) {
                g = S->gl[k * nv + a];
                for (int q = 0; q < ni; q++) {
                    const int i = k * ni + q;
                    double w = S->yi[i];
                    if (CACT(S, k, q)) {
                        const double sg = S->Ss[i] + dw, D = sg / (1.0 + (dc + RDIAG(S, N * nx + i)) * sg);
                        w += D * (rin[i] + RCORR(S, N * nx + i) + (S->gs[i] - S->yi[i]) / sg);
                    }
                    g += Ji[q * nv + a] * w;
                }
                if (a < nx) {
                    g += S->gx[k * nx + a] - (k > 0 ? S->lam[(k - 1) * nx + a] : 0.0);
                    for (int jj = 0; jj < nx; jj++) g += A[jj * nx + a] * S->lam[k * nx + jj];
                } else {
                    g += S->gu[k * nu + a - nx];
                    for (int jj = 0; jj < nx; jj++) g += B[jj * nu + a - nx] * S->lam[k * nx + jj];
                }
                for (int e = 0; e < ne; e++)
                    if (EQ_ON(S, k, e) && (e >= nes || a < nx)) g += Je[e * nv + a] * S->ye[k * ne + e];
            }
            vx[a] = g;
        }
        for (int j = 0; j < nx; j++) {
            double acc = pt[j];
            for (int l = 0; l < nx; l++) acc += Pk[j * nx + l] * rh[l];
            tv[j] = acc;
        }
        for (int a = 0; a < nk; a++) {
            double z = 0.0;
            if (a < nu) {
                if (!S->ufix[k * nu + a]) {
                    z = vx[nx + a];
                    for (int l = 0; l < nx; l++) z += B[l * nu + a] * tv[l];
                }
            } else if (a - nu >= nes) {
                z = req[k * ne + a - nu] + RCORR(S, oE + k * ne + a - nu);
            } else if (en) {
                const int ee = a - nu;
                z = req[(k + 1) * ne + ee] + RCORR(S, oE + (k + 1) * ne + ee);
                for (int l = 0; l < nx; l++)
                    z += Jn[ee * nx + l] * rh[l] - S->Je[(size_t)(k + 1) * ne * nv + ee * nv + l] * Dr[l] * pt[l];
            }
            zv[a] = z;
        }
        const double *Kk = S->Kst + (size_t)k * nk * nk, *Fk = S->Fg + (size_t)k * nk * nx;
        const int *pp = S->Kpp + (size_t)k * 2 * nk;
        for (int a = 0; a < nk; a++) duv[a] = -zv[a];
        bk_solve(Kk, nk, pp, pp + nk, duv);
        memcpy(S->kvg + (size_t)k * nk, duv, sizeof(double) * nk);
        if (k > 0) {
            for (int j = 0; j < nx; j++) {
                double acc = vx[j];
                for (int l = 0; l < nx; l++) acc += A[l * nx + j] * tv[l];
                for (int a = 0; a < nk; a++) acc += Fk[a * nx + j] * zv[a];
                dxn[j] = acc;
            }
            memcpy(pvs, dxn, sizeof(double) * nx);
        }
    }
    for (int j = 0; j < nx; j++) { dxs[j] = 0.0; S->dx[j] = 0.0; }
    for (int e = 0; e < ne; e++) S->dye[e] = 0.0;
    for (int k = 0; k < N; k++) {
        const double *A = S->Af + (size_t)k * nx * nx, *B = S->Bf + (size_t)k * nx * nu;
        const double *Jn = S->Jtg + (size_t)k * ne * nx, *Pk = S->Pg + (size_t)k * nx * nx;
        const double *Fk = S->Fg + (size_t)k * nk * nx, *kv = S->kvg + (size_t)k * nk;
        const double *Dr = S->Drg + (size_t)k * nx, *pk = S->pvg + (size_t)k * nx;
        const int en = (k + 1 < N) && EQ_ON(S, k + 1, 0) && nes > 0;
        for (int a = 0; a < nk; a++) {
            double acc = kv[a];
            for (int j = 0; j < nx; j++) acc += Fk[a * nx + j] * dxs[j];
            if (a < nu && S->ufix[k * nu + a]) acc = 0.0;
            duv[a] = acc;
            if (a < nu) S->du[k * nu + a] = acc;
        }
        /* z = A dx + B du + r; dlam = P~ z + p~ + J~^T dy_s; dx_{k+1} = z - D_r dlam */
        double pt[GX];
        ric_ptilde(S, k, pk, pt);
        for (int j = 0; j < nx; j++) {
            double acc = rdyn[k * nx + j] + RCORR(S, k * nx + j);
            for (int l = 0; l < nx; l++) acc += A[j * nx + l] * dxs[l];
            for (int c = 0; c < nu; c++) acc += B[j * nu + c] * duv[c];
            dxn[j] = acc;
        }
        for (int j = 0; j < nx; j++) {
            double acc = pt[j];
            for (int l = 0; l < nx; l++) acc += Pk[j * nx + l] * dxn[l];
            if (en)
                for (int ee = 0; ee < nes; ee++) acc += Jn[ee * nx + j] * duv[nu + ee];
            S->dlam[k * nx + j] = acc;
        }
        for (int j = 0; j < nx; j++) {
            dxn[j] -= Dr[j] * S->dlam[k * nx + j];
            S->dx[(k + 1) * nx + j] = dxn[j];
        }
        if (k + 1 < N)
            for (int ee = 0; ee < nes; ee++) S->dye[(k + 1) * ne + ee] = en ? duv[nu + ee] : 0.0;
        for (int m = nes; m < ne; m++) S->dye[k * ne + m] = duv[nu + m];
        memcpy(dxs, dxn, sizeof(double) * nx);
    }
    slack_and_bound_steps(S, mu, rin);
}

/* fraction to the boundary of the current direction */
#define FTB(v, dv, lo, hi, zl, dzl, zu, dzu)                                                      \
    do {                                                                                          \
        if (hasb(lo)) { if ((dv) < 0) ap = fmin(ap, -tau_fb * ((v) - (lo)) / (dv));                \
                        if ((dzl) < 0) az = fmin(az, -tau_fb * (zl) / (dzl)); }                   \
        if (hasb(hi)) { if ((dv) > 0) ap = fmin(ap, tau_fb * ((hi) - (v)) / (dv));                 \
                        if ((dzu) < 0) az = fmin(az, -tau_fb * (zu) / (dzu)); }                   \
    } while (0)
static void ftb(const ws_t *S, double tau_fb, double *ap_out, double *az_out) {
    const int N = S->N, nx = S->nx, nu = S->nu, ni = S->ni;
    double ap = 1.0, az = 1.0;
    for (int k = 1; k <= N; k++)
        for (int j = 0; j < nx; j++) {
            const int i = k * nx + j;
            FTB(S->x[i], S->dx[i], S->xlo[j], S->xhi[j], S->zxL[i], S->dzxL[i], S->zxU[i], S->dzxU[i]);
        }
    for (int i = 0; i < N * nu; i++)
        if (!S->ufix[i]) FTB(S->u[i], S->du[i], S->ulo[i], S->uhi[i], S->zuL[i], S->dzuL[i], S->zuU[i], S->dzuU[i]);
    for (int i = 0; i < N * ni; i++)
        FTB(S->s[i], S->ds[i], S->clo[i], S->chi[i], S->vL[i], S->dvL[i], S->vU[i], S->dvU[i]);
    if (S->resto)
        for (int r = 0; r < S->NR; r++)
            if (row_el(S, r)) {
                FTB(S->pr[r], S->dpr[r], 0.0, INFINITY, S->zp[r], S->dzp[r], 0.0, 0.0);
                FTB(S->nr[r], S->dnr[r], 0.0, INFINITY, S->zn[r], S->dzn[r], 0.0, 0.0);
            }
    *ap_out = ap;
    *az_out = az;
}
static void ftb_report(const ws_t *S, double tau_fb) {
    const int N = S->N, nx = S->nx, nu = S->nu, ni = S->ni;
    double ap = 1.0, az = 1.0;
    for (int k = 1; k <= N; k++)
        for (int j = 0; j < nx; j++) {
            const int i = k * nx + j;
            FTB(S->x[i], S->dx[i], S->xlo[j], S->xhi[j], S->zxL[i], S->dzxL[i], S->zxU[i], S->dzxU[i]);
        }
    for (int i = 0; i < N * nu; i++)
        if (!S->ufix[i]) FTB(S->u[i], S->du[i], S->ulo[i], S->uhi[i], S->zuL[i], S->dzuL[i], S->zuU[i], S->dzuU[i]);
    const double apx = ap;
    for (int i = 0; i < N * ni; i++) {
        const double a0 = ap;
        FTB(S->s[i], S->ds[i], S->clo[i], S->chi[i], S->vL[i], S->dvL[i], S->vU[i], S->dvU[i]);
        if (ap < a0)
            fprintf(stderr, "      ftb s k %d row %d s %.4e ds %.4e c %.4e [%g, %g] -> %.3e\n", i / ni, i % ni, S->s[i],
                    S->ds[i], S->ci[i], S->clo[i], S->chi[i], ap);
    }
    fprintf(stderr, "   ftb x/u %.3e all %.3e\n", apx, ap);
}
#undef FTB

/* directional derivative of the barrier objective and the curvature term of the penalty update */
static void direction_model(const ws_t *S, double *gdot_out, double *pHp_out) {
    const int N = S->N, nx = S->nx, nu = S->nu, nv = S->nv, ni = S->ni;
    double gdot = 0, pHp = 0;
    for (int k = 0; k < N; k++) {
        const double *W = S->W + (size_t)k * nv * nv;
        double d[GV];
        for (int a = 0; a < nx; a++) d[a] = S->dx[k * nx + a];
        for (int a = 0; a < nu; a++) d[nx + a] = S->du[k * nu + a];
        for (int a = 0; a < nv; a++) {
            gdot += S->gl[k * nv + a] * d[a];
            for (int b = 0; b < nv; b++) pHp += d[a] * W[a * nv + b] * d[b];
        }
        for (int a = 0; a < nu; a++) {
            const int i = k * nu + a;
            gdot += S->gu[i] * S->du[i];
            pHp += S->Su[i] * S->du[i] * S->du[i];
        }
        for (int q = 0; q < ni; q++) {
            const int i = k * ni + q;
            gdot += S->gs[i] * S->ds[i];
            pHp += S->Ss[i] * S->ds[i] * S->ds[i];
        }
    }
    for (int i = nx; i < (N + 1) * nx; i++) {
        gdot += S->gx[i] * S->dx[i];
        pHp += S->Sx[i] * S->dx[i] * S->dx[i];
    }
    if (S->resto)
        for (int r = 0; r < S->NR; r++)
            if (row_el(S, r)) gdot += (S->rho_r + S->gp[r]) * S->dpr[r] + (S->rho_r + S->gn[r]) * S->dnr[r];
    *gdot_out = gdot;
    *pHp_out = pHp;
}

static void trial_point(ws_t *S, double alpha) {
    const size_t NX1 = (size_t)(S->N + 1) * S->nx, NU = (size_t)S->N * S->nu, NI = (size_t)S->N * S->ni;
    for (size_t i = 0; i < NX1; i++) S->tx[i] = S->x[i] + alpha * S->dx[i];
    for (size_t i = 0; i < NU; i++) S->tu[i] = S->u[i] + alpha * S->du[i];
    for (size_t i = 0; i < NI; i++) S->ts[i] = S->s[i] + alpha * S->ds[i];
    if (S->resto)
        for (int r = 0; r < S->NR; r++) {
            S->tpr[r] = S->pr[r] + alpha * S->dpr[r];
            S->tnr[r] = S->nr[r] + alpha * S->dnr[r];
        }
}

/* the direction arrays, in a fixed order, for save / restore around second-order corrections */
static int dir_arrays(ws_t *S, double ***arr, size_t *len) {
    const size_t NX1 = (size_t)(S->N + 1) * S->nx, NXN = (size_t)S->N * S->nx, NU = (size_t)S->N * S->nu,
                 NI = (size_t)S->N * S->ni, NE = (size_t)S->N * S->ne;
    double **a[] = {&S->dx, &S->du, &S->ds, &S->dlam, &S->dye, &S->dyi, &S->dzxL, &S->dzxU, &S->dzuL, &S->dzuU,
                    &S->dvL, &S->dvU, &S->dpr, &S->dnr, &S->dzp, &S->dzn};
    const size_t l[] = {NX1, NU, NI, NXN, NE, NI, NX1, NX1, NU, NU, NI, NI, S->NR, S->NR, S->NR, S->NR};
    for (int i = 0; i < 16; i++) { arr[i] = a[i]; len[i] = l[i]; }
    return S->resto ? 16 : 12;
}
static void save_direction(ws_t *S) {
    double **arr[16];
    size_t len[16], off = 0;
    const int na = dir_arrays(S, arr, len);
    for (int i = 0; i < na; i++) { memcpy(S->bk + off, *arr[i], len[i] * sizeof(double)); off += len[i]; }
}
static void restore_direction(ws_t *S) {
    double **arr[16];
    size_t len[16], off = 0;
    const int na = dir_arrays(S, arr, len);
    for (int i = 0; i < na; i++) { memcpy(*arr[i], S->bk + off, len[i] * sizeof(double)); off += len[i]; }
}

/* the iterate arrays, in a fixed order, for the watchdog's stored point */
static int iter_arrays(ws_t *S, double ***arr, size_t *len) {
    const size_t NX1 = (size_t)(S->N + 1) * S->nx, NXN = (size_t)S->N * S->nx, NU = (size_t)S->N * S->nu,
                 NI = (size_t)S->N * S->ni, NE = (size_t)S->N * S->ne;
    double **a[] = {&S->x, &S->u, &S->s, &S->lam, &S->ye, &S->yi, &S->zxL, &S->zxU, &S->zuL, &S->zuU, &S->vL, &S->vU,
                    &S->pr, &S->nr, &S->zp, &S->zn};
    const size_t l[] = {NX1, NU, NI, NXN, NE, NI, NX1, NX1, NU, NU, NI, NI, S->NR, S->NR, S->NR, S->NR};
    for (int i = 0; i < 16; i++) { arr[i] = a[i]; len[i] = l[i]; }
    return S->resto ? 16 : 12;
}
static void copy_arrays(ws_t *S, int (*fn)(ws_t *, double ***, size_t *), double *buf, int to_buf) {
    double **arr[16];
    size_t len[16], off = 0;
    const int na = fn(S, arr, len);
    for (int i = 0; i < na; i++) {
        if (to_buf) memcpy(buf + off, *arr[i], len[i] * sizeof(double));
        else memcpy(*arr[i], buf + off, len[i] * sizeof(double));
        off += len[i];
    }
}

/* ---- IPOPT's filter line search (mfg_opts.filter) ----
 * Constants are IPOPT's defaults (IpFilterLSAcceptor.cpp): gamma_theta 1e-5, gamma_phi 1e-8, delta 1,
 * s_theta 1.1, s_phi 2.3, eta_phi 1e-8, theta_max = 1e4 max(1, theta_0), theta_min = 1e-4 max(1, theta_0),
 * alpha_min_frac 0.05, kappa_soc 0.99, obj_max_inc 5.  theta is the l1 norm of (c, d - s), phi the
 * barrier objective. */
typedef struct {
    double *fph, *fth;  /* filter entries (phi, theta), already margined */
    int nf, cap;
    double theta_max, theta_min;
    double rph, rth, rgd;  /* reference point: phi, theta, grad phi^T d */
} filt_t;

static int ls_le(double a, double b, double bas) { return a - b <= 10.0 * 2.220446049250313e-16 * fabs(bas); }
static int ls_ftype(const filt_t *L, double a) {
    return L->rgd < 0.0 && a * pow(-L->rgd, 2.3) > pow(L->rth, 1.1);
}
static int ls_armijo(const filt_t *L, double a, double ph) { return ls_le(ph - L->rph, 1e-8 * a * L->rgd, L->rph); }
static int ls_acceptable(const filt_t *L, double atest, double ph, double th, int ok) {
    if (!ok || !isfinite(ph) || !isfinite(th)) return 0;
    if (th > L->theta_max) return 0;
    if (atest > 0.0 && ls_ftype(L, atest) && L->rth <= L->theta_min) {
        if (!ls_armijo(L, atest, ph)) return 0;
    } else {
        if (ph > L->rph) {
            const double bas = fabs(L->rph) > 10.0 ? log10(fabs(L->rph)) : 1.0;
            if (log10(ph - L->rph) > 5.0 + bas) return 0;
        }
        if (!(ls_le(th, (1.0 - 1e-5) * L->rth, L->rth) || ls_le(ph - L->rph, -1e-8 * L->rth, L->rph))) return 0;
    }
    for (int j = 0; j < L->nf; j++)
        if (!(ph <= L->fph[j] || th <= L->fth[j])) return 0;
    return 1;
}
static void ls_augment(filt_t *L) {
    if (L->nf == L->cap) {
        L->cap = L->cap ? 2 * L->cap : 64;
        L->fph = (double *)realloc(L->fph, L->cap * sizeof(double));
        L->fth = (double *)realloc(L->fth, L->cap * sizeof(double));
    }
    L->fph[L->nf] = L->rph - 1e-8 * L->rth;
    L->fth[L->nf] = (1.0 - 1e-5) * L->rth;
    L->nf++;
}
static double ls_alpha_min(const filt_t *L) {
    double am = 1e-5;
    if (L->rgd < 0.0) {
        am = fmin(1e-5, 1e-8 * L->rth / (-L->rgd));
        if (L->rth <= L->theta_min) am = fmin(am, pow(L->rth, 1.1) / pow(-L->rgd, 2.3));
    }
    return 0.05 * am;
}

#define TP(S) ((S)->resto ? (S)->tpr : NULL)
#define TN(S) ((S)->resto ? (S)->tnr : NULL)
/* DoBacktrackingLineSearch (IpBacktrackingLineSearch.cpp): trial steps alpha_max, alpha_max/2, ... down to
 * alpha_min; a second-order correction after a rejected first trial point that did not lower theta below
 * the current one (thc); in the watchdog only the full step is tried, tested with the watchdog's alpha.
 * Returns 1 with the accepted step (alpha, az, and the SOC direction left in place when one was taken). */
static int filter_backtrack(ws_t *S, const filt_t *L, double mu, double tau_fb, double ap, double thc, int skip_first,
                            int in_wd, double wd_atest, double *alpha_out, double *az_io, double *atest_out,
                            int *nsteps_out, int *soc_out, double *ph_out, double *th_out, double *ts) {
    const int N = S->N, nx = S->nx, ni = S->ni, ne = S->ne;
    const double alpha_min = in_wd ? ap : ls_alpha_min(L);
    double alpha = ap, atest = in_wd ? wd_atest : ap, ph = 0, th = 0, t_ph, last = ap;
    int n_steps = 0, accept = 0, soc = 0, ok;
    if (skip_first) alpha *= 0.5;
    while (alpha > alpha_min || n_steps == 0) {
        if (!in_wd) atest = alpha;
        last = alpha;
        trial_point(S, alpha);
        t_ph = wall_s();
        merit_parts_e(S, S->tx, S->tu, S->ts, TP(S), TN(S), mu, &ph, &th, &ok, S->trdyn, S->trin, S->treq);
        ts[3] += wall_s() - t_ph;
        if (ls_acceptable(L, atest, ph, th, ok)) { accept = 1; break; }
        if (in_wd) break;
        if (ok && alpha == ap && thc <= th && S->O->max_soc > 0) {
            double th_trial = th, th_old = 0.0, a_soc = alpha;
            for (size_t i = 0; i < (size_t)N * nx; i++) S->sdyn[i] = S->rdyn[i];
            for (size_t i = 0; i < (size_t)N * ni; i++) S->sin_[i] = S->rin[i];
            for (size_t i = 0; i < (size_t)N * ne; i++) S->seq[i] = S->req[i];
            for (int cnt = 0; cnt < S->O->max_soc && (cnt == 0 || th_trial <= 0.99 * th_old); cnt++) {
                th_old = th_trial;
                for (size_t i = 0; i < (size_t)N * nx; i++) S->sdyn[i] = a_soc * S->sdyn[i] + S->trdyn[i];
                for (size_t i = 0; i < (size_t)N * ni; i++) S->sin_[i] = a_soc * S->sin_[i] + S->trin[i];
                for (size_t i = 0; i < (size_t)N * ne; i++) S->seq[i] = a_soc * S->seq[i] + S->treq[i];
                save_direction(S);
                t_ph = wall_s();
                (S->ric ? kkt_direction_ric : kkt_direction)(S, mu, S->sdyn, S->sin_, S->seq);
                ts[2] += wall_s() - t_ph;
                double azs;
                ftb(S, tau_fb, &a_soc, &azs);
                trial_point(S, a_soc);
                int oks;
                t_ph = wall_s();
                merit_parts_e(S, S->tx, S->tu, S->ts, TP(S), TN(S), mu, &ph, &th, &oks, S->trdyn, S->trin, S->treq);
                ts[3] += wall_s() - t_ph;
                if (S->O->verbose > 1)
                    fprintf(stderr, "      soc %d a %.3e th %.3e (ref %.3e) phi %.10e (ref %.10e)\n", cnt, a_soc, th,
                            L->rth, ph, L->rph);
                if (ls_acceptable(L, atest, ph, th, oks)) {
                    accept = 1; soc = 1; alpha = a_soc; *az_io = azs;
                    break;
                }
                restore_direction(S);
                if (!oks) break;
                th_trial = th;
            }
            if (accept) break;
        }
        alpha *= 0.5;
        n_steps++;
    }
    *alpha_out = accept ? alpha : last;  /* rejected: the last (shortest) trial step */
    *atest_out = atest;
    *nsteps_out = n_steps;
    *soc_out = soc;
    *ph_out = ph;
    *th_out = th;
    return accept;
}

/* relative-pose targets of the Centauro rows from x_0: RelativePosition / RelativeOrientationError at
 * q_0 (Centauro_functions.py:297-343).  The orientation target is optionally rounded as the MPC restart
 * rounds RelativeOrientation_0 (RepeatedMPCwithThermal.py:485-486, np.round: half to even); the position
 * rows chain node k to node k-1 in the reference (L255-272), so for k >= 1 they hold the exact value. */
static void cent_targets(mfg_ocp *P, const models_t *MM) {
    hd xu[GV], hl, hci[GI], hce[GE], hf[GX];
    for (int i = 0; i < P->nx + P->nu; i++) xu[i] = K(i < P->nx ? P->x0[i] : 0.0);
    for (int b = 0; b < 3; b++) P->relpos0[b] = P->orient0[b] = 0.0;
    node_hd(P, MM, xu, &hl, hci, hce, hf);
    const double sc = P->target_decimals >= 0 ? pow(10.0, P->target_decimals) : 0.0;
    for (int b = 0; b < 3; b++) {
        P->relpos0[b] = hce[b].a;
        P->orient0[b] = sc > 0 ? rint(hce[3 + b].a * sc) / sc : hce[3 + b].a;
    }
}


/* ==================================================================== IPOPT mode (mfg_opts.filter) ==== */
/* optimality measures at the current point (its derivatives evaluated): IPOPT's scaled E_0 pieces (max
 * norms) and the primal-dual system error of the soft restoration phase (1-norms / count).  In the
 * restoration phase they are those of the restoration problem. */
typedef struct {
    double dinf, pinf, cinf0, cinfm, sd, sc;
    double s1, n1;  /* sum of |dual inf| + |primal inf| + |z gap - mu|, and the number of terms */
} errs_t;

static void opt_error_f(const ws_t *S, double mu, errs_t *E) {
    const int N = S->N, nx = S->nx, nu = S->nu, nv = S->nv, ni = S->ni, ne = S->ne;
    const double s_max = 100.0;
    double dinf = 0, pinf = 0, cinf0 = 0, cinfm = 0, sum_mult = 0, sum_bmult = 0, s1 = 0, n1 = 0;
    int n_mult = 0, n_bmult = 0;
#define COMPF(z, gap)                                                                           \
    do {                                                                                        \
        double c_ = (z) * (gap);                                                                \
        cinf0 = fmax(cinf0, fabs(c_)); cinfm = fmax(cinfm, fabs(c_ - mu));                      \
        sum_bmult += (z); n_bmult++; s1 += fabs(c_ - mu); n1 += 1;                              \
    } while (0)
#define DUALF(r) do { dinf = fmax(dinf, fabs(r)); s1 += fabs(r); n1 += 1; } while (0)
#define PRIMF(r) do { pinf = fmax(pinf, fabs(r)); s1 += fabs(r); n1 += 1; } while (0)
    for (int k = 1; k <= N; k++)
        for (int j = 0; j < nx; j++) {
            const int i = k * nx + j;
            double r = -S->lam[(k - 1) * nx + j];
            if (k < N) {
                r += S->gl[k * nv + j];
                for (int jj = 0; jj < nx; jj++) r += S->Af[(k * nx + jj) * nx + j] * S->lam[k * nx + jj];
                for (int q = 0; q < ni; q++) r += S->Ji[((size_t)k * ni + q) * nv + j] * S->yi[k * ni + q];
                for (int e = 0; e < ne; e++)
                    if (EQ_ON(S, k, e)) r += S->Je[((size_t)k * ne + e) * nv + j] * S->ye[k * ne + e];
            }
            if (S->resto) r += S->zeta * S->dR[i] * (S->x[i] - S->wR[i]);
            r += -S->zxL[i] + S->zxU[i];
            DUALF(r);
            if (hasb(S->xlo[j])) COMPF(S->zxL[i], S->x[i] - S->xlo[j]);
            if (hasb(S->xhi[j])) COMPF(S->zxU[i], S->xhi[j] - S->x[i]);
        }
    for (int k = 0; k < N; k++) {
        for (int j = 0; j < nu; j++) {
            const int i = k * nu + j;
            if (S->ufix[i]) continue;
            double r = S->gl[k * nv + nx + j];
            for (int jj = 0; jj < nx; jj++) r += S->Bf[(k * nx + jj) * nu + j] * S->lam[k * nx + jj];
            for (int q = 0; q < ni; q++) r += S->Ji[((size_t)k * ni + q) * nv + nx + j] * S->yi[k * ni + q];
            for (int e = S->nes; e < ne; e++) r += S->Je[((size_t)k * ne + e) * nv + nx + j] * S->ye[k * ne + e];
            if (S->resto) {
                const int o = (N + 1) * nx + i;
                r += S->zeta * S->dR[o] * (S->u[i] - S->wR[o]);
            }
            r += -S->zuL[i] + S->zuU[i];
            DUALF(r);
            if (hasb(S->ulo[i])) COMPF(S->zuL[i], S->u[i] - S->ulo[i]);
            if (hasb(S->uhi[i])) COMPF(S->zuU[i], S->uhi[i] - S->u[i]);
        }
        for (int q = 0; q < ni; q++) {
            const int i = k * ni + q;
            if (!CACT(S, k, q)) continue;
            double r = -S->yi[i] - S->vL[i] + S->vU[i];
            DUALF(r);
            if (hasb(S->clo[i])) COMPF(S->vL[i], S->s[i] - S->clo[i]);
            if (hasb(S->chi[i])) COMPF(S->vU[i], S->chi[i] - S->s[i]);
            PRIMF(S->rin[i]);
            sum_mult += fabs(S->yi[i]); n_mult++;
        }
        for (int j = 0; j < nx; j++) {
            PRIMF(S->rdyn[k * nx + j]);
            sum_mult += fabs(S->lam[k * nx + j]); n_mult++;
        }
        for (int e = 0; e < ne; e++)
            if (EQ_ON(S, k, e)) {
                PRIMF(S->req[k * ne + e]);
                sum_mult += fabs(S->ye[k * ne + e]); n_mult++;
            }
    }
    if (S->resto)
        for (int r = 0; r < S->NR; r++) {
            if (!row_el(S, r)) continue;
            const double y = *row_y((ws_t *)S, r);
            DUALF(S->rho_r - y - S->zp[r]);
            DUALF(S->rho_r + y - S->zn[r]);
            COMPF(S->zp[r], S->pr[r]);
            COMPF(S->zn[r], S->nr[r]);
        }
#undef COMPF
#undef DUALF
#undef PRIMF
    E->dinf = dinf; E->pinf = pinf; E->cinf0 = cinf0; E->cinfm = cinfm;
    E->sd = fmax(s_max, (sum_mult + sum_bmult) / fmax(1, n_mult + n_bmult)) / s_max;
    E->sc = fmax(s_max, sum_bmult / fmax(1, n_bmult)) / s_max;
    E->s1 = s1; E->n1 = n1;
}

/* Sigma, barrier gradients (with kappa_d) and, in the restoration phase, the proximity term (folded into
 * Sigma / gradient of x, u) and the condensed elastic rows */
static void barrier_f(ws_t *S, double mu) {
    const int N = S->N, nx = S->nx, nu = S->nu;
#define SIGF(Sg, gg, z_l, z_u, v, lo, hi)                                                   \
    do {                                                                                   \
        Sg = 0; gg = 0;                                                                    \
        if (hasb(lo)) { Sg += (z_l) / ((v) - (lo)); gg -= mu / ((v) - (lo)); }             \
        if (hasb(hi)) { Sg += (z_u) / ((hi) - (v)); gg += mu / ((hi) - (v)); }             \
        if (hasb(lo) && !hasb(hi)) gg += KAPPA_D * mu;                                     \
        if (hasb(hi) && !hasb(lo)) gg -= KAPPA_D * mu;                                     \
    } while (0)
    for (int k = 0; k <= N; k++)
        for (int j = 0; j < nx; j++) {
            const int i = k * nx + j;
            if (k == 0) { S->Sx[i] = S->gx[i] = 0; continue; }
            SIGF(S->Sx[i], S->gx[i], S->zxL[i], S->zxU[i], S->x[i], S->xlo[j], S->xhi[j]);
            if (S->resto) { S->Sx[i] += S->zeta * S->dR[i]; S->gx[i] += S->zeta * S->dR[i] * (S->x[i] - S->wR[i]); }
        }
    for (int i = 0; i < N * nu; i++) {
        if (S->ufix[i]) { S->Su[i] = S->gu[i] = 0; continue; }
        SIGF(S->Su[i], S->gu[i], S->zuL[i], S->zuU[i], S->u[i], S->ulo[i], S->uhi[i]);
        if (S->resto) {
            const int o = (N + 1) * nx + i;
            S->Su[i] += S->zeta * S->dR[o];
            S->gu[i] += S->zeta * S->dR[o] * (S->u[i] - S->wR[o]);
        }
    }
    for (int i = 0; i < N * S->ni; i++) SIGF(S->Ss[i], S->gs[i], S->vL[i], S->vU[i], S->s[i], S->clo[i], S->chi[i]);
#undef SIGF
    if (S->resto)
        for (int r = 0; r < S->NR; r++) {
            if (!row_el(S, r)) { S->Sp[r] = S->Sn[r] = INFINITY; S->gp[r] = S->gn[r] = S->rowr[r] = 0.0; continue; }
            const double y = *row_y(S, r);
            S->Sp[r] = S->zp[r] / S->pr[r];
            S->Sn[r] = S->zn[r] / S->nr[r];
            S->gp[r] = -mu / S->pr[r] + KAPPA_D * mu;
            S->gn[r] = -mu / S->nr[r] + KAPPA_D * mu;
            S->rowr[r] = (S->rho_r + S->gp[r] - y) / S->Sp[r] - (S->rho_r + S->gn[r] + y) / S->Sn[r];
        }
}

/* IPOPT's inertia correction (IpPDPerturbationHandler.cpp get_deltas_for_wrong_inertia): delta_w = 0
 * first; on wrong inertia 1e-4 if no earlier perturbation, else max(1e-20, last / 3); then x100 (no earlier
 * one, or last far below) or x8 up to 1e40; a singular matrix first gets delta_c = 1e-8 mu^(1/4) */
static int factor_f(ws_t *S, double mu, double *ic_last, int *n_ic, double *ts) {
    double dw = 0.0, dc = (S->P->dc_always || S->O->dc_all) ? 1e-8 * pow(mu, 0.25) : 0.0;
    const int ric = S->ric;  /* off in the restoration phase unless riccati >= 2 */
    for (int tries = 0; tries < 200; tries++) {
        const double t0 = wall_s();
        const int fr = ric ? kkt_factor_ric(S, dw, dc, 0.0) : kkt_factor(S, dw, dc, 0.0);
        ts[1] += wall_s() - t0;
        if (fr == 0) {
            if (dw > 0.0) *ic_last = dw;
            return 1;
        }
        if (fr == 2 && dc == 0.0) { dc = 1e-8 * pow(mu, 0.25); continue; }
        (*n_ic)++;
        if (dw == 0.0) dw = (*ic_last == 0.0) ? 1e-4 : fmax(1e-20, *ic_last / 3.0);
        else dw *= (*ic_last == 0.0 || 1e5 * *ic_last < dw) ? 100.0 : 8.0;
        if (dw > 1e40) return 0;
    }
    return 0;
}

/* riccati = 3 (test mode): in the restoration phase factor and solve both ways, keep the Riccati
 * direction, and record the largest difference of the primal-dual steps relative to their size */
static double g_ric_check = 0.0;
/* test hook: searches after StopWatchDog that failed (the re-evaluated stored point goes to the restoration) */
static int g_wd_fail = 0;
int mfg_wdfail_count(int reset) {
    const int v = g_wd_fail;
    if (reset) g_wd_fail = 0;
    return v;
}
/* largest residual of the current step (dx, du, dlam, dye) in the unfactored KKT system (the rows kkt_factor
 * assembles: stationarity of the free x_k, u_k; dynamics; equality rows) */
static double kkt_resid(const ws_t *S, const double *rdyn, const double *rin, const double *req) {
    const int N = S->N, nx = S->nx, nu = S->nu, nv = S->nv, ni = S->ni, ne = S->ne;
    const double dw = S->dw, dc = S->dc, d1 = S->d1;
    double res = 0.0;
    for (int k = 0; k <= N; k++) {
        if (k == N) {
            for (int j = 0; j < nx; j++)
                res = fmax(res, fabs((S->Sx[N * nx + j] + dw) * S->dx[N * nx + j] - S->dlam[(N - 1) * nx + j] +
                                     S->gx[N * nx + j] - S->lam[(N - 1) * nx + j]));
            break;
        }
        const double *A = S->Af + (size_t)k * nx * nx, *B = S->Bf + (size_t)k * nx * nu;
        const double *W = S->W + (size_t)k * nv * nv, *Ji = S->Ji + (size_t)k * ni * nv;
        const double *Je = S->Je + (size_t)k * ne * nv;
        double dv[GV], Dd[GI], rdd[GI];
        for (int a = 0; a < nv; a++) dv[a] = !vfree(S, k, a) ? 0.0 : (a < nx ? S->dx[k * nx + a] : S->du[k * nu + a - nx]);
        for (int q = 0; q < ni; q++) {
            const int i = k * ni + q;
            if (CACT(S, k, q)) {
                const double sg = S->Ss[i] + dw;
                Dd[q] = sg / (1.0 + (dc + RDIAG(S, N * nx + i)) * sg);
                rdd[q] = rin[i] + RCORR(S, N * nx + i) + (S->gs[i] - S->yi[i]) / sg;
            } else { Dd[q] = 0; rdd[q] = 0; }
        }
        for (int a = 0; a < nv; a++) {
            if (!vfree(S, k, a)) continue;
            double g = S->gl[k * nv + a], v = 0.0;
            for (int q = 0; q < ni; q++) g += Ji[q * nv + a] * (S->yi[k * ni + q] + Dd[q] * rdd[q]);
            for (int c = 0; c < nv; c++) {
                double h = W[a * nv + c];
                for (int q = 0; q < ni; q++) h += Ji[q * nv + a] * Dd[q] * Ji[q * nv + c];
                v += h * dv[c];
            }
            if (a < nx) {
                v += (S->Sx[k * nx + a] + dw) * dv[a];
                g += S->gx[k * nx + a] - (k > 0 ? S->lam[(k - 1) * nx + a] : 0.0);
                if (k > 0) v -= S->dlam[(k - 1) * nx + a];
                for (int jj = 0; jj < nx; jj++) {
                    g += A[jj * nx + a] * S->lam[k * nx + jj];
                    v += A[jj * nx + a] * S->dlam[k * nx + jj];
                }
            } else {
                v += (S->Su[k * nu + a - nx] + dw) * dv[a];
                if (a - nx >= S->P->tier1_from && a - nx < S->P->tier1_to) v += d1 * dv[a];
                g += S->gu[k * nu + a - nx];
                for (int jj = 0; jj < nx; jj++) {
                    g += B[jj * nu + a - nx] * S->lam[k * nx + jj];
                    v += B[jj * nu + a - nx] * S->dlam[k * nx + jj];
                }
            }
            for (int e = 0; e < ne; e++)
                if (EQ_ON(S, k, e)) {
                    g += Je[e * nv + a] * S->ye[k * ne + e];
                    v += Je[e * nv + a] * S->dye[k * ne + e];
                }
            res = fmax(res, fabs(v + g));
        }
        for (int e = 0; e < ne; e++) {
            if (!EQ_ON(S, k, e)) continue;
            const int rr = N * nx + N * ni + k * ne + e;
            double v = -(dc + RDIAG(S, rr)) * S->dye[k * ne + e] + req[k * ne + e] + RCORR(S, rr);
            for (int a = 0; a < nv; a++) v += Je[e * nv + a] * dv[a];
            res = fmax(res, fabs(v));
        }
        for (int j = 0; j < nx; j++) {
            const int rr = k * nx + j;
            const double Dr = (S->O->dc_all ? dc : 0.0) + RDIAG(S, rr);
            double v = -S->dx[(k + 1) * nx + j] - Dr * S->dlam[rr] + rdyn[rr] + RCORR(S, rr);
            for (int l = 0; l < nx; l++) v += A[j * nx + l] * dv[l];
            for (int c = 0; c < nu; c++) v += B[j * nu + c] * dv[nx + c];
            res = fmax(res, fabs(v));
        }
    }
    return res;
}
double mfg_ric_check_max(int reset) {
    const double v = g_ric_check;
    if (reset) g_ric_check = 0.0;
    return v;
}
static void direction_f(ws_t *S, double mu, const double *rdyn, const double *rin, const double *req) {
    if (S->ric && S->resto && S->O->riccati == 3) {
        const int N = S->N, nx = S->nx, nu = S->nu, ne = S->ne;
        const size_t nX = (size_t)(N + 1) * nx, nU = (size_t)N * nu, nL = (size_t)N * nx, nE = (size_t)N * ne;
        double *sv = dal(nX + nU + nL + nE);
        const double dw = S->dw, dc = S->dc, d1 = S->d1;
        if (kkt_factor(S, dw, dc, d1) == 0) {
            kkt_direction(S, mu, rdyn, rin, req);
            const double res_b = getenv("MFG_RIC_DEBUG") ? kkt_resid(S, rdyn, rin, req) : 0.0;
            memcpy(sv, S->dx, nX * sizeof(double));
            memcpy(sv + nX, S->du, nU * sizeof(double));
            memcpy(sv + nX + nU, S->dlam, nL * sizeof(double));
            memcpy(sv + nX + nU + nL, S->dye, nE * sizeof(double));
            kkt_factor_ric(S, dw, dc, d1);
            kkt_direction_ric(S, mu, rdyn, rin, req);
            const double *cur[4] = {S->dx, S->du, S->dlam, S->dye};
            const size_t len[4] = {nX, nU, nL, nE};
            double dmax = 0.0, vmax = 1e-300;
            for (int t = 0, o = 0; t < 4; o += (int)len[t], t++)
                for (size_t i = 0; i < len[t]; i++) {
                    dmax = fmax(dmax, fabs(cur[t][i] - sv[o + i]));
                    vmax = fmax(vmax, fabs(sv[o + i]));
                }
            g_ric_check = fmax(g_ric_check, dmax / vmax);
            if (getenv("MFG_RIC_DEBUG") && dmax / vmax > 1e-6) {
                double drmax = 0, drmin = 1e300;
                for (size_t i = 0; i < nL; i++) { drmax = fmax(drmax, S->Drg[i]); drmin = fmin(drmin, S->Drg[i]); }
                fprintf(stderr, "ric check rel %.2e vmax %.2e Dr [%.2e, %.2e] dw %.2e dc %.2e  KKT residual banded %.2e riccati %.2e\n",
                        dmax / vmax, vmax, drmin, drmax, dw, dc, res_b, kkt_resid(S, rdyn, rin, req));
            }
        } else {
            kkt_factor_ric(S, dw, dc, d1);
            kkt_direction_ric(S, mu, rdyn, rin, req);
        }
        free(sv);
        return;
    }
    if (S->ric) kkt_direction_ric(S, mu, rdyn, rin, req);
    else kkt_direction(S, mu, rdyn, rin, req);
}

/* primal step alpha, dual step az; bound multipliers kept within kappa_sigma = 1e10 of mu / slack */
static void update_f(ws_t *S, double alpha, double az, double mu) {
    const int N = S->N, nx = S->nx, nu = S->nu, ni = S->ni;
    const size_t NX1 = (size_t)(N + 1) * nx, NU = (size_t)N * nu, NI = (size_t)N * ni, NE = (size_t)N * S->ne;
    const double ks = 1e10;
    for (size_t i = 0; i < NX1; i++) S->x[i] += alpha * S->dx[i];
    for (size_t i = 0; i < NU; i++) S->u[i] += alpha * S->du[i];
    for (size_t i = 0; i < NI; i++) { S->s[i] += alpha * S->ds[i]; S->yi[i] += alpha * S->dyi[i]; }
    for (int i = 0; i < N * nx; i++) S->lam[i] += alpha * S->dlam[i];
    for (size_t i = 0; i < NE; i++) S->ye[i] += alpha * S->dye[i];
#define ZUPF(z, dz, slack)                                                                \
    do {                                                                                  \
        double zz = (z) + az * (dz), sl = (slack);                                        \
        (z) = fmax(fmin(zz, ks * mu / sl), mu / (ks * sl));                               \
    } while (0)
    for (int k = 1; k <= N; k++)
        for (int j = 0; j < nx; j++) {
            const int i = k * nx + j;
            if (hasb(S->xlo[j])) ZUPF(S->zxL[i], S->dzxL[i], S->x[i] - S->xlo[j]);
            if (hasb(S->xhi[j])) ZUPF(S->zxU[i], S->dzxU[i], S->xhi[j] - S->x[i]);
        }
    for (int i = 0; i < N * nu; i++) {
        if (S->ufix[i]) continue;
        if (hasb(S->ulo[i])) ZUPF(S->zuL[i], S->dzuL[i], S->u[i] - S->ulo[i]);
        if (hasb(S->uhi[i])) ZUPF(S->zuU[i], S->dzuU[i], S->uhi[i] - S->u[i]);
    }
    for (int i = 0; i < N * ni; i++) {
        if (hasb(S->clo[i])) ZUPF(S->vL[i], S->dvL[i], S->s[i] - S->clo[i]);
        if (hasb(S->chi[i])) ZUPF(S->vU[i], S->dvU[i], S->chi[i] - S->s[i]);
    }
    if (S->resto)
        for (int r = 0; r < S->NR; r++) {
            if (!row_el(S, r)) continue;
            S->pr[r] += alpha * S->dpr[r];
            S->nr[r] += alpha * S->dnr[r];
            ZUPF(S->zp[r], S->dzp[r], S->pr[r]);
            ZUPF(S->zn[r], S->dzn[r], S->nr[r]);
        }
#undef ZUPF
}

static void eval_all(ws_t *S, double *ts) {
    const double t0 = wall_s();
#ifdef _OPENMP
#pragma omp parallel for schedule(dynamic, 1)
#endif
    for (int k = 0; k < S->N; k++) eval_derivs(S, k);
    ts[0] += wall_s() - t0;
    residuals_cached(S, S->rdyn, S->rin, S->req);
}

/* IPOPT's least-square constraint multipliers (DefaultIterateInitializer::least_square_mults, the
 * restoration problem's start): min |grad f + J^T y - z|^2 through [[I, J^T], [J, 0]]; 0 if the system is
 * singular or max |y| > constr_mult_init_max = 1000.  The derivatives of the current point must be
 * evaluated; Sigma / gradients are overwritten (recomputed by barrier_f). */
static void ls_mults(ws_t *S) {
    const int N = S->N, nx = S->nx, nu = S->nu, nv = S->nv, ni = S->ni, ne = S->ne;
    const size_t NXN = (size_t)N * nx, NI = (size_t)N * ni, NE = (size_t)N * ne;
    for (int k = 0; k < N; k++)
        for (int a = 0; a < nv; a++)
            for (int b = 0; b < nv; b++) S->W[(size_t)k * nv * nv + a * nv + b] = (a == b) ? 1.0 : 0.0;
    for (int k = 0; k <= N; k++)
        for (int j = 0; j < nx; j++) {
            const int i = k * nx + j;
            S->Sx[i] = 0.0;
            double g = -S->zxL[i] + S->zxU[i];
            if (S->resto) g += S->zeta * S->dR[i] * (S->x[i] - S->wR[i]);
            S->gx[i] = (k == 0) ? 0.0 : g;
        }
    if (N > 0) for (int j = 0; j < nx; j++) S->Sx[N * nx + j] = 1.0;  /* x_N's Hessian block is I too */
    for (int i = 0; i < N * nu; i++) {
        S->Su[i] = 0.0;
        double g = -S->zuL[i] + S->zuU[i];
        if (S->resto) g += S->zeta * S->dR[(N + 1) * nx + i] * (S->u[i] - S->wR[(N + 1) * nx + i]);
        S->gu[i] = S->ufix[i] ? 0.0 : g;
    }
    for (size_t i = 0; i < NI; i++) { S->Ss[i] = 1.0; S->gs[i] = -S->vL[i] + S->vU[i]; }
    if (S->resto)
        for (int r = 0; r < S->NR; r++) {
            const int el = row_el(S, r);
            S->Sp[r] = S->Sn[r] = el ? 1.0 : INFINITY;
            S->gp[r] = -S->zp[r]; S->gn[r] = -S->zn[r];
            S->rowr[r] = el ? S->zn[r] - S->zp[r] : 0.0;  /* (rho - zp) - (rho - zn), y = 0 */
        }
    memset(S->lam, 0, NXN * sizeof(double));
    memset(S->yi, 0, NI * sizeof(double));
    memset(S->ye, 0, NE * sizeof(double));
    double *z0 = dal(NXN + NI + NE);
    int ok = (kkt_factor(S, 0.0, 0.0, 0.0) == 0);
    if (ok) {
        kkt_direction(S, 0.0, z0, z0 + NXN, z0 + NXN + NI);
        double ym = 0;
        for (size_t i = 0; i < NXN; i++) ym = fmax(ym, fabs(S->dlam[i]));
        for (size_t i = 0; i < NI; i++) ym = fmax(ym, fabs(S->dyi[i]));
        for (size_t i = 0; i < NE; i++) ym = fmax(ym, fabs(S->dye[i]));
        if (ym <= 1e3) {
            memcpy(S->lam, S->dlam, NXN * sizeof(double));
            memcpy(S->yi, S->dyi, NI * sizeof(double));
            memcpy(S->ye, S->dye, NE * sizeof(double));
        }
        if (S->O->verbose) fprintf(stderr, "   least-square multipliers: max |y| %.3e%s\n", ym, ym > 1e3 ? " -> 0" : "");
    } else if (S->O->verbose) fprintf(stderr, "   least-square multipliers: singular system -> 0\n");
    free(z0);
}

/* state of one IPOPT algorithm instance (the main problem, or the restoration problem) */
typedef struct {
    double mu, ic_last;
    filt_t LS;
    int in_wd, wd_short, wd_trial, n_wd;
    double wd_ph, wd_th, wd_gd, wd_atest;
    double *wd_it, *wd_dir;
    int in_soft, soft_cnt, n_resto, n_soft;
} fst_t;

/* the restoration problem's link to the original one (RestoFilterConvergenceCheck) */
typedef struct {
    double mu_orig, th_R;
    const filt_t *LSo;
} resto_ctx;

static int ls_orig_ok(const filt_t *L, double ph, double th) {
    /* IsAcceptableToCurrentFilter && IsAcceptableToCurrentIterate(called_from_restoration = true) */
    if (!isfinite(ph) || !isfinite(th)) return 0;
    if (!(ls_le(th, (1.0 - 1e-5) * L->rth, L->rth) || ls_le(ph - L->rph, -1e-8 * L->rth, L->rph))) return 0;
    for (int j = 0; j < L->nf; j++)
        if (!(ph <= L->fph[j] || th <= L->fth[j])) return 0;
    return 1;
}

static void fst_init(fst_t *F, double mu, size_t nit) {
    memset(F, 0, sizeof *F);
    F->mu = mu;
    F->LS.theta_max = -1.0;
    F->wd_it = dal(nit);
    F->wd_dir = dal(nit);
}
static void fst_free(fst_t *F) { free(F->wd_it); free(F->wd_dir); free(F->LS.fph); free(F->LS.fth); }

typedef struct {
    int n_ls_fail, n_ic, n_soc;
    double E0, cviol;
    double ts[5];
    size_t nit;
} fcount_t;

static int ipm_filter(ws_t *S, fst_t *F, int *it, fcount_t *C, const resto_ctx *R);

/* TrySoftRestoStep: the full step min(alpha_primal, alpha_dual) for primal and dual variables, accepted if
 * the original criteria accept it (then the soft phase ends) or it reduces the primal-dual system error by
 * soft_resto_pderror_reduction_factor = 0.9999.  On success the iterate is updated in place. */
static int soft_resto_step(ws_t *S, fst_t *F, double ap, double az, int *satisfies, fcount_t *C) {
    const double a = fmin(ap, az), mu = F->mu;
    double ph, th;
    int ok;
    *satisfies = 0;
    trial_point(S, a);
    merit_parts(S, S->tx, S->tu, S->ts, mu, &ph, &th, &ok, NULL, NULL, NULL);
    if (ls_acceptable(&F->LS, 0.0, ph, th, ok)) {
        *satisfies = 1;
        update_f(S, a, a, mu);
        return 1;
    }
    if (!ok) return 0;
    errs_t E0;
    opt_error_f(S, mu, &E0);
    const double pd0 = E0.s1 / E0.n1;
    double *buf = dal(C->nit);
    copy_arrays(S, iter_arrays, buf, 1);
    update_f(S, a, a, mu);
    eval_all(S, C->ts);
    errs_t E1;
    opt_error_f(S, mu, &E1);
    const double pd1 = E1.s1 / E1.n1;
    if (S->O->verbose) fprintf(stderr, "   soft resto a %.3e pderr %.6e -> %.6e\n", a, pd0, pd1);
    if (pd1 <= 0.9999 * pd0) { free(buf); return 1; }
    copy_arrays(S, iter_arrays, buf, 0);
    eval_all(S, C->ts);
    free(buf);
    return 0;
}

/* MinC_1NrmRestorationPhase::PerformRestoration: set up the restoration problem at the current point,
 * solve it with the same algorithm until the original filter accepts its iterate with theta reduced to
 * 0.9 theta_R, then return to the original problem with y = 0 (constr_mult_reset_threshold = 0) and the
 * bound multipliers reset to 1 if any exceeds bound_mult_reset_threshold = 1000. */
static int resto_phase(ws_t *S, fst_t *Fm, double thc, int *it, fcount_t *C) {
    const int N = S->N, nx = S->nx, nu = S->nu, ni = S->ni, ne = S->ne;
    const double rho = 1000.0;
    const int ric_save = S->ric;
    double cmax = 0;
    for (int r = 0; r < S->NR; r++)
        if (row_on(S, r)) {
            const int nd = N * nx, nI = N * ni;
            const double c = r < nd ? S->rdyn[r] : (r < nd + nI ? S->rin[r - nd] : S->req[r - nd - nI]);
            cmax = fmax(cmax, fabs(c));
        }
    const double mu_r = fmax(Fm->mu, cmax);
    for (int r = 0; r < S->NR; r++) {
        if (!row_el(S, r)) { S->pr[r] = S->nr[r] = 1.0; S->zp[r] = S->zn[r] = 0.0; continue; }
        const int nd = N * nx, nI = N * ni;
        const double c = r < nd ? S->rdyn[r] : (r < nd + nI ? S->rin[r - nd] : S->req[r - nd - nI]);
        const double a = (mu_r - rho * c) / (2.0 * rho);
        S->nr[r] = a + sqrt(a * a + mu_r * c / (2.0 * rho));
        S->pr[r] = c + S->nr[r];
        S->zp[r] = mu_r / S->pr[r];
        S->zn[r] = mu_r / S->nr[r];
    }
    for (int k = 0; k <= N; k++)
        for (int j = 0; j < nx; j++) {
            const int i = k * nx + j;
            S->wR[i] = S->x[i];
            S->dR[i] = 1.0 / fmax(1.0, S->x[i] * S->x[i]);
        }
    for (int i = 0; i < N * nu; i++) {
        const int o = (N + 1) * nx + i;
        S->wR[o] = S->u[i];
        S->dR[o] = 1.0 / fmax(1.0, S->u[i] * S->u[i]);
    }
    /* bound multipliers of the original variables capped at rho */
    double *zs[] = {S->zxL, S->zxU, S->zuL, S->zuU, S->vL, S->vU};
    const size_t zl[] = {(size_t)(N + 1) * nx, (size_t)(N + 1) * nx, (size_t)N * nu, (size_t)N * nu, (size_t)N * ni,
                         (size_t)N * ni};
    for (int a = 0; a < 6; a++)
        for (size_t i = 0; i < zl[a]; i++) zs[a][i] = fmin(zs[a][i], rho);
    S->resto = 1; S->objw = 0.0; S->rho_r = rho; S->zeta = sqrt(mu_r);
    if (S->O->riccati < 2) S->ric = 0;
    eval_all(S, C->ts);
    ls_mults(S);
    fst_t Fr;
    fst_init(&Fr, mu_r, C->nit);
    resto_ctx R = {Fm->mu, thc, &Fm->LS};
    if (S->O->verbose)
        fprintf(stderr, "   ---- restoration phase: theta_R %.4e mu_R %.3e ----\n", thc, mu_r);
    const int st = ipm_filter(S, &Fr, it, C, &R);
    fst_free(&Fr);
    S->resto = 0; S->objw = 1.0; S->ric = ric_save;
    if (S->O->verbose) fprintf(stderr, "   ---- restoration phase end: status %d ----\n", st);
    if (st != 0) return st;
    memset(S->lam, 0, (size_t)N * nx * sizeof(double));
    memset(S->yi, 0, (size_t)N * ni * sizeof(double));
    memset(S->ye, 0, (size_t)N * ne * sizeof(double));
    double zmax = 0;
    for (int a = 0; a < 6; a++)
        for (size_t i = 0; i < zl[a]; i++) zmax = fmax(zmax, zs[a][i]);
    if (zmax > 1e3)
        for (int a = 0; a < 6; a++)
            for (size_t i = 0; i < zl[a]; i++)
                if (zs[a][i] > 0.0) zs[a][i] = 1.0;
    return 0;
}

/* IpoptAlgorithm::Optimize in filter mode: the main problem (R == NULL) or the restoration problem.
 * Returns the device's status codes (csrc/gipm.hip GS_*): 0 converged (resto: the original filter accepted),
 * 1 max_iter, 3 inertia correction failed, 4 restoration failure (the restoration problem's line search failed:
 * IPOPT's RESTORATION_FAILURE), 5 the restoration converged to a point of local infeasibility (IPOPT's
 * LOCAL_INFEASIBILITY). */
static int ipm_filter(ws_t *S, fst_t *F, int *it, fcount_t *C, const resto_ctx *R) {
    const mfg_opts *O = S->O;
    const double kappa_eps = 10.0, kappa_mu = 0.2, theta_mu = 1.5, tau_min = 0.99;
    const double mu_min = O->tol / (kappa_eps + 1.0);
    for (; *it <= O->max_iter; (*it)++) {
        eval_all(S, C->ts);
        errs_t E;
        opt_error_f(S, F->mu, &E);
        const double E0 = fmax(fmax(E.dinf / E.sd, E.pinf), E.cinf0 / E.sc);
        double Emu = fmax(fmax(E.dinf / E.sd, E.pinf), E.cinfm / E.sc);
        if (O->verbose) {
            double fo = 0;
            for (int k = 0; k < S->N; k++) fo += S->l[k];
            fprintf(stderr, "%sit %3d f %+.10e dinf %.2e pinf %.2e compl %.2e mu %.1e\n", R ? "r" : "", *it, fo,
                    E.dinf, E.pinf, E.cinf0, F->mu);
        }
        if (!R) {
            C->E0 = E0; C->cviol = E.pinf;
            if (E0 <= O->tol && E.pinf <= O->constr_viol_tol) return 0;
        } else {
            double ph, th;
            int ok;
            merit_parts(S, S->x, S->u, S->s, R->mu_orig, &ph, &th, &ok, NULL, NULL, NULL);
            if (O->verbose) fprintf(stderr, "   orig theta %.4e (resto start %.4e) phi %.8e\n", th, R->th_R, ph);
            if (ok && th <= 0.9 * R->th_R && ls_orig_ok(R->LSo, ph, th)) return 0;
            if (E0 <= O->tol) return 5;
        }
        if (*it == O->max_iter) return 1;
        while (Emu <= kappa_eps * F->mu && F->mu > mu_min) {
            const double mnew = fmax(mu_min, fmin(kappa_mu * F->mu, pow(F->mu, theta_mu)));
            if (mnew >= F->mu) break;
            F->mu = mnew;
            F->LS.nf = 0;  /* MonotoneMuUpdate resets the line search's filter on every barrier update */
            if (S->resto) S->zeta = sqrt(F->mu);
            errs_t E2;
            opt_error_f(S, F->mu, &E2);
            Emu = fmax(fmax(E2.dinf / E2.sd, E2.pinf), E2.cinfm / E2.sc);
        }
        const double mu = F->mu, tau_fb = fmax(tau_min, 1.0 - mu);
        barrier_f(S, mu);
        if (!factor_f(S, mu, &F->ic_last, &C->n_ic, C->ts)) return 3;
        double t_ph = wall_s();
        direction_f(S, mu, S->rdyn, S->rin, S->req);
        C->ts[2] += wall_s() - t_ph;
        double ap, az;
        ftb(S, tau_fb, &ap, &az);
        /* ---- FindAcceptableTrialPoint ---- */
        double phc, thc, gdc, pHp_unused;
        int okc;
        merit_parts_e(S, S->x, S->u, S->s, S->resto ? S->pr : NULL, S->resto ? S->nr : NULL, mu, &phc, &thc, &okc, NULL,
                      NULL, NULL);
        direction_model(S, &gdc, &pHp_unused);
        if (F->LS.theta_max < 0.0) {
            F->LS.theta_max = 1e4 * fmax(1.0, thc);
            F->LS.theta_min = 1e-4 * fmax(1.0, thc);
        }
        double alpha = ap, atest = ap, pht = 0, tht = 0;
        int accepted = 0, soc_used = 0, n_steps = 0, wd_step = 0, done = 0;
        if (F->in_soft) {  /* soft restoration phase: at most max_soft_resto_iters = 10 iterations */
            F->LS.rph = phc; F->LS.rth = thc; F->LS.rgd = gdc;
            int sat = 0;
            if (++F->soft_cnt <= 10 && soft_resto_step(S, F, ap, az, &sat, C)) {
                if (sat) { F->in_soft = 0; F->soft_cnt = 0; }
                F->n_soft++;
                if (O->verbose) fprintf(stderr, "   soft resto step (%s)\n", sat ? "S" : "s");
                continue;
            }
            F->in_soft = 0;
            if (R) return 4;
            F->n_resto++;
            const int st = resto_phase(S, F, thc, it, C);
            if (st) return st;
            F->in_wd = 0; F->wd_short = 0;
            continue;
        }
        if (!F->in_wd && F->wd_short >= 10) {  /* StartWatchDog */
            F->in_wd = 1; F->wd_trial = 0; F->n_wd++;
            F->wd_ph = phc; F->wd_th = thc; F->wd_gd = gdc; F->wd_atest = ap;
            copy_arrays(S, iter_arrays, F->wd_it, 1);
            copy_arrays(S, dir_arrays, F->wd_dir, 1);
        }
        F->LS.rph = F->in_wd ? F->wd_ph : phc;
        F->LS.rth = F->in_wd ? F->wd_th : thc;
        F->LS.rgd = F->in_wd ? F->wd_gd : gdc;
        accepted = filter_backtrack(S, &F->LS, mu, tau_fb, ap, thc, 0, F->in_wd, F->wd_atest, &alpha, &az, &atest,
                                    &n_steps, &soc_used, &pht, &tht, C->ts);
        if (F->in_wd) {
            if (accepted) F->in_wd = 0;
            else if (++F->wd_trial > 3) {  /* StopWatchDog: back to the stored point, backtrack from alpha_max/2 */
                F->in_wd = 0; F->wd_short = 0;
                copy_arrays(S, iter_arrays, F->wd_it, 0);
                copy_arrays(S, dir_arrays, F->wd_dir, 0);
                eval_all(S, C->ts);  /* value caches of the stored point */
                ftb(S, tau_fb, &ap, &az);
                F->LS.rph = F->wd_ph; F->LS.rth = F->wd_th; F->LS.rgd = F->wd_gd;
                merit_parts_e(S, S->x, S->u, S->s, S->resto ? S->pr : NULL, S->resto ? S->nr : NULL, mu, &phc, &thc,
                              &okc, NULL, NULL, NULL);
                accepted = filter_backtrack(S, &F->LS, mu, tau_fb, ap, thc, 1, 0, 0.0, &alpha, &az, &atest, &n_steps,
                                            &soc_used, &pht, &tht, C->ts);
                if (!accepted) {
#ifdef _OPENMP
#pragma omp atomic
#endif
                    g_wd_fail++;
                }
            } else {  /* the watchdog's full trial step, no filter update */
                accepted = 1; wd_step = 1; alpha = ap; n_steps = 0;
            }
        }
        if (accepted && !wd_step && (!ls_ftype(&F->LS, atest) || !ls_armijo(&F->LS, atest, pht))) ls_augment(&F->LS);
        if (O->verbose)
            fprintf(stderr, "   ap %.3e az %.3e alpha %.3e acc %d soc %d steps %d wd %d/%d filt %d th %.3e ph %.10e\n",
                    ap, az, alpha, accepted, soc_used, n_steps, F->in_wd, F->wd_trial, F->LS.nf, thc, phc);
        if (!accepted) {
            C->n_ls_fail++;
            if (R) return 4;  /* no restoration inside the restoration phase */
            /* PrepareRestoPhaseStart augments the filter with the current point; then the soft restoration
             * phase is tried, and the restoration phase if its step fails */
            F->LS.rph = phc; F->LS.rth = thc; F->LS.rgd = gdc;
            ls_augment(&F->LS);
            ftb(S, tau_fb, &ap, &az);
            int sat = 0;
            if (soft_resto_step(S, F, ap, az, &sat, C)) {
                F->in_soft = !sat; F->soft_cnt = 0; F->n_soft++;
                if (O->verbose) fprintf(stderr, "   soft resto start (%s)\n", sat ? "S" : "s");
                continue;
            }
            F->n_resto++;
            const int st = resto_phase(S, F, thc, it, C);
            if (st) return st;
            F->in_wd = 0; F->wd_short = 0;
            continue;
        }
        (void)done;
        C->n_soc += soc_used;
        if (!F->in_wd) F->wd_short = (n_steps == 0) ? 0 : F->wd_short + 1;
        update_f(S, alpha, az, mu);
    }
    return 1;
}

int mfg_solve(const double *blob0, const double *blob1, const mfg_ocp *P, const mfg_opts *O, double *w_out,
              mfg_result *res) {
    models_t MM;
    memset(&MM, 0, sizeof MM);
    if (mfo_model_from_blob(blob0, &MM.M[0])) return -1;
    frame_from_arr(P->frame[0], &MM.F[0]);
    if (P->family == MFG_BOX || P->family == MFG_CENT) {
        if (!blob1 || mfo_model_from_blob(blob1, &MM.M[1])) return -1;
        frame_from_arr(P->frame[1], &MM.F[1]);
    }
    const int N = P->N, nx = P->nx, nu = P->nu, nv = nx + nu, ni = P->ni, ne = P->ne + P->nem;
    const int mb = 2 * nx + nu + ne;
    if (N < 1 || nx > GX || nu > GU || ni > GI || ne > GE || mb > BKMAX) return -2;
    ws_t SS, *S = &SS;
    memset(S, 0, sizeof *S);
    mfg_ocp PL = *P;  /* local copy: the Centauro targets are set from x_0 */
    S->P = &PL; S->O = O; S->MM = &MM;
    S->N = N; S->nx = nx; S->nu = nu; S->nv = nv; S->ni = ni; S->ne = ne; S->mb = mb; S->nes = P->ne;
    if (P->family == MFG_CENT) cent_targets(&PL, &MM);
    const double h_unused = P->h; (void)h_unused;

    /* ---- bounds (IPOPT bound_relax_factor on every non-fixed bound) ---- */
    const double br = O->bound_relax;
#define RELAX_LO(b) ((b) - br * fmax(1.0, fabs(b)))
#define RELAX_HI(b) ((b) + br * fmax(1.0, fabs(b)))
    S->ulo = dal((size_t)N * nu); S->uhi = dal((size_t)N * nu); S->ufix = (unsigned char *)calloc((size_t)N * nu, 1);
    S->clo = dal((size_t)N * ni); S->chi = dal((size_t)N * ni);
    for (int j = 0; j < nx; j++) {
        S->xlo[j] = hasb(P->x_lo[j]) ? RELAX_LO(P->x_lo[j]) : P->x_lo[j];
        S->xhi[j] = hasb(P->x_hi[j]) ? RELAX_HI(P->x_hi[j]) : P->x_hi[j];
    }
    for (int i = 0; i < N * nu; i++) {
        double lo = P->u_lo[i], hi = P->u_hi[i];
        if (hasb(lo) && lo == hi) { S->ufix[i] = 1; S->ulo[i] = S->uhi[i] = lo; continue; }
        S->ulo[i] = hasb(lo) ? RELAX_LO(lo) : lo;
        S->uhi[i] = hasb(hi) ? RELAX_HI(hi) : hi;
    }
    for (int i = 0; i < N * ni; i++) {
        double lo = P->c_lo[i], hi = P->c_hi[i];
        S->clo[i] = hasb(lo) ? RELAX_LO(lo) : lo;
        S->chi[i] = hasb(hi) ? RELAX_HI(hi) : hi;
    }
#undef RELAX_LO
#undef RELAX_HI

    /* ---- allocation ---- */
    const size_t NX1 = (size_t)(N + 1) * nx, NU = (size_t)N * nu, NI = (size_t)N * ni, NE = (size_t)N * ne;
    S->x = dal(NX1); S->u = dal(NU); S->s = dal(NI); S->lam = dal((size_t)N * nx); S->ye = dal(NE); S->yi = dal(NI);
    S->zxL = dal(NX1); S->zxU = dal(NX1); S->zuL = dal(NU); S->zuU = dal(NU); S->vL = dal(NI); S->vU = dal(NI);
    S->tx = dal(NX1); S->tu = dal(NU); S->ts = dal(NI);
    S->l = dal(N); S->gl = dal((size_t)N * nv); S->ci = dal(NI); S->Ji = dal(NI * nv); S->ce = dal(NE);
    S->Je = dal(NE * nv); S->f = dal((size_t)N * nx); S->Af = dal((size_t)N * nx * nx); S->Bf = dal((size_t)N * nx * nu);
    S->W = dal((size_t)N * nv * nv);
    S->dx = dal(NX1); S->du = dal(NU); S->ds = dal(NI); S->dlam = dal((size_t)N * nx); S->dye = dal(NE);
    S->dyi = dal(NI); S->dzxL = dal(NX1); S->dzxU = dal(NX1); S->dzuL = dal(NU); S->dzuU = dal(NU);
    S->dvL = dal(NI); S->dvU = dal(NI);
    S->Sx = dal(NX1); S->gx = dal(NX1); S->Su = dal(NU); S->gu = dal(NU); S->Ss = dal(NI); S->gs = dal(NI);
    S->wv = dal((size_t)(N + 1) * mb); S->G = dal((size_t)(N + 1) * mb * nx);
    S->Dsave = dal((size_t)(N + 1) * mb * mb);
    S->rdyn = dal((size_t)N * nx); S->rin = dal(NI); S->req = dal(NE);
    S->trdyn = dal((size_t)N * nx); S->trin = dal(NI); S->treq = dal(NE);
    S->sdyn = dal((size_t)N * nx); S->sin_ = dal(NI); S->seq = dal(NE);
    S->bk = dal(3 * NX1 + 3 * NU + 4 * NI + (size_t)N * nx + NE);
    S->ric = O->riccati;
    S->nk = nu + ne;
    if (S->ric) {
        if (S->nk > BKMAX) return -2;
        S->Pg = dal((size_t)N * nx * nx); S->Kst = dal((size_t)N * S->nk * S->nk); S->Fg = dal((size_t)N * S->nk * nx);
        S->pvg = dal((size_t)N * nx); S->kvg = dal((size_t)N * S->nk);
        S->Kpp = (int *)calloc((size_t)N * 2 * S->nk, sizeof(int));
        S->Drg = dal((size_t)N * nx); S->Jtg = dal((size_t)N * ne * nx); S->LUg = dal((size_t)N * nx * nx);
        S->LUp = (int *)calloc((size_t)N * nx, sizeof(int));
    }
    S->perm = (int *)calloc((size_t)(N + 1) * mb, sizeof(int));
    S->piv = (int *)calloc((size_t)(N + 1) * mb, sizeof(int));
    S->objw = 1.0;
    S->NR = (int)((size_t)N * nx + NI + NE);
    const size_t NIT4 = 3 * NX1 + 3 * NU + 4 * NI + (size_t)N * nx + NE + 4 * (size_t)S->NR;
    if (O->filter) {  /* restoration-phase arrays; direction / iterate copies with the elastic variables */
        double **ra[] = {&S->pr, &S->nr, &S->zp, &S->zn, &S->dpr, &S->dnr, &S->dzp, &S->dzn, &S->tpr, &S->tnr,
                         &S->Sp, &S->Sn, &S->gp, &S->gn, &S->rowr};
        for (size_t i = 0; i < sizeof ra / sizeof ra[0]; i++) *ra[i] = dal(S->NR);
        S->wR = dal(NX1 + NU); S->dR = dal(NX1 + NU);
        free(S->bk);
        S->bk = dal(NIT4);
    }

    /* ---- initial point (IPOPT: x0 = 0 or the held state, bound_push / bound_frac = 1e-2) ---- */
    for (int k = 0; k <= N; k++)
        for (int j = 0; j < nx; j++) {
            double v = (k == 0 || !O->init_zero) ? P->x0[j] : 0.0;
            S->x[k * nx + j] = (k == 0) ? P->x0[j] : push_into(v, S->xlo[j], S->xhi[j]);
        }
    for (int k = 0; k < N; k++)
        for (int j = 0; j < nu; j++) {
            const int i = k * nu + j;
            double v = O->u_init ? O->u_init[j] : ((j >= P->force_from) ? O->F_init : 0.0);
            S->u[i] = S->ufix[i] ? S->ulo[i] : push_into(v, S->ulo[i], S->uhi[i]);
        }
    const int warm = O->warm_start && O->w0;
    const double kp = warm ? 1e-3 : 1e-2;  /* (warm_start_)bound_push = _frac */
    if (O->w0) {
        const int st = nu + nx;
        for (int k = 0; k < N; k++) {
            const double *wk = O->w0 + nx + (size_t)k * st;
            for (int j = 0; j < nu; j++) {
                const int i = k * nu + j;
                if (!S->ufix[i]) S->u[i] = push_into_k(wk[j], S->ulo[i], S->uhi[i], kp, kp);
            }
            for (int j = 0; j < nx; j++)
                S->x[(k + 1) * nx + j] = push_into_k(wk[nu + j], S->xlo[j], S->xhi[j], kp, kp);
        }
    }
    for (int k = 0; k < N; k++) {
        double l, ci[GI], ce[GE], f[GX];
        eval_values(S, k, S->x + k * nx, S->u + k * nu, &l, ci, ce, f);
        for (int r = 0; r < ni; r++)
            S->s[k * ni + r] = push_into_k(ci[r], S->clo[k * ni + r], S->chi[k * ni + r], kp, kp);
    }
    /* bound multipliers: bound_mult_init_val = 1 cold; warm: max(given (0 when none),
     * warm_start_mult_bound_push = 1e-3) */
    const double z0 = warm ? 1e-3 : 1.0;
    for (int k = 0; k <= N; k++)
        for (int j = 0; j < nx; j++) {
            S->zxL[k * nx + j] = (k > 0 && hasb(S->xlo[j])) ? z0 : 0.0;
            S->zxU[k * nx + j] = (k > 0 && hasb(S->xhi[j])) ? z0 : 0.0;
        }
    for (int i = 0; i < N * nu; i++) {
        S->zuL[i] = (!S->ufix[i] && hasb(S->ulo[i])) ? z0 : 0.0;
        S->zuU[i] = (!S->ufix[i] && hasb(S->uhi[i])) ? z0 : 0.0;
    }
    for (int i = 0; i < N * ni; i++) {
        S->vL[i] = hasb(S->clo[i]) ? z0 : 0.0;
        S->vU[i] = hasb(S->chi[i]) ? z0 : 0.0;
    }
    if (warm && O->dual_in) {
        const double *o = O->dual_in;
        double *dst[] = {S->lam, S->yi, S->ye, S->zxL, S->zxU, S->zuL, S->zuU, S->vL, S->vU};
        const size_t len[] = {(size_t)N * nx, NI, NE, NX1, NX1, NU, NU, NI, NI};
        for (int a = 0; a < 9; a++) {
            for (size_t i = 0; i < len[a]; i++)
                dst[a][i] = a < 3 ? o[i] : (dst[a][i] > 0.0 ? fmax(o[i], 1e-3) : 0.0);
            o += len[a];
        }
    }

    const double kappa_eps = 10.0, kappa_mu = 0.2, theta_mu = 1.5, tau_min = 0.99, s_max = 100.0;
    const double kappa_sigma = 1e10, eta = 1e-4, rho = 0.1;
    double mu = O->mu_init, nu_pen = 0.0, reg_last = 0.0;
    int reg_tier = 0, status = 1, it = 0, n_ls_fail = 0, n_ic = 0, consecutive_fail = 0, n_soc = 0;
    double E0 = INFINITY, cviol = INFINITY;
    const int has_tier1 = P->tier1_to > P->tier1_from;

    double ts[5] = {0, 0, 0, 0, 0}, t_solve0 = wall_s(), t_ph;
    if (O->kkt_at) {  /* the KKT measures at the given point (mfg_opts.kkt_at) */
        const int st = nu + nx;
        for (int k = 0; k < N; k++) {
            const double *wk = O->w0 + nx + (size_t)k * st;
            for (int j = 0; j < nu; j++)
                if (!S->ufix[k * nu + j]) S->u[k * nu + j] = wk[j];
            for (int j = 0; j < nx; j++) S->x[(k + 1) * nx + j] = wk[nu + j];
        }
        memcpy(S->s, O->s_in, NI * sizeof(double));
        const double *o = O->dual_in;
        double *dst[] = {S->lam, S->yi, S->ye, S->zxL, S->zxU, S->zuL, S->zuU, S->vL, S->vU};
        const size_t len[] = {(size_t)N * nx, NI, NE, NX1, NX1, NU, NU, NI, NI};
        for (int a = 0; a < 9; a++) {
            memcpy(dst[a], o, len[a] * sizeof(double));
            o += len[a];
        }
        eval_all(S, ts);
        errs_t Ek;
        opt_error_f(S, 0.0, &Ek);
        double fo = 0.0;
        for (int k = 0; k < N; k++) fo += S->l[k];
        double *ko = O->kkt_out;
        ko[0] = fmax(fmax(Ek.dinf / Ek.sd, Ek.pinf), Ek.cinf0 / Ek.sc);
        ko[1] = Ek.dinf; ko[2] = Ek.pinf; ko[3] = Ek.cinf0; ko[4] = Ek.sd; ko[5] = Ek.sc; ko[6] = fo;
        status = 0; it = 0; E0 = ko[0]; cviol = Ek.pinf;
    } else if (O->filter) {  /* IPOPT's globalisation (mfg_opts.filter) */
        fcount_t C;
        memset(&C, 0, sizeof C);
        C.nit = NIT4; C.E0 = INFINITY; C.cviol = INFINITY;
        fst_t F;
        fst_init(&F, O->mu_init, C.nit);
        it = 0;
        status = ipm_filter(S, &F, &it, &C, NULL);
        mu = F.mu; E0 = C.E0; cviol = C.cviol; n_ls_fail = C.n_ls_fail; n_ic = C.n_ic; n_soc = C.n_soc;
        for (int i = 0; i < 4; i++) ts[i] += C.ts[i];
        if (O->verbose)
            fprintf(stderr, "filter: watchdogs %d soft-restoration steps %d restoration phases %d\n", F.n_wd, F.n_soft,
                    F.n_resto);
        fst_free(&F);
    } else
    for (it = 0; it <= O->max_iter; it++) {
        /* ---- node derivatives ---- */
        t_ph = wall_s();
#ifdef _OPENMP
#pragma omp parallel for schedule(dynamic, 1)
#endif
        for (int k = 0; k < N; k++) eval_derivs(S, k);
        ts[0] += wall_s() - t_ph;

        /* ---- optimality error (IPOPT E_0 with s_max scaling) ---- */
        double dinf = 0, pinf = 0, cinf0 = 0, cinfm = 0, sum_mult = 0, sum_bmult = 0;
        int n_mult = 0, n_bmult = 0;
#define COMP(z, gap)                                                            \
    do {                                                                        \
        double c_ = (z) * (gap);                                                \
        cinf0 = fmax(cinf0, fabs(c_)); cinfm = fmax(cinfm, fabs(c_ - mu));      \
        sum_bmult += (z); n_bmult++;                                            \
    } while (0)
        for (int k = 1; k <= N; k++)
            for (int j = 0; j < nx; j++) {
                const int i = k * nx + j;
                double r = -S->lam[(k - 1) * nx + j];
                if (k < N) {
                    r += S->gl[k * nv + j];
                    for (int jj = 0; jj < nx; jj++) r += S->Af[(k * nx + jj) * nx + j] * S->lam[k * nx + jj];
                    for (int q = 0; q < ni; q++) r += S->Ji[((size_t)k * ni + q) * nv + j] * S->yi[k * ni + q];
                    for (int e = 0; e < ne; e++)
                        if (EQ_ON(S, k, e)) r += S->Je[((size_t)k * ne + e) * nv + j] * S->ye[k * ne + e];
                }
                r += -S->zxL[i] + S->zxU[i];
                dinf = fmax(dinf, fabs(r));
                if (hasb(S->xlo[j])) COMP(S->zxL[i], S->x[i] - S->xlo[j]);
                if (hasb(S->xhi[j])) COMP(S->zxU[i], S->xhi[j] - S->x[i]);
            }
        for (int k = 0; k < N; k++) {
            for (int j = 0; j < nu; j++) {
                const int i = k * nu + j;
                if (S->ufix[i]) continue;
                double r = S->gl[k * nv + nx + j];
                for (int jj = 0; jj < nx; jj++) r += S->Bf[(k * nx + jj) * nu + j] * S->lam[k * nx + jj];
                for (int q = 0; q < ni; q++) r += S->Ji[((size_t)k * ni + q) * nv + nx + j] * S->yi[k * ni + q];
                for (int e = S->nes; e < ne; e++) r += S->Je[((size_t)k * ne + e) * nv + nx + j] * S->ye[k * ne + e];
                r += -S->zuL[i] + S->zuU[i];
                dinf = fmax(dinf, fabs(r));
                if (hasb(S->ulo[i])) COMP(S->zuL[i], S->u[i] - S->ulo[i]);
                if (hasb(S->uhi[i])) COMP(S->zuU[i], S->uhi[i] - S->u[i]);
            }
            for (int q = 0; q < ni; q++) {
                const int i = k * ni + q;
                if (!CACT(S, k, q)) continue;
                double r = -S->yi[i] - S->vL[i] + S->vU[i];
                dinf = fmax(dinf, fabs(r));
                if (hasb(S->clo[i])) COMP(S->vL[i], S->s[i] - S->clo[i]);
                if (hasb(S->chi[i])) COMP(S->vU[i], S->chi[i] - S->s[i]);
                pinf = fmax(pinf, fabs(S->ci[i] - S->s[i]));
                sum_mult += fabs(S->yi[i]); n_mult++;
            }
            for (int j = 0; j < nx; j++) {
                pinf = fmax(pinf, fabs(S->f[k * nx + j] - S->x[(k + 1) * nx + j]));
                sum_mult += fabs(S->lam[k * nx + j]); n_mult++;
            }
            for (int e = 0; e < ne; e++)
                if (EQ_ON(S, k, e)) {
                    pinf = fmax(pinf, fabs(S->ce[k * ne + e]));
                    sum_mult += fabs(S->ye[k * ne + e]); n_mult++;
                }
        }
#undef COMP
        const double sd = fmax(s_max, (sum_mult + sum_bmult) / fmax(1, n_mult + n_bmult)) / s_max;
        const double sc = fmax(s_max, sum_bmult / fmax(1, n_bmult)) / s_max;
        E0 = fmax(fmax(dinf / sd, pinf), cinf0 / sc);
        cviol = pinf;
        double Emu = fmax(fmax(dinf / sd, pinf), cinfm / sc);
        if (O->verbose) {
            double fo = 0;
            for (int k = 0; k < N; k++) fo += S->l[k];
            fprintf(stderr, "it %3d f %+.10e dinf %.2e pinf %.2e compl %.2e mu %.1e nu %.2e\n", it, fo, dinf, pinf,
                    cinf0, mu, nu_pen);
        }
        if (E0 <= O->tol && cviol <= O->constr_viol_tol) { status = 0; break; }
        if (it == O->max_iter) { status = 1; break; }
        while (Emu <= kappa_eps * mu && mu > O->tol / 10.0) {
            double mnew = fmax(O->tol / 10.0, fmin(kappa_mu * mu, pow(mu, theta_mu)));
            if (mnew >= mu) break;
            mu = mnew;
            cinfm = 0;
            for (int k = 1; k <= N; k++)
                for (int j = 0; j < nx; j++) {
                    const int i = k * nx + j;
                    if (hasb(S->xlo[j])) cinfm = fmax(cinfm, fabs(S->zxL[i] * (S->x[i] - S->xlo[j]) - mu));
                    if (hasb(S->xhi[j])) cinfm = fmax(cinfm, fabs(S->zxU[i] * (S->xhi[j] - S->x[i]) - mu));
                }
            for (int i = 0; i < N * nu; i++) {
                if (S->ufix[i]) continue;
                if (hasb(S->ulo[i])) cinfm = fmax(cinfm, fabs(S->zuL[i] * (S->u[i] - S->ulo[i]) - mu));
                if (hasb(S->uhi[i])) cinfm = fmax(cinfm, fabs(S->zuU[i] * (S->uhi[i] - S->u[i]) - mu));
            }
            for (int i = 0; i < N * ni; i++) {
                if (hasb(S->clo[i])) cinfm = fmax(cinfm, fabs(S->vL[i] * (S->s[i] - S->clo[i]) - mu));
                if (hasb(S->chi[i])) cinfm = fmax(cinfm, fabs(S->vU[i] * (S->chi[i] - S->s[i]) - mu));
            }
            Emu = fmax(fmax(dinf / sd, pinf), cinfm / sc);
        }
        const double tau_fb = fmax(tau_min, 1.0 - mu);

        /* ---- barrier Sigma and gradients ---- */
#define SIGG(Sg, gg, z_l, z_u, v, lo, hi)                                                  \
    do {                                                                                   \
        Sg = 0; gg = 0;                                                                    \
        if (hasb(lo)) { Sg += (z_l) / ((v) - (lo)); gg -= mu / ((v) - (lo)); }             \
        if (hasb(hi)) { Sg += (z_u) / ((hi) - (v)); gg += mu / ((hi) - (v)); }             \
    } while (0)
        for (int k = 0; k <= N; k++)
            for (int j = 0; j < nx; j++) {
                const int i = k * nx + j;
                if (k == 0) { S->Sx[i] = S->gx[i] = 0; continue; }
                SIGG(S->Sx[i], S->gx[i], S->zxL[i], S->zxU[i], S->x[i], S->xlo[j], S->xhi[j]);
            }
        for (int i = 0; i < N * nu; i++) {
            if (S->ufix[i]) { S->Su[i] = S->gu[i] = 0; continue; }
            SIGG(S->Su[i], S->gu[i], S->zuL[i], S->zuU[i], S->u[i], S->ulo[i], S->uhi[i]);
        }
        for (int i = 0; i < N * ni; i++) SIGG(S->Ss[i], S->gs[i], S->vL[i], S->vU[i], S->s[i], S->clo[i], S->chi[i]);
#undef SIGG

        /* ---- inertia-corrected block factorisation ---- */
        /* delta_c = 1e-8 mu^(1/4) (IPOPT's perturbation of a singular KKT) from the first attempt when
         * the equality rows are rank deficient by construction (Centauro moment rows at the fixed
         * node 0: (p_L - p_R) x (F_L - F_R) has rank 2 in F), else only after a zero pivot */
        double dw = 0.0, dc = P->dc_always ? 1e-8 * pow(mu, 0.25) : 0.0, d1 = 0.0;
        int tier = reg_tier, step_no = 0, factor_ok = 0, tries;
        double reg = (reg_tier == 0) ? 0.0 : reg_last / 3.0;
        if (reg_tier != 0 && reg < 1e-8) { tier = 0; reg = 0.0; }
        if (tier == 1) d1 = reg; else if (tier == 2) dw = reg;
        for (tries = 0; tries < 60; tries++) {
            t_ph = wall_s();
            const int fr = S->ric ? kkt_factor_ric(S, dw, dc, d1) : kkt_factor(S, dw, dc, d1);
            ts[1] += wall_s() - t_ph;
            if (fr == 0) { factor_ok = 1; break; }
            if (fr == 2 && dc == 0.0) { dc = 1e-8 * pow(mu, 0.25); continue; }
            n_ic++;
            step_no++;
            if (tier == 0) {
                tier = has_tier1 ? 1 : 2;
                reg = 1e-4;
            } else if (step_no == 1 && reg_tier == tier && reg < reg_last) {
                reg = reg_last;
            } else {
                reg *= 8.0;
                if (tier == 1 && reg > 1e6) { tier = 2; reg = 1e-4; }
            }
            if (reg > 1e40) break;
            d1 = (tier == 1) ? reg : 0.0;
            dw = (tier == 2) ? reg : 0.0;
        }
        if (!factor_ok) { status = 3; break; }
        reg_tier = tier;
        reg_last = reg;
        if (O->verbose > 1) fprintf(stderr, "   d1 %.2e dw %.2e dc %.2e tries %d\n", d1, dw, dc, tries);

        /* ---- Newton direction for the residuals of the current point ---- */
        residuals_cached(S, S->rdyn, S->rin, S->req);
        t_ph = wall_s();
        (S->ric ? kkt_direction_ric : kkt_direction)(S, mu, S->rdyn, S->rin, S->req);
        ts[2] += wall_s() - t_ph;
        double ap, az;
        ftb(S, tau_fb, &ap, &az);
        if (O->verbose > 2) ftb_report(S, tau_fb);

        /* ---- l1-merit backtracking line search with second-order corrections ---- */
        double phi0, th0;
        int ok0;
        merit_parts(S, S->x, S->u, S->s, mu, &phi0, &th0, &ok0, NULL, NULL, NULL);
        double gdot = 0, pHp = 0;
        direction_model(S, &gdot, &pHp);
        if (th0 > 1e-300) {
            double nreq = (gdot + 0.5 * fmax(pHp, 0.0)) / ((1.0 - rho) * th0);
            if (nu_pen < nreq) nu_pen = nreq + 1.0;
        }
        const double Dphi = gdot - nu_pen * th0, m0 = phi0 + nu_pen * th0;
        const double slack_m = 10.0 * 2.220446049250313e-16 * fabs(m0);
        double alpha = ap;
        int accepted = 0, soc_used = 0;
        for (int ls = 0; ls < 40; ls++) {
            double ph, th;
            int okk;
            trial_point(S, alpha);
            t_ph = wall_s();
            merit_parts(S, S->tx, S->tu, S->ts, mu, &ph, &th, &okk, S->trdyn, S->trin, S->treq);
            ts[3] += wall_s() - t_ph;
            const double mt = ph + nu_pen * th;
            if (okk && isfinite(mt) && mt - m0 <= eta * alpha * fmin(Dphi, 0.0) + slack_m) { accepted = 1; break; }
            /* IPOPT A-5.5..A-5.9: second-order corrections after the first trial step when it raised the
             * infeasibility: c_soc = alpha c(x) + c(x_trial), same factorisation, up to O->max_soc tries */
            if (ls == 0 && O->max_soc > 0 && (!okk || th >= th0)) {
                double th_old = th, a_soc = alpha;
                for (size_t i = 0; i < (size_t)N * nx; i++) S->sdyn[i] = alpha * S->rdyn[i] + S->trdyn[i];
                for (size_t i = 0; i < (size_t)N * ni; i++) S->sin_[i] = alpha * S->rin[i] + S->trin[i];
                for (size_t i = 0; i < (size_t)N * ne; i++) S->seq[i] = alpha * S->req[i] + S->treq[i];
                for (int p = 0; p < O->max_soc; p++) {
                    save_direction(S);
                    t_ph = wall_s();
                    (S->ric ? kkt_direction_ric : kkt_direction)(S, mu, S->sdyn, S->sin_, S->seq);
                    ts[2] += wall_s() - t_ph;
                    double aps, azs;
                    ftb(S, tau_fb, &aps, &azs);
                    trial_point(S, aps);
                    double phs, ths;
                    int oks;
                    t_ph = wall_s();
                    merit_parts(S, S->tx, S->tu, S->ts, mu, &phs, &ths, &oks, S->trdyn, S->trin, S->treq);
                    ts[3] += wall_s() - t_ph;
                    const double ms = phs + nu_pen * ths;
                    if (O->verbose > 1)
                        fprintf(stderr, "      soc %d a %.3e th %.3e (th0 %.3e) m %.10e (m0 %.10e)\n", p, aps, ths, th0, ms, m0);
                    if (oks && isfinite(ms) && ms - m0 <= eta * a_soc * fmin(Dphi, 0.0) + slack_m) {
                        accepted = 1; soc_used = 1; alpha = aps; az = azs;
                        break;
                    }
                    restore_direction(S);
                    if (!oks || ths > 0.99 * th_old) break;
                    th_old = ths;
                    for (size_t i = 0; i < (size_t)N * nx; i++) S->sdyn[i] = aps * S->sdyn[i] + S->trdyn[i];
                    for (size_t i = 0; i < (size_t)N * ni; i++) S->sin_[i] = aps * S->sin_[i] + S->trin[i];
                    for (size_t i = 0; i < (size_t)N * ne; i++) S->seq[i] = aps * S->seq[i] + S->treq[i];
                }
                if (accepted) break;
            }
            alpha *= 0.5;
        }
        if (O->verbose) fprintf(stderr, "   ap %.3e az %.3e alpha %.3e acc %d soc %d\n", ap, az, alpha, accepted, soc_used);
        if (!accepted) {
            n_ls_fail++;
            if (++consecutive_fail >= 5) { status = 2; break; }
        } else consecutive_fail = 0;
        n_soc += soc_used;
        /* ---- update ---- */
        for (size_t i = 0; i < NX1; i++) S->x[i] += alpha * S->dx[i];
        for (size_t i = 0; i < NU; i++) S->u[i] += alpha * S->du[i];
        for (size_t i = 0; i < NI; i++) { S->s[i] += alpha * S->ds[i]; S->yi[i] += alpha * S->dyi[i]; }
        for (int i = 0; i < N * nx; i++) S->lam[i] += alpha * S->dlam[i];
        for (size_t i = 0; i < NE; i++) S->ye[i] += alpha * S->dye[i];
#define ZUPD(z, dz, slack)                                                                    \
    do {                                                                                      \
        double zz = (z) + az * (dz), sl = (slack);                                            \
        (z) = fmax(fmin(zz, kappa_sigma * mu / sl), mu / (kappa_sigma * sl));                  \
    } while (0)
        for (int k = 1; k <= N; k++)
            for (int j = 0; j < nx; j++) {
                const int i = k * nx + j;
                if (hasb(S->xlo[j])) ZUPD(S->zxL[i], S->dzxL[i], S->x[i] - S->xlo[j]);
                if (hasb(S->xhi[j])) ZUPD(S->zxU[i], S->dzxU[i], S->xhi[j] - S->x[i]);
            }
        for (int i = 0; i < N * nu; i++) {
            if (S->ufix[i]) continue;
            if (hasb(S->ulo[i])) ZUPD(S->zuL[i], S->dzuL[i], S->u[i] - S->ulo[i]);
            if (hasb(S->uhi[i])) ZUPD(S->zuU[i], S->dzuU[i], S->uhi[i] - S->u[i]);
        }
        for (int i = 0; i < N * ni; i++) {
            if (hasb(S->clo[i])) ZUPD(S->vL[i], S->dvL[i], S->s[i] - S->clo[i]);
            if (hasb(S->chi[i])) ZUPD(S->vU[i], S->dvU[i], S->chi[i] - S->s[i]);
        }
#undef ZUPD
    }
    ts[4] = wall_s() - t_solve0;
    for (int i = 0; i < 5; i++) {
#ifdef _OPENMP
#pragma omp atomic
#endif
        g_tsplit[i] += ts[i];
    }
    /* ---- output in the reference layout [x_0 | (u_k, x_{k+1}) x N] ---- */
    if (w_out) {
        double *o = w_out;
        memcpy(o, S->x, nx * sizeof(double));
        o += nx;
        for (int k = 0; k < N; k++) {
            memcpy(o, S->u + k * nu, nu * sizeof(double));
            o += nu;
            memcpy(o, S->x + (k + 1) * nx, nx * sizeof(double));
            o += nx;
        }
    }
    if (res) {
        double fo = 0;
        for (int k = 0; k < N; k++) {
            double l, ci[GI], ce[GE], f[GX];
            eval_values(S, k, S->x + k * nx, S->u + k * nu, &l, ci, ce, f);
            fo += l;
        }
        res->status = status; res->iter = it; res->kkt = E0; res->cviol = cviol; res->obj = fo; res->mu = mu;
        res->n_ls_fail = n_ls_fail; res->n_inertia_fix = n_ic;
    }
    if (O->verbose) fprintf(stderr, "second-order corrections accepted: %d\n", n_soc);
    if (O->s_out) memcpy(O->s_out, S->s, NI * sizeof(double));
    if (O->dual_out) {
        double *o = O->dual_out;
        const double *src[] = {S->lam, S->yi, S->ye, S->zxL, S->zxU, S->zuL, S->zuU, S->vL, S->vU};
        const size_t len[] = {(size_t)N * nx, NI, NE, NX1, NX1, NU, NU, NI, NI};
        for (int a = 0; a < 9; a++) { memcpy(o, src[a], len[a] * sizeof(double)); o += len[a]; }
        *o = mu;
    }
    double **pp[] = {&S->ulo, &S->uhi, &S->clo, &S->chi, &S->x, &S->u, &S->s, &S->lam, &S->ye, &S->yi, &S->zxL,
                     &S->zxU, &S->zuL, &S->zuU, &S->vL, &S->vU, &S->tx, &S->tu, &S->ts, &S->l, &S->gl, &S->ci,
                     &S->Ji, &S->ce, &S->Je, &S->f, &S->Af, &S->Bf, &S->W, &S->dx, &S->du, &S->ds, &S->dlam,
                     &S->dye, &S->dyi, &S->dzxL, &S->dzxU, &S->dzuL, &S->dzuU, &S->dvL, &S->dvU, &S->Sx, &S->gx,
                     &S->Su, &S->gu, &S->Ss, &S->gs, &S->wv, &S->G, &S->Dsave, &S->rdyn, &S->rin, &S->req,
                     &S->trdyn, &S->trin, &S->treq, &S->sdyn, &S->sin_, &S->seq, &S->bk};
    for (size_t i = 0; i < sizeof pp / sizeof pp[0]; i++) free(*pp[i]);
    free(S->ufix); free(S->perm); free(S->piv);
    if (S->ric) {
        free(S->Pg); free(S->Kst); free(S->Fg); free(S->pvg); free(S->kvg); free(S->Kpp); free(S->Drg); free(S->Jtg);
        free(S->LUg); free(S->LUp);
    }
    if (O->filter) {
        double **ra[] = {&S->pr, &S->nr, &S->zp, &S->zn, &S->dpr, &S->dnr, &S->dzp, &S->dzn, &S->tpr, &S->tnr,
                         &S->Sp, &S->Sn, &S->gp, &S->gn, &S->rowr, &S->wR, &S->dR};
        for (size_t i = 0; i < sizeof ra / sizeof ra[0]; i++) free(*ra[i]);
    }
    return 0;
}

/* Node values and derivatives for tests: l, c_in, c_eq, f and their Jacobians w.r.t. [x|u]
 * (row-major), and the Hessian of l + yi.c_in + ye.c_eq + lam.f (nv x nv). */
int mfg_node_derivs(const double *blob0, const double *blob1, const mfg_ocp *P, const double *xu, const double *yi,
                    const double *ye, const double *lam, double *vals, double *jac, double *H) {
    models_t MM;
    memset(&MM, 0, sizeof MM);
    if (mfo_model_from_blob(blob0, &MM.M[0])) return -1;
    frame_from_arr(P->frame[0], &MM.F[0]);
    if (P->family == MFG_BOX || P->family == MFG_CENT) {
        if (!blob1 || mfo_model_from_blob(blob1, &MM.M[1])) return -1;
        frame_from_arr(P->frame[1], &MM.F[1]);
    }
    const int nx = P->nx, nv = P->nx + P->nu, ni = P->ni, ne = P->ne + P->nem, no = 1 + ni + ne + nx;
    for (int a = 0; a < nv; a++)
        for (int b = a; b < nv; b++) {
            hd hx[GV], hl, hci[GI], hce[GE], hf[GX];
            for (int i = 0; i < nv; i++) hx[i] = K(xu[i]);
            hx[a].b = 1.0;
            hx[b].c = 1.0;
            node_hd(P, &MM, hx, &hl, hci, hce, hf);
            double h2 = hl.d;
            for (int r = 0; r < ni; r++) h2 += yi[r] * hci[r].d;
            for (int e = 0; e < ne; e++) h2 += ye[e] * hce[e].d;
            for (int j = 0; j < nx; j++) h2 += lam[j] * hf[j].d;
            H[a * nv + b] = H[b * nv + a] = h2;
            if (a == b) {
                jac[0 * nv + a] = hl.b;
                for (int r = 0; r < ni; r++) jac[(1 + r) * nv + a] = hci[r].b;
                for (int e = 0; e < ne; e++) jac[(1 + ni + e) * nv + a] = hce[e].b;
                for (int j = 0; j < nx; j++) jac[(1 + ni + ne + j) * nv + a] = hf[j].b;
                if (a == 0) {
                    vals[0] = hl.a;
                    for (int r = 0; r < ni; r++) vals[1 + r] = hci[r].a;
                    for (int e = 0; e < ne; e++) vals[1 + ni + e] = hce[e].a;
                    for (int j = 0; j < nx; j++) vals[1 + ni + ne + j] = hf[j].a;
                }
            }
        }
    (void)no;
    return 0;
}

/* Batch of independent horizons (OpenMP over problems when nthreads > 0, nodes otherwise). */
int mfg_solve_batch(const double *blob0, const double *blob1, const mfg_ocp *P, int batch, const mfg_opts *O,
                    double *w_out, int w_stride, mfg_result *res, int nthreads) {
    int err = 0;
#ifdef _OPENMP
    if (nthreads > 0) omp_set_num_threads(nthreads);
#pragma omp parallel for schedule(dynamic, 1) reduction(| : err)
#endif
    for (int b = 0; b < batch; b++)
        err |= mfg_solve(blob0, blob1, &P[b], O, w_out ? w_out + (size_t)b * w_stride : NULL, &res[b]);
    return err;
}
