/*
 * ORACLE — test infrastructure only.  CPU restatement (plain C99, FP64) of the
 * reference's hot path.  Only tests/, __graft_entry__.smoke() and bench.py's
 * cpu_baseline leg may load it, and only as the checker / timed CPU baseline.
 * The product path (mpc_fatigue_amd, libmpcfatigue.so) never links it.
 *
 * What it restates (reference file:line):
 *   - pinocchio::rnea traced by generate_inv_dyn   src/casadi_pinocchio_bridge.hpp:57-85
 *   - framesForwardKinematics / oMf[frame]          src/casadi_pinocchio_bridge.hpp:87-117
 *   - getFrameJacobian(LOCAL_WORLD_ALIGNED)         src/casadi_pinocchio_bridge.hpp:119-153
 *   - node torque  tau = ID(q,qd,0) - J^T [F;0]     python/Pilz_6_DOF/force_optimization_pilz_6DOF.py:129-135
 *   - exponential torque envelope (fatigue)         force_optimization_pilz_6DOF.py:136-148
 *   - line constraint fk(q)[0:2] = ref              force_optimization_pilz_6DOF.py:150-156
 *   - explicit-Euler continuity                     force_optimization_pilz_6DOF.py:159-172
 *   - stage costs -F^T F / tau^T tau + 100 qd^T qd  force_optimization_pilz_6DOF.py:177,
 *                                                   python/Pilz_3_DOF/inverse_dynamics_pilz_3DOF_working.py
 *   - nlpsol('ipopt') with CasADi exact Hessians    force_optimization_pilz_6DOF.py:195-197
 *     restated as an IPOPT-style primal-dual interior-point method (Waechter &
 *     Biegler 2006: monotone mu, fraction-to-boundary, inertia correction) with
 *     an l1-merit Armijo line search; the algorithm is specified in DESIGN.md
 *     section 4 and the HIP product implements the identical iteration.
 *
 * Derivatives: exact, by hyper-dual numbers (a + b e1 + c e2 + d e1e2) run
 * through the same world-frame Newton-Euler code -- obviously correct, slow.
 * The KKT: block-tridiagonal over shooting nodes, each dense stage block
 * factorised by Bunch-Kaufman LDL^T (LAPACK dsytf2 pivoting rule, full
 * symmetric permutations); inertia = sum over blocks (Sylvester).
 */
#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

#include "hd_kin.h"

#define MV (2 * MJ + 3)       /* max node variables (q, qd, F) */
#define MB (3 * MJ + 3 + 4)   /* max stage block size */

/* ------------------------------------------------------------------ */
/* plain-double entry points (the three Functions of the bridge)       */
static void to_hd(hd *o, const double *x, int n) { for (int i = 0; i < n; i++) o[i] = K(x[i]); }

int mfo_id(const double *blob, const double *q, const double *qd, const double *qdd, double *tau) {
    mfo_model M; if (mfo_model_from_blob(blob, &M)) return -1;
    hd hq[MJ], hqd[MJ], hqdd[MJ], ht[MJ];
    to_hd(hq, q, M.n); to_hd(hqd, qd, M.n); to_hd(hqdd, qdd, M.n);
    kin_t Kn; kinematics(&M, hq, &Kn); rnea(&M, &Kn, hqd, hqdd, ht);
    for (int i = 0; i < M.n; i++) tau[i] = ht[i].a;
    return 0;
}

int mfo_fk(const double *blob, const double *frame, const double *q, double *pos, double *rot_rowmajor) {
    mfo_model M; if (mfo_model_from_blob(blob, &M)) return -1;
    mfo_frame F; frame_from_arr(frame, &F);
    hd hq[MJ], p[3], R[9];
    to_hd(hq, q, M.n);
    kin_t Kn; kinematics(&M, hq, &Kn); frame_pose(&Kn, &F, p, R);
    for (int k = 0; k < 3; k++) pos[k] = p[k].a;
    for (int k = 0; k < 9; k++) rot_rowmajor[k] = R[k].a;
    return 0;
}

int mfo_jac(const double *blob, const double *frame, const double *q, double *J_rowmajor /* 6 x n */) {
    mfo_model M; if (mfo_model_from_blob(blob, &M)) return -1;
    mfo_frame F; frame_from_arr(frame, &F);
    hd hq[MJ], p[3], R[9];
    to_hd(hq, q, M.n);
    kin_t Kn; kinematics(&M, hq, &Kn); frame_pose(&Kn, &F, p, R);
    int n = M.n;
    memset(J_rowmajor, 0, 6 * n * sizeof(double));
    for (int j = F.parent; j >= 0; j = M.parent[j]) {
        hd d[3], c[3];
        for (int k = 0; k < 3; k++) d[k] = sub(p[k], Kn.o[j][k]);
        cross3(c, Kn.z[j], d);
        for (int k = 0; k < 3; k++) { J_rowmajor[k * n + j] = c[k].a; J_rowmajor[(3 + k) * n + j] = Kn.z[j][k].a; }
    }
    return 0;
}

/* ------------------------------------------------------------------ */
/* OCP (one horizon): the transcription of force_optimization_pilz_6DOF.py
 * generalised with flags so C1 (3-DOF, tau^T tau + 100 qd^T qd) fits too.   */
typedef struct {
    int N, nf, use_line;
    double h;
    double frame[13];             /* parent, R(9), t(3) */
    double fdir[9];               /* force component a -> world direction fdir[3a..3a+2] */
    double line_ref[2];
    double wF, wqd, wtau;
    double q0[MJ], qd0[MJ];
    double qd_lo[MJ], qd_hi[MJ];  /* stages k >= 1 */
    double q_lo[MJ], q_hi[MJ];    /* states k >= 1 */
    const double *tau_lo, *tau_hi;/* N*n */
} mfo_ocp;

typedef struct {
    double tol;            /* scaled KKT error E_0 */
    double constr_viol_tol;
    int max_iter;
    double mu_init;
    int init_zero;         /* 1: IPOPT x0 = 0 for free variables; 0: hold q0 */
    int verbose;
    double prox;           /* proximal primal regularisation prox*mu on (q, qd) */
    double F_init;         /* initial guess for every force component */
    const double *w0;      /* warm start (w layout) or NULL: q_k, qd_k (k >= 1) and F_k from w0, pushed
                              into their bounds; q_0, qd_0 stay the problem's (IPOPT warm_start_init_point
                              with x0 = the previous solution, RepeatedMPCwithThermal.py:445-448, 462-487) */
    int warm_start;        /* with w0: IPOPT warm_start_init_point = yes -- warm_start_bound_push = _frac =
                              1e-3 (slacks alike) and bound multipliers warm_start_mult_bound_push = 1e-3
                              (CasADi's lam_x0 = 0 pushed), constraint multipliers 0 (lam_g0 = 0) */
} mfo_opts;

typedef struct {
    int status;            /* 0 converged, 1 max_iter, 2 line-search failure, 3 inertia failure */
    int iter;
    double kkt, cviol, obj, mu;
    int n_ls_fail, n_inertia_fix;
} mfo_result;

typedef struct {
    const mfo_model *M;
    const mfo_ocp *P;
    mfo_frame F;
    int N, n, nf, nl, nv, mb;
    /* iterate */
    double *q, *qd, *Fv, *s, *yc, *yl, *yd;
    double *zqL, *zqU, *zdL, *zdU, *vL, *vU;
    /* trial */
    double *tq, *tqd, *tF, *ts;
    /* stage eval cache */
    double *tau, *Jt, *line, *Jl, *W, *gf;
    double *ttau, *tline;
    /* step */
    double *dq, *dqd, *dF, *ds, *dyc, *dyl, *dyd, *dzqL, *dzqU, *dzdL, *dzdU, *dvL, *dvU;
    /* kkt workspace */
    double *wv, *G;
    double mu;
    double push_k;         /* bound_push = bound_frac of the initial point (cold 1e-2, warm 1e-3) */
} ws_t;

static int has(double b) { return isfinite(b); }

/* node evaluation at stage k.  mode 0: values only into (tau,line); mode 1: + jac + Hessian of
 * phi = sum_j cw_j tau_j + sum_i yl_i pf_i with cw = yd + 2 wtau tau.                               */
static double stage_cost(const mfo_ocp *P, int n, int nf, const double *qd, const double *F, const double *tau) {
    double c = 0;
    for (int j = 0; j < nf; j++) c += P->wF * F[j] * F[j];
    for (int j = 0; j < n; j++) c += P->wqd * qd[j] * qd[j] + P->wtau * tau[j] * tau[j];
    return c;
}

static void node_eval_hd(const ws_t *S, const hd *hq, const hd *hqd, const hd *hF, hd *tau, hd *pf) {
    const mfo_model *M = S->M;
    kin_t Kn;
    kinematics(M, hq, &Kn);
    hd zero[MJ];
    for (int i = 0; i < M->n; i++) zero[i] = K(0);
    rnea(M, &Kn, hqd, zero, tau);
    hd R[9];
    frame_pose(&Kn, &S->F, pf, R);
    if (S->nf > 0) {
        hd Fw[3] = {K(0), K(0), K(0)};
        for (int a = 0; a < S->nf; a++)
            for (int k = 0; k < 3; k++) Fw[k] = add(Fw[k], muls(hF[a], S->P->fdir[3 * a + k]));
        sub_external(M, &Kn, &S->F, pf, Fw, tau);
    }
}

static void eval_values(const ws_t *S, const double *q, const double *qd, const double *F, double *tau, double *line) {
    hd hq[MJ], hqd[MJ], hF[3], ht[MJ], pf[3];
    to_hd(hq, q, S->n); to_hd(hqd, qd, S->n); to_hd(hF, F, S->nf);
    node_eval_hd(S, hq, hqd, hF, ht, pf);
    for (int j = 0; j < S->n; j++) tau[j] = ht[j].a;
    for (int i = 0; i < S->nl; i++) line[i] = pf[i].a - S->P->line_ref[i];
}

static void eval_derivs(ws_t *S, int k) {
    int n = S->n, nf = S->nf, nv = S->nv, nl = S->nl;
    const double *q = S->q + k * n, *qd = S->qd + k * n, *F = S->Fv + k * nf;
    double *tau = S->tau + k * n, *Jt = S->Jt + (size_t)k * n * nv, *line = S->line + k * nl;
    double *Jl = S->Jl + k * nl * n, *W = S->W + (size_t)k * nv * nv, *gf = S->gf + k * nv;
    const double *yd = S->yd + k * n, *yl = S->yl + k * nl;
    double x[MV];
    memcpy(x, q, n * sizeof(double)); memcpy(x + n, qd, n * sizeof(double)); memcpy(x + 2 * n, F, nf * sizeof(double));
    eval_values(S, q, qd, F, tau, line);
    double cw[MJ];
    for (int j = 0; j < n; j++) cw[j] = yd[j] + 2.0 * S->P->wtau * tau[j];
    for (int u = 0; u < nv; u++) {
        for (int v = u; v < nv; v++) {
            hd hx[MV], ht[MJ], pf[3];
            for (int i = 0; i < nv; i++) hx[i] = K(x[i]);
            hx[u].b = 1.0;
            hx[v].c = 1.0;
            node_eval_hd(S, hx, hx + n, hx + 2 * n, ht, pf);
            double h2 = 0;
            for (int j = 0; j < n; j++) h2 += cw[j] * ht[j].d;
            for (int i = 0; i < nl; i++) h2 += yl[i] * pf[i].d;
            W[u * nv + v] = W[v * nv + u] = h2;
            if (u == v) {
                for (int j = 0; j < n; j++) Jt[j * nv + u] = ht[j].b;
                if (u < n)
                    for (int i = 0; i < nl; i++) Jl[i * n + u] = pf[i].b;
            }
        }
    }
    /* cost: wF F^T F + wqd qd^T qd + wtau tau^T tau */
    for (int u = 0; u < nv; u++) {
        double g = 0;
        for (int j = 0; j < n; j++) g += 2.0 * S->P->wtau * tau[j] * Jt[j * nv + u];
        if (u >= n && u < 2 * n) g += 2.0 * S->P->wqd * x[u];
        if (u >= 2 * n) g += 2.0 * S->P->wF * x[u];
        gf[u] = g;
        for (int v = 0; v < nv; v++) {
            double gn = 0;
            for (int j = 0; j < n; j++) gn += Jt[j * nv + u] * Jt[j * nv + v];
            W[u * nv + v] += 2.0 * S->P->wtau * gn;
        }
        if (u >= n && u < 2 * n) W[u * nv + u] += 2.0 * S->P->wqd;
        if (u >= 2 * n) W[u * nv + u] += 2.0 * S->P->wF;
    }
}


/* ------------------------------------------------------------------ */
/* IPM                                                                 */
/* IPOPT bound_push = bound_frac = 1e-2; warm_start_bound_push = _frac = 1e-3 (push_k) */
#define PUSH_K1 push_k
#define PUSH_K2 push_k

static double push_into_k(double x, double lo, double hi, double push_k) {
    int hl = has(lo), hh = has(hi);
    if (hl && hh) {
        double pl = fmin(PUSH_K1 * fmax(1.0, fabs(lo)), PUSH_K2 * (hi - lo));
        double pu = fmin(PUSH_K1 * fmax(1.0, fabs(hi)), PUSH_K2 * (hi - lo));
        x = fmax(x, lo + pl);
        x = fmin(x, hi - pu);
    } else if (hl) {
        x = fmax(x, lo + PUSH_K1 * fmax(1.0, fabs(lo)));
    } else if (hh) {
        x = fmin(x, hi - PUSH_K1 * fmax(1.0, fabs(hi)));
    }
    return x;
}
#define push_into(x, lo, hi) push_into_k((x), (lo), (hi), S->push_k)

static double *dalloc(size_t n) { return (double *)calloc(n ? n : 1, sizeof(double)); }

static void ws_alloc(ws_t *S) {
    int N = S->N, n = S->n, nf = S->nf, nl = S->nl, nv = S->nv, mb = S->mb;
    S->q = dalloc((N + 1) * n); S->qd = dalloc(N * n); S->Fv = dalloc(N * nf); S->s = dalloc(N * n);
    S->yc = dalloc(N * n); S->yl = dalloc(N * nl); S->yd = dalloc(N * n);
    S->zqL = dalloc((N + 1) * n); S->zqU = dalloc((N + 1) * n); S->zdL = dalloc(N * n); S->zdU = dalloc(N * n);
    S->vL = dalloc(N * n); S->vU = dalloc(N * n);
    S->tq = dalloc((N + 1) * n); S->tqd = dalloc(N * n); S->tF = dalloc(N * nf); S->ts = dalloc(N * n);
    S->tau = dalloc(N * n); S->Jt = dalloc((size_t)N * n * nv); S->line = dalloc(N * nl); S->Jl = dalloc(N * nl * n);
    S->W = dalloc((size_t)N * nv * nv); S->gf = dalloc(N * nv);
    S->ttau = dalloc(N * n); S->tline = dalloc(N * nl);
    S->dq = dalloc((N + 1) * n); S->dqd = dalloc(N * n); S->dF = dalloc(N * nf); S->ds = dalloc(N * n);
    S->dyc = dalloc(N * n); S->dyl = dalloc(N * nl); S->dyd = dalloc(N * n);
    S->dzqL = dalloc((N + 1) * n); S->dzqU = dalloc((N + 1) * n); S->dzdL = dalloc(N * n); S->dzdU = dalloc(N * n);
    S->dvL = dalloc(N * n); S->dvU = dalloc(N * n);
    S->wv = dalloc((size_t)(N + 1) * mb); S->G = dalloc((size_t)N * mb * n);
}

static void ws_free(ws_t *S) {
    double **p[] = {&S->q, &S->qd, &S->Fv, &S->s, &S->yc, &S->yl, &S->yd, &S->zqL, &S->zqU, &S->zdL, &S->zdU,
                    &S->vL, &S->vU, &S->tq, &S->tqd, &S->tF, &S->ts, &S->tau, &S->Jt, &S->line, &S->Jl, &S->W,
                    &S->gf, &S->ttau, &S->tline, &S->dq, &S->dqd, &S->dF, &S->ds, &S->dyc, &S->dyl, &S->dyd,
                    &S->dzqL, &S->dzqU, &S->dzdL, &S->dzdU, &S->dvL, &S->dvU, &S->wv, &S->G};
    for (size_t i = 0; i < sizeof p / sizeof p[0]; i++) { free(*p[i]); *p[i] = NULL; }
}

/* bounds accessors: q state k (1..N), qd stage k (1..N-1), tau slack (k, j) */
#define QLO(j) (S->P->q_lo[j])
#define QHI(j) (S->P->q_hi[j])
#define DLO(j) (S->P->qd_lo[j])
#define DHI(j) (S->P->qd_hi[j])
#define TLO(k, j) (S->P->tau_lo[(k) * S->n + (j)])
#define THI(k, j) (S->P->tau_hi[(k) * S->n + (j)])
#define TACT(k, j) (has(TLO(k, j)) || has(THI(k, j)))
/* state-only (line) constraints act from k = 2: q_0 is fixed and q_1 = q_0 + h qd_0 with
 * qd_0 fixed, so at k = 0, 1 they constrain fixed data (rank-deficient rows) */
#define LINE_ON(k) ((k) >= 2)

/* barrier objective + constraint violation (l1) at a point */
static void merit_parts(const ws_t *S, const double *q, const double *qd, const double *F, const double *s,
                        double *tau, double *line, double mu, double *phi_out, double *theta_out, int *ok) {
    int N = S->N, n = S->n, nf = S->nf, nl = S->nl;
    double f = 0, bar = 0, th = 0;
    *ok = 1;
    for (int k = 0; k < N; k++) {
        eval_values(S, q + k * n, qd + k * n, F + k * nf, tau + k * n, line + k * nl);
        f += stage_cost(S->P, n, nf, qd + k * n, F + k * nf, tau + k * n);
        for (int j = 0; j < n; j++) {
            th += fabs(q[k * n + j] + S->P->h * qd[k * n + j] - q[(k + 1) * n + j]);
            if (TACT(k, j)) th += fabs(tau[k * n + j] - s[k * n + j]);
        }
        if (LINE_ON(k))
            for (int i = 0; i < nl; i++) th += fabs(line[k * nl + i]);
    }
    for (int k = 1; k <= N; k++)
        for (int j = 0; j < n; j++) {
            double x = q[k * n + j];
            if (has(QLO(j))) { if (x - QLO(j) <= 0) *ok = 0; else bar -= log(x - QLO(j)); }
            if (has(QHI(j))) { if (QHI(j) - x <= 0) *ok = 0; else bar -= log(QHI(j) - x); }
        }
    for (int k = 1; k < N; k++)
        for (int j = 0; j < n; j++) {
            double x = qd[k * n + j];
            if (has(DLO(j))) { if (x - DLO(j) <= 0) *ok = 0; else bar -= log(x - DLO(j)); }
            if (has(DHI(j))) { if (DHI(j) - x <= 0) *ok = 0; else bar -= log(DHI(j) - x); }
        }
    for (int k = 0; k < N; k++)
        for (int j = 0; j < n; j++) {
            double x = s[k * n + j];
            if (has(TLO(k, j))) { if (x - TLO(k, j) <= 0) *ok = 0; else bar -= log(x - TLO(k, j)); }
            if (has(THI(k, j))) { if (THI(k, j) - x <= 0) *ok = 0; else bar -= log(THI(k, j) - x); }
        }
    *phi_out = f + mu * bar;
    *theta_out = th;
}

/* Assemble stage block k (0..N-1) or terminal (k == N) into Dm (mb x mb); returns size. */
typedef struct { double *Sx_q, *Sx_d, *Ss, *gq, *gd, *gs; } sig_t;

int mfo_solve(const double *blob, const mfo_ocp *P, const mfo_opts *O, double *w_out, mfo_result *res) {
    mfo_model M;
    if (mfo_model_from_blob(blob, &M)) return -1;
    ws_t SS, *S = &SS;
    memset(S, 0, sizeof *S);
    S->M = &M; S->P = P;
    frame_from_arr(P->frame, &S->F);
    S->N = P->N; S->n = M.n; S->nf = P->nf; S->nl = P->use_line ? 2 : 0;
    S->nv = 2 * S->n + S->nf;
    S->mb = S->nv + S->nl + S->n;
    int N = S->N, n = S->n, nf = S->nf, nl = S->nl, nv = S->nv, mb = S->mb;
    if (mb > MB || N < 1) return -2;
    ws_alloc(S);
    double h = P->h;

    /* ---- initial point ---- */
    const int warm = O->warm_start && O->w0;
    const double z0 = warm ? 1e-3 : 1.0;  /* bound_mult_init_val / warm_start_mult_bound_push */
    S->push_k = 1e-2;
    for (int k = 0; k <= N; k++)
        for (int j = 0; j < n; j++) {
            double x = (k == 0 || !O->init_zero) ? P->q0[j] : 0.0;
            S->q[k * n + j] = (k == 0) ? x : push_into(x, QLO(j), QHI(j));
        }
    for (int k = 0; k < N; k++)
        for (int j = 0; j < n; j++)
            S->qd[k * n + j] = (k == 0) ? P->qd0[j] : push_into(0.0, DLO(j), DHI(j));
    for (int k = 0; k < N * nf; k++) S->Fv[k] = O->F_init;
    if (O->w0) {
        const int st = 2 * n + nf;
        if (warm) S->push_k = 1e-3;
        for (int k = 0; k < N; k++) {
            const double *wk = O->w0 + n + (size_t)k * st;
            for (int j = 0; j < n; j++) {
                if (k > 0) S->qd[k * n + j] = push_into(wk[j], DLO(j), DHI(j));
                S->q[(k + 1) * n + j] = push_into(wk[n + nf + j], QLO(j), QHI(j));
            }
            for (int a = 0; a < nf; a++) S->Fv[k * nf + a] = wk[n + a];
        }
    }
    for (int k = 0; k < N; k++) {
        eval_values(S, S->q + k * n, S->qd + k * n, S->Fv + k * nf, S->tau + k * n, S->line + k * nl);
        for (int j = 0; j < n; j++) S->s[k * n + j] = push_into(S->tau[k * n + j], TLO(k, j), THI(k, j));
    }
    for (int k = 0; k <= N; k++)
        for (int j = 0; j < n; j++) {
            S->zqL[k * n + j] = (k > 0 && has(QLO(j))) ? z0 : 0.0;
            S->zqU[k * n + j] = (k > 0 && has(QHI(j))) ? z0 : 0.0;
        }
    for (int k = 0; k < N; k++)
        for (int j = 0; j < n; j++) {
            S->zdL[k * n + j] = (k > 0 && has(DLO(j))) ? z0 : 0.0;
            S->zdU[k * n + j] = (k > 0 && has(DHI(j))) ? z0 : 0.0;
            S->vL[k * n + j] = has(TLO(k, j)) ? z0 : 0.0;
            S->vU[k * n + j] = has(THI(k, j)) ? z0 : 0.0;
        }

    const double kappa_eps = 10.0, kappa_mu = 0.2, theta_mu = 1.5, tau_min = 0.99, s_max = 100.0;
    const double kappa_sigma = 1e10, eta = 1e-4, rho = 0.1;
    double mu = O->mu_init, nu = 0.0, reg_last = 0.0;
    int reg_tier = 0;
    int status = 1, it = 0, n_ls_fail = 0, n_ic = 0, consecutive_fail = 0;
    double E0 = INFINITY, cviol = INFINITY;

    double *Dm = (double *)malloc(sizeof(double) * mb * mb);
    double *Dsave = (double *)malloc(sizeof(double) * (size_t)(N + 1) * mb * mb);
    int *perm = (int *)malloc(sizeof(int) * (N + 1) * mb), *piv = (int *)malloc(sizeof(int) * (N + 1) * mb);
    int *msz = (int *)malloc(sizeof(int) * (N + 1));
    /* barrier quantities */
    double *Sxq = dalloc((N + 1) * n), *Sxd = dalloc(N * n), *Ss = dalloc(N * n);
    double *gphq = dalloc((N + 1) * n), *gphd = dalloc(N * n), *gphs = dalloc(N * n);
    double *rhs = dalloc((size_t)(N + 1) * mb);

    for (it = 0; it <= O->max_iter; it++) {
        /* ---- evaluate derivatives ---- */
        for (int k = 0; k < N; k++) eval_derivs(S, k);
        /* ---- optimality error ---- */
        double dinf = 0, pinf = 0, cinf0 = 0, cinfm = 0, sum_mult = 0, sum_bmult = 0;
        int n_mult = 0, n_bmult = 0;
        for (int k = 0; k <= N; k++) {
            for (int j = 0; j < n; j++) {
                if (k == 0) continue;
                double r;
                if (k < N) {
                    r = S->gf[k * nv + j] + S->yc[k * n + j] - S->yc[(k - 1) * n + j];
                    for (int i = 0; i < nl; i++) r += S->Jl[(k * nl + i) * n + j] * S->yl[k * nl + i];
                    for (int jj = 0; jj < n; jj++) r += S->Jt[((size_t)k * n + jj) * nv + j] * S->yd[k * n + jj];
                } else {
                    r = -S->yc[(N - 1) * n + j];
                }
                r += -S->zqL[k * n + j] + S->zqU[k * n + j];
                dinf = fmax(dinf, fabs(r));
                double x = S->q[k * n + j];
                if (has(QLO(j))) { double c = S->zqL[k * n + j] * (x - QLO(j)); cinf0 = fmax(cinf0, fabs(c)); cinfm = fmax(cinfm, fabs(c - mu)); sum_bmult += S->zqL[k * n + j]; n_bmult++; }
                if (has(QHI(j))) { double c = S->zqU[k * n + j] * (QHI(j) - x); cinf0 = fmax(cinf0, fabs(c)); cinfm = fmax(cinfm, fabs(c - mu)); sum_bmult += S->zqU[k * n + j]; n_bmult++; }
            }
        }
        for (int k = 0; k < N; k++) {
            for (int j = 0; j < n; j++) {
                if (k > 0) {
                    double r = S->gf[k * nv + n + j] + h * S->yc[k * n + j];
                    for (int jj = 0; jj < n; jj++) r += S->Jt[((size_t)k * n + jj) * nv + n + j] * S->yd[k * n + jj];
                    r += -S->zdL[k * n + j] + S->zdU[k * n + j];
                    dinf = fmax(dinf, fabs(r));
                    double x = S->qd[k * n + j];
                    if (has(DLO(j))) { double c = S->zdL[k * n + j] * (x - DLO(j)); cinf0 = fmax(cinf0, fabs(c)); cinfm = fmax(cinfm, fabs(c - mu)); sum_bmult += S->zdL[k * n + j]; n_bmult++; }
                    if (has(DHI(j))) { double c = S->zdU[k * n + j] * (DHI(j) - x); cinf0 = fmax(cinf0, fabs(c)); cinfm = fmax(cinfm, fabs(c - mu)); sum_bmult += S->zdU[k * n + j]; n_bmult++; }
                }
                if (TACT(k, j)) {
                    double r = -S->yd[k * n + j] - S->vL[k * n + j] + S->vU[k * n + j];
                    dinf = fmax(dinf, fabs(r));
                    double x = S->s[k * n + j];
                    if (has(TLO(k, j))) { double c = S->vL[k * n + j] * (x - TLO(k, j)); cinf0 = fmax(cinf0, fabs(c)); cinfm = fmax(cinfm, fabs(c - mu)); sum_bmult += S->vL[k * n + j]; n_bmult++; }
                    if (has(THI(k, j))) { double c = S->vU[k * n + j] * (THI(k, j) - x); cinf0 = fmax(cinf0, fabs(c)); cinfm = fmax(cinfm, fabs(c - mu)); sum_bmult += S->vU[k * n + j]; n_bmult++; }
                    pinf = fmax(pinf, fabs(S->tau[k * n + j] - S->s[k * n + j]));
                    sum_mult += fabs(S->yd[k * n + j]); n_mult++;
                }
                pinf = fmax(pinf, fabs(S->q[k * n + j] + h * S->qd[k * n + j] - S->q[(k + 1) * n + j]));
                sum_mult += fabs(S->yc[k * n + j]); n_mult++;
            }
            for (int a = 0; a < nf; a++) {
                double r = S->gf[k * nv + 2 * n + a];
                for (int jj = 0; jj < n; jj++) r += S->Jt[((size_t)k * n + jj) * nv + 2 * n + a] * S->yd[k * n + jj];
                dinf = fmax(dinf, fabs(r));
            }
            if (LINE_ON(k))
                for (int i = 0; i < nl; i++) { pinf = fmax(pinf, fabs(S->line[k * nl + i])); sum_mult += fabs(S->yl[k * nl + i]); n_mult++; }
        }
        double sd = fmax(s_max, (sum_mult + sum_bmult) / fmax(1, n_mult + n_bmult)) / s_max;
        double sc = fmax(s_max, sum_bmult / fmax(1, n_bmult)) / s_max;
        E0 = fmax(fmax(dinf / sd, pinf), cinf0 / sc);
        cviol = pinf;
        double Emu = fmax(fmax(dinf / sd, pinf), cinfm / sc);
        if (O->verbose) {
            double f = 0;
            for (int k = 0; k < N; k++) f += stage_cost(P, n, nf, S->qd + k * n, S->Fv + k * nf, S->tau + k * n);
            fprintf(stderr, "it %3d f %+.8e dinf %.2e pinf %.2e compl %.2e mu %.1e nu %.2e\n", it, f, dinf, pinf, cinf0, mu, nu);
        }
        if (O->verbose > 2) {
            double myc = 0, myl = 0, myd = 0, mv = 0, mz = 0; int kyc = -1, kyl = -1, kyd = -1;
            for (int i = 0; i < N * n; i++) {
                if (fabs(S->yc[i]) > myc) { myc = fabs(S->yc[i]); kyc = i; }
                if (fabs(S->yd[i]) > myd) { myd = fabs(S->yd[i]); kyd = i; }
                mv = fmax(mv, fmax(S->vL[i], S->vU[i])); mz = fmax(mz, fmax(S->zdL[i], S->zdU[i]));
            }
            for (int i = 0; i < N * nl; i++) if (fabs(S->yl[i]) > myl) { myl = fabs(S->yl[i]); kyl = i; }
            fprintf(stderr, "   |yc| %.2e@%d |yl| %.2e@%d |yd| %.2e@%d |v| %.2e |z| %.2e\n", myc, kyc, myl, kyl, myd, kyd, mv, mz);
        }
        if (E0 <= O->tol && cviol <= O->constr_viol_tol) { status = 0; break; }
        if (it == O->max_iter) { status = 1; break; }
        while (Emu <= kappa_eps * mu && mu > O->tol / 10.0) {
            double mnew = fmax(O->tol / 10.0, fmin(kappa_mu * mu, pow(mu, theta_mu)));
            if (mnew >= mu) break;
            mu = mnew;
            cinfm = 0; /* recompute complementarity error at new mu */
            for (int k = 1; k <= N; k++)
                for (int j = 0; j < n; j++) {
                    double x = S->q[k * n + j];
                    if (has(QLO(j))) cinfm = fmax(cinfm, fabs(S->zqL[k * n + j] * (x - QLO(j)) - mu));
                    if (has(QHI(j))) cinfm = fmax(cinfm, fabs(S->zqU[k * n + j] * (QHI(j) - x) - mu));
                }
            for (int k = 0; k < N; k++)
                for (int j = 0; j < n; j++) {
                    if (k > 0) {
                        double x = S->qd[k * n + j];
                        if (has(DLO(j))) cinfm = fmax(cinfm, fabs(S->zdL[k * n + j] * (x - DLO(j)) - mu));
                        if (has(DHI(j))) cinfm = fmax(cinfm, fabs(S->zdU[k * n + j] * (DHI(j) - x) - mu));
                    }
                    double x = S->s[k * n + j];
                    if (has(TLO(k, j))) cinfm = fmax(cinfm, fabs(S->vL[k * n + j] * (x - TLO(k, j)) - mu));
                    if (has(THI(k, j))) cinfm = fmax(cinfm, fabs(S->vU[k * n + j] * (THI(k, j) - x) - mu));
                }
            Emu = fmax(fmax(dinf / sd, pinf), cinfm / sc);
        }
        double tau_fb = fmax(tau_min, 1.0 - mu);

        /* ---- barrier Sigma and gradients ---- */
        for (int k = 0; k <= N; k++)
            for (int j = 0; j < n; j++) {
                int i = k * n + j;
                Sxq[i] = 0; gphq[i] = 0;
                if (k == 0) continue;
                double x = S->q[i];
                if (has(QLO(j))) { Sxq[i] += S->zqL[i] / (x - QLO(j)); gphq[i] -= mu / (x - QLO(j)); }
                if (has(QHI(j))) { Sxq[i] += S->zqU[i] / (QHI(j) - x); gphq[i] += mu / (QHI(j) - x); }
            }
        for (int k = 0; k < N; k++)
            for (int j = 0; j < n; j++) {
                int i = k * n + j;
                Sxd[i] = 0; gphd[i] = 0; Ss[i] = 0; gphs[i] = 0;
                if (k > 0) {
                    double x = S->qd[i];
                    if (has(DLO(j))) { Sxd[i] += S->zdL[i] / (x - DLO(j)); gphd[i] -= mu / (x - DLO(j)); }
                    if (has(DHI(j))) { Sxd[i] += S->zdU[i] / (DHI(j) - x); gphd[i] += mu / (DHI(j) - x); }
                }
                double x = S->s[i];
                if (has(TLO(k, j))) { Ss[i] += S->vL[i] / (x - TLO(k, j)); gphs[i] -= mu / (x - TLO(k, j)); }
                if (has(THI(k, j))) { Ss[i] += S->vU[i] / (THI(k, j) - x); gphs[i] += mu / (THI(k, j) - x); }
            }

        /* ---- inertia-corrected factorisation + solve ----
         * Block k (0 <= k < N): [yc_{k-1} | q_k | qd_k | F_k | yl_k]  (yc_{-1}: dummy, masked)
         * Block N:             [yc_{N-1} | q_N]
         * Coupling: the continuity row yc_k (block k+1) has entries I on q_k and h I on qd_k
         * (block k), i.e. K_{k+1,k} = C = [0 I hI 0 0] restricted to the yc rows.
         * Forward block elimination D_{k+1}[yc,yc] -= C D_k^-1 C^T, G_k = D_k^-1 C^T. */
        const int oyc = 0, oq = n, oqd = 2 * n, oF = 3 * n, oyl = 3 * n + nf;
        /* Inertia correction: tier 1 regularises only the force block
         * (the concave -F^2 directions), tier 2 the whole primal block.  The previous
         * iteration's tier and value are remembered; attempts: last/3, last, then x8
         * (0 once the value has decayed below 1e-8).  Tier 1 escalates into tier 2 above 1e6. */
        double dw = 0.0, dc = 0.0, dF = 0.0, dprox = O->prox * mu;
        int tries = 0, factor_ok = 0;
        int tier = reg_tier, step_no = 0;
        double reg = (reg_tier == 0) ? 0.0 : reg_last / 3.0;
        if (reg_tier != 0 && reg < 1e-8) { tier = 0; reg = 0.0; }
        if (tier == 1) dF = reg; else if (tier == 2) dw = reg;
        for (tries = 0; tries < 60; tries++) {
            int npos_t = 0, nneg_t = 0, nzero_t = 0;
            for (int k = 0; k <= N; k++) {
                int m = (k < N) ? mb : 2 * n;
                memset(Dm, 0, sizeof(double) * mb * mb);
                double *r = rhs + (size_t)k * mb;
                memset(r, 0, sizeof(double) * mb);
#define D_(i, j) Dm[(i) * m + (j)]
                /* continuity row of yc_{k-1}: -I on q_k; rhs -(q_{k-1} + h qd_{k-1} - q_k) */
                for (int j = 0; j < n; j++) {
                    D_(oyc + j, oyc + j) = -dc;
                    if (k > 0) {
                        D_(oyc + j, oq + j) = D_(oq + j, oyc + j) = -1.0;
                        r[oyc + j] = -(S->q[(k - 1) * n + j] + h * S->qd[(k - 1) * n + j] - S->q[k * n + j]);
                    } else {
                        D_(oyc + j, oyc + j) = -1.0; /* dummy */
                    }
                }
                if (k < N) {
                    const double *W = S->W + (size_t)k * nv * nv, *Jt = S->Jt + (size_t)k * n * nv;
                    const double *Jl = S->Jl + k * nl * n;
                    double Dd[MJ], rdd[MJ];
                    for (int j = 0; j < n; j++) {
                        int i = k * n + j;
                        if (TACT(k, j)) {
                            double sg = Ss[i] + dw;
                            Dd[j] = sg / (1.0 + dc * sg);
                            rdd[j] = (S->tau[i] - S->s[i]) + (gphs[i] - S->yd[i]) / sg;
                        } else { Dd[j] = 0; rdd[j] = 0; }
                    }
                    /* primal block: W + Sigma_x + reg + Jt^T D Jt  (vars at offset oq) */
                    for (int u = 0; u < nv; u++)
                        for (int v = 0; v < nv; v++) {
                            double a = W[u * nv + v];
                            for (int j = 0; j < n; j++) a += Jt[j * nv + u] * Dd[j] * Jt[j * nv + v];
                            D_(oq + u, oq + v) = a;
                        }
                    for (int u = 0; u < nv; u++) D_(oq + u, oq + u) += dw + (u >= 2 * n ? dF : dprox);
                    for (int j = 0; j < n; j++) { D_(oq + j, oq + j) += Sxq[k * n + j]; D_(oqd + j, oqd + j) += Sxd[k * n + j]; }
                    for (int i = 0; i < nl; i++) {
                        for (int j = 0; j < n; j++) { D_(oyl + i, oq + j) = Jl[i * n + j]; D_(oq + j, oyl + i) = Jl[i * n + j]; }
                        D_(oyl + i, oyl + i) = -dc;
                    }
                    for (int u = 0; u < nv; u++) {
                        double g = S->gf[k * nv + u];
                        for (int j = 0; j < n; j++) g += Jt[j * nv + u] * (S->yd[k * n + j] + Dd[j] * rdd[j]);
                        if (u < n) {
                            g += gphq[k * n + u] + S->yc[k * n + u] - (k > 0 ? S->yc[(k - 1) * n + u] : 0.0);
                            for (int i = 0; i < nl; i++) g += Jl[i * n + u] * S->yl[k * nl + i];
                        } else if (u < 2 * n) {
                            g += gphd[k * n + u - n] + h * S->yc[k * n + u - n];
                        }
                        r[oq + u] = -g;
                    }
                    for (int i = 0; i < nl; i++) r[oyl + i] = -S->line[k * nl + i];
                    if (k == 0) { /* q_0, qd_0 fixed */
                        for (int u = oq; u < oF; u++) {
                            for (int v = 0; v < m; v++) { D_(u, v) = 0; D_(v, u) = 0; }
                            D_(u, u) = 1.0; r[u] = 0;
                        }
                    }
                    if (!LINE_ON(k))
                        for (int i = 0; i < nl; i++) {
                            for (int v = 0; v < m; v++) { D_(oyl + i, v) = 0; D_(v, oyl + i) = 0; }
                            D_(oyl + i, oyl + i) = -1.0; r[oyl + i] = 0;
                        }
                } else {
                    for (int j = 0; j < n; j++) {
                        D_(oq + j, oq + j) = Sxq[N * n + j] + dw + dprox;
                        r[oq + j] = -(gphq[N * n + j] - S->yc[(N - 1) * n + j]);
                    }
                }
                double *wk = S->wv + (size_t)k * mb;
                memcpy(wk, r, sizeof(double) * m);
                if (k > 0) {
                    /* D[yc,yc] -= C G_{k-1};  z[yc] -= C w_{k-1}  (C = 0 on the fixed block-0 columns) */
                    const double *Gp = S->G + (size_t)(k - 1) * mb * n;
                    const double *wp = S->wv + (size_t)(k - 1) * mb;
                    if (k - 1 > 0)
                        for (int a = 0; a < n; a++) {
                            for (int b2 = 0; b2 < n; b2++) D_(oyc + a, oyc + b2) -= Gp[(oq + a) * n + b2] + h * Gp[(oqd + a) * n + b2];
                            wk[oyc + a] -= wp[oq + a] + h * wp[oqd + a];
                        }
                }
                int np, nn, nz;
                double *Dk = Dsave + (size_t)k * mb * mb;
                memcpy(Dk, Dm, sizeof(double) * m * m);
                bk_factor(Dk, m, perm + k * mb, piv + k * mb, &np, &nn, &nz);
                npos_t += np; nneg_t += nn; nzero_t += nz;
                if (nz) break;
                bk_solve(Dk, m, perm + k * mb, piv + k * mb, wk);
                if (k < N) {
                    double *Gk = S->G + (size_t)k * mb * n;
                    for (int c = 0; c < n; c++) {
                        double e[MB];
                        memset(e, 0, sizeof e);
                        if (k > 0) { e[oq + c] = 1.0; e[oqd + c] = h; }
                        if (k > 0) bk_solve(Dk, m, perm + k * mb, piv + k * mb, e);
                        for (int i = 0; i < m; i++) Gk[i * n + c] = e[i];
                    }
                }
#undef D_
            }
            int want_pos = N * nv + n, want_neg = N * (n + nl) + n;
            if (nzero_t == 0 && npos_t == want_pos && nneg_t == want_neg) { factor_ok = 1; break; }
            if (nzero_t > 0 && dc == 0.0) { dc = 1e-8 * pow(mu, 0.25); continue; }
            n_ic++;
            step_no++;
            if (tier == 0) {
                tier = (nf > 0 && P->wF < 0) ? 1 : 2;
                reg = 1e-4;
            } else if (step_no == 1 && reg_tier == tier && reg < reg_last) {
                reg = reg_last;               /* last/3 failed: retry the value that worked */
            } else {
                reg *= 8.0;
                if (tier == 1 && reg > 1e6) { tier = 2; reg = 1e-4; }
            }
            if (reg > 1e40) break;
            dF = (tier == 1) ? reg : 0.0;
            dw = (tier == 2) ? reg : 0.0;
        }
        if (!factor_ok) { status = 3; break; }
        reg_tier = tier;
        reg_last = reg;
        if (O->verbose > 1) fprintf(stderr, "   dF %.2e dw %.2e dc %.2e tries %d\n", dF, dw, dc, tries);

        /* ---- back substitution: y_N = w_N, y_k = w_k - G_k y_{k+1}[yc] ---- */
        {
            double ynext[MB];
            const double *yN = S->wv + (size_t)N * mb;
            for (int j = 0; j < n; j++) { S->dq[N * n + j] = yN[oq + j]; S->dyc[(N - 1) * n + j] = yN[oyc + j]; }
            memcpy(ynext, yN, sizeof(double) * 2 * n);
            for (int k = N - 1; k >= 0; k--) {
                double y[MB];
                const double *wk = S->wv + (size_t)k * mb, *Gk = S->G + (size_t)k * mb * n;
                for (int i = 0; i < mb; i++) {
                    double a = wk[i];
                    for (int c = 0; c < n; c++) a -= Gk[i * n + c] * ynext[oyc + c];
                    y[i] = a;
                }
                for (int j = 0; j < n; j++) {
                    S->dq[k * n + j] = y[oq + j]; S->dqd[k * n + j] = y[oqd + j];
                    if (k > 0) S->dyc[(k - 1) * n + j] = y[oyc + j];
                }
                for (int a = 0; a < nf; a++) S->dF[k * nf + a] = y[oF + a];
                for (int i = 0; i < nl; i++) S->dyl[k * nl + i] = LINE_ON(k) ? y[oyl + i] : 0.0;
                memcpy(ynext, y, sizeof(double) * mb);
            }
            for (int j = 0; j < n; j++) { S->dq[j] = 0; S->dqd[j] = 0; }
        }
        /* dyd, ds, dz, dv */
        for (int k = 0; k < N; k++) {
            const double *Jt = S->Jt + (size_t)k * n * nv;
            for (int j = 0; j < n; j++) {
                int i = k * n + j;
                if (!TACT(k, j)) { S->dyd[i] = 0; S->ds[i] = 0; continue; }
                double jdx = 0;
                for (int u = 0; u < n; u++) jdx += Jt[j * nv + u] * S->dq[k * n + u] + Jt[j * nv + n + u] * S->dqd[k * n + u];
                for (int a = 0; a < nf; a++) jdx += Jt[j * nv + 2 * n + a] * S->dF[k * nf + a];
                double sg = Ss[i] + dw, Dd = sg / (1.0 + dc * sg);
                double rs = gphs[i] - S->yd[i], rd = S->tau[i] - S->s[i];
                S->dyd[i] = Dd * (jdx + rd + rs / sg);
                S->ds[i] = (S->dyd[i] - rs) / sg;
            }
        }
        for (int k = 0; k <= N; k++)
            for (int j = 0; j < n; j++) {
                int i = k * n + j;
                S->dzqL[i] = S->dzqU[i] = 0;
                if (k == 0) continue;
                double x = S->q[i], dx = S->dq[i];
                if (has(QLO(j))) S->dzqL[i] = mu / (x - QLO(j)) - S->zqL[i] - S->zqL[i] / (x - QLO(j)) * dx;
                if (has(QHI(j))) S->dzqU[i] = mu / (QHI(j) - x) - S->zqU[i] + S->zqU[i] / (QHI(j) - x) * dx;
            }
        for (int k = 0; k < N; k++)
            for (int j = 0; j < n; j++) {
                int i = k * n + j;
                S->dzdL[i] = S->dzdU[i] = S->dvL[i] = S->dvU[i] = 0;
                if (k > 0) {
                    double x = S->qd[i], dx = S->dqd[i];
                    if (has(DLO(j))) S->dzdL[i] = mu / (x - DLO(j)) - S->zdL[i] - S->zdL[i] / (x - DLO(j)) * dx;
                    if (has(DHI(j))) S->dzdU[i] = mu / (DHI(j) - x) - S->zdU[i] + S->zdU[i] / (DHI(j) - x) * dx;
                }
                double x = S->s[i], dx = S->ds[i];
                if (has(TLO(k, j))) S->dvL[i] = mu / (x - TLO(k, j)) - S->vL[i] - S->vL[i] / (x - TLO(k, j)) * dx;
                if (has(THI(k, j))) S->dvU[i] = mu / (THI(k, j) - x) - S->vU[i] + S->vU[i] / (THI(k, j) - x) * dx;
            }
        /* ---- fraction to boundary ---- */
        double ap = 1.0, az = 1.0;
#define FTB_L(x, dx, lo, a) do { if ((dx) < 0) a = fmin(a, -tau_fb * ((x) - (lo)) / (dx)); } while (0)
#define FTB_U(x, dx, hi, a) do { if ((dx) > 0) a = fmin(a, tau_fb * ((hi) - (x)) / (dx)); } while (0)
#define FTB_Z(z, dz, a) do { if ((dz) < 0) a = fmin(a, -tau_fb * (z) / (dz)); } while (0)
        for (int k = 1; k <= N; k++)
            for (int j = 0; j < n; j++) {
                int i = k * n + j;
                if (has(QLO(j))) { FTB_L(S->q[i], S->dq[i], QLO(j), ap); FTB_Z(S->zqL[i], S->dzqL[i], az); }
                if (has(QHI(j))) { FTB_U(S->q[i], S->dq[i], QHI(j), ap); FTB_Z(S->zqU[i], S->dzqU[i], az); }
            }
        for (int k = 0; k < N; k++)
            for (int j = 0; j < n; j++) {
                int i = k * n + j;
                if (k > 0) {
                    if (has(DLO(j))) { FTB_L(S->qd[i], S->dqd[i], DLO(j), ap); FTB_Z(S->zdL[i], S->dzdL[i], az); }
                    if (has(DHI(j))) { FTB_U(S->qd[i], S->dqd[i], DHI(j), ap); FTB_Z(S->zdU[i], S->dzdU[i], az); }
                }
                if (has(TLO(k, j))) { FTB_L(S->s[i], S->ds[i], TLO(k, j), ap); FTB_Z(S->vL[i], S->dvL[i], az); }
                if (has(THI(k, j))) { FTB_U(S->s[i], S->ds[i], THI(k, j), ap); FTB_Z(S->vU[i], S->dvU[i], az); }
            }
        if (O->verbose > 2) {
            /* which component limits the primal fraction-to-boundary step? */
            double aq = 1, ad = 1, as_ = 1;
            for (int k = 1; k <= N; k++) for (int j = 0; j < n; j++) { int i = k * n + j;
                if (has(QLO(j))) FTB_L(S->q[i], S->dq[i], QLO(j), aq);
                if (has(QHI(j))) FTB_U(S->q[i], S->dq[i], QHI(j), aq); }
            int ks = -1, js = -1;
            for (int k = 0; k < N; k++) for (int j = 0; j < n; j++) { int i = k * n + j; double old = as_;
                if (k > 0) { if (has(DLO(j))) FTB_L(S->qd[i], S->dqd[i], DLO(j), ad); if (has(DHI(j))) FTB_U(S->qd[i], S->dqd[i], DHI(j), ad); }
                if (has(TLO(k, j))) FTB_L(S->s[i], S->ds[i], TLO(k, j), as_);
                if (has(THI(k, j))) FTB_U(S->s[i], S->ds[i], THI(k, j), as_);
                if (as_ < old) { ks = k; js = j; } }
            fprintf(stderr, "   ftb: q %.2e qd %.2e s %.2e (k %d j %d s %.3f ds %.3f tau %.3f lo %.2f hi %.2f)\n", aq, ad, as_, ks, js,
                    ks >= 0 ? S->s[ks * n + js] : 0, ks >= 0 ? S->ds[ks * n + js] : 0, ks >= 0 ? S->tau[ks * n + js] : 0,
                    ks >= 0 ? TLO(ks, js) : 0, ks >= 0 ? THI(ks, js) : 0);
        }
        /* ---- merit line search ---- */
        double phi0, th0; int ok0;
        {
            /* phi at current point (values already in S->tau / S->line from eval_derivs) */
            merit_parts(S, S->q, S->qd, S->Fv, S->s, S->ttau, S->tline, mu, &phi0, &th0, &ok0);
        }
        double gdot = 0, pHp = 0;
        for (int k = 0; k < N; k++) {
            const double *W = S->W + (size_t)k * nv * nv;
            double dx[MV];
            for (int j = 0; j < n; j++) { dx[j] = S->dq[k * n + j]; dx[n + j] = S->dqd[k * n + j]; }
            for (int a = 0; a < nf; a++) dx[2 * n + a] = S->dF[k * nf + a];
            for (int u = 0; u < nv; u++) {
                gdot += S->gf[k * nv + u] * dx[u];
                for (int v = 0; v < nv; v++) pHp += dx[u] * W[u * nv + v] * dx[v];
            }
            for (int j = 0; j < n; j++) {
                int i = k * n + j;
                gdot += gphd[i] * S->dqd[i] + gphs[i] * S->ds[i];
                pHp += Sxd[i] * S->dqd[i] * S->dqd[i] + Ss[i] * S->ds[i] * S->ds[i];
            }
        }
        for (int k = 1; k <= N; k++)
            for (int j = 0; j < n; j++) {
                int i = k * n + j;
                gdot += gphq[i] * S->dq[i];
                pHp += Sxq[i] * S->dq[i] * S->dq[i];
            }
        if (th0 > 1e-300) {
            double nreq = (gdot + 0.5 * fmax(pHp, 0.0)) / ((1.0 - rho) * th0);
            if (nu < nreq) nu = nreq + 1.0;
        }
        double Dphi = gdot - nu * th0;
        double m0 = phi0 + nu * th0;
        double alpha = ap;
        int accepted = 0;
        for (int ls = 0; ls < 40; ls++) {
            for (int i = 0; i < (N + 1) * n; i++) S->tq[i] = S->q[i] + alpha * S->dq[i];
            for (int i = 0; i < N * n; i++) { S->tqd[i] = S->qd[i] + alpha * S->dqd[i]; S->ts[i] = S->s[i] + alpha * S->ds[i]; }
            for (int i = 0; i < N * nf; i++) S->tF[i] = S->Fv[i] + alpha * S->dF[i];
            double ph, th; int okk;
            merit_parts(S, S->tq, S->tqd, S->tF, S->ts, S->ttau, S->tline, mu, &ph, &th, &okk);
            double mt = ph + nu * th;
            if (O->verbose > 3) fprintf(stderr, "      ls a %.3e phi %.10e th %.4e (phi0 %.10e th0 %.4e) ok %d\n", alpha, ph, th, phi0, th0, okk);
            if (okk && isfinite(mt) && mt - m0 <= eta * alpha * fmin(Dphi, 0.0) + 10.0 * 2.220446049250313e-16 * fabs(m0)) { accepted = 1; break; }
            alpha *= 0.5;
        }
        if (O->verbose) fprintf(stderr, "   ap %.3e az %.3e alpha %.3e acc %d Dphi %.3e th0 %.3e pHp %.3e\n", ap, az, alpha, accepted, Dphi, th0, pHp);
        if (!accepted) { n_ls_fail++; consecutive_fail++; if (consecutive_fail >= 5) { status = 2; break; } }
        else consecutive_fail = 0;
        /* ---- update ---- */
        for (int i = 0; i < (N + 1) * n; i++) S->q[i] += alpha * S->dq[i];
        for (int i = 0; i < N * n; i++) {
            S->qd[i] += alpha * S->dqd[i]; S->s[i] += alpha * S->ds[i];
            S->yc[i] += alpha * S->dyc[i]; S->yd[i] += alpha * S->dyd[i];
        }
        for (int i = 0; i < N * nf; i++) S->Fv[i] += alpha * S->dF[i];
        for (int i = 0; i < N * nl; i++) S->yl[i] += alpha * S->dyl[i];
#define ZUPD(z, dz, slack) do { double zz = (z) + az * (dz); double sl = (slack); zz = fmax(fmin(zz, kappa_sigma * mu / sl), mu / (kappa_sigma * sl)); (z) = zz; } while (0)
        for (int k = 1; k <= N; k++)
            for (int j = 0; j < n; j++) {
                int i = k * n + j;
                if (has(QLO(j))) ZUPD(S->zqL[i], S->dzqL[i], S->q[i] - QLO(j));
                if (has(QHI(j))) ZUPD(S->zqU[i], S->dzqU[i], QHI(j) - S->q[i]);
            }
        for (int k = 0; k < N; k++)
            for (int j = 0; j < n; j++) {
                int i = k * n + j;
                if (k > 0) {
                    if (has(DLO(j))) ZUPD(S->zdL[i], S->dzdL[i], S->qd[i] - DLO(j));
                    if (has(DHI(j))) ZUPD(S->zdU[i], S->dzdU[i], DHI(j) - S->qd[i]);
                }
                if (has(TLO(k, j))) ZUPD(S->vL[i], S->dvL[i], S->s[i] - TLO(k, j));
                if (has(THI(k, j))) ZUPD(S->vU[i], S->dvU[i], THI(k, j) - S->s[i]);
            }
    }
    /* ---- output in the reference layout [q0 | (qd_k, F_k, q_{k+1}) x N] ---- */
    if (w_out) {
        double *o = w_out;
        memcpy(o, S->q, n * sizeof(double)); o += n;
        for (int k = 0; k < N; k++) {
            memcpy(o, S->qd + k * n, n * sizeof(double)); o += n;
            memcpy(o, S->Fv + k * nf, nf * sizeof(double)); o += nf;
            memcpy(o, S->q + (k + 1) * n, n * sizeof(double)); o += n;
        }
    }
    if (res) {
        double f = 0;
        for (int k = 0; k < N; k++) {
            eval_values(S, S->q + k * n, S->qd + k * n, S->Fv + k * nf, S->tau + k * n, S->line + k * nl);
            f += stage_cost(P, n, nf, S->qd + k * n, S->Fv + k * nf, S->tau + k * n);
        }
        res->status = status; res->iter = it; res->kkt = E0; res->cviol = cviol; res->obj = f; res->mu = mu;
        res->n_ls_fail = n_ls_fail; res->n_inertia_fix = n_ic;
    }
    free(Dm); free(Dsave); free(perm); free(piv); free(msz);
    free(Sxq); free(Sxd); free(Ss); free(gphq); free(gphd); free(gphs); free(rhs);
    ws_free(S);
    return 0;
}

/* Batch of independent horizons (OpenMP over problems): P[i] share the model. */
int mfo_solve_batch(const double *blob, const mfo_ocp *P, int batch, const mfo_opts *O, double *w_out, int w_stride,
                    mfo_result *res, int nthreads) {
    int err = 0;
#ifdef _OPENMP
    if (nthreads > 0) omp_set_num_threads(nthreads);
#pragma omp parallel for schedule(dynamic, 1) reduction(| : err)
#endif
    for (int b = 0; b < batch; b++)
        err |= mfo_solve(blob, &P[b], O, w_out ? w_out + (size_t)b * w_stride : NULL, &res[b]);
    return err;
}

/* Node-level evaluation for derivative tests: tau, d tau / d(q,qd,F) (n x nv, row-major),
 * pf (3), d pf / dq (3 x n), and Hessian of phi = cw . tau + yl . pf[0:nl] (nv x nv). */
int mfo_node_derivs(const double *blob, const mfo_ocp *P, const double *q, const double *qd, const double *F,
                    const double *cw, const double *yl, double *tau, double *Jt, double *pf, double *Jp, double *H) {
    mfo_model M;
    if (mfo_model_from_blob(blob, &M)) return -1;
    ws_t SS, *S = &SS;
    memset(S, 0, sizeof *S);
    S->M = &M; S->P = P;
    frame_from_arr(P->frame, &S->F);
    S->n = M.n; S->nf = P->nf; S->nl = P->use_line ? 2 : 0; S->nv = 2 * S->n + S->nf;
    int n = S->n, nv = S->nv;
    double x[MV];
    memcpy(x, q, n * sizeof(double)); memcpy(x + n, qd, n * sizeof(double)); memcpy(x + 2 * n, F, S->nf * sizeof(double));
    for (int u = 0; u < nv; u++)
        for (int v = u; v < nv; v++) {
            hd hx[MV], ht[MJ], p[3];
            for (int i = 0; i < nv; i++) hx[i] = K(x[i]);
            hx[u].b = 1.0; hx[v].c = 1.0;
            node_eval_hd(S, hx, hx + n, hx + 2 * n, ht, p);
            double h2 = 0;
            for (int j = 0; j < n; j++) h2 += cw[j] * ht[j].d;
            for (int i = 0; i < S->nl; i++) h2 += yl[i] * p[i].d;
            H[u * nv + v] = H[v * nv + u] = h2;
            if (u == v) {
                for (int j = 0; j < n; j++) Jt[j * nv + u] = ht[j].b;
                if (u < n) for (int k = 0; k < 3; k++) Jp[k * n + u] = p[k].b;
                if (u == 0) { for (int j = 0; j < n; j++) tau[j] = ht[j].a; for (int k = 0; k < 3; k++) pf[k] = p[k].a; }
            }
        }
    return 0;
}
