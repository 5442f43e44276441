/*
 * mpcfatigue.h — C ABI of libmpcfatigue.so, the MI355X-native drop-in for the
 * hot path of ADVRHumanoids/mpc_fatigue.
 *
 * What each entry point replaces (reference file:line):
 *
 *   mf_model_from_urdf   urdf::parseURDF + pinocchio::urdf::buildModel
 *                        (src/casadi_pinocchio_bridge.hpp:60-63, 92-95, 124-127)
 *   mf_frame_id          model.getFrameId(body_name)  (bridge:103, 135; throws on
 *                        unknown names there -> MF_ERR_FRAME here)
 *   mf_id / mf_id_dev    generate_inv_dyn -> Function "inverse_dynamics"
 *                        {q,qdot,qddot}->{tau} (bridge:57-85, rnea L76, Function L78)
 *   mf_fk / mf_fk_dev    generate_forward_kin -> Function "forward_kinematics"
 *                        {q}->{ee_pos,ee_rot} (bridge:87-117)
 *   mf_jac / mf_jac_dev  generate_jacobian -> Function "jacobian" {q}->{J},
 *                        LOCAL_WORLD_ALIGNED 6 x nv (bridge:119-153)
 *   mf_problem_create    the per-node NLP transcription loop of the OCP scripts
 *                        (python/Pilz_6_DOF/force_optimization_pilz_6DOF.py:103-172,
 *                         python/Pilz_3_DOF/inverse_dynamics_pilz_3DOF_working.py)
 *   mf_node_eval         the (x,u) -> (xnext, g, cost, jac) surface of one shooting
 *                        node (force_optimization_pilz_6DOF.py:129-177)
 *   mf_solve_batch       nlpsol('Solver','ipopt',...) + Solver(lbx,ubx,lbg,ubg)
 *                        (force_optimization_pilz_6DOF.py:195-197), for a batch of
 *                        independent horizons
 *   mf_last_error        the C++ exception text pybind11 would have raised
 *
 * Conventions: all arrays are caller-owned FP64.  Host-pointer entry points
 * copy in/out; *_dev variants take device pointers and a hipStream_t (as void*).
 * Matrices are column-major like CasADi DM (ee_rot 3x3, J 6 x nv).  Every
 * function returns 0 on success or a negative MF_ERR_* code; the message is in
 * mf_last_error() (thread-local).  The library never falls back to a CPU path:
 * with no usable gfx950 device every compute entry point returns MF_ERR_DEVICE.
 */
#ifndef MPCFATIGUE_H
#define MPCFATIGUE_H

#ifdef __cplusplus
extern "C" {
#endif

#define MF_OK 0
#define MF_ERR_ARG (-1)
#define MF_ERR_URDF (-2)
#define MF_ERR_FRAME (-3)
#define MF_ERR_DEVICE (-4)
#define MF_ERR_UNSUPPORTED (-5)
#define MF_ERR_NOMEM (-6)

/* Model blob layout (mf_model_export): [n, gx, gy, gz] then per joint
 * MF_BLOB_JSTRIDE doubles: parent, R(9, row-major), t(3), axis(3), mass, com(3),
 * Ic(9, row-major, about com, joint frame), lower, upper, effort, velocity.   */
#define MF_BLOB_HDR 4
#define MF_BLOB_JSTRIDE 33
#define MF_MAX_JOINTS 16

typedef struct mf_model mf_model;
typedef struct mf_problem mf_problem;

int mf_model_from_urdf(const char *urdf_xml, mf_model **out);
void mf_model_free(mf_model *m);
int mf_model_nq(const mf_model *m);
/* writes min(cap, needed) doubles; returns the needed size */
int mf_model_export(const mf_model *m, double *blob, int cap);
/* frame lookup by URDF link / joint name; MF_ERR_FRAME if unknown */
int mf_frame_id(const mf_model *m, const char *name);
/* frame record: parent joint (-1 = universe), R (9 row-major), t (3) */
int mf_frame_export(const mf_model *m, int frame, double *rec13);

/* Batched evaluation of the bridge Functions (batch rows contiguous). */
int mf_id(const mf_model *m, const double *q, const double *qd, const double *qdd, double *tau, int batch);
int mf_fk(const mf_model *m, int frame, const double *q, double *pos3, double *rot9_colmajor, int batch);
int mf_jac(const mf_model *m, int frame, const double *q, double *J_colmajor, int batch);
int mf_id_dev(const mf_model *m, const double *q, const double *qd, const double *qdd, double *tau, int batch,
              void *stream);
int mf_fk_dev(const mf_model *m, int frame, const double *q, double *pos3, double *rot9_colmajor, int batch,
              void *stream);
int mf_jac_dev(const mf_model *m, int frame, const double *q, double *J_colmajor, int batch, void *stream);

/* ---- OCP transcription (one spec per problem family) ---- */
typedef struct {
    int N;                 /* shooting nodes */
    double h;              /* T / N */
    int frame;             /* mf_frame_id of the frame for J^T F and the line constraint */
    int nf;                /* force components (0..3) */
    double fdir[9];        /* world direction of force component a: fdir[3a..3a+2] */
    int use_line;          /* fk(q_k)[0:2] = line_ref for k >= 2 */
    double line_ref[2];    /* default reference (per-problem override in mf_solve_batch) */
    double wF, wqd, wtau;  /* stage cost wF|F|^2 + wqd|qd|^2 + wtau|tau|^2 */
    double qd0[MF_MAX_JOINTS];                          /* fixed qd_0 */
    double qd_lo[MF_MAX_JOINTS], qd_hi[MF_MAX_JOINTS];  /* k >= 1, +-inf allowed */
    double q_lo[MF_MAX_JOINTS], q_hi[MF_MAX_JOINTS];    /* states k >= 1 */
    const double *tau_lo, *tau_hi;                      /* N x n, fatigue schedule */
} mf_problem_spec;

typedef struct {
    double tol;            /* scaled KKT error (IPOPT E_0) */
    double constr_viol_tol;
    int max_iter;
    double mu_init;
    double F_init;         /* initial force guess (breaks the F = 0 saddle of -F^2) */
    int verbose;
    int warm_start;        /* with a warm start w0: IPOPT warm_start_init_point = yes (RepeatedMPCwithThermal.py:
                              445-446, mpc_principal.py:349-351) -- warm_start_bound_push = _frac = 1e-3 for the
                              primal point and the slacks, bound multipliers warm_start_mult_bound_push = 1e-3
                              (CasADi passes lam_x0 = 0), constraint multipliers 0 (lam_g0 = 0); 0: cold
                              constants (bound_push = bound_frac = 1e-2, bound multipliers 1) */
} mf_solver_opts;

int mf_problem_create(const mf_model *m, const mf_problem_spec *spec, mf_problem **out);
void mf_problem_free(mf_problem *p);
/* w layout of the reference (force_optimization_pilz_6DOF.py:103-172):
 * [q_0 | (qd_k, F_k, q_{k+1}) for k < N]  ->  n + N (2n + nf) doubles */
int mf_problem_wsize(const mf_problem *p);

/* One shooting node, batched over `nodes` rows:
 *   x = q (n), u = [qd (n), F (nf)]
 *   xnext = q + h qd (n); g = [tau (n), line (2 if use_line)]; cost (1)
 *   jac = d[xnext; g; cost] / d[x; u], column-major (rows n+n+nl+1, cols 2n+nf)
 * line_ref: per-row reference (nodes x 2) or NULL for the spec default.      */
int mf_node_eval(const mf_problem *p, const double *x, const double *u, const double *line_ref, double *xnext,
                 double *g, double *cost, double *jac, int nodes);

/* Solve `batch` independent horizons from q0 (batch x n).  line_ref: batch x 2
 * or NULL.  Outputs: w (batch x wsize), status (0 converged, 1 max_iter,
 * 2 line-search failure, 3 inertia failure), iterations, final KKT error,
 * objective.  device: HIP device ordinal.  Inputs/outputs are host memory. */
int mf_solve_batch(mf_problem *p, int batch, const double *q0, const double *line_ref, const mf_solver_opts *opts,
                   double *w, int *status, int *iters, double *kkt, double *obj, int device);
/* Same, all arrays device-resident; runs on `stream`; timing-friendly. */
int mf_solve_batch_dev(mf_problem *p, int batch, const double *q0, const double *line_ref,
                       const mf_solver_opts *opts, double *w, int *status, int *iters, double *kkt, double *obj,
                       void *stream);

/* Batched inverse kinematics of a frame position.  Replaces the per-script IPOPT solve of
 * min ||fk(q) - p||^2 from q = 0 (python/Pilz_6_DOF/force_optimization_pilz_6DOF.py:55-63,
 * python/2_pilz_6_DOF/Box_Pilz_6DOF.py:123-156, Centauro_functions.py:207-260) that produces
 * each script's initial state: damped least squares (J J^T + lam I) y = e, dq = J^T y, steps
 * capped at max_step (max norm), stop when |p - fk(q)| < tol or after iters steps.
 * target: batch x 3; q_init: batch x n or NULL (q = 0, as the reference); q_out: batch x n;
 * residual: batch (|p - fk(q_out)|, may be NULL).  _dev: device pointers, async on stream. */
int mf_ik_batch(const mf_model *m, int frame, const double *target, const double *q_init, double *q_out,
                double *residual, int batch, int iters, double lam, double max_step, double tol);
int mf_ik_batch_dev(const mf_model *m, int frame, const double *target, const double *q_init, double *q_out,
                    double *residual, int batch, int iters, double lam, double max_step, double tol, void *stream);

/* Warm-started batch solve (the receding-horizon calls of mpc_principal.py:357-377 and
 * RepeatedMPCwithThermal.py:445-487: Solver(x0 = sol, ...) with ipopt warm_start_init_point):
 * qd0 (batch x n, or NULL = the spec's) is each problem's fixed qd_0; w0 (batch x wsize, or NULL
 * = cold start) supplies q_k, qd_k (k >= 1) and F_k, pushed into their bounds; q_0 is q0.
 * Multipliers start at IPOPT's cold (opts->warm_start = 0) or warm-start values.  w0 must not alias w. */
int mf_solve_batch_ws(mf_problem *p, int batch, const double *q0, const double *qd0, const double *w0,
                      const double *line_ref, const mf_solver_opts *opts, double *w, int *status, int *iters,
                      double *kkt, double *obj, int device);
int mf_solve_batch_ws_dev(mf_problem *p, int batch, const double *q0, const double *qd0, const double *w0,
                          const double *line_ref, const mf_solver_opts *opts, double *w, int *status, int *iters,
                          double *kkt, double *obj, void *stream);

/* Per-kernel device time of the solver's launches on the solve stream (HIP events),
 * MF_NKERNELS slots named by mf_kernel_name(slot), in launch order of one interior-point
 * iteration: 0 = node values, Jacobian and Hessian columns (k_eval_node), 1 = condensed
 * stage Hessians and cost gradients (k_eval_asm), 2 = optimality error and barrier terms
 * (k_ipm_pre), 3 = inertia-corrected Riccati recursion and step recovery (k_ipm_kkt),
 * 4 = line search and update (k_ipm_post).  Enabling resets the totals. */
#define MF_NKERNELS 5
int mf_problem_timing(mf_problem *p, int enable);
int mf_problem_kernel_stats(const mf_problem *p, double *ms_total, long *launches);
/* Per-chunk trace of the last solve run with timing on (the host polls the running count every 4
 * iterations): iteration at the chunk start, problems running at its start, GPU ms of its launches.
 * Fills up to `cap` entries of the non-null arrays; returns the number of chunks. */
int mf_problem_trace(const mf_problem *p, int *iter, int *running, double *ms, int cap);
const char *mf_kernel_name(int slot);

/* ---- generic stage-structured OCPs: dual-arm box (C3), thermal fatigue state (a8), Centauro (C4) ----
 * Replaces the per-node transcription loops of python/2_pilz_6_DOF/Box_Pilz_6DOF.py:219-456 and of
 * the thermal MPC (python/Centauro_script/RepeatedMPCwithThermal.py:183-402, Tmodel_library.py:9-41)
 * plus their nlpsol('ipopt') solves.  One horizon is the NLP
 *   w = [x_0 | (u_k, x_{k+1}) for k < N]   (the reference's CSV layout, Box_Pilz_6DOF.py:464-466)
 *   min sum_k l(x_k, u_k)   s.t.  x_{k+1} = f(x_k, u_k),  c_lo[k] <= c_in(x_k, u_k) <= c_hi[k],
 *   c_eq(x_k) = 0 (eq_from <= k < N),  x_lo <= x_k <= x_hi (k >= 1),  u_lo[k] <= u_k <= u_hi[k]
 * where u_lo == u_hi fixes a component (qd_0).  Families:
 *   MF_FAM_CHAIN  x = [q, (T)], u = [qd, F];  c_in = tau = ID(q, qd, 0) - J_f^T [sum F_a fdir_a; 0];
 *                 c_eq = p_f[0:2] - line_ref;  l = wF|F|^2 + wqd|qd|^2 + wtau|tau|^2 + wT|T|^2;
 *                 f = [q + h qd, th_a T + th_b (Ra (tau/ktau)^2 + qd^2/Rh)]   (thermal: nx = 2n)
 *   MF_FAM_BOX    two 6-DOF arms (model 0 = first, model 1 = second URDF), x = [q_L, q_R],
 *                 u = [qd_L, qd_R, F_L, F_R];  c_in = [F_L + F_R - (0, 0, m g) as (z, x, y),
 *                 (E1 - E2) x (F_L - F_R), tau_L, tau_R];  c_eq = |E1 - E2|^2 - L;
 *                 l = w_box |(E1 + E2)/2 - p_des|^2 + w_qd |qd|^2;  f = q + h qd
 *   MF_FAM_CENTAURO  two 7-DOF arms (models 0 / 1, frames mass1_ee / mass2_ee),
 *                 python/Centauro_script/RepeatedMPCwithThermal.py:154-402 (Const1): x = [q (14), T (14)],
 *                 u = [qd (14), F_L, F_R];  c_in = tau = ID(q, qd, 0) + J_LA^T [F_L; 0] + J_RA^T [F_R; 0];
 *                 c_eq = [R_L^T (p_R - p_L), skew(R_L R_R^T)] minus their values at x_0 (rounded to
 *                 target_decimals when >= 0, mpc_principal.py:371-373), k >= eq_from;  mixed rows for
 *                 every k: F_L + F_R - (0, 0, m g) as (z, x, y), (p_L - p_R) x (F_L - F_R);
 *                 l = w_box |(p_L + p_R)/2 - box_pdes|^2 + w_qd |qd|^2 + wF (|F_L|^2 + |F_R|^2) + wT |T|^2;
 *                 f = [q + h qd, th_a T + th_b (Ra (tau/ktau)^2 + qd^2/Rh)]                      */
#define MF_FAM_CHAIN 0
#define MF_FAM_BOX 1
#define MF_FAM_CENTAURO 2
#define MF_GX_MAX 32
typedef struct mf_gproblem mf_gproblem;
typedef struct {
    int family;            /* MF_FAM_* */
    int N;
    double h;
    int frame0, frame1;    /* mf_frame_id of the force / constraint frame in model 0 / model 1 */
    int eq_from;           /* first node carrying c_eq (2: q_0 and q_1 = q_0 + h qd_0 are fixed data) */
    int nf;                /* CHAIN: force components along fdir */
    double fdir[9];
    int use_line;
    double line_ref[2];    /* default line reference (per-problem override in mf_gsolve_batch) */
    double wF, wqd, wtau, wT;
    int thermal;
    double th_a, th_b, Ra, Rh;
    double ktau[MF_MAX_JOINTS];
    double box_mg, box_L, box_pdes[3], w_box, w_qd;  /* BOX */
    double x_lo[MF_GX_MAX], x_hi[MF_GX_MAX];         /* states k >= 1, +-inf allowed */
    const double *u_lo, *u_hi;                       /* N x nu */
    const double *c_lo, *c_hi;                       /* N x ni */
    int target_decimals;                             /* CENTAURO: rounding of the pose targets, -1: exact */
} mf_gspec;

typedef struct {
    double tol;            /* scaled KKT error (IPOPT E_0) */
    double constr_viol_tol;
    int max_iter;
    double mu_init;
    int init_zero;         /* 1: IPOPT's x0 = 0 for every free variable; 0: hold x_0 */
    double F_init;         /* initial force components when u_init is NULL */
    const double *u_init;  /* nu initial controls used at every node (host memory), or NULL */
    int max_soc;           /* second-order corrections per iteration (IPOPT max_soc; 0 = off) */
    int verbose;
    int warm_start;        /* as mf_solver_opts.warm_start (IPOPT warm_start_init_point with w0) */
    int filter;            /* 1: IPOPT's globalisation -- filter line search, watchdog, soft restoration and the
                              restoration phase (IPOPT's: elastic p, n on every constraint row, the dynamics rows
                              included); 0: the l1-merit search */
    double bound_relax;    /* IPOPT bound_relax_factor (1e-8 in IPOPT; 0 = exact bounds) */
    int resto_hard_dyn;    /* 1: the restoration problem keeps x_{k+1} = f(x_k, u_k) exact (no elastic variables on
                              the dynamics rows; the build's variant before round 5); 0: IPOPT's restoration */
    int inertia_spec;      /* IPOPT mode: while few horizons run (at most as many as can hold 4 tries each on the
                              device at once: C3 192, C4 128, chain 512 on MI355X, at least 64), the first 4
                              inertia-correction tries of each iteration are factored concurrently (same result as
                              the sequential search); -1: never */
} mf_gopts;

/* Fills *o with the library's defaults (tol = constr_viol_tol = 1e-8, max_iter 3000, mu_init 0.1, max_soc 4, every
 * other field 0 / NULL) and returns sizeof(mf_gopts).  C callers start from it and set what they need, so fields a
 * later version appends start at their defaults (the struct has no size field). */
int mf_gopts_init(mf_gopts *o);
int mf_gproblem_create(const mf_model *m0, const mf_model *m1, const mf_gspec *spec, mf_gproblem **out);
void mf_gproblem_free(mf_gproblem *p);
/* dims = {nx, nu, ni, ne, wsize} */
int mf_gproblem_dims(const mf_gproblem *p, int *dims5);
/* x0: batch x nx; u0: batch x nu values of the fixed controls at k = 0 (qd_0 carried by a receding
 * horizon, mpc_principal.py:365-374) or NULL = u_lo[0]; w0: batch x wsize warm start (primal) or NULL;
 * line_ref: batch x 2 or NULL.  Outputs as mf_solve_batch.  Host memory; _dev: device memory on stream. */
int mf_gsolve_batch(mf_gproblem *p, int batch, const double *x0, const double *u0, const double *w0,
                    const double *line_ref, const mf_gopts *opts, double *w, int *status, int *iters, double *kkt,
                    double *obj, int device);
int mf_gsolve_batch_dev(mf_gproblem *p, int batch, const double *x0, const double *u0, const double *w0,
                        const double *line_ref, const mf_gopts *opts, double *w, int *status, int *iters,
                        double *kkt, double *obj, void *stream);
/* Continuous batching (device memory, build-defined: the reference solves one problem per nlpsol call,
 * Box_Pilz_6DOF.py:455-456, RepeatedMPCwithThermal.py:466): `slots` solves run at once and work through
 * `total` independent problems -- a slot whose problem has finished is handed the next one, so a few long
 * solves do not hold the device at single-problem latency.  Inputs and outputs have `total` rows; every
 * problem's result equals mf_gsolve_batch_dev's for the same row. */
int mf_gsolve_stream_dev(mf_gproblem *p, int total, int slots, const double *x0, const double *u0, const double *w0,
                         const double *line_ref, const mf_gopts *opts, double *w, int *status, int *iters,
                         double *kkt, double *obj, void *stream);
/* One node record evaluated by the device kernel (tests): xu = [x | u], multipliers yi (ni), ye (ne),
 * lam (nx); rec = [l | grad l (nv) | c_in (ni) | d c_in (ni x nv) | c_eq (ne) | d c_eq / dx (ne x nx) |
 * f (nx) | A (nx x nx) | B (nx x nu) | W (nv x nv)], row-major blocks.  Returns the record size. */
int mf_gnode_record(mf_gproblem *p, const double *xu, const double *yi, const double *ye, const double *lam,
                    const double *line_ref, double *rec, int device);
/* Diagnostics: dual state of problem b after the last solve, [lam | yi | ye | zxL | zxU | zuL | zuU | vL | vU |
 * mu] (per-node blocks as the solver stores them).  Returns the number of doubles written. */
int mf_gdebug_duals(mf_gproblem *p, int b, double *out);
/* Diagnostics: the slack rows s (N x ni, node-major) of problem b after the last solve -- with mf_gdebug_duals the
 * primal-dual point an oracle-side KKT check of a device solution needs.  Returns N x ni. */
int mf_gdebug_slacks(mf_gproblem *p, int b, double *out);
/* Diagnostics: n stage blocks of the C2 chain (M x (M + 1) row-major, M = 9) factorised on the device by a Bunch-Kaufman
 * variant (0: registers with pivoting, 1: LDS with unrolled scans, 2: natural-order registers with variant 1 as
 * fallback (k_gkkt_chain), 3: registers with pivoting, runtime step loop) and by the LDS routine of k_gkkt: the two factors (same layout) and per block
 * meta[2M + 6] = {perm | piv << 8 (M, variant), the same (M, k_gkkt's), inertia (pos, neg, zero) x 2}.  Returns M. */
int mf_debug_bk_compare(const double *K, int n, int variant, double *out_var, double *out_wave, int *meta);
/* Per-phase timing of the generic solver (HIP events on the solve stream around every launch group; bench.py):
 * enable != 0 turns it on and resets the accumulators.  kernel_stats: total ms and launches per slot
 * {k_geval, k_gasm, k_gpre, k_gkkt (with k_gspec and the occupancy variant), k_gls}, and (node_evals, may be
 * NULL) the node evaluations k_geval made while timing was on. */
int mf_gproblem_timing(mf_gproblem *p, int enable);
int mf_gproblem_kernel_stats(mf_gproblem *p, double *ms5, long *launches5, long long *node_evals);
/* Diagnostics: solver counters of problem b after the last solve, out[10] = {iterations, status, inertia corrections,
 * line-search failures, second-order-correction steps, restoration phases, watchdog starts, soft-restoration steps,
 * failed searches after StopWatchDog, restoration-phase iterations}.  Returns 10. */
int mf_gdebug_counters(mf_gproblem *p, int b, int *out);
/* Diagnostics: IPOPT-mode trace of horizon 0 of the last solve made with opts.verbose >= 2, 2 x 4096 rows of 16
 * doubles (rows of the phase-0 kernel, then of the line-search kernel, indexed by iteration); returns 4096.
 * _reset zeroes it. */
int mf_gdebug_trace(double *out);
int mf_gdebug_trace_reset(void);

const char *mf_last_error(void);

#ifdef __cplusplus
}
#endif
#endif
