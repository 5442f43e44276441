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
 * Multipliers start cold.  w0 must not alias w. */
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
const char *mf_kernel_name(int slot);

const char *mf_last_error(void);

#ifdef __cplusplus
}
#endif
#endif
