// Device-side data structures of the batched interior-point solver.
#pragma once
#include <hip/hip_runtime.h>

#include "model.hpp"

namespace mf {

// Per-problem scalar state of the interior-point iteration.
struct ProbState {
    double mu, nu, reg_last, E0, cviol, obj;
    double tau_fb;         // fraction to the boundary parameter (k_ipm_pre -> k_kkt_recover)
    double kkt_dw, kkt_dc; // regularisation of the accepted factorisation (k_ipm_kkt -> k_kkt_recover)
    // step quantities for the line search (k_kkt_recover -> k_ipm_post): primal / dual step bounds
    // (fraction to the boundary), grad(phi)^T dx and dx^T (W + Sigma) dx
    double ap, az, gdot, pHp;
    double alpha;          // accepted primal step (k_ipm_post -> k_post_update)
    double phi0, th0;      // barrier objective and constraint violation at the iterate (k_kkt_recover -> k_ipm_post)
    int reg_tier;     // inertia correction of the last iteration: 0 none, 1 force block, 2 all primal
    int status;       // -1 running, 0 converged, 1 max_iter, 2 line-search failure, 3 inertia failure
    int iter, n_ls_fail, n_ic, consec_fail;
};

enum { ST_RUNNING = -1, ST_CONVERGED = 0, ST_MAXITER = 1, ST_LSFAIL = 2, ST_INERTIA = 3 };

// Problem constants shared by every horizon of a batch.
struct OcpConst {
    int N, n, nf, nl, nv, mb, npair;
    double h;
    double fdir[9];
    double wF, wqd, wtau;
    double qd0[MF_MAX_JOINTS];
    double qd_lo[MF_MAX_JOINTS], qd_hi[MF_MAX_JOINTS];
    double q_lo[MF_MAX_JOINTS], q_hi[MF_MAX_JOINTS];
    // solver options
    double tol, constr_viol_tol, mu_init, F_init;
    int max_iter;
    int warm_start;        // IPOPT warm_start_init_point constants for a w0 start (k_ipm_init)
};

// Device arrays; every per-problem array is [batch][size] with the size below.
struct IpmArrays {
    // iterate
    double *q, *qd, *F, *s, *yc, *yl, *yd, *zqL, *zqU, *zdL, *zdU, *vL, *vU;
    // step
    double *dq, *dqd, *dF, *ds, *dyc, *dyl, *dyd, *dzqL, *dzqU, *dzdL, *dzdU, *dvL, *dvU;
    // node evaluation (written by the eval kernels)
    double *tau, *Jt, *line, *Jl, *W, *gf, *cost;
    // barrier terms
    double *Sxq, *gphq, *Sxd, *gphd, *Ss, *gphs;
    // block LDL^T recursion
    double *G, *wv;
    // per-stage Riccati inputs [N x (g_k | c_k | e_k | dD_k)] then y_tau + D_tau r_tau (N x n)
    double *stg;
    // per-problem data
    double *q0, *lref;
    const double *tau_lo, *tau_hi;  // shared N x n
    ProbState *st;
    // optional per-solve inputs (device, may be null): per-problem fixed qd_0 (batch x n) and a
    // warm start in the w layout (batch x wsize)
    const double *qd0p, *w0;
    int *active;                    // device counter of running problems
    // compacted running set (k_compact, once per iteration): list[0..*nrun) = running problems in
    // index order; every per-iteration kernel maps its block / node slot through it
    int *list, *nrun;
};

// sizes (doubles) per problem
struct IpmSizes {
    size_t q, u, f, l, jt, jl, w, gf, cost, G, wv, stg;
};

__host__ __device__ inline IpmSizes ipm_sizes(const OcpConst &c) {
    IpmSizes s;
    s.q = (size_t)(c.N + 1) * c.n;
    s.u = (size_t)c.N * c.n;
    s.f = (size_t)c.N * (c.nf > 0 ? c.nf : 1);
    s.l = (size_t)c.N * (c.nl > 0 ? c.nl : 1);
    s.jt = (size_t)c.N * c.n * c.nv;
    s.jl = (size_t)c.N * (c.nl > 0 ? c.nl : 1) * c.n;
    s.w = (size_t)c.N * c.nv * c.nv;
    s.gf = (size_t)c.N * c.nv;
    s.cost = (size_t)c.N;
    s.G = (size_t)c.N * c.mb * c.n;
    s.wv = (size_t)(c.N + 1) * c.mb;
    s.stg = (size_t)c.N * (c.nv + 3 * c.n + (c.nl > 0 ? c.nl : 1));
    return s;
}

}  // namespace mf
