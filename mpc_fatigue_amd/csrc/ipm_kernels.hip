// Batched interior-point solve of the fatigue-aware OCP on MI355X (gfx950).
//
// One IPM iteration = three launches:
//   k_eval_jac  lanes (problem, node, direction u)   dual numbers: tau, line, cost
//                                                     and column u of their Jacobian
//   k_eval_hess lanes (problem, node, pair (u<=v))    hyper-dual numbers: entry (u,v)
//                                                     of the stage Lagrangian Hessian
//   k_ipm_iter  one wavefront per problem             optimality error, barrier update,
//               inertia-corrected block-tridiagonal LDL^T (Bunch-Kaufman stage blocks
//               in LDS), step recovery, fraction-to-boundary, l1-merit line search,
//               update.  Mirrors oracle/mf_oracle.c mfo_solve statement by statement.
// Model constants (URDF joint placements, inertias) are staged in LDS per
// workgroup; per-problem arrays are [problem][node][field] so a wave reading a
// node's data, and lanes (node, field) writing it, both touch contiguous bytes.
#include <hip/hip_runtime.h>

#include "bk_wave.hpp"
#include "dyn.hpp"
#include "ipm.hpp"

namespace mf {

#define LINE_ON(k) ((k) >= 2)

__device__ __forceinline__ bool hasb(double b) { return isfinite(b); }

// Diagnostic build only (-DMF_PHASE_STAMPS): per-phase cycle counts of k_ipm_iter,
// accumulated by lane 0 into a debug buffer (never read by the solver).
#ifdef MF_PHASE_STAMPS
__device__ unsigned long long mf_stamp_buf[16 * 4096];
#define STAMP(slot)                                                                   \
    do {                                                                              \
        unsigned long long t_ = __builtin_amdgcn_s_memtime();                         \
        if (lane == 0 && b < 4096) mf_stamp_buf[b * 16 + (slot)] += t_ - t_prev_;     \
        t_prev_ = t_;                                                                 \
    } while (0)
#define STAMP_INIT unsigned long long t_prev_ = __builtin_amdgcn_s_memtime()
#define STAMP_COUNT(slot, v) do { if (lane == 0 && b < 4096) mf_stamp_buf[b * 16 + (slot)] += (v); } while (0)
#else
#define STAMP(slot) do {} while (0)
#define STAMP_INIT do {} while (0)
#define STAMP_COUNT(slot, v) do {} while (0)
#endif

// cooperative copy of a POD struct into LDS
template <class T> __device__ __forceinline__ void stage_lds(T *dst, const T *src) {
    const int words = (int)(sizeof(T) / sizeof(double));
    const double *s = reinterpret_cast<const double *>(src);
    double *d = reinterpret_cast<double *>(dst);
    for (int i = threadIdx.x; i < words; i += blockDim.x) d[i] = s[i];
}

// ============================================================== eval: Jacobian lanes
template <int NJ, int NF>
__global__ __launch_bounds__(256) void k_eval_jac(const DevModel *__restrict__ Mg, const DevFrame *__restrict__ Fg,
                                                  OcpConst C, IpmArrays A, int batch) {
    __shared__ DevModel M;
    __shared__ DevFrame F;
    stage_lds(&M, Mg);
    stage_lds(&F, Fg);
    __syncthreads();
    constexpr int NV = 2 * NJ + NF;
    constexpr int NFA = NF > 0 ? NF : 1;
    long t = (long)blockIdx.x * blockDim.x + threadIdx.x;
    long total = (long)batch * C.N * NV;
    if (t >= total) return;
    const int u = (int)(t % NV);
    const long r = t / NV;
    const int k = (int)(r % C.N);
    const int b = (int)(r / C.N);
    if (A.st[b].status != ST_RUNNING) return;
    const IpmSizes S = ipm_sizes(C);
    const double *q = A.q + b * S.q + (size_t)k * NJ;
    const double *qd = A.qd + b * S.u + (size_t)k * NJ;
    const double *Fv = A.F + b * S.f + (size_t)k * NFA;
    Dual xq[NJ], xqd[NJ], xF[NFA], tau[NJ], pf[3];
#pragma unroll
    for (int i = 0; i < NJ; i++) {
        xq[i] = Dual(q[i], u == i ? 1.0 : 0.0);
        xqd[i] = Dual(qd[i], u == NJ + i ? 1.0 : 0.0);
    }
#pragma unroll
    for (int a = 0; a < NFA; a++) xF[a] = Dual(NF > 0 ? Fv[a] : 0.0, u == 2 * NJ + a ? 1.0 : 0.0);
    node_tau<Dual, NJ>(M, F, NF, C.fdir, xq, xqd, xF, tau, pf);
    double *Jt = A.Jt + b * S.jt + (size_t)k * NJ * NV;
#pragma unroll
    for (int j = 0; j < NJ; j++) Jt[j * NV + u] = tau[j].d;
    if (C.nl > 0 && u < NJ) {
        double *Jl = A.Jl + b * S.jl + (size_t)k * C.nl * NJ;
        for (int l = 0; l < C.nl; l++) Jl[l * NJ + u] = pf[l].d;
    }
    double g = 0.0;
#pragma unroll
    for (int j = 0; j < NJ; j++) g += 2.0 * C.wtau * tau[j].v * tau[j].d;
    if (u >= NJ && u < 2 * NJ) g += 2.0 * C.wqd * qd[u - NJ];
    if (NF > 0 && u >= 2 * NJ) g += 2.0 * C.wF * Fv[u - 2 * NJ];
    A.gf[b * S.gf + (size_t)k * NV + u] = g;
    if (u == 0) {
        double *tv = A.tau + b * S.u + (size_t)k * NJ;
        double c = 0.0;
        for (int a = 0; a < NF; a++) c += C.wF * Fv[a] * Fv[a];
#pragma unroll
        for (int j = 0; j < NJ; j++) {
            tv[j] = tau[j].v;
            c += C.wqd * qd[j] * qd[j] + C.wtau * tau[j].v * tau[j].v;
        }
        A.cost[b * S.cost + k] = c;
        if (C.nl > 0) {
            double *lv = A.line + b * S.l + (size_t)k * C.nl;
            for (int l = 0; l < C.nl; l++) lv[l] = pf[l].v - A.lref[b * 2 + l];
        }
    }
}

// ============================================================== eval: Hessian lanes
template <int NJ, int NF>
__global__ __launch_bounds__(256) void k_eval_hess(const DevModel *__restrict__ Mg, const DevFrame *__restrict__ Fg,
                                                   OcpConst C, IpmArrays A, int batch) {
    __shared__ DevModel M;
    __shared__ DevFrame F;
    stage_lds(&M, Mg);
    stage_lds(&F, Fg);
    __syncthreads();
    constexpr int NV = 2 * NJ + NF;
    constexpr int NFA = NF > 0 ? NF : 1;
    constexpr int NP = NV * (NV + 1) / 2;
    long t = (long)blockIdx.x * blockDim.x + threadIdx.x;
    long total = (long)batch * C.N * NP;
    if (t >= total) return;
    int p = (int)(t % NP);
    const long r = t / NP;
    const int k = (int)(r % C.N);
    const int b = (int)(r / C.N);
    if (A.st[b].status != ST_RUNNING) return;
    int u = 0;
    while (p >= NV - u) { p -= NV - u; u++; }
    const int v = u + p;
    const IpmSizes S = ipm_sizes(C);
    const double *q = A.q + b * S.q + (size_t)k * NJ;
    const double *qd = A.qd + b * S.u + (size_t)k * NJ;
    const double *Fv = A.F + b * S.f + (size_t)k * NFA;
    const double *tv = A.tau + b * S.u + (size_t)k * NJ;
    const double *yd = A.yd + b * S.u + (size_t)k * NJ;
    double cw[NJ], yl[2] = {0.0, 0.0};
#pragma unroll
    for (int j = 0; j < NJ; j++) cw[j] = yd[j] + 2.0 * C.wtau * tv[j];
    for (int l = 0; l < C.nl; l++) yl[l] = A.yl[b * S.l + (size_t)k * C.nl + l];
    HDual xq[NJ], xqd[NJ], xF[NFA];
#pragma unroll
    for (int i = 0; i < NJ; i++) {
        xq[i] = HDual(q[i], u == i ? 1.0 : 0.0, v == i ? 1.0 : 0.0, 0.0);
        xqd[i] = HDual(qd[i], u == NJ + i ? 1.0 : 0.0, v == NJ + i ? 1.0 : 0.0, 0.0);
    }
#pragma unroll
    for (int a = 0; a < NFA; a++)
        xF[a] = HDual(NF > 0 ? Fv[a] : 0.0, u == 2 * NJ + a ? 1.0 : 0.0, v == 2 * NJ + a ? 1.0 : 0.0, 0.0);
    PhiVis<HDual, NJ> vis;
    vis.F = &F;
    vis.cw = cw;
    vis.yl = yl;
    vis.nl = C.nl;
#pragma unroll
    for (int c = 0; c < 3; c++) {
        HDual acc(0.0);
        for (int a = 0; a < NF; a++) acc += xF[a] * C.fdir[3 * a + c];
        vis.Fw[c] = acc;
    }
    vis.init();
    ne_pass<HDual>(M, NJ, xq, xqd, (const HDual *)nullptr, vis);
    double h2 = vis.phi.d;
    const double *Jt = A.Jt + b * S.jt + (size_t)k * NJ * NV;
    double gn = 0.0;
#pragma unroll
    for (int j = 0; j < NJ; j++) gn += Jt[j * NV + u] * Jt[j * NV + v];
    h2 += 2.0 * C.wtau * gn;
    if (u == v && u >= NJ && u < 2 * NJ) h2 += 2.0 * C.wqd;
    if (u == v && u >= 2 * NJ) h2 += 2.0 * C.wF;
    double *W = A.W + b * S.w + (size_t)k * NV * NV;
    W[u * NV + v] = h2;
    W[v * NV + u] = h2;
}

// ============================================================== init
template <int NJ, int NF, int NL>
__global__ __launch_bounds__(64) void k_ipm_init(const DevModel *__restrict__ Mg, const DevFrame *__restrict__ Fg,
                                                 OcpConst C, IpmArrays A, int batch) {
    __shared__ DevModel M;
    __shared__ DevFrame F;
    stage_lds(&M, Mg);
    stage_lds(&F, Fg);
    __syncthreads();
    const int b = blockIdx.x, lane = threadIdx.x;
    if (b >= batch) return;
    constexpr int NFA = NF > 0 ? NF : 1;
    const IpmSizes S = ipm_sizes(C);
    const int N = C.N;
    double *q = A.q + b * S.q, *qd = A.qd + b * S.u, *Fv = A.F + b * S.f, *s = A.s + b * S.u;
    const double *q0 = A.q0 + (size_t)b * NJ;
    auto push = [&](double x, double lo, double hi) {
        const double k1 = 1e-2, k2 = 1e-2;
        bool hl = hasb(lo), hh = hasb(hi);
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
    };
    for (int e = lane; e < (N + 1) * NJ; e += 64) {
        int k = e / NJ, j = e % NJ;
        q[e] = (k == 0) ? q0[j] : push(q0[j], C.q_lo[j], C.q_hi[j]);
        A.zqL[b * S.q + e] = (k > 0 && hasb(C.q_lo[j])) ? 1.0 : 0.0;
        A.zqU[b * S.q + e] = (k > 0 && hasb(C.q_hi[j])) ? 1.0 : 0.0;
    }
    for (int e = lane; e < N * NJ; e += 64) {
        int k = e / NJ, j = e % NJ;
        qd[e] = (k == 0) ? C.qd0[j] : push(0.0, C.qd_lo[j], C.qd_hi[j]);
        A.zdL[b * S.u + e] = (k > 0 && hasb(C.qd_lo[j])) ? 1.0 : 0.0;
        A.zdU[b * S.u + e] = (k > 0 && hasb(C.qd_hi[j])) ? 1.0 : 0.0;
        A.vL[b * S.u + e] = hasb(A.tau_lo[e]) ? 1.0 : 0.0;
        A.vU[b * S.u + e] = hasb(A.tau_hi[e]) ? 1.0 : 0.0;
        A.yc[b * S.u + e] = 0.0;
        A.yd[b * S.u + e] = 0.0;
    }
    for (int e = lane; e < N * NFA; e += 64) Fv[e] = NF > 0 ? C.F_init : 0.0;
    for (int e = lane; e < (int)S.l; e += 64) A.yl[b * S.l + e] = 0.0;
    __syncthreads();
    // slacks from tau at the initial point
    for (int k = lane; k < N; k += 64) {
        double tau[NJ], pf[3];
        node_tau<double, NJ>(M, F, NF, C.fdir, q + (size_t)k * NJ, qd + (size_t)k * NJ, Fv + (size_t)k * NFA, tau, pf);
        for (int j = 0; j < NJ; j++) s[k * NJ + j] = push(tau[j], A.tau_lo[k * NJ + j], A.tau_hi[k * NJ + j]);
    }
    if (lane == 0) {
        ProbState st;
        st.mu = C.mu_init; st.nu = 0.0; st.reg_last = 0.0; st.reg_tier = 0;
        st.E0 = INFINITY; st.cviol = INFINITY; st.obj = 0.0;
        st.status = ST_RUNNING; st.iter = 0; st.n_ls_fail = 0; st.n_ic = 0; st.consec_fail = 0;
        A.st[b] = st;
    }
}

// ============================================================== one IPM iteration
template <int NJ, int NF, int NL>
__global__ __launch_bounds__(64) void k_ipm_iter(const DevModel *__restrict__ Mg, const DevFrame *__restrict__ Fg,
                                                 OcpConst C, IpmArrays A, int batch) {
    constexpr int n = NJ, nf = NF, nl = NL;
    constexpr int NV = 2 * NJ + NF;
    constexpr int NFA = NF > 0 ? NF : 1;
    constexpr int NLA = NL > 0 ? NL : 1;
    constexpr int MB = 3 * NJ + NF + NL;
    __shared__ DevModel M;
    __shared__ DevFrame F;
    __shared__ double Dd_s[NJ], rdd_s[NJ];
    __shared__ int perm[MB], piv[MB];
    const int b = blockIdx.x, lane = threadIdx.x;
    if (b >= batch) return;
    ProbState st = A.st[b];
    if (st.status != ST_RUNNING) return;
    stage_lds(&M, Mg);
    stage_lds(&F, Fg);
    __syncthreads();
    STAMP_INIT;

    const IpmSizes S = ipm_sizes(C);
    const int N = C.N;
    const double h = C.h;
    double *q = A.q + b * S.q, *qd = A.qd + b * S.u, *Fv = A.F + b * S.f, *s = A.s + b * S.u;
    double *yc = A.yc + b * S.u, *yl = A.yl + b * S.l, *yd = A.yd + b * S.u;
    double *zqL = A.zqL + b * S.q, *zqU = A.zqU + b * S.q, *zdL = A.zdL + b * S.u, *zdU = A.zdU + b * S.u;
    double *vL = A.vL + b * S.u, *vU = A.vU + b * S.u;
    double *dq = A.dq + b * S.q, *dqd = A.dqd + b * S.u, *dF = A.dF + b * S.f, *ds = A.ds + b * S.u;
    double *dyc = A.dyc + b * S.u, *dyl = A.dyl + b * S.l, *dyd = A.dyd + b * S.u;
    double *dzqL = A.dzqL + b * S.q, *dzqU = A.dzqU + b * S.q, *dzdL = A.dzdL + b * S.u, *dzdU = A.dzdU + b * S.u;
    double *dvL = A.dvL + b * S.u, *dvU = A.dvU + b * S.u;
    const double *tau = A.tau + b * S.u, *Jt = A.Jt + b * S.jt, *line = A.line + b * S.l, *Jl = A.Jl + b * S.jl;
    const double *W = A.W + b * S.w, *gf = A.gf + b * S.gf, *cost = A.cost + b * S.cost;
    double *Sxq = A.Sxq + b * S.q, *gphq = A.gphq + b * S.q, *Sxd = A.Sxd + b * S.u, *gphd = A.gphd + b * S.u;
    double *Ss = A.Ss + b * S.u, *gphs = A.gphs + b * S.u;
    double *G = A.G + b * S.G, *wv = A.wv + b * S.wv;
    const double *lref = A.lref + b * 2;
    const double *tlo = A.tau_lo, *thi = A.tau_hi;
    const double *QLO = C.q_lo, *QHI = C.q_hi, *DLO = C.qd_lo, *DHI = C.qd_hi;
#define TACT(k, j) (hasb(tlo[(k) * n + (j)]) || hasb(thi[(k) * n + (j)]))

    const double kappa_eps = 10.0, kappa_mu = 0.2, theta_mu = 1.5, tau_min = 0.99, s_max = 100.0;
    const double kappa_sigma = 1e10, eta = 1e-4, rho = 0.1;
    double mu = st.mu, nu = st.nu;

    // ---------------- optimality error
    double dinf = 0, pinf = 0, cinf0 = 0, cinfm = 0, sum_mult = 0, sum_bmult = 0;
    int n_mult = 0, n_bmult = 0;
    for (int e = lane; e < N * n; e += 64) {  // q rows, k = 1..N
        int k = e / n + 1, j = e % n, i = k * n + j;
        double r;
        if (k < N) {
            r = gf[k * NV + j] + yc[k * n + j] - yc[(k - 1) * n + j];
            for (int l = 0; l < nl; l++) r += Jl[(k * nl + l) * n + j] * yl[k * nl + l];
            for (int jj = 0; jj < n; jj++) r += Jt[((size_t)k * n + jj) * NV + j] * yd[k * n + jj];
        } else {
            r = -yc[(N - 1) * n + j];
        }
        r += -zqL[i] + zqU[i];
        dinf = fmax(dinf, fabs(r));
        double x = q[i];
        if (hasb(QLO[j])) { double c = zqL[i] * (x - QLO[j]); cinf0 = fmax(cinf0, fabs(c)); cinfm = fmax(cinfm, fabs(c - mu)); sum_bmult += zqL[i]; n_bmult++; }
        if (hasb(QHI[j])) { double c = zqU[i] * (QHI[j] - x); cinf0 = fmax(cinf0, fabs(c)); cinfm = fmax(cinfm, fabs(c - mu)); sum_bmult += zqU[i]; n_bmult++; }
    }
    for (int e = lane; e < N * n; e += 64) {
        int k = e / n, j = e % n, i = e;
        if (k > 0) {
            double r = gf[k * NV + n + j] + h * yc[i];
            for (int jj = 0; jj < n; jj++) r += Jt[((size_t)k * n + jj) * NV + n + j] * yd[k * n + jj];
            r += -zdL[i] + zdU[i];
            dinf = fmax(dinf, fabs(r));
            double x = qd[i];
            if (hasb(DLO[j])) { double c = zdL[i] * (x - DLO[j]); cinf0 = fmax(cinf0, fabs(c)); cinfm = fmax(cinfm, fabs(c - mu)); sum_bmult += zdL[i]; n_bmult++; }
            if (hasb(DHI[j])) { double c = zdU[i] * (DHI[j] - x); cinf0 = fmax(cinf0, fabs(c)); cinfm = fmax(cinfm, fabs(c - mu)); sum_bmult += zdU[i]; n_bmult++; }
        }
        if (TACT(k, j)) {
            double r = -yd[i] - vL[i] + vU[i];
            dinf = fmax(dinf, fabs(r));
            double x = s[i];
            if (hasb(tlo[i])) { double c = vL[i] * (x - tlo[i]); cinf0 = fmax(cinf0, fabs(c)); cinfm = fmax(cinfm, fabs(c - mu)); sum_bmult += vL[i]; n_bmult++; }
            if (hasb(thi[i])) { double c = vU[i] * (thi[i] - x); cinf0 = fmax(cinf0, fabs(c)); cinfm = fmax(cinfm, fabs(c - mu)); sum_bmult += vU[i]; n_bmult++; }
            pinf = fmax(pinf, fabs(tau[i] - s[i]));
            sum_mult += fabs(yd[i]); n_mult++;
        }
        pinf = fmax(pinf, fabs(q[k * n + j] + h * qd[i] - q[(k + 1) * n + j]));
        sum_mult += fabs(yc[i]); n_mult++;
    }
    for (int e = lane; e < N * nf; e += 64) {
        int k = e / nf, a = e % nf;
        double r = gf[k * NV + 2 * n + a];
        for (int jj = 0; jj < n; jj++) r += Jt[((size_t)k * n + jj) * NV + 2 * n + a] * yd[k * n + jj];
        dinf = fmax(dinf, fabs(r));
    }
    for (int e = lane; e < N * nl; e += 64) {
        int k = e / nl;
        if (LINE_ON(k)) { pinf = fmax(pinf, fabs(line[e])); sum_mult += fabs(yl[e]); n_mult++; }
    }
    dinf = wave_max(dinf); pinf = wave_max(pinf); cinf0 = wave_max(cinf0); cinfm = wave_max(cinfm);
    sum_mult = wave_sum(sum_mult); sum_bmult = wave_sum(sum_bmult);
    n_mult = wave_sum_i(n_mult); n_bmult = wave_sum_i(n_bmult);
    const double sd = fmax(s_max, (sum_mult + sum_bmult) / fmax(1.0, (double)(n_mult + n_bmult))) / s_max;
    const double sc = fmax(s_max, sum_bmult / fmax(1.0, (double)n_bmult)) / s_max;
    const double E0 = fmax(fmax(dinf / sd, pinf), cinf0 / sc);
    double Emu = fmax(fmax(dinf / sd, pinf), cinfm / sc);
    st.E0 = E0;
    st.cviol = pinf;
    auto finish = [&](int status) {
        double f = 0.0;
        for (int k = lane; k < N; k += 64) f += cost[k];
        f = wave_sum(f);
        if (lane == 0) {
            st.status = status;
            st.obj = f;
            st.mu = mu;
            st.nu = nu;
            A.st[b] = st;
            atomicSub(A.active, 1);
        }
    };
    if (E0 <= C.tol && pinf <= C.constr_viol_tol) { finish(ST_CONVERGED); return; }
    if (st.iter >= C.max_iter) { finish(ST_MAXITER); return; }
    while (Emu <= kappa_eps * mu && mu > C.tol / 10.0) {
        double mnew = fmax(C.tol / 10.0, fmin(kappa_mu * mu, pow(mu, theta_mu)));
        if (mnew >= mu) break;
        mu = mnew;
        double cm = 0.0;
        for (int e = lane; e < N * n; e += 64) {
            int k = e / n + 1, j = e % n, i = k * n + j;
            double x = q[i];
            if (hasb(QLO[j])) cm = fmax(cm, fabs(zqL[i] * (x - QLO[j]) - mu));
            if (hasb(QHI[j])) cm = fmax(cm, fabs(zqU[i] * (QHI[j] - x) - mu));
        }
        for (int e = lane; e < N * n; e += 64) {
            int k = e / n, j = e % n, i = e;
            if (k > 0) {
                double x = qd[i];
                if (hasb(DLO[j])) cm = fmax(cm, fabs(zdL[i] * (x - DLO[j]) - mu));
                if (hasb(DHI[j])) cm = fmax(cm, fabs(zdU[i] * (DHI[j] - x) - mu));
            }
            double x = s[i];
            if (hasb(tlo[i])) cm = fmax(cm, fabs(vL[i] * (x - tlo[i]) - mu));
            if (hasb(thi[i])) cm = fmax(cm, fabs(vU[i] * (thi[i] - x) - mu));
        }
        cinfm = wave_max(cm);
        Emu = fmax(fmax(dinf / sd, pinf), cinfm / sc);
    }
    const double tau_fb = fmax(tau_min, 1.0 - mu);
    STAMP(0);

    // ---------------- barrier Sigma and gradients
    for (int e = lane; e < (N + 1) * n; e += 64) {
        int k = e / n, j = e % n;
        double sx = 0, gp = 0;
        if (k > 0) {
            double x = q[e];
            if (hasb(QLO[j])) { sx += zqL[e] / (x - QLO[j]); gp -= mu / (x - QLO[j]); }
            if (hasb(QHI[j])) { sx += zqU[e] / (QHI[j] - x); gp += mu / (QHI[j] - x); }
        }
        Sxq[e] = sx; gphq[e] = gp;
    }
    for (int e = lane; e < N * n; e += 64) {
        int k = e / n, j = e % n;
        double sx = 0, gp = 0, ss = 0, gs = 0;
        if (k > 0) {
            double x = qd[e];
            if (hasb(DLO[j])) { sx += zdL[e] / (x - DLO[j]); gp -= mu / (x - DLO[j]); }
            if (hasb(DHI[j])) { sx += zdU[e] / (DHI[j] - x); gp += mu / (DHI[j] - x); }
        }
        double x = s[e];
        if (hasb(tlo[e])) { ss += vL[e] / (x - tlo[e]); gs -= mu / (x - tlo[e]); }
        if (hasb(thi[e])) { ss += vU[e] / (thi[e] - x); gs += mu / (thi[e] - x); }
        Sxd[e] = sx; gphd[e] = gp; Ss[e] = ss; gphs[e] = gs;
    }
    __threadfence_block();
    __syncthreads();

    STAMP(1);
    // ---------------- inertia-corrected Riccati recursion
    // Stage k (1 <= k < N): x = dq_k (n), u = (dqd_k, dF_k) (NU), dynamics dx_{k+1} = dx_k + B du_k + c_k
    // with B = [h I, 0].  The line constraint of stage k+1 is pushed back onto stage k:
    // Jl_{k+1} (dx_k + B du_k + c_k) + line_{k+1} = 0.  Per stage the (NU+NL) block
    // [[Quu, Du^T], [Du, -dc]] is factorised by Bunch-Kaufman; the KKT matrix has the inertia
    // (n_primal, n_dual) iff every stage block has inertia (NU, NL) (Sylvester),
    // which is the test the oracle's block LDL^T of the whole KKT performs.  Stage 0 has x, qd
    // fixed: only dF_0 with Hessian H_FF.  Slot k of G / wv keeps Ku, Kl, P_{k+1} / ku, kl, p_{k+1}.
    constexpr int NU = NJ + NF;
    constexpr int NK = NU + NL;
    constexpr int LDK = NK + 1;
    constexpr int NRK = NJ + 1;
    constexpr int NLA2 = NL > 0 ? NL : 1;
    __shared__ double Hs[NV * NV], gs[NV];
    __shared__ double Ps[NJ * NJ], ps[NJ], ss[NJ], cs[NJ], Pn[NJ * NJ];
    __shared__ double Ks[NK * LDK], Rk[NK * NRK], Yk[NK * NRK];
    __shared__ double Gl[NLA2 * NJ], el[NLA2];
    __shared__ double xs[NJ], us[NU + NLA2];
    double dw = 0.0, dc = 0.0, dFr = 0.0;
    const int reg_tier0 = st.reg_tier;
    const double reg_last0 = st.reg_last;
    int tier = reg_tier0, step_no = 0;
    double reg = (reg_tier0 == 0) ? 0.0 : reg_last0 / 3.0;
    if (reg_tier0 != 0 && reg < 1e-8) { tier = 0; reg = 0.0; }
    if (tier == 1) dFr = reg; else if (tier == 2) dw = reg;
    bool factor_ok = false;
    int ntries = 0;
    for (int tries = 0; tries < 60; tries++) {
        ntries++;
        bool ok = true, zero = false;
        // terminal value function V_N = 1/2 x^T P x + p^T x
        for (int e = lane; e < n * n; e += 64) {
            int i = e / n, j = e % n;
            Ps[e] = (i == j) ? Sxq[N * n + i] + dw : 0.0;
        }
        for (int j = lane; j < n; j += 64) ps[j] = gphq[N * n + j] - yc[(N - 1) * n + j];
        __syncthreads();
        for (int k = N - 1; k >= 0; k--) {
            const double *Wk = W + (size_t)k * NV * NV, *Jtk = Jt + (size_t)k * n * NV;
            // ---- stage Hessian H (NV x NV) and gradient g, exactly the primal rows of the KKT
            for (int j = lane; j < n; j += 64) {
                int i = k * n + j;
                if (TACT(k, j)) {
                    double sg = Ss[i] + dw;
                    Dd_s[j] = sg / (1.0 + dc * sg);
                    rdd_s[j] = (tau[i] - s[i]) + (gphs[i] - yd[i]) / sg;
                } else { Dd_s[j] = 0.0; rdd_s[j] = 0.0; }
                cs[j] = q[k * n + j] + h * qd[k * n + j] - q[(k + 1) * n + j];
            }
            __syncthreads();
            for (int e = lane; e < NV * NV; e += 64) {
                int u = e / NV, v = e % NV;
                double a = Wk[u * NV + v];
                for (int jj = 0; jj < n; jj++) a += Jtk[jj * NV + u] * Dd_s[jj] * Jtk[jj * NV + v];
                if (u == v) {
                    a += dw + (u >= 2 * n ? dFr : 0.0);
                    if (u < n) a += Sxq[k * n + u];
                    else if (u < 2 * n) a += Sxd[k * n + u - n];
                }
                Hs[e] = a;
            }
            for (int u = lane; u < NV; u += 64) {
                double g = gf[k * NV + u];
                for (int jj = 0; jj < n; jj++) g += Jtk[jj * NV + u] * (yd[k * n + jj] + Dd_s[jj] * rdd_s[jj]);
                if (u < n) {
                    g += gphq[k * n + u] + yc[k * n + u] - (k > 0 ? yc[(k - 1) * n + u] : 0.0);
                    for (int l = 0; l < nl; l++) g += Jl[(k * nl + l) * n + u] * yl[k * nl + l];
                } else if (u < 2 * n) {
                    g += gphd[k * n + u - n] + h * yc[k * n + u - n];
                }
                gs[u] = g;
            }
            // s = P c + p ; keep P_{k+1}, p_{k+1} for the forward sweep
            double *Gk = G + (size_t)k * MB * n, *wk = wv + (size_t)k * MB;
            for (int j = lane; j < n; j += 64) {
                double a = ps[j];
                for (int i = 0; i < n; i++) a += Ps[j * n + i] * cs[i];
                ss[j] = a;
                wk[NU + NL + j] = ps[j];
            }
            for (int e = lane; e < n * n; e += 64) Gk[(NU + NL) * n + e] = Ps[e];
            __syncthreads();
            if (k == 0) {
                // only dF_0 is free (q_0, qd_0 fixed; the stage-1 line constraint is masked)
                if (nf > 0) {
                    for (int e = lane; e < nf * nf; e += 64) Ks[(e / nf) * LDK + e % nf] = Hs[(2 * n + e / nf) * NV + 2 * n + e % nf];
                    for (int a = lane; a < nf; a += 64) Rk[a * NRK] = -gs[2 * n + a];
                    __syncthreads();
                    BKInertia in = bk_factor_wave<LDK>(Ks, nf, perm, piv);
                    if (in.zero) { ok = false; zero = true; break; }
                    if (in.pos != nf) { ok = false; break; }
                    bk_solve_wave<LDK, NRK>(Ks, nf, perm, piv, Rk, 1, Yk);
                    for (int a = lane; a < nf; a += 64) wk[NJ + a] = Rk[a * NRK];  // dF_0 (ku slot)
                }
                __syncthreads();
                break;
            }
            const bool con = (nl > 0) && LINE_ON(k + 1) && (k + 1 <= N - 1);
            if (con) {
                const double *Jl1 = Jl + (size_t)(k + 1) * nl * n;
                for (int e = lane; e < nl * n; e += 64) Gl[e] = Jl1[e];
                for (int l = lane; l < nl; l += 64) {
                    double a = line[(k + 1) * nl + l];
                    for (int i = 0; i < n; i++) a += Jl1[l * n + i] * cs[i];
                    el[l] = a;
                }
                __syncthreads();
            }
            // ---- stage block [[Quu, Du^T], [Du, -dc]] and right-hand sides -[Qux | qu ; G | e]
            for (int e = lane; e < NK * NK; e += 64) {
                int a = e / NK, c = e % NK;
                double val;
                if (a < NU && c < NU) {
                    val = Hs[(n + a) * NV + n + c];
                    if (a < n && c < n) val += h * h * Ps[a * n + c];
                } else if (a >= NU && c >= NU) {
                    val = (a == c) ? (con ? -dc : -1.0) : 0.0;
                } else {
                    int l = (a >= NU) ? a - NU : c - NU, v = (a >= NU) ? c : a;
                    val = (con && v < n) ? h * Gl[l * n + v] : 0.0;
                }
                Ks[a * LDK + c] = val;
            }
            for (int e = lane; e < NK * NRK; e += 64) {
                int a = e / NRK, c = e % NRK;
                double val;
                if (a < NU) {
                    if (c < n) val = -(Hs[(n + a) * NV + c] + (a < n ? h * Ps[a * n + c] : 0.0));
                    else val = -(gs[n + a] + (a < n ? h * ss[a] : 0.0));
                } else {
                    int l = a - NU;
                    val = con ? -(c < n ? Gl[l * n + c] : el[l]) : 0.0;
                }
                Rk[e] = val;
            }
            __syncthreads();
            BKInertia in = bk_factor_wave<LDK>(Ks, NK, perm, piv);
            if (in.zero) { ok = false; zero = true; break; }
            if (in.pos != NU || in.neg != NL) { ok = false; break; }
            bk_solve_wave<LDK, NRK>(Ks, NK, perm, piv, Rk, NRK, Yk);
            // ---- P_k = Qxx + Qxu Ku + G^T Kl ; p_k = qx + Qxu ku + G^T kl
            for (int e = lane; e < n * n; e += 64) {
                int i = e / n, j = e % n;
                double a = Hs[i * NV + j] + Ps[i * n + j];
                for (int c = 0; c < NU; c++) a += (Hs[i * NV + n + c] + (c < n ? h * Ps[i * n + c] : 0.0)) * Rk[c * NRK + j];
                if (con)
                    for (int l = 0; l < nl; l++) a += Gl[l * n + i] * Rk[(NU + l) * NRK + j];
                Pn[e] = a;
            }
            double pnew = 0.0;
            if (lane < n) {
                int i = lane;
                pnew = gs[i] + ss[i];
                for (int c = 0; c < NU; c++) pnew += (Hs[i * NV + n + c] + (c < n ? h * Ps[i * n + c] : 0.0)) * Rk[c * NRK + n];
                if (con)
                    for (int l = 0; l < nl; l++) pnew += Gl[l * n + i] * Rk[(NU + l) * NRK + n];
            }
            for (int e = lane; e < NK * n; e += 64) Gk[e] = Rk[(e / n) * NRK + e % n];  // Ku (NU x n), Kl (NL x n)
            for (int a = lane; a < NK; a += 64) wk[a] = Rk[a * NRK + n];              // ku, kl
            __syncthreads();
            for (int e = lane; e < n * n; e += 64) {
                int i = e / n, j = e % n;
                Ps[e] = 0.5 * (Pn[e] + Pn[j * n + i]);
            }
            if (lane < n) ps[lane] = pnew;
            __syncthreads();
        }
        if (ok) { factor_ok = true; break; }
        if (zero && dc == 0.0) { dc = 1e-8 * pow(mu, 0.25); continue; }
        st.n_ic++;
        step_no++;
        if (tier == 0) {
            tier = (nf > 0 && C.wF < 0) ? 1 : 2;
            reg = 1e-4;
        } else if (step_no == 1 && reg_tier0 == tier && reg < reg_last0) {
            reg = reg_last0;
        } else {
            reg *= 8.0;
            if (tier == 1 && reg > 1e6) { tier = 2; reg = 1e-4; }
        }
        if (reg > 1e40) break;
        dFr = (tier == 1) ? reg : 0.0;
        dw = (tier == 2) ? reg : 0.0;
    }
    STAMP(2);
    STAMP_COUNT(8, ntries);
    if (!factor_ok) { finish(ST_INERTIA); return; }
    st.reg_tier = tier;
    st.reg_last = reg;

    // ---------------- forward sweep: du_k = Ku dx_k + ku, dyl_{k+1} = Kl dx_k + kl,
    //                  dyc_k = P_{k+1} dx_{k+1} + p_{k+1}
    for (int j = lane; j < n; j += 64) {
        dq[j] = 0.0; dqd[j] = 0.0;
        xs[j] = q[j] + h * qd[j] - q[n + j];  // dx_1 = c_0 (dx_0 = 0, dqd_0 = 0)
    }
    for (int a = lane; a < nf; a += 64) dF[a] = wv[NJ + a];
    for (int l = lane; l < nl; l += 64) { dyl[l] = 0.0; dyl[nl + l] = 0.0; }
    __syncthreads();
    for (int j = lane; j < n; j += 64) {  // dyc_0 = P_1 dx_1 + p_1 (slot 0)
        double a = wv[NU + NL + j];
        for (int i = 0; i < n; i++) a += G[(NU + NL) * n + j * n + i] * xs[i];
        dyc[j] = a;
    }
    for (int k = 1; k < N; k++) {
        const double *Gk = G + (size_t)k * MB * n, *wk = wv + (size_t)k * MB;
        for (int a = lane; a < NK; a += 64) {
            double v = wk[a];
            for (int i = 0; i < n; i++) v += Gk[a * n + i] * xs[i];
            us[a] = v;
        }
        for (int j = lane; j < n; j += 64) dq[k * n + j] = xs[j];
        __syncthreads();
        for (int j = lane; j < n; j += 64) {
            dqd[k * n + j] = us[j];
            cs[j] = xs[j] + h * us[j] + (q[k * n + j] + h * qd[k * n + j] - q[(k + 1) * n + j]);
        }
        for (int a = lane; a < nf; a += 64) dF[k * NFA + a] = us[NJ + a];
        if (k + 1 < N)
            for (int l = lane; l < nl; l += 64) dyl[(k + 1) * nl + l] = ((nl > 0) && LINE_ON(k + 1)) ? us[NU + l] : 0.0;
        __syncthreads();
        for (int j = lane; j < n; j += 64) {
            double a = wk[NU + NL + j];
            for (int i = 0; i < n; i++) a += Gk[(NU + NL) * n + j * n + i] * cs[i];
            dyc[k * n + j] = a;
            xs[j] = cs[j];
        }
        __syncthreads();
    }
    for (int j = lane; j < n; j += 64) dq[N * n + j] = xs[j];
    __threadfence_block();
    __syncthreads();

    // ---------------- dyd, ds, dz, dv
    for (int e = lane; e < N * n; e += 64) {
        int k = e / n, j = e % n, i = e;
        if (!TACT(k, j)) { dyd[i] = 0.0; ds[i] = 0.0; continue; }
        const double *Jtk = Jt + (size_t)k * n * NV;
        double jdx = 0.0;
        for (int u = 0; u < n; u++) jdx += Jtk[j * NV + u] * dq[k * n + u] + Jtk[j * NV + n + u] * dqd[k * n + u];
        for (int a = 0; a < nf; a++) jdx += Jtk[j * NV + 2 * n + a] * dF[k * NFA + a];
        double sg = Ss[i] + dw, Dd = sg / (1.0 + dc * sg);
        double rs = gphs[i] - yd[i], rd = tau[i] - s[i];
        dyd[i] = Dd * (jdx + rd + rs / sg);
        ds[i] = (dyd[i] - rs) / sg;
    }
    for (int e = lane; e < (N + 1) * n; e += 64) {
        int k = e / n, j = e % n;
        double a = 0, bb = 0;
        if (k > 0) {
            double x = q[e], dx = dq[e];
            if (hasb(QLO[j])) a = mu / (x - QLO[j]) - zqL[e] - zqL[e] / (x - QLO[j]) * dx;
            if (hasb(QHI[j])) bb = mu / (QHI[j] - x) - zqU[e] + zqU[e] / (QHI[j] - x) * dx;
        }
        dzqL[e] = a; dzqU[e] = bb;
    }
    __threadfence_block();
    __syncthreads();
    for (int e = lane; e < N * n; e += 64) {
        int k = e / n, j = e % n;
        double a = 0, bb = 0, c = 0, d = 0;
        if (k > 0) {
            double x = qd[e], dx = dqd[e];
            if (hasb(DLO[j])) a = mu / (x - DLO[j]) - zdL[e] - zdL[e] / (x - DLO[j]) * dx;
            if (hasb(DHI[j])) bb = mu / (DHI[j] - x) - zdU[e] + zdU[e] / (DHI[j] - x) * dx;
        }
        double x = s[e], dx = ds[e];
        if (hasb(tlo[e])) c = mu / (x - tlo[e]) - vL[e] - vL[e] / (x - tlo[e]) * dx;
        if (hasb(thi[e])) d = mu / (thi[e] - x) - vU[e] + vU[e] / (thi[e] - x) * dx;
        dzdL[e] = a; dzdU[e] = bb; dvL[e] = c; dvU[e] = d;
    }
    __threadfence_block();
    __syncthreads();

    STAMP(3);
    // ---------------- fraction to boundary
    double ap = 1.0, az = 1.0;
    auto ftbL = [&](double x, double dx, double lo, double &a) { if (dx < 0) a = fmin(a, -tau_fb * (x - lo) / dx); };
    auto ftbU = [&](double x, double dx, double hi, double &a) { if (dx > 0) a = fmin(a, tau_fb * (hi - x) / dx); };
    auto ftbZ = [&](double z, double dz, double &a) { if (dz < 0) a = fmin(a, -tau_fb * z / dz); };
    for (int e = n + lane; e < (N + 1) * n; e += 64) {
        int j = e % n;
        if (hasb(QLO[j])) { ftbL(q[e], dq[e], QLO[j], ap); ftbZ(zqL[e], dzqL[e], az); }
        if (hasb(QHI[j])) { ftbU(q[e], dq[e], QHI[j], ap); ftbZ(zqU[e], dzqU[e], az); }
    }
    for (int e = lane; e < N * n; e += 64) {
        int k = e / n, j = e % n;
        if (k > 0) {
            if (hasb(DLO[j])) { ftbL(qd[e], dqd[e], DLO[j], ap); ftbZ(zdL[e], dzdL[e], az); }
            if (hasb(DHI[j])) { ftbU(qd[e], dqd[e], DHI[j], ap); ftbZ(zdU[e], dzdU[e], az); }
        }
        if (hasb(tlo[e])) { ftbL(s[e], ds[e], tlo[e], ap); ftbZ(vL[e], dvL[e], az); }
        if (hasb(thi[e])) { ftbU(s[e], ds[e], thi[e], ap); ftbZ(vU[e], dvU[e], az); }
    }
    ap = wave_min(ap);
    az = wave_min(az);

    // ---------------- merit at the current point, directional derivative, curvature
    // merit of a point (x + alpha dx); alpha = 0 uses the stored node values
    auto merit = [&](double alpha, double &phi, double &theta, bool &ok_out) {
        double f = 0, bar = 0, th = 0;
        int bad = 0;
        for (int k = lane; k < N; k += 64) {
            double tq[NJ], tqd[NJ], tF[NFA], tt[NJ], pf[3];
            for (int j = 0; j < n; j++) { tq[j] = q[k * n + j] + alpha * dq[k * n + j]; tqd[j] = qd[k * n + j] + alpha * dqd[k * n + j]; }
            for (int a = 0; a < NFA; a++) tF[a] = NF > 0 ? Fv[k * NFA + a] + alpha * dF[k * NFA + a] : 0.0;
            node_tau<double, NJ>(M, F, NF, C.fdir, tq, tqd, tF, tt, pf);
            double c = 0.0;
            for (int a = 0; a < nf; a++) c += C.wF * tF[a] * tF[a];
            for (int j = 0; j < n; j++) c += C.wqd * tqd[j] * tqd[j] + C.wtau * tt[j] * tt[j];
            f += c;
            for (int j = 0; j < n; j++) {
                double qn = q[(k + 1) * n + j] + alpha * dq[(k + 1) * n + j];
                th += fabs(tq[j] + h * tqd[j] - qn);
                if (TACT(k, j)) th += fabs(tt[j] - (s[k * n + j] + alpha * ds[k * n + j]));
            }
            if (LINE_ON(k))
                for (int l = 0; l < nl; l++) th += fabs(pf[l] - lref[l]);
        }
        for (int e = n + lane; e < (N + 1) * n; e += 64) {
            int j = e % n;
            double x = q[e] + alpha * dq[e];
            if (hasb(QLO[j])) { if (x - QLO[j] <= 0) bad = 1; else bar -= log(x - QLO[j]); }
            if (hasb(QHI[j])) { if (QHI[j] - x <= 0) bad = 1; else bar -= log(QHI[j] - x); }
        }
        for (int e = lane; e < N * n; e += 64) {
            int k = e / n, j = e % n;
            if (k > 0) {
                double x = qd[e] + alpha * dqd[e];
                if (hasb(DLO[j])) { if (x - DLO[j] <= 0) bad = 1; else bar -= log(x - DLO[j]); }
                if (hasb(DHI[j])) { if (DHI[j] - x <= 0) bad = 1; else bar -= log(DHI[j] - x); }
            }
            double x = s[e] + alpha * ds[e];
            if (hasb(tlo[e])) { if (x - tlo[e] <= 0) bad = 1; else bar -= log(x - tlo[e]); }
            if (hasb(thi[e])) { if (thi[e] - x <= 0) bad = 1; else bar -= log(thi[e] - x); }
        }
        f = wave_sum(f); bar = wave_sum(bar); th = wave_sum(th);
        bad = wave_sum_i(bad);
        phi = f + mu * bar;
        theta = th;
        ok_out = (bad == 0);
    };
    // merit at the current point from the node values the eval kernel stored
    double phi0, th0;
    {
        double f = 0, bar = 0, th = 0;
        for (int k = lane; k < N; k += 64) {
            f += cost[k];
            for (int j = 0; j < n; j++) {
                th += fabs(q[k * n + j] + h * qd[k * n + j] - q[(k + 1) * n + j]);
                if (TACT(k, j)) th += fabs(tau[k * n + j] - s[k * n + j]);
            }
            if (LINE_ON(k))
                for (int l = 0; l < nl; l++) th += fabs(line[k * nl + l]);
        }
        for (int e = n + lane; e < (N + 1) * n; e += 64) {
            int j = e % n;
            if (hasb(QLO[j])) bar -= log(q[e] - QLO[j]);
            if (hasb(QHI[j])) bar -= log(QHI[j] - q[e]);
        }
        for (int e = lane; e < N * n; e += 64) {
            int k = e / n, j = e % n;
            if (k > 0) {
                if (hasb(DLO[j])) bar -= log(qd[e] - DLO[j]);
                if (hasb(DHI[j])) bar -= log(DHI[j] - qd[e]);
            }
            if (hasb(tlo[e])) bar -= log(s[e] - tlo[e]);
            if (hasb(thi[e])) bar -= log(thi[e] - s[e]);
        }
        f = wave_sum(f); bar = wave_sum(bar); th = wave_sum(th);
        phi0 = f + mu * bar;
        th0 = th;
    }
    double gdot = 0, pHp = 0;
    for (int k = lane; k < N; k += 64) {
        const double *Wk = W + (size_t)k * NV * NV;
        double dx[NV];
        for (int j = 0; j < n; j++) { dx[j] = dq[k * n + j]; dx[n + j] = dqd[k * n + j]; }
        for (int a = 0; a < nf; a++) dx[2 * n + a] = dF[k * NFA + a];
        for (int u = 0; u < NV; u++) {
            gdot += gf[k * NV + u] * dx[u];
            for (int v = 0; v < NV; v++) pHp += dx[u] * Wk[u * NV + v] * dx[v];
        }
    }
    for (int e = lane; e < N * n; e += 64) {
        gdot += gphd[e] * dqd[e] + gphs[e] * ds[e];
        pHp += Sxd[e] * dqd[e] * dqd[e] + Ss[e] * ds[e] * ds[e];
    }
    for (int e = n + lane; e < (N + 1) * n; e += 64) {
        gdot += gphq[e] * dq[e];
        pHp += Sxq[e] * dq[e] * dq[e];
    }
    gdot = wave_sum(gdot);
    pHp = wave_sum(pHp);
    if (th0 > 1e-300) {
        double nreq = (gdot + 0.5 * fmax(pHp, 0.0)) / ((1.0 - rho) * th0);
        if (nu < nreq) nu = nreq + 1.0;
    }
    STAMP(4);
    const double Dphi = gdot - nu * th0;
    const double m0 = phi0 + nu * th0;
    int nls = 0;
    double alpha = ap;
    bool accepted = false;
    for (int ls = 0; ls < 40; ls++) {
        double ph, th;
        bool okk;
        merit(alpha, ph, th, okk);
        double mt = ph + nu * th;
        nls++;
        if (okk && isfinite(mt) && mt - m0 <= eta * alpha * fmin(Dphi, 0.0) + 10.0 * 2.220446049250313e-16 * fabs(m0)) {
            accepted = true;
            break;
        }
        alpha *= 0.5;
    }
    STAMP(5);
    STAMP_COUNT(9, nls);
    if (!accepted) {
        st.n_ls_fail++;
        st.consec_fail++;
        if (st.consec_fail >= 5) { st.mu = mu; st.nu = nu; finish(ST_LSFAIL); return; }
    } else {
        st.consec_fail = 0;
    }

    // ---------------- update
    for (int e = lane; e < (N + 1) * n; e += 64) q[e] += alpha * dq[e];
    for (int e = lane; e < N * n; e += 64) {
        qd[e] += alpha * dqd[e]; s[e] += alpha * ds[e];
        yc[e] += alpha * dyc[e]; yd[e] += alpha * dyd[e];
    }
    for (int e = lane; e < N * nf; e += 64) Fv[(e / nf) * NFA + e % nf] += alpha * dF[(e / nf) * NFA + e % nf];
    for (int e = lane; e < N * nl; e += 64) yl[e] += alpha * dyl[e];
    __threadfence_block();
    __syncthreads();
    auto zupd = [&](double &z, double dz, double slack) {
        double zz = z + az * dz;
        zz = fmax(fmin(zz, kappa_sigma * mu / slack), mu / (kappa_sigma * slack));
        z = zz;
    };
    for (int e = n + lane; e < (N + 1) * n; e += 64) {
        int j = e % n;
        if (hasb(QLO[j])) zupd(zqL[e], dzqL[e], q[e] - QLO[j]);
        if (hasb(QHI[j])) zupd(zqU[e], dzqU[e], QHI[j] - q[e]);
    }
    for (int e = lane; e < N * n; e += 64) {
        int k = e / n, j = e % n;
        if (k > 0) {
            if (hasb(DLO[j])) zupd(zdL[e], dzdL[e], qd[e] - DLO[j]);
            if (hasb(DHI[j])) zupd(zdU[e], dzdU[e], DHI[j] - qd[e]);
        }
        if (hasb(tlo[e])) zupd(vL[e], dvL[e], s[e] - tlo[e]);
        if (hasb(thi[e])) zupd(vU[e], dvU[e], thi[e] - s[e]);
    }
    STAMP(6);
    STAMP_COUNT(10, 1);
    if (lane == 0) {
        st.iter++;
        st.mu = mu;
        st.nu = nu;
        A.st[b] = st;
    }
#undef TACT
}

// ============================================================== output in the reference layout
template <int NJ, int NF>
__global__ __launch_bounds__(64) void k_ipm_output(OcpConst C, IpmArrays A, int batch, double *w, int *status,
                                                   int *iters, double *kkt, double *obj) {
    const int b = blockIdx.x, lane = threadIdx.x;
    if (b >= batch) return;
    constexpr int NFA = NF > 0 ? NF : 1;
    const IpmSizes S = ipm_sizes(C);
    const int N = C.N, n = NJ, stride = 2 * n + NF;
    const int ws = n + N * stride;
    double *o = w + (size_t)b * ws;
    const double *q = A.q + b * S.q, *qd = A.qd + b * S.u, *Fv = A.F + b * S.f;
    for (int e = lane; e < ws; e += 64) {
        double v;
        if (e < n) v = q[e];
        else {
            int k = (e - n) / stride, c = (e - n) % stride;
            if (c < n) v = qd[k * n + c];
            else if (c < n + NF) v = Fv[k * NFA + c - n];
            else v = q[(k + 1) * n + c - n - NF];
        }
        o[e] = v;
    }
    if (lane == 0) {
        ProbState st = A.st[b];
        if (status) status[b] = st.status;
        if (iters) iters[b] = st.iter;
        if (kkt) kkt[b] = st.E0;
        if (obj) obj[b] = st.obj;
    }
}

// ============================================================== host launchers
template <int NJ, int NF, int NL>
struct IpmLaunch {
    static void init(const DevModel *M, const DevFrame *F, const OcpConst &C, const IpmArrays &A, int batch,
                     hipStream_t s) {
        hipLaunchKernelGGL((k_ipm_init<NJ, NF, NL>), dim3(batch), dim3(64), 0, s, M, F, C, A, batch);
    }
    // phase 0: node values + Jacobians, 1: Lagrangian Hessians, 2: per-problem IPM step
    static void iter(int phase, const DevModel *M, const DevFrame *F, const OcpConst &C, const IpmArrays &A,
                     int batch, hipStream_t s) {
        constexpr int NV = 2 * NJ + NF;
        constexpr int NP = NV * (NV + 1) / 2;
        long tj = (long)batch * C.N * NV, th = (long)batch * C.N * NP;
        if (phase == 0)
            hipLaunchKernelGGL((k_eval_jac<NJ, NF>), dim3((unsigned)((tj + 255) / 256)), dim3(256), 0, s, M, F, C,
                               A, batch);
        else if (phase == 1)
            hipLaunchKernelGGL((k_eval_hess<NJ, NF>), dim3((unsigned)((th + 255) / 256)), dim3(256), 0, s, M, F,
                               C, A, batch);
        else
            hipLaunchKernelGGL((k_ipm_iter<NJ, NF, NL>), dim3(batch), dim3(64), 0, s, M, F, C, A, batch);
    }
    static void output(const OcpConst &C, const IpmArrays &A, int batch, double *w, int *status, int *iters,
                       double *kkt, double *obj, hipStream_t s) {
        hipLaunchKernelGGL((k_ipm_output<NJ, NF>), dim3(batch), dim3(64), 0, s, C, A, batch, w, status, iters, kkt,
                           obj);
    }
};

// explicit instantiations: Pilz 3-DOF (C1) and Pilz 6-DOF force problem (C2/C5)
using Ipm_3_0_0 = IpmLaunch<3, 0, 0>;
using Ipm_6_1_2 = IpmLaunch<6, 1, 2>;
using Ipm_6_0_0 = IpmLaunch<6, 0, 0>;

bool ipm_dispatch(int n, int nf, int nl, int what, const DevModel *M, const DevFrame *F, const OcpConst &C,
                  const IpmArrays &A, int batch, hipStream_t s, double *w, int *status, int *iters, double *kkt,
                  double *obj) {
#define MF_CASE(NJ, NF, NL)                                                       \
    if (n == NJ && nf == NF && nl == NL) {                                        \
        if (what == 0) IpmLaunch<NJ, NF, NL>::init(M, F, C, A, batch, s);          \
        else if (what >= 10 && what <= 12) IpmLaunch<NJ, NF, NL>::iter(what - 10, M, F, C, A, batch, s); \
        else IpmLaunch<NJ, NF, NL>::output(C, A, batch, w, status, iters, kkt, obj, s); \
        return true;                                                              \
    }
    MF_CASE(3, 0, 0)
    MF_CASE(6, 1, 2)
    MF_CASE(6, 0, 0)
#undef MF_CASE
    return false;
}

}  // namespace mf

#ifdef MF_PHASE_STAMPS
extern "C" int mf_debug_phase_stamps(unsigned long long *out, int nprob) {
    if (nprob > 4096) nprob = 4096;
    return hipMemcpyFromSymbol(out, HIP_SYMBOL(mf::mf_stamp_buf), sizeof(unsigned long long) * 16 * nprob) == hipSuccess ? 0 : -1;
}
#endif
