// Batched interior-point solve of the fatigue-aware OCP on MI355X (gfx950).
//
// One IPM iteration = two launches:
//   k_eval_node lanes (problem, node, direction v)   forward-over-reverse dual sweep
//               (adj.hpp): tau, line, cost, column v of their Jacobian and of the exact
//               Lagrangian Hessian; writes the condensed stage Hessian H0
//   k_ipm_iter  one wavefront per problem             optimality error, barrier update,
//               inertia-corrected Riccati recursion (Bunch-Kaufman stage blocks in LDS),
//               step recovery, fraction-to-boundary, l1-merit line search (node_values),
//               update.  Mirrors oracle/mf_oracle.c mfo_solve statement by statement.
// Model constants (URDF joint placements, inertias) are staged in LDS per
// workgroup; per-problem arrays are [problem][node][field] so a wave reading a
// node's data, and lanes (node, field) writing it, both touch contiguous bytes.
#include <hip/hip_runtime.h>

#include "adj.hpp"
#include "bk_wave.hpp"
#include "dyn.hpp"
#include "ipm.hpp"

namespace mf {

#define LINE_ON(k) ((k) >= 2)

__device__ __forceinline__ bool hasb(double b) { return isfinite(b); }

// primal-dual barrier Hessian of a scalar x in [lo, hi] (missing bound: +-inf, multiplier 0)
__device__ __forceinline__ double sigma_pair(double zL, double zU, double x, double lo, double hi) {
    double s = 0.0;
    if (hasb(lo)) s += zL / (x - lo);
    if (hasb(hi)) s += zU / (hi - x);
    return s;
}

// Diagnostic build only (-DMF_PHASE_STAMPS): per-phase cycle counts of k_ipm_iter,
// accumulated by lane 0 into a debug buffer (never read by the solver).
#ifdef MF_PHASE_STAMPS
__device__ unsigned long long mf_stamp_buf[32 * 4096];
// accumulated in registers (a global read-modify-write per stamp would wait, vmcnt being in
// order, for every prefetch in flight) and added to the buffer once per launch
#define STAMP(slot)                                                                   \
    do {                                                                              \
        unsigned long long t_ = __builtin_amdgcn_s_memtime();                         \
        stamp_acc_[slot] += t_ - t_prev_;                                             \
        t_prev_ = t_;                                                                 \
    } while (0)
#define STAMP_INIT                                                                    \
    unsigned long long stamp_acc_[32] = {0};                                          \
    unsigned long long t_prev_ = __builtin_amdgcn_s_memtime()
#define STAMP_COUNT(slot, v) do { stamp_acc_[slot] += (v); } while (0)
#define STAMP_FLUSH                                                                   \
    do {                                                                              \
        if (lane == 0 && b < 4096)                                                    \
            for (int s_ = 0; s_ < 32; s_++) mf_stamp_buf[b * 32 + s_] += stamp_acc_[s_]; \
    } while (0)
#else
#define STAMP(slot) do {} while (0)
#define STAMP_INIT do {} while (0)
#define STAMP_COUNT(slot, v) do {} while (0)
#define STAMP_FLUSH do {} while (0)
#endif

// IPOPT bound_push / bound_frac = 1e-2: move an initial value strictly inside its bounds
__device__ __forceinline__ double bound_push(double x, double lo, double hi) {
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
}

// Diagnostic build only (-DMF_TRACE): per-iteration record of the first 16 problems
// (16 doubles per iteration, read by mf_debug_trace; tools/trace_probe.py).
#ifdef MF_TRACE
__device__ double mf_trace_buf[16 * 512 * 16];
#define TRACE(slot, val)                                                                     \
    do {                                                                                     \
        if (lane == 0 && b < 16 && st.iter < 512) mf_trace_buf[(b * 512 + st.iter) * 16 + (slot)] = (val); \
    } while (0)
#else
#define TRACE(slot, val) do {} while (0)
#endif

// cooperative copy of a POD struct into LDS
template <class T> __device__ __forceinline__ void stage_lds(T *dst, const T *src) {
    const int words = (int)(sizeof(T) / sizeof(double));
    const double *s = reinterpret_cast<const double *>(src);
    double *d = reinterpret_cast<double *>(dst);
    for (int i = threadIdx.x; i < words; i += blockDim.x) d[i] = s[i];
}

// ============================================================== eval: node derivatives
// Lanes (problem, node, direction v), NV = 2 n + n_f lanes per node, NPB nodes per
// block.  Each lane runs node_fwd_rev<Dual> (adj.hpp) with tangent e_v and gets tau,
// column v of d tau / dw, the line Jacobian column and column v of the exact Hessian
// of phi = c.tau + yl.line, c = y_tau + 2 wtau tau.  The block exchanges the Jacobian
// columns through LDS to add the Gauss-Newton / barrier term and writes the condensed
// stage Hessian  H0_k = grad^2 L_k + J^T diag(2 wtau + Sigma_s) J + diag(Sigma_x)
// (what the Riccati recursion needs at delta_w = delta_c = 0).
template <int NJ, int NF> struct NodeIn {
    const double *xq, *xqd;
    int v;
    __device__ __forceinline__ Dual q(int i) const { return Dual(xq[i], v == i ? 1.0 : 0.0); }
    __device__ __forceinline__ Dual qd(int i) const { return Dual(xqd[i], v == NJ + i ? 1.0 : 0.0); }
};
template <int NJ, int NF, int NPB, int NV> struct NodeOut {
    double (*Js)[NJ][NV];  // LDS: Jacobian columns of the block's nodes
    double (*Hs)[NV][NV];  // LDS: Hessian columns of phi
    double (*Ts)[NJ];      // LDS: tau values
    int g, v;
    const double *fdir;
    double pfv[3], pfd[3];
    __device__ __forceinline__ void frame(const Dual *p) {
#pragma unroll
        for (int k = 0; k < 3; k++) { pfv[k] = p[k].v; pfd[k] = p[k].d; }
    }
    __device__ __forceinline__ void force(const Dual *gF) {
#pragma unroll
        for (int a = 0; a < NF; a++)
            Hs[g][2 * NJ + a][v] = fdir[3 * a] * gF[0].d + fdir[3 * a + 1] * gF[1].d + fdir[3 * a + 2] * gF[2].d;
    }
    __device__ __forceinline__ void joint(int i, const Dual &t, const Dual &gq, const Dual &gqd) {
        Js[g][i][v] = t.d;
        if (v == 0) Ts[g][i] = t.v;
        Hs[g][i][v] = gq.d;
        Hs[g][NJ + i][v] = gqd.d;
    }
};

template <int NJ, int NF, int NL>
__global__ __launch_bounds__(256) void k_eval_node(const DevModel *__restrict__ Mg, const DevFrame *__restrict__ Fg,
                                                   OcpConst C, IpmArrays A, int batch) {
    constexpr int NV = 2 * NJ + NF;
    constexpr int NFA = NF > 0 ? NF : 1;
    constexpr int NPB = 256 / NV;
    __shared__ DevModel M;
    __shared__ DevFrame F;
    __shared__ double Js[NPB][NJ][NV], Hs[NPB][NV][NV], Ts[NPB][NJ], Cs[NPB][NJ];
    stage_lds(&M, Mg);
    stage_lds(&F, Fg);
    const int tid = threadIdx.x, g = tid / NV, v = tid % NV;
    const int N = C.N;
    const long node = (long)blockIdx.x * NPB + g;
    bool run = (g < NPB) && node < (long)batch * N;
    int b = 0, k = 0;
    if (run) {
        b = (int)(node / N);
        k = (int)(node % N);
        run = A.st[b].status == ST_RUNNING;
    }
    const IpmSizes S = ipm_sizes(C);
    const double *q = A.q + b * S.q + (size_t)k * NJ;
    const double *qd = A.qd + b * S.u + (size_t)k * NJ;
    const double *Fv = A.F + b * S.f + (size_t)k * NFA;
    NodeOut<NJ, NF, NPB, NV> out;
    out.Js = Js;
    out.Hs = Hs;
    out.Ts = Ts;
    out.g = g;
    out.v = v;
    out.fdir = C.fdir;
    // torque weights c = y_tau + 2 wtau tau (tau at the iterate first when wtau != 0)
    if (run && v == 0) {
        const double *yd = A.yd + b * S.u + (size_t)k * NJ;
        if (C.wtau != 0.0) {
            struct WOut {
                double *c;
                const double *yd;
                double w2;
                __device__ void frame(const double *) {}
                __device__ void force(const double *) {}
                __device__ void joint(int j, double t, double, double) { c[j] = yd[j] + w2 * t; }
            } wo{Cs[g], yd, 2.0 * C.wtau};
            double Fw[3];
#pragma unroll
            for (int r = 0; r < 3; r++) {
                double acc = 0.0;
#pragma unroll
                for (int a = 0; a < NF; a++) acc += Fv[a] * C.fdir[3 * a + r];
                Fw[r] = acc;
            }
            ArrIn<NJ> in0{q, qd};
            node_values<NJ>(M, F, (NF > 0 || NL > 0) ? F.parent : -1, in0, Fw, wo);
        } else {
#pragma unroll
            for (int j = 0; j < NJ; j++) Cs[g][j] = yd[j];
        }
    }
    __syncthreads();
    if (run) {
        double yl3[3] = {0.0, 0.0, 0.0};
#pragma unroll
        for (int l = 0; l < NL; l++) yl3[l] = A.yl[b * S.l + (size_t)k * NL + l];
        Dual Fw[3];
#pragma unroll
        for (int r = 0; r < 3; r++) {
            Dual acc(0.0);
#pragma unroll
            for (int a = 0; a < NF; a++) acc += Dual(Fv[a], v == 2 * NJ + a ? 1.0 : 0.0) * C.fdir[3 * a + r];
            Fw[r] = acc;
        }
        const int fp = (NF > 0 || NL > 0) ? F.parent : -1;
        NodeIn<NJ, NF> in{q, qd, v};
        node_fwd_rev<Dual, NJ>(M, F, fp, in, Fw, Cs[g], yl3, out);
    }
    __syncthreads();
    if (!run) return;
    // barrier Hessian of the node: Sigma_s (torque slacks), Sigma_x (q_k, qd_k bounds, k >= 1)
    const double *tlo = A.tau_lo + (size_t)k * NJ, *thi = A.tau_hi + (size_t)k * NJ;
    const double *sk = A.s + b * S.u + (size_t)k * NJ;
    const double *vL = A.vL + b * S.u + (size_t)k * NJ, *vU = A.vU + b * S.u + (size_t)k * NJ;
    double wj[NJ];
#pragma unroll
    for (int j = 0; j < NJ; j++) wj[j] = 2.0 * C.wtau + sigma_pair(vL[j], vU[j], sk[j], tlo[j], thi[j]);
    double diag = 0.0;
    if (k > 0) {
        if (v < NJ) {
            const size_t e = b * S.q + (size_t)k * NJ + v;
            diag = sigma_pair(A.zqL[e], A.zqU[e], q[v], C.q_lo[v], C.q_hi[v]);
        } else if (v < 2 * NJ) {
            const size_t e = b * S.u + (size_t)k * NJ + v - NJ;
            diag = sigma_pair(A.zdL[e], A.zdU[e], qd[v - NJ], C.qd_lo[v - NJ], C.qd_hi[v - NJ]);
        }
    }
    if (v >= NJ && v < 2 * NJ) diag += 2.0 * C.wqd;
    if (v >= 2 * NJ) diag += 2.0 * C.wF;
    double *W = A.W + b * S.w + (size_t)k * NV * NV;
#pragma unroll
    for (int u = 0; u < NV; u++) {
        if (u < v) continue;
        double gn = 0.0;
#pragma unroll
        for (int j = 0; j < NJ; j++) gn += wj[j] * Js[g][j][u] * Js[g][j][v];
        double hh = Hs[g][u][v] + gn;
        if (u == v) hh += diag;
        W[u * NV + v] = hh;
        W[v * NV + u] = hh;
    }
    double *Jt = A.Jt + b * S.jt + (size_t)k * NJ * NV;
    double gfv = 0.0;
#pragma unroll
    for (int j = 0; j < NJ; j++) {
        const double jv = Js[g][j][v];
        Jt[j * NV + v] = jv;
        gfv += 2.0 * C.wtau * Ts[g][j] * jv;
    }
    if (v >= NJ && v < 2 * NJ) gfv += 2.0 * C.wqd * qd[v - NJ];
    if (NF > 0 && v >= 2 * NJ) gfv += 2.0 * C.wF * Fv[v - 2 * NJ];
    A.gf[b * S.gf + (size_t)k * NV + v] = gfv;
    if (NL > 0 && v < NJ) {
        double *Jl = A.Jl + b * S.jl + (size_t)k * NL * NJ;
#pragma unroll
        for (int l = 0; l < NL; l++) Jl[l * NJ + v] = out.pfd[l];
    }
    if (v == 0) {
        double *tvo = A.tau + b * S.u + (size_t)k * NJ;
        double c = 0.0;
#pragma unroll
        for (int a = 0; a < NF; a++) c += C.wF * Fv[a] * Fv[a];
#pragma unroll
        for (int j = 0; j < NJ; j++) {
            const double tj = Ts[g][j];
            tvo[j] = tj;
            c += C.wqd * qd[j] * qd[j] + C.wtau * tj * tj;
        }
        A.cost[b * S.cost + k] = c;
        if (NL > 0) {
            double *lv = A.line + b * S.l + (size_t)k * NL;
#pragma unroll
            for (int l = 0; l < NL; l++) lv[l] = out.pfv[l] - A.lref[b * 2 + l];
        }
    }
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
    for (int e = lane; e < (N + 1) * NJ; e += 64) {
        int k = e / NJ, j = e % NJ;
        q[e] = (k == 0) ? q0[j] : bound_push(q0[j], C.q_lo[j], C.q_hi[j]);
        A.zqL[b * S.q + e] = (k > 0 && hasb(C.q_lo[j])) ? 1.0 : 0.0;
        A.zqU[b * S.q + e] = (k > 0 && hasb(C.q_hi[j])) ? 1.0 : 0.0;
    }
    for (int e = lane; e < N * NJ; e += 64) {
        int k = e / NJ, j = e % NJ;
        qd[e] = (k == 0) ? C.qd0[j] : bound_push(0.0, C.qd_lo[j], C.qd_hi[j]);
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
    struct SlackOut {
        double *s;
        const double *lo, *hi;
        __device__ void frame(const double *) {}
        __device__ void force(const double *) {}
        __device__ void joint(int j, double t, double, double) { s[j] = bound_push(t, lo[j], hi[j]); }
    };
    const int fp = (NF > 0 || NL > 0) ? F.parent : -1;
    for (int k = lane; k < N; k += 64) {
        double Fw[3];
#pragma unroll
        for (int r = 0; r < 3; r++) {
            double acc = 0.0;
#pragma unroll
            for (int a = 0; a < NF; a++) acc += Fv[(size_t)k * NFA + a] * C.fdir[3 * a + r];
            Fw[r] = acc;
        }
        ArrIn<NJ> in{q + (size_t)k * NJ, qd + (size_t)k * NJ};
        SlackOut so{s + (size_t)k * NJ, A.tau_lo + (size_t)k * NJ, A.tau_hi + (size_t)k * NJ};
        node_values<NJ>(M, F, fp, in, Fw, so);
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
// line-search trial point x + alpha dx, read on use by node_values
struct TrialIn {
    const double *xq, *dxq, *xqd, *dxqd;
    double al;
    __device__ double q(int i) const { return xq[i] + al * dxq[i]; }
    __device__ double qd(int i) const { return xqd[i] + al * dxqd[i]; }
};
// accumulates wtau |tau|^2, |tau - s| on the bounded torque rows and |p - ref| on the line
struct MeritOut {
    const double *s, *ds, *tlo, *thi, *lref;
    double al, wtau, c, th;
    int nl;
    bool line;
    __device__ void frame(const double *p) {
        if (line)
            for (int l = 0; l < nl; l++) th += fabs(p[l] - lref[l]);
    }
    __device__ void force(const double *) {}
    __device__ void joint(int j, double t, double, double) {
        c += wtau * t * t;
        if (hasb(tlo[j]) || hasb(thi[j])) th += fabs(t - (s[j] + al * ds[j]));
    }
};


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
    __shared__ double Dd_s[NJ], Ss_s[NJ], rdd_s[NJ];
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
    TRACE(0, dinf); TRACE(1, pinf); TRACE(2, cinf0); TRACE(3, mu);
#ifdef MF_TRACE
    {
        double f = 0.0;
        for (int k = lane; k < N; k += 64) f += cost[k];
        f = wave_sum(f);
        TRACE(14, f);
    }
#endif
    double Emu = fmax(fmax(dinf / sd, pinf), cinfm / sc);
    st.E0 = E0;
    st.cviol = pinf;
    auto finish = [&](int status) {
        STAMP_FLUSH;
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
    TRACE(4, mu);
    STAMP(0);

    // ---------------- barrier Sigma and gradients
    for (int e = lane; e < (N + 1) * n; e += 64) {
        int k = e / n, j = e % n;
        double sx = 0, gp = 0;
        if (k > 0) {
            double x = q[e];
            sx = sigma_pair(zqL[e], zqU[e], x, QLO[j], QHI[j]);
            if (hasb(QLO[j])) gp -= mu / (x - QLO[j]);
            if (hasb(QHI[j])) gp += mu / (QHI[j] - x);
        }
        Sxq[e] = sx; gphq[e] = gp;
    }
    for (int e = lane; e < N * n; e += 64) {
        int k = e / n, j = e % n;
        double sx = 0, gp = 0, ss = 0, gs = 0;
        if (k > 0) {
            double x = qd[e];
            sx = sigma_pair(zdL[e], zdU[e], x, DLO[j], DHI[j]);
            if (hasb(DLO[j])) gp -= mu / (x - DLO[j]);
            if (hasb(DHI[j])) gp += mu / (DHI[j] - x);
        }
        double x = s[e];
        ss = sigma_pair(vL[e], vU[e], x, tlo[e], thi[e]);
        if (hasb(tlo[e])) gs -= mu / (x - tlo[e]);
        if (hasb(thi[e])) gs += mu / (thi[e] - x);
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
    //
    // Latency layout: everything a stage needs that does not depend on the recursion (the
    // gradient g_k, c_k, e_k = line_{k+1} + Jl_{k+1} c_k) is computed for all stages at once by
    // the whole wave into LDS; the stage Hessian H0_k and Jl_{k+1} are prefetched into registers
    // one stage ahead, so the serial chain itself issues no dependent global load.
    constexpr int NU = NJ + NF;
    constexpr int NK = NU + NL;
    constexpr int LDK = NK + 1;
    constexpr int NRK = NJ + 1;
    constexpr int NLA2 = NL > 0 ? NL : 1;
    constexpr int NVV = NV * NV;
    constexpr int NHR = (NVV + 63) / 64;     // H entries per lane
    constexpr int SLOT = MB * NJ + MB;       // Riccati slot (G_k | wv_k) doubles
    constexpr int NSR = (SLOT + 63) / 64;
    __shared__ double Hs[NVV];
    __shared__ double Ps[NJ * NJ], ps[NJ], ss[NJ], Pn[NJ * NJ];
    __shared__ double Ks[NK * LDK], Rk[NK * NRK], Yk[NK * NRK];
    __shared__ double Gl[NLA2 * NJ];
    __shared__ double xs[NJ], us[NU + NLA2], cs[NJ];
    __shared__ double Sl[SLOT];
    __shared__ double Jl_s[NJ * NV];  // J_k (torque Jacobian) of the stage, regularised tries only
    extern __shared__ double dyn_lds[];
    double *gst = dyn_lds;                    // N x NV   stage gradients g_k
    double *cst = gst + (size_t)N * NV;       // N x NJ   c_k = q_k + h qd_k - q_{k+1}
    double *est = cst + (size_t)N * NJ;       // N x NLA2 e_k = line_{k+1} + Jl_{k+1} c_k
    double *wst = est + (size_t)N * NLA2;     // N x NJ   y_tau + D_tau r_tau (torque rows)
    double *dst = wst + (size_t)N * NJ;       // N x NJ   D_tau(dw, dc) - Sigma_s (0 unless dw, dc != 0)
    // g_k for all stages at the current (dw, dc): exactly the primal rows of the KKT right-hand side
    auto prep_stages = [&](double dwv, double dcv) {
        for (int e = lane; e < N * n; e += 64) {
            const int k = e / n, j = e % n;
            double wv_ = yd[e], dD = 0.0;
            if (TACT(k, j)) {
                const double sg = Ss[e] + dwv;
                const double Dd = sg / (1.0 + dcv * sg);
                wv_ += Dd * ((tau[e] - s[e]) + (gphs[e] - yd[e]) / sg);
                dD = Dd - Ss[e];
            }
            wst[e] = wv_;
            dst[e] = dD;
            cst[e] = q[e] + h * qd[e] - q[e + n];
        }
        wave_lds_sync();
        for (int e = lane; e < N * NV; e += 64) {
            const int k = e / NV, u = e % NV;
            double g = gf[e];
            const double *Jtk = Jt + (size_t)k * n * NV;
#pragma unroll
            for (int jj = 0; jj < NJ; jj++) g += Jtk[jj * NV + u] * wst[k * n + jj];
            if (u < n) {
                g += gphq[k * n + u] + yc[k * n + u] - (k > 0 ? yc[(k - 1) * n + u] : 0.0);
#pragma unroll
                for (int l = 0; l < NL; l++) g += Jl[(k * nl + l) * n + u] * yl[k * nl + l];
            } else if (u < 2 * n) {
                g += gphd[k * n + u - n] + h * yc[k * n + u - n];
            }
            gst[e] = g;
        }
        for (int e = lane; e < N * nl; e += 64) {
            const int k = e / nl, l = e % nl;
            double a = 0.0;
            if (LINE_ON(k + 1) && k + 1 <= N - 1) {
                a = line[(k + 1) * nl + l];
#pragma unroll
                for (int i = 0; i < NJ; i++) a += Jl[((size_t)(k + 1) * nl + l) * n + i] * cst[k * n + i];
            }
            est[k * NLA2 + l] = a;
        }
        wave_lds_sync();
    };
    double dw = 0.0, dc = 0.0, dFr = 0.0;
    const int reg_tier0 = st.reg_tier;
    const double reg_last0 = st.reg_last;
    int tier = reg_tier0, step_no = 0;
    double reg = (reg_tier0 == 0) ? 0.0 : reg_last0 / 3.0;
    if (reg_tier0 != 0 && reg < 1e-8) { tier = 0; reg = 0.0; }
    if (tier == 1) dFr = reg; else if (tier == 2) dw = reg;
    bool factor_ok = false;
    int ntries = 0;
    double prep_dw = NAN, prep_dc = NAN;
    for (int tries = 0; tries < 60; tries++) {
        ntries++;
        bool ok = true, zero = false;
        if (!(dw == prep_dw && dc == prep_dc)) {
            prep_stages(dw, dc);
            prep_dw = dw;
            prep_dc = dc;
        }
        const bool dreg = (dw != 0.0 || dc != 0.0);
        // terminal value function V_N = 1/2 x^T P x + p^T x
        for (int e = lane; e < n * n; e += 64) {
            int i = e / n, j = e % n;
            Ps[e] = (i == j) ? Sxq[N * n + i] + dw : 0.0;
        }
        for (int j = lane; j < n; j += 64) ps[j] = gphq[N * n + j] - yc[(N - 1) * n + j];
        // prefetch H0_{N-1} (and J_{N-1} when the torque block is regularised)
        constexpr int NJV = NJ * NV, NJR = (NJV + 63) / 64;
        double hr[NHR], jr[NJR];
#pragma unroll
        for (int t = 0; t < NHR; t++) {
            const int e = lane + 64 * t;
            hr[t] = (e < NVV) ? W[(size_t)(N - 1) * NVV + e] : 0.0;
        }
#pragma unroll
        for (int t = 0; t < NJR; t++) {
            const int e = lane + 64 * t;
            jr[t] = (dreg && e < NJV) ? Jt[(size_t)(N - 1) * NJV + e] : 0.0;
        }
        double glr = 0.0;  // Jl_{k+1} entry of this lane for the next stage
        wave_lds_sync();
        for (int k = N - 1; k >= 0; k--) {
            // ---- H_k = H0_k (+ regularisation) into LDS; prefetch H0_{k-1}, Jl_k (, J_{k-1})
            if (dreg) {
#pragma unroll
                for (int t = 0; t < NJR; t++) {
                    const int e = lane + 64 * t;
                    if (e < NJV) Jl_s[e] = jr[t];
                }
                wave_lds_sync();
            }
            const double *dDk = dst + (size_t)k * n;
#pragma unroll
            for (int t = 0; t < NHR; t++) {
                const int e = lane + 64 * t;
                if (e < NVV) {
                    const int u = e / NV, v = e % NV;
                    double a = hr[t];
                    if (dreg)
#pragma unroll
                        for (int jj = 0; jj < NJ; jj++) a += Jl_s[jj * NV + u] * dDk[jj] * Jl_s[jj * NV + v];
                    if (u == v) a += dw + (u >= 2 * n ? dFr : 0.0);
                    Hs[e] = a;
                }
            }
            if (lane < nl * n) Gl[lane] = glr;
            STAMP(7);
            if (k > 0) {
#pragma unroll
                for (int t = 0; t < NHR; t++) {
                    const int e = lane + 64 * t;
                    hr[t] = (e < NVV) ? W[(size_t)(k - 1) * NVV + e] : 0.0;
                }
                glr = (lane < nl * n) ? Jl[(size_t)k * nl * n + lane] : 0.0;
                if (dreg)
#pragma unroll
                    for (int t = 0; t < NJR; t++) {
                        const int e = lane + 64 * t;
                        jr[t] = (e < NJV) ? Jt[(size_t)(k - 1) * NJV + e] : 0.0;
                    }
            }
            // s = P c + p ; keep P_{k+1}, p_{k+1} for the forward sweep
            double *Gk = G + (size_t)k * MB * n, *wk = wv + (size_t)k * MB;
            const double *ck = cst + (size_t)k * n;
            if (lane < n) {
                const int j = lane;
                double a = ps[j];
#pragma unroll
                for (int i = 0; i < NJ; i++) a += Ps[j * n + i] * ck[i];
                ss[j] = a;
                wk[NU + NL + j] = ps[j];
            }
            for (int e = lane; e < n * n; e += 64) Gk[(NU + NL) * n + e] = Ps[e];
            wave_lds_sync();
            STAMP(11);
            const double *gsk = gst + (size_t)k * NV;
            if (k == 0) {
                // only dF_0 is free (q_0, qd_0 fixed; the stage-1 line constraint is masked)
                if (nf > 0) {
                    for (int e = lane; e < nf * nf; e += 64) Ks[(e / nf) * LDK + e % nf] = Hs[(2 * n + e / nf) * NV + 2 * n + e % nf];
                    for (int a = lane; a < nf; a += 64) Rk[a * NRK] = -gsk[2 * n + a];
                    wave_lds_sync();
                    BKInertia in = bk_factor_fixed<LDK, NFA>(Ks, perm, piv);
                    if (in.zero) { ok = false; zero = true; break; }
                    if (in.pos != nf) { ok = false; break; }
                    bk_solve_cols<LDK, NRK, NFA>(Ks, perm, piv, Rk, 1);
                    for (int a = lane; a < nf; a += 64) wk[NJ + a] = Rk[a * NRK];  // dF_0 (ku slot)
                }
                wave_lds_sync();
                break;
            }
            const bool con = (nl > 0) && LINE_ON(k + 1) && (k + 1 <= N - 1);
            const double *elk = est + (size_t)k * NLA2;
            // ---- stage block [[Quu, Du^T], [Du, -dc]] and right-hand sides -[Qux | qu ; G | e]
            // Block rows order the controls as (F, qd): with active torque bounds the force
            // carries the large curvature Sigma_s (J^T F)^2 and the joint velocities couple to it
            // weakly, so natural-order 1x1 pivots pass the Bunch-Kaufman test (ldl_schur_regs).
            // uo(a): control index (qd 0..n-1, F n..) of block row a < NU.
            auto uo = [&](int a) { return a < NF ? NJ + a : a - NF; };
            for (int e = lane; e < NK * NK; e += 64) {
                int a = e / NK, c = e % NK;
                double val;
                if (a < NU && c < NU) {
                    const int ua = uo(a), uc = uo(c);
                    val = Hs[(n + ua) * NV + n + uc];
                    if (ua < n && uc < n) val += h * h * Ps[ua * n + uc];
                } else if (a >= NU && c >= NU) {
                    val = (a == c) ? (con ? -dc : -1.0) : 0.0;
                } else {
                    int l = (a >= NU) ? a - NU : c - NU, v = uo((a >= NU) ? c : a);
                    val = (con && v < n) ? h * Gl[l * n + v] : 0.0;
                }
                Ks[a * LDK + c] = val;
            }
            for (int e = lane; e < NK * NRK; e += 64) {
                int a = e / NRK, c = e % NRK;
                double val;
                if (a < NU) {
                    const int ua = uo(a);
                    if (c < n) val = -(Hs[(n + ua) * NV + c] + (ua < n ? h * Ps[ua * n + c] : 0.0));
                    else val = -(gsk[n + ua] + (ua < n ? h * ss[ua] : 0.0));
                } else {
                    int l = a - NU;
                    val = con ? -(c < n ? Gl[l * n + c] : elk[l]) : 0.0;
                }
                Rk[e] = val;
            }
            wave_lds_sync();
            STAMP(12);
            BKInertia in;
            const bool fast = ldl_schur_regs<LDK, NRK, NU, NL>(Ks, Rk, NRK, in);
            STAMP(13);
            STAMP_COUNT(16, fast ? 0 : 1);
            STAMP_COUNT(17, 1);
            if (fast) {
                if (in.pos != NU || in.neg != NL) { ok = false; break; }
            } else {
                in = bk_factor_fixed<LDK, NK>(Ks, perm, piv);
                if (in.zero) { ok = false; zero = true; break; }
                if (in.pos != NU || in.neg != NL) { ok = false; break; }
                bk_solve_cols<LDK, NRK, NK>(Ks, perm, piv, Rk, NRK);
            }
            STAMP(14);
            // ---- P_k = Qxx + Qxu Ku + G^T Kl ; p_k = qx + Qxu ku + G^T kl   (block row a <-> control uo(a))
            for (int e = lane; e < n * n; e += 64) {
                int i = e / n, j = e % n;
                double a = Hs[i * NV + j] + Ps[i * n + j];
                for (int r = 0; r < NU; r++) {
                    const int c = uo(r);
                    a += (Hs[i * NV + n + c] + (c < n ? h * Ps[i * n + c] : 0.0)) * Rk[r * NRK + j];
                }
                if (con)
                    for (int l = 0; l < nl; l++) a += Gl[l * n + i] * Rk[(NU + l) * NRK + j];
                Pn[e] = a;
            }
            double pnew = 0.0;
            if (lane < n) {
                int i = lane;
                pnew = gsk[i] + ss[i];
                for (int r = 0; r < NU; r++) {
                    const int c = uo(r);
                    pnew += (Hs[i * NV + n + c] + (c < n ? h * Ps[i * n + c] : 0.0)) * Rk[r * NRK + n];
                }
                if (con)
                    for (int l = 0; l < nl; l++) pnew += Gl[l * n + i] * Rk[(NU + l) * NRK + n];
            }
            // slot rows in control order (qd 0..n-1, F, then the NL line multipliers)
            auto brow = [&](int c) { return c < NU ? (c < NJ ? NF + c : c - NJ) : c; };
            for (int e = lane; e < NK * n; e += 64) Gk[e] = Rk[brow(e / n) * NRK + e % n];  // Ku (NU x n), Kl (NL x n)
            for (int a = lane; a < NK; a += 64) wk[a] = Rk[brow(a) * NRK + n];              // ku, kl
            wave_lds_sync();
            for (int e = lane; e < n * n; e += 64) {
                int i = e / n, j = e % n;
                Ps[e] = 0.5 * (Pn[e] + Pn[j * n + i]);
            }
            if (lane < n) ps[lane] = pnew;
            wave_lds_sync();
            STAMP(15);
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
    TRACE(5, dFr); TRACE(6, dw); TRACE(7, dc); TRACE(8, (double)ntries);
    if (!factor_ok) { finish(ST_INERTIA); return; }
    st.reg_tier = tier;
    st.reg_last = reg;

    wave_mem_sync();  // the Riccati slots stored above are read back by other lanes below
    // ---------------- forward sweep: du_k = Ku dx_k + ku, dyl_{k+1} = Kl dx_k + kl,
    //                  dyc_k = P_{k+1} dx_{k+1} + p_{k+1} + Jl_{k+1}^T dyl_{k+1}
    // (the node-(k+1) line constraint was pushed back onto stage k, so V_{k+1} does not contain
    // it but the q_{k+1} row of the KKT does).  Slot k+1 is prefetched while stage k runs.
    double sr[NSR];
#pragma unroll
    for (int t = 0; t < NSR; t++) {
        const int e = lane + 64 * t;
        sr[t] = (e < SLOT) ? ((e < MB * NJ) ? G[e] : wv[e - MB * NJ]) : 0.0;  // slot 0
    }
    for (int j = lane; j < n; j += 64) {
        dq[j] = 0.0; dqd[j] = 0.0;
        xs[j] = cst[j];  // dx_1 = c_0 (dx_0 = 0, dqd_0 = 0)
    }
    for (int l = lane; l < nl; l += 64) { dyl[l] = 0.0; dyl[nl + l] = 0.0; }
    for (int k = 0; k < N; k++) {
        // slot k -> LDS; prefetch slot k+1
#pragma unroll
        for (int t = 0; t < NSR; t++) {
            const int e = lane + 64 * t;
            if (e < SLOT) Sl[e] = sr[t];
        }
        if (k + 1 < N) {
            const double *Gn = G + (size_t)(k + 1) * MB * n, *wn = wv + (size_t)(k + 1) * MB;
#pragma unroll
            for (int t = 0; t < NSR; t++) {
                const int e = lane + 64 * t;
                sr[t] = (e < SLOT) ? ((e < MB * NJ) ? Gn[e] : wn[e - MB * NJ]) : 0.0;
            }
        }
        wave_lds_sync();
        const double *Gk = Sl, *wk = Sl + MB * NJ;
        if (k == 0) {
            for (int a = lane; a < nf; a += 64) dF[a] = wk[NJ + a];
            for (int j = lane; j < n; j += 64) {  // dyc_0 = P_1 dx_1 + p_1 (stage-1 line is masked)
                double a = wk[NU + NL + j];
                for (int i = 0; i < n; i++) a += Gk[(NU + NL) * n + j * n + i] * xs[i];
                dyc[j] = a;
            }
            wave_lds_sync();
            continue;
        }
        for (int a = lane; a < NK; a += 64) {
            double v = wk[a];
            for (int i = 0; i < n; i++) v += Gk[a * n + i] * xs[i];
            us[a] = v;
        }
        for (int j = lane; j < n; j += 64) dq[k * n + j] = xs[j];
        wave_lds_sync();
        for (int j = lane; j < n; j += 64) {
            dqd[k * n + j] = us[j];
            cs[j] = xs[j] + h * us[j] + cst[k * n + j];
        }
        for (int a = lane; a < nf; a += 64) dF[k * NFA + a] = us[NJ + a];
        const bool con1 = (nl > 0) && LINE_ON(k + 1) && (k + 1 <= N - 1);
        if (k + 1 < N)
            for (int l = lane; l < nl; l += 64) dyl[(k + 1) * nl + l] = con1 ? us[NU + l] : 0.0;
        wave_lds_sync();
        for (int j = lane; j < n; j += 64) {
            double a = wk[NU + NL + j];
            for (int i = 0; i < n; i++) a += Gk[(NU + NL) * n + j * n + i] * cs[i];
            if (con1)
                for (int l = 0; l < nl; l++) a += Jl[((size_t)(k + 1) * nl + l) * n + j] * us[NU + l];
            dyc[k * n + j] = a;
            xs[j] = cs[j];
        }
        wave_lds_sync();
    }
    for (int j = lane; j < n; j += 64) dq[N * n + j] = xs[j];
    __threadfence_block();
    __syncthreads();

    // ---------------- dyd, ds, dz, dv
    double pcorr = 0.0;  // sum Sigma_s (ds^2 - (J dx)^2): turns p^T H0 p into the oracle's p^T (W + Sigma) p
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
        pcorr += Ss[i] * (ds[i] * ds[i] - jdx * jdx);
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
    TRACE(9, ap); TRACE(10, az);

    // ---------------- merit at the current point, directional derivative, curvature
    // merit of a point (x + alpha dx); alpha = 0 uses the stored node values
    const int fpj = (NF > 0 || NL > 0) ? F.parent : -1;
    auto merit = [&](double alpha, double &phi, double &theta, bool &ok_out) {
        double f = 0, bar = 0, th = 0;
        int bad = 0;
        for (int k = lane; k < N; k += 64) {
            double Fw[3], c = 0.0;
#pragma unroll
            for (int r = 0; r < 3; r++) Fw[r] = 0.0;
#pragma unroll
            for (int a = 0; a < NF; a++) {
                const double tF = Fv[k * NFA + a] + alpha * dF[k * NFA + a];
                c += C.wF * tF * tF;
#pragma unroll
                for (int r = 0; r < 3; r++) Fw[r] += tF * C.fdir[3 * a + r];
            }
            TrialIn tin{q + (size_t)k * n, dq + (size_t)k * n, qd + (size_t)k * n, dqd + (size_t)k * n, alpha};
            MeritOut mo{s + (size_t)k * n, ds + (size_t)k * n, tlo + (size_t)k * n, thi + (size_t)k * n, lref,
                        alpha, C.wtau, 0.0, 0.0, nl, LINE_ON(k)};
            node_values<NJ>(M, F, fpj, tin, Fw, mo);
#pragma unroll
            for (int j = 0; j < NJ; j++) {
                const double tq = q[k * n + j] + alpha * dq[k * n + j], tqd = qd[k * n + j] + alpha * dqd[k * n + j];
                const double qn = q[(k + 1) * n + j] + alpha * dq[(k + 1) * n + j];
                c += C.wqd * tqd * tqd;
                th += fabs(tq + h * tqd - qn);
            }
            f += c + mo.c;
            th += mo.th;
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
    // merit at the current point through the same value sweep as the trial points, so that
    // m(alpha) - m(0) carries no round-off mismatch between two code paths
    double phi0, th0;
    {
        bool ok0;
        merit(0.0, phi0, th0, ok0);
    }
    double gdot = 0, pHp = pcorr;
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
    for (int e = lane; e < N * n; e += 64) gdot += gphd[e] * dqd[e] + gphs[e] * ds[e];
    for (int e = n + lane; e < (N + 1) * n; e += 64) {
        gdot += gphq[e] * dq[e];
        if (e >= N * n) pHp += Sxq[e] * dq[e] * dq[e];  // q_N (stages k < N carry Sigma_x in H0)
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
    TRACE(11, alpha); TRACE(12, accepted ? 1.0 : 0.0); TRACE(13, nu); TRACE(15, (double)nls);
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
    STAMP_FLUSH;
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
    // phase 0: node derivatives (k_eval_node), 1: per-problem IPM step (k_ipm_iter)
    static void iter(int phase, const DevModel *M, const DevFrame *F, const OcpConst &C, const IpmArrays &A,
                     int batch, hipStream_t s) {
        constexpr int NV = 2 * NJ + NF;
        constexpr int NPB = 256 / NV;
        long nodes = (long)batch * C.N;
        if (phase == 0)
            hipLaunchKernelGGL((k_eval_node<NJ, NF, NL>), dim3((unsigned)((nodes + NPB - 1) / NPB)), dim3(256), 0, s,
                               M, F, C, A, batch);
        else {
            const size_t dyn = ipm_dyn_lds(C.N);
            if (dyn > 64 * 1024)
                (void)hipFuncSetAttribute((const void *)k_ipm_iter<NJ, NF, NL>,
                                          hipFuncAttributeMaxDynamicSharedMemorySize, (int)dyn);
            hipLaunchKernelGGL((k_ipm_iter<NJ, NF, NL>), dim3(batch), dim3(64), dyn, s, M, F, C, A, batch);
        }
    }
    // dynamic LDS of k_ipm_iter: per-stage g_k (NV), c_k (NJ), e_k (NL), y_tau + D r_tau (NJ), dD (NJ)
    static size_t ipm_dyn_lds(int N) {
        constexpr int NV = 2 * NJ + NF;
        return (size_t)N * (NV + 3 * NJ + (NL > 0 ? NL : 1)) * sizeof(double);
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
        else if (what >= 10 && what <= 11) IpmLaunch<NJ, NF, NL>::iter(what - 10, M, F, C, A, batch, s); \
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

#ifdef MF_TRACE
extern "C" int mf_debug_trace(double *out, int nprob) {
    if (nprob > 16) nprob = 16;
    return hipMemcpyFromSymbol(out, HIP_SYMBOL(mf::mf_trace_buf), sizeof(double) * 512 * 16 * nprob) == hipSuccess ? 0 : -1;
}
#endif

#ifdef MF_PHASE_STAMPS
extern "C" int mf_debug_phase_stamps(unsigned long long *out, int nprob) {
    if (nprob > 4096) nprob = 4096;
    return hipMemcpyFromSymbol(out, HIP_SYMBOL(mf::mf_stamp_buf), sizeof(unsigned long long) * 32 * nprob) == hipSuccess ? 0 : -1;
}
#endif
