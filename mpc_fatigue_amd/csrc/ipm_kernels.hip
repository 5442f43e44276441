// Batched interior-point solve of the fatigue-aware OCP on MI355X (gfx950).
//
// One IPM iteration = six launches (IpmLaunch::iter):
//   k_eval_node<CLS> lanes (problem, node, direction v)   forward-over-reverse dual sweep
//               (adj.hpp): tau, line, cost, column v of their Jacobian and of the exact
//               Lagrangian Hessian; one launch per direction class (CLS 0: the q directions,
//               dual pose; CLS 1: the qd directions, plain-FP64 pose -- its own register
//               allocation, not the q class's)
//   k_eval_asm  lanes (problem, node, column)          condensed stage Hessian H0, grad f
//   k_ipm_pre / k_ipm_kkt / k_ipm_post  one wavefront per problem: optimality error and
//               barrier update; inertia-corrected Riccati recursion (null-space or
//               Bunch-Kaufman stage solves in LDS) and step recovery; fraction-to-boundary,
//               l1-merit line search (node_values) and update.  Together they mirror
//               oracle/mf_oracle.c mfo_solve statement by statement.
// Model constants (URDF joint placements, inertias) are staged in LDS per
// workgroup; per-problem arrays are [problem][node][field] so a wave reading a
// node's data, and lanes (node, field) writing it, both touch contiguous bytes.
#include <hip/hip_runtime.h>

#include "adj.hpp"
#include "bk_wave.hpp"
#include "dyn.hpp"
#include "ipm.hpp"
#include "stage_ns.hpp"

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

// IPOPT bound_push / bound_frac = 1e-2 (warm_start_bound_push / _frac = 1e-3 for a warm start): move an
// initial value strictly inside its bounds
__device__ __forceinline__ double bound_push(double x, double lo, double hi, double k1 = 1e-2) {
    const double k2 = k1;
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

// LDS image of a DevModel holding only its first NJ joints (the kernels of an NJ-joint
// instantiation never index past joint NJ-1): 0.4 KB per joint instead of the full
// MF_MAX_JOINTS table, which keeps more workgroups resident per CU.
template <int NJ> struct ModelLds {
    static constexpr int WORDS = (int)((offsetof(DevModel, j) + NJ * sizeof(DevJoint) + sizeof(double) - 1) / sizeof(double));
    double w[WORDS];
    __device__ __forceinline__ void load(const DevModel *g) {
        const double *s = reinterpret_cast<const double *>(g);
        for (int i = threadIdx.x; i < WORDS; i += blockDim.x) w[i] = s[i];
    }
    __device__ __forceinline__ const DevModel &get() const { return *reinterpret_cast<const DevModel *>(w); }
};

// ============================================================== eval: node derivatives
// Lanes (problem, node, direction v), NVL = 2 n lanes per node (the q and qd directions),
// NPB nodes per block.  Each lane runs node_fwd_rev<Dual> (adj.hpp) with tangent e_v and
// gets tau, column v of d tau / dw, the line Jacobian column and column v of the exact
// Hessian of phi = c.tau + yl.line, c = y_tau + 2 wtau tau.  The force directions need no
// lane of their own: phi is linear in F, so the force row of the Hessian comes out of the
// q / qd lanes (symmetry), H_FF = 0, and d tau / dF_a = -J_f^T fdir_a = -(fdir_a . dp_f/dq_j)
// is the frame-point tangent of the q lanes.  The block exchanges the Jacobian
// columns through LDS to add the Gauss-Newton / barrier term and writes the condensed
// stage Hessian  H0_k = grad^2 L_k + J^T diag(2 wtau + Sigma_s) J + diag(Sigma_x)
// (what the Riccati recursion needs at delta_w = delta_c = 0).
// TP = Dual: lane of a q direction (tangent e_v on the angle); TP = double: lane of a qd
// direction (the pose has no tangent, node_fwd_rev runs it in plain FP64)
template <int NJ, class TP> struct NodeIn {
    const double *xqd;
    const double (*sc)[2];  // LDS: sin / cos of the node's joint angles (one evaluation per node, not per lane)
    int v;
    __device__ __forceinline__ Dual qd(int i) const { return Dual(xqd[i], v == NJ + i ? 1.0 : 0.0); }
    __device__ __forceinline__ void sincos(int i, TP &s, TP &c) const {
        const double sv = sc[i][0], cv = sc[i][1];
        if constexpr (sizeof(TP) == sizeof(Dual)) {
            const double t = (v == i) ? 1.0 : 0.0;
            s = TP(sv, cv * t);
            c = TP(cv, -sv * t);
        } else {
            s = sv;
            c = cv;
        }
    }
};
// Per-lane results of node_fwd_rev, written straight to the node's global arrays: column v of
// d tau / dw (Jt) and column v of grad^2 phi (raw, into W; k_eval_asm completes W in place).
template <int NJ, int NF, int NV, int CLS> struct NodeOut {
    double *Jt, *W;  // the node's blocks
    double *Ts;      // LDS: tau values of the node (direction-0 lane)
    int v;
    const double *fdir;
    double pfv[3], pfd[3];
    template <class TP> __device__ __forceinline__ void frame(const TP *p) {
#pragma unroll
        for (int k = 0; k < 3; k++) { pfv[k] = val(p[k]); pfd[k] = dtan(p[k]); }
    }
    template <class TP> __device__ __forceinline__ void force(const TP *gF) {
#pragma unroll
        for (int a = 0; a < NF; a++)
            W[(2 * NJ + a) * NV + v] = fdir[3 * a] * dtan(gF[0]) + fdir[3 * a + 1] * dtan(gF[1]) + fdir[3 * a + 2] * dtan(gF[2]);
    }
    // k_eval_asm reads the lower triangle (row >= column) of the Hessian: a qd lane (CLS 1) writes
    // no q row (v >= NJ > i) and runs without the q-gradient adjoint (GQ = false); a q lane writes
    // its whole column (the rows above the diagonal are never read)
    __device__ __forceinline__ void joint(int i, const Dual &t, const Dual &gq, const Dual &gqd) {
        Jt[i * NV + v] = t.d;
        if (v == 0) Ts[i] = t.v;
        if constexpr (CLS == 0) {
            W[i * NV + v] = gq.d;
            W[(NJ + i) * NV + v] = gqd.d;
        } else {
            if (NJ + i >= v) W[(NJ + i) * NV + v] = gqd.d;
        }
    }
};

// Blocks hold one direction class each (blockIdx < nb: q directions, else qd directions) of
// NPB nodes, NJ lanes per node: a qd lane runs the sweep with a plain-FP64 pose and costs about
// half a q lane, and a block of one class never waits on the slower class (a block's waves
// keep their registers until the last one finishes).  Each lane writes its own Jacobian and
// Hessian columns; k_eval_asm adds the Gauss-Newton / barrier terms.  The q-class lanes also
// write the force columns (d tau / dF_a = -fdir_a . dp_f/dq_v), the line Jacobian, and the
// node's tau, line residual and cost.
template <int NJ, int NF, int NL, int CLS>
__global__ __launch_bounds__(256) void k_eval_node(const DevModel *__restrict__ Mg, const DevFrame *__restrict__ Fg,
                                                   OcpConst C, IpmArrays A, int batch, int nb) {
    constexpr int NV = 2 * NJ + NF;
    constexpr int NFA = NF > 0 ? NF : 1;
    constexpr int NPB = 4 * (64 / NJ);
    __shared__ ModelLds<NJ> Ml;
    const DevModel &M = Ml.get();
    __shared__ DevFrame F;
    __shared__ double Ts[NPB][NJ], Cs[NPB][NJ];
    __shared__ double SCs[NPB][NJ][2];  // sin / cos of each node's joint angles
    if ((long)blockIdx.x * NPB >= (long)*A.nrun * C.N) return;  // block past the running set (uniform)
    Ml.load(Mg);
    stage_lds(&F, Fg);
    constexpr int cls = CLS;  // direction class: 0 = q directions, 1 = qd directions (own launch)
    const int grp = blockIdx.x;
    const int tid = threadIdx.x, wv = tid >> 6, ln = tid & 63;
    const int g = wv * (64 / NJ) + ln / NJ, j0 = ln % NJ, v = cls * NJ + j0;
    const int N = C.N;
    const long nslots = (long)*A.nrun * N;  // nodes of the compacted running set
    const long node = (long)grp * NPB + g;
    bool run = (ln < (64 / NJ) * NJ) && node < nslots;
    int b = 0, k = 0;
    if (run) {
        b = A.list[node / N];
        k = (int)(node % N);
        run = A.st[b].status == ST_RUNNING;
    }
    const IpmSizes S = ipm_sizes(C);
    const double *q = A.q + b * S.q + (size_t)k * NJ;
    const double *qd = A.qd + b * S.u + (size_t)k * NJ;
    const double *Fv = A.F + b * S.f + (size_t)k * NFA;
    NodeOut<NJ, NF, NV, CLS> out;
    out.Jt = A.Jt + b * S.jt + (size_t)k * NJ * NV;
    out.W = A.W + b * S.w + (size_t)k * NV * NV;
    out.Ts = Ts[g];
    out.v = v;
    out.fdir = C.fdir;
    if (run) sincos(q[j0], &SCs[g][j0][0], &SCs[g][j0][1]);
    // torque weights c = y_tau + 2 wtau tau (tau at the iterate first when wtau != 0)
    if (run && j0 == 0) {
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
    if (!run) return;
    double yl3[3] = {0.0, 0.0, 0.0};
#pragma unroll
    for (int l = 0; l < NL; l++) yl3[l] = A.yl[b * S.l + (size_t)k * NL + l];
    double Fw[3];
#pragma unroll
    for (int r = 0; r < 3; r++) {
        double acc = 0.0;
#pragma unroll
        for (int a = 0; a < NF; a++) acc += Fv[a] * C.fdir[3 * a + r];
        Fw[r] = acc;
    }
    const int fp = (NF > 0 || NL > 0) ? F.parent : -1;
    if constexpr (cls == 0) {
        NodeIn<NJ, Dual> in{qd, SCs[g], v};
        node_fwd_rev<Dual, Dual, NJ>(M, F, fp, in, Fw, Cs[g], yl3, out);
    } else {
        NodeIn<NJ, double> in{qd, SCs[g], v};
        node_fwd_rev<double, Dual, NJ, true, false>(M, F, fp, in, Fw, Cs[g], yl3, out);
        return;
    }
    // ---- q lanes: force columns of d tau / dw, line Jacobian column; node values (lane 0)
#pragma unroll
    for (int a = 0; a < NF; a++)
        out.Jt[v * NV + 2 * NJ + a] = -(C.fdir[3 * a] * out.pfd[0] + C.fdir[3 * a + 1] * out.pfd[1] +
                                        C.fdir[3 * a + 2] * out.pfd[2]);
    if (NL > 0) {
        double *Jl = A.Jl + b * S.jl + (size_t)k * NL * NJ;
#pragma unroll
        for (int l = 0; l < NL; l++) Jl[l * NJ + v] = out.pfd[l];
    }
    if (v == 0) {
        __builtin_amdgcn_wave_barrier();
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

// ---- q directions: one wavefront = one direction v x 64 nodes (k_eval_q)
// A wave whose lanes all carry the tangent of the same angle q_v runs node_fwd_rev_split: plain FP64
// over the joints below v in the forward sweep and, in the reverse sweep, the qd-class arithmetic
// (plain pose, no q-gradient) over those joints -- the tangents it drops are exactly zero.  Block
// (node group, v) = blockIdx (grp * NJ + v): the NJ directions of a node group are adjacent.  Each
// lane writes column v of d tau / dw, the lower part (rows >= v) of column v of the raw Hessian, the
// force column entry of row v, the line-Jacobian column v and (v = 0) the node's tau, cost and line
// residual.
struct QIn {
    const double (*sc)[2];  // LDS: sin / cos of the lane's joint angles
    const double *xqd;      // LDS: the lane's joint velocities
    int v;
    __device__ __forceinline__ Dual qd(int i) const { return Dual(xqd[i], 0.0); }
    __device__ __forceinline__ void sincos(int i, double &s, double &c) const { s = sc[i][0]; c = sc[i][1]; }
    __device__ __forceinline__ void sincos(int i, Dual &s, Dual &c) const {
        const double sv = sc[i][0], cv = sc[i][1], t = (v == i) ? 1.0 : 0.0;
        s = Dual(sv, cv * t);
        c = Dual(cv, -sv * t);
    }
};
template <int NJ, int NF, int NV> struct QOut {
    double *Jt, *W;
    double *Ts;  // LDS: tau values of the lane's node
    int v;
    bool forced;
    const double *fdir;
    double pfv[3], pfd[3];
    template <class TP> __device__ __forceinline__ void frame(const TP *p) {
#pragma unroll
        for (int k = 0; k < 3; k++) { pfv[k] = val(p[k]); pfd[k] = dtan(p[k]); }
    }
    template <class TP> __device__ __forceinline__ void force(const TP *gF) {
        forced = true;
#pragma unroll
        for (int a = 0; a < NF; a++)
            W[(2 * NJ + a) * NV + v] = fdir[3 * a] * dtan(gF[0]) + fdir[3 * a + 1] * dtan(gF[1]) + fdir[3 * a + 2] * dtan(gF[2]);
    }
    __device__ __forceinline__ void joint(int i, const Dual &t, const Dual &gq, const Dual &gqd) {
        Jt[i * NV + v] = t.d;
        Ts[i] = t.v;
        if (i >= v) W[i * NV + v] = gq.d;
        W[(NJ + i) * NV + v] = gqd.d;
    }
};
// MF_EVALQ_WAVES (experiment builds only): ask the register allocator for that many waves per SIMD
#ifdef MF_EVALQ_WAVES
#define MF_EVALQ_ATTR __attribute__((amdgpu_waves_per_eu(MF_EVALQ_WAVES)))
#else
#define MF_EVALQ_ATTR
#endif
template <int NJ, int NF, int NL>
__global__ __launch_bounds__(64) MF_EVALQ_ATTR void k_eval_q(const DevModel *__restrict__ Mg, const DevFrame *__restrict__ Fg,
                                               OcpConst C, IpmArrays A, int batch) {
    constexpr int NV = 2 * NJ + NF;
    constexpr int NFA = NF > 0 ? NF : 1;
    __shared__ ModelLds<NJ> Ml;
    const DevModel &M = Ml.get();
    __shared__ DevFrame F;
    __shared__ double SCs[64][NJ][2], QDs[64][NJ], Cs[64][NJ], Ts[64][NJ];
    // XCD-aware block -> (node group, direction) map: workgroups are dealt round-robin over the 8 XCDs
    // (blockIdx % 8), each with its own L2.  The NJ direction blocks of a node group write interleaved
    // columns of the same W / Jt rows, so they are kept on one XCD (blockIdx % 8 = grp % 8) and issued
    // back to back there: the rows' lines fill in one L2 instead of leaving it as NJ partial lines from
    // NJ different L2s.  The grid is a multiple of 8 NJ blocks; blocks past the node groups exit.
    const int xcd = (int)(blockIdx.x & 7);
    const long slot = blockIdx.x >> 3;
    const int v = (int)(slot % NJ);
    const long grp = (slot / NJ) * 8 + xcd;
    const int lane = threadIdx.x;
    const int N = C.N;
    const long nslots = (long)*A.nrun * N;  // nodes of the compacted running set
    if (grp * 64 >= nslots) return;         // block past the running set (uniform)
    Ml.load(Mg);
    stage_lds(&F, Fg);
    const long node = grp * 64 + lane;
    bool run = node < nslots;
    int b = 0, k = 0;
    if (run) {
        b = A.list[node / N];
        k = (int)(node % N);
        run = A.st[b].status == ST_RUNNING;
    }
    const IpmSizes S = ipm_sizes(C);
    const double *q = A.q + b * S.q + (size_t)k * NJ;
    const double *qd = A.qd + b * S.u + (size_t)k * NJ;
    const double *Fv = A.F + b * S.f + (size_t)k * NFA;
    double Fw[3];
#pragma unroll
    for (int r = 0; r < 3; r++) {
        double acc = 0.0;
#pragma unroll
        for (int a = 0; a < NF; a++) acc += Fv[a] * C.fdir[3 * a + r];
        Fw[r] = acc;
    }
    const int fp = (NF > 0 || NL > 0) ? F.parent : -1;
    if (run) {
#pragma unroll
        for (int j = 0; j < NJ; j++) {
            sincos(q[j], &SCs[lane][j][0], &SCs[lane][j][1]);
            QDs[lane][j] = qd[j];
        }
        // torque weights c = y_tau + 2 wtau tau (tau at the iterate first when wtau != 0)
        const double *yd = A.yd + b * S.u + (size_t)k * NJ;
        if (C.wtau != 0.0) {
            struct WOut {
                double *c;
                const double *yd;
                double w2;
                __device__ void frame(const double *) {}
                __device__ void force(const double *) {}
                __device__ void joint(int j, double t, double, double) { c[j] = yd[j] + w2 * t; }
            } wo{Cs[lane], yd, 2.0 * C.wtau};
            ArrIn<NJ> in0{q, qd};
            node_values<NJ>(M, F, fp, in0, Fw, wo);
        } else {
#pragma unroll
            for (int j = 0; j < NJ; j++) Cs[lane][j] = yd[j];
        }
    }
    __syncthreads();
    if (!run) return;
    double yl3[3] = {0.0, 0.0, 0.0};
#pragma unroll
    for (int l = 0; l < NL; l++) yl3[l] = A.yl[b * S.l + (size_t)k * NL + l];
    QOut<NJ, NF, NV> out;
    out.Jt = A.Jt + b * S.jt + (size_t)k * NJ * NV;
    out.W = A.W + b * S.w + (size_t)k * NV * NV;
    out.Ts = Ts[lane];
    out.v = v;
    out.forced = false;
    out.fdir = C.fdir;
    QIn in{SCs[lane], QDs[lane], v};
    node_fwd_rev_split<NJ>(M, F, fp, v, in, Fw, Cs[lane], yl3, out);
    if (!out.forced)  // frame parent below v: the force row of column v is exactly zero
#pragma unroll
        for (int a = 0; a < NF; a++) out.W[(2 * NJ + a) * NV + v] = 0.0;
    // force columns of d tau / dw (row v), line Jacobian column v; node values (v = 0)
#pragma unroll
    for (int a = 0; a < NF; a++)
        out.Jt[v * NV + 2 * NJ + a] = -(C.fdir[3 * a] * out.pfd[0] + C.fdir[3 * a + 1] * out.pfd[1] +
                                        C.fdir[3 * a + 2] * out.pfd[2]);
    if (NL > 0) {
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
            const double tj = Ts[lane][j];
            tvo[j] = tj;
            c += C.wqd * QDs[lane][j] * QDs[lane][j] + C.wtau * tj * tj;
        }
        A.cost[b * S.cost + k] = c;
        if (NL > 0) {
            double *lv = A.line + b * S.l + (size_t)k * NL;
#pragma unroll
            for (int l = 0; l < NL; l++) lv[l] = out.pfv[l] - A.lref[b * 2 + l];
        }
    }
}

// Completes the condensed stage Hessian in place:
//   H0_k = grad^2 L_k + J^T diag(2 wtau + Sigma_s) J + diag(Sigma_x) (+ cost curvature)
// from the raw Hessian columns k_eval_node left in W and the Jacobian Jt; also the cost gradient
// gf.  One lane per (node, column v), NV lanes per node.  W holds the lower triangle only (row u
// >= column v), read and written in place; k_ipm_kkt mirrors it when it stages H0 in LDS.
template <int NJ, int NF, int NL>
__global__ __launch_bounds__(256) void k_eval_asm(OcpConst C, IpmArrays A, int batch) {
    constexpr int NV = 2 * NJ + NF;
    constexpr int NFA = NF > 0 ? NF : 1;
    constexpr int NPB = 256 / NV;
    __shared__ double Js[NPB][NJ][NV], Wj[NPB][NJ];
    const int tid = threadIdx.x, g = tid / NV, v = tid % NV;
    const int N = C.N;
    const long node = (long)blockIdx.x * NPB + g;
    if ((long)blockIdx.x * NPB >= (long)*A.nrun * N) return;  // block past the running set (uniform)
    bool run = g < NPB && node < (long)*A.nrun * N;
    int b = 0, k = 0;
    if (run) {
        b = A.list[node / N];
        k = (int)(node % N);
        run = A.st[b].status == ST_RUNNING;
    }
    const IpmSizes S = ipm_sizes(C);
    const double *Jt = A.Jt + b * S.jt + (size_t)k * NJ * NV;
    double *W = A.W + b * S.w + (size_t)k * NV * NV;
    const double *q = A.q + b * S.q + (size_t)k * NJ, *qd = A.qd + b * S.u + (size_t)k * NJ;
    const double *Fv = A.F + b * S.f + (size_t)k * NFA;
    double raw[NV];
    if (run) {
#pragma unroll
        for (int j = 0; j < NJ; j++) Js[g][j][v] = Jt[j * NV + v];
        if (v < NJ) {
            const size_t e = b * S.u + (size_t)k * NJ + v;
            Wj[g][v] = 2.0 * C.wtau + sigma_pair(A.vL[e], A.vU[e], A.s[e], A.tau_lo[(size_t)k * NJ + v],
                                                 A.tau_hi[(size_t)k * NJ + v]);
        }
#pragma unroll
        for (int u = 0; u < NV; u++) raw[u] = (u >= v && !(u >= 2 * NJ && v >= NJ)) ? W[u * NV + v] : 0.0;
    }
    __syncthreads();
    if (!run) return;
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
    // phi is linear in F and d phi / dF does not depend on qd: the force rows of the qd and force
    // columns of the raw Hessian are zero (no lane computed them; raw[] reads them as 0)
#pragma unroll
    for (int u = 0; u < NV; u++) {
        if (u < v) continue;
        double gn = 0.0;
#pragma unroll
        for (int j = 0; j < NJ; j++) gn += Wj[g][j] * Js[g][j][u] * Js[g][j][v];
        double hh = raw[u] + gn;
        if (u == v) hh += diag;
        W[u * NV + v] = hh;
    }
    const double *tv = A.tau + b * S.u + (size_t)k * NJ;
    double gfv = 0.0;
#pragma unroll
    for (int j = 0; j < NJ; j++) gfv += 2.0 * C.wtau * tv[j] * Js[g][j][v];
    if (v >= NJ && v < 2 * NJ) gfv += 2.0 * C.wqd * qd[v - NJ];
    if (NF > 0 && v >= 2 * NJ) gfv += 2.0 * C.wF * Fv[v - 2 * NJ];
    A.gf[b * S.gf + (size_t)k * NV + v] = gfv;
}

// ============================================================== init
template <int NJ, int NF, int NL>
__global__ __launch_bounds__(64) void k_ipm_init(const DevModel *__restrict__ Mg, const DevFrame *__restrict__ Fg,
                                                 OcpConst C, IpmArrays A, int batch) {
    __shared__ ModelLds<NJ> Ml;
    const DevModel &M = Ml.get();
    __shared__ DevFrame F;
    Ml.load(Mg);
    stage_lds(&F, Fg);
    __syncthreads();
    const int b = blockIdx.x, lane = threadIdx.x;
    if (b >= batch) return;
    constexpr int NFA = NF > 0 ? NF : 1;
    const IpmSizes S = ipm_sizes(C);
    const int N = C.N;
    double *q = A.q + b * S.q, *qd = A.qd + b * S.u, *Fv = A.F + b * S.f, *s = A.s + b * S.u;
    const double *q0 = A.q0 + (size_t)b * NJ;
    // warm start (w layout [q_0 | (qd_k, F_k, q_{k+1}) for k < N]): q_k, qd_k (k >= 1) and F_k from w0,
    // pushed into their bounds; q_0, qd_0 stay this problem's.  IPOPT warm_start_init_point (C.warm_start):
    // pushes 1e-3 instead of 1e-2 and bound multipliers 1e-3 instead of 1 (oracle/mf_oracle.c, same rule)
    const int wst = 2 * NJ + NF, wsz = NJ + N * wst;
    const double *w0 = A.w0 ? A.w0 + (size_t)b * wsz : nullptr;
    const bool warm = C.warm_start && w0;
    const double kp = warm ? 1e-3 : 1e-2, z0 = warm ? 1e-3 : 1.0;
    for (int e = lane; e < (N + 1) * NJ; e += 64) {
        int k = e / NJ, j = e % NJ;
        q[e] = (k == 0) ? q0[j] : bound_push(q0[j], C.q_lo[j], C.q_hi[j]);
        A.zqL[b * S.q + e] = (k > 0 && hasb(C.q_lo[j])) ? z0 : 0.0;
        A.zqU[b * S.q + e] = (k > 0 && hasb(C.q_hi[j])) ? z0 : 0.0;
    }
    if (w0) {
        for (int e = lane + NJ; e < (N + 1) * NJ; e += 64) {
            const int k = e / NJ, j = e % NJ;
            q[e] = bound_push(w0[NJ + (k - 1) * wst + NJ + NF + j], C.q_lo[j], C.q_hi[j], kp);
        }
    }
    for (int e = lane; e < N * NJ; e += 64) {
        int k = e / NJ, j = e % NJ;
        const double qd0j = A.qd0p ? A.qd0p[(size_t)b * NJ + j] : C.qd0[j];
        qd[e] = (k == 0) ? qd0j : bound_push(w0 ? w0[NJ + k * wst + j] : 0.0, C.qd_lo[j], C.qd_hi[j], kp);
        A.zdL[b * S.u + e] = (k > 0 && hasb(C.qd_lo[j])) ? z0 : 0.0;
        A.zdU[b * S.u + e] = (k > 0 && hasb(C.qd_hi[j])) ? z0 : 0.0;
        A.vL[b * S.u + e] = hasb(A.tau_lo[e]) ? z0 : 0.0;
        A.vU[b * S.u + e] = hasb(A.tau_hi[e]) ? z0 : 0.0;
        A.yc[b * S.u + e] = 0.0;
        A.yd[b * S.u + e] = 0.0;
    }
    for (int e = lane; e < N * NFA; e += 64)
        Fv[e] = NF > 0 ? (w0 ? w0[NJ + (e / NFA) * wst + NJ + e % NFA] : C.F_init) : 0.0;
    for (int e = lane; e < (int)S.l; e += 64) A.yl[b * S.l + e] = 0.0;
    __syncthreads();
    // slacks from tau at the initial point
    struct SlackOut {
        double *s;
        const double *lo, *hi;
        double kp;
        __device__ void frame(const double *) {}
        __device__ void force(const double *) {}
        __device__ void joint(int j, double t, double, double) { s[j] = bound_push(t, lo[j], hi[j], kp); }
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
        SlackOut so{s + (size_t)k * NJ, A.tau_lo + (size_t)k * NJ, A.tau_hi + (size_t)k * NJ, kp};
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
    __device__ void sincos(int i, double &s, double &c) const { sincos_t(q(i), s, c); }
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


// Block reductions over NT threads (NT / 64 waves): NMX maxima and NSM sums at once; every thread
// gets the results.  red: LDS scratch of (NMX + NSM) * (NT / 64) doubles, free on entry.
template <int NT, int NMX, int NSM>
__device__ __forceinline__ void block_reduce(double *mx, double *sm, double *red) {
    constexpr int NW = NT / 64;
    const int t = threadIdx.x;
#pragma unroll
    for (int i = 0; i < NMX; i++) mx[i] = wave_max(mx[i]);
#pragma unroll
    for (int i = 0; i < NSM; i++) sm[i] = wave_sum(sm[i]);
    __syncthreads();  // red is free: earlier readers are done
    if ((t & 63) == 0) {
#pragma unroll
        for (int i = 0; i < NMX; i++) red[i * NW + (t >> 6)] = mx[i];
#pragma unroll
        for (int i = 0; i < NSM; i++) red[(NMX + i) * NW + (t >> 6)] = sm[i];
    }
    __syncthreads();
#pragma unroll
    for (int i = 0; i < NMX; i++) {
        double r = red[i * NW];
        for (int w = 1; w < NW; w++) r = fmax(r, red[i * NW + w]);
        mx[i] = r;
    }
#pragma unroll
    for (int i = 0; i < NSM; i++) {
        double r = red[(NMX + i) * NW];
        for (int w = 1; w < NW; w++) r += red[(NMX + i) * NW + w];
        sm[i] = r;
    }
}
template <int NT> __device__ __forceinline__ double block_max(double v, double *red) {
    double mx[1] = {v};
    block_reduce<NT, 1, 0>(mx, nullptr, red);
    return mx[0];
}
template <int NT> __device__ __forceinline__ double block_sum(double v, double *red) {
    double sm[1] = {v};
    block_reduce<NT, 0, 1>(nullptr, sm, red);
    return sm[0];
}

// One interior-point iteration = the node evaluation (k_eval_q, k_eval_node<..,1>, k_eval_asm) + the
// per-problem launches (a launch boundary lets each phase have its own register budget and block shape):
//   k_ipm_pre     : optimality error, convergence test, barrier update, barrier Sigma / gradients, the
//                   first inertia try's Riccati stage inputs (256-thread block per problem)
//   k_ipm_kkt     : inertia-corrected Riccati recursion and forward sweep (one wave per problem)
//   k_kkt_recover : step recovery, fraction to the boundary, merit slope / curvature (block per problem)
//   k_ipm_post    : merit line search and the primal-dual update (two waves per problem)
// Scalars that cross a boundary travel in ProbState (mu, nu, tau_fb, regularisation, step bounds,
// directional derivative and curvature).
template <int NJ, int NF, int NL, int NT, class Sync>
__device__ __forceinline__ void prep_stage_inputs(const OcpConst &C, const IpmArrays &A, int b, int tid, double dwv,
                                                  double dcv, Sync sync);
__device__ __forceinline__ void kkt_first_try(const ProbState &st, int &tier, double &reg, double &dw, double &dFr);

template <int NJ, int NF, int NL>
__global__ __launch_bounds__(256) void k_ipm_pre(const DevModel *__restrict__ Mg, const DevFrame *__restrict__ Fg,
                                                 OcpConst C, IpmArrays A, int batch) {
    constexpr int n = NJ, nf = NF, nl = NL;
    constexpr int NV = 2 * NJ + NF;
    constexpr int NFA = NF > 0 ? NF : 1;
    constexpr int NLA = NL > 0 ? NL : 1;
    constexpr int MB = 3 * NJ + NF + NL;
    constexpr int NT = 256;  // a block per problem (element loops and block reductions)
    __shared__ double red[8 * (NT / 64)];
    const int lane = threadIdx.x;
    if ((int)blockIdx.x >= *A.nrun) return;
    const int b = A.list[blockIdx.x];
    ProbState st = A.st[b];
    if (st.status != ST_RUNNING) return;
    __shared__ double Bnd[4 * NJ];  // q_lo, q_hi, qd_lo, qd_hi (kernel-argument arrays read per element)
    if (lane < NJ) {
        Bnd[lane] = C.q_lo[lane];
        Bnd[NJ + lane] = C.q_hi[lane];
        Bnd[2 * NJ + lane] = C.qd_lo[lane];
        Bnd[3 * NJ + lane] = C.qd_hi[lane];
    }
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
    const double *QLO = Bnd, *QHI = Bnd + NJ, *DLO = Bnd + 2 * NJ, *DHI = Bnd + 3 * NJ;
#define TACT(k, j) (hasb(tlo[(k) * n + (j)]) || hasb(thi[(k) * n + (j)]))

    const double kappa_eps = 10.0, kappa_mu = 0.2, theta_mu = 1.5, tau_min = 0.99, s_max = 100.0;
    const double kappa_sigma = 1e10, eta = 1e-4, rho = 0.1;
    double mu = st.mu, nu = st.nu;
    constexpr int UB = 2;  // element-loop chunk (see the optimality-error phase)
    auto finish = [&](int status) {
        STAMP_FLUSH;
        double f = 0.0;
        for (int k = lane; k < N; k += NT) f += cost[k];
        f = block_sum<NT>(f, red);
        if (lane == 0) {
            st.status = status;
            st.obj = f;
            st.mu = mu;
            st.nu = nu;
            A.st[b] = st;
            atomicSub(A.active, 1);
        }
    };
    // ---------------- optimality error
    // Element loops of one problem run in chunks of UB elements per lane.  A chunk issues every
    // load first (indices clamped into range, results past the end discarded) and only then
    // computes and stores, so it costs one global-memory round trip instead of one per element:
    // one wave per problem has no other waves of its own to hide that latency behind.
    double dinf = 0, pinf = 0, cinf0 = 0, cinfm = 0, sum_mult = 0, sum_bmult = 0;
    int n_mult = 0, n_bmult = 0;
    auto comp = [&](double z, double gap) {
        const double c = z * gap;
        cinf0 = fmax(cinf0, fabs(c));
        cinfm = fmax(cinfm, fabs(c - mu));
        sum_bmult += z;
        n_bmult++;
    };
    for (int e0 = lane; e0 < N * n; e0 += NT * UB) {  // q rows, k = 1..N
        double r[UB], x[UB], zl[UB], zu[UB];
#pragma unroll
        for (int u = 0; u < UB; u++) {
            const int e = min(e0 + NT * u, N * n - 1);
            const int k = e / n + 1, j = e % n, i = k * n + j, kk = min(k, N - 1);
            double a = gf[kk * NV + j] + yc[kk * n + j] - yc[(k - 1) * n + j];
#pragma unroll
            for (int l = 0; l < NL; l++) a += Jl[(kk * nl + l) * n + j] * yl[kk * nl + l];
#pragma unroll
            for (int jj = 0; jj < NJ; jj++) a += Jt[((size_t)kk * n + jj) * NV + j] * yd[kk * n + jj];
            const double ycl = yc[(N - 1) * n + j];
            zl[u] = zqL[i];
            zu[u] = zqU[i];
            x[u] = q[i];
            r[u] = (k < N ? a : -ycl) - zl[u] + zu[u];
        }
#pragma unroll
        for (int u = 0; u < UB; u++) {
            const int e = e0 + NT * u;
            if (e < N * n) {
                const int j = e % n;
                dinf = fmax(dinf, fabs(r[u]));
                if (hasb(QLO[j])) comp(zl[u], x[u] - QLO[j]);
                if (hasb(QHI[j])) comp(zu[u], QHI[j] - x[u]);
            }
        }
    }
    for (int e0 = lane; e0 < N * n; e0 += NT * UB) {  // qd rows (k >= 1), torque rows, continuity
        double r[UB], x[UB], zl[UB], zu[UB], r2[UB], xs[UB], vl[UB], vu[UB], lo[UB], hi[UB], pt[UB], pc[UB], ydv[UB], ycv[UB];
#pragma unroll
        for (int u = 0; u < UB; u++) {
            const int e = min(e0 + NT * u, N * n - 1);
            const int k = e / n, j = e % n;
            double a = gf[k * NV + n + j] + h * yc[e];
#pragma unroll
            for (int jj = 0; jj < NJ; jj++) a += Jt[((size_t)k * n + jj) * NV + n + j] * yd[k * n + jj];
            zl[u] = zdL[e]; zu[u] = zdU[e]; x[u] = qd[e];
            r[u] = a - zl[u] + zu[u];
            vl[u] = vL[e]; vu[u] = vU[e]; xs[u] = s[e]; lo[u] = tlo[e]; hi[u] = thi[e];
            ydv[u] = yd[e]; ycv[u] = yc[e];
            r2[u] = -ydv[u] - vl[u] + vu[u];
            pt[u] = fabs(tau[e] - xs[u]);
            pc[u] = fabs(q[k * n + j] + h * x[u] - q[(k + 1) * n + j]);
        }
#pragma unroll
        for (int u = 0; u < UB; u++) {
            const int e = e0 + NT * u;
            if (e < N * n) {
                const int k = e / n, j = e % n;
                if (k > 0) {
                    dinf = fmax(dinf, fabs(r[u]));
                    if (hasb(DLO[j])) comp(zl[u], x[u] - DLO[j]);
                    if (hasb(DHI[j])) comp(zu[u], DHI[j] - x[u]);
                }
                if (hasb(lo[u]) || hasb(hi[u])) {
                    dinf = fmax(dinf, fabs(r2[u]));
                    if (hasb(lo[u])) comp(vl[u], xs[u] - lo[u]);
                    if (hasb(hi[u])) comp(vu[u], hi[u] - xs[u]);
                    pinf = fmax(pinf, pt[u]);
                    sum_mult += fabs(ydv[u]); n_mult++;
                }
                pinf = fmax(pinf, pc[u]);
                sum_mult += fabs(ycv[u]); n_mult++;
            }
        }
    }
    for (int e0 = lane; e0 < N * nf; e0 += NT * UB) {  // force rows
        double r[UB];
#pragma unroll
        for (int u = 0; u < UB; u++) {
            const int e = min(e0 + NT * u, N * nf - 1);
            const int k = e / nf, a = e % nf;
            double v = gf[k * NV + 2 * n + a];
#pragma unroll
            for (int jj = 0; jj < NJ; jj++) v += Jt[((size_t)k * n + jj) * NV + 2 * n + a] * yd[k * n + jj];
            r[u] = v;
        }
#pragma unroll
        for (int u = 0; u < UB; u++)
            if (e0 + NT * u < N * nf) dinf = fmax(dinf, fabs(r[u]));
    }
    for (int e0 = lane; e0 < N * nl; e0 += NT * UB) {  // line rows
        double lv[UB], yv[UB];
#pragma unroll
        for (int u = 0; u < UB; u++) {
            const int e = min(e0 + NT * u, N * nl - 1);
            lv[u] = line[e];
            yv[u] = yl[e];
        }
#pragma unroll
        for (int u = 0; u < UB; u++) {
            const int e = e0 + NT * u;
            if (e < N * nl && LINE_ON(e / nl)) { pinf = fmax(pinf, fabs(lv[u])); sum_mult += fabs(yv[u]); n_mult++; }
        }
    }
    {
        double mx[4] = {dinf, pinf, cinf0, cinfm}, sm[4] = {sum_mult, sum_bmult, (double)n_mult, (double)n_bmult};
        block_reduce<NT, 4, 4>(mx, sm, red);
        dinf = mx[0]; pinf = mx[1]; cinf0 = mx[2]; cinfm = mx[3];
        sum_mult = sm[0]; sum_bmult = sm[1]; n_mult = (int)sm[2]; n_bmult = (int)sm[3];
    }
    const double sd = fmax(s_max, (sum_mult + sum_bmult) / fmax(1.0, (double)(n_mult + n_bmult))) / s_max;
    const double sc = fmax(s_max, sum_bmult / fmax(1.0, (double)n_bmult)) / s_max;
    const double E0 = fmax(fmax(dinf / sd, pinf), cinf0 / sc);
    TRACE(0, dinf); TRACE(1, pinf); TRACE(2, cinf0); TRACE(3, mu);
#ifdef MF_TRACE
    {
        double f = 0.0;
        for (int k = lane; k < N; k += NT) f += cost[k];
        f = block_sum<NT>(f, red);
        TRACE(14, f);
    }
#endif
    double Emu = fmax(fmax(dinf / sd, pinf), cinfm / sc);
    st.E0 = E0;
    st.cviol = pinf;
    if (E0 <= C.tol && pinf <= C.constr_viol_tol) { finish(ST_CONVERGED); return; }
    if (st.iter >= C.max_iter) { finish(ST_MAXITER); return; }
    while (Emu <= kappa_eps * mu && mu > C.tol / 10.0) {
        double mnew = fmax(C.tol / 10.0, fmin(kappa_mu * mu, pow(mu, theta_mu)));
        if (mnew >= mu) break;
        mu = mnew;
        double cm = 0.0;
        for (int e0 = lane; e0 < N * n; e0 += NT * UB) {
            double cp[6][UB];
#pragma unroll
            for (int u = 0; u < UB; u++) {
                const int e = min(e0 + NT * u, N * n - 1);
                const int i = e + n, j = e % n;
                const double xq = q[i], xd = qd[e], xs = s[e], l = tlo[e], hh = thi[e];
                const bool in = e0 + NT * u < N * n, kq = e / n > 0;
                cp[0][u] = (in && hasb(QLO[j])) ? zqL[i] * (xq - QLO[j]) : NAN;
                cp[1][u] = (in && hasb(QHI[j])) ? zqU[i] * (QHI[j] - xq) : NAN;
                cp[2][u] = (in && kq && hasb(DLO[j])) ? zdL[e] * (xd - DLO[j]) : NAN;
                cp[3][u] = (in && kq && hasb(DHI[j])) ? zdU[e] * (DHI[j] - xd) : NAN;
                cp[4][u] = (in && hasb(l)) ? vL[e] * (xs - l) : NAN;
                cp[5][u] = (in && hasb(hh)) ? vU[e] * (hh - xs) : NAN;
            }
#pragma unroll
            for (int u = 0; u < UB; u++)
#pragma unroll
                for (int p = 0; p < 6; p++)
                    if (!isnan(cp[p][u])) cm = fmax(cm, fabs(cp[p][u] - mu));
        }
        cinfm = block_max<NT>(cm, red);
        Emu = fmax(fmax(dinf / sd, pinf), cinfm / sc);
    }
    const double tau_fb = fmax(tau_min, 1.0 - mu);
    TRACE(4, mu);
    STAMP(0);

    // ---------------- barrier Sigma and gradients
    for (int e0 = lane; e0 < (N + 1) * n; e0 += NT * UB) {
        double x[UB], zl[UB], zu[UB];
#pragma unroll
        for (int u = 0; u < UB; u++) {
            const int e = min(e0 + NT * u, (N + 1) * n - 1);
            x[u] = q[e]; zl[u] = zqL[e]; zu[u] = zqU[e];
        }
#pragma unroll
        for (int u = 0; u < UB; u++) {
            const int e = e0 + NT * u;
            if (e < (N + 1) * n) {
                const int k = e / n, j = e % n;
                double sx = 0, gp = 0;
                if (k > 0) {
                    sx = sigma_pair(zl[u], zu[u], x[u], QLO[j], QHI[j]);
                    if (hasb(QLO[j])) gp -= mu / (x[u] - QLO[j]);
                    if (hasb(QHI[j])) gp += mu / (QHI[j] - x[u]);
                }
                Sxq[e] = sx; gphq[e] = gp;
            }
        }
    }
    for (int e0 = lane; e0 < N * n; e0 += NT * UB) {
        double x[UB], zl[UB], zu[UB], xs[UB], vl[UB], vu[UB], lo[UB], hi[UB];
#pragma unroll
        for (int u = 0; u < UB; u++) {
            const int e = min(e0 + NT * u, N * n - 1);
            x[u] = qd[e]; zl[u] = zdL[e]; zu[u] = zdU[e];
            xs[u] = s[e]; vl[u] = vL[e]; vu[u] = vU[e]; lo[u] = tlo[e]; hi[u] = thi[e];
        }
#pragma unroll
        for (int u = 0; u < UB; u++) {
            const int e = e0 + NT * u;
            if (e < N * n) {
                const int k = e / n, j = e % n;
                double sx = 0, gp = 0, gs = 0;
                if (k > 0) {
                    sx = sigma_pair(zl[u], zu[u], x[u], DLO[j], DHI[j]);
                    if (hasb(DLO[j])) gp -= mu / (x[u] - DLO[j]);
                    if (hasb(DHI[j])) gp += mu / (DHI[j] - x[u]);
                }
                const double ss = sigma_pair(vl[u], vu[u], xs[u], lo[u], hi[u]);
                if (hasb(lo[u])) gs -= mu / (xs[u] - lo[u]);
                if (hasb(hi[u])) gs += mu / (hi[u] - xs[u]);
                Sxd[e] = sx; gphd[e] = gp; Ss[e] = ss; gphs[e] = gs;
            }
        }
    }
    __threadfence_block();
    __syncthreads();

    STAMP(1);
    STAMP_FLUSH;
    if (lane == 0) {
        st.mu = mu;
        st.nu = nu;
        st.tau_fb = tau_fb;
        A.st[b] = st;
    }
    // the first inertia try's per-stage inputs (Riccati stage blocks) from the Sigma and
    // barrier gradients this block has just written (the __syncthreads above orders them): one launch
    // and one re-read of those arrays per iteration less than a separate pass
    {
        int tier;
        double reg, dw, dFr;
        kkt_first_try(st, tier, reg, dw, dFr);
        prep_stage_inputs<NJ, NF, NL, NT>(C, A, b, lane, dw, 0.0, [] { __syncthreads(); });
    }
#undef TACT
}

// ---------------- per-stage inputs of the Riccati recursion
// For every stage k at once: g_k (NV), c_k = q_k + h qd_k - q_{k+1} (NJ), e_k = line_{k+1} +
// Jl_{k+1} c_k, dD_k = D_tau(dw, dc) - Sigma_s (NJ), into stg (stage k contiguous, SG doubles), and
// y_tau + D_tau r_tau (N x NJ) into the scratch behind it.  NT threads of one horizon (tid < NT)
// stride the elements; `sync` orders the phases (a wave: s_waitcnt; a block: __syncthreads).
// k_ipm_pre runs it for the first inertia try with a whole block per horizon; k_ipm_kkt reruns
// it in its own wave only when a retry changes (dw, dc).  Same per-element arithmetic either way.
template <int NJ, int NF, int NL, int NT, class Sync>
__device__ __forceinline__ void prep_stage_inputs(const OcpConst &C, const IpmArrays &A, int b, int tid, double dwv,
                                                  double dcv, Sync sync) {
    constexpr int n = NJ, nl = NL, NV = 2 * NJ + NF;
    constexpr int NLA2 = NL > 0 ? NL : 1;
    constexpr int SG = NV + 2 * NJ + NLA2;
    constexpr int UB = 2;
    const IpmSizes S = ipm_sizes(C);
    const int N = C.N;
    const double h = C.h;
    const double *q = A.q + b * S.q, *qd = A.qd + b * S.u, *s = A.s + b * S.u;
    const double *yc = A.yc + b * S.u, *yl = A.yl + b * S.l, *yd = A.yd + b * S.u;
    const double *tau = A.tau + b * S.u, *Jt = A.Jt + b * S.jt, *line = A.line + b * S.l, *Jl = A.Jl + b * S.jl;
    const double *gf = A.gf + b * S.gf;
    const double *gphq = A.gphq + b * S.q, *gphd = A.gphd + b * S.u, *Ss = A.Ss + b * S.u, *gphs = A.gphs + b * S.u;
    const double *tlo = A.tau_lo, *thi = A.tau_hi;
    double *stg = A.stg + b * S.stg;
    double *wst = stg + (size_t)N * SG;
    for (int e0 = tid; e0 < N * n; e0 += NT * UB) {
        double ydv[UB], ssv[UB], tv[UB], sv[UB], gv[UB], lo[UB], hi[UB], qa[UB], qdv[UB], qb[UB];
#pragma unroll
        for (int u = 0; u < UB; u++) {
            const int e = min(e0 + NT * u, N * n - 1);
            ydv[u] = yd[e]; ssv[u] = Ss[e]; tv[u] = tau[e]; sv[u] = s[e]; gv[u] = gphs[e];
            lo[u] = tlo[e]; hi[u] = thi[e]; qa[u] = q[e]; qdv[u] = qd[e]; qb[u] = q[e + n];
        }
#pragma unroll
        for (int u = 0; u < UB; u++) {
            const int e = e0 + NT * u;
            if (e < N * n) {
                double wv_ = ydv[u], dD = 0.0;
                if (hasb(lo[u]) || hasb(hi[u])) {
                    const double sg = ssv[u] + dwv;
                    const double Dd = sg / (1.0 + dcv * sg);
                    wv_ += Dd * ((tv[u] - sv[u]) + (gv[u] - ydv[u]) / sg);
                    dD = Dd - ssv[u];
                }
                const int k = e / n, j = e % n;
                wst[e] = wv_;
                stg[k * SG + NV + NJ + NLA2 + j] = dD;
                stg[k * SG + NV + j] = qa[u] + h * qdv[u] - qb[u];
            }
        }
    }
    sync();  // wst / c_k are read back by other threads
    for (int e0 = tid; e0 < N * NV; e0 += NT * UB) {
        double g[UB];
#pragma unroll
        for (int u = 0; u < UB; u++) {
            const int e = min(e0 + NT * u, N * NV - 1);
            const int k = e / NV, v = e % NV;
            const int vq = v < n ? v : 0, vd = (v >= n && v < 2 * n) ? v - n : 0;
            double a = gf[e];
            const double *Jtk = Jt + (size_t)k * n * NV;
#pragma unroll
            for (int jj = 0; jj < NJ; jj++) a += Jtk[jj * NV + v] * wst[k * n + jj];
            double aq = gphq[k * n + vq] + yc[k * n + vq] - (k > 0 ? yc[(k > 0 ? k - 1 : 0) * n + vq] : 0.0);
#pragma unroll
            for (int l = 0; l < NL; l++) aq += Jl[(k * nl + l) * n + vq] * yl[k * nl + l];
            const double ad = gphd[k * n + vd] + h * yc[k * n + vd];
            g[u] = a + (v < n ? aq : (v < 2 * n ? ad : 0.0));
        }
#pragma unroll
        for (int u = 0; u < UB; u++)
            if (e0 + NT * u < N * NV) stg[((e0 + NT * u) / NV) * SG + (e0 + NT * u) % NV] = g[u];
    }
    for (int e0 = tid; e0 < N * nl; e0 += NT * UB) {
        double a[UB];
#pragma unroll
        for (int u = 0; u < UB; u++) {
            const int e = min(e0 + NT * u, N * nl - 1);
            const int k = e / nl, l = e % nl, k1 = min(k + 1, N - 1);
            double v = line[k1 * nl + l];
#pragma unroll
            for (int i = 0; i < NJ; i++) v += Jl[((size_t)k1 * nl + l) * n + i] * stg[k * SG + NV + i];
            a[u] = (LINE_ON(k + 1) && k + 1 <= N - 1) ? v : 0.0;
        }
#pragma unroll
        for (int u = 0; u < UB; u++) {
            const int e = e0 + NT * u;
            if (e < N * nl) stg[(e / nl) * SG + NV + NJ + e % nl] = a[u];
        }
    }
    sync();  // the stage loop reads the blocks back
}

// Regularisation of an iteration's first inertia try (IPOPT's rule: a third of the last
// successful perturbation, dropped below 1e-8; k_ipm_kkt and k_ipm_pre must agree on it).
__device__ __forceinline__ void kkt_first_try(const ProbState &st, int &tier, double &reg, double &dw, double &dFr) {
    tier = st.reg_tier;
    reg = (st.reg_tier == 0) ? 0.0 : st.reg_last / 3.0;
    if (st.reg_tier != 0 && reg < 1e-8) { tier = 0; reg = 0.0; }
    dw = (tier == 2) ? reg : 0.0;
    dFr = (tier == 1) ? reg : 0.0;
}

// Step recovery after k_ipm_kkt's sweeps:
// dyc_k = P_{k+1} dx_{k+1} + p_{k+1} + Jl_{k+1}^T dyl_{k+1} for every stage, dyd, ds, the bound
// multiplier steps and the step-curvature correction pcorr.
// Step recovery of one horizon by the NT threads of its block (the first part of k_ipm_post since round 3;
// formerly its own launch): dy_c, dy_tau, ds, the bound-multiplier steps, the fraction to the boundary,
// grad(phi)^T dx, dx^T (W + Sigma) dx and the merit at the iterate.  Bnd: q_lo, q_hi, qd_lo, qd_hi in LDS;
// red: >= 7 NT / 64 doubles of LDS.  out = {ap, az, gdot, pHp, phi0, th0}, the same in every thread.
template <int NJ, int NF, int NL, int NT>
__device__ __forceinline__ void kkt_recover_body(const OcpConst &C, const IpmArrays &A, int b, const ProbState &st,
                                                 const double *Bnd, double *red, double *out) {
    constexpr int n = NJ, nl = NL;
    constexpr int NV = 2 * NJ + NF;
    constexpr int NFA = NF > 0 ? NF : 1;
    constexpr int MB = 3 * NJ + NF + NL;
    constexpr int NU = NJ + NF;
    constexpr int UB = 2;
    const int tid = threadIdx.x;
    const double *QLO = Bnd, *QHI = Bnd + NJ, *DLO = Bnd + 2 * NJ, *DHI = Bnd + 3 * NJ;
    const IpmSizes S = ipm_sizes(C);
    const int N = C.N;
    const double mu = st.mu, dw = st.kkt_dw, dc = st.kkt_dc;
    const double *q = A.q + b * S.q, *qd = A.qd + b * S.u, *s = A.s + b * S.u, *yd = A.yd + b * S.u;
    const double *zqL = A.zqL + b * S.q, *zqU = A.zqU + b * S.q, *zdL = A.zdL + b * S.u, *zdU = A.zdU + b * S.u;
    const double *vL = A.vL + b * S.u, *vU = A.vU + b * S.u;
    const double *dq = A.dq + b * S.q, *dqd = A.dqd + b * S.u, *dF = A.dF + b * S.f, *dyl = A.dyl + b * S.l;
    double *ds = A.ds + b * S.u, *dyc = A.dyc + b * S.u, *dyd = A.dyd + b * S.u;
    double *dzqL = A.dzqL + b * S.q, *dzqU = A.dzqU + b * S.q, *dzdL = A.dzdL + b * S.u, *dzdU = A.dzdU + b * S.u;
    double *dvL = A.dvL + b * S.u, *dvU = A.dvU + b * S.u;
    const double *tau = A.tau + b * S.u, *Jt = A.Jt + b * S.jt, *Jl = A.Jl + b * S.jl;
    const double *Ss = A.Ss + b * S.u, *gphs = A.gphs + b * S.u;
    const double *W = A.W + b * S.w, *gf = A.gf + b * S.gf, *cost = A.cost + b * S.cost, *line = A.line + b * S.l;
    const double *Sxq = A.Sxq + b * S.q, *gphq = A.gphq + b * S.q, *gphd = A.gphd + b * S.u;
    const double h = C.h;
    const double *G = A.G + b * S.G, *wv = A.wv + b * S.wv;
    const double *tlo = A.tau_lo, *thi = A.tau_hi;
    // fraction to the boundary (primal ap, bound multipliers az), accumulated where the steps are formed
    const double tau_fb = st.tau_fb;
    double ap = 1.0, az = 1.0;
    auto ftbL = [&](double x, double dx, double lo, double &a) { if (dx < 0) a = fmin(a, -tau_fb * (x - lo) / dx); };
    auto ftbU = [&](double x, double dx, double hi, double &a) { if (dx > 0) a = fmin(a, tau_fb * (hi - x) / dx); };
    auto ftbZ = [&](double z, double dz, double &a) { if (dz < 0) a = fmin(a, -tau_fb * z / dz); };
    // dyc_k for every stage
    for (int e0 = tid; e0 < N * n; e0 += NT * UB) {
        double a[UB];
#pragma unroll
        for (int u = 0; u < UB; u++) {
            const int e = min(e0 + NT * u, N * n - 1);
            const int k = e / n, j = e % n;
            const double *Pj = G + (size_t)k * MB * n + (size_t)(NU + NL + j) * n;
            double v = wv[(size_t)k * MB + NU + NL + j];
#pragma unroll
            for (int i = 0; i < NJ; i++) v += Pj[i] * dq[(k + 1) * n + i];
            const bool con1 = (nl > 0) && LINE_ON(k + 1) && (k + 1 <= N - 1);
            const int k1 = min(k + 1, N - 1);
#pragma unroll
            for (int l = 0; l < NL; l++) {
                const double jl = Jl[((size_t)k1 * nl + l) * n + j], yl1 = dyl[k1 * nl + l];
                if (con1) v += jl * yl1;  // (contracted like the sweep's own update: same round-off)
            }
            a[u] = v;
        }
#pragma unroll
        for (int u = 0; u < UB; u++)
            if (e0 + NT * u < N * n) dyc[e0 + NT * u] = a[u];
    }
    // dyd, ds; pcorr = sum Sigma_s (ds^2 - (J dx)^2) turns p^T H0 p into the oracle's p^T (W + Sigma) p
    double pcorr = 0.0;
    for (int e0 = tid; e0 < N * n; e0 += NT * UB) {
        double jdx[UB], ssv[UB], gv[UB], ydv[UB], tv[UB], sv[UB], lo[UB], hi[UB];
#pragma unroll
        for (int u = 0; u < UB; u++) {
            const int e = min(e0 + NT * u, N * n - 1);
            const int k = e / n, j = e % n;
            const double *Jtk = Jt + ((size_t)k * n + j) * NV;
            double a = 0.0;
#pragma unroll
            for (int v = 0; v < NJ; v++) a += Jtk[v] * dq[k * n + v] + Jtk[n + v] * dqd[k * n + v];
#pragma unroll
            for (int f = 0; f < NF; f++) a += Jtk[2 * n + f] * dF[k * NFA + f];
            jdx[u] = a;
            ssv[u] = Ss[e]; gv[u] = gphs[e]; ydv[u] = yd[e]; tv[u] = tau[e]; sv[u] = s[e];
            lo[u] = tlo[e]; hi[u] = thi[e];
        }
#pragma unroll
        for (int u = 0; u < UB; u++) {
            const int e = e0 + NT * u;
            if (e < N * n) {
                double dydv = 0.0, dsv = 0.0;
                if (hasb(lo[u]) || hasb(hi[u])) {
                    const double sg = ssv[u] + dw, Dd = sg / (1.0 + dc * sg);
                    const double rs = gv[u] - ydv[u], rd = tv[u] - sv[u];
                    dydv = Dd * (jdx[u] + rd + rs / sg);
                    dsv = (dydv - rs) / sg;
                    pcorr += ssv[u] * (dsv * dsv - jdx[u] * jdx[u]);
                }
                dyd[e] = dydv;
                ds[e] = dsv;
            }
        }
    }
    for (int e0 = tid; e0 < (N + 1) * n; e0 += NT * UB) {
        double x[UB], dx[UB], zl[UB], zu[UB];
#pragma unroll
        for (int u = 0; u < UB; u++) {
            const int e = min(e0 + NT * u, (N + 1) * n - 1);
            x[u] = q[e]; dx[u] = dq[e]; zl[u] = zqL[e]; zu[u] = zqU[e];
        }
#pragma unroll
        for (int u = 0; u < UB; u++) {
            const int e = e0 + NT * u;
            if (e < (N + 1) * n) {
                const int k = e / n, j = e % n;
                double a = 0, bb = 0;
                if (k > 0) {
                    if (hasb(QLO[j])) a = mu / (x[u] - QLO[j]) - zl[u] - zl[u] / (x[u] - QLO[j]) * dx[u];
                    if (hasb(QHI[j])) bb = mu / (QHI[j] - x[u]) - zu[u] + zu[u] / (QHI[j] - x[u]) * dx[u];
                    if (hasb(QLO[j])) { ftbL(x[u], dx[u], QLO[j], ap); ftbZ(zl[u], a, az); }
                    if (hasb(QHI[j])) { ftbU(x[u], dx[u], QHI[j], ap); ftbZ(zu[u], bb, az); }
                }
                dzqL[e] = a; dzqU[e] = bb;
            }
        }
    }
    __syncthreads();  // ds is read back by other threads
    for (int e0 = tid; e0 < N * n; e0 += NT * UB) {
        double x[UB], dx[UB], zl[UB], zu[UB], xs[UB], dxs[UB], vl[UB], vu[UB], lo[UB], hi[UB];
#pragma unroll
        for (int u = 0; u < UB; u++) {
            const int e = min(e0 + NT * u, N * n - 1);
            x[u] = qd[e]; dx[u] = dqd[e]; zl[u] = zdL[e]; zu[u] = zdU[e];
            xs[u] = s[e]; dxs[u] = ds[e]; vl[u] = vL[e]; vu[u] = vU[e]; lo[u] = tlo[e]; hi[u] = thi[e];
        }
#pragma unroll
        for (int u = 0; u < UB; u++) {
            const int e = e0 + NT * u;
            if (e < N * n) {
                const int k = e / n, j = e % n;
                double a = 0, bb = 0, c = 0, d = 0;
                if (k > 0) {
                    if (hasb(DLO[j])) a = mu / (x[u] - DLO[j]) - zl[u] - zl[u] / (x[u] - DLO[j]) * dx[u];
                    if (hasb(DHI[j])) bb = mu / (DHI[j] - x[u]) - zu[u] + zu[u] / (DHI[j] - x[u]) * dx[u];
                }
                if (hasb(lo[u])) c = mu / (xs[u] - lo[u]) - vl[u] - vl[u] / (xs[u] - lo[u]) * dxs[u];
                if (hasb(hi[u])) d = mu / (hi[u] - xs[u]) - vu[u] + vu[u] / (hi[u] - xs[u]) * dxs[u];
                dzdL[e] = a; dzdU[e] = bb; dvL[e] = c; dvU[e] = d;
                if (k > 0) {
                    if (hasb(DLO[j])) { ftbL(x[u], dx[u], DLO[j], ap); ftbZ(zl[u], a, az); }
                    if (hasb(DHI[j])) { ftbU(x[u], dx[u], DHI[j], ap); ftbZ(zu[u], bb, az); }
                }
                if (hasb(lo[u])) { ftbL(xs[u], dxs[u], lo[u], ap); ftbZ(vl[u], c, az); }
                if (hasb(hi[u])) { ftbU(xs[u], dxs[u], hi[u], ap); ftbZ(vu[u], d, az); }
            }
        }
    }
    // gdot = grad(phi)^T dx, pHp = dx^T (W + Sigma) dx = pcorr + dx^T H0 dx + the q_N barrier term;
    // thread e covers row v of node k's H0 (stored as its lower triangle)
    double gdot = 0.0, pHp = pcorr;
    for (int e0 = tid; e0 < N * NV; e0 += NT * 2) {
        double acc[2], gd[2];
#pragma unroll
        for (int u = 0; u < 2; u++) {
            const int e = min(e0 + NT * u, N * NV - 1);
            const int k = e / NV, v = e % NV;
            double dx[NV];
#pragma unroll
            for (int j = 0; j < NJ; j++) { dx[j] = dq[k * n + j]; dx[NJ + j] = dqd[k * n + j]; }
#pragma unroll
            for (int a = 0; a < NF; a++) dx[2 * NJ + a] = dF[k * NFA + a];
            const double *Wr = W + (size_t)k * NV * NV + (size_t)v * NV;
            double a = 0.0, dv = 0.0;
#pragma unroll
            for (int w = 0; w < NV; w++) {
                const double hw = Wr[w];  // loaded unconditionally; the upper part is stale, never used
                a += (w < v ? 2.0 * hw : (w == v ? hw : 0.0)) * dx[w];
                if (w == v) dv = dx[w];
            }
            acc[u] = a * dv;
            gd[u] = gf[e] * dv;
        }
#pragma unroll
        for (int u = 0; u < 2; u++)
            if (e0 + NT * u < N * NV) { pHp += acc[u]; gdot += gd[u]; }
    }
    for (int e0 = tid; e0 < N * n; e0 += NT * UB) {
        double g1[UB], g2[UB], g3[UB];
#pragma unroll
        for (int u = 0; u < UB; u++) {
            const int e = min(e0 + NT * u, N * n - 1);
            const double dqv = dq[e + n];
            g1[u] = gphd[e] * dqd[e] + gphs[e] * ds[e];
            g2[u] = gphq[e + n] * dqv;
            g3[u] = (e + n >= N * n) ? Sxq[e + n] * dqv * dqv : 0.0;  // q_N (stages k < N carry Sigma_x in H0)
        }
#pragma unroll
        for (int u = 0; u < UB; u++)
            if (e0 + NT * u < N * n) { gdot += g1[u] + g2[u]; pHp += g3[u]; }
    }
    // merit terms at the iterate from the node evaluation of this iteration (the same values the
    // line search's value sweep gives at alpha = 0, to round-off): objective, barrier, violation
    // the barrier term -sum log(gap) is taken as -log of the gaps' product, renormalised per element
    // (mantissa pm, binary exponent pe): one log per thread instead of one per bound
    double f0 = 0.0, bar0 = 0.0, th0 = 0.0, pm = 1.0;
    int pe = 0, pe_ = 0;
    for (int k = tid; k < N; k += NT) {
        f0 += cost[k];
        if (LINE_ON(k))
#pragma unroll
            for (int l = 0; l < NL; l++) th0 += fabs(line[k * nl + l]);
    }
    for (int e0 = tid; e0 < N * n; e0 += NT * UB) {
        double xq[UB], xd[UB], xs[UB], tv[UB], qa[UB], lo[UB], hi[UB];
#pragma unroll
        for (int u = 0; u < UB; u++) {
            const int e = min(e0 + NT * u, N * n - 1);
            xq[u] = q[e + n]; qa[u] = q[e]; xd[u] = qd[e]; xs[u] = s[e]; tv[u] = tau[e]; lo[u] = tlo[e]; hi[u] = thi[e];
        }
#pragma unroll
        for (int u = 0; u < UB; u++) {
            const int e = e0 + NT * u;
            if (e < N * n) {
                const int k = e / n, j = e % n;
                if (hasb(lo[u]) || hasb(hi[u])) th0 += fabs(tv[u] - xs[u]);
                th0 += fabs(qa[u] + h * xd[u] - xq[u]);
                if (hasb(QLO[j])) pm *= xq[u] - QLO[j];
                if (hasb(QHI[j])) pm *= QHI[j] - xq[u];
                if (k > 0) {
                    if (hasb(DLO[j])) pm *= xd[u] - DLO[j];
                    if (hasb(DHI[j])) pm *= DHI[j] - xd[u];
                }
                if (hasb(lo[u])) pm *= xs[u] - lo[u];
                if (hasb(hi[u])) pm *= hi[u] - xs[u];
                pm = frexp(pm, &pe_);
                pe += pe_;
            }
        }
    }
    bar0 = -(log(pm) + pe * 0.69314718055994530942);
    double mx[2] = {-ap, -az}, sm[5] = {gdot, pHp, f0, bar0, th0};
    block_reduce<NT, 2, 5>(mx, sm, red);
    out[0] = -mx[0];
    out[1] = -mx[1];
    out[2] = sm[0];
    out[3] = sm[1];
    out[4] = sm[2] + mu * sm[3];
    out[5] = sm[4];
}

template <int NJ, int NF, int NL>
__global__ __launch_bounds__(64, 3) void k_ipm_kkt(const DevModel *__restrict__ Mg, const DevFrame *__restrict__ Fg,
                                                 OcpConst C, IpmArrays A, int batch) {
    constexpr int n = NJ, nf = NF, nl = NL;
    constexpr int NV = 2 * NJ + NF;
    constexpr int NFA = NF > 0 ? NF : 1;
    constexpr int NLA = NL > 0 ? NL : 1;
    constexpr int MB = 3 * NJ + NF + NL;
    __shared__ ModelLds<NJ> Ml;
    const DevModel &M = Ml.get();
    __shared__ DevFrame F;
    __shared__ int perm[MB], piv[MB];
    const int lane = threadIdx.x;
    if ((int)blockIdx.x >= *A.nrun) return;
    const int b = A.list[blockIdx.x];
    ProbState st = A.st[b];
    if (st.status != ST_RUNNING) return;
    Ml.load(Mg);
    stage_lds(&F, Fg);
    __shared__ double Bnd[4 * NJ];  // q_lo, q_hi, qd_lo, qd_hi (kernel-argument arrays read per element)
    if (lane < NJ) {
        Bnd[lane] = C.q_lo[lane];
        Bnd[NJ + lane] = C.q_hi[lane];
        Bnd[2 * NJ + lane] = C.qd_lo[lane];
        Bnd[3 * NJ + lane] = C.qd_hi[lane];
    }
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
    const double *QLO = Bnd, *QHI = Bnd + NJ, *DLO = Bnd + 2 * NJ, *DHI = Bnd + 3 * NJ;
#define TACT(k, j) (hasb(tlo[(k) * n + (j)]) || hasb(thi[(k) * n + (j)]))

    const double kappa_eps = 10.0, kappa_mu = 0.2, theta_mu = 1.5, tau_min = 0.99, s_max = 100.0;
    const double kappa_sigma = 1e10, eta = 1e-4, rho = 0.1;
    double mu = st.mu, nu = st.nu;
    constexpr int UB = 2;  // element-loop chunk (see the optimality-error phase)
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
    // H0 is stored as its lower triangle (k_eval_asm): lane entry e = (u, v) reads (max, min)
    int hlo[NHR];
#pragma unroll
    for (int t = 0; t < NHR; t++) {
        const int e = min(lane + 64 * t, NVV - 1), u = e / NV, v = e % NV;
        hlo[t] = u >= v ? e : v * NV + u;
    }
    constexpr int SLOT = MB * NJ + MB;       // Riccati slot (G_k | wv_k) doubles
    __shared__ double Hs[NVV];
    __shared__ double Ps[NJ * NJ], ps[NJ], ss[NJ], Pn[NJ * (NJ + 1)];
    __shared__ double Ks[NK * LDK], Rk[NK * NRK];
    __shared__ double Gl[NLA2 * NJ];
    constexpr int NRS = NU > 2 ? NU - 2 : 1;
    __shared__ double Ss5[NRS * NRS + 4 * NRS + 3];  // reduced Hessian + tables (stage_ns.hpp)
    __shared__ double Jl_s[NJ * NV];  // J_k (torque Jacobian) of the stage, regularised tries only
    // per-stage inputs of the recursion, computed for all stages at once by the whole wave (global
    // scratch, stage k contiguous): g_k (NV), c_k = q_k + h qd_k - q_{k+1} (NJ),
    // e_k = line_{k+1} + Jl_{k+1} c_k (NLA2), dD_k = D_tau(dw, dc) - Sigma_s (NJ); then
    // y_tau + D_tau r_tau (N x NJ, used inside prep only)
    constexpr int SG = NV + 2 * NJ + NLA2;
    double *stg = A.stg + b * S.stg;
    double *wst = stg + (size_t)N * SG;
    __shared__ double Stg[SG];  // stage k's block, staged from a register prefetch
    auto prep_stages = [&](double dwv, double dcv) {
        prep_stage_inputs<NJ, NF, NL, 64>(C, A, b, lane, dwv, dcv, [] { wave_mem_sync(); });
    };
    double dw, dc = 0.0, dFr, reg;
    const int reg_tier0 = st.reg_tier;
    const double reg_last0 = st.reg_last;
    int tier, step_no = 0;
    kkt_first_try(st, tier, reg, dw, dFr);
    bool factor_ok = false;
    int ntries = 0;
    double prep_dw = dw, prep_dc = 0.0;  // k_ipm_pre wrote the first try's stage inputs
    for (int tries = 0; tries < 60; tries++) {
        ntries++;
        bool ok = true, zero = false;
        if (!(dw == prep_dw && dc == prep_dc)) {
            prep_stages(dw, dc);
            prep_dw = dw;
            prep_dc = dc;
        }
        const bool dreg = (dw != 0.0 || dc != 0.0);
        const bool dgreg = (dw != 0.0 || dFr != 0.0);  // diagonal regularisation of H
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
            hr[t] = (e < NVV) ? W[(size_t)(N - 1) * NVV + hlo[t]] : 0.0;
        }
#pragma unroll
        for (int t = 0; t < NJR; t++) {
            const int e = lane + 64 * t;
            jr[t] = (dreg && e < NJV) ? Jt[(size_t)(N - 1) * NJV + e] : 0.0;
        }
        double glr = 0.0;  // Jl_{k+1} entry of this lane for the next stage
        double sgr = (lane < SG) ? stg[(size_t)(N - 1) * SG + lane] : 0.0;  // stage block, one ahead
        // block row of Rk holding slot row c (slot rows in control order: qd 0..n-1, F, then the
        // NL line multipliers)
        auto brow = [&](int c) { return c < NU ? (c < NJ ? NF + c : c - NJ) : c; };
        wave_lds_sync();
        for (int k = N - 1; k >= 0; k--) {
            const int lane = lane_opaque();  // per-stage index arithmetic stays inside the stage
            // ---- H_k = H0_k (+ regularisation) into LDS; prefetch H0_{k-1}, Jl_k (, J_{k-1})
            STAMP(18);
            if (lane < SG) Stg[lane] = sgr;
            STAMP(19);
            if (dreg) {
#pragma unroll
                for (int t = 0; t < NJR; t++) {
                    const int e = lane + 64 * t;
                    if (e < NJV) Jl_s[e] = jr[t];
                }
                wave_lds_sync();
            }
            const double *dDk = Stg + NV + NJ + NLA2;
#pragma unroll
            for (int t = 0; t < NHR; t++) {
                const int e = lane + 64 * t;
                if (e < NVV) {
                    const int u = e / NV, v = e % NV;
                    double a = hr[t];
                    if (dreg)
#pragma unroll
                        for (int jj = 0; jj < NJ; jj++) a += Jl_s[jj * NV + u] * dDk[jj] * Jl_s[jj * NV + v];
                    if (dgreg && u == v) a += dw + (u >= 2 * n ? dFr : 0.0);
                    Hs[e] = a;
                }
            }
            if (lane < nl * n) Gl[lane] = glr;
            STAMP(7);
            // ---- Riccati slot stores, then the prefetch loads.  vmcnt retires in order, so the
            // next stage's wait for its prefetched operands also waits for every store issued
            // before it: stores issued at the end of a stage (where the slot used to be written)
            // put a full store round trip on the path of the next stage; issued here, they
            // complete behind the stage's own work.  P_{k+1}, p_{k+1} (slot k) are in Ps / ps;
            // stage k+1's Ku, Kl, ku, kl (slot k+1) are still in Rk.
            double *Gk = G + (size_t)k * MB * n, *wk = wv + (size_t)k * MB;
            if (lane < n) wk[NU + NL + lane] = ps[lane];
            for (int e = lane; e < n * n; e += 64) Gk[(NU + NL) * n + e] = Ps[e];
            if (k + 1 < N) {
                double *G1 = G + (size_t)(k + 1) * MB * n, *w1 = wv + (size_t)(k + 1) * MB;
                for (int e = lane; e < NK * n; e += 64) G1[e] = Rk[brow(e / n) * NRK + e % n];  // Ku (NU x n), Kl (NL x n)
                if (lane < NK) w1[lane] = Rk[brow(lane) * NRK + n];                             // ku, kl
            }
            if (k > 0) {
                // unconditional loads from clamped addresses (a load whose value is selected
                // against a constant is waited for on the spot)
#pragma unroll
                for (int t = 0; t < NHR; t++) hr[t] = W[(size_t)(k - 1) * NVV + hlo[t]];
                if constexpr (NL > 0) glr = Jl[(size_t)k * nl * n + min(lane, nl * n - 1)];
                sgr = stg[(size_t)(k - 1) * SG + min(lane, SG - 1)];
                if (dreg)
#pragma unroll
                    for (int t = 0; t < NJR; t++) jr[t] = Jt[(size_t)(k - 1) * NJV + min(lane + 64 * t, NJV - 1)];
            }
            // s = P c + p
            const double *ck = Stg + NV;
            if (lane < n) {
                const int j = lane;
                double a = ps[j];
#pragma unroll
                for (int i = 0; i < NJ; i++) a += Ps[j * n + i] * ck[i];
                ss[j] = a;
            }
            wave_lds_sync();
            STAMP(11);
            const double *gsk = Stg;
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
            const double *elk = Stg + NV + NJ;
            // ---- stage solve: null-space elimination (stage_ns.hpp) when the two line rows are
            // active and dc = 0, the pivoted Bunch-Kaufman block otherwise
            auto uo = [&](int a) { return a < NF ? NJ + a : a - NF; };
            int nsr = -1;
            if constexpr (NL == 2) {
                if (con && dc == 0.0) nsr = stage_nullspace<NJ, NF, NV, NRK>(Hs, Ps, ss, Gl, gsk, elk, h, Ss5, Rk);
            }
            STAMP(13);
            STAMP_COUNT(17, 1);
            STAMP_COUNT(16, nsr < 0 ? 1 : 0);
            if (nsr == 0) { ok = false; break; }
            if (nsr < 0) {
                // ---- stage block [[Quu, Du^T], [Du, -dc]] and right-hand sides -[Qux | qu ; G | e]
                // Block rows order the controls as (F, qd): with active torque bounds the force
                // carries the large curvature Sigma_s (J^T F)^2 and the joint velocities couple to it
                // weakly, so natural-order 1x1 pivots pass the Bunch-Kaufman test (ldl_schur_regs).
                // uo(a): control index (qd 0..n-1, F n..) of block row a < NU.
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
                if (fast) {
                    if (in.pos != NU || in.neg != NL) { ok = false; break; }
                } else {
                    in = bk_factor_fixed<LDK, NK>(Ks, perm, piv);
                    if (in.zero) { ok = false; zero = true; break; }
                    if (in.pos != NU || in.neg != NL) { ok = false; break; }
                    bk_solve_cols<LDK, NRK, NK>(Ks, perm, piv, Rk, NRK);
                }
            }
            STAMP(14);
            // ---- P_k = Qxx + Qxu Ku + G^T Kl ; p_k = qx + Qxu ku + G^T kl   (block row a <-> control uo(a))
            // one pass over the n x (n + 1) entries [P_k | p_k] (column n of Rk holds ku, kl)
            for (int e = lane; e < n * (n + 1); e += 64) {
                const int i = e / (n + 1), j = e % (n + 1);
                double a = (j < n) ? Hs[i * NV + j] + Ps[i * n + j] : gsk[i] + ss[i];
                for (int r = 0; r < NU; r++) {
                    const int c = uo(r);
                    a += (Hs[i * NV + n + c] + (c < n ? h * Ps[i * n + c] : 0.0)) * Rk[r * NRK + j];
                }
                if (con)
                    for (int l = 0; l < nl; l++) a += Gl[l * n + i] * Rk[(NU + l) * NRK + j];
                Pn[e] = a;
            }
            // (Ku, Kl, ku, kl stay in Rk: the next stage stores them, see the slot stores)
            wave_lds_sync();
            for (int e = lane; e < n * n; e += 64) {
                int i = e / n, j = e % n;
                Ps[e] = 0.5 * (Pn[i * (n + 1) + j] + Pn[j * (n + 1) + i]);
            }
            if (lane < n) ps[lane] = Pn[lane * (n + 1) + n];
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
    // ---------------- forward sweep, serial part: dx_{k+1} = dx_k + h du_k + c_k with
    //   (dqd_k, dF_k) = Ku dx_k + ku and dyl_{k+1} = Kl dx_k + kl (stage k's slot).  Lane a < NK
    //   holds row a of [Ku ku; Kl kl] in registers, fetched FD stages ahead straight from global
    //   memory, and dx_k is held uniformly by every lane (readlane broadcast of the six new
    //   entries): a stage is one dot product, one update and the broadcast -- no LDS round trip.
    //   dyc_k = P_{k+1} dx_{k+1} + p_{k+1} + Jl_{k+1}^T dyl_{k+1} does not feed the recursion and
    //   is recovered afterwards for all stages at once.
    // Every load is unconditional from a clamped address (a value selected between a load and a
    // constant makes the compiler wait for the load on the spot, which would empty the ring).
    constexpr int FD = 4;
    const int ra = min(lane, NK - 1);  // slot row of this lane: qd 0..n-1, F, then the line multipliers
    double rowr[FD][NJ], wkr[FD], ckr[FD];
    auto fetch = [&](int kk, double *row, double &wk, double &ck) {
        const double *src = G + (size_t)kk * MB * n + (size_t)ra * n;
        if constexpr (NJ % 2 == 0) {
            const double2 *s2 = reinterpret_cast<const double2 *>(src);  // 16-byte aligned: MB n, n even
#pragma unroll
            for (int t = 0; t < NJ / 2; t++) {
                const double2 v2 = s2[t];
                row[2 * t] = v2.x;
                row[2 * t + 1] = v2.y;
            }
        } else {
#pragma unroll
            for (int i = 0; i < NJ; i++) row[i] = src[i];
        }
        wk = wv[(size_t)kk * MB + ra];
        ck = stg[(size_t)kk * SG + NV + min(lane, NJ - 1)];
    };
#pragma unroll
    for (int r = 0; r < FD; r++) fetch(min(r, N - 1), rowr[r], wkr[r], ckr[r]);
    double xsv[NJ];  // dx_k, the same in every lane
#pragma unroll
    for (int j = 0; j < NJ; j++) xsv[j] = stg[NV + j];  // dx_1 = c_0 (dx_0 = 0, dqd_0 = 0)
    for (int j = lane; j < n; j += 64) { dq[j] = 0.0; dqd[j] = 0.0; }
    for (int l = lane; l < nl; l += 64) { dyl[l] = 0.0; dyl[nl + l] = 0.0; }
    for (int k0 = 0; k0 < N; k0 += FD) {
#pragma unroll
        for (int r = 0; r < FD; r++) {
            const int k = k0 + r;
            if (k >= N) break;
            double row[NJ], wk = wkr[r], ck = ckr[r];
#pragma unroll
            for (int i = 0; i < NJ; i++) row[i] = rowr[r][i];
            fetch(min(k + FD, N - 1), rowr[r], wkr[r], ckr[r]);  // past the end: slot N-1 again, unused
            if (k == 0) {  // only dF_0 is free; it sits in the ku slot of stage 0
                if (lane >= NJ && lane < NU) dF[lane - NJ] = wk;
                continue;
            }
            double us = wk;
#pragma unroll
            for (int i = 0; i < NJ; i++) us += row[i] * xsv[i];
            const bool con1 = (nl > 0) && LINE_ON(k + 1) && (k + 1 <= N - 1);
            double xj = xsv[0];
#pragma unroll
            for (int j = 1; j < NJ; j++) xj = (lane == j) ? xsv[j] : xj;
            const double cs = xj + h * us + ck;  // dx_{k+1}, entry `lane` (lanes < n)
            if (lane < n) {
                dq[k * n + lane] = xj;
                dqd[k * n + lane] = us;
            } else if (lane < NU) {
                dF[k * NFA + lane - NJ] = us;
            } else if (lane < NK) {
                if (k + 1 < N) dyl[(k + 1) * nl + lane - NU] = con1 ? us : 0.0;
            }
#pragma unroll
            for (int j = 0; j < NJ; j++) xsv[j] = readlane_d(cs, j);
        }
    }
    for (int j = lane; j < n; j += 64) dq[N * n + j] = xsv[j];
    // dyc, dyd, ds, the bound multiplier steps and pcorr: k_kkt_recover (a block per horizon)
    STAMP(3);
    STAMP_FLUSH;
    if (lane == 0) {
        st.kkt_dw = dw;
        st.kkt_dc = dc;
        A.st[b] = st;
    }
#undef TACT
}

template <int NJ, int NF, int NL>
__global__ __launch_bounds__(128) void k_ipm_post(const DevModel *__restrict__ Mg, const DevFrame *__restrict__ Fg,
                                                 OcpConst C, IpmArrays A, int batch) {
    constexpr int n = NJ, nf = NF, nl = NL;
    constexpr int NV = 2 * NJ + NF;
    constexpr int NFA = NF > 0 ? NF : 1;
    constexpr int NLA = NL > 0 ? NL : 1;
    constexpr int MB = 3 * NJ + NF + NL;
    __shared__ ModelLds<NJ> Ml;
    const DevModel &M = Ml.get();
    __shared__ DevFrame F;
    constexpr int NT = 128;  // two waves per horizon: every node of the merit sweep in one pass (N <= 128)
    __shared__ double red[8 * (NT / 64)];
    const int lane = threadIdx.x;
    if ((int)blockIdx.x >= *A.nrun) return;
    const int b = A.list[blockIdx.x];
    ProbState st = A.st[b];
    if (st.status != ST_RUNNING) return;
    Ml.load(Mg);
    stage_lds(&F, Fg);
    __shared__ double Bnd[4 * NJ];  // q_lo, q_hi, qd_lo, qd_hi (kernel-argument arrays read per element)
    if (lane < NJ) {
        Bnd[lane] = C.q_lo[lane];
        Bnd[NJ + lane] = C.q_hi[lane];
        Bnd[2 * NJ + lane] = C.qd_lo[lane];
        Bnd[3 * NJ + lane] = C.qd_hi[lane];
    }
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
    const double *QLO = Bnd, *QHI = Bnd + NJ, *DLO = Bnd + 2 * NJ, *DHI = Bnd + 3 * NJ;
#define TACT(k, j) (hasb(tlo[(k) * n + (j)]) || hasb(thi[(k) * n + (j)]))

    const double kappa_eps = 10.0, kappa_mu = 0.2, theta_mu = 1.5, tau_min = 0.99, s_max = 100.0;
    const double kappa_sigma = 1e10, eta = 1e-4, rho = 0.1;
    double mu = st.mu, nu = st.nu;
    constexpr int UB = 2;  // element-loop chunk (see the optimality-error phase)
    auto finish = [&](int status) {
        STAMP_FLUSH;
        double f = 0.0;
        for (int k = lane; k < N; k += NT) f += cost[k];
        f = block_sum<NT>(f, red);
        if (lane == 0) {
            st.status = status;
            st.obj = f;
            st.mu = mu;
            st.nu = nu;
            A.st[b] = st;
            atomicSub(A.active, 1);
        }
    };
    const double tau_fb = st.tau_fb;
    // ---------------- step recovery, fraction to the boundary, merit slope and curvature (kkt_recover_body)
    double rcv[6];
    kkt_recover_body<NJ, NF, NL, NT>(C, A, b, st, Bnd, red, rcv);
    __syncthreads();  // the recovered steps (ds, dy, dz, dv) are read by other threads below
    const double ap = rcv[0], az = rcv[1];
    st.ap = ap;
    st.az = az;
    TRACE(9, ap); TRACE(10, az);

    // ---------------- merit at the current point, directional derivative, curvature
    // merit of a point (x + alpha dx).  Each lane sweeps its nodes with node_values; the node's
    // iterate and step are loaded into registers before the sweep starts.
    const int fpj = (NF > 0 || NL > 0) ? F.parent : -1;
    auto merit = [&](double alpha, double &phi, double &theta, bool &ok_out) {
        double f = 0, bar = 0, th = 0, pm = 1.0;  // barrier: -log of the gaps' product, renormalised per element
        int pe = 0, pe_ = 0;
        int bad = 0;
        for (int k = lane; k < N; k += NT) {
            // only the sweep's inputs are held through the sweep; slacks, bounds and q_{k+1} are
            // read after it (register budget of the sweep)
            double tq[NJ], tqd[NJ], tv[NJ], Fw[3], c = 0.0;
#pragma unroll
            for (int j = 0; j < NJ; j++) {
                tq[j] = q[k * n + j] + alpha * dq[k * n + j];
                tqd[j] = qd[k * n + j] + alpha * dqd[k * n + j];
            }
#pragma unroll
            for (int r = 0; r < 3; r++) Fw[r] = 0.0;
#pragma unroll
            for (int a = 0; a < NF; a++) {
                const double tF = Fv[k * NFA + a] + alpha * dF[k * NFA + a];
                c += C.wF * tF * tF;
#pragma unroll
                for (int r = 0; r < 3; r++) Fw[r] += tF * C.fdir[3 * a + r];
            }
            struct MOut {
                double *tv;
                const double *lref;
                double th;
                int nl;
                bool line;
                __device__ void frame(const double *p) {
                    if (line)
                        for (int l = 0; l < nl; l++) th += fabs(p[l] - lref[l]);
                }
                __device__ void force(const double *) {}
                __device__ void joint(int j, double t, double, double) { tv[j] = t; }
            } mo{tv, lref, 0.0, nl, LINE_ON(k)};
            ArrIn<NJ> tin{tq, tqd};
            node_values<NJ>(M, F, fpj, tin, Fw, mo);
#pragma unroll
            for (int j = 0; j < NJ; j++) {
                const double sl = s[k * n + j] + alpha * ds[k * n + j];
                const double qn = q[(k + 1) * n + j] + alpha * dq[(k + 1) * n + j];
                const double lo = tlo[k * n + j], hi = thi[k * n + j];
                c += C.wqd * tqd[j] * tqd[j] + C.wtau * tv[j] * tv[j];
                if (hasb(lo) || hasb(hi)) th += fabs(tv[j] - sl);
                th += fabs(tq[j] + h * tqd[j] - qn);
            }
            f += c;
            th += mo.th;
        }
        for (int e0 = lane; e0 < N * n; e0 += NT * UB) {
            double xq[UB], xd[UB], xs[UB], lo[UB], hi[UB];
#pragma unroll
            for (int u = 0; u < UB; u++) {
                const int e = min(e0 + NT * u, N * n - 1);
                xq[u] = q[e + n] + alpha * dq[e + n];
                xd[u] = qd[e] + alpha * dqd[e];
                xs[u] = s[e] + alpha * ds[e];
                lo[u] = tlo[e];
                hi[u] = thi[e];
            }
#pragma unroll
            for (int u = 0; u < UB; u++) {
                const int e = e0 + NT * u;
                if (e < N * n) {
                    const int k = e / n, j = e % n;
                    if (hasb(QLO[j])) { if (xq[u] - QLO[j] <= 0) bad = 1; else pm *= xq[u] - QLO[j]; }
                    if (hasb(QHI[j])) { if (QHI[j] - xq[u] <= 0) bad = 1; else pm *= QHI[j] - xq[u]; }
                    if (k > 0) {
                        if (hasb(DLO[j])) { if (xd[u] - DLO[j] <= 0) bad = 1; else pm *= xd[u] - DLO[j]; }
                        if (hasb(DHI[j])) { if (DHI[j] - xd[u] <= 0) bad = 1; else pm *= DHI[j] - xd[u]; }
                    }
                    if (hasb(lo[u])) { if (xs[u] - lo[u] <= 0) bad = 1; else pm *= xs[u] - lo[u]; }
                    if (hasb(hi[u])) { if (hi[u] - xs[u] <= 0) bad = 1; else pm *= hi[u] - xs[u]; }
                    pm = frexp(pm, &pe_);
                    pe += pe_;
                }
            }
        }
        bar = -(log(pm) + pe * 0.69314718055994530942);
        {
            double sm[4] = {f, bar, th, (double)bad};
            block_reduce<NT, 0, 4>(nullptr, sm, red);
            f = sm[0]; bar = sm[1]; th = sm[2];
            bad = sm[3] != 0.0 ? 1 : 0;
        }
        phi = f + mu * bar;
        theta = th;
        ok_out = (bad == 0);
    };
    // merit at the current point from this iteration's node evaluation (k_kkt_recover); it equals the
    // value sweep at alpha = 0 to round-off, which the acceptance test's 10 eps |m0| allowance covers
    const double phi0 = rcv[4], th0 = rcv[5];
    // gdot = grad(phi)^T dx, pHp = dx^T (W + Sigma) dx (k_kkt_recover)
    const double gdot = rcv[2], pHp = rcv[3];
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

    st.alpha = alpha;
    STAMP(6);
    STAMP_COUNT(10, 1);
    STAMP_FLUSH;
    // ---------------- update: the primal-dual step with alpha, the bound multipliers with az and the new
    // slacks (formerly the k_post_update launch: the same element loops, now by this block's 128 threads)
    __syncthreads();  // every merit sweep has read the iterate
    {
        auto zupd = [&](double z, double dz, double slack) {
            const double zz = z + az * dz;
            return fmax(fmin(zz, kappa_sigma * mu / slack), mu / (kappa_sigma * slack));
        };
        for (int e0 = lane; e0 < (N + 1) * n; e0 += NT * UB) {
            double x[UB], dx[UB], zl[UB], dzl[UB], zu[UB], dzu[UB];
#pragma unroll
            for (int u = 0; u < UB; u++) {
                const int e = min(e0 + NT * u, (N + 1) * n - 1);
                x[u] = q[e]; dx[u] = dq[e]; zl[u] = zqL[e]; dzl[u] = dzqL[e]; zu[u] = zqU[e]; dzu[u] = dzqU[e];
            }
#pragma unroll
            for (int u = 0; u < UB; u++) {
                const int e = e0 + NT * u;
                if (e < (N + 1) * n) {
                    const int j = e % n;
                    const double xn = x[u] + alpha * dx[u];
                    q[e] = xn;
                    if (e >= n) {
                        if (hasb(QLO[j])) zqL[e] = zupd(zl[u], dzl[u], xn - QLO[j]);
                        if (hasb(QHI[j])) zqU[e] = zupd(zu[u], dzu[u], QHI[j] - xn);
                    }
                }
            }
        }
        for (int e0 = lane; e0 < N * n; e0 += NT * UB) {
            double x[UB], xs[UB], zl[UB], zu[UB], vl[UB], vu[UB], lo[UB], hi[UB], yn[UB], dn[UB];
#pragma unroll
            for (int u = 0; u < UB; u++) {
                const int e = min(e0 + NT * u, N * n - 1);
                x[u] = qd[e] + alpha * dqd[e];
                xs[u] = s[e] + alpha * ds[e];
                yn[u] = yc[e] + alpha * dyc[e];
                dn[u] = yd[e] + alpha * dyd[e];
                zl[u] = zdL[e] + az * dzdL[e]; zu[u] = zdU[e] + az * dzdU[e];
                vl[u] = vL[e] + az * dvL[e]; vu[u] = vU[e] + az * dvU[e];
                lo[u] = tlo[e]; hi[u] = thi[e];
            }
            auto clampz = [&](double zz, double slack) {
                return fmax(fmin(zz, kappa_sigma * mu / slack), mu / (kappa_sigma * slack));
            };
#pragma unroll
            for (int u = 0; u < UB; u++) {
                const int e = e0 + NT * u;
                if (e < N * n) {
                    const int k = e / n, j = e % n;
                    qd[e] = x[u]; s[e] = xs[u]; yc[e] = yn[u]; yd[e] = dn[u];
                    if (k > 0) {
                        if (hasb(DLO[j])) zdL[e] = clampz(zl[u], x[u] - DLO[j]);
                        if (hasb(DHI[j])) zdU[e] = clampz(zu[u], DHI[j] - x[u]);
                    }
                    if (hasb(lo[u])) vL[e] = clampz(vl[u], xs[u] - lo[u]);
                    if (hasb(hi[u])) vU[e] = clampz(vu[u], hi[u] - xs[u]);
                }
            }
        }
        if constexpr (NF > 0)
            for (int e = lane; e < N * nf; e += NT) Fv[(e / nf) * NFA + e % nf] += alpha * dF[(e / nf) * NFA + e % nf];
        if constexpr (NL > 0)
            for (int e = lane; e < N * nl; e += NT) yl[e] += alpha * dyl[e];
    }
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

// ============================================================== running-set compaction
// One block: list[0..nrun) = the problems still ST_RUNNING, in index order (wave ballots + a
// 16-entry scan per 1024-problem chunk).  Run after k_ipm_init and after every k_ipm_post; the
// per-iteration kernels then size their grids from the host's last count of running problems
// (an upper bound of nrun, which only falls) and map slots through the list.
__global__ __launch_bounds__(1024) void k_compact(IpmArrays A, int batch) {
    __shared__ int wsum[16];
    __shared__ int base;
    const int tid = threadIdx.x, ln = tid & 63, wv = tid >> 6;
    if (tid == 0) base = 0;
    __syncthreads();
    for (int c0 = 0; c0 < batch; c0 += 1024) {
        const int b = c0 + tid;
        const bool r = b < batch && A.st[b].status == ST_RUNNING;
        const unsigned long long m = __ballot(r);
        if (ln == 0) wsum[wv] = __popcll(m);
        __syncthreads();
        int off = base;
        for (int w = 0; w < wv; w++) off += wsum[w];
        if (r) A.list[off + __popcll(m & ((1ull << ln) - 1ull))] = b;
        __syncthreads();
        if (tid == 0) {
            int t = 0;
            for (int w = 0; w < 16; w++) t += wsum[w];
            base += t;
        }
        __syncthreads();
    }
    if (tid == 0) A.nrun[0] = base;
}

// ============================================================== host launchers
template <int NJ, int NF, int NL>
struct IpmLaunch {
    static void init(const DevModel *M, const DevFrame *F, const OcpConst &C, const IpmArrays &A, int batch,
                     hipStream_t s) {
        hipLaunchKernelGGL((k_ipm_init<NJ, NF, NL>), dim3(batch), dim3(64), 0, s, M, F, C, A, batch);
        hipLaunchKernelGGL(k_compact, dim3(1), dim3(1024), 0, s, A, batch);
    }
    // phase 0: node derivatives (k_eval_node), 1: stage-Hessian assembly (k_eval_asm),
    // 2..4: per-problem IPM phases (k_ipm_pre, k_ipm_kkt, k_ipm_post)
    // grids cover `nact` problems (>= the running count), slots mapped through A.list
    static void iter(int phase, const DevModel *M, const DevFrame *F, const OcpConst &C, const IpmArrays &A,
                     int batch, int nact, hipStream_t s) {
        constexpr int NPB = 4 * (64 / NJ);        // k_eval_node: nodes per block (one direction class)
        constexpr int NPBA = 256 / (2 * NJ + NF);  // k_eval_asm: nodes per block
        if (nact < 1) return;
        long nodes = (long)nact * C.N;
        if (phase == 0) {
            const int nb = (int)((nodes + NPB - 1) / NPB);
            const long ngrp8 = ((nodes + 63) / 64 + 7) / 8;  // node groups of 64, in rounds of 8 (one per XCD)
            hipLaunchKernelGGL((k_eval_q<NJ, NF, NL>), dim3((unsigned)(ngrp8 * 8 * NJ)), dim3(64), 0, s, M, F, C, A,
                               batch);
            hipLaunchKernelGGL((k_eval_node<NJ, NF, NL, 1>), dim3(nb), dim3(256), 0, s, M, F, C, A, batch, nb);
        } else if (phase == 1) {
            hipLaunchKernelGGL((k_eval_asm<NJ, NF, NL>), dim3((unsigned)((nodes + NPBA - 1) / NPBA)), dim3(256), 0, s,
                               C, A, batch);
        } else if (phase == 2) {
            hipLaunchKernelGGL((k_ipm_pre<NJ, NF, NL>), dim3(nact), dim3(256), 0, s, M, F, C, A, batch);
        } else if (phase == 3) {
            hipLaunchKernelGGL((k_ipm_kkt<NJ, NF, NL>), dim3(nact), dim3(64), 0, s, M, F, C, A, batch);
        } else {
            hipLaunchKernelGGL((k_ipm_post<NJ, NF, NL>), dim3(nact), dim3(128), 0, s, M, F, C, A, batch);
            hipLaunchKernelGGL(k_compact, dim3(1), dim3(1024), 0, s, A, batch);
        }
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
                  const IpmArrays &A, int batch, int nact, hipStream_t s, double *w, int *status, int *iters,
                  double *kkt, double *obj) {
#define MF_CASE(NJ, NF, NL)                                                       \
    if (n == NJ && nf == NF && nl == NL) {                                        \
        if (what == 0) IpmLaunch<NJ, NF, NL>::init(M, F, C, A, batch, s);          \
        else if (what >= 10 && what <= 14) IpmLaunch<NJ, NF, NL>::iter(what - 10, M, F, C, A, batch, nact, s); \
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
