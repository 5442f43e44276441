// Generic batched interior-point solver for stage-structured OCPs on MI355X (gfx950):
// the dual-arm box (C3, python/2_pilz_6_DOF/Box_Pilz_6DOF.py:219-456) and the thermal-fatigue
// transcriptions (Tmodel_library.py:9-41, RepeatedMPCwithThermal.py:371-376), plus the Pilz chain
// tasks through the same path.  The iteration is the one of DESIGN.md section 4 (IPOPT-style
// primal-dual interior point, monotone mu, inertia correction, l1-merit line search with IPOPT's
// second-order corrections); the CPU restatement is oracle/mf_ocp.c (block-tridiagonal
// Bunch-Kaufman), this file factorises the same KKT matrix by a Riccati recursion with general
// dynamics Jacobians A_k, B_k.
//
// One iteration = two launches:
//   k_geval<FAM>  lanes (problem, node, tangent direction): the node record (gfam.hpp) --
//                 forward-over-reverse sweeps per arm and direction, assembled in LDS, written as
//                 one contiguous record per node
//   k_giter<FAM>  one wavefront per horizon: optimality error, barrier update, inertia-corrected
//                 Riccati factorisation (stage blocks [[Quu, Du^T], [Du, -dc]] by Bunch-Kaufman in
//                 LDS), solve, fraction to the boundary, line search (trial values: one lane per
//                 node) with second-order corrections, update
// Layout: every per-problem array is [problem][node][field]; a node's record is contiguous.
// the phase kernels read their model images in LDS through generic pointers (dyn.hpp joint_at)
#define MF_GENERIC_MODEL_PTR 1
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <type_traits>
#include <vector>

#include "bk_wave.hpp"
#include "capi_internal.hpp"
#include "gfam.hpp"
#include "gcore.hpp"
#include "gchain.hpp"

namespace mf {

__device__ double mf_gdbg_pre[GDBG_ROWS * GDBG_W], mf_gdbg_ls[GDBG_ROWS * GDBG_W];

// Diagnostic build only (-DMF_GSTAMPS, libmpcfatigue_gstamps.so): per-phase cycle counts of k_giter
// accumulated in registers by every lane and added to a debug buffer by lane 0 once per launch
#ifdef MF_GSTAMPS
__device__ unsigned long long mf_gstamp_buf[32 * 1024];
#define GSTAMP(slot)                                                                  \
    do {                                                                              \
        unsigned long long t_ = __builtin_amdgcn_s_memtime();                         \
        gst_acc_[slot] += t_ - gst_prev_;                                             \
        gst_prev_ = t_;                                                               \
    } while (0)
#define GSTAMP_INIT                                                                   \
    unsigned long long gst_acc_[32] = {0};                                            \
    unsigned long long gst_prev_ = __builtin_amdgcn_s_memtime()
#define GSTAMP_COUNT(slot, v) do { gst_acc_[slot] += (v); } while (0)
#define GSTAMP_FLUSH                                                                  \
    do {                                                                              \
        if (lane == 0 && b < 1024)                                                    \
            for (int s_ = 0; s_ < 32; s_++) mf_gstamp_buf[b * 32 + s_] += gst_acc_[s_]; \
    } while (0)
#else
#define GSTAMP(slot) do {} while (0)
#define GSTAMP_INIT do {} while (0)
#define GSTAMP_COUNT(slot, v) do {} while (0)
#define GSTAMP_FLUSH do {} while (0)
#endif

// Diagnostic build only (-DMF_GCHK, libmpcfatigue_gchk.so): progress checkpoints of the phase kernels and index
// checks of the stored stage factorisations (0 <= perm < NK, piv in {0, 1, 2}), written by plain vector stores to
// mapped host memory (mf_gdebug_chk_attach); if the runtime aborts the process on a GPU fault, a SIGABRT handler
// writes that memory to a file.  Per problem b < GCHK_B four words: [0] (iter << 12) | (phase << 8) | checkpoint,
// [1] violation flags (1 perm, 2 piv, 4 perm at the factorisation, 8 piv at the factorisation), [2] auxiliary
// value (stage, trial), [3] the offending value.  Out-of-range indices are clamped in this build.
#define GCHK_B 4096
#define GCHK_W 68  // words per problem: the four above, then one per lane (GCHK_LANE)
#ifdef MF_GCHK
__device__ unsigned *mf_gchk_dev;
__device__ __forceinline__ void gchk_store(unsigned *p, unsigned v) {
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
#define GCHK(id, aux)                                                                                           \
    do {                                                                                                        \
        unsigned *g_ = mf_gchk_dev;                                                                             \
        if (lane == 0 && g_ && b < GCHK_B) {                                                                    \
            gchk_store(g_ + GCHK_W * b, ((unsigned)st.iter << 12) | ((unsigned)PH << 8) | (unsigned)(id));            \
            gchk_store(g_ + GCHK_W * b + 2, (unsigned)(aux));                                                         \
            __threadfence_system();                                                                             \
        }                                                                                                       \
    } while (0)
#define GCHK_BAD(code, val)                                                                                     \
    do {                                                                                                        \
        unsigned *g_ = mf_gchk_dev;                                                                             \
        if (g_ && b < GCHK_B) {                                                                                 \
            gchk_store(g_ + GCHK_W * b + 1, (unsigned)(code));                                                        \
            gchk_store(g_ + GCHK_W * b + 3, (unsigned)(val));                                                         \
            __threadfence_system();                                                                             \
        }                                                                                                       \
    } while (0)
#define GCHK_LANE(v)                                                                                            \
    do {                                                                                                        \
        unsigned *g_ = mf_gchk_dev;                                                                             \
        if (g_ && b < GCHK_B) {                                                                                 \
            gchk_store(g_ + GCHK_W * b + 4 + lane, (unsigned)(v));                                               \
            __threadfence_system();                                                                             \
        }                                                                                                       \
    } while (0)
#else
#define GCHK(id, aux) do {} while (0)
#define GCHK_BAD(code, val) do {} while (0)
#define GCHK_LANE(v) do {} while (0)
#endif


template <class FAM>
__global__ __launch_bounds__(256) void k_geval(const DevModel *M0, const DevModel *M1, const DevFrame *F0,
                                               const DevFrame *F1, GParams P, GArrays A, int batch) {
    using D = typename FAM::D;
    constexpr int L = FAM::LANES, NPB = 256 / L, SW = scr_words<FAM>();
#ifdef MF_GSTAMPS
    const unsigned long long gs0_ = __builtin_amdgcn_s_memtime();
#endif
    GMODELS(FAM);
    __shared__ typename FAM::Scratch S[NPB];
    const int tid = threadIdx.x, g = tid / L, t = tid % L;
    const int N = P.N;
    const long node0 = (long)blockIdx.x * NPB, node = node0 + g;
    bool run = g < NPB && node < (long)batch * N;
    int b = 0, k = 0;
    if (run) {
        b = (int)(node / N);
        k = (int)(node % N);
        run = A.st[b].status == GS_RUNNING;
    }
    const double ow = (run && A.st[b].mode == 1) ? 0.0 : 1.0;  // the restoration problem has no objective
    const GSz<D> Z(N);
    const double *x = A.x + b * Z.x() + (size_t)k * D::NX, *u = A.u + b * Z.u() + (size_t)k * D::NU;
    const double *yi = A.yi + b * Z.i() + (size_t)k * D::NIA, *ye = A.ye + b * Z.e() + (size_t)k * D::NET;
    const double *lam = A.lam + b * Z.l() + (size_t)k * D::NX;
    const bool eqon = D::NE > 0 && k >= P.eq_from && k < N;
    if (run && t < FAM::PRE) FAM::prepass(M, F, P, x, u, t, S[g]);
    __syncthreads();
    if (run && t == 0) FAM::seeds(P, u, yi, ye, lam, eqon, ow, S[g]);
    __syncthreads();
    if (run) FAM::lane(M, F, x, u, yi, t, S[g]);
    {
        const int nrun = __syncthreads_count(run && t == 0);  // (also the barrier before the scratch store)
        if (A.neval && tid == 0 && nrun > 0) atomicAdd(A.neval, (unsigned long long)nrun);
    }
#ifdef MF_GSTAMPS
    const unsigned long long gs1_ = __builtin_amdgcn_s_memtime();
#endif
    // the block's NPB scratch images are contiguous in LDS and (node-major) in A.scr
    const long nn = (long)batch * N - node0;
    const int nw = (int)((nn < NPB ? nn : NPB) * SW);
    const double *src = reinterpret_cast<const double *>(S);
    double *dst = A.scr + node0 * SW;
    for (int e = tid; e < nw; e += 256) dst[e] = src[e];
#ifdef MF_GSTAMPS  // slots 30 / 31: models + sweeps, scratch store (per block, charged to its first problem)
    __syncthreads();
    if (tid == 0 && b < 1024) {
        atomicAdd(&mf_gstamp_buf[b * 32 + 30], gs1_ - gs0_);
        atomicAdd(&mf_gstamp_buf[b * 32 + 31], __builtin_amdgcn_s_memtime() - gs1_);
    }
#endif
}

template <class FAM>
__global__ __launch_bounds__(256) void k_gasm(GParams P, GArrays A, int batch) {
    using D = typename FAM::D;
    constexpr int SW = scr_words<FAM>();
    constexpr int NX = D::NX, NU = D::NU, NIA = D::NIA, NET = D::NET;
    constexpr int VX = 0, VU = NX, VI = NX + NU, VE = VI + NIA, VL = VE + NET, NVEC = VL + NX;
    // the scratch and the node's primal / dual values in LDS: FAM::rec reads them per entry, and from global
    // memory every entry would wait on a load the record stores keep the compiler from hoisting
    __shared__ typename FAM::Scratch S[4];
    __shared__ double Vv[4][NVEC];
    const int w = threadIdx.x / 64, lane = threadIdx.x % 64;
    const int N = P.N;
    const long node = (long)blockIdx.x * 4 + w;
    bool run = node < (long)batch * N;
    int b = 0, k = 0;
    if (run) {
        b = (int)(node / N);
        k = (int)(node % N);
        run = A.st[b].status == GS_RUNNING;
    }
    const GSz<D> Z(N);
    double *V = Vv[w];
    if (run) {
        glds_copy(reinterpret_cast<double *>(&S[w]), A.scr + node * SW, SW, lane);
        glds_copy(V + VX, A.x + b * Z.x() + (size_t)k * NX, NX, lane);
        glds_copy(V + VU, A.u + b * Z.u() + (size_t)k * NU, NU, lane);
        glds_copy(V + VI, A.yi + b * Z.i() + (size_t)k * NIA, NIA, lane);
        if constexpr (NET > 0) glds_copy(V + VE, A.ye + b * Z.e() + (size_t)k * NET, NET, lane);
        glds_copy(V + VL, A.lam + b * Z.l() + (size_t)k * NX, NX, lane);
    }
    gsync();
#ifdef MF_GSTAMPS
    const unsigned long long gs0_ = __builtin_amdgcn_s_memtime();
#endif
    if (run) {
        const double *lref = A.lref + FAM::LREF * b;
        const bool eqon = D::NE > 0 && k >= P.eq_from && k < N;
        double *rec = A.rec + b * Z.rec() + (size_t)k * D::REC;
        for (int e = lane; e < D::REC; e += 64)
            rec[e] = FAM::rec(P, V + VX, V + VU, V + VI, V + VE, V + VL, eqon, S[w], e, lref);
    }
#ifdef MF_GSTAMPS  // slot 31 += record assembly (per wave, charged to its problem)
    if (run && lane == 0 && b < 1024) atomicAdd(&mf_gstamp_buf[b * 32 + 31], __builtin_amdgcn_s_memtime() - gs0_);
#endif
}

// ============================================================== initial point
template <class FAM>
__global__ __launch_bounds__(64) void k_ginit(const DevModel *M0, const DevModel *M1, const DevFrame *F0,
                                              const DevFrame *F1, GParams P, GArrays A, int batch) {
    using D = typename FAM::D;
    constexpr int NX = D::NX, NU = D::NU, NI = D::NI, NIA = D::NIA, NET = D::NET;
    if (blockIdx.x >= (unsigned)batch) return;
    if (A.init && !A.init[blockIdx.x]) return;  // continuous batching: only the slots handed a new problem
    GMODELS(FAM);
    const int b = blockIdx.x, lane = threadIdx.x;
    const int pb = A.pidx ? A.pidx[b] : b;  // the problem in this slot (its u_0 / warm-start rows)
    const int N = P.N;
    const GSz<D> Z(N);
    double *x = A.x + b * Z.x(), *u = A.u + b * Z.u(), *s = A.s + b * Z.i();
    const double *x0 = A.x0 + (size_t)b * NX;
    if (FAM::LREF > 2) {  // per-problem data of the family computed from x_0 (Centauro pose targets)
        if (lane == 0) FAM::targets(M, F, P, x0, A.lref + FAM::LREF * b);
        gsync();
    }
    const int wst = NU + NX, wsz = NX + N * wst;
    const double *w0 = A.w0 ? A.w0 + (size_t)pb * wsz : nullptr;
    // IPOPT initial point: bound_push = bound_frac = 1e-2 and bound multipliers 1 (bound_mult_init_val);
    // warm_start_init_point: 1e-3 and warm_start_mult_bound_push = 1e-3 (oracle/mf_ocp.c, same rule)
    const bool warm = P.warm_start && w0;
    const double kp = warm ? 1e-3 : 1e-2, z0 = warm ? 1e-3 : 1.0;
    for (int e = lane; e < (N + 1) * NX; e += 64) {
        const int k = e / NX, j = e % NX;
        double v = x0[j];
        if (k > 0)
            v = gpush(w0 ? w0[NX + (k - 1) * wst + NU + j] : (P.init_zero ? 0.0 : x0[j]), P.x_lo[j], P.x_hi[j], kp);
        x[e] = v;
        A.zxL[b * Z.x() + e] = (k > 0 && gb(P.x_lo[j])) ? z0 : 0.0;
        A.zxU[b * Z.x() + e] = (k > 0 && gb(P.x_hi[j])) ? z0 : 0.0;
    }
    for (int e = lane; e < N * NU; e += 64) {
        const int k = e / NU, j = e % NU;
        const double lo = A.u_lo[e], hi = A.u_hi[e];
        const bool fixed = gb(lo) && lo == hi;
        double v;
        if (fixed) {
            v = (k == 0 && A.u0) ? A.u0[(size_t)pb * NU + j] : lo;
        } else {
            double v0 = P.has_u_init ? P.u_init[j] : (j >= P.force_from ? P.F_init : 0.0);
            if (w0) v0 = w0[NX + k * wst + j];
            v = gpush(v0, lo, hi, kp);
        }
        u[e] = v;
        A.zuL[b * Z.u() + e] = (!fixed && gb(lo)) ? z0 : 0.0;
        A.zuU[b * Z.u() + e] = (!fixed && gb(hi)) ? z0 : 0.0;
    }
    for (int e = lane; e < N * NX; e += 64) A.lam[b * Z.l() + e] = 0.0;
    for (int e = lane; e < N * NET; e += 64) A.ye[b * Z.e() + e] = 0.0;
    for (int e = lane; e < N * NIA; e += 64) A.yi[b * Z.i() + e] = 0.0;
    gsync();
    for (int k = lane; k < N; k += 64) {
        double l, ci[NIA], ce[NET], f[NX];
        FAM::values(M, F, P, x + (size_t)k * NX, u + (size_t)k * NU, A.lref + FAM::LREF * b, l, ci, ce, f);
        for (int r = 0; r < NI; r++) {
            const int i = k * NIA + r;
            const double lo = A.c_lo[k * NI + r], hi = A.c_hi[k * NI + r];
            s[i] = gpush(ci[r], lo, hi, kp);
            A.vL[b * Z.i() + i] = gb(lo) ? z0 : 0.0;
            A.vU[b * Z.i() + i] = gb(hi) ? z0 : 0.0;
        }
    }
    if (lane == 0) {
        GState st;
        st.mu = P.mu_init; st.nu = 0.0; st.reg_last = 0.0; st.E0 = INFINITY; st.cviol = INFINITY; st.obj = 0.0;
        st.reg_tier = 0; st.status = GS_RUNNING; st.iter = 0; st.n_ls_fail = 0; st.n_ic = 0; st.consec_fail = 0;
        st.n_soc = 0; st.frow = -1; st.dw_c = 0.0; st.dc_c = 0.0;
        st.ic_last = st.ic_last_main = 0.0;
        st.thm[0][0] = st.thm[0][1] = st.thm[1][0] = st.thm[1][1] = -1.0;
        st.rs_ph = st.rs_th = st.mu_orig = st.zeta = 0.0;
        st.wd_ph = st.wd_th = st.wd_gd = st.wd_atest = st.pd_cur = 0.0;
        st.mode = 0; st.pend = GP_NONE; st.nf[0] = st.nf[1] = 0;
        st.in_wd = st.wd_short = st.wd_trial = st.in_soft = st.soft_cnt = st.n_resto = st.n_wd = st.n_soft = 0;
        st.n_wdfail = st.n_rit = 0;
        A.st[b] = st;
        if (A.init) A.init[b] = 0;
    }
}

// ============================================================== one interior-point iteration
// Three launches per iteration, one wavefront per horizon each (giter_phase<FAM, PH>):
//   PH 0 k_gpre  optimality error, convergence test, barrier update, Sigma / barrier gradients, residuals
//   PH 1 k_gkkt  inertia-corrected Riccati factorisation and the Newton direction
//   PH 2 k_gls   fraction to the boundary, l1-merit line search with second-order corrections, update
// The phases share this one body (same arithmetic as a single kernel); each launch keeps only its own
// phase's code and LDS, so register allocation and occupancy are per phase.
template <class FAM, int PH, bool FLT>
__device__ __forceinline__ void giter_phase(const DevModel *M0, const DevModel *M1, const DevFrame *F0,
                                            const DevFrame *F1, const GParams &P, const GArrays &A, int batch) {
    using D = typename FAM::D;
    constexpr int NX = D::NX, NU = D::NU, NV = D::NV, NI = D::NI, NE = D::NE, NIA = D::NIA, NEA = D::NEA;
    constexpr int NM = D::NM, NET = D::NET;  // mixed rows c_m(x_k, u_k): multipliers at ye[k NET + NEA + m]
    constexpr int NK = NU + NET, LDK = NK + 1;
    // (not const: the serial stage loops redefine it opaquely per stage, so the per-lane addresses are recomputed
    // inside them instead of being hoisted out and held in registers across the sweep)
    int lane = threadIdx.x;
    // PH 3 (k_gspec): block s GNSPEC + t is try t of the s-th running horizon, with factor storage row blockIdx.x
    const int b = PH == 3 ? (blockIdx.x < GNSPEC * A.spec_max ? A.slist[blockIdx.x / GNSPEC] : -1) : (int)blockIdx.x;
    if (b < 0 || b >= batch) return;
    // the horizon's state in LDS: a register copy of GState (~70 dwords) stays live across the whole phase body; every
    // lane reads the same values and the uniform updates below are the same store from every lane
    __shared__ GState st_lds;
    if (lane == 0) st_lds = A.st[b];
    wave_lds_sync();
    GState &st = st_lds;
    if (st.status != GS_RUNNING) {
        if (PH == 3 && lane == 0) A.sres[blockIdx.x] = -1;
        return;
    }
    GCHK(1, 0);
    __shared__ GModels<FAM> Gm;
    if constexpr (PH == 2) {
        Gm.load(M0, M1, F0, F1);
        __syncthreads();
        GCHK(2, 0);
    }
    // the LDS images' generic addresses made opaque: with many inlined users the optimiser otherwise folds the
    // {&Gm.m[0], &Gm.m[1]} aggregate into a constant global initialiser, which cannot hold LDS addresses
    const DevModel *gm0_ = nullptr, *gm1_ = nullptr;
    const DevFrame *gf0_ = nullptr, *gf1_ = nullptr;
    if constexpr (PH == 2) {  // (the other phases evaluate no node function: no model images in their LDS)
        gm0_ = &Gm.m[0].get(); gm1_ = &Gm.m[FAM::NM - 1].get();
        gf0_ = &Gm.f[0]; gf1_ = &Gm.f[FAM::NM - 1];
        __asm__ volatile("" : "+s"(gm0_), "+s"(gm1_), "+s"(gf0_), "+s"(gf1_));
    }
    const MArr M{gm0_, gm1_};
    const FArr F{gf0_, gf1_};
    GSTAMP_INIT;
    // LDS is what limits the phase kernels' occupancy, so buffers whose lives do not overlap share storage:
    // Rh (the stage's Q_ux / constraint rows) lives in T1 once Q_uu has consumed P B; the feedback Kf in rows
    // NX.. of Hs once K_k and Rh have been formed from them (Q_xx stays in place in the rows < NX of Hs);
    // the pivoted multi-column solve's scratch in A|B once the products are formed.
    constexpr int NT1 = NX * NU > NK * NX ? NX * NU : NK * NX;
    static_assert(NK * NX <= NU * NV, "Kf must fit in rows NX.. of Hs");
    static_assert(NK <= 24 || NK * NX <= NX * NX + NX * NU, "the solve's scratch must fit in A|B");
    __shared__ double Hs[NV * NV], Ps[NX * NX], T1[NT1], T2[NX * NX], AB[NX * NX + NX * NU];
    double *const Ab = AB, *const Bb = AB + NX * NX, *const Rh = T1, *const Kf = Hs + NX * NV;
    constexpr int KSTG = NK * LDK + 2 * NK;  // per stage: factored block, perm, piv
    __shared__ double Ks[NK * LDK], Ys[NK], Jn[NEA * NX], Dds[NIA];  // Ys: the one-column solve's scratch
    __shared__ int perm[NK], piv[NK];
    __shared__ double vx[NV], tv[NX], zv[NK], pvs[NX], dxs[NX], dxn[NX], duv[NK];
    // elastic dynamics rows of the restoration phase (relax_stage): D_r of the stage, J~ of node k+1, p~, the LU
    // permutation and the pivot data of G = I + S P S
    __shared__ double Drs[NX], Jts[NEA * NX], ptv[NX];
    __shared__ int pix[NX], permx[NX], pivx[NX];
    // stage k's record parts staged into LDS by coalesced lane-strided loads (stage_in): the inner
    // loops of the stage then read LDS, not global memory; fixed-control / active-row flags alike
    constexpr int NIA2 = NI > 0 ? NI : 1, NMA = NM > 0 ? NM : 1;
    __shared__ double JIs[NIA2 * NV], JMs[NMA * NV];
    __shared__ int fixs[NU], acts[NIA2];
    // the stage's bound rows (u_lo, u_hi, c_lo, c_hi) and slack-row vectors (y_i, Sigma_s, grad_s, r_i, the elastic
    // rows' correction and Sigma_p, Sigma_n) staged by LDS-DMA with the record parts, so that a stage's operands
    // arrive in one memory round trip: a plain load feeding an LDS store makes the wave wait (vmcnt, in order) for
    // everything issued before it, one more round trip per such loop.  The flags and weights are formed after it.
    constexpr int SL_YI = 0, SL_SS = NIA2, SL_GS = 2 * NIA2, SL_RI = 3 * NIA2, SL_RR = 4 * NIA2, SL_SP = 5 * NIA2,
                  SL_SN = 6 * NIA2, SL_END = 7 * NIA2;
    __shared__ double Bnd[2 * NU + 2 * NIA2], Sl[SL_END], PPd[2 * (NU + NET)];
    // stage vectors (stage_vec): barrier Sigma of the stage's x / u / slack rows (factor), and for the
    // direction's backward pass grad L_k, the barrier gradients, lambda_k, lambda_{k-1}, y_e,k, the slack
    // weights w_q, rd_k, re_k, re_{k+1} and J_E of node k
    constexpr int V_SX = 0, V_SU = V_SX + NX, V_SS = V_SU + NU, V_GL = V_SS + NIA2, V_GX = V_GL + NV,
                  V_LK = V_GX + NX, V_LP = V_LK + NX, V_YE = V_LP + NX, V_GU = V_YE + NET, V_W = V_GU + NU,
                  V_RD = V_W + NIA2, V_RE = V_RD + NX, V_RN = V_RE + NET, V_JE = V_RN + NEA, V_END = V_JE + NEA * NX;
    __shared__ double Vs[V_END];

    const int N = P.N;
    const GSz<D> Z(N);
    double *x = A.x + b * Z.x(), *u = A.u + b * Z.u(), *s = A.s + b * Z.i(), *lam = A.lam + b * Z.l();
    double *ye = A.ye + b * Z.e(), *yi = A.yi + b * Z.i();
    double *zxL = A.zxL + b * Z.x(), *zxU = A.zxU + b * Z.x(), *zuL = A.zuL + b * Z.u(), *zuU = A.zuU + b * Z.u();
    double *vL = A.vL + b * Z.i(), *vU = A.vU + b * Z.i();
    double *dx = A.dx + b * Z.x(), *du = A.du + b * Z.u(), *ds = A.ds + b * Z.i(), *dlam = A.dlam + b * Z.l();
    double *dye = A.dye + b * Z.e(), *dyi = A.dyi + b * Z.i();
    double *dzxL = A.dzxL + b * Z.x(), *dzxU = A.dzxU + b * Z.x(), *dzuL = A.dzuL + b * Z.u(), *dzuU = A.dzuU + b * Z.u();
    double *dvL = A.dvL + b * Z.i(), *dvU = A.dvU + b * Z.i();
    double *bkp = A.bk + b * Z.bk();
    const double *rec = A.rec + b * Z.rec();
    double *Sx = A.Sx + b * Z.x(), *gx = A.gx + b * Z.x(), *Su = A.Su + b * Z.u(), *gu = A.gu + b * Z.u();
    double *Ss = A.Ss + b * Z.i(), *gs = A.gs + b * Z.i();
    double *rdyn = A.rdyn + b * Z.l(), *rin = A.rin + b * Z.i(), *req = A.req + b * Z.e();
    double *trdyn = A.trdyn + b * Z.l(), *trin = A.trin + b * Z.i(), *treq = A.treq + b * Z.e();
    double *sdyn = A.sdyn + b * Z.l(), *sin_ = A.sin_ + b * Z.i(), *seq = A.seq + b * Z.e();
    double *tx = A.tx + b * Z.x(), *tu = A.tu + b * Z.u(), *ts = A.ts + b * Z.i();
    double *Pg = A.P + b * Z.P(), *Kg = A.Kinv + b * Z.Kinv(), *Fg = A.Kfb + b * Z.Kfb(), *pvg = A.pv + b * Z.l();
    double *LUb = A.LUg + b * Z.lu(), *Jtb = A.Jtg + b * Z.jt();  // elastic-dynamics factors (restoration)
    // a speculative try factors into its own storage row (PH 3); the line search's second-order corrections solve
    // with the factors k_gkkt took from such a row (PH 2, st.frow)
    auto use_row = [&](size_t r) __attribute__((always_inline)) {
        Pg = A.Psp + r * Z.P(); Kg = A.Ksp + r * Z.Kinv(); Fg = A.Fsp + r * Z.Kfb();
        LUb = A.LUsp + r * Z.lu(); Jtb = A.Jtsp + r * Z.jt();
    };
    if constexpr (PH == 3) use_row(blockIdx.x);
    if constexpr (PH == 2) {
        if (P.filter && st.frow >= 0) use_row((size_t)st.frow);
    }
    double *kvg = A.kv + b * Z.kv();
    const double *ulo = A.u_lo, *uhi = A.u_hi, *clo = A.c_lo, *chi = A.c_hi;
    const double *lref = A.lref + FAM::LREF * b;
    auto R = [&](int k) __attribute__((always_inline)) { return rec + (size_t)k * D::REC; };
    auto ufix = [&](int i) __attribute__((always_inline)) { return gb(ulo[i]) && ulo[i] == uhi[i]; };
    auto cact = [&](int k, int q) __attribute__((always_inline)) { return gb(clo[k * NI + q]) || gb(chi[k * NI + q]); };
    auto eqon = [&](int k) __attribute__((always_inline)) { return NE > 0 && k >= P.eq_from && k < N; };
    const double kappa_eps = 10.0, kappa_mu = 0.2, theta_mu = 1.5, tau_min = 0.99, s_max = 100.0;
    const double kappa_sigma = 1e10, eta = 1e-4, rho = 0.1;
    double mu = st.mu, nu = st.nu;

    auto finish = [&](int status) __attribute__((always_inline)) {
        GSTAMP_FLUSH;
        double f = 0.0;
        for (int k = lane; k < N; k += 64) f += R(k)[D::O_L];
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

    // ---------------- IPOPT mode (P.filter): restoration-phase arrays and row helpers
    // k_gpre / k_gkkt test the option at run time; k_gls is instantiated twice (merit / filter) so that each
    // line search has its own register allocation
    const bool flt = PH == 2 ? FLT : P.filter != 0;
    const bool rsm = flt && st.mode == 1;  // the restoration problem is being solved
    constexpr double RHO_R = 1000.0, KAPPA_D = 1e-5;
    const size_t NRo = (size_t)N * NIA;   // elastic rows: slack rows [k NIA + q], then equality rows [NRo + k NET + e],
    const size_t NRD = Z.nrd();            // then dynamics rows [NRD + k NX + j] (IPOPT's restoration; not resto_hard_dyn)
    const bool rlx = rsm && !P.resto_hard_dyn;  // the dynamics rows carry elastic variables now
    double *prr = A.pr + b * Z.nr(), *nrr = A.nr + b * Z.nr(), *zpr = A.zp + b * Z.nr(), *znr = A.zn + b * Z.nr();
    double *dpr = A.dpr + b * Z.nr(), *dnr = A.dnr + b * Z.nr(), *dzp = A.dzp + b * Z.nr(), *dzn = A.dzn + b * Z.nr();
    double *tpr = A.tpr + b * Z.nr(), *tnr = A.tnr + b * Z.nr(), *Spr = A.Sp + b * Z.nr(), *Snr = A.Sn + b * Z.nr();
    double *gpr = A.gp + b * Z.nr(), *gnr = A.gn + b * Z.nr(), *rowr = A.rowr + b * Z.nr();
    double *wR = A.wR + b * Z.wv(), *dR = A.dR + b * Z.wv();
    auto el_on = [&](int r) __attribute__((always_inline)) -> bool {  // elastic row r active
        if ((size_t)r < NRo) return (r % NIA) < NI && cact(r / NIA, r % NIA);
        if ((size_t)r >= NRD) return !P.resto_hard_dyn;
        const int e = r - (int)NRo, k = e / NET, ee = e % NET;
        return ee < NEA ? (ee < NE && eqon(k)) : true;
    };
    auto el_y = [&](int r) __attribute__((always_inline)) -> double {
        return (size_t)r < NRo ? yi[r] : ((size_t)r < NRD ? ye[r - NRo] : lam[r - NRD]);
    };
    // the constraint value of elastic row r at the current point (records current)
    auto el_c = [&](int r) __attribute__((always_inline)) -> double {
        if ((size_t)r < NRo) return R(r / NIA)[D::O_CI + r % NIA] - s[r];
        if ((size_t)r >= NRD) {
            const int e = r - (int)NRD, k = e / NX, j = e % NX;
            return R(k)[D::O_F + j] - x[(k + 1) * NX + j];
        }
        const int e = r - (int)NRo, k = e / NET, ee = e % NET;
        return ee < NEA ? R(k)[D::O_CE + ee] : R(k)[D::O_CM + ee - NEA];
    };
    const int NRI = (int)Z.nr();

    // ---------------- optimality measures at the current point (records current): IPOPT's E_0 pieces and, for
    // the soft restoration phase, the primal-dual system error (sum of 1-norms / number of terms); the
    // restoration problem's when rsm
    struct GErr { double dinf, pinf, cinf0, cinfm, sd, sc, s1, n1; };
    auto opt_err = [&](double mu_) __attribute__((always_inline)) -> GErr {
        double dinf = 0, pinf = 0, cinf0 = 0, cinfm = 0, sm = 0, sbm = 0, s1 = 0;
        int nm = 0, nbm = 0, n1 = 0;
        auto comp = [&](double z, double gap) __attribute__((always_inline)) {
            const double c = z * gap;
            cinf0 = fmax(cinf0, fabs(c));
            cinfm = fmax(cinfm, fabs(c - mu_));
            sbm += z;
            nbm++;
            s1 += fabs(c - mu_);
            n1++;
        };
        for (int e = lane; e < N * NX; e += 64) {  // x rows, k = 1..N
            const int k = e / NX + 1, j = e % NX, i = k * NX + j;
            double r = -lam[(k - 1) * NX + j];
            if (k < N) {
                const double *rk = R(k);
                r += rk[D::O_GL + j];
                for (int jj = 0; jj < NX; jj++) r += rk[D::O_A + jj * NX + j] * lam[k * NX + jj];
                for (int q = 0; q < NI; q++) r += rk[D::O_JI + q * NV + j] * yi[k * NIA + q];
                if (eqon(k))
                    for (int ee = 0; ee < NE; ee++) r += rk[D::O_JE + ee * NX + j] * ye[k * NET + ee];
                for (int m = 0; m < NM; m++) r += rk[D::O_JM + m * NV + j] * ye[k * NET + NEA + m];
            }
            if (rsm) r += st.zeta * dR[i] * (x[i] - wR[i]);
            r += -zxL[i] + zxU[i];
            dinf = fmax(dinf, fabs(r));
            s1 += fabs(r);
            n1++;
            if (gb(P.x_lo[j])) comp(zxL[i], x[i] - P.x_lo[j]);
            if (gb(P.x_hi[j])) comp(zxU[i], P.x_hi[j] - x[i]);
        }
        for (int e = lane; e < N * NU; e += 64) {  // u rows (free)
            if (ufix(e)) continue;
            const int k = e / NU, j = e % NU;
            const double *rk = R(k);
            double r = rk[D::O_GL + NX + j];
            for (int jj = 0; jj < NX; jj++) r += rk[D::O_B + jj * NU + j] * lam[k * NX + jj];
            for (int q = 0; q < NI; q++) r += rk[D::O_JI + q * NV + NX + j] * yi[k * NIA + q];
            for (int m = 0; m < NM; m++) r += rk[D::O_JM + m * NV + NX + j] * ye[k * NET + NEA + m];
            if (rsm) r += st.zeta * dR[Z.x() + e] * (u[e] - wR[Z.x() + e]);
            r += -zuL[e] + zuU[e];
            dinf = fmax(dinf, fabs(r));
            s1 += fabs(r);
            n1++;
            if (gb(ulo[e])) comp(zuL[e], u[e] - ulo[e]);
            if (gb(uhi[e])) comp(zuU[e], uhi[e] - u[e]);
        }
        for (int e = lane; e < N * NI; e += 64) {  // slack rows
            const int k = e / NI, q = e % NI, i = k * NIA + q;
            if (!cact(k, q)) continue;
            const double rd = -yi[i] - vL[i] + vU[i];
            dinf = fmax(dinf, fabs(rd));
            s1 += fabs(rd);
            n1++;
            if (gb(clo[e])) comp(vL[i], s[i] - clo[e]);
            if (gb(chi[e])) comp(vU[i], chi[e] - s[i]);
            const double rp = R(k)[D::O_CI + q] - s[i] + (rsm ? nrr[i] - prr[i] : 0.0);
            pinf = fmax(pinf, fabs(rp));
            s1 += fabs(rp);
            n1++;
            sm += fabs(yi[i]);
            nm++;
        }
        for (int e = lane; e < N * NX; e += 64) {  // dynamics
            const int k = e / NX, j = e % NX;
            const double rp = R(k)[D::O_F + j] - x[(k + 1) * NX + j] + (rlx ? nrr[NRD + e] - prr[NRD + e] : 0.0);
            pinf = fmax(pinf, fabs(rp));
            s1 += fabs(rp);
            n1++;
            sm += fabs(lam[e]);
            nm++;
        }
        if (NE > 0)
            for (int e = lane; e < N * NE; e += 64) {
                const int k = e / NE, ee = e % NE;
                if (!eqon(k)) continue;
                const size_t r = NRo + (size_t)k * NET + ee;
                const double rp = R(k)[D::O_CE + ee] + (rsm ? nrr[r] - prr[r] : 0.0);
                pinf = fmax(pinf, fabs(rp));
                s1 += fabs(rp);
                n1++;
                sm += fabs(ye[k * NET + ee]);
                nm++;
            }
        if (NM > 0)
            for (int e = lane; e < N * NM; e += 64) {
                const int k = e / NM, m = e % NM;
                const size_t r = NRo + (size_t)k * NET + NEA + m;
                const double rp = R(k)[D::O_CM + m] + (rsm ? nrr[r] - prr[r] : 0.0);
                pinf = fmax(pinf, fabs(rp));
                s1 += fabs(rp);
                n1++;
                sm += fabs(ye[k * NET + NEA + m]);
                nm++;
            }
        if (rsm)  // elastic variables: rho - y - z_p, rho + y - z_n, complementarity
            for (int r = lane; r < NRI; r += 64) {
                if (!el_on(r)) continue;
                const double y = el_y(r), a1 = RHO_R - y - zpr[r], a2 = RHO_R + y - znr[r];
                dinf = fmax(dinf, fmax(fabs(a1), fabs(a2)));
                s1 += fabs(a1) + fabs(a2);
                n1 += 2;
                comp(zpr[r], prr[r]);
                comp(znr[r], nrr[r]);
            }
        dinf = wave_max(dinf); pinf = wave_max(pinf); cinf0 = wave_max(cinf0); cinfm = wave_max(cinfm);
        sm = wave_sum(sm); sbm = wave_sum(sbm); nm = wave_sum_i(nm); nbm = wave_sum_i(nbm);
        s1 = wave_sum(s1); n1 = wave_sum_i(n1);
        GErr E;
        E.dinf = dinf; E.pinf = pinf; E.cinf0 = cinf0; E.cinfm = cinfm;
        E.sd = fmax(s_max, (sm + sbm) / fmax(1.0, (double)(nm + nbm))) / s_max;
        E.sc = fmax(s_max, sbm / fmax(1.0, (double)nbm)) / s_max;
        E.s1 = s1; E.n1 = (double)n1;
        return E;
    };

    // the filter of problem m (0 main, 1 restoration): acceptability and IPOPT's AddEntry
    double *filb = A.fil + (size_t)b * 4 * GFCAP;
    auto fil_ok = [&](int m, double ph, double th) __attribute__((always_inline)) -> bool {
        const double *f = filb + 2 * m * GFCAP;
        int bad = 0;
        for (int j = lane; j < st.nf[m]; j += 64)
            if (!(ph <= f[2 * j] || th <= f[2 * j + 1])) bad = 1;
        return wave_sum_i(bad) == 0;
    };
    auto fil_add = [&](int m, double ph, double th) __attribute__((always_inline)) {
        double *f = filb + 2 * m * GFCAP;
        int n = 0;
        if (lane == 0) {
            for (int j = 0; j < st.nf[m]; j++)
                if (!(ph <= f[2 * j] && th <= f[2 * j + 1])) { f[2 * n] = f[2 * j]; f[2 * n + 1] = f[2 * j + 1]; n++; }
            if (n == GFCAP) {  // full: the oldest entry goes (not reached on the reference problems)
                for (int j = 1; j < n; j++) { f[2 * j - 2] = f[2 * j]; f[2 * j - 1] = f[2 * j + 1]; }
                n--;
            }
            f[2 * n] = ph;
            f[2 * n + 1] = th;
            n++;
        }
        st.nf[m] = __shfl(n, 0, 64);
        gsync();
    };
    // barrier objective and l1 violation of the main problem at the current point (records), with mu_o
    auto orig_merit_cur = [&](double mu_o, double &phi, double &th, bool &okp) __attribute__((always_inline)) {
        double fs = 0.0, t = 0.0, bar = 0.0, lin = 0.0;
        int bad = 0;
        for (int k = lane; k < N; k += 64) {
            const double *rk = R(k);
            fs += rk[D::O_L];
            for (int j = 0; j < NX; j++) t += fabs(rk[D::O_F + j] - x[(k + 1) * NX + j]);
            for (int q = 0; q < NI; q++)
                if (cact(k, q)) t += fabs(rk[D::O_CI + q] - s[k * NIA + q]);
            if (eqon(k))
                for (int ee = 0; ee < NE; ee++) t += fabs(rk[D::O_CE + ee]);
            for (int m = 0; m < NM; m++) t += fabs(rk[D::O_CM + m]);
        }
        auto blog = [&](double v, double lo, double hi) __attribute__((always_inline)) {
            if (gb(lo)) { if (v - lo <= 0) bad = 1; else bar -= log(v - lo); }
            if (gb(hi)) { if (hi - v <= 0) bad = 1; else bar -= log(hi - v); }
            if (gb(lo) && !gb(hi)) lin += v - lo;
            if (gb(hi) && !gb(lo)) lin += hi - v;
        };
        for (int e = lane + NX; e < (N + 1) * NX; e += 64) blog(x[e], P.x_lo[e % NX], P.x_hi[e % NX]);
        for (int e = lane; e < N * NU; e += 64)
            if (!ufix(e)) blog(u[e], ulo[e], uhi[e]);
        for (int e = lane; e < N * NI; e += 64) blog(s[(e / NI) * NIA + e % NI], clo[e], chi[e]);
        fs = wave_sum(fs); t = wave_sum(t); bar = wave_sum(bar); lin = wave_sum(lin); bad = wave_sum_i(bad);
        phi = fs + mu_o * bar + KAPPA_D * mu_o * lin;
        th = t;
        okp = bad == 0;
    };

    if constexpr (PH == 0) {
    if (flt && st.pend == GP_WDSOFT) return;  // records of the restored point being evaluated (k_gls continues)
    if (flt && st.pend == GP_RESTO) {
        // ---------------- MinC_1NrmRestorationPhase / RestoIterateInitializer at the current point
        double cm = 0.0;
        for (int e = lane; e < N * NX; e += 64) cm = fmax(cm, fabs(R(e / NX)[D::O_F + e % NX] - x[(e / NX + 1) * NX + e % NX]));
        for (int r = lane; r < (int)NRD; r += 64)
            if (el_on(r)) cm = fmax(cm, fabs(el_c(r)));
        cm = wave_max(cm);
        const double mu_r = fmax(mu, cm);
        for (int r = lane; r < NRI; r += 64) {
            if (!el_on(r)) { prr[r] = nrr[r] = 1.0; zpr[r] = znr[r] = 0.0; continue; }
            const double c = el_c(r);
            const double a = (mu_r - RHO_R * c) / (2.0 * RHO_R);
            nrr[r] = a + sqrt(a * a + mu_r * c / (2.0 * RHO_R));
            prr[r] = c + nrr[r];
            zpr[r] = mu_r / prr[r];
            znr[r] = mu_r / nrr[r];
        }
        for (int e = lane; e < (int)Z.x(); e += 64) { wR[e] = x[e]; dR[e] = 1.0 / fmax(1.0, x[e] * x[e]); }
        for (int e = lane; e < N * NU; e += 64) { wR[Z.x() + e] = u[e]; dR[Z.x() + e] = 1.0 / fmax(1.0, u[e] * u[e]); }
        for (int e = lane; e < (int)Z.x(); e += 64) { zxL[e] = fmin(zxL[e], RHO_R); zxU[e] = fmin(zxU[e], RHO_R); }
        for (int e = lane; e < N * NU; e += 64) { zuL[e] = fmin(zuL[e], RHO_R); zuU[e] = fmin(zuU[e], RHO_R); }
        for (int e = lane; e < N * NIA; e += 64) { vL[e] = fmin(vL[e], RHO_R); vU[e] = fmin(vU[e], RHO_R); }
        // least-square multipliers (DefaultIterateInitializer::least_square_mults): the system [[I, J^T], [J, 0]]
        // through the stage factorisation -- Sigma = 0 (x_N: I), slacks and elastic variables with unit
        // Hessian, gradients grad f_R - z (grad f_R = 0 at w_R), zero constraint residuals and multipliers
        for (int e = lane; e < (N + 1) * NX; e += 64) {
            const int k = e / NX;
            Sx[e] = (k == N) ? 1.0 : 0.0;
            gx[e] = k > 0 ? -zxL[e] + zxU[e] : 0.0;
        }
        for (int e = lane; e < N * NU; e += 64) { Su[e] = 0.0; gu[e] = ufix(e) ? 0.0 : -zuL[e] + zuU[e]; }
        for (int e = lane; e < N * NIA; e += 64) { Ss[e] = 1.0; gs[e] = -vL[e] + vU[e]; }
        for (int r = lane; r < NRI; r += 64) {
            const bool on = el_on(r);
            Spr[r] = Snr[r] = on ? 1.0 : INFINITY;
            gpr[r] = -zpr[r];
            gnr[r] = -znr[r];
            rowr[r] = on ? znr[r] - zpr[r] : 0.0;
        }
        for (int e = lane; e < N * NX; e += 64) { lam[e] = 0.0; rdyn[e] = 0.0; }
        for (int e = lane; e < N * NIA; e += 64) { yi[e] = 0.0; rin[e] = 0.0; }
        for (int e = lane; e < N * NET; e += 64) { ye[e] = 0.0; req[e] = 0.0; }
        gsync();
        if (lane == 0) {
            st.mu_orig = mu;
            st.mu = mu_r;
            st.zeta = sqrt(mu_r);
            st.mode = 1;
            st.ic_last_main = st.ic_last;
            st.ic_last = 0.0;
            st.nf[1] = 0;
            st.thm[1][0] = st.thm[1][1] = -1.0;
            st.in_wd = 0; st.wd_short = 0; st.in_soft = 0; st.soft_cnt = 0;
            st.n_resto++;
            st.pend = GP_LSM;
            A.st[b] = st;
        }
        return;
    }
    // ---------------- optimality error (IPOPT E_0, s_max scaling)
    const GErr Eq = opt_err(mu);
    const double dinf = Eq.dinf, pinf = Eq.pinf, sd = Eq.sd, sc = Eq.sc;
    double cinfm = Eq.cinfm;
    const double E0 = fmax(fmax(dinf / sd, pinf), Eq.cinf0 / sc);
    double Emu = fmax(fmax(dinf / sd, pinf), cinfm / sc);
    if (flt && st.pend == GP_SOFT) {  // TrySoftRestoStep, second half: the pending step's primal-dual error
        if (Eq.s1 / Eq.n1 <= 0.9999 * st.pd_cur) {
            st.pend = GP_NONE;
            st.n_soft++;
        } else {  // undo the step; the restoration phase starts from the point it was taken at
            const GSz<D> &Zc = Z;
            double *arr[16] = {x, u, s, lam, ye, yi, zxL, zxU, zuL, zuU, vL, vU, prr, nrr, zpr, znr};
            const size_t len[16] = {Zc.x(), Zc.u(), Zc.i(), Zc.l(), Zc.e(), Zc.i(), Zc.x(), Zc.x(), Zc.u(), Zc.u(),
                                    Zc.i(), Zc.i(), Zc.nr(), Zc.nr(), Zc.nr(), Zc.nr()};
            const double *src = A.wdit + b * Z.bk();
            size_t off = 0;
            for (int a = 0; a < 12; a++) {
                for (size_t e = lane; e < len[a]; e += 64) arr[a][e] = src[off + e];
                off += len[a];
            }
            gsync();
            if (lane == 0) {
                st.in_soft = 0;
                st.soft_cnt = 0;
                st.pend = GP_IDLE_RESTO;
                st.iter--;  // the oracle starts the restoration phase in the iteration of the undone step
                A.st[b] = st;
            }
            return;
        }
    }
    st.E0 = E0;
    st.cviol = pinf;
    if (!rsm) {
        if (E0 <= P.tol && pinf <= P.constr_viol_tol) { finish(GS_CONVERGED); return; }
    } else {
        // RestoFilterConvergenceCheck: the main problem's filter and its reference point accept the iterate and
        // theta fell to kappa_resto = 0.9 of its value where the restoration started
        double pho, tho;
        bool oko;
        orig_merit_cur(st.mu_orig, pho, tho, oko);
        const bool cur_ok = (tho - (1.0 - 1e-5) * st.rs_th <= 10.0 * 2.220446049250313e-16 * fabs(st.rs_th)) ||
                            ((pho - st.rs_ph) - (-1e-8 * st.rs_th) <= 10.0 * 2.220446049250313e-16 * fabs(st.rs_ph));
        if (oko && isfinite(pho) && tho <= 0.9 * st.rs_th && cur_ok && fil_ok(0, pho, tho)) {
            // back to the main problem: y = 0 (constr_mult_reset_threshold = 0), bound multipliers reset to 1
            // when any exceeds bound_mult_reset_threshold = 1000
            double zm = 0.0;
            for (int e = lane; e < (int)Z.x(); e += 64) zm = fmax(zm, fmax(zxL[e], zxU[e]));
            for (int e = lane; e < N * NU; e += 64) zm = fmax(zm, fmax(zuL[e], zuU[e]));
            for (int e = lane; e < N * NIA; e += 64) zm = fmax(zm, fmax(vL[e], vU[e]));
            zm = wave_max(zm);
            if (zm > 1e3) {
                for (int e = lane; e < (int)Z.x(); e += 64) { if (zxL[e] > 0.0) zxL[e] = 1.0; if (zxU[e] > 0.0) zxU[e] = 1.0; }
                for (int e = lane; e < N * NU; e += 64) { if (zuL[e] > 0.0) zuL[e] = 1.0; if (zuU[e] > 0.0) zuU[e] = 1.0; }
                for (int e = lane; e < N * NIA; e += 64) { if (vL[e] > 0.0) vL[e] = 1.0; if (vU[e] > 0.0) vU[e] = 1.0; }
            }
            for (int e = lane; e < N * NX; e += 64) lam[e] = 0.0;
            for (int e = lane; e < N * NIA; e += 64) yi[e] = 0.0;
            for (int e = lane; e < N * NET; e += 64) ye[e] = 0.0;
            gsync();
            if (lane == 0) {
                st.mode = 0;
                st.mu = st.mu_orig;
                st.ic_last = st.ic_last_main;
                st.in_wd = 0; st.wd_short = 0; st.in_soft = 0; st.soft_cnt = 0;
                st.pend = GP_IDLE;
                A.st[b] = st;
            }
            return;
        }
        if (P.dbg && b == 0 && lane == 0 && st.iter < GDBG_ROWS) {
            double *t = mf_gdbg_pre + st.iter * GDBG_W;
            t[8] = tho; t[9] = pho; t[10] = oko; t[11] = st.rs_th; t[12] = st.rs_ph; t[13] = cur_ok;
        }
        if (E0 <= P.tol) { finish(GS_LOCINF); return; }
    }
    if (P.dbg && b == 0 && lane == 0 && st.iter < GDBG_ROWS) {
        double *t = mf_gdbg_pre + st.iter * GDBG_W;
        t[0] = st.iter; t[1] = st.mode; t[2] = mu; t[3] = E0; t[4] = pinf; t[5] = dinf; t[6] = Eq.cinf0; t[7] = st.nf[0];
        t[14] = st.nf[1]; t[15] = st.n_resto;
    }
    if (st.iter >= P.max_iter) { finish(GS_MAXITER); return; }
    const double mu_min = flt ? P.tol / (kappa_eps + 1.0) : P.tol / 10.0;
    while (Emu <= kappa_eps * mu && mu > mu_min) {
        const double mnew = fmax(mu_min, fmin(kappa_mu * mu, pow(mu, theta_mu)));
        if (mnew >= mu) break;
        mu = mnew;
        if (flt) {  // MonotoneMuUpdate resets the line search's filter; the proximity weight follows mu
            st.nf[st.mode] = 0;
            if (rsm) st.zeta = sqrt(mu);
        }
        double cmx = 0.0;
        for (int e = lane; e < N * NX; e += 64) {
            const int i = e + NX, j = e % NX;
            if (gb(P.x_lo[j])) cmx = fmax(cmx, fabs(zxL[i] * (x[i] - P.x_lo[j]) - mu));
            if (gb(P.x_hi[j])) cmx = fmax(cmx, fabs(zxU[i] * (P.x_hi[j] - x[i]) - mu));
        }
        for (int e = lane; e < N * NU; e += 64) {
            if (ufix(e)) continue;
            if (gb(ulo[e])) cmx = fmax(cmx, fabs(zuL[e] * (u[e] - ulo[e]) - mu));
            if (gb(uhi[e])) cmx = fmax(cmx, fabs(zuU[e] * (uhi[e] - u[e]) - mu));
        }
        for (int e = lane; e < N * NI; e += 64) {
            const int i = (e / NI) * NIA + e % NI;
            if (gb(clo[e])) cmx = fmax(cmx, fabs(vL[i] * (s[i] - clo[e]) - mu));
            if (gb(chi[e])) cmx = fmax(cmx, fabs(vU[i] * (chi[e] - s[i]) - mu));
        }
        if (rsm)
            for (int r = lane; r < NRI; r += 64)
                if (el_on(r)) cmx = fmax(cmx, fmax(fabs(zpr[r] * prr[r] - mu), fabs(znr[r] * nrr[r] - mu)));
        cinfm = wave_max(cmx);
        Emu = fmax(fmax(dinf / sd, pinf), cinfm / sc);
    }
    GSTAMP(0);

    // ---------------- barrier Sigma / gradients, residuals of the current point
    const double kd = flt ? KAPPA_D * mu : 0.0;  // IPOPT kappa_d: linear damping of single-bounded variables
    for (int e = lane; e < (N + 1) * NX; e += 64) {
        const int k = e / NX, j = e % NX;
        double sg = 0, g = 0;
        if (k > 0) {
            if (gb(P.x_lo[j])) { sg += zxL[e] / (x[e] - P.x_lo[j]); g -= mu / (x[e] - P.x_lo[j]); }
            if (gb(P.x_hi[j])) { sg += zxU[e] / (P.x_hi[j] - x[e]); g += mu / (P.x_hi[j] - x[e]); }
            if (flt && gb(P.x_lo[j]) && !gb(P.x_hi[j])) g += kd;
            if (flt && gb(P.x_hi[j]) && !gb(P.x_lo[j])) g -= kd;
            if (rsm) { sg += st.zeta * dR[e]; g += st.zeta * dR[e] * (x[e] - wR[e]); }
        }
        Sx[e] = sg;
        gx[e] = g;
    }
    for (int e = lane; e < N * NU; e += 64) {
        double sg = 0, g = 0;
        if (!ufix(e)) {
            if (gb(ulo[e])) { sg += zuL[e] / (u[e] - ulo[e]); g -= mu / (u[e] - ulo[e]); }
            if (gb(uhi[e])) { sg += zuU[e] / (uhi[e] - u[e]); g += mu / (uhi[e] - u[e]); }
            if (flt && gb(ulo[e]) && !gb(uhi[e])) g += kd;
            if (flt && gb(uhi[e]) && !gb(ulo[e])) g -= kd;
            if (rsm) { sg += st.zeta * dR[Z.x() + e]; g += st.zeta * dR[Z.x() + e] * (u[e] - wR[Z.x() + e]); }
        }
        Su[e] = sg;
        gu[e] = g;
    }
    for (int e = lane; e < N * NI; e += 64) {
        const int k = e / NI, q = e % NI, i = k * NIA + q;
        double sg = 0, g = 0;
        if (gb(clo[e])) { sg += vL[i] / (s[i] - clo[e]); g -= mu / (s[i] - clo[e]); }
        if (gb(chi[e])) { sg += vU[i] / (chi[e] - s[i]); g += mu / (chi[e] - s[i]); }
        if (flt && gb(clo[e]) && !gb(chi[e])) g += kd;
        if (flt && gb(chi[e]) && !gb(clo[e])) g -= kd;
        Ss[i] = sg;
        gs[i] = g;
        rin[i] = cact(k, q) ? R(k)[D::O_CI + q] - s[i] + (rsm ? nrr[i] - prr[i] : 0.0) : 0.0;
    }
    for (int e = lane; e < N * NX; e += 64)
        rdyn[e] = R(e / NX)[D::O_F + e % NX] - x[(e / NX + 1) * NX + e % NX] + (rlx ? nrr[NRD + e] - prr[NRD + e] : 0.0);
    for (int e = lane; e < N * NET; e += 64) {
        const int k = e / NET, ee = e % NET;
        double v = ee < NEA ? ((ee < NE && eqon(k)) ? R(k)[D::O_CE + ee] : 0.0) : R(k)[D::O_CM + ee - NEA];
        if (rsm && el_on((int)NRo + e)) v += nrr[NRo + e] - prr[NRo + e];
        req[e] = v;
    }
    if (rsm)  // the elastic variables condensed: Sp dp = dy - r_p, Sn dn = -dy - r_n (oracle barrier_f)
        for (int r = lane; r < NRI; r += 64) {
            if (!el_on(r)) { Spr[r] = Snr[r] = INFINITY; gpr[r] = gnr[r] = rowr[r] = 0.0; continue; }
            const double y = el_y(r);
            Spr[r] = zpr[r] / prr[r];
            Snr[r] = znr[r] / nrr[r];
            gpr[r] = -mu / prr[r] + kd;
            gnr[r] = -mu / nrr[r] + kd;
            rowr[r] = (RHO_R + gpr[r] - y) / Spr[r] - (RHO_R + gnr[r] + y) / Snr[r];
        }
    gsync();
    GSTAMP(1);
    GSTAMP_FLUSH;
    if (lane == 0) {
        st.mu = mu;
        A.st[b] = st;
    }
    return;
    }  // PH 0
    const double tau_fb = fmax(tau_min, 1.0 - mu);

    // ---------------- Riccati factorisation with inertia test (stage blocks [[Quu, Du^T], [Du, -dc]])
    double dw_c = 0.0, dc_c = 0.0;
    // the least-square multiplier pass of a restoration start: the stage Hessians are identities and the
    // objective gradient is left out
    const bool lsm = flt && st.pend == GP_LSM;
    auto rdiag = [&](size_t r) __attribute__((always_inline)) -> double { return rsm ? 1.0 / Spr[r] + 1.0 / Snr[r] : 0.0; };
    // the bound rows of stage k into LDS (LDS-DMA; flags_in forms fixs / acts from them once they have arrived)
    auto bounds_in = [&](int k) __attribute__((always_inline)) {
        glds_copy(Bnd, ulo + (size_t)k * NU, NU);
        glds_copy(Bnd + NU, uhi + (size_t)k * NU, NU);
        if (NI > 0) {
            glds_copy(Bnd + 2 * NU, clo + (size_t)k * NI, NI);
            glds_copy(Bnd + 2 * NU + NIA2, chi + (size_t)k * NI, NI);
        }
    };
    auto flags_in = [&](bool with_acts) __attribute__((always_inline)) {
        for (int c = lane; c < NU; c += 64) fixs[c] = (gb(Bnd[c]) && Bnd[c] == Bnd[NU + c]) ? 1 : 0;
        if (with_acts)
            for (int q = lane; q < NI; q += 64) acts[q] = (gb(Bnd[2 * NU + q]) || gb(Bnd[2 * NU + NIA2 + q])) ? 1 : 0;
        wave_lds_sync();
    };
    // stage k's A, B, J_I, J_M (and W into Hs), J_E of node k+1, the fixed-control and active-row flags
    auto stage_in = [&](int k, bool withW) __attribute__((always_inline)) {
        const double *rk = R(k);
        const bool en = eqon(k + 1);
        glds_copy(Ab, rk + D::O_A, NX * NX);
        glds_copy(Bb, rk + D::O_B, NX * NU);
        if (NI > 0) glds_copy(JIs, rk + D::O_JI, NI * NV);
        if (NM > 0) glds_copy(JMs, rk + D::O_JM, NM * NV);
        if (withW) glds_copy(Hs, rk + D::O_W, NV * NV);
        if (en && NE > 0) glds_copy(Jn, R(k + 1) + D::O_JE, NE * NX);
        for (int e = lane; e < NEA * NX; e += 64)
            if (!(en && e < NE * NX)) Jn[e] = 0.0;
        bounds_in(k);
    };
    // IPOPT's restoration problem puts elastic p, n on the dynamics rows too (oracle/mf_ocp.c ric_relax): row k reads
    // dx_{k+1} = A dx_k + B du_k + r - D_r dlam_k, D_r = 1/Sp + 1/Sn.  With L = I + P_{k+1} D_r (LU, partial
    // pivoting) the stage continues with P~ = L^-1 P_{k+1} (into Ps), J~^T = L^-1 J_n^T (Jts, node k+1's state
    // rows) and the state-equality block -dc - J~ D_r J_n^T; G = I + S P S (S = D_r^1/2) must be positive definite
    // for the eliminated (x_{k+1}, lam_k) pair to have the right inertia.  Hs is the scratch (W arrives after).
    // Returns 1 for wrong inertia or a singular L (the inertia correction then raises delta_w).
    auto relax_stage = [&](int k, bool en) __attribute__((always_inline)) -> int {
        double *Gm = Hs, *Lm = Hs + NX * NX;
        for (int j = lane; j < NX; j += 64) Drs[j] = rdiag(NRD + (size_t)k * NX + j);
        __syncthreads();
        for (int e = lane; e < NX * NX; e += 64) {
            const int i = e / NX, j = e % NX;
            const double id = (i == j) ? 1.0 : 0.0;
            Gm[e] = id + sqrt(Drs[i]) * Ps[e] * sqrt(Drs[j]);
            Lm[e] = id + Ps[e] * Drs[j];
        }
        __syncthreads();
        // (register factorisations where they give the LDS routines' results: natural-order Bunch-Kaufman for G,
        // the row-per-lane LU for L)
        BKInertia gi;
        if (!bk_factor_regs<NX, NX>(Gm, permx, pivx, gi)) gi = bk_factor_wave<NX>(Gm, NX, permx, pivx);
        if (gi.zero || gi.neg) return 1;
        if (lu_factor_regs<NX, NX>(Lm, pix)) return 1;
        // lane c < NX: column c of P~ (into Gm, free now); lanes NX.. NX + NE - 1: the rows of J~
        double y[NX];
        if (lane < NX) {
            lu_solve_lane<NX, NX>(Lm, pix, Ps + lane, NX, y);
#pragma unroll
            for (int i = 0; i < NX; i++) Gm[i * NX + lane] = y[i];
        } else if (NE > 0 && en && lane < NX + NE) {
            lu_solve_lane<NX, NX>(Lm, pix, R(k + 1) + D::O_JE + (lane - NX) * NX, 1, y);
#pragma unroll
            for (int i = 0; i < NX; i++) Jts[(lane - NX) * NX + i] = y[i];
        }
        __syncthreads();
        for (int e = lane; e < NX * NX; e += 64) {
            const int i = e / NX, j = e % NX;
            Ps[e] = (i == j) ? Gm[e] : 0.5 * (Gm[i * NX + j] + Gm[j * NX + i]);
        }
        double *lu = LUb + (size_t)k * (NX * NX + NX);
        for (int e = lane; e < NX * NX; e += 64) lu[e] = Lm[e];
        for (int e = lane; e < NX; e += 64) lu[NX * NX + e] = (double)pix[e];
        if (en)
            for (int e = lane; e < NE * NX; e += 64) Jtb[(size_t)k * NEA * NX + e] = Jts[e];
        __syncthreads();
        return 0;
    };
    auto factor = [&](double dw, double dc, double d1) __attribute__((always_inline)) -> int {
        for (int e = lane; e < NX * NX; e += 64) Ps[e] = (e / NX == e % NX) ? Sx[N * NX + e / NX] + dw : 0.0;
        __syncthreads();
        for (int k = N - 1; k >= 0; k--) {
            lane = lane_opaque();
            GSTAMP(2);
            const bool en = eqon(k + 1);
            if (rlx && relax_stage(k, en)) return 1;
            for (int e = lane; e < NX * NX; e += 64) Pg[(size_t)k * NX * NX + e] = Ps[e];
            stage_in(k, true);
            glds_copy(Vs + V_SX, Sx + k * NX, NX);
            glds_copy(Vs + V_SU, Su + k * NU, NU);
            if (NI > 0) glds_copy(Vs + V_SS, Ss + k * NIA, NI);
            if (rsm && NI > 0) {
                glds_copy(Sl + SL_SP, Spr + (size_t)k * NIA, NI);
                glds_copy(Sl + SL_SN, Snr + (size_t)k * NIA, NI);
            }
            gsync();
            flags_in(true);
            for (int q = lane; q < NI; q += 64) {
                const double sg = Vs[V_SS + q] + dw;
                const double rdq = rsm ? 1.0 / Sl[SL_SP + q] + 1.0 / Sl[SL_SN + q] : 0.0;  // rdiag(k NIA + q)
                Dds[q] = acts[q] ? sg / (1.0 + (dc + rdq) * sg) : 0.0;
            }
            if (lsm)
                for (int e = lane; e < NV * NV; e += 64) Hs[e] = (e / NV == e % NV) ? 1.0 : 0.0;
            gsync();
            GSTAMP(8);
            // H = W + J_I^T D J_I (+ diagonal terms), in place over W (each lane its own tile).  Small stages: the
            // fixed rows / columns and the diagonal terms in the tile epilogue; large ones (box, Centauro: a 6 x 6
            // tile per lane, whose unrolled per-entry tests cost more than the products) in a pass over the NV
            // indices after it -- lane a sets row and column a of a fixed index to the identity (entries shared by
            // two fixed lanes get the same 0) or adds + dw, + Sigma, (+ d1) to a free diagonal, in that order
            if constexpr (NV < 24) {
                tile_gemm<NV, NV, (NI > 0 ? NI : 1)>(
                    lane, [&](int a, int c) { return Hs[a * NV + c]; },
                    [&](int q, int a) { return NI > 0 ? JIs[q * NV + a] * Dds[q] : 0.0; },
                    [&](int q, int c) { return NI > 0 ? JIs[q * NV + c] : 0.0; },
                    [&](int a, int c, double v) {
                        const bool fa = a < NX ? (k == 0) : fixs[a - NX];
                        const bool fc = c < NX ? (k == 0) : fixs[c - NX];
                        if (fa || fc) {
                            v = (a == c) ? 1.0 : 0.0;
                        } else if (a == c) {
                            v += dw;
                            if (a < NX) v += Vs[V_SX + a];
                            else {
                                v += Vs[V_SU + a - NX];
                                if (a - NX >= P.tier1_from && a - NX < P.tier1_to) v += d1;
                            }
                        }
                        Hs[a * NV + c] = v;
                    });
            } else {
                tile_gemm<NV, NV, (NI > 0 ? NI : 1)>(
                    lane, [&](int a, int c) { return Hs[a * NV + c]; },
                    [&](int q, int a) { return NI > 0 ? JIs[q * NV + a] * Dds[q] : 0.0; },
                    [&](int q, int c) { return NI > 0 ? JIs[q * NV + c] : 0.0; },
                    [&](int a, int c, double v) { Hs[a * NV + c] = v; });
                wave_lds_sync();
                auto hdiag = [&](int a, double v) __attribute__((always_inline)) {
                    v += dw;
                    if (a < NX) v += Vs[V_SX + a];
                    else {
                        v += Vs[V_SU + a - NX];
                        if (a - NX >= P.tier1_from && a - NX < P.tier1_to) v += d1;
                    }
                    return v;
                };
                auto hfixed = [&](int a) __attribute__((always_inline)) { return a < NX ? (k == 0) : (fixs[a - NX] != 0); };
                for (int a = lane; a < NV; a += 64) {
                    if (hfixed(a)) {
                        for (int c = 0; c < NV; c++) {
                            const double e = (a == c) ? 1.0 : 0.0;
                            Hs[a * NV + c] = e;
                            Hs[c * NV + a] = e;
                        }
                    } else {
                        Hs[a * NV + a] = hdiag(a, Hs[a * NV + a]);
                    }
                }
            }
            GSTAMP(9);
            tile_gemm<NX, NU, NX>(
                lane, [](int, int) { return 0.0; }, [&](int l, int i) { return Ps[i * NX + l]; },
                [&](int l, int c) { return Bb[l * NU + c]; }, [&](int i, int c, double v) { T1[i * NU + c] = v; });
            tile_gemm<NX, NX, NX>(
                lane, [](int, int) { return 0.0; }, [&](int l, int i) { return Ps[i * NX + l]; },
                [&](int l, int j) { return Ab[l * NX + j]; }, [&](int i, int j, double v) { T2[i * NX + j] = v; });
            __syncthreads();
            GSTAMP(10);
            tile_gemm<NU, NU, NX>(
                lane, [&](int a, int c) { return Hs[(NX + a) * NV + NX + c]; },
                [&](int l, int a) { return Bb[l * NU + a]; }, [&](int l, int c) { return T1[l * NU + c]; },
                [&](int a, int c, double v) { Ks[a * LDK + c] = (fixs[a] || fixs[c]) ? ((a == c) ? 1.0 : 0.0) : v; });
            for (int e = lane; e < NK * NK; e += 64) {
                const int a = e / NK, c = e % NK;
                double v = 0.0;
                if (a < NU && c < NU) {
                    continue;  // the control block: tile_gemm above
                } else if (a >= NU && c >= NU) {
                    const int ee = a - NU, e2 = c - NU;
                    const size_t rr = NRo + (size_t)(ee >= NEA ? k : k + 1) * NET + ee;
                    v = (a == c) ? ((ee >= NEA || (en && ee < NE)) ? -dc - rdiag(rr) : -1.0) : 0.0;
                    if (rlx && en && ee < NE && e2 < NE) {  // - J~ D_r J_n^T (elastic dynamics rows)
                        double acc = 0.0;
                        for (int l = 0; l < NX; l++) acc += Jts[ee * NX + l] * Drs[l] * Jn[e2 * NX + l];
                        v -= acc;
                    }
                } else {
                    const int ee = (a >= NU ? a : c) - NU, uu = a >= NU ? c : a;
                    const double *Jx = rlx ? Jts : Jn;
                    if (fixs[uu]) v = 0.0;
                    else if (ee >= NEA) v = JMs[(ee - NEA) * NV + NX + uu];  // mixed row of stage k
                    else if (en && ee < NE)
                        for (int l = 0; l < NX; l++) v += Jx[ee * NX + l] * Bb[l * NU + uu];
                }
                Ks[a * LDK + c] = v;
            }
            tile_gemm<NU, NX, NX>(
                lane, [&](int a, int j) { return Hs[(NX + a) * NV + j]; },
                [&](int l, int a) { return Bb[l * NU + a]; }, [&](int l, int j) { return T2[l * NX + j]; },
                [&](int a, int j, double v) { Rh[a * NX + j] = (k > 0 && !fixs[a]) ? v : 0.0; });
            for (int e = NU * NX + lane; e < NK * NX; e += 64) {
                const int a = e / NX, j = e % NX;
                double v = 0.0;
                const double *Jx = rlx ? Jts : Jn;
                if (k > 0) {
                    if (a - NU >= NEA) {
                        v = JMs[(a - NU - NEA) * NV + j];
                    } else if (en && a - NU < NE) {
                        for (int l = 0; l < NX; l++) v += Jx[(a - NU) * NX + l] * Ab[l * NX + j];
                    }
                }
                Rh[e] = v;
            }
            tile_gemm<NX, NX, NX>(
                lane, [&](int i, int j) { return Hs[i * NV + j]; }, [&](int l, int i) { return Ab[l * NX + i]; },
                [&](int l, int j) { return T2[l * NX + j]; }, [&](int i, int j, double v) { Hs[i * NV + j] = v; });
            __syncthreads();
            GSTAMP(11);
            // natural-order pivots in registers (the common case), the pivoted LDS factorisation otherwise
            BKInertia in;
            // (stage blocks with at most two constraint rows: with more, the Schur rows usually need pivoting)
            // (the stamps build runs this same path: its round-5 variant, the whole block in registers on every family,
            // was the only code difference of that build and the r05c fault came with it)
            if constexpr (NET <= 2) {
                if (!bk_factor_regs<LDK, NK>(Ks, perm, piv, in)) in = bk_factor_fixed<LDK, NK>(Ks, perm, piv);
            } else {
                // many constraint rows (Centauro): the control rows in registers (they keep the natural order),
                // the Schur rows of the constraints by the pivoted LDS routine from column NU
                BKInertia in0;
                if (bk_factor_regs<LDK, NK, NU>(Ks, perm, piv, in0)) in = bk_factor_wave<LDK>(Ks, NK, perm, piv, NU, in0);
                else in = bk_factor_wave<LDK>(Ks, NK, perm, piv);
            }
            GSTAMP(12);
            if (in.zero) return 2;
            if (in.pos != NU || in.neg != NET) return 1;
            // the stage factorisation is kept (the solves of the vector pass and of the second-order
            // corrections reuse it: a backward-stable LDL^T solve, not an explicit inverse)
            double *kst = Kg + (size_t)k * KSTG;
#ifdef MF_GCHK
            for (int e = lane; e < NK; e += 64) {
                if (perm[e] < 0 || perm[e] >= NK) GCHK_BAD(4, perm[e]);
                if (piv[e] < 0 || piv[e] > 2) GCHK_BAD(8, piv[e]);
            }
#endif
            for (int e = lane; e < NK * LDK; e += 64) kst[e] = Ks[e];
            for (int e = lane; e < NK; e += 64) { kst[NK * LDK + e] = perm[e]; kst[NK * LDK + NK + e] = piv[e]; }
            for (int e = lane; e < NK * NX; e += 64) Kf[e] = -Rh[e];
            __syncthreads();
            // one lane per right-hand side with the column in registers up to NK = 24 (register budget)
            if constexpr (NK <= 24) bk_solve_cols<LDK, NX, NK>(Ks, perm, piv, Kf, NX);
            else bk_solve_wave<LDK, NX>(Ks, NK, perm, piv, Kf, NX, AB);
            for (int e = lane; e < NK * NX; e += 64) Fg[(size_t)k * NK * NX + e] = Kf[e];
            __syncthreads();
            GSTAMP(13);
            if (k > 0) {
                tile_gemm<NX, NX, NK>(
                    lane, [&](int i, int j) { return Hs[i * NV + j]; }, [&](int a, int i) { return Rh[a * NX + i]; },
                    [&](int a, int j) { return Kf[a * NX + j]; }, [&](int i, int j, double v) { T2[i * NX + j] = v; });
                __syncthreads();
                for (int e = lane; e < NX * NX; e += 64) Ps[e] = 0.5 * (T2[e] + T2[(e % NX) * NX + e / NX]);
                __syncthreads();
            }
            GSTAMP(14);
        }
        return 0;
    };

    // ---------------- direction for constraint residuals (rd, ri, re) with the stored factorisation
    auto direction = [&](const double *rd, const double *ri, const double *re) __attribute__((always_inline)) {
        const double dw = dw_c, dc = dc_c;
        for (int j = lane; j < NX; j += 64) pvs[j] = gx[N * NX + j] - lam[(N - 1) * NX + j];
        gsync();
        for (int k = N - 1; k >= 0; k--) {
            lane = lane_opaque();
            const double *rk = R(k);
            const bool en = eqon(k + 1);
            GSTAMP(26);
            if (!rlx)
                for (int j = lane; j < NX; j += 64) pvg[k * NX + j] = pvs[j];
            // every operand of the stage into LDS in one round trip: the record parts, P_{k+1} (T2),
            // the stored stage factorisation (Ks, perm, piv) and feedback (Kf), the stage vectors
            stage_in(k, false);
            {
                const double *kst = Kg + (size_t)k * KSTG;
                glds_copy(T2, Pg + (size_t)k * NX * NX, NX * NX);
                glds_copy(Ks, kst, NK * LDK);
                glds_copy(Kf, Fg + (size_t)k * NK * NX, NK * NX);
                glds_copy(Vs + V_GL, rk + D::O_GL, NV);
                glds_copy(Vs + V_GX, gx + k * NX, NX);
                glds_copy(Vs + V_LK, lam + k * NX, NX);
                glds_copy(Vs + V_RD, rd + k * NX, NX);
                glds_copy(Vs + V_GU, gu + k * NU, NU);
                glds_copy(Vs + V_YE, ye + k * NET, NET);
                glds_copy(Vs + V_RE, re + k * NET, NET);
                if (k > 0) glds_copy(Vs + V_LP, lam + (k - 1) * NX, NX);
                if (k + 1 < N) glds_copy(Vs + V_RN, re + (k + 1) * NET, NEA);
                if (eqon(k) && NE > 0) glds_copy(Vs + V_JE, rk + D::O_JE, NE * NX);
                glds_copy(PPd, kst + NK * LDK, 2 * NK);  // perm, piv (stored as doubles)
                if (NI > 0) {
                    glds_copy(Sl + SL_YI, yi + (size_t)k * NIA, NI);
                    glds_copy(Sl + SL_SS, Ss + (size_t)k * NIA, NI);
                    glds_copy(Sl + SL_GS, gs + (size_t)k * NIA, NI);
                    glds_copy(Sl + SL_RI, ri + (size_t)k * NIA, NI);
                    if (rsm) {
                        glds_copy(Sl + SL_RR, rowr + (size_t)k * NIA, NI);
                        glds_copy(Sl + SL_SP, Spr + (size_t)k * NIA, NI);
                        glds_copy(Sl + SL_SN, Snr + (size_t)k * NIA, NI);
                    }
                }
                if (rlx) {  // elastic dynamics rows: the stage's LU of I + P D_r and permutation, J~ (Hs rows < NX: free)
                    glds_copy(Hs, LUb + (size_t)k * (NX * NX + NX), NX * NX + NX);
                    if (en && NE > 0) glds_copy(Jts, Jtb + (size_t)k * NEA * NX, NE * NX);
                    for (int j = lane; j < NX; j += 64) Drs[j] = rdiag(NRD + (size_t)k * NX + j);
                }
            }
            GCHK(21, k);
            for (int j = lane; j < NX; j += 64)
                if (k == 0) Vs[V_LP + j] = 0.0;
            for (int ee = lane; ee < NEA; ee += 64)
                if (k + 1 >= N) Vs[V_RN + ee] = 0.0;
            for (int e = lane; e < NEA * NX; e += 64)
                if (!(eqon(k) && e < NE * NX)) Vs[V_JE + e] = 0.0;
            gsync();  // the stage's operands have arrived (one round trip)
            flags_in(true);
            for (int e = lane; e < NK; e += 64) {
                perm[e] = (int)PPd[e];
                piv[e] = (int)PPd[NK + e];
#ifdef MF_GCHK
                if (perm[e] < 0 || perm[e] >= NK) { GCHK_BAD(1, perm[e]); perm[e] = e; }
                if (piv[e] < 0 || piv[e] > 2) { GCHK_BAD(2, piv[e]); piv[e] = 1; }
#endif
            }
            if (rlx) {  // p~ = L^-1 p_{k+1} (stored for the forward sweep), rd + the elastic rows' correction
                for (int j = lane; j < NX; j += 64) {
                    pix[j] = (int)Hs[NX * NX + j];
                    Vs[V_RD + j] += rowr[NRD + (size_t)k * NX + j];
                }
                wave_lds_sync();
                if (lane == 0) {
                    double y[NX];
                    lu_solve_lane<NX, NX>(Hs, pix, pvs, 1, y);
#pragma unroll
                    for (int i = 0; i < NX; i++) ptv[i] = y[i];
                }
                wave_lds_sync();
                for (int j = lane; j < NX; j += 64) pvg[k * NX + j] = ptv[j];
            }
            // slack-row weights of the stage (vx: the J_I^T w term), from the staged rows
            for (int q = lane; q < NI; q += 64) {
                double w = Sl[SL_YI + q];
                if (acts[q]) {
                    const double rdq = rsm ? 1.0 / Sl[SL_SP + q] + 1.0 / Sl[SL_SN + q] : 0.0;  // rdiag(k NIA + q)
                    const double sg = Sl[SL_SS + q] + dw, Dd = sg / (1.0 + (dc + rdq) * sg);
                    w += Dd * (Sl[SL_RI + q] + (rsm ? Sl[SL_RR + q] : 0.0) + (Sl[SL_GS + q] - Sl[SL_YI + q]) / sg);
                }
                Vs[V_W + q] = w;
            }
            wave_lds_sync();
            GSTAMP(19);
            for (int a = lane; a < NV; a += 64) {
                const bool fa = a < NX ? (k == 0) : fixs[a - NX];
                double g = 0.0;
                if (!fa) {
                    g = lsm ? 0.0 : Vs[V_GL + a];
                    for (int q = 0; q < NI; q++) g += JIs[q * NV + a] * Vs[V_W + q];
                    if (a < NX) {
                        g += Vs[V_GX + a] - Vs[V_LP + a];
                        for (int jj = 0; jj < NX; jj++) g += Ab[jj * NX + a] * Vs[V_LK + jj];
                        if (eqon(k))
                            for (int ee = 0; ee < NE; ee++) g += Vs[V_JE + ee * NX + a] * Vs[V_YE + ee];
                    } else {
                        g += Vs[V_GU + a - NX];
                        for (int jj = 0; jj < NX; jj++) g += Bb[jj * NU + a - NX] * Vs[V_LK + jj];
                    }
                    for (int m = 0; m < NM; m++) g += JMs[m * NV + a] * Vs[V_YE + NEA + m];
                }
                vx[a] = g;
            }
            for (int j = lane; j < NX; j += 64) {
                double acc = rlx ? ptv[j] : pvs[j];
                for (int l = 0; l < NX; l++) acc += T2[j * NX + l] * Vs[V_RD + l];
                tv[j] = acc;
            }
            gsync();
            GSTAMP(23);
            for (int a = lane; a < NK; a += 64) {
                double z = 0.0;
                if (a < NU) {
                    if (!fixs[a]) {
                        z = vx[NX + a];
                        for (int l = 0; l < NX; l++) z += Bb[l * NU + a] * tv[l];
                    }
                } else if (a - NU >= NEA) {
                    z = Vs[V_RE + a - NU];  // mixed row of stage k
                    if (rsm) z += rowr[NRo + (size_t)k * NET + a - NU];
                } else if (en && a - NU < NE) {
                    const int ee = a - NU;
                    z = Vs[V_RN + ee];
                    if (rsm) z += rowr[NRo + (size_t)(k + 1) * NET + ee];
                    if (rlx)  // J~ rh - J_n D_r p~
                        for (int l = 0; l < NX; l++) z += Jts[ee * NX + l] * Vs[V_RD + l] - Jn[ee * NX + l] * Drs[l] * ptv[l];
                    else
                        for (int l = 0; l < NX; l++) z += Jn[ee * NX + l] * Vs[V_RD + l];
                }
                zv[a] = z;
                duv[a] = -z;
            }
            wave_lds_sync();
            GSTAMP(24);
            if constexpr (NK <= 24 && PH == 1) bk_solve_cols<LDK, 1, NK>(Ks, perm, piv, duv, 1);  // (k_gls: register budget)
            else bk_solve_wave<LDK, 1>(Ks, NK, perm, piv, duv, 1, Ys);
            GCHK(22, k);
            for (int a = lane; a < NK; a += 64) kvg[k * NK + a] = duv[a];
            GSTAMP(25);
            if (k > 0)
                for (int j = lane; j < NX; j += 64) {
                    double acc = vx[j];
                    for (int l = 0; l < NX; l++) acc += Ab[l * NX + j] * tv[l];
                    for (int a = 0; a < NK; a++) acc += Kf[a * NX + j] * zv[a];
                    pvs[j] = acc;
                }
            gsync();
        }
        GSTAMP(26);
        // forward sweep
        GCHK(23, 0);
        for (int j = lane; j < NX; j += 64) { dxs[j] = 0.0; dx[j] = 0.0; }
        for (int ee = lane; ee < NEA; ee += 64) dye[ee] = 0.0;  // state rows of node 0 (inactive)
        gsync();
        for (int k = 0; k < N; k++) {
            lane = lane_opaque();
            const double *rk = R(k);
            const bool en = eqon(k + 1);
            // the stage's operands into LDS first (one round trip), then three LDS-only phases
            glds_copy(Ab, rk + D::O_A, NX * NX);
            glds_copy(T2, Pg + (size_t)k * NX * NX, NX * NX);
            glds_copy(Bb, rk + D::O_B, NX * NU);
            glds_copy(Kf, Fg + (size_t)k * NK * NX, NK * NX);
            if (en && NE > 0) glds_copy(Jn, R(k + 1) + D::O_JE, NE * NX);
            glds_copy(zv, kvg + k * NK, NK);
            glds_copy(tv, pvg + k * NX, NX);
            glds_copy(vx, rd + k * NX, NX);
            if (rlx && en && NE > 0) glds_copy(Jts, Jtb + (size_t)k * NEA * NX, NE * NX);
            for (int e = lane; e < NEA * NX; e += 64)
                if (!(en && e < NE * NX)) Jn[e] = 0.0;
            bounds_in(k);
            gsync();
            flags_in(false);
            for (int a = lane; a < NK; a += 64) {
                double acc = zv[a];
                for (int j = 0; j < NX; j++) acc += Kf[a * NX + j] * dxs[j];
                if (a < NU && fixs[a]) acc = 0.0;
                duv[a] = acc;
                if (a < NU) du[k * NU + a] = acc;
            }
            double drj = 0.0, dlj = 0.0;  // (elastic dynamics rows) D_r and dlam of this lane's state j
            if (rlx)
                for (int j = lane; j < NX; j += 64) {
                    vx[j] += rowr[NRD + (size_t)k * NX + j];
                    drj = rdiag(NRD + (size_t)k * NX + j);
                }
            wave_lds_sync();
            for (int j = lane; j < NX; j += 64) {
                double acc = vx[j];
                for (int l = 0; l < NX; l++) acc += Ab[j * NX + l] * dxs[l];
                for (int c = 0; c < NU; c++) acc += Bb[j * NU + c] * duv[c];
                dxn[j] = acc;
            }
            wave_lds_sync();
            for (int j = lane; j < NX; j += 64) {
                // dlam = P~ z + p~ + J~^T dy_s, dx_{k+1} = z - D_r dlam (hard rows: P, p, J_n, D_r = 0)
                double acc = tv[j];
                for (int l = 0; l < NX; l++) acc += T2[j * NX + l] * dxn[l];
                const double *Jx = rlx ? Jts : Jn;
                if (en)
                    for (int ee = 0; ee < NE; ee++) acc += Jx[ee * NX + j] * duv[NU + ee];
                dlam[k * NX + j] = acc;
                dlj = acc;
                dx[(k + 1) * NX + j] = rlx ? dxn[j] - drj * acc : dxn[j];
            }
            if (k + 1 < N)
                for (int ee = lane; ee < NEA; ee += 64) dye[(k + 1) * NET + ee] = (en && ee < NE) ? duv[NU + ee] : 0.0;
            for (int m = lane; m < NM; m += 64) dye[k * NET + NEA + m] = duv[NU + NEA + m];
            wave_lds_sync();
            for (int j = lane; j < NX; j += 64) dxs[j] = rlx ? dxn[j] - drj * dlj : dxn[j];
            wave_lds_sync();
        }
        gsync();  // (the sweep's global stores retired before anything reads them back)
        GSTAMP(17);
        GCHK(24, 0);
        // slack rows and bound multipliers
        for (int e = lane; e < N * NI; e += 64) {
            const int k = e / NI, q = e % NI, i = k * NIA + q;
            double dyv = 0.0, dsv = 0.0;
            if (cact(k, q)) {
                const double *rk = R(k);
                double jd = 0.0;
                for (int a = 0; a < NX; a++) jd += rk[D::O_JI + q * NV + a] * dx[k * NX + a];
                for (int a = 0; a < NU; a++) jd += rk[D::O_JI + q * NV + NX + a] * du[k * NU + a];
                const double sg = Ss[i] + dw, Dd = sg / (1.0 + (dc + rdiag(i)) * sg), rs = gs[i] - yi[i];
                dyv = Dd * (jd + ri[i] + (rsm ? rowr[i] : 0.0) + rs / sg);
                dsv = (dyv - rs) / sg;
            }
            dyi[i] = dyv;
            ds[i] = dsv;
        }
        gsync();
        for (int e = lane; e < (N + 1) * NX; e += 64) {
            const int k = e / NX, j = e % NX;
            double a = 0.0, c = 0.0;
            if (k > 0) {
                if (gb(P.x_lo[j])) a = mu / (x[e] - P.x_lo[j]) - zxL[e] - zxL[e] / (x[e] - P.x_lo[j]) * dx[e];
                if (gb(P.x_hi[j])) c = mu / (P.x_hi[j] - x[e]) - zxU[e] + zxU[e] / (P.x_hi[j] - x[e]) * dx[e];
            }
            dzxL[e] = a;
            dzxU[e] = c;
        }
        for (int e = lane; e < N * NU; e += 64) {
            double a = 0.0, c = 0.0;
            if (!ufix(e)) {
                if (gb(ulo[e])) a = mu / (u[e] - ulo[e]) - zuL[e] - zuL[e] / (u[e] - ulo[e]) * du[e];
                if (gb(uhi[e])) c = mu / (uhi[e] - u[e]) - zuU[e] + zuU[e] / (uhi[e] - u[e]) * du[e];
            }
            dzuL[e] = a;
            dzuU[e] = c;
        }
        for (int e = lane; e < N * NI; e += 64) {
            const int i = (e / NI) * NIA + e % NI;
            double a = 0.0, c = 0.0;
            if (gb(clo[e])) a = mu / (s[i] - clo[e]) - vL[i] - vL[i] / (s[i] - clo[e]) * ds[i];
            if (gb(chi[e])) c = mu / (chi[e] - s[i]) - vU[i] + vU[i] / (chi[e] - s[i]) * ds[i];
            dvL[i] = a;
            dvU[i] = c;
        }
        if (rsm)  // elastic variables: Sp dp = dy - r_p, Sn dn = -dy - r_n, and their bound multipliers
            for (int r = lane; r < NRI; r += 64) {
                if (!el_on(r)) { dpr[r] = dnr[r] = dzp[r] = dzn[r] = 0.0; continue; }
                const double dy = (size_t)r < NRo ? dyi[r] : ((size_t)r < NRD ? dye[r - NRo] : dlam[r - NRD]), y = el_y(r);
                const double rp = RHO_R + gpr[r] - y, rn = RHO_R + gnr[r] + y;
                dpr[r] = (dy - rp) / Spr[r];
                dnr[r] = (-dy - rn) / Snr[r];
                dzp[r] = mu / prr[r] - zpr[r] - zpr[r] / prr[r] * dpr[r];
                dzn[r] = mu / nrr[r] - znr[r] - znr[r] / nrr[r] * dnr[r];
            }
        gsync();
        GSTAMP(18);
    };

    auto ftb = [&](double &ap_o, double &az_o) __attribute__((always_inline)) {
        double ap = 1.0, az = 1.0;
        auto one = [&](double v, double dv, double lo, double hi, double zl, double dzl, double zu, double dzu) __attribute__((always_inline)) {
            if (gb(lo)) {
                if (dv < 0) ap = fmin(ap, -tau_fb * (v - lo) / dv);
                if (dzl < 0) az = fmin(az, -tau_fb * zl / dzl);
            }
            if (gb(hi)) {
                if (dv > 0) ap = fmin(ap, tau_fb * (hi - v) / dv);
                if (dzu < 0) az = fmin(az, -tau_fb * zu / dzu);
            }
        };
        for (int e = lane + NX; e < (N + 1) * NX; e += 64) {
            const int j = e % NX;
            one(x[e], dx[e], P.x_lo[j], P.x_hi[j], zxL[e], dzxL[e], zxU[e], dzxU[e]);
        }
        for (int e = lane; e < N * NU; e += 64)
            if (!ufix(e)) one(u[e], du[e], ulo[e], uhi[e], zuL[e], dzuL[e], zuU[e], dzuU[e]);
        for (int e = lane; e < N * NI; e += 64) {
            const int i = (e / NI) * NIA + e % NI;
            one(s[i], ds[i], clo[e], chi[e], vL[i], dvL[i], vU[i], dvU[i]);
        }
        if (rsm)
            for (int r = lane; r < NRI; r += 64)
                if (el_on(r)) {
                    one(prr[r], dpr[r], 0.0, INFINITY, zpr[r], dzp[r], 0.0, 0.0);
                    one(nrr[r], dnr[r], 0.0, INFINITY, znr[r], dzn[r], 0.0, 0.0);
                }
        ap_o = wave_min(ap);
        az_o = wave_min(az);
    };

    // barrier objective + l1 violation at (xx, uu, ss): cur = the current point (values in the records)
    auto merit = [&](const double *xx, const double *uu, const double *ss, bool cur, double *trd, double *tri,
                     double *tre, double &phi, double &th, bool &okp) __attribute__((always_inline)) {
        double fs = 0.0, t = 0.0, bar = 0.0, lin = 0.0;
        int bad = 0;
        const double *pe = cur ? prr : tpr, *ne_ = cur ? nrr : tnr;  // elastic variables of the point (rsm)
        GCHK(40, cur);
        for (int k = lane; k < N; k += 64) {
            double l, ci[NIA], ce[NET], f[NX];
            GCHK_LANE((k << 8) | 1);
            if (cur) {
                const double *rk = R(k);
                l = rk[D::O_L];
                for (int q = 0; q < NI; q++) ci[q] = rk[D::O_CI + q];
                for (int ee = 0; ee < NE; ee++) ce[ee] = rk[D::O_CE + ee];
                for (int m = 0; m < NM; m++) ce[NE + m] = rk[D::O_CM + m];
                for (int j = 0; j < NX; j++) f[j] = rk[D::O_F + j];
            } else {
#ifdef MF_GCHK
                {  // which operand of the node function faults
                    volatile double sink;
                    sink = xx[(size_t)k * NX];
                    GCHK_LANE((k << 8) | 11);
                    sink = uu[(size_t)k * NU + NU - 1];
                    GCHK_LANE((k << 8) | 12);
                    sink = lref[0];
                    GCHK_LANE((k << 8) | 13);
                    sink = P.fdir[0] + P.h;
                    GCHK_LANE((k << 8) | 14);
                    sink = M[0].g[2] + (double)M[0].n;
                    GCHK_LANE((k << 8) | 15);
                    sink = M[0].j[FAM::NJ - 1].m;
                    GCHK_LANE((k << 8) | 16);
                    sink = F[0].t[2] + (double)F[0].parent;
                    GCHK_LANE((k << 8) | 17);
                    (void)sink;
                }
#endif
                FAM::values(M, F, P, xx + (size_t)k * NX, uu + (size_t)k * NU, lref, l, ci, ce, f);
            }
            GCHK_LANE((k << 8) | 2);
            if (!rsm) fs += l;
            for (int j = 0; j < NX; j++) {
                const size_t rr = NRD + (size_t)k * NX + j;
                const double r = f[j] - xx[(k + 1) * NX + j] + (rlx ? ne_[rr] - pe[rr] : 0.0);
                t += fabs(r);
                if (trd) trd[k * NX + j] = r;
            }
            GCHK_LANE((k << 8) | 3);
            for (int q = 0; q < NI; q++) {
                const int i = k * NIA + q;
                const double r = cact(k, q) ? ci[q] - ss[i] + (rsm ? ne_[i] - pe[i] : 0.0) : 0.0;
                t += fabs(r);
                if (tri) tri[i] = r;
            }
            GCHK_LANE((k << 8) | 4);
            const bool eo = eqon(k);
            for (int ee = 0; ee < NEA; ee++) {
                const size_t rr = NRo + (size_t)k * NET + ee;
                const double r = (eo && ee < NE) ? ce[ee] + (rsm ? ne_[rr] - pe[rr] : 0.0) : 0.0;
                t += fabs(r);
                if (tre) tre[k * NET + ee] = r;
            }
            for (int m = 0; m < NM; m++) {  // families write the mixed rows after their NE state rows
                const size_t rr = NRo + (size_t)k * NET + NEA + m;
                const double r = ce[NE + m] + (rsm ? ne_[rr] - pe[rr] : 0.0);
                t += fabs(r);
                if (tre) tre[k * NET + NEA + m] = r;
            }
            GCHK_LANE((k << 8) | 5);
        }
        GCHK(41, cur);
        auto blog = [&](double v, double lo, double hi) __attribute__((always_inline)) {
            if (gb(lo)) { if (v - lo <= 0) bad = 1; else bar -= log(v - lo); }
            if (gb(hi)) { if (hi - v <= 0) bad = 1; else bar -= log(hi - v); }
            if (flt && gb(lo) && !gb(hi)) lin += v - lo;
            if (flt && gb(hi) && !gb(lo)) lin += hi - v;
        };
        for (int e = lane + NX; e < (N + 1) * NX; e += 64) blog(xx[e], P.x_lo[e % NX], P.x_hi[e % NX]);
        for (int e = lane; e < N * NU; e += 64)
            if (!ufix(e)) blog(uu[e], ulo[e], uhi[e]);
        for (int e = lane; e < N * NI; e += 64) blog(ss[(e / NI) * NIA + e % NI], clo[e], chi[e]);
        if (rsm) {  // restoration objective: rho sum(p + n) + zeta/2 |D_R (w - w_R)|^2, barrier and damping on p, n
            double pn = 0.0, prox = 0.0;
            for (int r = lane; r < NRI; r += 64)
                if (el_on(r)) {
                    pn += pe[r] + ne_[r];
                    if (pe[r] <= 0 || ne_[r] <= 0) bad = 1;
                    else bar -= log(pe[r]) + log(ne_[r]);
                }
            for (int e = lane + NX; e < (N + 1) * NX; e += 64) prox += dR[e] * (xx[e] - wR[e]) * (xx[e] - wR[e]);
            for (int e = lane; e < N * NU; e += 64)
                if (!ufix(e)) prox += dR[Z.x() + e] * (uu[e] - wR[Z.x() + e]) * (uu[e] - wR[Z.x() + e]);
            fs += RHO_R * pn + 0.5 * st.zeta * prox;
            lin += pn;
        }
        fs = wave_sum(fs);
        t = wave_sum(t);
        bar = wave_sum(bar);
        bad = wave_sum_i(bad);
        phi = fs + mu * bar;
        if (flt) phi += KAPPA_D * mu * wave_sum(lin);
        th = t;
        okp = bad == 0;
        gsync();
        GCHK(42, cur);
    };
    auto trial = [&](double al) __attribute__((always_inline)) {
        for (int e = lane; e < (N + 1) * NX; e += 64) tx[e] = x[e] + al * dx[e];
        for (int e = lane; e < N * NU; e += 64) tu[e] = u[e] + al * du[e];
        for (int e = lane; e < N * NIA; e += 64) ts[e] = s[e] + al * ds[e];
        if (rsm)
            for (int r = lane; r < NRI; r += 64) { tpr[r] = prr[r] + al * dpr[r]; tnr[r] = nrr[r] + al * dnr[r]; }
        gsync();
    };
    // direction arrays (save / restore around second-order corrections)
    // the direction's / the iterate's arrays (with the elastic variables in the restoration phase) to / from buf
    auto dir_copy_to = [&](double *buf, bool save) __attribute__((always_inline)) {
        double *arr[16] = {dx, du, ds, dlam, dye, dyi, dzxL, dzxU, dzuL, dzuU, dvL, dvU, dpr, dnr, dzp, dzn};
        const size_t len[16] = {Z.x(), Z.u(), Z.i(), Z.l(), Z.e(), Z.i(), Z.x(), Z.x(), Z.u(), Z.u(), Z.i(), Z.i(),
                                Z.nr(), Z.nr(), Z.nr(), Z.nr()};
        size_t off = 0;
        const int na = rsm ? 16 : 12;
        for (int a = 0; a < na; a++) {
            for (size_t e = lane; e < len[a]; e += 64) {
                if (save) buf[off + e] = arr[a][e];
                else arr[a][e] = buf[off + e];
            }
            off += len[a];
        }
        gsync();
    };
    auto dir_copy = [&](bool save) __attribute__((always_inline)) { dir_copy_to(bkp, save); };
    auto iter_copy_to = [&](double *buf, bool save) __attribute__((always_inline)) {
        double *arr[16] = {x, u, s, lam, ye, yi, zxL, zxU, zuL, zuU, vL, vU, prr, nrr, zpr, znr};
        const size_t len[16] = {Z.x(), Z.u(), Z.i(), Z.l(), Z.e(), Z.i(), Z.x(), Z.x(), Z.u(), Z.u(), Z.i(), Z.i(),
                                Z.nr(), Z.nr(), Z.nr(), Z.nr()};
        size_t off = 0;
        const int na = rsm ? 16 : 12;
        for (int a = 0; a < na; a++) {
            for (size_t e = lane; e < len[a]; e += 64) {
                if (save) buf[off + e] = arr[a][e];
                else arr[a][e] = buf[off + e];
            }
            off += len[a];
        }
        gsync();
    };

    if constexpr (PH == 3) {
    // ---------------- speculative inertia try t (IPOPT mode): the t-th delta_w of the search k_gkkt will make
    const int t = blockIdx.x % GNSPEC;
    if (!flt || lsm || st.pend == GP_IDLE || st.pend == GP_IDLE_RESTO || st.pend == GP_WDSOFT) {
        if (lane == 0) A.sres[blockIdx.x] = -1;
        return;
    }
    double dw = 0.0;
    if (t > 0) {
        dw = (st.ic_last == 0.0) ? 1e-4 : fmax(1e-20, st.ic_last / 3.0);
        for (int i = 1; i < t; i++) dw *= (st.ic_last == 0.0 || 1e5 * st.ic_last < dw) ? 100.0 : 8.0;
    }
    const double dc = P.dc_always ? 1e-8 * pow(mu, 0.25) : 0.0;
    const int fr = factor(dw, dc, 0.0);
    if (lane == 0) {
        A.sres[blockIdx.x] = fr;
        A.sdw[blockIdx.x] = dw;
        A.sdc[blockIdx.x] = dc;
    }
    return;
    }  // PH 3

    if constexpr (PH == 1) {
    if (flt && (st.pend == GP_IDLE || st.pend == GP_IDLE_RESTO || st.pend == GP_WDSOFT)) return;
    if (flt && A.fast_kkt && st.mode == 0 && st.pend == GP_NONE) return;  // taken by k_gkkt_chain (gchain.hip)
    // a try k_gspec has made with exactly these parameters: its result, and on success the direction (and the line
    // search's corrections, st.frow) use its factors where they lie
    const int srow = (flt && !lsm && A.spec_of) ? A.spec_of[b] : -1;
    st.frow = -1;
    auto spec_try = [&](double dw_, double dc_, double d1_, int &fr_) __attribute__((always_inline)) -> bool {
        if (srow < 0 || d1_ != 0.0) return false;
        for (int t = 0; t < GNSPEC; t++) {
            const size_t r = (size_t)srow * GNSPEC + t;
            if (A.sres[r] < 0 || A.sdw[r] != dw_ || A.sdc[r] != dc_) continue;
            fr_ = A.sres[r];
            if (fr_ == 0) {
                use_row(r);
                st.frow = (int)r;
            }
            return true;
        }
        return false;
    };
    // ---------------- inertia correction.  Merit mode: DESIGN.md section 4 (tiers).  IPOPT mode
    // (IpPDPerturbationHandler.cpp, oracle/mf_ocp.c factor_f): delta_w = 0 first; on wrong inertia 1e-4 if no
    // earlier perturbation, else max(1e-20, last / 3); then x100 (no earlier one, or last far below) or x8 up to
    // 1e40.  A singular matrix first gets delta_c = 1e-8 mu^(1/4).  The least-square multiplier pass of a
    // restoration start factors once, unperturbed.  (One factor / direction call site: the kernel's registers.)
    double dw = 0.0, dc = (P.dc_always && !lsm) ? 1e-8 * pow(mu, 0.25) : 0.0, d1 = 0.0;
    int tier = st.reg_tier, step_no = 0;
    double reg = (st.reg_tier == 0) ? 0.0 : st.reg_last / 3.0;
    if (st.reg_tier != 0 && reg < 1e-8) { tier = 0; reg = 0.0; }
    if (tier == 1) d1 = reg; else if (tier == 2) dw = reg;
    if (flt) { dw = 0.0; d1 = 0.0; }
    const bool has_t1 = P.tier1_to > P.tier1_from;
    bool factor_ok = false;
    const int max_tries = flt ? 200 : 60;
    for (int tries = 0; tries < max_tries; tries++) {
        GSTAMP_COUNT(20, 1);
        int fr;
        if (!spec_try(dw, dc, d1, fr)) fr = factor(dw, dc, d1);
        if (fr == 0) { factor_ok = true; break; }
        if (lsm) break;
        if (fr == 2 && dc == 0.0) { dc = 1e-8 * pow(mu, 0.25); continue; }
        st.n_ic++;
        if (flt) {
            if (dw == 0.0) dw = (st.ic_last == 0.0) ? 1e-4 : fmax(1e-20, st.ic_last / 3.0);
            else dw *= (st.ic_last == 0.0 || 1e5 * st.ic_last < dw) ? 100.0 : 8.0;
            if (dw > 1e40) break;
            continue;
        }
        step_no++;
        if (tier == 0) {
            tier = has_t1 ? 1 : 2;
            reg = 1e-4;
        } else if (step_no == 1 && st.reg_tier == tier && reg < st.reg_last) {
            reg = st.reg_last;
        } else {
            reg *= 8.0;
            if (tier == 1 && reg > 1e6) { tier = 2; reg = 1e-4; }
        }
        if (reg > 1e40) break;
        d1 = (tier == 1) ? reg : 0.0;
        dw = (tier == 2) ? reg : 0.0;
    }
    GCHK(30, factor_ok);
    if (!factor_ok && !lsm) { finish(GS_INERTIA); return; }
    if (lsm) {
        dw_c = 0.0;
        dc_c = factor_ok ? 0.0 : -1.0;  // -1: singular system, the multipliers stay 0 (k_gls)
    } else {
        if (flt) {
            if (dw > 0.0) st.ic_last = dw;
        } else {
            st.reg_tier = tier;
            st.reg_last = reg;
        }
        dw_c = dw;
        dc_c = dc;
    }
    GSTAMP(2);
    if (factor_ok) direction(rdyn, rin, req);
    GSTAMP(3);
    GSTAMP_FLUSH;
    if (lane == 0) {
        st.dw_c = dw_c;
        st.dc_c = dc_c;
        A.st[b] = st;
    }
    return;
    }  // PH 1

    // ---------------- step, line search with second-order corrections, update
    dw_c = st.dw_c;
    dc_c = st.dc_c;
    if (flt) {
    // ================= IPOPT's FindAcceptableTrialPoint (oracle/mf_ocp.c ipm_filter / filter_backtrack)
    if (st.pend == GP_IDLE || st.pend == GP_IDLE_RESTO) {
        if (lane == 0) {
            if (st.pend == GP_IDLE) st.iter++;  // (the restoration's exit ends an iteration; an undone soft step not)
            st.pend = st.pend == GP_IDLE_RESTO ? GP_RESTO : GP_NONE;
            A.st[b] = st;
        }
        return;
    }
    if (lsm) {  // least-square multipliers of the restoration start: 0 if singular or max |y| > 1000
        double ym = 0.0;
        for (int e = lane; e < N * NX; e += 64) ym = fmax(ym, fabs(dlam[e]));
        for (int e = lane; e < N * NIA; e += 64) ym = fmax(ym, fabs(dyi[e]));
        for (int e = lane; e < N * NET; e += 64) ym = fmax(ym, fabs(dye[e]));
        ym = wave_max(ym);
        if (dc_c == 0.0 && ym <= 1e3) {
            for (int e = lane; e < N * NX; e += 64) lam[e] = dlam[e];
            for (int e = lane; e < N * NIA; e += 64) yi[e] = dyi[e];
            for (int e = lane; e < N * NET; e += 64) ye[e] = dye[e];
        }
        gsync();
        if (lane == 0) {
            st.pend = GP_NONE;
            A.st[b] = st;
        }
        return;
    }
    const int m = st.mode;
    auto apply_step = [&](double al, double azz) __attribute__((always_inline)) {
        for (int e = lane; e < (N + 1) * NX; e += 64) x[e] += al * dx[e];
        for (int e = lane; e < N * NU; e += 64) u[e] += al * du[e];
        for (int e = lane; e < N * NIA; e += 64) { s[e] += al * ds[e]; yi[e] += al * dyi[e]; }
        for (int e = lane; e < N * NX; e += 64) lam[e] += al * dlam[e];
        for (int e = lane; e < N * NET; e += 64) ye[e] += al * dye[e];
        if (rsm)
            for (int r = lane; r < NRI; r += 64)
                if (el_on(r)) { prr[r] += al * dpr[r]; nrr[r] += al * dnr[r]; }
        gsync();
        auto zupd = [&](double &z, double dz, double sl) __attribute__((always_inline)) {
            const double zz = z + azz * dz;
            z = fmax(fmin(zz, kappa_sigma * mu / sl), mu / (kappa_sigma * sl));
        };
        for (int e = lane + NX; e < (N + 1) * NX; e += 64) {
            const int j = e % NX;
            if (gb(P.x_lo[j])) zupd(zxL[e], dzxL[e], x[e] - P.x_lo[j]);
            if (gb(P.x_hi[j])) zupd(zxU[e], dzxU[e], P.x_hi[j] - x[e]);
        }
        for (int e = lane; e < N * NU; e += 64) {
            if (ufix(e)) continue;
            if (gb(ulo[e])) zupd(zuL[e], dzuL[e], u[e] - ulo[e]);
            if (gb(uhi[e])) zupd(zuU[e], dzuU[e], uhi[e] - u[e]);
        }
        for (int e = lane; e < N * NI; e += 64) {
            const int i = (e / NI) * NIA + e % NI;
            if (gb(clo[e])) zupd(vL[i], dvL[i], s[i] - clo[e]);
            if (gb(chi[e])) zupd(vU[i], dvU[i], chi[e] - s[i]);
        }
        if (rsm)
            for (int r = lane; r < NRI; r += 64)
                if (el_on(r)) { zupd(zpr[r], dzp[r], prr[r]); zupd(znr[r], dzn[r], nrr[r]); }
        gsync();
    };
    auto store = [&]() __attribute__((always_inline)) {
        if (lane == 0) {
            if (m == 1) st.n_rit++;
            st.iter++;
            st.mu = mu;
            A.st[b] = st;
        }
    };
    double ap, az;
    ftb(ap, az);
    double phc, thc, gdc = 0.0;
    bool okc;
    merit(x, u, s, true, nullptr, nullptr, nullptr, phc, thc, okc);
    for (int k = lane; k < N; k += 64) {
        const double *rk = R(k);
        for (int a = 0; a < NV; a++) gdc += rk[D::O_GL + a] * (a < NX ? dx[k * NX + a] : du[k * NU + a - NX]);
    }
    for (int e = lane; e < N * NU; e += 64) gdc += gu[e] * du[e];
    for (int e = lane; e < N * NIA; e += 64) gdc += gs[e] * ds[e];
    for (int e = lane + NX; e < (N + 1) * NX; e += 64) gdc += gx[e] * dx[e];
    if (rsm)
        for (int r = lane; r < NRI; r += 64)
            if (el_on(r)) gdc += (RHO_R + gpr[r]) * dpr[r] + (RHO_R + gnr[r]) * dnr[r];
    gdc = wave_sum(gdc);
    if (st.thm[m][0] < 0.0) {
        st.thm[m][0] = 1e4 * fmax(1.0, thc);
        st.thm[m][1] = 1e-4 * fmax(1.0, thc);
    }
    constexpr double EPS10 = 10.0 * 2.220446049250313e-16;
    auto ftype = [&](double a, double rth, double rgd) __attribute__((always_inline)) { return rgd < 0.0 && a * pow(-rgd, 2.3) > pow(rth, 1.1); };
    auto armijo = [&](double a, double ph, double rph, double rgd) __attribute__((always_inline)) { return ph - rph - 1e-8 * a * rgd <= EPS10 * fabs(rph); };
    // CheckAcceptabilityOfTrialPoint (IpFilterLSAcceptor.cpp); every argument is wave-uniform
    auto acceptable = [&](double atest, double ph, double th, bool ok, double rph, double rth, double rgd) __attribute__((always_inline)) -> bool {
        if (!ok || !isfinite(ph) || !isfinite(th)) return false;
        if (th > st.thm[m][0]) return false;
        if (atest > 0.0 && ftype(atest, rth, rgd) && rth <= st.thm[m][1]) {
            if (!armijo(atest, ph, rph, rgd)) return false;
        } else {
            if (ph > rph) {
                const double bas = fabs(rph) > 10.0 ? log10(fabs(rph)) : 1.0;
                if (log10(ph - rph) > 5.0 + bas) return false;
            }
            if (!((th - (1.0 - 1e-5) * rth <= EPS10 * fabs(rth)) || (ph - rph + 1e-8 * rth <= EPS10 * fabs(rph))))
                return false;
        }
        return fil_ok(m, ph, th);
    };
    auto alpha_min = [&](double rth, double rgd) __attribute__((always_inline)) {
        double am = 1e-5;
        if (rgd < 0.0) {
            am = fmin(1e-5, 1e-8 * rth / (-rgd));
            if (rth <= st.thm[m][1]) am = fmin(am, pow(rth, 1.1) / pow(-rgd, 2.3));
        }
        return 0.05 * am;
    };
    // DoBacktrackingLineSearch with second-order corrections
    auto backtrack = [&](bool skip_first, bool inwd, double ap_, double th_cur, double rph, double rth, double rgd,
                         double &alpha_o, double &atest_o, int &ns_o, int &soc_o, double &ph_o, double &azz) __attribute__((always_inline)) -> bool {
        const double amin = inwd ? ap_ : alpha_min(rth, rgd);
        double alpha = ap_, atest = inwd ? st.wd_atest : ap_, ph = 0.0, th = 0.0, last = ap_;
        int ns = 0, soc = 0;
        bool acc = false;
        if (skip_first) alpha *= 0.5;
        while (alpha > amin || ns == 0) {
            if (!inwd) atest = alpha;
            last = alpha;
            trial(alpha);
            bool ok;
            merit(tx, tu, ts, false, trdyn, trin, treq, ph, th, ok);
            if (acceptable(atest, ph, th, ok, rph, rth, rgd)) { acc = true; break; }
            if (inwd) break;
            if (ok && alpha == ap_ && th_cur <= th && P.max_soc > 0) {
                double th_trial = th, th_old = 0.0, a_soc = alpha;
                for (int e = lane; e < N * NX; e += 64) sdyn[e] = rdyn[e];
                for (int e = lane; e < N * NIA; e += 64) sin_[e] = rin[e];
                for (int e = lane; e < N * NET; e += 64) seq[e] = req[e];
                gsync();
                for (int cnt = 0; cnt < P.max_soc && (cnt == 0 || th_trial <= 0.99 * th_old); cnt++) {
                    th_old = th_trial;
                    for (int e = lane; e < N * NX; e += 64) sdyn[e] = a_soc * sdyn[e] + trdyn[e];
                    for (int e = lane; e < N * NIA; e += 64) sin_[e] = a_soc * sin_[e] + trin[e];
                    for (int e = lane; e < N * NET; e += 64) seq[e] = a_soc * seq[e] + treq[e];
                    gsync();
                    dir_copy(true);
                    direction(sdyn, sin_, seq);
                    double azs;
                    ftb(a_soc, azs);
                    trial(a_soc);
                    bool oks;
                    merit(tx, tu, ts, false, trdyn, trin, treq, ph, th, oks);
                    if (acceptable(atest, ph, th, oks, rph, rth, rgd)) {
                        acc = true; soc = 1; alpha = a_soc; azz = azs;
                        break;
                    }
                    dir_copy(false);
                    if (!oks) break;
                    th_trial = th;
                }
                if (acc) break;
            }
            alpha *= 0.5;
            ns++;
        }
        alpha_o = acc ? alpha : last;
        atest_o = atest;
        ns_o = ns;
        soc_o = soc;
        ph_o = ph;
        return acc;
    };
    // TrySoftRestoStep (first half): the step min(alpha_primal, alpha_dual) for primal and dual variables;
    // 1: the original criteria accept it, 2: taken pending the primal-dual error test of the next k_gpre (the
    // point is kept in wdit), 0: failed
    auto soft_step = [&](double &a_o) __attribute__((always_inline)) -> int {
        const double a = fmin(ap, az);
        a_o = a;
        trial(a);
        double ph, th;
        bool ok;
        merit(tx, tu, ts, false, nullptr, nullptr, nullptr, ph, th, ok);
        if (acceptable(0.0, ph, th, ok, phc, thc, gdc)) return 1;
        if (!ok) return 0;
        const GErr E = opt_err(mu);
        st.pd_cur = E.s1 / E.n1;
        iter_copy_to(A.wdit + b * Z.bk(), true);
        return 2;
    };
    bool want_soft = false, soft_entry = false, go_resto = false, do_step = false;
    double step_a = 0.0, step_az = 0.0;
    if (st.pend == GP_WDSOFT) {
        // the failed search after StopWatchDog, continued with the stored point's records: PrepareRestoPhaseStart
        // (the filter takes the point, phc / thc evaluated there above), then the soft restoration phase
        st.pend = GP_NONE;
        st.n_ls_fail++;
        fil_add(0, phc - 1e-8 * thc, (1.0 - 1e-5) * thc);
        want_soft = true;
        soft_entry = true;
    } else if (m == 0 && st.in_soft) {  // soft restoration phase: at most max_soft_resto_iters = 10 iterations
        if (++st.soft_cnt <= 10) want_soft = true;
        else go_resto = true;
    } else {
        if (!st.in_wd && st.wd_short >= 10) {  // StartWatchDog
            st.in_wd = 1; st.wd_trial = 0; st.n_wd++;
            st.wd_ph = phc; st.wd_th = thc; st.wd_gd = gdc; st.wd_atest = ap;
            iter_copy_to(A.wdit + b * Z.bk(), true);
            dir_copy_to(A.wddir + b * Z.bk(), true);
        }
        double rph = st.in_wd ? st.wd_ph : phc, rth = st.in_wd ? st.wd_th : thc, rgd = st.in_wd ? st.wd_gd : gdc;
        double alpha = ap, atest = ap, pht = 0.0, th_cur = thc;
        int n_steps = 0, soc_used = 0;
        bool wd_step = false, accepted = false, wd_stopped = false;
        for (int pass = 0; pass < 2; pass++) {
            const bool inwd = pass == 0 && st.in_wd;
            accepted = backtrack(pass == 1, inwd, ap, th_cur, rph, rth, rgd, alpha, atest, n_steps, soc_used, pht, az);
            if (!inwd) break;
            if (accepted) { st.in_wd = 0; break; }
            if (++st.wd_trial > 3) {  // StopWatchDog: the stored point and direction, backtrack from alpha_max / 2
                st.in_wd = 0;
                st.wd_short = 0;
                iter_copy_to(A.wdit + b * Z.bk(), false);
                dir_copy_to(A.wddir + b * Z.bk(), false);
                ftb(ap, az);
                rph = st.wd_ph; rth = st.wd_th; rgd = st.wd_gd;
                th_cur = INFINITY;  // (no second-order correction after a skipped first trial point)
                wd_stopped = true;
                continue;
            }
            accepted = true;  // the watchdog's full trial step, no filter update
            wd_step = true;
            alpha = ap;
            n_steps = 0;
            break;
        }
        if (accepted && !wd_step && (!ftype(atest, rth, rgd) || !armijo(atest, pht, rph, rgd)))
            fil_add(m, rph - 1e-8 * rth, (1.0 - 1e-5) * rth);
        if (accepted) {
            st.n_soc += soc_used;
            if (!st.in_wd) st.wd_short = (n_steps == 0) ? 0 : st.wd_short + 1;
            do_step = true;
            step_a = alpha;
            step_az = az;
        } else if (wd_stopped && m == 0) {
            // the records describe the abandoned watchdog point: re-evaluate at the restored one first (GP_WDSOFT)
            if (lane == 0) {
                st.pend = GP_WDSOFT;
                st.frow = -1;  // (the next round's k_gspec may reuse this round's storage rows)
                st.n_wdfail++;
                st.mu = mu;
                A.st[b] = st;
            }
            return;
        } else {
            st.n_ls_fail++;
            if (m == 1) { finish(GS_RESTOFAIL); return; }  // no restoration inside the restoration phase
            // PrepareRestoPhaseStart (the filter takes the current point), then the soft restoration phase, then
            // the restoration phase if its first step fails
            fil_add(0, phc - 1e-8 * thc, (1.0 - 1e-5) * thc);
            ftb(ap, az);
            want_soft = true;
            soft_entry = true;
        }
    }
    if (want_soft) {
        // the point a restoration would start from (MinC_1NrmRestorationPhase's reference): this iteration's, also
        // when k_gpre undoes the pending step
        st.rs_ph = phc;
        st.rs_th = thc;
        double a = 0.0;
        const int r = soft_step(a);
        if (r == 0) {
            go_resto = true;
        } else {
            do_step = true;
            step_a = step_az = a;
            if (r == 1) {
                st.in_soft = 0;
                st.soft_cnt = 0;
                st.n_soft++;
            } else {
                if (soft_entry) { st.in_soft = 1; st.soft_cnt = 0; }
                st.pend = GP_SOFT;
            }
        }
    }
    if (go_resto) {
        st.rs_ph = phc;
        st.rs_th = thc;
        st.in_soft = 0;
        st.soft_cnt = 0;
        st.pend = GP_RESTO;
    }
    if (P.dbg && b == 0 && lane == 0 && st.iter < GDBG_ROWS) {
        double *t = mf_gdbg_ls + st.iter * GDBG_W;
        t[0] = st.iter; t[1] = m; t[2] = thc; t[3] = phc; t[4] = gdc; t[5] = ap; t[6] = az; t[7] = step_a;
        t[8] = do_step; t[9] = want_soft; t[10] = go_resto; t[11] = st.nf[0]; t[12] = st.nf[1]; t[13] = st.in_wd;
        t[14] = st.pend; t[15] = st.in_soft;
    }
    if (do_step) apply_step(step_a, step_az);
    if (go_resto) {  // the restoration phase starts within this iteration (oracle resto_phase): not counted here
        if (lane == 0) {
            st.mu = mu;
            A.st[b] = st;
        }
        return;
    }
    store();
    return;
    }  // flt
    double ap, az;
    GCHK(3, 0);
    ftb(ap, az);
    double phi0, th0;
    bool ok0;
    GCHK(4, 0);
    merit(x, u, s, true, nullptr, nullptr, nullptr, phi0, th0, ok0);
    GCHK(5, 0);
    double gdot = 0.0, pHp = 0.0;
    for (int k = lane; k < N; k += 64) {
        const double *rk = R(k);
        for (int a = 0; a < NV; a++) {
            const double da = a < NX ? dx[k * NX + a] : du[k * NU + a - NX];
            gdot += rk[D::O_GL + a] * da;
            double hd = 0.0;
            for (int c = 0; c < NV; c++) hd += rk[D::O_W + a * NV + c] * (c < NX ? dx[k * NX + c] : du[k * NU + c - NX]);
            pHp += da * hd;
        }
    }
    for (int e = lane; e < N * NU; e += 64) { gdot += gu[e] * du[e]; pHp += Su[e] * du[e] * du[e]; }
    for (int e = lane; e < N * NIA; e += 64) { gdot += gs[e] * ds[e]; pHp += Ss[e] * ds[e] * ds[e]; }
    for (int e = lane + NX; e < (N + 1) * NX; e += 64) { gdot += gx[e] * dx[e]; pHp += Sx[e] * dx[e] * dx[e]; }
    gdot = wave_sum(gdot);
    pHp = wave_sum(pHp);
    if (th0 > 1e-300) {
        const double nreq = (gdot + 0.5 * fmax(pHp, 0.0)) / ((1.0 - rho) * th0);
        if (nu < nreq) nu = nreq + 1.0;
    }
    const double Dphi = gdot - nu * th0, m0 = phi0 + nu * th0;
    const double slack_m = 10.0 * 2.220446049250313e-16 * fabs(m0);
    GSTAMP(4);
    double alpha = ap;
    bool accepted = false;
    int soc_used = 0;
    for (int ls = 0; ls < 40; ls++) {
        GSTAMP(7);
        GCHK(6, ls);
        trial(alpha);
        double ph, th;
        bool okk;
        GCHK(7, ls);
        merit(tx, tu, ts, false, trdyn, trin, treq, ph, th, okk);
        GCHK(8, ls);
        GSTAMP_COUNT(21, 1);
        GSTAMP(5);
        const double mt = ph + nu * th;
        if (okk && isfinite(mt) && mt - m0 <= eta * alpha * fmin(Dphi, 0.0) + slack_m) { accepted = true; break; }
        if (ls == 0 && P.max_soc > 0 && (!okk || th >= th0)) {
            double th_old = th;
            const double a_soc = alpha;
            for (int e = lane; e < N * NX; e += 64) sdyn[e] = alpha * rdyn[e] + trdyn[e];
            for (int e = lane; e < N * NIA; e += 64) sin_[e] = alpha * rin[e] + trin[e];
            for (int e = lane; e < N * NET; e += 64) seq[e] = alpha * req[e] + treq[e];
            gsync();
            for (int p = 0; p < P.max_soc; p++) {
                GSTAMP_COUNT(22, 1);
                GCHK(9, p);
                dir_copy(true);
                GCHK(10, p);
                direction(sdyn, sin_, seq);
                GCHK(11, p);
                double aps, azs;
                ftb(aps, azs);
                trial(aps);
                double phs, ths;
                bool oks;
                GCHK(12, p);
                merit(tx, tu, ts, false, trdyn, trin, treq, phs, ths, oks);
                GCHK(13, p);
                const double ms = phs + nu * ths;
                if (oks && isfinite(ms) && ms - m0 <= eta * a_soc * fmin(Dphi, 0.0) + slack_m) {
                    accepted = true;
                    soc_used = 1;
                    alpha = aps;
                    az = azs;
                    break;
                }
                dir_copy(false);
                GCHK(14, p);
                if (!oks || ths > 0.99 * th_old) break;
                th_old = ths;
                for (int e = lane; e < N * NX; e += 64) sdyn[e] = aps * sdyn[e] + trdyn[e];
                for (int e = lane; e < N * NIA; e += 64) sin_[e] = aps * sin_[e] + trin[e];
                for (int e = lane; e < N * NET; e += 64) seq[e] = aps * seq[e] + treq[e];
                gsync();
            }
            GSTAMP(15);
            if (accepted) break;
        }
        alpha *= 0.5;
    }
    if (!accepted) {
        st.n_ls_fail++;
        if (++st.consec_fail >= 5) { finish(GS_LSFAIL); return; }
    } else {
        st.consec_fail = 0;
    }
    st.n_soc += soc_used;
    GSTAMP(6);
    GCHK(15, 0);
    for (int e = lane; e < (N + 1) * NX; e += 64) x[e] += alpha * dx[e];
    for (int e = lane; e < N * NU; e += 64) u[e] += alpha * du[e];
    for (int e = lane; e < N * NIA; e += 64) { s[e] += alpha * ds[e]; yi[e] += alpha * dyi[e]; }
    for (int e = lane; e < N * NX; e += 64) lam[e] += alpha * dlam[e];
    for (int e = lane; e < N * NET; e += 64) ye[e] += alpha * dye[e];
    gsync();
    auto zupd = [&](double &z, double dz, double sl) __attribute__((always_inline)) {
        const double zz = z + az * dz;
        z = fmax(fmin(zz, kappa_sigma * mu / sl), mu / (kappa_sigma * sl));
    };
    for (int e = lane + NX; e < (N + 1) * NX; e += 64) {
        const int j = e % NX;
        if (gb(P.x_lo[j])) zupd(zxL[e], dzxL[e], x[e] - P.x_lo[j]);
        if (gb(P.x_hi[j])) zupd(zxU[e], dzxU[e], P.x_hi[j] - x[e]);
    }
    for (int e = lane; e < N * NU; e += 64) {
        if (ufix(e)) continue;
        if (gb(ulo[e])) zupd(zuL[e], dzuL[e], u[e] - ulo[e]);
        if (gb(uhi[e])) zupd(zuU[e], dzuU[e], uhi[e] - u[e]);
    }
    for (int e = lane; e < N * NI; e += 64) {
        const int i = (e / NI) * NIA + e % NI;
        if (gb(clo[e])) zupd(vL[i], dvL[i], s[i] - clo[e]);
        if (gb(chi[e])) zupd(vU[i], dvU[i], chi[e] - s[i]);
    }
    GSTAMP(7);
    GSTAMP_FLUSH;
    GCHK(16, 0);
    if (lane == 0) {
        st.iter++;
        st.mu = mu;
        st.nu = nu;
        A.st[b] = st;
    }
}

// Occupancy variants of k_gkkt / k_gls for full launches.  The chain families' stage arrays take ~6 KB of LDS, so
// these kernels are register-limited: the compiler's own allocation (k_gkkt 256 + 40 accumulation registers, k_gls
// about 430) leaves one wave per SIMD, four horizons per CU, and a 4096-horizon launch runs in four rounds of waves
// that are latency-bound (lone and fully loaded waves take nearly the same cycles per stage).  k_gkkt capped at 128
// registers (4 waves per SIMD, 253 spilled) and k_gls at 256 (2 waves, 208 spilled) hold 4x / 2x the horizons: the host takes them while more horizons run than the default kernels hold (four per CU),
// the defaults (no spills, faster lone waves) in the tail.  The box and Centauro families are LDS-limited (~50 KB:
// three horizons per CU) and have only the defaults.
template <class FAM> struct GOcc { static constexpr int KKT = 1, LS = 1; };
template <int NJ, int NF, int NE, bool TH> struct GOcc<ChainFam<NJ, NF, NE, TH>> {
    static constexpr int KKT = 4, LS = 2;
};

template <class FAM>
__global__ __launch_bounds__(64) void k_gpre(const DevModel *M0, const DevModel *M1, const DevFrame *F0,
                                             const DevFrame *F1, GParams P, GArrays A, int batch) {
    giter_phase<FAM, 0, true>(M0, M1, F0, F1, P, A, batch);
}
template <class FAM>
__global__ __launch_bounds__(64) void k_gkkt(const DevModel *M0, const DevModel *M1, const DevFrame *F0,
                                             const DevFrame *F1, GParams P, GArrays A, int batch) {
    giter_phase<FAM, 1, true>(M0, M1, F0, F1, P, A, batch);
}
// the register-capped variant (GOcc): its own kernel, so the default one keeps the compiler's own allocation
template <class FAM, int OCC>
__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(OCC))) void k_gkkt_occ(
    const DevModel *M0, const DevModel *M1, const DevFrame *F0, const DevFrame *F1, GParams P, GArrays A, int batch) {
    giter_phase<FAM, 1, true>(M0, M1, F0, F1, P, A, batch);
}
template <class FAM>
__global__ __launch_bounds__(64) void k_gspec(const DevModel *M0, const DevModel *M1, const DevFrame *F0,
                                              const DevFrame *F1, GParams P, GArrays A, int batch) {
    giter_phase<FAM, 3, true>(M0, M1, F0, F1, P, A, batch);
}
// the running horizons (at most A.spec_max, the host's condition for launching k_gspec) listed for k_gspec
// nonfast: only the horizons k_gkkt_chain leaves to k_gkkt (restoration phase, pending actions): their tries run
// concurrently while the chain kernel takes the others
__global__ __launch_bounds__(1024) void k_gspec_list(GArrays A, int batch, int nonfast) {
    __shared__ int cnt;
    if (threadIdx.x == 0) cnt = 0;
    __syncthreads();
    for (int b = threadIdx.x; b < batch; b += blockDim.x) {
        int s = -1;
        const GState &g = A.st[b];
        if (g.status == GS_RUNNING && !(nonfast && g.mode == 0 && g.pend == GP_NONE)) {
            s = atomicAdd(&cnt, 1);
            if (s >= A.spec_max) s = -1;
            else A.slist[s] = b;
        }
        A.spec_of[b] = s;
    }
    __syncthreads();
    for (int s = cnt + threadIdx.x; s < A.spec_max; s += blockDim.x) A.slist[s] = -1;
}
template <class FAM, bool FLT>
__global__ __launch_bounds__(64) void k_gls(const DevModel *M0, const DevModel *M1, const DevFrame *F0,
                                            const DevFrame *F1, GParams P, GArrays A, int batch) {
    giter_phase<FAM, 2, FLT>(M0, M1, F0, F1, P, A, batch);
}
template <class FAM, bool FLT, int OCC>
__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(OCC))) void k_gls_occ(
    const DevModel *M0, const DevModel *M1, const DevFrame *F0, const DevFrame *F1, GParams P, GArrays A, int batch) {
    giter_phase<FAM, 2, FLT>(M0, M1, F0, F1, P, A, batch);
}


// ============================================================== outputs
template <class D>
__global__ void k_gout(GArrays A, int N, int batch, double *w, int *status, int *iters, double *kkt, double *obj) {
    const int b = blockIdx.x, lane = threadIdx.x;
    if (b >= batch) return;
    const GSz<D> Z(N);
    constexpr int NX = D::NX, NU = D::NU;
    const int ws = NX + N * (NU + NX);
    const double *x = A.x + b * Z.x(), *u = A.u + b * Z.u();
    double *wb = w + (size_t)b * ws;
    for (int e = lane; e < ws; e += blockDim.x) {
        double v;
        if (e < NX) v = x[e];
        else {
            const int k = (e - NX) / (NU + NX), r = (e - NX) % (NU + NX);
            v = r < NU ? u[k * NU + r] : x[(k + 1) * NX + r - NU];
        }
        wb[e] = v;
    }
    if (lane == 0) {
        const GState st = A.st[b];
        if (status) status[b] = st.status == GS_RUNNING ? GS_MAXITER : st.status;  // (host launch bound reached)
        if (iters) iters[b] = st.iter;
        if (kkt) kkt[b] = st.E0;
        if (obj) obj[b] = st.obj;
    }
}

// Continuous batching: every problem's status row starts as max_iter with no iterations, so a problem the host's launch
// bound leaves unassigned to a slot reads as not converged (not as an uninitialised row)
__global__ void k_gout_init(int total, int *status, int *iters, double *kkt, double *obj) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= total) return;
    if (status) status[i] = GS_MAXITER;
    if (iters) iters[i] = 0;
    if (kkt) kkt[i] = INFINITY;
    if (obj) obj[i] = NAN;
}

// Continuous batching: a finished slot's solution goes to its problem's output row, and the slot takes the next
// unsolved problem (x_0 and line reference staged into the slot; k_ginit initialises it).  force: the host's
// launch bound was reached -- running slots are written out as max_iter and no problem is handed out.
template <class FAM>
__global__ __launch_bounds__(64) void k_gharvest(GArrays A, int N, int batch, int force) {
    using D = typename FAM::D;
    constexpr int NX = D::NX, NU = D::NU;
    const int b = blockIdx.x, lane = threadIdx.x;
    if (b >= batch) return;
    const int pb = A.pidx[b];
    if (pb < 0) return;
    const GState st = A.st[b];
    if (st.status == GS_RUNNING && !force) return;
    const GSz<D> Z(N);
    const int ws = NX + N * (NU + NX);
    const double *x = A.x + b * Z.x(), *u = A.u + b * Z.u();
    double *wb = A.ow + (size_t)pb * ws;
    for (int e = lane; e < ws; e += 64) {
        double v;
        if (e < NX) v = x[e];
        else {
            const int k = (e - NX) / (NU + NX), r = (e - NX) % (NU + NX);
            v = r < NU ? u[k * NU + r] : x[(k + 1) * NX + r - NU];
        }
        wb[e] = v;
    }
    int q = A.total;
    if (lane == 0) {
        if (A.ost) A.ost[pb] = st.status == GS_RUNNING ? GS_MAXITER : st.status;
        if (A.oit) A.oit[pb] = st.iter;
        if (A.okkt) A.okkt[pb] = st.E0;
        if (A.oobj) A.oobj[pb] = st.obj;
        if (st.status == GS_RUNNING) atomicSub(A.active, 1);
        if (!force) q = atomicAdd(A.next, 1);
    }
    q = __shfl(q, 0, 64);
    if (q < A.total) {
        for (int j = lane; j < NX; j += 64) A.x0[(size_t)b * NX + j] = A.x0all[(size_t)q * NX + j];
        if (FAM::LREF == 2 && A.lrall)
            for (int j = lane; j < 2; j += 64) A.lref[2 * (size_t)b + j] = A.lrall[2 * (size_t)q + j];
        if (lane == 0) {
            A.pidx[b] = q;
            A.init[b] = 1;
            atomicAdd(A.active, 1);
        }
    } else if (lane == 0) {
        A.pidx[b] = -1;
    }
}

// single node record for tests (batch of one node, multipliers given)
template <class FAM>
__global__ __launch_bounds__(256) void k_grec(const DevModel *M0, const DevModel *M1, const DevFrame *F0,
                                              const DevFrame *F1, GParams P, const double *xu, const double *yi,
                                              const double *ye, const double *lam, const double *lref, double *out) {
    using D = typename FAM::D;
    GMODELS(FAM);
    __shared__ typename FAM::Scratch S;
    const int t = threadIdx.x;
    const double *x = xu, *u = xu + D::NX;
    if (t < FAM::PRE) FAM::prepass(M, F, P, x, u, t, S);
    __syncthreads();
    if (t == 0) FAM::seeds(P, u, yi, ye, lam, true, 1.0, S);
    __syncthreads();
    if (t < FAM::LANES) FAM::lane(M, F, x, u, yi, t, S);
    __syncthreads();
    for (int e = t; e < D::REC; e += blockDim.x) out[e] = FAM::rec(P, x, u, yi, ye, lam, true, S, e, lref);
}

}  // namespace mf

// ====================================================================== host side / C ABI
using namespace mf;

#define GHIPCHK(x)                                                                                    \
    do {                                                                                              \
        hipError_t e_ = (x);                                                                          \
        if (e_ != hipSuccess) return capi_fail(MF_ERR_DEVICE, std::string("HIP error: ") + hipGetErrorString(e_) + " at " #x); \
    } while (0)

// the kernel instantiations (family, dims) and their dispatch
enum GKind { GK_BOX = 0, GK_CH6F = 1, GK_CH6FT = 2, GK_CH3 = 3, GK_CH3T = 4, GK_CENT = 5, GK_BOXT = 6 };
using FamBox = BoxFam;
using FamCh6F = ChainFam<6, 1, 2, false>;
using FamCh6FT = ChainFam<6, 1, 2, true>;
using FamCh3 = ChainFam<3, 0, 0, false>;
using FamCh3T = ChainFam<3, 0, 0, true>;
using FamCent = CentauroFam;
using FamBoxT = BoxThermFam;

struct mf_gproblem {
    mf_model *m0 = nullptr, *m1 = nullptr;
    mf_gspec spec;
    int kind = 0, nx = 0, nu = 0, ni = 0, ne = 0;
    GParams P;
    std::vector<double> ulo, uhi, clo, chi;
    const DevModel *dM0 = nullptr, *dM1 = nullptr;
    DevFrame *dF0 = nullptr, *dF1 = nullptr;
    double *d_ulo = nullptr, *d_uhi = nullptr, *d_clo = nullptr, *d_chi = nullptr;
    // the bound tables relaxed by IPOPT's bound_relax_factor (mf_gopts.bound_relax), made on demand
    double relax = 0.0;
    double *d_ulo_r = nullptr, *d_uhi_r = nullptr, *d_clo_r = nullptr, *d_chi_r = nullptr;
    int cap = 0;
    int last_batch = 0;  // batch of the last solve (diagnostic reads are bounded by it)
    std::vector<double *> bufs;
    GArrays A;
    GState *d_st = nullptr;
    int *d_active = nullptr;
    int *d_slots = nullptr;  // continuous batching: pidx (cap) | init (cap) | next (1)
    std::vector<void *> sbufs;  // per-horizon slot of the concurrent inertia tries (spec_of)
    std::vector<void *> spec_bufs;  // their storage rows, result codes, horizon list (gensure_spec)
    int spec_cap = 0;               // running horizons whose tries fit on the device at once (gensure_ws)
    // per-phase timing (HIP events on the solve stream around every launch group), mf_gproblem_timing:
    // slots k_geval, k_gasm, k_gpre, k_gkkt (with k_gspec / the occupancy variant), k_gls
    int timing = 0;
    unsigned long long *d_neval = nullptr;
    std::vector<hipEvent_t> ev;
    // the chain family's Newton step: k_gkkt_chain (main-problem horizons) on the solve stream and the generic k_gkkt
    // (restoration, least-square multipliers) on this side stream, concurrently (fork / join by events)
    hipStream_t side = nullptr;
    hipEvent_t ev_fork = nullptr, ev_join = nullptr;
    double t_ms[5] = {0, 0, 0, 0, 0};
    long t_launch[5] = {0, 0, 0, 0, 0};
};

template <class FAM> static void sizes_of(int N, std::vector<std::pair<double **, size_t>> &items, GArrays &A) {
    using D = typename FAM::D;
    const GSz<D> Z(N);
    items = {{&A.x, Z.x()},    {&A.u, Z.u()},    {&A.s, Z.i()},    {&A.lam, Z.l()},  {&A.ye, Z.e()},
             {&A.yi, Z.i()},   {&A.zxL, Z.x()},  {&A.zxU, Z.x()},  {&A.zuL, Z.u()},  {&A.zuU, Z.u()},
             {&A.vL, Z.i()},   {&A.vU, Z.i()},   {&A.dx, Z.x()},   {&A.du, Z.u()},   {&A.ds, Z.i()},
             {&A.dlam, Z.l()}, {&A.dye, Z.e()},  {&A.dyi, Z.i()},  {&A.dzxL, Z.x()}, {&A.dzxU, Z.x()},
             {&A.dzuL, Z.u()}, {&A.dzuU, Z.u()}, {&A.dvL, Z.i()},  {&A.dvU, Z.i()},  {&A.bk, Z.bk()},
             {&A.rec, Z.rec()}, {&A.Sx, Z.x()},  {&A.gx, Z.x()},   {&A.Su, Z.u()},   {&A.gu, Z.u()},
             {&A.Ss, Z.i()},   {&A.gs, Z.i()},   {&A.rdyn, Z.l()}, {&A.rin, Z.i()},  {&A.req, Z.e()},
             {&A.trdyn, Z.l()}, {&A.trin, Z.i()}, {&A.treq, Z.e()}, {&A.sdyn, Z.l()}, {&A.sin_, Z.i()},
             {&A.seq, Z.e()},  {&A.tx, Z.x()},   {&A.tu, Z.u()},   {&A.ts, Z.i()},   {&A.P, Z.P()},
             {&A.Kinv, Z.Kinv()}, {&A.Kfb, Z.Kfb()}, {&A.pv, Z.l()}, {&A.kv, Z.kv()}, {&A.x0, (size_t)D::NX},
             {&A.lref, (size_t)FAM::LREF}, {&A.scr, (size_t)N * scr_words<FAM>()},
             {&A.fil, (size_t)4 * GFCAP}, {&A.wdit, Z.bk()}, {&A.wddir, Z.bk()},
             {&A.pr, Z.nr()}, {&A.nr, Z.nr()}, {&A.zp, Z.nr()}, {&A.zn, Z.nr()}, {&A.dpr, Z.nr()},
             {&A.dnr, Z.nr()}, {&A.dzp, Z.nr()}, {&A.dzn, Z.nr()}, {&A.tpr, Z.nr()}, {&A.tnr, Z.nr()},
             {&A.Sp, Z.nr()}, {&A.Sn, Z.nr()}, {&A.gp, Z.nr()}, {&A.gn, Z.nr()}, {&A.rowr, Z.nr()},
             {&A.wR, Z.wv()}, {&A.dR, Z.wv()}, {&A.LUg, Z.lu()}, {&A.Jtg, Z.jt()}};
}

static void gfree_ws(mf_gproblem *p) {
    for (double *b : p->bufs) (void)hipFree(b);
    p->bufs.clear();
    for (void *b : p->sbufs) (void)hipFree(b);
    p->sbufs.clear();
    for (void *b : p->spec_bufs) (void)hipFree(b);
    p->spec_bufs.clear();
    p->A.spec_max = 0;
    if (p->d_st) (void)hipFree(p->d_st);
    if (p->d_active) (void)hipFree(p->d_active);
    if (p->d_slots) (void)hipFree(p->d_slots);
    p->d_st = nullptr;
    p->d_active = nullptr;
    p->d_slots = nullptr;
    p->cap = 0;
}

// the workspace is zeroed on the solve's stream s (ordering as capi.hip ensure_ws)
template <class FAM> static int gensure_ws(mf_gproblem *p, int batch, hipStream_t s) {
    if (p->cap >= batch) return MF_OK;
    gfree_ws(p);
    std::vector<std::pair<double **, size_t>> items;
    GArrays &A = p->A;
    sizes_of<FAM>(p->spec.N, items, A);
    for (auto &it : items) {
        double *ptr = nullptr;
        hipError_t he = hipMalloc(&ptr, it.second * (size_t)batch * sizeof(double));
        if (he != hipSuccess) {
            gfree_ws(p);
            return capi_fail(MF_ERR_NOMEM, std::string("workspace allocation failed: ") + hipGetErrorString(he));
        }
        p->bufs.push_back(ptr);
        *it.first = ptr;
        GHIPCHK(hipMemsetAsync(ptr, 0, it.second * (size_t)batch * sizeof(double), s));
    }
    GHIPCHK(hipMalloc(&p->d_st, sizeof(GState) * (size_t)batch));
    GHIPCHK(hipMalloc(&p->d_active, sizeof(int)));
    GHIPCHK(hipMalloc(&p->d_slots, sizeof(int) * (2 * (size_t)batch + 1)));
    {  // concurrent inertia tries (k_gspec): the running count whose GNSPEC tries all fit on the device at once; the
       // factor-storage rows themselves are made on demand by gensure_spec (IPOPT mode with the tries on only)
        hipFuncAttributes fa{};
        int dev = 0, ncu = 0, lds_cu = 0;
        GHIPCHK(hipFuncGetAttributes(&fa, reinterpret_cast<const void *>(k_gspec<FAM>)));
        GHIPCHK(hipGetDevice(&dev));
        GHIPCHK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev));
        GHIPCHK(hipDeviceGetAttribute(&lds_cu, hipDeviceAttributeMaxSharedMemoryPerMultiprocessor, dev));
        // k_gspec waves resident per CU: LDS, and the architectural VGPRs (512 per SIMD lane; a kernel that also
        // uses accumulation registers is LDS-limited below that anyway)
        const int w_lds = fa.sharedSizeBytes > 0 ? lds_cu / (int)fa.sharedSizeBytes : 32;
        const int w_reg = 4 * (512 / std::max(8, (fa.numRegs + 7) / 8 * 8));
        p->spec_cap = std::min(GSPEC_MAX, std::max(GSPEC_MIN, ncu * std::min(w_lds, w_reg) / GNSPEC));
        A.spec_max = 0;
        A.Psp = A.Ksp = A.Fsp = A.LUsp = A.Jtsp = A.sdw = A.sdc = nullptr;
        A.sres = A.slist = nullptr;
        void *ptr = nullptr;
        hipError_t he = hipMalloc(&ptr, (size_t)batch * 4);
        if (he != hipSuccess) {
            gfree_ws(p);
            return capi_fail(MF_ERR_NOMEM, std::string("workspace allocation failed: ") + hipGetErrorString(he));
        }
        p->sbufs.push_back(ptr);
        A.spec_of = static_cast<int *>(ptr);
    }
    A.st = p->d_st;
    A.active = p->d_active;
    A.u_lo = p->d_ulo;
    A.u_hi = p->d_uhi;
    A.c_lo = p->d_clo;
    A.c_hi = p->d_chi;
    p->cap = batch;
    return MF_OK;
}

// the factor-storage rows of the concurrent inertia tries for `rows` running horizons (GNSPEC tries each; made on
// the first IPOPT-mode solve that uses them, never for merit mode or inertia_spec < 0; kept with the workspace)
template <class FAM> static int gensure_spec(mf_gproblem *p, int rows) {
    using D = typename FAM::D;
    GArrays &A = p->A;
    if (A.spec_max >= rows) return MF_OK;
    for (void *b : p->spec_bufs) (void)hipFree(b);
    p->spec_bufs.clear();
    A.spec_max = 0;
    const GSz<D> Z(p->spec.N);
    const size_t R = (size_t)GNSPEC * rows;
    std::pair<void **, size_t> sp[] = {{(void **)&A.Psp, R * Z.P() * 8},   {(void **)&A.Ksp, R * Z.Kinv() * 8},
                                       {(void **)&A.Fsp, R * Z.Kfb() * 8}, {(void **)&A.LUsp, R * Z.lu() * 8},
                                       {(void **)&A.Jtsp, R * Z.jt() * 8}, {(void **)&A.sdw, R * 8},
                                       {(void **)&A.sdc, R * 8},           {(void **)&A.sres, R * 4},
                                       {(void **)&A.slist, (size_t)rows * 4}};
    for (auto &it : sp) {
        void *ptr = nullptr;
        hipError_t he = hipMalloc(&ptr, it.second);
        if (he != hipSuccess) {
            for (void *b : p->spec_bufs) (void)hipFree(b);
            p->spec_bufs.clear();
            return capi_fail(MF_ERR_NOMEM, std::string("workspace allocation failed: ") + hipGetErrorString(he));
        }
        p->spec_bufs.push_back(ptr);
        *it.first = ptr;
    }
    A.spec_max = rows;
    return MF_OK;
}

template <class FAM>
static int gsolve_core(mf_gproblem *p, int batch, const double *d_x0, const double *d_u0, const double *d_w0,
                       const double *d_lref, const mf_gopts *o, double *d_w, int *d_status, int *d_iters,
                       double *d_kkt, double *d_obj, hipStream_t s, int total = 0) {
    using D = typename FAM::D;
    // total > batch: continuous batching -- `batch` slots work through `total` problems (input and output
    // arrays have `total` rows); a slot whose problem finished takes the next one (k_gharvest)
    const bool stream_mode = total > batch;
    if (!stream_mode) total = batch;
    int e = gensure_ws<FAM>(p, batch, s);
    if (e) return e;
    GParams P = p->P;
    P.tol = o ? o->tol : 1e-8;
    P.constr_viol_tol = o ? o->constr_viol_tol : 1e-8;
    P.max_iter = o ? o->max_iter : 300;
    P.mu_init = o ? o->mu_init : 0.1;
    P.init_zero = o ? o->init_zero : 0;
    P.F_init = o ? o->F_init : 0.0;
    P.max_soc = o ? o->max_soc : 4;
    P.warm_start = (o && d_w0) ? o->warm_start : 0;
    P.filter = o ? o->filter : 0;
    P.dbg = (o && o->verbose >= 2) ? 1 : 0;
    P.resto_hard_dyn = o ? o->resto_hard_dyn : 0;
    p->last_batch = batch;
    // IPOPT bound_relax_factor: every finite bound of a non-fixed variable or row moves out by
    // br max(1, |b|) (oracle/mf_ocp.c, same rule); fixed controls (lo == hi) stay parameters
    const double br = o ? o->bound_relax : 0.0;
    const double *ulo = p->d_ulo, *uhi = p->d_uhi, *clo = p->d_clo, *chi = p->d_chi;
    if (br != 0.0) {
        auto lo_r = [&](double v) { return std::isfinite(v) ? v - br * fmax(1.0, fabs(v)) : v; };
        auto hi_r = [&](double v) { return std::isfinite(v) ? v + br * fmax(1.0, fabs(v)) : v; };
        for (int j = 0; j < D::NX; j++) { P.x_lo[j] = lo_r(P.x_lo[j]); P.x_hi[j] = hi_r(P.x_hi[j]); }
        if (br != p->relax || !p->d_ulo_r) {
            std::vector<double> a(p->ulo), bb(p->uhi), c(p->clo), d(p->chi);
            for (size_t i = 0; i < a.size(); i++)
                if (!(std::isfinite(a[i]) && a[i] == bb[i])) { a[i] = lo_r(a[i]); bb[i] = hi_r(bb[i]); }
            for (size_t i = 0; i < c.size(); i++) { c[i] = lo_r(c[i]); d[i] = hi_r(d[i]); }
            double **dst[4] = {&p->d_ulo_r, &p->d_uhi_r, &p->d_clo_r, &p->d_chi_r};
            const std::vector<double> *srcv[4] = {&a, &bb, &c, &d};
            for (int t = 0; t < 4; t++) {
                if (!*dst[t]) GHIPCHK(hipMalloc(dst[t], srcv[t]->size() * sizeof(double)));
                GHIPCHK(hipMemcpyAsync(*dst[t], srcv[t]->data(), srcv[t]->size() * sizeof(double), hipMemcpyHostToDevice, s));
            }
            GHIPCHK(hipStreamSynchronize(s));
            p->relax = br;
        }
        ulo = p->d_ulo_r; uhi = p->d_uhi_r; clo = p->d_clo_r; chi = p->d_chi_r;
    }
    P.has_u_init = (o && o->u_init) ? 1 : 0;
    if (P.has_u_init)
        for (int j = 0; j < D::NU; j++) P.u_init[j] = o->u_init[j];
    GArrays A = p->A;
    A.u0 = d_u0;
    A.w0 = d_w0;
    A.u_lo = ulo; A.u_hi = uhi; A.c_lo = clo; A.c_hi = chi;
    A.pidx = A.next = A.init = nullptr;
    A.total = total;
    A.neval = nullptr;
    A.fast_kkt = 0;
    if (p->timing) {
        if (!p->d_neval) {
            GHIPCHK(hipMalloc(&p->d_neval, sizeof(unsigned long long)));
            GHIPCHK(hipMemsetAsync(p->d_neval, 0, sizeof(unsigned long long), s));
        }
        A.neval = p->d_neval;
    }
    A.x0all = d_x0;
    A.lrall = FAM::LREF == 2 ? d_lref : nullptr;
    A.ow = d_w; A.okkt = d_kkt; A.oobj = d_obj; A.ost = d_status; A.oit = d_iters;
    if (stream_mode) {
        std::vector<int> h(2 * (size_t)batch + 1, 0);
        for (int b = 0; b < batch; b++) h[b] = b;  // slot b starts on problem b
        h[2 * (size_t)batch] = batch;               // the next problem to hand out
        GHIPCHK(hipMemcpyAsync(p->d_slots, h.data(), sizeof(int) * h.size(), hipMemcpyHostToDevice, s));
        GHIPCHK(hipStreamSynchronize(s));
        A.pidx = p->d_slots;
        A.init = p->d_slots + batch;
        A.next = p->d_slots + 2 * batch;
        hipLaunchKernelGGL(k_gout_init, dim3((total + 255) / 256), dim3(256), 0, s, total, d_status, d_iters, d_kkt, d_obj);
        GHIPCHK(hipGetLastError());
    }
    GHIPCHK(hipMemcpyAsync(A.x0, d_x0, sizeof(double) * D::NX * (size_t)batch, hipMemcpyDeviceToDevice, s));
    if (FAM::LREF != 2) {
        // per-problem data computed by k_ginit from x_0
    } else if (d_lref) {
        GHIPCHK(hipMemcpyAsync(A.lref, d_lref, sizeof(double) * 2 * (size_t)batch, hipMemcpyDeviceToDevice, s));
    } else {
        std::vector<double> lr(2 * (size_t)batch);
        for (int b = 0; b < batch; b++) { lr[2 * b] = p->spec.line_ref[0]; lr[2 * b + 1] = p->spec.line_ref[1]; }
        GHIPCHK(hipMemcpyAsync(A.lref, lr.data(), sizeof(double) * lr.size(), hipMemcpyHostToDevice, s));
        GHIPCHK(hipStreamSynchronize(s));
    }
    GHIPCHK(hipMemcpyAsync(A.active, &batch, sizeof(int), hipMemcpyHostToDevice, s));
    GHIPCHK(hipStreamSynchronize(s));
    const DevModel *M0 = p->dM0, *M1 = p->dM1 ? p->dM1 : p->dM0;
    const DevFrame *F0 = p->dF0, *F1 = p->dF1 ? p->dF1 : p->dF0;
    {
        GArrays A0 = A;
        A0.init = nullptr;  // the first launch initialises every slot
        hipLaunchKernelGGL(k_ginit<FAM>, dim3(batch), dim3(64), 0, s, M0, M1, F0, F1, P, A0, batch);
    }
    GHIPCHK(hipGetLastError());
    constexpr int NPB = 256 / FAM::LANES;
    const int eval_blocks = (int)(((long)batch * P.N + NPB - 1) / NPB);
    const int rec_blocks = (int)(((long)batch * P.N + 3) / 4);
    int active = batch;
    const int chunk = 4;
    // every running horizon ends at the latest when its own iteration count reaches max_iter; in IPOPT mode
    // some launches advance no iteration (the restoration phase's start and end), so the host bound is on
    // launches, with room for those, not on iterations
    // (IPOPT mode: a soft step undone, the restoration's start and one of its iterations take up to 5 launch rounds
    // for 2 iterations)
    const long max_launches = (3L * P.max_iter + 64) * (stream_mode ? (total + batch - 1) / batch + 1 : 1);
    // concurrent inertia tries while few horizons run (IPOPT mode; mf_gopts.inertia_spec < 0: never)
    const bool spec_ok = P.filter && !(o && o->inertia_spec < 0);
    if (spec_ok) {
        if ((e = gensure_spec<FAM>(p, std::min(p->spec_cap, batch)))) return e;
        A.Psp = p->A.Psp; A.Ksp = p->A.Ksp; A.Fsp = p->A.Fsp; A.LUsp = p->A.LUsp; A.Jtsp = p->A.Jtsp;
        A.sdw = p->A.sdw; A.sdc = p->A.sdc; A.sres = p->A.sres; A.slist = p->A.slist;
        A.spec_max = std::min(p->spec_cap, batch);
    } else {
        A.spec_max = 0;
    }
    if (o && o->verbose && spec_ok) fprintf(stderr, "[mf gipm] concurrent inertia tries from %d running horizons\n", A.spec_max);
    GArrays As = A;  // k_gkkt's view: spec_of set while k_gspec runs
    // the chain family's main-problem Newton step by k_gkkt_chain (IPOPT mode, not while k_gspec runs);
    // MF_CHAIN_KKT=0 in the environment keeps k_gkkt for every horizon (A/B diagnostics)
    bool chain_kkt = false, chain_rspec = false;
    if constexpr (ChainEuler<FAM>::value) {
        const char *ev = getenv("MF_CHAIN_KKT");
        chain_kkt = P.filter && P.N <= GCHAIN_NMAX && !(ev && ev[0] == '0');
        const char *er = getenv("MF_CHAIN_RSPEC");
        // (MF_CHAIN_RSPEC=1: the left-over horizons' inertia tries concurrently as well; measured no faster, DESIGN s.9)
        chain_rspec = chain_kkt && spec_ok && A.spec_max > 0 && (er && er[0] == '1');
        if (chain_kkt && !p->side) {
            GHIPCHK(hipStreamCreateWithFlags(&p->side, hipStreamNonBlocking));
            GHIPCHK(hipEventCreateWithFlags(&p->ev_fork, hipEventDisableTiming));
            GHIPCHK(hipEventCreateWithFlags(&p->ev_join, hipEventDisableTiming));
        }
    }
    // the C2 chain's node evaluation direction-major (k_geval_chain; MF_CHAIN_EVAL=0: k_geval, the same lanes)
    bool chain_eval = false;
    int chain_blocks = 0;
    if constexpr (FAM::SPLIT) {
        const char *ev = getenv("MF_CHAIN_EVAL");
        chain_eval = !(ev && ev[0] == '0');
        const long groups = ((long)batch * P.N + 63) / 64;
        chain_blocks = (int)(8 * FAM::NJ * ((groups + 7) / 8));
    }
    // the occupancy variants while more horizons run than the default kernels hold (four per CU; measured on the C2
    // leg: launches at ~1000 running horizons take the same time with either k_gkkt, fewer run faster without spills)
    int kkt_occ_from = batch;
    // MF_GLS_OCC=0 in the environment keeps the default k_gls at every running count (A/B diagnostics)
    const char *egl = getenv("MF_GLS_OCC");
    const bool gls_occ_on = !(egl && egl[0] == '0');
    // MF_GKKT_OCC=0: the default k_gkkt at every running count
    const char *egk = getenv("MF_GKKT_OCC");
    const bool gkkt_occ_on = !(egk && egk[0] == '0');
    if constexpr (GOcc<FAM>::KKT > 1) {
        int dev = 0, ncu = 0;
        GHIPCHK(hipGetDevice(&dev));
        GHIPCHK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev));
        kkt_occ_from = 4 * ncu;
        if (o && o->verbose) fprintf(stderr, "[mf gipm] k_gkkt occupancy variant above %d running horizons\n", kkt_occ_from);
    }
    const auto t_start = std::chrono::steady_clock::now();
    constexpr int NPH = 5;
    if (p->timing && p->ev.size() < (size_t)(2 * NPH * chunk)) {
        for (auto e2 : p->ev) (void)hipEventDestroy(e2);
        p->ev.assign(2 * NPH * chunk, nullptr);
        for (auto &e2 : p->ev) GHIPCHK(hipEventCreate(&e2));
    }
    auto mark = [&](int c, int ph, int end) {
        if (p->timing) (void)hipEventRecord(p->ev[(c * NPH + ph) * 2 + end], s);
    };
    for (long it = 0; it < max_launches && active > 0; it += chunk) {
        const bool spec = spec_ok && active <= A.spec_max;
        As.spec_of = spec ? A.spec_of : nullptr;
        for (int c = 0; c < chunk; c++) {
            mark(c, 0, 0);
            if constexpr (FAM::SPLIT) {
                if (chain_eval) {
                    static_assert(std::is_same<FAM, ChainC2>::value, "the split evaluation is the C2 chain's");
                    gchain_eval(s, chain_blocks, M0, F0, P, A, batch);
                } else {
                    hipLaunchKernelGGL(k_geval<FAM>, dim3(eval_blocks), dim3(256), 0, s, M0, M1, F0, F1, P, A, batch);
                }
            } else {
                hipLaunchKernelGGL(k_geval<FAM>, dim3(eval_blocks), dim3(256), 0, s, M0, M1, F0, F1, P, A, batch);
            }
            mark(c, 0, 1);
            mark(c, 1, 0);
            hipLaunchKernelGGL(k_gasm<FAM>, dim3(rec_blocks), dim3(256), 0, s, P, A, batch);
            mark(c, 1, 1);
            mark(c, 2, 0);
            hipLaunchKernelGGL(k_gpre<FAM>, dim3(batch), dim3(64), 0, s, M0, M1, F0, F1, P, A, batch);
            mark(c, 2, 1);
            mark(c, 3, 0);
            As.fast_kkt = 0;
            hipStream_t ks = s;  // the generic k_gkkt's stream
            if constexpr (ChainEuler<FAM>::value) {
                if (chain_kkt && !spec) {
                    // fork: the two kernels take disjoint horizons (k_gkkt skips the ones k_gkkt_chain takes and only
                    // reads their state's mode / pend, which k_gkkt_chain does not write)
                    GHIPCHK(hipEventRecord(p->ev_fork, s));
                    GHIPCHK(hipStreamWaitEvent(p->side, p->ev_fork, 0));
                    gchain_kkt(s, P, A, batch);
                    As.fast_kkt = 1;
                    ks = p->side;
                    if (chain_rspec) {
                        // the left-over horizons' inertia tries concurrently as well (k_gspec on the side stream)
                        hipLaunchKernelGGL(k_gspec_list, dim3(1), dim3(1024), 0, ks, A, batch, 1);
                        hipLaunchKernelGGL(k_gspec<FAM>, dim3(GNSPEC * A.spec_max), dim3(64), 0, ks, M0, M1, F0, F1, P,
                                           A, batch);
                        As.spec_of = A.spec_of;
                    }
                }
            }
            if (spec) {
                hipLaunchKernelGGL(k_gspec_list, dim3(1), dim3(1024), 0, s, A, batch, 0);
                hipLaunchKernelGGL(k_gspec<FAM>, dim3(GNSPEC * std::min(active, A.spec_max)), dim3(64), 0, s, M0, M1, F0,
                                   F1, P, A, batch);
            }
            bool occ = false;
            if constexpr (GOcc<FAM>::KKT > 1) {
                occ = gkkt_occ_on && active > kkt_occ_from;
                if (occ)
                    hipLaunchKernelGGL((k_gkkt_occ<FAM, GOcc<FAM>::KKT>), dim3(batch), dim3(64), 0, ks, M0, M1, F0, F1, P,
                                       As, batch);
            }
            if (!occ) hipLaunchKernelGGL(k_gkkt<FAM>, dim3(batch), dim3(64), 0, ks, M0, M1, F0, F1, P, As, batch);
            if (ks != s) {  // join
                GHIPCHK(hipEventRecord(p->ev_join, ks));
                GHIPCHK(hipStreamWaitEvent(s, p->ev_join, 0));
            }
            mark(c, 3, 1);
            mark(c, 4, 0);
            bool occ_ls = false;
            if constexpr (GOcc<FAM>::LS > 1) {
                occ_ls = gls_occ_on && active > kkt_occ_from;
                if (occ_ls && P.filter)
                    hipLaunchKernelGGL((k_gls_occ<FAM, true, GOcc<FAM>::LS>), dim3(batch), dim3(64), 0, s, M0, M1, F0, F1,
                                       P, A, batch);
                else if (occ_ls)
                    hipLaunchKernelGGL((k_gls_occ<FAM, false, GOcc<FAM>::LS>), dim3(batch), dim3(64), 0, s, M0, M1, F0,
                                       F1, P, A, batch);
            }
            if (!occ_ls && P.filter)
                hipLaunchKernelGGL((k_gls<FAM, true>), dim3(batch), dim3(64), 0, s, M0, M1, F0, F1, P, A, batch);
            else if (!occ_ls)
                hipLaunchKernelGGL((k_gls<FAM, false>), dim3(batch), dim3(64), 0, s, M0, M1, F0, F1, P, A, batch);
            mark(c, 4, 1);
        }
        GHIPCHK(hipGetLastError());
        GHIPCHK(hipMemcpyAsync(&active, A.active, sizeof(int), hipMemcpyDeviceToHost, s));
        GHIPCHK(hipStreamSynchronize(s));
        if (p->timing)
            for (int c = 0; c < chunk; c++)
                for (int ph = 0; ph < NPH; ph++) {
                    float ms = 0.f;
                    GHIPCHK(hipEventElapsedTime(&ms, p->ev[(c * NPH + ph) * 2], p->ev[(c * NPH + ph) * 2 + 1]));
                    p->t_ms[ph] += ms;
                    p->t_launch[ph]++;
                }
        if (stream_mode && active < batch) {  // finished slots: outputs written, next problems handed out
            hipLaunchKernelGGL(k_gharvest<FAM>, dim3(batch), dim3(64), 0, s, A, P.N, batch, 0);
            hipLaunchKernelGGL(k_ginit<FAM>, dim3(batch), dim3(64), 0, s, M0, M1, F0, F1, P, A, batch);
            GHIPCHK(hipGetLastError());
            GHIPCHK(hipMemcpyAsync(&active, A.active, sizeof(int), hipMemcpyDeviceToHost, s));
            GHIPCHK(hipStreamSynchronize(s));
        }
        if (o && o->verbose)
            fprintf(stderr, "[mf gipm] after %ld launches: %d running, %.3f ms\n", it + chunk, active,
                    std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t_start).count());
    }
    if (stream_mode) {  // launch bound reached with slots still running: written out as max_iter
        hipLaunchKernelGGL(k_gharvest<FAM>, dim3(batch), dim3(64), 0, s, A, P.N, batch, 1);
    } else {
        hipLaunchKernelGGL(k_gout<D>, dim3(batch), dim3(256), 0, s, A, P.N, batch, d_w, d_status, d_iters, d_kkt,
                           d_obj);
    }
    GHIPCHK(hipGetLastError());
    return MF_OK;
}

static int gdispatch_solve(mf_gproblem *p, int batch, const double *x0, const double *u0, const double *w0,
                           const double *lref, const mf_gopts *o, double *w, int *st, int *it, double *kkt,
                           double *obj, hipStream_t s, int total = 0) {
    switch (p->kind) {
        case GK_BOX: return gsolve_core<FamBox>(p, batch, x0, u0, w0, lref, o, w, st, it, kkt, obj, s, total);
        case GK_CH6F: return gsolve_core<FamCh6F>(p, batch, x0, u0, w0, lref, o, w, st, it, kkt, obj, s, total);
        case GK_CH6FT: return gsolve_core<FamCh6FT>(p, batch, x0, u0, w0, lref, o, w, st, it, kkt, obj, s, total);
        case GK_CH3: return gsolve_core<FamCh3>(p, batch, x0, u0, w0, lref, o, w, st, it, kkt, obj, s, total);
        case GK_CH3T: return gsolve_core<FamCh3T>(p, batch, x0, u0, w0, lref, o, w, st, it, kkt, obj, s, total);
        case GK_CENT: return gsolve_core<FamCent>(p, batch, x0, u0, w0, lref, o, w, st, it, kkt, obj, s, total);
        case GK_BOXT: return gsolve_core<FamBoxT>(p, batch, x0, u0, w0, lref, o, w, st, it, kkt, obj, s, total);
    }
    return capi_fail(MF_ERR_UNSUPPORTED, "no kernel instantiation");
}

template <class FAM> static void dims_of(int &nx, int &nu, int &ni, int &ne) {
    nx = FAM::D::NX; nu = FAM::D::NU; ni = FAM::D::NI; ne = FAM::D::NE;
}

// mf_gopts with the library's defaults (include/mpcfatigue.h): callers fill this and change what they need, so a
// field added in a later version starts at its default instead of at whatever a shorter struct leaves behind
extern "C" int mf_gopts_init(mf_gopts *o) {
    if (!o) return capi_fail(MF_ERR_ARG, "null argument");
    memset(o, 0, sizeof *o);
    o->tol = 1e-8;
    o->constr_viol_tol = 1e-8;
    o->max_iter = 3000;
    o->mu_init = 0.1;
    o->max_soc = 4;
    return (int)sizeof *o;
}

extern "C" int mf_gproblem_create(const mf_model *m0c, const mf_model *m1c, const mf_gspec *spec, mf_gproblem **out) {
    mf_model *m0 = const_cast<mf_model *>(m0c), *m1 = const_cast<mf_model *>(m1c);
    if (!m0 || !spec || !out) return capi_fail(MF_ERR_ARG, "null argument");
    if (spec->N < 1 || spec->h <= 0) return capi_fail(MF_ERR_ARG, "N >= 1 and h > 0 required");
    if (!spec->u_lo || !spec->u_hi || !spec->c_lo || !spec->c_hi) return capi_fail(MF_ERR_ARG, "bounds required");
    int e = capi_ensure_device();
    if (e) return e;
    const DevModel *dM0 = nullptr, *dM1 = nullptr;
    const Model *h0 = nullptr, *h1 = nullptr;
    if ((e = capi_model_dev(m0, &dM0, &h0))) return e;
    int kind = -1;
    const int n0 = (int)h0->joints.size();
    if (spec->family == MF_FAM_BOX) {
        if (!m1) return capi_fail(MF_ERR_ARG, "the box family needs two models");
        if ((e = capi_model_dev(m1, &dM1, &h1))) return e;
        if (n0 != 6 || (int)h1->joints.size() != 6) return capi_fail(MF_ERR_UNSUPPORTED, "box family: two 6-joint arms");
        kind = spec->thermal ? GK_BOXT : GK_BOX;
    } else if (spec->family == MF_FAM_CENTAURO) {
        if (!m1) return capi_fail(MF_ERR_ARG, "the Centauro family needs two models");
        if ((e = capi_model_dev(m1, &dM1, &h1))) return e;
        if (n0 != 7 || (int)h1->joints.size() != 7)
            return capi_fail(MF_ERR_UNSUPPORTED, "Centauro family: two 7-joint arms");
        kind = GK_CENT;
    } else if (spec->family == MF_FAM_CHAIN) {
        const int ne = spec->use_line ? 2 : 0;
        if (n0 == 6 && spec->nf == 1 && ne == 2) kind = spec->thermal ? GK_CH6FT : GK_CH6F;
        else if (n0 == 3 && spec->nf == 0 && ne == 0) kind = spec->thermal ? GK_CH3T : GK_CH3;
        else
            return capi_fail(MF_ERR_UNSUPPORTED, "no chain instantiation for (n, nf, line) = (" + std::to_string(n0) +
                                                     ", " + std::to_string(spec->nf) + ", " + std::to_string(ne) + ")");
    } else {
        return capi_fail(MF_ERR_ARG, "unknown family");
    }
    for (const Model *h : {h0, h1}) {
        if (!h) continue;
        for (size_t i = 0; i < h->joints.size(); i++)
            if (h->joints[i].parent != (int)i - 1) return capi_fail(MF_ERR_UNSUPPORTED, "serial chains only");
    }
    mf_gproblem *p = new mf_gproblem();
    p->m0 = m0;
    p->m1 = m1;
    p->spec = *spec;
    p->kind = kind;
    p->dM0 = dM0;
    p->dM1 = dM1;
    switch (kind) {
        case GK_BOX: dims_of<FamBox>(p->nx, p->nu, p->ni, p->ne); break;
        case GK_CH6F: dims_of<FamCh6F>(p->nx, p->nu, p->ni, p->ne); break;
        case GK_CH6FT: dims_of<FamCh6FT>(p->nx, p->nu, p->ni, p->ne); break;
        case GK_CH3: dims_of<FamCh3>(p->nx, p->nu, p->ni, p->ne); break;
        case GK_CH3T: dims_of<FamCh3T>(p->nx, p->nu, p->ni, p->ne); break;
        case GK_CENT: dims_of<FamCent>(p->nx, p->nu, p->ni, p->ne); break;
        case GK_BOXT: dims_of<FamBoxT>(p->nx, p->nu, p->ni, p->ne); break;
    }
    const int N = spec->N;
    int rc = capi_frame_dev(m0, spec->frame0, &p->dF0);
    if (!rc && m1) rc = capi_frame_dev(m1, spec->frame1, &p->dF1);
    if (rc) { delete p; return rc; }
    p->ulo.assign(spec->u_lo, spec->u_lo + (size_t)N * p->nu);
    p->uhi.assign(spec->u_hi, spec->u_hi + (size_t)N * p->nu);
    p->clo.assign(spec->c_lo, spec->c_lo + (size_t)N * p->ni);
    p->chi.assign(spec->c_hi, spec->c_hi + (size_t)N * p->ni);
    p->spec.u_lo = p->ulo.data(); p->spec.u_hi = p->uhi.data();
    p->spec.c_lo = p->clo.data(); p->spec.c_hi = p->chi.data();
    GParams &P = p->P;
    memset(&P, 0, sizeof P);
    P.N = N; P.h = spec->h; P.eq_from = spec->eq_from;
    P.nf = spec->nf; P.use_line = spec->use_line; P.thermal = spec->thermal;
    memcpy(P.fdir, spec->fdir, sizeof P.fdir);
    P.wF = spec->wF; P.wqd = spec->wqd; P.wtau = spec->wtau; P.wT = spec->wT;
    P.th_a = spec->th_a; P.th_b = spec->th_b; P.Ra = spec->Ra; P.Rh = spec->Rh;
    memcpy(P.ktau, spec->ktau, sizeof P.ktau);
    P.box_mg = spec->box_mg; P.box_L = spec->box_L; memcpy(P.box_pdes, spec->box_pdes, sizeof P.box_pdes);
    P.w_box = spec->w_box; P.w_qdb = spec->w_qd;
    memcpy(P.x_lo, spec->x_lo, sizeof P.x_lo);
    memcpy(P.x_hi, spec->x_hi, sizeof P.x_hi);
    P.target_decimals = spec->target_decimals;
    if (kind == GK_BOX || kind == GK_BOXT) { P.force_from = 12; P.tier1_from = P.tier1_to = 0; }
    else if (kind == GK_CENT) {
        // the moment rows at the fixed node 0 have rank 2 in F: IPOPT sees a singular KKT every
        // iteration and perturbs it with delta_c; the solver does so from the first factorisation
        P.force_from = 14; P.tier1_from = P.tier1_to = 0; P.dc_always = 1;
        P.w_qdb = spec->w_qd;
    } else {
        P.force_from = n0;
        const bool concave = spec->nf > 0 && spec->wF < 0;
        P.tier1_from = concave ? n0 : 0;
        P.tier1_to = concave ? n0 + spec->nf : 0;
    }
    auto up = [&](double **d, const std::vector<double> &h) -> int {
        GHIPCHK(hipMalloc(d, h.size() * sizeof(double)));
        GHIPCHK(hipMemcpy(*d, h.data(), h.size() * sizeof(double), hipMemcpyHostToDevice));
        return MF_OK;
    };
    if ((rc = up(&p->d_ulo, p->ulo)) || (rc = up(&p->d_uhi, p->uhi)) || (rc = up(&p->d_clo, p->clo)) ||
        (rc = up(&p->d_chi, p->chi))) {
        delete p;
        return rc;
    }
    *out = p;
    return MF_OK;
}

extern "C" void mf_gproblem_free(mf_gproblem *p) {
    if (!p) return;
    gfree_ws(p);
    for (auto e : p->ev) (void)hipEventDestroy(e);
    if (p->ev_fork) (void)hipEventDestroy(p->ev_fork);
    if (p->ev_join) (void)hipEventDestroy(p->ev_join);
    if (p->side) (void)hipStreamDestroy(p->side);
    if (p->d_neval) (void)hipFree(p->d_neval);
    for (double *d : {p->d_ulo, p->d_uhi, p->d_clo, p->d_chi, p->d_ulo_r, p->d_uhi_r, p->d_clo_r, p->d_chi_r})
        if (d) (void)hipFree(d);
    delete p;
}

// per-phase timing of the generic solver's launches (HIP events on the solve stream; diagnostics and bench.py):
// enable resets the accumulators; stats: total ms and launch count per slot
// {k_geval, k_gasm, k_gpre, k_gkkt (+ k_gspec, occupancy variant), k_gls}
extern "C" int mf_gproblem_timing(mf_gproblem *p, int enable) {
    if (!p) return capi_fail(MF_ERR_ARG, "null argument");
    p->timing = enable ? 1 : 0;
    for (int k = 0; k < 5; k++) { p->t_ms[k] = 0; p->t_launch[k] = 0; }
    if (p->d_neval) GHIPCHK(hipMemset(p->d_neval, 0, sizeof(unsigned long long)));
    return MF_OK;
}
extern "C" int mf_gproblem_kernel_stats(mf_gproblem *p, double *ms5, long *launches5, long long *node_evals) {
    if (!p || !ms5 || !launches5) return capi_fail(MF_ERR_ARG, "null argument");
    for (int k = 0; k < 5; k++) { ms5[k] = p->t_ms[k]; launches5[k] = p->t_launch[k]; }
    if (node_evals) {
        unsigned long long v = 0;
        if (p->d_neval) {
            GHIPCHK(hipDeviceSynchronize());
            GHIPCHK(hipMemcpy(&v, p->d_neval, sizeof v, hipMemcpyDeviceToHost));
        }
        *node_evals = (long long)v;
    }
    return MF_OK;
}

extern "C" int mf_gproblem_dims(const mf_gproblem *p, int *dims5) {
    if (!p || !dims5) return capi_fail(MF_ERR_ARG, "null argument");
    dims5[0] = p->nx; dims5[1] = p->nu; dims5[2] = p->ni; dims5[3] = p->ne;
    dims5[4] = p->nx + p->spec.N * (p->nu + p->nx);
    return MF_OK;
}

extern "C" int mf_gsolve_batch_dev(mf_gproblem *p, int batch, const double *x0, const double *u0, const double *w0,
                                   const double *line_ref, const mf_gopts *opts, double *w, int *status, int *iters,
                                   double *kkt, double *obj, void *stream) {
    if (!p || !x0 || !w || batch < 1) return capi_fail(MF_ERR_ARG, "bad argument");
    int e = capi_ensure_device();
    if (e) return e;
    return gdispatch_solve(p, batch, x0, u0, w0, line_ref, opts, w, status, iters, kkt, obj, (hipStream_t)stream);
}

// continuous batching (device memory): `slots` concurrent solves work through `total` problems; the inputs
// (x0, u0, w0, line_ref) and outputs have `total` rows, results identical to mf_gsolve_batch_dev's
extern "C" int mf_gsolve_stream_dev(mf_gproblem *p, int total, int slots, const double *x0, const double *u0,
                                    const double *w0, const double *line_ref, const mf_gopts *opts, double *w,
                                    int *status, int *iters, double *kkt, double *obj, void *stream) {
    if (!p || !x0 || !w || total < 1 || slots < 1) return capi_fail(MF_ERR_ARG, "bad argument");
    int e = capi_ensure_device();
    if (e) return e;
    if (slots > total) slots = total;
    return gdispatch_solve(p, slots, x0, u0, w0, line_ref, opts, w, status, iters, kkt, obj, (hipStream_t)stream,
                           total);
}

namespace {
struct GBuf {
    double *p = nullptr;
    ~GBuf() { if (p) (void)hipFree(p); }
};
struct GIBuf {
    int *p = nullptr;
    ~GIBuf() { if (p) (void)hipFree(p); }
};
struct GOwnStream {
    hipStream_t s = nullptr;
    ~GOwnStream() { if (s) { (void)hipStreamSynchronize(s); (void)hipStreamDestroy(s); } }
};
int gh2d(GBuf &b, const double *h, size_t n, hipStream_t s = nullptr) {
    GHIPCHK(hipMalloc(&b.p, n * sizeof(double)));
    if (s) GHIPCHK(hipMemcpyAsync(b.p, h, n * sizeof(double), hipMemcpyHostToDevice, s));
    else GHIPCHK(hipMemcpy(b.p, h, n * sizeof(double), hipMemcpyHostToDevice));
    return MF_OK;
}
int galloc(GBuf &b, size_t n) {
    GHIPCHK(hipMalloc(&b.p, n * sizeof(double)));
    return MF_OK;
}
}  // namespace

extern "C" int mf_gsolve_batch(mf_gproblem *p, int batch, const double *x0, const double *u0, const double *w0,
                               const double *line_ref, const mf_gopts *opts, double *w, int *status, int *iters,
                               double *kkt, double *obj, int device) {
    if (!p || !x0 || !w || batch < 1) return capi_fail(MF_ERR_ARG, "bad argument");
    int e = capi_ensure_device();
    if (e) return e;
    GHIPCHK(hipSetDevice(device));
    const int ws = p->nx + p->spec.N * (p->nu + p->nx);
    GBuf dx0, du0, dw0, dl, dw, dk, dob;
    GIBuf dst, dit;
    // this call's own stream: uploads, solve and copies back are ordered on it, and synchronising it
    // leaves other handles / streams of the device running
    GOwnStream os;
    GHIPCHK(hipStreamCreateWithFlags(&os.s, hipStreamNonBlocking));
    if ((e = gh2d(dx0, x0, (size_t)p->nx * batch, os.s))) return e;
    if (u0 && (e = gh2d(du0, u0, (size_t)p->nu * batch, os.s))) return e;
    if (w0 && (e = gh2d(dw0, w0, (size_t)ws * batch, os.s))) return e;
    if (line_ref && (e = gh2d(dl, line_ref, 2 * (size_t)batch, os.s))) return e;
    if ((e = galloc(dw, (size_t)ws * batch)) || (e = galloc(dk, batch)) || (e = galloc(dob, batch))) return e;
    GHIPCHK(hipMalloc(&dst.p, sizeof(int) * batch));
    GHIPCHK(hipMalloc(&dit.p, sizeof(int) * batch));
    e = gdispatch_solve(p, batch, dx0.p, du0.p, dw0.p, line_ref ? dl.p : nullptr, opts, dw.p, dst.p, dit.p, dk.p,
                        dob.p, os.s);
    if (e) return e;
    GHIPCHK(hipMemcpyAsync(w, dw.p, sizeof(double) * ws * (size_t)batch, hipMemcpyDeviceToHost, os.s));
    if (status) GHIPCHK(hipMemcpyAsync(status, dst.p, sizeof(int) * batch, hipMemcpyDeviceToHost, os.s));
    if (iters) GHIPCHK(hipMemcpyAsync(iters, dit.p, sizeof(int) * batch, hipMemcpyDeviceToHost, os.s));
    if (kkt) GHIPCHK(hipMemcpyAsync(kkt, dk.p, sizeof(double) * batch, hipMemcpyDeviceToHost, os.s));
    if (obj) GHIPCHK(hipMemcpyAsync(obj, dob.p, sizeof(double) * batch, hipMemcpyDeviceToHost, os.s));
    GHIPCHK(hipStreamSynchronize(os.s));
    return MF_OK;
}

template <class FAM>
static int grec_core(mf_gproblem *p, const double *xu, const double *yi, const double *ye, const double *lam,
                     const double *lref, double *rec) {
    using D = typename FAM::D;
    GBuf a, b2, c, d, l, o;
    int e;
    if ((e = gh2d(a, xu, D::NV)) || (e = gh2d(b2, yi, D::NIA)) || (e = gh2d(l, lref, FAM::LREF)) ||
        (e = galloc(o, D::REC)))
        return e;
    // ye = [state rows (NE) | mixed rows (NM)] -> the device layout [NEA | NM]
    std::vector<double> yev(D::NET, 0.0);
    for (int i = 0; i < D::NE; i++) yev[i] = ye[i];
    for (int i = 0; i < D::NM; i++) yev[D::NEA + i] = ye[D::NE + i];
    if ((e = gh2d(c, yev.data(), D::NET)) || (e = gh2d(d, lam, D::NX))) return e;
    const DevModel *M1 = p->dM1 ? p->dM1 : p->dM0;
    const DevFrame *F1 = p->dF1 ? p->dF1 : p->dF0;
    hipLaunchKernelGGL(k_grec<FAM>, dim3(1), dim3(256), 0, 0, p->dM0, M1, p->dF0, F1, p->P, a.p, b2.p, c.p, d.p, l.p, o.p);
    GHIPCHK(hipGetLastError());
    GHIPCHK(hipStreamSynchronize(0));  // the launch's own (null) stream
    GHIPCHK(hipMemcpy(rec, o.p, sizeof(double) * D::REC, hipMemcpyDeviceToHost));
    return D::REC;
}

// diagnostics: dual state of problem b, [lam | yi | ye | zxL | zxU | zuL | zuU | vL | vU | mu]
template <class FAM> static int gdual_core(mf_gproblem *p, int b, double *out) {
    using D = typename FAM::D;
    const GSz<D> Z(p->spec.N);
    const GArrays &A = p->A;
    if (b < 0 || b >= p->last_batch) return capi_fail(MF_ERR_ARG, "problem index out of range (last solve's batch)");
    double *src[] = {A.lam, A.yi, A.ye, A.zxL, A.zxU, A.zuL, A.zuU, A.vL, A.vU};
    const size_t len[] = {Z.l(), Z.i(), Z.e(), Z.x(), Z.x(), Z.u(), Z.u(), Z.i(), Z.i()};
    size_t off = 0;
    // diagnostic read of the last solve, whichever stream it ran on: the whole device is synchronised
    GHIPCHK(hipDeviceSynchronize());
    for (int a = 0; a < 9; a++) {
        GHIPCHK(hipMemcpy(out + off, src[a] + (size_t)b * len[a], len[a] * sizeof(double), hipMemcpyDeviceToHost));
        off += len[a];
    }
    GState st;
    GHIPCHK(hipMemcpy(&st, A.st + b, sizeof st, hipMemcpyDeviceToHost));
    out[off] = st.mu;
    return (int)off + 1;
}
#ifdef MF_GSTAMPS
extern "C" int mf_debug_gstamps(unsigned long long *out, int nprob) {
    if (nprob > 1024) nprob = 1024;
    return hipMemcpyFromSymbol(out, HIP_SYMBOL(mf::mf_gstamp_buf), sizeof(unsigned long long) * 32 * nprob) == hipSuccess ? 0 : -1;
}
extern "C" int mf_debug_gstamps_reset(void) {
    static unsigned long long z[32 * 1024];
    return hipMemcpyToSymbol(HIP_SYMBOL(mf::mf_gstamp_buf), z, sizeof z) == hipSuccess ? 0 : -1;
}
#endif

// diagnostics: the IPOPT-mode trace of horizon 0 of the last solve with verbose >= 2 (rows of GDBG_W doubles:
// rows [0, GDBG_ROWS) from k_gpre, then [GDBG_ROWS, 2 GDBG_ROWS) from k_gls, indexed by the iteration)
extern "C" int mf_gdebug_trace(double *out) {
    if (!out) return capi_fail(MF_ERR_ARG, "null argument");
    GHIPCHK(hipMemcpyFromSymbol(out, HIP_SYMBOL(mf_gdbg_pre), sizeof(double) * GDBG_ROWS * GDBG_W));
    GHIPCHK(hipMemcpyFromSymbol(out + GDBG_ROWS * GDBG_W, HIP_SYMBOL(mf_gdbg_ls), sizeof(double) * GDBG_ROWS * GDBG_W));
    return GDBG_ROWS;
}
extern "C" int mf_gdebug_trace_reset(void) {
    static std::vector<double> z((size_t)GDBG_ROWS * GDBG_W, 0.0);
    GHIPCHK(hipMemcpyToSymbol(HIP_SYMBOL(mf_gdbg_pre), z.data(), sizeof(double) * z.size()));
    GHIPCHK(hipMemcpyToSymbol(HIP_SYMBOL(mf_gdbg_ls), z.data(), sizeof(double) * z.size()));
    return MF_OK;
}

#ifdef MF_GCHK
// diagnostic build: the checkpoint words live in mapped host memory; the SIGABRT handler (the runtime aborts the
// process on a GPU fault) and mf_gdebug_chk_dump write them to the file named at attach time
#include <csignal>
#include <fcntl.h>
#include <unistd.h>
namespace {
unsigned *g_chk_host = nullptr;
char g_chk_path[512];
void gchk_write() {
    const int fd = open(g_chk_path, O_WRONLY | O_CREAT | O_TRUNC, 0644);
    if (fd < 0) return;
    const ssize_t n = write(fd, g_chk_host, sizeof(unsigned) * GCHK_W * GCHK_B);
    (void)n;
    close(fd);
}
void gchk_on_abort(int sig) {
    if (g_chk_host) gchk_write();
    signal(sig, SIG_DFL);
    raise(sig);
}
}  // namespace
extern "C" int mf_gdebug_chk_attach(const char *path) {
    if (!path) return capi_fail(MF_ERR_ARG, "null path");
    snprintf(g_chk_path, sizeof g_chk_path, "%s", path);
    if (!g_chk_host) {
        GHIPCHK(hipHostMalloc(reinterpret_cast<void **>(&g_chk_host), sizeof(unsigned) * GCHK_W * GCHK_B, hipHostMallocMapped));
        unsigned *d = nullptr;
        GHIPCHK(hipHostGetDevicePointer(reinterpret_cast<void **>(&d), g_chk_host, 0));
        GHIPCHK(hipMemcpyToSymbol(HIP_SYMBOL(mf::mf_gchk_dev), &d, sizeof d));
        signal(SIGABRT, gchk_on_abort);
    }
    memset(g_chk_host, 0, sizeof(unsigned) * GCHK_W * GCHK_B);
    return MF_OK;
}
extern "C" int mf_gdebug_chk_dump(void) {
    if (!g_chk_host) return capi_fail(MF_ERR_ARG, "not attached");
    gchk_write();
    return MF_OK;
}
#endif

// diagnostics: the solver counters of problem b after the last solve (IPOPT mode): iterations, status, inertia
// corrections, line-search failures, second-order-correction steps, restoration phases, watchdog starts,
// soft-restoration steps, failed searches after StopWatchDog, restoration-phase iterations
extern "C" int mf_gdebug_counters(mf_gproblem *p, int b, int *out) {
    if (!p || !out) return capi_fail(MF_ERR_ARG, "null argument");
    if (b < 0 || b >= p->last_batch || !p->d_st) return capi_fail(MF_ERR_ARG, "no such problem in the last solve");
    int e = capi_ensure_device();
    if (e) return e;
    GState st;
    GHIPCHK(hipMemcpy(&st, p->d_st + b, sizeof st, hipMemcpyDeviceToHost));
    const int v[10] = {st.iter, st.status, st.n_ic, st.n_ls_fail, st.n_soc, st.n_resto, st.n_wd, st.n_soft,
                       st.n_wdfail, st.n_rit};
    for (int i = 0; i < 10; i++) out[i] = v[i];
    return 10;
}

// diagnostics: the slack rows s (N x NI) of problem b after the last solve (with mf_gdebug_duals, the primal-dual
// point an oracle-side KKT check of the device's solution needs)
template <class FAM> static int gslack_core(mf_gproblem *p, int b, double *out) {
    using D = typename FAM::D;
    const GSz<D> Z(p->spec.N);
    if (b < 0 || b >= p->last_batch) return capi_fail(MF_ERR_ARG, "problem index out of range (last solve's batch)");
    GHIPCHK(hipDeviceSynchronize());
    std::vector<double> s(Z.i());
    GHIPCHK(hipMemcpy(s.data(), p->A.s + (size_t)b * Z.i(), Z.i() * sizeof(double), hipMemcpyDeviceToHost));
    for (int k = 0; k < p->spec.N; k++)
        for (int q = 0; q < D::NI; q++) out[(size_t)k * D::NI + q] = s[(size_t)k * D::NIA + q];
    return p->spec.N * D::NI;
}

extern "C" int mf_gdebug_slacks(mf_gproblem *p, int b, double *out) {
    if (!p || !out) return capi_fail(MF_ERR_ARG, "null argument");
    switch (p->kind) {
        case GK_BOX: return gslack_core<FamBox>(p, b, out);
        case GK_CH6F: return gslack_core<FamCh6F>(p, b, out);
        case GK_CH6FT: return gslack_core<FamCh6FT>(p, b, out);
        case GK_CH3: return gslack_core<FamCh3>(p, b, out);
        case GK_CH3T: return gslack_core<FamCh3T>(p, b, out);
        case GK_CENT: return gslack_core<FamCent>(p, b, out);
        case GK_BOXT: return gslack_core<FamBoxT>(p, b, out);
    }
    return capi_fail(MF_ERR_UNSUPPORTED, "no kernel instantiation");
}

extern "C" int mf_gdebug_duals(mf_gproblem *p, int b, double *out) {
    if (!p || !out) return capi_fail(MF_ERR_ARG, "null argument");
    switch (p->kind) {
        case GK_BOX: return gdual_core<FamBox>(p, b, out);
        case GK_CH6F: return gdual_core<FamCh6F>(p, b, out);
        case GK_CH6FT: return gdual_core<FamCh6FT>(p, b, out);
        case GK_CH3: return gdual_core<FamCh3>(p, b, out);
        case GK_CH3T: return gdual_core<FamCh3T>(p, b, out);
        case GK_CENT: return gdual_core<FamCent>(p, b, out);
        case GK_BOXT: return gdual_core<FamBoxT>(p, b, out);
    }
    return capi_fail(MF_ERR_UNSUPPORTED, "no kernel instantiation");
}

extern "C" int mf_gnode_record(mf_gproblem *p, const double *xu, const double *yi, const double *ye, const double *lam,
                               const double *line_ref, double *rec, int device) {
    if (!p || !xu || !yi || !lam || !rec) return capi_fail(MF_ERR_ARG, "null argument");
    int e = capi_ensure_device();
    if (e) return e;
    GHIPCHK(hipSetDevice(device));
    const double zero2[6] = {p->spec.line_ref[0], p->spec.line_ref[1], 0, 0, 0, 0};
    const double *lr = line_ref ? line_ref : zero2;  // CENTAURO: the 6 pose targets
    const double ye0[16] = {0};
    const double *yv = ye ? ye : ye0;
    switch (p->kind) {
        case GK_BOX: return grec_core<FamBox>(p, xu, yi, yv, lam, lr, rec);
        case GK_CH6F: return grec_core<FamCh6F>(p, xu, yi, yv, lam, lr, rec);
        case GK_CH6FT: return grec_core<FamCh6FT>(p, xu, yi, yv, lam, lr, rec);
        case GK_CH3: return grec_core<FamCh3>(p, xu, yi, yv, lam, lr, rec);
        case GK_CH3T: return grec_core<FamCh3T>(p, xu, yi, yv, lam, lr, rec);
        case GK_CENT: return grec_core<FamCent>(p, xu, yi, yv, lam, lr, rec);
        case GK_BOXT: return grec_core<FamBoxT>(p, xu, yi, yv, lam, lr, rec);
    }
    return capi_fail(MF_ERR_UNSUPPORTED, "no kernel instantiation");
}
