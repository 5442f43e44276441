// The C2 chain family's own kernels (their own translation unit; gipm.hip launches them through gchain.hpp):
// k_geval_chain, the node evaluation direction-major, and k_gkkt_chain, the main problem's Newton step in IPOPT mode.
//
// k_gkkt does the same for every family: one inertia-corrected Riccati factorisation per try, then a second backward
// sweep for the direction's vectors and the forward sweep.  For the Pilz chain with explicit Euler dynamics
// (force_optimization_pilz_6DOF.py:159-172: x_{k+1} = q_k + h qd_k, A = I, B = [h I | 0]) this kernel
//   * forms the stage block and the feedback rows from the stage Hessian H = W + J_I^T D J_I in one pass per stage:
//     Q_uu = H_uu + h (h P) on the qd block, Q_ux = H_ux + h P, Q_xx = H_xx + P, constraint rows h J_n / J_n (the
//     products B^T P B, B^T P A, A^T P A of k_gkkt's tile GEMMs, with the same per-entry arithmetic);
//   * runs the vector pass of the first direction inside the factorisation sweep (the stage's right-hand side -z is a
//     seventh column of the feedback solve), so a successful try leaves P, the factors, the feedback and the
//     direction's backward vectors stored in one sweep;
//   * keeps one wavefront per horizon with wave-local synchronisation only (no workgroup barrier inside a stage) and a
//     small register / LDS footprint, so several horizons share each SIMD.
// The stored factors have k_gkkt's layout (Bunch-Kaufman factor with perm / piv per stage, P_{k+1}, feedback, p_{k+1},
// k_k): the line search's second-order corrections (k_gls, direction()) solve with them unchanged.  Horizons in the
// restoration problem, in a least-square-multiplier pass or in an idle round stay with k_gkkt.  The IPOPT-mode inertia
// correction is IpPDPerturbationHandler's sequence as in k_gkkt (delta_w = 0, then 1e-4 or last / 3, then x100 / x8;
// delta_c = 1e-8 mu^(1/4) on a singular block).

#include "gchain.hpp"

namespace mf {

// bk_solve_cols (bk_wave.hpp) with the factor's LDS reads issued step by step (a compiler fence per column): the same
// arithmetic in the same order, without the whole factor hoisted into registers ahead of the sweeps
template <int LD, int NR, int M>
__device__ __forceinline__ void bk_solve_cols_lean(const double *A, const int *perm, const int *piv, double *B, int nr) {
    const int c = lane_opaque();
    double y[M];
    int pv[M];
    if (c < nr) {
#pragma unroll
        for (int i = 0; i < M; i++) {
            pv[i] = piv[i];
            y[i] = B[perm[i] * NR + c];
        }
#pragma unroll
        for (int t = 0; t < M; t++) {
            __asm__ volatile("" ::: "memory");
            const int start = t + 1 + (pv[t] == 2 ? 1 : 0);
#pragma unroll
            for (int i = t + 1; i < M; i++)
                if (i >= start) y[i] -= A[i * LD + t] * y[t];
        }
#pragma unroll
        for (int i = 0; i < M; i++) {
            __asm__ volatile("" ::: "memory");
            if (pv[i] == 1) {
                y[i] = y[i] / A[i * LD + i];
            } else if (pv[i] == 2 && i + 1 < M) {
                const double a = A[i * LD + i], bb = A[(i + 1) * LD + i], cc = A[(i + 1) * LD + i + 1];
                const double det = a * cc - bb * bb;
                const double y0 = y[i], y1 = y[i + 1];
                y[i] = (cc * y0 - bb * y1) / det;
                y[i + 1] = (a * y1 - bb * y0) / det;
            }
        }
#pragma unroll
        for (int t = M - 1; t >= 0; t--) {
            __asm__ volatile("" ::: "memory");
            const int start = t + 1 + (pv[t] == 2 ? 1 : 0);
            double acc = y[t];
#pragma unroll
            for (int i = t + 1; i < M; i++)
                if (i >= start) acc -= A[i * LD + t] * y[i];
            y[t] = acc;
        }
    }
    wave_lds_sync();
    if (c < nr) {
#pragma unroll
        for (int i = 0; i < M; i++) B[perm[i] * NR + c] = y[i];
    }
    wave_lds_sync();
}

// ============================================================== node evaluation, direction-major (C2's chain)
// k_geval lays a node's 12 tangent directions side by side in a wavefront, so the q lanes' split sweeps (plain FP64
// below joint v, Dual from v on) and the qd lanes' sweeps diverge and the wave runs every path in turn.  Here one
// wavefront runs ONE direction v for 64 consecutive nodes (the specialised solver's k_eval_q layout): no divergence,
// the split pays.  Each lane computes its node's values and sweep weights itself (one plain Newton-Euler pass),
// writes its direction's column straight into the node's scratch image (FAM::Scratch in A.scr, as k_geval leaves it
// for k_gasm), and the v = 0 wave writes the image's header.  XCD-aware block map: workgroups are dealt round-robin
// over the 8 XCDs, so the NDIR direction blocks of node group grp get blockIdx = grp % 8 (mod 8) and their column
// writes to the same scratch lines meet in one L2.  CLS 0: the q directions, CLS 1: the qd directions (separate
// launches, each with its own register allocation).
template <class FAM, int CLS>
__global__ __launch_bounds__(64) void k_geval_chain(const DevModel *M0, const DevFrame *F0, GParams P, GArrays A,
                                                    int batch) {
    using D = typename FAM::D;
    using S = typename FAM::Scratch;
    constexpr int NJ = FAM::NJ, NX = D::NX, NU = D::NU, NE = D::NE, SW = scr_words<FAM>();
    static_assert(FAM::SPLIT, "the chain family's split lanes");
    constexpr int COL0 = (int)(offsetof(S, col) / sizeof(double)), LCOL = GLaneOut<NJ>::LCOL;
    __shared__ GModelLds<NJ> Mm;
    __shared__ DevFrame Ff;
    Mm.load(M0);
    {
        const double *s0 = reinterpret_cast<const double *>(F0);
        double *d0 = reinterpret_cast<double *>(&Ff);
        for (int i = threadIdx.x; i < (int)(sizeof(DevFrame) / sizeof(double)); i += blockDim.x) d0[i] = s0[i];
    }
    __syncthreads();
    const DevModel *mp = &Mm.get();
    const DevFrame *fp = &Ff;
    __asm__ volatile("" : "+s"(mp), "+s"(fp));  // (LDS images behind opaque generic pointers, as giter_phase)
    const DevModel &M = *mp;
    const DevFrame &F = *fp;
    const int xcd = blockIdx.x % 8, r = blockIdx.x / 8, vv = r % NJ, grp = 8 * (r / NJ) + xcd;
    const int v = CLS * NJ + vv, lane = threadIdx.x;
    const int N = P.N;
    const long node = (long)grp * 64 + lane;
    if (node >= (long)batch * N) return;
    const int b = (int)(node / N), k = (int)(node % N);
    const GState *stp = A.st + b;
    if (stp->status != GS_RUNNING) return;
    const double ow = stp->mode == 1 ? 0.0 : 1.0;  // the restoration problem has no objective
    const GSz<D> Z(N);
    double x[NX], u[NU];
    const double *xg = A.x + b * Z.x() + (size_t)k * NX, *ug = A.u + b * Z.u() + (size_t)k * NU;
#pragma unroll
    for (int j = 0; j < NX; j++) x[j] = xg[j];
#pragma unroll
    for (int j = 0; j < NU; j++) u[j] = ug[j];
    double Fw[3], tau[NJ], pf[3], cw[NJ], om[NJ], seed[3];
    FAM::world_force(P, u, Fw);
    arm_values<NJ>(M, F, x, u, Fw, tau, pf);
    const double *yi = A.yi + b * Z.i() + (size_t)k * D::NIA, *ye = A.ye + b * Z.e() + (size_t)k * D::NET;
#pragma unroll
    for (int j = 0; j < NJ; j++) {
        const double w = ow * P.wtau;
        om[j] = 2.0 * w;
        cw[j] = yi[j] + 2.0 * w * tau[j];
    }
    const bool eqon = k >= P.eq_from && k < N;
#pragma unroll
    for (int q = 0; q < 3; q++) seed[q] = (eqon && q < NE) ? ye[q] : 0.0;
    double *img = A.scr + node * SW;
    if (CLS == 0 && vv == 0) {  // the image's header (FAM::Scratch fields before col)
        S *sp = reinterpret_cast<S *>(img);
#pragma unroll
        for (int q = 0; q < 3; q++) {
            sp->E[0][q] = 0.0;
            sp->pf[q] = pf[q];
            sp->seed[q] = seed[q];
            sp->Fw[q] = Fw[q];
        }
#pragma unroll
        for (int j = 0; j < NJ; j++) {
            sp->tau[0][j] = tau[j];
            sp->cw[j] = cw[j];
            sp->om[j] = om[j];
        }
        sp->ow = ow;
    }
    arm_lane_split<NJ>(M, F, x, u, Fw, cw, seed, v, img + COL0 + v * LCOL);
    if (A.neval && CLS == 0 && vv == 0) {
        const int nrun = __popcll(__ballot(1));
        if (lane == 0) atomicAdd(A.neval, (unsigned long long)nrun);
    }
}

// the horizon's state that k_gkkt_chain takes (k_gkkt skips exactly these when the chain kernel ran)
__device__ __forceinline__ bool chain_fast_state(const GState &st) {
    return st.status == GS_RUNNING && st.mode == 0 && st.pend == GP_NONE;
}

// Diagnostic build only (-DMF_CSTAMPS, libmpcfatigue_cstamps.so): cycle counts of k_gkkt_chain's phases summed over
// all waves (slots: 0 setup, 1 stage loads, 2 slack weights / tv, 3 stage block + rows + vector pass, 4 BK factor,
// 5 factor stores + feedback solve, 6 P update, 7 forward sweep, 8 slack rows and multipliers, 12 pivoted BK factor;
// counters 9 sweeps, 10 stages, 11 launches of a running horizon, 13 pivoted factorisations, 14 sweeps ended by a
// wrong inertia, 15 by a singular block), read by mf_debug_cstamps
#ifdef MF_CSTAMPS
__device__ unsigned long long mf_cstamp_buf[16];
#define CST_INIT                                 \
    unsigned long long cst_acc_[16] = {0};       \
    unsigned long long cst_prev_ = __builtin_amdgcn_s_memtime()
#define CST(slot)                                                  \
    do {                                                           \
        unsigned long long t_ = __builtin_amdgcn_s_memtime();      \
        cst_acc_[slot] += t_ - cst_prev_;                          \
        cst_prev_ = t_;                                            \
    } while (0)
#define CST_COUNT(slot, v) do { cst_acc_[slot] += (v); } while (0)
#define CST_FLUSH                                                                        \
    do {                                                                                 \
        if (threadIdx.x == 0)                                                            \
            for (int s_ = 0; s_ < 16; s_++) atomicAdd(&mf_cstamp_buf[s_], cst_acc_[s_]); \
    } while (0)
#else
#define CST_INIT do {} while (0)
#define CST(slot) do {} while (0)
#define CST_COUNT(slot, v) do {} while (0)
#define CST_FLUSH do {} while (0)
#endif

// one stage's inputs to k_gkkt_chain's backward sweep: the record's W, J_I, the Lagrangian gradient row, the
// next / this node's line-row Jacobians, and the stage's vectors V (offsets below)
template <int NV, int NI, int NE, int NX, int NU, int NIA, int NET, int NEA> struct ChainStageIn {
    static constexpr int SX = 0, SU = SX + NX, SS = SU + NU, GX = SS + NIA, GU = GX + NX, GS = GU + NU, YI = GS + NIA,
                         LK = YI + NIA, LP = LK + NX, YE = LP + NX, RD = YE + NET, RI = RD + NX, RN = RI + NIA,
                         END = RN + NEA;
    double W[NV * NV], JI[NI * NV], GL[NV], Jn[NE * NX], JE[NE * NX], V[END];
    // LDS-DMA instructions of one stage's copy (glds_copy)
    static constexpr int nc(int nd) { return glds_instr(nd); }
    static constexpr int DMA = nc(NV * NV) + nc(NI * NV) + nc(NV) + 2 * nc(NE * NX) + 5 * nc(NX) + 2 * nc(NU) +
                               4 * nc(NIA) + nc(NET) + nc(NEA);
};

// s_waitcnt vmcnt(C), also a compiler barrier for memory operations (no LDS-DMA moves across it)
template <int C> __device__ __forceinline__ void wait_vm() {
    static_assert(C >= 0 && C < 64, "vmcnt range");
    __asm__ volatile("s_waitcnt vmcnt(%0)" ::"n"(C) : "memory");
}

template <class FAM>
__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(4))) void k_gkkt_chain(GParams P, GArrays A, int batch) {
    using D = typename FAM::D;
    constexpr int NX = D::NX, NU = D::NU, NV = D::NV, NI = D::NI, NE = D::NE, NIA = D::NIA, NEA = D::NEA, NET = D::NET;
    constexpr int NK = NU + NET, LDK = NK + 1, KSTG = NK * LDK + 2 * NK, NR = NX + 1;
    static_assert(ChainEuler<FAM>::value && D::NM == 0 && NE == NEA && NX == NU - 1, "Euler chain with line rows");
    const int b = blockIdx.x, lane = threadIdx.x;
    if (b >= batch) return;
    // the horizon's state in LDS, not in registers: a GState copy is ~70 dwords the compiler would keep live in VGPRs
    // for the whole kernel (every lane reads the same values; lane 0 writes)
    __shared__ GState st;
    if (lane == 0) st = A.st[b];
    wave_lds_sync();
    if (!P.filter || !chain_fast_state(st)) return;
    CST_INIT;
    CST_COUNT(11, 1);
    const int N = P.N;
    const double h = P.h, mu = st.mu;  // (read once: wave-uniform)
    const GSz<D> Z(N);
    const double *rec = A.rec + b * Z.rec();
    const double *x = A.x + b * Z.x(), *u = A.u + b * Z.u(), *s = A.s + b * Z.i(), *lam = A.lam + b * Z.l();
    const double *ye = A.ye + b * Z.e(), *yi = A.yi + b * Z.i();
    const double *zxL = A.zxL + b * Z.x(), *zxU = A.zxU + b * Z.x(), *zuL = A.zuL + b * Z.u(), *zuU = A.zuU + b * Z.u();
    const double *vL = A.vL + b * Z.i(), *vU = A.vU + b * Z.i();
    double *dx = A.dx + b * Z.x(), *du = A.du + b * Z.u(), *ds = A.ds + b * Z.i(), *dlam = A.dlam + b * Z.l();
    double *dye = A.dye + b * Z.e(), *dyi = A.dyi + b * Z.i();
    double *dzxL = A.dzxL + b * Z.x(), *dzxU = A.dzxU + b * Z.x(), *dzuL = A.dzuL + b * Z.u(), *dzuU = A.dzuU + b * Z.u();
    double *dvL = A.dvL + b * Z.i(), *dvU = A.dvU + b * Z.i();
    const double *Sx = A.Sx + b * Z.x(), *gx = A.gx + b * Z.x(), *Su = A.Su + b * Z.u(), *gu = A.gu + b * Z.u();
    const double *Ss = A.Ss + b * Z.i(), *gs = A.gs + b * Z.i();
    const double *rdyn = A.rdyn + b * Z.l(), *rin = A.rin + b * Z.i(), *req = A.req + b * Z.e();
    double *Pg = A.P + b * Z.P(), *Kg = A.Kinv + b * Z.Kinv(), *Fg = A.Kfb + b * Z.Kfb(), *pvg = A.pv + b * Z.l();
    double *kvg = A.kv + b * Z.kv();
    const double *ulo = A.u_lo, *uhi = A.u_hi, *clo = A.c_lo, *chi = A.c_hi;
    auto R = [&](int k) __attribute__((always_inline)) { return rec + (size_t)k * D::REC; };
    auto ufix = [&](int i) __attribute__((always_inline)) { return gb(ulo[i]) && ulo[i] == uhi[i]; };
    auto cact = [&](int k, int q) __attribute__((always_inline)) { return gb(clo[k * NI + q]) || gb(chi[k * NI + q]); };
    auto eqon = [&](int k) __attribute__((always_inline)) { return k >= P.eq_from && k < N; };

    // per-stage flags, once per launch: fixed controls (u_lo == u_hi) and active slack rows as bit masks in LDS (the
    // stage loop would otherwise wait on these shared-array loads every stage)
    static_assert(NU <= 8 && NI <= 8, "byte masks");
    __shared__ unsigned char fixm[GCHAIN_NMAX], actm[GCHAIN_NMAX];
    for (int k = lane; k < N; k += 64) {
        unsigned f = 0, c = 0;
        for (int a = 0; a < NU; a++) f |= ufix(k * NU + a) ? 1u << a : 0u;
        for (int q = 0; q < NI; q++) c |= cact(k, q) ? 1u << q : 0u;
        fixm[k] = (unsigned char)f;
        actm[k] = (unsigned char)c;
    }
    wave_lds_sync();

    // stage inputs, double-buffered: stage k - 1's inputs arrive by LDS-DMA while stage k computes.  The compiler does
    // not order LDS reads after LDS-DMA, so each stage waits explicitly, s_waitcnt vmcnt(SI::DMA) right after issuing
    // the prefetch: every copy issues exactly SI::DMA instructions (pieces a stage does not have -- J_n past the
    // horizon, lam_{-1}, the next equality residual -- are copied from a valid dummy source and skipped by the
    // readers), so the wait retires this stage's inputs and everything older, never the prefetch.  The global stores
    // of a stage's results are deferred to the next stage, after its wait (stores issued between two stages' copies
    // would have to retire before the second wait).  Nothing writes into a buffer after its DMA.
    using SI = ChainStageIn<NV, NI, NE, NX, NU, NIA, NET, NEA>;
    __shared__ SI SIb2[2];  // (indexed by a runtime slot: every access stays an LDS access, ds_read / ds_write)
    __shared__ double Ks[NK * LDK], Bm[NK * NR], Rh[NK * NX], Qx[NX * NX], Ps[NX * NX], T2[NX * NX];
    __shared__ double Dd[NIA], wq[NIA], vx[NX], tv[NX], pvs[NX], zv[NK];
    __shared__ int perm[NK], piv[NK];

    auto issue = [&](int k, int slot) __attribute__((always_inline)) {
        SI &T = SIb2[slot];
        const int lane = lane_opaque();
        const double *rk = R(k), *rn = k + 1 < N ? R(k + 1) : rk;
        glds_copy(T.W, rk + D::O_W, NV * NV, lane);
        glds_copy(T.JI, rk + D::O_JI, NI * NV, lane);
        glds_copy(T.GL, rk + D::O_GL, NV, lane);
        glds_copy(T.Jn, rn + D::O_JE, NE * NX, lane);
        glds_copy(T.JE, rk + D::O_JE, NE * NX, lane);
        glds_copy(T.V + SI::SX, Sx + k * NX, NX, lane);
        glds_copy(T.V + SI::SU, Su + k * NU, NU, lane);
        glds_copy(T.V + SI::SS, Ss + k * NIA, NIA, lane);
        glds_copy(T.V + SI::GX, gx + k * NX, NX, lane);
        glds_copy(T.V + SI::GU, gu + k * NU, NU, lane);
        glds_copy(T.V + SI::GS, gs + k * NIA, NIA, lane);
        glds_copy(T.V + SI::YI, yi + k * NIA, NIA, lane);
        glds_copy(T.V + SI::LK, lam + k * NX, NX, lane);
        glds_copy(T.V + SI::LP, lam + (k > 0 ? k - 1 : 0) * NX, NX, lane);
        glds_copy(T.V + SI::YE, ye + k * NET, NET, lane);
        glds_copy(T.V + SI::RD, rdyn + k * NX, NX, lane);
        glds_copy(T.V + SI::RI, rin + k * NIA, NIA, lane);
        glds_copy(T.V + SI::RN, req + (k + 1 < N ? k + 1 : k) * NET, NEA, lane);
    };
    // stage k's factor (with perm / piv), feedback and step, from LDS (k_gkkt's storage layout)
    auto store_factors = [&](int k) __attribute__((always_inline)) {
        const int lane = lane_opaque();
        double *kst = Kg + (size_t)k * KSTG;
        for (int e = lane; e < NK * LDK; e += 64) kst[e] = Ks[e];
        for (int e = lane; e < NK; e += 64) { kst[NK * LDK + e] = perm[e]; kst[NK * LDK + NK + e] = piv[e]; }
        for (int e = lane; e < NK * NX; e += 64) Fg[(size_t)k * NK * NX + e] = Bm[(e / NX) * NR + e % NX];
        for (int a = lane; a < NK; a += 64) kvg[k * NK + a] = Bm[a * NR + NX];
    };

    // one stage of the backward sweep from the inputs in C, prefetching stage k - 1's into Nx (0 ok, 1 wrong inertia,
    // 2 singular block)
    auto stage = [&](int k, int slot, double dw, double dc) __attribute__((always_inline)) -> int {
        const SI &C = SIb2[slot];
        CST_COUNT(10, 1);
        if (k >= 1) {
            issue(k - 1, slot ^ 1);
            wait_vm<SI::DMA>();
        } else {
            wait_vm<0>();
        }
        // the lane index made opaque per stage: the per-lane LDS / global addresses are recomputed inside the
        // loop instead of being hoisted out of it and held in registers across the whole sweep
        const int lane = lane_opaque();
        const bool en = eqon(k + 1), ek = eqon(k);
        const unsigned fm = fixm[k], am = actm[k];
        auto fixd = [&](int a) __attribute__((always_inline)) { return ((fm >> a) & 1u) != 0; };
        const double *Wl = C.W, *JIl = C.JI, *GL = C.GL, *Jn = C.Jn, *JEk = C.JE, *Vs = C.V;
        // the previous stage's results; P_{k+1} and p_{k+1} of this stage (the direction's forward sweep and the
        // corrections read them)
        if (k + 1 < N) store_factors(k + 1);
        for (int e = lane; e < NX * NX; e += 64) Pg[(size_t)k * NX * NX + e] = Ps[e];
        for (int j = lane; j < NX; j += 64) pvg[k * NX + j] = pvs[j];
        CST(1);
        // slack-row weights: D (the condensed Hessian term) and w (the J_I^T w term of the vector pass);
        // tv = p_{k+1} + P_{k+1} r_d
        if (lane < NI) {
            const int q = lane;
            double dd = 0.0, w = Vs[SI::YI + q];
            if ((am >> q) & 1u) {
                const double sg = Vs[SI::SS + q] + dw;
                dd = sg / (1.0 + dc * sg);
                w += dd * (Vs[SI::RI + q] + (Vs[SI::GS + q] - Vs[SI::YI + q]) / sg);
            }
            Dd[q] = dd;
            wq[q] = w;
        } else if (lane >= 8 && lane < 8 + NX) {
            const int j = lane - 8;
            double acc = pvs[j];
            for (int l = 0; l < NX; l++) acc += Ps[j * NX + l] * Vs[SI::RD + l];
            tv[j] = acc;
        }
        wave_lds_sync();
        CST(2);
        // stage block K, feedback rows Rh, Q_xx, and the vector pass's right-hand side, one pass
        auto Hel = [&](int a, int c) __attribute__((always_inline)) -> double {  // W + J_I^T D J_I (+ diagonal)
            double v = Wl[a * NV + c];
            for (int q = 0; q < NI; q++) v += (JIl[q * NV + a] * Dd[q]) * JIl[q * NV + c];
            if (a == c) {
                v += dw;
                v += a < NX ? Vs[SI::SX + a] : Vs[SI::SU + a - NX];
            }
            return v;
        };
        for (int e = lane; e < NK * NK; e += 64) {
            const int a = e / NK, c = e % NK;
            double v = 0.0;
            if (a < NU && c < NU) {
                if (fixd(a) || fixd(c)) v = (a == c) ? 1.0 : 0.0;
                else {
                    v = Hel(NX + a, NX + c);
                    if (a < NX && c < NX) v += h * (Ps[a * NX + c] * h);
                }
            } else if (a >= NU && c >= NU) {
                v = (a == c) ? (en ? -dc : -1.0) : 0.0;
            } else {
                const int ee = (a >= NU ? a : c) - NU, uu = a >= NU ? c : a;
                if (!fixd(uu) && en && uu < NX) v = Jn[ee * NX + uu] * h;
            }
            Ks[a * LDK + c] = v;
        }
        for (int e = lane; e < NK * NX; e += 64) {
            const int a = e / NX, j = e % NX;
            double v = 0.0;
            if (k > 0) {
                if (a < NU) {
                    if (!fixd(a)) {
                        v = Hel(NX + a, j);
                        if (a < NX) v += h * Ps[a * NX + j];
                    }
                } else if (en) {
                    v = Jn[(a - NU) * NX + j];
                }
            }
            Rh[e] = v;
            Bm[a * NR + j] = -v;
        }
        if (k > 0)
            for (int e = lane; e < NX * NX; e += 64) Qx[e] = Hel(e / NX, e % NX) + Ps[e];
        // the vector pass: vx = the stage's gradient row of the Lagrangian with the slack weights, z = its
        // projection through the dynamics and the next node's state rows
        auto vxel = [&](int a) __attribute__((always_inline)) -> double {
            const bool fa = a < NX ? (k == 0) : fixd(a - NX);
            if (fa) return 0.0;
            double g = GL[a];
            for (int q = 0; q < NI; q++) g += JIl[q * NV + a] * wq[q];
            if (a < NX) {
                g += Vs[SI::GX + a];
                if (k > 0) g -= Vs[SI::LP + a];
                g += Vs[SI::LK + a];  // A^T lam_k (A = I)
                if (ek)
                    for (int ee = 0; ee < NE; ee++) g += JEk[ee * NX + a] * Vs[SI::YE + ee];
            } else {
                g += Vs[SI::GU + a - NX];
                if (a - NX < NX) g += h * Vs[SI::LK + a - NX];  // B^T lam_k
            }
            return g;
        };
        if (lane >= 64 - NK) {
            const int a = lane - (64 - NK);
            double z = 0.0;
            if (a < NU) {
                if (!fixd(a)) {
                    z = vxel(NX + a);
                    if (a < NX) z += h * tv[a];
                }
            } else if (en) {
                const int ee = a - NU;
                z = Vs[SI::RN + ee];
                for (int l = 0; l < NX; l++) z += Jn[ee * NX + l] * Vs[SI::RD + l];
            }
            zv[a] = z;
            Bm[a * NR + NX] = -z;
        } else if (lane >= 64 - NK - NX) {
            const int j = lane - (64 - NK - NX);
            vx[j] = vxel(j);
        }
        wave_lds_sync();
        CST(3);
        // the stage block: natural-order pivots in registers, else Bunch-Kaufman in LDS with unrolled scans (both with
        // bk_factor_wave's arithmetic and pivoting, bit for bit; in 2 of 3 stages the q-dot rows' small diagonal
        // against h J_n takes a 2x2 pivot).  Measured per 9 x 9 block, one wavefront (tools/bk_bench.hip): natural
        // order in registers 5.0k cycles, pivoting 17.8k (bk_factor_fixed) / 17.4k (bk_factor_regs_piv, whose code
        // is also 33 KB) / 23.5k (bk_factor_wave).
        BKInertia in;
        if (!bk_factor_regs<LDK, NK>(Ks, perm, piv, in)) {
            in = bk_factor_fixed<LDK, NK>(Ks, perm, piv);
            CST_COUNT(13, 1);
        }
        CST(4);
        if (in.zero) { CST_COUNT(15, 1); return 2; }
        if (in.pos != NU || in.neg != NET) { CST_COUNT(14, 1); return 1; }
        // feedback K^-1 (-Rh) and the step k_k = K^-1 (-z), one column per lane
        bk_solve_cols_lean<LDK, NR, NK>(Ks, perm, piv, Bm, NR);
        CST(5);
        if (k > 0) {
            // P_k = sym(Q_xx + Rh^T Kf), p_k = vx + A^T tv + Kf^T z
            if (lane < NX * NX) {
                const int i = lane / NX, j = lane % NX;
                double v = Qx[lane];
                for (int a = 0; a < NK; a++) v += Rh[a * NX + i] * Bm[a * NR + j];
                T2[lane] = v;
            } else if (lane < NX * NX + NX) {
                const int j = lane - NX * NX;
                double acc = vx[j] + tv[j];
                for (int a = 0; a < NK; a++) acc += Bm[a * NR + j] * zv[a];
                pvs[j] = acc;
            }
            wave_lds_sync();
            for (int e = lane; e < NX * NX; e += 64) Ps[e] = 0.5 * (T2[e] + T2[(e % NX) * NX + e / NX]);
            wave_lds_sync();
        }
        CST(6);
        return 0;
    };

    // one try: the backward sweep with the direction's vectors (0 ok, 1 wrong inertia, 2 singular block); stage k's
    // inputs in SIa for even N - 1 - k, SIb for odd
    auto sweep = [&](double dw, double dc) __attribute__((always_inline)) -> int {
        for (int e = lane; e < NX * NX; e += 64) Ps[e] = (e / NX == e % NX) ? Sx[N * NX + e / NX] + dw : 0.0;
        for (int j = lane; j < NX; j += 64) pvs[j] = gx[N * NX + j] - lam[(N - 1) * NX + j];
        wave_mem_sync();  // (a failed try may have left a prefetch in flight)
        CST_COUNT(9, 1);
        CST(0);
        issue(N - 1, 0);
        int fr = 0;
#pragma unroll 1
        for (int k = N - 1; k >= 0; k--) {
            // (one stage body for both buffers: the waits are explicit, so nothing needs to name the buffer)
            fr = stage(k, (N - 1 - k) & 1, dw, dc);
            if (fr) break;
            wave_lds_sync();  // (the current buffer's readers done before the next DMA overwrites it)
        }
        if (fr == 0) store_factors(0);
        return fr;
    };

    // inertia correction (IPOPT mode, k_gkkt's sequence)
    double dw = 0.0, dc = P.dc_always ? 1e-8 * pow(mu, 0.25) : 0.0;
    const double ic_last = st.ic_last;
    int n_ic = 0;
    bool ok = false;
    for (int tries = 0; tries < 200; tries++) {
        const int fr = sweep(dw, dc);
        if (fr == 0) { ok = true; break; }
        if (fr == 2 && dc == 0.0) { dc = 1e-8 * pow(mu, 0.25); continue; }
        n_ic++;
        if (dw == 0.0) dw = (ic_last == 0.0) ? 1e-4 : fmax(1e-20, ic_last / 3.0);
        else dw *= (ic_last == 0.0 || 1e5 * ic_last < dw) ? 100.0 : 8.0;
        if (dw > 1e40) break;
    }
    if (!ok) {  // k_gkkt's finish(GS_INERTIA)
        double f = 0.0;
        for (int k = lane; k < N; k += 64) f += R(k)[D::O_L];
        f = wave_sum(f);
        if (lane == 0) {
            GState *g = A.st + b;
            g->n_ic = st.n_ic + n_ic;
            g->status = GS_INERTIA;
            g->obj = f;
            g->frow = -1;
            atomicSub(A.active, 1);
        }
        CST_FLUSH;
        return;
    }
    const double dw_c = dw, dc_c = dc;
    CST(0);

    // forward sweep: du_k = k_k + Kf dx_k, dx_{k+1} = r_d + dx_k + h du_qd, dlam_k = p_{k+1} + P_{k+1} dx_{k+1} +
    // J_n^T dy_{k+1}
    __shared__ double dxs[NX], dxn[NX], duv[NK];
    double *Jn = SIb2[0].Jn;  // (the backward sweep's buffers are free now)
    wave_mem_sync();
    for (int j = lane; j < NX; j += 64) { dxs[j] = 0.0; dx[j] = 0.0; }
    for (int ee = lane; ee < NEA; ee += 64) dye[ee] = 0.0;
    wave_lds_sync();
#pragma unroll 1
    for (int k = 0; k < N; k++) {
        const int lane = lane_opaque();
        const bool en = eqon(k + 1);
        glds_copy(T2, Pg + (size_t)k * NX * NX, NX * NX, lane);
        glds_copy(Rh, Fg + (size_t)k * NK * NX, NK * NX, lane);
        glds_copy(zv, kvg + k * NK, NK, lane);
        glds_copy(tv, pvg + k * NX, NX, lane);
        glds_copy(vx, rdyn + k * NX, NX, lane);
        if (en) glds_copy(Jn, R(k + 1) + D::O_JE, NE * NX, lane);
        gsync();
        const unsigned fm = fixm[k];
        if (lane < NK) {
            const int a = lane;
            double acc = zv[a];
            for (int j = 0; j < NX; j++) acc += Rh[a * NX + j] * dxs[j];
            if (a < NU && ((fm >> a) & 1u)) acc = 0.0;
            duv[a] = acc;
            if (a < NU) du[k * NU + a] = acc;
        }
        wave_lds_sync();
        if (lane < NX) {
            const int j = lane;
            double acc = vx[j] + dxs[j];
            acc += h * duv[j];
            dxn[j] = acc;
        }
        wave_lds_sync();
        if (lane < NX) {
            const int j = lane;
            double acc = tv[j];
            for (int l = 0; l < NX; l++) acc += T2[j * NX + l] * dxn[l];
            if (en)
                for (int ee = 0; ee < NE; ee++) acc += Jn[ee * NX + j] * duv[NU + ee];
            dlam[k * NX + j] = acc;
            dx[(k + 1) * NX + j] = dxn[j];
            dxs[j] = dxn[j];
        }
        if (k + 1 < N)
            for (int ee = lane; ee < NEA; ee += 64) dye[(k + 1) * NET + ee] = en ? duv[NU + ee] : 0.0;
        wave_lds_sync();
    }
    gsync();
    CST(7);
    // slack rows and bound multipliers (k_gkkt's direction() tail, main problem)
    const int ln = lane_opaque();
#pragma unroll 1
    for (int e = ln; e < N * NI; e += 64) {
        const int k = e / NI, q = e % NI, i = k * NIA + q;
        double dyv = 0.0, dsv = 0.0;
        if (cact(k, q)) {
            const double *rk = R(k);
            double jd = 0.0;
            for (int a = 0; a < NX; a++) jd += rk[D::O_JI + q * NV + a] * dx[k * NX + a];
            for (int a = 0; a < NU; a++) jd += rk[D::O_JI + q * NV + NX + a] * du[k * NU + a];
            const double sg = Ss[i] + dw_c, Dq = sg / (1.0 + dc_c * sg), rs = gs[i] - yi[i];
            dyv = Dq * (jd + rin[i] + rs / sg);
            dsv = (dyv - rs) / sg;
        }
        dyi[i] = dyv;
        ds[i] = dsv;
    }
    gsync();
#pragma unroll 1
    for (int e = lane_opaque(); e < (N + 1) * NX; e += 64) {
        const int k = e / NX, j = e % NX;
        double a = 0.0, c = 0.0;
        if (k > 0) {
            if (gb(P.x_lo[j])) a = mu / (x[e] - P.x_lo[j]) - zxL[e] - zxL[e] / (x[e] - P.x_lo[j]) * dx[e];
            if (gb(P.x_hi[j])) c = mu / (P.x_hi[j] - x[e]) - zxU[e] + zxU[e] / (P.x_hi[j] - x[e]) * dx[e];
        }
        dzxL[e] = a;
        dzxU[e] = c;
    }
#pragma unroll 1
    for (int e = lane_opaque(); e < N * NU; e += 64) {
        double a = 0.0, c = 0.0;
        if (!ufix(e)) {
            if (gb(ulo[e])) a = mu / (u[e] - ulo[e]) - zuL[e] - zuL[e] / (u[e] - ulo[e]) * du[e];
            if (gb(uhi[e])) c = mu / (uhi[e] - u[e]) - zuU[e] + zuU[e] / (uhi[e] - u[e]) * du[e];
        }
        dzuL[e] = a;
        dzuU[e] = c;
    }
#pragma unroll 1
    for (int e = lane_opaque(); e < N * NI; e += 64) {
        const int i = (e / NI) * NIA + e % NI;
        double a = 0.0, c = 0.0;
        if (gb(clo[e])) a = mu / (s[i] - clo[e]) - vL[i] - vL[i] / (s[i] - clo[e]) * ds[i];
        if (gb(chi[e])) c = mu / (chi[e] - s[i]) - vU[i] + vU[i] / (chi[e] - s[i]) * ds[i];
        dvL[i] = a;
        dvU[i] = c;
    }
    gsync();
    if (lane == 0) {
        GState *g = A.st + b;
        g->n_ic = st.n_ic + n_ic;
        if (dw_c > 0.0) g->ic_last = dw_c;
        g->frow = -1;
        g->dw_c = dw_c;
        g->dc_c = dc_c;
    }
    CST(8);
    CST_FLUSH;
}

// ============================================================== launchers (gchain.hpp)
void gchain_eval(hipStream_t s, int blocks, const DevModel *M0, const DevFrame *F0, const GParams &P, const GArrays &A,
                 int batch) {
    hipLaunchKernelGGL((k_geval_chain<ChainC2, 0>), dim3(blocks), dim3(64), 0, s, M0, F0, P, A, batch);
    hipLaunchKernelGGL((k_geval_chain<ChainC2, 1>), dim3(blocks), dim3(64), 0, s, M0, F0, P, A, batch);
}

void gchain_kkt(hipStream_t s, const GParams &P, const GArrays &A, int batch) {
    hipLaunchKernelGGL(k_gkkt_chain<ChainC2>, dim3(batch), dim3(64), 0, s, P, A, batch);
}

}  // namespace mf

// ============================================================== diagnostics
namespace mf {
// one 9 x 9 stage block per workgroup factorised twice, by a variant (V = 0 bk_factor_regs_piv, 1 bk_factor_fixed,
// 2 bk_factor_regs with the bk_factor_fixed fallback, 3 bk_factor_regs_loop) and by bk_factor_wave (k_gkkt): both factors, perm | piv << 8
// per row and the inertia
template <int M, int V>
__global__ __launch_bounds__(64) void k_bk_compare(const double *K, int n, double *outR, double *outW, int *meta) {
    constexpr int LD = M + 1;
    __shared__ double A1[M * LD], A2[M * LD];
    __shared__ int p1[M], v1[M], p2[M], v2[M];
    const int b = blockIdx.x, lane = threadIdx.x;
    if (b >= n) return;
    for (int e = lane; e < M * LD; e += 64) A1[e] = A2[e] = K[(size_t)b * M * LD + e];
    __syncthreads();
    BKInertia r;
    if constexpr (V == 0) r = bk_factor_regs_piv<LD, M>(A1, p1, v1);
    if constexpr (V == 1) r = bk_factor_fixed<LD, M>(A1, p1, v1);
    if constexpr (V == 2) {
        if (!bk_factor_regs<LD, M>(A1, p1, v1, r)) r = bk_factor_fixed<LD, M>(A1, p1, v1);
    }
    if constexpr (V == 3) r = bk_factor_regs_loop<LD, M>(A1, p1, v1);
    __syncthreads();
    const BKInertia w = bk_factor_wave<LD>(A2, M, p2, v2);
    __syncthreads();
    for (int e = lane; e < M * LD; e += 64) {
        outR[(size_t)b * M * LD + e] = A1[e];
        outW[(size_t)b * M * LD + e] = A2[e];
    }
    int *mb = meta + b * (2 * M + 6);
    if (lane < M) {
        mb[lane] = p1[lane] | (v1[lane] << 8);
        mb[M + lane] = p2[lane] | (v2[lane] << 8);
    }
    if (lane == 0) {
        mb[2 * M] = r.pos; mb[2 * M + 1] = r.neg; mb[2 * M + 2] = r.zero;
        mb[2 * M + 3] = w.pos; mb[2 * M + 4] = w.neg; mb[2 * M + 5] = w.zero;
    }
}
}  // namespace mf

extern "C" int mf_debug_bk_compare(const double *K, int n, int variant, double *outR, double *outW, int *meta) {
    constexpr int M = mf::ChainC2::D::NU + mf::ChainC2::D::NET, LD = M + 1;
    if (!K || !outR || !outW || !meta || n <= 0 || variant < 0 || variant > 3)
        return mf::capi_fail(MF_ERR_ARG, "bad argument");
    double *dK = nullptr, *dR = nullptr, *dW = nullptr;
    int *dm = nullptr;
    const size_t nb = (size_t)n * M * LD * sizeof(double), mb = (size_t)n * (2 * M + 6) * sizeof(int);
    hipError_t e = hipMalloc(&dK, nb);
    if (e == hipSuccess) e = hipMalloc(&dR, nb);
    if (e == hipSuccess) e = hipMalloc(&dW, nb);
    if (e == hipSuccess) e = hipMalloc(&dm, mb);
    if (e == hipSuccess) e = hipMemcpy(dK, K, nb, hipMemcpyHostToDevice);
    if (e == hipSuccess) {
        if (variant == 0) hipLaunchKernelGGL((mf::k_bk_compare<M, 0>), dim3(n), dim3(64), 0, 0, dK, n, dR, dW, dm);
        if (variant == 1) hipLaunchKernelGGL((mf::k_bk_compare<M, 1>), dim3(n), dim3(64), 0, 0, dK, n, dR, dW, dm);
        if (variant == 2) hipLaunchKernelGGL((mf::k_bk_compare<M, 2>), dim3(n), dim3(64), 0, 0, dK, n, dR, dW, dm);
        if (variant == 3) hipLaunchKernelGGL((mf::k_bk_compare<M, 3>), dim3(n), dim3(64), 0, 0, dK, n, dR, dW, dm);
        e = hipGetLastError();
    }
    if (e == hipSuccess) e = hipMemcpy(outR, dR, nb, hipMemcpyDeviceToHost);
    if (e == hipSuccess) e = hipMemcpy(outW, dW, nb, hipMemcpyDeviceToHost);
    if (e == hipSuccess) e = hipMemcpy(meta, dm, mb, hipMemcpyDeviceToHost);
    (void)hipFree(dK); (void)hipFree(dR); (void)hipFree(dW); (void)hipFree(dm);
    if (e != hipSuccess) return mf::capi_fail(MF_ERR_DEVICE, std::string("HIP error: ") + hipGetErrorString(e));
    return M;
}

#ifdef MF_CSTAMPS
extern "C" int mf_debug_cstamps(unsigned long long *out) {
    return hipMemcpyFromSymbol(out, HIP_SYMBOL(mf::mf_cstamp_buf), sizeof(unsigned long long) * 16) == hipSuccess ? 0 : -1;
}
extern "C" int mf_debug_cstamps_reset(void) {
    static unsigned long long z[16];
    return hipMemcpyToSymbol(HIP_SYMBOL(mf::mf_cstamp_buf), z, sizeof z) == hipSuccess ? 0 : -1;
}
#endif
