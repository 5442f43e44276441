// Shared definitions of the generic stage-structured IPM (csrc/gipm.hip) and of the chain family's kernels
// (csrc/gchain.hip): per-horizon solver state, the device arrays, sizes, LDS model images, copy helpers.
#pragma once
// the phase kernels read their model images in LDS through generic pointers (dyn.hpp joint_at)
#ifndef MF_GENERIC_MODEL_PTR
#define MF_GENERIC_MODEL_PTR 1
#endif
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstddef>

#include "bk_wave.hpp"
#include "capi_internal.hpp"
#include "gfam.hpp"

namespace mf {

struct GState {
    double mu, nu, reg_last, E0, cviol, obj;
    double dw_c, dc_c;  // the regularisation the accepted factorisation was made with (k_gkkt -> k_gls)
    int reg_tier, status, iter, n_ls_fail, n_ic, consec_fail, n_soc;
    int frow;  // >= 0: this iteration's factors are k_gspec's storage row frow (k_gkkt -> k_gls), -1: the horizon's own
    // IPOPT mode (GParams::filter; the same algorithm as oracle/mf_ocp.c mfg_opts.filter with resto_hard_dyn)
    double ic_last, ic_last_main;  // last nonzero inertia perturbation: current problem / main problem in a restoration
    double thm[2][2];              // theta_max / theta_min of the main / restoration filter (< 0: unset)
    double rs_ph, rs_th;           // main problem's line-search reference where the restoration started
    double mu_orig, zeta;          // main problem's mu during a restoration; proximity weight sqrt(mu_resto)
    double wd_ph, wd_th, wd_gd, wd_atest;  // watchdog reference
    double pd_cur;                 // soft restoration: primal-dual error before the pending step
    int mode;                      // 0 main problem, 1 restoration problem
    int pend;                      // GP_*: pending action of the next phases
    int nf[2];                     // filter entries (main, restoration)
    int in_wd, wd_short, wd_trial, in_soft, soft_cnt, n_resto, n_wd, n_soft;
    int n_wdfail, n_rit;  // failed searches after StopWatchDog (GP_WDSOFT rounds), restoration-phase iterations
};
enum { GS_RUNNING = -1, GS_CONVERGED = 0, GS_MAXITER = 1, GS_LSFAIL = 2, GS_INERTIA = 3, GS_RESTOFAIL = 4,
       GS_LOCINF = 5 };
// pending actions (IPOPT mode):
//   GP_SOFT        the last k_gls took a soft-restoration step: k_gpre compares the primal-dual errors
//   GP_RESTO       k_gpre sets up the restoration problem at the current point (records current)
//   GP_LSM         k_gkkt / k_gls compute the restoration problem's least-square multipliers
//   GP_IDLE(_RESTO) the records are stale (a restoration ended / a soft step was undone): k_gkkt and k_gls idle,
//                  the next iteration re-evaluates (and then sets up the restoration)
//   GP_WDSOFT      the watchdog stopped (iterate and direction restored) and the backtracking search from the
//                  stored point failed: the records describe the abandoned point, so k_gpre / k_gkkt idle while they
//                  are re-evaluated, and k_gls then augments the filter with the stored point and starts the soft
//                  restoration from it (oracle/mf_ocp.c ipm_filter: eval_all after StopWatchDog)
// Iteration counts follow the oracle's: the launch rounds that only switch state (a soft step undone, the start
// of the restoration phase, a re-evaluation) advance no iteration.
enum { GP_NONE = 0, GP_SOFT = 1, GP_RESTO = 2, GP_LSM = 3, GP_IDLE = 4, GP_IDLE_RESTO = 5, GP_WDSOFT = 6 };
constexpr int GFCAP = 512;  // filter entries per filter (dominated entries are dropped as IPOPT does)
// Concurrent inertia tries: IPOPT's inertia correction is a sequential search over delta_w (0, then last / 3 or 1e-4,
// then x8 / x100 ...), one whole Riccati factorisation per try (2.3-2.5 per iteration on C3 / C4).  When at most
// GArrays::spec_max horizons are running -- the tail, where each horizon's serial factorisations set the batch time and
// the device is otherwise idle -- k_gspec factors the first GNSPEC candidates of that sequence at once, one wavefront
// each, into storage of their own; k_gkkt then replays the sequential search and takes a try's result (and copies its
// factors) wherever the parameters match exactly, so the outcome is the sequential one bit for bit.  spec_max: the
// running count whose GNSPEC tries all fit on the device at once (k_gspec's LDS and registers; gensure_ws), at least
// GSPEC_MIN and at most GSPEC_MAX.
constexpr int GNSPEC = 4, GSPEC_MIN = 64, GSPEC_MAX = 1024;
// diagnostic trace of horizon 0 in IPOPT mode (mf_gopts.verbose >= 2; mf_gdebug_trace): per iteration one row
// from k_gpre (E_0 pieces, the restoration exit test) and one from k_gls (line search)
constexpr int GDBG_ROWS = 4096, GDBG_W = 16;

struct GArrays {
    double *x, *u, *s, *lam, *ye, *yi, *zxL, *zxU, *zuL, *zuU, *vL, *vU;
    double *dx, *du, *ds, *dlam, *dye, *dyi, *dzxL, *dzxU, *dzuL, *dzuU, *dvL, *dvU;
    double *bk;     // saved direction (second-order corrections)
    double *rec;    // node records
    double *scr;    // per-node sweep scratch (FAM::Scratch images, k_geval -> k_gasm)
    double *Sx, *gx, *Su, *gu, *Ss, *gs;
    double *rdyn, *rin, *req, *trdyn, *trin, *treq, *sdyn, *sin_, *seq;
    double *tx, *tu, *ts;
    double *P, *Kinv, *Kfb, *pv, *kv;
    // IPOPT's restoration problem with elastic dynamics rows (oracle ric_relax): per stage the LU factor of
    // I + P_{k+1} D_r with its row permutation, and J~ = J_e,k+1 (I + D_r P_{k+1})^-1
    double *LUg, *Jtg;
    // concurrent inertia tries (IPOPT mode, few horizons running; k_gspec): rows r = s * GNSPEC + t of the factor
    // storage for try t of the s-th running horizon (slist[s]; spec_of[b] = s or -1), its result code and (dw, dc)
    double *Psp, *Ksp, *Fsp, *LUsp, *Jtsp, *sdw, *sdc;
    int *slist, *spec_of, *sres;
    int spec_max;
    const double *u_lo, *u_hi, *c_lo, *c_hi;  // shared, N x NU / N x NI
    double *x0, *lref;                        // per problem: NX, FAM::LREF (line reference / pose targets)
    const double *u0, *w0;                    // optional per-problem fixed u_0 values / warm start
    GState *st;
    int *active;
    // IPOPT mode: filters (2 x GFCAP x (phi, theta)), watchdog / soft-restoration copies of the iterate and of
    // the direction, and the restoration problem's elastic variables p, n >= 0 on the slack rows, the equality rows
    // and the dynamics rows (rows [k NIA + q | N NIA + k NET + e | N (NIA + NET) + k NX + j]; the oracle orders the
    // same rows [dynamics | slack | equality]), with their bound multipliers, steps, trial values,
    // condensed Sigma / barrier gradients / residual corrections, and the reference point w_R, D_R^2
    double *fil, *wdit, *wddir;
    double *pr, *nr, *zp, *zn, *dpr, *dnr, *dzp, *dzn, *tpr, *tnr, *Sp, *Sn, *gp, *gn, *rowr, *wR, *dR;
    // continuous batching (mf_gsolve_stream_dev): slot b holds problem pidx[b] (-1: none); k_gharvest writes a
    // finished slot's result to its problem's output row and hands the slot the next unsolved problem, which
    // k_ginit then initialises (init[b] = 1).  pidx == nullptr: slot b is problem b (mf_gsolve_batch*).
    int *pidx, *next, *init;
    int total;
    unsigned long long *neval;  // timing mode (mf_gproblem_timing): node evaluations made by k_geval, else nullptr
    int fast_kkt;               // k_gkkt_chain ran before this k_gkkt launch: skip the horizons it took
    const double *x0all, *lrall;  // every problem's x_0 and line reference (total rows)
    double *ow, *okkt, *oobj;     // every problem's outputs
    int *ost, *oit;
};

template <class D> struct GSz {
    static constexpr int NX = D::NX, NU = D::NU, NI = D::NIA, NE = D::NET, NK = D::NU + D::NET;
    size_t N;
    __host__ __device__ GSz(int n) : N(n) {}
    __host__ __device__ size_t x() const { return (N + 1) * NX; }
    __host__ __device__ size_t u() const { return N * NU; }
    __host__ __device__ size_t i() const { return N * NI; }
    __host__ __device__ size_t e() const { return N * NE; }
    __host__ __device__ size_t l() const { return N * NX; }
    __host__ __device__ size_t rec() const { return N * D::REC; }
    __host__ __device__ size_t nr() const { return N * (NI + NE + NX); }  // elastic rows (restoration)
    __host__ __device__ size_t nrd() const { return N * (NI + NE); }      // the first elastic dynamics row
    __host__ __device__ size_t lu() const { return N * (NX * NX + NX); }  // stage LU factors + permutations
    __host__ __device__ size_t jt() const { return N * D::NEA * NX; }
    __host__ __device__ size_t bk() const { return 3 * x() + 3 * u() + 4 * i() + l() + e() + 4 * nr(); }
    __host__ __device__ size_t wv() const { return x() + u(); }
    __host__ __device__ size_t P() const { return N * NX * NX; }
    __host__ __device__ size_t Kinv() const { return N * (NK * (NK + 1) + 2 * NK); }  // BK factor + perm/piv
    __host__ __device__ size_t Kfb() const { return N * NK * NX; }
    __host__ __device__ size_t kv() const { return N * NK; }
};

__device__ __forceinline__ bool gb(double b) { return isfinite(b); }

// IPOPT bound_push = bound_frac (k1 = k2): 1e-2 cold, warm_start_bound_push = _frac = 1e-3 warm
__device__ __forceinline__ double gpush(double x, double lo, double hi, double k1 = 1e-2) {
    const double k2 = k1;
    const bool hl = gb(lo), hh = gb(hi);
    if (hl && hh) {
        const double pl = fmin(k1 * fmax(1.0, fabs(lo)), k2 * (hi - lo));
        const double pu = fmin(k1 * fmax(1.0, fabs(hi)), k2 * (hi - lo));
        x = fmax(x, lo + pl);
        x = fmin(x, hi - pu);
    } else if (hl) {
        x = fmax(x, lo + k1 * fmax(1.0, fabs(lo)));
    } else if (hh) {
        x = fmin(x, hi - k1 * fmax(1.0, fabs(hi)));
    }
    return x;
}

__device__ __forceinline__ void gsync() {
    __threadfence_block();
    __syncthreads();
}

// nd contiguous doubles global -> LDS by LDS-DMA (no VGPR destination, every instruction of the copy in flight at
// once; the next gsync()'s vmcnt(0) retires them).  16 bytes per lane (global_load_lds_dwordx4: 128 doubles per
// wave-instruction; 8-byte-aligned sources and destinations are fine, tools/glds16_check.hip), the last double of an
// odd count by two 4-byte lanes.  The LDS destination of one instruction is the wave-uniform base + size x lane, so
// lanes past the end are masked off (they would write beyond the array).  Instructions issued: glds_instr(nd).
__host__ __device__ constexpr int glds_instr(int nd) { return (nd / 2 + 63) / 64 + (nd & 1); }
__device__ __forceinline__ void glds_copy(double *lds, const double *src, int nd, int lane = threadIdx.x) {
    const int n2 = nd & ~1;
    for (int t = 0; t < n2; t += 128)
        if (t + 2 * lane < n2)
            __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void *)(src + t + 2 * lane),
                                             (__attribute__((address_space(3))) void *)(lds + t), 16, 0, 0);
    if (nd & 1) {
        const unsigned *s4 = reinterpret_cast<const unsigned *>(src + n2);
        unsigned *d4 = reinterpret_cast<unsigned *>(lds + n2);
        if (lane < 2)
            __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void *)(s4 + lane),
                                             (__attribute__((address_space(3))) void *)d4, 4, 0, 0);
    }
}

// first NJ joints of a DevModel in LDS
template <int NJ> struct GModelLds {
    static constexpr int WORDS = (int)((offsetof(DevModel, j) + NJ * sizeof(DevJoint) + sizeof(double) - 1) / sizeof(double));
    double w[WORDS];
    __device__ __forceinline__ void load(const DevModel *g) {
        const double *s = reinterpret_cast<const double *>(g);
        for (int i = threadIdx.x; i < WORDS; i += blockDim.x) w[i] = s[i];
    }
    __device__ const DevModel &get() const { return *reinterpret_cast<const DevModel *>(w); }
};

template <class FAM> struct GModels {
    GModelLds<FAM::NJ> m[FAM::NM];
    DevFrame f[FAM::NM];
    __device__ __forceinline__ void load(const DevModel *M0, const DevModel *M1, const DevFrame *F0, const DevFrame *F1) {
        m[0].load(M0);
        if (FAM::NM > 1) m[FAM::NM - 1].load(M1);
        const double *s0 = reinterpret_cast<const double *>(F0);
        double *d0 = reinterpret_cast<double *>(&f[0]);
        for (int i = threadIdx.x; i < (int)(sizeof(DevFrame) / sizeof(double)); i += blockDim.x) d0[i] = s0[i];
        if (FAM::NM > 1) {
            const double *s1 = reinterpret_cast<const double *>(F1);
            double *d1 = reinterpret_cast<double *>(&f[FAM::NM - 1]);
            for (int i = threadIdx.x; i < (int)(sizeof(DevFrame) / sizeof(double)); i += blockDim.x) d1[i] = s1[i];
        }
    }
};

// the family functions take DevModel / DevFrame arrays indexed by arm; in LDS the images are
// separate objects, so a small adaptor forwards by arm
// (two named members and a select, not a pointer array: a lane-indexed array of pointers is a
// private alloca that the backend promotes into a per-thread LDS table)
struct MArr {
    const DevModel *p0, *p1;
    __device__ __forceinline__ const DevModel &operator[](int a) const { return a ? *p1 : *p0; }
};
struct FArr {
    const DevFrame *p0, *p1;
    __device__ __forceinline__ const DevFrame &operator[](int a) const { return a ? *p1 : *p0; }
};


#define GMODELS(FAM)                                                                               \
    __shared__ GModels<FAM> Gm;                                                                    \
    Gm.load(M0, M1, F0, F1);                                                                       \
    __syncthreads();                                                                               \
    const MArr M{&Gm.m[0].get(), &Gm.m[FAM::NM - 1].get()};                                        \
    const FArr F{&Gm.f[0], &Gm.f[FAM::NM - 1]}

// ============================================================== node records
// Two kernels per evaluation.  k_geval: lanes (problem, node, tangent direction) run the models and the
// forward-over-reverse sweeps (FAM::prepass / seeds / lane); the per-node scratch they leave in LDS is
// written to A.scr.  The sweeps need ~512 VGPRs (one wave per SIMD), so the record assembly, which is
// branchy per-entry work over LDS (FAM::rec), runs in k_gasm instead: one wave per node, 64 lanes over the
// record entries, at the occupancy its own registers allow.
template <class FAM> constexpr int scr_words() {
    static_assert(sizeof(typename FAM::Scratch) % sizeof(double) == 0, "scratch is a double array");
    return (int)(sizeof(typename FAM::Scratch) / sizeof(double));
}

}  // namespace mf
