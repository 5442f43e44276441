// Newton step of the chain family's main problem in IPOPT mode (included by gipm.hip after giter_phase).
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

template <class FAM> struct ChainEuler { static constexpr bool value = false; };
template <> struct ChainEuler<ChainFam<6, 1, 2, false>> { static constexpr bool value = true; };

// the horizon's state that k_gkkt_chain takes (k_gkkt skips exactly these when the chain kernel ran)
__device__ __forceinline__ bool chain_fast_state(const GState &st) {
    return st.status == GS_RUNNING && st.mode == 0 && st.pend == GP_NONE;
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

    // stage inputs (staged by LDS-DMA at the top of each stage), working arrays
    __shared__ double Wl[NV * NV], JIl[NI * NV], Jn[NE * NX], GL[NV], JEk[NE * NX];
    constexpr int V_SX = 0, V_SU = V_SX + NX, V_SS = V_SU + NU, V_GX = V_SS + NIA, V_GU = V_GX + NX, V_GS = V_GU + NU,
                  V_YI = V_GS + NIA, V_LK = V_YI + NIA, V_LP = V_LK + NX, V_YE = V_LP + NX, V_RD = V_YE + NET,
                  V_RI = V_RD + NX, V_RN = V_RI + NIA, V_END = V_RN + NEA;
    __shared__ double Vs[V_END];
    __shared__ double Ks[NK * LDK], Bm[NK * NR], Rh[NK * NX], Qx[NX * NX], Ps[NX * NX], T2[NX * NX];
    __shared__ double Dd[NIA], wq[NIA], vx[NX], tv[NX], pvs[NX], zv[NK];
    __shared__ int perm[NK], piv[NK], fixs[NU];

    // one try: the backward sweep with the direction's vectors (0 ok, 1 wrong inertia, 2 singular block)
    auto sweep = [&](double dw, double dc) __attribute__((always_inline)) -> int {
        for (int e = lane; e < NX * NX; e += 64) Ps[e] = (e / NX == e % NX) ? Sx[N * NX + e / NX] + dw : 0.0;
        for (int j = lane; j < NX; j += 64) pvs[j] = gx[N * NX + j] - lam[(N - 1) * NX + j];
        wave_lds_sync();
#pragma unroll 1
        for (int k = N - 1; k >= 0; k--) {
            // the lane index made opaque per stage: the per-lane LDS / global addresses are recomputed inside the
            // loop instead of being hoisted out of it and held in registers across the whole sweep
            const int lane = lane_opaque();
            const bool en = eqon(k + 1), ek = eqon(k);
            const double *rk = R(k);
            // P_{k+1} and p_{k+1} of this stage (the direction's forward sweep and the corrections read them)
            for (int e = lane; e < NX * NX; e += 64) Pg[(size_t)k * NX * NX + e] = Ps[e];
            for (int j = lane; j < NX; j += 64) pvg[k * NX + j] = pvs[j];
            glds_copy(Wl, rk + D::O_W, NV * NV, lane);
            glds_copy(JIl, rk + D::O_JI, NI * NV, lane);
            glds_copy(GL, rk + D::O_GL, NV, lane);
            if (en) glds_copy(Jn, R(k + 1) + D::O_JE, NE * NX, lane);
            if (ek) glds_copy(JEk, rk + D::O_JE, NE * NX, lane);
            glds_copy(Vs + V_SX, Sx + k * NX, NX, lane);
            glds_copy(Vs + V_SU, Su + k * NU, NU, lane);
            glds_copy(Vs + V_SS, Ss + k * NIA, NIA, lane);
            glds_copy(Vs + V_GX, gx + k * NX, NX, lane);
            glds_copy(Vs + V_GU, gu + k * NU, NU, lane);
            glds_copy(Vs + V_GS, gs + k * NIA, NIA, lane);
            glds_copy(Vs + V_YI, yi + k * NIA, NIA, lane);
            glds_copy(Vs + V_LK, lam + k * NX, NX, lane);
            if (k > 0) glds_copy(Vs + V_LP, lam + (k - 1) * NX, NX, lane);
            glds_copy(Vs + V_YE, ye + k * NET, NET, lane);
            glds_copy(Vs + V_RD, rdyn + k * NX, NX, lane);
            glds_copy(Vs + V_RI, rin + k * NIA, NIA, lane);
            if (k + 1 < N) glds_copy(Vs + V_RN, req + (k + 1) * NET, NEA, lane);
            if (lane < NU) fixs[lane] = ufix(k * NU + lane) ? 1 : 0;
            gsync();  // the LDS-DMA copies retired (vmcnt) and visible
            if (!en)
                for (int e = lane; e < NE * NX; e += 64) Jn[e] = 0.0;
            if (!ek)
                for (int e = lane; e < NE * NX; e += 64) JEk[e] = 0.0;
            if (k == 0)
                for (int j = lane; j < NX; j += 64) Vs[V_LP + j] = 0.0;
            if (k + 1 >= N)
                for (int ee = lane; ee < NEA; ee += 64) Vs[V_RN + ee] = 0.0;
            // slack-row weights: D (the condensed Hessian term) and w (the J_I^T w term of the vector pass);
            // tv = p_{k+1} + P_{k+1} r_d
            if (lane < NI) {
                const int q = lane;
                double dd = 0.0, w = Vs[V_YI + q];
                if (cact(k, q)) {
                    const double sg = Vs[V_SS + q] + dw;
                    dd = sg / (1.0 + dc * sg);
                    w += dd * (Vs[V_RI + q] + (Vs[V_GS + q] - Vs[V_YI + q]) / sg);
                }
                Dd[q] = dd;
                wq[q] = w;
            } else if (lane >= 8 && lane < 8 + NX) {
                const int j = lane - 8;
                double acc = pvs[j];
                for (int l = 0; l < NX; l++) acc += Ps[j * NX + l] * Vs[V_RD + l];
                tv[j] = acc;
            }
            wave_lds_sync();
            // stage block K, feedback rows Rh, Q_xx, and the vector pass's right-hand side, one pass
            auto Hel = [&](int a, int c) __attribute__((always_inline)) -> double {  // W + J_I^T D J_I (+ diagonal)
                double v = Wl[a * NV + c];
                for (int q = 0; q < NI; q++) v += (JIl[q * NV + a] * Dd[q]) * JIl[q * NV + c];
                if (a == c) {
                    v += dw;
                    v += a < NX ? Vs[V_SX + a] : Vs[V_SU + a - NX];
                }
                return v;
            };
            for (int e = lane; e < NK * NK; e += 64) {
                const int a = e / NK, c = e % NK;
                double v = 0.0;
                if (a < NU && c < NU) {
                    if (fixs[a] || fixs[c]) v = (a == c) ? 1.0 : 0.0;
                    else {
                        v = Hel(NX + a, NX + c);
                        if (a < NX && c < NX) v += h * (Ps[a * NX + c] * h);
                    }
                } else if (a >= NU && c >= NU) {
                    v = (a == c) ? (en ? -dc : -1.0) : 0.0;
                } else {
                    const int ee = (a >= NU ? a : c) - NU, uu = a >= NU ? c : a;
                    if (!fixs[uu] && en && uu < NX) v = Jn[ee * NX + uu] * h;
                }
                Ks[a * LDK + c] = v;
            }
            for (int e = lane; e < NK * NX; e += 64) {
                const int a = e / NX, j = e % NX;
                double v = 0.0;
                if (k > 0) {
                    if (a < NU) {
                        if (!fixs[a]) {
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
                const bool fa = a < NX ? (k == 0) : (fixs[a - NX] != 0);
                if (fa) return 0.0;
                double g = GL[a];
                for (int q = 0; q < NI; q++) g += JIl[q * NV + a] * wq[q];
                if (a < NX) {
                    g += Vs[V_GX + a] - Vs[V_LP + a];
                    g += Vs[V_LK + a];  // A^T lam_k (A = I)
                    if (ek)
                        for (int ee = 0; ee < NE; ee++) g += JEk[ee * NX + a] * Vs[V_YE + ee];
                } else {
                    g += Vs[V_GU + a - NX];
                    if (a - NX < NX) g += h * Vs[V_LK + a - NX];  // B^T lam_k
                }
                return g;
            };
            if (lane >= 64 - NK) {
                const int a = lane - (64 - NK);
                double z = 0.0;
                if (a < NU) {
                    if (!fixs[a]) {
                        z = vxel(NX + a);
                        if (a < NX) z += h * tv[a];
                    }
                } else if (en) {
                    const int ee = a - NU;
                    z = Vs[V_RN + ee];
                    for (int l = 0; l < NX; l++) z += Jn[ee * NX + l] * Vs[V_RD + l];
                }
                zv[a] = z;
                Bm[a * NR + NX] = -z;
            } else if (lane >= 64 - NK - NX) {
                const int j = lane - (64 - NK - NX);
                vx[j] = vxel(j);
            }
            wave_lds_sync();
            // the stage block: natural-order pivots in registers, the pivoted LDS factorisation otherwise
            BKInertia in;
            if (!bk_factor_regs<LDK, NK>(Ks, perm, piv, in)) in = bk_factor_wave<LDK>(Ks, NK, perm, piv);
            if (in.zero) return 2;
            if (in.pos != NU || in.neg != NET) return 1;
            double *kst = Kg + (size_t)k * KSTG;
            for (int e = lane; e < NK * LDK; e += 64) kst[e] = Ks[e];
            for (int e = lane; e < NK; e += 64) { kst[NK * LDK + e] = perm[e]; kst[NK * LDK + NK + e] = piv[e]; }
            // feedback K^-1 (-Rh) and the step k_k = K^-1 (-z), one column per lane
            bk_solve_cols_lean<LDK, NR, NK>(Ks, perm, piv, Bm, NR);
            for (int e = lane; e < NK * NX; e += 64) Fg[(size_t)k * NK * NX + e] = Bm[(e / NX) * NR + e % NX];
            for (int a = lane; a < NK; a += 64) kvg[k * NK + a] = Bm[a * NR + NX];
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
        }
        return 0;
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
        return;
    }
    const double dw_c = dw, dc_c = dc;

    // forward sweep: du_k = k_k + Kf dx_k, dx_{k+1} = r_d + dx_k + h du_qd, dlam_k = p_{k+1} + P_{k+1} dx_{k+1} +
    // J_n^T dy_{k+1}
    __shared__ double dxs[NX], dxn[NX], duv[NK];
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
        if (lane < NU) fixs[lane] = ufix(k * NU + lane) ? 1 : 0;
        gsync();
        if (!en)
            for (int e = lane; e < NE * NX; e += 64) Jn[e] = 0.0;
        if (lane < NK) {
            const int a = lane;
            double acc = zv[a];
            for (int j = 0; j < NX; j++) acc += Rh[a * NX + j] * dxs[j];
            if (a < NU && fixs[a]) acc = 0.0;
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
}

}  // namespace mf
