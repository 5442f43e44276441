// Test harness (CPU): runs the device template node_fwd_rev of
// mpc_fatigue_amd/csrc/adj.hpp on the host, one tangent direction at a time,
// exactly as the GPU kernel's 2n lanes per node do (force columns derived).  Used by
// tests/test_adjoint_cpu.py to check the forward-over-reverse Hessian against
// the oracle's hyper-dual one without a GPU.  Not part of the product library.
#include <cstring>
#include <stdexcept>

#include "../../mpc_fatigue_amd/csrc/adj.hpp"
#include "../../mpc_fatigue_amd/csrc/model.hpp"

using namespace mf;

// Lanes of a q direction run TP = Dual (the angle carries the tangent), lanes of a qd direction
// TP = double (plain-FP64 pose), exactly as k_eval_node's two block classes do.
template <int NJ, class TP> struct In {
    const double *xq, *xqd;
    int v;
    Dual qd(int i) const { return Dual(xqd[i], v == NJ + i ? 1.0 : 0.0); }
    void sincos(int i, TP &s, TP &c) const {
        if constexpr (sizeof(TP) == sizeof(Dual)) {
            sincos_t(Dual(xq[i], v == i ? 1.0 : 0.0), s, c);
        } else {
            sincos_t(xq[i], s, c);
        }
    }
};

// inputs for the split q-direction sweep (node_fwd_rev_split): sincos / qd for both scalar types
template <int NJ> struct InSplit {
    const double *xq, *xqd;
    int v;
    Dual qd(int i) const { return Dual(xqd[i], 0.0); }
    void sincos(int i, double &s, double &c) const { sincos_t(xq[i], s, c); }
    void sincos(int i, Dual &s, Dual &c) const { sincos_t(Dual(xq[i], v == i ? 1.0 : 0.0), s, c); }
};

static int g_split = 0;  // 1: the q directions run node_fwd_rev_split, as k_eval_node's q class does
extern "C" void adj_set_split(int on) { g_split = on; }

template <int NJ> struct Out {
    Dual tau[NJ], gq[NJ], gqd[NJ];
    double pfv[3], pfd[3], gFd[3] = {0.0, 0.0, 0.0};
    template <class TP> void frame(const TP *p) { for (int k = 0; k < 3; k++) { pfv[k] = val(p[k]); pfd[k] = dtan(p[k]); } }
    template <class TP> void force(const TP *g) { for (int k = 0; k < 3; k++) gFd[k] = dtan(g[k]); }
    void joint(int i, const Dual &t, const Dual &a, const Dual &b) { tau[i] = t; gq[i] = a; gqd[i] = b; }
};

template <int NJ>
static void run(const DevModel &M, const DevFrame &F, int fp, int nf, const double *fdir, const double *q,
                const double *qd, const double *Fv, const double *c, const double *yl3, double *tau, double *Jt,
                double *pf, double *Jp, double *H) {
    const int nv = 2 * NJ + nf;
    double Fw[3];
    for (int k = 0; k < 3; k++) {
        double acc = 0.0;
        for (int a = 0; a < nf; a++) acc += Fv[a] * fdir[3 * a + k];
        Fw[k] = acc;
    }
    for (int v = 0; v < 2 * NJ; v++) {
        Out<NJ> o;
        if (v < NJ && g_split) {
            InSplit<NJ> in{q, qd, v};
            node_fwd_rev_split<NJ>(M, F, fp, v, in, Fw, c, yl3, o);
        } else if (v < NJ) {
            In<NJ, Dual> in{q, qd, v};
            node_fwd_rev<Dual, Dual, NJ>(M, F, fp, in, Fw, c, yl3, o);
        } else {
            // as k_eval_node's qd class: no q-gradient adjoint (GQ = false), no force row
            In<NJ, double> in{q, qd, v};
            node_fwd_rev<double, Dual, NJ, true, false>(M, F, fp, in, Fw, c, yl3, o);
        }
        for (int j = 0; j < NJ; j++) Jt[j * nv + v] = o.tau[j].d;
        if (v < NJ) {
            for (int k = 0; k < 3; k++) Jp[k * NJ + v] = o.pfd[k];
            // force column: d tau_v / dF_a = -fdir_a . dp_f/dq_v
            for (int a = 0; a < nf; a++)
                Jt[v * nv + 2 * NJ + a] = -(fdir[3 * a] * o.pfd[0] + fdir[3 * a + 1] * o.pfd[1] + fdir[3 * a + 2] * o.pfd[2]);
        }
        if (v == 0) {
            for (int j = 0; j < NJ; j++) tau[j] = o.tau[j].v;
            for (int k = 0; k < 3; k++) pf[k] = o.pfv[k];
        }
        for (int u = 0; u < NJ; u++) {
            // q rows of a qd column: from the q lanes (already run) by symmetry
            // (the split sweep computes no q rows above the diagonal: those follow by symmetry too)
            H[u * nv + v] = (v < NJ && !(g_split && u < v)) ? o.gq[u].d : H[v * nv + u];
            H[(NJ + u) * nv + v] = o.gqd[u].d;
        }
        for (int a = 0; a < nf; a++) {
            const double hv = fdir[3 * a] * o.gFd[0] + fdir[3 * a + 1] * o.gFd[1] + fdir[3 * a + 2] * o.gFd[2];
            H[(2 * NJ + a) * nv + v] = hv;
            H[v * nv + 2 * NJ + a] = hv;  // symmetry: the force columns have no lane of their own
        }
    }
    for (int a = 0; a < nf; a++)
        for (int b = 0; b < nf; b++) H[(2 * NJ + a) * nv + 2 * NJ + b] = 0.0;  // phi is linear in F
}

extern "C" int adj_node(const char *urdf, const char *frame, int nf, const double *fdir, int nl, const double *q,
                        const double *qd, const double *Fv, const double *c, const double *yl, double *tau,
                        double *Jt, double *pf, double *Jp, double *H) {
    try {
        Model m = build_model_from_urdf(urdf);
        int fid = -1;
        for (int i = 0; i < (int)m.frames.size(); i++)
            if (m.frames[i].name == frame) fid = i;
        if (fid < 0) return -3;
        DevModel M = make_dev_model(m);
        DevFrame F = make_dev_frame(m, fid);
        double yl3[3] = {0, 0, 0};
        for (int l = 0; l < nl; l++) yl3[l] = yl[l];
        const int fp = F.parent;
        switch (M.n) {
            case 3: run<3>(M, F, fp, nf, fdir, q, qd, Fv, c, yl3, tau, Jt, pf, Jp, H); break;
            case 6: run<6>(M, F, fp, nf, fdir, q, qd, Fv, c, yl3, tau, Jt, pf, Jp, H); break;
            default: return -5;
        }
        return 0;
    } catch (const std::exception &) {
        return -2;
    }
}
