// Test harness (CPU): runs the device template node_fwd_rev<Dual, n> of
// mpc_fatigue_amd/csrc/adj.hpp on the host, one tangent direction at a time,
// exactly as the GPU kernel's 13 lanes per node do.  Used by
// tests/test_adjoint_cpu.py to check the forward-over-reverse Hessian against
// the oracle's hyper-dual one without a GPU.  Not part of the product library.
#include <cstring>
#include <stdexcept>

#include "../../mpc_fatigue_amd/csrc/adj.hpp"
#include "../../mpc_fatigue_amd/csrc/model.hpp"

using namespace mf;

template <int NJ> struct In {
    const double *xq, *xqd;
    int v;
    Dual q(int i) const { return Dual(xq[i], v == i ? 1.0 : 0.0); }
    Dual qd(int i) const { return Dual(xqd[i], v == NJ + i ? 1.0 : 0.0); }
};

template <int NJ> struct Out {
    Dual tau[NJ], gq[NJ], gqd[NJ], pf[3], gF[3];
    void frame(const Dual *p) { for (int k = 0; k < 3; k++) pf[k] = p[k]; }
    void force(const Dual *g) { for (int k = 0; k < 3; k++) gF[k] = g[k]; }
    void joint(int i, const Dual &t, const Dual &a, const Dual &b) { tau[i] = t; gq[i] = a; gqd[i] = b; }
};

template <int NJ>
static void run(const DevModel &M, const DevFrame &F, int fp, int nf, const double *fdir, const double *q,
                const double *qd, const double *Fv, const double *c, const double *yl3, double *tau, double *Jt,
                double *pf, double *Jp, double *H) {
    const int nv = 2 * NJ + nf;
    for (int v = 0; v < nv; v++) {
        In<NJ> in{q, qd, v};
        Out<NJ> o;
        Dual Fw[3];
        for (int k = 0; k < 3; k++) {
            Dual acc(0.0);
            for (int a = 0; a < nf; a++) acc += Dual(Fv[a], v == 2 * NJ + a ? 1.0 : 0.0) * fdir[3 * a + k];
            Fw[k] = acc;
        }
        node_fwd_rev<Dual, NJ>(M, F, fp, in, Fw, c, yl3, o);
        for (int j = 0; j < NJ; j++) Jt[j * nv + v] = o.tau[j].d;
        if (v < NJ)
            for (int k = 0; k < 3; k++) Jp[k * NJ + v] = o.pf[k].d;
        if (v == 0) {
            for (int j = 0; j < NJ; j++) tau[j] = o.tau[j].v;
            for (int k = 0; k < 3; k++) pf[k] = o.pf[k].v;
        }
        for (int u = 0; u < NJ; u++) {
            H[u * nv + v] = o.gq[u].d;
            H[(NJ + u) * nv + v] = o.gqd[u].d;
        }
        for (int a = 0; a < nf; a++)
            H[(2 * NJ + a) * nv + v] = fdir[3 * a] * o.gF[0].d + fdir[3 * a + 1] * o.gF[1].d + fdir[3 * a + 2] * o.gF[2].d;
    }
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
