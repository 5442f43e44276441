// ORACLE-side CPU baseline helper (not the checker): the product's node functions
// (mpc_fatigue_amd/csrc/gfam.hpp -- forward-over-reverse lanes of adj.hpp plus closed-form assembly)
// compiled for the host, exposed as the node-record provider of the generic oracle IPM
// (oracle/mf_ocp.c, mfg_opts.node_cb).  bench.py's cpu_baseline leg uses it so that the CPU figure is
// the same algorithm with efficient derivatives, not the hyper-dual restatement.  Tests compare it
// with the hyper-dual records (tests/test_gfam_cpu.py covers the same functions).
#include <cstring>
#include <new>
#include <stdexcept>

#include "../mpc_fatigue_amd/csrc/gfam.hpp"
#include "../mpc_fatigue_amd/csrc/model.hpp"

using namespace mf;

namespace {
struct Ctx {
    int family;
    DevModel M[2];
    DevFrame F[2];
    GParams P;
};

template <class FAM>
int record(const Ctx *c, const double *xu, const double *yi, const double *ye, const double *lam, const double *lref,
           int eqon, double *rec) {
    using D = typename FAM::D;
    typename FAM::Scratch S;
    std::memset(&S, 0, sizeof S);
    const double *x = xu, *u = xu + D::NX;
    // the oracle passes ye = [state rows (NE) | mixed rows (NM)]; the families read [NEA | NM]
    double yev[D::NET];
    for (int i = 0; i < D::NET; i++) yev[i] = 0.0;
    for (int i = 0; i < D::NE; i++) yev[i] = ye[i];
    for (int i = 0; i < D::NM; i++) yev[D::NEA + i] = ye[D::NE + i];
    const double *tg = lref;  // line reference (chain) or the 6 pose targets (Centauro)
    for (int t = 0; t < FAM::PRE; t++) FAM::prepass(c->M, c->F, c->P, x, u, t, S);
    FAM::seeds(c->P, u, yi, yev, lam, eqon != 0, 1.0, S);
    for (int t = 0; t < FAM::LANES; t++) FAM::lane(c->M, c->F, x, u, yi, t, S);
    for (int e = 0; e < D::REC; e++) rec[e] = FAM::rec(c->P, x, u, yi, yev, lam, eqon != 0, S, e, tg);
    return D::REC;
}

int frame_of(const Model &m, const char *name) {
    for (int i = 0; i < (int)m.frames.size(); i++)
        if (m.frames[i].name == name) return i;
    throw std::runtime_error("unknown frame");
}
}  // namespace

// family: 0 box, 1 chain 6-DOF force + line, 2 the same with thermal state, 3 Centauro (two 7-DOF arms),
// 4 box with thermal state and shared fatigue budget
extern "C" void *mfc_create(int family, const char *urdf0, const char *urdf1, const char *frame0, const char *frame1,
                            const GParams *P) {
    try {
        Ctx *c = new Ctx();
        c->family = family;
        Model m0 = build_model_from_urdf(urdf0);
        c->M[0] = make_dev_model(m0);
        c->F[0] = make_dev_frame(m0, frame_of(m0, frame0));
        if (family == 0 || family == 3 || family == 4) {
            Model m1 = build_model_from_urdf(urdf1);
            c->M[1] = make_dev_model(m1);
            c->F[1] = make_dev_frame(m1, frame_of(m1, frame1));
        } else {
            c->M[1] = c->M[0];
            c->F[1] = c->F[0];
        }
        c->P = *P;
        return c;
    } catch (const std::exception &) {
        return nullptr;
    }
}

extern "C" void mfc_free(void *ctx) { delete static_cast<Ctx *>(ctx); }

extern "C" int mfc_node(void *ctx, const double *xu, const double *yi, const double *ye, const double *lam,
                        const double *lref, int eqon, double *rec) {
    const Ctx *c = static_cast<const Ctx *>(ctx);
    switch (c->family) {
        case 0: return record<BoxFam>(c, xu, yi, ye, lam, lref, eqon, rec);
        case 1: return record<ChainFam<6, 1, 2, false>>(c, xu, yi, ye, lam, lref, eqon, rec);
        case 2: return record<ChainFam<6, 1, 2, true>>(c, xu, yi, ye, lam, lref, eqon, rec);
        case 3: return record<CentauroFam>(c, xu, yi, ye, lam, lref, eqon, rec);
        case 4: return record<BoxThermFam>(c, xu, yi, ye, lam, lref, eqon, rec);
    }
    return -5;
}

template <class FAM>
int values(const Ctx *c, const double *x, const double *u, const double *lref, double *l, double *ci, double *ce,
           double *f) {
    double ce0[16];
    FAM::values(c->M, c->F, c->P, x, u, lref, *l, ci, FAM::D::NE + FAM::D::NM > 0 ? ce : ce0, f);
    return 0;
}

extern "C" int mfc_values(void *ctx, const double *x, const double *u, const double *lref, double *l, double *ci,
                          double *ce, double *f) {
    const Ctx *c = static_cast<const Ctx *>(ctx);
    switch (c->family) {
        case 0: return values<BoxFam>(c, x, u, lref, l, ci, ce, f);
        case 1: return values<ChainFam<6, 1, 2, false>>(c, x, u, lref, l, ci, ce, f);
        case 2: return values<ChainFam<6, 1, 2, true>>(c, x, u, lref, l, ci, ce, f);
        case 3: return values<CentauroFam>(c, x, u, lref, l, ci, ce, f);
        case 4: return values<BoxThermFam>(c, x, u, lref, l, ci, ce, f);
    }
    return -5;
}

extern "C" int mfc_gparams_size(void) { return (int)sizeof(GParams); }
