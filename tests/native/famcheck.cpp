// Test harness (CPU): builds the node record of the generic families (mpc_fatigue_amd/csrc/gfam.hpp)
// on the host with exactly the functions the device kernel k_geval runs -- the pre-pass lanes, the
// seeds, one forward-over-reverse lane per tangent direction, then every record entry -- so that
// tests/test_gfam_cpu.py can compare it with the oracle's hyper-dual restatement
// (oracle/mf_ocp.c mfg_node_derivs) without a GPU.  Not part of the product library.
#include <cstring>
#include <stdexcept>
#include <vector>

#include "../../mpc_fatigue_amd/csrc/gfam.hpp"
#include "../../mpc_fatigue_amd/csrc/model.hpp"

using namespace mf;

template <class FAM>
static void run(const DevModel *M, const DevFrame *F, const GParams &P, const double *xu, const double *yi,
                const double *ye, const double *lam, const double *lref, double *rec) {
    using D = typename FAM::D;
    typename FAM::Scratch S;
    std::memset(&S, 0, sizeof S);
    const double *x = xu, *u = xu + D::NX;
    double yev[D::NET];  // [state rows (NE) | mixed rows (NM)] -> [NEA | NM]
    for (int i = 0; i < D::NET; i++) yev[i] = 0.0;
    for (int i = 0; i < D::NE; i++) yev[i] = ye[i];
    for (int i = 0; i < D::NM; i++) yev[D::NEA + i] = ye[D::NE + i];
    for (int t = 0; t < FAM::PRE; t++) FAM::prepass(M, F, P, x, u, t, S);
    FAM::seeds(P, u, yi, yev, lam, true, 1.0, S);
    for (int t = 0; t < FAM::LANES; t++) FAM::lane(M, F, x, u, yi, t, S);
    for (int e = 0; e < D::REC; e++) rec[e] = FAM::rec(P, x, u, yi, yev, lam, true, S, e, lref);
}

static int frame_of(const Model &m, const char *name) {
    for (int i = 0; i < (int)m.frames.size(); i++)
        if (m.frames[i].name == name) return i;
    throw std::runtime_error("frame");
}

// family: 0 box (urdf0, urdf1), 1 chain 6-DOF force+line, 2 chain 6-DOF force+line+thermal,
// 3 Centauro (urdf0 / urdf1 with frames mass1_ee / mass2_ee; lref = the 6 pose targets).
// P: GParams filled by the caller (layout shared with the product's ctypes mirror).  Returns the record size.
extern "C" int fam_node_record(int family, const char *urdf0, const char *urdf1, const char *frame, const GParams *P,
                               const double *xu, const double *yi, const double *ye, const double *lam,
                               const double *lref, double *rec) {
    try {
        Model m0 = build_model_from_urdf(urdf0);
        DevModel M[2];
        DevFrame F[2];
        M[0] = make_dev_model(m0);
        F[0] = make_dev_frame(m0, frame_of(m0, frame));
        if (family == 0) {
            Model m1 = build_model_from_urdf(urdf1);
            M[1] = make_dev_model(m1);
            F[1] = make_dev_frame(m1, frame_of(m1, frame));
            run<BoxFam>(M, F, *P, xu, yi, ye, lam, lref, rec);
            return BoxFam::D::REC;
        }
        if (family == 4) {
            Model m1 = build_model_from_urdf(urdf1);
            M[1] = make_dev_model(m1);
            F[1] = make_dev_frame(m1, frame_of(m1, frame));
            run<BoxThermFam>(M, F, *P, xu, yi, ye, lam, lref, rec);
            return BoxThermFam::D::REC;
        }
        if (family == 3) {
            Model m1 = build_model_from_urdf(urdf1);
            M[0] = make_dev_model(m0);
            F[0] = make_dev_frame(m0, frame_of(m0, "mass1_ee"));
            M[1] = make_dev_model(m1);
            F[1] = make_dev_frame(m1, frame_of(m1, "mass2_ee"));
            run<CentauroFam>(M, F, *P, xu, yi, ye, lam, lref, rec);
            return CentauroFam::D::REC;
        }
        if (family == 1) {
            run<ChainFam<6, 1, 2, false>>(M, F, *P, xu, yi, ye, lam, lref, rec);
            return ChainFam<6, 1, 2, false>::D::REC;
        }
        if (family == 2) {
            run<ChainFam<6, 1, 2, true>>(M, F, *P, xu, yi, ye, lam, lref, rec);
            return ChainFam<6, 1, 2, true>::D::REC;
        }
        return -5;
    } catch (const std::exception &) {
        return -2;
    }
}

extern "C" int fam_gparams_size(void) { return (int)sizeof(GParams); }
