// Op-counted FP64 work of one node evaluation (tests/test_flopcount_cpu.py, bench.py's
// roofline.fp64).  The device's node sweeps (mpc_fatigue_amd/csrc/adj.hpp: fwd_range / rev_range, templated
// on the pose and velocity scalar types) are instantiated on the host with counting scalars that perform the
// same arithmetic as the device's types and add up the FP64 operations they execute:
//   CD   ~ double  (one op per +, -, *; a division 1)
//   CDu  ~ Dual    (value + tangent, built on CD: Dual*Dual = 3 mul + 1 add = the device's mul + fma (2) + mul,
//                   Dual*double = 2 mul, Dual+double = 1 add -- the device's zero-tangent shortcuts)
// and run exactly the lanes k_eval_q / k_eval_node<..,1> run per node: for each q direction v the split
// sweep (plain FP64 forward below joint v, Dual from v on, qd-class reverse below v), for each qd direction
// the q-gradient-free sweep; sin / cos are counted apart (the q lanes read them from LDS, computed once per
// node).  Not part of the product library.  Arithmetic on model constants alone (the per-joint axis
// products of the reverse sweep) is plain double in adj.hpp and not counted: a few dozen ops per lane.
#include <cmath>
#include <stdexcept>

#include "../../mpc_fatigue_amd/csrc/model.hpp"

namespace mf {
static long long g_ops = 0, g_trans = 0;
struct CD {
    double x;
    CD() : x(0) {}
    CD(double v) : x(v) {}
};
inline CD operator+(CD a, CD b) { g_ops++; return CD(a.x + b.x); }
inline CD operator-(CD a, CD b) { g_ops++; return CD(a.x - b.x); }
inline CD operator*(CD a, CD b) { g_ops++; return CD(a.x * b.x); }
inline CD operator-(CD a) { return CD(-a.x); }
inline CD operator+(CD a, double b) { g_ops++; return CD(a.x + b); }
inline CD operator+(double a, CD b) { g_ops++; return CD(a + b.x); }
inline CD operator-(CD a, double b) { g_ops++; return CD(a.x - b); }
inline CD operator-(double a, CD b) { g_ops++; return CD(a - b.x); }
inline CD operator*(CD a, double b) { g_ops++; return CD(a.x * b); }
inline CD operator*(double a, CD b) { g_ops++; return CD(a * b.x); }
inline CD &operator+=(CD &a, CD b) { a = a + b; return a; }
inline CD &operator-=(CD &a, CD b) { a = a - b; return a; }
inline CD &operator+=(CD &a, double b) { a = a + b; return a; }
inline CD &operator-=(CD &a, double b) { a = a - b; return a; }

struct CDu {
    CD v, d;
    CDu() {}
    CDu(double a) : v(a), d(0.0) {}
    CDu(CD a) : v(a), d(0.0) {}
    CDu(CD a, CD b) : v(a), d(b) {}
};
inline CDu operator+(CDu a, CDu b) { return CDu(a.v + b.v, a.d + b.d); }
inline CDu operator-(CDu a, CDu b) { return CDu(a.v - b.v, a.d - b.d); }
inline CDu operator-(CDu a) { return CDu(-a.v, -a.d); }
inline CDu operator*(CDu a, CDu b) { return CDu(a.v * b.v, a.v * b.d + a.d * b.v); }
// with a plain (zero-tangent) operand: the device's Dual shortcuts
inline CDu operator*(CDu a, CD s) { return CDu(a.v * s, a.d * s); }
inline CDu operator*(CD s, CDu a) { return CDu(a.v * s, a.d * s); }
inline CDu operator*(CDu a, double s) { return CDu(a.v * s, a.d * s); }
inline CDu operator*(double s, CDu a) { return CDu(a.v * s, a.d * s); }
inline CDu operator+(CDu a, CD b) { return CDu(a.v + b, a.d); }
inline CDu operator+(CD a, CDu b) { return CDu(a + b.v, b.d); }
inline CDu operator-(CDu a, CD b) { return CDu(a.v - b, a.d); }
inline CDu operator-(CD a, CDu b) { return CDu(a - b.v, -b.d); }
inline CDu operator+(CDu a, double b) { return CDu(a.v + b, a.d); }
inline CDu operator+(double a, CDu b) { return CDu(a + b.v, b.d); }
inline CDu operator-(CDu a, double b) { return CDu(a.v - b, a.d); }
inline CDu operator-(double a, CDu b) { return CDu(a - b.v, -b.d); }
inline CDu &operator+=(CDu &a, CDu b) { a = a + b; return a; }
inline CDu &operator-=(CDu &a, CDu b) { a = a - b; return a; }
inline CDu &operator+=(CDu &a, CD b) { a = a + b; return a; }
inline CDu &operator-=(CDu &a, CD b) { a = a - b; return a; }
inline CDu &operator+=(CDu &a, double b) { a = a + b; return a; }
inline CDu &operator-=(CDu &a, double b) { a = a - b; return a; }

inline double val(CD x) { return x.x; }
inline double val(CDu x) { return x.v.x; }
inline double dtan(CD) { return 0.0; }
inline double dtan(CDu x) { return x.d.x; }
}  // namespace mf

#include "../../mpc_fatigue_amd/csrc/adj.hpp"

using namespace mf;

namespace {
// inputs as k_eval_q / k_eval_node read them: sin / cos per node from LDS (counted apart), the q tangent
// applied as the device's NodeIn does (s = (sv, cv t), c = (cv, -sv t): 2 mul)
template <int NJ> struct CIn {
    const double *xq, *xqd;
    int v;
    CDu qd(int i) const { return CDu(CD(xqd[i]), CD(v == NJ + i ? 1.0 : 0.0)); }
    void sincos(int i, CD &s, CD &c) const { s = CD(std::sin(xq[i])); c = CD(std::cos(xq[i])); }
    void sincos(int i, CDu &s, CDu &c) const {
        const double sv = std::sin(xq[i]), cv = std::cos(xq[i]);
        const CD t(v == i ? 1.0 : 0.0);
        s = CDu(CD(sv), CD(cv) * t);
        c = CDu(CD(cv), CD(-sv) * t);
    }
};
struct CEmit {
    template <class TP> void frame(const TP *) {}
    template <class TP> void force(const TP *) {}
    template <class A, class B, class C2> void joint(int, const A &, const B &, const C2 &) {}
};

template <int NJ>
void count(const DevModel &M, const DevFrame &F, const double *q, const double *qd, const double *Fw, const double *c,
           const double *yl, long long *qlanes, long long *qdlanes) {
    CEmit em;
    const int fp = F.parent;
    for (int v = 0; v < NJ; v++) {  // node_fwd_rev_split with the counting types
        g_ops = 0;
        CIn<NJ> in{q, qd, v};
        SweepState<CD, CD> S0;
        sweep_init(M, S0);
        fwd_range<CD, CD, NJ, true>(M, 0, v, in, c, S0);
        SweepState<CDu, CDu> S1;
        for (int k = 0; k < 9; k++) S1.R[k] = CDu(S0.R[k]);
        for (int k = 0; k < 3; k++) {
            S1.o[k] = CDu(S0.o[k]); S1.Lz[k] = CDu(S0.Lz[k]); S1.Loz[k] = CDu(S0.Loz[k]);
            S1.w[k] = CDu(S0.w[k]); S1.dw[k] = CDu(S0.dw[k]); S1.a[k] = CDu(S0.a[k]);
            S1.Mt[k] = CDu(0.0); S1.Ft[k] = CDu(0.0); S1.wb[k] = CDu(0.0); S1.dwb[k] = CDu(0.0);
            S1.ab[k] = CDu(0.0); S1.G[k] = CDu(0.0); S1.Ob[k] = CDu(0.0);
        }
        fwd_range<CDu, CDu, NJ, true>(M, v, NJ, in, c, S1);
        rev_range<CDu, CDu, NJ, true, true>(M, F, fp, NJ - 1, v, in, Fw, c, yl, em, S1);
        if (v > 0) {
            SweepState<CD, CDu> S2;
            for (int k = 0; k < 9; k++) S2.R[k] = S1.R[k].v;
            for (int k = 0; k < 3; k++) {
                S2.o[k] = S1.o[k].v; S2.Lz[k] = S1.Lz[k].v; S2.Loz[k] = S1.Loz[k].v;
                S2.w[k] = S1.w[k]; S2.dw[k] = S1.dw[k]; S2.a[k] = S1.a[k];
                S2.Mt[k] = S1.Mt[k]; S2.Ft[k] = S1.Ft[k]; S2.wb[k] = S1.wb[k]; S2.dwb[k] = S1.dwb[k];
                S2.ab[k] = S1.ab[k]; S2.G[k] = S1.G[k]; S2.Ob[k] = S1.Ob[k];
            }
            rev_range<CD, CDu, NJ, true, false>(M, F, fp, v - 1, 0, in, Fw, c, yl, em, S2);
        }
        qlanes[v] = g_ops;
    }
    for (int v = NJ; v < 2 * NJ; v++) {  // qd class: node_fwd_rev<double, Dual, NJ, true, false>
        g_ops = 0;
        CIn<NJ> in{q, qd, v};
        SweepState<CD, CDu> S;
        sweep_init(M, S);
        fwd_range<CD, CDu, NJ, true>(M, 0, NJ, in, c, S);
        rev_range<CD, CDu, NJ, true, false>(M, F, fp, NJ - 1, 0, in, Fw, c, yl, em, S);
        qdlanes[v - NJ] = g_ops;
    }
}
}  // namespace

// ops[0..n): q lanes, ops[n..2n): qd lanes; returns the joint count or < 0
extern "C" int flop_node(const char *urdf, const char *frame, const double *q, const double *qd, const double *Fw,
                         const double *c, const double *yl3, long long *ops) {
    try {
        Model m = build_model_from_urdf(urdf);
        int fid = -1;
        for (int i = 0; i < (int)m.frames.size(); i++)
            if (m.frames[i].name == frame) fid = i;
        if (fid < 0) return -3;
        DevModel M = make_dev_model(m);
        DevFrame F = make_dev_frame(m, fid);
        switch (M.n) {
            case 3: count<3>(M, F, q, qd, Fw, c, yl3, ops, ops + 3); break;
            case 6: count<6>(M, F, q, qd, Fw, c, yl3, ops, ops + 6); break;
            default: return -5;
        }
        return M.n;
    } catch (const std::exception &) {
        return -2;
    }
}
