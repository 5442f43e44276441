// extern "C" ABI of libmpcfatigue.so (declared in include/mpcfatigue.h).
//
// Host side: URDF ingestion (urdf.cpp), device model images, problem objects
// and the batched solve driver.  Device side: the bridge kernels below
// (inverse dynamics / FK / frame Jacobian, one lane per sample) and the
// interior-point kernels in ipm_kernels.hip.  There is no CPU compute path:
// without a usable device every compute entry point fails with MF_ERR_DEVICE.
#include <hip/hip_runtime.h>

#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <exception>
#include <string>
#include <vector>

#include "dyn.hpp"
#include "ipm.hpp"
#include "model.hpp"

namespace mf {
bool ipm_dispatch(int n, int nf, int nl, int what, const DevModel *M, const DevFrame *F, const OcpConst &C,
                  const IpmArrays &A, int batch, int nact, hipStream_t s, double *w, int *status, int *iters,
                  double *kkt, double *obj);
}

using namespace mf;

static thread_local std::string g_err;
static int fail(int code, const std::string &msg) {
    g_err = msg;
    return code;
}
extern "C" const char *mf_last_error(void) { return g_err.c_str(); }

#define HIPCHK(x)                                                                                     \
    do {                                                                                              \
        hipError_t e_ = (x);                                                                          \
        if (e_ != hipSuccess) return fail(MF_ERR_DEVICE, std::string("HIP error: ") + hipGetErrorString(e_) + " at " #x); \
    } while (0)

static int ensure_device() {
    int n = 0;
    hipError_t e = hipGetDeviceCount(&n);
    if (e != hipSuccess || n == 0) return fail(MF_ERR_DEVICE, "no HIP device available (libmpcfatigue has no CPU path)");
    return MF_OK;
}

struct mf_model {
    Model host;
    DevModel dev;
    DevModel *d_model = nullptr;
    std::vector<DevFrame *> d_frames;  // lazily uploaded
};

static int upload_model(mf_model *m) {
    if (m->d_model) return MF_OK;
    int e = ensure_device();
    if (e) return e;
    HIPCHK(hipMalloc(&m->d_model, sizeof(DevModel)));
    HIPCHK(hipMemcpy(m->d_model, &m->dev, sizeof(DevModel), hipMemcpyHostToDevice));
    m->d_frames.assign(m->host.frames.size(), nullptr);
    return MF_OK;
}
static int frame_dev(mf_model *m, int frame, DevFrame **out) {
    int e = upload_model(m);
    if (e) return e;
    if (frame < 0 || frame >= (int)m->host.frames.size()) return fail(MF_ERR_FRAME, "frame index out of range");
    if (!m->d_frames[frame]) {
        DevFrame F = make_dev_frame(m->host, frame);
        HIPCHK(hipMalloc(&m->d_frames[frame], sizeof(DevFrame)));
        HIPCHK(hipMemcpy(m->d_frames[frame], &F, sizeof F, hipMemcpyHostToDevice));
    }
    *out = m->d_frames[frame];
    return MF_OK;
}

// ---- internal entry points for the generic solver (csrc/capi_internal.hpp)
namespace mf {
int capi_fail(int code, const std::string &msg) { return fail(code, msg); }
int capi_model_dev(mf_model *m, const DevModel **dev, const Model **host) {
    int e = upload_model(m);
    if (e) return e;
    if (dev) *dev = m->d_model;
    if (host) *host = &m->host;
    return MF_OK;
}
int capi_frame_dev(mf_model *m, int frame, DevFrame **out) { return frame_dev(m, frame, out); }
int capi_ensure_device() { return ensure_device(); }
}  // namespace mf

extern "C" int mf_model_from_urdf(const char *urdf_xml, mf_model **out) {
    if (!urdf_xml || !out) return fail(MF_ERR_ARG, "null argument");
    try {
        mf_model *m = new mf_model();
        m->host = build_model_from_urdf(urdf_xml);
        m->dev = make_dev_model(m->host);
        *out = m;
        return MF_OK;
    } catch (const std::exception &ex) {
        return fail(MF_ERR_URDF, ex.what());
    }
}

extern "C" void mf_model_free(mf_model *m) {
    if (!m) return;
    if (m->d_model) (void)hipFree(m->d_model);
    for (auto *f : m->d_frames)
        if (f) (void)hipFree(f);
    delete m;
}

extern "C" int mf_model_nq(const mf_model *m) { return m ? (int)m->host.joints.size() : MF_ERR_ARG; }

extern "C" int mf_model_export(const mf_model *m, double *blob, int cap) {
    if (!m) return fail(MF_ERR_ARG, "null model");
    int n = (int)m->host.joints.size();
    int need = MF_BLOB_HDR + MF_BLOB_JSTRIDE * n;
    std::vector<double> b(need, 0.0);
    b[0] = n;
    for (int k = 0; k < 3; k++) b[1 + k] = m->host.gravity[k];
    for (int j = 0; j < n; j++) {
        const Joint &J = m->host.joints[j];
        double *o = b.data() + MF_BLOB_HDR + MF_BLOB_JSTRIDE * j;
        o[0] = J.parent;
        memcpy(o + 1, J.R, 9 * sizeof(double));
        memcpy(o + 10, J.t, 3 * sizeof(double));
        memcpy(o + 13, J.axis, 3 * sizeof(double));
        o[16] = J.mass;
        memcpy(o + 17, J.com, 3 * sizeof(double));
        memcpy(o + 20, J.Ic, 9 * sizeof(double));
        o[29] = J.lower; o[30] = J.upper; o[31] = J.effort; o[32] = J.velocity;
    }
    if (blob) memcpy(blob, b.data(), sizeof(double) * (size_t)(cap < need ? cap : need));
    return need;
}

extern "C" int mf_frame_id(const mf_model *m, const char *name) {
    if (!m || !name) return fail(MF_ERR_ARG, "null argument");
    for (size_t i = 0; i < m->host.frames.size(); i++)
        if (m->host.frames[i].name == name) return (int)i;
    return fail(MF_ERR_FRAME, std::string("unknown frame '") + name + "'");
}

extern "C" int mf_frame_export(const mf_model *m, int frame, double *rec13) {
    if (!m || !rec13) return fail(MF_ERR_ARG, "null argument");
    if (frame < 0 || frame >= (int)m->host.frames.size()) return fail(MF_ERR_FRAME, "frame index out of range");
    const Frame &f = m->host.frames[frame];
    rec13[0] = f.parent;
    memcpy(rec13 + 1, f.R, 9 * sizeof(double));
    memcpy(rec13 + 10, f.t, 3 * sizeof(double));
    return MF_OK;
}

// ====================================================================== bridge kernels
// One lane per sample; runtime n <= MF_MAX_JOINTS (these are the drop-in numeric calls,
// not the solver hot loop).
template <int NJ>
__global__ __launch_bounds__(256) void k_bridge_id(const DevModel *__restrict__ Mg, const double *q, const double *qd,
                                                   const double *qdd, double *tau, int batch) {
    __shared__ DevModel M;
    {
        const double *s = reinterpret_cast<const double *>(Mg);
        double *d = reinterpret_cast<double *>(&M);
        for (int i = threadIdx.x; i < (int)(sizeof(DevModel) / sizeof(double)); i += blockDim.x) d[i] = s[i];
    }
    __syncthreads();
    int b = blockIdx.x * blockDim.x + threadIdx.x;
    if (b >= batch) return;
    const int n = M.n;
    double xq[NJ], xqd[NJ], xqdd[NJ];
    for (int i = 0; i < n; i++) { xq[i] = q[b * n + i]; xqd[i] = qd[b * n + i]; xqdd[i] = qdd[b * n + i]; }
    TotVis<double> tv;
    tv.F = nullptr;
    tv.init();
    ne_pass<double>(M, n, xq, xqd, xqdd, tv);
    EmitVis<double, NJ> ev;
    ev.tot = &tv;
    ev.fp = -1;
    for (int k = 0; k < 3; k++) ev.Fw[k] = 0.0;
    ev.init();
    ne_pass<double>(M, n, xq, xqd, xqdd, ev);
    for (int i = 0; i < n; i++) tau[b * n + i] = ev.tau[i];
}

template <int NJ>
__global__ __launch_bounds__(256) void k_bridge_kin(const DevModel *__restrict__ Mg, const DevFrame *__restrict__ Fg,
                                                    const double *q, double *pos, double *rot, double *J, int batch) {
    __shared__ DevModel M;
    __shared__ DevFrame F;
    {
        const double *s = reinterpret_cast<const double *>(Mg);
        double *d = reinterpret_cast<double *>(&M);
        for (int i = threadIdx.x; i < (int)(sizeof(DevModel) / sizeof(double)); i += blockDim.x) d[i] = s[i];
        const double *s2 = reinterpret_cast<const double *>(Fg);
        double *d2 = reinterpret_cast<double *>(&F);
        for (int i = threadIdx.x; i < (int)(sizeof(DevFrame) / sizeof(double)); i += blockDim.x) d2[i] = s2[i];
    }
    __syncthreads();
    int b = blockIdx.x * blockDim.x + threadIdx.x;
    if (b >= batch) return;
    const int n = M.n;
    double xq[NJ], zero[NJ];
    for (int i = 0; i < n; i++) { xq[i] = q[b * n + i]; zero[i] = 0.0; }
    JacVis<double, NJ> jv;
    jv.F = &F;
    if (F.parent < 0) {
        for (int k = 0; k < 3; k++) jv.pf[k] = F.t[k];
        for (int k = 0; k < 9; k++) jv.Rf[k] = F.R[k];
    }
    ne_pass<double>(M, n, xq, zero, (const double *)nullptr, jv);
    if (pos)
        for (int k = 0; k < 3; k++) pos[b * 3 + k] = jv.pf[k];
    if (rot)
        for (int r = 0; r < 3; r++)
            for (int c = 0; c < 3; c++) rot[b * 9 + c * 3 + r] = jv.Rf[r * 3 + c];
    if (J) {
        double *Jb = J + (size_t)b * 6 * n;
        for (int j = 0; j < n; j++) {
            bool anc = false;
            for (int a = F.parent; a >= 0; a = M.j[a].parent)
                if (a == j) { anc = true; break; }
            double lin[3] = {0, 0, 0}, ang[3] = {0, 0, 0};
            if (anc) {
                double d[3] = {jv.pf[0] - jv.o[j][0], jv.pf[1] - jv.o[j][1], jv.pf[2] - jv.o[j][2]};
                cross3(lin, jv.z[j], d);
                for (int k = 0; k < 3; k++) ang[k] = jv.z[j][k];
            }
            for (int k = 0; k < 3; k++) { Jb[j * 6 + k] = lin[k]; Jb[j * 6 + 3 + k] = ang[k]; }
        }
    }
}

static int check_serial(const mf_model *m) {
    if (!m->dev.serial) return fail(MF_ERR_UNSUPPORTED, "branching kinematic trees are not supported by the kernels yet");
    return MF_OK;
}

extern "C" int mf_id_dev(const mf_model *mc, const double *q, const double *qd, const double *qdd, double *tau,
                         int batch, void *stream) {
    mf_model *m = const_cast<mf_model *>(mc);
    if (!m || batch < 0) return fail(MF_ERR_ARG, "bad argument");
    int e = check_serial(m);
    if (e) return e;
    if ((e = upload_model(m))) return e;
    if (batch == 0) return MF_OK;
    hipLaunchKernelGGL(k_bridge_id<MF_MAX_JOINTS>, dim3((batch + 255) / 256), dim3(256), 0, (hipStream_t)stream,
                       m->d_model, q, qd, qdd, tau, batch);
    HIPCHK(hipGetLastError());
    return MF_OK;
}

static int kin_dev(const mf_model *mc, int frame, const double *q, double *pos, double *rot, double *J, int batch,
                   void *stream) {
    mf_model *m = const_cast<mf_model *>(mc);
    if (!m || batch < 0) return fail(MF_ERR_ARG, "bad argument");
    int e = check_serial(m);
    if (e) return e;
    DevFrame *F;
    if ((e = frame_dev(m, frame, &F))) return e;
    if (batch == 0) return MF_OK;
    hipLaunchKernelGGL(k_bridge_kin<MF_MAX_JOINTS>, dim3((batch + 255) / 256), dim3(256), 0, (hipStream_t)stream,
                       m->d_model, F, q, pos, rot, J, batch);
    HIPCHK(hipGetLastError());
    return MF_OK;
}
extern "C" int mf_fk_dev(const mf_model *m, int frame, const double *q, double *pos3, double *rot9, int batch,
                         void *stream) {
    return kin_dev(m, frame, q, pos3, rot9, nullptr, batch, stream);
}
extern "C" int mf_jac_dev(const mf_model *m, int frame, const double *q, double *J, int batch, void *stream) {
    return kin_dev(m, frame, q, nullptr, nullptr, J, batch, stream);
}

// ====================================================================== batched IK
// The reference solves min ||fk(q) - p||^2 with IPOPT from q = 0 once per script
// (force_optimization_pilz_6DOF.py:55-63, Box_Pilz_6DOF.py:123-156).  Here one lane per target
// runs damped least squares on the frame position: e = p - fk(q), (J J^T + lam I) y = e
// (3 x 3 Cholesky), dq = J^T y, the step capped at max_step in the max norm so the iterate
// stays on the branch nearest its start; stop at |e| < tol.  Same iteration as the fixture
// generator tests/golden/make_fixtures.py:ik (numpy), which pins it.
template <int NJ>
__global__ __launch_bounds__(256) void k_ik(const DevModel *__restrict__ Mg, const DevFrame *__restrict__ Fg,
                                            const double *target, const double *q_init, double *q_out,
                                            double *residual, int batch, int iters, double lam, double max_step,
                                            double tol) {
    __shared__ DevModel M;
    __shared__ DevFrame F;
    {
        const double *s = reinterpret_cast<const double *>(Mg);
        double *d = reinterpret_cast<double *>(&M);
        for (int i = threadIdx.x; i < (int)(sizeof(DevModel) / sizeof(double)); i += blockDim.x) d[i] = s[i];
        const double *s2 = reinterpret_cast<const double *>(Fg);
        double *d2 = reinterpret_cast<double *>(&F);
        for (int i = threadIdx.x; i < (int)(sizeof(DevFrame) / sizeof(double)); i += blockDim.x) d2[i] = s2[i];
    }
    __syncthreads();
    const int b = blockIdx.x * blockDim.x + threadIdx.x;
    if (b >= batch) return;
    const int n = M.n;
    double q[NJ], zero[NJ];
    for (int i = 0; i < n; i++) { q[i] = q_init ? q_init[b * n + i] : 0.0; zero[i] = 0.0; }
    const double t0 = target[3 * b], t1 = target[3 * b + 1], t2 = target[3 * b + 2];
    double en = INFINITY;
    for (int it = 0; it <= iters; it++) {
        JacVis<double, NJ> jv;
        jv.F = &F;
        if (F.parent < 0) {
            for (int k = 0; k < 3; k++) jv.pf[k] = F.t[k];
            for (int k = 0; k < 9; k++) jv.Rf[k] = F.R[k];
        }
        ne_pass<double>(M, n, q, zero, (const double *)nullptr, jv);
        const double e[3] = {t0 - jv.pf[0], t1 - jv.pf[1], t2 - jv.pf[2]};
        en = sqrt(e[0] * e[0] + e[1] * e[1] + e[2] * e[2]);
        if (en < tol || it == iters) break;
        // position Jacobian columns: z_j x (p - o_j) for the frame's ancestors
        double Jc[NJ][3];
        for (int j = 0; j < n; j++) {
            bool anc = false;
            for (int a = F.parent; a >= 0; a = M.j[a].parent)
                if (a == j) { anc = true; break; }
            double d[3] = {jv.pf[0] - jv.o[j][0], jv.pf[1] - jv.o[j][1], jv.pf[2] - jv.o[j][2]};
            double c[3];
            cross3(c, jv.z[j], d);
            for (int k = 0; k < 3; k++) Jc[j][k] = anc ? c[k] : 0.0;
        }
        double A[3][3];
        for (int r = 0; r < 3; r++)
            for (int c = 0; c < 3; c++) {
                double a = (r == c) ? lam : 0.0;
                for (int j = 0; j < n; j++) a += Jc[j][r] * Jc[j][c];
                A[r][c] = a;
            }
        // Cholesky of the SPD 3 x 3 system
        const double l00 = sqrt(A[0][0]), l10 = A[1][0] / l00, l20 = A[2][0] / l00;
        const double l11 = sqrt(A[1][1] - l10 * l10), l21 = (A[2][1] - l20 * l10) / l11;
        const double l22 = sqrt(A[2][2] - l20 * l20 - l21 * l21);
        const double z0 = e[0] / l00, z1 = (e[1] - l10 * z0) / l11, z2 = (e[2] - l20 * z0 - l21 * z1) / l22;
        const double y2 = z2 / l22, y1 = (z1 - l21 * y2) / l11, y0 = (z0 - l10 * y1 - l20 * y2) / l00;
        double dq[NJ], step = 0.0;
        for (int j = 0; j < n; j++) {
            dq[j] = Jc[j][0] * y0 + Jc[j][1] * y1 + Jc[j][2] * y2;
            step = fmax(step, fabs(dq[j]));
        }
        const double sc = (step > max_step) ? max_step / step : 1.0;
        for (int j = 0; j < n; j++) q[j] += dq[j] * sc;
    }
    for (int i = 0; i < n; i++) q_out[b * n + i] = q[i];
    if (residual) residual[b] = en;
}

extern "C" int mf_ik_batch_dev(const mf_model *mc, int frame, const double *target, const double *q_init,
                               double *q_out, double *residual, int batch, int iters, double lam, double max_step,
                               double tol, void *stream) {
    mf_model *m = const_cast<mf_model *>(mc);
    if (!m || !target || !q_out || batch < 0 || iters < 0 || !(lam > 0.0) || !(max_step > 0.0))
        return fail(MF_ERR_ARG, "bad argument");
    int e = check_serial(m);
    if (e) return e;
    DevFrame *F;
    if ((e = frame_dev(m, frame, &F))) return e;
    if (batch == 0) return MF_OK;
    hipLaunchKernelGGL(k_ik<MF_MAX_JOINTS>, dim3((batch + 255) / 256), dim3(256), 0, (hipStream_t)stream, m->d_model,
                       F, target, q_init, q_out, residual, batch, iters, lam, max_step, tol);
    HIPCHK(hipGetLastError());
    return MF_OK;
}

// host-pointer wrappers: stage through device buffers
struct DBuf {
    double *p = nullptr;
    ~DBuf() { if (p) (void)hipFree(p); }
};
struct IBuf {
    int *p = nullptr;
    ~IBuf() { if (p) (void)hipFree(p); }
};
// a host-path call's own stream (destroyed on every return path)
struct OwnStream {
    hipStream_t s = nullptr;
    ~OwnStream() { if (s) { (void)hipStreamSynchronize(s); (void)hipStreamDestroy(s); } }
};
static int dalloc(DBuf &b, size_t n) {
    HIPCHK(hipMalloc(&b.p, (n ? n : 1) * sizeof(double)));
    return MF_OK;
}
// upload: on `s` when given (ordered before the launches on that stream by the stream itself), else the
// blocking copy the single-stream bridge functions use
static int h2d(DBuf &b, const double *h, size_t n, hipStream_t s = nullptr) {
    int e = dalloc(b, n);
    if (e) return e;
    if (n && s) HIPCHK(hipMemcpyAsync(b.p, h, n * sizeof(double), hipMemcpyHostToDevice, s));
    else if (n) HIPCHK(hipMemcpy(b.p, h, n * sizeof(double), hipMemcpyHostToDevice));
    return MF_OK;
}

extern "C" int mf_id(const mf_model *m, const double *q, const double *qd, const double *qdd, double *tau, int batch) {
    if (!m || !q || !qd || !qdd || !tau || batch < 0) return fail(MF_ERR_ARG, "null argument");
    int e = ensure_device();
    if (e) return e;
    size_t n = (size_t)m->host.joints.size() * batch;
    DBuf a, b, c, t;
    if ((e = h2d(a, q, n)) || (e = h2d(b, qd, n)) || (e = h2d(c, qdd, n)) || (e = dalloc(t, n))) return e;
    if ((e = mf_id_dev(m, a.p, b.p, c.p, t.p, batch, nullptr))) return e;
    HIPCHK(hipMemcpy(tau, t.p, n * sizeof(double), hipMemcpyDeviceToHost));
    return MF_OK;
}
extern "C" int mf_fk(const mf_model *m, int frame, const double *q, double *pos3, double *rot9, int batch) {
    if (!m || !q || batch < 0) return fail(MF_ERR_ARG, "null argument");
    int e = ensure_device();
    if (e) return e;
    size_t n = (size_t)m->host.joints.size() * batch;
    DBuf a, p, r;
    if ((e = h2d(a, q, n)) || (e = dalloc(p, 3 * (size_t)batch)) || (e = dalloc(r, 9 * (size_t)batch))) return e;
    if ((e = mf_fk_dev(m, frame, a.p, p.p, r.p, batch, nullptr))) return e;
    if (pos3) HIPCHK(hipMemcpy(pos3, p.p, 3 * (size_t)batch * sizeof(double), hipMemcpyDeviceToHost));
    if (rot9) HIPCHK(hipMemcpy(rot9, r.p, 9 * (size_t)batch * sizeof(double), hipMemcpyDeviceToHost));
    return MF_OK;
}
extern "C" int mf_jac(const mf_model *m, int frame, const double *q, double *J, int batch) {
    if (!m || !q || !J || batch < 0) return fail(MF_ERR_ARG, "null argument");
    int e = ensure_device();
    if (e) return e;
    size_t n = (size_t)m->host.joints.size() * batch;
    DBuf a, j;
    if ((e = h2d(a, q, n)) || (e = dalloc(j, 6 * n))) return e;
    if ((e = mf_jac_dev(m, frame, a.p, j.p, batch, nullptr))) return e;
    HIPCHK(hipMemcpy(J, j.p, 6 * n * sizeof(double), hipMemcpyDeviceToHost));
    return MF_OK;
}

extern "C" int mf_ik_batch(const mf_model *m, int frame, const double *target, const double *q_init, double *q_out,
                           double *residual, int batch, int iters, double lam, double max_step, double tol) {
    if (!m || !target || !q_out || batch < 0) return fail(MF_ERR_ARG, "null argument");
    int e = ensure_device();
    if (e) return e;
    size_t n = (size_t)m->host.joints.size() * batch;
    DBuf t, qi, qo, r;
    if ((e = h2d(t, target, 3 * (size_t)batch)) || (e = dalloc(qo, n)) || (e = dalloc(r, (size_t)batch))) return e;
    if (q_init && (e = h2d(qi, q_init, n))) return e;
    if ((e = mf_ik_batch_dev(m, frame, t.p, q_init ? qi.p : nullptr, qo.p, r.p, batch, iters, lam, max_step, tol,
                             nullptr)))
        return e;
    HIPCHK(hipMemcpy(q_out, qo.p, n * sizeof(double), hipMemcpyDeviceToHost));
    if (residual) HIPCHK(hipMemcpy(residual, r.p, (size_t)batch * sizeof(double), hipMemcpyDeviceToHost));
    return MF_OK;
}

// ====================================================================== problems
struct mf_problem {
    mf_model *model;
    mf_problem_spec spec;
    std::vector<double> tau_lo, tau_hi;
    OcpConst C;
    DevFrame *d_frame = nullptr;
    double *d_tlo = nullptr, *d_thi = nullptr;
    // per-kernel timing (HIP events on the solve stream), enabled by mf_problem_timing
    int timing = 0;
    std::vector<hipEvent_t> ev;
    double t_ms[MF_NKERNELS] = {0};
    long t_launch[MF_NKERNELS] = {0};
    // solver workspace (grown on demand)
    int cap = 0;
    std::vector<double *> bufs;
    IpmArrays A;
    ProbState *d_st = nullptr;
    int *d_active = nullptr;
    int *d_list = nullptr;  // compacted running set (batch) + its count
    // per-chunk trace of the last timed solve: (iteration, running count, GPU ms of the chunk)
    std::vector<int> tr_iter, tr_run;
    std::vector<double> tr_ms;
};

static void free_ws(mf_problem *p) {
    for (double *b : p->bufs) (void)hipFree(b);
    p->bufs.clear();
    if (p->d_st) (void)hipFree(p->d_st);
    if (p->d_active) (void)hipFree(p->d_active);
    if (p->d_list) (void)hipFree(p->d_list);
    p->d_st = nullptr;
    p->d_active = nullptr;
    p->d_list = nullptr;
    p->cap = 0;
}

extern "C" int mf_problem_create(const mf_model *mc, const mf_problem_spec *spec, mf_problem **out) {
    mf_model *m = const_cast<mf_model *>(mc);
    if (!m || !spec || !out) return fail(MF_ERR_ARG, "null argument");
    int n = (int)m->host.joints.size();
    if (spec->N < 1 || spec->h <= 0) return fail(MF_ERR_ARG, "N >= 1 and h > 0 required");
    if (spec->nf < 0 || spec->nf > 3) return fail(MF_ERR_ARG, "nf must be 0..3");
    if (spec->frame < 0 || spec->frame >= (int)m->host.frames.size()) return fail(MF_ERR_FRAME, "frame index out of range");
    if (!spec->tau_lo || !spec->tau_hi) return fail(MF_ERR_ARG, "tau bounds required");
    int e = check_serial(m);
    if (e) return e;
    int nl = spec->use_line ? 2 : 0;
    if (!((n == 3 && spec->nf == 0 && nl == 0) || (n == 6 && spec->nf == 1 && nl == 2) || (n == 6 && spec->nf == 0 && nl == 0)))
        return fail(MF_ERR_UNSUPPORTED, "no kernel instantiation for (n, nf, nl) = (" + std::to_string(n) + ", " +
                                            std::to_string(spec->nf) + ", " + std::to_string(nl) + ")");
    mf_problem *p = new mf_problem();
    p->model = m;
    p->spec = *spec;
    size_t nb = (size_t)spec->N * n;
    p->tau_lo.assign(spec->tau_lo, spec->tau_lo + nb);
    p->tau_hi.assign(spec->tau_hi, spec->tau_hi + nb);
    p->spec.tau_lo = p->tau_lo.data();
    p->spec.tau_hi = p->tau_hi.data();
    OcpConst &C = p->C;
    memset(&C, 0, sizeof C);
    C.N = spec->N; C.n = n; C.nf = spec->nf; C.nl = nl;
    C.nv = 2 * n + spec->nf;
    C.mb = 3 * n + spec->nf + nl;
    C.npair = C.nv * (C.nv + 1) / 2;
    C.h = spec->h;
    memcpy(C.fdir, spec->fdir, sizeof C.fdir);
    C.wF = spec->wF; C.wqd = spec->wqd; C.wtau = spec->wtau;
    memcpy(C.qd0, spec->qd0, sizeof C.qd0);
    memcpy(C.qd_lo, spec->qd_lo, sizeof C.qd_lo);
    memcpy(C.qd_hi, spec->qd_hi, sizeof C.qd_hi);
    memcpy(C.q_lo, spec->q_lo, sizeof C.q_lo);
    memcpy(C.q_hi, spec->q_hi, sizeof C.q_hi);
    *out = p;
    return MF_OK;
}

extern "C" void mf_problem_free(mf_problem *p) {
    if (!p) return;
    free_ws(p);
    for (auto e : p->ev) (void)hipEventDestroy(e);
    if (p->d_tlo) (void)hipFree(p->d_tlo);
    if (p->d_thi) (void)hipFree(p->d_thi);
    delete p;
}

extern "C" int mf_problem_wsize(const mf_problem *p) {
    if (!p) return fail(MF_ERR_ARG, "null problem");
    return p->C.n + p->C.N * (2 * p->C.n + p->C.nf);
}

// s: the solve's stream.  The workspace is zeroed on it, so the solve's kernels are ordered after the
// zeroing (a hipMemset on the legacy null stream is asynchronous and does not order a non-blocking stream:
// a first solve on a torch stream then raced it).
static int ensure_ws(mf_problem *p, int batch, hipStream_t s) {
    int e = upload_model(p->model);
    if (e) return e;
    if (!p->d_frame && (e = frame_dev(p->model, p->spec.frame, &p->d_frame))) return e;
    const OcpConst &C = p->C;
    size_t nb = (size_t)C.N * C.n;
    if (!p->d_tlo) {
        HIPCHK(hipMalloc(&p->d_tlo, nb * sizeof(double)));
        HIPCHK(hipMalloc(&p->d_thi, nb * sizeof(double)));
        HIPCHK(hipMemcpy(p->d_tlo, p->tau_lo.data(), nb * sizeof(double), hipMemcpyHostToDevice));
        HIPCHK(hipMemcpy(p->d_thi, p->tau_hi.data(), nb * sizeof(double), hipMemcpyHostToDevice));
    }
    if (p->cap >= batch) return MF_OK;
    free_ws(p);
    IpmSizes S = ipm_sizes(C);
    IpmArrays &A = p->A;
    struct Item { double **ptr; size_t n; };
    Item items[] = {
        {&A.q, S.q}, {&A.qd, S.u}, {&A.F, S.f}, {&A.s, S.u}, {&A.yc, S.u}, {&A.yl, S.l}, {&A.yd, S.u},
        {&A.zqL, S.q}, {&A.zqU, S.q}, {&A.zdL, S.u}, {&A.zdU, S.u}, {&A.vL, S.u}, {&A.vU, S.u},
        {&A.dq, S.q}, {&A.dqd, S.u}, {&A.dF, S.f}, {&A.ds, S.u}, {&A.dyc, S.u}, {&A.dyl, S.l}, {&A.dyd, S.u},
        {&A.dzqL, S.q}, {&A.dzqU, S.q}, {&A.dzdL, S.u}, {&A.dzdU, S.u}, {&A.dvL, S.u}, {&A.dvU, S.u},
        {&A.tau, S.u}, {&A.Jt, S.jt}, {&A.line, S.l}, {&A.Jl, S.jl}, {&A.W, S.w}, {&A.gf, S.gf}, {&A.cost, S.cost},
        {&A.Sxq, S.q}, {&A.gphq, S.q}, {&A.Sxd, S.u}, {&A.gphd, S.u}, {&A.Ss, S.u}, {&A.gphs, S.u},
        {&A.G, S.G}, {&A.wv, S.wv}, {&A.stg, S.stg}, {&A.q0, (size_t)C.n}, {&A.lref, 2},
    };
    for (auto &it : items) {
        double *ptr = nullptr;
        hipError_t he = hipMalloc(&ptr, it.n * (size_t)batch * sizeof(double));
        if (he != hipSuccess) {
            free_ws(p);
            return fail(MF_ERR_NOMEM, std::string("workspace allocation failed: ") + hipGetErrorString(he));
        }
        p->bufs.push_back(ptr);
        *it.ptr = ptr;
        HIPCHK(hipMemsetAsync(ptr, 0, it.n * (size_t)batch * sizeof(double), s));
    }
    HIPCHK(hipMalloc(&p->d_st, sizeof(ProbState) * (size_t)batch));
    HIPCHK(hipMalloc(&p->d_active, sizeof(int)));
    HIPCHK(hipMalloc(&p->d_list, sizeof(int) * ((size_t)batch + 1)));
    A.st = p->d_st;
    A.active = p->d_active;
    A.list = p->d_list;
    A.nrun = p->d_list + batch;
    A.tau_lo = p->d_tlo;
    A.tau_hi = p->d_thi;
    p->cap = batch;
    return MF_OK;
}

static int solve_core(mf_problem *p, int batch, const double *d_q0, const double *d_qd0, const double *d_w0,
                      const double *d_lref, const mf_solver_opts *o,
                      double *d_w, int *d_status, int *d_iters, double *d_kkt, double *d_obj, hipStream_t s) {
    int e = ensure_ws(p, batch, s);
    if (e) return e;
    OcpConst C = p->C;
    C.tol = o ? o->tol : 1e-8;
    C.constr_viol_tol = o ? o->constr_viol_tol : 1e-8;
    C.max_iter = o ? o->max_iter : 200;
    C.mu_init = o ? o->mu_init : 0.1;
    C.F_init = o ? o->F_init : 0.0;
    C.warm_start = (o && d_w0) ? o->warm_start : 0;
    IpmArrays A = p->A;
    A.qd0p = d_qd0;
    A.w0 = d_w0;
    const int n = C.n;
    HIPCHK(hipMemcpyAsync(A.q0, d_q0, sizeof(double) * n * (size_t)batch, hipMemcpyDeviceToDevice, s));
    if (d_lref) {
        HIPCHK(hipMemcpyAsync(A.lref, d_lref, sizeof(double) * 2 * (size_t)batch, hipMemcpyDeviceToDevice, s));
    } else {
        std::vector<double> lr(2 * (size_t)batch);
        for (int b = 0; b < batch; b++) { lr[2 * b] = p->spec.line_ref[0]; lr[2 * b + 1] = p->spec.line_ref[1]; }
        HIPCHK(hipMemcpyAsync(A.lref, lr.data(), sizeof(double) * lr.size(), hipMemcpyHostToDevice, s));
        HIPCHK(hipStreamSynchronize(s));
    }
    HIPCHK(hipMemcpyAsync(A.active, &batch, sizeof(int), hipMemcpyHostToDevice, s));
    DevFrame *F = p->d_frame;
    if (!ipm_dispatch(n, C.nf, C.nl, 0, p->model->d_model, F, C, A, batch, batch, s, nullptr, nullptr, nullptr, nullptr,
                      nullptr))
        return fail(MF_ERR_UNSUPPORTED, "no kernel instantiation");
    HIPCHK(hipGetLastError());
    int active = batch;
    const int chunk = 4, NPH = 5;  // launches per iteration: k_eval_node, k_eval_asm, k_ipm_pre, k_ipm_kkt, k_ipm_post
    if (p->timing && p->ev.size() < (size_t)(2 * NPH * chunk)) {
        for (auto e2 : p->ev) (void)hipEventDestroy(e2);
        p->ev.assign(2 * NPH * chunk, nullptr);
        for (auto &e2 : p->ev) HIPCHK(hipEventCreate(&e2));
    }
    if (p->timing) {
        p->tr_iter.clear();
        p->tr_run.clear();
        p->tr_ms.clear();
    }
    for (int it = 0; it <= C.max_iter && active > 0; it += chunk) {
        const int run_before = active;
        for (int c = 0; c < chunk; c++)
            for (int ph = 0; ph < NPH; ph++) {
                if (p->timing) HIPCHK(hipEventRecord(p->ev[(c * NPH + ph) * 2], s));
                ipm_dispatch(n, C.nf, C.nl, 10 + ph, p->model->d_model, F, C, A, batch, active, s, nullptr, nullptr,
                             nullptr, nullptr, nullptr);
                if (p->timing) HIPCHK(hipEventRecord(p->ev[(c * NPH + ph) * 2 + 1], s));
            }
        HIPCHK(hipGetLastError());
        HIPCHK(hipMemcpyAsync(&active, A.active, sizeof(int), hipMemcpyDeviceToHost, s));
        HIPCHK(hipStreamSynchronize(s));
        if (p->timing) {
            double chunk_ms = 0.0;
            for (int c = 0; c < chunk; c++)
                for (int ph = 0; ph < NPH; ph++) {
                    float ms = 0;
                    HIPCHK(hipEventElapsedTime(&ms, p->ev[(c * NPH + ph) * 2], p->ev[(c * NPH + ph) * 2 + 1]));
                    p->t_ms[ph] += ms;
                    p->t_launch[ph]++;
                    chunk_ms += ms;
                }
            p->tr_iter.push_back(it);
            p->tr_run.push_back(run_before);
            p->tr_ms.push_back(chunk_ms);
        }
        if (o && o->verbose) {
            static thread_local std::chrono::steady_clock::time_point t_start;
            if (it == 0) t_start = std::chrono::steady_clock::now();
            const double ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t_start).count();
            fprintf(stderr, "[mf] after %d iterations: %d running  t=%.2f ms\n", it + chunk, active, ms);
        }
    }
    ipm_dispatch(n, C.nf, C.nl, 2, p->model->d_model, F, C, A, batch, batch, s, d_w, d_status, d_iters, d_kkt, d_obj);
    HIPCHK(hipGetLastError());
    return MF_OK;
}

extern "C" int mf_solve_batch_dev(mf_problem *p, int batch, const double *q0, const double *line_ref,
                                  const mf_solver_opts *opts, double *w, int *status, int *iters, double *kkt,
                                  double *obj, void *stream) {
    if (!p || !q0 || !w || batch < 1) return fail(MF_ERR_ARG, "bad argument");
    int e = ensure_device();
    if (e) return e;
    return solve_core(p, batch, q0, nullptr, nullptr, line_ref, opts, w, status, iters, kkt, obj, (hipStream_t)stream);
}

static int solve_host(mf_problem *p, int batch, const double *q0, const double *qd0, const double *w0,
                      const double *line_ref, const mf_solver_opts *opts, double *w, int *status, int *iters,
                      double *kkt, double *obj, int device) {
    if (!p || !q0 || !w || batch < 1) return fail(MF_ERR_ARG, "bad argument");
    int e = ensure_device();
    if (e) return e;
    HIPCHK(hipSetDevice(device));
    const int n = p->C.n, ws = mf_problem_wsize(p);
    DBuf dq0, dqd0, dw0, dl, dw, dk, dob;
    IBuf dst, dit;
    // a stream of this call's own: uploads, solve and copies back are ordered on it and synchronise with
    // it alone, so host calls on other handles / streams of the device keep running (reentrant)
    OwnStream os;
    HIPCHK(hipStreamCreateWithFlags(&os.s, hipStreamNonBlocking));
    if ((e = h2d(dq0, q0, (size_t)n * batch, os.s))) return e;
    if (qd0 && (e = h2d(dqd0, qd0, (size_t)n * batch, os.s))) return e;
    if (w0 && (e = h2d(dw0, w0, (size_t)ws * batch, os.s))) return e;
    if (line_ref && (e = h2d(dl, line_ref, 2 * (size_t)batch, os.s))) return e;
    if ((e = dalloc(dw, (size_t)ws * batch)) || (e = dalloc(dk, batch)) || (e = dalloc(dob, batch))) return e;
    HIPCHK(hipMalloc(&dst.p, sizeof(int) * batch));
    HIPCHK(hipMalloc(&dit.p, sizeof(int) * batch));
    e = solve_core(p, batch, dq0.p, dqd0.p, dw0.p, line_ref ? dl.p : nullptr, opts, dw.p, dst.p, dit.p, dk.p, dob.p,
                   os.s);
    if (e) return e;
    HIPCHK(hipMemcpyAsync(w, dw.p, sizeof(double) * ws * (size_t)batch, hipMemcpyDeviceToHost, os.s));
    if (status) HIPCHK(hipMemcpyAsync(status, dst.p, sizeof(int) * batch, hipMemcpyDeviceToHost, os.s));
    if (iters) HIPCHK(hipMemcpyAsync(iters, dit.p, sizeof(int) * batch, hipMemcpyDeviceToHost, os.s));
    if (kkt) HIPCHK(hipMemcpyAsync(kkt, dk.p, sizeof(double) * batch, hipMemcpyDeviceToHost, os.s));
    if (obj) HIPCHK(hipMemcpyAsync(obj, dob.p, sizeof(double) * batch, hipMemcpyDeviceToHost, os.s));
    HIPCHK(hipStreamSynchronize(os.s));
    return MF_OK;
}
extern "C" int mf_solve_batch(mf_problem *p, int batch, const double *q0, const double *line_ref,
                              const mf_solver_opts *opts, double *w, int *status, int *iters, double *kkt, double *obj,
                              int device) {
    return solve_host(p, batch, q0, nullptr, nullptr, line_ref, opts, w, status, iters, kkt, obj, device);
}
extern "C" int mf_solve_batch_ws(mf_problem *p, int batch, const double *q0, const double *qd0, const double *w0,
                                 const double *line_ref, const mf_solver_opts *opts, double *w, int *status,
                                 int *iters, double *kkt, double *obj, int device) {
    return solve_host(p, batch, q0, qd0, w0, line_ref, opts, w, status, iters, kkt, obj, device);
}
extern "C" int mf_solve_batch_ws_dev(mf_problem *p, int batch, const double *q0, const double *qd0, const double *w0,
                                     const double *line_ref, const mf_solver_opts *opts, double *w, int *status,
                                     int *iters, double *kkt, double *obj, void *stream) {
    if (!p || !q0 || !w || batch < 1) return fail(MF_ERR_ARG, "bad argument");
    if (w0 && w0 == w) return fail(MF_ERR_ARG, "w0 and w must not alias (w is written while w0 is read)");
    int e = ensure_device();
    if (e) return e;
    return solve_core(p, batch, q0, qd0, w0, line_ref, opts, w, status, iters, kkt, obj, (hipStream_t)stream);
}

// ====================================================================== node evaluation
template <int NJ, int NF>
__global__ __launch_bounds__(256) void k_node_eval(const DevModel *__restrict__ Mg, const DevFrame *__restrict__ Fg,
                                                   OcpConst C, const double *x, const double *uu, const double *lref,
                                                   double dl0, double dl1, double *xnext, double *g, double *cost,
                                                   double *jac, int nodes) {
    __shared__ DevModel M;
    __shared__ DevFrame F;
    {
        const double *s = reinterpret_cast<const double *>(Mg);
        double *d = reinterpret_cast<double *>(&M);
        for (int i = threadIdx.x; i < (int)(sizeof(DevModel) / sizeof(double)); i += blockDim.x) d[i] = s[i];
        const double *s2 = reinterpret_cast<const double *>(Fg);
        double *d2 = reinterpret_cast<double *>(&F);
        for (int i = threadIdx.x; i < (int)(sizeof(DevFrame) / sizeof(double)); i += blockDim.x) d2[i] = s2[i];
    }
    __syncthreads();
    constexpr int NV = 2 * NJ + NF;
    constexpr int NFA = NF > 0 ? NF : 1;
    long t = (long)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= (long)nodes * NV) return;
    const int col = (int)(t % NV);
    const int r = (int)(t / NV);
    const int nl = C.nl, nrow = 2 * NJ + nl + 1;
    const double *q = x + (size_t)r * NJ, *u = uu + (size_t)r * (NJ + NF);
    Dual xq[NJ], xqd[NJ], xF[NFA], tau[NJ], pf[3];
    for (int i = 0; i < NJ; i++) {
        xq[i] = Dual(q[i], col == i ? 1.0 : 0.0);
        xqd[i] = Dual(u[i], col == NJ + i ? 1.0 : 0.0);
    }
    for (int a = 0; a < NFA; a++) xF[a] = Dual(NF > 0 ? u[NJ + a] : 0.0, col == 2 * NJ + a ? 1.0 : 0.0);
    node_tau<Dual, NJ>(M, F, NF, C.fdir, xq, xqd, xF, tau, pf);
    Dual c(0.0);
    for (int a = 0; a < NF; a++) c += xF[a] * xF[a] * C.wF;
    for (int j = 0; j < NJ; j++) c += xqd[j] * xqd[j] * C.wqd + tau[j] * tau[j] * C.wtau;
    double *J = jac + (size_t)r * nrow * NV + (size_t)col * nrow;  // column-major per node
    for (int j = 0; j < NJ; j++) J[j] = (col == j ? 1.0 : 0.0) + (col == NJ + j ? C.h : 0.0);
    for (int j = 0; j < NJ; j++) J[NJ + j] = tau[j].d;
    for (int l = 0; l < nl; l++) J[2 * NJ + l] = pf[l].d;
    J[2 * NJ + nl] = c.d;
    if (col == 0) {
        for (int j = 0; j < NJ; j++) xnext[(size_t)r * NJ + j] = q[j] + C.h * u[j];
        for (int j = 0; j < NJ; j++) g[(size_t)r * (NJ + nl) + j] = tau[j].v;
        for (int l = 0; l < nl; l++) {
            double ref = lref ? lref[(size_t)r * 2 + l] : (l == 0 ? dl0 : dl1);
            g[(size_t)r * (NJ + nl) + NJ + l] = pf[l].v - ref;
        }
        cost[r] = c.v;
    }
}

extern "C" int mf_node_eval(const mf_problem *pc, const double *x, const double *u, const double *line_ref,
                            double *xnext, double *g, double *cost, double *jac, int nodes) {
    mf_problem *p = const_cast<mf_problem *>(pc);
    if (!p || !x || !u || !xnext || !g || !cost || !jac || nodes < 0) return fail(MF_ERR_ARG, "null argument");
    int e = ensure_device();
    if (e) return e;
    if ((e = upload_model(p->model))) return e;
    if (!p->d_frame && (e = frame_dev(p->model, p->spec.frame, &p->d_frame))) return e;
    if (nodes == 0) return MF_OK;
    const OcpConst &C = p->C;
    const int n = C.n, nf = C.nf, nl = C.nl, nv = C.nv, nrow = 2 * n + nl + 1;
    DBuf dx, du, dl, dxn, dg, dc, dj;
    if ((e = h2d(dx, x, (size_t)n * nodes)) || (e = h2d(du, u, (size_t)(n + nf) * nodes))) return e;
    if (line_ref && (e = h2d(dl, line_ref, 2 * (size_t)nodes))) return e;
    if ((e = dalloc(dxn, (size_t)n * nodes)) || (e = dalloc(dg, (size_t)(n + nl) * nodes)) || (e = dalloc(dc, nodes)) ||
        (e = dalloc(dj, (size_t)nrow * nv * nodes)))
        return e;
    long total = (long)nodes * nv;
    dim3 grid((unsigned)((total + 255) / 256)), blk(256);
    const double *lr = line_ref ? dl.p : nullptr;
    if (n == 6 && nf == 1)
        hipLaunchKernelGGL((k_node_eval<6, 1>), grid, blk, 0, 0, p->model->d_model, p->d_frame, C, dx.p, du.p, lr,
                           p->spec.line_ref[0], p->spec.line_ref[1], dxn.p, dg.p, dc.p, dj.p, nodes);
    else if (n == 6 && nf == 0)
        hipLaunchKernelGGL((k_node_eval<6, 0>), grid, blk, 0, 0, p->model->d_model, p->d_frame, C, dx.p, du.p, lr,
                           p->spec.line_ref[0], p->spec.line_ref[1], dxn.p, dg.p, dc.p, dj.p, nodes);
    else if (n == 3 && nf == 0)
        hipLaunchKernelGGL((k_node_eval<3, 0>), grid, blk, 0, 0, p->model->d_model, p->d_frame, C, dx.p, du.p, lr,
                           p->spec.line_ref[0], p->spec.line_ref[1], dxn.p, dg.p, dc.p, dj.p, nodes);
    else
        return fail(MF_ERR_UNSUPPORTED, "no node-eval instantiation for this problem");
    HIPCHK(hipGetLastError());
    HIPCHK(hipStreamSynchronize(0));  // the launch's own (null) stream, not every stream of the device
    HIPCHK(hipMemcpy(xnext, dxn.p, sizeof(double) * n * (size_t)nodes, hipMemcpyDeviceToHost));
    HIPCHK(hipMemcpy(g, dg.p, sizeof(double) * (n + nl) * (size_t)nodes, hipMemcpyDeviceToHost));
    HIPCHK(hipMemcpy(cost, dc.p, sizeof(double) * (size_t)nodes, hipMemcpyDeviceToHost));
    HIPCHK(hipMemcpy(jac, dj.p, sizeof(double) * nrow * nv * (size_t)nodes, hipMemcpyDeviceToHost));
    return MF_OK;
}

extern "C" int mf_problem_timing(mf_problem *p, int enable) {
    if (!p) return fail(MF_ERR_ARG, "null problem");
    p->timing = enable ? 1 : 0;
    for (int k = 0; k < MF_NKERNELS; k++) { p->t_ms[k] = 0; p->t_launch[k] = 0; }
    return MF_OK;
}

extern "C" const char *mf_kernel_name(int slot) {
    static const char *names[MF_NKERNELS] = {"k_eval_node", "k_eval_asm", "k_ipm_pre", "k_ipm_kkt", "k_ipm_post"};
    return (slot >= 0 && slot < MF_NKERNELS) ? names[slot] : "";
}

extern "C" int mf_problem_trace(const mf_problem *p, int *iter, int *running, double *ms, int cap) {
    if (!p) return fail(MF_ERR_ARG, "null problem");
    const int n = (int)p->tr_iter.size();
    for (int i = 0; i < n && i < cap; i++) {
        if (iter) iter[i] = p->tr_iter[i];
        if (running) running[i] = p->tr_run[i];
        if (ms) ms[i] = p->tr_ms[i];
    }
    return n;
}

extern "C" int mf_problem_kernel_stats(const mf_problem *p, double *ms_total3, long *launches3) {
    if (!p || !ms_total3 || !launches3) return fail(MF_ERR_ARG, "null argument");
    for (int k = 0; k < MF_NKERNELS; k++) { ms_total3[k] = p->t_ms[k]; launches3[k] = p->t_launch[k]; }
    return MF_OK;
}

#ifdef MF_TRACE
// Diagnostic build only: copy `count` doubles of one solver array (problem 0 first) to the host.
// which: 0 q 1 qd 2 F 3 s 4 yc 5 yl 6 yd 7 zqL 8 zqU 9 zdL 10 zdU 11 vL 12 vU 13 tau 14 Jt
//        15 Jl 16 W 17 gf 18 line 19 cost
extern "C" int mf_debug_array(const mf_problem *p, int which, double *out, long count) {
    const IpmArrays &A = p->A;
    double *src[20] = {A.q, A.qd, A.F, A.s, A.yc, A.yl, A.yd, A.zqL, A.zqU, A.zdL, A.zdU, A.vL, A.vU,
                       A.tau, A.Jt, A.Jl, A.W, A.gf, A.line, A.cost};
    if (which < 0 || which >= 20 || !src[which]) return -1;
    return hipMemcpy(out, src[which], sizeof(double) * count, hipMemcpyDeviceToHost) == hipSuccess ? 0 : -1;
}
#endif

