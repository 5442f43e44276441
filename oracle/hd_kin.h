/*
 * ORACLE — test infrastructure only.  Hyper-dual scalar, model blob and the
 * world-frame kinematics / Newton-Euler restatement shared by mf_oracle.c (the
 * Pilz-specialised IPM) and mf_ocp.c (the generic stage-structured IPM).
 * Restates pinocchio::rnea / framesForwardKinematics / getFrameJacobian as the
 * reference's bridge traces them (src/casadi_pinocchio_bridge.hpp:57-153).
 */
#ifndef MF_HD_KIN_H
#define MF_HD_KIN_H
#include <math.h>
#include <string.h>
#define MJ 16                 /* max joints */
#define BLOB_HDR 4
#define BLOB_JSTRIDE 33

typedef struct {
    int n;
    int parent[MJ];
    double RX[MJ][9], tX[MJ][3], axis[MJ][3];
    double m[MJ], c[MJ][3], Ic[MJ][9];
    double g[3];
} mfo_model;

/* ------------------------------------------------------------------ */
/* hyper-dual scalar                                                   */
typedef struct { double a, b, c, d; } hd;

static inline hd K(double x) { hd r = {x, 0, 0, 0}; return r; }
static inline hd add(hd x, hd y) { hd r = {x.a + y.a, x.b + y.b, x.c + y.c, x.d + y.d}; return r; }
static inline hd sub(hd x, hd y) { hd r = {x.a - y.a, x.b - y.b, x.c - y.c, x.d - y.d}; return r; }
static inline hd mul(hd x, hd y) {
    hd r = {x.a * y.a, x.a * y.b + x.b * y.a, x.a * y.c + x.c * y.a,
            x.a * y.d + x.b * y.c + x.c * y.b + x.d * y.a};
    return r;
}
static inline hd muls(hd x, double s) { hd r = {x.a * s, x.b * s, x.c * s, x.d * s}; return r; }
static inline hd hsin(hd x) {
    double s = sin(x.a), c = cos(x.a);
    hd r = {s, c * x.b, c * x.c, c * x.d - s * x.b * x.c};
    return r;
}
static inline hd hcos(hd x) {
    double s = sin(x.a), c = cos(x.a);
    hd r = {c, -s * x.b, -s * x.c, -s * x.d - c * x.b * x.c};
    return r;
}

static void cross3(hd *o, const hd *a, const hd *b) {
    hd t0 = sub(mul(a[1], b[2]), mul(a[2], b[1]));
    hd t1 = sub(mul(a[2], b[0]), mul(a[0], b[2]));
    hd t2 = sub(mul(a[0], b[1]), mul(a[1], b[0]));
    o[0] = t0; o[1] = t1; o[2] = t2;
}
static hd dot3(const hd *a, const hd *b) { return add(add(mul(a[0], b[0]), mul(a[1], b[1])), mul(a[2], b[2])); }
static void mv3(hd *o, const hd *R, const hd *v) { /* o = R v, R row-major */
    hd t[3];
    for (int i = 0; i < 3; i++) t[i] = add(add(mul(R[3 * i], v[0]), mul(R[3 * i + 1], v[1])), mul(R[3 * i + 2], v[2]));
    memcpy(o, t, sizeof t);
}
static void mtv3(hd *o, const hd *R, const hd *v) { /* o = R^T v */
    hd t[3];
    for (int i = 0; i < 3; i++) t[i] = add(add(mul(R[i], v[0]), mul(R[3 + i], v[1])), mul(R[6 + i], v[2]));
    memcpy(o, t, sizeof t);
}
static void mvc3(hd *o, const hd *R, const double *v) {
    for (int i = 0; i < 3; i++)
        o[i] = add(add(muls(R[3 * i], v[0]), muls(R[3 * i + 1], v[1])), muls(R[3 * i + 2], v[2]));
}
static void mmc3(hd *o, const hd *A, const double *B) { /* o = A B, B constant */
    for (int i = 0; i < 3; i++)
        for (int j = 0; j < 3; j++)
            o[3 * i + j] = add(add(muls(A[3 * i], B[j]), muls(A[3 * i + 1], B[3 + j])), muls(A[3 * i + 2], B[6 + j]));
}
static void mm3(hd *o, const hd *A, const hd *B) {
    hd t[9];
    for (int i = 0; i < 3; i++)
        for (int j = 0; j < 3; j++)
            t[3 * i + j] = add(add(mul(A[3 * i], B[j]), mul(A[3 * i + 1], B[3 + j])), mul(A[3 * i + 2], B[6 + j]));
    memcpy(o, t, sizeof t);
}

/* ------------------------------------------------------------------ */
/* model blob <-> struct (blob layout documented in include/mpcfatigue.h) */
static int mfo_model_from_blob(const double *blob, mfo_model *M) {
    int n = (int)blob[0];
    if (n < 1 || n > MJ) return -1;
    memset(M, 0, sizeof *M);
    M->n = n;
    M->g[0] = blob[1]; M->g[1] = blob[2]; M->g[2] = blob[3];
    for (int j = 0; j < n; j++) {
        const double *b = blob + BLOB_HDR + BLOB_JSTRIDE * j;
        M->parent[j] = (int)b[0];
        if (M->parent[j] >= j) return -2; /* topological order required */
        memcpy(M->RX[j], b + 1, 9 * sizeof(double));
        memcpy(M->tX[j], b + 10, 3 * sizeof(double));
        memcpy(M->axis[j], b + 13, 3 * sizeof(double));
        M->m[j] = b[16];
        memcpy(M->c[j], b + 17, 3 * sizeof(double));
        memcpy(M->Ic[j], b + 20, 9 * sizeof(double));
    }
    return 0;
}

typedef struct { int parent; double R[9], t[3]; } mfo_frame;

static void frame_from_arr(const double *f, mfo_frame *F) {
    F->parent = (int)f[0];
    memcpy(F->R, f + 1, 9 * sizeof(double));
    memcpy(F->t, f + 10, 3 * sizeof(double));
}

/* ------------------------------------------------------------------ */
/* world-frame kinematics + Newton-Euler (revolute joints)            */
typedef struct { hd R[MJ][9], o[MJ][3], z[MJ][3]; } kin_t;

static void kinematics(const mfo_model *M, const hd *q, kin_t *Kn) {
    for (int i = 0; i < M->n; i++) {
        int p = M->parent[i];
        hd A[9], o[3];
        if (p < 0) {
            for (int k = 0; k < 9; k++) A[k] = K(M->RX[i][k]);
            for (int k = 0; k < 3; k++) o[k] = K(M->tX[i][k]);
        } else {
            mmc3(A, Kn->R[p], M->RX[i]);
            mvc3(o, Kn->R[p], M->tX[i]);
            for (int k = 0; k < 3; k++) o[k] = add(o[k], Kn->o[p][k]);
        }
        mvc3(Kn->z[i], A, M->axis[i]);
        memcpy(Kn->o[i], o, sizeof o);
        /* joint rotation Rot(axis,q) = I + s [a] + (1-c) [a]^2 */
        const double *a = M->axis[i];
        double Sk[9] = {0, -a[2], a[1], a[2], 0, -a[0], -a[1], a[0], 0};
        double S2[9];
        for (int r = 0; r < 3; r++)
            for (int cc = 0; cc < 3; cc++)
                S2[3 * r + cc] = Sk[3 * r] * Sk[cc] + Sk[3 * r + 1] * Sk[3 + cc] + Sk[3 * r + 2] * Sk[6 + cc];
        hd s = hsin(q[i]), c = hcos(q[i]);
        hd omc = sub(K(1.0), c);
        hd Rot[9];
        for (int k = 0; k < 9; k++) Rot[k] = add(add(K((k % 4 == 0) ? 1.0 : 0.0), muls(s, Sk[k])), muls(omc, S2[k]));
        mm3(Kn->R[i], A, Rot);
    }
}

static void rnea(const mfo_model *M, const kin_t *Kn, const hd *qd, const hd *qdd, hd *tau) {
    hd w[MJ][3], dw[MJ][3], a[MJ][3], Fn[MJ][3], Nn[MJ][3];
    int n = M->n;
    for (int i = 0; i < n; i++) {
        int p = M->parent[i];
        hd wp[3], dwp[3], ap[3];
        if (p < 0) {
            for (int k = 0; k < 3; k++) { wp[k] = K(0); dwp[k] = K(0); ap[k] = K(-M->g[k]); }
        } else {
            hd d[3], t1[3], t2[3];
            memcpy(wp, w[p], sizeof wp);
            memcpy(dwp, dw[p], sizeof dwp);
            for (int k = 0; k < 3; k++) d[k] = sub(Kn->o[i][k], Kn->o[p][k]);
            cross3(t1, dwp, d);
            cross3(t2, wp, d);
            cross3(t2, wp, t2);
            for (int k = 0; k < 3; k++) ap[k] = add(add(a[p][k], t1[k]), t2[k]);
        }
        hd zq[3], t[3];
        for (int k = 0; k < 3; k++) zq[k] = mul(Kn->z[i][k], qd[i]);
        cross3(t, wp, zq);
        for (int k = 0; k < 3; k++) {
            w[i][k] = add(wp[k], zq[k]);
            dw[i][k] = add(add(dwp[k], mul(Kn->z[i][k], qdd[i])), t[k]);
            a[i][k] = ap[k];
        }
        /* com acceleration */
        hd r[3], t1[3], t2[3], ac[3];
        hd cl[3] = {K(M->c[i][0]), K(M->c[i][1]), K(M->c[i][2])};
        mv3(r, Kn->R[i], cl);
        cross3(t1, dw[i], r);
        cross3(t2, w[i], r);
        cross3(t2, w[i], t2);
        for (int k = 0; k < 3; k++) ac[k] = add(add(a[i][k], t1[k]), t2[k]);
        hd f[3];
        for (int k = 0; k < 3; k++) f[k] = muls(ac[k], M->m[i]);
        /* I_w v = R Ic R^T v */
        hd lb[3], Ib[3], Iw_dw[3], Iw_w[3];
        mtv3(lb, Kn->R[i], dw[i]);
        for (int k = 0; k < 3; k++) Ib[k] = add(add(muls(lb[0], M->Ic[i][3 * k]), muls(lb[1], M->Ic[i][3 * k + 1])), muls(lb[2], M->Ic[i][3 * k + 2]));
        mv3(Iw_dw, Kn->R[i], Ib);
        mtv3(lb, Kn->R[i], w[i]);
        for (int k = 0; k < 3; k++) Ib[k] = add(add(muls(lb[0], M->Ic[i][3 * k]), muls(lb[1], M->Ic[i][3 * k + 1])), muls(lb[2], M->Ic[i][3 * k + 2]));
        mv3(Iw_w, Kn->R[i], Ib);
        hd gyro[3], rf[3];
        cross3(gyro, w[i], Iw_w);
        cross3(rf, r, f);
        for (int k = 0; k < 3; k++) {
            Fn[i][k] = f[k];
            Nn[i][k] = add(add(Iw_dw[k], gyro[k]), rf[k]);
        }
    }
    for (int i = n - 1; i >= 0; i--) {
        tau[i] = dot3(Kn->z[i], Nn[i]);
        int p = M->parent[i];
        if (p >= 0) {
            hd d[3], t[3];
            for (int k = 0; k < 3; k++) d[k] = sub(Kn->o[i][k], Kn->o[p][k]);
            cross3(t, d, Fn[i]);
            for (int k = 0; k < 3; k++) {
                Fn[p][k] = add(Fn[p][k], Fn[i][k]);
                Nn[p][k] = add(add(Nn[p][k], Nn[i][k]), t[k]);
            }
        }
    }
}

static void frame_pose(const kin_t *Kn, const mfo_frame *F, hd *pos, hd *R) {
    if (F->parent < 0) {
        for (int k = 0; k < 3; k++) pos[k] = K(F->t[k]);
        for (int k = 0; k < 9; k++) R[k] = K(F->R[k]);
        return;
    }
    mvc3(pos, Kn->R[F->parent], F->t);
    for (int k = 0; k < 3; k++) pos[k] = add(pos[k], Kn->o[F->parent][k]);
    mmc3(R, Kn->R[F->parent], F->R);
}

/* tau_j -= J_f[:,j]^T [Fw; 0] = (z_j x (p_f - o_j)) . Fw for ancestors j of the frame joint */
static void sub_external(const mfo_model *M, const kin_t *Kn, const mfo_frame *F, const hd *pf, const hd *Fw, hd *tau) {
    for (int j = F->parent; j >= 0; j = M->parent[j]) {
        hd d[3], c[3];
        for (int k = 0; k < 3; k++) d[k] = sub(pf[k], Kn->o[j][k]);
        cross3(c, Kn->z[j], d);
        tau[j] = sub(tau[j], dot3(c, Fw));
    }
}
#ifndef BKMAX
#define BKMAX 160
#endif
/* ------------------------------------------------------------------ */
/* Bunch-Kaufman LDL^T of a dense symmetric m x m matrix (row-major, full
 * storage) with full symmetric permutations: P A P^T = L D L^T.
 * On return A holds L (strict lower) and D (diagonal + subdiagonal of 2x2
 * blocks); piv[k] = size of pivot block starting at k (1 or 2; 0 for the
 * second row of a 2x2); perm = permutation.  Returns inertia counts.      */
static int bk_factor(double *A, int m, int *perm, int *piv, int *npos, int *nneg, int *nzero) {
    const double alpha = (1.0 + sqrt(17.0)) / 8.0;
    for (int i = 0; i < m; i++) perm[i] = i;
    *npos = *nneg = *nzero = 0;
#define A_(i, j) A[(i) * m + (j)]
    int k = 0;
    while (k < m) {
        int kstep = 1, kp = k;
        double absakk = fabs(A_(k, k));
        int imax = k;
        double colmax = 0;
        for (int i = k + 1; i < m; i++)
            if (fabs(A_(i, k)) > colmax) { colmax = fabs(A_(i, k)); imax = i; }
        if (fmax(absakk, colmax) == 0.0) {
            (*nzero)++;
            piv[k] = 1;
            k++;
            continue;
        }
        if (absakk >= alpha * colmax) {
            kp = k;
        } else {
            double rowmax = 0;
            for (int j = k; j < m; j++)
                if (j != imax && fabs(A_(imax, j)) > rowmax) rowmax = fabs(A_(imax, j));
            if (absakk >= alpha * colmax * (colmax / rowmax)) kp = k;
            else if (fabs(A_(imax, imax)) >= alpha * rowmax) kp = imax;
            else { kp = imax; kstep = 2; }
        }
        int kk = k + kstep - 1;
        if (kp != kk) {
            /* symmetric swap of rows/cols kk <-> kp over the whole matrix (L part included) */
            for (int j = 0; j < m; j++) { double t = A_(kk, j); A_(kk, j) = A_(kp, j); A_(kp, j) = t; }
            for (int i = 0; i < m; i++) { double t = A_(i, kk); A_(i, kk) = A_(i, kp); A_(i, kp) = t; }
            int t = perm[kk]; perm[kk] = perm[kp]; perm[kp] = t;
        }
        if (kstep == 1) {
            double d = A_(k, k);
            if (d > 0) (*npos)++; else if (d < 0) (*nneg)++; else (*nzero)++;
            double inv = 1.0 / d, col[BKMAX];
            for (int i = k + 1; i < m; i++) col[i] = A_(i, k);
            for (int i = k + 1; i < m; i++) {
                double lik = col[i] * inv;
                for (int j = k + 1; j <= i; j++) A_(i, j) -= lik * col[j];
                A_(i, k) = lik;
            }
            for (int i = k + 1; i < m; i++)
                for (int j = i + 1; j < m; j++) A_(i, j) = A_(j, i);
            for (int j = k + 1; j < m; j++) A_(k, j) = A_(j, k);
            piv[k] = 1;
        } else {
            double a = A_(k, k), b = A_(k + 1, k), c = A_(k + 1, k + 1);
            double det = a * c - b * b;
            if (det < 0) { (*npos)++; (*nneg)++; }
            else if (det > 0) { if (a + c > 0) *npos += 2; else *nneg += 2; }
            else *nzero += 2;
            /* inverse of [[a,b],[b,c]] */
            double ia = c / det, ib = -b / det, ic = a / det, c0[BKMAX], c1[BKMAX];
            for (int i = k + 2; i < m; i++) { c0[i] = A_(i, k); c1[i] = A_(i, k + 1); }
            for (int i = k + 2; i < m; i++) {
                double l0 = c0[i] * ia + c1[i] * ib, l1 = c0[i] * ib + c1[i] * ic;
                for (int j = k + 2; j <= i; j++) A_(i, j) -= l0 * c0[j] + l1 * c1[j];
                A_(i, k) = l0;
                A_(i, k + 1) = l1;
            }
            for (int i = k + 2; i < m; i++)
                for (int j = i + 1; j < m; j++) A_(i, j) = A_(j, i);
            piv[k] = 2;
            piv[k + 1] = 0;
        }
        k += kstep;
    }
    return 0;
}

/* solve A x = b given bk_factor output; b overwritten with x */
static void bk_solve(const double *A, int m, const int *perm, const int *piv, double *b) {
    double y[BKMAX];
    for (int i = 0; i < m; i++) y[i] = b[perm[i]];
    /* L u = y  (unit lower; 2x2 blocks have L(k+1,k) = 0) */
    for (int k = 0; k < m;) {
        int s = piv[k] == 2 ? 2 : 1;
        for (int i = k + s; i < m; i++)
            for (int t = 0; t < s; t++) y[i] -= A_(i, k + t) * y[k + t];
        k += s;
    }
    /* D v = u */
    for (int k = 0; k < m;) {
        if (piv[k] == 2) {
            double a = A_(k, k), bb = A_(k + 1, k), c = A_(k + 1, k + 1);
            double det = a * c - bb * bb;
            double y0 = y[k], y1 = y[k + 1];
            y[k] = (c * y0 - bb * y1) / det;
            y[k + 1] = (a * y1 - bb * y0) / det;
            k += 2;
        } else {
            y[k] = y[k] / A_(k, k);
            k += 1;
        }
    }
    /* L^T x = v */
    for (int k = m - 1; k >= 0;) {
        int k0 = (k > 0 && piv[k] == 0) ? k - 1 : k;
        int s = k - k0 + 1;
        for (int t = 0; t < s; t++) {
            double acc = y[k0 + t];
            for (int i = k0 + s; i < m; i++) acc -= A_(i, k0 + t) * y[i];
            y[k0 + t] = acc;
        }
        k = k0 - 1;
    }
    for (int i = 0; i < m; i++) b[perm[i]] = y[i];
#undef A_
}

#endif
