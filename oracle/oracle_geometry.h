/*
 * TEST INFRASTRUCTURE ONLY — CPU oracle (see oracle/README.md).
 *
 * Restated geometric primitives of the absent dependencies (Eigen 3.2/3.3-beta,
 * arc_utilities, sdf_tools).  None of these libraries is present in the
 * container, so each primitive below is a documented choice,
 * written in the operation order Eigen evaluates the corresponding expression
 * (DESIGN.md §"Restated external primitives").  The HIP kernel implements the
 * same definitions independently.
 *
 * Canonical evaluation orders used everywhere:
 *   dot3(a,b)           = (a0*b0 + a1*b1) + a2*b2
 *   3x4 compose C = A*B = rotation: dot3(row_i(A), col_j(B));
 *                         translation: dot3(row_i(A), B.t) + A.t_i      (Eigen Transform*Transform)
 *   T * p (4-vector)    = dot3(row_i(R), p.xyz) + t_i * p.w, w copied   (Eigen Isometry3d * Vector4d)
 *   squaredNorm(4-vec)  = ((x*x + y*y) + z*z) + w*w
 *   AngleAxis -> matrix = Eigen::AngleAxis::toRotationMatrix (sin_axis, (1-c)*axis, tmp form)
 */
#ifndef FKS_ORACLE_GEOMETRY_H
#define FKS_ORACLE_GEOMETRY_H

#include <stdint.h>

#include "fks_portable_math.h"

namespace oracle {

struct V3 {
    double x, y, z;
};
struct V4 {
    double x, y, z, w;
};

struct Iso {
    double r[9]; /* row-major linear part */
    double t[3];
};

inline Iso iso_identity() {
    Iso I;
    for (int i = 0; i < 9; ++i) I.r[i] = (i % 4 == 0) ? 1.0 : 0.0;
    I.t[0] = I.t[1] = I.t[2] = 0.0;
    return I;
}

inline Iso iso_from12(const double* m) {
    Iso T;
    T.r[0] = m[0];
    T.r[1] = m[1];
    T.r[2] = m[2];
    T.t[0] = m[3];
    T.r[3] = m[4];
    T.r[4] = m[5];
    T.r[5] = m[6];
    T.t[1] = m[7];
    T.r[6] = m[8];
    T.r[7] = m[9];
    T.r[8] = m[10];
    T.t[2] = m[11];
    return T;
}

inline void iso_to12(const Iso& T, double* m) {
    m[0] = T.r[0];
    m[1] = T.r[1];
    m[2] = T.r[2];
    m[3] = T.t[0];
    m[4] = T.r[3];
    m[5] = T.r[4];
    m[6] = T.r[5];
    m[7] = T.t[1];
    m[8] = T.r[6];
    m[9] = T.r[7];
    m[10] = T.r[8];
    m[11] = T.t[2];
}

inline double dot3(double a0, double a1, double a2, double b0, double b1, double b2) {
    return (a0 * b0 + a1 * b1) + a2 * b2;
}

inline Iso compose(const Iso& A, const Iso& B) {
    Iso C;
    for (int i = 0; i < 3; ++i) {
        for (int j = 0; j < 3; ++j)
            C.r[i * 3 + j] = dot3(A.r[i * 3 + 0], A.r[i * 3 + 1], A.r[i * 3 + 2], B.r[0 * 3 + j],
                                  B.r[1 * 3 + j], B.r[2 * 3 + j]);
        C.t[i] = dot3(A.r[i * 3 + 0], A.r[i * 3 + 1], A.r[i * 3 + 2], B.t[0], B.t[1], B.t[2]) + A.t[i];
    }
    return C;
}

/* Eigen Isometry3d::inverse(): linear^T, -(linear^T * t) */
inline Iso inverse(const Iso& T) {
    Iso I;
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j) I.r[i * 3 + j] = T.r[j * 3 + i];
    for (int i = 0; i < 3; ++i)
        I.t[i] = -dot3(I.r[i * 3 + 0], I.r[i * 3 + 1], I.r[i * 3 + 2], T.t[0], T.t[1], T.t[2]);
    return I;
}

inline V4 xform4(const Iso& T, const V4& p) {
    V4 o;
    o.x = dot3(T.r[0], T.r[1], T.r[2], p.x, p.y, p.z) + T.t[0] * p.w;
    o.y = dot3(T.r[3], T.r[4], T.r[5], p.x, p.y, p.z) + T.t[1] * p.w;
    o.z = dot3(T.r[6], T.r[7], T.r[8], p.x, p.y, p.z) + T.t[2] * p.w;
    o.w = p.w;
    return o;
}

inline V3 xform3(const Iso& T, const V3& p) {
    V3 o;
    o.x = dot3(T.r[0], T.r[1], T.r[2], p.x, p.y, p.z) + T.t[0];
    o.y = dot3(T.r[3], T.r[4], T.r[5], p.x, p.y, p.z) + T.t[1];
    o.z = dot3(T.r[6], T.r[7], T.r[8], p.x, p.y, p.z) + T.t[2];
    return o;
}

inline V3 rotate(const Iso& T, const V3& v) {
    V3 o;
    o.x = dot3(T.r[0], T.r[1], T.r[2], v.x, v.y, v.z);
    o.y = dot3(T.r[3], T.r[4], T.r[5], v.x, v.y, v.z);
    o.z = dot3(T.r[6], T.r[7], T.r[8], v.x, v.y, v.z);
    return o;
}

/* Eigen cross(): (y*z' - z*y', z*x' - x*z', x*y' - y*x') */
inline V3 cross(const V3& a, const V3& b) {
    V3 c;
    c.x = a.y * b.z - a.z * b.y;
    c.y = a.z * b.x - a.x * b.z;
    c.z = a.x * b.y - a.y * b.x;
    return c;
}

/* Eigen Vector4d squaredNorm (and norm, dot): the vectorised redux over two Packet2d
 * lanes, (x + z) + (y + w) -- the reference's -O3 x86-64 (SSE2, no FMA) build
 * (CMakeLists.txt:66).  ORACLE_AUDIT_V4_SEQUENTIAL is the restatement
 * audit's alternative (tools/restatement_audit.py), never the parity oracle. */
#ifdef ORACLE_AUDIT_V4_SEQUENTIAL
inline double sqnorm4(const V4& v) { return ((v.x * v.x + v.y * v.y) + v.z * v.z) + v.w * v.w; }
#else
inline double sqnorm4(const V4& v) { return (v.x * v.x + v.z * v.z) + (v.y * v.y + v.w * v.w); }
#endif
inline double sqnorm3(const V3& v) { return (v.x * v.x + v.y * v.y) + v.z * v.z; }

/* EigenHelpers::SafeNormal: v / norm if norm > DBL_EPSILON else v */
inline V4 safe_normal4(const V4& v) {
    const double n = fks_math::dsqrt(sqnorm4(v));
    if (n > 2.220446049250313e-16) return V4{v.x / n, v.y / n, v.z / n, v.w / n};
    return v;
}
inline V3 safe_normal3(const V3& v) {
    const double n = fks_math::dsqrt(sqnorm3(v));
    if (n > 2.220446049250313e-16) return V3{v.x / n, v.y / n, v.z / n};
    return v;
}

/* Eigen::AngleAxisd(angle, axis).toRotationMatrix() */
inline void angle_axis_matrix(double angle, const double a[3], double R[9]) {
    const double s = fks_math::sin(angle);
    const double c = fks_math::cos(angle);
    const double sa0 = s * a[0], sa1 = s * a[1], sa2 = s * a[2];
    const double omc = 1.0 - c;
    const double c1a0 = omc * a[0], c1a1 = omc * a[1], c1a2 = omc * a[2];
    double tmp = c1a0 * a[1];
    R[1] = tmp - sa2;
    R[3] = tmp + sa2;
    tmp = c1a0 * a[2];
    R[2] = tmp + sa1;
    R[6] = tmp - sa1;
    tmp = c1a1 * a[2];
    R[5] = tmp - sa0;
    R[7] = tmp + sa0;
    R[0] = c1a0 * a[0] + c;
    R[4] = c1a1 * a[1] + c;
    R[8] = c1a2 * a[2] + c;
}

/* ---- SE(3) exponential / logarithm of body twists (v, w) ----
 * arc_utilities EigenHelpers::ExpTwist / TwistBetweenTransforms are absent; they
 * are restated as the closed-form SE(3) exp/log.  A = sin t / t,
 * B = (1 - cos t)/t^2 = 2 sin^2(t/2)/t^2, C = (t - sin t)/t^3, series below 1e-3. */
inline void se3_coeffs(double theta, double* A, double* B, double* C) {
    if (theta < 1e-3) {
        const double t2 = theta * theta;
        *A = 1.0 - t2 / 6.0 + (t2 * t2) / 120.0;
        *B = 0.5 - t2 / 24.0 + (t2 * t2) / 720.0;
        *C = 1.0 / 6.0 - t2 / 120.0 + (t2 * t2) / 5040.0;
    } else {
        const double s = fks_math::sin(theta);
        const double sh = fks_math::sin(0.5 * theta);
        *A = s / theta;
        *B = (2.0 * (sh * sh)) / (theta * theta);
        *C = (theta - s) / ((theta * theta) * theta);
    }
}

/* W = skew(w); returns W*v */
inline V3 skew_mul(const V3& w, const V3& v) { return cross(w, v); }

inline Iso exp_twist(const double twist[6]) {
    const V3 v{twist[0], twist[1], twist[2]};
    const V3 w{twist[3], twist[4], twist[5]};
    const double theta = fks_math::dsqrt(sqnorm3(w));
    double A, B, C;
    se3_coeffs(theta, &A, &B, &C);
    Iso T;
    /* R = I + A W + B W^2, W^2 = w w^T - theta^2 I  (element form) */
    const double wv[3] = {w.x, w.y, w.z};
    const double th2 = (w.x * w.x + w.y * w.y) + w.z * w.z;
    for (int i = 0; i < 3; ++i) {
        for (int j = 0; j < 3; ++j) {
            double Wij = 0.0;
            if (i == 0 && j == 1) Wij = -w.z;
            if (i == 0 && j == 2) Wij = w.y;
            if (i == 1 && j == 0) Wij = w.z;
            if (i == 1 && j == 2) Wij = -w.x;
            if (i == 2 && j == 0) Wij = -w.y;
            if (i == 2 && j == 1) Wij = w.x;
            const double W2ij = wv[i] * wv[j] - ((i == j) ? th2 : 0.0);
            T.r[i * 3 + j] = ((i == j) ? 1.0 : 0.0) + A * Wij + B * W2ij;
        }
    }
    /* t = v + B (W v) + C (W (W v)) */
    const V3 Wv = skew_mul(w, v);
    const V3 WWv = skew_mul(w, Wv);
    T.t[0] = (v.x + B * Wv.x) + C * WWv.x;
    T.t[1] = (v.y + B * Wv.y) + C * WWv.y;
    T.t[2] = (v.z + B * Wv.z) + C * WWv.z;
    return T;
}

inline void log_twist(const Iso& T, double twist[6]) {
    const double* R = T.r;
    const double cos_arg = (((R[0] + R[4]) + R[8]) - 1.0) * 0.5;
    const V3 vee{(R[7] - R[5]) * 0.5, (R[2] - R[6]) * 0.5, (R[3] - R[1]) * 0.5};
    const double s = fks_math::dsqrt(sqnorm3(vee));
    const double theta = fks_math::atan2(s, cos_arg);
    V3 w;
    if (theta < 1e-3) {
        const double f = 1.0 + (theta * theta) / 6.0;
        w = V3{vee.x * f, vee.y * f, vee.z * f};
    } else if (s < 1e-6 && cos_arg < 0.0) {
        /* rotation by ~pi: axis from the largest diagonal entry */
        int k = 0;
        if (R[4] > R[0]) k = 1;
        if (R[8] > R[k * 4]) k = 2;
        double ax[3];
        ax[k] = fks_math::dsqrt((R[k * 4] + 1.0) * 0.5);
        for (int i = 0; i < 3; ++i)
            if (i != k) ax[i] = (R[i * 3 + k] + R[k * 3 + i]) / (4.0 * ax[k]);
        w = V3{ax[0] * theta, ax[1] * theta, ax[2] * theta};
    } else {
        const double f = theta / s;
        w = V3{vee.x * f, vee.y * f, vee.z * f};
    }
    const double th = fks_math::dsqrt(sqnorm3(w));
    double A, B, C;
    se3_coeffs(th, &A, &B, &C);
    /* V^-1 = I - W/2 + D W^2, D = (1 - A/(2B)) / th^2 */
    double D;
    if (th < 1e-3) {
        const double t2 = th * th;
        D = 1.0 / 12.0 + t2 / 720.0;
    } else {
        D = (1.0 - A / (2.0 * B)) / (th * th);
    }
    const V3 t{T.t[0], T.t[1], T.t[2]};
    const V3 Wt = skew_mul(w, t);
    const V3 WWt = skew_mul(w, Wt);
    twist[0] = (t.x - 0.5 * Wt.x) + D * WWt.x;
    twist[1] = (t.y - 0.5 * Wt.y) + D * WWt.y;
    twist[2] = (t.z - 0.5 * Wt.z) + D * WWt.z;
    twist[3] = w.x;
    twist[4] = w.y;
    twist[5] = w.z;
}

}  // namespace oracle

#endif
