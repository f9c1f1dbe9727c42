/*
 * fks_se3.h — the SE(3) primitives of the robot models, shared by the kernels
 * (fks_kernels.hip) and the host-side robot control of the C-ABI (fks_robot_control.cpp),
 * so both evaluate the same expression trees: EigenHelpers::ExpTwist / TwistBetweenTransforms
 * (the body-twist exp / log of TNUVA:360, 389, closed forms as oracle_geometry.h) and the
 * 3x4 composition / inverse in Eigen's Transform product order.
 */
#ifndef FKS_SE3_H
#define FKS_SE3_H

#include "fks_portable_math.h"

namespace fks_se3 {

using fks_math::dsqrt;

struct V3 {
    double x, y, z;
};
FKS_HD inline double dot3(double a0, double a1, double a2, double b0, double b1, double b2) {
    return (a0 * b0 + a1 * b1) + a2 * b2;
}
FKS_HD inline V3 cross(const V3& a, const V3& b) {
    V3 c;
    c.x = a.y * b.z - a.z * b.y;
    c.y = a.z * b.x - a.x * b.z;
    c.z = a.x * b.y - a.y * b.x;
    return c;
}
FKS_HD inline double sqnorm3(const V3& v) { return (v.x * v.x + v.y * v.y) + v.z * v.z; }

/* SE(3) exp/log of body twists: same closed forms as oracle_geometry.h */
FKS_HD inline void se3_coeffs(double theta, double* A, double* B, double* C) {
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
FKS_HD inline void exp_twist34(const double* tw, double* M) {
    const V3 v{tw[0], tw[1], tw[2]};
    const V3 w{tw[3], tw[4], tw[5]};
    const double theta = dsqrt(sqnorm3(w));
    double A, B, C;
    se3_coeffs(theta, &A, &B, &C);
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
            M[4 * i + j] = ((i == j) ? 1.0 : 0.0) + A * Wij + B * W2ij;
        }
    }
    const V3 Wv = cross(w, v);
    const V3 WWv = cross(w, Wv);
    M[3] = (v.x + B * Wv.x) + C * WWv.x;
    M[7] = (v.y + B * Wv.y) + C * WWv.y;
    M[11] = (v.z + B * Wv.z) + C * WWv.z;
}
FKS_HD inline void log_twist34(const double* T, double* tw) {
    const double R0 = T[0], R1 = T[1], R2 = T[2], R3 = T[4], R4 = T[5], R5 = T[6], R6 = T[8], R7 = T[9], R8 = T[10];
    const double cos_arg = (((R0 + R4) + R8) - 1.0) * 0.5;
    const V3 vee{(R7 - R5) * 0.5, (R2 - R6) * 0.5, (R3 - R1) * 0.5};
    const double s = dsqrt(sqnorm3(vee));
    const double theta = fks_math::atan2(s, cos_arg);
    V3 w;
    if (theta < 1e-3) {
        const double f = 1.0 + (theta * theta) / 6.0;
        w = V3{vee.x * f, vee.y * f, vee.z * f};
    } else if (s < 1e-6 && cos_arg < 0.0) {
        const double Rm[9] = {R0, R1, R2, R3, R4, R5, R6, R7, R8};
        int k = 0;
        if (Rm[4] > Rm[0]) k = 1;
        if (Rm[8] > Rm[k * 4]) k = 2;
        double ax[3];
        ax[k] = dsqrt((Rm[k * 4] + 1.0) * 0.5);
        for (int i = 0; i < 3; ++i)
            if (i != k) ax[i] = (Rm[i * 3 + k] + Rm[k * 3 + i]) / (4.0 * ax[k]);
        w = V3{ax[0] * theta, ax[1] * theta, ax[2] * theta};
    } else {
        const double f = theta / s;
        w = V3{vee.x * f, vee.y * f, vee.z * f};
    }
    const double th = dsqrt(sqnorm3(w));
    double A, B, C;
    se3_coeffs(th, &A, &B, &C);
    double D;
    if (th < 1e-3) {
        const double t2 = th * th;
        D = 1.0 / 12.0 + t2 / 720.0;
    } else {
        D = (1.0 - A / (2.0 * B)) / (th * th);
    }
    const V3 t{T[3], T[7], T[11]};
    const V3 Wt = cross(w, t);
    const V3 WWt = cross(w, Wt);
    tw[0] = (t.x - 0.5 * Wt.x) + D * WWt.x;
    tw[1] = (t.y - 0.5 * Wt.y) + D * WWt.y;
    tw[2] = (t.z - 0.5 * Wt.z) + D * WWt.z;
    tw[3] = w.x;
    tw[4] = w.y;
    tw[5] = w.z;
}
/* C = A * B (3x4 row-major), Eigen Transform product order */
FKS_HD inline void compose34(const double* A, const double* B, double* C) {
    for (int i = 0; i < 3; ++i) {
        for (int j = 0; j < 3; ++j)
            C[4 * i + j] = dot3(A[4 * i + 0], A[4 * i + 1], A[4 * i + 2], B[j], B[4 + j], B[8 + j]);
        C[4 * i + 3] = dot3(A[4 * i + 0], A[4 * i + 1], A[4 * i + 2], B[3], B[7], B[11]) + A[4 * i + 3];
    }
}
FKS_HD inline void inverse34(const double* T, double* I) {
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j) I[4 * i + j] = T[4 * j + i];
    for (int i = 0; i < 3; ++i) I[4 * i + 3] = -dot3(I[4 * i + 0], I[4 * i + 1], I[4 * i + 2], T[3], T[7], T[11]);
}

}  // namespace fks_se3

#endif
