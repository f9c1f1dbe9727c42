/*
 * fks_portable_math.h — deterministic double-precision libm subset, compiled
 * identically for the gfx950 device (hipcc) and the host (g++/hipcc).
 *
 * Why this exists: the reference simulator calls std::sin/std::cos (through
 * Eigen::AngleAxisd, SPCS FK via arc_utilities), std::log (through
 * std::normal_distribution inside arc_helpers::TruncatedNormalDistribution,
 * UNC:86) and atan2 (SE(3) log map, TNUVA:389).  glibc and the ROCm device
 * library (ocml) differ from each other by an ulp here and there; one ulp in a
 * joint angle is enough to flip a voxel index a few thousand microsteps
 * later.  Every transcendental used on the hot path therefore goes through
 * the functions below, which use only IEEE-754 +, -, *, / (correctly rounded
 * on both sides), integer bit manipulation and no fused multiply-add (every
 * translation unit that includes this header must be compiled with
 * -ffp-contract=off).  The algorithms are the classic fdlibm ones (Sun
 * Microsystems, freely redistributable), re-expressed here: sin/cos = Cody-
 * Waite reduction by pi/2 + degree-13/14 minimax kernels (<1 ulp), log =
 * reduction to [sqrt(2)/2, sqrt(2)) + Remez series in s=f/(2+f) (<1 ulp),
 * atan = 4-interval reduction + odd minimax polynomial (<1 ulp).
 *
 * Valid domain: |x| < 1.6e6 for sin/cos (the medium-range reduction; larger
 * arguments return NaN — joint angles never get there).
 *
 * This header is part of the product (include/).  The CPU oracle under
 * oracle/ includes it too so that both sides evaluate the same libm; it is
 * tested against glibc in tests/test_portable_math.py.
 */
#ifndef FKS_PORTABLE_MATH_H
#define FKS_PORTABLE_MATH_H

#if !defined(__HIPCC_RTC__)
#include <stdint.h>
#endif

#if defined(__HIPCC__)
#define FKS_HD __host__ __device__
#else
#define FKS_HD
#endif

#ifdef FKS_MATH_AUDIT_SYSTEM_LIBM
/* restatement audit only (oracle/Makefile `audit`, host code): the system libm in place
 * of the portable kernels, to measure how far results depend on them */
#include <math.h>
#define FKS_MATH_AUDIT_RETURN(expr) return (expr)
#else
#define FKS_MATH_AUDIT_RETURN(expr) (void)0
#endif

namespace fks_math {

FKS_HD inline uint64_t bits(double x) { return __builtin_bit_cast(uint64_t, x); }
FKS_HD inline double from_bits(uint64_t b) { return __builtin_bit_cast(double, b); }
FKS_HD inline uint32_t hi_word(double x) { return (uint32_t)(bits(x) >> 32); }
FKS_HD inline uint32_t lo_word(double x) { return (uint32_t)(bits(x) & 0xffffffffu); }
FKS_HD inline double with_hi_word(double x, uint32_t hi) {
    return from_bits(((uint64_t)hi << 32) | (bits(x) & 0xffffffffull));
}

/* round-to-nearest-even for |x| < 2^51 via the 1.5*2^52 shifter (exact) */
FKS_HD inline double rint_small(double x) {
    const double shifter = 6755399441055744.0; /* 0x1.8p52 */
    const double t = x + shifter; /* no reassociation without -ffast-math */
    return t - shifter;
}

/* std::max / std::min / arc_helpers::ClampValue semantics (NaN/+-0 ordering
 * of the C++ library, not IEEE maxNum) */
FKS_HD inline double dmax(double a, double b) { return (a < b) ? b : a; }
FKS_HD inline double dmin(double a, double b) { return (b < a) ? b : a; }
FKS_HD inline double clamp(double v, double lo, double hi) { return dmin(hi, dmax(lo, v)); }
FKS_HD inline double dabs(double x) { return from_bits(bits(x) & 0x7fffffffffffffffull); }
FKS_HD inline double dsqrt(double x) { return __builtin_sqrt(x); }

/* ---------------- sin / cos ---------------- */
FKS_HD inline double kernel_sin(double x, double y, int iy) {
    const double S1 = -1.66666666666666324348e-01, S2 = 8.33333333332248946124e-03,
                 S3 = -1.98412698298579493134e-04, S4 = 2.75573137070700676789e-06,
                 S5 = -2.50507602534068634195e-08, S6 = 1.58969099521155010221e-10;
    const double z = x * x;
    const double w = z * z;
    const double r = S2 + z * (S3 + z * S4) + z * w * (S5 + z * S6);
    const double v = z * x;
    if (iy == 0) return x + v * (S1 + z * r);
    return x - ((z * (0.5 * y - v * r) - y) - v * S1);
}

FKS_HD inline double kernel_cos(double x, double y) {
    const double C1 = 4.16666666666666019037e-02, C2 = -1.38888888888741095749e-03,
                 C3 = 2.48015872894767294178e-05, C4 = -2.75573143513906633035e-07,
                 C5 = 2.08757232129817482790e-09, C6 = -1.13596475577881948265e-11;
    const double z = x * x;
    double w = z * z;
    const double r = z * (C1 + z * (C2 + z * C3)) + w * w * (C4 + z * (C5 + z * C6));
    const double hz = 0.5 * z;
    w = 1.0 - hz;
    return w + (((1.0 - w) - hz) + (z * r - x * y));
}

/* x = n*pi/2 + (y0 + y1), medium range only; returns n (or INT32_MIN if out of range) */
FKS_HD inline int32_t rem_pio2(double x, double* y0, double* y1) {
    const double invpio2 = 6.36619772367581382433e-01, pio2_1 = 1.57079632673412561417e+00,
                 pio2_1t = 6.07710050650619224932e-11, pio2_2 = 6.07710050630396597660e-11,
                 pio2_2t = 2.02226624879595063154e-21, pio2_3 = 2.02226624871116645580e-21,
                 pio2_3t = 8.47842766036889956997e-32;
    const uint32_t ix = hi_word(x) & 0x7fffffffu;
    if (ix > 0x413921fbu) { /* |x| > 2^20*pi/2 */
        *y0 = 0.0;
        *y1 = 0.0;
        return INT32_MIN;
    }
    const double fn = rint_small(x * invpio2);
    const int32_t n = (int32_t)fn;
    double r = x - fn * pio2_1;
    double w = fn * pio2_1t;
    const int32_t j = (int32_t)(ix >> 20);
    double yy0 = r - w;
    int32_t i = j - (int32_t)((hi_word(yy0) >> 20) & 0x7ffu);
    if (i > 16) {
        double t = r;
        w = fn * pio2_2;
        r = t - w;
        w = fn * pio2_2t - ((t - r) - w);
        yy0 = r - w;
        i = j - (int32_t)((hi_word(yy0) >> 20) & 0x7ffu);
        if (i > 49) {
            t = r;
            w = fn * pio2_3;
            r = t - w;
            w = fn * pio2_3t - ((t - r) - w);
            yy0 = r - w;
        }
    }
    *y0 = yy0;
    *y1 = (r - yy0) - w;
    return n;
}

FKS_HD inline double sin(double x) {
    FKS_MATH_AUDIT_RETURN(::sin(x));
    const uint32_t ix = hi_word(x) & 0x7fffffffu;
    if (ix <= 0x3fe921fbu) {
        if (ix < 0x3e500000u) return x;
        return kernel_sin(x, 0.0, 0);
    }
    if (ix >= 0x7ff00000u) return x - x;
    double y0, y1;
    const int32_t n = rem_pio2(x, &y0, &y1);
    if (n == INT32_MIN) return from_bits(0x7ff8000000000000ull);
    switch (n & 3) {
        case 0: return kernel_sin(y0, y1, 1);
        case 1: return kernel_cos(y0, y1);
        case 2: return -kernel_sin(y0, y1, 1);
        default: return -kernel_cos(y0, y1);
    }
}

FKS_HD inline double cos(double x) {
    FKS_MATH_AUDIT_RETURN(::cos(x));
    const uint32_t ix = hi_word(x) & 0x7fffffffu;
    if (ix <= 0x3fe921fbu) {
        if (ix < 0x3e46a09eu) return 1.0;
        return kernel_cos(x, 0.0);
    }
    if (ix >= 0x7ff00000u) return x - x;
    double y0, y1;
    const int32_t n = rem_pio2(x, &y0, &y1);
    if (n == INT32_MIN) return from_bits(0x7ff8000000000000ull);
    switch (n & 3) {
        case 0: return kernel_cos(y0, y1);
        case 1: return -kernel_sin(y0, y1, 1);
        case 2: return -kernel_cos(y0, y1);
        default: return kernel_sin(y0, y1, 1);
    }
}

/* sin and cos of one argument sharing the argument reduction; bit-identical to
 * sin(x) and cos(x) */
FKS_HD inline void sincos(double x, double* s, double* c) {
#ifdef FKS_MATH_AUDIT_SYSTEM_LIBM
    *s = ::sin(x);
    *c = ::cos(x);
    return;
#endif
    const uint32_t ix = hi_word(x) & 0x7fffffffu;
    if (ix <= 0x3fe921fbu) {
        *s = (ix < 0x3e500000u) ? x : kernel_sin(x, 0.0, 0);
        *c = (ix < 0x3e46a09eu) ? 1.0 : kernel_cos(x, 0.0);
        return;
    }
    if (ix >= 0x7ff00000u) {
        *s = x - x;
        *c = x - x;
        return;
    }
    double y0, y1;
    const int32_t n = rem_pio2(x, &y0, &y1);
    if (n == INT32_MIN) {
        *s = from_bits(0x7ff8000000000000ull);
        *c = *s;
        return;
    }
    const double ks = kernel_sin(y0, y1, 1), kc = kernel_cos(y0, y1);
    switch (n & 3) {
        case 0:
            *s = ks;
            *c = kc;
            break;
        case 1:
            *s = kc;
            *c = -ks;
            break;
        case 2:
            *s = -ks;
            *c = -kc;
            break;
        default:
            *s = -kc;
            *c = ks;
            break;
    }
}

/* ---------------- log ---------------- */
FKS_HD inline double log(double x) {
    FKS_MATH_AUDIT_RETURN(::log(x));
    const double ln2_hi = 6.93147180369123816490e-01, ln2_lo = 1.90821492927058770002e-10,
                 two54 = 1.80143985094819840000e+16, Lg1 = 6.666666666666735130e-01,
                 Lg2 = 3.999999999940941908e-01, Lg3 = 2.857142874366239149e-01,
                 Lg4 = 2.222219843214978396e-01, Lg5 = 1.818357216161805012e-01,
                 Lg6 = 1.531383769920937332e-01, Lg7 = 1.479819860511658591e-01;
    int32_t hx = (int32_t)hi_word(x);
    const uint32_t lx = lo_word(x);
    int32_t k = 0;
    if (hx < 0x00100000) {
        if (((hx & 0x7fffffff) | (int32_t)lx) == 0) return -from_bits(0x7ff0000000000000ull);
        if (hx < 0) return from_bits(0x7ff8000000000000ull);
        k -= 54;
        x *= two54;
        hx = (int32_t)hi_word(x);
    }
    if (hx >= 0x7ff00000) return x + x;
    k += (hx >> 20) - 1023;
    hx &= 0x000fffff;
    int32_t i = (hx + 0x95f64) & 0x100000;
    x = with_hi_word(x, (uint32_t)(hx | (i ^ 0x3ff00000)));
    k += (i >> 20);
    const double f = x - 1.0;
    double dk, R;
    if ((0x000fffff & (2 + hx)) < 3) {
        if (f == 0.0) {
            if (k == 0) return 0.0;
            dk = (double)k;
            return dk * ln2_hi + dk * ln2_lo;
        }
        R = f * f * (0.5 - 0.33333333333333333 * f);
        if (k == 0) return f - R;
        dk = (double)k;
        return dk * ln2_hi - ((R - dk * ln2_lo) - f);
    }
    const double s = f / (2.0 + f);
    dk = (double)k;
    const double z = s * s;
    i = hx - 0x6147a;
    const double w = z * z;
    const int32_t j = 0x6b851 - hx;
    const double t1 = w * (Lg2 + w * (Lg4 + w * Lg6));
    const double t2 = z * (Lg1 + w * (Lg3 + w * (Lg5 + w * Lg7)));
    i |= j;
    R = t2 + t1;
    if (i > 0) {
        const double hfsq = 0.5 * f * f;
        if (k == 0) return f - (hfsq - s * (hfsq + R));
        return dk * ln2_hi - ((hfsq - (s * (hfsq + R) + dk * ln2_lo)) - f);
    }
    if (k == 0) return f - s * (f - R);
    return dk * ln2_hi - ((s * (f - R) - dk * ln2_lo) - f);
}

/* ---------------- atan / atan2 ---------------- */
FKS_HD inline double atan(double x) {
    FKS_MATH_AUDIT_RETURN(::atan(x));
    const double atanhi[4] = {4.63647609000806093515e-01, 7.85398163397448278999e-01,
                              9.82793723247329054082e-01, 1.57079632679489655800e+00};
    const double atanlo[4] = {2.26987774529616870924e-17, 3.06161699786838301793e-17,
                              1.39033110312309984516e-17, 6.12323399573676603587e-17};
    const double aT[11] = {3.33333333333329318027e-01,  -1.99999999998764832476e-01,
                           1.42857142725034663711e-01,  -1.11111104054623557880e-01,
                           9.09088713343650656196e-02,  -7.69187620504482999495e-02,
                           6.66107313738753120669e-02,  -5.83357013379057348645e-02,
                           4.97687799461593236017e-02,  -3.65315727442169155270e-02,
                           1.62858201153657823623e-02};
    const int32_t hx = (int32_t)hi_word(x);
    const uint32_t ix = (uint32_t)hx & 0x7fffffffu;
    int id;
    if (ix >= 0x44100000u) { /* |x| >= 2^66 */
        if (ix > 0x7ff00000u || (ix == 0x7ff00000u && lo_word(x) != 0)) return x + x;
        return (hx > 0) ? atanhi[3] + atanlo[3] : -atanhi[3] - atanlo[3];
    }
    if (ix < 0x3fdc0000u) { /* |x| < 0.4375 */
        if (ix < 0x3e400000u) return x;
        id = -1;
    } else {
        x = dabs(x);
        if (ix < 0x3ff30000u) {
            if (ix < 0x3fe60000u) {
                id = 0;
                x = (2.0 * x - 1.0) / (2.0 + x);
            } else {
                id = 1;
                x = (x - 1.0) / (x + 1.0);
            }
        } else {
            if (ix < 0x40038000u) {
                id = 2;
                x = (x - 1.5) / (1.0 + 1.5 * x);
            } else {
                id = 3;
                x = -1.0 / x;
            }
        }
    }
    const double z = x * x;
    const double w = z * z;
    const double s1 = z * (aT[0] + w * (aT[2] + w * (aT[4] + w * (aT[6] + w * (aT[8] + w * aT[10])))));
    const double s2 = w * (aT[1] + w * (aT[3] + w * (aT[5] + w * (aT[7] + w * aT[9]))));
    if (id < 0) return x - x * (s1 + s2);
    const double zz = atanhi[id] - ((x * (s1 + s2) - atanlo[id]) - x);
    return (hx < 0) ? -zz : zz;
}

/* atan2 for finite arguments (the hot path never passes inf/nan) */
FKS_HD inline double atan2(double y, double x) {
    FKS_MATH_AUDIT_RETURN(::atan2(y, x));
    const double pi_o_2 = 1.5707963267948965580e+00, pi = 3.1415926535897931160e+00,
                 pi_lo = 1.2246467991473531772e-16;
    if (x != x || y != y) return x + y;
    if (x == 1.0) return atan(y);
    const uint32_t hx = hi_word(x), hy = hi_word(y);
    const uint32_t ix = hx & 0x7fffffffu, iy = hy & 0x7fffffffu;
    const int m = (int)(((hy >> 31) & 1u) | ((hx >> 30) & 2u));
    if (y == 0.0) {
        switch (m) {
            case 0:
            case 1: return y;
            case 2: return pi;
            default: return -pi;
        }
    }
    if (x == 0.0) return ((int32_t)hy < 0) ? -pi_o_2 : pi_o_2;
    const int32_t k = ((int32_t)iy - (int32_t)ix) >> 20;
    double z;
    if (k > 60) {
        z = pi_o_2 + 0.5 * pi_lo;
    } else if ((int32_t)hx < 0 && k < -60) {
        z = 0.0;
    } else {
        z = atan(dabs(y / x));
    }
    switch (m) {
        case 0: return z;
        case 1: return -z;
        case 2: return pi - (z - pi_lo);
        default: return (z - pi_lo) - pi;
    }
}

/* fmod(x, 2*pi) without a libm call, for the kernel's continuous-joint wrap: binary long
 * division of |x| by 2*pi.  Each step subtracts s = 2*pi*2^m with s <= r < 2*s, which is exact
 * (Sterbenz), so the result is the exact remainder fmod returns, with the sign of x; a
 * non-finite x gives the quiet NaN.  At most one step per binade of |x| / (2*pi).  Pinned
 * against glibc's fmod by tests/test_portable_math.py. */
FKS_HD inline double fmod_two_pi(double x) {
    const double y = 2.0 * 3.14159265358979323846;
    const uint64_t yb = bits(y);
    double r = dabs(x);
    if (!(r <= 1.7976931348623157e308)) return from_bits(0x7ff8000000000000ull);
    while (r >= y) {
        const uint64_t shift = (uint64_t)((hi_word(r) >> 20) - (uint32_t)(yb >> 52)) << 52;
        double s = from_bits(yb + shift);
        if (s > r) s = from_bits(yb + shift - (1ull << 52));
        r = r - s;
    }
    return from_bits(bits(r) | (bits(x) & 0x8000000000000000ull));
}

/* the same wrap as enforce_continuous_revolute_bounds below, through fmod_two_pi: the kernel's
 * form (ocml's fmod is a large inlined loop that costs the hot loops registers) */
FKS_HD inline double wrap_revolute(double value) {
    const double kPi = 3.14159265358979323846;
    if ((value <= -kPi) || (value > kPi)) {
        const double remainder = fmod_two_pi(value);
        if (remainder <= -kPi) return remainder + (2.0 * kPi);
        if (remainder > kPi) return remainder - (2.0 * kPi);
        return remainder;
    }
    return value;
}

/* arc_utilities EigenHelpers::EnforceContinuousRevoluteBounds restated:
 * wrap into (-pi, pi]; fmod is exact on both glibc and ocml. */
FKS_HD inline double enforce_continuous_revolute_bounds(double value) {
    const double kPi = 3.14159265358979323846;
    if ((value <= -kPi) || (value > kPi)) {
        const double remainder = __builtin_fmod(value, 2.0 * kPi);
        if (remainder <= -kPi) return remainder + (2.0 * kPi);
        if (remainder > kPi) return remainder - (2.0 * kPi);
        return remainder;
    }
    return value;
}

}  // namespace fks_math

#endif  // FKS_PORTABLE_MATH_H
