/*
 * wololo/wmath.h -- host-side scalar/vector/quaternion types of the wololo scene API.
 *
 * ABI contract (must not change, `wololo_demo` links against it unchanged):
 *   Wo_Scalar      = double                               (ref: src/wololo/wmath.decl.h:13)
 *   Wo_Vec3        = { double x, y, z }       24 bytes    (ref: src/wololo/wmath.decl.h:19-24)
 *   Wo_Quaternion  = { double real; Wo_Vec3 imaginary }   (ref: src/wololo/wmath.decl.h:41-45)
 *
 * All helpers are header-only `static inline`, as in the reference
 * (src/wololo/wmath.impl.h:11-69).  One deliberate difference: the reference's
 * `wo_vec3_normalized` divides by the SQUARED length (wmath.impl.h:48-55, see
 * SURVEY.md Appendix A); here it divides by the length.  Nothing on the render
 * path uses it -- the scene compiler normalises in its own code.
 */
#ifndef WOLOLO_WMATH_H
#define WOLOLO_WMATH_H

#include <math.h>

typedef double Wo_Scalar;

typedef struct Wo_Vec3 Wo_Vec3;
struct Wo_Vec3 {
    Wo_Scalar x;
    Wo_Scalar y;
    Wo_Scalar z;
};

/* q = real + imaginary.(i, j, k); a rotation when |q| = 1. */
typedef struct Wo_Quaternion Wo_Quaternion;
struct Wo_Quaternion {
    Wo_Scalar real;
    Wo_Vec3 imaginary;
};

static inline Wo_Vec3 wo_vec3_0(void) {
    Wo_Vec3 z;
    z.x = 0.0; z.y = 0.0; z.z = 0.0;
    return z;
}

static inline Wo_Vec3 wo_vec3_make(Wo_Scalar x, Wo_Scalar y, Wo_Scalar z) {
    Wo_Vec3 v;
    v.x = x; v.y = y; v.z = z;
    return v;
}

static inline Wo_Vec3 wo_vec3_add(Wo_Vec3 a, Wo_Vec3 b) {
    return wo_vec3_make(a.x + b.x, a.y + b.y, a.z + b.z);
}

static inline Wo_Vec3 wo_vec3_subtract(Wo_Vec3 a, Wo_Vec3 b) {
    return wo_vec3_make(a.x - b.x, a.y - b.y, a.z - b.z);
}

static inline Wo_Vec3 wo_vec3_scale(Wo_Vec3 a, Wo_Scalar s) {
    return wo_vec3_make(a.x * s, a.y * s, a.z * s);
}

static inline Wo_Scalar wo_vec3_dot(Wo_Vec3 a, Wo_Vec3 b) {
    return a.x * b.x + a.y * b.y + a.z * b.z;
}

static inline Wo_Scalar wo_vec3_lengthsqr(Wo_Vec3 a) {
    return wo_vec3_dot(a, a);
}

static inline Wo_Scalar wo_vec3_length(Wo_Vec3 a) {
    return sqrt(wo_vec3_lengthsqr(a));
}

/* Unit vector along `a`; the zero vector is returned unchanged. */
static inline Wo_Vec3 wo_vec3_normalized(Wo_Vec3 a) {
    Wo_Scalar len = wo_vec3_length(a);
    if (len == 0.0) {
        return a;
    }
    return wo_vec3_scale(a, 1.0 / len);
}

static inline Wo_Vec3 wo_vec3_cross(Wo_Vec3 a, Wo_Vec3 b) {
    return wo_vec3_make(a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x);
}

static inline Wo_Quaternion wo_quaternion_identity(void) {
    Wo_Quaternion q;
    q.real = 1.0;
    q.imaginary = wo_vec3_0();
    return q;
}

/* Rotation by `angle_rad` about `axis` (axis need not be unit length). */
static inline Wo_Quaternion wo_quaternion_from_axis_angle(Wo_Vec3 axis, Wo_Scalar angle_rad) {
    Wo_Quaternion q;
    Wo_Vec3 u = wo_vec3_normalized(axis);
    q.real = cos(0.5 * angle_rad);
    q.imaginary = wo_vec3_scale(u, sin(0.5 * angle_rad));
    return q;
}

/* Hamilton product a*b (apply b first, then a). */
static inline Wo_Quaternion wo_quaternion_multiply(Wo_Quaternion a, Wo_Quaternion b) {
    Wo_Quaternion r;
    r.real = a.real * b.real - wo_vec3_dot(a.imaginary, b.imaginary);
    r.imaginary = wo_vec3_add(
        wo_vec3_add(wo_vec3_scale(b.imaginary, a.real), wo_vec3_scale(a.imaginary, b.real)),
        wo_vec3_cross(a.imaginary, b.imaginary));
    return r;
}

#endif /* WOLOLO_WMATH_H */
