"""glm::inverse of a mat4 in float32, restated with numpy scalars for the
tests (independent of the C/C++ restatements in vr_camera.cpp and the oracle).

glm/detail/func_matrix.inl, compute_inverse<4, 4, T, Q> (the scalar path: the
reference defines no GLM_FORCE_INTRINSICS, VulkanHeader.h:9-11), as published
in glm 0.9.9: eighteen 2x2 cofactors Coef = a*b - c*d; Fac0..Fac5; Vec0..Vec3 =
(m[1][k], m[0][k], m[0][k], m[0][k]); Inv0 = Vec1*Fac0 - Vec2*Fac1 + Vec3*Fac2,
Inv1 = Vec0*Fac0 - Vec2*Fac3 + Vec3*Fac4, Inv2 = Vec0*Fac1 - Vec1*Fac3 +
Vec3*Fac5, Inv3 = Vec0*Fac2 - Vec1*Fac4 + Vec2*Fac5 (left to right); columns
Inv0*SignA, Inv1*SignB, Inv2*SignA, Inv3*SignB with SignA = (+,-,+,-),
SignB = (-,+,-,+); Dot1 = (x + y) + (z + w) of m[0] * (Inverse[0][0],
Inverse[1][0], Inverse[2][0], Inverse[3][0]); Inverse * (1 / Dot1).  Every
float32 operation rounds on its own (numpy float32 scalars), as the
reference's build does without FMA contraction.
"""
import numpy as np

f = np.float32


def inverse(m16):
    """m16: 16 floats, column-major (m[c*4 + r]); returns 16 float32."""
    mm = [f(v) for v in m16]

    def m(c, r):
        return mm[c * 4 + r]

    def cof(a, b, c, d):
        return f(f(a * b) - f(c * d))
    c00 = cof(m(2, 2), m(3, 3), m(3, 2), m(2, 3))
    c02 = cof(m(1, 2), m(3, 3), m(3, 2), m(1, 3))
    c03 = cof(m(1, 2), m(2, 3), m(2, 2), m(1, 3))
    c04 = cof(m(2, 1), m(3, 3), m(3, 1), m(2, 3))
    c06 = cof(m(1, 1), m(3, 3), m(3, 1), m(1, 3))
    c07 = cof(m(1, 1), m(2, 3), m(2, 1), m(1, 3))
    c08 = cof(m(2, 1), m(3, 2), m(3, 1), m(2, 2))
    c10 = cof(m(1, 1), m(3, 2), m(3, 1), m(1, 2))
    c11 = cof(m(1, 1), m(2, 2), m(2, 1), m(1, 2))
    c12 = cof(m(2, 0), m(3, 3), m(3, 0), m(2, 3))
    c14 = cof(m(1, 0), m(3, 3), m(3, 0), m(1, 3))
    c15 = cof(m(1, 0), m(2, 3), m(2, 0), m(1, 3))
    c16 = cof(m(2, 0), m(3, 2), m(3, 0), m(2, 2))
    c18 = cof(m(1, 0), m(3, 2), m(3, 0), m(1, 2))
    c19 = cof(m(1, 0), m(2, 2), m(2, 0), m(1, 2))
    c20 = cof(m(2, 0), m(3, 1), m(3, 0), m(2, 1))
    c22 = cof(m(1, 0), m(3, 1), m(3, 0), m(1, 1))
    c23 = cof(m(1, 0), m(2, 1), m(2, 0), m(1, 1))
    fac = [(c00, c00, c02, c03), (c04, c04, c06, c07), (c08, c08, c10, c11),
           (c12, c12, c14, c15), (c16, c16, c18, c19), (c20, c20, c22, c23)]
    vec = [(m(1, k), m(0, k), m(0, k), m(0, k)) for k in range(4)]
    terms = [((1, 0), (2, 1), (3, 2)), ((0, 0), (2, 3), (3, 4)), ((0, 1), (1, 3), (3, 5)), ((0, 2), (1, 4), (2, 5))]
    sign_a, sign_b = (f(1), f(-1), f(1), f(-1)), (f(-1), f(1), f(-1), f(1))
    inv = [f(0)] * 16
    for col, ((va, fa), (vb, fb), (vc, fc)) in enumerate(terms):
        sign = sign_a if col % 2 == 0 else sign_b
        for i in range(4):
            t = f(f(f(vec[va][i] * fac[fa][i]) - f(vec[vb][i] * fac[fb][i])) + f(vec[vc][i] * fac[fc][i]))
            inv[col * 4 + i] = f(t * sign[i])
    dot = f(f(f(m(0, 0) * inv[0]) + f(m(0, 1) * inv[4])) + f(f(m(0, 2) * inv[8]) + f(m(0, 3) * inv[12])))
    one_over = f(f(1) / dot)
    return np.array([f(v * one_over) for v in inv], dtype=np.float32)
