// vr_camera.cpp -- host camera math of the C ABI.
//
// * reference_shader_data: the per-frame uniform producer of TestMain.cpp:
//   219-245 with GLM semantics in fp32 (GLM_FORCE_DEPTH_ZERO_TO_ONE,
//   GLM_FORCE_RADIANS: VulkanHeader.h:9-10).
// * make_ray_basis: replaces vert.glsl:17-22 and rasterisation.  The
//   fragment's ray direction normalize(W2L*fragPos - W2L*cam) (frag.glsl:36-38)
//   is the direction of the camera ray through the pixel centre.  That
//   direction is affine in the pixel coordinates:
//   dir(x,y) = o + (x+.5)*px + (y+.5)*py in box-local space.
//   It is computed in double with the fixed order of DESIGN.md sec. 3.1.
//   Built with -ffp-contract=off.
#include <cmath>
#include <cstring>

#include "vr_internal.h"

namespace vr {
namespace {

void m4_identity(float* m)
{
    std::memset(m, 0, 16 * sizeof(float));
    m[0] = m[5] = m[10] = m[15] = 1.0f;
}

// glm::rotate(m, angle, axis)
void m4_rotate(const float* m, float angle, float ax, float ay, float az, float* o)
{
    const float c = std::cos(angle), s = std::sin(angle);
    const float len = std::sqrt(ax * ax + ay * ay + az * az);
    ax /= len; ay /= len; az /= len;
    const float tx = (1.0f - c) * ax, ty = (1.0f - c) * ay, tz = (1.0f - c) * az;
    float R[3][3];
    R[0][0] = c + tx * ax;      R[0][1] = tx * ay + s * az; R[0][2] = tx * az - s * ay;
    R[1][0] = ty * ax - s * az; R[1][1] = c + ty * ay;      R[1][2] = ty * az + s * ax;
    R[2][0] = tz * ax + s * ay; R[2][1] = tz * ay - s * ax; R[2][2] = c + tz * az;
    float t[16];
    for (int col = 0; col < 3; ++col)
        for (int r = 0; r < 4; ++r)
            t[col * 4 + r] = (m[0 * 4 + r] * R[col][0] + m[1 * 4 + r] * R[col][1]) + m[2 * 4 + r] * R[col][2];
    for (int r = 0; r < 4; ++r) t[12 + r] = m[12 + r];
    std::memcpy(o, t, sizeof t);
}

// glm::lookAtRH
void m4_lookat(const float* eye, const float* ctr, const float* up, float* o)
{
    float f[3] = {ctr[0] - eye[0], ctr[1] - eye[1], ctr[2] - eye[2]};
    const float fl = 1.0f / std::sqrt(f[0] * f[0] + f[1] * f[1] + f[2] * f[2]);
    for (float& v : f) v *= fl;
    float s[3] = {f[1] * up[2] - up[1] * f[2], f[2] * up[0] - up[2] * f[0], f[0] * up[1] - up[0] * f[1]};
    const float sl = 1.0f / std::sqrt(s[0] * s[0] + s[1] * s[1] + s[2] * s[2]);
    for (float& v : s) v *= sl;
    const float u[3] = {s[1] * f[2] - f[1] * s[2], s[2] * f[0] - f[2] * s[0], s[0] * f[1] - f[0] * s[1]};
    m4_identity(o);
    o[0] = s[0]; o[4] = s[1]; o[8] = s[2];
    o[1] = u[0]; o[5] = u[1]; o[9] = u[2];
    o[2] = -f[0]; o[6] = -f[1]; o[10] = -f[2];
    o[12] = -(s[0] * eye[0] + s[1] * eye[1] + s[2] * eye[2]);
    o[13] = -(u[0] * eye[0] + u[1] * eye[1] + u[2] * eye[2]);
    o[14] = (f[0] * eye[0] + f[1] * eye[1] + f[2] * eye[2]);
}

// glm::perspectiveRH_ZO
void m4_perspective(float fovy, float aspect, float zn, float zf, float* o)
{
    const float th = std::tan(fovy / 2.0f);
    std::memset(o, 0, 16 * sizeof(float));
    o[0] = 1.0f / (aspect * th);
    o[5] = 1.0f / th;
    o[10] = zf / (zn - zf);
    o[11] = -1.0f;
    o[14] = -(zf * zn) / (zf - zn);
}

// glm::inverse of a mat4 in float (glm/detail/func_matrix.inl,
// compute_inverse<4, 4, T, Q>; the scalar path -- the reference defines no
// GLM_FORCE_INTRINSICS, VulkanHeader.h:9-11), operation for operation: the
// 18 2x2 cofactors a*b - c*d, the four Inv columns (Vec*Fac - Vec*Fac) +
// Vec*Fac, the sign flips, the determinant (x + y) + (z + w) of column 0 of
// m times row 0 of the adjugate, and each element times 1/det.  Each fp32
// operation rounds on its own (-ffp-contract=off).  The W2L of TestMain.cpp:230.
void inverse_glm(const float* mm, float* out)
{
    auto m = [mm](int c, int r) { return mm[c * 4 + r]; };
    const float c00 = m(2, 2) * m(3, 3) - m(3, 2) * m(2, 3);
    const float c02 = m(1, 2) * m(3, 3) - m(3, 2) * m(1, 3);
    const float c03 = m(1, 2) * m(2, 3) - m(2, 2) * m(1, 3);
    const float c04 = m(2, 1) * m(3, 3) - m(3, 1) * m(2, 3);
    const float c06 = m(1, 1) * m(3, 3) - m(3, 1) * m(1, 3);
    const float c07 = m(1, 1) * m(2, 3) - m(2, 1) * m(1, 3);
    const float c08 = m(2, 1) * m(3, 2) - m(3, 1) * m(2, 2);
    const float c10 = m(1, 1) * m(3, 2) - m(3, 1) * m(1, 2);
    const float c11 = m(1, 1) * m(2, 2) - m(2, 1) * m(1, 2);
    const float c12 = m(2, 0) * m(3, 3) - m(3, 0) * m(2, 3);
    const float c14 = m(1, 0) * m(3, 3) - m(3, 0) * m(1, 3);
    const float c15 = m(1, 0) * m(2, 3) - m(2, 0) * m(1, 3);
    const float c16 = m(2, 0) * m(3, 2) - m(3, 0) * m(2, 2);
    const float c18 = m(1, 0) * m(3, 2) - m(3, 0) * m(1, 2);
    const float c19 = m(1, 0) * m(2, 2) - m(2, 0) * m(1, 2);
    const float c20 = m(2, 0) * m(3, 1) - m(3, 0) * m(2, 1);
    const float c22 = m(1, 0) * m(3, 1) - m(3, 0) * m(1, 1);
    const float c23 = m(1, 0) * m(2, 1) - m(2, 0) * m(1, 1);
    const float fac[6][4] = {{c00, c00, c02, c03}, {c04, c04, c06, c07}, {c08, c08, c10, c11},
                             {c12, c12, c14, c15}, {c16, c16, c18, c19}, {c20, c20, c22, c23}};
    float vec[4][4];   // Vec0..Vec3: (m[1][k], m[0][k], m[0][k], m[0][k])
    for (int k = 0; k < 4; ++k) {
        vec[k][0] = m(1, k);
        vec[k][1] = vec[k][2] = vec[k][3] = m(0, k);
    }
    // Inv0 = Vec1*Fac0 - Vec2*Fac1 + Vec3*Fac2, Inv1 = Vec0*Fac0 - Vec2*Fac3 + Vec3*Fac4,
    // Inv2 = Vec0*Fac1 - Vec1*Fac3 + Vec3*Fac5, Inv3 = Vec0*Fac2 - Vec1*Fac4 + Vec2*Fac5
    static const int kv[4][3] = {{1, 2, 3}, {0, 2, 3}, {0, 1, 3}, {0, 1, 2}};
    static const int kf[4][3] = {{0, 1, 2}, {0, 3, 4}, {1, 3, 5}, {2, 4, 5}};
    float inv[16];
    for (int col = 0; col < 4; ++col)
        for (int i = 0; i < 4; ++i) {
            const float t = (vec[kv[col][0]][i] * fac[kf[col][0]][i] - vec[kv[col][1]][i] * fac[kf[col][1]][i]) +
                            vec[kv[col][2]][i] * fac[kf[col][2]][i];
            // SignA (+,-,+,-) on columns 0 and 2, SignB (-,+,-,+) on 1 and 3
            const bool neg = ((col & 1) == 0) ? (i & 1) : !(i & 1);
            inv[col * 4 + i] = neg ? -t : t;
        }
    const float d0 = m(0, 0) * inv[0 * 4 + 0], d1 = m(0, 1) * inv[1 * 4 + 0];
    const float d2 = m(0, 2) * inv[2 * 4 + 0], d3 = m(0, 3) * inv[3 * 4 + 0];
    const float det = (d0 + d1) + (d2 + d3);
    const float one_over = 1.0f / det;
    for (int i = 0; i < 16; ++i) out[i] = inv[i] * one_over;
}

// 4x4 inverse by cofactors, double precision (fixed evaluation order).
bool inverse_d(const double* m, double* inv)
{
    double t[16];
    t[0] = m[5] * m[10] * m[15] - m[5] * m[11] * m[14] - m[9] * m[6] * m[15] + m[9] * m[7] * m[14] + m[13] * m[6] * m[11] - m[13] * m[7] * m[10];
    t[4] = -m[4] * m[10] * m[15] + m[4] * m[11] * m[14] + m[8] * m[6] * m[15] - m[8] * m[7] * m[14] - m[12] * m[6] * m[11] + m[12] * m[7] * m[10];
    t[8] = m[4] * m[9] * m[15] - m[4] * m[11] * m[13] - m[8] * m[5] * m[15] + m[8] * m[7] * m[13] + m[12] * m[5] * m[11] - m[12] * m[7] * m[9];
    t[12] = -m[4] * m[9] * m[14] + m[4] * m[10] * m[13] + m[8] * m[5] * m[14] - m[8] * m[6] * m[13] - m[12] * m[5] * m[10] + m[12] * m[6] * m[9];
    t[1] = -m[1] * m[10] * m[15] + m[1] * m[11] * m[14] + m[9] * m[2] * m[15] - m[9] * m[3] * m[14] - m[13] * m[2] * m[11] + m[13] * m[3] * m[10];
    t[5] = m[0] * m[10] * m[15] - m[0] * m[11] * m[14] - m[8] * m[2] * m[15] + m[8] * m[3] * m[14] + m[12] * m[2] * m[11] - m[12] * m[3] * m[10];
    t[9] = -m[0] * m[9] * m[15] + m[0] * m[11] * m[13] + m[8] * m[1] * m[15] - m[8] * m[3] * m[13] - m[12] * m[1] * m[11] + m[12] * m[3] * m[9];
    t[13] = m[0] * m[9] * m[14] - m[0] * m[10] * m[13] - m[8] * m[1] * m[14] + m[8] * m[2] * m[13] + m[12] * m[1] * m[10] - m[12] * m[2] * m[9];
    t[2] = m[1] * m[6] * m[15] - m[1] * m[7] * m[14] - m[5] * m[2] * m[15] + m[5] * m[3] * m[14] + m[13] * m[2] * m[7] - m[13] * m[3] * m[6];
    t[6] = -m[0] * m[6] * m[15] + m[0] * m[7] * m[14] + m[4] * m[2] * m[15] - m[4] * m[3] * m[14] - m[12] * m[2] * m[7] + m[12] * m[3] * m[6];
    t[10] = m[0] * m[5] * m[15] - m[0] * m[7] * m[13] - m[4] * m[1] * m[15] + m[4] * m[3] * m[13] + m[12] * m[1] * m[7] - m[12] * m[3] * m[5];
    t[14] = -m[0] * m[5] * m[14] + m[0] * m[6] * m[13] + m[4] * m[1] * m[14] - m[4] * m[2] * m[13] - m[12] * m[1] * m[6] + m[12] * m[2] * m[5];
    t[3] = -m[1] * m[6] * m[11] + m[1] * m[7] * m[10] + m[5] * m[2] * m[11] - m[5] * m[3] * m[10] - m[9] * m[2] * m[7] + m[9] * m[3] * m[6];
    t[7] = m[0] * m[6] * m[11] - m[0] * m[7] * m[10] - m[4] * m[2] * m[11] + m[4] * m[3] * m[10] + m[8] * m[2] * m[7] - m[8] * m[3] * m[6];
    t[11] = -m[0] * m[5] * m[11] + m[0] * m[7] * m[9] + m[4] * m[1] * m[11] - m[4] * m[3] * m[9] - m[8] * m[1] * m[7] + m[8] * m[3] * m[5];
    t[15] = m[0] * m[5] * m[10] - m[0] * m[6] * m[9] - m[4] * m[1] * m[10] + m[4] * m[2] * m[9] + m[8] * m[1] * m[6] - m[8] * m[2] * m[5];
    const double det = m[0] * t[0] + m[1] * t[4] + m[2] * t[8] + m[3] * t[12];
    if (det == 0.0 || !std::isfinite(det)) return false;
    const double id = 1.0 / det;
    for (int i = 0; i < 16; ++i) inv[i] = t[i] * id;
    return true;
}

void mul_d(const double* a, const double* b, double* o)  // o = a * b, column-major
{
    for (int c = 0; c < 4; ++c)
        for (int r = 0; r < 4; ++r)
            o[c * 4 + r] = ((a[0 * 4 + r] * b[c * 4 + 0] + a[1 * 4 + r] * b[c * 4 + 1]) + a[2 * 4 + r] * b[c * 4 + 2]) +
                           a[3 * 4 + r] * b[c * 4 + 3];
}

}  // namespace

bool invert4_d(const double* m, double* inv) { return inverse_d(m, inv); }

void reference_shader_data(float aspect, float phi_deg, float theta_deg, float frame_time, float* obj48,
                           float* glob36)
{
    const float d2r = 0.01745329251994329576923690768489f;  // glm::radians
    float I[16], rot[16], model[16], view[16], proj[16];
    m4_identity(I);
    m4_rotate(I, phi_deg * d2r, 0.0f, 0.0f, 1.0f, rot);          // TestMain.cpp:222
    m4_rotate(rot, theta_deg * d2r, 0.0f, 1.0f, 0.0f, model);    // :224
    const float eye[3] = {3.0f, 3.0f, 3.0f}, ctr[3] = {0.0f, 0.0f, 0.0f}, up[3] = {0.0f, 0.0f, 1.0f};
    m4_lookat(eye, ctr, up, view);                                // :225
    m4_perspective(45.0f * d2r, aspect, 0.1f, 10.0f, proj);       // :226
    proj[5] *= -1.0f;                                             // :228
    std::memcpy(obj48, model, 64);
    std::memcpy(obj48 + 16, view, 64);
    std::memcpy(obj48 + 32, proj, 64);
    inverse_glm(model, glob36);                                   // :230 glm::inverse(Model), in float
    glob36[16] = 3.0f; glob36[17] = 3.0f; glob36[18] = 3.0f; glob36[19] = 0.0f;   // :242
    float* ms = glob36 + 20;                                      // :233-238
    std::memset(ms, 0, 16 * sizeof(float));
    ms[0] = -frame_time;
}

bool make_ray_basis(const float* obj48, const float* glob36, int W, int H, RayBasis* b)
{
    double M[16], V[16], P[16], L[16], PV[16], PVM[16], inv[16];
    for (int i = 0; i < 16; ++i) {
        M[i] = obj48[i]; V[i] = obj48[16 + i]; P[i] = obj48[32 + i]; L[i] = glob36[i];
    }
    const double cam_pos[3] = {glob36[16], glob36[17], glob36[18]};
    mul_d(P, V, PV);
    mul_d(PV, M, PVM);
    if (!inverse_d(PV, inv)) return false;
    // The rasteriser's rays leave the View eye, inverse(View) * (0,0,0,1).  The
    // fragment shader's ray leaves CameraPosition through the rasterised point
    // (frag.glsl:36-38).  While the two agree to float rounding the ray is the
    // camera ray through the pixel centre (cam_mode 0, the reference's case,
    // TestMain.cpp:225 / :242); otherwise the kernel finds the front-face
    // point along the eye's ray and turns towards it (cam_mode 1).
    double Vi[16];
    if (!inverse_d(V, Vi) || Vi[15] == 0.0) return false;
    const double eye[3] = {Vi[12] / Vi[15], Vi[13] / Vi[15], Vi[14] / Vi[15]};
    double err = 0.0, mag = 1.0;
    for (int i = 0; i < 3; ++i) {
        err = std::fmax(err, std::fabs(eye[i] - cam_pos[i]));
        mag = std::fmax(mag, std::fabs(eye[i]));
    }
    b->cam_mode = err > 1e-6 * mag ? 1 : 0;
    const double* cam = b->cam_mode ? eye : cam_pos;   // where the basis' rays start
    // Unprojected pixel ray minus the camera, scaled by the homogeneous w:
    // columns x, y and the far-plane point (z_ndc = 1) of inverse(P*V).
    double D[3][3];
    for (int i = 0; i < 3; ++i) {
        D[0][i] = inv[0 * 4 + i] - cam[i] * inv[0 * 4 + 3];
        D[1][i] = inv[1 * 4 + i] - cam[i] * inv[1 * 4 + 3];
        D[2][i] = (inv[2 * 4 + i] + inv[3 * 4 + i]) - cam[i] * (inv[2 * 4 + 3] + inv[3 * 4 + 3]);
    }
    double Dl[3][3];  // to box-local space with the linear part of W2L
    for (int k = 0; k < 3; ++k)
        for (int i = 0; i < 3; ++i) Dl[k][i] = (L[0 * 4 + i] * D[k][0] + L[1 * 4 + i] * D[k][1]) + L[2 * 4 + i] * D[k][2];
    const double s = 1.0 / std::sqrt((Dl[2][0] * Dl[2][0] + Dl[2][1] * Dl[2][1]) + Dl[2][2] * Dl[2][2]);
    if (!std::isfinite(s)) return false;
    const double sx = 2.0 / (double)W, sy = 2.0 / (double)H;
    for (int i = 0; i < 3; ++i) {
        b->o[i] = (float)(((Dl[2][i] - Dl[0][i]) - Dl[1][i]) * s);
        b->px[i] = (float)((Dl[0][i] * sx) * s);
        b->py[i] = (float)((Dl[1][i] * sy) * s);
        b->org[i] = (float)(((L[0 * 4 + i] * cam[0] + L[1 * 4 + i] * cam[1]) + L[2 * 4 + i] * cam[2]) + L[3 * 4 + i]);
        b->cam[i] = (float)(((L[0 * 4 + i] * cam_pos[0] + L[1 * 4 + i] * cam_pos[1]) + L[2 * 4 + i] * cam_pos[2]) +
                            L[3 * 4 + i]);
    }
    // clip rows of P*V*M act on box-local points (vert.glsl:19)
    for (int c = 0; c < 4; ++c) {
        b->r2[c] = (float)PVM[c * 4 + 2];
        b->r3[c] = (float)PVM[c * 4 + 3];
    }
    return true;
}

}  // namespace vr
