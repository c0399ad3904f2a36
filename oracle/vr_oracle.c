/*
 * vr_oracle.c -- CPU restatement of the reference ray-march hot path.
 *
 * TEST INFRASTRUCTURE ONLY (see vr_oracle.h): the checker for the HIP
 * product path and the CPU baseline of bench.py.  Never linked into, or
 * called by, the product library.
 *
 * Parity unpinned against reference outputs (the reference cannot run here
 * and ships no golden vectors); every function cites the reference lines it
 * restates.  Build: oracle/Makefile (-O3 -ffp-contract=off -fopenmp).
 */
#include "vr_oracle.h"

#include <float.h>
#include <math.h>
#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

/* ======================================================================
 * Noise: restatement of FastNoise2's Perlin / Simplex / CellularDistance
 * (vendor/noise, absent here; called at TestMain.cpp:43-45, 59-62).
 * FastNoise2 commit unknown (.gitmodules:10-12, no gitlink in the mount):
 * values are NOT pinned to FastNoise2, only to our own KAT fixtures.
 * ==================================================================== */
#define PRIME_X 501125321
#define PRIME_Y 1136930381
#define PRIME_Z 1720413743

static inline int32_t wmul(int32_t a, int32_t b) { return (int32_t)((uint32_t)a * (uint32_t)b); }
static inline int32_t wadd(int32_t a, int32_t b) { return (int32_t)((uint32_t)a + (uint32_t)b); }

/* FastNoise2 HashPrimes: seed ^ x ^ y ^ z, * 0x27d4eb2d, fold >>15 (arith). */
static inline int32_t hash_primes(int32_t seed, int32_t x, int32_t y, int32_t z)
{
    int32_t h = seed ^ x ^ y ^ z;
    h = wmul(h, 0x27d4eb2d);
    return (h >> 15) ^ h;
}
/* FastNoise2 HashPrimesHB: no final fold (high bits used by cellular). */
static inline int32_t hash_primes_hb(int32_t seed, int32_t x, int32_t y, int32_t z)
{
    int32_t h = seed ^ x ^ y ^ z;
    return wmul(h, 0x27d4eb2d);
}
/* FastNoise2 GetGradientDot (3D): 12-edge gradient set selected by hash&13. */
static inline float grad_dot(int32_t h, float fx, float fy, float fz)
{
    int32_t h13 = h & 13;
    float u = h13 < 8 ? fx : fy;
    float v = h13 < 2 ? fy : (h13 == 12 ? fx : fz);
    if (h & 1) u = -u;
    if (h & 2) v = -v;
    return u + v;
}
static inline float quintic(float t)
{
    float q = fmaf(t, 6.0f, -15.0f);
    q = fmaf(t, q, 10.0f);
    return ((t * t) * t) * q;
}
static inline float lerpf_(float a, float b, float t) { return fmaf(t, b - a, a); }

float vro_perlin3(int32_t seed, float x, float y, float z)
{
    float xs = floorf(x), ys = floorf(y), zs = floorf(z);
    int32_t x0 = wmul((int32_t)xs, PRIME_X), y0 = wmul((int32_t)ys, PRIME_Y), z0 = wmul((int32_t)zs, PRIME_Z);
    int32_t x1 = wadd(x0, PRIME_X), y1 = wadd(y0, PRIME_Y), z1 = wadd(z0, PRIME_Z);
    float xf0 = x - xs, yf0 = y - ys, zf0 = z - zs;
    float xf1 = xf0 - 1.0f, yf1 = yf0 - 1.0f, zf1 = zf0 - 1.0f;
    float u = quintic(xf0), v = quintic(yf0), w = quintic(zf0);
    float l00 = lerpf_(grad_dot(hash_primes(seed, x0, y0, z0), xf0, yf0, zf0),
                       grad_dot(hash_primes(seed, x1, y0, z0), xf1, yf0, zf0), u);
    float l10 = lerpf_(grad_dot(hash_primes(seed, x0, y1, z0), xf0, yf1, zf0),
                       grad_dot(hash_primes(seed, x1, y1, z0), xf1, yf1, zf0), u);
    float l01 = lerpf_(grad_dot(hash_primes(seed, x0, y0, z1), xf0, yf0, zf1),
                       grad_dot(hash_primes(seed, x1, y0, z1), xf1, yf0, zf1), u);
    float l11 = lerpf_(grad_dot(hash_primes(seed, x0, y1, z1), xf0, yf1, zf1),
                       grad_dot(hash_primes(seed, x1, y1, z1), xf1, yf1, zf1), u);
    return 0.964921414852142333984375f * lerpf_(lerpf_(l00, l10, v), lerpf_(l01, l11, v), w);
}

static inline float simplex_corner(int32_t seed, int32_t xp, int32_t yp, int32_t zp,
                                   float x, float y, float z)
{
    float t = 0.6f - fmaf(z, z, fmaf(y, y, x * x));
    if (!(t > 0.0f)) return 0.0f;
    float t2 = t * t;
    return (t2 * t2) * grad_dot(hash_primes(seed, xp, yp, zp), x, y, z);
}

float vro_simplex3(int32_t seed, float x, float y, float z)
{
    const float F3 = 1.0f / 3.0f, G3 = 1.0f / 6.0f, G3x2 = 1.0f / 3.0f;
    float s = ((x + y) + z) * F3;
    float xs = floorf(x + s), ys = floorf(y + s), zs = floorf(z + s);
    float t = ((xs + ys) + zs) * G3;
    float x0 = (x - xs) + t, y0 = (y - ys) + t, z0 = (z - zs) + t;
    int i1, j1, k1, i2, j2, k2;
    if (x0 >= y0) {
        if (y0 >= z0)      { i1 = 1; j1 = 0; k1 = 0; i2 = 1; j2 = 1; k2 = 0; }
        else if (x0 >= z0) { i1 = 1; j1 = 0; k1 = 0; i2 = 1; j2 = 0; k2 = 1; }
        else               { i1 = 0; j1 = 0; k1 = 1; i2 = 1; j2 = 0; k2 = 1; }
    } else {
        if (y0 < z0)       { i1 = 0; j1 = 0; k1 = 1; i2 = 0; j2 = 1; k2 = 1; }
        else if (x0 < z0)  { i1 = 0; j1 = 1; k1 = 0; i2 = 0; j2 = 1; k2 = 1; }
        else               { i1 = 0; j1 = 1; k1 = 0; i2 = 1; j2 = 1; k2 = 0; }
    }
    float x1 = (x0 - (float)i1) + G3, y1 = (y0 - (float)j1) + G3, z1 = (z0 - (float)k1) + G3;
    float x2 = (x0 - (float)i2) + G3x2, y2 = (y0 - (float)j2) + G3x2, z2 = (z0 - (float)k2) + G3x2;
    float x3 = (x0 - 1.0f) + 0.5f, y3 = (y0 - 1.0f) + 0.5f, z3 = (z0 - 1.0f) + 0.5f;
    int32_t xp = wmul((int32_t)xs, PRIME_X), yp = wmul((int32_t)ys, PRIME_Y), zp = wmul((int32_t)zs, PRIME_Z);
    float n0 = simplex_corner(seed, xp, yp, zp, x0, y0, z0);
    float n1 = simplex_corner(seed, wadd(xp, i1 ? PRIME_X : 0), wadd(yp, j1 ? PRIME_Y : 0),
                              wadd(zp, k1 ? PRIME_Z : 0), x1, y1, z1);
    float n2 = simplex_corner(seed, wadd(xp, i2 ? PRIME_X : 0), wadd(yp, j2 ? PRIME_Y : 0),
                              wadd(zp, k2 ? PRIME_Z : 0), x2, y2, z2);
    float n3 = simplex_corner(seed, wadd(xp, PRIME_X), wadd(yp, PRIME_Y), wadd(zp, PRIME_Z), x3, y3, z3);
    return 32.69428253173828125f * (((n0 + n1) + n2) + n3);
}

/* CellularDistance, EuclideanSquared, return F1 - 1, jitter 0.39614353. */
float vro_cellular3(int32_t seed, float x, float y, float z)
{
    const float jitter = 0.39614353f;
    float xr = rintf(x), yr = rintf(y), zr = rintf(z);
    int32_t xc = wmul((int32_t)xr, PRIME_X), yc = wmul((int32_t)yr, PRIME_Y), zc = wmul((int32_t)zr, PRIME_Z);
    float d0 = FLT_MAX;
    for (int xi = -1; xi <= 1; ++xi) {
        float xcf = (xr + (float)xi) - x;
        int32_t xp = wadd(xc, wmul(xi, PRIME_X));
        for (int yi = -1; yi <= 1; ++yi) {
            float ycf = (yr + (float)yi) - y;
            int32_t yp = wadd(yc, wmul(yi, PRIME_Y));
            for (int zi = -1; zi <= 1; ++zi) {
                float zcf = (zr + (float)zi) - z;
                int32_t zp = wadd(zc, wmul(zi, PRIME_Z));
                int32_t h = hash_primes_hb(seed, xp, yp, zp);
                float xd = (float)(h & 0x3ff) - 511.5f;
                float yd = (float)((h >> 10) & 0x3ff) - 511.5f;
                float zd = (float)((h >> 20) & 0x3ff) - 511.5f;
                float inv = jitter / sqrtf(fmaf(zd, zd, fmaf(yd, yd, xd * xd)));
                xd = fmaf(xd, inv, xcf);
                yd = fmaf(yd, inv, ycf);
                zd = fmaf(zd, inv, zcf);
                float dist = fmaf(zd, zd, fmaf(yd, yd, xd * xd));
                d0 = fminf(d0, dist);
            }
        }
    }
    return d0 - 1.0f;
}

static inline float noise_eval(int kind, int32_t seed, float x, float y, float z)
{
    switch (kind) {
    case VRO_NOISE_CELLULAR: return vro_cellular3(seed, x, y, z);
    case VRO_NOISE_PERLIN:   return vro_perlin3(seed, x, y, z);
    default:                 return vro_simplex3(seed, x, y, z);
    }
}

/* FastNoise2 Generator::GenUniformGrid3D: pos = (start + idx) * frequency,
 * output x-fastest, returns {min, max} over the grid (TestMain.cpp:59-62). */
void vro_gen_uniform_grid3d(int kind, float* out, int x0, int y0, int z0,
                            int nx, int ny, int nz, float freq, int32_t seed,
                            float* out_min, float* out_max)
{
    float gmin = INFINITY, gmax = -INFINITY;
#pragma omp parallel for schedule(dynamic, 1) reduction(min : gmin) reduction(max : gmax)
    for (int z = 0; z < nz; ++z) {
        float pz = (float)(z0 + z) * freq;
        for (int y = 0; y < ny; ++y) {
            float py = (float)(y0 + y) * freq;
            for (int x = 0; x < nx; ++x) {
                float px = (float)(x0 + x) * freq;
                float v = noise_eval(kind, seed, px, py, pz);
                if (out) out[((size_t)z * ny + y) * nx + x] = v;
                gmin = fminf(gmin, v);
                gmax = fmaxf(gmax, v);
            }
        }
    }
    if (out_min) *out_min = gmin;
    if (out_max) *out_max = gmax;
}

/* float -> unsigned char as x86-64 compiles static_cast<unsigned char>(float)
 * (cvttss2si to int32, keep the low byte): TestMain.cpp:84-87.            */
static inline uint8_t f2u8_trunc(float f)
{
    if (!(f > -2147483648.0f && f < 2147483648.0f)) return 0;
    return (uint8_t)(uint32_t)(int32_t)f;
}

/* TestMain.cpp:51-92: four noise grids -> normalise -> invert -> pow4 (R)
 * -> RGBA8.  literal_overwrite replicates :60 writing into noiseOutput1, so
 * R uses the f=.03 data with the f=.01 min/max and G is a constant.       */
int vro_build_volume(const vro_recipe* r, uint8_t* rgba)
{
    const int N = r->size;
    const size_t total = (size_t)N * N * N;
    float* b1 = (float*)malloc(total * sizeof(float));
    float* b2 = (float*)calloc(total, sizeof(float));
    float* b3 = (float*)malloc(total * sizeof(float));
    float* b4 = (float*)malloc(total * sizeof(float));
    if (!b1 || !b2 || !b3 || !b4) { free(b1); free(b2); free(b3); free(b4); return 1; }
    float mn[4], mx[4];
    vro_gen_uniform_grid3d(VRO_NOISE_CELLULAR, b1, 0, 0, 0, N, N, N, r->freq[0], r->seed[0], &mn[0], &mx[0]);
    vro_gen_uniform_grid3d(VRO_NOISE_CELLULAR, r->literal_overwrite ? b1 : b2, 0, 0, 0, N, N, N,
                           r->freq[1], r->seed[1], &mn[1], &mx[1]);
    vro_gen_uniform_grid3d(VRO_NOISE_PERLIN, b3, 0, 0, 0, N, N, N, r->freq[2], r->seed[2], &mn[2], &mx[2]);
    vro_gen_uniform_grid3d(VRO_NOISE_SIMPLEX, b4, 0, 0, 0, N, N, N, r->freq[3], r->seed[3], &mn[3], &mx[3]);
    float inv[4];
    for (int k = 0; k < 4; ++k) inv[k] = 1.0f / (mx[k] - mn[k]);   /* :64-67 */
#pragma omp parallel for schedule(static)
    for (long long i = 0; i < (long long)total; ++i) {
        float s1 = 1.0f - (b1[i] - mn[0]) * inv[0];                 /* :75-78 */
        float s2 = 1.0f - (b2[i] - mn[1]) * inv[1];
        float s3 = 1.0f - (b3[i] - mn[2]) * inv[2];
        float s4 = 1.0f - (b4[i] - mn[3]) * inv[3];
        s1 = s1 * ((s1 * s1) * s1);                                   /* :80 */
        rgba[4 * i + 0] = f2u8_trunc(s1 * 255.0f);                    /* :84-87 */
        rgba[4 * i + 1] = f2u8_trunc(s2 * 255.0f);
        rgba[4 * i + 2] = f2u8_trunc(s3 * 255.0f);
        rgba[4 * i + 3] = f2u8_trunc(s4 * 255.0f);
    }
    free(b1); free(b2); free(b3); free(b4);
    return 0;
}

/* ======================================================================
 * Camera producer: TestMain.cpp:219-245 with GLM semantics (float),
 * GLM_FORCE_DEPTH_ZERO_TO_ONE + GLM_FORCE_RADIANS (VulkanHeader.h:9-10).
 * Matrices column-major: m[c*4 + r].
 * ==================================================================== */
static void m4_identity(float* m) { memset(m, 0, 16 * sizeof(float)); m[0] = m[5] = m[10] = m[15] = 1.0f; }
/* glm::rotate(m, angle, axis) */
static void m4_rotate(const float* m, float angle, float ax, float ay, float az, float* o)
{
    float c = cosf(angle), s = sinf(angle);
    float len = sqrtf(ax * ax + ay * ay + az * az);
    ax /= len; ay /= len; az /= len;
    float tx = (1.0f - c) * ax, ty = (1.0f - c) * ay, tz = (1.0f - c) * az;
    float R[9];
    R[0] = c + tx * ax;      R[1] = tx * ay + s * az; R[2] = tx * az - s * ay;
    R[3] = ty * ax - s * az; R[4] = c + ty * ay;      R[5] = ty * az + s * ax;
    R[6] = tz * ax + s * ay; R[7] = tz * ay - s * ax; R[8] = c + tz * az;
    float t[16];
    for (int col = 0; col < 3; ++col)
        for (int r = 0; r < 4; ++r)
            t[col * 4 + r] = (m[0 * 4 + r] * R[col * 3 + 0] + m[1 * 4 + r] * R[col * 3 + 1]) + m[2 * 4 + r] * R[col * 3 + 2];
    for (int r = 0; r < 4; ++r) t[12 + r] = m[12 + r];
    memcpy(o, t, sizeof t);
}
/* glm::lookAtRH */
static void m4_lookat(const float* eye, const float* ctr, const float* up, float* o)
{
    float f[3] = {ctr[0] - eye[0], ctr[1] - eye[1], ctr[2] - eye[2]};
    float fl = 1.0f / sqrtf(f[0] * f[0] + f[1] * f[1] + f[2] * f[2]);
    f[0] *= fl; f[1] *= fl; f[2] *= fl;
    float s[3] = {f[1] * up[2] - up[1] * f[2], f[2] * up[0] - up[2] * f[0], f[0] * up[1] - up[0] * f[1]};
    float sl = 1.0f / sqrtf(s[0] * s[0] + s[1] * s[1] + s[2] * s[2]);
    s[0] *= sl; s[1] *= sl; s[2] *= sl;
    float u[3] = {s[1] * f[2] - f[1] * s[2], s[2] * f[0] - f[2] * s[0], s[0] * f[1] - f[0] * s[1]};
    m4_identity(o);
    o[0] = s[0]; o[4] = s[1]; o[8] = s[2];
    o[1] = u[0]; o[5] = u[1]; o[9] = u[2];
    o[2] = -f[0]; o[6] = -f[1]; o[10] = -f[2];
    o[12] = -(s[0] * eye[0] + s[1] * eye[1] + s[2] * eye[2]);
    o[13] = -(u[0] * eye[0] + u[1] * eye[1] + u[2] * eye[2]);
    o[14] = (f[0] * eye[0] + f[1] * eye[1] + f[2] * eye[2]);
}
/* glm::perspectiveRH_ZO */
static void m4_perspective(float fovy, float aspect, float zn, float zf, float* o)
{
    float th = tanf(fovy / 2.0f);
    memset(o, 0, 16 * sizeof(float));
    o[0] = 1.0f / (aspect * th);
    o[5] = 1.0f / th;
    o[10] = zf / (zn - zf);
    o[11] = -1.0f;
    o[14] = -(zf * zn) / (zf - zn);
}
/* glm::inverse of a mat4 in float (glm/detail/func_matrix.inl,
 * compute_inverse<4,4>; the scalar path, no GLM_FORCE_INTRINSICS in
 * VulkanHeader.h:9-11), op for op, each fp32 op rounded on its own
 * (-ffp-contract=off): 18 cofactors a*b - c*d; columns
 * Inv_c = (Vec_a*Fac_x - Vec_b*Fac_y) + Vec_d*Fac_z with the SignA/SignB
 * flips; det = (x + y) + (z + w) of m[0] * row 0; out = inv * (1/det). */
static void m4_inverse_glm(const float* mm, float* out)
{
#define M(c, r) mm[(c) * 4 + (r)]
    const float c00 = M(2, 2) * M(3, 3) - M(3, 2) * M(2, 3);
    const float c02 = M(1, 2) * M(3, 3) - M(3, 2) * M(1, 3);
    const float c03 = M(1, 2) * M(2, 3) - M(2, 2) * M(1, 3);
    const float c04 = M(2, 1) * M(3, 3) - M(3, 1) * M(2, 3);
    const float c06 = M(1, 1) * M(3, 3) - M(3, 1) * M(1, 3);
    const float c07 = M(1, 1) * M(2, 3) - M(2, 1) * M(1, 3);
    const float c08 = M(2, 1) * M(3, 2) - M(3, 1) * M(2, 2);
    const float c10 = M(1, 1) * M(3, 2) - M(3, 1) * M(1, 2);
    const float c11 = M(1, 1) * M(2, 2) - M(2, 1) * M(1, 2);
    const float c12 = M(2, 0) * M(3, 3) - M(3, 0) * M(2, 3);
    const float c14 = M(1, 0) * M(3, 3) - M(3, 0) * M(1, 3);
    const float c15 = M(1, 0) * M(2, 3) - M(2, 0) * M(1, 3);
    const float c16 = M(2, 0) * M(3, 2) - M(3, 0) * M(2, 2);
    const float c18 = M(1, 0) * M(3, 2) - M(3, 0) * M(1, 2);
    const float c19 = M(1, 0) * M(2, 2) - M(2, 0) * M(1, 2);
    const float c20 = M(2, 0) * M(3, 1) - M(3, 0) * M(2, 1);
    const float c22 = M(1, 0) * M(3, 1) - M(3, 0) * M(1, 1);
    const float c23 = M(1, 0) * M(2, 1) - M(2, 0) * M(1, 1);
    const float f0[4] = {c00, c00, c02, c03}, f1[4] = {c04, c04, c06, c07}, f2[4] = {c08, c08, c10, c11};
    const float f3[4] = {c12, c12, c14, c15}, f4[4] = {c16, c16, c18, c19}, f5[4] = {c20, c20, c22, c23};
    const float v0[4] = {M(1, 0), M(0, 0), M(0, 0), M(0, 0)}, v1[4] = {M(1, 1), M(0, 1), M(0, 1), M(0, 1)};
    const float v2[4] = {M(1, 2), M(0, 2), M(0, 2), M(0, 2)}, v3[4] = {M(1, 3), M(0, 3), M(0, 3), M(0, 3)};
    const float sa[4] = {1.0f, -1.0f, 1.0f, -1.0f}, sb[4] = {-1.0f, 1.0f, -1.0f, 1.0f};
    float inv[16];
    for (int i = 0; i < 4; ++i) {
        inv[0 * 4 + i] = ((v1[i] * f0[i] - v2[i] * f1[i]) + v3[i] * f2[i]) * sa[i];
        inv[1 * 4 + i] = ((v0[i] * f0[i] - v2[i] * f3[i]) + v3[i] * f4[i]) * sb[i];
        inv[2 * 4 + i] = ((v0[i] * f1[i] - v1[i] * f3[i]) + v3[i] * f5[i]) * sa[i];
        inv[3 * 4 + i] = ((v0[i] * f2[i] - v1[i] * f4[i]) + v2[i] * f5[i]) * sb[i];
    }
    const float dot = (M(0, 0) * inv[0] + M(0, 1) * inv[4]) + (M(0, 2) * inv[8] + M(0, 3) * inv[12]);
    const float one_over = 1.0f / dot;
    for (int i = 0; i < 16; ++i) out[i] = inv[i] * one_over;
#undef M
}

void vro_reference_shader_data(float aspect, float phi_deg, float theta_deg,
                               float frame_time, float* obj48, float* glob36)
{
    const float d2r = 0.01745329251994329576923690768489f;  /* glm::radians */
    float I[16], rot[16], model[16], view[16], proj[16];
    m4_identity(I);
    m4_rotate(I, phi_deg * d2r, 0.0f, 0.0f, 1.0f, rot);           /* :222 */
    m4_rotate(rot, theta_deg * d2r, 0.0f, 1.0f, 0.0f, model);     /* :224 */
    const float eye[3] = {3.0f, 3.0f, 3.0f}, ctr[3] = {0.0f, 0.0f, 0.0f}, up[3] = {0.0f, 0.0f, 1.0f};
    m4_lookat(eye, ctr, up, view);                                 /* :225 */
    m4_perspective(45.0f * d2r, aspect, 0.1f, 10.0f, proj);        /* :226 */
    proj[5] *= -1.0f;                                              /* :228 */
    memcpy(obj48, model, 64);
    memcpy(obj48 + 16, view, 64);
    memcpy(obj48 + 32, proj, 64);
    m4_inverse_glm(model, glob36);                                 /* :230 glm::inverse(Model), float */
    glob36[16] = 3.0f; glob36[17] = 3.0f; glob36[18] = 3.0f; glob36[19] = 0.0f;  /* :242 */
    float* ms = glob36 + 20;                                       /* :233-238 */
    memset(ms, 0, 16 * sizeof(float));
    ms[0] = -frame_time;
}

/* ======================================================================
 * Ray basis (replaces vert.glsl:17-22 + rasterisation): direction of the
 * pixel-centre ray, affine in the pixel coordinates.  Computed in double with
 * a fixed operation order; the product's host code restates the same.
 * ==================================================================== */
/* 4x4 inverse by cofactors in double (the ray basis, not a glm call) */
static int m4_inverse_d(const double* m, double* inv)
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
    double det = m[0] * t[0] + m[1] * t[4] + m[2] * t[8] + m[3] * t[12];
    if (det == 0.0) return 1;
    double id = 1.0 / det;
    for (int i = 0; i < 16; ++i) inv[i] = t[i] * id;
    return 0;
}
static void m4_mul_d(const double* a, const double* b, double* o)
{
    for (int c = 0; c < 4; ++c)
        for (int r = 0; r < 4; ++r)
            o[c * 4 + r] = ((a[0 * 4 + r] * b[c * 4 + 0] + a[1 * 4 + r] * b[c * 4 + 1]) + a[2 * 4 + r] * b[c * 4 + 2]) +
                           a[3 * 4 + r] * b[c * 4 + 3];
}

typedef struct {
    float org[3];   /* camera in box-local space  (frag.glsl:36)          */
    float o[3], px[3], py[3];  /* dir(x,y) = o + (x+.5) px + (y+.5) py    */
    float r2[4], r3[4];        /* rows 2,3 of P*V*M: clip z, clip w        */
    /* cam_mode 1: CameraPosition is not the View eye; org/o/px/py are the
     * eye's (the rasteriser's rays, vert.glsl:20) and cam is the box-local
     * CameraPosition the fragment's ray starts from (frag.glsl:36-38).     */
    int cam_mode;
    float cam[3];
} ray_basis;

static int make_basis(const float* obj48, const float* glob36, int W, int H, ray_basis* b)
{
    double M[16], V[16], P[16], L[16], PV[16], PVM[16], inv[16];
    for (int i = 0; i < 16; ++i) {
        M[i] = obj48[i]; V[i] = obj48[16 + i]; P[i] = obj48[32 + i]; L[i] = glob36[i];
    }
    const double cam_pos[3] = {glob36[16], glob36[17], glob36[18]};
    m4_mul_d(P, V, PV);
    m4_mul_d(PV, M, PVM);
    if (m4_inverse_d(PV, inv)) return 1;
    /* the View eye, inverse(View) * (0,0,0,1): where the rasteriser's rays
     * start.  Equal to CameraPosition up to float rounding in the reference
     * (TestMain.cpp:225, :242): then the fragment's ray is the camera ray
     * through the pixel centre (cam_mode 0).                                 */
    double Vi[16];
    if (m4_inverse_d(V, Vi) || Vi[15] == 0.0) return 1;
    const double eye[3] = {Vi[12] / Vi[15], Vi[13] / Vi[15], Vi[14] / Vi[15]};
    double err = 0.0, mag = 1.0;
    for (int i = 0; i < 3; ++i) {
        err = fmax(err, fabs(eye[i] - cam_pos[i]));
        mag = fmax(mag, fabs(eye[i]));
    }
    b->cam_mode = err > 1e-6 * mag ? 1 : 0;
    const double* cam = b->cam_mode ? eye : cam_pos;
    double D[3][3]; /* Dx, Dy, D0 (far plane, z_ndc = 1) in world space */
    for (int i = 0; i < 3; ++i) {
        D[0][i] = inv[0 * 4 + i] - cam[i] * inv[0 * 4 + 3];
        D[1][i] = inv[1 * 4 + i] - cam[i] * inv[1 * 4 + 3];
        D[2][i] = (inv[2 * 4 + i] + inv[3 * 4 + i]) - cam[i] * (inv[2 * 4 + 3] + inv[3 * 4 + 3]);
    }
    double Dl[3][3];
    for (int k = 0; k < 3; ++k)
        for (int i = 0; i < 3; ++i)
            Dl[k][i] = (L[0 * 4 + i] * D[k][0] + L[1 * 4 + i] * D[k][1]) + L[2 * 4 + i] * D[k][2];
    double s = 1.0 / sqrt((Dl[2][0] * Dl[2][0] + Dl[2][1] * Dl[2][1]) + Dl[2][2] * Dl[2][2]);
    const double sx = 2.0 / (double)W, sy = 2.0 / (double)H;
    for (int i = 0; i < 3; ++i) {
        b->o[i] = (float)(((Dl[2][i] - Dl[0][i]) - Dl[1][i]) * s);
        b->px[i] = (float)((Dl[0][i] * sx) * s);
        b->py[i] = (float)((Dl[1][i] * sy) * s);
        b->org[i] = (float)(((L[0 * 4 + i] * cam[0] + L[1 * 4 + i] * cam[1]) + L[2 * 4 + i] * cam[2]) + L[3 * 4 + i]);
        b->cam[i] = (float)(((L[0 * 4 + i] * cam_pos[0] + L[1 * 4 + i] * cam_pos[1]) + L[2 * 4 + i] * cam_pos[2]) +
                            L[3 * 4 + i]);
    }
    /* clip rows act on box-local points: P*V*M*inverse(W2L)... the reference
     * transforms local->world with Model (vert.glsl:20), so local == model
     * space and the clip rows are those of P*V*M.                          */
    for (int c = 0; c < 4; ++c) {
        b->r2[c] = (float)PVM[c * 4 + 2];
        b->r3[c] = (float)PVM[c * 4 + 3];
    }
    return 0;
}

/* ======================================================================
 * Sampler: VK_FORMAT_R8G8B8A8_UNORM 3D, LINEAR mag/min, MIRRORED_REPEAT
 * (VulkanCore.cpp:676-710, VulkanTexture.cpp:111-156), LOD 0.  Vulkan spec
 * texel-space u*N - 0.5, floor/frac, mirrored-repeat on integer indices.
 * ==================================================================== */
int vro_mirror(int i, int n)
{
    int two = 2 * n;
    int m = i % two;
    if (m < 0) m += two;
    return m < n ? m : two - 1 - m;
}

static inline float texel(const uint8_t* v, int nx, int ny, int c, int i, int j, int k)
{
    return (float)v[4 * (((size_t)k * ny + j) * nx + i) + c];
}

/* One tap at padded texel coordinate g = u*N - 0.5 + 1 (so that floor(g) is
 * the base texel + 1): weight = fract(g) clamped below 1 (v_fract_f32
 * semantics), base texel floor(g) - 1, mirrored repeat on both indices.   */
static float sample_g(const uint8_t* v, int nx, int ny, int nz, int c, float gx, float gy, float gz)
{
    float fx = floorf(gx), fy = floorf(gy), fz = floorf(gz);
    float ax = fminf(gx - fx, 0x1.fffffep-1f), ay = fminf(gy - fy, 0x1.fffffep-1f), az = fminf(gz - fz, 0x1.fffffep-1f);
    int ix = (int)fx - 1, iy = (int)fy - 1, iz = (int)fz - 1;
    int i0 = vro_mirror(ix, nx), i1 = vro_mirror(ix + 1, nx);
    int j0 = vro_mirror(iy, ny), j1 = vro_mirror(iy + 1, ny);
    int k0 = vro_mirror(iz, nz), k1 = vro_mirror(iz + 1, nz);
    float c000 = texel(v, nx, ny, c, i0, j0, k0), c100 = texel(v, nx, ny, c, i1, j0, k0);
    float c010 = texel(v, nx, ny, c, i0, j1, k0), c110 = texel(v, nx, ny, c, i1, j1, k0);
    float c001 = texel(v, nx, ny, c, i0, j0, k1), c101 = texel(v, nx, ny, c, i1, j0, k1);
    float c011 = texel(v, nx, ny, c, i0, j1, k1), c111 = texel(v, nx, ny, c, i1, j1, k1);
    float x00 = lerpf_(c000, c100, ax), x10 = lerpf_(c010, c110, ax);
    float x01 = lerpf_(c001, c101, ax), x11 = lerpf_(c011, c111, ax);
    float y0 = lerpf_(x00, x10, ay), y1 = lerpf_(x01, x11, ay);
    return lerpf_(y0, y1, az) * (1.0f / 255.0f);
}

float vro_sample(const uint8_t* v, int nx, int ny, int nz, int c, float px, float py, float pz)
{
    return sample_g(v, nx, ny, nz, c, fmaf(px, (float)nx, 0.5f), fmaf(py, (float)ny, 0.5f),
                    fmaf(pz, (float)nz, 0.5f));
}

/* exp for x <= 0, fma-only polynomial (Cephes expf coefficients): an exactly
 * specified function so the CPU and GPU agree bit for bit.                 */
float vro_expf(float x)
{
    if (x < -80.0f) return 0.0f;
    float k = rintf(x * 1.44269504088896341f);
    float r = fmaf(k, -0.693359375f, x);
    r = fmaf(k, 2.12194440e-4f, r);
    float p = 1.9875691500e-4f;
    p = fmaf(p, r, 1.3981999507e-3f);
    p = fmaf(p, r, 8.3334519073e-3f);
    p = fmaf(p, r, 4.1665795894e-2f);
    p = fmaf(p, r, 1.6666665459e-1f);
    p = fmaf(p, r, 5.0000001201e-1f);
    p = fmaf(p, r * r, r);
    p = p + 1.0f;
    int ki = (int)k;
    union { uint32_t u; float f; } sc;
    sc.u = (uint32_t)(ki + 127) << 23;
    return p * sc.f;
}

/* ======================================================================
 * The hot path: frag.glsl:34-81 per pixel.
 * ==================================================================== */
typedef struct {
    float step_size, box_min[3], box_range[3];
    float tap_S[4][3], tap_T[4][3]; /* padded texel coordinate g = fma(P, S, T) */
    float acc_limit;   /* early-out threshold on acc, +inf when off */
} march_consts;

/* tap t at ray point P samples u = P*s_t + o_t (frag.glsl:66-69); in padded
 * texel space g = u*N + 0.5 = fma(P, s_t*N, o_t*N + 0.5).                   */
static void make_consts(const vro_march* m, const float* glob36, int nx, int ny, int nz, march_consts* k)
{
    const float dims[3] = {(float)nx, (float)ny, (float)nz};
    k->step_size = (1.0f / (float)m->max_steps) * m->step_scale;          /* :42 */
    for (int a = 0; a < 3; ++a) {
        k->box_min[a] = m->box_min[a];
        k->box_range[a] = fabsf(m->box_max[a] - m->box_min[a]);          /* :51 */
    }
    const float* ms = glob36 + 20;  /* MediaScroll, column-major; tap t uses row t */
    for (int t = 0; t < 4; ++t)
        for (int a = 0; a < 3; ++a) {
            const float off = ms[a * 4 + t] * m->tap_weight[t];
            k->tap_S[t][a] = m->tap_scale[t] * dims[a];
            k->tap_T[t][a] = off * dims[a] + 0.5f;
        }
    if (m->early_out > 0.0f)
        k->acc_limit = (float)(-log((double)m->early_out) / ((double)m->density * (double)k->step_size));
    else
        k->acc_limit = INFINITY;
}

/* Returns n (>=0) for covered pixels, -1 otherwise; fills P0/step. */
static inline int ray_setup(const ray_basis* b, const vro_march* m, const march_consts* k,
                            int x, int y, float P[3], float st[3])
{
    float fx = (float)x + 0.5f, fy = (float)y + 0.5f;
    float v[3], d[3];
    for (int a = 0; a < 3; ++a) v[a] = fmaf(fy, b->py[a], fmaf(fx, b->px[a], b->o[a]));
    float len = sqrtf(fmaf(v[2], v[2], fmaf(v[1], v[1], v[0] * v[0])));   /* :38 normalize */
    for (int a = 0; a < 3; ++a) d[a] = v[a] / len;
    float tlo[3], thi[3];                                                    /* :18-27 */
    for (int a = 0; a < 3; ++a) {
        float t0 = (m->box_min[a] - b->org[a]) / d[a];
        float t1 = (m->box_max[a] - b->org[a]) / d[a];
        tlo[a] = fminf(t0, t1);
        thi[a] = fmaxf(t0, t1);
    }
    float tn = fmaxf(fmaxf(tlo[0], tlo[1]), tlo[2]);
    float tf = fminf(fminf(thi[0], thi[1]), thi[2]);
    if (!(tn <= tf)) return -1;
    float pin[3], pout[3], c[3];                                             /* :43-44 */
    for (int a = 0; a < 3; ++a) {
        pin[a] = fmaf(d[a], tn, b->org[a]);
        c[a] = b->org[a];
    }
    /* coverage: the front-face fragment survives clipping (0 <= z <= w)   */
    float zc = fmaf(b->r2[2], pin[2], fmaf(b->r2[1], pin[1], fmaf(b->r2[0], pin[0], b->r2[3])));
    float wc = fmaf(b->r3[2], pin[2], fmaf(b->r3[1], pin[1], fmaf(b->r3[0], pin[0], b->r3[3])));
    if (!(wc > 0.0f && zc >= 0.0f && zc <= wc)) return -1;
    if (b->cam_mode) {
        /* pin is the rasterised front-face point (vert.glsl:20); the
         * fragment's ray leaves CameraPosition through it (frag.glsl:36-38)
         * and IntersectAABB runs again from CameraPosition (:39).          */
        float f[3];
        for (int a = 0; a < 3; ++a) { c[a] = b->cam[a]; f[a] = pin[a] - c[a]; }
        float fl = sqrtf(fmaf(f[2], f[2], fmaf(f[1], f[1], f[0] * f[0])));
        for (int a = 0; a < 3; ++a) d[a] = f[a] / fl;
        for (int a = 0; a < 3; ++a) {
            float t0 = (m->box_min[a] - c[a]) / d[a];
            float t1 = (m->box_max[a] - c[a]) / d[a];
            tlo[a] = fminf(t0, t1);
            thi[a] = fmaxf(t0, t1);
        }
        tn = fmaxf(fmaxf(tlo[0], tlo[1]), tlo[2]);
        tf = fminf(fminf(thi[0], thi[1]), thi[2]);
        for (int a = 0; a < 3; ++a) pin[a] = fmaf(d[a], tn, c[a]);
    }
    for (int a = 0; a < 3; ++a) pout[a] = fmaf(d[a], tf, c[a]);
    float dd[3] = {pout[0] - pin[0], pout[1] - pin[1], pout[2] - pin[2]};
    float dist = sqrtf(fmaf(dd[2], dd[2], fmaf(dd[1], dd[1], dd[0] * dd[0])));
    float q = dist / k->step_size;                                           /* :46 */
    /* int(NaN) (a camera on the fragment) is undefined in GLSL: 0 here      */
    int n = q >= (float)m->max_steps ? m->max_steps : q >= 0.0f ? (int)q : 0;
    for (int a = 0; a < 3; ++a) {                                            /* :45,49-54 */
        P[a] = (pin[a] - k->box_min[a]) / k->box_range[a];
        st[a] = (k->step_size * d[a]) / k->box_range[a];
    }
    return n;
}

int vro_step_counts(const float* obj48, const float* glob36, const vro_march* m,
                    int width, int height, int32_t* n_out)
{
    ray_basis b;
    march_consts k;
    if (make_basis(obj48, glob36, width, height, &b)) return 1;
    make_consts(m, glob36, 1, 1, 1, &k);
#pragma omp parallel for schedule(dynamic, 4)
    for (int y = 0; y < height; ++y)
        for (int x = 0; x < width; ++x) {
            float P[3], st[3];
            n_out[(size_t)y * width + x] = ray_setup(&b, m, &k, x, y, P, st);
        }
    return 0;
}

static inline void store_px(void* out, size_t pitch, int row, int x, int fmt, float g, int covered)
{
    char* base = (char*)out + (size_t)row * pitch;
    if (fmt == VRO_FMT_RGBA32F) {
        float* p = (float*)base + 4 * (size_t)x;
        p[0] = p[1] = p[2] = covered ? g : 0.0f;
        p[3] = 1.0f;
        return;
    }
    uint8_t* p = (uint8_t*)base + 4 * (size_t)x;
    uint8_t q = 0;
    if (covered) {
        float c = fminf(fmaxf(g, 0.0f), 1.0f);
        if (fmt == VRO_FMT_RGBA8_SRGB)
            c = c <= 0.0031308f ? c * 12.92f : fmaf(1.055f, powf(c, 1.0f / 2.4f), -0.055f);
        q = (uint8_t)rintf(c * 255.0f);
    }
    p[0] = p[1] = p[2] = q;
    p[3] = 255;
}

int vro_render(const uint8_t* vol, int nx, int ny, int nz,
               const float* obj48, const float* glob36, const vro_march* m,
               int width, int height, int format, void* out, size_t pitch,
               int band_rows, int band_stride, int band_first,
               int64_t* steps_out, int threads)
{
    ray_basis b;
    march_consts k;
    if (m->max_steps <= 0 || nx <= 0 || ny <= 0 || nz <= 0 || width <= 0 || height <= 0) return 2;
    if (make_basis(obj48, glob36, width, height, &b)) return 1;
    make_consts(m, glob36, nx, ny, nz, &k);
    if (band_rows <= 0) { band_rows = height; band_stride = 1; band_first = 0; }
    if (band_stride <= 0) band_stride = 1;
    const int nbands = (height + band_rows - 1) / band_rows;
    /* packed output rows for the selected bands */
    int nsel = 0;
    for (int bb = band_first; bb < nbands; bb += band_stride) nsel++;
    const int out_rows = nsel * band_rows;
    int64_t total = 0;
#ifdef _OPENMP
    if (threads > 0) omp_set_num_threads(threads);
#else
    (void)threads;
#endif
#pragma omp parallel for schedule(dynamic, 1) reduction(+ : total)
    for (int orow = 0; orow < out_rows; ++orow) {
        const int sel = orow / band_rows, r = orow % band_rows;
        const int y = (band_first + sel * band_stride) * band_rows + r;
        if (y >= height) continue;
        for (int x = 0; x < width; ++x) {
            float P[3], st[3];
            int n = ray_setup(&b, m, &k, x, y, P, st);
            if (n < 0) { store_px(out, pitch, orow, x, format, 0.0f, 0); continue; }
            float acc = 0.0f;
            int i = 0;
            for (; i < n; ++i) {                                              /* :57-75 */
                float s[4];
                for (int t = 0; t < 4; ++t)
                    s[t] = sample_g(vol, nx, ny, nz, t, fmaf(P[0], k.tap_S[t][0], k.tap_T[t][0]),
                                    fmaf(P[1], k.tap_S[t][1], k.tap_T[t][1]),
                                    fmaf(P[2], k.tap_S[t][2], k.tap_T[t][2]));
                float cur = ((s[0] * s[1]) * (s[2] + s[3])) * m->scale;      /* :71 */
                acc = acc + cur;                                             /* :73 */
                P[0] = P[0] + st[0]; P[1] = P[1] + st[1]; P[2] = P[2] + st[2]; /* :74 */
                if (acc > k.acc_limit) { ++i; break; }
            }
            total += i;
            float a = acc * k.step_size;                                     /* :76 */
            float e = vro_expf(m->density * fminf(-a, 0.0f));               /* :79 */
            store_px(out, pitch, orow, x, format, 1.0f - e, 1);
        }
    }
    if (steps_out) *steps_out = total;
    return 0;
}

/* ======================================================================
 * Procedural medium (BASELINE configs 2/3): build-defined, no reference
 * counterpart.  Same ray setup and march as the
 * grid path; the density comes from the noise functions above.
 * ==================================================================== */
float vro_procedural_density(const vro_procedural* p, float scale, float px, float py, float pz)
{
    const float qx = px * p->grid_scale, qy = py * p->grid_scale, qz = pz * p->grid_scale;
    float f = p->freq0, amp = 1.0f, fbm = 0.0f;
    for (int o = 0; o < p->octaves; ++o) {
        fbm = fmaf(amp, vro_perlin3(p->seed_fbm, qx * f, qy * f, qz * f), fbm);
        f = f * p->lacunarity;
        amp = amp * p->gain;
    }
    const float wf = p->worley_freq;
    const float f1 = vro_cellular3(p->seed_worley, qx * wf, qy * wf, qz * wf) + 1.0f;
    return fmaxf(fbm * (1.0f - f1), 0.0f) * scale;
}

/* Worley cells the device computes for this evaluation (vr option "count" =
 * 2; test infrastructure, mirrors noise::cellular_table9's pruning decision):
 * the 8 cells of the unit cube around the sample, and all 27 of
 * vro_cellular3's block again when the cube's minimum does not provably hold
 * F1: sqrt(d_cube) + 0.3962 squared > T + 1 + 2 min g.  The device's square
 * root is v_sqrt_f32 and this one is correctly rounded, so a sample whose
 * test sits within an ulp of the bound may count differently (tests allow for
 * it). */
int vro_worley_cells(const vro_procedural* p, float px, float py, float pz)
{
    const float wf = p->worley_freq;
    const float x = (px * p->grid_scale) * wf, y = (py * p->grid_scale) * wf, z = (pz * p->grid_scale) * wf;
    const float jitter = 0.39614353f;
    const float xf = floorf(x), yf = floorf(y), zf = floorf(z);
    const float c0[3] = {xf - x, yf - y, zf - z}, c1[3] = {(xf + 1.0f) - x, (yf + 1.0f) - y, (zf + 1.0f) - z};
    float d0 = FLT_MAX;
    for (int xi = 0; xi <= 1; ++xi)
        for (int yi = 0; yi <= 1; ++yi)
            for (int zi = 0; zi <= 1; ++zi) {
                const int32_t h = hash_primes_hb(p->seed_worley, wmul((int32_t)xf + xi, PRIME_X),
                                                 wmul((int32_t)yf + yi, PRIME_Y), wmul((int32_t)zf + zi, PRIME_Z));
                float xd = (float)(h & 0x3ff) - 511.5f;
                float yd = (float)((h >> 10) & 0x3ff) - 511.5f;
                float zd = (float)((h >> 20) & 0x3ff) - 511.5f;
                const float inv = jitter / sqrtf(fmaf(zd, zd, fmaf(yd, yd, xd * xd)));
                xd = fmaf(xd, inv, xi ? c1[0] : c0[0]);
                yd = fmaf(yd, inv, yi ? c1[1] : c0[1]);
                zd = fmaf(zd, inv, zi ? c1[2] : c0[2]);
                d0 = fminf(d0, fmaf(zd, zd, fmaf(yd, yd, xd * xd)));
            }
    const float gx = fminf(-c0[0], c1[0]), gy = fminf(-c0[1], c1[1]), gz = fminf(-c0[2], c1[2]);
    const float bound = fmaf(2.0f, fminf(gx, fminf(gy, gz)), fmaf(gz, gz, fmaf(gy, gy, fmaf(gx, gx, 1.0f))));
    const float e = sqrtf(d0) + 0.3962f;
    return e * e > bound ? 35 : 8;
}

static inline int inside01(const float q[3])
{
    return q[0] >= 0.0f && q[0] <= 1.0f && q[1] >= 0.0f && q[1] <= 1.0f && q[2] >= 0.0f && q[2] <= 1.0f;
}

int vro_render_procedural(const vro_procedural* p, const float* obj48, const float* glob36, const vro_march* m,
                          int width, int height, int format, void* out, size_t pitch,
                          int band_rows, int band_stride, int band_first, int64_t* steps_out,
                          int64_t* evals_out, int64_t* cells_out, int threads)
{
    ray_basis b;
    march_consts k;
    if (m->max_steps <= 0 || width <= 0 || height <= 0) return 2;
    if (make_basis(obj48, glob36, width, height, &b)) return 1;
    make_consts(m, glob36, 1, 1, 1, &k);
    float lstep[3];
    for (int a = 0; a < 3; ++a) lstep[a] = (k.step_size * p->sun_dir[a]) / k.box_range[a];
    const float od = k.step_size * m->density;   /* optical depth per unit density */
    if (band_rows <= 0) { band_rows = height; band_stride = 1; band_first = 0; }
    if (band_stride <= 0) band_stride = 1;
    const int nbands = (height + band_rows - 1) / band_rows;
    int nsel = 0;
    for (int bb = band_first; bb < nbands; bb += band_stride) nsel++;
    const int out_rows = nsel * band_rows;
    int64_t total = 0, shadow_total = 0, cells_total = 0;
    const int count_cells = cells_out != NULL;
#ifdef _OPENMP
    if (threads > 0) omp_set_num_threads(threads);
#else
    (void)threads;
#endif
#pragma omp parallel for schedule(dynamic, 1) reduction(+ : total, shadow_total, cells_total)
    for (int orow = 0; orow < out_rows; ++orow) {
        const int sel = orow / band_rows, r = orow % band_rows;
        const int y = (band_first + sel * band_stride) * band_rows + r;
        if (y >= height) continue;
        for (int x = 0; x < width; ++x) {
            float P[3], st[3];
            int n = ray_setup(&b, m, &k, x, y, P, st);
            if (n < 0) { store_px(out, pitch, orow, x, format, 0.0f, 0); continue; }
            float acc = 0.0f, rad = 0.0f, tv = 1.0f;
            int64_t shadow = 0;
            int i = 0;
            for (; i < n; ++i) {
                const float rho = vro_procedural_density(p, m->scale, P[0], P[1], P[2]);
                if (count_cells) cells_total += vro_worley_cells(p, P[0], P[1], P[2]);
                if (p->shadow_steps > 0 && rho > 0.0f) {
                    float q[3] = {P[0], P[1], P[2]}, sl = 0.0f;
                    for (int j = 0; j < p->shadow_steps; ++j) {
                        q[0] = q[0] + lstep[0]; q[1] = q[1] + lstep[1]; q[2] = q[2] + lstep[2];
                        if (inside01(q)) {
                            sl = sl + vro_procedural_density(p, m->scale, q[0], q[1], q[2]);
                            if (count_cells) cells_total += vro_worley_cells(p, q[0], q[1], q[2]);
                            ++shadow;
                        }
                    }
                    const float tl = vro_expf(-(sl * od));
                    rad = fmaf((tv * (rho * od)), tl, rad);
                }
                acc = acc + rho;
                if (p->shadow_steps > 0) tv = vro_expf(-(acc * od));
                P[0] = P[0] + st[0]; P[1] = P[1] + st[1]; P[2] = P[2] + st[2];
                if (acc > k.acc_limit) { ++i; break; }
            }
            total += i;
            if (n > 0) shadow_total += shadow;
            float g;
            if (p->shadow_steps > 0) {
                g = rad;
            } else {
                const float a = acc * k.step_size;
                g = 1.0f - vro_expf(m->density * fminf(-a, 0.0f));
            }
            store_px(out, pitch, orow, x, format, g, 1);
        }
    }
    if (steps_out) *steps_out = total;
    if (evals_out) *evals_out = total + shadow_total;
    if (cells_out) *cells_out = cells_total;
    return 0;
}
