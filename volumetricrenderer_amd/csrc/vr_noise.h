// vr_noise.h -- device noise generators for the volume producer
// (reference call sites TestMain.cpp:43-45, 59-62).
//
// FastNoise2 (vendor/noise) is absent from the reference mount and its commit
// is unknown (.gitmodules:10-12).  These are restatements of its published
// generators -- HashPrimes with primes 501125321 / 1136930381 / 1720413743 and
// multiplier 0x27d4eb2d, the hash&13 gradient set, quintic interpolation,
// 3D simplex with the 0.6 falloff, cellular F1 with hash-derived jitter --
// with a fixed fp32 operation order.  Values are pinned
// to our own known-answer fixtures, not to FastNoise2 (parity unpinned).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace vr {
namespace noise {

constexpr int32_t kPX = 501125321, kPY = 1136930381, kPZ = 1720413743;

__device__ __forceinline__ int32_t wmul(int32_t a, int32_t b) { return (int32_t)((uint32_t)a * (uint32_t)b); }
__device__ __forceinline__ int32_t wadd(int32_t a, int32_t b) { return (int32_t)((uint32_t)a + (uint32_t)b); }

__device__ __forceinline__ int32_t hash(int32_t seed, int32_t x, int32_t y, int32_t z)
{
    const int32_t h = wmul(seed ^ x ^ y ^ z, 0x27d4eb2d);
    return (h >> 15) ^ h;
}
__device__ __forceinline__ int32_t hash_hb(int32_t seed, int32_t x, int32_t y, int32_t z)
{
    return wmul(seed ^ x ^ y ^ z, 0x27d4eb2d);
}
__device__ __forceinline__ float grad(int32_t h, float fx, float fy, float fz)
{
    const int32_t h13 = h & 13;
    float u = h13 < 8 ? fx : fy;
    float v = h13 < 2 ? fy : (h13 == 12 ? fx : fz);
    u = (h & 1) ? -u : u;
    v = (h & 2) ? -v : v;
    return u + v;
}
__device__ __forceinline__ float quintic(float t)
{
    float q = fmaf(t, 6.0f, -15.0f);
    q = fmaf(t, q, 10.0f);
    return ((t * t) * t) * q;
}
__device__ __forceinline__ float lerp(float a, float b, float t) { return fmaf(t, b - a, a); }

__device__ inline float perlin(int32_t seed, float x, float y, float z)
{
    const float xs = floorf(x), ys = floorf(y), zs = floorf(z);
    const int32_t x0 = wmul((int32_t)xs, kPX), y0 = wmul((int32_t)ys, kPY), z0 = wmul((int32_t)zs, kPZ);
    const int32_t x1 = wadd(x0, kPX), y1 = wadd(y0, kPY), z1 = wadd(z0, kPZ);
    const float xf0 = x - xs, yf0 = y - ys, zf0 = z - zs;
    const float xf1 = xf0 - 1.0f, yf1 = yf0 - 1.0f, zf1 = zf0 - 1.0f;
    const float u = quintic(xf0), v = quintic(yf0), w = quintic(zf0);
    const float l00 = lerp(grad(hash(seed, x0, y0, z0), xf0, yf0, zf0), grad(hash(seed, x1, y0, z0), xf1, yf0, zf0), u);
    const float l10 = lerp(grad(hash(seed, x0, y1, z0), xf0, yf1, zf0), grad(hash(seed, x1, y1, z0), xf1, yf1, zf0), u);
    const float l01 = lerp(grad(hash(seed, x0, y0, z1), xf0, yf0, zf1), grad(hash(seed, x1, y0, z1), xf1, yf0, zf1), u);
    const float l11 = lerp(grad(hash(seed, x0, y1, z1), xf0, yf1, zf1), grad(hash(seed, x1, y1, z1), xf1, yf1, zf1), u);
    return 0.964921414852142333984375f * lerp(lerp(l00, l10, v), lerp(l01, l11, v), w);
}

// Perlin with the gradient dot product from a table (the LDS table of the
// procedural march): for hash bits k = hash & 15, grad_entry(k) is the
// (gx, gy, gz) in {-1, 0, 1} that grad() selects, and the dot is
// fma(gx, fx, fma(gy, fy, gz * fz)).  Exactly one component is 0, so each
// fma adds one exact term to an exact term: the value is grad()'s u + v,
// correctly rounded once.  Only the sign of an exact zero can differ, and a
// zero (of either sign) leaves every later sum, lerp and max unchanged, so
// the rendered pixels are identical.
__device__ __forceinline__ float4 grad_entry(int k)
{
    float g[3] = {0.0f, 0.0f, 0.0f};
    const int h13 = k & 13;
    const int ua = h13 < 8 ? 0 : 1;
    const int va = h13 < 2 ? 1 : (h13 == 12 ? 0 : 2);
    g[ua] += (k & 1) ? -1.0f : 1.0f;
    g[va] += (k & 2) ? -1.0f : 1.0f;
    return make_float4(g[0], g[1], g[2], 0.0f);
}
// perlin_gp: the two x-neighbour corners of each (y, z) edge are done
// together in packed math: a 256-entry table of gradient PAIRS, entry
// e = ka | kb << 4.  Part 0 {gx_a, gx_b, gy_a, gy_b} is gp[e], part 1
// {gz_a, gz_b, 0, 0} is gp[256 + e]: both at 16-B stride from one address
// register (the second read takes a 4 KiB immediate offset), so a 16-lane
// ds_read_b128 group spreads over 16 bank slots (e & 15), not the 8 of
// interleaved 32-B entries.  One b128 + one b64 read yields register pairs
// that feed v_pk_mul / v_pk_fma directly: 3 packed ops per corner pair.  A
// packed fma is two IEEE fmas.  Per octave 114 VALU + 8 LDS reads, against
// ~193 VALU for perlin().
typedef float vr_pf2 __attribute__((ext_vector_type(2)));
// A loop-invariant value pinned to a VGPR.  gfx950 issues a VALU op that reads
// an SGPR (kernel parameters, wave-uniform constants) at half rate, like the
// 4-cycle ops (tools/valu_calib.hip), so values many VALU ops read in the
// hot loops are copied to VGPRs once (the empty asm is hoisted).
__device__ __forceinline__ float in_vgpr(float x) { asm("" : "+v"(x)); return x; }
__device__ __forceinline__ uint32_t in_vgpr(uint32_t x) { asm("" : "+v"(x)); return x; }
__device__ __forceinline__ void grad_pair_entry(int e, float4* gp)
{
    const float4 a = grad_entry(e & 15), b = grad_entry(e >> 4);
    gp[e] = make_float4(a.x, b.x, a.y, b.y);
    gp[256 + e] = make_float4(a.z, b.z, 0.0f, 0.0f);
}
// Byte offset 16 e of the pair entry e = k_a | k_b << 4 of two corners with
// hash inputs va, vb, where k = ((h >> 15) ^ h) & 15 and h = va * M (hash()).
// The shifts are folded into the multiplier: h << 4 = va * (M << 4), and bits
// 15..18 of h sit at 19..22 of that, so k_a << 4 = ((A >> 15) ^ A) & 0xf0 with
// A = va * (M << 4); likewise k_b << 8 with M << 8.  Only right shifts, xor,
// and, or: no 4-cycle left shifts (tools/valu_calib.hip).
// The masks come in VGPRs (in_vgpr): as an SGPR or literal operand of the
// 3-operand bitop3 they would halve its issue rate.
__device__ __forceinline__ unsigned pair_offset(int32_t va, int32_t vb, uint32_t m0, uint32_t m1)
{
    const uint32_t A = (uint32_t)va * (0x27d4eb2du << 4), B = (uint32_t)vb * (0x27d4eb2du << 8);
    return (((A >> 15) ^ A) & m0) | (((B >> 15) ^ B) & m1);
}
__device__ __forceinline__ float gdot_pair_lerp(const float4* __restrict__ gp, unsigned off16, vr_pf2 fx,
                                                float fy, float fz, float u)
{
    const float4* e = reinterpret_cast<const float4*>(reinterpret_cast<const char*>(gp) + off16);
    const float4 g0 = e[0];
    const float2 g1 = *reinterpret_cast<const float2*>(e + 256);
    const vr_pf2 dz = vr_pf2{g1.x, g1.y} * vr_pf2{fz, fz};
    const vr_pf2 dy = __builtin_elementwise_fma(vr_pf2{g0.z, g0.w}, vr_pf2{fy, fy}, dz);
    const vr_pf2 d = __builtin_elementwise_fma(vr_pf2{g0.x, g0.y}, fx, dy);
    return lerp(d.x, d.y, u);
}
__device__ inline float perlin_gp(const float4* __restrict__ gp, int32_t seed, float x, float y, float z)
{
    const float xs = floorf(x), ys = floorf(y), zs = floorf(z);
    const int32_t x0 = wmul((int32_t)xs, kPX), y0 = wmul((int32_t)ys, kPY), z0 = wmul((int32_t)zs, kPZ);
    const int32_t x1 = wadd(x0, kPX), y1 = wadd(y0, kPY), z1 = wadd(z0, kPZ);
    const float xf0 = x - xs, yf0 = y - ys, zf0 = z - zs;
    const float xf1 = xf0 - 1.0f, yf1 = yf0 - 1.0f, zf1 = zf0 - 1.0f;
    const float u = quintic(xf0), v = quintic(yf0), w = quintic(zf0);
    const vr_pf2 fx = {xf0, xf1};
    const int32_t s0 = seed ^ x0, s1 = seed ^ x1;   // hash inputs seed ^ x ^ y ^ z (hash())
    const int32_t y0z0 = y0 ^ z0, y1z0 = y1 ^ z0, y0z1 = y0 ^ z1, y1z1 = y1 ^ z1;
    const uint32_t m0 = in_vgpr(0xf0u), m1 = in_vgpr(0xf00u);
    const float l00 = gdot_pair_lerp(gp, pair_offset(s0 ^ y0z0, s1 ^ y0z0, m0, m1), fx, yf0, zf0, u);
    const float l10 = gdot_pair_lerp(gp, pair_offset(s0 ^ y1z0, s1 ^ y1z0, m0, m1), fx, yf1, zf0, u);
    const float l01 = gdot_pair_lerp(gp, pair_offset(s0 ^ y0z1, s1 ^ y0z1, m0, m1), fx, yf0, zf1, u);
    const float l11 = gdot_pair_lerp(gp, pair_offset(s0 ^ y1z1, s1 ^ y1z1, m0, m1), fx, yf1, zf1, u);
    return 0.964921414852142333984375f * lerp(lerp(l00, l10, v), lerp(l01, l11, v), w);
}

// Perlin lattice table (the procedural march's global table, TABLE 3): for
// every lattice cell (xs, ys, zs) the four byte offsets perlin_gp derives by
// hashing for the cell's (y, z) edges -- (y0,z0), (y1,z0) in the low and high
// 16 bits of .x, (y0,z1), (y1,z1) of .y.  The hash depends only on the seed
// and the integer corners, and every octave of the fBm uses the same seed, so
// one table serves all octaves.  Per octave the sample then costs one 8-byte
// load and 4 mask/shift ops instead of 3 conversions, 11 multiplies, 14 xors
// and the offset extraction.
__device__ inline uint2 perlin_lattice_entry(int32_t seed, int ix, int iy, int iz)
{
    const int32_t x0 = wmul(ix, kPX), y0 = wmul(iy, kPY), z0 = wmul(iz, kPZ);
    const int32_t x1 = wadd(x0, kPX), y1 = wadd(y0, kPY), z1 = wadd(z0, kPZ);
    const int32_t s0 = seed ^ x0, s1 = seed ^ x1;
    const int32_t y0z0 = y0 ^ z0, y1z0 = y1 ^ z0, y0z1 = y0 ^ z1, y1z1 = y1 ^ z1;
    const unsigned o00 = pair_offset(s0 ^ y0z0, s1 ^ y0z0, 0xf0u, 0xf00u);
    const unsigned o10 = pair_offset(s0 ^ y1z0, s1 ^ y1z0, 0xf0u, 0xf00u);
    const unsigned o01 = pair_offset(s0 ^ y0z1, s1 ^ y0z1, 0xf0u, 0xf00u);
    const unsigned o11 = pair_offset(s0 ^ y1z1, s1 ^ y1z1, 0xf0u, 0xf00u);
    return make_uint2(o00 | (o10 << 16), o01 | (o11 << 16));
}
// perlin_gp with the edge offsets from the lattice table word w of cell
// (xs, ys, zs) = floor(x, y, z): the same gradient pairs, fractions, fades and
// lerps in the same order, so the value is perlin_gp's bit for bit.
__device__ inline float perlin_lat(const float4* __restrict__ gp, uint2 w, float x, float y, float z, float xs,
                                   float ys, float zs)
{
    const float xf0 = x - xs, yf0 = y - ys, zf0 = z - zs;
    const float xf1 = xf0 - 1.0f, yf1 = yf0 - 1.0f, zf1 = zf0 - 1.0f;
    const float u = quintic(xf0), v = quintic(yf0), w_ = quintic(zf0);
    const vr_pf2 fx = {xf0, xf1};
    const float l00 = gdot_pair_lerp(gp, w.x & 0xffffu, fx, yf0, zf0, u);
    const float l10 = gdot_pair_lerp(gp, w.x >> 16, fx, yf1, zf0, u);
    const float l01 = gdot_pair_lerp(gp, w.y & 0xffffu, fx, yf0, zf1, u);
    const float l11 = gdot_pair_lerp(gp, w.y >> 16, fx, yf1, zf1, u);
    return 0.964921414852142333984375f * lerp(lerp(l00, l10, v), lerp(l01, l11, v), w_);
}

__device__ __forceinline__ float simplex_corner(int32_t seed, int32_t xp, int32_t yp, int32_t zp,
                                                float x, float y, float z)
{
    const float t = 0.6f - fmaf(z, z, fmaf(y, y, x * x));
    if (!(t > 0.0f)) return 0.0f;
    const float t2 = t * t;
    return (t2 * t2) * grad(hash(seed, xp, yp, zp), x, y, z);
}

__device__ inline float simplex(int32_t seed, float x, float y, float z)
{
    const float F3 = 1.0f / 3.0f, G3 = 1.0f / 6.0f, G3x2 = 1.0f / 3.0f;
    const float s = ((x + y) + z) * F3;
    const float xs = floorf(x + s), ys = floorf(y + s), zs = floorf(z + s);
    const float t = ((xs + ys) + zs) * G3;
    const float x0 = (x - xs) + t, y0 = (y - ys) + t, z0 = (z - zs) + t;
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
    const float x1 = (x0 - (float)i1) + G3, y1 = (y0 - (float)j1) + G3, z1 = (z0 - (float)k1) + G3;
    const float x2 = (x0 - (float)i2) + G3x2, y2 = (y0 - (float)j2) + G3x2, z2 = (z0 - (float)k2) + G3x2;
    const float x3 = (x0 - 1.0f) + 0.5f, y3 = (y0 - 1.0f) + 0.5f, z3 = (z0 - 1.0f) + 0.5f;
    const int32_t xp = wmul((int32_t)xs, kPX), yp = wmul((int32_t)ys, kPY), zp = wmul((int32_t)zs, kPZ);
    const float n0 = simplex_corner(seed, xp, yp, zp, x0, y0, z0);
    const float n1 = simplex_corner(seed, wadd(xp, i1 ? kPX : 0), wadd(yp, j1 ? kPY : 0), wadd(zp, k1 ? kPZ : 0), x1, y1, z1);
    const float n2 = simplex_corner(seed, wadd(xp, i2 ? kPX : 0), wadd(yp, j2 ? kPY : 0), wadd(zp, k2 ? kPZ : 0), x2, y2, z2);
    const float n3 = simplex_corner(seed, wadd(xp, kPX), wadd(yp, kPY), wadd(zp, kPZ), x3, y3, z3);
    return 32.69428253173828125f * (((n0 + n1) + n2) + n3);
}

// Cell-point magnitude jitter / sqrt(d2) (correctly rounded division of the
// correctly rounded square root, as the oracle computes it).  d2 is a sum of
// three squared half-integers in [-511.5, 511.5]: d2 = K / 4 with integer
// K = 3 (mod 8), K <= 3 * 1023^2, always exact in fp32.  Candidate fast
// sequences are verified exhaustively over that domain by vr_selftest
// ("cell_inv_a" .. "cell_inv_c"); the one cellular() uses must report 0.
constexpr float kCellJitter = 0.39614353f;
__device__ __forceinline__ float cell_inv_ieee(float d2) { return kCellJitter / sqrtf(d2); }
__device__ __forceinline__ float cell_inv_a(float d2) { return kCellJitter * __builtin_amdgcn_rsqf(d2); }
__device__ __forceinline__ float cell_inv_b(float d2)
{
    const float s = __builtin_amdgcn_sqrtf(d2);
    const float r = __builtin_amdgcn_rcpf(s);
    const float q = kCellJitter * r;
    return fmaf(fmaf(-q, s, kCellJitter), r, q);
}
__device__ __forceinline__ float cell_inv_c(float d2)
{
    float s = __builtin_amdgcn_sqrtf(d2);   // <= 1 ulp; d2 is normal, no scaling needed
    const float sdn = __uint_as_float(__float_as_uint(s) - 1u), sup = __uint_as_float(__float_as_uint(s) + 1u);
    const float rdn = fmaf(-sdn, s, d2), rup = fmaf(-sup, s, d2);
    s = rdn <= 0.0f ? sdn : s;
    s = rup > 0.0f ? sup : s;
    const float r = __builtin_amdgcn_rcpf(s);
    const float q = kCellJitter * r;
    return fmaf(fmaf(-q, s, kCellJitter), r, q);
}
__device__ __forceinline__ float cell_inv(float d2) { return cell_inv_c(d2); }

__device__ inline float cellular(int32_t seed, float x, float y, float z)
{
    const float xr = rintf(x), yr = rintf(y), zr = rintf(z);
    const int32_t xc = wmul((int32_t)xr, kPX), yc = wmul((int32_t)yr, kPY), zc = wmul((int32_t)zr, kPZ);
    float d0 = 3.402823466e+38f;
#pragma unroll
    for (int xi = -1; xi <= 1; ++xi) {
        const float xcf = (xr + (float)xi) - x;
        const int32_t xp = wadd(xc, wmul(xi, kPX));
#pragma unroll
        for (int yi = -1; yi <= 1; ++yi) {
            const float ycf = (yr + (float)yi) - y;
            const int32_t yp = wadd(yc, wmul(yi, kPY));
#pragma unroll
            for (int zi = -1; zi <= 1; ++zi) {
                const float zcf = (zr + (float)zi) - z;
                const int32_t zp = wadd(zc, wmul(zi, kPZ));
                const int32_t h = hash_hb(seed, xp, yp, zp);
                float xd = (float)(h & 0x3ff) - 511.5f;
                float yd = (float)((h >> 10) & 0x3ff) - 511.5f;
                float zd = (float)((h >> 20) & 0x3ff) - 511.5f;
                const float inv = cell_inv(fmaf(zd, zd, fmaf(yd, yd, xd * xd)));
                xd = fmaf(xd, inv, xcf);
                yd = fmaf(yd, inv, ycf);
                zd = fmaf(zd, inv, zcf);
                d0 = fminf(d0, fmaf(zd, zd, fmaf(yd, yd, xd * xd)));
            }
        }
    }
    return d0 - 1.0f;
}

// Cellular F1 from a table of per-cell feature-point data (the LDS table of
// the procedural march; vr_march.hip).  Entry (ix, iy, iz) - lo (at
// index iz * pz + iy * n + ix; the z pitch pz >= n * n is padded so that
// lanes in neighbouring cells do not hit the same LDS bank slot) holds
// {xd, yd, zd, inv} of cellular() for that integer cell, so each of the 27
// cells costs one 16-byte LDS read and 7 VALU ops instead of the hash,
// bit-field, sqrt and reciprocal.  The arithmetic per cell is cellular()'s,
// op for op, and fminf is exact, so the result is bit-identical.  The caller
// guarantees every cell rint(coord) - 1 .. + 1 lies in [lo, lo + n).
__device__ inline float cellular_table(const float4* __restrict__ tab, int lo, int n, int pz, float x, float y,
                                      float z)
{
    const float xr = rintf(x), yr = rintf(y), zr = rintf(z);
    const int ix = (int)xr - 1 - lo, iy = (int)yr - 1 - lo, iz = (int)zr - 1 - lo;
    const float4* t0 = tab + iz * pz + iy * n + ix;
    float d0 = 3.402823466e+38f;
#pragma unroll
    for (int xi = -1; xi <= 1; ++xi) {
        const float xcf = (xr + (float)xi) - x;
#pragma unroll
        for (int yi = -1; yi <= 1; ++yi) {
            const float ycf = (yr + (float)yi) - y;
#pragma unroll
            for (int zi = -1; zi <= 1; ++zi) {
                const float zcf = (zr + (float)zi) - z;
                const float4 c = t0[(zi + 1) * pz + (yi + 1) * n + (xi + 1)];
                const float xd = fmaf(c.x, c.w, xcf);
                const float yd = fmaf(c.y, c.w, ycf);
                const float zd = fmaf(c.z, c.w, zcf);
                d0 = fminf(d0, fmaf(zd, zd, fmaf(yd, yd, xd * xd)));
            }
        }
    }
    return d0 - 1.0f;
}

// cellular_table with the fixed geometry the host picks for tables of at most
// 9 cells per axis (kWorleyN = 9, z pitch kWorleyPz = 83: no bank aliasing
// between cells one apart): the base offset is computed in fp32 (small exact
// integers, one conversion) and the reads take immediate offsets.
//
// Pruned: feature points sit at distance kCellJitter (0.396) from their
// cell's integer corner, so the 8 corners of the unit cube around the sample
// (cells floor .. floor + 1 per axis, a subset of cellular()'s 27) usually
// hold the minimum.  Each of the other 19 cells has one axis at distance
// >= 1 + g_a from the sample (g_a = |coord - rint(coord)|) and the others
// at >= g_b, so its point is at least sqrt(T + 1 + 2 min g) - jitter away
// (T = sum g^2).  Only lanes whose cube minimum d does not beat that bound
// evaluate all 27 cells; a wave with no such lane skips them.  fminf is exact
// and order-free, and skipped cells are provably farther than d (margin
// kPruneR - jitter = 5.6e-5 in distance, >> fp32 rounding of the distance
// sums), so the result is bit-identical to cellular().  Modelled on config 2
// (tools/worley_prune_model.py): 94 % of wave-steps need the cube only.
#ifndef VR_CUBE_BATCH
#define VR_CUBE_BATCH 0
#endif
constexpr int kWorleyN = 9, kWorleyPz = 83;
constexpr float kPruneR = 0.3962f;
// The table's base byte offset term, negated: -16 lo (1 + kWorleyN + kWorleyPz)
// for the cube's (floor) cells.  Negated once per kernel (pinned in a VGPR,
// DensityK::wt_nc), so that fmaf(x, 16, nc) is one v_fmamk with a literal
// instead of a v_fma whose 16.0 sits in an SGPR (half issue rate, sec. 5.5).
__device__ __forceinline__ float worley9_nc(int lo) { return -(float)(16 * lo * (1 + kWorleyN + kWorleyPz)); }
// Cell distances are finite (table entries and sample coordinates are), so
// the minimum starts from the first cell instead of FLT_MAX: the same value,
// one min operand fewer.
__device__ inline float cellular_table9_full(const float4* __restrict__ tab, float nc, float x, float y, float z)
{
    const float xr = rintf(x), yr = rintf(y), zr = rintf(z);
    // cells rint - 1 ..: the base one cell lower on every axis (exact small integers)
    const float ncf = nc - (float)(16 * (1 + kWorleyN + kWorleyPz));
    const float fo = fmaf(zr, (float)(16 * kWorleyPz), fmaf(yr, (float)(16 * kWorleyN), fmaf(xr, 16.0f, ncf)));
    const float4* t0 = reinterpret_cast<const float4*>(reinterpret_cast<const char*>(tab) + (int)fo);
    float d0 = 0.0f;
#pragma unroll
    for (int xi = -1; xi <= 1; ++xi) {
        const float xcf = (xr + (float)xi) - x;
#pragma unroll
        for (int yi = -1; yi <= 1; ++yi) {
            const float ycf = (yr + (float)yi) - y;
#pragma unroll
            for (int zi = -1; zi <= 1; ++zi) {
                const float zcf = (zr + (float)zi) - z;
                const float4 cc = t0[(zi + 1) * kWorleyPz + (yi + 1) * kWorleyN + (xi + 1)];
                const float xd = fmaf(cc.x, cc.w, xcf);
                const float yd = fmaf(cc.y, cc.w, ycf);
                const float zd = fmaf(cc.z, cc.w, zcf);
                const float dd = fmaf(zd, zd, fmaf(yd, yd, xd * xd));
                d0 = (xi == -1 && yi == -1 && zi == -1) ? dd : fminf(d0, dd);
            }
        }
    }
    return d0;
}
// `full` (out): this lane evaluated all 27 cells after the cube's 8 (35 cell
// evaluations instead of 8) -- what vr option "count" = 2 sums.
__device__ inline float cellular_table9(const float4* __restrict__ tab, float nc, float x, float y, float z, bool& full)
{
    const float xf = floorf(x), yf = floorf(y), zf = floorf(z);
    // cellular()'s xcf = (integer cell coordinate) - x for the cube's two cells per axis
    const float x0 = xf - x, x1 = (xf + 1.0f) - x;
    const float y0 = yf - y, y1 = (yf + 1.0f) - y;
    const float z0 = zf - z, z1 = (zf + 1.0f) - z;
    const float fo = fmaf(zf, (float)(16 * kWorleyPz), fmaf(yf, (float)(16 * kWorleyN), fmaf(xf, 16.0f, nc)));
    const float4* t0 = reinterpret_cast<const float4*>(reinterpret_cast<const char*>(tab) + (int)fo);
#if VR_CUBE_BATCH
    // the cube's 8 LDS reads all in flight before the first use (one LDS round
    // trip per sample instead of up to 8): the empty asm takes every entry as
    // an operand, so the reads are issued ahead of it and used after it
    // entry k = xi * 4 + yi * 2 + zi, as native 4-vectors (register tuples for the asm)
    typedef float v4f __attribute__((ext_vector_type(4)));
    const v4f* tv = reinterpret_cast<const v4f*>(t0);
    v4f c0 = tv[0], c1 = tv[kWorleyPz], c2 = tv[kWorleyN], c3 = tv[kWorleyN + kWorleyPz];
    v4f c4 = tv[1], c5 = tv[1 + kWorleyPz], c6 = tv[1 + kWorleyN], c7 = tv[1 + kWorleyN + kWorleyPz];
    asm volatile("" : "+v"(c0), "+v"(c1), "+v"(c2), "+v"(c3), "+v"(c4), "+v"(c5), "+v"(c6), "+v"(c7));
    const v4f cv[8] = {c0, c1, c2, c3, c4, c5, c6, c7};
#endif
    float d0 = 0.0f;
#pragma unroll
    for (int xi = 0; xi <= 1; ++xi) {
#pragma unroll
        for (int yi = 0; yi <= 1; ++yi) {
#pragma unroll
            for (int zi = 0; zi <= 1; ++zi) {
#if VR_CUBE_BATCH
                const v4f cq = cv[xi * 4 + yi * 2 + zi];
                const float4 cc = make_float4(cq.x, cq.y, cq.z, cq.w);
#else
                const float4 cc = t0[zi * kWorleyPz + yi * kWorleyN + xi];
#endif
                const float xd = fmaf(cc.x, cc.w, xi ? x1 : x0);
                const float yd = fmaf(cc.y, cc.w, yi ? y1 : y0);
                const float zd = fmaf(cc.z, cc.w, zi ? z1 : z0);
                const float dd = fmaf(zd, zd, fmaf(yd, yd, xd * xd));
                d0 = (xi | yi | zi) == 0 ? dd : fminf(d0, dd);
            }
        }
    }
    const float gx = fminf(-x0, x1), gy = fminf(-y0, y1), gz = fminf(-z0, z1);
    const float bound = fmaf(2.0f, fminf(gx, fminf(gy, gz)), fmaf(gz, gz, fmaf(gy, gy, fmaf(gx, gx, 1.0f))));
    const float e = __builtin_amdgcn_sqrtf(d0) + kPruneR;
    full = e * e > bound;
    if (full) d0 = fminf(d0, cellular_table9_full(tab, nc, x, y, z));
    return d0 - 1.0f;
}

// cellular_table9 for a lane that evaluates a run of nearby samples (the
// deferred shadow pass: a sun ray's samples are ~2 texels apart, Worley cells
// at f = .03 ~33): the unit cube's 8 table entries stay in registers while
// the cube's base cell is unchanged (key = its table offset), so the LDS is
// read only when a sample crosses a cell face.  The same entries, the same
// ops: bit-identical to cellular_table9.
struct WorleyCube {
    int fo = -1;   // byte offset of the cached cube's base entry (-1: none)
    float4 c[8];
};
__device__ inline float cellular_table9_cached(const float4* __restrict__ tab, float nc, float x, float y, float z,
                                               bool& full, WorleyCube& wc)
{
    const float xf = floorf(x), yf = floorf(y), zf = floorf(z);
    const float x0 = xf - x, x1 = (xf + 1.0f) - x;
    const float y0 = yf - y, y1 = (yf + 1.0f) - y;
    const float z0 = zf - z, z1 = (zf + 1.0f) - z;
    const int fo = (int)fmaf(zf, (float)(16 * kWorleyPz), fmaf(yf, (float)(16 * kWorleyN), fmaf(xf, 16.0f, nc)));
    if (fo != wc.fo) {
        wc.fo = fo;
        const float4* t0 = reinterpret_cast<const float4*>(reinterpret_cast<const char*>(tab) + fo);
#pragma unroll
        for (int k = 0; k < 8; ++k) wc.c[k] = t0[(k & 1) * kWorleyPz + ((k >> 1) & 1) * kWorleyN + (k >> 2)];
    }
    float d0 = 0.0f;
#pragma unroll
    for (int xi = 0; xi <= 1; ++xi) {
#pragma unroll
        for (int yi = 0; yi <= 1; ++yi) {
#pragma unroll
            for (int zi = 0; zi <= 1; ++zi) {
                const float4 cc = wc.c[xi * 4 + yi * 2 + zi];
                const float xd = fmaf(cc.x, cc.w, xi ? x1 : x0);
                const float yd = fmaf(cc.y, cc.w, yi ? y1 : y0);
                const float zd = fmaf(cc.z, cc.w, zi ? z1 : z0);
                const float dd = fmaf(zd, zd, fmaf(yd, yd, xd * xd));
                d0 = (xi | yi | zi) == 0 ? dd : fminf(d0, dd);
            }
        }
    }
    const float gx = fminf(-x0, x1), gy = fminf(-y0, y1), gz = fminf(-z0, z1);
    const float bound = fmaf(2.0f, fminf(gx, fminf(gy, gz)), fmaf(gz, gz, fmaf(gy, gy, fmaf(gx, gx, 1.0f))));
    const float e = __builtin_amdgcn_sqrtf(d0) + kPruneR;
    full = e * e > bound;
    if (full) d0 = fminf(d0, cellular_table9_full(tab, nc, x, y, z));
    return d0 - 1.0f;
}

// One table entry: cellular()'s feature-point data for integer cell (ix, iy, iz).
__device__ inline float4 cellular_cell(int32_t seed, int ix, int iy, int iz)
{
    const int32_t h = hash_hb(seed, wmul(ix, kPX), wmul(iy, kPY), wmul(iz, kPZ));
    const float xd = (float)(h & 0x3ff) - 511.5f;
    const float yd = (float)((h >> 10) & 0x3ff) - 511.5f;
    const float zd = (float)((h >> 20) & 0x3ff) - 511.5f;
    return make_float4(xd, yd, zd, cell_inv(fmaf(zd, zd, fmaf(yd, yd, xd * xd))));
}

}  // namespace noise
}  // namespace vr
