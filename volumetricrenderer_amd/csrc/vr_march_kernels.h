// vr_march_kernels.h -- device code of the ray march: the tap and blend
// helpers, the per-pixel march for the grid layouts and the procedural
// medium, and the kernels with their templated launcher launch_lw.  Included
// by vr_march.hip (all launchers) and vr_march_c8.hip (the CORNER8 launcher,
// compiled with different vectoriser flags).  Everything
// is in an anonymous namespace, so each translation unit keeps its own copy.
#pragma once
#include "vr_internal.h"
#include "vr_noise.h"

namespace vr {
namespace {

constexpr int kTile = 16;           // static schedule: workgroup tile edge, pixels
constexpr int kThreads = 256;       // 4 waves

typedef float f2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ float lerp_(float a, float b, float t) { return fmaf(t, b - a, a); }
__device__ __forceinline__ f2 lerp2(f2 a, f2 b, f2 t) { return __builtin_elementwise_fma(t, b - a, a); }
__device__ __forceinline__ int clampi(int v, int lo, int hi) { return min(max(v, lo), hi); }

// floor(x) as int in one instruction, and x - floor(x) clamped below 1.0
// (v_fract_f32).  The spec defines the tap weight as
// fminf(g - floorf(g), 0x1.fffffep-1f), which is what v_fract_f32 returns.
__device__ __forceinline__ int cvt_flr(float x)
{
    int r;
    asm("v_cvt_flr_i32_f32 %0, %1" : "=v"(r) : "v"(x));
    return r;
}
__device__ __forceinline__ float fract_(float x) { return __builtin_amdgcn_fractf(x); }

// byte k of a dword as float: one v_cvt_f32_ubyteK.  Opaque on purpose: given
// (float)hi - (float)lo of two bytes, hipcc otherwise subtracts in packed
// int16 and converts the difference, which costs more instructions.
template <int K>
__device__ __forceinline__ float ubyte(unsigned v)
{
    float r;
    if constexpr (K == 0) asm("v_cvt_f32_ubyte0 %0, %1" : "=v"(r) : "v"(v));
    else if constexpr (K == 1) asm("v_cvt_f32_ubyte1 %0, %1" : "=v"(r) : "v"(v));
    else if constexpr (K == 2) asm("v_cvt_f32_ubyte2 %0, %1" : "=v"(r) : "v"(v));
    else asm("v_cvt_f32_ubyte3 %0, %1" : "=v"(r) : "v"(v));
    return r;
}

// VK_SAMPLER_ADDRESS_MODE_MIRRORED_REPEAT on an integer texel index
// (VulkanCore.cpp:683-685; Vulkan spec "Texel coordinate wrapping").
__device__ __forceinline__ int mirror_(int i, int n)
{
    int two = n + n;
    int m = i % two;
    m = m < 0 ? m + two : m;
    return m < n ? m : two - 1 - m;
}

// exp(x) for x <= 0, the fma-only polynomial of the spec.
__device__ __forceinline__ float spec_expf(float x)
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
    return p * __int_as_float(((int)k + 127) << 23);
}

// Trilinear blend of the 8 footprint texels, two lerps per packed op:
// x-lerps of (y0,z0|y0,z1) and (y1,z0|y1,z1), then y, then z.  Each element
// is the spec's fma(t, b - a, a), in the spec's order.
__device__ __forceinline__ float blend(f2 lo_a, f2 hi_a, f2 lo_b, f2 hi_b, float wx, float wy, float wz)
{
    const f2 xa = lerp2(lo_a, hi_a, f2{wx, wx});   // {x00, x01}
    const f2 xb = lerp2(lo_b, hi_b, f2{wx, wx});   // {x10, x11}
    const f2 y = lerp2(xa, xb, f2{wy, wy});        // {y0, y1}
    return lerp_(y.x, y.y, wz) * (1.0f / 255.0f);
}

// Per-launch state of a fast-layout tap: the channel's buffer descriptor and
// the LDS offset tables TX | TY | TZ (vr_internal.h Layout).
struct FastCtx {
    __amdgpu_buffer_rsrc_t rsrc[4];
    const unsigned* tx;
    const unsigned* ty;
    const unsigned* tz;
    const unsigned* tx3;   // COL48Z: channel 3's ZPAIR offset tables (a second set in LDS)
    const unsigned* ty3;
    const unsigned* tz3;
    float s1x16, s2x16;   // CORNERH: 16 (nx+1), 16 (nx+1)(ny+1) (byte strides of y, z)
    // CORNERH: the z tap constants and the sample scale pinned to VGPRs (an fp32
    // op reading an SGPR issues at ~4.1 instead of ~2.2 cycles, sec. 5.5)
    float sz[4], oz[4], scale;
};

// x-lerp of one CORNERH footprint row: fma(w, b - a, a) with the f16 pair
// {a, b - a} of dword q (a low, b - a high), converted exactly inside the
// one v_fma_mix_f32.  Equal to the spec's fmaf(w, b - a, a) bit for bit.
__device__ __forceinline__ float mix_lerp(float w, unsigned q)
{
    float r;
    asm("v_fma_mix_f32 %0, %1, %2, %2 op_sel:[0,1,0] op_sel_hi:[0,1,1]" : "=v"(r) : "v"(w), "v"(q));
    return r;
}

// A fast-layout tap in two parts: fetch (issue the loads, keep the weights)
// and blend.  The pipelined march issues step i+1's fetches before blending
// step i, so each wave keeps two steps of loads in flight.
struct TapRaw {
    unsigned q0, q1, q2, q3;
    float wx, wy, wz;
};
template <int LAYOUT>
__device__ __forceinline__ TapRaw tap_fetch(const FastCtx& f, int ch, float gx, float gy, float gz)
{
    TapRaw r{};
    if constexpr (LAYOUT == LAYOUT_CORNERH) {
        // floor(g) in fp32 and the weight g - floor(g): exact and equal to
        // v_fract_f32 because g >= 0 here (clamp_is_exact); the byte offset
        // 16 (a + (nx+1) b + (nx+1)(ny+1) c) is an integer below 2^28 with at
        // most 24 significant bits, so both fmas are exact
        const float fx = floorf(gx), fy = floorf(gy), fz = floorf(gz);
        r.wx = gx - fx; r.wy = gy - fy; r.wz = gz - fz;
        const unsigned off = (unsigned)fmaf(fz, f.s2x16, fmaf(fy, f.s1x16, fx * 16.0f));
        const auto v = __builtin_amdgcn_raw_buffer_load_b128(f.rsrc[ch], off, 0, 0);
        r.q0 = v[0]; r.q1 = v[1]; r.q2 = v[2]; r.q3 = v[3];
        return r;
    }
    r.wx = fract_(gx); r.wy = fract_(gy); r.wz = fract_(gz);
    const unsigned off = f.tx[cvt_flr(gx)] + f.ty[cvt_flr(gy)] + f.tz[cvt_flr(gz)];
    if constexpr (LAYOUT == LAYOUT_CORNER8) {
        r.q0 = __builtin_amdgcn_raw_buffer_load_b32(f.rsrc[ch], off, 0, 0);
        r.q1 = __builtin_amdgcn_raw_buffer_load_b32(f.rsrc[ch], off + 4, 0, 0);
    } else if constexpr (LAYOUT == LAYOUT_BRICK5) {
        // R = 5: one load per z-slice, bytes off..off+6 (c000 c100 . . . c010
        // c110) and the same 25 bytes on.  Each is a dword-ALIGNED 12-byte
        // load from off & ~3 and two v_alignbyte_b32 that shift the slice
        // down by off & 3: an 8-byte load at a byte-granular offset costs
        // the L1 twice the tag lookups of a dword-aligned one, and a 12-byte
        // one costs the same as 8 bytes (tools/tcp_calib.hip, DESIGN.md
        // sec. 5.1): 0.264 -> 0.225 ms at 512^3, 0.195 -> 0.122 ms at 256^3.
        // Narrow row loads (4 x u16 or u32 per tap) were 20 % slower than the
        // byte-offset 8-byte loads: more instructions, more lookups.
        const unsigned o1 = off + 25;
        const auto s0 = __builtin_amdgcn_raw_buffer_load_b96(f.rsrc[ch], off & ~3u, 0, 0);
        const auto s1 = __builtin_amdgcn_raw_buffer_load_b96(f.rsrc[ch], o1 & ~3u, 0, 0);
        r.q0 = __builtin_amdgcn_alignbyte(s0[1], s0[0], off);
        r.q1 = __builtin_amdgcn_alignbyte(s0[2], s0[1], off);
        r.q2 = __builtin_amdgcn_alignbyte(s1[1], s1[0], o1);
        r.q3 = __builtin_amdgcn_alignbyte(s1[2], s1[1], o1);
    } else if constexpr (is_b4_family(LAYOUT)) {
        // R = 4: a slice's rows y and y+1 are the two dwords at off & ~3
        // (x = off & 3 <= 2), so one dword-aligned 8-byte load per z-slice,
        // the z+1 slice 16 bytes on (32 for BRICK488's 8-row slices): 2
        // dwords per lane and slice where BRICK5 needs 3.  q0/q2 = bytes x,
        // x+1 of row y, q1/q3 of row y+1.
        constexpr unsigned kZ = LAYOUT == LAYOUT_BRICK41616 ? 64u
                             : LAYOUT == LAYOUT_BRICK488 || LAYOUT == LAYOUT_BRICK4816 || LAYOUT == LAYOUT_BRICK4832 ||
                                      LAYOUT == LAYOUT_BRICK4864 || LAYOUT == LAYOUT_COL48 ? 32u : 16u;
        const unsigned a0 = off & ~3u;
        const auto s0 = __builtin_amdgcn_raw_buffer_load_b64(f.rsrc[ch], a0, 0, 0);
        const auto s1 = __builtin_amdgcn_raw_buffer_load_b64(f.rsrc[ch], a0 + kZ, 0, 0);
        r.q0 = __builtin_amdgcn_alignbyte(s0[1], s0[0], off);
        r.q1 = __builtin_amdgcn_alignbyte(s0[1], s0[1], off);
        r.q2 = __builtin_amdgcn_alignbyte(s1[1], s1[0], off);
        r.q3 = __builtin_amdgcn_alignbyte(s1[1], s1[1], off);
    } else if constexpr (LAYOUT == LAYOUT_ZPAIR) {
        // the whole footprint is the 16 bytes at off & ~3 (x = off & 3 <= 2):
        // dwords = rows (y,z) (y,z+1) (y+1,z) (y+1,z+1); one load per tap
        const auto s0 = __builtin_amdgcn_raw_buffer_load_b128(f.rsrc[ch], off & ~3u, 0, 0);
        r.q0 = __builtin_amdgcn_alignbyte(s0[0], s0[0], off);
        r.q2 = __builtin_amdgcn_alignbyte(s0[1], s0[1], off);
        r.q1 = __builtin_amdgcn_alignbyte(s0[2], s0[2], off);
        r.q3 = __builtin_amdgcn_alignbyte(s0[3], s0[3], off);
    } else if constexpr (LAYOUT == LAYOUT_BRICK8) {
        // R = 8: rows y and y+1 of a slice are 8 bytes apart, so one
        // dword-aligned 16-byte load from off & ~3 holds both (bytes off,
        // off+1, off+8, off+9); the z+1 slice is 64 bytes on.  Two loads per
        // tap instead of four byte-offset u16 loads: 0.271 -> 0.235 ms at
        // 512^3, 0.185 -> 0.119 ms at 128^3.
        const unsigned o1 = off + 64;
        const auto s0 = __builtin_amdgcn_raw_buffer_load_b128(f.rsrc[ch], off & ~3u, 0, 0);
        const auto s1 = __builtin_amdgcn_raw_buffer_load_b128(f.rsrc[ch], o1 & ~3u, 0, 0);
        r.q0 = __builtin_amdgcn_alignbyte(s0[1], s0[0], off);   // c000 c100 in bytes 0-1
        r.q1 = __builtin_amdgcn_alignbyte(s0[3], s0[2], off);   // c010 c110
        r.q2 = __builtin_amdgcn_alignbyte(s1[1], s1[0], o1);    // c001 c101
        r.q3 = __builtin_amdgcn_alignbyte(s1[3], s1[2], o1);    // c011 c111
    } else {
        constexpr int R = LAYOUT == LAYOUT_BRICK8 ? 8 : 16;
        r.q0 = __builtin_amdgcn_raw_buffer_load_b16(f.rsrc[ch], off, 0, 0);
        r.q1 = __builtin_amdgcn_raw_buffer_load_b16(f.rsrc[ch], off + R, 0, 0);
        r.q2 = __builtin_amdgcn_raw_buffer_load_b16(f.rsrc[ch], off + R * R, 0, 0);
        r.q3 = __builtin_amdgcn_raw_buffer_load_b16(f.rsrc[ch], off + R * R + R, 0, 0);
    }
    return r;
}
template <int LAYOUT>
__device__ __forceinline__ float tap_blend(const TapRaw& r)
{
    if constexpr (LAYOUT == LAYOUT_CORNERH) {
        // rows q0 (y0,z0) q1 (y1,z0) q2 (y0,z1) q3 (y1,z1): x-lerps, then y, then z
        const float x00 = mix_lerp(r.wx, r.q0), x10 = mix_lerp(r.wx, r.q1);
        const float x01 = mix_lerp(r.wx, r.q2), x11 = mix_lerp(r.wx, r.q3);
        const float y0 = lerp_(x00, x10, r.wy), y1 = lerp_(x01, x11, r.wy);
        return lerp_(y0, y1, r.wz) * (1.0f / 255.0f);
    } else if constexpr (LAYOUT == LAYOUT_CORNER8) {
        return blend(f2{ubyte<0>(r.q0), ubyte<0>(r.q1)}, f2{ubyte<1>(r.q0), ubyte<1>(r.q1)},
                     f2{ubyte<2>(r.q0), ubyte<2>(r.q1)}, f2{ubyte<3>(r.q0), ubyte<3>(r.q1)}, r.wx, r.wy, r.wz);
    } else if constexpr (LAYOUT == LAYOUT_BRICK5) {
        return blend(f2{ubyte<0>(r.q0), ubyte<0>(r.q2)}, f2{ubyte<1>(r.q0), ubyte<1>(r.q2)},
                     f2{ubyte<1>(r.q1), ubyte<1>(r.q3)}, f2{ubyte<2>(r.q1), ubyte<2>(r.q3)}, r.wx, r.wy, r.wz);
    } else {
        return blend(f2{ubyte<0>(r.q0), ubyte<0>(r.q2)}, f2{ubyte<1>(r.q0), ubyte<1>(r.q2)},
                     f2{ubyte<0>(r.q1), ubyte<0>(r.q3)}, f2{ubyte<1>(r.q1), ubyte<1>(r.q3)}, r.wx, r.wy, r.wz);
    }
}
// One trilinear tap of one channel from a fast layout, at padded texel
// coordinate g (floor(g) = base texel + 1, fract(g) = weight).  Loads go
// through a range-checked buffer descriptor: an offset outside the plane
// reads 0 instead of faulting.
template <int LAYOUT>
__device__ __forceinline__ float tap_fast(const FastCtx& f, int ch, float gx, float gy, float gz)
{
    return tap_blend<LAYOUT>(tap_fetch<LAYOUT>(f, ch, gx, gy, gz));
}

template <int LAYOUT, bool ZO = false>
__device__ __forceinline__ TapRaw tap_fetch_at(const MarchArgs& a, const FastCtx& f, int t, f2 pxy, float pz)
{
    const f2 T = ZO ? f2{0.5f, 0.5f} : f2{a.tap_T[t][0], a.tap_T[t][1]};
    const f2 gxy = __builtin_elementwise_fma(pxy, f2{a.tap_S[t][0], a.tap_S[t][1]}, T);
    const float gz = LAYOUT == LAYOUT_CORNERH ? fmaf(pz, f.sz[t], ZO ? 0.5f : f.oz[t])
                                             : fmaf(pz, a.tap_S[t][2], ZO ? 0.5f : a.tap_T[t][2]);
    return tap_fetch<LAYOUT>(f, t, gxy.x, gxy.y, gz);
}

// One trilinear tap from the planar layout with full wrap semantics.
template <int WRAP>
__device__ __forceinline__ float tap_planar(const uint8_t* __restrict__ pl, const MarchArgs& a, float gx,
                                            float gy, float gz)
{
    const float wx = fract_(gx), wy = fract_(gy), wz = fract_(gz);
    const int ix = cvt_flr(gx) - 1, iy = cvt_flr(gy) - 1, iz = cvt_flr(gz) - 1;
    int i0, i1, j0, j1, k0, k1;
    if constexpr (WRAP == WRAP_CLAMP) {
        i0 = clampi(ix, 0, a.nx - 1); i1 = clampi(ix + 1, 0, a.nx - 1);
        j0 = clampi(iy, 0, a.ny - 1); j1 = clampi(iy + 1, 0, a.ny - 1);
        k0 = clampi(iz, 0, a.nz - 1); k1 = clampi(iz + 1, 0, a.nz - 1);
    } else {
        i0 = mirror_(ix, a.nx); i1 = mirror_(ix + 1, a.nx);
        j0 = mirror_(iy, a.ny); j1 = mirror_(iy + 1, a.ny);
        k0 = mirror_(iz, a.nz); k1 = mirror_(iz + 1, a.nz);
    }
    const int r00 = (k0 * a.ny + j0) * a.nx, r10 = (k0 * a.ny + j1) * a.nx;
    const int r01 = (k1 * a.ny + j0) * a.nx, r11 = (k1 * a.ny + j1) * a.nx;
    return blend(f2{ubyte<0>(pl[r00 + i0]), ubyte<0>(pl[r01 + i0])}, f2{ubyte<0>(pl[r00 + i1]), ubyte<0>(pl[r01 + i1])},
                 f2{ubyte<0>(pl[r10 + i0]), ubyte<0>(pl[r11 + i0])}, f2{ubyte<0>(pl[r10 + i1]), ubyte<0>(pl[r11 + i1])},
                 wx, wy, wz);
}

// Tap t at ray point P: padded texel coordinate g = fma(P, S_t, T_t).
template <int LAYOUT, int WRAP>
__device__ __forceinline__ float tap(const MarchArgs& a, const FastCtx& f, int t, f2 pxy, float pz)
{
    const f2 gxy = __builtin_elementwise_fma(pxy, f2{a.tap_S[t][0], a.tap_S[t][1]}, f2{a.tap_T[t][0], a.tap_T[t][1]});
    const float gz = fmaf(pz, a.tap_S[t][2], a.tap_T[t][2]);
    if constexpr (LAYOUT == LAYOUT_PLANAR)
        return tap_planar<WRAP>(a.vol + (size_t)t * a.plane_stride, a, gxy.x, gxy.y, gz);
    else
        return tap_fast<LAYOUT>(f, t, gxy.x, gxy.y, gz);
}

// Per-ray state after ray setup (frag.glsl:36-55).
struct Ray {
    bool live;     // pixel exists (inside the target and the frame)
    int n;         // steps (frag.glsl:46); -1 = not covered
    f2 pxy;        // box-normalised ray point (frag.glsl:49-54)
    float pz;
    f2 sxy;        // step vector (frag.glsl:45, 54)
    float sz;
};

__device__ __forceinline__ Ray setup_ray(const MarchArgs& a, int x, int orow)
{
    Ray r{};
    r.n = -1;
    const bool inside = x < a.width && orow < a.out_rows;
    int y = 0;
    if (inside) {
        const int bl = orow / a.band_rows;
        y = set_band(bl, a.band_first, a.band_stride, a.band_flip) * a.band_rows + (orow - bl * a.band_rows);
    }
    r.live = inside && y < a.height;
    if (!r.live) return r;
    const float fx = (float)x + 0.5f, fy = (float)y + 0.5f;
    const float v0 = fmaf(fy, a.py[0], fmaf(fx, a.px[0], a.o[0]));
    const float v1 = fmaf(fy, a.py[1], fmaf(fx, a.px[1], a.o[1]));
    const float v2 = fmaf(fy, a.py[2], fmaf(fx, a.px[2], a.o[2]));
    const float len = sqrtf(fmaf(v2, v2, fmaf(v1, v1, v0 * v0)));
    float d0 = v0 / len, d1 = v1 / len, d2 = v2 / len;
    // IntersectAABB, frag.glsl:18-27
    float ta0 = (a.box_min[0] - a.org[0]) / d0, tb0 = (a.box_max[0] - a.org[0]) / d0;
    float ta1 = (a.box_min[1] - a.org[1]) / d1, tb1 = (a.box_max[1] - a.org[1]) / d1;
    float ta2 = (a.box_min[2] - a.org[2]) / d2, tb2 = (a.box_max[2] - a.org[2]) / d2;
    float tn = fmaxf(fmaxf(fminf(ta0, tb0), fminf(ta1, tb1)), fminf(ta2, tb2));
    float tf = fminf(fminf(fmaxf(ta0, tb0), fmaxf(ta1, tb1)), fmaxf(ta2, tb2));
    if (!(tn <= tf)) return r;
    float pi0 = fmaf(d0, tn, a.org[0]), pi1 = fmaf(d1, tn, a.org[1]), pi2 = fmaf(d2, tn, a.org[2]);
    // coverage: the front-face fragment survives clipping (0 <= z <= w)
    const float zc = fmaf(a.r2[2], pi2, fmaf(a.r2[1], pi1, fmaf(a.r2[0], pi0, a.r2[3])));
    const float wc = fmaf(a.r3[2], pi2, fmaf(a.r3[1], pi1, fmaf(a.r3[0], pi0, a.r3[3])));
    if (!(wc > 0.0f && zc >= 0.0f && zc <= wc)) return r;
    float c0 = a.org[0], c1 = a.org[1], c2 = a.org[2];
    if (a.cam_mode) {
        // CameraPosition is not the View eye: pi is the rasterised front-face
        // point (vert.glsl:20); the fragment's ray leaves CameraPosition through
        // it (frag.glsl:36-38), and IntersectAABB runs again from there
        c0 = a.cam[0]; c1 = a.cam[1]; c2 = a.cam[2];
        const float f0 = pi0 - c0, f1 = pi1 - c1, f2 = pi2 - c2;
        const float fl = sqrtf(fmaf(f2, f2, fmaf(f1, f1, f0 * f0)));
        d0 = f0 / fl; d1 = f1 / fl; d2 = f2 / fl;
        ta0 = (a.box_min[0] - c0) / d0; tb0 = (a.box_max[0] - c0) / d0;
        ta1 = (a.box_min[1] - c1) / d1; tb1 = (a.box_max[1] - c1) / d1;
        ta2 = (a.box_min[2] - c2) / d2; tb2 = (a.box_max[2] - c2) / d2;
        tn = fmaxf(fmaxf(fminf(ta0, tb0), fminf(ta1, tb1)), fminf(ta2, tb2));
        tf = fminf(fminf(fmaxf(ta0, tb0), fmaxf(ta1, tb1)), fmaxf(ta2, tb2));
        pi0 = fmaf(d0, tn, c0); pi1 = fmaf(d1, tn, c1); pi2 = fmaf(d2, tn, c2);
    }
    const float po0 = fmaf(d0, tf, c0), po1 = fmaf(d1, tf, c1), po2 = fmaf(d2, tf, c2);
    const float e0 = po0 - pi0, e1 = po1 - pi1, e2 = po2 - pi2;
    const float dist = sqrtf(fmaf(e2, e2, fmaf(e1, e1, e0 * e0)));
    const float q = dist / a.step_size;                                   // :46
    // int(NaN) (a degenerate camera on the fragment) is undefined in GLSL: 0 here
    r.n = q >= (float)a.max_steps ? a.max_steps : q >= 0.0f ? (int)q : 0;
    r.pxy = f2{(pi0 - a.box_min[0]) / a.box_range[0], (pi1 - a.box_min[1]) / a.box_range[1]};   // :49-54
    r.pz = (pi2 - a.box_min[2]) / a.box_range[2];
    r.sxy = f2{(a.step_size * d0) / a.box_range[0], (a.step_size * d1) / a.box_range[1]};       // :45
    r.sz = (a.step_size * d2) / a.box_range[2];
    return r;
}

// Render-target store: grey g (frag.glsl:80), uncovered pixels keep the
// clear colour (0,0,0,1) (VulkanRenderPass.cpp:17-24).  Formats 3-5 store the
// R channel only (include/vr.h grey targets).
__device__ __forceinline__ void store_pixel(const MarchArgs& a, int x, int orow, bool covered, float g)
{
    int trow = orow;
    if (a.bands_in_place) {   // the band's frame row (vr.h VR_TARGET_BANDS_IN_PLACE)
        const int bl = orow / a.band_rows;
        trow = set_band(bl, a.band_first, a.band_stride, a.band_flip) * a.band_rows + (orow - bl * a.band_rows);
    }
    char* row = (char*)a.out + (long long)trow * a.pitch;
    if (a.format == 0 || a.format == 5) {
        g = covered ? g : 0.0f;
        if (a.format == 0) reinterpret_cast<float4*>(row)[x] = make_float4(g, g, g, 1.0f);
        else reinterpret_cast<float*>(row)[x] = g;
    } else {
        unsigned int q = 0;
        if (covered) {
            float c = fminf(fmaxf(g, 0.0f), 1.0f);
            if (a.format == 2 || a.format == 4)
                c = c <= 0.0031308f ? c * 12.92f : fmaf(1.055f, powf(c, 1.0f / 2.4f), -0.055f);
            q = (unsigned int)rintf(c * 255.0f);
        }
        if (a.format <= 2) reinterpret_cast<unsigned int*>(row)[x] = q | (q << 8) | (q << 16) | 0xff000000u;
        else reinterpret_cast<unsigned char*>(row)[x] = (unsigned char)q;
    }
}

// One ray of the grid path: setup, the march (frag.glsl:57-75), the
// epilogue (:76-80) and the store.  Returns the executed steps.
// The brick layouts run software-pipelined: step i+1's loads are issued
// before step i is blended, so a wave has two steps of gathers in flight.
// This costs VGPRs (67-73, 6-7 waves/SIMD) and is still faster: at 512^3
// brick5 0.334 -> 0.280 ms (before the aligned loads), brick8 unchanged.
// Fetching two steps ahead spilled to scratch and was 2.6x slower.  CORNER8 (the cache-resident
// layout, one load per tap) is not: 0.51 -> 0.56 ms at 3840x2160x256.
// Forcing 6 or 8 waves/SIMD (amdgpu_waves_per_eu) was slower in every case,
// with or without pipelining.
#ifndef VR_PIPE
#define VR_PIPE 1
#endif
// Taps of a march with uniform channels UM (MarchArgs.umask): a uniform
// channel's tap is the constant uv[T], with no load.
// COL48Z: taps 0-2 are COL48's, tap 3 ZPAIR's (its own tables and plane).
template <int UM, int T, int LAYOUT, bool ZO>
__device__ __forceinline__ TapRaw fetch_u(const MarchArgs& a, const FastCtx& f, f2 pxy, float pz)
{
    if constexpr ((UM >> T) & 1) {
        return TapRaw{};
    } else if constexpr (LAYOUT == LAYOUT_COL48Z) {
        if constexpr (T == 3) {
            FastCtx g = f;
            g.tx = f.tx3; g.ty = f.ty3; g.tz = f.tz3;
            return tap_fetch_at<LAYOUT_ZPAIR, ZO>(a, g, T, pxy, pz);
        } else {
            return tap_fetch_at<LAYOUT_COL48, ZO>(a, f, T, pxy, pz);
        }
    } else {
        return tap_fetch_at<LAYOUT, ZO>(a, f, T, pxy, pz);
    }
}
template <int UM, int T, int LAYOUT>
__device__ __forceinline__ float blend_u(const TapRaw& c, const float* uv)
{
    if constexpr ((UM >> T) & 1) return uv[T];
    else if constexpr (LAYOUT == LAYOUT_COL48Z) return tap_blend<T == 3 ? LAYOUT_ZPAIR : LAYOUT_COL48>(c);
    else return tap_blend<LAYOUT>(c);
}
template <int LAYOUT, int WRAP, bool EARLY, bool ZO = false, int UM = 0>
__device__ __forceinline__ unsigned march_pixel(const MarchArgs& a, const FastCtx& f, int x, int orow)
{
    const Ray r = setup_ray(a, x, orow);
    float uv[4] = {};
    if constexpr (UM != 0)
        for (int t = 0; t < 4; ++t)
            if ((UM >> t) & 1) uv[t] = noise::in_vgpr(a.uval[t]);
    if constexpr (VR_PIPE && LAYOUT != LAYOUT_PLANAR && LAYOUT != LAYOUT_CORNER8 && LAYOUT != LAYOUT_CORNERH) {
        f2 pxy = r.pxy;
        float pz = r.pz;
        float acc = 0.0f;
        int i = 0;
        if (r.n > 0) {
            TapRaw c0 = fetch_u<UM, 0, LAYOUT, ZO>(a, f, pxy, pz), c1 = fetch_u<UM, 1, LAYOUT, ZO>(a, f, pxy, pz);
            TapRaw c2 = fetch_u<UM, 2, LAYOUT, ZO>(a, f, pxy, pz), c3 = fetch_u<UM, 3, LAYOUT, ZO>(a, f, pxy, pz);
            for (; i < r.n; ++i) {
                const f2 cxy = pxy;
                const float cz = pz;
                pxy = pxy + r.sxy;                                                        // :74
                pz = pz + r.sz;
                // the last step re-fetches its own (in-box) point: no branch
                const bool more = i + 1 < r.n;
                const f2 qxy = more ? pxy : cxy;
                const float qz = more ? pz : cz;
                const TapRaw n0 = fetch_u<UM, 0, LAYOUT, ZO>(a, f, qxy, qz), n1 = fetch_u<UM, 1, LAYOUT, ZO>(a, f, qxy, qz);
                const TapRaw n2 = fetch_u<UM, 2, LAYOUT, ZO>(a, f, qxy, qz), n3 = fetch_u<UM, 3, LAYOUT, ZO>(a, f, qxy, qz);
                const float t0 = blend_u<UM, 0, LAYOUT>(c0, uv), t1 = blend_u<UM, 1, LAYOUT>(c1, uv);
                const float t2 = blend_u<UM, 2, LAYOUT>(c2, uv), t3 = blend_u<UM, 3, LAYOUT>(c3, uv);
                acc = acc + ((t0 * t1) * (t2 + t3)) * a.scale;                           // :71-73
                c0 = n0; c1 = n1; c2 = n2; c3 = n3;
                if constexpr (EARLY) {
                    if (acc > a.acc_limit) { ++i; break; }
                }
            }
        }
        if (r.live) {
            const float at = acc * a.step_size;
            store_pixel(a, x, orow, r.n >= 0, 1.0f - spec_expf(a.density * fminf(-at, 0.0f)));
        }
        return r.n > 0 ? (unsigned)i : 0u;
    }
    f2 pxy = r.pxy;
    float pz = r.pz;
    float acc = 0.0f;
    int i = 0;
    for (; i < r.n; ++i) {
        float t0, t1, t2, t3;
        if constexpr (LAYOUT != LAYOUT_PLANAR) {
            t0 = blend_u<UM, 0, LAYOUT>(fetch_u<UM, 0, LAYOUT, ZO>(a, f, pxy, pz), uv);
            t1 = blend_u<UM, 1, LAYOUT>(fetch_u<UM, 1, LAYOUT, ZO>(a, f, pxy, pz), uv);
            t2 = blend_u<UM, 2, LAYOUT>(fetch_u<UM, 2, LAYOUT, ZO>(a, f, pxy, pz), uv);
            t3 = blend_u<UM, 3, LAYOUT>(fetch_u<UM, 3, LAYOUT, ZO>(a, f, pxy, pz), uv);
        } else {
            t0 = tap<LAYOUT, WRAP>(a, f, 0, pxy, pz);
            t1 = tap<LAYOUT, WRAP>(a, f, 1, pxy, pz);
            t2 = tap<LAYOUT, WRAP>(a, f, 2, pxy, pz);
            t3 = tap<LAYOUT, WRAP>(a, f, 3, pxy, pz);
        }
        acc = acc + ((t0 * t1) * (t2 + t3)) * (LAYOUT == LAYOUT_CORNERH ? f.scale : a.scale);   // :71-73
        pxy = pxy + r.sxy;                                                            // :74
        pz = pz + r.sz;
        if constexpr (EARLY) {
            if (acc > a.acc_limit) { ++i; break; }
        }
    }
    if (r.live) {
        const float at = acc * a.step_size;                                          // :76
        store_pixel(a, x, orow, r.n >= 0, 1.0f - spec_expf(a.density * fminf(-at, 0.0f)));   // :79
    }
    return r.n > 0 ? (unsigned)i : 0u;
}

// Procedural medium (BASELINE configs 2/3, build-defined; spec in
// oracle/vr_oracle.h vro_procedural): fBm Perlin x (1 - Worley F1).
// TABLE: 0 = direct noise, 1 = LDS tables with runtime Worley geometry,
// 2 = LDS tables with the fixed 9-cell geometry (noise::cellular_table9),
// 3 = 2 + the global Perlin lattice table (noise::perlin_lat)
// `cells` accumulates the Worley cells this evaluation computed (8, or 35 when
// the pruned lane also ran the 27-cell block; 27 without the pruned table) --
// vr option "count" = 2, the algorithmic work of the roofline (bench.py)
// WC: the Worley cube comes from the lane's register cache *wc
// (noise::cellular_table9_cached; the deferred shadow pass)
// The loop-invariant operands of proc_density, pinned to VGPRs ONCE, before
// a kernel's step / sample loops: a VALU op reading an SGPR issues at half
// rate, and an in_vgpr() inside the density is re-done
// (v_mov from the SGPR) at every evaluation -- the round-4 shadow pass spent
// 7 of its ~44 per-sample instructions outside the octaves on those copies.
#ifndef VR_PROC_WAVES   // the primary procedural marches (unrolled fBm) held to 4 waves per SIMD (<= 128 VGPRs)
#define VR_PROC_WAVES 4
#endif
#ifndef VR_PROC_ATTR
#if VR_PROC_WAVES > 0
#define VR_PROC_ATTR __attribute__((amdgpu_waves_per_eu(VR_PROC_WAVES)))
#else
#define VR_PROC_ATTR
#endif
#endif
// the deferred-shadow primary march (config 3): the unrolled fBm without the
// occupancy cap -- 0.905 ms vs 0.937 capped at 4 waves and 0.910 for round 4's
// build (profiles/r05/ab_defer.txt)
#ifndef VR_DEFER_UNROLL
#define VR_DEFER_UNROLL 1
#endif
#ifndef VR_DEFER_ATTR
#define VR_DEFER_ATTR
#endif
struct DensityK {
    float gs, lac, gain, f0, wf, scale;
    float lat_sy, lat_sz, lat_nc;   // TABLE 3: the lattice table's byte-offset fma constants (lat_nc = -lat_c)
    float wt_nc;                    // TABLE >= 2: noise::worley9_nc(wt_lo)
};
template <int TABLE>
__device__ __forceinline__ DensityK density_k(const ProcParams& p, float scale)
{
    DensityK k;
    k.gs = noise::in_vgpr(p.grid_scale);
    k.lac = noise::in_vgpr(p.lacunarity);
    k.gain = noise::in_vgpr(p.gain);
    k.f0 = noise::in_vgpr(p.freq0);
    k.wf = noise::in_vgpr(p.worley_freq);
    k.scale = noise::in_vgpr(scale);
    if constexpr (TABLE == 3) {
        k.lat_sy = noise::in_vgpr(p.lat_sy);
        k.lat_sz = noise::in_vgpr(p.lat_sz);
        k.lat_nc = noise::in_vgpr(-p.lat_c);
    } else {
        k.lat_sy = k.lat_sz = k.lat_nc = 0.0f;
    }
    // the negated constant terms make the offset fmas v_fmamk (literal 8 / 16)
    k.wt_nc = TABLE >= 2 ? noise::in_vgpr(noise::worley9_nc(p.wt_lo)) : 0.0f;
    return k;
}

// fBm over the lattice table (TABLE 3): the lattice word of octave o + 1 is
// loaded while octave o computes.  OCT > 0: exactly OCT octaves, fully
// unrolled (no loop-carried register copies, no loop control; the recipe's 4,
// vr_procedural_defaults); OCT = 0: p.octaves, a loop.  The same operations in
// the same order either way.
#ifndef VR_FBM_FENCE
#define VR_FBM_FENCE 0
#endif
#ifndef VR_FBM_UNROLL_BY
#define VR_FBM_UNROLL_BY 1
#endif
#ifndef VR_FBM_PREFETCH   // fbm_lat<0>: the next octave's lattice word loaded during this one
#define VR_FBM_PREFETCH 0   // off: config 3 -0.7 % (the shadow pass: 10 % fewer issue cycles, its loads now wait), profiles/r05/ab_nopf.txt
#endif
#ifndef VR_FBM_UNROLL
// the primary marches' fBm with the recipe's 4 octaves unrolled (no
// loop-carried register copies): config 2 -4 % at 4 waves per SIMD
// (VR_PROC_WAVES), profiles/r05/ab_proc_diet_*.txt; the shadow pass keeps the
// loop (unrolled it needs 104 VGPRs, and was level or slower)
#define VR_FBM_UNROLL 4
#endif
template <int OCT>
__device__ __forceinline__ float fbm_lat(const ProcParams& p, const DensityK& k, const float4* gp, float qx, float qy,
                                         float qz)
{
    const auto rsrc = __builtin_amdgcn_make_buffer_rsrc((void*)p.lat, (short)0, (int)p.lat_bytes, 0x00020000);
#if !VR_FBM_PREFETCH
    if constexpr (OCT == 0) {   // no loop-carried prefetch: each octave loads its own word
        float f = k.f0, amp = 1.0f, fbm = 0.0f;
#pragma unroll VR_FBM_UNROLL_BY
        for (int o = 0; o < p.octaves; ++o) {
            const float x = qx * f, y = qy * f, z = qz * f;
            const float xs = floorf(x), ys = floorf(y), zs = floorf(z);
            const auto w = __builtin_amdgcn_raw_buffer_load_b64(
                rsrc, (unsigned)fmaf(zs, k.lat_sz, fmaf(ys, k.lat_sy, fmaf(xs, 8.0f, k.lat_nc))), 0, 0);
            const float pn = noise::perlin_lat(gp, make_uint2(w[0], w[1]), x, y, z, xs, ys, zs);
            fbm = fmaf(amp, pn, fbm);
            f = f * k.lac;
            amp = amp * k.gain;
        }
        return fbm;
    }
#endif
    float f = k.f0, amp = 1.0f, fbm = 0.0f;
    float x = qx * f, y = qy * f, z = qz * f;
    float xs = floorf(x), ys = floorf(y), zs = floorf(z);
    auto word = __builtin_amdgcn_raw_buffer_load_b64(
        rsrc, (unsigned)fmaf(zs, k.lat_sz, fmaf(ys, k.lat_sy, fmaf(xs, 8.0f, k.lat_nc))), 0, 0);
    const int n = OCT > 0 ? OCT : p.octaves;
    auto octave = [&](int o) {
        const uint2 w = make_uint2(word[0], word[1]);
        const float cx = x, cy = y, cz = z, cxs = xs, cys = ys, czs = zs;
        f = f * k.lac;
        if (o + 1 < n) {
            x = qx * f; y = qy * f; z = qz * f;
            xs = floorf(x); ys = floorf(y); zs = floorf(z);
            word = __builtin_amdgcn_raw_buffer_load_b64(
                rsrc, (unsigned)fmaf(zs, k.lat_sz, fmaf(ys, k.lat_sy, fmaf(xs, 8.0f, k.lat_nc))), 0, 0);
        }
        const float pn = noise::perlin_lat(gp, w, cx, cy, cz, cxs, cys, czs);
        fbm = fmaf(amp, pn, fbm);
        amp = amp * k.gain;
    };
    if constexpr (OCT > 0) {
#pragma unroll
        for (int o = 0; o < OCT; ++o) {
            octave(o);
#if VR_FBM_FENCE
            // keep each octave's instructions in their own block, so that the
            // scheduler does not hoist later octaves' loads and LDS reads (and
            // their registers) into earlier ones
            __builtin_amdgcn_sched_barrier(0);
#endif
        }
    } else {
#pragma unroll VR_FBM_UNROLL_BY
        for (int o = 0; o < n; ++o) octave(o);
    }
    return fbm;
}

// The recipe's density (TABLE 3, OCT octaves unrolled) in three phases: the
// lattice words of every octave are loaded first, the Worley cube is computed
// while they are in flight (its LDS reads and ~100 VALU ops hide the global
// load latency that fbm_lat<OCT> waits out at its first octave), then the
// octaves.  The same operations on the same values as proc_density: the fBm
// and F1 are independent until the final combine.
#ifndef VR_PROC_PHASES
#define VR_PROC_PHASES 1   // config 2 -2.8 %, config 3 -1.7 % (profiles/r05/ab_phases.txt)
#endif
#ifndef VR_PHASE_FENCE
#define VR_PHASE_FENCE 1
#endif
template <int OCT>
__device__ __forceinline__ float proc_density_phased(const ProcParams& p, const DensityK& k, const float4* wt,
                                                     float px, float py, float pz, unsigned& cells)
{
    const float qx = px * k.gs, qy = py * k.gs, qz = pz * k.gs;
    const float4* gp = wt + noise::kWorleyN * noise::kWorleyPz;
    const auto rsrc = __builtin_amdgcn_make_buffer_rsrc((void*)p.lat, (short)0, (int)p.lat_bytes, 0x00020000);
    float X[OCT], Y[OCT], Z[OCT], XS[OCT], YS[OCT], ZS[OCT];
    uint2 W[OCT];
    float f = k.f0;
#pragma unroll
    for (int o = 0; o < OCT; ++o) {
        if (o > 0) f = f * k.lac;
        X[o] = qx * f; Y[o] = qy * f; Z[o] = qz * f;
        XS[o] = floorf(X[o]); YS[o] = floorf(Y[o]); ZS[o] = floorf(Z[o]);
        const auto w = __builtin_amdgcn_raw_buffer_load_b64(
            rsrc, (unsigned)fmaf(ZS[o], k.lat_sz, fmaf(YS[o], k.lat_sy, fmaf(XS[o], 8.0f, k.lat_nc))), 0, 0);
        W[o] = make_uint2(w[0], w[1]);
    }
#if VR_PHASE_FENCE
    __builtin_amdgcn_sched_barrier(0);
#endif
    const float wf = k.wf;
    bool full;
    const float f1 = noise::cellular_table9(wt, k.wt_nc, qx * wf, qy * wf, qz * wf, full) + 1.0f;
    if (p.count_evals == 2) cells += full ? 35u : 8u;
#if VR_PHASE_FENCE
    __builtin_amdgcn_sched_barrier(0);
#endif
    float amp = 1.0f, fbm = 0.0f;
#pragma unroll
    for (int o = 0; o < OCT; ++o) {
        const float pn = noise::perlin_lat(gp, W[o], X[o], Y[o], Z[o], XS[o], YS[o], ZS[o]);
        fbm = fmaf(amp, pn, fbm);
        amp = amp * k.gain;
    }
    return fmaxf(fbm * (1.0f - f1), 0.0f) * k.scale;
}

template <int TABLE, bool WC = false, bool UNROLL = false>
__device__ __forceinline__ float proc_density(const ProcParams& p, const DensityK& k, const float4* wt, float px,
                                              float py, float pz, unsigned& cells, noise::WorleyCube* wc = nullptr)
{
#if VR_PROC_PHASES && VR_FBM_UNROLL
    if constexpr (TABLE == 3 && UNROLL && !WC)
        if (p.octaves == VR_FBM_UNROLL) return proc_density_phased<VR_FBM_UNROLL>(p, k, wt, px, py, pz, cells);
#endif
    const float qx = px * k.gs, qy = py * k.gs, qz = pz * k.gs;
    float fbm = 0.0f;
    if constexpr (TABLE == 3) {
        const float4* gp = wt + noise::kWorleyN * noise::kWorleyPz;
#if VR_FBM_UNROLL
        if constexpr (UNROLL)
            fbm = p.octaves == VR_FBM_UNROLL ? fbm_lat<VR_FBM_UNROLL>(p, k, gp, qx, qy, qz) : fbm_lat<0>(p, k, gp, qx, qy, qz);
        else
            fbm = fbm_lat<0>(p, k, gp, qx, qy, qz);
#else
        fbm = fbm_lat<0>(p, k, gp, qx, qy, qz);
#endif
    } else {
        float f = k.f0, amp = 1.0f;
        for (int o = 0; o < p.octaves; ++o) {
            float pn;
            if constexpr (TABLE == 2) pn = noise::perlin_gp(wt + noise::kWorleyN * noise::kWorleyPz, p.seed_fbm, qx * f, qy * f, qz * f);
            else if constexpr (TABLE == 1) pn = noise::perlin_gp(wt + p.wt_n * p.wt_pz, p.seed_fbm, qx * f, qy * f, qz * f);
            else pn = noise::perlin(p.seed_fbm, qx * f, qy * f, qz * f);
            fbm = fmaf(amp, pn, fbm);
            f = f * k.lac;
            amp = amp * k.gain;
        }
    }
    const float wf = k.wf;
    float f1;
    if constexpr (TABLE >= 2) {
        bool full;
        if constexpr (WC) f1 = noise::cellular_table9_cached(wt, k.wt_nc, qx * wf, qy * wf, qz * wf, full, *wc) + 1.0f;
        else f1 = noise::cellular_table9(wt, k.wt_nc, qx * wf, qy * wf, qz * wf, full) + 1.0f;
        if (p.count_evals == 2) cells += full ? 35u : 8u;
    } else {
        if constexpr (TABLE == 1) f1 = noise::cellular_table(wt, p.wt_lo, p.wt_n, p.wt_pz, qx * wf, qy * wf, qz * wf) + 1.0f;
        else f1 = noise::cellular(p.seed_worley, qx * wf, qy * wf, qz * wf) + 1.0f;
        if (p.count_evals == 2) cells += 27u;
    }
    return fmaxf(fbm * (1.0f - f1), 0.0f) * k.scale;
}

// Pixel value of the procedural march: single scatter, or frag.glsl:76-80.
template <bool SHADOW>
__device__ __forceinline__ float proc_epilogue(const MarchArgs& a, float acc, float rad)
{
    if constexpr (SHADOW) {
        return rad;
    } else {
        const float at = acc * a.step_size;
        return 1.0f - spec_expf(a.density * fminf(-at, 0.0f));
    }
}

template <bool SHADOW, bool EARLY, int TABLE>
__device__ __forceinline__ unsigned march_pixel_proc(const MarchArgs& a, const float4* wt, int x, int orow)
{
    const Ray r = setup_ray(a, x, orow);
    const ProcParams& p = a.proc;
    float P0 = r.pxy.x, P1 = r.pxy.y, P2 = r.pz;
    float acc = 0.0f, rad = 0.0f, tv = 1.0f;
    int i = 0;
    unsigned evals = 0;   // shadow density evaluations
    unsigned cells = 0;   // Worley cells computed (count mode 2)
    const DensityK dk = density_k<TABLE>(p, a.scale);
    for (; i < r.n; ++i) {
        const float rho = proc_density<TABLE, false, true>(p, dk, wt, P0, P1, P2, cells);
        if constexpr (SHADOW) {
            if (rho > 0.0f) {
                float q0 = P0, q1 = P1, q2 = P2, sl = 0.0f;
                for (int j = 0; j < p.shadow_steps; ++j) {
                    q0 = q0 + p.lstep[0]; q1 = q1 + p.lstep[1]; q2 = q2 + p.lstep[2];
                    if (q0 >= 0.0f && q0 <= 1.0f && q1 >= 0.0f && q1 <= 1.0f && q2 >= 0.0f && q2 <= 1.0f) {
                        sl = sl + proc_density<TABLE>(p, dk, wt, q0, q1, q2, cells);
                        ++evals;
                    }
                }
                const float tl = spec_expf(-(sl * p.od));
                rad = fmaf((tv * (rho * p.od)), tl, rad);
            }
        }
        acc = acc + rho;
        if constexpr (SHADOW) tv = spec_expf(-(acc * p.od));
        P0 = P0 + r.sxy.x; P1 = P1 + r.sxy.y; P2 = P2 + r.sz;
        if constexpr (EARLY) {
            if (acc > a.acc_limit) { ++i; break; }
        }
    }
    if (r.live) store_pixel(a, x, orow, r.n >= 0, proc_epilogue<SHADOW>(a, acc, rad));
    if (r.n <= 0) return 0u;
    if (p.count_evals == 2) return cells;
    return p.count_evals ? (unsigned)i + evals : (unsigned)i;
}

// Shadow-ray compaction (config 3).  In march_pixel_proc a wave runs all
// shadow_steps density evaluations whenever ANY lane has rho > 0, so most
// lanes idle.  Here a wave instead deals the (lane, shadow step) pairs of the
// lanes that need them over all 64 lanes: cnt lanes need cnt * S evaluations,
// done in ceil(cnt * S / 64) rounds.  The results go through LDS and each lane
// then sums its own S values in step order, so the arithmetic (and the
// repeated-addition shadow positions) is exactly march_pixel_proc's.
// Requires wave-uniform control flow: every lane of the wave calls it.
// The pairs are dealt owner-major (a lane's run of steps is contiguous).  A
// step-major deal -- all owners' step 0, then step 1, ..., so that a round's
// neighbouring lanes evaluate neighbouring rays at one shadow step and share
// lattice cells -- cut the bank conflicts from 2.6 to 2.2 cycles per LDS
// instruction (1.4 together with the 64x64-region enumeration, option
// "proc_enum") and the VALU count by 2-6 %, yet ran 2-5 % slower
// (profiles/r03/ab_config3_deal_enum.txt, pmc_config3_deal_enum.txt): the
// conflicts are not on config 3's critical path.  Removed after measuring.
constexpr int kMaxCompactShadow = 8;
// Distance from the box faces beyond which the shadow-run fast path needs no
// per-sample test: 8 sequential adds drift < 8 * 6e-8 from the exact segment.
constexpr float kShadowInMargin = 1.0e-6f;
// Dealt pair pid lives at slot pid + pid / 32: an owner lane writes (and later
// reads) its run at off_k + c, and the offsets of neighbouring lanes step by
// their run lengths (~8), which without the pad puts 32 lanes on 4 LDS banks.
__device__ __forceinline__ int shadow_slot(int pid) { return pid + (pid >> 5); }
constexpr int kShadowSlots = 64 * kMaxCompactShadow + 64 * kMaxCompactShadow / 32;
struct ShadowLds {
    float4 p[64];                        // primary positions of the lanes that need shadow rays, [lane]
                                         // (one 16-B LDS access each way)
    union {
        unsigned code[kShadowSlots];   // dealt (lane << 3 | step) pairs, inside the box only
        float d[kShadowSlots];         // then their densities, same slot
    };
};

template <bool EARLY, int TABLE>
__device__ __forceinline__ unsigned march_pixel_proc_compact(const MarchArgs& a, const float4* wt, int x, int orow,
                                                             bool valid,
                                                             ShadowLds* sh, unsigned* shadow_evals)
{
    Ray r{};
    r.n = -1;
    if (valid) r = setup_ray(a, x, orow);
    const ProcParams& p = a.proc;
    const int S = p.shadow_steps;
    const int lane = threadIdx.x & 63;
    // the sun step in VGPRs: an add reading an SGPR issues at half rate
    const float l0 = noise::in_vgpr(p.lstep[0]), l1 = noise::in_vgpr(p.lstep[1]), l2 = noise::in_vgpr(p.lstep[2]);
    float P0 = r.pxy.x, P1 = r.pxy.y, P2 = r.pz;
    float acc = 0.0f, rad = 0.0f, tv = 1.0f;
    int i = 0;
    bool act = r.n > 0;
    unsigned evals = 0;
    unsigned cells = 0;   // Worley cells this lane computed (count mode 2), primary and dealt
    const DensityK dk = density_k<TABLE>(p, a.scale);
    for (;;) {
        act = act && i < r.n;
        if (__ballot(act) == 0) break;
        float rho = 0.0f;
        if (act) rho = proc_density<TABLE, false, true>(p, dk, wt, P0, P1, P2, cells);
        const bool need = act && rho > 0.0f;
        const unsigned long long m = __ballot(need);
        if (m) {
            // The samples q_j = P + (j+1) lstep (sequential adds) that fall inside the box form
            // one run j in [lo, lo+cnt): each coordinate moves monotonically, so its inside set
            // along j is an interval, and so is their intersection.  Only those are dealt, so
            // no lane of a round idles on an outside sample (they contribute exactly +0).
            int lo = 0, cnt = 0;
            // Fast path: the shadow samples lie on the segment from P + L to
            // P + S L (convex), and the sequential adds drift from it by at most
            // S half-ulps (< 6e-8 each below 2).  When both ends are inside the
            // box by kShadowInMargin, every sample is: the run is j = 0..S-1.
            bool slow = false;
            if (need) {
                const float fs = (float)S;
                const float a0 = fmaf(fs, l0, P0), a1 = fmaf(fs, l1, P1), a2 = fmaf(fs, l2, P2);
                const float b0 = P0 + l0, b1 = P1 + l1, b2 = P2 + l2;
                const float lo3 = fminf(fminf(fminf(a0, a1), a2), fminf(fminf(b0, b1), b2));
                const float hi3 = fmaxf(fmaxf(fmaxf(a0, a1), a2), fmaxf(fmaxf(b0, b1), b2));
                slow = !(lo3 >= kShadowInMargin && hi3 <= 1.0f - kShadowInMargin);
                cnt = slow ? 0 : S;
                sh->p[lane] = make_float4(P0, P1, P2, 0.0f);
            }
            if (__ballot(slow)) {
                if (slow) {
                    float q0 = P0, q1 = P1, q2 = P2;
                    for (int j = 0; j < S; ++j) {
                        q0 = q0 + l0; q1 = q1 + l1; q2 = q2 + l2;
                        // the box test as min3 / max3 (q is never NaN): 4 ops, not 6 compares
                        const bool in = fminf(fminf(q0, q1), q2) >= 0.0f && fmaxf(fmaxf(q0, q1), q2) <= 1.0f;
                        if (in && cnt == 0) lo = j;
                        cnt += in ? 1 : 0;
                    }
                }
            }
            // Exclusive prefix of cnt (0..8, four bits) over the wave, by bit-plane ballots.
            int off = 0, total = 0;
#pragma unroll
            for (int b = 0; b < 4; ++b) {
                const unsigned long long bb = __ballot((cnt >> b) & 1);
                off += __popcll(bb & ((1ull << lane) - 1ull)) << b;
                total += __popcll(bb) << b;
            }
            for (int c = 0; c < cnt; ++c) sh->code[shadow_slot(off + c)] = ((unsigned)lane << 3) | (unsigned)(lo + c);
            __builtin_amdgcn_wave_barrier();
            for (int base = 0; base < total; base += 64) {
                const int pid = base + lane;
                if (pid < total) {
                    const unsigned code = sh->code[shadow_slot(pid)];
                    const int kk = (int)(code >> 3), j = (int)(code & 7u);
                    const float4 pk = sh->p[kk];
                    float q0 = pk.x, q1 = pk.y, q2 = pk.z;
                    for (int jj = 0; jj <= j; ++jj) { q0 = q0 + l0; q1 = q1 + l1; q2 = q2 + l2; }
                    sh->d[shadow_slot(pid)] = proc_density<TABLE>(p, dk, wt, q0, q1, q2, cells);
                    ++evals;
                }
            }
            __builtin_amdgcn_wave_barrier();
            if (need) {
                float sl = 0.0f;
                for (int c = 0; c < cnt; ++c) sl = sl + sh->d[shadow_slot(off + c)];
                const float tl = spec_expf(-(sl * p.od));
                rad = fmaf((tv * (rho * p.od)), tl, rad);
            }
            __builtin_amdgcn_wave_barrier();
        }
        if (act) {
            acc = acc + rho;
            tv = spec_expf(-(acc * p.od));
            P0 = P0 + r.sxy.x; P1 = P1 + r.sxy.y; P2 = P2 + r.sz;
            ++i;
            if constexpr (EARLY) {
                if (acc > a.acc_limit) act = false;
            }
        }
    }
    if (r.live) store_pixel(a, x, orow, r.n >= 0, rad);
    if (p.count_evals == 2) {   // every lane's cells, also those a lane computed for another's shadow ray
        *shadow_evals = 0;
        return cells;
    }
    *shadow_evals = evals;
    return r.n > 0 ? (unsigned)i : 0u;
}

// Lane -> pixel inside an 8x8 wave tile.  Default row-major, so each 16-lane
// TA group of a narrow load (tools/tcp_calib.hip) is an 8x2 strip; compact
// 4x4 groups were measured no better for brick5 and 15 % slower for brick8's
// u16 loads.  BRICK5's 12-byte loads are looked up per 4 lanes, and there 2x2
// pixel quads (4x4 of them per tile) are 2.6 % faster at 512^3 than 4x1 rows
// (neutral for the other layouts, 20 % slower for planar).
#ifndef VR_LANEMAP
#define VR_LANEMAP 0   // timing experiments: COL48 lanes 1 = 4x1 row quads, 2 = 1x4 column quads
#endif
template <int LAYOUT = 0>
__device__ __forceinline__ int lane_x(int lane)
{
    if constexpr (LAYOUT == LAYOUT_COL48 && VR_LANEMAP == 1) return lane & 7;
    else if constexpr (LAYOUT == LAYOUT_COL48 && VR_LANEMAP == 2) return lane >> 3;
    else if constexpr (LAYOUT == LAYOUT_BRICK5 || LAYOUT == LAYOUT_ZPAIR || LAYOUT == LAYOUT_COL48Z || is_b4_family(LAYOUT)) return ((lane >> 2) & 3) * 2 + (lane & 1);
    else return lane & 7;
}
template <int LAYOUT = 0>
__device__ __forceinline__ int lane_y(int lane)
{
    if constexpr (LAYOUT == LAYOUT_COL48 && VR_LANEMAP == 1) return lane >> 3;
    else if constexpr (LAYOUT == LAYOUT_COL48 && VR_LANEMAP == 2) return lane & 7;
    else if constexpr (LAYOUT == LAYOUT_BRICK5 || LAYOUT == LAYOUT_ZPAIR || LAYOUT == LAYOUT_COL48Z || is_b4_family(LAYOUT)) return (lane >> 4) * 2 + ((lane >> 1) & 1);
    else return lane >> 3;
}

#ifdef VR_TIMELINE
// Timing experiments only (make timeline -> libvr_tl.so, tools/timeline.py):
// per wave of a regions launch, {start, end} in s_memrealtime ticks (100 MHz),
// the wave's XCD (blockIdx % 8), its SIMD / CU / SE (HW_ID) and its executed
// lane-steps.
constexpr int kTimelineWaves = 1 << 16;
__device__ unsigned long long g_timeline[kTimelineWaves][3];
__device__ __forceinline__ void timeline_record(unsigned long long t_begin, unsigned long long steps)
{
    for (int off = 32; off > 0; off >>= 1) steps += __shfl_xor(steps, off);
    const unsigned long long t_end = __builtin_amdgcn_s_memrealtime();
    const int wid = (int)blockIdx.x * (int)(blockDim.x >> 6) + (threadIdx.x >> 6);
    if ((threadIdx.x & 63) == 0 && wid < kTimelineWaves) {
        g_timeline[wid][0] = t_begin;
        g_timeline[wid][1] = t_end;
        // HW_ID (hwreg 4): wave slot [3:0], SIMD [5:4], pipe [7:6], CU [11:8], SH [12], SE [15:13]
        const unsigned hw = (unsigned)__builtin_amdgcn_s_getreg((31 << 11) | 4);
        g_timeline[wid][2] = (steps << 24) | ((unsigned long long)((hw >> 4) & 0xfffu) << 8) | (blockIdx.x & 7);
    }
}
#endif

__device__ __forceinline__ void add_steps(const MarchArgs& a, unsigned long long cnt)
{
    for (int off = 32; off > 0; off >>= 1) cnt += __shfl_xor(cnt, off);
    if ((threadIdx.x & 63) == 0 && cnt) atomicAdd(a.step_counter, cnt);
}

// Kernel prologue for the fast layouts: buffer descriptors (wave-uniform,
// from kernargs only) and the per-axis offset tables, built in LDS by the
// whole workgroup.  The tables are the only LDS use and are read-only after
// the barrier.
template <int LAYOUT>
__device__ __forceinline__ FastCtx fast_prologue(const MarchArgs& a, unsigned* lds)
{
    FastCtx f{};
    if constexpr (LAYOUT == LAYOUT_CORNERH) {
        // no offset tables: the index is arithmetic (tap_fetch)
        for (int c = 0; c < 4; ++c)
            f.rsrc[c] = __builtin_amdgcn_make_buffer_rsrc((void*)(a.vol + (size_t)c * a.plane_stride), (short)0,
                                                          (int)a.plane_stride, 0x00020000);
        f.s1x16 = (float)(16 * a.geom.nbx);
        f.s2x16 = (float)(16 * a.geom.nbx) * (float)a.geom.nby;
        for (int c = 0; c < 4; ++c) {
            f.sz[c] = noise::in_vgpr(a.tap_S[c][2]);
            f.oz[c] = noise::in_vgpr(a.tap_T[c][2]);
        }
        f.scale = noise::in_vgpr(a.scale);
    } else if constexpr (LAYOUT == LAYOUT_COL48Z) {
        for (int c = 0; c < 4; ++c)
            f.rsrc[c] = __builtin_amdgcn_make_buffer_rsrc((void*)(a.vol + (size_t)c * a.plane_stride), (short)0,
                                                          (int)(c < 3 ? a.plane_stride : a.plane3_bytes), 0x00020000);
        const int nx1 = a.nx + 1, ny1 = a.ny + 1, nz1 = a.nz + 1, n3 = nx1 + ny1 + nz1;
        for (int i = threadIdx.x; i < 2 * n3; i += (int)blockDim.x) {
            const int set = i >= n3, j = i - set * n3;
            const int axis = j < nx1 ? 0 : j < nx1 + ny1 ? 1 : 2;
            const int pos = axis == 0 ? j : axis == 1 ? j - nx1 : j - nx1 - ny1;
            lds[i] = set ? axis_offset(a.geom3, LAYOUT_ZPAIR, axis, pos) : axis_offset(a.geom, LAYOUT_COL48, axis, pos);
        }
        __syncthreads();
        f.tx = lds;
        f.ty = lds + nx1;
        f.tz = lds + nx1 + ny1;
        f.tx3 = lds + n3;
        f.ty3 = lds + n3 + nx1;
        f.tz3 = lds + n3 + nx1 + ny1;
    } else if constexpr (LAYOUT != LAYOUT_PLANAR) {
        for (int c = 0; c < 4; ++c)
            f.rsrc[c] = __builtin_amdgcn_make_buffer_rsrc((void*)(a.vol + (size_t)c * a.plane_stride), (short)0,
                                                          (int)a.plane_stride, 0x00020000);
        const int nx1 = a.nx + 1, ny1 = a.ny + 1, nz1 = a.nz + 1;
        for (int i = threadIdx.x; i < nx1 + ny1 + nz1; i += (int)blockDim.x) {
            const int axis = i < nx1 ? 0 : i < nx1 + ny1 ? 1 : 2;
            const int pos = axis == 0 ? i : axis == 1 ? i - nx1 : i - nx1 - ny1;
            lds[i] = axis_offset(a.geom, LAYOUT, axis, pos);   // once per workgroup
        }
        __syncthreads();
        f.tx = lds;
        f.ty = lds + nx1;
        f.tz = lds + nx1 + ny1;
    }
    return f;
}

// Static schedule: one 16x16 tile per workgroup, one 8x8 sub-tile per wave.
// Tile rows are dealt to XCDs round-robin: XCD x (= blockIdx % 8 under the
// observed dispatch, a speed-only assumption) walks tile rows x, x+8, ...
template <int LAYOUT, int WRAP, bool EARLY>
__global__ __launch_bounds__(kThreads) void march_grid(const MarchArgs a)
{
    extern __shared__ __attribute__((aligned(16))) unsigned lds[];
    const int xcd = blockIdx.x & 7, j = blockIdx.x >> 3;
    const int k = j / a.tiles_x, tx = j - k * a.tiles_x;
    const int ty = xcd + 8 * k;
    if (ty >= a.tiles_y) return;   // whole workgroup: uniform, before the barrier
    const FastCtx f = fast_prologue<LAYOUT>(a, lds);
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int x = tx * kTile + (wave & 1) * 8 + lane_x<LAYOUT>(lane);
    const int orow = ty * kTile + (wave >> 1) * 8 + lane_y<LAYOUT>(lane);
    const unsigned steps = march_pixel<LAYOUT, WRAP, EARLY>(a, f, x, orow);
    if (a.step_counter) add_steps(a, steps);
}

// Strided schedule: wave g (of nw) renders 8x8 tiles g, g + nw, g + 2nw, ...
// of the row-major tile grid.  Its tiles sit 1/T of the image apart, so the
// per-wave (and per-SIMD) work evens out without atomics.
template <int LAYOUT, int WRAP, bool EARLY>
__global__ __launch_bounds__(kThreads) void march_strided(const MarchArgs a, int nw)
{
    extern __shared__ __attribute__((aligned(16))) unsigned lds[];
    const FastCtx f = fast_prologue<LAYOUT>(a, lds);
    const int lane = threadIdx.x & 63;
    const int g = blockIdx.x * (kThreads / 64) + (threadIdx.x >> 6);
    const int tiles_x8 = (a.width + 7) >> 3, rows8 = (a.out_rows + 7) >> 3;
    const int ntiles = tiles_x8 * rows8;
    unsigned long long steps = 0;
    for (int t = g; t < ntiles; t += nw) {
        const int ty = t / tiles_x8, tx = t - ty * tiles_x8;
        steps += march_pixel<LAYOUT, WRAP, EARLY>(a, f, tx * 8 + lane_x<LAYOUT>(lane), ty * 8 + lane_y<LAYOUT>(lane));
    }
    if (a.step_counter) add_steps(a, steps);
}

// Ring schedule: wave k renders the k-th 8x8 tile of square rings around the
// tile (cx, cy) under the projected box centre, where rays are longest.  The
// longest-running waves start first (longest-processing-time order), so no
// long wave is left to run alone at the end.  Ring r >= 1 holds 8r tiles and
// starts at wave (2r-1)^2; waves whose tile is off the target exit at once.
__device__ __forceinline__ bool ring_tile(int k, int cx, int cy, int* tx, int* ty)
{
    if (k == 0) { *tx = cx; *ty = cy; return true; }
    const int r = (int)((sqrtf((float)k) + 1.0f) * 0.5f);
    const int j = k - (2 * r - 1) * (2 * r - 1), side = j / (2 * r), t = j - side * 2 * r;
    if (side == 0) { *tx = cx - r + t; *ty = cy - r; }
    else if (side == 1) { *tx = cx + r; *ty = cy - r + t; }
    else if (side == 2) { *tx = cx + r - t; *ty = cy + r; }
    else { *tx = cx - r; *ty = cy + r - t; }
    return true;
}

template <int LAYOUT, int WRAP, bool EARLY, bool ZO>
__global__ __launch_bounds__(kThreads) void march_rings(const MarchArgs a, int cx, int cy, int nw, int npos)
{
    extern __shared__ __attribute__((aligned(16))) unsigned lds[];
    const FastCtx f = fast_prologue<LAYOUT>(a, lds);
    const int lane = threadIdx.x & 63;
    const int tiles_x8 = (a.width + 7) >> 3, rows8 = (a.out_rows + 7) >> 3;
    unsigned long long steps = 0;
    // wave g takes ring positions g, g + nw, ... (nw = all waves): fewer
    // workgroups, so fewer LDS-table prologues, in the same inside-out order
    for (int k = blockIdx.x * (kThreads / 64) + (threadIdx.x >> 6); k < npos; k += nw) {
        int tx, ty;
        ring_tile(k, cx, cy, &tx, &ty);
        if (tx >= 0 && tx < tiles_x8 && ty >= 0 && ty < rows8)
            steps += march_pixel<LAYOUT, WRAP, EARLY, ZO>(a, f, tx * 8 + lane_x<LAYOUT>(lane),
                                                      ty * 8 + lane_y<LAYOUT>(lane));
    }
    if (a.step_counter) add_steps(a, steps);
}

// Regions schedule: each XCD renders one host-built list of 8x8 tiles, a few
// contiguous angular wedges of the frame around the box centre with equal
// estimated work, inside-out (vr_api.cpp build_regions).  Rays of neighbouring
// tiles read the same 128-B bricks, so keeping neighbours on one XCD lets its
// L2 serve them once: the lines the eight L2s fetch per 1080p frame at 512^3
// drop from ~900 MB (ring positions dealt round-robin over XCDs) to ~620 MB
// (DESIGN.md sec. 5.3).  XCD = blockIdx % 8 is a speed-only assumption.
// WGW waves per workgroup (option wg_waves): the waves of one workgroup run on
// one CU and share its L1, and they render consecutive list entries.
// The regions lists' empty tiles (MarchArgs.empty_fill; vr_internal.h
// tile_is_empty): XCD x's entries [marched, count) after the marched ones.
// Wave w of the XCD writes the uncovered value -- what the march stores for a
// ray that misses (setup_ray, store_pixel) -- to the pixels of entries
// marched + w, marched + w + nwx, ...: one store per lane, no ray setup.
__device__ __forceinline__ void fill_empty_tiles(const MarchArgs& a, const unsigned* __restrict__ tiles, int begin,
                                                 int marched, int count, int w, int nwx)
{
    const int lane = threadIdx.x & 63, lx = lane & 7, ly = lane >> 3;
    for (int k = marched + w; w < nwx && k < count; k += nwx) {
        const unsigned t = tiles[begin + k];
        const int x = (int)(t & 0xffffu) * 8 + lx, orow = (int)(t >> 16) * 8 + ly;
        if (x < a.width && orow < a.out_rows) {
            const int bl = orow / a.band_rows;
            const int y = set_band(bl, a.band_first, a.band_stride, a.band_flip) * a.band_rows + (orow - bl * a.band_rows);
            if (y < a.height) store_pixel(a, x, orow, false, 0.0f);
        }
    }
}

template <int LAYOUT, int WRAP, bool EARLY, bool ZO, int WGW, int UM>
__device__ __forceinline__ void regions_body(const MarchArgs& a, const unsigned* __restrict__ tiles, const int* __restrict__ hdr, int nwx,
                                             unsigned* lds)
{
    const int xcd = blockIdx.x & 7;
    const int w = (int)(blockIdx.x >> 3) * WGW + (threadIdx.x >> 6);
    const int begin = hdr[xcd], all = hdr[xcd + 1] - begin;
    const int count = a.empty_fill ? min(hdr[kRegionWork + xcd], all) : all;   // marched entries
    if (a.empty_fill) fill_empty_tiles(a, tiles, begin, count, all, w, nwx);
    if ((int)(blockIdx.x >> 3) * WGW >= count) return;   // whole workgroup, before the barrier
#ifdef VR_TIMELINE
    const unsigned long long t_begin = __builtin_amdgcn_s_memrealtime();
#endif
    const FastCtx f = fast_prologue<LAYOUT>(a, lds);
    const int lane = threadIdx.x & 63;
    unsigned long long steps = 0;
    for (int k = w; w < nwx && k < count; k += nwx) {   // the grid rounds nwx up to whole workgroups
        const unsigned t = tiles[begin + k];
        const int tx = (int)(t & 0xffffu), ty = (int)(t >> 16);
        steps += march_pixel<LAYOUT, WRAP, EARLY, ZO, UM>(a, f, tx * 8 + lane_x<LAYOUT>(lane),
                                                          ty * 8 + lane_y<LAYOUT>(lane));
    }
#ifdef VR_TIMELINE
    timeline_record(t_begin, steps);
#endif
    if (a.step_counter) add_steps(a, steps);
}
template <int LAYOUT, int WRAP, bool EARLY, bool ZO, int WGW = kThreads / 64>
__global__ __launch_bounds__(64 * WGW) void march_regions(const MarchArgs a, const unsigned* __restrict__ tiles,
                                                         const int* __restrict__ hdr, int nwx)
{
    extern __shared__ __attribute__((aligned(16))) unsigned lds[];
    regions_body<LAYOUT, WRAP, EARLY, ZO, WGW, 0>(a, tiles, hdr, nwx, lds);
}
// with uniform channels UM (march_pixel's fetch_u / blend_u)
#ifndef VR_UM_ATTR
#ifdef VR_UM_WAVES   // timing experiments: the _u kernels built for this many waves per SIMD
#define VR_UM_ATTR __attribute__((amdgpu_waves_per_eu(VR_UM_WAVES)))
#else
#define VR_UM_ATTR
#endif
#endif
template <int LAYOUT, int WRAP, bool EARLY, bool ZO, int UM>
__global__ __launch_bounds__(kThreads) VR_UM_ATTR void march_regions_u(const MarchArgs a, const unsigned* __restrict__ tiles,
                                                                      const int* __restrict__ hdr, int nwx)
{
    extern __shared__ __attribute__((aligned(16))) unsigned lds[];
    regions_body<LAYOUT, WRAP, EARLY, ZO, kThreads / 64, UM>(a, tiles, hdr, nwx, lds);
}


// ---- step-split rays (regions schedule) ----
// A wave whose rays march alone on their SIMD waits ~110 dependent memory
// round trips (the longest ray's steps): with a small share of the frame per
// GPU (N GPUs strong-scaled) there are too few waves to hide that.  Here K
// lanes share one ray: lane k computes the terms of steps k, k+K, k+2K, ...
// and the K terms of each round are added to `acc` in step order, so the sum
// is frag.glsl:71-73's sequential one, bit for bit.  A lane reaches its own
// ray points by the same sequence of fp32 adds as the reference loop (k adds,
// then K per round): P_i is never formed as P_0 + i*step.  The K lanes of a
// ray share n, so they loop, shuffle and stop together.  Lanes beyond the
// last step fetch the ray's entry point (in the box) and their terms are not
// added.
template <int LAYOUT, bool EARLY, bool ZO, int K, int UM = 0>
__device__ __forceinline__ unsigned march_pixel_split(const MarchArgs& a, const FastCtx& f, int x, int orow,
                                                      int k, int ray_lane)
{
    constexpr int R = 64 / K;
    const Ray r = setup_ray(a, x, orow);
    float uv[4] = {};
    if constexpr (UM != 0)
        for (int t = 0; t < 4; ++t)
            if ((UM >> t) & 1) uv[t] = noise::in_vgpr(a.uval[t]);
    const int n = r.n;
    f2 pxy = r.pxy;
    float pz = r.pz;
    for (int j = 0; j < k; ++j) { pxy = pxy + r.sxy; pz = pz + r.sz; }   // this lane's first step
    float acc = 0.0f;
    int i = 0;
    if (n > 0) {
        const bool mine0 = k < n;
        TapRaw c0 = fetch_u<UM, 0, LAYOUT, ZO>(a, f, mine0 ? pxy : r.pxy, mine0 ? pz : r.pz);
        TapRaw c1 = fetch_u<UM, 1, LAYOUT, ZO>(a, f, mine0 ? pxy : r.pxy, mine0 ? pz : r.pz);
        TapRaw c2 = fetch_u<UM, 2, LAYOUT, ZO>(a, f, mine0 ? pxy : r.pxy, mine0 ? pz : r.pz);
        TapRaw c3 = fetch_u<UM, 3, LAYOUT, ZO>(a, f, mine0 ? pxy : r.pxy, mine0 ? pz : r.pz);
        for (int base = 0; base < n; base += K) {
            for (int j = 0; j < K; ++j) { pxy = pxy + r.sxy; pz = pz + r.sz; }   // step base + K + k
            const bool mine = base + K + k < n;
            const f2 qxy = mine ? pxy : r.pxy;
            const float qz = mine ? pz : r.pz;
            const TapRaw n0 = fetch_u<UM, 0, LAYOUT, ZO>(a, f, qxy, qz), n1 = fetch_u<UM, 1, LAYOUT, ZO>(a, f, qxy, qz);
            const TapRaw n2 = fetch_u<UM, 2, LAYOUT, ZO>(a, f, qxy, qz), n3 = fetch_u<UM, 3, LAYOUT, ZO>(a, f, qxy, qz);
            const float t0 = blend_u<UM, 0, LAYOUT>(c0, uv), t1 = blend_u<UM, 1, LAYOUT>(c1, uv);
            const float t2 = blend_u<UM, 2, LAYOUT>(c2, uv), t3 = blend_u<UM, 3, LAYOUT>(c3, uv);
            const float term = ((t0 * t1) * (t2 + t3)) * a.scale;                        // :71-73
            bool stop = false;
#pragma unroll
            for (int j = 0; j < K; ++j) {
                const float tj = __shfl(term, ray_lane + j * R);
                if (base + j < n && !stop) {
                    acc = acc + tj;
                    ++i;
                    if constexpr (EARLY) stop = acc > a.acc_limit;
                }
            }
            if constexpr (EARLY) {
                if (stop) break;
            }
            c0 = n0; c1 = n1; c2 = n2; c3 = n3;
        }
    }
    if (r.live && k == 0) {
        const float at = acc * a.step_size;
        store_pixel(a, x, orow, n >= 0, 1.0f - spec_expf(a.density * fminf(-at, 0.0f)));
    }
    return (n > 0 && k == 0) ? (unsigned)i : 0u;
}

// Regions schedule with step-split rays: an 8x8 tile is K sub-blocks of 64/K
// rays (8x8, 8x4, 4x4, 4x2 pixels), one per wave; wave w of its XCD's nwx
// renders the units (tile, sub-block) w, w + nwx, ...  Lane = k * (64/K) + ray,
// so 4 adjacent lanes are a 2x2 pixel quad at the same step offset.
template <int LAYOUT, bool EARLY, bool ZO, int K, int UM = 0>
__global__ __launch_bounds__(kThreads) void march_regions_split(const MarchArgs a, const unsigned* __restrict__ tiles,
                                                               const int* __restrict__ hdr, int nwx)
{
    constexpr int R = 64 / K, SW = K >= 4 ? 4 : 8, SH = R / SW, NSX = 8 / SW;
    extern __shared__ __attribute__((aligned(16))) unsigned lds[];
    const int xcd = blockIdx.x & 7;
    const int w = (int)(blockIdx.x >> 3) * (kThreads / 64) + (threadIdx.x >> 6);
    const int begin = hdr[xcd], all = hdr[xcd + 1] - begin;
    const int marched = a.empty_fill ? min(hdr[kRegionWork + xcd], all) : all;
    if (a.empty_fill) fill_empty_tiles(a, tiles, begin, marched, all, w, nwx);
    const int units = marched * K;
    if ((int)(blockIdx.x >> 3) * (kThreads / 64) >= units) return;   // whole workgroup, before the barrier
    const FastCtx f = fast_prologue<LAYOUT>(a, lds);
#ifdef VR_TIMELINE
    const unsigned long long t_begin = __builtin_amdgcn_s_memrealtime();
#endif
    const int lane = threadIdx.x & 63, k = lane / R, rho = lane % R;
    const int px = ((rho >> 2) % (SW / 2)) * 2 + (rho & 1), py = ((rho >> 2) / (SW / 2)) * 2 + ((rho >> 1) & 1);
    unsigned long long steps = 0;
    for (int u = w; w < nwx && u < units; u += nwx) {
        const unsigned t = tiles[begin + u / K];
        const int s = u % K;
        const int x = (int)(t & 0xffffu) * 8 + (s % NSX) * SW + px, orow = (int)(t >> 16) * 8 + (s / NSX) * SH + py;
        steps += march_pixel_split<LAYOUT, EARLY, ZO, K, UM>(a, f, x, orow, k, rho);
    }
#ifdef VR_TIMELINE
    timeline_record(t_begin, steps);
#endif
    if (a.step_counter) add_steps(a, steps);
}

template <int L, int K>
void launch_regions_split(const MarchArgs& a, bool early, const Schedule& sc, dim3 grid, size_t lds, hipStream_t s)
{
    const dim3 block(kThreads);
    if constexpr (L == LAYOUT_COL48 || L == LAYOUT_BRICK4832 || L == LAYOUT_CORNERH || L == LAYOUT_COL48Z) {
        const int um = a.umask;   // one uniform channel: no loads for it (march_regions' launcher)
        if (!early && a.zero_offsets && (um == 1 || um == 2 || um == 4 || um == 8)) {
#define VR_UMS(U) hipLaunchKernelGGL((march_regions_split<L, false, true, K, U>), grid, block, lds, s, a, sc.tiles, sc.hdr, sc.map.nwx)
            if (um == 1) VR_UMS(1);
            else if (um == 2) VR_UMS(2);
            else if (um == 4) VR_UMS(4);
            else VR_UMS(8);
#undef VR_UMS
            return;
        }
    }
    if (early && a.zero_offsets)
        hipLaunchKernelGGL((march_regions_split<L, true, true, K>), grid, block, lds, s, a, sc.tiles, sc.hdr, sc.map.nwx);
    else if (early)
        hipLaunchKernelGGL((march_regions_split<L, true, false, K>), grid, block, lds, s, a, sc.tiles, sc.hdr, sc.map.nwx);
    else if (a.zero_offsets)
        hipLaunchKernelGGL((march_regions_split<L, false, true, K>), grid, block, lds, s, a, sc.tiles, sc.hdr, sc.map.nwx);
    else
        hipLaunchKernelGGL((march_regions_split<L, false, false, K>), grid, block, lds, s, a, sc.tiles, sc.hdr, sc.map.nwx);
}

// XCD-row schedule: one 8x8 tile per wave, 4 horizontally adjacent tiles per
// workgroup.  8-px tile rows are dealt to XCDs round-robin: XCD x walks rows
// x, x+8, ... (blockIdx % 8, speed-only).  Rows interleave, so the balance
// holds, and a row's neighbours share one L2.
template <int LAYOUT, int WRAP, bool EARLY>
__global__ __launch_bounds__(kThreads) void march_xcdrows(const MarchArgs a)
{
    extern __shared__ __attribute__((aligned(16))) unsigned lds[];
    const int tiles_x8 = (a.width + 7) >> 3, rows8 = (a.out_rows + 7) >> 3;
    const int groups = (tiles_x8 + 3) >> 2;
    const int xcd = blockIdx.x & 7, j = blockIdx.x >> 3;
    const int k = j / groups, gx = j - k * groups;
    const int ty = xcd + 8 * k;
    if (ty >= rows8) return;   // whole workgroup, before the barrier
    const FastCtx f = fast_prologue<LAYOUT>(a, lds);
    const int lane = threadIdx.x & 63, tx = gx * 4 + (threadIdx.x >> 6);
    unsigned long long steps = 0;
    if (tx < tiles_x8) steps = march_pixel<LAYOUT, WRAP, EARLY>(a, f, tx * 8 + lane_x<LAYOUT>(lane), ty * 8 + lane_y<LAYOUT>(lane));
    if (a.step_counter) add_steps(a, steps);
}

// Queue schedule: persistent waves pull 8x8 tiles from 8 queues, one per
// XCD group (blockIdx % 8, speed-only).  Queue q owns the 16-row tile pairs
// p = q, q+8, ..., walked column by column.  heads[] is zeroed by a memset
// before every launch.  Every wave leaves once its queue is drained, so the
// grid always completes.
template <int LAYOUT, int WRAP, bool EARLY>
__global__ __launch_bounds__(kThreads) void march_queue(const MarchArgs a, int* __restrict__ heads)
{
    extern __shared__ __attribute__((aligned(16))) unsigned lds[];
    const FastCtx f = fast_prologue<LAYOUT>(a, lds);
    const int q = blockIdx.x & 7, lane = threadIdx.x & 63;
    const int tiles_x8 = (a.width + 7) >> 3, rows8 = (a.out_rows + 7) >> 3;
    const int pairs = (rows8 + 1) >> 1;
    const int per_pair = 2 * tiles_x8;
    const int count = q < pairs ? ((pairs - q + 7) >> 3) * per_pair : 0;
    unsigned long long steps = 0;
    for (;;) {
        int k = 0;
        if (lane == 0) k = atomicAdd(&heads[q], 1);
        k = __shfl(k, 0);
        if (k >= count) break;
        const int m = k / per_pair, rem = k - m * per_pair;
        const int row8 = 2 * (q + 8 * m) + (rem & 1), tx = rem >> 1;
        if (row8 >= rows8) continue;
        steps += march_pixel<LAYOUT, WRAP, EARLY>(a, f, tx * 8 + lane_x<LAYOUT>(lane), row8 * 8 + lane_y<LAYOUT>(lane));
    }
    if (a.step_counter) add_steps(a, steps);
}

// Procedural medium: one 8x8 tile per wave (compute-bound; no volume), in
// row order (cx < 0) or in rings around tile (cx, cy) (see march_rings).
// Noise tables for the workgroup (dynamic LDS): the Worley cell table
// (wt_n^3 float4) followed by the 256 Perlin gradient pairs (2 float4 each),
// built before any wave may leave.  Returns null when the tables are off
// (wt_n = 0).
template <int TABLE>
__device__ __forceinline__ const float4* worley_table(const ProcParams& p, float4* lds)
{
    // TABLE > 0 only when the host sized the tables (wt_n > 0): the returned
    // pointer is the LDS symbol itself, so table reads fold its address
    if constexpr (TABLE == 0) return nullptr;
    const int n = p.wt_n, cells = n * p.wt_pz;   // z pitch wt_pz >= n * n
    for (int i = threadIdx.x; i < n * n * n; i += kThreads) {
        const int ix = i % n, iy = (i / n) % n, iz = i / (n * n);
        lds[iz * p.wt_pz + iy * n + ix] = noise::cellular_cell(p.seed_worley, p.wt_lo + ix, p.wt_lo + iy, p.wt_lo + iz);
    }
    noise::grad_pair_entry(threadIdx.x, lds + cells);   // 256 pairs, one per thread
    __syncthreads();
    return lds;
}

template <bool SHADOW, bool EARLY, int TABLE>
__global__ __launch_bounds__(kThreads) void march_proc(const MarchArgs a, int cx, int cy)
{
    extern __shared__ float4 wt_lds[];
    const float4* wt = worley_table<TABLE>(a.proc, wt_lds);
    const int lane = threadIdx.x & 63;
    const int t = blockIdx.x * (kThreads / 64) + (threadIdx.x >> 6);
    const int tiles_x8 = (a.width + 7) >> 3, rows8 = (a.out_rows + 7) >> 3;
    unsigned long long steps = 0;
    int tx, ty;
    if (cx >= 0) {
        ring_tile(t, cx, cy, &tx, &ty);
    } else {
        ty = t / tiles_x8;
        tx = t - ty * tiles_x8;
    }
    if (tx >= 0 && tx < tiles_x8 && ty >= 0 && ty < rows8) {
        steps = march_pixel_proc<SHADOW, EARLY, TABLE>(a, wt, tx * 8 + lane_x(lane), ty * 8 + lane_y(lane));
    }
    if (a.step_counter) add_steps(a, steps);
}

// ---- procedural, cost-sorted schedule ----
// A ray's cost is its step count n (a3), known after the ray setup.  Pass 1
// writes every pixel with n <= 0 and builds a histogram of n; pass 2 turns it
// into descending-n offsets; pass 3 scatters the packed pixel ids (orow << 16
// | x) in that order; the march then gives wave w the sorted pixels
// [64w, 64w + 64).  Lanes of a wave share n (no loop divergence) and the
// longest rays start first (longest-processing-time order, no tail).
constexpr int kKeyBins = 1024;
// Pixels per thread of the sort passes: fewer blocks -> fewer global atomics
// on hot bins.  Measured 2/4/8/16: 16 is best (bin 21 us, scatter 11 us at
// 1080p).  Wave-aggregated LDS increments (one atomic per distinct key) were
// slower than the plain LDS atomics.
constexpr int kSortPixelsPerThread = 16;
__device__ __forceinline__ int cost_key(int n) { return n < kKeyBins - 1 ? n : kKeyBins - 1; }
// The sort passes enumerate pixels by 64x64 regions (one region per block of
// 256 threads x 16 pixels), regions in row-major order.  A key's pixels then
// come out region by region, so the 64 lanes of a sorted wave are one compact
// segment of the n-contour instead of pixels from both sides of the ring
// (row-major enumeration): neighbouring rays share Worley cells and Perlin
// corners, so their LDS table reads broadcast instead of conflicting (config
// 2: 9 % faster together with the fixed table geometry).  With shadow rays
// (config 3) row-major order is kept: there compact waves are all-or-nothing
// in shadow work, which the per-wave compaction balances worse (4 % slower).
constexpr int kSortRegion = 64;
__device__ __forceinline__ bool sort_pixel(const MarchArgs& a, unsigned idx, int* x, int* orow)
{
    if (a.proc.shadow_steps > 0 && !a.proc.enum_regions) {
        *orow = (int)(idx / (unsigned)a.width);
        *x = (int)(idx - (unsigned)*orow * (unsigned)a.width);
        return *orow < a.out_rows;
    }
    const unsigned rx = (unsigned)(a.width + kSortRegion - 1) / kSortRegion;
    const unsigned reg = idx / (kSortRegion * kSortRegion), loc = idx % (kSortRegion * kSortRegion);
    *x = (int)((reg % rx) * kSortRegion + loc % kSortRegion);
    *orow = (int)((reg / rx) * kSortRegion + loc / kSortRegion);
    return *x < a.width && *orow < a.out_rows;
}

template <bool SHADOW>
__global__ __launch_bounds__(256) void proc_bin(const MarchArgs a, unsigned* __restrict__ hist,
                                                unsigned short* __restrict__ keys)
{
    __shared__ unsigned h[kKeyBins];
    for (int i = threadIdx.x; i < kKeyBins; i += 256) h[i] = 0;
    __syncthreads();
    for (int it = 0; it < kSortPixelsPerThread; ++it) {
        const unsigned pix = (blockIdx.x * kSortPixelsPerThread + it) * 256u + threadIdx.x;   // < 2^31 (host check)
        int x, orow;
        if (!sort_pixel(a, pix, &x, &orow)) {
            keys[pix] = 0;
            continue;
        }
        const Ray r = setup_ray(a, x, orow);
        int key = 0;
        if (r.n > 0) {
            key = cost_key(r.n);
            atomicAdd(&h[key], 1u);
        } else if (r.live) {
            store_pixel(a, x, orow, r.n >= 0, proc_epilogue<SHADOW>(a, 0.0f, 0.0f));   // 0 steps
        }
        keys[pix] = (unsigned short)key;
    }
    __syncthreads();
    for (int i = threadIdx.x; i < kKeyBins; i += 256)
        if (h[i]) atomicAdd(&hist[i], h[i]);
}

// hist[kKeyBins] -> cursor[kKeyBins] (start of each key, descending keys) and
// total at cursor[kKeyBins].  One workgroup of kKeyBins threads.
// It also zeroes the histogram for the next frame (the buffer is zeroed once
// when allocated), which saves a memset launch per frame.
// Background of a frame whose sorted order is reused (same geometry): the
// pixels with no steps (key 0 in the bin pass) get (0,0,0,1), which is both
// the clear colour and the epilogue of zero steps in every format, so this is
// exactly what proc_bin stores for them.
// Run by the trailing blocks of march_proc_sorted (one launch per reused frame).
__device__ __forceinline__ void proc_fill_background(const MarchArgs& a, const unsigned short* __restrict__ keys,
                                                     unsigned positions, unsigned block, unsigned blocks)
{
    for (unsigned i = block * kThreads + threadIdx.x; i < positions; i += blocks * kThreads) {
        int x, orow;
        if (!sort_pixel(a, i, &x, &orow) || keys[i] != 0) continue;
        const int bl = orow / a.band_rows;
        const int y = set_band(bl, a.band_first, a.band_stride, a.band_flip) * a.band_rows + (orow - bl * a.band_rows);
        if (y < a.height) store_pixel(a, x, orow, false, 0.0f);
    }
}

// With shadow rays (config 3) it also lays out the deferred passes' scratch
// (ScanOut; went = null: not needed).  Sorted wave w covers the sorted
// positions [64w, 64w + 64), whose keys bound their step counts (key = n below
// kKeyBins - 1, the last key holds every n >= kKeyBins - 1, bounded by
// max_steps).  Its lanes append at most one entry per step, so its entries fit
// the sum of its lanes' bounds, and it marches at most its first (largest)
// key's bound of wave-steps.  went / wrec are the exclusive prefixes of those
// two bounds over the waves -- the thread of a key writes the waves whose
// first position falls in its key's range -- and need[] their totals, which the
// host sizes the scratch from (vr_api.cpp ensure_defer).
struct ScanOut {
    unsigned long long* went;        // [waves + 1]: first entry of sorted wave w
    unsigned* wrec;                  // [waves + 1]: first step record (saturated at 2^32 - 1)
    unsigned long long* need;        // [0] entries, [1] step records of the frame
    unsigned long long* need_host;   // the same, host-mapped (optional)
    int max_steps;
};
[[maybe_unused]] __global__ __launch_bounds__(kKeyBins) void proc_scan(unsigned* __restrict__ hist, unsigned* __restrict__ cursor,
                                                                       ScanOut so)
{
    __shared__ unsigned sc[kKeyBins];
    __shared__ unsigned long long ce[kKeyBins], cr[kKeyBins];
    const int t = threadIdx.x;
    const unsigned own = hist[kKeyBins - 1 - t];
    sc[t] = own;   // descending key order
    __syncthreads();
    for (int off = 1; off < kKeyBins; off <<= 1) {
        const unsigned v = t >= off ? sc[t - off] : 0u;
        __syncthreads();
        sc[t] += v;
        __syncthreads();
    }
    const int key = kKeyBins - 1 - t;
    const unsigned start = sc[t] - own, end = sc[t];
    cursor[key] = start;   // exclusive
    if (t == kKeyBins - 1) cursor[kKeyBins] = end;
    hist[key] = 0u;              // each thread clears the bin it read
    if (!so.went) return;        // kernel-uniform
    const unsigned long long val = key < kKeyBins - 1 ? (unsigned long long)key
                                                      : (unsigned long long)max(so.max_steps, key);
    const unsigned ws0 = (start + 63u) / 64u, ws1 = (end + 63u) / 64u;   // waves whose first position has this key
    const unsigned long long e_own = (unsigned long long)own * val, r_own = (unsigned long long)(ws1 - ws0) * val;
    ce[t] = e_own;
    cr[t] = r_own;
    __syncthreads();
    for (int off = 1; off < kKeyBins; off <<= 1) {
        const unsigned long long ve = t >= off ? ce[t - off] : 0ull, vr = t >= off ? cr[t - off] : 0ull;
        __syncthreads();
        ce[t] += ve;
        cr[t] += vr;
        __syncthreads();
    }
    const unsigned long long e0 = ce[t] - e_own, r0 = cr[t] - r_own;
    for (unsigned w = ws0; w < ws1; ++w) {
        so.went[w] = e0 + (unsigned long long)(64u * w - start) * val;
        const unsigned long long rw = r0 + (unsigned long long)(w - ws0) * val;
        so.wrec[w] = rw < 0xffffffffull ? (unsigned)rw : 0xffffffffu;
    }
    if (t == kKeyBins - 1) {   // key 0 holds no pixel: its start is the frame's end
        so.went[ws1] = ce[t];
        so.wrec[ws1] = cr[t] < 0xffffffffull ? (unsigned)cr[t] : 0xffffffffu;
        so.need[0] = ce[t];
        so.need[1] = cr[t];
        if (so.need_host) {
            so.need_host[0] = ce[t];
            so.need_host[1] = cr[t];
        }
    }
}

[[maybe_unused]] __global__ __launch_bounds__(256) void proc_scatter(const MarchArgs a, const unsigned short* __restrict__ keys,
                                                    unsigned* __restrict__ cursor, unsigned* __restrict__ order)
{
    __shared__ unsigned h[kKeyBins];
    for (int i = threadIdx.x; i < kKeyBins; i += 256) h[i] = 0;
    __syncthreads();
    int key[kSortPixelsPerThread];
    unsigned rank[kSortPixelsPerThread], packed[kSortPixelsPerThread];
    for (int it = 0; it < kSortPixelsPerThread; ++it) {
        key[it] = -1;
        const unsigned pix = (blockIdx.x * kSortPixelsPerThread + it) * 256u + threadIdx.x;
        int x, orow;
        if (sort_pixel(a, pix, &x, &orow)) {
            const int k = keys[pix];
            if (k > 0) {
                key[it] = k;
                rank[it] = atomicAdd(&h[k], 1u);
                packed[it] = ((unsigned)orow << 16) | (unsigned)x;
            }
        }
    }
    __syncthreads();
    for (int i = threadIdx.x; i < kKeyBins; i += 256)
        if (h[i]) h[i] = atomicAdd(&cursor[i], h[i]);   // block's base in the sorted list
    __syncthreads();
    for (int it = 0; it < kSortPixelsPerThread; ++it)
        if (key[it] >= 0) order[h[key[it]] + rank[it]] = packed[it];
}

template <bool SHADOW, bool EARLY, int TABLE>
__global__ __launch_bounds__(kThreads) VR_PROC_ATTR void march_proc_sorted(const MarchArgs a, const unsigned* __restrict__ order,
                                                              const unsigned* __restrict__ total_ptr,
                                                              const unsigned short* __restrict__ keys,
                                                              unsigned fill_positions, unsigned fill_first, int stale)
{
    extern __shared__ float4 wt_lds[];
    // A reused sort order (vr_render): blocks from fill_first on write the
    // pixels without steps instead of marching, so a frame is one launch.
    // A stale order (an older camera, same target): the pixels it left out
    // may have steps now, so those blocks march them (unsorted; a 1.6-degree
    // turn moves only the silhouette) -- every pixel is still written once.
    if (blockIdx.x >= fill_first) {
        if (!stale) {
            proc_fill_background(a, keys, fill_positions, blockIdx.x - fill_first, gridDim.x - fill_first);
            return;
        }
        const float4* wt = worley_table<TABLE>(a.proc, wt_lds);
        unsigned long long steps = 0;
        const unsigned blocks = gridDim.x - fill_first;
        for (unsigned i = (blockIdx.x - fill_first) * kThreads + threadIdx.x; i < fill_positions; i += blocks * kThreads) {
            int x, orow;
            if (sort_pixel(a, i, &x, &orow) && keys[i] == 0) steps += march_pixel_proc<SHADOW, EARLY, TABLE>(a, wt, x, orow);
        }
        if (a.step_counter) add_steps(a, steps);
        return;
    }
    const float4* wt = worley_table<TABLE>(a.proc, wt_lds);
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const unsigned total = *total_ptr;
    const unsigned base = (blockIdx.x * (kThreads / 64) + wave) * 64u;
    if (base >= total) return;   // wave-uniform
    const unsigned idx = base + lane;
    const bool valid = idx < total;
    int x = 0, orow = 0;
    if (valid) {
        const unsigned pk = order[idx];
        x = (int)(pk & 0xffffu);
        orow = (int)(pk >> 16);
    }
    unsigned long long steps;
    if constexpr (SHADOW) {
        __shared__ ShadowLds sh[kThreads / 64];
        if (a.proc.shadow_steps <= kMaxCompactShadow) {
            unsigned ev = 0;
            steps = march_pixel_proc_compact<EARLY, TABLE>(a, wt, x, orow, valid, &sh[wave], &ev);
            if (a.proc.count_evals) steps += ev;
        } else {
            steps = valid ? march_pixel_proc<true, EARLY, TABLE>(a, wt, x, orow) : 0u;
        }
    } else {
        steps = valid ? march_pixel_proc<false, EARLY, TABLE>(a, wt, x, orow) : 0u;
    }
    if (a.step_counter) add_steps(a, steps);
}

// ---- deferred shadow rays (config 3; vr option "shadow_defer") ----
// The compaction above deals a wave's shadow samples over its own lanes at
// every primary step, so each step ends in a partial round (lane use ~0.85)
// and pays the dealing (box scan, ballot prefix, LDS round trips).  Deferred,
// the frame runs in passes instead:
//  1. march_proc_defer: the primary march of the sorted waves (config 2's loop,
//     64x64-region enumeration).  At a step with rho > 0 a lane appends the
//     entry (P, tv * (rho * od)) -- its ray point and the coefficient the
//     single-scatter term multiplies by the sun transmittance -- to its wave's
//     own region (a running count, no atomics: one device-scope counter for
//     all waves saturates at ~88 adds/us, MI355X_MICROARCH.md, and ran the
//     frame at 3.7 ms), and the wave records {first entry, lane mask} per step.
//  2. proc_shadow_scan / proc_shadow_map: the waves' entries in chunks of 64,
//     numbered across the frame: chunk -> (wave, chunk of the wave, count).
//  3. proc_shadow_eval: one lane per entry walks the S sun samples
//     P + (j+1) L (sequential adds) and sums the in-box densities in step
//     order, tl = exp(-(sl * od)); it rewrites the entry as (coef, tl).  Lanes
//     are busy whatever the owner rays (one partial chunk per wave).
//  4. proc_shadow_resolve: the sorted waves again; a lane folds
//     rad = fma(coef, tl, rad) over its entries in step order and stores the
//     pixel.
// Every value is computed by the same ops in the same order as
// march_pixel_proc<true>, so the frame stays bit-exact.
// (struct ShadowDefer: vr_internal.h)
template <bool EARLY, int TABLE>
__global__ __launch_bounds__(kThreads) VR_DEFER_ATTR void march_proc_defer(const MarchArgs a, const unsigned* __restrict__ order,
                                                             const unsigned* __restrict__ total_ptr,
                                                             const unsigned short* __restrict__ keys,
                                                             unsigned fill_positions, unsigned fill_first, int stale,
                                                             ShadowDefer d)
{
    extern __shared__ float4 wt_lds[];
    if (blockIdx.x >= fill_first) {   // as march_proc_sorted: background, or a stale order's leftovers
        if (!stale) {
            proc_fill_background(a, keys, fill_positions, blockIdx.x - fill_first, gridDim.x - fill_first);
            return;
        }
        const float4* wt = worley_table<TABLE>(a.proc, wt_lds);
        unsigned long long steps = 0;
        const unsigned blocks = gridDim.x - fill_first;
        for (unsigned i = (blockIdx.x - fill_first) * kThreads + threadIdx.x; i < fill_positions; i += blocks * kThreads) {
            int x, orow;
            if (sort_pixel(a, i, &x, &orow) && keys[i] == 0) steps += march_pixel_proc<true, EARLY, TABLE>(a, wt, x, orow);
        }
        if (a.step_counter) add_steps(a, steps);
        return;
    }
    const float4* wt = worley_table<TABLE>(a.proc, wt_lds);
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const unsigned total = *total_ptr;
    const unsigned wid = blockIdx.x * (kThreads / 64) + wave;
    const unsigned base = wid * 64u;
    if (base >= total) return;   // wave-uniform
    const unsigned idx = base + lane;
    // the wave's ranges of entries and step records (proc_scan); past the
    // scratch (a frame larger than the one it was sized for) the wave marches
    // its shadow rays in place, and the later passes skip it
    const unsigned long long eb = d.went[wid];
    const unsigned rb = d.wrec[wid];
    if (d.went[wid + 1] > d.ent_cap || d.wrec[wid + 1] > d.rec_cap) {   // wave-uniform
        unsigned steps = 0;
        if (idx < total) {
            const unsigned pk = order[idx];
            steps = march_pixel_proc<true, EARLY, TABLE>(a, wt, (int)(pk & 0xffffu), (int)(pk >> 16));
        }
        if (lane == 0) {
            d.wsteps[wid] = kDeferInPlace;
            d.wcount[wid] = 0;
        }
        if (a.step_counter) add_steps(a, steps);
        return;
    }
    Ray r{};
    r.n = -1;
    if (idx < total) {
        const unsigned pk = order[idx];
        r = setup_ray(a, (int)(pk & 0xffffu), (int)(pk >> 16));
    }
    const ProcParams& p = a.proc;
    const unsigned long long lt = (1ull << lane) - 1ull;
    uint4* rec = d.rec + rb;
    float4* ent = d.ent + eb;
    float P0 = r.pxy.x, P1 = r.pxy.y, P2 = r.pz;
    float acc = 0.0f, tv = 1.0f;
    int i = 0;
    bool act = r.n > 0;
    unsigned cells = 0, s = 0, b = 0;   // b: entries the wave appended so far (wave-uniform)
    const DensityK dk = density_k<TABLE>(p, a.scale);
    for (;;) {
        act = act && i < r.n;
        if (__ballot(act) == 0) break;
        float rho = 0.0f;
        if (act) rho = proc_density<TABLE, false, (VR_DEFER_UNROLL != 0)>(p, dk, wt, P0, P1, P2, cells);
        const bool need = act && rho > 0.0f;
        const unsigned long long m = __ballot(need);
        if (need) ent[b + (unsigned)__popcll(m & lt)] = make_float4(P0, P1, P2, tv * (rho * p.od));
        if (lane == 0) rec[s] = make_uint4(b, (unsigned)m, (unsigned)(m >> 32), 0u);
        b += (unsigned)__popcll(m);
        ++s;
        if (act) {
            acc = acc + rho;
            tv = spec_expf(-(acc * p.od));
            P0 = P0 + r.sxy.x; P1 = P1 + r.sxy.y; P2 = P2 + r.sz;
            ++i;
            if constexpr (EARLY) {
                if (acc > a.acc_limit) act = false;
            }
        }
    }
    if (lane == 0) {
        d.wsteps[wid] = s;
        d.wcount[wid] = b;
    }
    if (a.step_counter) add_steps(a, p.count_evals == 2 ? cells : r.n > 0 ? (unsigned)i : 0u);
}

// Exclusive prefix of the waves' chunk counts (one workgroup; waves past the
// frame's sorted total count 0) and the frame's chunk total in count[0].
constexpr int kScanThreads = 1024;
[[maybe_unused]] __global__ __launch_bounds__(kScanThreads) void proc_shadow_scan(const unsigned* __restrict__ total_ptr,
                                                                                  ShadowDefer d)
{
    __shared__ unsigned sc[kScanThreads];
    const int t = threadIdx.x;
    const unsigned nw = min((*total_ptr + 63u) / 64u, d.waves);
    const unsigned per = (nw + kScanThreads - 1) / kScanThreads;
    const unsigned w0 = min((unsigned)t * per, nw), w1 = min(w0 + per, nw);
    unsigned own = 0;
    for (unsigned w = w0; w < w1; ++w) own += (d.wcount[w] + 63u) / 64u;
    sc[t] = own;
    __syncthreads();
    for (int off = 1; off < kScanThreads; off <<= 1) {
        const unsigned v = t >= off ? sc[t - off] : 0u;
        __syncthreads();
        sc[t] += v;
        __syncthreads();
    }
    unsigned c = sc[t] - own;
    for (unsigned w = w0; w < w1; ++w) {
        d.wchunk[w] = c;
        c += (d.wcount[w] + 63u) / 64u;
    }
    if (t == kScanThreads - 1) d.count[0] = sc[t];
}

// chunk -> (wave, chunk of the wave, entries): one wave per sorted wave.
[[maybe_unused]] __global__ __launch_bounds__(kThreads) void proc_shadow_map(const unsigned* __restrict__ total_ptr,
                                                                             ShadowDefer d)
{
    const unsigned w = blockIdx.x * (kThreads / 64) + (threadIdx.x >> 6);
    const unsigned lane = threadIdx.x & 63;
    if (w >= min((*total_ptr + 63u) / 64u, d.waves)) return;
    const unsigned n = d.wcount[w], c0 = d.wchunk[w];
    const unsigned e0 = (unsigned)d.went[w];   // < ent_cap < 2^32 for a wave with entries
    for (unsigned k = lane; k * 64u < n; k += 64u) d.map[c0 + k] = make_uint4(e0 + k * 64u, 0u, min(64u, n - k * 64u), 0u);
}

// the shadow pass's density through proc_density_phased (unrolled octaves),
// held to 5 waves per SIMD: config 3 -2.3 % (profiles/r05/ab_shadow_phased.txt;
// 4 waves, uncapped at 107 VGPRs: level)
#ifndef VR_SHADOW_PHASED
#define VR_SHADOW_PHASED 1
#endif
#if VR_SHADOW_PHASED && !defined(VR_SHADOW_WAVES)
#define VR_SHADOW_WAVES 5
#endif
#ifndef VR_SHADOW_ATTR
#ifdef VR_SHADOW_WAVES   // timing experiments: the shadow pass built for this many waves per SIMD
#define VR_SHADOW_ATTR __attribute__((amdgpu_waves_per_eu(VR_SHADOW_WAVES)))
#else
#define VR_SHADOW_ATTR
#endif
#endif
template <int TABLE, bool WC>
__global__ __launch_bounds__(kThreads) VR_SHADOW_ATTR void proc_shadow_eval(const MarchArgs a, ShadowDefer d)
{
    noise::WorleyCube wc;   // WC: the lane's Worley cube, kept across its samples (and entries)
    extern __shared__ float4 wt_lds[];
    const float4* wt = worley_table<TABLE>(a.proc, wt_lds);
    const ProcParams& p = a.proc;
    const unsigned chunks = *d.count;
    const int S = p.shadow_steps;
    const unsigned lane = threadIdx.x & 63;
    const float l0 = noise::in_vgpr(p.lstep[0]), l1 = noise::in_vgpr(p.lstep[1]), l2 = noise::in_vgpr(p.lstep[2]);
    unsigned evals = 0, cells = 0;
    for (unsigned c = blockIdx.x * (kThreads / 64) + (threadIdx.x >> 6); c < chunks; c += gridDim.x * (kThreads / 64)) {
        const uint4 mc = d.map[c];   // wave-uniform
#if defined(VR_COUNT_SLOTS) && VR_COUNT_SLOTS == 2
        if (lane == 0) evals += 64u * (unsigned)S;   // lane-slots of the chunk (timing experiment)
#endif
        if (lane >= mc.z) continue;
#if defined(VR_COUNT_SLOTS) && VR_COUNT_SLOTS == 1
        evals += (unsigned)S;   // slots of the entry (timing experiment)
#endif
        float4* e = d.ent + mc.x + lane;
        const float4 en = *e;
        float q0 = en.x, q1 = en.y, q2 = en.z, sl = 0.0f;
        for (int j = 0; j < S; ++j) {
            q0 = q0 + l0; q1 = q1 + l1; q2 = q2 + l2;
            // march_pixel_proc's box test as min3 / max3 (q is never NaN)
            if (fminf(fminf(q0, q1), q2) >= 0.0f && fmaxf(fmaxf(q0, q1), q2) <= 1.0f) {
                // the operands pinned per sample, as before round 5: hoisted out
                // of the loops they take the pass from 75 to 86 VGPRs (6 -> 5
                // waves per SIMD) and it ran 0.4 % slower (profiles/r05)
                const DensityK dk = density_k<TABLE>(p, a.scale);
                sl = sl + proc_density<TABLE, WC, (VR_SHADOW_PHASED != 0)>(p, dk, wt, q0, q1, q2, cells, &wc);
#ifndef VR_COUNT_SLOTS
                ++evals;
#endif
            }
        }
        const float tl = spec_expf(-(sl * p.od));
        *reinterpret_cast<float2*>(e) = make_float2(en.w, tl);
    }
    if (a.step_counter) add_steps(a, p.count_evals == 2 ? cells : p.count_evals ? evals : 0u);
}

// The shadow pass with 8 lanes per entry (option shadow_cache = 2): lane j of
// an entry's group of 8 evaluates the sun samples j, j + 8, ... of its ray
// (reached by the same sequential adds, P + (s+1) L), and the group sums them
// in sample order through __shfl, so sl is the per-lane loop's, bit for bit
// (an out-of-box sample adds +0, which leaves sl >= +0 unchanged).  The 8
// lanes of a group sample one sun ray a few texels apart, so their Worley
// cube and Perlin corners mostly coincide: their LDS table reads broadcast
// instead of spreading over 64 rays' cells (bank conflicts, verdict r03 #5).
template <int TABLE>
__global__ __launch_bounds__(kThreads) void proc_shadow_eval8(const MarchArgs a, ShadowDefer d)
{
    extern __shared__ float4 wt_lds[];
    const float4* wt = worley_table<TABLE>(a.proc, wt_lds);
    const ProcParams& p = a.proc;
    const unsigned units = *d.count * 8u;   // 8 entries per unit
    const int S = p.shadow_steps;
    const unsigned lane = threadIdx.x & 63, g = lane >> 3, j = lane & 7;
    const float l0 = noise::in_vgpr(p.lstep[0]), l1 = noise::in_vgpr(p.lstep[1]), l2 = noise::in_vgpr(p.lstep[2]);
    unsigned evals = 0, cells = 0;
    const DensityK dk = density_k<TABLE>(p, a.scale);
    for (unsigned u = blockIdx.x * (kThreads / 64) + (threadIdx.x >> 6); u < units; u += gridDim.x * (kThreads / 64)) {
        const uint4 mc = d.map[u >> 3];   // wave-uniform
        const unsigned k = (u & 7u) * 8u + g;   // the group's entry within the chunk
        const bool has = k < mc.z;
        float4* e = d.ent + mc.x + k;
        float4 en = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
        if (has) en = *e;
        float q0 = en.x, q1 = en.y, q2 = en.z, sl = 0.0f;
        for (unsigned t = 0; t <= j; ++t) { q0 = q0 + l0; q1 = q1 + l1; q2 = q2 + l2; }   // sample j
        for (int r = 0; r < S; r += 8) {
            float v = 0.0f;
            // march_pixel_proc's box test as min3 / max3 (q is never NaN)
            if (has && r + (int)j < S && fminf(fminf(q0, q1), q2) >= 0.0f && fmaxf(fmaxf(q0, q1), q2) <= 1.0f) {
                v = proc_density<TABLE>(p, dk, wt, q0, q1, q2, cells);
                ++evals;
            }
#pragma unroll
            for (int t = 0; t < 8; ++t) {   // the group's samples r .. r + 7, in order
                const float vt = __shfl(v, (int)(g * 8u) + t);
                if (r + t < S) sl = sl + vt;
            }
            for (int t = 0; t < 8; ++t) { q0 = q0 + l0; q1 = q1 + l1; q2 = q2 + l2; }   // sample j + r + 8
        }
        if (has && j == 0) *reinterpret_cast<float2*>(e) = make_float2(en.w, spec_expf(-(sl * p.od)));
    }
    if (a.step_counter) add_steps(a, p.count_evals == 2 ? cells : p.count_evals ? evals : 0u);
}

// Steps folded per batch in the resolve pass: lanes 0..31 load the batch's
// step records with one vector load, v_readlane hands each record to the
// wave, and every lane issues its entry loads back to back (the fold itself is
// a serial fma chain; the loads are independent): two round trips per batch.
constexpr int kResolveBatch = 32;
[[maybe_unused]] __global__ __launch_bounds__(kThreads) void proc_shadow_resolve(const MarchArgs a, const unsigned* __restrict__ order,
                                                                const unsigned* __restrict__ total_ptr, ShadowDefer d)
{
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const unsigned total = *total_ptr;
    const unsigned wid = __builtin_amdgcn_readfirstlane(blockIdx.x * (kThreads / 64) + wave);
    const unsigned base = wid * 64u;
    if (base >= total) return;
    const unsigned ns = d.wsteps[wid];
    if (ns == kDeferInPlace) return;   // the primary pass stored this wave's pixels
    const unsigned long long lt = (1ull << lane) - 1ull;
    const uint4* rec = d.rec + d.wrec[wid];
    const float4* ent = d.ent + d.went[wid];
    float rad = 0.0f;
    for (unsigned s0 = 0; s0 < ns; s0 += kResolveBatch) {
        uint4 rc = make_uint4(0u, 0u, 0u, 0u);
        if (lane < kResolveBatch && s0 + lane < ns) rc = rec[s0 + lane];
        float2 v[kResolveBatch];
        bool h[kResolveBatch];
#pragma unroll
        for (int k = 0; k < kResolveBatch; ++k) {
            // (readlane returns int: widen the low word unsigned, not sign-extended)
            const unsigned bk = (unsigned)__builtin_amdgcn_readlane(rc.x, k);
            const unsigned long long m = ((unsigned long long)(unsigned)__builtin_amdgcn_readlane(rc.z, k) << 32) |
                                         (unsigned long long)(unsigned)__builtin_amdgcn_readlane(rc.y, k);
            h[k] = (m >> lane) & 1ull;
            v[k] = make_float2(0.0f, 0.0f);
            if (h[k]) v[k] = *reinterpret_cast<const float2*>(ent + bk + (unsigned)__popcll(m & lt));
        }
#pragma unroll
        for (int k = 0; k < kResolveBatch; ++k)
            if (h[k]) rad = fmaf(v[k].x, v[k].y, rad);
    }
    const unsigned idx = base + lane;
    if (idx < total) {
        const unsigned pk = order[idx];
        const int x = (int)(pk & 0xffffu), orow = (int)(pk >> 16);
        const Ray r = setup_ray(a, x, orow);
        if (r.live) store_pixel(a, x, orow, r.n >= 0, rad);
    }
}

template <int L, int W>
hipError_t launch_lw(const MarchArgs& a, bool early, const Schedule& sc, hipStream_t s)
{
    const size_t lds = L == LAYOUT_PLANAR || L == LAYOUT_CORNERH ? 0
                     : (size_t)(a.nx + a.ny + a.nz + 3) * sizeof(unsigned) * (L == LAYOUT_COL48Z ? 2 : 1);
    const dim3 block(kThreads);
#if VR_EXPERIMENTS
    if (sc.kind == SCHED_STRIDED) {
        const int tiles = ((a.width + 7) >> 3) * ((a.out_rows + 7) >> 3);
        const int tpw = sc.tiles_per_wave > 0 ? sc.tiles_per_wave : 1;
        const int nw = (tiles + tpw - 1) / tpw;
        const dim3 grid((nw + 3) / 4);
        if (early)
            hipLaunchKernelGGL((march_strided<L, W, true>), grid, block, lds, s, a, 4 * (int)grid.x);
        else
            hipLaunchKernelGGL((march_strided<L, W, false>), grid, block, lds, s, a, 4 * (int)grid.x);
        return hipGetLastError();
    }
#endif
    if (sc.kind == SCHED_RINGS) {
        const int tiles_x8 = (a.width + 7) >> 3, rows8 = (a.out_rows + 7) >> 3;
        const int cx = min(max(sc.center_x >> 3, 0), tiles_x8 - 1), cy = min(max(sc.center_y >> 3, 0), rows8 - 1);
        const int R = max(max(cx, tiles_x8 - 1 - cx), max(cy, rows8 - 1 - cy));
        const int npos = (2 * R + 1) * (2 * R + 1);
        const int tpw = sc.tiles_per_wave > 0 ? sc.tiles_per_wave : 1;
        const dim3 grid((unsigned)(((npos + tpw - 1) / tpw + 3) / 4));
        const int nw = 4 * (int)grid.x;
        if (early && a.zero_offsets)
            hipLaunchKernelGGL((march_rings<L, W, true, true>), grid, block, lds, s, a, cx, cy, nw, npos);
        else if (early)
            hipLaunchKernelGGL((march_rings<L, W, true, false>), grid, block, lds, s, a, cx, cy, nw, npos);
        else if (a.zero_offsets)
            hipLaunchKernelGGL((march_rings<L, W, false, true>), grid, block, lds, s, a, cx, cy, nw, npos);
        else
            hipLaunchKernelGGL((march_rings<L, W, false, false>), grid, block, lds, s, a, cx, cy, nw, npos);
        return hipGetLastError();
    }
    if constexpr (is_b4_family(L) || L == LAYOUT_ZPAIR || L == LAYOUT_CORNER8 || L == LAYOUT_CORNERH ||
                  L == LAYOUT_COL48Z) {
        if (sc.kind == SCHED_REGIONS && sc.split > 1) {
            const dim3 grid((unsigned)(8 * ((sc.map.nwx + 3) / 4)));
            if (sc.split == 2) launch_regions_split<L, 2>(a, early, sc, grid, lds, s);
            else if (sc.split == 4) launch_regions_split<L, 4>(a, early, sc, grid, lds, s);
            else launch_regions_split<L, 8>(a, early, sc, grid, lds, s);
            return hipGetLastError();
        }
    }
#if VR_EXPERIMENTS
    if constexpr (L == LAYOUT_COL48 || L == LAYOUT_BRICK4832 || L == LAYOUT_CORNERH) {
        if (sc.kind == SCHED_REGIONS && (sc.wg_waves == 8 || sc.wg_waves == 16)) {
            const int g = sc.wg_waves;
            const dim3 grid((unsigned)(8 * ((sc.map.nwx + g - 1) / g))), blk(64 * g);
#define VR_RW(G) \
    if (early && a.zero_offsets) hipLaunchKernelGGL((march_regions<L, W, true, true, G>), grid, blk, lds, s, a, sc.tiles, sc.hdr, sc.map.nwx); \
    else if (early) hipLaunchKernelGGL((march_regions<L, W, true, false, G>), grid, blk, lds, s, a, sc.tiles, sc.hdr, sc.map.nwx); \
    else if (a.zero_offsets) hipLaunchKernelGGL((march_regions<L, W, false, true, G>), grid, blk, lds, s, a, sc.tiles, sc.hdr, sc.map.nwx); \
    else hipLaunchKernelGGL((march_regions<L, W, false, false, G>), grid, blk, lds, s, a, sc.tiles, sc.hdr, sc.map.nwx)
            if (g == 8) { VR_RW(8); } else { VR_RW(16); }
#undef VR_RW
            return hipGetLastError();
        }
    }
#endif
    if constexpr (L == LAYOUT_COL48 || L == LAYOUT_BRICK4832 || L == LAYOUT_CORNERH || L == LAYOUT_COL48Z) {
        // one uniform channel (the reference recipe's G, TestMain.cpp:60/76):
        // its loads are skipped; other masks run the general kernel (exact too)
        const int um = a.umask;
        if (sc.kind == SCHED_REGIONS && !early && a.zero_offsets && (um == 1 || um == 2 || um == 4 || um == 8)) {
            const dim3 grid((unsigned)(8 * ((sc.map.nwx + 3) / 4)));
#define VR_UM(U) hipLaunchKernelGGL((march_regions_u<L, W, false, true, U>), grid, block, lds, s, a, sc.tiles, sc.hdr, sc.map.nwx)
            if (um == 1) VR_UM(1);
            else if (um == 2) VR_UM(2);
            else if (um == 4) VR_UM(4);
            else VR_UM(8);
#undef VR_UM
            return hipGetLastError();
        }
#ifdef VR_UM_EXPERIMENT
        if (sc.kind == SCHED_REGIONS && !early && a.zero_offsets && um == 10) {   // G and A (timing experiment)
            const dim3 grid((unsigned)(8 * ((sc.map.nwx + 3) / 4)));
            hipLaunchKernelGGL((march_regions_u<L, W, false, true, 10>), grid, block, lds, s, a, sc.tiles, sc.hdr, sc.map.nwx);
            return hipGetLastError();
        }
#endif
    }
    if (sc.kind == SCHED_REGIONS) {
        const dim3 grid((unsigned)(8 * ((sc.map.nwx + 3) / 4)));
        if (early && a.zero_offsets)
            hipLaunchKernelGGL((march_regions<L, W, true, true>), grid, block, lds, s, a, sc.tiles, sc.hdr, sc.map.nwx);
        else if (early)
            hipLaunchKernelGGL((march_regions<L, W, true, false>), grid, block, lds, s, a, sc.tiles, sc.hdr, sc.map.nwx);
        else if (a.zero_offsets)
            hipLaunchKernelGGL((march_regions<L, W, false, true>), grid, block, lds, s, a, sc.tiles, sc.hdr, sc.map.nwx);
        else
            hipLaunchKernelGGL((march_regions<L, W, false, false>), grid, block, lds, s, a, sc.tiles, sc.hdr, sc.map.nwx);
        return hipGetLastError();
    }
#if VR_EXPERIMENTS
    if (sc.kind == SCHED_XCDROWS) {
        const int groups = (((a.width + 7) >> 3) + 3) >> 2, rows8 = (a.out_rows + 7) >> 3;
        const dim3 grid(8 * ((rows8 + 7) / 8) * groups);
        if (early)
            hipLaunchKernelGGL((march_xcdrows<L, W, true>), grid, block, lds, s, a);
        else
            hipLaunchKernelGGL((march_xcdrows<L, W, false>), grid, block, lds, s, a);
        return hipGetLastError();
    }
    if (sc.kind == SCHED_QUEUE) {
        hipError_t e = hipMemsetAsync(sc.heads, 0, 32, s);
        if (e != hipSuccess) return e;
        const dim3 grid(256 * sc.waves_per_simd);
        if (early)
            hipLaunchKernelGGL((march_queue<L, W, true>), grid, block, lds, s, a, sc.heads);
        else
            hipLaunchKernelGGL((march_queue<L, W, false>), grid, block, lds, s, a, sc.heads);
        return hipGetLastError();
    }
#endif
    const dim3 grid(a.num_blocks);
    if (early)
        hipLaunchKernelGGL((march_grid<L, W, true>), grid, block, lds, s, a);
    else
        hipLaunchKernelGGL((march_grid<L, W, false>), grid, block, lds, s, a);
    return hipGetLastError();
}

}  // namespace
}  // namespace vr
