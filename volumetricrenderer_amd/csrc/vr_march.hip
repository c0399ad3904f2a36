// vr_march.hip -- the hot path: per-pixel volumetric ray march for gfx950.
//
// Replaces shaders/frag.glsl:34-81 (and the coverage that vert.glsl:17-22
// plus rasterisation provide).  Each lane traces one ray; a wave64 owns an
// 8x8 pixel tile; a 256-thread workgroup owns a 16x16 tile.  There is no LDS
// and no barrier: neighbouring rays share the volume through L1/L2.  Work is
// ALU/gather-bound, so nothing here uses MFMA.
//
// The op sequence is the fp32 spec of DESIGN.md sec. 3.  The oracle
// (oracle/vr_oracle.c) restates the same spec, and results agree bit for bit.
// Build with -ffp-contract=off: the only fused ops are the explicit fmaf().
#include "vr_internal.h"

namespace vr {
namespace {

constexpr int kTile = 16;           // workgroup tile edge, pixels
constexpr int kThreads = 256;       // 4 waves, each an 8x8 sub-tile

__device__ __forceinline__ float lerp_(float a, float b, float t) { return fmaf(t, b - a, a); }
__device__ __forceinline__ int clampi(int v, int lo, int hi) { return min(max(v, lo), hi); }
// clamp to [0, hi] in one v_med3_i32
__device__ __forceinline__ int clamp0(int v, int hi)
{
    int r;
    asm("v_med3_i32 %0, %1, 0, %2" : "=v"(r) : "v"(v), "v"(hi));
    return r;
}

// unaligned u16 load at a 32-bit byte offset from a wave-uniform base
// (gfx950 runs in unaligned-access mode; one global_load_ushort)
__device__ __forceinline__ unsigned ld_u16(const uint8_t* __restrict__ base, unsigned off)
{
    uint16_t v;
    __builtin_memcpy(&v, base + off, 2);
    return v;
}

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

// byte k of a dword as float (v_cvt_f32_ubyteK)
template <int K>
__device__ __forceinline__ float ubyte(unsigned v) { return (float)((v >> (8 * K)) & 0xffu); }

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

// One trilinear tap of one channel: Vulkan LINEAR filter, LOD 0, at padded
// texel coordinate g = u*N - 0.5 + 1.  floor(g) is the padded base texel,
// fract(g) the weight.  Then 8 texels and 7 lerps.
template <int LAYOUT, int WRAP>
__device__ __forceinline__ float tap(const uint8_t* __restrict__ pl, const MarchArgs& a,
                                     float gx, float gy, float gz)
{
    const float ax = fract_(gx), ay = fract_(gy), az = fract_(gz);
    const int px = cvt_flr(gx), py = cvt_flr(gy), pz = cvt_flr(gz);
    float c000, c100, c010, c110, c001, c101, c011, c111;
    if constexpr (LAYOUT != LAYOUT_PLANAR) {
        // padded base position, clamped to [0, N]
        const int a0 = clamp0(px, a.nx), b0 = clamp0(py, a.ny), c0 = clamp0(pz, a.nz);
        if constexpr (LAYOUT == LAYOUT_PAD16) {
            const unsigned off = __umul24((unsigned)c0, (unsigned)a.pslice) + __umul24((unsigned)b0, (unsigned)a.prow) + (unsigned)a0;
            const unsigned v00 = ld_u16(pl, off), v10 = ld_u16(pl, off + a.prow);
            const unsigned v01 = ld_u16(pl, off + a.pslice), v11 = ld_u16(pl, off + a.pslice + a.prow);
            c000 = (float)(v00 & 0xffu); c100 = (float)(v00 >> 8);
            c010 = (float)(v10 & 0xffu); c110 = (float)(v10 >> 8);
            c001 = (float)(v01 & 0xffu); c101 = (float)(v01 >> 8);
            c011 = (float)(v11 & 0xffu); c111 = (float)(v11 >> 8);
        } else if constexpr (LAYOUT == LAYOUT_BRICK5) {
            // 5x5x5 bytes of brick (a0>>2, b0>>2, c0>>2) hold the whole footprint
            const unsigned brick = __umul24(__umul24((unsigned)(c0 >> 2), (unsigned)a.nby) + (unsigned)(b0 >> 2),
                                            (unsigned)a.nbx) + (unsigned)(a0 >> 2);
            const unsigned off = (brick << 7) + (unsigned)((c0 & 3) * 25 + (b0 & 3) * 5 + (a0 & 3));
            const unsigned v00 = ld_u16(pl, off), v10 = ld_u16(pl, off + 5);
            const unsigned v01 = ld_u16(pl, off + 25), v11 = ld_u16(pl, off + 30);
            c000 = (float)(v00 & 0xffu); c100 = (float)(v00 >> 8);
            c010 = (float)(v10 & 0xffu); c110 = (float)(v10 >> 8);
            c001 = (float)(v01 & 0xffu); c101 = (float)(v01 >> 8);
            c011 = (float)(v11 & 0xffu); c111 = (float)(v11 >> 8);
        } else if constexpr (LAYOUT == LAYOUT_CORNER8) {
            const unsigned brick = __umul24(__umul24((unsigned)(c0 >> 2), (unsigned)a.nby) + (unsigned)(b0 >> 2),
                                            (unsigned)a.nbx) + (unsigned)(a0 >> 2);
            const unsigned off = (brick << 9) + ((unsigned)(((c0 & 3) << 4) + ((b0 & 3) << 2) + (a0 & 3)) << 3);
            const uint2 q = *reinterpret_cast<const uint2*>(pl + off);
            c000 = ubyte<0>(q.x); c100 = ubyte<1>(q.x);
            c010 = ubyte<2>(q.x); c110 = ubyte<3>(q.x);
            c001 = ubyte<0>(q.y); c101 = ubyte<1>(q.y);
            c011 = ubyte<2>(q.y); c111 = ubyte<3>(q.y);
        } else {  // LAYOUT_QUAD: 4x4x5 positions x 4 B per brick; z0 quad then z1 quad at +64 B
            const unsigned brick = __umul24(__umul24((unsigned)(c0 >> 2), (unsigned)a.nby) + (unsigned)(b0 >> 2),
                                            (unsigned)a.nbx) + (unsigned)(a0 >> 2);
            const unsigned off = __umul24(brick, 320u) + ((unsigned)(((c0 & 3) << 4) + ((b0 & 3) << 2) + (a0 & 3)) << 2);
            const unsigned q0 = *reinterpret_cast<const unsigned*>(pl + off);
            const unsigned q1 = *reinterpret_cast<const unsigned*>(pl + off + 64);
            c000 = ubyte<0>(q0); c100 = ubyte<1>(q0);
            c010 = ubyte<2>(q0); c110 = ubyte<3>(q0);
            c001 = ubyte<0>(q1); c101 = ubyte<1>(q1);
            c011 = ubyte<2>(q1); c111 = ubyte<3>(q1);
        }
    } else {
        const int ix = px - 1, iy = py - 1, iz = pz - 1;
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
        c000 = pl[r00 + i0]; c100 = pl[r00 + i1];
        c010 = pl[r10 + i0]; c110 = pl[r10 + i1];
        c001 = pl[r01 + i0]; c101 = pl[r01 + i1];
        c011 = pl[r11 + i0]; c111 = pl[r11 + i1];
    }
    const float x00 = lerp_(c000, c100, ax), x10 = lerp_(c010, c110, ax);
    const float x01 = lerp_(c001, c101, ax), x11 = lerp_(c011, c111, ax);
    const float y0 = lerp_(x00, x10, ay), y1 = lerp_(x01, x11, ay);
    return lerp_(y0, y1, az) * (1.0f / 255.0f);
}

// One ray: ray setup (frag.glsl:36-55), the march (:57-75), the epilogue
// (:76-80) and the store.  Returns the executed steps (0 if uncovered).
template <int LAYOUT, int WRAP, bool EARLY>
__device__ __forceinline__ unsigned march_pixel(const MarchArgs& a, int x, int orow)
{
    const bool inside = x < a.width && orow < a.out_rows;
    int y = 0;
    if (inside) {
        const int bl = orow / a.band_rows;
        y = (a.band_first + bl * a.band_stride) * a.band_rows + (orow - bl * a.band_rows);
    }
    const bool live = inside && y < a.height;

    // ---- ray setup: frag.glsl:36-55 ---------------------------------------
    int n = -1;
    float P0 = 0.f, P1 = 0.f, P2 = 0.f, s0 = 0.f, s1 = 0.f, s2 = 0.f;
    if (live) {
        const float fx = (float)x + 0.5f, fy = (float)y + 0.5f;
        const float v0 = fmaf(fy, a.py[0], fmaf(fx, a.px[0], a.o[0]));
        const float v1 = fmaf(fy, a.py[1], fmaf(fx, a.px[1], a.o[1]));
        const float v2 = fmaf(fy, a.py[2], fmaf(fx, a.px[2], a.o[2]));
        const float len = sqrtf(fmaf(v2, v2, fmaf(v1, v1, v0 * v0)));
        const float d0 = v0 / len, d1 = v1 / len, d2 = v2 / len;
        // IntersectAABB, frag.glsl:18-27
        const float ta0 = (a.box_min[0] - a.org[0]) / d0, tb0 = (a.box_max[0] - a.org[0]) / d0;
        const float ta1 = (a.box_min[1] - a.org[1]) / d1, tb1 = (a.box_max[1] - a.org[1]) / d1;
        const float ta2 = (a.box_min[2] - a.org[2]) / d2, tb2 = (a.box_max[2] - a.org[2]) / d2;
        const float tn = fmaxf(fmaxf(fminf(ta0, tb0), fminf(ta1, tb1)), fminf(ta2, tb2));
        const float tf = fminf(fminf(fmaxf(ta0, tb0), fmaxf(ta1, tb1)), fmaxf(ta2, tb2));
        if (tn <= tf) {
            const float pi0 = fmaf(d0, tn, a.org[0]), pi1 = fmaf(d1, tn, a.org[1]), pi2 = fmaf(d2, tn, a.org[2]);
            const float zc = fmaf(a.r2[2], pi2, fmaf(a.r2[1], pi1, fmaf(a.r2[0], pi0, a.r2[3])));
            const float wc = fmaf(a.r3[2], pi2, fmaf(a.r3[1], pi1, fmaf(a.r3[0], pi0, a.r3[3])));
            if (wc > 0.0f && zc >= 0.0f && zc <= wc) {
                const float po0 = fmaf(d0, tf, a.org[0]), po1 = fmaf(d1, tf, a.org[1]), po2 = fmaf(d2, tf, a.org[2]);
                const float e0 = po0 - pi0, e1 = po1 - pi1, e2 = po2 - pi2;
                const float dist = sqrtf(fmaf(e2, e2, fmaf(e1, e1, e0 * e0)));
                const float q = dist / a.step_size;                                   // :46
                n = q >= (float)a.max_steps ? a.max_steps : (int)q;
                P0 = (pi0 - a.box_min[0]) / a.box_range[0];                           // :49-54
                P1 = (pi1 - a.box_min[1]) / a.box_range[1];
                P2 = (pi2 - a.box_min[2]) / a.box_range[2];
                s0 = (a.step_size * d0) / a.box_range[0];                             // :45
                s1 = (a.step_size * d1) / a.box_range[1];
                s2 = (a.step_size * d2) / a.box_range[2];
            }
        }
    }

    // ---- the hot loop: frag.glsl:57-75 ------------------------------------
    const uint8_t* __restrict__ pl0 = a.vol;
    const uint8_t* __restrict__ pl1 = a.vol + a.plane_stride;
    const uint8_t* __restrict__ pl2 = a.vol + 2 * a.plane_stride;
    const uint8_t* __restrict__ pl3 = a.vol + 3 * a.plane_stride;
    float acc = 0.0f;
    int i = 0;
    for (; i < n; ++i) {
        const float t0 = tap<LAYOUT, WRAP>(pl0, a, fmaf(P0, a.tap_S[0][0], a.tap_T[0][0]),
                                           fmaf(P1, a.tap_S[0][1], a.tap_T[0][1]),
                                           fmaf(P2, a.tap_S[0][2], a.tap_T[0][2]));
        const float t1 = tap<LAYOUT, WRAP>(pl1, a, fmaf(P0, a.tap_S[1][0], a.tap_T[1][0]),
                                           fmaf(P1, a.tap_S[1][1], a.tap_T[1][1]),
                                           fmaf(P2, a.tap_S[1][2], a.tap_T[1][2]));
        const float t2 = tap<LAYOUT, WRAP>(pl2, a, fmaf(P0, a.tap_S[2][0], a.tap_T[2][0]),
                                           fmaf(P1, a.tap_S[2][1], a.tap_T[2][1]),
                                           fmaf(P2, a.tap_S[2][2], a.tap_T[2][2]));
        const float t3 = tap<LAYOUT, WRAP>(pl3, a, fmaf(P0, a.tap_S[3][0], a.tap_T[3][0]),
                                           fmaf(P1, a.tap_S[3][1], a.tap_T[3][1]),
                                           fmaf(P2, a.tap_S[3][2], a.tap_T[3][2]));
        acc = acc + ((t0 * t1) * (t2 + t3)) * a.scale;                               // :71-73
        P0 = P0 + s0; P1 = P1 + s1; P2 = P2 + s2;                                     // :74
        if constexpr (EARLY) {
            if (acc > a.acc_limit) { ++i; break; }
        }
    }

    // ---- epilogue: frag.glsl:76-80 + the render-target format --------------
    if (live) {
        float g = 0.0f;
        if (n >= 0) {
            const float at = acc * a.step_size;
            const float e = spec_expf(a.density * fminf(-at, 0.0f));
            g = 1.0f - e;
        }
        char* row = (char*)a.out + (long long)orow * a.pitch;
        if (a.format == 0) {
            reinterpret_cast<float4*>(row)[x] = make_float4(g, g, g, 1.0f);
        } else {
            unsigned int q = 0;
            if (n >= 0) {
                float c = fminf(fmaxf(g, 0.0f), 1.0f);
                if (a.format == 2)
                    c = c <= 0.0031308f ? c * 12.92f : fmaf(1.055f, powf(c, 1.0f / 2.4f), -0.055f);
                q = (unsigned int)rintf(c * 255.0f);
            }
            reinterpret_cast<unsigned int*>(row)[x] = q | (q << 8) | (q << 16) | 0xff000000u;
        }
    }
    return n > 0 ? (unsigned)i : 0u;
}

__device__ __forceinline__ void add_steps(const MarchArgs& a, unsigned long long cnt)
{
    for (int off = 32; off > 0; off >>= 1) cnt += __shfl_xor(cnt, off);
    if ((threadIdx.x & 63) == 0 && cnt) atomicAdd(a.step_counter, cnt);
}

// Static schedule: one 16x16 tile per workgroup, one 8x8 sub-tile per wave.
template <int LAYOUT, int WRAP, bool EARLY>
__global__ __launch_bounds__(kThreads) void march_grid(const MarchArgs a)
{
    // Tile rows are dealt to XCDs round-robin: XCD x (= blockIdx % 8 under
    // the observed dispatch, a speed-only assumption) walks tile rows
    // x, x+8, ...  Work is balanced (the silhouette is centred) and
    // horizontally adjacent tiles share one L2.
    const int xcd = blockIdx.x & 7, j = blockIdx.x >> 3;
    const int k = j / a.tiles_x, tx = j - k * a.tiles_x;
    const int ty = xcd + 8 * k;
    if (ty >= a.tiles_y) return;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int x = tx * kTile + (wave & 1) * 8 + (lane & 7);
    const int orow = ty * kTile + (wave >> 1) * 8 + (lane >> 3);
    const unsigned steps = march_pixel<LAYOUT, WRAP, EARLY>(a, x, orow);
    if (a.step_counter) add_steps(a, steps);
}

// Dynamic schedule: persistent waves pull 8x8 tiles from 8 queues, one per
// XCD group (blockIdx % 8, speed-only).  Queue q owns the 16-row tile pairs
// p = q, q+8, ..., walked column by column.  heads[] is zeroed by a memset
// before every launch.  Every wave leaves once its queue is drained, so the
// grid always completes.
template <int LAYOUT, int WRAP, bool EARLY>
__global__ __launch_bounds__(kThreads) void march_queue(const MarchArgs a, int* __restrict__ heads)
{
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
        steps += march_pixel<LAYOUT, WRAP, EARLY>(a, tx * 8 + (lane & 7), row8 * 8 + (lane >> 3));
    }
    if (a.step_counter) add_steps(a, steps);
}

// Strided static schedule: wave g (of nw) renders 8x8 tiles g, g + nw,
// g + 2nw, ... of the row-major tile grid.  Its T = ceil(ntiles / nw) tiles
// sit 1/T of the image apart, so every wave mixes silhouette centre and edge.
// Per-wave (and per-SIMD) work evens out without atomics.
template <int LAYOUT, int WRAP, bool EARLY>
__global__ __launch_bounds__(kThreads) void march_strided(const MarchArgs a, int nw)
{
    const int lane = threadIdx.x & 63;
    const int g = blockIdx.x * (kThreads / 64) + (threadIdx.x >> 6);
    const int tiles_x8 = (a.width + 7) >> 3, rows8 = (a.out_rows + 7) >> 3;
    const int ntiles = tiles_x8 * rows8;
    unsigned long long steps = 0;
    for (int t = g; t < ntiles; t += nw) {
        const int ty = t / tiles_x8, tx = t - ty * tiles_x8;
        steps += march_pixel<LAYOUT, WRAP, EARLY>(a, tx * 8 + (lane & 7), ty * 8 + (lane >> 3));
    }
    if (a.step_counter) add_steps(a, steps);
}

template <int L, int W>
hipError_t launch_lw(const MarchArgs& a, bool early, const Schedule& sc, hipStream_t s)
{
    if (sc.strided) {
        const int tiles = ((a.width + 7) >> 3) * ((a.out_rows + 7) >> 3);
        const int nw = (tiles + sc.tiles_per_wave - 1) / sc.tiles_per_wave;
        dim3 grid((nw + 3) / 4), block(kThreads);
        if (early)
            hipLaunchKernelGGL((march_strided<L, W, true>), grid, block, 0, s, a, 4 * (int)grid.x);
        else
            hipLaunchKernelGGL((march_strided<L, W, false>), grid, block, 0, s, a, 4 * (int)grid.x);
        return hipGetLastError();
    }
    if (sc.queue) {
        hipError_t e = hipMemsetAsync(sc.heads, 0, 32, s);
        if (e != hipSuccess) return e;
        dim3 grid(256 * sc.waves_per_simd), block(kThreads);
        if (early)
            hipLaunchKernelGGL((march_queue<L, W, true>), grid, block, 0, s, a, sc.heads);
        else
            hipLaunchKernelGGL((march_queue<L, W, false>), grid, block, 0, s, a, sc.heads);
        return hipGetLastError();
    }
    dim3 grid(a.num_blocks), block(kThreads);
    if (early)
        hipLaunchKernelGGL((march_grid<L, W, true>), grid, block, 0, s, a);
    else
        hipLaunchKernelGGL((march_grid<L, W, false>), grid, block, 0, s, a);
    return hipGetLastError();
}

}  // namespace

hipError_t launch_march(const MarchArgs& a, int layout, int wrap, bool early, const Schedule& sc, hipStream_t s)
{
    if (a.num_blocks <= 0) return hipSuccess;
    if (layout == LAYOUT_PAD16) return launch_lw<LAYOUT_PAD16, WRAP_CLAMP>(a, early, sc, s);
    if (layout == LAYOUT_BRICK5) return launch_lw<LAYOUT_BRICK5, WRAP_CLAMP>(a, early, sc, s);
    if (layout == LAYOUT_CORNER8) return launch_lw<LAYOUT_CORNER8, WRAP_CLAMP>(a, early, sc, s);
    if (layout == LAYOUT_QUAD) return launch_lw<LAYOUT_QUAD, WRAP_CLAMP>(a, early, sc, s);
    if (wrap == WRAP_CLAMP) return launch_lw<LAYOUT_PLANAR, WRAP_CLAMP>(a, early, sc, s);
    return launch_lw<LAYOUT_PLANAR, WRAP_MIRROR>(a, early, sc, s);
}

}  // namespace vr
