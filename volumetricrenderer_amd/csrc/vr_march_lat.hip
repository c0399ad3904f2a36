// vr_march_lat.hip -- the latency-mode grid march for small frame shares
// (multi-GPU strong scaling).
//
// Same ray setup, taps, blend and accumulation as march_pixel_split (frag.glsl:
// 36-80, the fp32 spec of DESIGN.md sec. 3): K lanes per ray, lane k marching
// steps k, k+K, k+2K, ..., reaching each of its points by the reference's own
// sequence of fp32 adds (frag.glsl:74), and the K terms of a round added to
// `acc` in step order through __shfl -- so results and step counts are bit for
// bit those of the one-lane march.
//
// What differs is the depth of the load pipeline.  With 1/8 of a 1080p frame
// per GPU the share has ~950 8x8 tiles with work: ~1 wave per SIMD even at
// K = 4, so each wave waits out its longest ray's dependent memory round trips
// (rank-0 band sets at 0.029 ms against 0.015 for 1/8 of the
// frame).  The one-lane and split marches keep one step (round) of loads in
// flight, and they finish the loaded bytes (v_alignbyte) in the iteration that
// issued them, which makes the wave wait for them there.  Here:
//   - D rounds of loads are in flight: round r + D's addresses need only the
//     ray point (sequential adds), not `acc`, so they are issued D rounds
//     before their blend;
//   - the loaded dwords stay raw until the blend of their round (TapLat), so
//     the s_waitcnt for a round lands at its blend, D - 1 rounds of other
//     loads later;
//   - the D rounds rotate through a register ring indexed at compile time (the
//     group loop is unrolled by D), under a register budget of 2 waves per
//     SIMD (amdgpu_waves_per_eu), with no scratch (checked on the code object,
//     DESIGN.md sec. 7.1).
#include "vr_march_kernels.h"

namespace vr {
namespace {

// A tap's loaded dwords before the byte alignment (b4 family: the two 8-B
// z-slice loads s0, s1 and the byte offset; CORNERH: the 16-B row pairs), and
// its weights.
struct TapLat {
    unsigned d0, d1, d2, d3, off;
    float wx, wy, wz;
};

template <int LAYOUT>
__device__ __forceinline__ TapLat lat_fetch(const FastCtx& f, int ch, float gx, float gy, float gz)
{
    TapLat r{};
    if constexpr (is_b4_family(LAYOUT)) {
        // tap_fetch's b4 loads (a slice's rows y, y+1 are the
        // two dwords at off & ~3), without the v_alignbyte_b32 that would wait
        constexpr unsigned kZ = LAYOUT == LAYOUT_BRICK41616 ? 64u
                             : LAYOUT == LAYOUT_BRICK488 || LAYOUT == LAYOUT_BRICK4816 || LAYOUT == LAYOUT_BRICK4832 ||
                                      LAYOUT == LAYOUT_BRICK4864 || LAYOUT == LAYOUT_COL48 ? 32u : 16u;
        r.wx = fract_(gx); r.wy = fract_(gy); r.wz = fract_(gz);
        const unsigned off = f.tx[cvt_flr(gx)] + f.ty[cvt_flr(gy)] + f.tz[cvt_flr(gz)];
        const unsigned a0 = off & ~3u;
        const auto s0 = __builtin_amdgcn_raw_buffer_load_b64(f.rsrc[ch], a0, 0, 0);
        const auto s1 = __builtin_amdgcn_raw_buffer_load_b64(f.rsrc[ch], a0 + kZ, 0, 0);
        r.d0 = s0[0]; r.d1 = s0[1]; r.d2 = s1[0]; r.d3 = s1[1];
        r.off = off;
    } else {
        static_assert(LAYOUT == LAYOUT_CORNERH, "latency march: b4 family or CORNERH");
        const TapRaw t = tap_fetch<LAYOUT>(f, ch, gx, gy, gz);
        r.d0 = t.q0; r.d1 = t.q1; r.d2 = t.q2; r.d3 = t.q3;
        r.wx = t.wx; r.wy = t.wy; r.wz = t.wz;
    }
    return r;
}

template <int LAYOUT>
__device__ __forceinline__ float lat_blend(const TapLat& r)
{
    TapRaw t{};
    t.wx = r.wx; t.wy = r.wy; t.wz = r.wz;
    if constexpr (is_b4_family(LAYOUT)) {
        t.q0 = __builtin_amdgcn_alignbyte(r.d1, r.d0, r.off);
        t.q1 = __builtin_amdgcn_alignbyte(r.d1, r.d1, r.off);
        t.q2 = __builtin_amdgcn_alignbyte(r.d3, r.d2, r.off);
        t.q3 = __builtin_amdgcn_alignbyte(r.d3, r.d3, r.off);
    } else {
        t.q0 = r.d0; t.q1 = r.d1; t.q2 = r.d2; t.q3 = r.d3;
    }
    return tap_blend<LAYOUT>(t);
}

// tap T of a march with uniform channels UM at ray point (pxy, pz)
template <int UM, int T, int LAYOUT, bool ZO>
__device__ __forceinline__ TapLat lat_fetch_u(const MarchArgs& a, const FastCtx& f, f2 pxy, float pz)
{
    if constexpr ((UM >> T) & 1) {
        return TapLat{};
    } else {
        const f2 Tt = ZO ? f2{0.5f, 0.5f} : f2{a.tap_T[T][0], a.tap_T[T][1]};
        const f2 gxy = __builtin_elementwise_fma(pxy, f2{a.tap_S[T][0], a.tap_S[T][1]}, Tt);
        const float gz = LAYOUT == LAYOUT_CORNERH ? fmaf(pz, f.sz[T], ZO ? 0.5f : f.oz[T])
                                                 : fmaf(pz, a.tap_S[T][2], ZO ? 0.5f : a.tap_T[T][2]);
        return lat_fetch<LAYOUT>(f, T, gxy.x, gxy.y, gz);
    }
}
template <int UM, int T, int LAYOUT>
__device__ __forceinline__ float lat_blend_u(const TapLat& c, const float* uv)
{
    if constexpr ((UM >> T) & 1) return uv[T];
    else return lat_blend<LAYOUT>(c);
}

struct LatRound {
    TapLat t[4];
};
template <int UM, int LAYOUT, bool ZO>
__device__ __forceinline__ LatRound lat_fetch_round(const MarchArgs& a, const FastCtx& f, f2 pxy, float pz)
{
    LatRound r;
    r.t[0] = lat_fetch_u<UM, 0, LAYOUT, ZO>(a, f, pxy, pz);
    r.t[1] = lat_fetch_u<UM, 1, LAYOUT, ZO>(a, f, pxy, pz);
    r.t[2] = lat_fetch_u<UM, 2, LAYOUT, ZO>(a, f, pxy, pz);
    r.t[3] = lat_fetch_u<UM, 3, LAYOUT, ZO>(a, f, pxy, pz);
    return r;
}

// One ray, K lanes (this is lane k of the ray; ray_lane = the ray's lane 0),
// D rounds of loads in flight.  Returns the executed steps (lane k = 0).
template <int LAYOUT, bool EARLY, bool ZO, int K, int D, int UM>
__device__ __forceinline__ unsigned march_pixel_lat(const MarchArgs& a, const FastCtx& f, int x, int orow, int k,
                                                    int ray_lane)
{
    constexpr int R = 64 / K;
    const Ray r = setup_ray(a, x, orow);
    float uv[4] = {};
    if constexpr (UM != 0)
        for (int t = 0; t < 4; ++t)
            if ((UM >> t) & 1) uv[t] = noise::in_vgpr(a.uval[t]);
    const float scale = LAYOUT == LAYOUT_CORNERH ? f.scale : a.scale;
    const int n = r.n;
    f2 pxy = r.pxy;
    float pz = r.pz;
    for (int j = 0; j < k; ++j) { pxy = pxy + r.sxy; pz = pz + r.sz; }   // step k: k sequential adds
    float acc = 0.0f;
    int i = 0;
    if (n > 0) {
        LatRound c[D];
        // prologue: rounds 0 .. D-1 (steps k + jK); a round past the ray's
        // last step fetches its entry point (inside the box) and is not added
#pragma unroll
        for (int j = 0; j < D; ++j) {
            const bool mine = j * K + k < n;
            c[j] = lat_fetch_round<UM, LAYOUT, ZO>(a, f, mine ? pxy : r.pxy, mine ? pz : r.pz);
            for (int q = 0; q < K; ++q) { pxy = pxy + r.sxy; pz = pz + r.sz; }
            // issue the rounds in slot order, as the loop refills them: the
            // s_waitcnt at a blend counts the loads issued after that slot's
            __builtin_amdgcn_sched_barrier(0);
        }
        // (pxy, pz) is step k + DK now
        bool stop = false;
        for (int base = 0; base < n; base += D * K) {
#pragma unroll
            for (int j = 0; j < D; ++j) {
                const int rb = base + j * K;   // this round's first step
                const float t0 = lat_blend_u<UM, 0, LAYOUT>(c[j].t[0], uv), t1 = lat_blend_u<UM, 1, LAYOUT>(c[j].t[1], uv);
                const float t2 = lat_blend_u<UM, 2, LAYOUT>(c[j].t[2], uv), t3 = lat_blend_u<UM, 3, LAYOUT>(c[j].t[3], uv);
                const float term = ((t0 * t1) * (t2 + t3)) * scale;                        // :71-73
                // refill the slot with round rb + DK, D rounds ahead of its blend
                const bool mine = rb + D * K + k < n;
                c[j] = lat_fetch_round<UM, LAYOUT, ZO>(a, f, mine ? pxy : r.pxy, mine ? pz : r.pz);
                for (int q = 0; q < K; ++q) { pxy = pxy + r.sxy; pz = pz + r.sz; }
                // the K terms of the round, in step order (frag.glsl:71-73's sequential sum)
#pragma unroll
                for (int q = 0; q < K; ++q) {
                    const float tq = K == 1 ? term : __shfl(term, ray_lane + q * R);
                    if (rb + q < n && !stop) {
                        acc = acc + tq;
                        ++i;
                        if constexpr (EARLY) stop = acc > a.acc_limit;
                    }
                }
                if constexpr (EARLY) {
                    if (stop) break;
                }
                // keep the rounds in program order: the scheduler would otherwise
                // hoist every round's blend (and its s_waitcnt) to the top of the
                // group, so the D rounds' loads would be waited for together
                __builtin_amdgcn_sched_barrier(0);
            }
            if constexpr (EARLY) {
                if (stop) break;
            }
        }
    }
    if (r.live && k == 0) {
        const float at = acc * a.step_size;                                              // :76
        store_pixel(a, x, orow, n >= 0, 1.0f - spec_expf(a.density * fminf(-at, 0.0f)));   // :79
    }
    return (n > 0 && k == 0) ? (unsigned)i : 0u;
}

#ifndef VR_LAT_WAVES
#define VR_LAT_WAVES 2   // register budget: waves per SIMD (256 VGPRs at 2)
#endif

// Regions schedule, latency mode: the units of march_regions_split (8x8 tile
// = K sub-blocks of 64/K rays; lane = k * (64/K) + ray, so 4 adjacent lanes
// are a 2x2 pixel quad at the same step offset), each ray marched by
// march_pixel_lat.
template <int LAYOUT, bool EARLY, bool ZO, int K, int D, int UM>
__global__ __launch_bounds__(kThreads) __attribute__((amdgpu_waves_per_eu(1, VR_LAT_WAVES))) void march_regions_lat(
    const MarchArgs a, const unsigned* __restrict__ tiles, const int* __restrict__ hdr, int nwx)
{
    constexpr int R = 64 / K, SW = K >= 4 ? 4 : 8, SH = R / SW, NSX = 8 / SW;
    extern __shared__ __attribute__((aligned(16))) unsigned lds[];
    const int xcd = blockIdx.x & 7;
    const int w = (int)(blockIdx.x >> 3) * (kThreads / 64) + (threadIdx.x >> 6);
    const int begin = hdr[xcd], units = (hdr[xcd + 1] - begin) * K;
    if ((int)(blockIdx.x >> 3) * (kThreads / 64) >= units) return;   // whole workgroup, before the barrier
    const FastCtx f = fast_prologue<LAYOUT>(a, lds);
    const int lane = threadIdx.x & 63, k = lane / R, rho = lane % R;
    const int px = ((rho >> 2) % (SW / 2)) * 2 + (rho & 1), py = ((rho >> 2) / (SW / 2)) * 2 + ((rho >> 1) & 1);
    unsigned long long steps = 0;
    for (int u = w; w < nwx && u < units; u += nwx) {
        const unsigned t = tiles[begin + u / K];
        const int s = u % K;
        const int x = (int)(t & 0xffffu) * 8 + (s % NSX) * SW + px, orow = (int)(t >> 16) * 8 + (s / NSX) * SH + py;
        steps += march_pixel_lat<LAYOUT, EARLY, ZO, K, D, UM>(a, f, x, orow, k, rho);
    }
    if (a.step_counter) add_steps(a, steps);
}

template <int L, int K, int D>
void launch_lat_kd(const MarchArgs& a, bool early, const Schedule& sc, dim3 grid, size_t lds, hipStream_t s)
{
    const dim3 block(kThreads);
    const int um = a.umask;
    if (!early && a.zero_offsets && (um == 1 || um == 2 || um == 4 || um == 8)) {
#define VR_LU(U) hipLaunchKernelGGL((march_regions_lat<L, false, true, K, D, U>), grid, block, lds, s, a, sc.tiles, sc.hdr, sc.map.nwx)
        if (um == 1) VR_LU(1);
        else if (um == 2) VR_LU(2);
        else if (um == 4) VR_LU(4);
        else VR_LU(8);
#undef VR_LU
        return;
    }
    if (early && a.zero_offsets)
        hipLaunchKernelGGL((march_regions_lat<L, true, true, K, D, 0>), grid, block, lds, s, a, sc.tiles, sc.hdr, sc.map.nwx);
    else if (early)
        hipLaunchKernelGGL((march_regions_lat<L, true, false, K, D, 0>), grid, block, lds, s, a, sc.tiles, sc.hdr, sc.map.nwx);
    else if (a.zero_offsets)
        hipLaunchKernelGGL((march_regions_lat<L, false, true, K, D, 0>), grid, block, lds, s, a, sc.tiles, sc.hdr, sc.map.nwx);
    else
        hipLaunchKernelGGL((march_regions_lat<L, false, false, K, D, 0>), grid, block, lds, s, a, sc.tiles, sc.hdr, sc.map.nwx);
}

template <int L, int K>
void launch_lat_k(const MarchArgs& a, bool early, const Schedule& sc, dim3 grid, size_t lds, hipStream_t s)
{
    if (sc.lat == 2) launch_lat_kd<L, K, 2>(a, early, sc, grid, lds, s);
    else if (sc.lat == 4) launch_lat_kd<L, K, 4>(a, early, sc, grid, lds, s);
    else launch_lat_kd<L, K, 3>(a, early, sc, grid, lds, s);
}

template <int L>
hipError_t launch_lat_l(const MarchArgs& a, bool early, const Schedule& sc, hipStream_t s)
{
    const size_t lds = L == LAYOUT_CORNERH ? 0 : (size_t)(a.nx + a.ny + a.nz + 3) * sizeof(unsigned);
    const int K = sc.split > 1 ? sc.split : 1;
    const dim3 grid((unsigned)(8 * ((sc.map.nwx + 3) / 4)));
    if (K == 1) launch_lat_k<L, 1>(a, early, sc, grid, lds, s);
    else if (K == 2) launch_lat_k<L, 2>(a, early, sc, grid, lds, s);
    else if (K == 4) launch_lat_k<L, 4>(a, early, sc, grid, lds, s);
    else launch_lat_k<L, 8>(a, early, sc, grid, lds, s);
    return hipGetLastError();
}

}  // namespace

bool lat_supported(int layout) { return layout == LAYOUT_COL48 || layout == LAYOUT_BRICK4832 || layout == LAYOUT_CORNERH; }

hipError_t launch_march_lat(const MarchArgs& a, int layout, bool early, const Schedule& sc, hipStream_t s)
{
    if (a.width <= 0 || a.out_rows <= 0) return hipSuccess;
    switch (layout) {
    case LAYOUT_COL48: return launch_lat_l<LAYOUT_COL48>(a, early, sc, s);
    case LAYOUT_BRICK4832: return launch_lat_l<LAYOUT_BRICK4832>(a, early, sc, s);
    case LAYOUT_CORNERH: return launch_lat_l<LAYOUT_CORNERH>(a, early, sc, s);
    default: return hipErrorInvalidValue;
    }
}

}  // namespace vr
