// vr_march_slab.hip -- the LDS-slab variant of the grid march (BASELINE
// north star: "per-tile density slabs staged in LDS").
//
// Same ray setup, taps, blend and accumulation as march_pixel (frag.glsl:
// 36-80, the fp32 spec of DESIGN.md sec. 3), on the COL48 layout: each
// channel plane is a grid of columns of 4 x 8 texels (3 x 7 padded
// positions) through the whole z extent, one 32-B slice per z position, so a
// run of slices of one column is contiguous.
//
// Per step, a wave (one 8x8 tile) takes the bounding box of its live rays'
// points -- six DPP wave reductions of P; the tap coordinate fma(P, S, T) is
// monotone in P, so the box maps to every channel's box of padded positions
// -- and, per channel, fills the columns x 64-B chunks (two slices) that box
// covers into its LDS slab: 16-B loads, four lanes per chunk, so one L1
// lookup per chunk, packed densely (nbx x nby columns of nk chunks), then
// written to LDS.  The footprint reads of the step are then ds_reads from the
// slab.  A channel whose box exceeds the slab (slab_cap chunks) reads its
// taps straight from the layout for that step, as the plain march does.
//
// The per-lane gathers of the plain march cost the L1 one tag lookup per
// quad of lanes and distinct 128-B line: 26.6 per b64 load, 8 loads per
// step (profiles/r02_pmc/brick4832_512.json).  The fill needs one lookup per
// 64-B chunk, ~26 per channel-step (tools/slab_fill_model.py), but pays the
// box reductions and the per-lane fill addresses in VALU.  Register-staged
// fills, not LDS-DMA: a buffer_load ... lds of 16 scattered 64-B pieces costs
// the TA 37 cycles against 16.8 for the same loads into VGPRs
// (tools/lds_dma_calib.hip, profiles/r03/lds_dma_calib.txt).
#include "vr_march_kernels.h"

namespace vr {
namespace {

constexpr int kSlabWaves = kThreads / 64;
constexpr int kSlabChannelBytes = kSlabMaxChunks * 64;
constexpr int kSlabWaveBytes = 4 * kSlabChannelBytes;
constexpr int kSlabFillInstr = kSlabMaxChunks / 16;   // 16-B loads of 64 lanes per channel and step, at most

// min (MAX = false) or max of v over the 64 lanes, result in every lane
// (wave-uniform control flow; lanes that must not count pass +inf / -inf):
// row_shr 1, 2, 4, 8 inside each row of 16, then row_bcast 15 and 31.
template <bool MAX>
__device__ __forceinline__ float wave_reduce(float v)
{
    const auto step = [&](auto ctrl, auto rmask) {
        const float t = __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(__builtin_bit_cast(int, v),
                                                                              __builtin_bit_cast(int, v),
                                                                              decltype(ctrl)::value,
                                                                              decltype(rmask)::value, 0xf, false));
        v = MAX ? fmaxf(v, t) : fminf(v, t);
    };
    step(std::integral_constant<int, 0x111>{}, std::integral_constant<int, 0xf>{});
    step(std::integral_constant<int, 0x112>{}, std::integral_constant<int, 0xf>{});
    step(std::integral_constant<int, 0x114>{}, std::integral_constant<int, 0xf>{});
    step(std::integral_constant<int, 0x118>{}, std::integral_constant<int, 0xf>{});
    step(std::integral_constant<int, 0x142>{}, std::integral_constant<int, 0xa>{});
    step(std::integral_constant<int, 0x143>{}, std::integral_constant<int, 0xc>{});
    return __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, v), 63));
}

// One channel's slab box for this step (wave-uniform values).
struct SlabBox {
    bool fit;
    float bx0, by0, k0;       // first column (x, y) and chunk of the box
    float nbx, nk;            // columns along x, chunks per column
    float pieces;             // 16-B pieces of the fill (4 per chunk)
    float xs, ys, cb;         // LDS address = fma(qb, ys, fma(qa, xs, fma(c, 32, qb.y + qa.y + cb)))
};

// Padded positions floor(fma(P, S, T)) of the box corners -> columns and
// chunks.  a / 3 and b / 7 as floor(v * fl(1/k)): fl(1/3) and fl(1/7) exceed
// 1/3 and 1/7, and v <= 2^12, so no quotient falls below an integer.
__device__ __forceinline__ SlabBox slab_box(const MarchArgs& a, int ch, bool zo, float mnx, float mny, float mnz,
                                            float mxx, float mxy, float mxz, int chan_off)
{
    const float Sx = a.tap_S[ch][0], Sy = a.tap_S[ch][1], Sz = a.tap_S[ch][2];
    const float Tx = zo ? 0.5f : a.tap_T[ch][0], Ty = zo ? 0.5f : a.tap_T[ch][1], Tz = zo ? 0.5f : a.tap_T[ch][2];
    const float alo = floorf(fmaf(mnx, Sx, Tx)), ahi = floorf(fmaf(mxx, Sx, Tx));
    const float blo = floorf(fmaf(mny, Sy, Ty)), bhi = floorf(fmaf(mxy, Sy, Ty));
    const float clo = floorf(fmaf(mnz, Sz, Tz)), chi = floorf(fmaf(mxz, Sz, Tz));
    SlabBox b;
    b.bx0 = floorf(alo * (1.0f / 3.0f));
    b.by0 = floorf(blo * (1.0f / 7.0f));
    b.k0 = floorf(clo * 0.5f);
    b.nbx = floorf(ahi * (1.0f / 3.0f)) - b.bx0 + 1.0f;
    const float nby = floorf(bhi * (1.0f / 7.0f)) - b.by0 + 1.0f;
    b.nk = floorf((chi + 1.0f) * 0.5f) - b.k0 + 1.0f;
    const float chunks = (b.nbx * nby) * b.nk;
    b.fit = chunks <= (float)a.slab_cap;
    b.pieces = 4.0f * chunks;
    b.xs = 64.0f * b.nk;
    b.ys = b.xs * b.nbx;
    b.cb = (float)chan_off - fmaf(b.by0, b.ys, fmaf(b.bx0, b.xs, 64.0f * b.k0));
    return b;
}

template <bool EARLY, bool ZO>
__device__ __forceinline__ unsigned march_pixel_slab(const MarchArgs& a, const __amdgpu_buffer_rsrc_t* rsrc,
                                                     const float2* tx2, const float2* ty2, unsigned char* slab,
                                                     unsigned slab_lds, int x, int orow)
{
    const Ray r = setup_ray(a, x, orow);
    const int lane = threadIdx.x & 63;
    const float nbx_all = (float)a.geom.nbx;
    const unsigned colb = a.geom.brick;
    f2 pxy = r.pxy;
    float pz = r.pz;
    float acc = 0.0f;
    int i = 0;
    bool act = r.n > 0;
    for (;;) {
        act = act && i < r.n;
        if (__ballot(act) == 0) break;
        const float inf = __builtin_inff();
        const float mnx = wave_reduce<false>(act ? pxy.x : inf), mxx = wave_reduce<true>(act ? pxy.x : -inf);
        const float mny = wave_reduce<false>(act ? pxy.y : inf), mxy = wave_reduce<true>(act ? pxy.y : -inf);
        const float mnz = wave_reduce<false>(act ? pz : inf), mxz = wave_reduce<true>(act ? pz : -inf);
        SlabBox bx[4];
#pragma unroll
        for (int ch = 0; ch < 4; ++ch)
            bx[ch] = slab_box(a, ch, ZO, mnx, mny, mnz, mxx, mxy, mxz, ch * kSlabChannelBytes);
        // fill: every channel's loads first (in VGPRs), then their LDS writes
        uint4 fill[4][kSlabFillInstr];
        const float pf0 = (float)lane;
#pragma unroll
        for (int ch = 0; ch < 4; ++ch) {
            const SlabBox& b = bx[ch];
            const float pc = 4.0f * b.nk, rpc = __builtin_amdgcn_rcpf(pc), rnbx = __builtin_amdgcn_rcpf(b.nbx);
#pragma unroll
            for (int j = 0; j < kSlabFillInstr; ++j) {
                fill[ch][j] = make_uint4(0, 0, 0, 0);
                const float pf = pf0 + 64.0f * (float)j;
                if (b.fit && pf < b.pieces) {
                    const float col = floorf((pf + 0.5f) * rpc);
                    const float wq = fmaf(col, -pc, pf);
                    const float iy = floorf((col + 0.5f) * rnbx);
                    const float ix = fmaf(iy, -b.nbx, col);
                    const unsigned colg = (unsigned)fmaf(b.by0 + iy, nbx_all, b.bx0 + ix);
                    const unsigned off = __umul24(colg, colb) + (unsigned)fmaf(wq, 16.0f, 64.0f * b.k0);
                    const auto v = __builtin_amdgcn_raw_buffer_load_b128(rsrc[ch], off, 0, 0);
                    fill[ch][j] = make_uint4(v[0], v[1], v[2], v[3]);
                }
            }
        }
#pragma unroll
        for (int ch = 0; ch < 4; ++ch)
#pragma unroll
            for (int j = 0; j < kSlabFillInstr; ++j)
                if (bx[ch].fit && pf0 + 64.0f * (float)j < bx[ch].pieces)
                    *reinterpret_cast<uint4*>(slab + ch * kSlabChannelBytes + (j * 64 + lane) * 16) = fill[ch][j];
        __builtin_amdgcn_wave_barrier();
        if (act) {
            float t[4];
#pragma unroll
            for (int ch = 0; ch < 4; ++ch) {
                const f2 T = ZO ? f2{0.5f, 0.5f} : f2{a.tap_T[ch][0], a.tap_T[ch][1]};
                const f2 gxy = __builtin_elementwise_fma(pxy, f2{a.tap_S[ch][0], a.tap_S[ch][1]}, T);
                const float gz = fmaf(pz, a.tap_S[ch][2], ZO ? 0.5f : a.tap_T[ch][2]);
                TapRaw q{};
                q.wx = fract_(gxy.x); q.wy = fract_(gxy.y); q.wz = fract_(gz);
                const float2 qa = tx2[cvt_flr(gxy.x)], qb = ty2[cvt_flr(gxy.y)];
                const float cf = floorf(gz);
                const float row = qb.y + qa.y;   // 4 (b % 7) + a % 3: the byte in its slice
                if (bx[ch].fit) {
                    const SlabBox& b = bx[ch];
                    const unsigned ad = (unsigned)fmaf(qb.x, b.ys, fmaf(qa.x, b.xs, fmaf(cf, 32.0f, row + b.cb)));
                    const unsigned a0 = ad & ~3u;
                    const unsigned* s0 = reinterpret_cast<const unsigned*>(slab + a0);
                    const unsigned d0 = s0[0], d1 = s0[1], d2 = s0[8], d3 = s0[9];
                    q.q0 = __builtin_amdgcn_alignbyte(d1, d0, ad);
                    q.q1 = __builtin_amdgcn_alignbyte(d1, d1, ad);
                    q.q2 = __builtin_amdgcn_alignbyte(d3, d2, ad);
                    q.q3 = __builtin_amdgcn_alignbyte(d3, d3, ad);
                } else {
                    const unsigned colg = (unsigned)fmaf(qb.x, nbx_all, qa.x);
                    const unsigned off = __umul24(colg, colb) + (unsigned)fmaf(cf, 32.0f, row);
                    const unsigned a0 = off & ~3u;
                    const auto s0 = __builtin_amdgcn_raw_buffer_load_b64(rsrc[ch], a0, 0, 0);
                    const auto s1 = __builtin_amdgcn_raw_buffer_load_b64(rsrc[ch], a0 + 32u, 0, 0);
                    q.q0 = __builtin_amdgcn_alignbyte(s0[1], s0[0], off);
                    q.q1 = __builtin_amdgcn_alignbyte(s0[1], s0[1], off);
                    q.q2 = __builtin_amdgcn_alignbyte(s1[1], s1[0], off);
                    q.q3 = __builtin_amdgcn_alignbyte(s1[1], s1[1], off);
                }
                t[ch] = tap_blend<LAYOUT_COL48>(q);
            }
            acc = acc + ((t[0] * t[1]) * (t[2] + t[3])) * a.scale;                   // frag.glsl:71-73
            pxy = pxy + r.sxy;                                                        // :74
            pz = pz + r.sz;
            ++i;
            if constexpr (EARLY) {
                if (acc > a.acc_limit) act = false;
            }
        }
        __builtin_amdgcn_wave_barrier();   // the slab's reads before the next step's writes
    }
    if (r.live) {
        const float at = acc * a.step_size;                                          // :76
        store_pixel(a, x, orow, r.n >= 0, 1.0f - spec_expf(a.density * fminf(-at, 0.0f)));   // :79
    }
    (void)slab_lds;
    return r.n > 0 ? (unsigned)i : 0u;
}

// Regions schedule (march_regions), COL48, one lane per ray.  Dynamic LDS:
// the per-wave slabs (kSlabWaveBytes each), then the per-axis tables
// {a / 3, a % 3} and {b / 7, 4 (b % 7)} as float2.
template <bool EARLY, bool ZO>
__global__ __launch_bounds__(kThreads) void march_regions_slab(const MarchArgs a, const unsigned* __restrict__ tiles,
                                                              const int* __restrict__ hdr, int nwx)
{
    extern __shared__ __attribute__((aligned(16))) unsigned char lds_raw[];
    const int xcd = blockIdx.x & 7;
    const int w = (int)(blockIdx.x >> 3) * kSlabWaves + (threadIdx.x >> 6);
    const int begin = hdr[xcd], count = hdr[xcd + 1] - begin;
    if ((int)(blockIdx.x >> 3) * kSlabWaves >= count) return;   // whole workgroup, before the barrier
    float2* tx2 = reinterpret_cast<float2*>(lds_raw + kSlabWaves * kSlabWaveBytes);
    float2* ty2 = tx2 + (a.nx + 1);
    for (int i = threadIdx.x; i < a.nx + 1 + a.ny + 1; i += kThreads) {
        if (i <= a.nx) tx2[i] = make_float2((float)(i / 3), (float)(i % 3));
        else {
            const int b = i - a.nx - 1;
            ty2[b] = make_float2((float)(b / 7), (float)(4 * (b % 7)));
        }
    }
    __syncthreads();
    __amdgpu_buffer_rsrc_t rsrc[4];
    for (int c = 0; c < 4; ++c)
        rsrc[c] = __builtin_amdgcn_make_buffer_rsrc((void*)(a.vol + (size_t)c * a.plane_stride), (short)0,
                                                    (int)a.plane_stride, 0x00020000);
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    unsigned char* slab = lds_raw + wave * kSlabWaveBytes;
    unsigned long long steps = 0;
    for (int k = w; w < nwx && k < count; k += nwx) {   // the grid rounds nwx up to whole workgroups
        const unsigned t = tiles[begin + k];
        const int tx = (int)(t & 0xffffu), ty = (int)(t >> 16);
        steps += march_pixel_slab<EARLY, ZO>(a, rsrc, tx2, ty2, slab, 0u, tx * 8 + lane_x<LAYOUT_COL48>(lane),
                                             ty * 8 + lane_y<LAYOUT_COL48>(lane));
    }
    if (a.step_counter) add_steps(a, steps);
}

}  // namespace

size_t slab_lds_bytes(int nx, int ny) { return (size_t)kSlabWaves * kSlabWaveBytes + (size_t)(nx + 1 + ny + 1) * 8u; }

hipError_t launch_march_slab(const MarchArgs& a, bool early, const Schedule& sc, hipStream_t s)
{
    const dim3 grid((unsigned)(8 * ((sc.map.nwx + 3) / 4))), block(kThreads);
    const size_t lds = slab_lds_bytes(a.nx, a.ny);
    if (early && a.zero_offsets)
        hipLaunchKernelGGL((march_regions_slab<true, true>), grid, block, lds, s, a, sc.tiles, sc.hdr, sc.map.nwx);
    else if (early)
        hipLaunchKernelGGL((march_regions_slab<true, false>), grid, block, lds, s, a, sc.tiles, sc.hdr, sc.map.nwx);
    else if (a.zero_offsets)
        hipLaunchKernelGGL((march_regions_slab<false, true>), grid, block, lds, s, a, sc.tiles, sc.hdr, sc.map.nwx);
    else
        hipLaunchKernelGGL((march_regions_slab<false, false>), grid, block, lds, s, a, sc.tiles, sc.hdr, sc.map.nwx);
    return hipGetLastError();
}

}  // namespace vr
