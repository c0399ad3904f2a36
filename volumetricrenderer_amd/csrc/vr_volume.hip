// vr_volume.hip -- volume producer and layout kernels, plus band assembly.
//
//  * repack: RGBA8 interleaved (the Texture3D input, TestMain.cpp:69-87)
//    -> per-channel planes (planar and padded), the layouts vr_march reads.
//  * noise + min/max + pack: TestMain.cpp:43-92 on the GPU.
//  * assemble: gathered band sets of N ranks -> one frame (SURVEY.md e).
// All are HBM-bound streaming kernels: wide coalesced accesses, grid-stride.
#include <algorithm>
#include <cmath>
#include <cstdlib>

#include "vr_internal.h"
#include "vr_noise.h"

namespace vr {
namespace {

constexpr int kBlock = 256;

__device__ __forceinline__ int clampi(int v, int lo, int hi) { return min(max(v, lo), hi); }

// One thread per texel: read 4 B, write 1 B to each of 4 planes.  The padded
// planes get their own pass over (nx+2)(ny+2)(nz+2) positions.
__global__ __launch_bounds__(kBlock) void k_repack_planar(const uchar4* __restrict__ src, long long total,
                                                          uint8_t* __restrict__ dst)
{
    for (long long i = blockIdx.x * (long long)kBlock + threadIdx.x; i < total;
         i += (long long)gridDim.x * kBlock) {
        const uchar4 v = src[i];
        dst[i] = v.x;
        dst[i + total] = v.y;
        dst[i + 2 * total] = v.z;
        dst[i + 3 * total] = v.w;
    }
}

// Fast layouts, built from the planar planes.  Every element stores
// clamp-to-edge texels of the padded base position (a, b, c), where texel
// index = padded index - 1 (vr_internal.h Layout).
struct PlaneSrc {
    const uint8_t* p;
    int nx, ny, nz;
    __device__ __forceinline__ unsigned int at(int a, int b, int c) const  // padded coordinates
    {
        const int x = clampi(a - 1, 0, nx - 1), y = clampi(b - 1, 0, ny - 1), z = clampi(c - 1, 0, nz - 1);
        return p[((long long)z * ny + y) * nx + x];
    }
};

// One thread per output element: a byte of an apron brick, or one 8-byte
// footprint word (CORNER8).  Brick order and in-brick order match
// axis_offset() in vr_internal.h, which the march kernel's LDS tables use.
template <int LAYOUT>
__global__ __launch_bounds__(kBlock) void k_build_layout(const uint8_t* __restrict__ planar, int nx, int ny,
                                                         int nz, LayoutGeom g, long long plane_elems,
                                                         long long plane_bytes, uint8_t* __restrict__ out, int nch = 4)
{
    const long long total_planar = (long long)nx * ny * nz;
    for (long long i = blockIdx.x * (long long)kBlock + threadIdx.x; i < nch * plane_elems;
         i += (long long)gridDim.x * kBlock) {
        const int ch = (int)(i / plane_elems);
        const long long e = i - ch * plane_elems;
        const PlaneSrc src{planar + ch * total_planar, nx, ny, nz};
        uint8_t* dst = out + ch * plane_bytes;
        if constexpr (LAYOUT == LAYOUT_CORNER8) {
            const long long brick = e >> 6;
            const int pos = (int)(e & 63);
            const int bx = (int)(brick % g.nbx);
            const long long t = brick / g.nbx;
            const int by = (int)(t % g.nby), bz = (int)(t / g.nby);
            const int a = 4 * bx + (pos & 3), b = 4 * by + ((pos >> 2) & 3), c = 4 * bz + (pos >> 4);
            unsigned long long q = 0;
            for (int k = 0; k < 8; ++k)
                q |= (unsigned long long)src.at(a + (k & 1), b + ((k >> 1) & 1), c + (k >> 2)) << (8 * k);
            reinterpret_cast<unsigned long long*>(dst)[e] = q;
        } else if constexpr (LAYOUT == LAYOUT_CORNERH) {
            // position (a, b, c), x fastest; dword k = footprint row (y, z) =
            // (b + (k & 1), c + (k >> 1)): f16 a in the low half, f16 (b - a)
            // in the high half (both exact: |values| <= 255)
            const int a = (int)(e % g.nbx);
            const long long t = e / g.nbx;
            const int b = (int)(t % g.nby), c = (int)(t / g.nby);
            unsigned w[4];
            for (int k = 0; k < 4; ++k) {
                const int y = b + (k & 1), z = c + (k >> 1);
                const int va = (int)src.at(a, y, z), vb = (int)src.at(a + 1, y, z);
                const _Float16 ha = (_Float16)(float)va, hd = (_Float16)(float)(vb - va);
                w[k] = (unsigned)__builtin_bit_cast(unsigned short, ha) |
                       ((unsigned)__builtin_bit_cast(unsigned short, hd) << 16);
            }
            reinterpret_cast<uint4*>(dst)[e] = make_uint4(w[0], w[1], w[2], w[3]);
        } else if constexpr (LAYOUT == LAYOUT_ZPAIR) {
            // byte = x + 4 * (z + 2 * y): 4-byte rows, z fastest
            const long long brick = e >> 7;
            const int byte = (int)(e & 127);
            const int bx = (int)(brick % g.nbx);
            const long long t = brick / g.nbx;
            const int by = (int)(t % g.nby), bz = (int)(t / g.nby);
            dst[e] = src.at(3 * bx + (byte & 3), 15 * by + (byte >> 3), bz + ((byte >> 2) & 1));
        } else {
            const long long brick = e / g.brick;
            const int byte = (int)(e - brick * g.brick);
            unsigned int v = 0;
            if (byte < g.Rn[0] * g.Rn[1] * g.Rn[2]) {
                const int u = byte % g.Rn[0], vv = (byte / g.Rn[0]) % g.Rn[1], w = byte / (g.Rn[0] * g.Rn[1]);
                const int bx = (int)(brick % g.nbx);
                const long long t = brick / g.nbx;
                const int by = (int)(t % g.nby), bz = (int)(t / g.nby);
                v = src.at(g.Ba[0] * bx + u, g.Ba[1] * by + vv, g.Ba[2] * bz + w);
            }
            dst[e] = (uint8_t)v;
        }
    }
}

// The apron-brick layouts (BRICK4 family, BRICK5/8/16), staged through LDS.
// A workgroup builds a run of `run` consecutive bricks along x at one
// (by, bz): it loads their source box -- Rn[1] x Rn[2] planar rows of
// Ba[0] (run - 1) + Rn[0] bytes, clamped to the edge -- with coalesced byte
// loads (consecutive lanes, consecutive x), then writes the run, which is
// contiguous in the layout, as 16-B stores gathered from LDS.  The per-byte
// kernel before it (a 1-B store and 8 scattered planar reads per thread,
// 64-bit decode) took 4.0 ms at 512^3.
constexpr int kBrickStageBytes = 16 * 1024;
//
// zseg > 0 (COL48, whose columns run through the whole z extent): a workgroup
// builds segment blockIdx.y -- slices [zseg * seg, zseg * (seg + 1)) -- of a
// run of columns; a column's segment is contiguous, the run's columns sit a
// column (g.brick bytes) apart.
__global__ __launch_bounds__(kBlock) void k_build_bricks(const uint8_t* __restrict__ planar, int nx, int ny, int nz,
                                                         LayoutGeom g, int run, long long plane_bytes, int zseg,
                                                         uint8_t* __restrict__ out)
{
    __shared__ uint8_t st[kBrickStageBytes];
    const int ch = blockIdx.z;
    const uint8_t* __restrict__ p = planar + (long long)ch * nx * ny * nz;
    const int runs_x = (g.nbx + run - 1) / run;
    const int rx = (int)blockIdx.x % runs_x, by = (int)blockIdx.x / runs_x, bz = (int)blockIdx.y;
    const int bx0 = rx * run, nb = min(run, g.nbx - bx0);
    const int rn0 = g.Rn[0], rn1 = g.Rn[1], rn2 = zseg > 0 ? min(zseg, g.Rn[2] - zseg * bz) : g.Rn[2];
    // slice w of a COL48 column holds padded z position w (texel w - 1)
    const int x0 = g.Ba[0] * bx0 - 1, y0 = g.Ba[1] * by - 1, z0 = zseg > 0 ? zseg * bz - 1 : g.Ba[2] * bz - 1;
    const int xe = x0 + g.Ba[0] * (nb - 1) + rn0;    // one past the last staged x
    const int rows = rn1 * rn2;
    // stage: rows (v, w) of the source box, x fastest over the whole workgroup.
    // Runs inside the volume along x with dword-aligned planar rows take
    // aligned dword loads (xa = x0 & ~3 .. xe rounded up); the edge runs
    // clamp byte by byte.
    const int xa = x0 & ~3, wx = ((xe + 3) & ~3) - xa;   // staged row: [xa, xa + wx)
    if (xa >= 0 && xa + wx <= nx && (nx & 3) == 0) {
        const int wd = wx >> 2, total = rows * wd;
        unsigned* st4 = reinterpret_cast<unsigned*>(st);
#pragma unroll 4
        for (int i = threadIdx.x; i < total; i += kBlock) {
            const int row = i / wd, xi = i - row * wd;
            const int w = row / rn1, v = row - w * rn1;
            const int y = clampi(y0 + v, 0, ny - 1), z = clampi(z0 + w, 0, nz - 1);
            st4[i] = *reinterpret_cast<const unsigned*>(
                p + ((unsigned)z * (unsigned)ny + (unsigned)y) * (unsigned)nx + (unsigned)(xa + 4 * xi));
        }
    } else {
        const int total = rows * wx;
        for (int i = threadIdx.x; i < total; i += kBlock) {
            const int row = i / wx, xi = i - row * wx;
            const int w = row / rn1, v = row - w * rn1;
            const int x = clampi(xa + xi, 0, nx - 1), y = clampi(y0 + v, 0, ny - 1), z = clampi(z0 + w, 0, nz - 1);
            st[i] = p[((unsigned)z * (unsigned)ny + (unsigned)y) * (unsigned)nx + (unsigned)x];
        }
    }
    __syncthreads();
    // write: the run's bricks are contiguous, brick by brick in-brick order x
    // fastest (COL48: each column's segment is contiguous, columns g.brick apart)
    const unsigned used = (unsigned)(rn0 * rn1 * rn2);
    const unsigned per_brick = zseg > 0 ? used / 16u : g.brick / 16u;   // COL48: 32 B per slice
    uint8_t* __restrict__ dst0 = out + (long long)ch * plane_bytes +
                                 (zseg > 0 ? ((long long)by * g.nbx + bx0) * g.brick + (long long)bz * rn0 * rn1 * zseg
                                           : ((long long)(bz * g.nby + by) * g.nbx + bx0) * g.brick);
    for (unsigned c = threadIdx.x; c < (unsigned)nb * per_brick; c += kBlock) {
        const unsigned j = c / per_brick, b0 = (c - j * per_brick) * 16u;
        uint4* __restrict__ dst = reinterpret_cast<uint4*>(dst0 + (long long)j * g.brick) - j * per_brick;
        unsigned u = b0 % (unsigned)rn0, v = (b0 / (unsigned)rn0) % (unsigned)rn1, w = b0 / (unsigned)(rn0 * rn1);
        const unsigned xb = j * (unsigned)g.Ba[0] + (unsigned)(x0 - xa);
        unsigned word[4] = {0u, 0u, 0u, 0u};
#pragma unroll
        for (int k = 0; k < 16; ++k) {
            if (b0 + (unsigned)k < used)
                word[k >> 2] |= (unsigned)st[(w * (unsigned)rn1 + v) * (unsigned)wx + xb + u] << (8 * (k & 3));
            if (++u == (unsigned)rn0) { u = 0; if (++v == (unsigned)rn1) { v = 0; ++w; } }
        }
        dst[c] = make_uint4(word[0], word[1], word[2], word[3]);
    }
}

__global__ __launch_bounds__(kBlock) void k_unpack_planar(const uint8_t* __restrict__ src, long long total,
                                                          uchar4* __restrict__ dst)
{
    for (long long i = blockIdx.x * (long long)kBlock + threadIdx.x; i < total;
         i += (long long)gridDim.x * kBlock)
        dst[i] = make_uchar4(src[i], src[i + total], src[i + 2 * total], src[i + 3 * total]);
}

// GenUniformGrid3D: pos = (start + idx) * freq, x fastest.  Each block also
// writes its {min, max}; k_minmax folds them (exact, order-independent).
// kind 0 cellular, 1 Perlin, 2 simplex.  cell_n > 0 (cellular only): the
// workgroup first puts the feature-point data of the cells [cell_lo,
// cell_lo + cell_n)^3 in LDS (noise::cellular_cell, the procedural march's
// table) and evaluates F1 with noise::cellular_table -- bit-identical to
// noise::cellular, 7 VALU ops per cell instead of the hash, sqrt and
// reciprocal.  The host sizes the cell range from the grid's coordinate range.
constexpr int kNoiseTableMaxN = 12;
__global__ __launch_bounds__(kBlock) void k_noise(int kind, float* __restrict__ out, int x0, int y0, int z0,
                                                  int nx, int ny, int nz, float freq, int32_t seed,
                                                  int cell_lo, int cell_n, float2* __restrict__ partials)
{
    extern __shared__ float4 cells[];   // cell_n^3 entries (dynamic: none for Perlin / simplex)
    if (cell_n > 0) {
        const int n = cell_n;
        for (int i = threadIdx.x; i < n * n * n; i += kBlock) {
            const int ix = i % n, iy = (i / n) % n, iz = i / (n * n);
            cells[i] = noise::cellular_cell(seed, cell_lo + ix, cell_lo + iy, cell_lo + iz);
        }
        __syncthreads();
    }
    const unsigned total = (unsigned)nx * (unsigned)ny * (unsigned)nz;   // < 2^32 (host check)
    float mn = __builtin_inff(), mx = -__builtin_inff();
    for (unsigned i = blockIdx.x * kBlock + threadIdx.x; i < total; i += gridDim.x * kBlock) {
        const unsigned t = i / (unsigned)nx;
        const int x = (int)(i - t * (unsigned)nx);
        const int y = (int)(t % (unsigned)ny), z = (int)(t / (unsigned)ny);
        const float px = (float)(x0 + x) * freq, py = (float)(y0 + y) * freq, pz = (float)(z0 + z) * freq;
        float v;
        if (kind == 0) v = cell_n > 0 ? noise::cellular_table(cells, cell_lo, cell_n, cell_n * cell_n, px, py, pz)
                                      : noise::cellular(seed, px, py, pz);
        else if (kind == 1) v = noise::perlin(seed, px, py, pz);
        else v = noise::simplex(seed, px, py, pz);
        if (out) out[i] = v;
        mn = fminf(mn, v);
        mx = fmaxf(mx, v);
    }
    for (int off = 32; off > 0; off >>= 1) {
        mn = fminf(mn, __shfl_xor(mn, off));
        mx = fmaxf(mx, __shfl_xor(mx, off));
    }
    __shared__ float2 red[kBlock / 64];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    if (lane == 0) red[wave] = make_float2(mn, mx);
    __syncthreads();
    if (threadIdx.x == 0) {
        float2 r = red[0];
        for (int w = 1; w < kBlock / 64; ++w) { r.x = fminf(r.x, red[w].x); r.y = fmaxf(r.y, red[w].y); }
        partials[blockIdx.x] = r;
    }
}

__global__ __launch_bounds__(kBlock) void k_minmax(const float2* __restrict__ partials, int n, float* __restrict__ out)
{
    float mn = __builtin_inff(), mx = -__builtin_inff();
    for (int i = threadIdx.x; i < n; i += kBlock) { mn = fminf(mn, partials[i].x); mx = fmaxf(mx, partials[i].y); }
    for (int off = 32; off > 0; off >>= 1) {
        mn = fminf(mn, __shfl_xor(mn, off));
        mx = fmaxf(mx, __shfl_xor(mx, off));
    }
    __shared__ float2 red[kBlock / 64];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    if (lane == 0) red[wave] = make_float2(mn, mx);
    __syncthreads();
    if (threadIdx.x == 0) {
        float2 r = red[0];
        for (int w = 1; w < kBlock / 64; ++w) { r.x = fminf(r.x, red[w].x); r.y = fmaxf(r.y, red[w].y); }
        out[0] = r.x;
        out[1] = r.y;
    }
}

// static_cast<unsigned char>(float) as x86-64 compiles it (cvttss2si, keep
// the low byte): TestMain.cpp:84-87.
__device__ __forceinline__ unsigned int f2u8_trunc(float f)
{
    if (!(f > -2147483648.0f && f < 2147483648.0f)) return 0u;
    return (unsigned int)(int)f & 0xffu;
}

// TestMain.cpp:64-92.  g2 == nullptr means the zero-filled noiseOutput2 of
// the literal recipe.  minmax = {min1,max1, min2,max2, min3,max3, min4,max4}.
__global__ __launch_bounds__(kBlock) void k_pack_recipe(const float* __restrict__ g1, const float* __restrict__ g2,
                                                        const float* __restrict__ g3, const float* __restrict__ g4,
                                                        const float* __restrict__ mm, long long total,
                                                        uchar4* __restrict__ out)
{
    const float inv1 = 1.0f / (mm[1] - mm[0]), inv2 = 1.0f / (mm[3] - mm[2]);
    const float inv3 = 1.0f / (mm[5] - mm[4]), inv4 = 1.0f / (mm[7] - mm[6]);
    for (long long i = blockIdx.x * (long long)kBlock + threadIdx.x; i < total;
         i += (long long)gridDim.x * kBlock) {
        float s1 = 1.0f - (g1[i] - mm[0]) * inv1;
        const float s2 = 1.0f - ((g2 ? g2[i] : 0.0f) - mm[2]) * inv2;
        const float s3 = 1.0f - (g3[i] - mm[4]) * inv3;
        const float s4 = 1.0f - (g4[i] - mm[6]) * inv4;
        s1 = s1 * ((s1 * s1) * s1);
        out[i] = make_uchar4(f2u8_trunc(s1 * 255.0f), f2u8_trunc(s2 * 255.0f), f2u8_trunc(s3 * 255.0f),
                             f2u8_trunc(s4 * 255.0f));
    }
}

// frame row y lives in band b = y / band_rows, rendered by rank b % nranks as
// its (b / nranks)-th band.  16-byte chunks when rows allow it.  Rows of ranks
// below first_rank are left as they are (rendered in place into the frame,
// vr.h VR_TARGET_BANDS_IN_PLACE).
//
// Row q (from rank first_rank's slot on) of the gathered band sets -> its
// frame row y: rank r's slot holds its bands lb = 0, 1, ... packed, and band
// lb of rank r is frame band lb * nranks + r -- or, serpentine (vr_target
// band_flip nranks - 1 - 2r), lb * nranks + nranks - 1 - r for odd lb.  -1 for slot rows past the
// frame (a rank with fewer rows than the slot).  Block-uniform: the divisions
// are scalar, once per row.
__device__ __forceinline__ int assembled_row(int q, int rows_per_rank, int nranks, int band_rows, int first_rank,
                                             int serp, int height)
{
    const int r = first_rank + q / rows_per_rank, lr = q % rows_per_rank;
    const int lb = lr / band_rows, rr = lr - lb * band_rows;
    const int y = (lb * nranks + ((serp && (lb & 1)) ? nranks - 1 - r : r)) * band_rows + rr;
    return y < height ? y : -1;
}

// The assembly kernels (vr_assemble_frame): rows x elements.  Each lane moves
// up to kAsmBatch rows' elements with all the loads in flight before the
// first store (frames taller than the grid); the frame row comes from
// block-uniform scalar arithmetic, with no per-element division.
constexpr int kAsmBatch = 8;
template <typename S, typename D, typename F>
__device__ __forceinline__ void assemble_rows(const S* __restrict__ src, int rows_per_rank, int nranks, int row_elems,
                                              int height, int band_rows, int first_rank, int serp, D* __restrict__ dst,
                                              F expand)
{
    const int rows = (nranks - first_rank) * rows_per_rank;
    const int e = blockIdx.x * kBlock + threadIdx.x;
    if (e >= row_elems) return;
    const size_t base = (size_t)first_rank * rows_per_rank;
    for (int q0 = blockIdx.y; q0 < rows; q0 += gridDim.y * kAsmBatch) {
        S v[kAsmBatch];
        int y[kAsmBatch];
#pragma unroll
        for (int j = 0; j < kAsmBatch; ++j) {
            const int q = q0 + j * (int)gridDim.y;
            y[j] = q < rows ? assembled_row(q, rows_per_rank, nranks, band_rows, first_rank, serp, height) : -1;
            if (y[j] >= 0) v[j] = src[(base + q) * row_elems + e];
        }
#pragma unroll
        for (int j = 0; j < kAsmBatch; ++j)
            if (y[j] >= 0) dst[(size_t)y[j] * row_elems + e] = expand(v[j]);
    }
}

template <typename T>
__global__ __launch_bounds__(kBlock) void k_assemble(const T* __restrict__ src, int rows_per_rank, int nranks,
                                                     int row_elems, int height, int band_rows, int first_rank,
                                                     int serp, T* __restrict__ dst)
{
    assemble_rows(src, rows_per_rank, nranks, row_elems, height, band_rows, first_rank, serp, dst,
                  [](T v) { return v; });
}

// Grey band sets -> RGBA frame (vr_assemble_frame): element e of frame row y
// comes from the same place k_assemble reads, expanded.  P pixels per element:
// u8 x 4 (uchar4 -> 4 RGBA8 words, rows of a multiple of 4 pixels), u8 x 1,
// or fp32 x 1 (-> float4).
template <typename S, typename D>
__device__ __forceinline__ D grey_expand(S v);
template <>
__device__ __forceinline__ uint4 grey_expand<unsigned int, uint4>(unsigned int v)
{
    uint4 o;
    unsigned q = v & 0xffu;
    o.x = q * 0x010101u | 0xff000000u;
    q = (v >> 8) & 0xffu;
    o.y = q * 0x010101u | 0xff000000u;
    q = (v >> 16) & 0xffu;
    o.z = q * 0x010101u | 0xff000000u;
    q = v >> 24;
    o.w = q * 0x010101u | 0xff000000u;
    return o;
}
template <>
__device__ __forceinline__ unsigned int grey_expand<unsigned char, unsigned int>(unsigned char v)
{
    return (unsigned)v * 0x010101u | 0xff000000u;
}
template <>
__device__ __forceinline__ float4 grey_expand<float, float4>(float v)
{
    return make_float4(v, v, v, 1.0f);
}
template <typename S, typename D>
__global__ __launch_bounds__(kBlock) void k_assemble_grey(const S* __restrict__ src, int rows_per_rank,
                                                          int nranks, int row_elems, int height, int band_rows,
                                                          int first_rank, int serp, D* __restrict__ dst)
{
    assemble_rows(src, rows_per_rank, nranks, row_elems, height, band_rows, first_rank, serp, dst,
                  [](S v) { return grey_expand<S, D>(v); });
}

// grid of the assembly kernels: ceil(elems / kBlock) workgroups across a row,
// rows over blockIdx.y -- about 2048 workgroups in all, so 7/8 of a 1080p
// frame is one row per workgroup row (more, smaller workgroups run faster
// beside the other stream's march: profiles/r05/assembly_grid.txt)
dim3 grid_rows(size_t rows_per_rank, int nranks, int first_rank, long long elems)
{
    const long long rows = (long long)(nranks - first_rank) * (long long)rows_per_rank;
    const long long gx = (elems + kBlock - 1) / kBlock;
    constexpr long long target = 2048;   // rank 0 at N = 8: 0.0212 ms/frame, 0.0215 at 1024, 0.0220 at 512, 0.0245 at 128
    const long long gy = std::max(1LL, std::min({rows, (target + gx - 1) / gx, 65535LL}));
    return dim3((unsigned)gx, (unsigned)gy);
}

int grid_for(long long n)
{
    long long g = (n + kBlock - 1) / kBlock;
    if (g > 256 * 16) g = 256 * 16;
    if (g < 1) g = 1;
    return (int)g;
}

}  // namespace

// Byte min / max of each plane (blockIdx.y = plane): grid-stride bytes, a
// wave reduction, one atomicMin / atomicMax per wave.
__global__ __launch_bounds__(kBlock) void k_plane_minmax(const uint8_t* __restrict__ planes, long long total,
                                                         unsigned* __restrict__ mm)
{
    const uint8_t* pl = planes + (size_t)blockIdx.y * (size_t)total;
    unsigned lo = 255u, hi = 0u;
    // the 4-byte-aligned body as words, the rest as bytes
    const long long mis = (long long)((4u - (unsigned)((uintptr_t)pl & 3u)) & 3u);
    const long long head = mis < total ? mis : total;
    const long long words = (total - head) / 4;
    const unsigned* w = reinterpret_cast<const unsigned*>(pl + head);
    const long long stride = (long long)gridDim.x * kBlock;
    for (long long i = blockIdx.x * (long long)kBlock + threadIdx.x; i < words; i += stride) {
        const unsigned v = w[i];
        const unsigned b0 = v & 0xffu, b1 = (v >> 8) & 0xffu, b2 = (v >> 16) & 0xffu, b3 = v >> 24;
        lo = min(lo, min(min(b0, b1), min(b2, b3)));
        hi = max(hi, max(max(b0, b1), max(b2, b3)));
    }
    const long long tail0 = head + words * 4;
    for (long long i = blockIdx.x * (long long)kBlock + threadIdx.x; i < head + (total - tail0); i += stride) {
        const unsigned b = i < head ? pl[i] : pl[tail0 + (i - head)];
        lo = min(lo, b);
        hi = max(hi, b);
    }
    for (int off = 32; off > 0; off >>= 1) {
        lo = min(lo, (unsigned)__shfl_xor((int)lo, off));
        hi = max(hi, (unsigned)__shfl_xor((int)hi, off));
    }
    if ((threadIdx.x & 63) == 0) {
        atomicMin(&mm[blockIdx.y], lo);
        atomicMax(&mm[4 + blockIdx.y], hi);
    }
}

hipError_t launch_plane_minmax(const uint8_t* d_planar, long long total, unsigned* mm, hipStream_t s)
{
    long long g = (total / 4 + kBlock - 1) / kBlock;
    g = g < 1 ? 1 : g > 1024 ? 1024 : g;
    hipLaunchKernelGGL(k_plane_minmax, dim3((unsigned)g, 4), dim3(kBlock), 0, s, d_planar, total, mm);
    return hipGetLastError();
}

hipError_t launch_repack(const uint8_t* d_rgba, int nx, int ny, int nz, uint8_t* d_planar, hipStream_t s)
{
    const long long total = (long long)nx * ny * nz;
    hipLaunchKernelGGL(k_repack_planar, dim3(grid_for(total)), dim3(kBlock), 0, s,
                       reinterpret_cast<const uchar4*>(d_rgba), total, d_planar);
    return hipGetLastError();
}

namespace {
long long layout_elems(int layout, int nx, int ny, int nz)
{
    const LayoutGeom g = layout_geom(layout, nx, ny, nz);
    const long long nb = (long long)g.nbx * g.nby * g.nbz;
    return layout == LAYOUT_CORNER8 ? nb * 64 : layout == LAYOUT_CORNERH ? nb : nb * g.brick;
}
int elem_bytes(int layout) { return layout == LAYOUT_CORNER8 ? 8 : layout == LAYOUT_CORNERH ? 16 : 1; }
}  // namespace

size_t layout_plane_bytes(int layout, int nx, int ny, int nz)
{
    const size_t b = (size_t)layout_elems(layout, nx, ny, nz) * elem_bytes(layout);
    return (b + 255) & ~(size_t)255;
}

size_t layout_total_bytes(int layout, int nx, int ny, int nz)
{
    if (layout == LAYOUT_COL48Z)   // three COL48 planes, then channel 3's ZPAIR plane
        return 3 * layout_plane_bytes(LAYOUT_COL48, nx, ny, nz) + layout_plane_bytes(LAYOUT_ZPAIR, nx, ny, nz);
    return 4 * layout_plane_bytes(layout, nx, ny, nz);
}

hipError_t launch_build_layout(int layout, const uint8_t* d_planar, int nx, int ny, int nz, uint8_t* d_out,
                               hipStream_t s)
{
    const LayoutGeom g = layout_geom(layout, nx, ny, nz);
    const long long elems = layout_elems(layout, nx, ny, nz);
    const long long pb = (long long)layout_plane_bytes(layout, nx, ny, nz);
    const dim3 gr(grid_for(4 * elems)), b(kBlock);
    const long long rows = (long long)g.Rn[1] * g.Rn[2];
    if (layout == LAYOUT_COL48 || layout == LAYOUT_COL48Z) {
        const int nch = layout == LAYOUT_COL48Z ? 3 : 4;   // COL48Z: channel 3 is ZPAIR's, below
        // columns in z segments of 32 slices (1 KiB of a column: BRICK4832's stage)
        constexpr int kSeg = 32;
        const long long srows = (long long)g.Rn[1] * kSeg;
        const int run = (int)std::min<long long>(g.nbx, (kBrickStageBytes / srows - g.Rn[0] - 7) / g.Ba[0] + 1);
        const int runs_x = (g.nbx + run - 1) / run;
        const dim3 gb((unsigned)(runs_x * g.nby), (unsigned)((g.Rn[2] + kSeg - 1) / kSeg), nch);   // last segment partial
        hipLaunchKernelGGL(k_build_bricks, gb, b, 0, s, d_planar, nx, ny, nz, g, run, pb, kSeg, d_out);
        if (layout == LAYOUT_COL48Z) {
            const LayoutGeom gz = layout_geom(LAYOUT_ZPAIR, nx, ny, nz);
            const long long ez = layout_elems(LAYOUT_ZPAIR, nx, ny, nz);
            hipLaunchKernelGGL(k_build_layout<LAYOUT_ZPAIR>, dim3(grid_for(ez)), b, 0, s,
                               d_planar + 3 * (long long)nx * ny * nz, nx, ny, nz, gz, ez,
                               (long long)layout_plane_bytes(LAYOUT_ZPAIR, nx, ny, nz), d_out + 3 * pb, 1);
        }
        return hipGetLastError();
    }
    if (layout != LAYOUT_CORNER8 && layout != LAYOUT_CORNERH && layout != LAYOUT_ZPAIR && g.brick % 16u == 0 &&
        rows * (g.Ba[0] + g.Rn[0] + 8) <= kBrickStageBytes) {
        // bricks per workgroup: the longest run whose source box (+ up to 7
        // bytes of dword alignment per row) fits the stage
        const int run = (int)std::min<long long>(g.nbx, (kBrickStageBytes / rows - g.Rn[0] - 7) / g.Ba[0] + 1);
        const int runs_x = (g.nbx + run - 1) / run;
        const dim3 gb((unsigned)(runs_x * g.nby), (unsigned)g.nbz, 4);
        hipLaunchKernelGGL(k_build_bricks, gb, b, 0, s, d_planar, nx, ny, nz, g, run, pb, 0, d_out);
        return hipGetLastError();
    }
    switch (layout) {
    case LAYOUT_BRICK4: hipLaunchKernelGGL(k_build_layout<LAYOUT_BRICK4>, gr, b, 0, s, d_planar, nx, ny, nz, g, elems, pb, d_out); break;
    case LAYOUT_BRICK5: hipLaunchKernelGGL(k_build_layout<LAYOUT_BRICK5>, gr, b, 0, s, d_planar, nx, ny, nz, g, elems, pb, d_out); break;
    case LAYOUT_BRICK8: hipLaunchKernelGGL(k_build_layout<LAYOUT_BRICK8>, gr, b, 0, s, d_planar, nx, ny, nz, g, elems, pb, d_out); break;
    case LAYOUT_BRICK16: hipLaunchKernelGGL(k_build_layout<LAYOUT_BRICK16>, gr, b, 0, s, d_planar, nx, ny, nz, g, elems, pb, d_out); break;
    case LAYOUT_BRICK448: hipLaunchKernelGGL(k_build_layout<LAYOUT_BRICK448>, gr, b, 0, s, d_planar, nx, ny, nz, g, elems, pb, d_out); break;
    case LAYOUT_BRICK488: hipLaunchKernelGGL(k_build_layout<LAYOUT_BRICK488>, gr, b, 0, s, d_planar, nx, ny, nz, g, elems, pb, d_out); break;
    case LAYOUT_BRICK4816: hipLaunchKernelGGL(k_build_layout<LAYOUT_BRICK4816>, gr, b, 0, s, d_planar, nx, ny, nz, g, elems, pb, d_out); break;
    case LAYOUT_BRICK4864: hipLaunchKernelGGL(k_build_layout<LAYOUT_BRICK4864>, gr, b, 0, s, d_planar, nx, ny, nz, g, elems, pb, d_out); break;
    case LAYOUT_BRICK4832: hipLaunchKernelGGL(k_build_layout<LAYOUT_BRICK4832>, gr, b, 0, s, d_planar, nx, ny, nz, g, elems, pb, d_out); break;
    case LAYOUT_COL48: hipLaunchKernelGGL(k_build_layout<LAYOUT_COL48>, gr, b, 0, s, d_planar, nx, ny, nz, g, elems, pb, d_out); break;
    case LAYOUT_BRICK41616: hipLaunchKernelGGL(k_build_layout<LAYOUT_BRICK41616>, gr, b, 0, s, d_planar, nx, ny, nz, g, elems, pb, d_out); break;
    case LAYOUT_ZPAIR: hipLaunchKernelGGL(k_build_layout<LAYOUT_ZPAIR>, gr, b, 0, s, d_planar, nx, ny, nz, g, elems, pb, d_out); break;
    case LAYOUT_CORNER8: hipLaunchKernelGGL(k_build_layout<LAYOUT_CORNER8>, gr, b, 0, s, d_planar, nx, ny, nz, g, elems, pb, d_out); break;
    case LAYOUT_CORNERH: hipLaunchKernelGGL(k_build_layout<LAYOUT_CORNERH>, gr, b, 0, s, d_planar, nx, ny, nz, g, elems, pb, d_out); break;
    default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

hipError_t launch_unpack(const uint8_t* d_planar, int nx, int ny, int nz, uint8_t* d_rgba, hipStream_t s)
{
    const long long total = (long long)nx * ny * nz;
    hipLaunchKernelGGL(k_unpack_planar, dim3(grid_for(total)), dim3(kBlock), 0, s, d_planar, total,
                       reinterpret_cast<uchar4*>(d_rgba));
    return hipGetLastError();
}

int noise_partials_needed(int nx, int ny, int nz) { return grid_for((long long)nx * ny * nz); }

hipError_t launch_noise(int kind, float* d_out, int x0, int y0, int z0, int nx, int ny, int nz, float freq,
                        int32_t seed, float* d_partials, int* num_partials, hipStream_t s)
{
    const int g = grid_for((long long)nx * ny * nz);
    *num_partials = g;
    // k_noise strides a 32-bit index by gridDim * kBlock (<= 4096 * kBlock): a
    // total within one stride of 2^32 would wrap it and loop forever
    if ((long long)nx * ny * nz > (1ll << 32) - 4096ll * kBlock) return hipErrorInvalidValue;
    // cellular: the cell range the grid's coordinates (start + i) * freq can
    // reach, +-1 neighbour and a cell of margin for rint (cellular_table)
    int lo = 0, n = 0;
    if (kind == 0) {
        double cmin = 0.0, cmax = 0.0;
        bool first = true;
        for (int ax = 0; ax < 3; ++ax) {
            const int o = ax == 0 ? x0 : ax == 1 ? y0 : z0, m = ax == 0 ? nx : ax == 1 ? ny : nz;
            for (const int e : {o, o + m - 1}) {
                const double c = (double)(float)((float)e * freq);
                cmin = first ? c : std::min(cmin, c);
                cmax = first ? c : std::max(cmax, c);
                first = false;
            }
        }
        if (std::isfinite(cmin) && std::isfinite(cmax) && cmax - cmin < 64.0) {
            lo = (int)std::floor(cmin) - 2;
            n = (int)std::ceil(cmax) + 2 - lo + 1;
            if (n > kNoiseTableMaxN) n = 0;
        }
    }
    const size_t lds = (size_t)n * n * n * sizeof(float4);
    hipLaunchKernelGGL(k_noise, dim3(g), dim3(kBlock), lds, s, kind, d_out, x0, y0, z0, nx, ny, nz, freq, seed, lo, n,
                       reinterpret_cast<float2*>(d_partials));
    return hipGetLastError();
}

__global__ __launch_bounds__(kBlock) void k_perlin_lattice(uint2* __restrict__ out, int seed, int lo, int n)
{
    const long long total = (long long)n * n * n;
    for (long long i = (long long)blockIdx.x * kBlock + threadIdx.x; i < total; i += (long long)gridDim.x * kBlock) {
        const int ix = (int)(i % n), iy = (int)((i / n) % n), iz = (int)(i / ((long long)n * n));
        out[i] = noise::perlin_lattice_entry(seed, lo + ix, lo + iy, lo + iz);
    }
}

hipError_t launch_perlin_lattice(uint2* d_out, int seed, int lo, int n, hipStream_t s)
{
    const long long total = (long long)n * n * n;
    const long long blocks = std::min<long long>((total + kBlock - 1) / kBlock, 8192);
    hipLaunchKernelGGL(k_perlin_lattice, dim3((unsigned)blocks), dim3(kBlock), 0, s, d_out, seed, lo, n);
    return hipGetLastError();
}

hipError_t launch_minmax_reduce(const float* d_partials, int num_partials, float* d_minmax, hipStream_t s)
{
    hipLaunchKernelGGL(k_minmax, dim3(1), dim3(kBlock), 0, s, reinterpret_cast<const float2*>(d_partials),
                       num_partials, d_minmax);
    return hipGetLastError();
}

hipError_t launch_pack_recipe(const float* d_g1, const float* d_g2, const float* d_g3, const float* d_g4,
                              const float* d_minmax, long long total, uint8_t* d_rgba, hipStream_t s)
{
    hipLaunchKernelGGL(k_pack_recipe, dim3(grid_for(total)), dim3(kBlock), 0, s, d_g1, d_g2, d_g3, d_g4,
                       d_minmax, total, reinterpret_cast<uchar4*>(d_rgba));
    return hipGetLastError();
}

// Streaming kernels for the measured HBM roofline (vr_measure_bandwidth):
// 16 B per lane, one pass over the buffer, the grid as large as the buffer
// (each workgroup owns PL x 256 x 16 B; a persistent 2,048-workgroup
// grid-stride loop read 4.6-4.7 TB/s).  PL independent loads per lane are
// issued before anything consumes them.
//  * copy: the float4 copy of MI355X_MICROARCH.md's measured HBM rate
//    (counted as 2 x bytes moved);
//  * read: loads only, folded into one register per lane (xor), which is
//    stored only if it equals a value the 0x5a fill never produces -- every
//    lane's loads stay live, nothing is written.  The ray march is 98 % reads
//    (profiles/traffic.json), so this is its roofline denominator.
template <int PL>
__global__ __launch_bounds__(256) void k_stream_copy(const uint4* __restrict__ src, uint4* __restrict__ dst,
                                                     long long n)
{
    const long long base = (long long)blockIdx.x * (256 * PL) + threadIdx.x;
    uint4 v[PL];
#pragma unroll
    for (int k = 0; k < PL; ++k)
        if (base + k * 256 < n) v[k] = src[base + k * 256];
#pragma unroll
    for (int k = 0; k < PL; ++k)
        if (base + k * 256 < n) dst[base + k * 256] = v[k];
}

constexpr unsigned kReadSinkMagic = 0x9e3779b9u;

template <int PL>
__global__ __launch_bounds__(256) void k_stream_read(const uint4* __restrict__ src, unsigned* __restrict__ sink,
                                                     long long n)
{
    const long long base = (long long)blockIdx.x * (256 * PL) + threadIdx.x;
    uint4 v[PL];
#pragma unroll
    for (int k = 0; k < PL; ++k) v[k] = base + k * 256 < n ? src[base + k * 256] : make_uint4(0u, 0u, 0u, 0u);
    unsigned x = 0u;
#pragma unroll
    for (int k = 0; k < PL; ++k) x ^= (v[k].x ^ v[k].y) ^ (v[k].z ^ v[k].w);
    if (x == kReadSinkMagic) sink[threadIdx.x] = x;   // never taken for the 0x5a fill
}

template <int PL>
static hipError_t launch_stream_pl(int kind, const void* src, void* dst, long long n, hipStream_t s)
{
    const long long blocks = (n + 256 * PL - 1) / (256 * PL);
    if (blocks <= 0) return hipSuccess;
    if (blocks > 0x7fffffffLL) return hipErrorInvalidValue;
    if (kind == 0)
        hipLaunchKernelGGL(k_stream_copy<PL>, dim3((unsigned)blocks), dim3(256), 0, s, static_cast<const uint4*>(src),
                           static_cast<uint4*>(dst), n);
    else
        hipLaunchKernelGGL(k_stream_read<PL>, dim3((unsigned)blocks), dim3(256), 0, s, static_cast<const uint4*>(src),
                           static_cast<unsigned*>(dst), n);
    return hipGetLastError();
}

hipError_t launch_stream_bw(int kind, int loads_per_lane, const void* src, void* dst, size_t bytes, hipStream_t s)
{
    const long long n = (long long)(bytes / 16);
    switch (loads_per_lane) {
    case 4: return launch_stream_pl<4>(kind, src, dst, n, s);
    case 8: return launch_stream_pl<8>(kind, src, dst, n, s);
    case 16: return launch_stream_pl<16>(kind, src, dst, n, s);
    default: return hipErrorInvalidValue;
    }
}

hipError_t launch_stream_copy(const void* src, void* dst, size_t bytes, hipStream_t s)
{
    return launch_stream_bw(0, 4, src, dst, bytes, s);
}

hipError_t launch_assemble(const uint8_t* d_gathered, size_t rows_per_rank, int nranks, int width, int height,
                           int band_rows, int bpp, int first_rank, uint8_t* d_frame, hipStream_t s, bool serp)
{
    const long long row_bytes = (long long)width * bpp;
    if (row_bytes % 16 == 0) {
        const int elems = (int)(row_bytes / 16);
        hipLaunchKernelGGL(k_assemble<uint4>, grid_rows(rows_per_rank, nranks, first_rank, elems), dim3(kBlock), 0, s,
                           reinterpret_cast<const uint4*>(d_gathered), (int)rows_per_rank, nranks, elems,
                           height, band_rows, first_rank, (int)serp, reinterpret_cast<uint4*>(d_frame));
    } else if (row_bytes % 4 == 0) {
        const int elems = (int)(row_bytes / 4);
        hipLaunchKernelGGL(k_assemble<unsigned int>, grid_rows(rows_per_rank, nranks, first_rank, elems), dim3(kBlock), 0,
                           s, reinterpret_cast<const unsigned int*>(d_gathered), (int)rows_per_rank, nranks,
                           elems, height, band_rows, first_rank, (int)serp, reinterpret_cast<unsigned int*>(d_frame));
    } else {   // 1-byte pixels, rows of any width
        const int elems = (int)row_bytes;
        hipLaunchKernelGGL(k_assemble<unsigned char>, grid_rows(rows_per_rank, nranks, first_rank, elems), dim3(kBlock), 0,
                           s, d_gathered, (int)rows_per_rank, nranks, elems, height, band_rows, first_rank, (int)serp,
                           d_frame);
    }
    return hipGetLastError();
}

hipError_t launch_assemble_grey(const uint8_t* d_gathered, size_t rows_per_rank, int nranks, int width, int height,
                                int band_rows, bool f32, int first_rank, uint8_t* d_frame, hipStream_t s, bool serp)
{
    const dim3 blk(kBlock);
    if (f32) {
        hipLaunchKernelGGL((k_assemble_grey<float, float4>), grid_rows(rows_per_rank, nranks, first_rank, width), blk, 0, s,
                           reinterpret_cast<const float*>(d_gathered), (int)rows_per_rank, nranks, width, height,
                           band_rows, first_rank, (int)serp, reinterpret_cast<float4*>(d_frame));
    } else if (width % 4 == 0) {
        const int elems = width / 4;
        hipLaunchKernelGGL((k_assemble_grey<unsigned int, uint4>), grid_rows(rows_per_rank, nranks, first_rank, elems), blk, 0,
                           s, reinterpret_cast<const unsigned int*>(d_gathered), (int)rows_per_rank, nranks,
                           elems, height, band_rows, first_rank, (int)serp, reinterpret_cast<uint4*>(d_frame));
    } else {
        hipLaunchKernelGGL((k_assemble_grey<unsigned char, unsigned int>), grid_rows(rows_per_rank, nranks, first_rank, width),
                           blk, 0, s, d_gathered, (int)rows_per_rank, nranks, width, height, band_rows, first_rank, (int)serp,
                           reinterpret_cast<unsigned int*>(d_frame));
    }
    return hipGetLastError();
}

// ---- self tests (vr_selftest) ----
namespace {
__global__ __launch_bounds__(256) void k_selftest_cell_inv(int variant, unsigned long long* __restrict__ bad)
{
    constexpr unsigned kMaxK = 3u * 1023u * 1023u;
    const unsigned i = blockIdx.x * 256u + threadIdx.x;
    const unsigned K = 8u * i + 3u;
    unsigned miss = 0;
    if (K <= kMaxK) {
        const float d2 = (float)K * 0.25f;
        const float want = noise::cell_inv_ieee(d2);
        const float got = variant == 0 ? noise::cell_inv_a(d2) : variant == 1 ? noise::cell_inv_b(d2)
                        : variant == 2 ? noise::cell_inv_c(d2) : noise::cell_inv(d2);
        miss = __float_as_uint(got) != __float_as_uint(want);
    }
    unsigned long long c = miss;
    for (int off = 32; off > 0; off >>= 1) c += __shfl_xor(c, off);
    if ((threadIdx.x & 63) == 0 && c) atomicAdd(bad, c);
}
}  // namespace

// Worley pruning (noise::cellular_table9) against the unpruned cellular():
// bit-equal F1 on points drawn uniformly and at the edge cases of the bound
// -- coordinates a few ulps around half-integers (the rint switch) and
// integers (the floor switch), and points next to a feature point (F1 ~ 0)
// or between two (near ties).  The table is the march's, cells [0, 9)^3
// with z pitch 83; points keep rint +- 1 inside it.
constexpr int kWorleyTestBlocks = 2048, kWorleyTestPerThread = 16;
__global__ __launch_bounds__(256) void k_selftest_worley(int seed, unsigned long long* __restrict__ bad)
{
    __shared__ float4 tab[noise::kWorleyN * noise::kWorleyPz];
    for (int i = threadIdx.x; i < noise::kWorleyN * noise::kWorleyN * noise::kWorleyN; i += 256) {
        const int ix = i % noise::kWorleyN, iy = (i / noise::kWorleyN) % noise::kWorleyN, iz = i / (noise::kWorleyN * noise::kWorleyN);
        tab[iz * noise::kWorleyPz + iy * noise::kWorleyN + ix] = noise::cellular_cell(seed, ix, iy, iz);
    }
    __syncthreads();
    unsigned miss = 0;
    for (int j = 0; j < kWorleyTestPerThread; ++j) {
        const unsigned id = (blockIdx.x * 256u + threadIdx.x) * kWorleyTestPerThread + (unsigned)j;
        unsigned h = id * 0x9E3779B1u + 0x85EBCA77u;
        auto next = [&h]() { h ^= h >> 15; h *= 0x2C1B3C6Du; h ^= h >> 12; h *= 0x297A2D39u; h ^= h >> 15; return h; };
        auto unit = [&]() { return (float)(next() >> 8) * (1.0f / 16777216.0f); };   // [0, 1)
        float c[3];
        const unsigned kind = id % 5u;
        for (int a = 0; a < 3; ++a) c[a] = 1.0f + 6.0f * unit();   // [1, 7)
        if (kind == 1 || kind == 2) {
            // a few ulps around k + 0.5 (rint) or k (floor) on a random subset of axes
            for (int a = 0; a < 3; ++a) {
                if (next() & 1u) continue;
                const float k = (float)(1 + (int)(next() % 6u)) + (kind == 1 ? 0.5f : 0.0f);
                const int ulps = (int)(next() % 7u) - 3;
                c[a] = __int_as_float(__float_as_int(k) + ulps);
            }
        } else if (kind == 3 || kind == 4) {
            // next to a feature point (3), or between two neighbouring ones (4)
            const int cx = 2 + (int)(next() % 5u), cy = 2 + (int)(next() % 5u), cz = 2 + (int)(next() % 5u);
            const float4 f = tab[cz * noise::kWorleyPz + cy * noise::kWorleyN + cx];
            float p[3] = {fmaf(f.x, f.w, (float)cx), fmaf(f.y, f.w, (float)cy), fmaf(f.z, f.w, (float)cz)};
            if (kind == 4) {
                const int a = (int)(next() % 3u);
                const int dx = a == 0, dy = a == 1, dz = a == 2;
                const float4 g = tab[(cz + dz) * noise::kWorleyPz + (cy + dy) * noise::kWorleyN + cx + dx];
                const float q[3] = {fmaf(g.x, g.w, (float)(cx + dx)), fmaf(g.y, g.w, (float)(cy + dy)), fmaf(g.z, g.w, (float)(cz + dz))};
                for (int b = 0; b < 3; ++b) p[b] = 0.5f * (p[b] + q[b]);
            }
            const float r = kind == 3 ? 1e-3f : 1e-5f;
            for (int b = 0; b < 3; ++b) c[b] = fminf(fmaxf(p[b] + r * (2.0f * unit() - 1.0f), 0.51f), 7.49f);
        }
        bool full;
        const float got = noise::cellular_table9(tab, noise::worley9_nc(0), c[0], c[1], c[2], full);
        const float want = noise::cellular(seed, c[0], c[1], c[2]);
        miss += __float_as_uint(got) != __float_as_uint(want);
    }
    unsigned long long cnt = miss;
    for (int off = 32; off > 0; off >>= 1) cnt += __shfl_xor(cnt, off);
    if ((threadIdx.x & 63) == 0 && cnt) atomicAdd(bad, cnt);
}

hipError_t launch_selftest_worley(int seed, unsigned long long* d_bad, hipStream_t s)
{
    hipLaunchKernelGGL(k_selftest_worley, dim3(kWorleyTestBlocks), dim3(256), 0, s, seed, d_bad);
    return hipGetLastError();
}

hipError_t launch_selftest_cell_inv(int variant, unsigned long long* d_bad, hipStream_t s)
{
    constexpr unsigned kCount = (3u * 1023u * 1023u - 3u) / 8u + 1u;
    hipLaunchKernelGGL(k_selftest_cell_inv, dim3((kCount + 255) / 256), dim3(256), 0, s, variant, d_bad);
    return hipGetLastError();
}

}  // namespace vr
