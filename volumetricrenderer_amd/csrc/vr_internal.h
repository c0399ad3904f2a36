// vr_internal.h -- internal structures shared by the HIP kernels and the C ABI
// (not installed; the public interface is include/vr.h).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stddef.h>

namespace vr {

// Volume layouts in HBM.  Each keeps one array per
// channel, so a tap reads only the channel it needs (frag.glsl:66-69 read
// .x, .y, .z, .w at four different coordinates).
//
// LAYOUT_PLANAR is the canonical copy and the source of every other layout.
// It is u8 plane[z][y][x], takes any wrap mode, and does 8 byte loads per tap.
//
// The fast layouts are indexed by the *padded* base texel a = floor(g), with
// g = u*N + 0.5 and a in [0, N].  They store the clamp-to-edge values of the
// 2x2x2 trilinear footprint, so a tap needs no index wrapping.  They are
// exact wherever clamp-to-edge equals mirrored repeat.  The host checks that
// per frame; otherwise LAYOUT_PLANAR runs.  A tap's byte offset is
// TX[a] + TY[b] + TZ[c], from three per-axis tables the kernel keeps in LDS,
// so the brick geometry costs two adds per tap.
enum Layout : int {
    LAYOUT_PLANAR = 1,
    LAYOUT_BRICK5 = 2,    // B=4: 4^3 texels + 1-texel apron = 5^3 B in one 128-B
                          // line (2.0x bytes); a footprint never leaves its line
    LAYOUT_BRICK8 = 3,    // B=7: 8^3 = 512 B bricks (1.49x bytes)
    LAYOUT_BRICK16 = 4,   // B=15: 16^3 = 4 KiB bricks (1.21x bytes)
    LAYOUT_CORNER8 = 5,   // per base texel its 8 footprint bytes (u64) in 4^3
                          // position bricks of 512 B (8x bytes); 1 load per tap
    LAYOUT_BRICK4 = 6,    // B=3: 3^3 texels + apron = 4^3 = 64 B (2.37x bytes);
                          // a z-slice of a footprint is one dword-aligned 8-B load
    LAYOUT_ZPAIR = 7,     // 4x16x2 texels = 128 B (3x15x1 positions, 2.93x bytes),
                          // 4-byte rows ordered z-fastest: rows (y,z) (y,z+1)
                          // (y+1,z) (y+1,z+1) are 16 contiguous bytes, so a whole
                          // footprint is one dword-aligned 16-B load
    LAYOUT_BRICK448 = 8,  // 4x4x8 texels = 128 B (3x3x7 positions, 2.03x bytes);
                          // BRICK4's in-brick order, so the same two 8-B loads
    LAYOUT_BRICK488 = 9,  // 4x8x8 texels = 256 B (3x7x7 positions, 1.74x bytes);
                          // slices 32 B apart
    LAYOUT_BRICK4816 = 10,   // 4x8x16 texels = 512 B (3x7x15 positions, 1.60x bytes)
    LAYOUT_BRICK41616 = 11,  // 4x16x16 texels = 1 KiB (3x15x15 positions, 1.52x
                             // bytes); slices 64 B apart
    LAYOUT_BRICK4832 = 12,   // 4x8x32 texels = 1 KiB (3x7x31 positions, 1.53x bytes)
    LAYOUT_BRICK4864 = 13,   // 4x8x64 texels = 2 KiB (3x7x63 positions, 1.51x bytes)
    LAYOUT_CORNERH = 14,     // per base position 16 B: for each footprint row (y,z)
                             // the f16 pair {a, b - a} of its x-neighbours a, b, so
                             // each x-lerp is one v_fma_mix_f32; x fastest, no
                             // bricks: the index is computed in fp32 (16x bytes)
    LAYOUT_COL48 = 15,       // columns of 4x8 texels (3x7 positions) through the whole
                             // z extent, slices 32 B apart (1.52x bytes): BRICK4832
                             // without z bricks, so any run of slices of a column is
                             // contiguous -- the fill unit of the LDS slab march
                             // (vr_march_slab.hip); also a plain BRICK4-family layout
    LAYOUT_COL48Z = 16,      // channels 0-2 as COL48, channel 3 as ZPAIR (one 16-B load per
                             // tap): the reference's smallest-scale tap (A at 0.7,
                             // frag.glsl:69) trades 1.9x its bytes for half its loads
};
constexpr int kNumLayouts = 17;
// CORNERH's fp32 index a + (nx+1)(b + (ny+1)c) is exact below 2^24 positions
constexpr long long kCornerHMaxPositions = 1ll << 24;
// the layouts whose taps are BRICK4's two dword-aligned 8-B loads
__host__ __device__ constexpr bool is_b4_family(int l)
{
    return l == LAYOUT_BRICK4 || l == LAYOUT_BRICK448 || l == LAYOUT_BRICK488 || l == LAYOUT_BRICK4816 ||
           l == LAYOUT_BRICK41616 || l == LAYOUT_BRICK4832 ||
           l == LAYOUT_BRICK4864 || l == LAYOUT_COL48;
}

// Variants measured slower than the defaults and kept as the record of that
// (DESIGN.md sec. 4, 5.1-5.4): the layouts other than the auto ones, the
// queue / strided / XCD-row schedules, 8- and 16-wave workgroups, and the
// procedural sort_reuse / proc_enum options.  They are compiled only with
// VR_EXPERIMENTS=1 (make EXPERIMENTS=1); the default library refuses their
// options.  The LDS slab march (north star; option slab, off by default) is
// in every build so that its parity test runs in the default GPU suite.
#ifndef VR_EXPERIMENTS
#define VR_EXPERIMENTS 0
#endif
__host__ __device__ constexpr bool layout_built(int l)
{
    return VR_EXPERIMENTS || l == LAYOUT_PLANAR || l == LAYOUT_CORNER8 || l == LAYOUT_CORNERH || l == LAYOUT_COL48 ||
           l == LAYOUT_BRICK4832;
}

enum Wrap : int { WRAP_CLAMP = 0, WRAP_MIRROR = 1 };

// Geometry of a fast layout for one channel (host and device).
struct LayoutGeom {
    int B;          // useful positions per brick edge (cubic layouts)
    int R;          // stored edge of an apron brick, R = B + 1
    int Ba[3];      // useful positions per brick along x, y, z
    int Rn[3];      // stored texels per brick along x, y, z (in-brick order x fastest)
    unsigned brick; // bytes per brick
    int nbx, nby, nbz;
};
__host__ __device__ inline LayoutGeom layout_geom(int layout, int nx, int ny, int nz)
{
    LayoutGeom g{};
    if (layout == LAYOUT_CORNER8) {
        g.B = 4; g.R = 4; g.brick = 512;
    } else if (layout == LAYOUT_CORNERH) {
        g.B = 1; g.R = 1; g.brick = 16;
    } else if (layout == LAYOUT_ZPAIR) {
        g.B = 3; g.R = 4; g.brick = 128;
    } else if (layout == LAYOUT_COL48 || layout == LAYOUT_COL48Z) {
        // slices c and c + 1 for every padded position c in [0, nz]: nz + 2
        // slices, rounded up to an even count (64-B chunks of two slices)
        g.B = 3; g.R = 4;
        g.brick = 32u * (unsigned)((nz + 3) & ~1);
    } else if (layout == LAYOUT_BRICK448 || layout == LAYOUT_BRICK488 || layout == LAYOUT_BRICK4816 ||
               layout == LAYOUT_BRICK41616 || layout == LAYOUT_BRICK4832 || layout == LAYOUT_BRICK4864) {
        g.B = 3; g.R = 4;
        g.brick = layout == LAYOUT_BRICK448 ? 128u : layout == LAYOUT_BRICK488 ? 256u
                : layout == LAYOUT_BRICK4816 ? 512u : layout == LAYOUT_BRICK4864 ? 2048u : 1024u;
    } else {
        g.B = layout == LAYOUT_BRICK4 ? 3 : layout == LAYOUT_BRICK5 ? 4 : layout == LAYOUT_BRICK8 ? 7 : 15;
        g.R = g.B + 1;
        const unsigned r3 = (unsigned)(g.R * g.R * g.R);
        // whole 128-B lines; BRICK4's 64-B bricks pair up in one line
        g.brick = layout == LAYOUT_BRICK4 ? 64u : (r3 + 127u) & ~127u;
    }
    g.Ba[0] = g.Ba[1] = g.Ba[2] = g.B;
    g.Rn[0] = g.Rn[1] = g.Rn[2] = g.R;
    if (layout == LAYOUT_ZPAIR) { g.Ba[1] = 15; g.Ba[2] = 1; }
    if (layout == LAYOUT_BRICK448) { g.Ba[2] = 7; g.Rn[2] = 8; }
    if (layout == LAYOUT_BRICK488) { g.Ba[1] = g.Ba[2] = 7; g.Rn[1] = g.Rn[2] = 8; }
    if (layout == LAYOUT_BRICK4816) { g.Ba[1] = 7; g.Rn[1] = 8; g.Ba[2] = 15; g.Rn[2] = 16; }
    if (layout == LAYOUT_BRICK4864) { g.Ba[1] = 7; g.Rn[1] = 8; g.Ba[2] = 63; g.Rn[2] = 64; }
    if (layout == LAYOUT_BRICK4832) { g.Ba[1] = 7; g.Rn[1] = 8; g.Ba[2] = 31; g.Rn[2] = 32; }
    if (layout == LAYOUT_BRICK41616) { g.Ba[1] = g.Ba[2] = 15; g.Rn[1] = g.Rn[2] = 16; }
    if (layout == LAYOUT_COL48 || layout == LAYOUT_COL48Z) { g.Ba[1] = 7; g.Rn[1] = 8; g.Ba[2] = nz + 1; g.Rn[2] = (nz + 3) & ~1; }
    // padded base positions a in [0, N] -> bricks a / B in [0, N / B]
    g.nbx = nx / g.Ba[0] + 1;
    g.nby = ny / g.Ba[1] + 1;
    g.nbz = nz / g.Ba[2] + 1;
    return g;
}
// byte offset of padded position a along axis 0/1/2 inside one channel plane
__host__ __device__ inline unsigned axis_offset(const LayoutGeom& g, int layout, int axis, int a)
{
    const unsigned q = (unsigned)(a / g.Ba[axis]), r = (unsigned)(a % g.Ba[axis]);
    const unsigned stride = axis == 0 ? g.brick : axis == 1 ? g.brick * (unsigned)g.nbx
                                                            : g.brick * (unsigned)g.nbx * (unsigned)g.nby;
    if (layout == LAYOUT_CORNER8) return q * stride + (r << (3 + 2 * axis));   // 8 B per position
    if (layout == LAYOUT_ZPAIR) return q * stride + (axis == 0 ? r : axis == 1 ? 8u * r : 0u);
    return q * stride + r * (axis == 0 ? 1u : axis == 1 ? (unsigned)g.Rn[0] : (unsigned)(g.Rn[0] * g.Rn[1]));
}

// Procedural medium parameters (vr_procedural; BASELINE configs 2/3).
struct ProcParams {
    float grid_scale;
    int octaves;
    float freq0, lacunarity, gain;
    int seed_fbm;
    float worley_freq;
    int seed_worley;
    int shadow_steps;
    float lstep[3];   // (step_size * sun_dir) / box_range
    float od;         // step_size * density
    int count_evals;  // step_counter counts: 0 ray-steps, 1 density evaluations (incl. shadow
                      // samples), 2 Worley cells computed (8 or 35 per evaluation when pruned, else 27)
    int wt_lo, wt_n;  // Worley cell table in LDS: cells [wt_lo, wt_lo + wt_n)^3; wt_n = 0: none
    int wt_pz;        // its z pitch in entries (>= wt_n^2, padded against LDS bank aliasing)
    int wt_fixed;     // 1: the fixed geometry wt_n = 9, wt_pz = 83 (noise::cellular_table9)
    int enum_regions; // sort passes: 1 = 64x64-region enumeration also with shadow rays
    // Perlin lattice table (global, noise::perlin_lattice_entry): cells
    // [lat_lo, lat_lo + lat_n)^3, entry (x, y, z) at byte offset
    // 8 x + lat_sy y + lat_sz z - lat_c, all exact in fp32.  Null: none.
    const uint2* lat;
    unsigned lat_bytes;
    float lat_c, lat_sy, lat_sz;
};

// Everything one launch of the march kernel needs.  Passed by value
// (kernarg segment), computed on the host per vr_render call.
struct MarchArgs {
    // ray basis in box-local space: dir(x,y) = o + (x+.5)*px + (y+.5)*py
    float org[3], o[3], px[3], py[3];
    float r2[4], r3[4];          // rows 2/3 of P*V*M (coverage clip test)
    int cam_mode;                // 1: org/o/px/py are the View eye's, the march starts at cam (RayBasis)
    float cam[3];
    float box_min[3], box_max[3], box_range[3];
    float step_size, density, scale, acc_limit;
    int max_steps;
    // tap t samples padded texel coordinate g = fma(P, tap_S, tap_T)
    // (= u*N + 0.5 with u = P*s_t + o_t, frag.glsl:66-69)
    float tap_S[4][3], tap_T[4][3];
    int zero_offsets;            // every tap_T is exactly 0.5 (no MediaScroll offsets)
    // uniform channels (vr_api.cpp install_volume: min == max over the plane):
    // bit t set = every texel of channel t is v_t, so tap t is exactly
    // uval[t] = v_t * (1/255) (the spec's lerps of equal values return them,
    // DESIGN.md sec. 3.2) and the march needs no load for it
    int umask;
    float uval[4];
    // COL48Z: channel 3's ZPAIR plane (geometry, bytes) after the three COL48 planes
    LayoutGeom geom3;
    unsigned plane3_bytes;
    // volume
    int nx, ny, nz;
    const uint8_t* vol;          // channel plane 0; plane c at vol + c*plane_stride
    unsigned plane_stride;       // bytes (< 2^31)
    LayoutGeom geom;             // fast layouts
    // target
    int width, height, band_rows, band_stride, band_first, out_rows;
    int band_flip;               // vr_target.band_flip: odd bands of the set shifted (set_band)
    int tiles_x, tiles_y, num_blocks;   // static schedule: 16x16 tiles
    void* out;
    long long pitch;
    int format;
    int empty_fill;              // regions lists: march each XCD's first hdr[kRegionWork + x] entries, fill the
                                 // rest (tiles no ray of which meets the box) with the uncovered value
    int bands_in_place;          // vr.h VR_TARGET_BANDS_IN_PLACE: packed row orow is stored at its frame row
    unsigned long long* step_counter;
    ProcParams proc;
    int slab_cap;                // LDS slab march (COL48): chunks per channel the slab holds
};

// The frame band of a band set's k-th band (vr_target): band_first + k *
// band_stride, every odd one shifted by band_flip (the serpentine deal)
__host__ __device__ inline int set_band(int k, int first, int stride, int flip)
{
    return first + k * stride + ((k & 1) ? flip : 0);
}

// How the march kernel maps tiles to waves.
enum ScheduleKind : int {
    SCHED_STATIC = 0, SCHED_QUEUE = 1, SCHED_STRIDED = 2, SCHED_XCDROWS = 3, SCHED_RINGS = 4, SCHED_REGIONS = 5
};
// Regions schedule: XCD x (blockIdx % 8) renders the 8x8 tiles
// tiles[off[x] .. off[x+1]) (packed ty << 16 | tx), wave w of its nwx waves
// the tiles w, w + nwx, ...  Built on the host (vr_api.cpp build_regions).
struct TileMap {
    int off[9];
    int nwx;
};
// The regions schedule's lists in device memory: a header of kRegionHeader
// ints, then the list entries.  The header:
//   [0..8]   off[]: XCD x renders the entries [off[x], off[x+1])
//   [9]      tiles with estimated work    [10] the longest list
//   [11]     entries
//   [16..23] marched tiles of XCD x (kRegionWork): its list holds the tiles
//            with estimated work, then the other tiles some ray of which may
//            meet the box, then the empty ones (tile_is_empty) -- those last
//            are written with the uncovered value, not marched
// Built on the host (vr_api.cpp build_regions) or, for a moving camera, on
// the GPU (vr_regions.hip launch_region_build, the same dealing).
constexpr int kRegionHeader = 24;
constexpr int kRegionWork = 16;
struct RegionBuild {
    int tw, th, width, out_rows, band_rows, band_stride, band_first, max_steps;
    int height, band_flip;
    float step_size;
    float org[3], o[3], px[3], py[3], box_min[3], box_max[3];
    float r3[4];           // row 3 of P*V*M (clip w), for tile_is_empty
    double ccx, ccy;       // box-centre tile (fractional), S x S block of it
    int ctx, cty;
    int supertile, wedges;
    int order;             // option region_order: 0 inside-out, 1 longest tile first, 2 longest S x S block first
};
// True when no ray of tile (tx, ty) of the target can be covered (setup_ray,
// vr_march_kernels.h), so the march would write the uncovered value at every
// pixel of it.  Conservative, in double: the box lies wholly in front of the
// camera (clip w > 0 at its 8 corners: no line through the eye meets it
// behind), and one side plane of the tile's frustum -- through the eye and
// two corner rays of the tile's pixel-edge rectangle, half a pixel outside
// every pixel centre -- has all 8 box corners strictly outside.  The pixel
// centre rays then pass half a pixel or more from any point of the box; the
// fp32 ray setup cannot close that.  Tiles whose rows span two bands (band
// rows not a multiple of 8) are never empty.  Host and GPU list builds.
__host__ __device__ inline bool tile_is_empty(const float org[3], const float o[3], const float px[3], const float py[3],
                                              const float bmin[3], const float bmax[3], const float r3[4], int width,
                                              int out_rows, int height, int band_rows, int band_stride, int band_first,
                                              int band_flip, int tx, int ty)
{
    if (band_rows > 0 && band_rows % 8 != 0) return false;
    const int x0 = tx * 8, x1 = x0 + 8 < width ? x0 + 8 : width;
    const int r0 = ty * 8, rows = r0 + 8 < out_rows ? 8 : out_rows - r0;
    if (x1 <= x0 || rows <= 0) return true;   // no pixels
    int y0 = r0;
    if (band_rows > 0) {
        const int bl = r0 / band_rows;
        y0 = set_band(bl, band_first, band_stride, band_flip) * band_rows + (r0 - bl * band_rows);
    }
    if (y0 >= height) return true;   // rows past the frame: never stored
    double c[8][3];
    for (int k = 0; k < 8; ++k) {
        c[k][0] = (double)((k & 1) ? bmax[0] : bmin[0]) - (double)org[0];
        c[k][1] = (double)((k & 2) ? bmax[1] : bmin[1]) - (double)org[1];
        c[k][2] = (double)((k & 4) ? bmax[2] : bmin[2]) - (double)org[2];
        const double w = (double)r3[0] * (c[k][0] + (double)org[0]) + (double)r3[1] * (c[k][1] + (double)org[1]) +
                         (double)r3[2] * (c[k][2] + (double)org[2]) + (double)r3[3];
        if (!(w > 1e-6)) return false;   // some of the box at or behind the eye
    }
    const double fxs[4] = {(double)x0, (double)x1, (double)x1, (double)x0};
    const double fys[4] = {(double)y0, (double)y0, (double)(y0 + rows), (double)(y0 + rows)};
    double d[4][3], m[3];
    for (int j = 0; j < 3; ++j)
        m[j] = (double)o[j] + 0.5 * (x0 + x1) * (double)px[j] + (y0 + 0.5 * rows) * (double)py[j];
    for (int i = 0; i < 4; ++i)
        for (int j = 0; j < 3; ++j) d[i][j] = (double)o[j] + fxs[i] * (double)px[j] + fys[i] * (double)py[j];
    for (int i = 0; i < 4; ++i) {
        const double* a = d[i];
        const double* b = d[(i + 1) & 3];
        double n[3] = {a[1] * b[2] - a[2] * b[1], a[2] * b[0] - a[0] * b[2], a[0] * b[1] - a[1] * b[0]};
        const double sm = n[0] * m[0] + n[1] * m[1] + n[2] * m[2];
        if (sm == 0.0) continue;
        if (sm > 0.0) { n[0] = -n[0]; n[1] = -n[1]; n[2] = -n[2]; }   // outward: away from the tile's centre ray
        const double nn = sqrt(n[0] * n[0] + n[1] * n[1] + n[2] * n[2]);
        bool out = true;
        for (int k = 0; k < 8 && out; ++k) {
            const double cl = sqrt(c[k][0] * c[k][0] + c[k][1] * c[k][1] + c[k][2] * c[k][2]);
            out = n[0] * c[k][0] + n[1] * c[k][1] + n[2] * c[k][2] > 1e-9 * nn * cl;
        }
        if (out) return true;
    }
    return false;
}
size_t region_build_bytes(int ntiles);
hipError_t region_build_preload();   // load the build's code object (first host build, once)
// h_hdr (optional, host-mapped): a copy of the header, for sizing later launches
hipError_t launch_region_build(const RegionBuild& b, void* scratch, unsigned* d_list, int* d_hdr, int* h_hdr,
                               hipStream_t s);

struct Schedule {
    int kind;
    int center_x, center_y;   // rings: target pixel under the projected box centre
    int tiles_per_wave;    // strided: 8x8 tiles per wave
    int waves_per_simd;    // queue: persistent waves per SIMD (grid = 256 CUs x this)
    int* heads;            // queue: 8 device ints, zeroed before each launch
    const unsigned* tiles; // regions: device tile lists
    TileMap map;           // regions (nwx counts waves of split units)
    int split;             // regions: lanes per ray (1, 2, 4, 8; BRICK4 / CORNER8 only)
    int slab;              // regions + COL48: the LDS slab march (vr_march_slab.hip)
    int wg_waves;          // regions (one lane per ray): waves per workgroup, 4 (default), 8 or 16
    const int* hdr;        // regions: the lists' device header (kRegionHeader; off[x] per XCD)
};

// Cost-sort scratch of the procedural march (vr_march.hip launch_march_procedural),
// byte offsets for a target of width x out_rows: the key histogram, the bin
// cursors, the sorted order, the keys per enumerated position, and for the
// deferred shadow passes the per-sorted-wave first entry / first step record
// (proc_scan; waves + 1 entries each) and the frame's totals (need[0] entries,
// need[1] step records).
struct SortLayout {
    size_t hist, cursor, order, keys, went, wrec, need, bytes;
    unsigned waves;   // sorted waves a frame can have: ceil(pixels / 64)
};
SortLayout sort_layout(int width, int out_rows);

// Deferred shadow rays (vr_march_kernels.h march_proc_defer): device scratch,
// sized from the frame (vr_api.cpp ensure_defer).  Sorted wave w appends at most
// went[w + 1] - went[w] entries (the sum of its lanes' step counts, bounded by
// their cost keys) and marches at most wrec[w + 1] - wrec[w] wave-steps (its
// first lane's key); proc_scan computes both prefixes from the cost histogram.
// A wave whose range lies beyond the capacities marches its shadow rays in
// place (march_pixel_proc) and is skipped by the later passes, so any capacity
// gives the exact frame.
struct ShadowDefer {
    unsigned* count;      // [0]: chunks of 64 entries this frame (written by proc_shadow_scan)
    unsigned* wsteps;     // per sorted wave: wave-steps marched; kDeferInPlace = its shadow rays were marched in place
    unsigned* wcount;     // per sorted wave: entries appended (dense from went[w])
    unsigned* wchunk;     // per sorted wave: its first chunk (exclusive prefix of ceil(wcount / 64))
    uint4* map;           // per chunk: {index of its first entry, 0, entries in it, 0}
    uint4* rec;           // step records {wave-local first entry, lane mask lo, hi, 0}, wave w's from wrec[w]
    float4* ent;          // entries (P, coef), wave w's from went[w]; pass 2 rewrites .xy as (coef, tl)
    const unsigned long long* went;   // sort buffer (SortLayout::went)
    const unsigned* wrec;             // sort buffer (SortLayout::wrec)
    unsigned long long ent_cap;       // entries the scratch holds (< 2^32)
    unsigned rec_cap;                 // step records it holds
    unsigned map_cap;                 // chunk map entries (ent_cap / 64 + waves)
    unsigned waves;                   // sorted waves the per-wave arrays hold
    unsigned eval_blocks;             // workgroups of the shadow pass (0 = kShadowEvalBlocks)
    int worley_cache;                 // shadow pass: keep each lane's Worley cube in registers (option shadow_cache)
};
constexpr unsigned kDeferInPlace = 0xffffffffu;

// launchers (vr_march.hip / vr_volume.hip); return hipError_t
hipError_t launch_march(const MarchArgs& a, int layout, int wrap, bool early, const Schedule& sc, hipStream_t s);
// per-plane byte min (mm[0..3]) and max (mm[4..7]) of the planar volume; mm
// must hold 0xffffffff x 4 then 0 x 4 (atomicMin / atomicMax)
hipError_t launch_plane_minmax(const uint8_t* d_planar, long long total, unsigned* mm, hipStream_t s);
// bytes per pixel of a vr_format (include/vr.h), and the grey format of an RGBA one
__host__ __device__ constexpr int format_bytes(int f) { return f == 0 ? 16 : f <= 2 ? 4 : f <= 4 ? 1 : 4; }
__host__ __device__ constexpr int grey_of(int f) { return f == 0 ? 5 : f == 1 ? 3 : f == 2 ? 4 : -1; }
// grey band sets (1 B or fp32 per pixel) -> RGBA frame rows (vr_assemble_frame)
hipError_t launch_assemble_grey(const uint8_t* d_gathered, size_t rows_per_rank, int nranks, int width, int height,
                                int band_rows, bool f32, int first_rank, uint8_t* d_frame, hipStream_t s,
                                bool serp = false);
hipError_t launch_march_corner8(const MarchArgs& a, int layout, bool early, const Schedule& sc,
                                hipStream_t s);   // CORNER8 / CORNERH, vr_march_c8.hip
hipError_t launch_march_slab(const MarchArgs& a, bool early, const Schedule& sc, hipStream_t s);   // vr_march_slab.hip
constexpr int kSlabMaxChunks = 32;   // per channel and wave (64 B each): 8 KiB of LDS per wave
// sort_buf (sort_layout) selects the cost-sorted schedule; null = 8x8
// tiles, in rings when sc.kind == SCHED_RINGS, else in row order
// reuse_sort (vr_api.cpp sort key): SORT_BUILD = sort this frame; SORT_REUSE =
// sort_buf holds the order of a frame with the same geometry (skip the sort
// passes, write the background only); SORT_STALE = the order of an older camera
// with the same target (skip the sort passes, march the pixels it left out too)
enum { SORT_BUILD = 0, SORT_REUSE = 1, SORT_STALE = 2 };
// need_host (optional, host-mapped, 2 entries): a frame that sorts with shadow rays
// writes there the deferred scratch it needs (entries, step records; ensure_defer)
hipError_t launch_march_procedural(const MarchArgs& a, bool early, void* sort_buf, int reuse_sort, const Schedule& sc,
                                   hipStream_t s, const ShadowDefer* defer = nullptr,
                                   unsigned long long* need_host = nullptr);
// blocks of the deferred shadow pass (proc_shadow_eval), at least: a grid-stride loop over
// the chunks (vr_api.cpp ensure_defer sizes the grid from the frame)
constexpr unsigned kShadowEvalBlocks = 256 * 6;
hipError_t launch_repack(const uint8_t* d_rgba, int nx, int ny, int nz, uint8_t* d_planar, hipStream_t s);
// Build a fast layout from the planar planes.
hipError_t launch_build_layout(int layout, const uint8_t* d_planar, int nx, int ny, int nz, uint8_t* d_out,
                               hipStream_t s);
size_t layout_plane_bytes(int layout, int nx, int ny, int nz);
// bytes of all four planes of a fast layout (COL48Z's planes differ in size)
size_t layout_total_bytes(int layout, int nx, int ny, int nz);
hipError_t launch_unpack(const uint8_t* d_planar, int nx, int ny, int nz, uint8_t* d_rgba,
                         hipStream_t s);
// Perlin lattice table: entry (x, y, z) - lo of n^3 = noise::perlin_lattice_entry(seed, x, y, z)
hipError_t launch_perlin_lattice(uint2* d_out, int seed, int lo, int n, hipStream_t s);
hipError_t launch_noise(int kind, float* d_out, int x0, int y0, int z0, int nx, int ny, int nz,
                        float freq, int32_t seed, float* d_partials, int* num_partials,
                        hipStream_t s);
hipError_t launch_minmax_reduce(const float* d_partials, int num_partials, float* d_minmax,
                                hipStream_t s);
hipError_t launch_pack_recipe(const float* d_g1, const float* d_g2, const float* d_g3,
                              const float* d_g4, const float* d_minmax, long long total,
                              uint8_t* d_rgba, hipStream_t s);
hipError_t launch_assemble(const uint8_t* d_gathered, size_t rows_per_rank, int nranks,
                           int width, int height, int band_rows, int bpp, int first_rank, uint8_t* d_frame,
                           hipStream_t s, bool serp = false);   // serp: vr.h VR_ASSEMBLE_SERPENTINE
int noise_partials_needed(int nx, int ny, int nz);
// 16-B-per-lane grid-stride copy of `bytes` (a multiple of 16): the measured HBM roofline
hipError_t launch_stream_copy(const void* src, void* dst, size_t bytes, hipStream_t s);
// kind 0 = that copy, 1 = a read-only stream (loads folded into a register);
// loads_per_lane 4, 8 or 16 in flight per lane; dst of a read is a 1 KiB sink
hipError_t launch_stream_bw(int kind, int loads_per_lane, const void* src, void* dst, size_t bytes, hipStream_t s);
// variant 0..2 = noise::cell_inv_a..c, 3 = the sequence cellular() uses
hipError_t launch_selftest_cell_inv(int variant, unsigned long long* d_bad, hipStream_t s);
// noise::cellular_table9 (pruned) vs noise::cellular on 2^23 points per seed
hipError_t launch_selftest_worley(int seed, unsigned long long* d_bad, hipStream_t s);

// host camera math (vr_camera.cpp)
struct RayBasis {
    float org[3], o[3], px[3], py[3], r2[4], r3[4];
    // cam_mode 0: CameraPosition is the View eye (to float rounding): org is
    // the camera, o/px/py its pixel-ray directions.  cam_mode 1: org and
    // o/px/py are the View EYE's (they find the rasterised front-face point,
    // vert.glsl:20), cam the box-local CameraPosition the march starts from
    // (frag.glsl:36-38).  DESIGN.md sec. 3.1.
    int cam_mode;
    float cam[3];
};
bool invert4_d(const double* m, double* inv);
bool make_ray_basis(const float* obj48, const float* glob36, int width, int height, RayBasis* b);
void reference_shader_data(float aspect, float phi_deg, float theta_deg, float frame_time,
                           float* obj48, float* glob36);

}  // namespace vr
