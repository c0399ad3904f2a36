// vr_internal.h -- internal structures shared by the HIP kernels and the C ABI
// (not installed; the public interface is include/vr.h).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stddef.h>

namespace vr {

// Volume layouts in HBM.  All keep one array per channel,
// so a tap reads only the channel it needs (frag.glsl:66-69 read .x, .y, .z,
// .w at four different coordinates).  LAYOUT_PLANAR is the canonical copy:
// any wrap mode, and the source of every other layout.  The others are
// indexed by the *padded* base texel a = floor(u*N - .5) + 1, clamped to
// [0, N].  They store the clamp-to-edge values of the 2x2x2 trilinear
// footprint, so a tap needs no index clamping.  They are exact wherever
// clamp-to-edge equals mirrored repeat (checked per frame on the host).
enum Layout : int {
    LAYOUT_PLANAR = 1,   // u8 plane[z][y][x]; 8 byte loads per tap
    LAYOUT_PAD16 = 2,    // u8 plane[z+1][y+1][x+1] with a 1-texel apron; 4 u16 loads
    LAYOUT_BRICK5 = 3,   // 4^3 bricks + 1-texel apron = 5^3 B in one 128-B line;
                         // a footprint never leaves its line; 4 u16 loads
    LAYOUT_CORNER8 = 4,  // per base texel the 8 footprint bytes (u64), in 4^3
                         // position bricks of 512 B; 1 dwordx2 load per tap
    LAYOUT_QUAD = 5,     // per base texel the 2x2 xy quad (u32), 4x4x5 position
                         // bricks of 320 B; 2 dword loads per tap
};
constexpr int kNumLayouts = 6;

enum Wrap : int { WRAP_CLAMP = 0, WRAP_MIRROR = 1 };

// Everything one launch of the march kernel needs.  Passed by value
// (kernarg segment), computed on the host per vr_render call.
struct MarchArgs {
    // ray basis in box-local space: dir(x,y) = o + (x+.5)*px + (y+.5)*py
    float org[3], o[3], px[3], py[3];
    float r2[4], r3[4];          // rows 2/3 of P*V*M (coverage clip test)
    float box_min[3], box_max[3], box_range[3];
    float step_size, density, scale, acc_limit;
    int max_steps;
    // tap t samples padded texel coordinate g = fma(P, tap_S, tap_T)
    // (= u*N + 0.5 with u = P*s_t + o_t, frag.glsl:66-69)
    float tap_S[4][3], tap_T[4][3];
    // volume
    int nx, ny, nz;
    const uint8_t* vol;          // channel plane 0; plane c at vol + c*plane_stride
    long long plane_stride;
    int prow, pslice;            // PAD16: (nx+2), (nx+2)*(ny+2)
    int nbx, nby;                // bricked layouts: bricks along x, y
    // target
    int width, height, band_rows, band_stride, band_first, out_rows;
    int tiles_x, tiles_y, num_blocks;   // 16x16 tiles; blocks = 8 XCD row-groups
    void* out;
    long long pitch;
    int format;
    unsigned long long* step_counter;
};

// How the march kernel maps tiles to waves.
struct Schedule {
    bool strided;          // true: each wave renders tiles_per_wave strided 8x8 tiles
    int tiles_per_wave;
    bool queue;            // false: static 16x16 tile per workgroup
    int waves_per_simd;    // queue: persistent waves per SIMD (grid = 256 CUs x this)
    int* heads;            // queue: 8 device ints, zeroed before each launch
};

// launchers (vr_march.hip / vr_volume.hip); return hipError_t
hipError_t launch_march(const MarchArgs& a, int layout, int wrap, bool early, const Schedule& sc, hipStream_t s);
hipError_t launch_repack(const uint8_t* d_rgba, int nx, int ny, int nz, uint8_t* d_planar, hipStream_t s);
// Build a fast layout (PAD16/BRICK5/CORNER8/QUAD) from the planar planes.
hipError_t launch_build_layout(int layout, const uint8_t* d_planar, int nx, int ny, int nz, uint8_t* d_out,
                               hipStream_t s);
size_t layout_plane_bytes(int layout, int nx, int ny, int nz);
hipError_t launch_unpack(const uint8_t* d_planar, int nx, int ny, int nz, uint8_t* d_rgba,
                         hipStream_t s);
hipError_t launch_noise(int kind, float* d_out, int x0, int y0, int z0, int nx, int ny, int nz,
                        float freq, int32_t seed, float* d_partials, int* num_partials,
                        hipStream_t s);
hipError_t launch_minmax_reduce(const float* d_partials, int num_partials, float* d_minmax,
                                hipStream_t s);
hipError_t launch_pack_recipe(const float* d_g1, const float* d_g2, const float* d_g3,
                              const float* d_g4, const float* d_minmax, long long total,
                              uint8_t* d_rgba, hipStream_t s);
hipError_t launch_assemble(const uint8_t* d_gathered, size_t rows_per_rank, int nranks,
                           int width, int height, int band_rows, int bpp, uint8_t* d_frame,
                           hipStream_t s);
int noise_partials_needed(int nx, int ny, int nz);

// host camera math (vr_camera.cpp)
struct RayBasis {
    float org[3], o[3], px[3], py[3], r2[4], r3[4];
};
bool invert4_d(const double* m, double* inv);
bool make_ray_basis(const float* obj48, const float* glob36, int width, int height, RayBasis* b);
void reference_shader_data(float aspect, float phi_deg, float theta_deg, float frame_time,
                           float* obj48, float* glob36);

}  // namespace vr
