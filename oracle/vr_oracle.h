/*
 * vr_oracle.h -- CPU restatement of the reference ray-march hot path.
 *
 * TEST INFRASTRUCTURE ONLY.  Only tests/, __graft_entry__.smoke() and
 * bench.py's cpu_baseline leg may load this library, and only as the checker
 * or the CPU baseline -- never as the product path.  The product is the HIP
 * library volumetricrenderer_amd/libvr.so (include/vr.h).
 *
 * Parity status: the reference (Vulkan + GLSL + FastNoise2) cannot be built or
 * run in this environment and ships no tests, fixtures or golden vectors
 * (SURVEY.md sec. 4, sec. 8c).  This restatement is therefore "parity
 * unpinned" against reference *outputs*; it is anchored instead on
 *   - the reference's code, cited file:line at every function below,
 *   - independent analytic known-answer tests (tests/test_oracle_kat.py):
 *     constant / linear-ramp volumes, mirrored-repeat addressing, and the
 *     SURVEY.md sec. 6 coverage / step-count figures for the reference camera.
 * Noise values (FastNoise2, absent from /root/reference, commit unknown) are
 * a restatement of FastNoise2's published algorithms and are unpinned.
 *
 * Floating point: fp32, round-to-nearest; the only fused multiply-adds are the
 * explicit fmaf() calls (built with -ffp-contract=off).  The sequence of
 * operations is the spec the HIP kernels follow.
 */
#ifndef VR_ORACLE_H
#define VR_ORACLE_H
#include <stdint.h>
#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

/* Shader-data blocks, column-major mat4 as in GLM.
 * obj  = 48 floats: Model, View, Projection          (TestMain.cpp:27-32)
 * glob = 36 floats: WorldToLocal, CameraPosition+pad, MediaScroll
 *        (TestMain.cpp:34-39 laid out std140, frag.glsl:9-14)            */

typedef struct {
    int32_t max_steps;      /* frag.glsl:30  maxSteps = 128            */
    float   step_scale;     /* frag.glsl:42  (1/maxSteps) * 4          */
    float   density;        /* frag.glsl:29  density = 1               */
    float   scale;          /* frag.glsl:63  scale = 0.2               */
    float   box_min[3];     /* frag.glsl:31                            */
    float   box_max[3];     /* frag.glsl:32                            */
    float   tap_scale[4];   /* frag.glsl:66-69  1, .8, .75, .7         */
    float   tap_weight[4];  /* frag.glsl:66-69  0, .2, .25, .3 (scroll)*/
    float   early_out;      /* transmittance early-out; 0 = off (ref)  */
    int32_t reserved[3];
} vro_march;

enum { VRO_FMT_RGBA32F = 0, VRO_FMT_RGBA8_UNORM = 1, VRO_FMT_RGBA8_SRGB = 2 };

/* ---- noise (restated FastNoise2 generators, TestMain.cpp:43-45,59-62) ---- */
enum { VRO_NOISE_CELLULAR = 0, VRO_NOISE_PERLIN = 1, VRO_NOISE_SIMPLEX = 2 };
float vro_perlin3(int32_t seed, float x, float y, float z);
float vro_simplex3(int32_t seed, float x, float y, float z);
float vro_cellular3(int32_t seed, float x, float y, float z);
/* GenUniformGrid3D(out, x0,y0,z0, nx,ny,nz, freq, seed) -> {min,max}.
 * out may be NULL (min/max only).                                          */
void vro_gen_uniform_grid3d(int kind, float* out, int x0, int y0, int z0,
                            int nx, int ny, int nz, float freq, int32_t seed,
                            float* out_min, float* out_max);

/* Volume recipe of TestMain.cpp:51-92 into an interleaved RGBA8 volume
 * (x fastest, then y, then z: TestMain.cpp:69-73).  literal_overwrite = 1
 * replicates the reference's noiseOutput1 overwrite (TestMain.cpp:60).    */
typedef struct {
    int32_t size;            /* 128 (TestMain.cpp:51)                     */
    float   freq[4];         /* .01 .03 .19 .15 (TestMain.cpp:59-62)      */
    int32_t seed[4];         /* 1 2 3 4                                   */
    int32_t literal_overwrite;
} vro_recipe;
int vro_build_volume(const vro_recipe* r, uint8_t* rgba_out);

/* ---- camera producer, TestMain.cpp:219-245 (GLM, float) ---- */
void vro_reference_shader_data(float aspect, float phi_deg, float theta_deg,
                               float frame_time, float* obj48, float* glob36);

/* ---- sampler, VulkanCore.cpp:676-710 + VulkanTexture.cpp:111-156 ---- */
float vro_sample(const uint8_t* rgba, int nx, int ny, int nz, int channel,
                 float px, float py, float pz);
int   vro_mirror(int i, int n);
float vro_expf(float x);

/* ---- the hot path: vert.glsl:17-22 + raster coverage + frag.glsl:34-81 ----
 * Renders rows of bands: band b covers rows [b*band_rows, (b+1)*band_rows),
 * bands band_first, band_first+band_stride, ... are written packed, in
 * order, to `out` (row pitch in bytes).  band_rows = 0 -> whole frame.
 * steps_out (nullable) receives the total executed steps (a3's n summed).
 * Returns 0 on success.                                                    */
int vro_render(const uint8_t* rgba, int nx, int ny, int nz,
               const float* obj48, const float* glob36, const vro_march* m,
               int width, int height, int format, void* out, size_t pitch,
               int band_rows, int band_stride, int band_first,
               int64_t* steps_out, int threads);

/* ---- procedural medium (BASELINE configs 2/3; build-defined, SURVEY.md
 * sec. 8d: no reference counterpart).  Density at box point P in [0,1]^3:
 *   q = P * grid_scale
 *   fbm = sum_o gain^o * perlin(seed_fbm, q * freq0 * lacunarity^o)
 *   F1  = cellular(seed_worley, q * worley_freq) + 1
 *   rho = max(fbm * (1 - F1), 0) * march.scale
 * shadow_steps = 0: Beer-Lambert of frag.glsl:76-80 on sum(rho).
 * shadow_steps > 0: single scatter toward sun_dir (box-local, normalised),
 *   L += Tview * (rho*ds*density) * Tsun, Tsun = exp(-density*ds*sum rho_sun)
 *   over shadow_steps samples at P + k*ds*sun (inside the box only).       */
typedef struct {
    int32_t enabled;
    float   grid_scale;     /* 128: the reference's texel-grid frequency units */
    int32_t octaves;        /* 4 */
    float   freq0;          /* 0.19 (TestMain.cpp:61 Perlin frequency) */
    float   lacunarity;     /* 2 */
    float   gain;           /* 0.5 */
    int32_t seed_fbm;       /* 3 */
    float   worley_freq;    /* 0.03 (TestMain.cpp:60) */
    int32_t seed_worley;    /* 2 */
    int32_t shadow_steps;   /* 0 (config 2) or 8 (config 3) */
    float   sun_dir[3];     /* normalize(1,1,2) */
    int32_t reserved;
} vro_procedural;
float vro_procedural_density(const vro_procedural* p, float scale, float px, float py, float pz);
int vro_render_procedural(const vro_procedural* p, const float* obj48, const float* glob36, const vro_march* m,
                          int width, int height, int format, void* out, size_t pitch,
                          int band_rows, int band_stride, int band_first, int64_t* steps_out,
                          int64_t* evals_out, int64_t* cells_out, int threads);
/* evals_out (nullable): density evaluations = executed steps + shadow samples.
 * cells_out (nullable): the Worley cells the device's pruned evaluation
 * computes, summed (vro_worley_cells; vr option "count" = 2).              */
int vro_worley_cells(const vro_procedural* p, float px, float py, float pz);

/* Per-pixel step count n (frag.glsl:46) and coverage, for KAT tests.
 * n_out[y*width+x] = -1 for uncovered pixels.                              */
int vro_step_counts(const float* obj48, const float* glob36, const vro_march* m,
                    int width, int height, int32_t* n_out);

#ifdef __cplusplus
}
#endif
#endif
