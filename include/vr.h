/*
 * vr.h -- C-ABI of the MI355X-native volumetric ray-march integrator
 *         (libvr.so, built from volumetricrenderer_amd/csrc/).
 *
 * The reference runs its hot path, shaders/frag.glsl, behind the Vulkan
 * render-pass / descriptor API.  Each entry point below
 * replaces one piece of that API; the reference interface it replaces is cited
 * in the comment above it.  Plain C types only: device buffers are passed as
 * void*, streams as void* (hipStream_t), no torch and no C++ types.
 *
 * Errors: every call returns a vr_status.  0 is success.  On failure,
 * vr_last_error() holds a message for the calling thread.  Exceptions never
 * cross the ABI.  (The reference instead throws from Error(), Utils.h:22-29.)
 *
 * Threading: one vr_ctx per device and host thread.  Calls on one vr_ctx are
 * not reentrant.  vr_render is asynchronous on the given stream.  It does not
 * allocate or synchronise, so a caller may capture it in a hipGraph -- except
 * that the first vr_render after a volume install waits (host) for that
 * install's uniform-channel scan (a few microseconds of GPU work queued with
 * the install), and the first procedural render of a
 * larger target allocates the context's cost-sort scratch (with shadow rays
 * also the deferred-shadow scratch, option "shadow_defer") after a device
 * synchronisation.  That scratch belongs to the context.  vr_render orders
 * procedural renders of one vr_ctx across streams itself: a frame that
 * writes the scratch (a new cost order, deferred shadow rays) waits for every
 * earlier procedural render, and a frame that only reads it (the same camera's
 * order) waits for the last writer, so readers overlap on alternating streams.
 */
#ifndef VR_H
#define VR_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define VR_ABI_VERSION 2

typedef enum {
    VR_OK = 0,
    VR_ERR_INVALID = 1,     /* bad argument (null pointer, bad size or enum) */
    VR_ERR_HIP = 2,         /* HIP runtime error (see vr_last_error)       */
    VR_ERR_NO_VOLUME = 3,   /* vr_render before vr_set_volume/generate     */
    VR_ERR_NO_CAMERA = 4,   /* vr_render before vr_set_shader_data         */
    VR_ERR_OOM = 5,         /* device allocation failed                    */
    VR_ERR_NO_DEVICE = 6,   /* no HIP device / bad device index            */
    VR_ERR_TIMEOUT = 7,     /* a collective (vr_shard.h) missed its deadline; communicator aborted */
    VR_ERR_COMM = 8         /* communicator error (RCCL, vr_shard.h); communicator aborted */
} vr_status;

typedef enum {
    VR_FMT_RGBA32F = 0,      /* 16 B/pixel, linear                          */
    VR_FMT_RGBA8_UNORM = 1,  /* 4 B/pixel, linear, round-to-nearest-even    */
    VR_FMT_RGBA8_SRGB = 2,   /* 4 B/pixel, sRGB-encoded on store, as the
                                reference's swapchain format
                                (VulkanSwapchain.cpp:181-191)               */
    /* Grey targets: frag.glsl:79-80 writes vec4(vec3(c), 1.0), so one channel
     * holds the whole pixel.  The value is the RGBA format's R (bit for bit);
     * G = B = R and A = 1 (255) are implied.  The multi-GPU band sets travel
     * in these (vr_shard.h), and vr_assemble_frame expands them.           */
    VR_FMT_R8_UNORM = 3,     /* 1 B/pixel: VR_FMT_RGBA8_UNORM's R           */
    VR_FMT_R8_SRGB = 4,      /* 1 B/pixel: VR_FMT_RGBA8_SRGB's R            */
    VR_FMT_R32F = 5          /* 4 B/pixel: VR_FMT_RGBA32F's R               */
} vr_format;

/* Replaces the binding-0 UBO `ObjectShaderData` (TestMain.cpp:27-32,
 * vert.glsl:4-9).  Column-major mat4, as in GLM.  192 bytes.              */
typedef struct {
    float model[16];
    float view[16];
    float projection[16];
} vr_object_shader_data;

/* Replaces the binding-1 UBO `GlobalShaderData` (TestMain.cpp:34-39,
 * frag.glsl:9-14).  The std140 layout is made explicit: the vec3 is padded
 * to 16 bytes, so media_scroll sits at byte 80.  The reference's C++ struct
 * put it at byte 76.  144 bytes.                     */
typedef struct {
    float world_to_local[16];
    float camera_position[3];
    float _pad0;
    float media_scroll[16];
} vr_global_shader_data;

/* Constants that the reference hard-codes in frag.glsl.  Fill it with
 * vr_march_defaults() to get the reference values.                        */
typedef struct {
    int32_t max_steps;      /* frag.glsl:30  maxSteps = 128                 */
    float   step_scale;     /* frag.glsl:42  stepSize = (1/maxSteps) * 4    */
    float   density;        /* frag.glsl:29  density = 1                    */
    float   scale;          /* frag.glsl:63  scale = 0.2                    */
    float   box_min[3];     /* frag.glsl:31  (-1,-1,-1)                     */
    float   box_max[3];     /* frag.glsl:32  ( 1, 1, 1)                     */
    float   tap_scale[4];   /* frag.glsl:66-69  Pin * {1, .8, .75, .7}      */
    float   tap_weight[4];  /* frag.glsl:66-69  MediaScroll * {0,.2,.25,.3} */
    float   early_out;      /* stop a ray once its transmittance is below this
                               value.  0 = off, which is the reference.      */
    int32_t reserved[3];    /* must be 0                                    */
} vr_march_params;

/* The volume recipe of TestMain.cpp:43-92: four FastNoise2-style grids
 * (Cellular f=.01 s1, Cellular f=.03 s2, Perlin f=.19 s3, Simplex f=.15 s4),
 * normalised, inverted, R raised to the 4th power, packed to RGBA8.       */
typedef struct {
    int32_t size;               /* N, for an N^3 volume (TestMain.cpp:51: 128) */
    float   freq[4];            /* TestMain.cpp:59-62                        */
    int32_t seed[4];
    int32_t literal_overwrite;  /* 1: replicate TestMain.cpp:60, where the
                                   f=.03 grid is written into noiseOutput1   */
} vr_volume_recipe;

/* Procedural medium: BASELINE configs 2/3, build-defined extensions with no
 * reference counterpart.  When enabled, vr_render
 * marches a density evaluated in-kernel instead of the volume:
 *   q = P * grid_scale              (P: box point in [0,1]^3)
 *   fbm = sum_o gain^o * perlin(seed_fbm, q * freq0 * lacunarity^o)
 *   F1  = cellular(seed_worley, q * worley_freq) + 1
 *   rho = max(fbm * (1 - F1), 0) * march.scale
 * With shadow_steps = 0, the output is Beer-Lambert 1 - exp(-density*sum(rho)*ds).
 * With shadow_steps > 0, each step adds single scatter lit from sun_dir
 * (box-local): Tview * rho*ds*density * exp(-density*ds*sum rho_sun), with
 * shadow_steps sun samples at P + k*ds*sun_dir, inside the box only.       */
typedef struct {
    int32_t enabled;
    float   grid_scale;     /* 128 */
    int32_t octaves;        /* 4 */
    float   freq0;          /* 0.19 */
    float   lacunarity;     /* 2 */
    float   gain;           /* 0.5 */
    int32_t seed_fbm;       /* 3 */
    float   worley_freq;    /* 0.03 */
    int32_t seed_worley;    /* 2 */
    int32_t shadow_steps;   /* 0 (config 2) or 8 (config 3) */
    float   sun_dir[3];     /* normalize(1,1,2); normalised by the library */
    int32_t reserved;       /* must be 0 */
} vr_procedural;

/* A render target.  `pixels` is a DEVICE pointer that the caller owns.
 * With band_rows > 0 only bands b = band_first, band_first + band_stride, ...
 * are rendered.  Band b covers frame rows [b*band_rows, (b+1)*band_rows).
 * band_flip (ABI 2) shifts every second band of the set: its k-th band is
 * band_first + k*band_stride + (k odd ? band_flip : 0), |band_flip| <
 * band_stride.  A world of S renderers with flips S-1-2i (renderer i) deals
 * the bands serpentine: forwards in even periods of S bands, backwards in odd
 * ones, so a cost that drifts down the frame does not load one renderer
 * more in every period (vr_shard.h vr_shard_set_serpentine).
 * The bands are written packed and in order, from row 0 of `pixels`; the
 * rows of a last, partial band that lie past `height` are left untouched.
 * This is how the frame is split across GPUs.  band_rows = 0 renders the whole
 * frame.  step_counter (device u64, may be NULL) has the executed ray-steps
 * added to it (the sum of n, frag.glsl:46).                                */
/* OR'ed into vr_target.format with band_rows > 0: each band is written at its
 * own frame rows of `pixels` (a whole-frame buffer, `height` rows) instead of
 * packed from row 0 -- rank 0 of the multi-GPU loop renders its bands straight
 * into the frame (vr_shard.h), and the assembly skips them
 * (vr_assemble_frame_ranks).                                               */
#define VR_TARGET_BANDS_IN_PLACE 0x100
/* OR'ed into vr_target.format: the target is one contiguous range of frame
 * rows, [band_first, band_first + band_rows), instead of a band set.
 * band_first must be a multiple of 8 and band_stride must be 1; rows past
 * `height` are not written.  The rows are packed from row 0 of `pixels`, or
 * stored at their frame rows with VR_TARGET_BANDS_IN_PLACE.  The multi-GPU
 * loop's balanced row ranges (vr_shard.h vr_shard_balance_rows).            */
#define VR_TARGET_ROW_RANGE 0x200

typedef struct {
    int32_t   width, height;
    int32_t   format;        /* vr_format, optionally | VR_TARGET_BANDS_IN_PLACE
                              * and/or VR_TARGET_ROW_RANGE                   */
    int32_t   band_rows, band_stride, band_first;
    void*     pixels;
    size_t    row_pitch;     /* bytes; 0 = tightly packed                  */
    uint64_t* step_counter;
    int32_t   band_flip;     /* 0 = plain band set; see above              */
    int32_t   reserved;      /* must be 0                                  */
} vr_target;

/* ---- context (replaces Renderer::Init/Shutdown, VulkanRenderer.h:68-72) */
vr_status   vr_create(int device, void** out_ctx);
vr_status   vr_destroy(void* ctx);
const char* vr_last_error(void);
int         vr_abi_version(void);
/* Hash of the sources this library was built from (tools/build_id.py; a
 * "-exp" suffix for the VR_EXPERIMENTS build): the tests and smoke() check
 * that the prebuilt library matches the checked-out code.  Static string.  */
const char* vr_build_id(void);

/* ---- volume: replaces vkc::Texture3D(unsigned char*, VkExtent3D)
 *      (VulkanTexture.h:55-60, VulkanTexture.cpp:111-156).  RGBA8 UNORM,
 *      x fastest (the TestMain.cpp:69-73 pack order).  The library copies the
 *      data into its own device layout.  The host call is synchronous.     */
vr_status vr_set_volume(void* ctx, const uint8_t* rgba8, int nx, int ny, int nz);
vr_status vr_set_volume_device(void* ctx, const void* d_rgba8, int nx, int ny, int nz, void* stream);
/* read the volume back as RGBA8 (host); for tests and tools             */
vr_status vr_get_volume(void* ctx, uint8_t* rgba8_out);
vr_status vr_volume_dims(void* ctx, int* nx, int* ny, int* nz);
/* 1 if vr_set_volume / vr_set_volume_device accept an nx x ny x nz extent
 * (the device layouts index a plane with 32-bit offsets), else 0          */
int       vr_volume_extent_ok(int nx, int ny, int nz);

/* ---- volume generation on the GPU: replaces the host start-up loops of
 *      TestMain.cpp:43-92.  Synchronous.             */
vr_status vr_volume_recipe_defaults(vr_volume_recipe* r);
vr_status vr_generate_volume(void* ctx, const vr_volume_recipe* r, void* stream);
/* one noise grid, for parity tests: kind 0 cellular, 1 perlin, 2 simplex.
 * d_out: device float[nx*ny*nz] (may be NULL); min/max to host.           */
vr_status vr_noise_grid(void* ctx, int kind, void* d_out, int x0, int y0, int z0,
                        int nx, int ny, int nz, float freq, int32_t seed,
                        float* out_min, float* out_max, void* stream);
/* Exhaustive device self-test of an arithmetic shortcut against its IEEE
 * definition; *failures = number of mismatching inputs (synchronous).
 * "cell_inv" (the cellular cell-point magnitude that the noise kernels use)
 * and the candidates "cell_inv_a", "cell_inv_b", "cell_inv_c";
 * "worley_prune": the procedural march's pruned Worley F1 against the full
 * 27-cell one on 2^23 points per seed (uniform, and at the bound's edge
 * cases: rint and floor switches, feature points, near ties).            */
vr_status vr_selftest(void* ctx, const char* name, long long* failures);

/* ---- uniforms: replaces UniformBuffer<T>::Update x2 (TestMain.cpp:248-249,
 *      VulkanUniformBuffer.h:58-61).  The data is copied.                  */
vr_status vr_set_shader_data(void* ctx, const vr_object_shader_data* osd,
                             const vr_global_shader_data* gsd);
/* host camera producer of TestMain.cpp:219-245: Model = rotZ(phi)*rotY(theta),
 * lookAt((3,3,3), 0, +Z), perspective(45deg, aspect, .1, 10) with y flipped,
 * W2L = inverse(Model), MediaScroll[0][0] = -frame_time.                   */
vr_status vr_reference_shader_data(float aspect, float phi_deg, float theta_deg,
                                   float frame_time, vr_object_shader_data* osd,
                                   vr_global_shader_data* gsd);

/* ---- procedural medium (configs 2/3) ----------------------------------- */
vr_status vr_procedural_defaults(vr_procedural* p);   /* enabled = 0 */
vr_status vr_set_procedural(void* ctx, const vr_procedural* p);

/* ---- march constants (frag.glsl:29-32, 42, 63-69) ---------------------- */
vr_status vr_march_defaults(vr_march_params* m);
vr_status vr_set_march(void* ctx, const vr_march_params* m);

/* ---- the hot path: replaces EnqueueRenderPass("BasePass") + the draw of
 *      TestMain.cpp:194-217 + vert.glsl/frag.glsl (VulkanRenderer.h:84-87).
 *      A procedural medium, when enabled, needs no volume.

 *      stream = hipStream_t (NULL = default stream).                       */
vr_status vr_render(void* ctx, const vr_target* target, void* stream);
/* The frame loop of TestMain.cpp:173-256 with a moving camera: `frames`
 * renders into `target`, frame i with shader data (osd[i], gsd[i]) -- the
 * per-frame UBO updates of :219-249 -- all queued on `stream` without a host
 * wait.  The ctx keeps the last frame's shader data.                       */
vr_status vr_render_sequence(void* ctx, const vr_target* target, int frames, const vr_object_shader_data* osd,
                             const vr_global_shader_data* gsd, void* stream);

/* ---- multi-GPU frame assembly.  The band sets of `nranks` ranks are
 *      gathered into one device buffer, d_gathered = [rank][packed rows].
 *      Each rank's set holds `rows_per_rank` rows.  This call scatters them
 *      into the full frame.  Rank r rendered with band_stride = nranks and
 *      band_first = r.  The layout matches vr_render's packed output.
 *      bytes_per_pixel: 1, 4 or 16 (the target format's pixel size).      */
vr_status vr_assemble_bands(void* ctx, const void* d_gathered, size_t rows_per_rank,
                            int nranks, int width, int height, int band_rows,
                            int bytes_per_pixel, void* d_frame, void* stream);
/* The same scatter between formats: band sets gathered in `gathered_format`
 * into a frame in `frame_format`.  Equal formats copy (vr_assemble_bands);
 * a grey set expands into its RGBA format: R8_UNORM -> RGBA8_UNORM,
 * R8_SRGB -> RGBA8_SRGB, R32F -> RGBA32F (G = B = R, A = 255 / 1.0), so the
 * gather moves a quarter of the bytes.  Other pairs are VR_ERR_INVALID.   */
vr_status vr_assemble_frame(void* ctx, const void* d_gathered, int gathered_format, size_t rows_per_rank,
                            int nranks, int width, int height, int band_rows, int frame_format,
                            void* d_frame, void* stream);
/* vr_assemble_frame for the ranks first_rank .. nranks-1 only: the rows of
 * ranks below first_rank are left untouched (rendered in place, with
 * VR_TARGET_BANDS_IN_PLACE); their gather slots are not read.
 * frame_format | VR_ASSEMBLE_SERPENTINE: rank r rendered its set with
 * band_flip nranks-1-2r (the serpentine deal, vr_target).                 */
#define VR_ASSEMBLE_SERPENTINE 0x400
vr_status vr_assemble_frame_ranks(void* ctx, const void* d_gathered, int gathered_format, size_t rows_per_rank,
                                  int nranks, int first_rank, int width, int height, int band_rows,
                                  int frame_format, void* d_frame, void* stream);
/* rows that vr_render writes for a band set (for sizing buffers): whole
 * bands, the set's last partial one included                             */
int vr_band_rows_packed(int height, int band_rows, int band_stride, int band_first, int band_flip);
/* Split the frame's rows into `parts` contiguous ranges of equal estimated
 * march work for the ctx's current camera and march constants (host, double;
 * the same inputs give the same split on every rank).  row_begin[parts + 1]:
 * range k is [row_begin[k], row_begin[k + 1]); row_begin[0] = 0,
 * row_begin[parts] = height, the others multiples of 8 or height
 * (VR_TARGET_ROW_RANGE).  The estimate per ray that meets the box is
 * n^(row_pow / 100) + row_setup, n its a3 step count (frag.glsl:46), sampled
 * every 8th pixel of every 8th row (vr_set_option "row_pow", default 130,
 * and "row_setup", default 40: long rays cost more than their steps, the
 * longest waves bound a small share's launch); range 0 takes
 * "row_first_pct" (default 100) % of a mean share.                        */
vr_status vr_row_partition(void* ctx, int width, int height, int parts, int* row_begin);
/* vr_row_partition corrected by measurement: range k of the previous split
 * prev_begin[parts + 1] took prev_ms[k] (any unit, >= 0; 0 = not measured);
 * each of its strips' estimated work is scaled by prev_ms[k] / (the model's
 * work of range k), and the frame is split again (vr_shard_rebalance_rows). */
vr_status vr_row_partition_measured(void* ctx, int width, int height, int parts, const int* prev_begin,
                                    const double* prev_ms, int* row_begin);

/* The estimate vr_row_partition splits: the march work of every 8-row strip
 * of a width x height frame for the ctx's current camera and march constants
 * (strip_work[nstrips], nstrips = ceil(height / 8); host, double; the same
 * inputs give the same values on every rank).  vr_shard_balance_lead sizes
 * rank 0's lead rows from it.  New (no reference counterpart).            */
vr_status vr_row_work(void* ctx, int width, int height, double* strip_work, int nstrips);

/* ---- introspection: the kernel variant vr_render will launch ----------- */
/* returns a static string, e.g. "grid_pad16_clamp"                        */
const char* vr_kernel_variant(void* ctx);
/* Choose the device volume layout: 0 = auto (default),
 * 1 = planar only, 2 = 4^3 apron bricks in 128-B lines ("brick5"),
 * 3 = 7^3 apron bricks of 512 B ("brick8"), 4 = 15^3 apron bricks of 4 KiB
 * ("brick16"), 5 = 8-corner footprint words ("corner8"), 6 = 3^3 apron
 * bricks of 64 B ("brick4"), 7 = 4x16x2-texel bricks of 128 B whose
 * rows run z-fastest, one 16-B load per tap ("zpair"), 8 = 4x4x8-texel
 * bricks of 128 B ("brick448"), 9 = 4x8x8-texel bricks of 256 B
 * ("brick488"), 10 = 4x8x16-texel bricks of 512 B ("brick4816"),
 * 11 = 4x16x16-texel bricks of 1 KiB ("brick41616"), 12 = 4x8x32-texel
 * bricks of 1 KiB ("brick4832"), 13 = 4x8x64-texel bricks of 2 KiB
 * ("brick4864"), 14 = per position the f16 pairs {a, b - a} of the four
 * footprint rows, one 16-B load and four v_fma_mix_f32 per tap ("cornerh";
 * volumes below 2^24 positions), 15 = columns of 4x8 texels through the
 * whole z extent, slices 32 B apart ("col48"; auto above 160 MiB), 16 = col48
 * for channels 0-2 and zpair for channel 3 ("col48z").  Layouts 2-16 are
 * used only where clamp-to-edge equals mirrored repeat.  Otherwise the
 * planar, mirrored-repeat kernel runs.  Rebuilds the layout (synchronous). */
vr_status vr_set_layout_preference(void* ctx, int pref);
/* Tuning knobs.
 *   "layout"          as vr_set_layout_preference.
 *   "schedule"        -1 = auto (the default); 0 = one static 16x16 tile per
 *                     workgroup, tile rows dealt to XCDs; 1 = persistent waves
 *                     pulling 8x8 tiles from per-XCD queues; 2 = each wave
 *                     renders "tiles_per_wave" strided 8x8 tiles; 3 = 8-px
 *                     tile rows dealt to XCDs; 4 = rings of 8x8 tiles around
 *                     the projected box centre, longest rays first; 5 =
 *                     regions: each XCD renders "wedges" contiguous angular
 *                     wedges of tiles around the box centre with equal
 *                     estimated work, inside-out (auto for the volume; the
 *                     lists are rebuilt on the host when the geometry
 *                     changes, at most every 32 renders for a moving camera).
 *                     Procedural medium: auto = cost-sorted pixels, 0 = 8x8
 *                     tiles in row order, 4 = rings.
 *   "waves_per_simd"  1-8, queue schedule.
 *   "tiles_per_wave"  1-64, strided, ring and region schedules; 0 = auto,
 *                     the default: 2 for rings, 3 for regions on the col48
 *                     layout and 2 on the others, 1 for strided.
 *   "wedges"          1-64, regions schedule: wedges per XCD; 0 = auto (the
 *                     default): 4 while frames_overlap is set (frames in
 *                     flight on several streams), else 8.  vr_get_option
 *                     returns the count in force.
 *   "supertile"       1, 2, 4, regions schedule: the tile lists are ordered by
 *                     S x S blocks of 8x8 tiles (default 2), so a workgroup's
 *                     waves render one block.
 *   "region_order"    regions schedule, each XCD's list: 2 (default) = S x S
 *                     blocks by their longest estimated tile, longest first;
 *                     1 = tiles by estimate, longest first; 0 = inside-out
 *                     (ring around the projected box centre, then angle).
 *   "wg_waves"        4 (default), 8, 16: waves per workgroup of the regions
 *                     march (col48, brick4832, cornerh).
 *   "slab"            0/1, col48 + regions: the per-wave LDS slab march
 *                     (the north star's "per-tile density slabs staged in
 *                     LDS", bit-exact; measured slower, so 0 is the
 *                     default); "slab_cap" 0-32 chunks per channel.
 *   "split"           regions schedule, brick4/448/488/zpair/corner8: lanes per ray
 *                     (1, 2, 4, 8; each lane marches every K-th step and the
 *                     terms are summed in step order, bit-exact); 0 = auto,
 *                     the default: 2 or 4 when the target has too few rays
 *                     to fill the GPU (a 1/N share of a frame).
 *   "count"           0 = vr_target.step_counter sums executed ray-steps (the
 *                     default); 1 = it sums density evaluations, i.e.
 *                     ray-steps plus the procedural shadow samples -- the unit
 *                     of the procedural roofline; 2 = the Worley cells those
 *                     evaluations computed.
 *   "uniform_skip"    1 (default) = a channel whose texels all hold one byte value
 *                     (found when the volume is installed; the reference recipe's
 *                     G, TestMain.cpp:60) is sampled as the exact constant v/255
 *                     with no loads; 0 = every channel is loaded.
 *   "uniform_mask"    read-only (vr_get_option): bit c set = channel c uniform.
 *   "region_work_tiles" read-only: 8x8 tiles with estimated work in the current
 *                     region lists (what the auto split K is chosen from).
 *   "sort_reuse"      0-64, procedural sorted schedule: renders that may march
 *                     the cost order of an older camera (default 0).
 *   "proc_enum"       0/1, procedural sort with shadow rays: enumerate
 *                     64x64 regions (default 0, row-major; the deferred
 *                     shadow passes always enumerate regions).
 *   "shadow_defer"    procedural medium with shadow rays, sorted schedule:
 *                     1 (default) = the primary march appends its
 *                     shadow-ray origins, one pass evaluates them all and a
 *                     resolve pass folds them per ray in step order;
 *                     0 = each wave deals its own shadow samples at every
 *                     step (at most 8 shadow steps).  Results are identical.
 *                     The deferred passes keep a device scratch sized from
 *                     the frame: ~16 B per executed ray-step x 5/4 (0.35 GB at
 *                     1080p x 128, ~2.7 GB at 3840 x 2160 x 256), grown when a
 *                     frame needs more (a wave past it marches its shadow rays
 *                     in place, exactly); setting "shadow_defer" 0 or
 *                     "shadow_defer_mib" 0 frees it (after a device sync).
 *                     "shadow_blocks" 0-65536: workgroups of the deferred
 *                     shadow pass (0 = auto, 3/8 of the sorted waves).
 *                     "shadow_defer_mib": the largest scratch the deferred
 *                     passes may allocate (default 4096); "shadow_defer_entries"
 *                     a fixed entry capacity (tests; 0 = from the frame).
 *                     Read-only: "shadow_defer_kib" the scratch held now,
 *                     "shadow_defer_last" 1 if the last procedural render ran
 *                     the deferred passes.
 *   "lattice"         procedural medium, sorted schedule: 1 = the fBm reads its
 *                     per-cell gradient-pair offsets from a lattice table in
 *                     global memory (the default; built when the seed or the
 *                     lattice range changes, at most 2^24 cells, 128 MiB);
 *                     0 = it hashes every corner.  Results are identical.
 * vr_get_option returns -1 for an unknown name.                            */
vr_status vr_set_option(void* ctx, const char* name, int value);
int       vr_get_option(void* ctx, const char* name);

/* ---- measurement: the device's streaming bandwidth, the measured HBM
 *      roofline the bench reports next to the 8 TB/s spec.
 *      vr_measure_bandwidth: one pass of 16 B per lane over `bytes`, the grid
 *      as large as the buffer, `loads_per_lane` (4, 8 or 16) independent loads
 *      in flight per lane, 0 = each of 4, 8, 16 (the best is reported), `reps`
 *      times on `stream`, each timed with HIP events.
 *        kind VR_BW_COPY: float4 copy between two fresh buffers; bytes moved
 *                         = read + written (2 x bytes);
 *        kind VR_BW_READ: loads only, folded into a register, nothing stored;
 *                         bytes moved = bytes (the ray march is ~98 % reads).
 *      *gbs_best and *gbs_median in GB/s; *loads_best (may be NULL) = the
 *      loads per lane of the best rep.  Synchronous.
 *      vr_measure_copy_bandwidth = kind VR_BW_COPY at 4 loads per lane.     */
#define VR_BW_COPY 0
#define VR_BW_READ 1
vr_status vr_measure_bandwidth(void* ctx, int kind, int loads_per_lane, size_t bytes, int reps, void* stream,
                               double* gbs_best, double* gbs_median, int* loads_best);
vr_status vr_measure_copy_bandwidth(void* ctx, size_t bytes, int reps, void* stream, double* gbs_best,
                                    double* gbs_median);

#ifdef __cplusplus
}
#endif
#endif /* VR_H */
