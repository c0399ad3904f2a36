// vr_ctx.h -- the library context (Ctx) and the host helpers shared by the
// translation units of the C ABI: vr_api.cpp (context, volume, render,
// assembly), vr_options.cpp (vr_set_option / vr_get_option / the kernel
// variant), vr_regions_host.cpp (region lists, row partition) and
// vr_proc_host.cpp (procedural medium scratch and tables).  Internal: not
// part of include/vr.h.
#pragma once

#include <algorithm>
#include <cmath>
#include <cstdarg>
#include <cstdio>
#include <cstring>
#include <exception>
#include <new>
#include <stdexcept>
#include <string>
#include <vector>

#include "../../include/vr.h"
#include "vr_internal.h"

namespace vrapi {
using namespace vr;

extern thread_local std::string g_err;
vr_status fail(vr_status st, const char* fmt, ...);
vr_status caught_exception(const char* fn) noexcept;

#define HIP_TRY(expr)                                                                        \
    do {                                                                                     \
        hipError_t e_ = (expr);                                                              \
        if (e_ != hipSuccess)                                                                \
            return fail(e_ == hipErrorOutOfMemory ? VR_ERR_OOM : VR_ERR_HIP, "%s: %s (%s:%d)", \
                        #expr, hipGetErrorString(e_), __FILE__, __LINE__);                   \
    } while (0)

constexpr int kDefaultSchedule = -1;     // -1 auto, 0 static tiles, 1 persistent queue, 2 strided
constexpr int kDefaultWavesPerSimd = 4;
constexpr int kDefaultTilesPerWave = 0;   // 0 = auto: 2 for rings and regions, 1 for strided (measured)
constexpr int kDefaultWedges = 8;         // regions schedule: wedges per XCD (measured; 4 until round 4)
// with consecutive frames overlapping (option frames_overlap): 4 -- config 5
// 0.1050 against 0.1078 ms per frame on the GPU clock (4 rounds), 0.0187 against
// 0.0193-0.0196 at 8 ranks; config 4 level (profiles/r06/c17, c18)
constexpr int kDefaultWedgesOverlap = 4;
// a moving camera reuses the current (still complete, maybe less balanced)
// region lists for this many renders before they are rebuilt
constexpr int kRegionRebuildInterval = 32;
// Procedural cost sort under a moving camera: with option sort_reuse = R > 0 a
// frame with the same target and march settings but another camera marches the
// order built for an older one, for R renders after the build (vr_render; the
// march then also checks the pixels the old order left out, so every frame
// stays exact).
constexpr size_t kSortKeyGridPart = 11;   // leading sort-key entries a stale order must match
constexpr int kMaxRegionStreams = 4;
// largest deferred-shadow scratch (option "shadow_defer_mib"): the scratch is
// sized from the frame (ensure_defer: ~0.35 GB at 1080p x 128, ~2.7 GB at
// 3840 x 2160 x 256); a frame needing more marches its last waves' shadow rays
// in place
constexpr int kMaxDeferMiB = 4 << 10;
// retired deferred scratch buffers kept before a device sync frees them
constexpr size_t kMaxDeferRetired = 4;
constexpr int kRegionKeyLen = 40;
// auto split (lanes per ray) from the frame share's tiles with work: K = 1 at
// >= 6000, 2 at >= 1400, else 4.  Measured on 1/N of the 1080p frame at 512^3
// (~7,500 tiles with work): K = 1, 2, 2, 4 at N = 1, 2, 4, 8.
// K = 2 beats K = 1 by 17 % at N = 2 and K = 4 by 2-5 % at N = 4; at 4K x 256
// (4x the tiles) it keeps K = 1 up to N = 4.
constexpr long long kSplitOneLane = 6000, kSplitTwoLanes = 1400;
// With consecutive frames overlapping on two streams (option frames_overlap,
// set by vr_shard_run_frames) the next frame's waves fill the SIMDs while this
// one's longest rays finish, so one lane per ray pays from fewer tiles on:
// K = 1 from 2500 (1080p at 512^3, N = 2: 0.0583 ms per frame at K = 1 against
// 0.0632 at K = 2; on one stream 0.0921 against 0.0744; profiles/r05/split_overlap.txt)
constexpr long long kSplitOneLaneOverlap = 2500;

struct Plan {
    int layout, wrap;
    bool early;
};

struct Ctx {
    int device = 0;
    // volume (channel planes; see vr_internal.h Layout)
    int nx = 0, ny = 0, nz = 0;
    uint8_t* d_planar = nullptr;   // canonical planes (LAYOUT_PLANAR)
    int uniform_mask = 0;          // channels whose every texel is uniform_val[c] (install_volume)
    uint8_t uniform_val[4] = {};
    // the install's per-plane min / max scan, read back asynchronously and
    // resolved at first use (resolve_uniform): no host wait inside the install,
    // so a collective volume share keeps its deadline (vr_shard.cpp)
    unsigned* d_mm = nullptr;      // device [min x 4, max x 4]
    unsigned* h_mm = nullptr;      // pinned copy
    hipEvent_t mm_ready = nullptr;
    bool mm_pending = false;
    int uniform_skip = 1;          // option "uniform_skip": 0 = load uniform channels anyway
    uint8_t* d_fast = nullptr;     // one fast layout, built from d_planar
    int fast_layout = 0;           // which one (0 = none)
    size_t fast_plane_bytes = 0;
    // uniforms
    bool has_camera = false;
    float obj[48];
    float glob[36];
    vr_march_params march;
    int layout_pref = 0;           // 0 = auto (kDefaultFastLayout), else a Layout
    // schedule of the march kernel (vr_set_option "schedule", "waves_per_simd")
    int schedule = kDefaultSchedule;
    int waves_per_simd = kDefaultWavesPerSimd;
    int tiles_per_wave = kDefaultTilesPerWave;
    int* d_heads = nullptr;        // 8 queue heads (+ padding), zeroed per launch
    vr_procedural proc{};          // procedural medium (configs 2/3), off by default
    int count = 0;                 // step_counter: 0 = executed ray-steps, 1 = density evaluations,
                                   // 2 = Worley cells computed (procedural)
    void* d_sort = nullptr;        // procedural cost-sort scratch (sort_layout), grown on demand
    size_t sort_bytes = 0;
    // deferred shadow rays (option "shadow_defer", vr_internal.h ShadowDefer):
    // counter, per-wave step counts and records, entries; grown on demand
    int shadow_defer_mib = kMaxDeferMiB;   // largest deferred-shadow scratch; a frame needing more compacts in-wave
    int shadow_blocks = 0;         // option "shadow_blocks": workgroups of the deferred shadow pass (0 = auto)
    int shadow_defer = 1;          // measured 1.25 -> 0.99 ms at config 3
    int shadow_cache = 0;          // deferred shadow pass: Worley cube cached in registers per lane
    // The deferred passes' scratch, one set per render stream (round 6): a
    // frame that reuses the cost order writes only its stream's set, so it
    // reads the shared sort scratch like any reader and overlaps the frames
    // of other streams (config 3 with 2 frames in flight).  Past
    // kMaxDeferSets streams a frame shares set 0 and renders as a writer.
    struct DeferSet {
        hipStream_t s = nullptr;
        void* d = nullptr;
        size_t bytes = 0;
        unsigned long long ent_cap = 0;   // entries / step records / waves it holds
        unsigned rec_cap = 0, waves = 0;
    };
    std::vector<DeferSet> defer_sets;
    // entries / step records per pixel-step (per wave-step) of the frame: 5/4 of
    // the largest need seen (proc_scan -> need_host); 1/12 and 1/8 until one is
    double want_ent = 0.0, want_rec = 0.0;
    double need_pixsteps = 0.0, need_wavesteps = 0.0;   // of the frame whose need is pending
    unsigned defer_entries = 0;    // option "shadow_defer_entries": entry capacity override (tests; 0 = sized from the frame)
    int defer_last = 0;            // the last procedural render ran the deferred passes
    // outgrown scratch buffers: queued frames may still use them.  Each gets an
    // event recorded on the render stream of the frame that outgrew it -- after
    // that stream has waited for every earlier procedural render if the frame
    // writes, else on its own stream, the only one that used its set -- and is
    // freed by a later ensure_defer once the event has completed
    struct Retired {
        void* p;
        hipEvent_t ev;             // nullptr until recorded
    };
    std::vector<Retired> defer_retired;
    // The procedural scratch (d_sort, d_defer) is written by a frame that
    // sorts (SORT_BUILD) or defers its shadow rays, and only read by a frame
    // that reuses the order.  A writer waits for every earlier procedural
    // render on other streams; a reader only for the last writer.  So frames
    // that reuse one camera's order overlap on alternating streams (2 in
    // flight), and a frame that writes never races a reader.
    struct ProcUse {
        hipStream_t s;
        hipEvent_t ev;     // recorded after the stream's last procedural render
    };
    std::vector<ProcUse> proc_uses;      // one per stream (at most kMaxProcStreams)
    hipEvent_t proc_wev = nullptr;       // after the last writer
    hipStream_t proc_wstream = nullptr;
    bool proc_wpending = false;
    unsigned long long* h_need = nullptr;   // host-mapped [entries, records] written by the last sorting frame
    unsigned long long* d_need = nullptr;   // its device address
    hipEvent_t need_ev = nullptr;
    bool need_pending = false;
    // regions schedule (build_regions): per-XCD tile lists, double-buffered
    // so a rebuild never waits for more than the render that last used the
    // other buffer (2 frames in flight, VulkanRenderer.cpp:13)
    int wedges = 0;                // wedges per XCD; 0 = auto (wedges_of)
    int split = 0;                 // lanes per ray: 0 = auto, 1, 2, 4, 8
    int slab = 0;                  // COL48 + regions: the LDS slab march (vr_march_slab.hip)
    int proc_enum = 0;             // procedural sort: 1 = 64x64-region enumeration with shadow rays too
    int slab_cap = kSlabMaxChunks; // its chunks per channel (<= kSlabMaxChunks; smaller forces the fallback)
    // regions: each XCD's list 0 = inside-out (ring, angle); 1 = longest tile first;
    // 2 = longest S x S block first (the default since round 4)
    int region_order = 2;
    int wg_waves = 4;              // regions: waves per workgroup (4, 8, 16)
    int supertile = 2;             // regions: list order by S x S blocks of tiles (1 = per tile; 2 measured 1 % faster)
    int region_interval = kRegionRebuildInterval;   // option "region_interval": renders a moved camera reuses the lists
    int region_gpu = 1;            // option "region_gpu": 1 = a moved camera's lists are rebuilt on the GPU
    void* d_rg = nullptr;          // GPU list build scratch (region_build_bytes), zeroed when allocated
    size_t rg_bytes = 0;
    int* h_rghdr = nullptr;        // host-mapped copy of the last GPU build's header (kRegionHeader ints)
    hipEvent_t rg_ev = nullptr;    // recorded after that build
    bool rg_pending = false;
    int rg_buf = -1;               // the region buffer it built
    long long gpu_builds = 0;      // read-only option "region_gpu_builds"
    bool rg_preloaded = false;     // region_build_preload done
    struct RegionBuf {
        unsigned* d = nullptr;     // device: kRegionHeader ints (off[9], tiles with work, longest, tiles), then the list
        unsigned* h = nullptr;     // pinned staging copy (host builds)
        size_t cap = 0;            // entries
        TileMap map{};             // host copy: nwx (and off[] for host builds)
        int most = 0;              // the longest per-XCD list (sizes the launch)
        int most_marched = 0;         // the most marched entries of one XCD (hdr[kRegionWork + x])
        int nwork = 0;             // tiles with estimated work
        int nempty = -1;           // empty tiles (tile_is_empty) in the lists (-1: GPU build not yet complete)
        // The streams that rendered with these lists, and per stream an event
        // recorded after its FIRST render with them (one event per stream and
        // build, never one per render).  These lists are rewritten two builds
        // later; by then every stream that used them has either rendered with
        // the newer lists -- and the newer lists' first-render event on that
        // stream follows all its renders with these -- or it is the rebuilding
        // stream itself, whose order covers them.  A stream that is neither
        // costs a device sync (as do more than kMaxRegionStreams streams).  An
        // event is never recorded on a remembered stream, which the caller may
        // have destroyed since (r04's abort), only on the rendering one.
        hipStream_t streams[kMaxRegionStreams] = {};
        hipEvent_t used[kMaxRegionStreams] = {};
        bool first_rec[kMaxRegionStreams] = {};   // used[i] recorded after stream i's first render
        int nstreams = 0;          // -1: more streams than tracked
        hipEvent_t uploaded = nullptr;   // the list upload (on streams[0]); other streams wait for it
        hipStream_t upload_stream = nullptr;
    } region[2];
    int region_cur = -1;           // buffer of the current lists (-1 = none)
    int region_slot = -1;          // the last render stream's slot in them (note_region_stream)
    float region_key[kRegionKeyLen] = {};   // geometry the current lists were built for
    bool region_exact = false;   // the current lists were built for this render's camera (their empty tiles hold)
    long long renders_since_build = 0;
    // procedural cost sort: the geometry whose order d_sort holds (n per pixel
    // depends only on it, not on the medium), valid until the buffer changes
    std::vector<float> sort_key;
    long long renders_since_sort = 0;   // renders with a stale order since it was built
    int sort_reuse = 0;                 // option "sort_reuse": renders a stale order serves (0 = sort every changed frame)
    // Perlin lattice table of the procedural march (noise::perlin_lattice_entry),
    // built when (seed, lo, n) changes; option "lattice" 0 turns it off
    int lattice = 1;
    // option "inject_throw" (tests of the exception guard): the next vr_render
    // throws std::runtime_error (1) or std::bad_alloc (2) in its host path
    int inject_throw = 0;
    // Launch cache of the grid march (option "launch_cache", default 1): the
    // last few renders' kernel arguments keyed by target and stream, valid
    // while `gen` is unchanged -- every call that can change a grid launch
    // (shader data, march constants, volume, options, a region-list build or
    // a GPU build's sizing) bumps it.  A repeated render of an unchanged frame
    // (the static camera of a frame stream; the two parities of the multi-GPU
    // loop) then skips the basis, plan and list bookkeeping and only launches.
    unsigned long long gen = 1;
    int launch_cache = 1;
    int empty_fill = 1;          // option "empty_fill": regions launches fill the lists' empty tiles, not march them
    int frames_overlap = 0;      // option "frames_overlap": consecutive renders overlap (auto split rule)
    // vr_row_partition's work model: a ray costs steps^(row_pow / 100) + row_setup
    int row_setup = 40, row_pow = 130;   // config 4 at 8 ranks, profiles/r05/row_ranges_c4.txt
    int row_first_pct = 100;     // range 0's share of the work, % of the mean (the loop's rank 0 also assembles)
    struct Cached {
        bool valid = false;
        unsigned long long gen = 0;
        vr_target t{};
        hipStream_t stream = nullptr;
        MarchArgs a{};
        Plan pl{};
        Schedule sc{};
        int kind = 0;
        int slot = -1;   // the stream's slot in the region lists (note_region_render)
    } lc[4];
    int lc_next = 0;
    long long lc_hits = 0;         // read-only option "launch_cache_hits"
    uint2* d_lat = nullptr;
    size_t lat_cap = 0;            // bytes allocated
    long long lat_key[3] = {0, 0, -1};
};

constexpr long long kMaxWorleyTableBytes = 32 << 10;   // LDS per workgroup for the procedural cell table

// ---- vr_api.cpp
int auto_layout(int nx, int ny, int nz);
Ctx* as_ctx(void* p);
void free_volume(Ctx* c);
bool dims_ok(int nx, int ny, int nz);
int wanted_fast_layout(const Ctx* c);
vr_status ensure_fast_layout(Ctx* c, hipStream_t s);
vr_status install_volume(Ctx* c, const uint8_t* d_rgba, int nx, int ny, int nz, hipStream_t s);
vr_status resolve_uniform(Ctx* c);
void tap_constants(const Ctx* c, float S[4][3], float T[4][3]);
bool clamp_is_exact(const Ctx* c, const float S[4][3], const float T[4][3]);
int band_rows_packed(int height, int band_rows, int band_stride, int band_first, int band_flip = 0);
vr_status make_plan(Ctx* c, MarchArgs* a, Plan* p);
const char* variant_name(const Plan& p);

// ---- vr_regions_host.cpp
inline int wedges_of(const Ctx* c)
{
    return c->wedges > 0 ? c->wedges : c->frames_overlap ? kDefaultWedgesOverlap : kDefaultWedges;
}
void box_centre_pixel(const Ctx* c, const MarchArgs& a, int* px, int* prow);
vr_status stream_wait_pending(hipStream_t s, hipEvent_t ev);
vr_status note_region_stream(Ctx::RegionBuf& rb, hipStream_t s, int* slot);
vr_status note_region_render(Ctx* c, hipStream_t s);
int auto_split(const Ctx* c, long long nwork);
void poll_region_header(Ctx* c);
vr_status build_regions(Ctx* c, const MarchArgs& a, int tpw, int cpx, int cprow, hipStream_t stream);

// ---- vr_proc_host.cpp
int worley_z_pitch(int n);
vr_status ensure_lattice(Ctx* c, ProcParams* q, hipStream_t s);
vr_status release_defer(Ctx* c);
vr_status ensure_defer(Ctx* c, const MarchArgs& a, void* sort_buf, hipStream_t s, ShadowDefer* d, bool* ok, bool* shared);
constexpr size_t kMaxDeferSets = 4;

}  // namespace vrapi
