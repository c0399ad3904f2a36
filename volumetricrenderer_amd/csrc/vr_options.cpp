// vr_options.cpp -- vr_set_layout_preference, vr_set_option, vr_get_option and
// vr_kernel_variant (include/vr.h): the tuning and measurement options of a
// context and the name of the march kernel a render would launch.
#include "vr_ctx.h"

using namespace vrapi;

extern "C" {

vr_status vr_set_layout_preference(void* p, int pref)
try {
    if (!p || pref < 0 || pref >= kNumLayouts) return fail(VR_ERR_INVALID, "vr_set_layout_preference: bad argument");
    if (pref > 0 && !layout_built(pref))
        return fail(VR_ERR_INVALID, "vr_set_layout_preference: layout %d is built only with VR_EXPERIMENTS "
                                    "(make EXPERIMENTS=1; measured slower, DESIGN.md sec. 4)", pref);
    Ctx* c = as_ctx(p);
    ++c->gen;
    HIP_TRY(hipSetDevice(c->device));
    c->layout_pref = pref;
    vr_status st = ensure_fast_layout(c, nullptr);
    if (st == VR_OK && hipDeviceSynchronize() != hipSuccess) return fail(VR_ERR_HIP, "vr_set_layout_preference: sync");
    return st;
} catch (...) {
    return caught_exception("vr_set_layout_preference");
}

vr_status vr_set_option(void* p, const char* name, int value)
try {
    if (!p || !name) return fail(VR_ERR_INVALID, "vr_set_option: null argument");
    Ctx* c = as_ctx(p);
    ++c->gen;
    const std::string n(name);
    // variants measured slower than the defaults (vr_internal.h VR_EXPERIMENTS)
    const bool experimental = (n == "schedule" && (value == SCHED_QUEUE || value == SCHED_STRIDED ||
                                                   value == SCHED_XCDROWS)) ||
                              (n == "wg_waves" && value != 4) ||
                              (n == "segment" && value != 0) ||
                              (n == "sort_reuse" && value != 0) ||
                              (n == "proc_enum" && value != 0);
    if (experimental && !VR_EXPERIMENTS)
        return fail(VR_ERR_INVALID, "vr_set_option: %s = %d is built only with VR_EXPERIMENTS (make EXPERIMENTS=1; "
                                    "measured slower, DESIGN.md)", name, value);
    if (n == "layout") return vr_set_layout_preference(p, value);
    if (n == "launch_cache") {
        if (value < 0 || value > 1) return fail(VR_ERR_INVALID, "vr_set_option: launch_cache is 0 or 1");
        c->launch_cache = value;
        return VR_OK;
    }
    if (n == "row_setup" || n == "row_pow" || n == "row_first_pct") {   // vr_row_partition's work model
        if (value < 0 || value > 1000 || (n == "row_pow" && value < 50) || (n == "row_first_pct" && value > 100))
            return fail(VR_ERR_INVALID, "vr_set_option: %s out of range", n.c_str());
        (n == "row_setup" ? c->row_setup : n == "row_pow" ? c->row_pow : c->row_first_pct) = value;
        return VR_OK;
    }
    if (n == "frames_overlap") {   // the caller overlaps consecutive frames on two streams (auto split)
        if (value < 0 || value > 1) return fail(VR_ERR_INVALID, "vr_set_option: frames_overlap is 0 or 1");
        if (c->frames_overlap != value) ++c->gen;
        c->frames_overlap = value;
        return VR_OK;
    }
    if (n == "empty_fill") {   // regions: fill the lists' empty tiles instead of marching them
        if (value < 0 || value > 1) return fail(VR_ERR_INVALID, "vr_set_option: empty_fill is 0 or 1");
        c->empty_fill = value;
        ++c->gen;
        return VR_OK;
    }
    if (n == "inject_throw") {   // test hook: the next vr_render throws in its host path
        if (value < 0 || value > 2)
            return fail(VR_ERR_INVALID, "vr_set_option: inject_throw is 0, 1 (std::runtime_error) or 2 (std::bad_alloc)");
        c->inject_throw = value;
        return VR_OK;
    }
    if (n == "schedule") {
        if (value < -1 || value > 5)
            return fail(VR_ERR_INVALID, "vr_set_option: schedule is -1 (auto), 0 (static), 1 (queue), "
                                        "2 (strided), 3 (xcd rows), 4 (rings) or 5 (regions)");
        c->schedule = value;
        return VR_OK;
    }
    if (n == "waves_per_simd") {
        if (value < 1 || value > 8) return fail(VR_ERR_INVALID, "vr_set_option: waves_per_simd in [1, 8]");
        c->waves_per_simd = value;
        return VR_OK;
    }
    if (n == "tiles_per_wave") {
        if (value < 0 || value > 64)
            return fail(VR_ERR_INVALID, "vr_set_option: tiles_per_wave in [1, 64], or 0 for auto");
        c->tiles_per_wave = value;
        return VR_OK;
    }
    if (n == "split") {
        if (value != 0 && value != 1 && value != 2 && value != 4 && value != 8)
            return fail(VR_ERR_INVALID, "vr_set_option: split is 0 (auto), 1, 2, 4 or 8");
        c->split = value;
        return VR_OK;
    }
    if (n == "wedges") {
        if (value < 0 || value > 64) return fail(VR_ERR_INVALID, "vr_set_option: wedges in [0 (auto), 64]");
        c->wedges = value;
        return VR_OK;
    }
    if (n == "proc_enum") {
        if (value < 0 || value > 1) return fail(VR_ERR_INVALID, "vr_set_option: proc_enum is 0 or 1");
        c->proc_enum = value;
        return VR_OK;
    }
    if (n == "shadow_defer_mib") {
        if (value < 0) return fail(VR_ERR_INVALID, "vr_set_option: shadow_defer_mib >= 0");
        c->shadow_defer_mib = value;
        return value == 0 ? release_defer(c) : VR_OK;
    }
    if (n == "shadow_defer_entries") {
        if (value < 0) return fail(VR_ERR_INVALID, "vr_set_option: shadow_defer_entries >= 0");
        c->defer_entries = (unsigned)value;
        return release_defer(c);
    }
    if (n == "shadow_cache") {
        if (value < 0 || value > 2)
            return fail(VR_ERR_INVALID, "vr_set_option: shadow_cache is 0 (lane per entry), 1 (+ register Worley cube) "
                                        "or 2 (8 lanes per entry)");
        c->shadow_cache = value;
        return VR_OK;
    }
    if (n == "shadow_blocks") {
        if (value < 0 || value > 65536) return fail(VR_ERR_INVALID, "vr_set_option: shadow_blocks in [0, 65536]");
        c->shadow_blocks = value;
        return VR_OK;
    }
    if (n == "shadow_defer") {
        if (value < 0 || value > 1) return fail(VR_ERR_INVALID, "vr_set_option: shadow_defer is 0 or 1");
        c->shadow_defer = value;
        return value == 0 ? release_defer(c) : VR_OK;
    }
    if (n == "slab") {
        if (value < 0 || value > 1) return fail(VR_ERR_INVALID, "vr_set_option: slab is 0 or 1");
        c->slab = value;
        return VR_OK;
    }
    if (n == "slab_cap") {
        if (value < 0 || value > kSlabMaxChunks)
            return fail(VR_ERR_INVALID, "vr_set_option: slab_cap in [0, %d]", kSlabMaxChunks);
        c->slab_cap = value;
        return VR_OK;
    }
    if (n == "region_order") {
        if (value < 0 || value > 2)
            return fail(VR_ERR_INVALID, "vr_set_option: region_order is 0 (inside-out), 1 (longest tile first) or "
                                        "2 (longest block first)");
        c->region_order = value;
        return VR_OK;
    }
    if (n == "wg_waves") {
        if (value != 4 && value != 8 && value != 16) return fail(VR_ERR_INVALID, "vr_set_option: wg_waves is 4, 8 or 16");
        c->wg_waves = value;
        return VR_OK;
    }
    if (n == "supertile") {
        if (value != 1 && value != 2 && value != 4) return fail(VR_ERR_INVALID, "vr_set_option: supertile is 1, 2 or 4");
        c->supertile = value;
        return VR_OK;
    }
    if (n == "region_interval") {
        if (value < 1 || value > 1 << 20) return fail(VR_ERR_INVALID, "vr_set_option: region_interval in [1, 2^20]");
        c->region_interval = value;
        return VR_OK;
    }
    if (n == "region_gpu") {
        if (value < 0 || value > 1) return fail(VR_ERR_INVALID, "vr_set_option: region_gpu is 0 or 1");
        c->region_gpu = value;
        return VR_OK;
    }
    if (n == "uniform_skip") {
        if (value < 0 || value > 1) return fail(VR_ERR_INVALID, "vr_set_option: uniform_skip is 0 or 1");
        c->uniform_skip = value;
        return VR_OK;
    }
    if (n == "sort_reuse") {
        if (value < 0 || value > 64) return fail(VR_ERR_INVALID, "vr_set_option: sort_reuse in [0, 64] renders");
        c->sort_reuse = value;
        return VR_OK;
    }
    if (n == "count") {
        if (value < 0 || value > 2)
            return fail(VR_ERR_INVALID, "vr_set_option: count is 0 (steps), 1 (evals) or 2 (Worley cells)");
        c->count = value;
        return VR_OK;
    }
    if (n == "lattice") {
        if (value < 0 || value > 1) return fail(VR_ERR_INVALID, "vr_set_option: lattice is 0 or 1");
        c->lattice = value;
        return VR_OK;
    }
    return fail(VR_ERR_INVALID, "vr_set_option: unknown option '%s'", name);
} catch (...) {
    return caught_exception("vr_set_option");
}

int vr_get_option(void* p, const char* name)
try {
    if (!p || !name) return -1;
    Ctx* c = as_ctx(p);
    const std::string n(name);
    if (n == "layout") return c->fast_layout ? c->fast_layout : LAYOUT_PLANAR;
    if (n == "schedule") return c->schedule;
    if (n == "waves_per_simd") return c->waves_per_simd;
    if (n == "tiles_per_wave") return c->tiles_per_wave;
    if (n == "count") return c->count;
    if (n == "wedges") return wedges_of(c);   // (the effective count; set 0 for auto)
    if (n == "split") return c->split;
    if (n == "lattice") return c->lattice;
    if (n == "slab") return c->slab;
    if (n == "proc_enum") return c->proc_enum;
    if (n == "shadow_defer") return c->shadow_defer;
    if (n == "shadow_blocks") return c->shadow_blocks;
    if (n == "shadow_cache") return c->shadow_cache;
    if (n == "shadow_defer_mib") return c->shadow_defer_mib;
    if (n == "shadow_defer_entries") return (int)c->defer_entries;
    if (n == "shadow_defer_last") return c->defer_last;   // read-only
    // read-only: 0 = a grid medium; 1 = procedural, frames that reuse one
    // camera's order only read the ctx's scratch (they overlap on two
    // streams); 2 = procedural with deferred shadow rays (round 6: a frame
    // that reuses the order writes only its stream's scratch set, so these
    // overlap too)
    if (n == "procedural") return !c->proc.enabled ? 0 : c->proc.shadow_steps > 0 && c->shadow_defer ? 2 : 1;
    if (n == "shadow_defer_kib") {                        // read-only: the scratch held now (every stream's set), KiB
        size_t b = 0;
        for (const auto& ds : c->defer_sets) b += ds.bytes;
        return (int)std::min<size_t>((b + 1023) / 1024, 0x7fffffff);
    }
    if (n == "slab_cap") return c->slab_cap;
    if (n == "region_order") return c->region_order;
    if (n == "sort_reuse") return c->sort_reuse;
    if (n == "wg_waves") return c->wg_waves;
    if (n == "uniform_skip") return c->uniform_skip;
    if (n == "region_work_tiles")   // read-only: tiles with estimated work in the current region lists
        return c->region_cur >= 0 ? c->region[c->region_cur].nwork : -1;
    if (n == "region_empty_tiles") {   // read-only: tiles of the current lists that are filled, not marched
        poll_region_header(c);   // (a completed GPU build's counts)
        return c->region_cur >= 0 ? c->region[c->region_cur].nempty : -1;
    }
    if (n == "uniform_mask") {   // read-only
        if (!c->d_planar || resolve_uniform(c) != VR_OK) return -1;
        return c->uniform_mask;
    }
    if (n == "supertile") return c->supertile;
    if (n == "launch_cache") return c->launch_cache;
    if (n == "empty_fill") return c->empty_fill;
    if (n == "frames_overlap") return c->frames_overlap;
    if (n == "row_setup") return c->row_setup;
    if (n == "row_pow") return c->row_pow;
    if (n == "row_first_pct") return c->row_first_pct;
    if (n == "launch_cache_hits") return (int)std::min<long long>(c->lc_hits, 0x7fffffff);
    if (n == "experiments") return VR_EXPERIMENTS;   // read-only: the measured-slower variants are built
    if (n == "region_interval") return c->region_interval;
    if (n == "region_gpu") return c->region_gpu;
    if (n == "region_gpu_builds") return (int)std::min<long long>(c->gpu_builds, 0x7fffffff);   // read-only
    return -1;
} catch (...) {
    (void)caught_exception("vr_get_option");
    return -1;
}

const char* vr_kernel_variant(void* p)
try {
    if (!p) return "none";
    Ctx* c = as_ctx(p);
    if (c->proc.enabled) {
        if (c->schedule == SCHED_STATIC) return c->proc.shadow_steps > 0 ? "procedural_shadow_tiles" : "procedural_tiles";
        if (c->schedule == SCHED_RINGS) return c->proc.shadow_steps > 0 ? "procedural_shadow_rings" : "procedural_rings";
        return c->proc.shadow_steps > 0 ? "procedural_shadow" : "procedural";
    }
    if (!c->d_planar || !c->has_camera) return "none";
    if (resolve_uniform(c) != VR_OK) return "none";
    MarchArgs a{};
    Plan pl{};
    make_plan(c, &a, &pl);
    const int kind = c->schedule >= 0 ? c->schedule : SCHED_REGIONS;
    if (pl.layout == LAYOUT_COL48 && c->slab && kind == SCHED_REGIONS && c->split <= 1)
        return pl.early ? "grid_col48_slab_clamp_early" : "grid_col48_slab_clamp";
    const int um = c->uniform_skip ? c->uniform_mask : 0;
    int ch = -1;   // one uniform channel, no loads for it (launch_lw / launch_lat_kd): "_u" + the channel
    if (kind == SCHED_REGIONS && !pl.early && a.zero_offsets && c->wg_waves == 4 &&
        (um == 1 || um == 2 || um == 4 || um == 8) &&
        (pl.layout == LAYOUT_COL48 || pl.layout == LAYOUT_BRICK4832 || pl.layout == LAYOUT_CORNERH ||
         pl.layout == LAYOUT_COL48Z))
        ch = um == 1 ? 0 : um == 2 ? 1 : um == 4 ? 2 : 3;
    if (ch < 0) return variant_name(pl);
    // built once, thread-safe (a function-local static): every layout x early x channel
    struct Names {
        std::string n[kNumLayouts][2][5];
    };
    static const Names table = [] {
        Names t;
        for (int l = 1; l < kNumLayouts; ++l)
            for (int e = 0; e < 2; ++e)
                for (int u = 0; u < 5; ++u) {
                    std::string v = variant_name(Plan{l, WRAP_CLAMP, e == 1});
                    if (u > 0) v += std::string("_u") + "RGBA"[u - 1];
                    t.n[l][e][u] = v;
                }
        return t;
    }();
    return table.n[pl.layout][pl.early ? 1 : 0][ch + 1].c_str();
} catch (...) {
    (void)caught_exception("vr_kernel_variant");
    return "error";
}

}  // extern "C"
