// vr_march.hip -- the hot path: per-pixel volumetric ray march for gfx950.
//
// Replaces shaders/frag.glsl:34-81 (and the coverage that vert.glsl:17-22
// plus rasterisation provide).  Each lane traces one ray and a wave64 owns an
// 8x8 pixel tile.  The work is gather + fp32 VALU; there is no dense
// contraction, so nothing here uses MFMA.
//
// The op sequence is the fp32 spec of DESIGN.md sec. 3.  The oracle
// (oracle/vr_oracle.c) restates the same spec, and results agree bit for bit.
// Packed fp32 ops (v_pk_fma_f32 / v_pk_add_f32) compute two independent IEEE
// lerps per instruction.  Built with -ffp-contract=off: the only fused ops
// are the explicit fma calls.
#include "vr_march_kernels.h"

namespace vr {

SortLayout sort_layout(int width, int out_rows)
{
    // hist, cursor (+ total), order (u32 per pixel), keys (u16 per enumerated
    // position: whole 64x64 regions, kSortRegion), then the deferred shadow
    // passes' per-wave prefixes (proc_scan) and the frame's totals
    auto up = [](size_t v) { return (v + 255) & ~(size_t)255; };
    SortLayout L{};
    const size_t pixels = (size_t)width * (size_t)out_rows;
    const size_t regions = (size_t)((width + kSortRegion - 1) / kSortRegion) * ((out_rows + kSortRegion - 1) / kSortRegion);
    L.waves = (unsigned)((pixels + 63) / 64);
    L.hist = 0;
    L.cursor = kKeyBins * sizeof(unsigned);
    L.order = (size_t)(2 * kKeyBins + 64) * sizeof(unsigned);
    L.keys = L.order + pixels * 4u;
    L.went = up(L.keys + regions * kSortRegion * kSortRegion * 2u);
    L.wrec = up(L.went + ((size_t)L.waves + 1) * sizeof(unsigned long long));
    L.need = up(L.wrec + ((size_t)L.waves + 1) * sizeof(unsigned));
    L.bytes = L.need + 2 * sizeof(unsigned long long);
    return L;
}

hipError_t launch_march_procedural(const MarchArgs& a, bool early, void* sort_buf, int reuse_sort, const Schedule& sc,
                                   hipStream_t s, const ShadowDefer* defer, unsigned long long* need_host)
{
    if (a.width <= 0 || a.out_rows <= 0) return hipSuccess;
    const bool shadow = a.proc.shadow_steps > 0;
    const size_t wt_bytes =
        a.proc.wt_n > 0 ? ((size_t)a.proc.wt_n * a.proc.wt_pz + 512) * sizeof(float4) : 0;
    if (sort_buf) {
        const SortLayout L = sort_layout(a.width, a.out_rows);
        char* sb = static_cast<char*>(sort_buf);
        unsigned* hist = reinterpret_cast<unsigned*>(sb + L.hist);
        unsigned* cursor = reinterpret_cast<unsigned*>(sb + L.cursor);   // kKeyBins + 1 entries
        unsigned* order = reinterpret_cast<unsigned*>(sb + L.order);
        unsigned short* keys = reinterpret_cast<unsigned short*>(sb + L.keys);
        // hist is all zero here: zeroed when the buffer was allocated, and by
        // the previous frame's proc_scan after it read it
        const long long pixels = (long long)a.width * a.out_rows;
        static_assert(kSortRegion * kSortRegion == 256 * kSortPixelsPerThread, "one 64x64 region per sort block");
        const dim3 g1((unsigned)(((a.width + kSortRegion - 1) / kSortRegion) * ((a.out_rows + kSortRegion - 1) / kSortRegion)));
        // same geometry as the frame that built keys / order / total: only the
        // pixels without steps need writing, by trailing blocks of the march
        const unsigned positions = reuse_sort != SORT_BUILD ? g1.x * 256u * kSortPixelsPerThread : 0u;
        if (reuse_sort == SORT_BUILD) {
            if (shadow) hipLaunchKernelGGL((proc_bin<true>), g1, dim3(256), 0, s, a, hist, keys);
            else hipLaunchKernelGGL((proc_bin<false>), g1, dim3(256), 0, s, a, hist, keys);
            // with shadow rays proc_scan also lays out the deferred passes' per-wave ranges
            ScanOut so{};
            if (shadow) {
                so.went = reinterpret_cast<unsigned long long*>(sb + L.went);
                so.wrec = reinterpret_cast<unsigned*>(sb + L.wrec);
                so.need = reinterpret_cast<unsigned long long*>(sb + L.need);
                so.need_host = need_host;
                so.max_steps = a.max_steps;
            }
            hipLaunchKernelGGL(proc_scan, dim3(1), dim3(kKeyBins), 0, s, hist, cursor, so);
            hipLaunchKernelGGL(proc_scatter, g1, dim3(256), 0, s, a, keys, cursor, order);
        }
        // the scatter advanced cursor[k] to the end of key k; total stays at cursor[kKeyBins]
        const unsigned march_blocks = (unsigned)((pixels + kThreads - 1) / kThreads);
        const dim3 g4(march_blocks + (positions + kThreads * 16 - 1) / (kThreads * 16));
        const unsigned* total = cursor + kKeyBins;
        // tables: 2 = the fixed 9-cell Worley geometry (compile-time offsets), 1 = runtime geometry,
        // 3 = 2 + the Perlin lattice table
        const int tm = wt_bytes ? (a.proc.wt_fixed ? (a.proc.lat ? 3 : 2) : 1) : 0;
        if (shadow && defer && tm >= 2) {   // deferred shadow rays: three passes (vr_march_kernels.h)
            const ShadowDefer d = *defer;
            const bool stale = reuse_sort == SORT_STALE;
#define VR_PD(E, T)                                                                                                  \
    do {                                                                                                             \
        hipLaunchKernelGGL((march_proc_defer<E, T>), g4, dim3(kThreads), wt_bytes, s, a, order, total, keys,        \
                           positions, march_blocks, stale, d);                                                       \
        hipLaunchKernelGGL(proc_shadow_scan, dim3(1), dim3(kScanThreads), 0, s, total, d);                          \
        hipLaunchKernelGGL(proc_shadow_map, dim3((d.waves + 3) / 4), dim3(kThreads), 0, s, total, d);               \
        if (d.worley_cache == 2) hipLaunchKernelGGL((proc_shadow_eval8<T>), dim3(d.eval_blocks ? d.eval_blocks : kShadowEvalBlocks), dim3(kThreads), wt_bytes, s, a, d); \
        else if (d.worley_cache) hipLaunchKernelGGL((proc_shadow_eval<T, true>), dim3(d.eval_blocks ? d.eval_blocks : kShadowEvalBlocks), dim3(kThreads), wt_bytes, s, a, d); \
        else hipLaunchKernelGGL((proc_shadow_eval<T, false>), dim3(d.eval_blocks ? d.eval_blocks : kShadowEvalBlocks), dim3(kThreads), wt_bytes, s, a, d); \
    } while (0)
            if (tm == 3) {
                if (early) VR_PD(true, 3); else VR_PD(false, 3);
            } else {
                if (early) VR_PD(true, 2); else VR_PD(false, 2);
            }
#undef VR_PD
            hipLaunchKernelGGL(proc_shadow_resolve, dim3(march_blocks), dim3(kThreads), 0, s, a, order, total, d);
            return hipGetLastError();
        }
        const int v = (shadow ? 4 : 0) | (early ? 2 : 0);
#define VR_PS(S, E, T) \
    hipLaunchKernelGGL((march_proc_sorted<S, E, T>), g4, dim3(kThreads), wt_bytes, s, a, order, total, keys, positions, \
                       march_blocks, reuse_sort == SORT_STALE)
#define VR_PS3(S, E) \
    if (tm == 3) VR_PS(S, E, 3); \
    else if (tm == 2) VR_PS(S, E, 2); \
    else if (tm == 1) VR_PS(S, E, 1); \
    else VR_PS(S, E, 0)
        switch (v) {
        case 0: VR_PS3(false, false); break;
        case 2: VR_PS3(false, true); break;
        case 4: VR_PS3(true, false); break;
        default: VR_PS3(true, true); break;
        }
#undef VR_PS3
#undef VR_PS
        return hipGetLastError();
    }
    const int tiles_x8 = (a.width + 7) >> 3, rows8 = (a.out_rows + 7) >> 3;
    long long waves = (long long)tiles_x8 * rows8;
    int cx = -1, cy = -1;
    if (sc.kind == SCHED_RINGS) {
        cx = min(max(sc.center_x >> 3, 0), tiles_x8 - 1);
        cy = min(max(sc.center_y >> 3, 0), rows8 - 1);
        const int R = max(max(cx, tiles_x8 - 1 - cx), max(cy, rows8 - 1 - cy));
        waves = (2ll * R + 1) * (2ll * R + 1);
    }
    const dim3 grid((unsigned)((waves + 3) / 4)), block(kThreads);
    // the fixed geometry is also a valid runtime geometry (n = 9, pz = 83)
    const int v = (shadow ? 4 : 0) | (early ? 2 : 0) | (wt_bytes ? 1 : 0);
#define VR_PT(S, E, T) hipLaunchKernelGGL((march_proc<S, E, T>), grid, block, wt_bytes, s, a, cx, cy)
    switch (v) {
    case 0: VR_PT(false, false, 0); break;
    case 1: VR_PT(false, false, 1); break;
    case 2: VR_PT(false, true, 0); break;
    case 3: VR_PT(false, true, 1); break;
    case 4: VR_PT(true, false, 0); break;
    case 5: VR_PT(true, false, 1); break;
    case 6: VR_PT(true, true, 0); break;
    default: VR_PT(true, true, 1); break;
    }
#undef VR_PT
    return hipGetLastError();
}

hipError_t launch_march(const MarchArgs& a, int layout, int wrap, bool early, const Schedule& sc, hipStream_t s)
{
    if (a.width <= 0 || a.out_rows <= 0) return hipSuccess;
    switch (layout) {
    case LAYOUT_BRICK4832: return launch_lw<LAYOUT_BRICK4832, WRAP_CLAMP>(a, early, sc, s);
    case LAYOUT_COL48:
        if (sc.kind == SCHED_REGIONS && sc.slab && sc.split <= 1) return launch_march_slab(a, early, sc, s);
        return launch_lw<LAYOUT_COL48, WRAP_CLAMP>(a, early, sc, s);
#if VR_EXPERIMENTS
    case LAYOUT_BRICK4: return launch_lw<LAYOUT_BRICK4, WRAP_CLAMP>(a, early, sc, s);
    case LAYOUT_BRICK448: return launch_lw<LAYOUT_BRICK448, WRAP_CLAMP>(a, early, sc, s);
    case LAYOUT_BRICK488: return launch_lw<LAYOUT_BRICK488, WRAP_CLAMP>(a, early, sc, s);
    case LAYOUT_BRICK4816: return launch_lw<LAYOUT_BRICK4816, WRAP_CLAMP>(a, early, sc, s);
    case LAYOUT_BRICK4864: return launch_lw<LAYOUT_BRICK4864, WRAP_CLAMP>(a, early, sc, s);
    case LAYOUT_BRICK41616: return launch_lw<LAYOUT_BRICK41616, WRAP_CLAMP>(a, early, sc, s);
    case LAYOUT_COL48Z: return launch_lw<LAYOUT_COL48Z, WRAP_CLAMP>(a, early, sc, s);
    case LAYOUT_ZPAIR: return launch_lw<LAYOUT_ZPAIR, WRAP_CLAMP>(a, early, sc, s);
    case LAYOUT_BRICK5: return launch_lw<LAYOUT_BRICK5, WRAP_CLAMP>(a, early, sc, s);
    case LAYOUT_BRICK8: return launch_lw<LAYOUT_BRICK8, WRAP_CLAMP>(a, early, sc, s);
    case LAYOUT_BRICK16: return launch_lw<LAYOUT_BRICK16, WRAP_CLAMP>(a, early, sc, s);
#endif
    case LAYOUT_CORNER8:
    case LAYOUT_CORNERH: return launch_march_corner8(a, layout, early, sc, s);   // vr_march_c8.hip
    default: break;
    }
    if (wrap == WRAP_CLAMP) return launch_lw<LAYOUT_PLANAR, WRAP_CLAMP>(a, early, sc, s);
    return launch_lw<LAYOUT_PLANAR, WRAP_MIRROR>(a, early, sc, s);
}

}  // namespace vr

#ifdef VR_TIMELINE
// timing experiments only (make timeline): copy / clear the per-wave records
// of the regions kernels compiled in this translation unit
extern "C" int vr_timeline_fetch(unsigned long long* host, int waves)
{
    waves = waves < vr::kTimelineWaves ? waves : vr::kTimelineWaves;
    return (int)hipMemcpyFromSymbol(host, HIP_SYMBOL(vr::g_timeline), (size_t)waves * 3 * sizeof(unsigned long long));
}
extern "C" int vr_timeline_clear()
{
    static unsigned long long zero[vr::kTimelineWaves][3];
    return (int)hipMemcpyToSymbol(HIP_SYMBOL(vr::g_timeline), zero, sizeof(zero));
}
#endif
