// vr_march_c8.hip -- the CORNER8 / CORNERH (cache-resident volume) instantiations of
// the ray march, in a translation unit of their own so that they compile in
// parallel with vr_march.hip's.  Like vr_march.hip it is built with
// -fno-slp-vectorize (Makefile FLAGS_*): the SLP vectoriser packs pairs of
// scalar lerps into v_pk_* ops, no faster than two plain ones on gfx950, whose
// operands then need v_mov pairs -- 5 % slower for this VALU-bound kernel at
// 128^3 (0.097 -> 0.092 ms without it).
#include "vr_march_kernels.h"

namespace vr {

hipError_t launch_march_corner8(const MarchArgs& a, int layout, bool early, const Schedule& sc, hipStream_t s)
{
    if (layout == LAYOUT_CORNERH) return launch_lw<LAYOUT_CORNERH, WRAP_CLAMP>(a, early, sc, s);
    return launch_lw<LAYOUT_CORNER8, WRAP_CLAMP>(a, early, sc, s);
}

}  // namespace vr

#ifdef VR_TIMELINE
// timing experiments only (make timeline): this translation unit's records
extern "C" int vr_timeline_fetch_c8(unsigned long long* host, int waves)
{
    waves = waves < vr::kTimelineWaves ? waves : vr::kTimelineWaves;
    return (int)hipMemcpyFromSymbol(host, HIP_SYMBOL(vr::g_timeline), (size_t)waves * 3 * sizeof(unsigned long long));
}
extern "C" int vr_timeline_clear_c8()
{
    static unsigned long long zero[vr::kTimelineWaves][3];
    return (int)hipMemcpyToSymbol(HIP_SYMBOL(vr::g_timeline), zero, sizeof(zero));
}
#endif
