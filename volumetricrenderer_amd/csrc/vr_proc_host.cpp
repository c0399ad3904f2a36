// vr_proc_host.cpp -- the host side of the procedural medium (BASELINE configs
// 2/3): its parameters (vr_procedural_defaults, vr_set_procedural), the Worley
// table pitch, the Perlin lattice table and the deferred-shadow scratch.
#include "vr_ctx.h"

namespace vrapi {

// z pitch of the Worley cell table (entries): the smallest pz >= n*n for which
// no two cells at most one apart on each axis share a ds_read_b128 bank slot
// (index mod 16), fewest aliases among cells two apart.  The lanes of a sorted
// wave sit in neighbouring cells; with pz = n*n (81 = 1 mod 16) cells
// (x+1, y, z-1) and (x, y, z) collide.
int worley_z_pitch(int n)
{
    int best = n * n, best_al = 1 << 30;
    for (int pz = n * n; pz < n * n + 16; ++pz) {
        int al1 = 0, al2 = 0;
        for (int dz = -2; dz <= 2; ++dz)
            for (int dy = -2; dy <= 2; ++dy)
                for (int dx = -2; dx <= 2; ++dx) {
                    if (!dx && !dy && !dz) continue;
                    if (((dx + n * dy + pz * dz) % 16 + 16) % 16) continue;
                    (std::abs(dx) <= 1 && std::abs(dy) <= 1 && std::abs(dz) <= 1 ? al1 : al2) += 1;
                }
        const int score = al1 * 1000 + al2;
        if (score < best_al) { best_al = score; best = pz; }
    }
    return best;
}

// Perlin lattice table (global memory) of the procedural march: the fBm's
// octave o samples lattice coordinates P * grid_scale * f_o with P in the
// box, [0, 1]^3 up to rounding; the table covers the cells of every octave,
// with 2 cells of margin, when that is at most 2^24 cells (byte offsets
// then stay exact in fp32; 128 MiB).  Built on `s` and waited for when the
// seed or the range changes (a parameter change, not per frame).
vr_status ensure_lattice(Ctx* c, ProcParams* q, hipStream_t s)
{
    double lo_c = 0.0, hi_c = 0.0;
    float f = q->freq0;
    for (int o = 0; o < q->octaves; ++o) {
        const double G = (double)q->grid_scale * (double)f;
        lo_c = std::min(lo_c, G);
        hi_c = std::max(hi_c, G);
        f = f * q->lacunarity;
    }
    if (!(hi_c - lo_c < 1.0e4) || q->octaves <= 0) return VR_OK;
    const long long lo = (long long)std::floor(lo_c) - 2, n = (long long)std::ceil(hi_c) + 2 - lo + 1;
    if (n * n * n > (1ll << 24)) return VR_OK;
    const size_t bytes = (size_t)(n * n * n) * sizeof(uint2);
    if (!(c->lat_key[0] == q->seed_fbm && c->lat_key[1] == lo && c->lat_key[2] == n)) {
        // renders queued on other streams may still read the old table
        HIP_TRY(hipDeviceSynchronize());
        c->lat_key[2] = -1;
        if (bytes > c->lat_cap) {
            if (c->d_lat) (void)hipFree(c->d_lat);
            c->d_lat = nullptr;
            c->lat_cap = 0;
            if (hipMalloc(&c->d_lat, bytes) != hipSuccess) return fail(VR_ERR_OOM, "vr_render: lattice table");
            c->lat_cap = bytes;
        }
        HIP_TRY(launch_perlin_lattice(c->d_lat, q->seed_fbm, (int)lo, (int)n, s));
        HIP_TRY(hipStreamSynchronize(s));
        c->lat_key[0] = q->seed_fbm;
        c->lat_key[1] = lo;
        c->lat_key[2] = n;
    }
    q->lat = c->d_lat;
    q->lat_bytes = (unsigned)bytes;
    q->lat_c = (float)(8 * lo * (1 + n + n * n));
    q->lat_sy = (float)(8 * n);
    q->lat_sz = (float)(8 * n * n);
    return VR_OK;
}

// Scratch of the deferred shadow passes (ShadowDefer), sized from the frame:
// [chunk count | per-wave step counts, entry counts, first chunks | chunk map |
// step records | entries].  Sorted wave w owns the entries [went[w],
// went[w+1]) and step records [wrec[w], wrec[w+1]) that proc_scan lays out
// from the cost histogram (the sum of its lanes' step-count bounds), so a
// frame needs about its executed lane-steps of entries: 16.7 M (0.27 GB) at
// 1080p x 128 where the old per-wave worst case (64 x max_steps) took 4.2 GB.
// The capacity follows the largest need seen (written by every sorting frame
// into host-mapped memory, read once its event has completed: no host wait),
// x 5/4; before one is known it starts at pixels x max_steps / 16 entries.
// A wave beyond the capacity marches its shadow rays in place, so a frame
// larger than the scratch is still exact, and the next one gets more.
// Growing keeps the outgrown buffer until the frames queued before the growth
// have run (an event, Ctx::Retired; queued frames on other streams may still
// use it): vr_render never waits for the device.
// *ok = false (and VR_OK): no usable scratch (shadow_defer_mib too small, or
// the allocation failed) -- the render then takes the in-wave compaction.
vr_status release_defer(Ctx* c)
{
    if (c->defer_sets.empty() && c->defer_retired.empty()) return VR_OK;
    HIP_TRY(hipSetDevice(c->device));
    HIP_TRY(hipDeviceSynchronize());   // an option change, not a frame: queued renders may use the scratch
    for (const auto& ds : c->defer_sets)
        if (ds.d) (void)hipFree(ds.d);
    for (const auto& q : c->defer_retired) {
        (void)hipFree(q.p);
        if (q.ev) (void)hipEventDestroy(q.ev);
    }
    c->defer_retired.clear();
    c->defer_sets.clear();
    c->want_ent = c->want_rec = 0.0;
    return VR_OK;
}

vr_status ensure_defer(Ctx* c, const MarchArgs& a, void* sort_buf, hipStream_t s, ShadowDefer* d, bool* ok, bool* shared)
{
    *ok = false;
    *shared = false;
    // free the outgrown buffers whose frames have run
    for (size_t i = 0; i < c->defer_retired.size();) {
        Ctx::Retired& q = c->defer_retired[i];
        const hipError_t st = q.ev ? hipEventQuery(q.ev) : hipErrorNotReady;
        if (st == hipSuccess) {
            (void)hipFree(q.p);
            (void)hipEventDestroy(q.ev);
            c->defer_retired.erase(c->defer_retired.begin() + (long)i);
        } else {
            if (q.ev) (void)hipGetLastError();   // not an error: still queued
            ++i;
        }
    }
    if (c->shadow_defer_mib == 0) return VR_OK;
    const SortLayout L = sort_layout(a.width, a.out_rows);
    const unsigned long long pixels = (unsigned long long)a.width * (unsigned long long)a.out_rows;
    if (!c->h_need) {
        HIP_TRY(hipHostMalloc(&c->h_need, 2 * sizeof(unsigned long long), hipHostMallocMapped));
        HIP_TRY(hipHostGetDevicePointer(reinterpret_cast<void**>(&c->d_need), c->h_need, 0));
        HIP_TRY(hipEventCreateWithFlags(&c->need_ev, hipEventDisableTiming));
    }
    if (c->need_pending) {   // the last sorting frame's need, if it has run
        const hipError_t q = hipEventQuery(c->need_ev);
        if (q == hipSuccess) {
            c->need_pending = false;
            c->want_ent = std::max(c->want_ent, 1.25 * (double)c->h_need[0] / c->need_pixsteps);
            c->want_rec = std::max(c->want_rec, 1.25 * (double)c->h_need[1] / c->need_wavesteps);
        } else if (q == hipErrorNotReady) {
            (void)hipGetLastError();   // not an error: the frame is still queued
        } else {
            return fail(VR_ERR_HIP, "vr_render: need event: %s", hipGetErrorString(q));
        }
    }
    const unsigned long long steps = (unsigned long long)std::max(a.max_steps, 1);
    constexpr unsigned long long kMaxCap = 0xffff0000ull;   // entry / record indices stay 32-bit
    const double pixsteps = (double)pixels * (double)steps, wavesteps = (double)L.waves * (double)steps;
    unsigned long long ent = (unsigned long long)std::min(4.0e9, pixsteps * std::max(c->want_ent, 1.0 / 12.0));
    unsigned long long rec = (unsigned long long)std::min(4.0e9, wavesteps * std::max(c->want_rec, 0.125));
    ent = std::max(ent, 4096ull);
    rec = std::max(rec, 1024ull);
    if (c->defer_entries) ent = c->defer_entries;   // test override
    auto up = [](size_t v) { return (v + 255) & ~(size_t)255; };
    struct Off { size_t ws, wc, wk, map, rec, ent, bytes; };
    auto layout = [&](unsigned long long e, unsigned long long r, unsigned w) {
        Off o{};
        o.ws = 256;
        o.wc = up(o.ws + (size_t)w * 4);
        o.wk = up(o.wc + (size_t)w * 4);
        o.map = up(o.wk + (size_t)w * 4);
        o.rec = up(o.map + (size_t)(e / 64 + w) * sizeof(uint4));
        o.ent = up(o.rec + (size_t)r * sizeof(uint4));
        o.bytes = o.ent + (size_t)e * sizeof(float4);
        return o;
    };
    // this stream's set (a new one for a new stream, up to kMaxDeferSets)
    Ctx::DeferSet* set = nullptr;
    for (auto& x : c->defer_sets)
        if (x.s == s) set = &x;
    if (!set) {
        if (c->defer_sets.size() < kMaxDeferSets) {
            c->defer_sets.push_back(Ctx::DeferSet{});
            set = &c->defer_sets.back();
            set->s = s;
        } else {
            set = &c->defer_sets[0];   // shared: the frame renders as a writer
            *shared = true;
        }
    }
    Ctx::DeferSet& ds = *set;
    const unsigned waves = std::max(L.waves, ds.waves);
    const bool fits = ds.d && L.waves <= ds.waves && rec <= ds.rec_cap &&
                      (c->defer_entries ? ent == ds.ent_cap : ent <= ds.ent_cap);
    if (!fits) {
        if (ds.d && !c->defer_entries) {   // grow by at least 1/4: a slowly growing need reallocates rarely
            ent = std::max(ent, ds.ent_cap + ds.ent_cap / 4);
            rec = std::max(rec, (unsigned long long)ds.rec_cap + ds.rec_cap / 4);
        }
        ent = std::min(ent, kMaxCap);
        rec = std::min(rec, kMaxCap);
        const size_t limit = (size_t)c->shadow_defer_mib << 20;
        if (layout(ent, rec, waves).bytes > limit) {   // fewer entries: the last waves march in place
            const size_t base = layout(0, rec, waves).bytes + 256;
            ent = base < limit ? (limit - base) / (sizeof(float4) + sizeof(uint4) / 64 + 1) : 0;
        }
        void* nb = nullptr;
        const Off o = layout(ent, rec, waves);
        if (ent < 4096 || o.bytes > limit || hipMalloc(&nb, o.bytes) != hipSuccess) {
            (void)hipGetLastError();   // clear an allocation error; keep what there is
            if (!ds.d || L.waves > ds.waves) return VR_OK;
        } else {
            if (ds.d) {
                c->defer_retired.push_back({ds.d, nullptr});   // its event: vr_render, before the launch
                if (c->defer_retired.size() > kMaxDeferRetired) {   // rare: a device sync frees them
                    HIP_TRY(hipDeviceSynchronize());
                    for (const auto& q : c->defer_retired) {
                        (void)hipFree(q.p);
                        if (q.ev) (void)hipEventDestroy(q.ev);
                    }
                    c->defer_retired.clear();   // the device is idle: the old scratch too
                }
            }
            ds.d = nb;
            ds.bytes = o.bytes;
            ds.ent_cap = ent;
            ds.rec_cap = (unsigned)rec;
            ds.waves = waves;
        }
    }
    const Off o = layout(ds.ent_cap, ds.rec_cap, ds.waves);
    *ok = true;
    char* b = static_cast<char*>(ds.d);
    char* sb = static_cast<char*>(sort_buf);
    d->count = reinterpret_cast<unsigned*>(b);
    d->wsteps = reinterpret_cast<unsigned*>(b + o.ws);
    d->wcount = reinterpret_cast<unsigned*>(b + o.wc);
    d->wchunk = reinterpret_cast<unsigned*>(b + o.wk);
    d->map = reinterpret_cast<uint4*>(b + o.map);
    d->rec = reinterpret_cast<uint4*>(b + o.rec);
    d->ent = reinterpret_cast<float4*>(b + o.ent);
    d->went = reinterpret_cast<const unsigned long long*>(sb + L.went);
    d->wrec = reinterpret_cast<const unsigned*>(sb + L.wrec);
    d->ent_cap = ds.ent_cap;
    d->rec_cap = ds.rec_cap;
    d->map_cap = (unsigned)(ds.ent_cap / 64 + ds.waves);
    d->waves = L.waves;
    // the shadow pass's grid: ~2-3 chunks per wave rather than one persistent
    // round (1,536 workgroups at 6 per CU), so the hardware dispatcher balances
    // the tail -- 3/8 of the sorted waves measured 0.90-0.91 ms against 0.98 at
    // config 3 (profiles/r03/ab_shadow_blocks_*.txt)
    d->worley_cache = c->shadow_cache;
    d->eval_blocks = c->shadow_blocks ? (unsigned)c->shadow_blocks
                                      : (unsigned)std::max<size_t>(kShadowEvalBlocks, (size_t)L.waves * 3 / 8);
    return VR_OK;
}
}  // namespace vrapi

using namespace vrapi;

extern "C" {

vr_status vr_procedural_defaults(vr_procedural* p)
try {
    if (!p) return fail(VR_ERR_INVALID, "vr_procedural_defaults: null");
    std::memset(p, 0, sizeof *p);
    p->enabled = 0;
    p->grid_scale = 128.0f;     // TestMain.cpp:51 grid, frequencies in texel units
    p->octaves = 4;
    p->freq0 = 0.19f;           // TestMain.cpp:61
    p->lacunarity = 2.0f;
    p->gain = 0.5f;
    p->seed_fbm = 3;
    p->worley_freq = 0.03f;     // TestMain.cpp:60
    p->seed_worley = 2;
    p->shadow_steps = 0;
    const double n = std::sqrt(1.0 + 1.0 + 4.0);
    p->sun_dir[0] = (float)(1.0 / n); p->sun_dir[1] = (float)(1.0 / n); p->sun_dir[2] = (float)(2.0 / n);
    return VR_OK;
} catch (...) {
    return caught_exception("vr_procedural_defaults");
}


vr_status vr_set_procedural(void* ctx, const vr_procedural* p)
try {
    if (!ctx || !p) return fail(VR_ERR_INVALID, "vr_set_procedural: null argument");
    if (p->enabled) {
        if (p->octaves < 0 || p->octaves > 16) return fail(VR_ERR_INVALID, "vr_set_procedural: octaves in [0,16]");
        if (p->shadow_steps < 0 || p->shadow_steps > 256)
            return fail(VR_ERR_INVALID, "vr_set_procedural: shadow_steps in [0,256]");
        const double l = std::sqrt((double)p->sun_dir[0] * p->sun_dir[0] + (double)p->sun_dir[1] * p->sun_dir[1] +
                                   (double)p->sun_dir[2] * p->sun_dir[2]);
        if (p->shadow_steps > 0 && !(l > 0.0)) return fail(VR_ERR_INVALID, "vr_set_procedural: zero sun_dir");
        if (p->reserved) return fail(VR_ERR_INVALID, "vr_set_procedural: reserved must be 0");
        if (!std::isfinite(p->grid_scale) || !std::isfinite(p->freq0) || !std::isfinite(p->lacunarity) ||
            !std::isfinite(p->gain) || !std::isfinite(p->worley_freq) || !std::isfinite(p->sun_dir[0]) ||
            !std::isfinite(p->sun_dir[1]) || !std::isfinite(p->sun_dir[2]))
            return fail(VR_ERR_INVALID, "vr_set_procedural: parameters must be finite");
    }
    Ctx* c = as_ctx(ctx);
    ++c->gen;
    c->proc = *p;
    if (p->enabled && p->shadow_steps > 0) {   // normalise in double, round once
        const double l = std::sqrt((double)p->sun_dir[0] * p->sun_dir[0] + (double)p->sun_dir[1] * p->sun_dir[1] +
                                   (double)p->sun_dir[2] * p->sun_dir[2]);
        for (int a = 0; a < 3; ++a) c->proc.sun_dir[a] = (float)((double)p->sun_dir[a] / l);
    }
    return VR_OK;
} catch (...) {
    return caught_exception("vr_set_procedural");
}

}  // extern "C"
