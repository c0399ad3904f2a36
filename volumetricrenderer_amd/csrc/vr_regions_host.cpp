// vr_regions_host.cpp -- the host side of the regions schedule: the box-centre
// pixel, the per-XCD tile lists (build_regions; the GPU build for a moving
// camera is vr_regions.hip), their stream bookkeeping, and the balanced row
// partition of the multi-GPU loop (vr_row_partition).
#include "vr_ctx.h"

namespace vrapi {

// Target pixel (x, packed output row) under the projected box centre: the
// centre of the ring schedule.  Model, View, Projection are column-major
// (vr_object_shader_data); the product is applied to the box-centre point.
void box_centre_pixel(const Ctx* c, const MarchArgs& a, int* px, int* prow)
{
    const float* M = c->obj;
    const float* V = c->obj + 16;
    const float* P = c->obj + 32;
    double v[4] = {0.5 * ((double)a.box_min[0] + a.box_max[0]), 0.5 * ((double)a.box_min[1] + a.box_max[1]),
                   0.5 * ((double)a.box_min[2] + a.box_max[2]), 1.0};
    for (const float* m : {M, V, P}) {
        double o[4];
        for (int r = 0; r < 4; ++r) o[r] = m[r] * v[0] + m[4 + r] * v[1] + m[8 + r] * v[2] + m[12 + r] * v[3];
        for (int r = 0; r < 4; ++r) v[r] = o[r];
    }
    double sx = 0.5 * a.width, sy = 0.5 * a.height;
    if (v[3] > 0.0) {
        sx = (v[0] / v[3] * 0.5 + 0.5) * a.width;
        sy = (v[1] / v[3] * 0.5 + 0.5) * a.height;
    }
    const int y = (int)std::min(std::max(sy, 0.0), (double)(a.height - 1));
    int row = y;
    if (a.band_rows > 0 && (a.band_stride > 1 || a.band_first > 0)) {   // near this rank's packed rows (flips aside)
        const int b = y / a.band_rows;
        const int sel = b >= a.band_first ? (b - a.band_first) / a.band_stride : 0;
        row = sel * a.band_rows + y % a.band_rows;
    }
    *px = (int)std::min(std::max(sx, 0.0), (double)(a.width - 1));
    *prow = std::min(std::max(row, 0), std::max(a.out_rows - 1, 0));
}

// Regions schedule (SCHED_REGIONS): deal the 8x8 tiles of
// the target to the 8 XCDs as contiguous angular wedges around the projected
// box centre, `wedges` per XCD, with equal estimated work, so that the tiles
// one L2 serves are mostly neighbours (their rays read the same bricks).  The
// work estimate of a tile is the longest a3 step count of the rays through its
// 4 corners (double, no clip test; one ray per tile corner of the frame).
// Each XCD walks its tiles inside-out (Chebyshev ring, then angle), so its
// longest rays start first; tiles without estimated work (background, or a
// silhouette edge missing every corner) follow, dealt round-robin.  Every tile
// is in exactly one list whatever the estimate, so a list built for an older
// camera stays correct: a moving camera reuses it for kRegionRebuildInterval
// renders.  Rebuilds go to the other of two buffers, once the renders that
// last read it are done (an event recorded when it was retired, on its one
// render stream; a device sync if several streams used it), uploaded on the
// render stream.
//
// `s` waits for `ev` unless it has already completed (an event recorded on a
// stream the caller has destroyed since is complete: no wait is queued for it)
vr_status stream_wait_pending(hipStream_t s, hipEvent_t ev)
{
    const hipError_t q = hipEventQuery(ev);
    if (q == hipSuccess) return VR_OK;
    if (q != hipErrorNotReady) return fail(VR_ERR_HIP, "vr_render: event query: %s", hipGetErrorString(q));
    (void)hipGetLastError();   // not an error: still queued
    HIP_TRY(hipStreamWaitEvent(s, ev, 0));
    return VR_OK;
}

// The render stream s uses the lists: *slot = its index in rb.streams (-1:
// untracked, more streams than kMaxRegionStreams)
vr_status note_region_stream(Ctx::RegionBuf& rb, hipStream_t s, int* slot)
{
    *slot = -1;
    if (rb.nstreams < 0) return VR_OK;
    for (int i = 0; i < rb.nstreams; ++i)
        if (rb.streams[i] == s) {
            *slot = i;
            return VR_OK;
        }
    if (s != rb.upload_stream) {   // first use on another stream
        const vr_status st = stream_wait_pending(s, rb.uploaded);
        if (st != VR_OK) return st;
    }
    if (rb.nstreams == kMaxRegionStreams) {
        rb.nstreams = -1;
        return VR_OK;
    }
    if (!rb.used[rb.nstreams]) HIP_TRY(hipEventCreateWithFlags(&rb.used[rb.nstreams], hipEventDisableTiming));
    rb.first_rec[rb.nstreams] = false;
    *slot = rb.nstreams;
    rb.streams[rb.nstreams++] = s;
    return VR_OK;
}

// After a regions launch on stream s (slot c->region_slot of the current
// lists): the stream's first render with these lists records its event
vr_status note_region_render(Ctx* c, hipStream_t s)
{
    if (c->region_cur < 0 || c->region_slot < 0) return VR_OK;
    Ctx::RegionBuf& rb = c->region[c->region_cur];
    if (c->region_slot >= rb.nstreams || rb.first_rec[c->region_slot]) return VR_OK;
    HIP_TRY(hipEventRecord(rb.used[c->region_slot], s));
    rb.first_rec[c->region_slot] = true;
    return VR_OK;
}

// lanes per ray of a regions frame: option split, or auto from the tiles with work
int auto_split(const Ctx* c, long long nwork)
{
    if (c->split > 0) return c->split;
    return nwork >= (c->frames_overlap ? kSplitOneLaneOverlap : kSplitOneLane) ? 1 : nwork >= kSplitTwoLanes ? 2 : 4;
}

// The lists of the GPU build that last completed (host-mapped header, read
// once its event is done -- never waited for): tiles with work and the longest
// list, which size the next launches of the same target.
void poll_region_header(Ctx* c)
{
    if (!c->rg_pending) return;
    const hipError_t q = hipEventQuery(c->rg_ev);
    if (q == hipErrorNotReady) {
        (void)hipGetLastError();   // not an error: the build is still queued
        return;
    }
    c->rg_pending = false;
    ++c->gen;   // the next launches are sized from the completed build
    if (q != hipSuccess) return;
    Ctx::RegionBuf& rb = c->region[c->rg_buf];
    rb.nwork = c->h_rghdr[9];
    rb.most = c->h_rghdr[10];
    rb.most_marched = 0;
    rb.nempty = 0;
    for (int x = 0; x < 8; ++x) {
        rb.most_marched = std::max(rb.most_marched, c->h_rghdr[kRegionWork + x]);
        rb.nempty += c->h_rghdr[x + 1] - c->h_rghdr[x] - c->h_rghdr[kRegionWork + x];
    }
}

// Pick the buffer for new lists, sized for n entries: the one the current
// lists replaced (two builds old), once the renders that used it are done --
// the new lists are written on `stream` (GPU build, or the upload of a host
// build), so `stream` waits for the other streams' renders (RegionBuf);
// host_staging: the host also rewrites that buffer's pinned staging copy,
// once its last upload has run.
vr_status next_region_buf(Ctx* c, size_t n, bool host_staging, hipStream_t stream, int* out)
{
    c->region_slot = -1;
    const int b = c->region_cur < 0 ? 0 : c->region_cur ^ 1;
    Ctx::RegionBuf& rb = c->region[b];
    if (c->rg_pending && c->rg_buf == b) {   // a GPU build into this buffer is still queued
        HIP_TRY(hipEventSynchronize(c->rg_ev));
        poll_region_header(c);
    }
    if (host_staging && rb.uploaded && rb.h) HIP_TRY(hipEventSynchronize(rb.uploaded));   // the staging copy is free
    const Ctx::RegionBuf* newer = c->region_cur >= 0 ? &c->region[c->region_cur] : nullptr;
    bool sync = rb.nstreams < 0;
    for (int i = 0; i < rb.nstreams && !sync; ++i) {
        if (rb.streams[i] == stream) continue;   // this stream's order covers its renders
        int j = -1;
        for (int k = 0; newer && k < newer->nstreams; ++k)
            if (newer->streams[k] == rb.streams[i] && newer->first_rec[k]) j = k;
        if (j < 0) {
            sync = true;   // a stream that never rendered with the newer lists
        } else {
            const vr_status st = stream_wait_pending(stream, newer->used[j]);
            if (st != VR_OK) return st;
        }
    }
    if (sync) HIP_TRY(hipDeviceSynchronize());
    rb.nstreams = 0;
    if (n > rb.cap) {
        if (rb.d) {
            HIP_TRY(hipStreamSynchronize(stream));   // the stream may have queued work on the old list
            (void)hipFree(rb.d);
        }
        if (rb.h) (void)hipHostFree(rb.h);
        rb.d = rb.h = nullptr;
        rb.cap = 0;
        HIP_TRY(hipMalloc(&rb.d, (n + kRegionHeader) * sizeof(unsigned)));
        HIP_TRY(hipHostMalloc(&rb.h, (n + kRegionHeader) * sizeof(unsigned), hipHostMallocDefault));
        rb.cap = n;
    }
    *out = b;
    return VR_OK;
}

vr_status build_regions(Ctx* c, const MarchArgs& a, int tpw, int cpx, int cprow, hipStream_t stream)
{
    const int tw = (a.width + 7) >> 3, th = (a.out_rows + 7) >> 3;
    float key[kRegionKeyLen] = {(float)tw, (float)th, (float)a.width, (float)a.height, (float)a.out_rows,
                                (float)a.band_rows, (float)a.band_stride, (float)a.band_first, (float)tpw,
                                (float)wedges_of(c), (float)(65536 * c->region_order), (float)c->split, (float)c->supertile,
                                (float)a.band_flip};
    constexpr int grid_part = 14;   // the part a reused list must match
    int kn = grid_part;
    for (float v : {(float)a.max_steps, a.step_size, (float)cpx, (float)cprow}) key[kn++] = v;
    for (const float* v : {a.org, a.o, a.px, a.py, a.box_min, a.box_max})
        for (int k = 0; k < 3; ++k) key[kn++] = v[k];
    for (int k = 0; k < 4; ++k) key[kn++] = a.r3[k];   // the clip w row (tile_is_empty)
    ++c->renders_since_build;
    poll_region_header(c);
    const bool same_grid = c->region_cur >= 0 && std::memcmp(key, c->region_key, grid_part * sizeof(float)) == 0;
    const bool exact = same_grid && std::memcmp(key, c->region_key, sizeof key) == 0;
    if (exact || (same_grid && c->renders_since_build < c->region_interval)) {
        // lists of an older camera order the work of this one correctly, but
        // their empty tiles are that camera's: they are then marched too
        c->region_exact = exact;
        return note_region_stream(c->region[c->region_cur], stream, &c->region_slot);
    }
    c->region_exact = true;   // (either build below is for this key)

    const int S = c->supertile;
    // a moved camera over the same target: the lists come from
    // the GPU build on the render stream (vr_regions.hip) -- no host loop, no
    // host wait; tiles with work and the longest list are the last completed
    // build's (they size the launch, not the result)
    if (same_grid && c->region_gpu && th < 65536 && tw < 65536) {
        const size_t n = (size_t)tw * th;
        const Ctx::RegionBuf& cur = c->region[c->region_cur];
        const int nwork = cur.nwork, most = cur.most;
        const size_t need = region_build_bytes((int)n);
        if (need > c->rg_bytes) {
            if (c->d_rg) {
                // the last build may have been queued on another stream
                if (c->rg_pending) HIP_TRY(hipEventSynchronize(c->rg_ev));
                HIP_TRY(hipStreamSynchronize(stream));
                (void)hipFree(c->d_rg);
            }
            c->d_rg = nullptr;
            c->rg_bytes = 0;
            HIP_TRY(hipMalloc(&c->d_rg, need));   // every build zeroes its own counters (launch_region_build)
            c->rg_bytes = need;
        }
        if (!c->h_rghdr) {
            HIP_TRY(hipHostMalloc(&c->h_rghdr, kRegionHeader * sizeof(int), hipHostMallocMapped));
            HIP_TRY(hipEventCreateWithFlags(&c->rg_ev, hipEventDisableTiming));
        }
        int b = 0;
        const vr_status st0 = next_region_buf(c, n, false, stream, &b);
        if (st0 != VR_OK) return st0;
        Ctx::RegionBuf& rb = c->region[b];
        RegionBuild g{};
        g.tw = tw; g.th = th; g.width = a.width; g.out_rows = a.out_rows;
        g.band_rows = a.band_rows; g.band_stride = a.band_stride; g.band_first = a.band_first; g.band_flip = a.band_flip;
        g.max_steps = a.max_steps; g.step_size = a.step_size;
        for (int k = 0; k < 3; ++k) {
            g.org[k] = a.org[k]; g.o[k] = a.o[k]; g.px[k] = a.px[k]; g.py[k] = a.py[k];
            g.box_min[k] = a.box_min[k]; g.box_max[k] = a.box_max[k];
        }
        for (int k = 0; k < 4; ++k) g.r3[k] = a.r3[k];
        g.height = a.height;
        g.ccx = (cpx + 0.5) / 8.0; g.ccy = (cprow + 0.5) / 8.0;
        g.ctx = (cpx >> 3) / S; g.cty = (cprow >> 3) / S;
        g.supertile = S; g.wedges = wedges_of(c); g.order = c->region_order;
        int* dev_hdr = nullptr;
        HIP_TRY(hipHostGetDevicePointer(reinterpret_cast<void**>(&dev_hdr), c->h_rghdr, 0));
        // one build scratch per context: a build on another stream waits for the last one
        if (c->gpu_builds > 0) {
            const vr_status sw = stream_wait_pending(stream, c->rg_ev);
            if (sw != VR_OK) return sw;
        }
        HIP_TRY(launch_region_build(g, c->d_rg, rb.d + kRegionHeader, reinterpret_cast<int*>(rb.d), dev_hdr, stream));
        HIP_TRY(hipEventRecord(c->rg_ev, stream));
        c->rg_pending = true;
        c->rg_buf = b;
        ++c->gpu_builds;
        if (!rb.uploaded) HIP_TRY(hipEventCreateWithFlags(&rb.uploaded, hipEventDisableTiming));
        HIP_TRY(hipEventRecord(rb.uploaded, stream));
        rb.upload_stream = stream;
        rb.nwork = nwork;
        rb.most = most;
        rb.most_marched = 0;   // known once the build completes (poll_region_header)
        rb.nempty = -1;
        rb.map = TileMap{};
        rb.map.nwx = std::max(1, (most + tpw - 1) / tpw);
        rb.nstreams = 0;
        const vr_status st = note_region_stream(rb, stream, &c->region_slot);
        if (st != VR_OK) return st;
        c->region_cur = b;
        std::memcpy(c->region_key, key, sizeof key);
        c->renders_since_build = 0;
        ++c->gen;   // new lists: cached launches point at the old ones
        return VR_OK;
    }

    // a host build (a new target or band set) is already the slow path: load the
    // GPU build's code object here, not at the first GPU rebuild mid-sequence
    if (c->region_gpu && !c->rg_preloaded) {
        HIP_TRY(region_build_preload());
        c->rg_preloaded = true;
    }
    // a3 step estimate of the ray through pixel-corner (fx, fy) of the packed target
    auto steps_at = [&](double fx, int orow) {
        const int bl = orow / a.band_rows;
        const double fy = (double)(set_band(bl, a.band_first, a.band_stride, a.band_flip) * a.band_rows + (orow - bl * a.band_rows));
        double d[3], len = 0.0;
        for (int k = 0; k < 3; ++k) {
            d[k] = a.o[k] + fx * a.px[k] + fy * a.py[k];
            len += d[k] * d[k];
        }
        len = std::sqrt(len);
        double tn = -INFINITY, tf = INFINITY;
        for (int k = 0; k < 3; ++k) {
            const double ta = (a.box_min[k] - a.org[k]) * len / d[k], tb = (a.box_max[k] - a.org[k]) * len / d[k];
            tn = std::max(tn, std::min(ta, tb));
            tf = std::min(tf, std::max(ta, tb));
        }
        return (tn <= tf && std::isfinite(tf)) ? std::min((double)a.max_steps, (tf - tn) / a.step_size) : 0.0;
    };
    std::vector<double> corner((size_t)(tw + 1) * (th + 1));
    for (int j = 0; j <= th; ++j) {
        const int orow = std::min(j * 8, a.out_rows);   // the row a packed-row edge starts
        for (int i = 0; i <= tw; ++i) corner[(size_t)j * (tw + 1) + i] = steps_at(std::min(i * 8, a.width), orow);
    }
    // supertile S: tiles are ordered by S x S blocks (angle and ring of the
    // block, then row-major inside it), so consecutive entries -- the waves of
    // one workgroup, on one CU -- are a compact block sharing the CU's L1
    struct T { unsigned id; double cost, ang; int ring, sub; };
    std::vector<T> work, idle;
    const double ccx = (cpx + 0.5) / 8.0, ccy = (cprow + 0.5) / 8.0;
    const int ctx = (cpx >> 3) / S, cty = (cprow >> 3) / S;
    for (int ty = 0; ty < th; ++ty)
        for (int tx = 0; tx < tw; ++tx) {
            const double* c0 = &corner[(size_t)ty * (tw + 1) + tx];
            const double cost = std::max(std::max(c0[0], c0[1]), std::max(c0[tw + 1], c0[tw + 2]));
            const int sx = tx / S, sy = ty / S;
            const T t{((unsigned)ty << 16) | (unsigned)tx, cost,
                      std::atan2(sy * S + 0.5 * S - ccy, sx * S + 0.5 * S - ccx),
                      std::max(std::abs(sx - ctx), std::abs(sy - cty)), (ty % S) * S + tx % S};
            (cost >= 1.0 ? work : idle).push_back(t);
        }
    std::sort(work.begin(), work.end(), [](const T& u, const T& v) { return u.ang != v.ang ? u.ang < v.ang : u.sub < v.sub; });
    double total = 0.0;
    for (const T& t : work) total += t.cost;
    std::vector<std::vector<T>> xl(8);
    const int K = 8 * wedges_of(c);
    double run = 0.0;
    for (const T& t : work) {   // wedge k = the k-th K-quantile of the work, dealt to XCD k % 8
        xl[std::min(K - 1, (int)((run + 0.5 * t.cost) / total * K)) % 8].push_back(t);
        run += t.cost;
    }
    auto inside_out = [](const T& u, const T& v) {
        return u.ring != v.ring ? u.ring < v.ring : u.ang != v.ang ? u.ang < v.ang : u.sub < v.sub;
    };
    if (c->region_order == 1) {   // longest estimated work first (LPT), inside-out among equals
        for (auto& l : xl)
            std::stable_sort(l.begin(), l.end(), [&](const T& u, const T& v) {
                return u.cost != v.cost ? u.cost > v.cost : inside_out(u, v);
            });
    } else if (c->region_order == 2) {   // S x S blocks by their longest tile, a block's tiles together
        const int bw = (tw + S - 1) / S;
        std::vector<double> bmax((size_t)bw * ((th + S - 1) / S), 0.0);
        auto bidx = [&](const T& t) { return (size_t)((t.id >> 16) / S) * bw + (size_t)((t.id & 0xffffu) / S); };
        for (const auto& l : xl)
            for (const T& t : l) bmax[bidx(t)] = std::max(bmax[bidx(t)], t.cost);
        for (auto& l : xl)
            std::stable_sort(l.begin(), l.end(), [&](const T& u, const T& v) {
                const double cu = bmax[bidx(u)], cv = bmax[bidx(v)];
                if (cu != cv) return cu > cv;
                if (bidx(u) != bidx(v)) return bidx(u) < bidx(v);
                return u.sub < v.sub;
            });
    } else {
        for (auto& l : xl) std::sort(l.begin(), l.end(), inside_out);
    }
    std::sort(idle.begin(), idle.end(), inside_out);
    // idle tiles some ray of which may meet the box, dealt round-robin after
    // the work, then the empty ones (tile_is_empty: filled, not marched),
    // likewise -- the GPU build's order
    std::vector<T> empty_tiles;
    {
        std::vector<T> edge;
        for (const T& t : idle)
            (tile_is_empty(a.org, a.o, a.px, a.py, a.box_min, a.box_max, a.r3, a.width, a.out_rows, a.height,
                           a.band_rows, a.band_stride, a.band_first, a.band_flip, (int)(t.id & 0xffffu),
                           (int)(t.id >> 16))
                 ? empty_tiles : edge).push_back(t);
        for (size_t i = 0; i < edge.size(); ++i) xl[i % 8].push_back(edge[i]);
    }
    std::vector<int> marched(8);
    for (int x = 0; x < 8; ++x) marched[x] = (int)xl[x].size();
    for (size_t i = 0; i < empty_tiles.size(); ++i) xl[i % 8].push_back(empty_tiles[i]);

    size_t nent = 0;
    for (int x = 0; x < 8; ++x) nent += xl[x].size();
    const size_t n = nent;   // words after the header
    int b = 0;
    const vr_status st0 = next_region_buf(c, n, true, stream, &b);
    if (st0 != VR_OK) return st0;
    Ctx::RegionBuf& rb = c->region[b];
    int* hdr = reinterpret_cast<int*>(rb.h);
    std::memset(hdr, 0, kRegionHeader * sizeof(int));
    unsigned* list = rb.h + kRegionHeader;
    int most_marched = 0;
    TileMap m{};
    size_t pos = 0, most = 0;
    for (int x = 0; x < 8; ++x) {
        m.off[x] = (int)pos;
        for (const T& t : xl[x]) list[pos++] = t.id;
        most = std::max(most, pos - (size_t)m.off[x]);
    }
    m.off[8] = (int)pos;
    m.nwx = std::max(1, (int)((most + tpw - 1) / tpw));
    for (int x = 0; x < 9; ++x) hdr[x] = m.off[x];
    hdr[9] = (int)work.size();
    hdr[10] = (int)most;
    hdr[11] = (int)pos;
    for (int x = 0; x < 8; ++x) {   // the marched entries lead each XCD's list
        const int nm = marched[x];
        hdr[kRegionWork + x] = nm;
        most_marched = std::max(most_marched, nm);
    }
    HIP_TRY(hipMemcpyAsync(rb.d, rb.h, (n + kRegionHeader) * sizeof(unsigned), hipMemcpyHostToDevice, stream));
    if (!rb.uploaded) HIP_TRY(hipEventCreateWithFlags(&rb.uploaded, hipEventDisableTiming));
    HIP_TRY(hipEventRecord(rb.uploaded, stream));
    rb.upload_stream = stream;
    rb.map = m;
    rb.most = (int)most;
    rb.most_marched = most_marched;
    rb.nempty = (int)empty_tiles.size();
    rb.nwork = (int)work.size();
    rb.nstreams = 0;
    const vr_status st = note_region_stream(rb, stream, &c->region_slot);
    if (st != VR_OK) return st;
    c->region_cur = b;
    std::memcpy(c->region_key, key, sizeof key);
    c->renders_since_build = 0;
    ++c->gen;   // new lists: cached launches point at the old ones
    return VR_OK;
}


// Balanced contiguous row ranges (vr.h; the multi-GPU loop's row partition,
// DESIGN.md sec. 7.3).  Work of an 8-row strip: over the rays through pixel
// (8i + 4, 8s + 4), the a3 step count of the box chord (frag.glsl:42-46, as
// the region build's estimate: double, no clip test) plus kRaySetup for a ray
// that meets the box, kRayMiss for one that does not.  Boundary k is the strip
// edge nearest to the k/parts quantile of the prefix sums.
// prev / prev_ms (vr_row_partition_measured): every strip of range k of the
// previous partition `prev` is weighted by prev_ms[k] / (the model's work of
// range k), so the split follows the measured times where the model is off
// Estimated march work of every 8-row strip of the frame (row_partition's
// model, below): the rays through pixel (8i + 4, 8s + 4), each costed at
// n^(row_pow / 100) + row_setup when it meets the box, 2 when it does not.
vr_status strip_work(void* p, int width, int height, std::vector<double>* out, const char* fn)
{
    Ctx* c = as_ctx(p);
    if (!c->has_camera) return fail(VR_ERR_NO_CAMERA, "%s: no shader data (vr_set_shader_data)", fn);
    RayBasis b;
    if (!make_ray_basis(c->obj, c->glob, width, height, &b))
        return fail(VR_ERR_INVALID, "%s: Projection*View is singular", fn);
    const double kRaySetup = (double)c->row_setup, kRayMiss = 2.0, pw = c->row_pow / 100.0;
    const vr_march_params& m = c->march;
    const double step = (1.0 / (double)m.max_steps) * (double)m.step_scale;
    const int ns = (height + 7) / 8;
    std::vector<double>& w = *out;
    w.assign((size_t)ns, 0.0);
    for (int s = 0; s < ns; ++s) {
        const double fy = std::min(8.0 * s + 4.0, height - 0.5);
        for (int x = 4; x < width + 4; x += 8) {
            const double fx = std::min((double)x, width - 0.5);
            double d[3], len = 0.0;
            for (int k = 0; k < 3; ++k) {
                d[k] = (double)b.o[k] + fx * (double)b.px[k] + fy * (double)b.py[k];
                len += d[k] * d[k];
            }
            len = std::sqrt(len);
            double tn = -INFINITY, tf = INFINITY;
            for (int k = 0; k < 3; ++k) {
                const double ta = ((double)m.box_min[k] - (double)b.org[k]) * len / d[k];
                const double tb = ((double)m.box_max[k] - (double)b.org[k]) * len / d[k];
                tn = std::max(tn, std::min(ta, tb));
                tf = std::min(tf, std::max(ta, tb));
            }
            const bool hit = tn <= tf && std::isfinite(tf) && tf > 0.0;
            w[(size_t)s] += hit ? std::pow(std::min((double)m.max_steps, (tf - std::max(tn, 0.0)) / step), pw) + kRaySetup
                                : kRayMiss;
        }
    }
    return VR_OK;
}

static vr_status row_partition(void* p, int width, int height, int parts, const int* prev, const double* prev_ms,
                               int* row_begin, const char* fn)
{
    if (!p || !row_begin) return fail(VR_ERR_INVALID, "%s: null argument", fn);
    if (width <= 0 || height <= 0 || parts <= 0 || parts > 4096)
        return fail(VR_ERR_INVALID, "%s: bad frame %dx%d or parts %d", fn, width, height, parts);
    if (prev) {
        bool ok = prev[0] == 0 && prev[parts] == height;
        for (int k = 1; k <= parts && ok; ++k) ok = prev[k] >= prev[k - 1] && (prev[k] % 8 == 0 || prev[k] == height);
        for (int k = 0; k < parts && ok; ++k) ok = std::isfinite(prev_ms[k]) && prev_ms[k] >= 0.0;
        if (!ok) return fail(VR_ERR_INVALID, "%s: bad previous partition or times", fn);
    }
    std::vector<double> w;
    const vr_status st = strip_work(p, width, height, &w, fn);
    if (st != VR_OK) return st;
    const int ns = (int)w.size();
    Ctx* c = as_ctx(p);
    if (prev) {   // measured / modelled time of each previous range, on its strips
        for (int k = 0; k < parts; ++k) {
            const int s0 = prev[k] / 8, s1 = std::min(ns, (prev[k + 1] + 7) / 8);
            double est = 0.0;
            for (int s = s0; s < s1; ++s) est += w[(size_t)s];
            if (s1 > s0 && est > 0.0 && prev_ms[k] > 0.0)
                for (int s = s0; s < s1; ++s) w[(size_t)s] *= prev_ms[k] / est;
        }
    }
    std::vector<double> prefix((size_t)ns + 1, 0.0);
    for (int s = 0; s < ns; ++s) prefix[(size_t)s + 1] = prefix[(size_t)s] + w[(size_t)s];
    const double total = prefix[(size_t)ns];
    row_begin[0] = 0;
    int j = 0;
    // range 0 takes f of a mean share, the others equal shares of the rest
    const double f = parts > 1 ? c->row_first_pct / 100.0 : 1.0, g = parts > 1 ? (parts - f) / (parts - 1) : 1.0;
    for (int k = 1; k < parts; ++k) {
        const double target = total * (f + (k - 1) * g) / parts;
        while (j < ns && prefix[(size_t)j + 1] < target) ++j;
        // strip edge j or j + 1, whichever prefix is nearer the quantile
        int e = j;
        if (j < ns && prefix[(size_t)j + 1] - target < target - prefix[(size_t)j]) e = j + 1;
        row_begin[k] = std::max(row_begin[k - 1], std::min(8 * e, height));
    }
    row_begin[parts] = height;
    return VR_OK;
}

}  // namespace vrapi

using namespace vrapi;

extern "C" {

vr_status vr_row_work(void* p, int width, int height, double* strip_work_out, int nstrips)
try {
    if (!p || !strip_work_out) return fail(VR_ERR_INVALID, "vr_row_work: null argument");
    if (width <= 0 || height <= 0 || nstrips != (height + 7) / 8)
        return fail(VR_ERR_INVALID, "vr_row_work: frame %dx%d needs %d strips, got %d", width, height,
                    height > 0 ? (height + 7) / 8 : 0, nstrips);
    std::vector<double> w;
    const vr_status st = strip_work(p, width, height, &w, "vr_row_work");
    if (st != VR_OK) return st;
    std::copy(w.begin(), w.end(), strip_work_out);
    return VR_OK;
} catch (...) {
    return caught_exception("vr_row_work");
}

vr_status vr_row_partition(void* p, int width, int height, int parts, int* row_begin)
try {
    return row_partition(p, width, height, parts, nullptr, nullptr, row_begin, "vr_row_partition");
} catch (...) {
    return caught_exception("vr_row_partition");
}

vr_status vr_row_partition_measured(void* p, int width, int height, int parts, const int* prev_begin,
                                    const double* prev_ms, int* row_begin)
try {
    if (!prev_begin || !prev_ms) return fail(VR_ERR_INVALID, "vr_row_partition_measured: null argument");
    return row_partition(p, width, height, parts, prev_begin, prev_ms, row_begin, "vr_row_partition_measured");
} catch (...) {
    return caught_exception("vr_row_partition_measured");
}

}  // extern "C"
