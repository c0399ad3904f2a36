// vr_shard.cpp -- the multi-GPU frame pipeline of include/vr_shard.h
// (libvr_shard.so: libvr + RCCL).  SURVEY.md sec. 8e; DESIGN.md sec. 7.
//
// Per frame i (buffers of parity p = i & 1):
//   render stream p: wait done[p] (frame i-2's exchange / assembly has read
//                   the parity-p buffers) -> vr_render of this rank's bands
//                   (rank 0 renders straight into its gather slot 0)
//                   -> record rendered[p]
//   comm stream:    wait rendered[p] -> grouped ncclSend (rank r > 0, its
//                   packed rows) / ncclRecv x (N-1) (rank 0, into slots
//                   1..N-1) -> rank 0: vr_assemble_frame into frame[p]
//                   -> record done[p]
// The band sets are rendered in the grey format of the frame's (include/vr.h
// VR_FMT_R8_* / R32F: the pixel is vec4(vec3(c), 1), frag.glsl:79-80), so the
// exchange moves 1 B (or 4 B) per pixel instead of 4 B (16 B), and rank 0's
// assembly expands them into the RGBA frame.
// Two render streams, one per parity (vr_shard_set_render_streams; 1 = the
// caller's stream renders every frame): frame i+1's render waits only for
// done[p^1], never for frame i's render, so its waves fill the SIMDs while
// frame i's longest rays finish, and frame i's exchange overlaps frame i+1's
// render -- the reference's 2 frames in flight (VulkanRenderer.cpp:13,
// :142-172).  Each vr_render captures its frame's shader data in its launch
// arguments, so frames in flight with different cameras stay exact.  No host
// synchronisation in the loop: the host cost per frame is one render launch,
// one RCCL group and (rank 0) one assembly launch.
//
// Failure handling: the communicator is non-blocking (ncclConfig_t.blocking
// = 0).  Every host wait on a collective -- the init, the barrier, the volume
// agreement and broadcast -- polls the stream and ncclCommGetAsyncError
// against a deadline (vr_shard_set_timeout; VR_SHARD_TIMEOUT_S; default
// 120 s).  On an asynchronous error or at the deadline the communicator is
// aborted (ncclCommAbort) and the call returns VR_ERR_COMM / VR_ERR_TIMEOUT,
// so a rank whose peer died fails with a message instead of hanging; every
// later collective call on that shard fails at once.
#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <exception>
#include <new>
#include <string>
#include <atomic>
#include <thread>
#include <vector>

#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include "../../include/vr_shard.h"

static_assert(sizeof(ncclUniqueId) == VR_SHARD_ID_BYTES, "ncclUniqueId size");

// frames in flight per rank, at most (vr_shard_set_render_streams)
constexpr int kMaxFramesInFlight = 4;

namespace {

thread_local std::string g_err;

vr_status fail(vr_status st, const char* fmt, ...)
{
    char buf[512];
    va_list ap;
    va_start(ap, fmt);
    std::vsnprintf(buf, sizeof buf, fmt, ap);
    va_end(ap);
    g_err = buf;
    return st;
}

// Every extern "C" entry is a function-try-block ending in caught_exception:
// no C++ exception crosses the ABI (a std::bad_alloc -> VR_ERR_OOM, anything
// else VR_ERR_HIP, the message in vr_shard_last_error()).  Called inside a
// catch handler: `throw;` rethrows the exception being handled.
vr_status caught_exception(const char* fn) noexcept
{
    try {
        throw;
    } catch (const std::bad_alloc&) {
        return fail(VR_ERR_OOM, "%s: host allocation failed (std::bad_alloc)", fn);
    } catch (const std::exception& e) {
        return fail(VR_ERR_HIP, "%s: unexpected exception: %s", fn, e.what());
    } catch (...) {
        return fail(VR_ERR_HIP, "%s: unexpected exception", fn);
    }
}

#define HIP_TRY(expr)                                                                                     \
    do {                                                                                                  \
        hipError_t e_ = (expr);                                                                           \
        if (e_ != hipSuccess)                                                                             \
            return fail(e_ == hipErrorOutOfMemory ? VR_ERR_OOM : VR_ERR_HIP, "%s: %s (%s:%d)", #expr,     \
                        hipGetErrorString(e_), __FILE__, __LINE__);                                       \
    } while (0)
// a non-blocking communicator may answer ncclInProgress: settle() then
// waits (with the deadline) until the call has taken effect
#define NCCL_TRY(expr)                                                                                    \
    do {                                                                                                  \
        ncclResult_t r_ = (expr);                                                                         \
        if (r_ == ncclInProgress) {                                                                       \
            const vr_status s2_ = settle(sh, #expr);                                                      \
            if (s2_ != VR_OK) return s2_;                                                                 \
        } else if (r_ != ncclSuccess) {                                                                   \
            abort_comm(sh);                                                                               \
            return fail(VR_ERR_COMM, "%s: %s (%s:%d)", #expr, ncclGetErrorString(r_), __FILE__, __LINE__); \
        }                                                                                                 \
    } while (0)
// a shard helper that has already set the message
#define SH_TRY(expr)                  \
    do {                              \
        vr_status t_ = (expr);        \
        if (t_ != VR_OK) return t_;   \
    } while (0)
#define VR_TRY(expr)                                                                                      \
    do {                                                                                                  \
        vr_status s_ = (expr);                                                                            \
        if (s_ != VR_OK) return fail(s_, "%s: %s", #expr, vr_last_error());                               \
    } while (0)

// Poll `state()` -- 0 done, 1 pending, 2 failed -- until it is not pending or
// `timeout_s` has passed: 0 done, 1 failed, 2 timed out.  Spins for the first
// 20 ms (a barrier at the end of a timed window of frames costs microseconds,
// not a sleep's granularity), then sleeps 50 us between polls.  Shared by the collective waits and the CPU
// self-test of the deadline logic (vr_shard_poll_selftest).
template <class State>
int poll_until(State state, double timeout_s)
{
    using clk = std::chrono::steady_clock;
    const auto t0 = clk::now();
    for (;;) {
        const int st = state();
        if (st == 0) return 0;
        if (st == 2) return 1;
        const double el = std::chrono::duration<double>(clk::now() - t0).count();
        if (el > timeout_s) return 2;
        if (el > 20e-3) std::this_thread::sleep_for(std::chrono::microseconds(50));
    }
}

double default_timeout()
{
    const char* e = std::getenv("VR_SHARD_TIMEOUT_S");
    const double v = e ? std::atof(e) : 0.0;
    return v > 0.0 ? v : 120.0;
}

}  // namespace

struct vr_shard {
    void* ctx = nullptr;
    int device = 0;
    int nranks = 1, rank = 0;
    int width = 0, height = 0, format = 0, band_rows = 0, bpp = 4;
    size_t pitch = 0;                 // tight frame rows (format)
    int gformat = 3;                  // grey format of the band sets (exchanged)
    size_t gpitch = 0;                // tight band-set rows
    int my_rows = 0, rows_per_rank = 0;
    std::vector<int> rows_of;         // packed rows of every rank
    // compositor (vr_shard_set_compositor): rank 0 renders no bands and only
    // assembles; ranks 1..N-1 render the band sets of a world of N-1 renderers
    // (rank r: band_first r - 1), received into gather slot r - 1
    bool compositor = false;
    // compositor with band sets: rank 0 also renders the lead rows [0,
    // lead_rows) of the frame in place (a multiple of band_rows; 0 = none),
    // and the renderers' band sets cover the rows below them
    // (vr_shard_set_lead_rows / vr_shard_balance_lead)
    int lead_rows = 0;
    // serpentine band sets (vr_shard_set_serpentine): renderer k's odd bands
    // shifted by R - 1 - 2k (vr_target.band_flip), so the deal runs backwards
    // in every other period of R bands
    bool serpentine = true;
    // balanced row ranges (vr_shard_set_rows / vr_shard_balance_rows): renderer
    // k renders frame rows [row_begin[k], row_begin[k + 1]) (VR_TARGET_ROW_RANGE)
    // and rank 0 gathers them into a grey frame; empty = interleaved band sets
    std::vector<int> row_begin;
    bool started = false;             // a run has queued frames (the geometry is fixed)
    ncclComm_t comm = nullptr;
    hipStream_t comm_stream = nullptr;
    // render streams: frame i renders on stream i mod render_streams with the
    // buffer set of that index (the comm-stream paths use at most 2)
    hipStream_t render_stream[kMaxFramesInFlight] = {};
    int render_streams = 2;           // 1: every frame renders on the caller's stream
    int host_threads = 1;             // 2: a second host thread issues the exchange half of every frame
    // exchange on the render streams (vr_shard_set_exchange_streams): frame i's
    // exchange (and rank 0's assembly) follows its render on render_stream[p],
    // over a communicator of its own per parity (comm for p = 0, comm2 for
    // p = 1, split from comm at the first such run), with no events at all
    bool on_render = true;   // vr_shard_set_exchange_streams
    ncclComm_t comm2 = nullptr;
    ncclComm_t comm_more[kMaxFramesInFlight - 2] = {};   // streams 2.. (split like comm2)
    uint8_t* local[kMaxFramesInFlight] = {};      // rank > 0: band sets (gformat)
    uint8_t* gathered[kMaxFramesInFlight] = {};   // rank 0: nranks slots of rows_per_rank rows (gformat)
    uint8_t* frame[kMaxFramesInFlight] = {};      // rank 0
    hipEvent_t rendered[kMaxFramesInFlight] = {}, done[kMaxFramesInFlight] = {};
    hipEvent_t tail[kMaxFramesInFlight] = {};     // the end of the render streams' frames (vr_shard_run_frames)
    hipEvent_t fence = nullptr;       // vr_shard_barrier: the caller's stream -> comm stream
    int* token = nullptr;             // [0]: vr_shard_barrier's all-reduced int; [1..7]:
                                      // vr_shard_share_volume's agreement vector
    bool pending[kMaxFramesInFlight] = {};        // done[p] recorded and not yet waited on
    int last = -1;                    // parity of the last frame
    bool loopback = false;            // one process emulates all ranks (no RCCL)
    bool solo = false;                // loopback rehearsal of one rank: its own band set only, no exchange
    std::vector<hipEvent_t> timing;   // sampled render brackets (pairs)
    double sampled_busy_ms = 0.0;     // the last run's sampled renders: union of their intervals
    double sampled_span_ms = 0.0;     // and first start -> last end (vr_shard_sampled_busy)
    // the ctx's option frames_overlap before this pipeline first ran frames on
    // 2+ render streams (-1: not changed).  It stays set while the pipeline
    // overlaps frames -- a set / reset per run would invalidate the ctx's
    // launch cache twice per run -- and is restored by vr_shard_destroy or a
    // switch to one render stream.
    int overlap_prev = -1;
    double timeout_s = 120.0;         // deadline of every host wait on a collective
    bool aborted = false;             // the communicator was aborted (error or deadline)
};

namespace {

void abort_comm(vr_shard* sh)
{
    if (sh)
        for (ncclComm_t& c : sh->comm_more)
            if (c) {
                (void)ncclCommAbort(c);
                c = nullptr;
            }
    if (sh && sh->comm2) {
        (void)ncclCommAbort(sh->comm2);
        sh->comm2 = nullptr;
    }
    if (sh && sh->comm) {
        (void)ncclCommAbort(sh->comm);
        sh->comm = nullptr;
        sh->aborted = true;
    }
}

// the communicators' asynchronous state: 0 ok, 1 in progress, 2 failed
int comm_state(vr_shard* sh)
{
    if (!sh->comm) return sh->aborted ? 2 : 0;
    int st = 0;
    for (int i = -2; i < kMaxFramesInFlight - 2; ++i) {
        const ncclComm_t c = i == -2 ? sh->comm : i == -1 ? sh->comm2 : sh->comm_more[i];
        if (!c) continue;
        ncclResult_t r = ncclSuccess;
        if (ncclCommGetAsyncError(c, &r) != ncclSuccess) return 2;
        if (r != ncclSuccess && r != ncclInProgress) return 2;
        if (r == ncclInProgress) st = 1;
    }
    return st;
}

vr_status deadline_fail(vr_shard* sh, int res, const char* what)
{
    ncclResult_t r = ncclSuccess;
    if (sh->comm) (void)ncclCommGetAsyncError(sh->comm, &r);
    abort_comm(sh);
    if (res == 2)
        return fail(VR_ERR_TIMEOUT, "%s: no completion within %.3g s (a peer rank failed or stalled); communicator aborted",
                    what, sh->timeout_s);
    return fail(VR_ERR_COMM, "%s: communicator error: %s; communicator aborted", what, ncclGetErrorString(r));
}

// A non-blocking NCCL call returned ncclInProgress: wait until it has taken effect.
vr_status settle(vr_shard* sh, const char* what)
{
    const int res = poll_until([&] { return comm_state(sh); }, sh->timeout_s);
    return res == 0 ? VR_OK : deadline_fail(sh, res, what);
}

// Host wait for stream `s` (which may hold collectives), with the deadline and
// the communicator's error state.
vr_status wait_stream(vr_shard* sh, hipStream_t s, const char* what)
{
    hipError_t he = hipSuccess;
    const int res = poll_until([&] {
        const int c = comm_state(sh);
        if (c == 2) return 2;
        he = hipStreamQuery(s);
        if (he == hipSuccess) return 0;
        return he == hipErrorNotReady ? 1 : 2;
    }, sh->timeout_s);
    if (res == 0) return VR_OK;
    if (res == 1 && he != hipSuccess && he != hipErrorNotReady) {
        abort_comm(sh);
        return fail(VR_ERR_HIP, "%s: %s; communicator aborted", what, hipGetErrorString(he));
    }
    return deadline_fail(sh, res, what);
}

vr_status wait_event(vr_shard* sh, hipEvent_t e, const char* what)
{
    hipError_t he = hipSuccess;
    const int res = poll_until([&] {
        if (comm_state(sh) == 2) return 2;
        he = hipEventQuery(e);
        if (he == hipSuccess) return 0;
        return he == hipErrorNotReady ? 1 : 2;
    }, sh->timeout_s);
    if (res == 0) return VR_OK;
    if (res == 1 && he != hipSuccess && he != hipErrorNotReady) {
        abort_comm(sh);   // as wait_stream: every later collective fails at once
        return fail(VR_ERR_HIP, "%s: %s; communicator aborted", what, hipGetErrorString(he));
    }
    return deadline_fail(sh, res, what);
}

vr_status check_usable(vr_shard* sh, const char* what)
{
    if (sh->aborted) return fail(VR_ERR_COMM, "%s: the communicator was aborted by an earlier error or deadline", what);
    return VR_OK;
}

void restore_overlap(vr_shard* sh)
{
    if (sh->overlap_prev == 0) (void)vr_set_option(sh->ctx, "frames_overlap", 0);
    sh->overlap_prev = -1;
}

void release(vr_shard* sh)
{
    restore_overlap(sh);
    for (hipStream_t rs : sh->render_stream)
        if (rs) (void)hipStreamSynchronize(rs);
    if (sh->comm_stream) (void)hipStreamSynchronize(sh->comm_stream);
    for (int p = 0; p < kMaxFramesInFlight; ++p) {
        if (sh->local[p]) (void)hipFree(sh->local[p]);
        if (sh->gathered[p]) (void)hipFree(sh->gathered[p]);
        if (sh->frame[p]) (void)hipFree(sh->frame[p]);
        if (sh->rendered[p]) (void)hipEventDestroy(sh->rendered[p]);
        if (sh->done[p]) (void)hipEventDestroy(sh->done[p]);
        if (sh->tail[p]) (void)hipEventDestroy(sh->tail[p]);
    }
    for (hipEvent_t e : sh->timing) (void)hipEventDestroy(e);
    if (sh->fence) (void)hipEventDestroy(sh->fence);
    if (sh->token) (void)hipFree(sh->token);
    for (ncclComm_t c : sh->comm_more)
        if (c) (void)ncclCommDestroy(c);
    if (sh->comm2) (void)ncclCommDestroy(sh->comm2);
    if (sh->comm) (void)ncclCommDestroy(sh->comm);   // an aborted communicator is already gone
    if (sh->comm_stream) (void)hipStreamDestroy(sh->comm_stream);
    for (hipStream_t rs : sh->render_stream)
        if (rs) (void)hipStreamDestroy(rs);
    delete sh;
}

// Rank 0 renders its bands straight into the frame (vr.h
// VR_TARGET_BANDS_IN_PLACE), so its render and the exchange + assembly of the
// other ranks' rows share no buffer: neither waits for the other, and the
// frame needs no event per frame on rank 0 (host time: an event record costs
// ~2.7 us, a frame of the 1/8 share ~20 us; profiles/r05/host_frame*).  The
// run's end joins the streams (vr_shard_run_frames).  Other ranks (and
// loopback, which renders the other ranks' sets here) order render ->
// exchange -> the next render of the parity with rendered[p] / done[p].
bool others_here(const vr_shard* sh) { return sh->loopback && !sh->solo; }

// Band geometry: renderers, a rank's band set (stride, first) and its gather slot.
int renderers(const vr_shard* sh) { return sh->compositor ? sh->nranks - 1 : sh->nranks; }
int band_first_of(const vr_shard* sh, int r) { return sh->compositor ? r - 1 : r; }
bool rows_mode(const vr_shard* sh) { return !sh->row_begin.empty(); }
// the renderers' band sets start below rank 0's lead rows: frame band b0 + k
// is renderer k's first (a band set over the whole frame, band_first >= stride)
int lead_band(const vr_shard* sh) { return sh->lead_rows / sh->band_rows; }
int set_first_of(const vr_shard* sh, int r) { return band_first_of(sh, r) + lead_band(sh); }
bool leads(const vr_shard* sh, int r) { return r == 0 && sh->lead_rows > 0; }
// the k-th band of a set (vr.h vr_target.band_flip)
int set_band(int k, int first, int stride, int flip) { return first + k * stride + ((k & 1) ? flip : 0); }
// rank r's band_flip: R - 1 - 2k for renderer k of a serpentine band-set deal
int flip_of(const vr_shard* sh, int r)
{
    const int R = renderers(sh), k = band_first_of(sh, r);
    if (!sh->serpentine || rows_mode(sh) || leads(sh, r) || k < 0 || R < 2) return 0;
    return R - 1 - 2 * k;
}
// rank 0's gather buffer: a slot of rows_per_rank rows per rank, or (row
// ranges) a grey frame that every renderer's range lands in at its own rows
size_t gather_rows(const vr_shard* sh)
{
    return rows_mode(sh) ? (size_t)sh->height : (size_t)sh->nranks * sh->rows_per_rank;
}
uint8_t* slot_of(const vr_shard* sh, int p, int r)
{
    if (rows_mode(sh)) return sh->gathered[p] + (size_t)sh->row_begin[band_first_of(sh, r)] * sh->gpitch;
    return sh->gathered[p] + (size_t)band_first_of(sh, r) * sh->rows_per_rank * sh->gpitch;
}
// rank r's render target: its band set or its row range (format and buffer set by the caller)
vr_target target_of(const vr_shard* sh, int r)
{
    vr_target t{};
    t.width = sh->width;
    t.height = sh->height;
    if (rows_mode(sh)) {
        const int k = band_first_of(sh, r);
        if (k < 0) return t;   // the compositor renders nothing
        t.band_rows = sh->row_begin[k + 1] - sh->row_begin[k];
        t.band_stride = 1;
        t.band_first = sh->row_begin[k];
    } else if (leads(sh, r)) {   // rank 0's lead rows (VR_TARGET_ROW_RANGE)
        t.band_rows = sh->lead_rows;
        t.band_stride = 1;
        t.band_first = 0;
    } else {
        t.band_rows = sh->band_rows;
        t.band_stride = renderers(sh);
        t.band_first = set_first_of(sh, r);
        t.band_flip = flip_of(sh, r);
    }
    return t;
}
int range_flag(const vr_shard* sh, int r) { return rows_mode(sh) || leads(sh, r) ? VR_TARGET_ROW_RANGE : 0; }
// the assembly: every renderer's rows, or (rank 0 rendering in place) all but rank 0's
vr_status assemble(vr_shard* sh, int p, hipStream_t s)
{
    if (rows_mode(sh)) {   // the other ranks' ranges are contiguous: one expansion of the rows below rank 0's
        const int start = sh->compositor ? 0 : sh->row_begin[1];
        const int n = sh->height - start;
        if (n > 0)
            VR_TRY(vr_assemble_frame_ranks(sh->ctx, sh->gathered[p] + (size_t)start * sh->gpitch, sh->gformat, (size_t)n,
                                           1, 0, sh->width, n, n, sh->format, sh->frame[p] + (size_t)start * sh->pitch,
                                           s));
        return VR_OK;
    }
    // (rank 0's lead rows, rendered in place, are above the band sets: the
    // assembly expands the frame below them, where renderer k's set is the
    // sub-frame's band set k)
    const int lead = sh->lead_rows;
    const int serp = sh->serpentine && renderers(sh) > 1 ? VR_ASSEMBLE_SERPENTINE : 0;
    VR_TRY(vr_assemble_frame_ranks(sh->ctx, sh->gathered[p], sh->gformat, (size_t)sh->rows_per_rank, renderers(sh),
                                   sh->compositor ? 0 : 1, sh->width, sh->height - lead, sh->band_rows,
                                   sh->format | serp, sh->frame[p] + (size_t)lead * sh->pitch, s));
    return VR_OK;
}

// The render-stream half of frame (parity p): wait for the exchange that last
// read the parity's buffers (not rank 0, which renders in place), render, and
// (not rank 0) mark the render for the exchange.
vr_status render_half(vr_shard* sh, int p, hipStream_t s, hipEvent_t t0, hipEvent_t t1)
{
    const bool r0 = sh->rank == 0, here = others_here(sh);
    if ((!r0 || here) && sh->pending[p]) HIP_TRY(hipStreamWaitEvent(s, sh->done[p], 0));
    vr_target t = target_of(sh, sh->rank);
    if (r0) {   // in place: the frame's own rows, the frame's format
        t.format = sh->format | VR_TARGET_BANDS_IN_PLACE | range_flag(sh, sh->rank);
        t.pixels = sh->frame[p];
        t.row_pitch = sh->pitch;
    } else {
        t.format = sh->gformat | range_flag(sh, sh->rank);
        t.pixels = sh->local[p];
        t.row_pitch = sh->gpitch;
    }
    if (t0) HIP_TRY(hipEventRecord(t0, s));
    if (sh->my_rows > 0) VR_TRY(vr_render(sh->ctx, &t, s));
    if (t1) HIP_TRY(hipEventRecord(t1, s));
    if (here) {   // the other ranks' band sets, rendered here into their gather slots
        for (int r = 1; r < sh->nranks; ++r) {
            t = target_of(sh, r);
            t.format = sh->gformat | range_flag(sh, r);
            t.row_pitch = sh->gpitch;
            t.pixels = slot_of(sh, p, r);
            if (sh->rows_of[r] > 0) VR_TRY(vr_render(sh->ctx, &t, s));
        }
    }
    if (!r0 || here) HIP_TRY(hipEventRecord(sh->rendered[p], s));
    return VR_OK;
}

// The communication-stream half: the exchange of the band sets (rank 0 receives
// into its gather slots, the others send), rank 0's assembly of the other
// ranks' rows, and (not rank 0) the mark that frees the parity's buffers.
vr_status comm_half(vr_shard* sh, int p)
{
    const bool r0 = sh->rank == 0, here = others_here(sh);
    if (!r0 || here) HIP_TRY(hipStreamWaitEvent(sh->comm_stream, sh->rendered[p], 0));
    if (r0 && !here && sh->pending[p]) {   // an earlier run's frame of this parity (its assembly read gathered[p])
        HIP_TRY(hipStreamWaitEvent(sh->comm_stream, sh->done[p], 0));
        sh->pending[p] = false;
    }
    if (sh->nranks > 1 && !sh->loopback) {
        NCCL_TRY(ncclGroupStart());
        if (r0) {
            for (int r = 1; r < sh->nranks; ++r)
                if (sh->rows_of[r] > 0)
                    NCCL_TRY(ncclRecv(slot_of(sh, p, r), (size_t)sh->rows_of[r] * sh->gpitch, ncclUint8, r, sh->comm,
                                      sh->comm_stream));
        } else if (sh->my_rows > 0) {
            NCCL_TRY(ncclSend(sh->local[p], (size_t)sh->my_rows * sh->gpitch, ncclUint8, 0, sh->comm,
                              sh->comm_stream));
        }
        NCCL_TRY(ncclGroupEnd());
    }
    if (r0 && sh->nranks > 1)   // (a solo rehearsal expands whatever its slots hold: the same work)
        SH_TRY(assemble(sh, p, sh->comm_stream));
    if (!r0 || here) {
        HIP_TRY(hipEventRecord(sh->done[p], sh->comm_stream));
        sh->pending[p] = true;
    }
    return VR_OK;
}

vr_status one_frame(vr_shard* sh, int p, hipStream_t s, hipEvent_t t0, hipEvent_t t1)
{
    SH_TRY(render_half(sh, p, s, t0, t1));
    SH_TRY(comm_half(sh, p));
    sh->last = p;
    return VR_OK;
}

// Frame (parity p) with its exchange on the render stream rs = render_stream[p]
// (vr_shard_set_exchange_streams): render -> send / receive over the parity's
// communicator -> (rank 0) assembly, in rs's order.  The next frame of the
// parity follows in the same order, so no event is recorded or waited for;
// the other parity's frame overlaps on the other stream and communicator.
vr_status one_frame_on_render(vr_shard* sh, int p, hipStream_t rs, hipEvent_t t0, hipEvent_t t1)
{
    const bool r0 = sh->rank == 0, here = others_here(sh);
    vr_target t = target_of(sh, sh->rank);
    if (r0) {
        t.format = sh->format | VR_TARGET_BANDS_IN_PLACE | range_flag(sh, sh->rank);
        t.pixels = sh->frame[p];
        t.row_pitch = sh->pitch;
    } else {
        t.format = sh->gformat | range_flag(sh, sh->rank);
        t.pixels = sh->local[p];
        t.row_pitch = sh->gpitch;
    }
    if (t0) HIP_TRY(hipEventRecord(t0, rs));
    if (sh->my_rows > 0) VR_TRY(vr_render(sh->ctx, &t, rs));
    if (t1) HIP_TRY(hipEventRecord(t1, rs));
    if (here) {
        for (int r = 1; r < sh->nranks; ++r) {
            t = target_of(sh, r);
            t.format = sh->gformat | range_flag(sh, r);
            t.row_pitch = sh->gpitch;
            t.pixels = slot_of(sh, p, r);
            if (sh->rows_of[r] > 0) VR_TRY(vr_render(sh->ctx, &t, rs));
        }
    }
    if (sh->nranks > 1 && !sh->loopback) {
        ncclComm_t c = p == 0 ? sh->comm : p == 1 ? sh->comm2 : sh->comm_more[p - 2];
        NCCL_TRY(ncclGroupStart());
        if (r0) {
            for (int r = 1; r < sh->nranks; ++r)
                if (sh->rows_of[r] > 0)
                    NCCL_TRY(ncclRecv(slot_of(sh, p, r), (size_t)sh->rows_of[r] * sh->gpitch, ncclUint8, r, c, rs));
        } else if (sh->my_rows > 0) {
            NCCL_TRY(ncclSend(sh->local[p], (size_t)sh->my_rows * sh->gpitch, ncclUint8, 0, c, rs));
        }
        NCCL_TRY(ncclGroupEnd());
    }
    if (r0 && sh->nranks > 1) SH_TRY(assemble(sh, p, rs));
    sh->last = p;
    return VR_OK;
}

// Rank 0 as a compositor by default (vr_shard_set_compositor) from this many
// ranks on.  Config 5 (1080p) at N = 8: rank 0 rendering its own 1/8 beside
// the assembly of the other 7/8 takes 0.0208 ms per frame against 0.0165 on
// the other ranks; as a compositor the slowest of 7 renderers takes 0.0198
// (profiles/r05/compositor_ab.txt).  Round 6: a compositor that also renders
// lead rows (vr_shard_balance_lead) beside serpentine band sets beats row
// ranges at 4K too -- config 4 at N = 8 0.0402-0.0406 against 0.0431-0.0434
// (profiles/r06/c4_lead/) -- so the default no longer depends on the size.
constexpr int kCompositorRanks = 8;

void set_geometry(vr_shard* sh, bool compositor)
{
    sh->compositor = compositor && sh->nranks >= 2;
    const int R = renderers(sh);
    if ((int)sh->row_begin.size() != R + 1) sh->row_begin.clear();   // ranges of another renderer count
    if (!sh->compositor || rows_mode(sh)) sh->lead_rows = 0;          // lead rows: compositor + band sets only
    sh->rows_of.assign(sh->nranks, 0);
    for (int r = 0; r < sh->nranks; ++r)
        if (!sh->compositor || r > 0) {
            const int k = band_first_of(sh, r);
            sh->rows_of[r] = rows_mode(sh) ? sh->row_begin[k + 1] - sh->row_begin[k]
                                           : vr_band_rows_packed(sh->height, sh->band_rows, R, set_first_of(sh, r),
                                                                 flip_of(sh, r));
        }
    // a gather slot holds the largest set (ranges: the longest range); rank
    // 0's lead rows are rendered in place, not gathered
    sh->rows_per_rank = 0;
    for (int r = 0; r < sh->nranks; ++r)
        if (!leads(sh, r)) sh->rows_per_rank = std::max(sh->rows_per_rank, sh->rows_of[r]);
    if (leads(sh, 0)) sh->rows_of[0] = sh->lead_rows;
    sh->my_rows = sh->rows_of[sh->rank];
}

// rank 0's gather slots / another rank's band sets, for the current geometry
vr_status alloc_band_buffers(vr_shard* sh)
{
    for (int p = 0; p < kMaxFramesInFlight; ++p) {
        uint8_t*& b = sh->rank == 0 ? sh->gathered[p] : sh->local[p];
        if (b) (void)hipFree(b);
        b = nullptr;
        const size_t bytes = sh->rank == 0 ? gather_rows(sh) * sh->gpitch
                                           : (size_t)std::max(sh->my_rows, 1) * sh->gpitch;
        const hipError_t e = hipMalloc(&b, std::max(bytes, (size_t)1));
        if (e != hipSuccess) {
            b = nullptr;
            return fail(e == hipErrorOutOfMemory ? VR_ERR_OOM : VR_ERR_HIP, "vr_shard: band buffers: %s",
                        hipGetErrorString(e));
        }
    }
    return VR_OK;
}

// Spin (then yield) until `ready()` or `stop`; false at the deadline.
template <class F>
bool wait_host(F ready, const std::atomic<bool>& stop, double timeout_s)
{
    const auto t0 = std::chrono::steady_clock::now();
    for (int k = 0;; ++k) {
        if (ready()) return true;
        if (stop.load(std::memory_order_acquire)) return false;
        if ((k & 1023) == 1023) {
            if (std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() > timeout_s) return false;
            std::this_thread::yield();
        }
    }
}

}  // namespace

extern "C" {

const char* vr_shard_last_error(void) { return g_err.c_str(); }

vr_status vr_shard_unique_id(uint8_t id[VR_SHARD_ID_BYTES])
try {
    if (!id) return fail(VR_ERR_INVALID, "vr_shard_unique_id: null");
    ncclUniqueId u;
    const ncclResult_t r = ncclGetUniqueId(&u);
    if (r != ncclSuccess) return fail(VR_ERR_COMM, "ncclGetUniqueId: %s", ncclGetErrorString(r));
    std::memcpy(id, &u, sizeof u);
    return VR_OK;
} catch (...) {
    return caught_exception("vr_shard_unique_id");
}

vr_status vr_shard_alloc(void* ctx, int nranks, int rank, int width, int height, int format, int band_rows,
                         vr_shard** out)
try {
    if (!ctx || !out) return fail(VR_ERR_INVALID, "vr_shard_alloc: null argument");
    *out = nullptr;
    if (nranks < 1 || rank < 0 || rank >= nranks) return fail(VR_ERR_INVALID, "vr_shard_alloc: rank %d of %d", rank, nranks);
    if (width <= 0 || height <= 0 || band_rows <= 0 || format < 0 || format > 2)
        return fail(VR_ERR_INVALID, "vr_shard_alloc: bad frame %dx%d format %d bands %d", width, height, format, band_rows);
    vr_shard* sh = new (std::nothrow) vr_shard();
    if (!sh) return fail(VR_ERR_OOM, "vr_shard_alloc: host allocation");
    sh->ctx = ctx;
    sh->loopback = true;   // until vr_shard_connect joins a communicator
    sh->timeout_s = default_timeout();
    sh->nranks = nranks;
    sh->rank = rank;
    sh->width = width;
    sh->height = height;
    sh->format = format;
    sh->band_rows = band_rows;
    sh->bpp = format == VR_FMT_RGBA32F ? 16 : 4;
    sh->pitch = (size_t)width * sh->bpp;
    sh->gformat = format == VR_FMT_RGBA32F ? VR_FMT_R32F : format == VR_FMT_RGBA8_SRGB ? VR_FMT_R8_SRGB : VR_FMT_R8_UNORM;
    sh->gpitch = (size_t)width * (format == VR_FMT_RGBA32F ? 4 : 1);
    set_geometry(sh, nranks >= kCompositorRanks);
    int dev = 0;
    hipError_t e = hipGetDevice(&dev);
    vr_status st = VR_OK;
    auto hip_ok = [&](hipError_t r, const char* what) {
        if (st == VR_OK && r != hipSuccess)
            st = fail(r == hipErrorOutOfMemory ? VR_ERR_OOM : VR_ERR_HIP, "vr_shard_alloc: %s: %s", what,
                      hipGetErrorString(r));
        return st == VR_OK;
    };
    hip_ok(e, "hipGetDevice");
    sh->device = dev;
    hip_ok(hipStreamCreateWithFlags(&sh->comm_stream, hipStreamNonBlocking), "comm stream");
    for (hipStream_t& rs : sh->render_stream) hip_ok(hipStreamCreateWithFlags(&rs, hipStreamNonBlocking), "render stream");
    hip_ok(hipEventCreateWithFlags(&sh->fence, hipEventDisableTiming), "event");
    if (hip_ok(hipMalloc(&sh->token, 8 * sizeof(int)), "barrier token"))
        hip_ok(hipMemset(sh->token, 0, 8 * sizeof(int)), "barrier token");
    for (int p = 0; p < kMaxFramesInFlight && st == VR_OK; ++p) {
        hip_ok(hipEventCreateWithFlags(&sh->rendered[p], hipEventDisableTiming), "event");
        hip_ok(hipEventCreateWithFlags(&sh->done[p], hipEventDisableTiming), "event");
        hip_ok(hipEventCreateWithFlags(&sh->tail[p], hipEventDisableTiming), "event");
        if (rank == 0) hip_ok(hipMalloc(&sh->frame[p], (size_t)height * sh->pitch), "frame buffer");
    }
    if (st == VR_OK) st = alloc_band_buffers(sh);
    if (st != VR_OK) {
        const std::string msg = g_err;
        release(sh);
        g_err = msg;
        return st;
    }
    *out = sh;
    return VR_OK;
} catch (...) {
    return caught_exception("vr_shard_alloc");
}

vr_status vr_shard_connect(vr_shard* sh, const uint8_t id[VR_SHARD_ID_BYTES])
try {
    if (!sh || !id) return fail(VR_ERR_INVALID, "vr_shard_connect: null argument");
    if (sh->comm) return fail(VR_ERR_INVALID, "vr_shard_connect: already connected");
    if (sh->last >= 0) return fail(VR_ERR_INVALID, "vr_shard_connect: frames already rendered in loopback");
    if (sh->aborted) return fail(VR_ERR_COMM, "vr_shard_connect: communicator already aborted");
    if (sh->solo) return fail(VR_ERR_INVALID, "vr_shard_connect: a solo rehearsal shard does not connect");
    ncclUniqueId u;
    std::memcpy(&u, id, sizeof u);
    // non-blocking: the init returns at once and completes as the peers join;
    // a peer that never joins ends in the deadline, not in a hang
    ncclConfig_t cfg = NCCL_CONFIG_INITIALIZER;
    cfg.blocking = 0;
    const ncclResult_t r = ncclCommInitRankConfig(&sh->comm, sh->nranks, u, sh->rank, &cfg);
    if (r != ncclSuccess && r != ncclInProgress) {
        sh->comm = nullptr;
        return fail(VR_ERR_COMM, "vr_shard_connect: ncclCommInitRankConfig: %s", ncclGetErrorString(r));
    }
    const vr_status st = settle(sh, "vr_shard_connect: ncclCommInitRankConfig");
    if (st != VR_OK) return st;
    sh->loopback = false;
    return VR_OK;
} catch (...) {
    return caught_exception("vr_shard_connect");
}

vr_status vr_shard_create(void* ctx, const uint8_t id[VR_SHARD_ID_BYTES], int nranks, int rank, int width,
                          int height, int format, int band_rows, vr_shard** out)
try {
    if (!ctx || !out) return fail(VR_ERR_INVALID, "vr_shard_create: null argument");
    *out = nullptr;
    if (!id && rank != 0) return fail(VR_ERR_INVALID, "vr_shard_create: null id (loopback needs rank 0)");
    vr_shard* sh = nullptr;
    vr_status st = vr_shard_alloc(ctx, nranks, rank, width, height, format, band_rows, &sh);
    if (st != VR_OK) return st;
    if (id) {
        st = vr_shard_connect(sh, id);
        if (st != VR_OK) {
            const std::string msg = g_err;
            release(sh);
            g_err = msg;
            return st;
        }
    }
    *out = sh;
    return VR_OK;
} catch (...) {
    return caught_exception("vr_shard_create");
}

vr_status vr_shard_destroy(vr_shard* sh)
try {
    if (sh) release(sh);
    return VR_OK;
} catch (...) {
    return caught_exception("vr_shard_destroy");
}

vr_status vr_shard_run(vr_shard* sh, int frames, void* stream, int sample_every, float* kernel_ms)
try {
    return vr_shard_run_frames(sh, frames, nullptr, nullptr, stream, sample_every, kernel_ms, nullptr);
} catch (...) {
    return caught_exception("vr_shard_run");
}

vr_status vr_shard_run_frames(vr_shard* sh, int frames, const vr_object_shader_data* osd,
                              const vr_global_shader_data* gsd, void* stream, int sample_every, float* kernel_ms,
                              double* host_ms)
try {
    if (!sh || frames < 0 || (!osd) != (!gsd)) return fail(VR_ERR_INVALID, "vr_shard_run: bad argument");
    if (kernel_ms && sample_every <= 0) return fail(VR_ERR_INVALID, "vr_shard_run: sample_every must be > 0");
    if (sh->loopback && sh->rank != 0 && !sh->solo)
        return fail(VR_ERR_INVALID, "vr_shard_run: rank %d is not connected (vr_shard_connect)", sh->rank);
    SH_TRY(check_usable(sh, "vr_shard_run"));
    hipStream_t s = static_cast<hipStream_t>(stream);
    const int nsamp = kernel_ms ? (frames + sample_every - 1) / sample_every : 0;
    while ((int)sh->timing.size() < 2 * nsamp) {
        hipEvent_t ev;
        HIP_TRY(hipEventCreate(&ev));
        sh->timing.push_back(ev);
    }
    int next = 0;
    const auto h0 = std::chrono::steady_clock::now();
    // a procedural medium with deferred shadow rays renders on one stream:
    // its frames could overlap since round 6 (a frame that reuses the cost
    // order writes only its stream's deferred scratch set), but two in flight
    // measured slower (config 3: 0.783 against 0.756 ms, profiles/r06/c10)
    const int P = vr_get_option(sh->ctx, "procedural") == 2 ? 1
                  : sh->on_render ? sh->render_streams : std::min(sh->render_streams, 2);
    const bool two = P >= 2;   // frames overlap on P render streams
    if (frames > 0) sh->started = true;   // the band geometry is fixed from here
    // two render streams: tell the ctx its consecutive renders overlap (its
    // auto split rule), from this pipeline's first such run until it is
    // destroyed or set to one render stream (restore_overlap)
    if (two && frames > 0 && sh->overlap_prev < 0) {
        sh->overlap_prev = vr_get_option(sh->ctx, "frames_overlap");
        if (sh->overlap_prev == 0) VR_TRY(vr_set_option(sh->ctx, "frames_overlap", 1));
    }
    if (two && frames > 0) {   // the render streams start after the caller's queued work (e.g. the volume)
        HIP_TRY(hipEventRecord(sh->fence, s));
        for (hipStream_t rs : sh->render_stream) HIP_TRY(hipStreamWaitEvent(rs, sh->fence, 0));
    }
    const bool on_render = sh->on_render && two;
    if (on_render && frames > 0) {
        // the communicators of streams 1..P-1, once each, split from the
        // first (collective: every rank runs its first such frames together,
        // in the same order; a one-rank communicator splits too, so its test
        // covers the call)
        for (int q = 1; q < P && !sh->loopback; ++q) {
            ncclComm_t& cq = q == 1 ? sh->comm2 : sh->comm_more[q - 2];
            if (cq) continue;
            ncclConfig_t cfg = NCCL_CONFIG_INITIALIZER;
            cfg.blocking = 0;
            const ncclResult_t r = ncclCommSplit(sh->comm, 0, sh->rank, &cq, &cfg);
            if (r != ncclSuccess && r != ncclInProgress) {
                cq = nullptr;
                abort_comm(sh);
                return fail(VR_ERR_COMM, "vr_shard_run: ncclCommSplit: %s; communicator aborted", ncclGetErrorString(r));
            }
            SH_TRY(settle(sh, "vr_shard_run: ncclCommSplit"));
        }
        // the buffer sets were last used by frames of the comm-stream path,
        // if any: their exchanges must be done
        for (int q = 0; q < kMaxFramesInFlight; ++q)
            if (sh->pending[q]) {
                for (hipStream_t rs : sh->render_stream) HIP_TRY(hipStreamWaitEvent(rs, sh->done[q], 0));
                sh->pending[q] = false;
            }
        for (int i = 0; i < frames; ++i) {
            const int p = sh->last < 0 ? 0 : (sh->last + 1) % P;
            const bool samp = kernel_ms && i % sample_every == 0;
            hipEvent_t t0 = samp ? sh->timing[2 * next] : nullptr, t1 = samp ? sh->timing[2 * next + 1] : nullptr;
            if (samp) ++next;
            if (osd) VR_TRY(vr_set_shader_data(sh->ctx, &osd[i], &gsd[i]));   // this frame's camera
            SH_TRY(one_frame_on_render(sh, p, sh->render_stream[p], t0, t1));
        }
        // join: the caller's stream after every render stream's last frame
        for (int q = 0; q < P; ++q) {
            HIP_TRY(hipEventRecord(sh->tail[q], sh->render_stream[q]));
            HIP_TRY(hipStreamWaitEvent(s, sh->tail[q], 0));
            // a later comm-stream frame of parity q waits for this one
            HIP_TRY(hipEventRecord(sh->done[q], sh->render_stream[q]));
            sh->pending[q] = true;
        }
    } else if (sh->host_threads == 2 && frames > 1) {
        // Two host threads: this one issues the render halves, a worker the
        // exchange halves, so a frame's host time is the longer half, not the
        // sum (an event record or a launch costs ~3-5 us).
        // Frame i's exchange is issued after its render (rendered[p] recorded);
        // frame i's render after frame i-2's exchange (done[p] recorded, and
        // rendered[p] no longer awaited).
        const int p0 = sh->last < 0 ? 0 : (sh->last + 1) % 2;
        std::atomic<int> rdone{0}, cdone{0};
        std::atomic<bool> stop{false};
        vr_status wst = VR_OK;
        std::string werr;
        std::thread worker([&] {
            if (hipSetDevice(sh->device) != hipSuccess) {
                wst = fail(VR_ERR_HIP, "vr_shard_run: worker hipSetDevice");
            } else {
                for (int i = 0; i < frames; ++i) {
                    if (!wait_host([&] { return rdone.load(std::memory_order_acquire) > i; }, stop, sh->timeout_s)) {
                        if (!stop.load()) wst = fail(VR_ERR_TIMEOUT, "vr_shard_run: render thread stalled");
                        break;
                    }
                    wst = comm_half(sh, (p0 + i) & 1);
                    if (wst != VR_OK) break;
                    cdone.store(i + 1, std::memory_order_release);
                }
            }
            if (wst != VR_OK) {
                werr = g_err;
                stop.store(true, std::memory_order_release);
            }
        });
        // if anything below throws, the worker is stopped and joined before
        // the exception leaves (a joinable std::thread's destructor would
        // call std::terminate past the function-try-block)
        struct JoinGuard {
            std::thread& t;
            std::atomic<bool>& stop;
            ~JoinGuard()
            {
                if (t.joinable()) {
                    stop.store(true, std::memory_order_release);
                    t.join();
                }
            }
        } join_guard{worker, stop};
        vr_status mst = VR_OK;
        for (int i = 0; i < frames && mst == VR_OK; ++i) {
            if (i >= 2 && !wait_host([&] { return cdone.load(std::memory_order_acquire) >= i - 1; }, stop, sh->timeout_s))
                break;   // the worker failed (its status is reported) or stalled
            const int p = (p0 + i) & 1;
            const bool samp = kernel_ms && i % sample_every == 0;
            hipEvent_t t0 = samp ? sh->timing[2 * next] : nullptr, t1 = samp ? sh->timing[2 * next + 1] : nullptr;
            if (samp) ++next;
            if (osd) {
                mst = vr_set_shader_data(sh->ctx, &osd[i], &gsd[i]);
                if (mst != VR_OK) mst = fail(mst, "vr_set_shader_data: %s", vr_last_error());
            }
            if (mst == VR_OK) mst = render_half(sh, p, two ? sh->render_stream[p] : s, t0, t1);
            if (mst == VR_OK) rdone.store(i + 1, std::memory_order_release);
        }
        if (mst != VR_OK) stop.store(true, std::memory_order_release);
        worker.join();
        if (mst != VR_OK) return mst;
        if (wst != VR_OK) {
            g_err = werr;
            return wst;
        }
        if (cdone.load() != frames) return fail(VR_ERR_TIMEOUT, "vr_shard_run: render thread stalled");
        sh->last = (p0 + frames - 1) & 1;
    } else {
        for (int i = 0; i < frames; ++i) {
            const int p = sh->last < 0 ? 0 : (sh->last + 1) % 2;
            const bool samp = kernel_ms && i % sample_every == 0;
            hipEvent_t t0 = samp ? sh->timing[2 * next] : nullptr, t1 = samp ? sh->timing[2 * next + 1] : nullptr;
            if (samp) ++next;
            if (osd) VR_TRY(vr_set_shader_data(sh->ctx, &osd[i], &gsd[i]));   // this frame's camera
            const vr_status st = one_frame(sh, p, two ? sh->render_stream[p] : s, t0, t1);
            if (st != VR_OK) return st;
        }
    }
    if (sh->last >= 0 && frames > 0 && !on_render) {   // the caller's stream sees the frame
        if (sh->rank == 0 && !others_here(sh)) {
            // rank 0 recorded no event per frame: join the exchange / assembly
            // stream and the render streams now (the render streams' frames
            // are the rank's own rows of the frames)
            HIP_TRY(hipEventRecord(sh->done[sh->last], sh->comm_stream));
            sh->pending[sh->last] = true;
            if (two)
                for (int q = 0; q < 2; ++q) {   // (the comm-stream paths use streams 0 and 1)
                    HIP_TRY(hipEventRecord(sh->tail[q], sh->render_stream[q]));
                    HIP_TRY(hipStreamWaitEvent(s, sh->tail[q], 0));
                }
        }
        HIP_TRY(hipStreamWaitEvent(s, sh->done[sh->last], 0));
    }
    if (host_ms)
        *host_ms = frames ? std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - h0).count() / frames
                          : 0.0;
    if (kernel_ms) {
        double sum = 0.0;
        std::vector<std::pair<double, double>> iv;   // sampled renders on one clock: ms after the first start
        for (int k = 0; k < next; ++k) {
            SH_TRY(wait_event(sh, sh->timing[2 * k + 1], "vr_shard_run: sampled render"));
            float ms = 0.0f, a = 0.0f, b = 0.0f;
            HIP_TRY(hipEventElapsedTime(&ms, sh->timing[2 * k], sh->timing[2 * k + 1]));
            HIP_TRY(hipEventElapsedTime(&a, sh->timing[0], sh->timing[2 * k]));
            HIP_TRY(hipEventElapsedTime(&b, sh->timing[0], sh->timing[2 * k + 1]));
            sum += ms;
            iv.emplace_back(a, b);
        }
        *kernel_ms = next ? (float)(sum / next) : 0.0f;
        // busy: the union of the sampled intervals (overlapping renders on
        // several streams count once); with sample_every = 1, the GPU time
        // the run's renders held the machine
        std::sort(iv.begin(), iv.end());
        double busy = 0.0, lo = 0.0, hi = -1.0, end = 0.0;
        for (const auto& x : iv) {
            if (x.first > hi) {
                if (hi >= lo) busy += hi - lo;
                lo = x.first;
                hi = x.second;
            } else {
                hi = std::max(hi, x.second);
            }
            end = std::max(end, x.second);
        }
        if (hi >= lo && !iv.empty()) busy += hi - lo;
        sh->sampled_busy_ms = busy;
        sh->sampled_span_ms = iv.empty() ? 0.0 : end - iv.front().first;
    }
    return VR_OK;
} catch (...) {
    return caught_exception("vr_shard_run_frames");
}

vr_status vr_shard_barrier(vr_shard* sh, void* stream)
try {
    if (!sh) return fail(VR_ERR_INVALID, "vr_shard_barrier: null");
    if (sh->loopback && sh->rank != 0 && !sh->solo)
        return fail(VR_ERR_INVALID, "vr_shard_barrier: rank %d is not connected (vr_shard_connect)", sh->rank);
    SH_TRY(check_usable(sh, "vr_shard_barrier"));
    hipStream_t s = static_cast<hipStream_t>(stream);
    HIP_TRY(hipEventRecord(sh->fence, s));
    HIP_TRY(hipStreamWaitEvent(sh->comm_stream, sh->fence, 0));
    // The all-reduce completes on a rank only once every rank's streams have
    // reached it: a device-side barrier over xGMI, then the host waits for it.
    if (sh->nranks > 1 && !sh->loopback)
        NCCL_TRY(ncclAllReduce(sh->token, sh->token, 1, ncclInt32, ncclSum, sh->comm, sh->comm_stream));
    SH_TRY(wait_stream(sh, sh->comm_stream, "vr_shard_barrier"));
    SH_TRY(wait_stream(sh, s, "vr_shard_barrier"));
    return VR_OK;
} catch (...) {
    return caught_exception("vr_shard_barrier");
}

// SURVEY.md sec. 8e collective (1): the volume, once, from rank 0 to every
// rank over xGMI (the reference uploads it once per process, Texture3D,
// VulkanTexture.cpp:111-156).  The ranks first agree -- one all-reduce (max)
// of {failed, nx, ny, nz, -nx, -ny, -nz} -- that every receive buffer exists
// and every rank named the same extent, so no rank enters the broadcast
// alone; then one ncclBroadcast of the RGBA8 bytes and, on every rank,
// vr_set_volume_device (repack + fast layout), ordered on `stream`.
vr_status vr_shard_share_volume(vr_shard* sh, const void* d_rgba8, int nx, int ny, int nz, void* stream)
try {
    if (!sh) return fail(VR_ERR_INVALID, "vr_shard_share_volume: null shard");
    if (sh->loopback && sh->rank != 0)
        return fail(VR_ERR_INVALID, "vr_shard_share_volume: rank %d is not connected (vr_shard_connect)", sh->rank);
    SH_TRY(check_usable(sh, "vr_shard_share_volume"));
    hipStream_t s = static_cast<hipStream_t>(stream);
    if (sh->loopback) {   // one process holds every rank's work: nothing to send
        HIP_TRY(hipSetDevice(sh->device));
        if (!d_rgba8) return fail(VR_ERR_INVALID, "vr_shard_share_volume: rank 0 needs the volume");
        VR_TRY(vr_set_volume_device(sh->ctx, d_rgba8, nx, ny, nz, stream));
        HIP_TRY(hipStreamSynchronize(s));
        return VR_OK;
    }
    // Every local failure before the broadcast -- the device, the extent (the
    // same test vr_set_volume_device applies), rank 0's missing volume, the
    // receive buffer -- is folded into `failed` and still takes part in the
    // agreement all-reduce, so no rank returns while its peers wait in it.
    int failed = hipSetDevice(sh->device) != hipSuccess ? 1 : 0;
    if (!vr_volume_extent_ok(nx, ny, nz) || (sh->rank == 0 && !d_rgba8)) failed = 1;
    const size_t bytes = failed ? 0 : (size_t)nx * ny * nz * 4;
    uint8_t* buf = nullptr;
    if (!failed && sh->rank != 0 && hipMalloc(&buf, bytes) != hipSuccess) {
        buf = nullptr;
        failed = 1;
    }
    const int agree[7] = {failed, nx, ny, nz, -nx, -ny, -nz};
    int got[7] = {};
    hipError_t he = hipMemcpyAsync(sh->token + 1, agree, sizeof agree, hipMemcpyHostToDevice, sh->comm_stream);
    ncclResult_t nr = ncclSuccess;
    vr_status st = VR_OK;   // a settle()/wait failure keeps its own status and message (VR_ERR_TIMEOUT / _COMM)
    if (he == hipSuccess) {
        nr = ncclAllReduce(sh->token + 1, sh->token + 1, 7, ncclInt32, ncclMax, sh->comm, sh->comm_stream);
        if (nr == ncclInProgress) {
            st = settle(sh, "vr_shard_share_volume: agreement");
            nr = ncclSuccess;
        }
    }
    if (he == hipSuccess && nr == ncclSuccess && st == VR_OK)
        he = hipMemcpyAsync(got, sh->token + 1, sizeof got, hipMemcpyDeviceToHost, sh->comm_stream);
    if (he == hipSuccess && nr == ncclSuccess && st == VR_OK)
        st = wait_stream(sh, sh->comm_stream, "vr_shard_share_volume: agreement");
    if (he != hipSuccess || nr != ncclSuccess || st != VR_OK) {
        if (buf && !sh->aborted) (void)hipFree(buf);
        if (st != VR_OK) return st;
        if (nr != ncclSuccess) {
            if (!sh->aborted) abort_comm(sh);
            return fail(VR_ERR_COMM, "vr_shard_share_volume: agreement: %s", ncclGetErrorString(nr));
        }
        return fail(VR_ERR_HIP, "vr_shard_share_volume: agreement: %s", hipGetErrorString(he));
    }
    if (got[0] || got[1] != -got[4] || got[2] != -got[5] || got[3] != -got[6]) {
        if (buf) (void)hipFree(buf);
        if (failed) return fail(VR_ERR_INVALID, "vr_shard_share_volume: rank %d: bad extent, no volume, no device or no memory", sh->rank);
        if (got[0]) return fail(VR_ERR_INVALID, "vr_shard_share_volume: failed on another rank");
        return fail(VR_ERR_INVALID, "vr_shard_share_volume: ranks named different extents");
    }
    void* data = sh->rank == 0 ? const_cast<void*>(d_rgba8) : buf;
    // the broadcast after the caller's stream (rank 0 may have produced the volume
    // on it), the install after the broadcast
    he = hipEventRecord(sh->fence, s);
    if (he == hipSuccess) he = hipStreamWaitEvent(sh->comm_stream, sh->fence, 0);
    if (he == hipSuccess) {
        nr = ncclBroadcast(data, data, bytes, ncclUint8, 0, sh->comm, sh->comm_stream);
        if (nr == ncclInProgress) {
            st = settle(sh, "vr_shard_share_volume: broadcast");   // keeps its status and message
            nr = ncclSuccess;
        }
        if (nr == ncclSuccess && st == VR_OK) {
            he = hipEventRecord(sh->fence, sh->comm_stream);
            if (he == hipSuccess) he = hipStreamWaitEvent(s, sh->fence, 0);
        }
    }
    if (st != VR_OK) {
        // settle() aborted the communicator and set the message
    } else if (nr != ncclSuccess) {
        if (!sh->aborted) abort_comm(sh);
        st = fail(VR_ERR_COMM, "vr_shard_share_volume: ncclBroadcast: %s", ncclGetErrorString(nr));
    } else if (he != hipSuccess) {
        st = fail(VR_ERR_HIP, "vr_shard_share_volume: %s", hipGetErrorString(he));
    } else if (vr_set_volume_device(sh->ctx, data, nx, ny, nz, stream) != VR_OK) {
        st = fail(VR_ERR_HIP, "vr_shard_share_volume: vr_set_volume_device: %s", vr_last_error());
    }
    // the broadcast must be finished (or the communicator aborted) before buf
    // goes; after an abort the waits are skipped, so they cannot overwrite the
    // message of the real cause
    if (!sh->aborted) {
        const vr_status w1 = wait_stream(sh, sh->comm_stream, "vr_shard_share_volume: broadcast");
        const vr_status w2 = w1 == VR_OK ? wait_stream(sh, s, "vr_shard_share_volume: install") : w1;
        if (st == VR_OK) st = w2;
    }
    if (buf && !sh->aborted) (void)hipFree(buf);   // an aborted broadcast may still own it: leak, not corrupt
    return st;
} catch (...) {
    return caught_exception("vr_shard_share_volume");
}

vr_status vr_shard_set_render_streams(vr_shard* sh, int n)
try {
    if (!sh || n < 1 || n > kMaxFramesInFlight)
        return fail(VR_ERR_INVALID, "vr_shard_set_render_streams: need a shard and n in 1..%d", kMaxFramesInFlight);
    if (n != sh->render_streams && sh->last >= 0) {
        // frames of the old arrangement may still be in flight: the next
        // frame's stream must see them (each set's done[] covers its render)
        for (int p = 0; p < kMaxFramesInFlight; ++p)
            if (sh->pending[p]) SH_TRY(wait_event(sh, sh->done[p], "vr_shard_set_render_streams"));
    }
    sh->render_streams = n;
    if (n == 1) restore_overlap(sh);   // the frames no longer overlap
    return VR_OK;
} catch (...) {
    return caught_exception("vr_shard_set_render_streams");
}

int vr_shard_get_render_streams(vr_shard* sh) { return sh ? sh->render_streams : 0; }

vr_status vr_shard_set_exchange_streams(vr_shard* sh, int on_render)
try {
    if (!sh || on_render < 0 || on_render > 1)
        return fail(VR_ERR_INVALID, "vr_shard_set_exchange_streams: need a shard and 0 or 1");
    sh->on_render = on_render == 1;
    return VR_OK;
} catch (...) {
    return caught_exception("vr_shard_set_exchange_streams");
}

vr_status vr_shard_set_host_threads(vr_shard* sh, int n)
try {
    if (!sh || (n != 1 && n != 2)) return fail(VR_ERR_INVALID, "vr_shard_set_host_threads: need a shard and n = 1 or 2");
    sh->host_threads = n;
    return VR_OK;
} catch (...) {
    return caught_exception("vr_shard_set_host_threads");
}

vr_status vr_shard_set_solo(vr_shard* sh, int on)
try {
    if (!sh) return fail(VR_ERR_INVALID, "vr_shard_set_solo: null");
    if (!sh->loopback) return fail(VR_ERR_INVALID, "vr_shard_set_solo: only an unconnected (loopback) shard rehearses alone");
    sh->solo = on != 0;
    return VR_OK;
} catch (...) {
    return caught_exception("vr_shard_set_solo");
}

vr_status vr_shard_set_timeout(vr_shard* sh, double seconds)
try {
    if (!sh || !(seconds > 0.0)) return fail(VR_ERR_INVALID, "vr_shard_set_timeout: need a shard and seconds > 0");
    sh->timeout_s = seconds;
    return VR_OK;
} catch (...) {
    return caught_exception("vr_shard_set_timeout");
}

int vr_shard_aborted(vr_shard* sh) { return sh && sh->aborted ? 1 : 0; }

vr_status vr_shard_sampled_busy(vr_shard* sh, double* busy_ms, double* span_ms)
try {
    if (!sh || !busy_ms || !span_ms) return fail(VR_ERR_INVALID, "vr_shard_sampled_busy: null argument");
    *busy_ms = sh->sampled_busy_ms;
    *span_ms = sh->sampled_span_ms;
    return VR_OK;
} catch (...) {
    return caught_exception("vr_shard_sampled_busy");
}

// CPU self-test of the deadline logic (no HIP, no RCCL): mode 0 -- the state
// settles after a few polls; 1 -- it reports an error; 2 -- it never settles
// (the deadline).  Returns poll_until's 0 / 1 / 2, or -1 for a bad mode.
int vr_shard_poll_selftest(int mode, double timeout_s, int* polls)
try {
    if (mode < 0 || mode > 2) return -1;
    int n = 0;
    const int res = poll_until([&] {
        ++n;
        if (mode == 0) return n >= 5 ? 0 : 1;
        if (mode == 1) return n >= 3 ? 2 : 1;
        return 1;
    }, timeout_s);
    if (polls) *polls = n;
    return res;
} catch (...) {
    (void)caught_exception("vr_shard_poll_selftest");
    return -1;
}

vr_status vr_shard_frame(vr_shard* sh, void** pixels, size_t* row_pitch, int* rows)
try {
    if (!sh || !pixels) return fail(VR_ERR_INVALID, "vr_shard_frame: null argument");
    if (sh->last < 0) return fail(VR_ERR_INVALID, "vr_shard_frame: no frame rendered yet");
    *pixels = sh->rank == 0 ? sh->frame[sh->last] : sh->local[sh->last];
    if (row_pitch) *row_pitch = sh->rank == 0 ? sh->pitch : sh->gpitch;
    if (rows) *rows = sh->rank == 0 ? sh->height : sh->my_rows;
    return VR_OK;
} catch (...) {
    return caught_exception("vr_shard_frame");
}

vr_status vr_shard_copy_frame(vr_shard* sh, void* dst, size_t dst_pitch, void* stream)
try {
    void* src = nullptr;
    size_t pitch = 0;
    int rows = 0;
    const vr_status st = vr_shard_frame(sh, &src, &pitch, &rows);
    if (st != VR_OK) return st;
    if (!dst) return fail(VR_ERR_INVALID, "vr_shard_copy_frame: null dst");
    if (dst_pitch == 0) dst_pitch = pitch;
    if (dst_pitch < pitch) return fail(VR_ERR_INVALID, "vr_shard_copy_frame: dst_pitch %zu < %zu", dst_pitch, pitch);
    HIP_TRY(hipMemcpy2DAsync(dst, dst_pitch, src, pitch, pitch, (size_t)rows, hipMemcpyDeviceToDevice,
                             static_cast<hipStream_t>(stream)));
    return VR_OK;
} catch (...) {
    return caught_exception("vr_shard_copy_frame");
}

vr_status vr_shard_set_compositor(vr_shard* sh, int on)
try {
    if (!sh || on < 0 || on > 1) return fail(VR_ERR_INVALID, "vr_shard_set_compositor: bad argument");
    if (on && sh->nranks < 2) return fail(VR_ERR_INVALID, "vr_shard_set_compositor: needs 2 or more ranks");
    if ((on == 1) == sh->compositor) return VR_OK;
    if (sh->started) return fail(VR_ERR_INVALID, "vr_shard_set_compositor: set before the first frames");
    set_geometry(sh, on == 1);
    return alloc_band_buffers(sh);
} catch (...) {
    return caught_exception("vr_shard_set_compositor");
}

int vr_shard_get_compositor(vr_shard* sh)
try {
    return sh ? (sh->compositor ? 1 : 0) : -1;
} catch (...) {
    return -1;
}

vr_status vr_shard_bands(vr_shard* sh, int* band_stride, int* band_first, int* band_flip)
try {
    if (!sh) return fail(VR_ERR_INVALID, "vr_shard_bands: null");
    if (band_stride) *band_stride = renderers(sh);
    if (band_first) *band_first = leads(sh, sh->rank) ? -1 : set_first_of(sh, sh->rank);
    if (band_flip) *band_flip = flip_of(sh, sh->rank);
    return VR_OK;
} catch (...) {
    return caught_exception("vr_shard_bands");
}

vr_status vr_shard_set_serpentine(vr_shard* sh, int on)
try {
    if (!sh || on < 0 || on > 1) return fail(VR_ERR_INVALID, "vr_shard_set_serpentine: bad argument");
    if ((on == 1) == sh->serpentine) return VR_OK;
    if (sh->started) return fail(VR_ERR_INVALID, "vr_shard_set_serpentine: set before the first frames");
    sh->serpentine = on == 1;
    set_geometry(sh, sh->compositor);
    return alloc_band_buffers(sh);
} catch (...) {
    return caught_exception("vr_shard_set_serpentine");
}

int vr_shard_get_serpentine(vr_shard* sh)
try {
    return sh ? (sh->serpentine ? 1 : 0) : -1;
} catch (...) {
    return -1;
}

vr_status vr_shard_set_rows(vr_shard* sh, const int* row_begin)
try {
    if (!sh) return fail(VR_ERR_INVALID, "vr_shard_set_rows: null");
    const int R = renderers(sh);
    std::vector<int> rb;
    if (row_begin) {
        rb.assign(row_begin, row_begin + R + 1);
        bool ok = rb[0] == 0 && rb[R] == sh->height;
        for (int k = 1; k <= R && ok; ++k) ok = rb[k] >= rb[k - 1] && (rb[k] % 8 == 0 || rb[k] == sh->height);
        if (!ok) return fail(VR_ERR_INVALID, "vr_shard_set_rows: need %d + 1 non-decreasing row starts from 0 to %d, "
                             "multiples of 8", R, sh->height);
    }
    if (rb == sh->row_begin) return VR_OK;
    if (sh->started) {
        // new ranges between runs (vr_shard_rebalance_rows): the frames in
        // flight still use the band buffers; the interleaved / row-range mode
        // itself is fixed once frames are queued
        if (rb.empty() != sh->row_begin.empty())
            return fail(VR_ERR_INVALID, "vr_shard_set_rows: band sets or row ranges are chosen before the first frames");
        for (hipStream_t rs : sh->render_stream) HIP_TRY(hipStreamSynchronize(rs));
        HIP_TRY(hipStreamSynchronize(sh->comm_stream));
        HIP_TRY(hipDeviceSynchronize());   // (frames rendered on the caller's stream)
    }
    sh->row_begin = rb;
    set_geometry(sh, sh->compositor);
    return alloc_band_buffers(sh);
} catch (...) {
    return caught_exception("vr_shard_set_rows");
}

}  // extern "C"

namespace {

// Rank 0's ints to every rank over the shard's communicator (after a
// connect; a no-op in loopback or with one rank): v[0] is rank 0's failure
// flag, so a rank-0 failure reaches every rank after the one collective.
vr_status bcast_ints(vr_shard* sh, std::vector<int>& rb, const char* fn)
{
    if (sh->nranks > 1 && !sh->loopback) {
        HIP_TRY(hipSetDevice(sh->device));
        int* d = nullptr;
        HIP_TRY(hipMalloc(&d, rb.size() * sizeof(int)));
        hipError_t he = hipMemcpyAsync(d, rb.data(), rb.size() * sizeof(int), hipMemcpyHostToDevice, sh->comm_stream);
        vr_status st = VR_OK;
        ncclResult_t nr = ncclSuccess;
        if (he == hipSuccess) {
            nr = ncclBroadcast(d, d, rb.size(), ncclInt32, 0, sh->comm, sh->comm_stream);
            if (nr == ncclInProgress) {
                st = settle(sh, fn);
                nr = ncclSuccess;
            }
        }
        if (he == hipSuccess && nr == ncclSuccess && st == VR_OK)
            he = hipMemcpyAsync(rb.data(), d, rb.size() * sizeof(int), hipMemcpyDeviceToHost, sh->comm_stream);
        if (he == hipSuccess && nr == ncclSuccess && st == VR_OK) st = wait_stream(sh, sh->comm_stream, fn);
        if (!sh->aborted) (void)hipFree(d);
        if (st != VR_OK) return st;
        if (nr != ncclSuccess) {
            abort_comm(sh);
            return fail(VR_ERR_COMM, "%s: ncclBroadcast: %s", fn, ncclGetErrorString(nr));
        }
        if (he != hipSuccess) return fail(VR_ERR_HIP, "%s: %s", fn, hipGetErrorString(he));
    }
    return VR_OK;
}

// Rank 0's partition, on every rank: broadcast with a failure flag (a rank-0
// failure reaches every rank after the one collective, not a hang).  all_ms
// (every rank's measured ms, by rank): vr_row_partition_measured over the
// current ranges; else vr_row_partition.
vr_status share_partition(vr_shard* sh, const std::vector<double>* all_ms, const char* fn)
{
    const int R = renderers(sh);
    std::vector<int> rb((size_t)R + 2, 0);   // [0]: failed, [1..R+1]: row starts
    vr_status mine = VR_OK;
    std::string msg;
    if (sh->rank == 0 || sh->loopback) {
        // rank 0 rendering in place also expands the other (N-1)/N of the
        // frame: its range takes 2 % less than a mean share per other rank
        // (config 4: 0.0461 ms per frame at 8 ranks with 85 %, 0.0491 with
        // 100 %; profiles/r05/row_ranges_c4.txt)
        const int prev = vr_get_option(sh->ctx, "row_first_pct");
        const int pct = sh->compositor ? 100 : std::max(50, 100 - 2 * (sh->nranks - 1));
        (void)vr_set_option(sh->ctx, "row_first_pct", pct);
        if (all_ms) {
            std::vector<double> ms((size_t)R, 0.0);
            for (int r = 0; r < sh->nranks; ++r)
                if (band_first_of(sh, r) >= 0) ms[(size_t)band_first_of(sh, r)] = (*all_ms)[(size_t)r];
            mine = vr_row_partition_measured(sh->ctx, sh->width, sh->height, R, sh->row_begin.data(), ms.data(),
                                             rb.data() + 1);
        } else {
            mine = vr_row_partition(sh->ctx, sh->width, sh->height, R, rb.data() + 1);
        }
        (void)vr_set_option(sh->ctx, "row_first_pct", prev);
        if (mine != VR_OK) {
            msg = vr_last_error();
            rb[0] = 1;
        }
    }
    SH_TRY(bcast_ints(sh, rb, fn));
    if (rb[0]) {
        if (mine != VR_OK) return fail(mine, "%s: %s", fn, msg.c_str());
        return fail(VR_ERR_INVALID, "%s: rank 0's partition failed", fn);
    }
    return vr_shard_set_rows(sh, rb.data() + 1);
}

}  // namespace

extern "C" {

vr_status vr_shard_balance_rows(vr_shard* sh)
try {
    if (!sh) return fail(VR_ERR_INVALID, "vr_shard_balance_rows: null");
    if (sh->loopback && sh->rank != 0 && !sh->solo)
        return fail(VR_ERR_INVALID, "vr_shard_balance_rows: rank %d is not connected (vr_shard_connect)", sh->rank);
    SH_TRY(check_usable(sh, "vr_shard_balance_rows"));
    return share_partition(sh, nullptr, "vr_shard_balance_rows");
} catch (...) {
    return caught_exception("vr_shard_balance_rows");
}

// Collective: every rank's measured ms (one all-reduce of a vector holding
// each rank's own entry), then rank 0's measured partition, broadcast.
vr_status vr_shard_rebalance_rows(vr_shard* sh, double my_ms)
try {
    if (!sh || !std::isfinite(my_ms) || my_ms < 0.0) return fail(VR_ERR_INVALID, "vr_shard_rebalance_rows: bad argument");
    if (sh->loopback) return fail(VR_ERR_INVALID, "vr_shard_rebalance_rows: needs the ranks' times (a connected shard)");
    if (!rows_mode(sh)) return fail(VR_ERR_INVALID, "vr_shard_rebalance_rows: the shard renders band sets");
    SH_TRY(check_usable(sh, "vr_shard_rebalance_rows"));
    HIP_TRY(hipSetDevice(sh->device));
    std::vector<double> ms((size_t)sh->nranks, 0.0);
    ms[(size_t)sh->rank] = my_ms;
    if (sh->nranks > 1) {
        double* d = nullptr;
        HIP_TRY(hipMalloc(&d, ms.size() * sizeof(double)));
        hipError_t he = hipMemcpyAsync(d, ms.data(), ms.size() * sizeof(double), hipMemcpyHostToDevice, sh->comm_stream);
        vr_status st = VR_OK;
        ncclResult_t nr = ncclSuccess;
        if (he == hipSuccess) {
            nr = ncclAllReduce(d, d, ms.size(), ncclFloat64, ncclSum, sh->comm, sh->comm_stream);
            if (nr == ncclInProgress) {
                st = settle(sh, "vr_shard_rebalance_rows: all-reduce");
                nr = ncclSuccess;
            }
        }
        if (he == hipSuccess && nr == ncclSuccess && st == VR_OK)
            he = hipMemcpyAsync(ms.data(), d, ms.size() * sizeof(double), hipMemcpyDeviceToHost, sh->comm_stream);
        if (he == hipSuccess && nr == ncclSuccess && st == VR_OK)
            st = wait_stream(sh, sh->comm_stream, "vr_shard_rebalance_rows: all-reduce");
        if (!sh->aborted) (void)hipFree(d);
        if (st != VR_OK) return st;
        if (nr != ncclSuccess) {
            abort_comm(sh);
            return fail(VR_ERR_COMM, "vr_shard_rebalance_rows: ncclAllReduce: %s", ncclGetErrorString(nr));
        }
        if (he != hipSuccess) return fail(VR_ERR_HIP, "vr_shard_rebalance_rows: %s", hipGetErrorString(he));
    }
    return share_partition(sh, &ms, "vr_shard_rebalance_rows");
} catch (...) {
    return caught_exception("vr_shard_rebalance_rows");
}

vr_status vr_shard_set_lead_rows(vr_shard* sh, int rows)
try {
    if (!sh) return fail(VR_ERR_INVALID, "vr_shard_set_lead_rows: null");
    if (rows < 0 || rows % sh->band_rows != 0 || rows >= sh->height)
        return fail(VR_ERR_INVALID, "vr_shard_set_lead_rows: %d rows: a multiple of the band rows (%d) below the "
                                    "frame height %d", rows, sh->band_rows, sh->height);
    if (rows > 0 && (!sh->compositor || rows_mode(sh)))
        return fail(VR_ERR_INVALID, "vr_shard_set_lead_rows: lead rows need rank 0 as a compositor over band sets");
    if (rows == sh->lead_rows) return VR_OK;
    if (sh->started) return fail(VR_ERR_INVALID, "vr_shard_set_lead_rows: set before the first frames");
    sh->lead_rows = rows;
    set_geometry(sh, sh->compositor);
    return alloc_band_buffers(sh);
} catch (...) {
    return caught_exception("vr_shard_set_lead_rows");
}

int vr_shard_get_lead_rows(vr_shard* sh) { return sh ? sh->lead_rows : -1; }

// Collective: rank 0 sizes its lead rows for the ctx's camera and every rank
// takes them.  Rank 0 counts as pct % of a renderer (the rest of its time is
// the assembly): over every lead of whole bands, the estimated work per row
// (vr_row_work, the row partition's model) gives rank 0's cost -- the lead
// rows' work / (pct / 100) -- and each renderer's -- the work of its band set
// below the lead --, and the lead with the smallest largest cost wins.  The
// renderers' band counts are part of that: a lead that leaves a whole number
// of bands per renderer keeps them level.
vr_status vr_shard_balance_lead(vr_shard* sh, int pct)
try {
    if (!sh || pct < 0 || pct > 100) return fail(VR_ERR_INVALID, "vr_shard_balance_lead: bad argument");
    if (sh->loopback && sh->rank != 0 && !sh->solo)
        return fail(VR_ERR_INVALID, "vr_shard_balance_lead: rank %d is not connected (vr_shard_connect)", sh->rank);
    if (!sh->compositor || rows_mode(sh))
        return fail(VR_ERR_INVALID, "vr_shard_balance_lead: lead rows need rank 0 as a compositor over band sets");
    SH_TRY(check_usable(sh, "vr_shard_balance_lead"));
    std::vector<int> v(2, 0);   // [0]: failed, [1]: lead rows
    vr_status mine = VR_OK;
    std::string msg;
    if ((sh->rank == 0 || sh->loopback) && pct > 0) {
        const int H = sh->height, br = sh->band_rows, R = renderers(sh), nb = (H + br - 1) / br;
        const int ns = (H + 7) / 8;
        std::vector<double> sw((size_t)ns, 0.0);
        mine = vr_row_work(sh->ctx, sh->width, H, sw.data(), ns);
        if (mine != VR_OK) {
            msg = vr_last_error();
            v[0] = 1;
        } else {
            std::vector<double> band((size_t)nb, 0.0);   // work per band: its rows' share of their strips
            for (int y = 0; y < H; ++y) band[(size_t)(y / br)] += sw[(size_t)(y / 8)] / 8.0;
            double best = INFINITY;
            for (int lb = 0; lb + R <= nb; ++lb) {
                double cost = 0.0;
                for (int b = 0; b < lb; ++b) cost += band[(size_t)b];
                cost /= pct / 100.0;
                for (int k = 0; k < R; ++k) {   // renderer k's set below the lead (flip_of)
                    const int fl = sh->serpentine && R > 1 ? R - 1 - 2 * k : 0;
                    double ck = 0.0;
                    for (int j = 0, b = lb + k; b < nb; b = lb + set_band(++j, k, R, fl))
                        ck += band[(size_t)b];
                    cost = std::max(cost, ck);
                }
                if (cost < best) {
                    best = cost;
                    v[1] = lb * br;
                }
            }
        }
    }
    SH_TRY(bcast_ints(sh, v, "vr_shard_balance_lead"));
    if (v[0]) {
        if (mine != VR_OK) return fail(mine, "vr_shard_balance_lead: %s", msg.c_str());
        return fail(VR_ERR_INVALID, "vr_shard_balance_lead: rank 0's partition failed");
    }
    return vr_shard_set_lead_rows(sh, v[1]);
} catch (...) {
    return caught_exception("vr_shard_balance_lead");
}

int vr_shard_partition(vr_shard* sh)
try {
    return sh ? (rows_mode(sh) ? 1 : 0) : -1;
} catch (...) {
    return -1;
}

vr_status vr_shard_row_range(vr_shard* sh, int rank, int* row_first, int* rows)
try {
    if (!sh || rank < 0 || rank >= sh->nranks) return fail(VR_ERR_INVALID, "vr_shard_row_range: bad argument");
    if (!rows_mode(sh)) return fail(VR_ERR_INVALID, "vr_shard_row_range: the shard renders band sets (vr_shard_set_rows)");
    const int k = band_first_of(sh, rank);
    if (row_first) *row_first = k < 0 ? 0 : sh->row_begin[k];
    if (rows) *rows = k < 0 ? 0 : sh->row_begin[k + 1] - sh->row_begin[k];
    return VR_OK;
} catch (...) {
    return caught_exception("vr_shard_row_range");
}

vr_status vr_shard_rows(vr_shard* sh, int* my_rows, int* rows_per_rank)
try {
    if (!sh) return fail(VR_ERR_INVALID, "vr_shard_rows: null");
    if (my_rows) *my_rows = sh->my_rows;
    if (rows_per_rank) *rows_per_rank = sh->rows_per_rank;
    return VR_OK;
} catch (...) {
    return caught_exception("vr_shard_rows");
}

}  // extern "C"
