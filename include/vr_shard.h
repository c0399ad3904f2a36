/*
 * vr_shard.h -- multi-GPU frame pipeline over RCCL (libvr_shard.so).
 *
 * pixels are independent, so a frame shards by screen
 * rows over the GPUs of one node.  Band b of `band_rows` rows goes to rank
 * b mod nranks (interleaved bands: the centred hexagonal silhouette makes
 * contiguous strips 2.45x imbalanced at 8 ranks, interleaved bands 1.00-1.02).
 * Each rank renders its packed band set with vr_render; one RCCL exchange
 * per frame sends the sets to rank 0 over xGMI (grouped point-to-point
 * sends/receives), and rank 0 scatters them into the frame with
 * vr_assemble_frame.  The band sets travel in the grey format of the frame's
 * (vr.h VR_FMT_R8_UNORM / R8_SRGB / R32F: the shader's pixel is
 * vec4(vec3(c), 1), frag.glsl:79-80), a quarter of the RGBA bytes, and the
 * assembly expands them.  The reference has no multi-GPU code at all (SURVEY.md
 * sec. 2); this replaces its single-queue frame loop (VulkanRenderer.cpp:
 * 142-230) for N GPUs and keeps its 2 frames in flight (:13): frame i's
 * exchange and assembly run on a communication stream while frame i+1
 * renders, with double-buffered band sets and frames.  The whole frame loop
 * is native, so the host cost per frame is a few HIP/RCCL calls (strong
 * scaling of a ~0.2 ms frame to 8 GPUs is host-bound from Python).
 *
 * One process per GPU.  The communicator is this library's own: rank 0 makes
 * an id with vr_shard_unique_id, the caller broadcasts its bytes (e.g. over
 * torch.distributed), and every rank calls vr_shard_create with it.
 * Status codes are vr_status (vr.h); messages via vr_shard_last_error().
 */
#ifndef VR_SHARD_H
#define VR_SHARD_H
#include "vr.h"

#ifdef __cplusplus
extern "C" {
#endif

#define VR_SHARD_ID_BYTES 128

typedef struct vr_shard vr_shard;

const char* vr_shard_last_error(void);
/* vr_build_id of the sources libvr_shard.so was built from (vr.h).       */
const char* vr_shard_build_id(void);

/* A new communicator id (call on rank 0, then share the bytes). */
vr_status vr_shard_unique_id(uint8_t id[VR_SHARD_ID_BYTES]);

/* Collective over the nranks processes: joins the communicator on ctx's
 * device and allocates the double-buffered band sets (every rank), gather
 * buffers and frames (rank 0) for W x H frames of `format`.  The ctx keeps
 * its volume, shader data and march constants; vr_shard_run renders with
 * whatever they are when it is called.
 * Loopback (id = NULL, rank 0): no communicator; this process renders every
 * rank's band set into its gather slot and assembles the frame -- the
 * N-rank data layout and assembly on one GPU (tests, rehearsals). */
vr_status vr_shard_create(void* ctx, const uint8_t id[VR_SHARD_ID_BYTES], int nranks, int rank,
                          int width, int height, int format, int band_rows, vr_shard** out);
/* The two halves of vr_shard_create, so that ranks can agree that every
 * allocation succeeded before any of them enters the collective
 * ncclCommInitRank (a rank that failed to allocate would otherwise leave its
 * peers blocked in the init):
 *   vr_shard_alloc   -- streams, events and buffers only (local, never
 *                       blocks); the result behaves as loopback on rank 0
 *                       until it is connected;
 *   vr_shard_connect -- collective: joins the communicator with `id`.
 * The caller agrees on success between the two (e.g. an all-reduce over a
 * torch.distributed group) and destroys the shard on every rank otherwise. */
vr_status vr_shard_alloc(void* ctx, int nranks, int rank, int width, int height, int format, int band_rows,
                         vr_shard** out);
vr_status vr_shard_connect(vr_shard* sh, const uint8_t id[VR_SHARD_ID_BYTES]);
vr_status vr_shard_destroy(vr_shard* sh);

/* Render `frames` frames (collective: every rank, same count), 2 in flight.
 * Asynchronous on `stream`: the frames start after the work queued on it,
 * and when the call returns the work is queued and `stream` is ordered after
 * the last frame's exchange (and, on rank 0, its assembly).  By default the
 * renders alternate between two streams of the shard, one per buffer parity
 * (vr_shard_set_render_streams): frame i+1's render waits only for frame
 * i-1's exchange, never for frame i's render, so consecutive renders overlap.
 * If kernel_ms is not null, every `sample_every`-th render is bracketed by
 * HIP events on its render stream and their mean duration is written there
 * (this call then waits for that last sample; overlapping renders make it
 * longer than the frame period). */
vr_status vr_shard_run(vr_shard* sh, int frames, void* stream, int sample_every, float* kernel_ms);
/* vr_shard_run with a moving camera (the reference's held A/D/W/S key,
 * TestMain.cpp:171-184, and its per-frame UBO updates, :219-249): frame i
 * renders with shader data (osd[i], gsd[i]) -- every rank passes the same
 * arrays -- set on the ctx before its render; osd = gsd = NULL keeps the ctx's.
 * host_ms (optional): host time per frame spent queueing the frames (before
 * any wait for the sampled renders), ms. */
vr_status vr_shard_run_frames(vr_shard* sh, int frames, const vr_object_shader_data* osd,
                              const vr_global_shader_data* gsd, void* stream, int sample_every, float* kernel_ms,
                              double* host_ms);

/* Collective barrier + synchronisation: returns once the work queued on
 * `stream` and on the communication stream of EVERY rank before the call has
 * finished (one 4-byte RCCL all-reduce over xGMI, ordered after `stream`,
 * then a host wait).  Costs microseconds where a host-side gloo barrier
 * across 8 processes costs a large fraction of a 1/8-frame; the bench
 * brackets its timed frames with it.  Loopback: a stream synchronisation. */
vr_status vr_shard_barrier(vr_shard* sh, void* stream);

/* Collective, once per volume (SURVEY.md sec. 8e collective 1): rank 0's
 * RGBA8 volume (device pointer, nz x ny x nx x 4 bytes, x fastest; ignored on
 * the other ranks) goes to every rank with one ncclBroadcast over xGMI, and
 * every rank's ctx installs it as vr_set_volume_device would.  All ranks
 * name the same extent; they agree on it and on every receive buffer (one
 * all-reduce) before the broadcast, so a failure on one rank fails all of
 * them instead of leaving peers blocked.  Synchronous: returns once this
 * rank's ctx holds the volume.  Loopback: vr_set_volume_device. */
vr_status vr_shard_share_volume(vr_shard* sh, const void* d_rgba8, int nx, int ny, int nz, void* stream);

/* Rank 0: the last assembled frame (device pointer, tight rows, the shard's
 * format) once `stream` of the last vr_shard_run has reached it.  Other ranks:
 * their last band set, in the grey format of the frame's (1 B per pixel, or
 * 4 B for VR_FMT_RGBA32F frames). */
vr_status vr_shard_frame(vr_shard* sh, void** pixels, size_t* row_pitch, int* rows);

/* Copy what vr_shard_frame points at into a caller-owned device buffer
 * (rows of `dst_pitch` bytes; 0 = tight), ordered on `stream`. */
vr_status vr_shard_copy_frame(vr_shard* sh, void* dst, size_t dst_pitch, void* stream);

/* This rank's rows (packed) and every rank's slot rows (rank 0's count). */
vr_status vr_shard_rows(vr_shard* sh, int* my_rows, int* rows_per_rank);

/* Failure handling.  The communicator is non-blocking: every host wait on a
 * collective (vr_shard_connect's init, vr_shard_barrier, vr_shard_share_volume,
 * the sampled renders of vr_shard_run) polls the stream and the
 * communicator's asynchronous error against a deadline -- `seconds`, default
 * the environment's VR_SHARD_TIMEOUT_S or 120.  On an error or at the
 * deadline the communicator is aborted (ncclCommAbort) and the call returns
 * VR_ERR_COMM or VR_ERR_TIMEOUT: a rank whose peer died fails with a message
 * instead of waiting forever.  Every later collective on the shard fails at
 * once (vr_shard_aborted = 1); vr_shard_destroy still frees it. */
vr_status vr_shard_set_timeout(vr_shard* sh, double seconds);
/* Render streams of vr_shard_run, 1 to 4: n >= 2 = frame i renders on stream
 * i mod n of the shard with buffer set i mod n, so n consecutive frames are in
 * flight and their renders overlap (with the exchange on the render streams;
 * on the communication stream at most 2); the default is 2;
 * 1 = every render on the caller's stream, after the previous one.  Results
 * are identical.  Switching waits (host) for the frames in flight.  A
 * procedural medium with shadow rays always takes one stream: each of its
 * frames writes the ctx's deferred-shadow scratch, so they cannot overlap
 * (two streams cost 12 % in waits). */
vr_status vr_shard_set_render_streams(vr_shard* sh, int n);
int       vr_shard_get_render_streams(vr_shard* sh);
/* Per-rank rehearsal on one GPU (an unconnected shard, any rank): 1 = each
 * frame renders only this rank's band set, on the same streams and buffers
 * as the N-rank loop, with no exchange (rank 0 still assembles, from its own
 * set and whatever the other slots hold).  The frame period and host cost of
 * one rank without its peers (tools/band_scaling.py --native). */
vr_status vr_shard_set_solo(vr_shard* sh, int on);
/* Host threads of vr_shard_run: 1 (default) = the caller's thread issues
 * every frame; 2 = a worker thread issues each frame's exchange half (wait
 * for the render, RCCL send / receive, rank 0's assembly) while the caller's
 * thread issues the renders, so the host time per frame is the longer half
 * instead of the sum.  Results are identical.                             */
vr_status vr_shard_set_host_threads(vr_shard* sh, int n);
/* Where the exchange runs (with 2 render streams): 1 (default) = on the
 * frame's own render stream, after its render, over one communicator per
 * buffer parity (the second split from the first at the first such run,
 * collectively): no event per frame, the host cost of a frame is its
 * launches alone (host_threads does not apply); 0 = on the shard's
 * communication stream, ordered after each render by events.  Every rank
 * must choose the same.  Results are identical.                           */
vr_status vr_shard_set_exchange_streams(vr_shard* sh, int on_render);
/* Rank 0 as a compositor: 1 = rank 0 renders no bands and only receives and
 * assembles; ranks 1..N-1 render the interleaved band sets of a world of N-1
 * renderers (rank r: band_stride N-1, band_first r-1).  0 = every rank
 * renders (band_stride N, band_first rank) and rank 0 renders its own bands
 * in place.  Default: 1 from 8 ranks on (the assembly of 7/8 of a frame
 * beside rank 0's render made it the slowest rank; with lead rows,
 * vr_shard_balance_lead, a compositor also beats row ranges at 4K).  Every
 * rank must choose the same, before its first frames (band buffers are
 * resized).
 * Results are identical. */
vr_status vr_shard_set_compositor(vr_shard* sh, int on);
int       vr_shard_get_compositor(vr_shard* sh);
/* This rank's band set: band_stride, band_first and band_flip of its
 * vr_render target (rank 0 as a compositor: stride N-1, first -1, no rows). */
vr_status vr_shard_bands(vr_shard* sh, int* band_stride, int* band_first, int* band_flip);
/* Serpentine band sets (round 6; new, no reference counterpart): 1 (the
 * default) = renderer k of R deals its bands forwards in even periods of R
 * bands and backwards in odd ones (vr.h vr_target.band_flip R-1-2k), and the
 * assembly follows (VR_ASSEMBLE_SERPENTINE); 0 = the plain interleave, band
 * k + jR.  With the plain interleave renderer 0 takes the first band of every
 * period, and below the cube's widest rows the work per band falls down the
 * frame, so it was the slowest of 7 in every config-5 rehearsal at 8 ranks
 * (DESIGN.md sec. 7.5).  Every rank must choose the same, before its first
 * frames.  Results are identical. */
vr_status vr_shard_set_serpentine(vr_shard* sh, int on);
int       vr_shard_get_serpentine(vr_shard* sh);
/* Contiguous row ranges instead of interleaved band sets.  Renderer k (rank
 * k, or rank k + 1 with rank 0 as a compositor) renders frame rows
 * [row_begin[k], row_begin[k + 1]) (vr.h VR_TARGET_ROW_RANGE); rank 0 gathers
 * them at their own rows of a grey frame and expands the rows below its own
 * range in one launch.  A rank's rays then cover one slab of the volume, and
 * its L2s serve its rows' neighbours: the 4K frame of a 128^3 grid (config 4)
 * at 8 ranks takes 0.0480 ms per frame against 0.0562 with 16-row bands
 * (DESIGN.md sec. 7.3).  Rank 0 rendering in place takes a smaller share of
 * the work (2 % less per other rank): it also expands the other ranks' rows.  row_begin[renderers + 1]: 0, non-decreasing,
 * multiples of 8, the frame height last; NULL = back to band sets.  Every
 * rank must set the same ranges.  The choice of band sets or ranges is fixed
 * by the first frames; new ranges between runs wait for the frames in flight.
 * A later vr_shard_set_compositor returns the shard to band sets.
 * vr_shard_balance_rows: the ranges of equal estimated work for the ctx's
 * current camera (vr_row_partition), computed by rank 0 and broadcast -- a
 * collective: every rank calls it.  vr_shard_partition: 1 = row ranges,
 * 0 = band sets.  vr_shard_row_range: a rank's range (row ranges only). */
vr_status vr_shard_set_rows(vr_shard* sh, const int* row_begin);
vr_status vr_shard_balance_rows(vr_shard* sh);
/* Collective, between runs, with row ranges: every rank passes its measured
 * time per frame (e.g. vr_shard_run's kernel_ms); rank 0 splits the frame
 * again with the ranges' times (vr_row_partition_measured) and every rank
 * takes the new ranges.  The frames in flight finish first.  The model's
 * split leaves ranks 2 and 5 of config 4 at 8 ranks 8-10 % above the others;
 * one measured round evens them. */
vr_status vr_shard_rebalance_rows(vr_shard* sh, double my_ms);
int       vr_shard_partition(vr_shard* sh);
vr_status vr_shard_row_range(vr_shard* sh, int rank, int* row_first, int* rows);
int       vr_shard_aborted(vr_shard* sh);
/* The last vr_shard_run_frames call that sampled renders (sample_every > 0):
 * the union of the sampled renders' intervals (busy_ms; renders that overlap
 * on several render streams count once) and the span from the first sampled
 * start to the last sampled end (span_ms), both totals in ms on the GPU's
 * clock.  With sample_every = 1, busy_ms / frames is the GPU time per frame
 * the renders held the machine (bench.py roofline.kernel_busy_ms_per_frame).
 * New (no reference counterpart). */
vr_status vr_shard_sampled_busy(vr_shard* sh, double* busy_ms, double* span_ms);
/* Rank 0's lead rows (round 6; new, no reference counterpart): with rank 0 as
 * a compositor over band sets, rank 0 also renders the frame rows
 * [0, rows) in place -- a row range beside its assembly -- and renderer k's
 * band set starts below them (frame band rows/band_rows + k - 1, stride
 * nranks - 1).  rows: a multiple of band_rows below the frame height; 0 = none
 * (the default).  Set before the first frames; vr_shard_set_compositor(0)
 * and row ranges clear it.  vr_shard_balance_lead (collective) sizes it for
 * the ctx's camera: rank 0 counts as pct % of a renderer, and of every lead
 * of whole bands it takes the one whose largest estimated cost -- rank 0's
 * lead work / (pct / 100), or a renderer's band-set work (vr_row_work) -- is
 * smallest, and broadcasts it.  vr_shard_bands reports band_first -1 for rank 0
 * and the offset sets of the renderers. */
vr_status vr_shard_set_lead_rows(vr_shard* sh, int rows);
int       vr_shard_get_lead_rows(vr_shard* sh);
vr_status vr_shard_balance_lead(vr_shard* sh, int pct);
/* Self-test of the deadline loop on the host (no GPU, no RCCL): mode 0 a
 * state that completes after 5 polls, 1 one that fails at the 3rd, 2 one that
 * never completes.  Returns 0 done, 1 failed, 2 deadline (-1 bad mode) and
 * the number of polls. */
int       vr_shard_poll_selftest(int mode, double timeout_s, int* polls);

#ifdef __cplusplus
}
#endif
#endif /* VR_SHARD_H */
