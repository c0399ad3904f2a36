// Host cost of the HIP / RCCL / libvr calls one frame of the native frame
// loop (volumetricrenderer_amd/csrc/vr_shard.cpp) makes, each timed alone
// over many calls on an otherwise idle GPU (tiny 64x64 frames, so no call
// waits for the device).  One rank, no peers: what RCCL adds per peer is not
// measured here.
//
//   tools/host_cost [iterations]
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <functional>

#include "vr.h"

namespace {

double per_call_us(int n, const std::function<void()>& f)
{
    const auto t0 = std::chrono::steady_clock::now();
    for (int i = 0; i < n; ++i) f();
    const auto t1 = std::chrono::steady_clock::now();
    return std::chrono::duration<double, std::micro>(t1 - t0).count() / n;
}

#define CHECK(x)                                                         \
    do {                                                                 \
        if ((x) != 0) {                                                  \
            std::fprintf(stderr, "%s failed at %s:%d\n", #x, __FILE__, __LINE__); \
            std::exit(1);                                                \
        }                                                                \
    } while (0)

}  // namespace

int main(int argc, char** argv)
{
    const int n = argc > 1 ? std::atoi(argv[1]) : 2000;
    const int W = 64, H = 64;
    void* ctx = nullptr;
    CHECK(vr_create(0, &ctx));
    vr_volume_recipe rec;
    CHECK(vr_volume_recipe_defaults(&rec));
    rec.size = 32;
    CHECK(vr_generate_volume(ctx, &rec, nullptr));
    vr_object_shader_data osd;
    vr_global_shader_data gsd;
    CHECK(vr_reference_shader_data(1.0f, 0.0f, 0.0f, 0.0f, &osd, &gsd));
    CHECK(vr_set_shader_data(ctx, &osd, &gsd));
    vr_march_params m;
    CHECK(vr_march_defaults(&m));
    m.max_steps = 8;
    CHECK(vr_set_march(ctx, &m));

    hipStream_t s, s2;
    CHECK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    CHECK(hipStreamCreateWithFlags(&s2, hipStreamNonBlocking));
    hipEvent_t e, et;
    CHECK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    CHECK(hipEventCreate(&et));
    void *d_frame = nullptr, *d_gather = nullptr;
    CHECK(hipMalloc(&d_frame, (size_t)W * H * 4));
    CHECK(hipMalloc(&d_gather, (size_t)W * H * 4));
    vr_target t{};
    t.width = W;
    t.height = H;
    t.format = VR_FMT_RGBA8_UNORM;
    t.pixels = d_frame;
    t.row_pitch = (size_t)W * 4;
    CHECK(vr_render(ctx, &t, s));
    CHECK(hipStreamSynchronize(s));

    ncclUniqueId id;
    ncclComm_t comm;
    CHECK(ncclGetUniqueId(&id));
    CHECK(ncclCommInitRank(&comm, 1, id, 0));

    const double render = per_call_us(n, [&] { vr_render(ctx, &t, s); });
    CHECK(hipStreamSynchronize(s));
    const double assemble = per_call_us(n, [&] {
        vr_assemble_bands(ctx, d_gather, (size_t)H, 1, W, H, 16, 4, d_frame, s);
    });
    CHECK(hipStreamSynchronize(s));
    const double rec_notiming = per_call_us(n, [&] { (void)hipEventRecord(e, s); });
    const double rec_timing = per_call_us(n, [&] { (void)hipEventRecord(et, s); });
    CHECK(hipStreamSynchronize(s));
    const double wait = per_call_us(n, [&] { (void)hipStreamWaitEvent(s2, e, 0); });
    CHECK(hipStreamSynchronize(s2));
    const double group = per_call_us(n, [&] {
        (void)ncclGroupStart();
        (void)ncclGroupEnd();
    });
    const double selfp2p = per_call_us(n / 4, [&] {
        (void)ncclGroupStart();
        (void)ncclSend(d_gather, 4096, ncclUint8, 0, comm, s2);
        (void)ncclRecv(d_frame, 4096, ncclUint8, 0, comm, s2);
        (void)ncclGroupEnd();
    });
    CHECK(hipStreamSynchronize(s2));
    double selfk[8] = {};
    for (int k : {2, 4, 7}) {
        selfk[k] = per_call_us(n / 4, [&] {
            (void)ncclGroupStart();
            for (int j = 0; j < k; ++j) {
                (void)ncclSend(static_cast<char*>(d_gather) + 512 * j, 512, ncclUint8, 0, comm, s2);
                (void)ncclRecv(static_cast<char*>(d_frame) + 512 * j, 512, ncclUint8, 0, comm, s2);
            }
            (void)ncclGroupEnd();
        });
        CHECK(hipStreamSynchronize(s2));
    }
    // the native loop's per-frame sequence (vr_shard.cpp one_frame), 2 in flight,
    // with pieces left out to see what they cost
    hipEvent_t rendered[2], done[2];
    for (int p = 0; p < 2; ++p) {
        CHECK(hipEventCreateWithFlags(&rendered[p], hipEventDisableTiming));
        CHECK(hipEventCreateWithFlags(&done[p], hipEventDisableTiming));
    }
    auto loop = [&](bool waits, bool group_on, bool assemble_on) {
        bool pending[2] = {false, false};
        return per_call_us(n, [&] {
            static int p = 0;
            p ^= 1;
            if (waits && pending[p]) (void)hipStreamWaitEvent(s, done[p], 0);
            vr_render(ctx, &t, s);
            if (waits) {
                (void)hipEventRecord(rendered[p], s);
                (void)hipStreamWaitEvent(s2, rendered[p], 0);
            }
            if (group_on) {
                (void)ncclGroupStart();
                (void)ncclGroupEnd();
            }
            if (assemble_on) vr_assemble_bands(ctx, d_gather, (size_t)H, 1, W, H, 16, 4, d_frame, s2);
            if (waits) (void)hipEventRecord(done[p], s2);
            pending[p] = true;
        });
    };
    const double l_full = loop(true, true, true);
    CHECK(hipDeviceSynchronize());
    const double l_noasm = loop(true, true, false);
    CHECK(hipDeviceSynchronize());
    const double l_nowait = loop(false, true, true);
    CHECK(hipDeviceSynchronize());
    const double l_render = loop(false, false, false);
    CHECK(hipDeviceSynchronize());
    std::printf("frame loop per frame: full %.2f  without assembly %.2f  without events/waits %.2f  render only %.2f us\n",
                l_full, l_noasm, l_nowait, l_render);
    const double launch_empty = per_call_us(n, [&] { (void)hipMemsetAsync(d_frame, 0, 4, s); });
    CHECK(hipStreamSynchronize(s));
    std::printf("host us per call (%d calls, idle GPU): vr_render %.2f  vr_assemble_bands %.2f  "
                "hipEventRecord %.2f (timing %.2f)  hipStreamWaitEvent %.2f  ncclGroupStart+End %.2f  "
                "group of send+recv to self %.2f  hipMemsetAsync 4 B %.2f\n",
                n, render, assemble, rec_notiming, rec_timing, wait, group, selfp2p, launch_empty);
    std::printf("groups of k send+recv pairs to self: k=2 %.2f  k=4 %.2f  k=7 %.2f us\n", selfk[2], selfk[4], selfk[7]);
    ncclCommDestroy(comm);
    vr_destroy(ctx);
    return 0;
}
