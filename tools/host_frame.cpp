// Host cost per frame of the native frame loop at the BASELINE config-5 frame
// (1080p x 128 over the 512^3 recipe volume), and of its pieces, on an idle
// GPU: every measurement enqueues batches of 8 and synchronises between
// batches, so no call waits for a full queue.  Also what a captured hipGraph
// of one render costs to launch.
//
//   tools/host_frame [batches]
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <functional>
#include <vector>

#include "vr.h"
#include "vr_shard.h"

namespace {

#define CHECK(x)                                                                                        \
    do {                                                                                                \
        if ((x) != 0) {                                                                                 \
            std::fprintf(stderr, "%s failed at %s:%d (%s | %s)\n", #x, __FILE__, __LINE__, vr_last_error(), \
                         vr_shard_last_error());                                                        \
            std::exit(1);                                                                               \
        }                                                                                               \
    } while (0)

struct Big {
    float v[120];
};

__global__ void k_empty(Big b, int* out)
{
    if (b.v[0] == 12345.0f && threadIdx.x == 0) out[0] = 1;
}

__global__ void k_small(float v, int* out)
{
    if (v == 12345.0f && threadIdx.x == 0) out[0] = 1;
}

// median over batches of the host microseconds per call of f, 8 calls per batch
double per_call_us(int batches, const std::function<void()>& f, const std::function<void()>& sync)
{
    std::vector<double> v;
    for (int b = 0; b < batches; ++b) {
        sync();
        const auto t0 = std::chrono::steady_clock::now();
        for (int i = 0; i < 8; ++i) f();
        const auto t1 = std::chrono::steady_clock::now();
        v.push_back(std::chrono::duration<double, std::micro>(t1 - t0).count() / 8);
    }
    sync();
    std::sort(v.begin(), v.end());
    return v[v.size() / 2];
}

}  // namespace

int main(int argc, char** argv)
{
    const int nb = argc > 1 ? std::atoi(argv[1]) : 50;
    const int W = 1920, H = 1080;
    void* ctx = nullptr;
    CHECK(vr_create(0, &ctx));
    vr_volume_recipe rec;
    CHECK(vr_volume_recipe_defaults(&rec));
    rec.size = 512;
    for (float& f : rec.freq) f *= 128.0f / 512.0f;   // vr.scaled_recipe
    CHECK(vr_generate_volume(ctx, &rec, nullptr));
    vr_object_shader_data osd;
    vr_global_shader_data gsd;
    CHECK(vr_reference_shader_data(1280.0f / 720.0f, 0.0f, 0.0f, 0.0f, &osd, &gsd));
    CHECK(vr_set_shader_data(ctx, &osd, &gsd));
    vr_march_params m;
    CHECK(vr_march_defaults(&m));
    CHECK(vr_set_march(ctx, &m));
    hipStream_t s, s2;
    CHECK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    CHECK(hipStreamCreateWithFlags(&s2, hipStreamNonBlocking));
    auto sync = [&] { CHECK(hipDeviceSynchronize()); };
    hipEvent_t e;
    CHECK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    int* d_out = nullptr;
    void* d_frame = nullptr;
    CHECK(hipMalloc(&d_out, 64));
    CHECK(hipMalloc(&d_frame, (size_t)W * H * 4));
    Big big{};
    std::printf("variant %s\n", vr_kernel_variant(ctx));

    const double t_empty = per_call_us(nb, [&] { hipLaunchKernelGGL(k_empty, dim3(1), dim3(64), 0, s, big, d_out); }, sync);
    const double t_small = per_call_us(nb, [&] { hipLaunchKernelGGL(k_small, dim3(1), dim3(64), 0, s, 1.0f, d_out); }, sync);
    const double t_bigg = per_call_us(nb, [&] { hipLaunchKernelGGL(k_empty, dim3(9000), dim3(256), 0, s, big, d_out); }, sync);
    // the same kernel through hipModuleLaunchKernel with its arguments as one buffer
    hipFunction_t fn = nullptr;
    CHECK(hipGetFuncBySymbol(&fn, reinterpret_cast<const void*>(&k_empty)));
    struct {
        Big b;
        int* out;
    } argbuf{big, d_out};
    size_t argsz = sizeof argbuf;
    void* extra[] = {HIP_LAUNCH_PARAM_BUFFER_POINTER, &argbuf, HIP_LAUNCH_PARAM_BUFFER_SIZE, &argsz, HIP_LAUNCH_PARAM_END};
    hipError_t me = hipSuccess;
    const double t_mod = per_call_us(nb, [&] {
        const hipError_t r = hipModuleLaunchKernel(fn, 1, 1, 1, 64, 1, 1, 0, s, nullptr, extra);
        if (r != hipSuccess) me = r;
    }, sync);
    (void)hipGetLastError();
    std::printf("hipModuleLaunchKernel (480-B arg buffer) %.2f us (%s)\n", t_mod, hipGetErrorString(me));
    // a launch that records an event at its end (hipExtLaunchKernel's stopEvent)
    hipEvent_t es;
    CHECK(hipEventCreateWithFlags(&es, hipEventDisableTiming));
    void* kargs[] = {&big, &d_out};
    hipError_t xe = hipSuccess;
    const double t_ext = per_call_us(nb, [&] {
        const hipError_t r = hipExtLaunchKernel(reinterpret_cast<const void*>(&k_empty), dim3(1), dim3(64), kargs, 0, s,
                                                nullptr, es, 0);
        if (r != hipSuccess) xe = r;
    }, sync);
    (void)hipGetLastError();
    const double t_ext_wait = per_call_us(nb, [&] {
        (void)hipExtLaunchKernel(reinterpret_cast<const void*>(&k_empty), dim3(1), dim3(64), kargs, 0, s, nullptr, es, 0);
        (void)hipStreamWaitEvent(s2, es, 0);
    }, sync);
    const double t_plain_rec_wait = per_call_us(nb, [&] {
        hipLaunchKernelGGL(k_empty, dim3(1), dim3(64), 0, s, big, d_out);
        (void)hipEventRecord(es, s);
        (void)hipStreamWaitEvent(s2, es, 0);
    }, sync);
    std::printf("hipExtLaunchKernel with stopEvent %.2f us (%s); + hipStreamWaitEvent on it %.2f; plain launch + "
                "hipEventRecord + hipStreamWaitEvent %.2f\n", t_ext, hipGetErrorString(xe), t_ext_wait,
                t_plain_rec_wait);
    const double t_rec = per_call_us(nb, [&] { (void)hipEventRecord(e, s); }, sync);
    hipEvent_t ef;
    CHECK(hipEventCreateWithFlags(&ef, hipEventDisableTiming | hipEventDisableSystemFence));
    const double t_recf = per_call_us(nb, [&] { (void)hipEventRecord(ef, s); }, sync);
    const double t_wait = per_call_us(nb, [&] { (void)hipStreamWaitEvent(s2, e, 0); }, sync);
    uint32_t* flag = nullptr;
    CHECK(hipMalloc(&flag, 64));
    CHECK(hipMemset(flag, 0, 64));
    uint32_t val = 0;
    const double t_wv = per_call_us(nb, [&] { (void)hipStreamWriteValue32(s, flag, ++val, 0); }, sync);
    const double t_wtv = per_call_us(nb, [&] { (void)hipStreamWaitValue32(s2, flag, 1, hipStreamWaitValueGte, 0xffffffffu); }, sync);
    void* pinned = nullptr;
    CHECK(hipHostMalloc(&pinned, 4096, hipHostMallocDefault));
    const double t_cp = per_call_us(nb, [&] { (void)hipMemcpyAsync(d_out, pinned, 512, hipMemcpyHostToDevice, s); }, sync);
    int dev = 0;
    const double t_setdev = per_call_us(nb, [&] { (void)hipSetDevice(0); }, sync);
    const double t_getdev = per_call_us(nb, [&] { (void)hipGetDevice(&dev); }, sync);
    std::printf("hipLaunchKernel: 480-B args 1 block %.2f us, 4-B args %.2f, 480-B args 9000 blocks %.2f; "
                "hipEventRecord %.2f (no system fence %.2f), hipStreamWaitEvent %.2f, hipStreamWriteValue32 %.2f, "
                "hipStreamWaitValue32 %.2f, hipMemcpyAsync 512 B H2D %.2f, hipSetDevice %.2f, hipGetDevice %.2f\n",
                t_empty, t_small, t_bigg, t_rec, t_recf, t_wait, t_wv, t_wtv, t_cp, t_setdev, t_getdev);

    (void)hipGetLastError();
    CHECK(hipDeviceSynchronize());
    for (int n : {1, 8}) {
        vr_target t{};
        t.width = W;
        t.height = H;
        t.format = n == 1 ? VR_FMT_RGBA8_UNORM : VR_FMT_R8_UNORM;
        t.band_rows = n == 1 ? 0 : 16;
        t.band_stride = n;
        t.band_first = 0;
        t.pixels = d_frame;
        CHECK(vr_render(ctx, &t, s));   // region lists
        sync();
        CHECK(vr_set_option(ctx, "launch_cache", 0));
        const double t_r0 = per_call_us(nb, [&] { CHECK(vr_render(ctx, &t, s)); }, sync);
        CHECK(vr_set_option(ctx, "launch_cache", 1));
        const double t_r = per_call_us(nb, [&] { CHECK(vr_render(ctx, &t, s)); }, sync);
        // the same render captured in a hipGraph, replayed
        hipGraph_t g;
        hipGraphExec_t ge;
        CHECK(hipStreamBeginCapture(s, hipStreamCaptureModeRelaxed));
        CHECK(vr_render(ctx, &t, s));
        CHECK(hipStreamEndCapture(s, &g));
        CHECK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
        const double t_g = per_call_us(nb, [&] { CHECK(hipGraphLaunch(ge, s)); }, sync);
        std::printf("N=%d band set: vr_render %.2f us (launch cache off: %.2f), hipGraphLaunch of it %.2f us\n", n, t_r,
                    t_r0, t_g);
        (void)hipGraphExecDestroy(ge);
        (void)hipGraphDestroy(g);
    }
    for (int th : {1, 2})
    for (int lc : {1, 0})
    for (int n : {1, 8})
        for (int rank : {0, 1})
            for (int rs : {1, 2}) {
                if (lc == 0 && (n == 1 || rs == 1 || th == 2)) continue;
                if (th == 2 && (n == 1 || rs == 1)) continue;
                CHECK(vr_set_option(ctx, "launch_cache", lc));
                if (n == 1 && rank == 1) continue;
                vr_shard* sh = nullptr;
                CHECK(vr_shard_alloc(ctx, n, rank, W, H, VR_FMT_RGBA8_UNORM, 16, &sh));
                CHECK(vr_shard_set_solo(sh, 1));
                CHECK(vr_shard_set_render_streams(sh, rs));
                CHECK(vr_shard_set_host_threads(sh, th));
                CHECK(vr_shard_run(sh, 8, s, 0, nullptr));
                sync();
                std::vector<double> hv;
                for (int b = 0; b < nb; ++b) {
                    double h = 0.0;
                    CHECK(vr_shard_run_frames(sh, 8, nullptr, nullptr, s, 0, nullptr, &h));
                    hv.push_back(h * 1e3);
                    sync();
                }
                std::sort(hv.begin(), hv.end());
                std::printf("solo loop N=%d rank %d, %d render stream(s)%s, %d host thread(s): host %.2f us per frame\n", n,
                            rank, rs, lc ? "" : ", launch cache off", th, hv[hv.size() / 2]);
                CHECK(vr_shard_destroy(sh));
            }
    vr_destroy(ctx);
    return 0;
}
