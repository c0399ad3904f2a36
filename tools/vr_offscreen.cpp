// vr_offscreen -- thin C++ offscreen driver for libvr.
//
// Replaces the reference application's start-up and frame loop
// (TestMain.cpp:41-263): it builds the noise volume (:43-92, here on the GPU),
// produces the per-frame uniforms (:219-245), renders frames (:194-217,
// :251-255) and writes the last frame as a PNG.  The window, GLFW key loop and
// ImGui are replaced by command-line arguments:
//   --width W --height H --steps S --size N --frames F
//   --phi DEG --theta DEG --spin DEG_PER_FRAME   (the A/D keys, :177-180)
//   --format unorm|srgb  --out frame.png
//   --procedural 0|1 --shadow K   (BASELINE configs 2/3: in-kernel Perlin-Worley medium)
// and it prints one timing line (hipEvent per frame, median).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "png_writer.hpp"
#include "vr_renderer.hpp"

#define HIPCHECK(x)                                                                            \
    do {                                                                                       \
        hipError_t e_ = (x);                                                                   \
        if (e_ != hipSuccess) {                                                                \
            std::fprintf(stderr, "%s failed: %s\n", #x, hipGetErrorString(e_));                \
            return 2;                                                                          \
        }                                                                                      \
    } while (0)

int main(int argc, char** argv)
{
    int width = 1280, height = 720, steps = 128, size = 128, frames = 10;
    float phi = 0.f, theta = 0.f, spin = 0.f;
    int procedural = 0, shadow = 0;
    std::string out = "frame.png", fmt = "unorm";
    for (int i = 1; i + 1 < argc; i += 2) {
        const std::string k = argv[i], v = argv[i + 1];
        if (k == "--width") width = std::atoi(v.c_str());
        else if (k == "--height") height = std::atoi(v.c_str());
        else if (k == "--steps") steps = std::atoi(v.c_str());
        else if (k == "--size") size = std::atoi(v.c_str());
        else if (k == "--frames") frames = std::atoi(v.c_str());
        else if (k == "--phi") phi = (float)std::atof(v.c_str());
        else if (k == "--theta") theta = (float)std::atof(v.c_str());
        else if (k == "--spin") spin = (float)std::atof(v.c_str());
        else if (k == "--format") fmt = v;
        else if (k == "--out") out = v;
        else if (k == "--procedural") procedural = std::atoi(v.c_str());
        else if (k == "--shadow") shadow = std::atoi(v.c_str());
        else {
            std::fprintf(stderr, "unknown option %s\n", k.c_str());
            return 1;
        }
    }
    if (frames < 1) frames = 1;
    try {
        vr::Renderer renderer(0);
        vr_volume_recipe recipe;
        vr_volume_recipe_defaults(&recipe);
        recipe.size = size;
        for (int k = 0; k < 4; ++k) recipe.freq[k] *= 128.0f / (float)size;  // same field at any N
        if (procedural) {
            vr_procedural p;
            vr_procedural_defaults(&p);
            p.enabled = 1;
            p.shadow_steps = shadow;
            renderer.SetProcedural(p);
        } else {
            renderer.GenerateVolume(recipe);
        }
        vr_march_params m;
        vr_march_defaults(&m);
        m.max_steps = steps;
        renderer.SetMarch(m);

        const vr_format vf = fmt == "srgb" ? VR_FMT_RGBA8_SRGB : VR_FMT_RGBA8_UNORM;
        void* d_pixels = nullptr;
        HIPCHECK(hipMalloc(&d_pixels, (size_t)width * height * 4));
        hipStream_t s;
        HIPCHECK(hipStreamCreate(&s));
        hipEvent_t e0, e1;
        HIPCHECK(hipEventCreate(&e0));
        HIPCHECK(hipEventCreate(&e1));
        std::vector<float> ms;
        for (int f = 0; f < frames; ++f) {
            vr::ObjectShaderData osd;
            vr::GlobalShaderData gsd;
            // Model = rotZ(phi) * rotY(theta); the reference's aspect is the
            // window's, 1280/720 (TestMain.cpp:226), here the target's.
            vr::Renderer::ReferenceShaderData((float)width / (float)height, phi + spin * f, theta, 0.0f, &osd, &gsd);
            renderer.UpdateObjectData(osd);
            renderer.UpdateGlobalData(gsd);
            HIPCHECK(hipEventRecord(e0, s));
            renderer.EnqueueRenderPass({width, height}, vf, d_pixels, s);
            HIPCHECK(hipEventRecord(e1, s));
            HIPCHECK(hipEventSynchronize(e1));
            float t = 0.f;
            HIPCHECK(hipEventElapsedTime(&t, e0, e1));
            ms.push_back(t);
        }
        std::vector<unsigned char> host((size_t)width * height * 4);
        HIPCHECK(hipMemcpy(host.data(), d_pixels, host.size(), hipMemcpyDeviceToHost));
        if (!vr::tools::WritePng(out, host.data(), width, height)) {
            std::fprintf(stderr, "could not write %s\n", out.c_str());
            return 3;
        }
        std::sort(ms.begin(), ms.end());
        const double med = ms[ms.size() / 2];
        std::printf("vr_offscreen: %dx%d steps %d volume %d^3 kernel %s frames %d median %.3f ms "
                    "(%.1f Mray/s nominal) -> %s\n",
                    width, height, steps, size, renderer.KernelVariant(), frames, med,
                    (double)width * height * steps / (med * 1e-3) / 1e6, out.c_str());
        (void)hipFree(d_pixels);
        (void)hipStreamDestroy(s);
    } catch (const vr::Error& e) {
        std::fprintf(stderr, "vr_offscreen: %s\n", e.what());
        return 4;
    }
    return 0;
}
