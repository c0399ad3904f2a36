// vr_renderer.hpp -- C++ host interface over the C ABI of vr.h.
//
// A thin RAII layer that gives C++ callers the shape of the reference's own
// host API for this path:
//
//   reference (file:line)                                  here
//   vkc::Renderer::Init / Shutdown (VulkanRenderer.h:68-72) Renderer ctor / dtor
//   vkc::Texture3D(data, extent) (VulkanTexture.h:55-60)    Renderer::SetVolume
//   noise -> pixelData start-up (TestMain.cpp:43-92)        Renderer::GenerateVolume
//   UniformBuffer<ObjectShaderData>::Update (TestMain:248)  Renderer::UpdateObjectData
//   UniformBuffer<GlobalShaderData>::Update (TestMain:249)  Renderer::UpdateGlobalData
//   EnqueueRenderPass("BasePass", rect, ...) + draw
//     (VulkanRenderer.h:84-87, TestMain.cpp:194-217)       Renderer::EnqueueRenderPass
//
// Errors are thrown as vr::Error on the C++ side, as the reference throws from
// Error() (Utils.h:22-29).  They become status codes at the C ABI.
#pragma once

#include <stdexcept>
#include <string>

#include "vr.h"

namespace vr {

using ObjectShaderData = vr_object_shader_data;   // TestMain.cpp:27-32
using GlobalShaderData = vr_global_shader_data;   // TestMain.cpp:34-39

class Error : public std::runtime_error {
public:
    Error(vr_status s, const std::string& what) : std::runtime_error(what), status(s) {}
    vr_status status;
};

inline void Check(vr_status s, const char* where)
{
    if (s != VR_OK) throw Error(s, std::string(where) + ": " + vr_last_error());
}

struct Rect2D {  // VkRect2D analogue: the rows/columns of the frame to draw
    int width = 0, height = 0;
};

class Renderer {
public:
    explicit Renderer(int device = 0) { Check(vr_create(device, &ctx_), "vr_create"); }
    ~Renderer() { vr_destroy(ctx_); }
    Renderer(const Renderer&) = delete;
    Renderer& operator=(const Renderer&) = delete;

    void SetVolume(const uint8_t* rgba, int nx, int ny, int nz)
    {
        Check(vr_set_volume(ctx_, rgba, nx, ny, nz), "vr_set_volume");
    }
    void GenerateVolume(const vr_volume_recipe& r, void* stream = nullptr)
    {
        Check(vr_generate_volume(ctx_, &r, stream), "vr_generate_volume");
    }
    void UpdateObjectData(const ObjectShaderData& o)
    {
        osd_ = o;
        has_osd_ = true;
        Flush();
    }
    void UpdateGlobalData(const GlobalShaderData& g)
    {
        gsd_ = g;
        has_gsd_ = true;
        Flush();
    }
    void SetMarch(const vr_march_params& m) { Check(vr_set_march(ctx_, &m), "vr_set_march"); }
    // BASELINE configs 2/3: the procedural medium replaces the volume (enabled = 0 restores it)
    void SetProcedural(const vr_procedural& p) { Check(vr_set_procedural(ctx_, &p), "vr_set_procedural"); }
    void SetOption(const char* name, int value) { Check(vr_set_option(ctx_, name, value), "vr_set_option"); }

    // Render the whole frame (or a band set) into a device buffer.
    void EnqueueRenderPass(const Rect2D& rect, vr_format fmt, void* d_pixels, void* stream = nullptr,
                           uint64_t* d_step_counter = nullptr, int band_rows = 0, int band_stride = 1,
                           int band_first = 0, int band_flip = 0)
    {
        vr_target t{};
        t.width = rect.width;
        t.height = rect.height;
        t.format = fmt;
        t.band_rows = band_rows;
        t.band_stride = band_stride;
        t.band_first = band_first;
        t.band_flip = band_flip;   // vr.h: odd bands of the set shifted (the serpentine deal)
        t.pixels = d_pixels;
        t.row_pitch = 0;
        t.step_counter = d_step_counter;
        Check(vr_render(ctx_, &t, stream), "vr_render");
    }
    const char* KernelVariant() const { return vr_kernel_variant(ctx_); }
    void* Handle() const { return ctx_; }

    static void ReferenceShaderData(float aspect, float phi_deg, float theta_deg, float frame_time,
                                    ObjectShaderData* o, GlobalShaderData* g)
    {
        Check(vr_reference_shader_data(aspect, phi_deg, theta_deg, frame_time, o, g),
              "vr_reference_shader_data");
    }

private:
    void Flush()
    {
        if (has_osd_ && has_gsd_) Check(vr_set_shader_data(ctx_, &osd_, &gsd_), "vr_set_shader_data");
    }
    void* ctx_ = nullptr;
    ObjectShaderData osd_{};
    GlobalShaderData gsd_{};
    bool has_osd_ = false, has_gsd_ = false;
};

}  // namespace vr
