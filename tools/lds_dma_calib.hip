// lds_dma_calib.hip -- what an LDS-DMA fill (buffer_load_dwordx4 ... lds) costs
// the vector-memory pipe on gfx950, for the slab march of DESIGN.md sec. 5.1.2.
// Each kernel issues ITER 16-B-per-lane loads per wave with one pattern:
//   k_dma<ACTIVE, SPREAD>: LDS-DMA, the first ACTIVE lanes active, each quad of
//       lanes 64 contiguous bytes; SPREAD = 0: the quads contiguous (1 KiB),
//       1: every quad in its own 128-B line (a column stride of 16448 B, as
//       the COL48 layout's columns at 512^3)
//   k_reg<ACTIVE, SPREAD>: the same addresses, loaded into VGPRs
//   k_b64: the shipped march's access (one dword-aligned 8-B load per lane,
//       quads of lanes mostly in one line)
// Run under rocprofv3 --pmc TA_TA_BUSY_sum / TD_TD_BUSY_sum /
// TCP_TOTAL_CACHE_ACCESSES_sum and --kernel-trace; divide by waves x ITER.
//   hipcc --offload-arch=gfx950 -O3 tools/lds_dma_calib.hip -o tools/lds_dma_calib
#include <hip/hip_runtime.h>
#include <cstdio>

constexpr int ITER = 64;
constexpr unsigned kColStride = 16448;   // COL48 column bytes at 512^3 (32 x 514)
constexpr unsigned kWindow = 64u << 20;  // bytes the bases walk over

__device__ __forceinline__ unsigned base_of(unsigned wave, int it)
{
    return ((wave * 131u + (unsigned)it * 7919u) & 0x7ffu) * 16384u;   // inside kWindow - 1 MiB
}
__device__ __forceinline__ unsigned off_of(int lane, int spread)
{
    return spread ? (unsigned)(lane >> 2) * kColStride + (unsigned)(lane & 3) * 16u : (unsigned)lane * 16u;
}

template <int ACTIVE, int SPREAD>
__global__ __launch_bounds__(256) void k_dma(const unsigned char* __restrict__ buf, unsigned* __restrict__ out)
{
    __shared__ __attribute__((aligned(16))) unsigned char slab[4][2048];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const unsigned wave = blockIdx.x * 4u + (unsigned)w;
    const auto rsrc = __builtin_amdgcn_make_buffer_rsrc((void*)buf, (short)0, (int)kWindow, 0x00020000);
    for (int it = 0; it < ITER; ++it) {
        if (lane < ACTIVE)
            __builtin_amdgcn_raw_ptr_buffer_load_lds(rsrc, (__attribute__((address_space(3))) void*)&slab[w][(it & 1) * 1024],
                                                     16, off_of(lane, SPREAD), base_of(wave, it), 0, 0);
    }
    __builtin_amdgcn_s_waitcnt(0);
    out[blockIdx.x * 256 + threadIdx.x] = slab[w][lane * 16];
}

template <int ACTIVE, int SPREAD>
__global__ __launch_bounds__(256) void k_reg(const unsigned char* __restrict__ buf, unsigned* __restrict__ out)
{
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const unsigned wave = blockIdx.x * 4u + (unsigned)w;
    const auto rsrc = __builtin_amdgcn_make_buffer_rsrc((void*)buf, (short)0, (int)kWindow, 0x00020000);
    unsigned acc = 0;
    for (int it = 0; it < ITER; ++it) {
        if (lane < ACTIVE) {
            const auto v = __builtin_amdgcn_raw_buffer_load_b128(rsrc, off_of(lane, SPREAD), base_of(wave, it), 0);
            acc += v[0] ^ v[1] ^ v[2] ^ v[3];
        }
    }
    out[blockIdx.x * 256 + threadIdx.x] = acc;
}

// CORNERH's tap load at config 4 (4K x 256 at 128^3): the four lanes of a
// 2x2 quad read the same 16 B, neighbouring quads neighbouring 16-B pieces.
// LEAD = 1: only the quad leaders load (the quad-dedup idea of verdict r02
// #5), the other lanes are masked off.
template <int LEAD>
__global__ __launch_bounds__(256) void k_quad(const unsigned char* __restrict__ buf, unsigned* __restrict__ out)
{
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const unsigned wave = blockIdx.x * 4u + (unsigned)w;
    const auto rsrc = __builtin_amdgcn_make_buffer_rsrc((void*)buf, (short)0, (int)kWindow, 0x00020000);
    unsigned acc = 0;
    for (int it = 0; it < ITER; ++it) {
        if (!LEAD || (lane & 3) == 0) {
            const auto v = __builtin_amdgcn_raw_buffer_load_b128(rsrc, (unsigned)(lane >> 2) * 16u, base_of(wave, it), 0);
            acc += v[0] ^ v[1] ^ v[2] ^ v[3];
        }
    }
    out[blockIdx.x * 256 + threadIdx.x] = acc;
}

// the shipped march's b64 tap load: lanes of a 2x2 pixel quad 0-1 texels
// apart inside 4x8x32 bricks (brick4832), quads of a tile 2 texels apart
__global__ __launch_bounds__(256) void k_b64(const unsigned char* __restrict__ buf, unsigned* __restrict__ out)
{
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const unsigned wave = blockIdx.x * 4u + (unsigned)w;
    const auto rsrc = __builtin_amdgcn_make_buffer_rsrc((void*)buf, (short)0, (int)kWindow, 0x00020000);
    unsigned acc = 0;
    const int qx = (lane >> 2) & 3, qy = lane >> 4;
    const int a = 2 * qx + (lane & 1), b = 2 * qy + ((lane >> 1) & 1);
    for (int it = 0; it < ITER; ++it) {
        const unsigned o = (unsigned)(a / 3) * 1024u + (unsigned)(b / 7) * 1024u * 171u + (unsigned)(a % 3) +
                           (unsigned)(b % 7) * 4u + (unsigned)(it & 15) * 32u;
        const auto v = __builtin_amdgcn_raw_buffer_load_b64(rsrc, o & ~3u, base_of(wave, it), 0);
        acc += v[0] ^ v[1];
    }
    out[blockIdx.x * 256 + threadIdx.x] = acc;
}

int main()
{
    unsigned char* buf;
    unsigned* out;
    if (hipMalloc(&buf, kWindow) != hipSuccess || hipMalloc(&out, 2048 * 256 * 4) != hipSuccess) return 1;
    (void)hipMemset(buf, 1, kWindow);
    const dim3 g(2048), b(256);
#define DMA(A, S) hipLaunchKernelGGL((k_dma<A, S>), g, b, 0, 0, buf, out)
#define REG(A, S) hipLaunchKernelGGL((k_reg<A, S>), g, b, 0, 0, buf, out)
    for (int rep = 0; rep < 3; ++rep) {
        DMA(64, 0); DMA(64, 1); DMA(32, 1); DMA(24, 1); DMA(16, 1); DMA(8, 1); DMA(4, 1);
        REG(64, 0); REG(64, 1); REG(24, 1); REG(8, 1);
        hipLaunchKernelGGL(k_b64, g, b, 0, 0, buf, out);
        hipLaunchKernelGGL(k_quad<0>, g, b, 0, 0, buf, out);
        hipLaunchKernelGGL(k_quad<1>, g, b, 0, 0, buf, out);
    }
    if (hipDeviceSynchronize() != hipSuccess) return 2;
    std::printf("lds_dma_calib done: %u blocks x 4 waves x %d loads per kernel\n", g.x, ITER);
    return 0;
}
