// tcp_calib.hip -- calibrate the L1 (TCP) lookup / TA cost of gather
// patterns on gfx950, for the layout choice of DESIGN.md sec. 4.
// Each kernel issues ITER loads per lane with one addressing pattern.  Run
// under rocprofv3 --pmc TCP_TOTAL_CACHE_ACCESSES_sum TA_TA_BUSY_sum
// --kernel-trace and divide by (waves * ITER).
//   hipcc --offload-arch=gfx950 -O3 tools/tcp_calib.hip -o tools/tcp_calib
#include <hip/hip_runtime.h>
#include <cstdio>

constexpr int ITER = 64;

struct B12 { unsigned a, b, c; };
struct alignas(16) B16 { unsigned a, b, c, d; };
__device__ __forceinline__ unsigned fold(unsigned short v) { return v; }
__device__ __forceinline__ unsigned fold(unsigned v) { return v; }
__device__ __forceinline__ unsigned fold(unsigned long long v) { return (unsigned)v ^ (unsigned)(v >> 32); }
__device__ __forceinline__ unsigned fold(B12 v) { return v.a ^ v.b ^ v.c; }
__device__ __forceinline__ unsigned fold(B16 v) { return v.a ^ v.b ^ v.c ^ v.d; }

// Wide (12/16-byte) loads at dword-aligned offsets.
template <int PATTERN, typename T>
__global__ void k_wide(const unsigned char* __restrict__ buf, unsigned* __restrict__ out)
{
    const int lane = threadIdx.x & 63;
    const unsigned wave = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
    unsigned acc = 0;
    for (int it = 0; it < ITER; ++it) {
        const unsigned base = ((wave * 131u + it * 7919u) & 0xfffu) * 4096u;
        unsigned off;
        if constexpr (PATTERN == 0) off = base + lane * sizeof(T);                         // contiguous
        else if constexpr (PATTERN == 1) off = base + (lane >> 4) * 128 + (lane & 15) * 4;  // a line per 16 lanes
        else if constexpr (PATTERN == 2) off = base + (lane >> 2) * 128 + (lane & 3) * 20;  // a line per 4 lanes
        else off = base + (lane >> 4) * 256 + (lane & 15) * 4 + (lane & 1) * 64;            // 16 lanes over 2 lines
        const T v = *reinterpret_cast<const T*>(buf + off);
        acc += fold(v);
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = acc;
}

template <int PATTERN, typename T>
__global__ void k_pattern(const unsigned char* __restrict__ buf, unsigned* __restrict__ out)
{
    const int lane = threadIdx.x & 63;
    const unsigned wave = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
    unsigned acc = 0;
    for (int it = 0; it < ITER; ++it) {
        const unsigned base = ((wave * 131u + it * 7919u) & 0xfffu) * 4096u;   // 16 MiB window
        unsigned off;
        if constexpr (PATTERN == 0) off = base;                                  // all lanes same address
        else if constexpr (PATTERN == 1) off = base + lane * sizeof(T);          // contiguous
        else if constexpr (PATTERN == 2) off = base + lane * 128;                // one line per lane
        else if constexpr (PATTERN == 3) off = base + (lane >> 2) * 128;         // one line per quad
        else if constexpr (PATTERN == 4) off = base + (lane & 3) * 128;          // 4 lines, each shared by 16 lanes (stride 4)
        else if constexpr (PATTERN == 5) off = base + (lane >> 4) * 128;         // 4 lines, 16 consecutive lanes each
        else if constexpr (PATTERN == 6) off = base + lane * sizeof(T) + 1;      // contiguous, misaligned by 1
        else if constexpr (PATTERN == 7) off = base + (lane >> 3) * 128 + (lane & 7) * sizeof(T);  // 8 lines x 8 lanes
        else if constexpr (PATTERN == 8) off = base + (lane & 7) * 128 + (lane >> 3) * sizeof(T);  // 8 lines, lanes interleaved
        else if constexpr (PATTERN == 9) off = base + lane * 8 + 1;             // contiguous 8-B slots, misaligned by 1
        else if constexpr (PATTERN == 10) off = base + lane * 8 + 4;            // contiguous 8-B slots, dword aligned
        else if constexpr (PATTERN == 11) off = base + (lane * 7) % 120;        // all lanes in one line, misaligned
        else if constexpr (PATTERN == 12) off = base + (lane >> 2) * 128 + (lane & 3) * 29;  // a line per 4 lanes, misaligned
        else if constexpr (PATTERN == 13) off = base + (lane >> 2) * 128 + (lane & 3) * 24;  // a line per 4 lanes, aligned
        else if constexpr (PATTERN == 14) off = base + (lane >> 4) * 128 + (lane & 15) * 7;  // a line per 16 lanes, misaligned
        else off = base + (lane >> 4) * 128 + (lane & 15) * 8;                  // a line per 16 lanes, aligned
        T v;
        __builtin_memcpy(&v, buf + off, sizeof(T));
        acc += fold(v);   // use every loaded byte
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = acc;
}

int main()
{
    unsigned char* buf;
    unsigned* out;
    const size_t bytes = 16u << 20;
    if (hipMalloc(&buf, bytes + 8192) != hipSuccess || hipMalloc(&out, 1024 * 256 * 4) != hipSuccess) return 1;
    (void)hipMemset(buf, 1, bytes + 8192);
    dim3 g(1024), b(256);
#define RUN(P, T) hipLaunchKernelGGL((k_pattern<P, T>), g, b, 0, 0, buf, out)
    for (int rep = 0; rep < 3; ++rep) {
        RUN(0, unsigned short); RUN(1, unsigned short); RUN(2, unsigned short); RUN(3, unsigned short);
        RUN(4, unsigned short); RUN(5, unsigned short); RUN(6, unsigned short); RUN(7, unsigned short);
        RUN(8, unsigned short);
        RUN(0, unsigned); RUN(1, unsigned); RUN(2, unsigned); RUN(3, unsigned); RUN(6, unsigned);
        RUN(0, unsigned long long); RUN(1, unsigned long long); RUN(2, unsigned long long);
        RUN(3, unsigned long long); RUN(7, unsigned long long); RUN(8, unsigned long long);
        RUN(9, unsigned long long); RUN(10, unsigned long long); RUN(11, unsigned long long);
        RUN(12, unsigned long long); RUN(13, unsigned long long); RUN(14, unsigned long long);
        RUN(15, unsigned long long);
#define RUNW(P, T) hipLaunchKernelGGL((k_wide<P, T>), g, b, 0, 0, buf, out)
        RUNW(0, B12); RUNW(1, B12); RUNW(2, B12); RUNW(3, B12);
        RUNW(0, B16); RUNW(1, B16); RUNW(2, B16); RUNW(3, B16);
        RUNW(1, unsigned long long); RUNW(2, unsigned long long); RUNW(3, unsigned long long);
    }
    if (hipDeviceSynchronize() != hipSuccess) return 2;
    std::printf("tcp_calib done: 1024 blocks x 4 waves x %d loads per pattern\n", ITER);
    return 0;
}
