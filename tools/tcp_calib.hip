// tcp_calib.hip -- calibrate the L1 (TCP) lookup / TA cost of gather
// patterns on gfx950, for the layout choice of DESIGN.md sec. 4.
// Each kernel issues ITER loads per lane with one addressing pattern.  Run
// under rocprofv3 --pmc TCP_TOTAL_CACHE_ACCESSES_sum TA_TA_BUSY_sum
// --kernel-trace and divide by (waves * ITER).
//   hipcc --offload-arch=gfx950 -O3 tools/tcp_calib.hip -o tools/tcp_calib
#include <hip/hip_runtime.h>
#include <cstdio>

constexpr int ITER = 64;

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
        else off = base + (lane & 7) * 128 + (lane >> 3) * sizeof(T);            // 8 lines, lanes interleaved
        T v;
        __builtin_memcpy(&v, buf + off, sizeof(T));
        acc += (unsigned)v;
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
    }
    if (hipDeviceSynchronize() != hipSuccess) return 2;
    std::printf("tcp_calib done: 1024 blocks x 4 waves x %d loads per pattern\n", ITER);
    return 0;
}
