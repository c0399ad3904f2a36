// valu_calib.hip -- issue throughput of single VALU opcodes on gfx950, the cost
// table behind the procedural kernel's instruction budget.
// Each kernel runs ITER x 16 independent instances of one opcode per lane
// (16 accumulators, so no dependent-latency stalls), at W waves per SIMD.
// The shader clock is measured in-kernel (s_memtime against the 100 MHz
// s_memrealtime), so the result is SIMD cycles per wave64 instruction.
//   hipcc --offload-arch=gfx950 -O3 tools/valu_calib.hip -o tools/valu_calib
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

constexpr int ITER = 4096;

#define R16(M) M(0) M(1) M(2) M(3) M(4) M(5) M(6) M(7) M(8) M(9) M(10) M(11) M(12) M(13) M(14) M(15)

template <int OP>
__device__ __forceinline__ void body(float (&f)[16], unsigned (&u)[16], float s)
{
#define FMA(i) asm volatile("v_fma_f32 %0, %0, %1, %1" : "+v"(f[i]) : "v"(s));
#define MUL(i) asm volatile("v_mul_f32 %0, %0, %1" : "+v"(f[i]) : "v"(s));
#define MULLO(i) asm volatile("v_mul_lo_u32 %0, %0, %1" : "+v"(u[i]) : "v"(u[(i + 1) & 15]));
#define XOR(i) asm volatile("v_xor_b32 %0, %0, %1" : "+v"(u[i]) : "v"(u[(i + 3) & 15]));
#define CVT(i) asm volatile("v_cvt_i32_f32 %0, %1" : "=v"(u[i]) : "v"(f[i]));
#define FLOOR(i) asm volatile("v_floor_f32 %0, %0" : "+v"(f[i]));
#define EXP(i) asm volatile("v_exp_f32 %0, %0" : "+v"(f[i]));
#define MIN3(i) asm volatile("v_min3_f32 %0, %0, %1, %1" : "+v"(f[i]) : "v"(s));
#define FMAMIX(i) asm volatile("v_fma_f32 %0, %0, %1, %1\n\tv_mul_lo_u32 %2, %2, %3" : "+v"(f[i]), "+v"(u[i]) : "v"(s), "v"(u[(i + 1) & 15]));
#define FMA3(i) asm volatile("v_fma_f32 %0, %1, %2, %0" : "+v"(f[i]) : "v"(f[(i + 5) & 15]), "v"(s));
#define FMAC(i) asm volatile("v_fmac_f32 %0, %1, %2" : "+v"(f[i]) : "v"(f[(i + 5) & 15]), "v"(s));
#define ADD(i) asm volatile("v_add_f32 %0, %0, %1" : "+v"(f[i]) : "v"(f[(i + 5) & 15]));
#define CND(i) asm volatile("v_cndmask_b32 %0, %0, %1, vcc" : "+v"(u[i]) : "v"(u[(i + 5) & 15]));
#define U24(i) asm volatile("v_mul_u32_u24 %0, %0, %1" : "+v"(u[i]) : "v"(u[(i + 1) & 15]));
#define MAD24(i) asm volatile("v_mad_u32_u24 %0, %0, %1, %2" : "+v"(u[i]) : "v"(u[(i + 1) & 15]), "v"(u[(i + 2) & 15]));
#define LSHLADD(i) asm volatile("v_lshl_add_u32 %0, %0, 3, %1" : "+v"(u[i]) : "v"(u[(i + 1) & 15]));
#define MOV(i) asm volatile("v_mov_b32 %0, %1" : "=v"(u[i]) : "v"(u[(i + 1) & 15]));
#define MULHI(i) asm volatile("v_mul_hi_u32 %0, %0, %1" : "+v"(u[i]) : "v"(u[(i + 1) & 15]));
#define CVTF(i) asm volatile("v_cvt_f32_i32 %0, %1" : "=v"(f[i]) : "v"(u[i]));
#define FRACT(i) asm volatile("v_fract_f32 %0, %0" : "+v"(f[i]));
    if constexpr (OP == 10) { R16(FMA3) }
    if constexpr (OP == 11) { R16(FMAC) }
    if constexpr (OP == 12) { R16(ADD) }
    if constexpr (OP == 13) { R16(CND) }
    if constexpr (OP == 14) { R16(U24) }
    if constexpr (OP == 15) { R16(MAD24) }
    if constexpr (OP == 16) { R16(LSHLADD) }
    if constexpr (OP == 17) { R16(MOV) }
    if constexpr (OP == 18) { R16(MULHI) }
    if constexpr (OP == 19) { R16(CVTF) }
    if constexpr (OP == 20) { R16(FRACT) }
    if constexpr (OP == 21 || OP == 22 || OP == 23) {
        for (int i = 0; i < 16; i += 2) {
            float2 v = make_float2(f[i], f[i + 1]);
            const float2 w = make_float2(f[(i + 4) & 15], f[(i + 5) & 15]);
            if constexpr (OP == 21) asm volatile("v_pk_mul_f32 %0, %0, %1" : "+v"(v) : "v"(w));
            if constexpr (OP == 22) asm volatile("v_pk_add_f32 %0, %0, %1" : "+v"(v) : "v"(w));
            if constexpr (OP == 23) asm volatile("v_pk_fma_f32 %0, %1, %0, %0" : "+v"(v) : "v"(w));
            f[i] = v.x; f[i + 1] = v.y;
        }
    }
    if constexpr (OP == 24) asm volatile("v_fma_f32 v64, v1, v2, v3\n\tv_fma_f32 v65, v1, v2, v3\n\tv_fma_f32 v66, v1, v2, v3\n\tv_fma_f32 v67, v1, v2, v3\n\tv_fma_f32 v68, v1, v2, v3\n\tv_fma_f32 v69, v1, v2, v3\n\tv_fma_f32 v70, v1, v2, v3\n\tv_fma_f32 v71, v1, v2, v3\n\tv_fma_f32 v72, v1, v2, v3\n\tv_fma_f32 v73, v1, v2, v3\n\tv_fma_f32 v74, v1, v2, v3\n\tv_fma_f32 v75, v1, v2, v3\n\tv_fma_f32 v76, v1, v2, v3\n\tv_fma_f32 v77, v1, v2, v3\n\tv_fma_f32 v78, v1, v2, v3\n\tv_fma_f32 v79, v1, v2, v3" ::: "v64","v65","v66","v67","v68","v69","v70","v71","v72","v73","v74","v75","v76","v77","v78","v79", "v1","v2","v3","v4","v5","v6","v8","v12","v13");
    if constexpr (OP == 25) asm volatile("v_fma_f32 v64, v4, v8, v12\n\tv_fma_f32 v65, v4, v8, v12\n\tv_fma_f32 v66, v4, v8, v12\n\tv_fma_f32 v67, v4, v8, v12\n\tv_fma_f32 v68, v4, v8, v12\n\tv_fma_f32 v69, v4, v8, v12\n\tv_fma_f32 v70, v4, v8, v12\n\tv_fma_f32 v71, v4, v8, v12\n\tv_fma_f32 v72, v4, v8, v12\n\tv_fma_f32 v73, v4, v8, v12\n\tv_fma_f32 v74, v4, v8, v12\n\tv_fma_f32 v75, v4, v8, v12\n\tv_fma_f32 v76, v4, v8, v12\n\tv_fma_f32 v77, v4, v8, v12\n\tv_fma_f32 v78, v4, v8, v12\n\tv_fma_f32 v79, v4, v8, v12" ::: "v64","v65","v66","v67","v68","v69","v70","v71","v72","v73","v74","v75","v76","v77","v78","v79", "v1","v2","v3","v4","v5","v6","v8","v12","v13");
    if constexpr (OP == 26) asm volatile("v_fma_f32 v64, v5, v5, v6\n\tv_fma_f32 v65, v5, v5, v6\n\tv_fma_f32 v66, v5, v5, v6\n\tv_fma_f32 v67, v5, v5, v6\n\tv_fma_f32 v68, v5, v5, v6\n\tv_fma_f32 v69, v5, v5, v6\n\tv_fma_f32 v70, v5, v5, v6\n\tv_fma_f32 v71, v5, v5, v6\n\tv_fma_f32 v72, v5, v5, v6\n\tv_fma_f32 v73, v5, v5, v6\n\tv_fma_f32 v74, v5, v5, v6\n\tv_fma_f32 v75, v5, v5, v6\n\tv_fma_f32 v76, v5, v5, v6\n\tv_fma_f32 v77, v5, v5, v6\n\tv_fma_f32 v78, v5, v5, v6\n\tv_fma_f32 v79, v5, v5, v6" ::: "v64","v65","v66","v67","v68","v69","v70","v71","v72","v73","v74","v75","v76","v77","v78","v79", "v1","v2","v3","v4","v5","v6","v8","v12","v13");
    if constexpr (OP == 27) asm volatile("v_mul_f32 v64, v5, v5\n\tv_mul_f32 v65, v5, v5\n\tv_mul_f32 v66, v5, v5\n\tv_mul_f32 v67, v5, v5\n\tv_mul_f32 v68, v5, v5\n\tv_mul_f32 v69, v5, v5\n\tv_mul_f32 v70, v5, v5\n\tv_mul_f32 v71, v5, v5\n\tv_mul_f32 v72, v5, v5\n\tv_mul_f32 v73, v5, v5\n\tv_mul_f32 v74, v5, v5\n\tv_mul_f32 v75, v5, v5\n\tv_mul_f32 v76, v5, v5\n\tv_mul_f32 v77, v5, v5\n\tv_mul_f32 v78, v5, v5\n\tv_mul_f32 v79, v5, v5" ::: "v64","v65","v66","v67","v68","v69","v70","v71","v72","v73","v74","v75","v76","v77","v78","v79", "v1","v2","v3","v4","v5","v6","v8","v12","v13");
    if constexpr (OP == 28) asm volatile("v_mul_f32 v64, v4, v8\n\tv_mul_f32 v65, v4, v8\n\tv_mul_f32 v66, v4, v8\n\tv_mul_f32 v67, v4, v8\n\tv_mul_f32 v68, v4, v8\n\tv_mul_f32 v69, v4, v8\n\tv_mul_f32 v70, v4, v8\n\tv_mul_f32 v71, v4, v8\n\tv_mul_f32 v72, v4, v8\n\tv_mul_f32 v73, v4, v8\n\tv_mul_f32 v74, v4, v8\n\tv_mul_f32 v75, v4, v8\n\tv_mul_f32 v76, v4, v8\n\tv_mul_f32 v77, v4, v8\n\tv_mul_f32 v78, v4, v8\n\tv_mul_f32 v79, v4, v8" ::: "v64","v65","v66","v67","v68","v69","v70","v71","v72","v73","v74","v75","v76","v77","v78","v79", "v1","v2","v3","v4","v5","v6","v8","v12","v13");
    if constexpr (OP == 29) asm volatile("v_mul_f32 v64, v5, v6\n\tv_mul_f32 v65, v5, v6\n\tv_mul_f32 v66, v5, v6\n\tv_mul_f32 v67, v5, v6\n\tv_mul_f32 v68, v5, v6\n\tv_mul_f32 v69, v5, v6\n\tv_mul_f32 v70, v5, v6\n\tv_mul_f32 v71, v5, v6\n\tv_mul_f32 v72, v5, v6\n\tv_mul_f32 v73, v5, v6\n\tv_mul_f32 v74, v5, v6\n\tv_mul_f32 v75, v5, v6\n\tv_mul_f32 v76, v5, v6\n\tv_mul_f32 v77, v5, v6\n\tv_mul_f32 v78, v5, v6\n\tv_mul_f32 v79, v5, v6" ::: "v64","v65","v66","v67","v68","v69","v70","v71","v72","v73","v74","v75","v76","v77","v78","v79", "v1","v2","v3","v4","v5","v6","v8","v12","v13");
    if constexpr (OP == 30) asm volatile("v_fma_f32 v64, v4, v8, v13\n\tv_fma_f32 v65, v4, v8, v13\n\tv_fma_f32 v66, v4, v8, v13\n\tv_fma_f32 v67, v4, v8, v13\n\tv_fma_f32 v68, v4, v8, v13\n\tv_fma_f32 v69, v4, v8, v13\n\tv_fma_f32 v70, v4, v8, v13\n\tv_fma_f32 v71, v4, v8, v13\n\tv_fma_f32 v72, v4, v8, v13\n\tv_fma_f32 v73, v4, v8, v13\n\tv_fma_f32 v74, v4, v8, v13\n\tv_fma_f32 v75, v4, v8, v13\n\tv_fma_f32 v76, v4, v8, v13\n\tv_fma_f32 v77, v4, v8, v13\n\tv_fma_f32 v78, v4, v8, v13\n\tv_fma_f32 v79, v4, v8, v13" ::: "v64","v65","v66","v67","v68","v69","v70","v71","v72","v73","v74","v75","v76","v77","v78","v79", "v1","v2","v3","v4","v5","v6","v8","v12","v13");
    if constexpr (OP == 31) asm volatile("v_fma_f32 v64, v64, v2, v3\n\tv_fma_f32 v65, v65, v2, v3\n\tv_fma_f32 v66, v66, v2, v3\n\tv_fma_f32 v67, v67, v2, v3\n\tv_fma_f32 v68, v68, v2, v3\n\tv_fma_f32 v69, v69, v2, v3\n\tv_fma_f32 v70, v70, v2, v3\n\tv_fma_f32 v71, v71, v2, v3\n\tv_fma_f32 v72, v72, v2, v3\n\tv_fma_f32 v73, v73, v2, v3\n\tv_fma_f32 v74, v74, v2, v3\n\tv_fma_f32 v75, v75, v2, v3\n\tv_fma_f32 v76, v76, v2, v3\n\tv_fma_f32 v77, v77, v2, v3\n\tv_fma_f32 v78, v78, v2, v3\n\tv_fma_f32 v79, v79, v2, v3" ::: "v64","v65","v66","v67","v68","v69","v70","v71","v72","v73","v74","v75","v76","v77","v78","v79", "v1","v2","v3","v4","v5","v6","v8","v12","v13");
    if constexpr (OP == 32) asm volatile("v_fma_f32 v64, v5, v6, v6\n\tv_fma_f32 v65, v5, v6, v6\n\tv_fma_f32 v66, v5, v6, v6\n\tv_fma_f32 v67, v5, v6, v6\n\tv_fma_f32 v68, v5, v6, v6\n\tv_fma_f32 v69, v5, v6, v6\n\tv_fma_f32 v70, v5, v6, v6\n\tv_fma_f32 v71, v5, v6, v6\n\tv_fma_f32 v72, v5, v6, v6\n\tv_fma_f32 v73, v5, v6, v6\n\tv_fma_f32 v74, v5, v6, v6\n\tv_fma_f32 v75, v5, v6, v6\n\tv_fma_f32 v76, v5, v6, v6\n\tv_fma_f32 v77, v5, v6, v6\n\tv_fma_f32 v78, v5, v6, v6\n\tv_fma_f32 v79, v5, v6, v6" ::: "v64","v65","v66","v67","v68","v69","v70","v71","v72","v73","v74","v75","v76","v77","v78","v79", "v1","v2","v3","v4","v5","v6","v7","s40","s41","vcc");
    if constexpr (OP == 33) asm volatile("v_min3_f32 v64, v1, v2, v3\n\tv_min3_f32 v65, v1, v2, v3\n\tv_min3_f32 v66, v1, v2, v3\n\tv_min3_f32 v67, v1, v2, v3\n\tv_min3_f32 v68, v1, v2, v3\n\tv_min3_f32 v69, v1, v2, v3\n\tv_min3_f32 v70, v1, v2, v3\n\tv_min3_f32 v71, v1, v2, v3\n\tv_min3_f32 v72, v1, v2, v3\n\tv_min3_f32 v73, v1, v2, v3\n\tv_min3_f32 v74, v1, v2, v3\n\tv_min3_f32 v75, v1, v2, v3\n\tv_min3_f32 v76, v1, v2, v3\n\tv_min3_f32 v77, v1, v2, v3\n\tv_min3_f32 v78, v1, v2, v3\n\tv_min3_f32 v79, v1, v2, v3" ::: "v64","v65","v66","v67","v68","v69","v70","v71","v72","v73","v74","v75","v76","v77","v78","v79", "v1","v2","v3","v4","v5","v6","v7","s40","s41","vcc");
    if constexpr (OP == 34) asm volatile("v_bitop3_b32 v64, v1, v2, v3 bitop3:0x48\n\tv_bitop3_b32 v65, v1, v2, v3 bitop3:0x48\n\tv_bitop3_b32 v66, v1, v2, v3 bitop3:0x48\n\tv_bitop3_b32 v67, v1, v2, v3 bitop3:0x48\n\tv_bitop3_b32 v68, v1, v2, v3 bitop3:0x48\n\tv_bitop3_b32 v69, v1, v2, v3 bitop3:0x48\n\tv_bitop3_b32 v70, v1, v2, v3 bitop3:0x48\n\tv_bitop3_b32 v71, v1, v2, v3 bitop3:0x48\n\tv_bitop3_b32 v72, v1, v2, v3 bitop3:0x48\n\tv_bitop3_b32 v73, v1, v2, v3 bitop3:0x48\n\tv_bitop3_b32 v74, v1, v2, v3 bitop3:0x48\n\tv_bitop3_b32 v75, v1, v2, v3 bitop3:0x48\n\tv_bitop3_b32 v76, v1, v2, v3 bitop3:0x48\n\tv_bitop3_b32 v77, v1, v2, v3 bitop3:0x48\n\tv_bitop3_b32 v78, v1, v2, v3 bitop3:0x48\n\tv_bitop3_b32 v79, v1, v2, v3 bitop3:0x48" ::: "v64","v65","v66","v67","v68","v69","v70","v71","v72","v73","v74","v75","v76","v77","v78","v79", "v1","v2","v3","v4","v5","v6","v7","s40","s41","vcc");
    if constexpr (OP == 35) asm volatile("v_and_or_b32 v64, v1, v2, v3\n\tv_and_or_b32 v65, v1, v2, v3\n\tv_and_or_b32 v66, v1, v2, v3\n\tv_and_or_b32 v67, v1, v2, v3\n\tv_and_or_b32 v68, v1, v2, v3\n\tv_and_or_b32 v69, v1, v2, v3\n\tv_and_or_b32 v70, v1, v2, v3\n\tv_and_or_b32 v71, v1, v2, v3\n\tv_and_or_b32 v72, v1, v2, v3\n\tv_and_or_b32 v73, v1, v2, v3\n\tv_and_or_b32 v74, v1, v2, v3\n\tv_and_or_b32 v75, v1, v2, v3\n\tv_and_or_b32 v76, v1, v2, v3\n\tv_and_or_b32 v77, v1, v2, v3\n\tv_and_or_b32 v78, v1, v2, v3\n\tv_and_or_b32 v79, v1, v2, v3" ::: "v64","v65","v66","v67","v68","v69","v70","v71","v72","v73","v74","v75","v76","v77","v78","v79", "v1","v2","v3","v4","v5","v6","v7","s40","s41","vcc");
    if constexpr (OP == 36) asm volatile("v_add3_u32 v64, v1, v2, v3\n\tv_add3_u32 v65, v1, v2, v3\n\tv_add3_u32 v66, v1, v2, v3\n\tv_add3_u32 v67, v1, v2, v3\n\tv_add3_u32 v68, v1, v2, v3\n\tv_add3_u32 v69, v1, v2, v3\n\tv_add3_u32 v70, v1, v2, v3\n\tv_add3_u32 v71, v1, v2, v3\n\tv_add3_u32 v72, v1, v2, v3\n\tv_add3_u32 v73, v1, v2, v3\n\tv_add3_u32 v74, v1, v2, v3\n\tv_add3_u32 v75, v1, v2, v3\n\tv_add3_u32 v76, v1, v2, v3\n\tv_add3_u32 v77, v1, v2, v3\n\tv_add3_u32 v78, v1, v2, v3\n\tv_add3_u32 v79, v1, v2, v3" ::: "v64","v65","v66","v67","v68","v69","v70","v71","v72","v73","v74","v75","v76","v77","v78","v79", "v1","v2","v3","v4","v5","v6","v7","s40","s41","vcc");
    if constexpr (OP == 37) asm volatile("v_lshl_or_b32 v64, v1, 4, v3\n\tv_lshl_or_b32 v65, v1, 4, v3\n\tv_lshl_or_b32 v66, v1, 4, v3\n\tv_lshl_or_b32 v67, v1, 4, v3\n\tv_lshl_or_b32 v68, v1, 4, v3\n\tv_lshl_or_b32 v69, v1, 4, v3\n\tv_lshl_or_b32 v70, v1, 4, v3\n\tv_lshl_or_b32 v71, v1, 4, v3\n\tv_lshl_or_b32 v72, v1, 4, v3\n\tv_lshl_or_b32 v73, v1, 4, v3\n\tv_lshl_or_b32 v74, v1, 4, v3\n\tv_lshl_or_b32 v75, v1, 4, v3\n\tv_lshl_or_b32 v76, v1, 4, v3\n\tv_lshl_or_b32 v77, v1, 4, v3\n\tv_lshl_or_b32 v78, v1, 4, v3\n\tv_lshl_or_b32 v79, v1, 4, v3" ::: "v64","v65","v66","v67","v68","v69","v70","v71","v72","v73","v74","v75","v76","v77","v78","v79", "v1","v2","v3","v4","v5","v6","v7","s40","s41","vcc");
    if constexpr (OP == 38) asm volatile("v_bfe_u32 v64, v1, 15, 4\n\tv_bfe_u32 v65, v1, 15, 4\n\tv_bfe_u32 v66, v1, 15, 4\n\tv_bfe_u32 v67, v1, 15, 4\n\tv_bfe_u32 v68, v1, 15, 4\n\tv_bfe_u32 v69, v1, 15, 4\n\tv_bfe_u32 v70, v1, 15, 4\n\tv_bfe_u32 v71, v1, 15, 4\n\tv_bfe_u32 v72, v1, 15, 4\n\tv_bfe_u32 v73, v1, 15, 4\n\tv_bfe_u32 v74, v1, 15, 4\n\tv_bfe_u32 v75, v1, 15, 4\n\tv_bfe_u32 v76, v1, 15, 4\n\tv_bfe_u32 v77, v1, 15, 4\n\tv_bfe_u32 v78, v1, 15, 4\n\tv_bfe_u32 v79, v1, 15, 4" ::: "v64","v65","v66","v67","v68","v69","v70","v71","v72","v73","v74","v75","v76","v77","v78","v79", "v1","v2","v3","v4","v5","v6","v7","s40","s41","vcc");
    if constexpr (OP == 39) asm volatile("v_alignbyte_b32 v64, v1, v2, v3\n\tv_alignbyte_b32 v65, v1, v2, v3\n\tv_alignbyte_b32 v66, v1, v2, v3\n\tv_alignbyte_b32 v67, v1, v2, v3\n\tv_alignbyte_b32 v68, v1, v2, v3\n\tv_alignbyte_b32 v69, v1, v2, v3\n\tv_alignbyte_b32 v70, v1, v2, v3\n\tv_alignbyte_b32 v71, v1, v2, v3\n\tv_alignbyte_b32 v72, v1, v2, v3\n\tv_alignbyte_b32 v73, v1, v2, v3\n\tv_alignbyte_b32 v74, v1, v2, v3\n\tv_alignbyte_b32 v75, v1, v2, v3\n\tv_alignbyte_b32 v76, v1, v2, v3\n\tv_alignbyte_b32 v77, v1, v2, v3\n\tv_alignbyte_b32 v78, v1, v2, v3\n\tv_alignbyte_b32 v79, v1, v2, v3" ::: "v64","v65","v66","v67","v68","v69","v70","v71","v72","v73","v74","v75","v76","v77","v78","v79", "v1","v2","v3","v4","v5","v6","v7","s40","s41","vcc");
    if constexpr (OP == 40) asm volatile("v_cvt_flr_i32_f32 v64, v1\n\tv_cvt_flr_i32_f32 v65, v1\n\tv_cvt_flr_i32_f32 v66, v1\n\tv_cvt_flr_i32_f32 v67, v1\n\tv_cvt_flr_i32_f32 v68, v1\n\tv_cvt_flr_i32_f32 v69, v1\n\tv_cvt_flr_i32_f32 v70, v1\n\tv_cvt_flr_i32_f32 v71, v1\n\tv_cvt_flr_i32_f32 v72, v1\n\tv_cvt_flr_i32_f32 v73, v1\n\tv_cvt_flr_i32_f32 v74, v1\n\tv_cvt_flr_i32_f32 v75, v1\n\tv_cvt_flr_i32_f32 v76, v1\n\tv_cvt_flr_i32_f32 v77, v1\n\tv_cvt_flr_i32_f32 v78, v1\n\tv_cvt_flr_i32_f32 v79, v1" ::: "v64","v65","v66","v67","v68","v69","v70","v71","v72","v73","v74","v75","v76","v77","v78","v79", "v1","v2","v3","v4","v5","v6","v7","s40","s41","vcc");
    if constexpr (OP == 41) asm volatile("v_cvt_f32_ubyte0 v64, v1\n\tv_cvt_f32_ubyte0 v65, v1\n\tv_cvt_f32_ubyte0 v66, v1\n\tv_cvt_f32_ubyte0 v67, v1\n\tv_cvt_f32_ubyte0 v68, v1\n\tv_cvt_f32_ubyte0 v69, v1\n\tv_cvt_f32_ubyte0 v70, v1\n\tv_cvt_f32_ubyte0 v71, v1\n\tv_cvt_f32_ubyte0 v72, v1\n\tv_cvt_f32_ubyte0 v73, v1\n\tv_cvt_f32_ubyte0 v74, v1\n\tv_cvt_f32_ubyte0 v75, v1\n\tv_cvt_f32_ubyte0 v76, v1\n\tv_cvt_f32_ubyte0 v77, v1\n\tv_cvt_f32_ubyte0 v78, v1\n\tv_cvt_f32_ubyte0 v79, v1" ::: "v64","v65","v66","v67","v68","v69","v70","v71","v72","v73","v74","v75","v76","v77","v78","v79", "v1","v2","v3","v4","v5","v6","v7","s40","s41","vcc");
    if constexpr (OP == 42) asm volatile("v_max_f32 v64, v1, v2\n\tv_max_f32 v65, v1, v2\n\tv_max_f32 v66, v1, v2\n\tv_max_f32 v67, v1, v2\n\tv_max_f32 v68, v1, v2\n\tv_max_f32 v69, v1, v2\n\tv_max_f32 v70, v1, v2\n\tv_max_f32 v71, v1, v2\n\tv_max_f32 v72, v1, v2\n\tv_max_f32 v73, v1, v2\n\tv_max_f32 v74, v1, v2\n\tv_max_f32 v75, v1, v2\n\tv_max_f32 v76, v1, v2\n\tv_max_f32 v77, v1, v2\n\tv_max_f32 v78, v1, v2\n\tv_max_f32 v79, v1, v2" ::: "v64","v65","v66","v67","v68","v69","v70","v71","v72","v73","v74","v75","v76","v77","v78","v79", "v1","v2","v3","v4","v5","v6","v7","s40","s41","vcc");
    if constexpr (OP == 43) asm volatile("v_rndne_f32 v64, v1\n\tv_rndne_f32 v65, v1\n\tv_rndne_f32 v66, v1\n\tv_rndne_f32 v67, v1\n\tv_rndne_f32 v68, v1\n\tv_rndne_f32 v69, v1\n\tv_rndne_f32 v70, v1\n\tv_rndne_f32 v71, v1\n\tv_rndne_f32 v72, v1\n\tv_rndne_f32 v73, v1\n\tv_rndne_f32 v74, v1\n\tv_rndne_f32 v75, v1\n\tv_rndne_f32 v76, v1\n\tv_rndne_f32 v77, v1\n\tv_rndne_f32 v78, v1\n\tv_rndne_f32 v79, v1" ::: "v64","v65","v66","v67","v68","v69","v70","v71","v72","v73","v74","v75","v76","v77","v78","v79", "v1","v2","v3","v4","v5","v6","v7","s40","s41","vcc");
    if constexpr (OP == 44) asm volatile("v_cmp_lt_f32 vcc, v1, v64\n\tv_cmp_lt_f32 vcc, v1, v65\n\tv_cmp_lt_f32 vcc, v1, v66\n\tv_cmp_lt_f32 vcc, v1, v67\n\tv_cmp_lt_f32 vcc, v1, v68\n\tv_cmp_lt_f32 vcc, v1, v69\n\tv_cmp_lt_f32 vcc, v1, v70\n\tv_cmp_lt_f32 vcc, v1, v71\n\tv_cmp_lt_f32 vcc, v1, v72\n\tv_cmp_lt_f32 vcc, v1, v73\n\tv_cmp_lt_f32 vcc, v1, v74\n\tv_cmp_lt_f32 vcc, v1, v75\n\tv_cmp_lt_f32 vcc, v1, v76\n\tv_cmp_lt_f32 vcc, v1, v77\n\tv_cmp_lt_f32 vcc, v1, v78\n\tv_cmp_lt_f32 vcc, v1, v79" ::: "v64","v65","v66","v67","v68","v69","v70","v71","v72","v73","v74","v75","v76","v77","v78","v79", "v1","v2","v3","v4","v5","v6","v7","s40","s41","vcc");
    if constexpr (OP == 45) asm volatile("v_cndmask_b32_e64 v64, v1, v2, s[40:41]\n\tv_cndmask_b32_e64 v65, v1, v2, s[40:41]\n\tv_cndmask_b32_e64 v66, v1, v2, s[40:41]\n\tv_cndmask_b32_e64 v67, v1, v2, s[40:41]\n\tv_cndmask_b32_e64 v68, v1, v2, s[40:41]\n\tv_cndmask_b32_e64 v69, v1, v2, s[40:41]\n\tv_cndmask_b32_e64 v70, v1, v2, s[40:41]\n\tv_cndmask_b32_e64 v71, v1, v2, s[40:41]\n\tv_cndmask_b32_e64 v72, v1, v2, s[40:41]\n\tv_cndmask_b32_e64 v73, v1, v2, s[40:41]\n\tv_cndmask_b32_e64 v74, v1, v2, s[40:41]\n\tv_cndmask_b32_e64 v75, v1, v2, s[40:41]\n\tv_cndmask_b32_e64 v76, v1, v2, s[40:41]\n\tv_cndmask_b32_e64 v77, v1, v2, s[40:41]\n\tv_cndmask_b32_e64 v78, v1, v2, s[40:41]\n\tv_cndmask_b32_e64 v79, v1, v2, s[40:41]" ::: "v64","v65","v66","v67","v68","v69","v70","v71","v72","v73","v74","v75","v76","v77","v78","v79", "v1","v2","v3","v4","v5","v6","v7","s40","s41","vcc");
    if constexpr (OP == 46) asm volatile("v_lshrrev_b32 v64, 15, v1\n\tv_lshrrev_b32 v65, 15, v1\n\tv_lshrrev_b32 v66, 15, v1\n\tv_lshrrev_b32 v67, 15, v1\n\tv_lshrrev_b32 v68, 15, v1\n\tv_lshrrev_b32 v69, 15, v1\n\tv_lshrrev_b32 v70, 15, v1\n\tv_lshrrev_b32 v71, 15, v1\n\tv_lshrrev_b32 v72, 15, v1\n\tv_lshrrev_b32 v73, 15, v1\n\tv_lshrrev_b32 v74, 15, v1\n\tv_lshrrev_b32 v75, 15, v1\n\tv_lshrrev_b32 v76, 15, v1\n\tv_lshrrev_b32 v77, 15, v1\n\tv_lshrrev_b32 v78, 15, v1\n\tv_lshrrev_b32 v79, 15, v1" ::: "v64","v65","v66","v67","v68","v69","v70","v71","v72","v73","v74","v75","v76","v77","v78","v79", "v1","v2","v3","v4","v5","v6","v7","s40","s41","vcc");
    if constexpr (OP == 47) asm volatile("v_add_u32 v64, v1, v2\n\tv_add_u32 v65, v1, v2\n\tv_add_u32 v66, v1, v2\n\tv_add_u32 v67, v1, v2\n\tv_add_u32 v68, v1, v2\n\tv_add_u32 v69, v1, v2\n\tv_add_u32 v70, v1, v2\n\tv_add_u32 v71, v1, v2\n\tv_add_u32 v72, v1, v2\n\tv_add_u32 v73, v1, v2\n\tv_add_u32 v74, v1, v2\n\tv_add_u32 v75, v1, v2\n\tv_add_u32 v76, v1, v2\n\tv_add_u32 v77, v1, v2\n\tv_add_u32 v78, v1, v2\n\tv_add_u32 v79, v1, v2" ::: "v64","v65","v66","v67","v68","v69","v70","v71","v72","v73","v74","v75","v76","v77","v78","v79", "v1","v2","v3","v4","v5","v6","v7","s40","s41","vcc");
    if constexpr (OP == 48) asm volatile("v_fmamk_f32 v64, v1, 0x40c00000, v2\n\tv_fmamk_f32 v65, v1, 0x40c00000, v2\n\tv_fmamk_f32 v66, v1, 0x40c00000, v2\n\tv_fmamk_f32 v67, v1, 0x40c00000, v2\n\tv_fmamk_f32 v68, v1, 0x40c00000, v2\n\tv_fmamk_f32 v69, v1, 0x40c00000, v2\n\tv_fmamk_f32 v70, v1, 0x40c00000, v2\n\tv_fmamk_f32 v71, v1, 0x40c00000, v2\n\tv_fmamk_f32 v72, v1, 0x40c00000, v2\n\tv_fmamk_f32 v73, v1, 0x40c00000, v2\n\tv_fmamk_f32 v74, v1, 0x40c00000, v2\n\tv_fmamk_f32 v75, v1, 0x40c00000, v2\n\tv_fmamk_f32 v76, v1, 0x40c00000, v2\n\tv_fmamk_f32 v77, v1, 0x40c00000, v2\n\tv_fmamk_f32 v78, v1, 0x40c00000, v2\n\tv_fmamk_f32 v79, v1, 0x40c00000, v2" ::: "v64","v65","v66","v67","v68","v69","v70","v71","v72","v73","v74","v75","v76","v77","v78","v79", "v1","v2","v3","v4","v5","v6","v7","s40","s41","vcc");
    if constexpr (OP == 49) asm volatile("v_mul_f32 v64, s40, v1\n\tv_mul_f32 v65, s40, v1\n\tv_mul_f32 v66, s40, v1\n\tv_mul_f32 v67, s40, v1\n\tv_mul_f32 v68, s40, v1\n\tv_mul_f32 v69, s40, v1\n\tv_mul_f32 v70, s40, v1\n\tv_mul_f32 v71, s40, v1\n\tv_mul_f32 v72, s40, v1\n\tv_mul_f32 v73, s40, v1\n\tv_mul_f32 v74, s40, v1\n\tv_mul_f32 v75, s40, v1\n\tv_mul_f32 v76, s40, v1\n\tv_mul_f32 v77, s40, v1\n\tv_mul_f32 v78, s40, v1\n\tv_mul_f32 v79, s40, v1" ::: "v64","v65","v66","v67","v68","v69","v70","v71","v72","v73","v74","v75","v76","v77","v78","v79", "v1","v2","v3","v4","v5","v6","v7","s40","s41","vcc");
    if constexpr (OP == 51) asm volatile("v_pk_fma_f32 v[64:65], v[2:3], v[4:5], v[6:7]\n\tv_pk_fma_f32 v[66:67], v[2:3], v[4:5], v[6:7]\n\tv_pk_fma_f32 v[68:69], v[2:3], v[4:5], v[6:7]\n\tv_pk_fma_f32 v[70:71], v[2:3], v[4:5], v[6:7]\n\tv_pk_fma_f32 v[72:73], v[2:3], v[4:5], v[6:7]\n\tv_pk_fma_f32 v[74:75], v[2:3], v[4:5], v[6:7]\n\tv_pk_fma_f32 v[76:77], v[2:3], v[4:5], v[6:7]\n\tv_pk_fma_f32 v[78:79], v[2:3], v[4:5], v[6:7]" ::: "v64","v65","v66","v67","v68","v69","v70","v71","v72","v73","v74","v75","v76","v77","v78","v79", "v1","v2","v3","v4","v5","v6","v7","s40","s41","vcc");
    if constexpr (OP == 52) asm volatile("v_mul_f32 v64, s40, v1\n\tv_mul_f32 v65, s41, v1\n\tv_mul_f32 v66, s42, v1\n\tv_mul_f32 v67, s43, v1\n\tv_mul_f32 v68, s44, v1\n\tv_mul_f32 v69, s45, v1\n\tv_mul_f32 v70, s46, v1\n\tv_mul_f32 v71, s47, v1\n\tv_mul_f32 v72, s40, v1\n\tv_mul_f32 v73, s41, v1\n\tv_mul_f32 v74, s42, v1\n\tv_mul_f32 v75, s43, v1\n\tv_mul_f32 v76, s44, v1\n\tv_mul_f32 v77, s45, v1\n\tv_mul_f32 v78, s46, v1\n\tv_mul_f32 v79, s47, v1" ::: "v64","v65","v66","v67","v68","v69","v70","v71","v72","v73","v74","v75","v76","v77","v78","v79", "v1","v2","v3","s40","s41","s42","s43","s44","s45","s46","s47","vcc");
    if constexpr (OP == 53) asm volatile("v_add_f32 v64, s40, v1\n\tv_add_f32 v65, s40, v1\n\tv_add_f32 v66, s40, v1\n\tv_add_f32 v67, s40, v1\n\tv_add_f32 v68, s40, v1\n\tv_add_f32 v69, s40, v1\n\tv_add_f32 v70, s40, v1\n\tv_add_f32 v71, s40, v1\n\tv_add_f32 v72, s40, v1\n\tv_add_f32 v73, s40, v1\n\tv_add_f32 v74, s40, v1\n\tv_add_f32 v75, s40, v1\n\tv_add_f32 v76, s40, v1\n\tv_add_f32 v77, s40, v1\n\tv_add_f32 v78, s40, v1\n\tv_add_f32 v79, s40, v1" ::: "v64","v65","v66","v67","v68","v69","v70","v71","v72","v73","v74","v75","v76","v77","v78","v79", "v1","v2","v3","s40","s41","s42","s43","s44","s45","s46","s47","vcc");
    if constexpr (OP == 54) asm volatile("v_xor_b32 v64, s40, v1\n\tv_xor_b32 v65, s40, v1\n\tv_xor_b32 v66, s40, v1\n\tv_xor_b32 v67, s40, v1\n\tv_xor_b32 v68, s40, v1\n\tv_xor_b32 v69, s40, v1\n\tv_xor_b32 v70, s40, v1\n\tv_xor_b32 v71, s40, v1\n\tv_xor_b32 v72, s40, v1\n\tv_xor_b32 v73, s40, v1\n\tv_xor_b32 v74, s40, v1\n\tv_xor_b32 v75, s40, v1\n\tv_xor_b32 v76, s40, v1\n\tv_xor_b32 v77, s40, v1\n\tv_xor_b32 v78, s40, v1\n\tv_xor_b32 v79, s40, v1" ::: "v64","v65","v66","v67","v68","v69","v70","v71","v72","v73","v74","v75","v76","v77","v78","v79", "v1","v2","v3","s40","s41","s42","s43","s44","s45","s46","s47","vcc");
    if constexpr (OP == 55) asm volatile("v_fma_f32 v64, s40, v1, v2\n\tv_fma_f32 v65, s40, v1, v2\n\tv_fma_f32 v66, s40, v1, v2\n\tv_fma_f32 v67, s40, v1, v2\n\tv_fma_f32 v68, s40, v1, v2\n\tv_fma_f32 v69, s40, v1, v2\n\tv_fma_f32 v70, s40, v1, v2\n\tv_fma_f32 v71, s40, v1, v2\n\tv_fma_f32 v72, s40, v1, v2\n\tv_fma_f32 v73, s40, v1, v2\n\tv_fma_f32 v74, s40, v1, v2\n\tv_fma_f32 v75, s40, v1, v2\n\tv_fma_f32 v76, s40, v1, v2\n\tv_fma_f32 v77, s40, v1, v2\n\tv_fma_f32 v78, s40, v1, v2\n\tv_fma_f32 v79, s40, v1, v2" ::: "v64","v65","v66","v67","v68","v69","v70","v71","v72","v73","v74","v75","v76","v77","v78","v79", "v1","v2","v3","s40","s41","s42","s43","s44","s45","s46","s47","vcc");
    if constexpr (OP == 56) asm volatile("v_mul_f32 v64, 0.5, v1\n\tv_mul_f32 v65, 0.5, v1\n\tv_mul_f32 v66, 0.5, v1\n\tv_mul_f32 v67, 0.5, v1\n\tv_mul_f32 v68, 0.5, v1\n\tv_mul_f32 v69, 0.5, v1\n\tv_mul_f32 v70, 0.5, v1\n\tv_mul_f32 v71, 0.5, v1\n\tv_mul_f32 v72, 0.5, v1\n\tv_mul_f32 v73, 0.5, v1\n\tv_mul_f32 v74, 0.5, v1\n\tv_mul_f32 v75, 0.5, v1\n\tv_mul_f32 v76, 0.5, v1\n\tv_mul_f32 v77, 0.5, v1\n\tv_mul_f32 v78, 0.5, v1\n\tv_mul_f32 v79, 0.5, v1" ::: "v64","v65","v66","v67","v68","v69","v70","v71","v72","v73","v74","v75","v76","v77","v78","v79", "v1","v2","v3","s40","s41","s42","s43","s44","s45","s46","s47","vcc");
    if constexpr (OP == 57) asm volatile("v_min_f32 v64, v1, v2\n\tv_min_f32 v65, v1, v2\n\tv_min_f32 v66, v1, v2\n\tv_min_f32 v67, v1, v2\n\tv_min_f32 v68, v1, v2\n\tv_min_f32 v69, v1, v2\n\tv_min_f32 v70, v1, v2\n\tv_min_f32 v71, v1, v2\n\tv_min_f32 v72, v1, v2\n\tv_min_f32 v73, v1, v2\n\tv_min_f32 v74, v1, v2\n\tv_min_f32 v75, v1, v2\n\tv_min_f32 v76, v1, v2\n\tv_min_f32 v77, v1, v2\n\tv_min_f32 v78, v1, v2\n\tv_min_f32 v79, v1, v2" ::: "v64","v65","v66","v67","v68","v69","v70","v71","v72","v73","v74","v75","v76","v77","v78","v79", "v1","v2","v3","s40","s41","s42","s43","s44","s45","s46","s47","vcc");
    if constexpr (OP == 58) asm volatile("v_sub_f32 v64, v1, v2\n\tv_sub_f32 v65, v1, v2\n\tv_sub_f32 v66, v1, v2\n\tv_sub_f32 v67, v1, v2\n\tv_sub_f32 v68, v1, v2\n\tv_sub_f32 v69, v1, v2\n\tv_sub_f32 v70, v1, v2\n\tv_sub_f32 v71, v1, v2\n\tv_sub_f32 v72, v1, v2\n\tv_sub_f32 v73, v1, v2\n\tv_sub_f32 v74, v1, v2\n\tv_sub_f32 v75, v1, v2\n\tv_sub_f32 v76, v1, v2\n\tv_sub_f32 v77, v1, v2\n\tv_sub_f32 v78, v1, v2\n\tv_sub_f32 v79, v1, v2" ::: "v64","v65","v66","v67","v68","v69","v70","v71","v72","v73","v74","v75","v76","v77","v78","v79", "v1","v2","v3","s40","s41","s42","s43","s44","s45","s46","s47","vcc");
    if constexpr (OP == 59) asm volatile("v_mul_f32 v64, v1, v2\n\tv_mul_f32 v65, v1, v2\n\tv_mul_f32 v66, v1, v2\n\tv_mul_f32 v67, v1, v2\n\tv_mul_f32 v68, v1, v2\n\tv_mul_f32 v69, v1, v2\n\tv_mul_f32 v70, v1, v2\n\tv_mul_f32 v71, v1, v2\n\tv_mul_f32 v72, v1, v2\n\tv_mul_f32 v73, v1, v2\n\tv_mul_f32 v74, v1, v2\n\tv_mul_f32 v75, v1, v2\n\tv_mul_f32 v76, v1, v2\n\tv_mul_f32 v77, v1, v2\n\tv_mul_f32 v78, v1, v2\n\tv_mul_f32 v79, v1, v2" ::: "v64","v65","v66","v67","v68","v69","v70","v71","v72","v73","v74","v75","v76","v77","v78","v79", "v1","v2","v3","s40","s41","s42","s43","s44","s45","s46","s47","vcc");
    if constexpr (OP == 60) asm volatile("v_cndmask_b32 v64, v1, v2, vcc\n\tv_cndmask_b32 v65, v1, v2, vcc\n\tv_cndmask_b32 v66, v1, v2, vcc\n\tv_cndmask_b32 v67, v1, v2, vcc\n\tv_cndmask_b32 v68, v1, v2, vcc\n\tv_cndmask_b32 v69, v1, v2, vcc\n\tv_cndmask_b32 v70, v1, v2, vcc\n\tv_cndmask_b32 v71, v1, v2, vcc\n\tv_cndmask_b32 v72, v1, v2, vcc\n\tv_cndmask_b32 v73, v1, v2, vcc\n\tv_cndmask_b32 v74, v1, v2, vcc\n\tv_cndmask_b32 v75, v1, v2, vcc\n\tv_cndmask_b32 v76, v1, v2, vcc\n\tv_cndmask_b32 v77, v1, v2, vcc\n\tv_cndmask_b32 v78, v1, v2, vcc\n\tv_cndmask_b32 v79, v1, v2, vcc" ::: "v64","v65","v66","v67","v68","v69","v70","v71","v72","v73","v74","v75","v76","v77","v78","v79", "v1","v2","v3","s40","s41","s42","s43","s44","s45","s46","s47","vcc");
    if constexpr (OP == 61) asm volatile("v_mul_f32_e64 v64, v1, s40\n\tv_mul_f32_e64 v65, v1, s40\n\tv_mul_f32_e64 v66, v1, s40\n\tv_mul_f32_e64 v67, v1, s40\n\tv_mul_f32_e64 v68, v1, s40\n\tv_mul_f32_e64 v69, v1, s40\n\tv_mul_f32_e64 v70, v1, s40\n\tv_mul_f32_e64 v71, v1, s40\n\tv_mul_f32_e64 v72, v1, s40\n\tv_mul_f32_e64 v73, v1, s40\n\tv_mul_f32_e64 v74, v1, s40\n\tv_mul_f32_e64 v75, v1, s40\n\tv_mul_f32_e64 v76, v1, s40\n\tv_mul_f32_e64 v77, v1, s40\n\tv_mul_f32_e64 v78, v1, s40\n\tv_mul_f32_e64 v79, v1, s40" ::: "v64","v65","v66","v67","v68","v69","v70","v71","v72","v73","v74","v75","v76","v77","v78","v79", "v1","v2","v3","s40","s41","s42","s43","s44","s45","s46","s47","vcc");
    if constexpr (OP == 62) asm volatile("v_mul_lo_u32 v64, v1, s40\n\tv_mul_lo_u32 v65, v1, s40\n\tv_mul_lo_u32 v66, v1, s40\n\tv_mul_lo_u32 v67, v1, s40\n\tv_mul_lo_u32 v68, v1, s40\n\tv_mul_lo_u32 v69, v1, s40\n\tv_mul_lo_u32 v70, v1, s40\n\tv_mul_lo_u32 v71, v1, s40\n\tv_mul_lo_u32 v72, v1, s40\n\tv_mul_lo_u32 v73, v1, s40\n\tv_mul_lo_u32 v74, v1, s40\n\tv_mul_lo_u32 v75, v1, s40\n\tv_mul_lo_u32 v76, v1, s40\n\tv_mul_lo_u32 v77, v1, s40\n\tv_mul_lo_u32 v78, v1, s40\n\tv_mul_lo_u32 v79, v1, s40" ::: "v64","v65","v66","v67","v68","v69","v70","v71","v72","v73","v74","v75","v76","v77","v78","v79", "v1","v2","v3","s40","s41","s42","s43","s44","s45","s46","s47","vcc");
    if constexpr (OP == 63) asm volatile("v_and_b32 v64, 15, v1\n\tv_and_b32 v65, 15, v1\n\tv_and_b32 v66, 15, v1\n\tv_and_b32 v67, 15, v1\n\tv_and_b32 v68, 15, v1\n\tv_and_b32 v69, 15, v1\n\tv_and_b32 v70, 15, v1\n\tv_and_b32 v71, 15, v1\n\tv_and_b32 v72, 15, v1\n\tv_and_b32 v73, 15, v1\n\tv_and_b32 v74, 15, v1\n\tv_and_b32 v75, 15, v1\n\tv_and_b32 v76, 15, v1\n\tv_and_b32 v77, 15, v1\n\tv_and_b32 v78, 15, v1\n\tv_and_b32 v79, 15, v1" ::: "v64","v65","v66","v67","v68","v69","v70","v71","v72","v73","v74","v75","v76","v77","v78","v79", "v1","v2","v3","s40","s41","s42","s43","s44","s45","s46","s47","vcc");
    if constexpr (OP == 64) asm volatile("v_or_b32 v64, v1, v2\n\tv_or_b32 v65, v1, v2\n\tv_or_b32 v66, v1, v2\n\tv_or_b32 v67, v1, v2\n\tv_or_b32 v68, v1, v2\n\tv_or_b32 v69, v1, v2\n\tv_or_b32 v70, v1, v2\n\tv_or_b32 v71, v1, v2\n\tv_or_b32 v72, v1, v2\n\tv_or_b32 v73, v1, v2\n\tv_or_b32 v74, v1, v2\n\tv_or_b32 v75, v1, v2\n\tv_or_b32 v76, v1, v2\n\tv_or_b32 v77, v1, v2\n\tv_or_b32 v78, v1, v2\n\tv_or_b32 v79, v1, v2" ::: "v64","v65","v66","v67","v68","v69","v70","v71","v72","v73","v74","v75","v76","v77","v78","v79", "v1","v2","v3","s40","s41","s42","s43","s44","s45","s46","s47","vcc");
    if constexpr (OP == 65) asm volatile("v_cmp_eq_u32 vcc, v1, v64\n\tv_cmp_eq_u32 vcc, v1, v65\n\tv_cmp_eq_u32 vcc, v1, v66\n\tv_cmp_eq_u32 vcc, v1, v67\n\tv_cmp_eq_u32 vcc, v1, v68\n\tv_cmp_eq_u32 vcc, v1, v69\n\tv_cmp_eq_u32 vcc, v1, v70\n\tv_cmp_eq_u32 vcc, v1, v71\n\tv_cmp_eq_u32 vcc, v1, v72\n\tv_cmp_eq_u32 vcc, v1, v73\n\tv_cmp_eq_u32 vcc, v1, v74\n\tv_cmp_eq_u32 vcc, v1, v75\n\tv_cmp_eq_u32 vcc, v1, v76\n\tv_cmp_eq_u32 vcc, v1, v77\n\tv_cmp_eq_u32 vcc, v1, v78\n\tv_cmp_eq_u32 vcc, v1, v79" ::: "v64","v65","v66","v67","v68","v69","v70","v71","v72","v73","v74","v75","v76","v77","v78","v79", "v1","v2","v3","s40","s41","s42","s43","s44","s45","s46","s47","vcc");
    if constexpr (OP == 66) asm volatile("v_max_i32 v64, v1, v2\n\tv_max_i32 v65, v1, v2\n\tv_max_i32 v66, v1, v2\n\tv_max_i32 v67, v1, v2\n\tv_max_i32 v68, v1, v2\n\tv_max_i32 v69, v1, v2\n\tv_max_i32 v70, v1, v2\n\tv_max_i32 v71, v1, v2\n\tv_max_i32 v72, v1, v2\n\tv_max_i32 v73, v1, v2\n\tv_max_i32 v74, v1, v2\n\tv_max_i32 v75, v1, v2\n\tv_max_i32 v76, v1, v2\n\tv_max_i32 v77, v1, v2\n\tv_max_i32 v78, v1, v2\n\tv_max_i32 v79, v1, v2" ::: "v64","v65","v66","v67","v68","v69","v70","v71","v72","v73","v74","v75","v76","v77","v78","v79", "v1","v2","v3","s40","s41","s42","s43","s44","s45","s46","s47","vcc");
    if constexpr (OP == 67) asm volatile("v_med3_f32 v64, v1, v2, v3\n\tv_med3_f32 v65, v1, v2, v3\n\tv_med3_f32 v66, v1, v2, v3\n\tv_med3_f32 v67, v1, v2, v3\n\tv_med3_f32 v68, v1, v2, v3\n\tv_med3_f32 v69, v1, v2, v3\n\tv_med3_f32 v70, v1, v2, v3\n\tv_med3_f32 v71, v1, v2, v3\n\tv_med3_f32 v72, v1, v2, v3\n\tv_med3_f32 v73, v1, v2, v3\n\tv_med3_f32 v74, v1, v2, v3\n\tv_med3_f32 v75, v1, v2, v3\n\tv_med3_f32 v76, v1, v2, v3\n\tv_med3_f32 v77, v1, v2, v3\n\tv_med3_f32 v78, v1, v2, v3\n\tv_med3_f32 v79, v1, v2, v3" ::: "v64","v65","v66","v67","v68","v69","v70","v71","v72","v73","v74","v75","v76","v77","v78","v79", "v1","v2","v3","s40","s41","s42","s43","s44","s45","s46","s47","vcc");
    if constexpr (OP == 68) asm volatile("v_fma_mix_f32 v64, v1, v2, v3 op_sel_hi:[0,0,1]\n\tv_fma_mix_f32 v65, v1, v2, v3 op_sel_hi:[0,0,1]\n\tv_fma_mix_f32 v66, v1, v2, v3 op_sel_hi:[0,0,1]\n\tv_fma_mix_f32 v67, v1, v2, v3 op_sel_hi:[0,0,1]\n\tv_fma_mix_f32 v68, v1, v2, v3 op_sel_hi:[0,0,1]\n\tv_fma_mix_f32 v69, v1, v2, v3 op_sel_hi:[0,0,1]\n\tv_fma_mix_f32 v70, v1, v2, v3 op_sel_hi:[0,0,1]\n\tv_fma_mix_f32 v71, v1, v2, v3 op_sel_hi:[0,0,1]\n\tv_fma_mix_f32 v72, v1, v2, v3 op_sel_hi:[0,0,1]\n\tv_fma_mix_f32 v73, v1, v2, v3 op_sel_hi:[0,0,1]\n\tv_fma_mix_f32 v74, v1, v2, v3 op_sel_hi:[0,0,1]\n\tv_fma_mix_f32 v75, v1, v2, v3 op_sel_hi:[0,0,1]\n\tv_fma_mix_f32 v76, v1, v2, v3 op_sel_hi:[0,0,1]\n\tv_fma_mix_f32 v77, v1, v2, v3 op_sel_hi:[0,0,1]\n\tv_fma_mix_f32 v78, v1, v2, v3 op_sel_hi:[0,0,1]\n\tv_fma_mix_f32 v79, v1, v2, v3 op_sel_hi:[0,0,1]" ::: "v64","v65","v66","v67","v68","v69","v70","v71","v72","v73","v74","v75","v76","v77","v78","v79", "v1","v2","v3","s40","s41","s42","s43","s44","s45","s46","s47","vcc");
    if constexpr (OP == 69) asm volatile("v_lshlrev_b32 v64, 16, v1\n\tv_lshlrev_b32 v65, 16, v1\n\tv_lshlrev_b32 v66, 16, v1\n\tv_lshlrev_b32 v67, 16, v1\n\tv_lshlrev_b32 v68, 16, v1\n\tv_lshlrev_b32 v69, 16, v1\n\tv_lshlrev_b32 v70, 16, v1\n\tv_lshlrev_b32 v71, 16, v1\n\tv_lshlrev_b32 v72, 16, v1\n\tv_lshlrev_b32 v73, 16, v1\n\tv_lshlrev_b32 v74, 16, v1\n\tv_lshlrev_b32 v75, 16, v1\n\tv_lshlrev_b32 v76, 16, v1\n\tv_lshlrev_b32 v77, 16, v1\n\tv_lshlrev_b32 v78, 16, v1\n\tv_lshlrev_b32 v79, 16, v1" ::: "v64","v65","v66","v67","v68","v69","v70","v71","v72","v73","v74","v75","v76","v77","v78","v79", "v1","v2","v3","s40","s41","s42","s43","s44","s45","s46","s47","vcc");
    if constexpr (OP == 70) asm volatile("v_cvt_f32_bf16 v64, v1\n\tv_cvt_f32_bf16 v65, v1\n\tv_cvt_f32_bf16 v66, v1\n\tv_cvt_f32_bf16 v67, v1\n\tv_cvt_f32_bf16 v68, v1\n\tv_cvt_f32_bf16 v69, v1\n\tv_cvt_f32_bf16 v70, v1\n\tv_cvt_f32_bf16 v71, v1\n\tv_cvt_f32_bf16 v72, v1\n\tv_cvt_f32_bf16 v73, v1\n\tv_cvt_f32_bf16 v74, v1\n\tv_cvt_f32_bf16 v75, v1\n\tv_cvt_f32_bf16 v76, v1\n\tv_cvt_f32_bf16 v77, v1\n\tv_cvt_f32_bf16 v78, v1\n\tv_cvt_f32_bf16 v79, v1" ::: "v64","v65","v66","v67","v68","v69","v70","v71","v72","v73","v74","v75","v76","v77","v78","v79", "v1","v2","v3","s40","s41","s42","s43","s44","s45","s46","s47","vcc");
    if constexpr (OP == 71) asm volatile("v_perm_b32 v64, v1, v2, v3\n\tv_perm_b32 v65, v1, v2, v3\n\tv_perm_b32 v66, v1, v2, v3\n\tv_perm_b32 v67, v1, v2, v3\n\tv_perm_b32 v68, v1, v2, v3\n\tv_perm_b32 v69, v1, v2, v3\n\tv_perm_b32 v70, v1, v2, v3\n\tv_perm_b32 v71, v1, v2, v3\n\tv_perm_b32 v72, v1, v2, v3\n\tv_perm_b32 v73, v1, v2, v3\n\tv_perm_b32 v74, v1, v2, v3\n\tv_perm_b32 v75, v1, v2, v3\n\tv_perm_b32 v76, v1, v2, v3\n\tv_perm_b32 v77, v1, v2, v3\n\tv_perm_b32 v78, v1, v2, v3\n\tv_perm_b32 v79, v1, v2, v3" ::: "v64","v65","v66","v67","v68","v69","v70","v71","v72","v73","v74","v75","v76","v77","v78","v79", "v1","v2","v3","s40","s41","s42","s43","s44","s45","s46","s47","vcc");
    if constexpr (OP == 72) asm volatile("v_cvt_f32_ubyte1 v64, v1\n\tv_cvt_f32_ubyte1 v65, v1\n\tv_cvt_f32_ubyte1 v66, v1\n\tv_cvt_f32_ubyte1 v67, v1\n\tv_cvt_f32_ubyte1 v68, v1\n\tv_cvt_f32_ubyte1 v69, v1\n\tv_cvt_f32_ubyte1 v70, v1\n\tv_cvt_f32_ubyte1 v71, v1\n\tv_cvt_f32_ubyte1 v72, v1\n\tv_cvt_f32_ubyte1 v73, v1\n\tv_cvt_f32_ubyte1 v74, v1\n\tv_cvt_f32_ubyte1 v75, v1\n\tv_cvt_f32_ubyte1 v76, v1\n\tv_cvt_f32_ubyte1 v77, v1\n\tv_cvt_f32_ubyte1 v78, v1\n\tv_cvt_f32_ubyte1 v79, v1" ::: "v64","v65","v66","v67","v68","v69","v70","v71","v72","v73","v74","v75","v76","v77","v78","v79", "v1","v2","v3","s40","s41","s42","s43","s44","s45","s46","s47","vcc");
    if constexpr (OP == 73) asm volatile("v_and_b32 v64, v2, v1\n\tv_and_b32 v65, v2, v1\n\tv_and_b32 v66, v2, v1\n\tv_and_b32 v67, v2, v1\n\tv_and_b32 v68, v2, v1\n\tv_and_b32 v69, v2, v1\n\tv_and_b32 v70, v2, v1\n\tv_and_b32 v71, v2, v1\n\tv_and_b32 v72, v2, v1\n\tv_and_b32 v73, v2, v1\n\tv_and_b32 v74, v2, v1\n\tv_and_b32 v75, v2, v1\n\tv_and_b32 v76, v2, v1\n\tv_and_b32 v77, v2, v1\n\tv_and_b32 v78, v2, v1\n\tv_and_b32 v79, v2, v1" ::: "v64","v65","v66","v67","v68","v69","v70","v71","v72","v73","v74","v75","v76","v77","v78","v79", "v1","v2","v3","s40","s41","s42","s43","s44","s45","s46","s47","vcc");
    if constexpr (OP == 74) asm volatile("v_fma_mix_f32 v64, v1, v2, v3 op_sel:[0,0,1] op_sel_hi:[0,0,1]\n\tv_fma_mix_f32 v65, v1, v2, v3 op_sel:[0,0,1] op_sel_hi:[0,0,1]\n\tv_fma_mix_f32 v66, v1, v2, v3 op_sel:[0,0,1] op_sel_hi:[0,0,1]\n\tv_fma_mix_f32 v67, v1, v2, v3 op_sel:[0,0,1] op_sel_hi:[0,0,1]\n\tv_fma_mix_f32 v68, v1, v2, v3 op_sel:[0,0,1] op_sel_hi:[0,0,1]\n\tv_fma_mix_f32 v69, v1, v2, v3 op_sel:[0,0,1] op_sel_hi:[0,0,1]\n\tv_fma_mix_f32 v70, v1, v2, v3 op_sel:[0,0,1] op_sel_hi:[0,0,1]\n\tv_fma_mix_f32 v71, v1, v2, v3 op_sel:[0,0,1] op_sel_hi:[0,0,1]\n\tv_fma_mix_f32 v72, v1, v2, v3 op_sel:[0,0,1] op_sel_hi:[0,0,1]\n\tv_fma_mix_f32 v73, v1, v2, v3 op_sel:[0,0,1] op_sel_hi:[0,0,1]\n\tv_fma_mix_f32 v74, v1, v2, v3 op_sel:[0,0,1] op_sel_hi:[0,0,1]\n\tv_fma_mix_f32 v75, v1, v2, v3 op_sel:[0,0,1] op_sel_hi:[0,0,1]\n\tv_fma_mix_f32 v76, v1, v2, v3 op_sel:[0,0,1] op_sel_hi:[0,0,1]\n\tv_fma_mix_f32 v77, v1, v2, v3 op_sel:[0,0,1] op_sel_hi:[0,0,1]\n\tv_fma_mix_f32 v78, v1, v2, v3 op_sel:[0,0,1] op_sel_hi:[0,0,1]\n\tv_fma_mix_f32 v79, v1, v2, v3 op_sel:[0,0,1] op_sel_hi:[0,0,1]" ::: "v64","v65","v66","v67","v68","v69","v70","v71","v72","v73","v74","v75","v76","v77","v78","v79", "v1","v2","v3","s40","s41","s42","s43","s44","s45","s46","s47","vcc");
    if constexpr (OP == 75) asm volatile("v_lshlrev_b32 v64, 4, v1\n\tv_lshlrev_b32 v65, 4, v1\n\tv_lshlrev_b32 v66, 4, v1\n\tv_lshlrev_b32 v67, 4, v1\n\tv_lshlrev_b32 v68, 4, v1\n\tv_lshlrev_b32 v69, 4, v1\n\tv_lshlrev_b32 v70, 4, v1\n\tv_lshlrev_b32 v71, 4, v1\n\tv_lshlrev_b32 v72, 4, v1\n\tv_lshlrev_b32 v73, 4, v1\n\tv_lshlrev_b32 v74, 4, v1\n\tv_lshlrev_b32 v75, 4, v1\n\tv_lshlrev_b32 v76, 4, v1\n\tv_lshlrev_b32 v77, 4, v1\n\tv_lshlrev_b32 v78, 4, v1\n\tv_lshlrev_b32 v79, 4, v1" ::: "v64","v65","v66","v67","v68","v69","v70","v71","v72","v73","v74","v75","v76","v77","v78","v79", "v1","v2","v3","s40","s41","s42","s43","s44","s45","s46","s47","vcc");
    if constexpr (OP == 76) asm volatile("v_lshlrev_b32 v64, v2, v1\n\tv_lshlrev_b32 v65, v2, v1\n\tv_lshlrev_b32 v66, v2, v1\n\tv_lshlrev_b32 v67, v2, v1\n\tv_lshlrev_b32 v68, v2, v1\n\tv_lshlrev_b32 v69, v2, v1\n\tv_lshlrev_b32 v70, v2, v1\n\tv_lshlrev_b32 v71, v2, v1\n\tv_lshlrev_b32 v72, v2, v1\n\tv_lshlrev_b32 v73, v2, v1\n\tv_lshlrev_b32 v74, v2, v1\n\tv_lshlrev_b32 v75, v2, v1\n\tv_lshlrev_b32 v76, v2, v1\n\tv_lshlrev_b32 v77, v2, v1\n\tv_lshlrev_b32 v78, v2, v1\n\tv_lshlrev_b32 v79, v2, v1" ::: "v64","v65","v66","v67","v68","v69","v70","v71","v72","v73","v74","v75","v76","v77","v78","v79", "v1","v2","v3","s40","s41","s42","s43","s44","s45","s46","s47","vcc");
    if constexpr (OP == 77) asm volatile("v_ashrrev_i32 v64, 4, v1\n\tv_ashrrev_i32 v65, 4, v1\n\tv_ashrrev_i32 v66, 4, v1\n\tv_ashrrev_i32 v67, 4, v1\n\tv_ashrrev_i32 v68, 4, v1\n\tv_ashrrev_i32 v69, 4, v1\n\tv_ashrrev_i32 v70, 4, v1\n\tv_ashrrev_i32 v71, 4, v1\n\tv_ashrrev_i32 v72, 4, v1\n\tv_ashrrev_i32 v73, 4, v1\n\tv_ashrrev_i32 v74, 4, v1\n\tv_ashrrev_i32 v75, 4, v1\n\tv_ashrrev_i32 v76, 4, v1\n\tv_ashrrev_i32 v77, 4, v1\n\tv_ashrrev_i32 v78, 4, v1\n\tv_ashrrev_i32 v79, 4, v1" ::: "v64","v65","v66","v67","v68","v69","v70","v71","v72","v73","v74","v75","v76","v77","v78","v79", "v1","v2","v3","s40","s41","s42","s43","s44","s45","s46","s47","vcc");
    if constexpr (OP == 78) asm volatile("v_cmp_lt_f32 vcc, v1, v64\n\tv_cndmask_b32 v64, v1, v2, vcc\n\tv_cmp_lt_f32 vcc, v1, v65\n\tv_cndmask_b32 v65, v1, v2, vcc\n\tv_cmp_lt_f32 vcc, v1, v66\n\tv_cndmask_b32 v66, v1, v2, vcc\n\tv_cmp_lt_f32 vcc, v1, v67\n\tv_cndmask_b32 v67, v1, v2, vcc\n\tv_cmp_lt_f32 vcc, v1, v68\n\tv_cndmask_b32 v68, v1, v2, vcc\n\tv_cmp_lt_f32 vcc, v1, v69\n\tv_cndmask_b32 v69, v1, v2, vcc\n\tv_cmp_lt_f32 vcc, v1, v70\n\tv_cndmask_b32 v70, v1, v2, vcc\n\tv_cmp_lt_f32 vcc, v1, v71\n\tv_cndmask_b32 v71, v1, v2, vcc\n\tv_cmp_lt_f32 vcc, v1, v72\n\tv_cndmask_b32 v72, v1, v2, vcc\n\tv_cmp_lt_f32 vcc, v1, v73\n\tv_cndmask_b32 v73, v1, v2, vcc\n\tv_cmp_lt_f32 vcc, v1, v74\n\tv_cndmask_b32 v74, v1, v2, vcc\n\tv_cmp_lt_f32 vcc, v1, v75\n\tv_cndmask_b32 v75, v1, v2, vcc\n\tv_cmp_lt_f32 vcc, v1, v76\n\tv_cndmask_b32 v76, v1, v2, vcc\n\tv_cmp_lt_f32 vcc, v1, v77\n\tv_cndmask_b32 v77, v1, v2, vcc\n\tv_cmp_lt_f32 vcc, v1, v78\n\tv_cndmask_b32 v78, v1, v2, vcc\n\tv_cmp_lt_f32 vcc, v1, v79\n\tv_cndmask_b32 v79, v1, v2, vcc" ::: "v64","v65","v66","v67","v68","v69","v70","v71","v72","v73","v74","v75","v76","v77","v78","v79", "v1","v2","v3","s40","s41","s42","s43","s44","s45","s46","s47","vcc");
    if constexpr (OP == 79) asm volatile("v_cmp_lt_f32 s[40:41], v1, v64\n\tv_cndmask_b32_e64 v64, v1, v2, s[40:41]\n\tv_cmp_lt_f32 s[40:41], v1, v65\n\tv_cndmask_b32_e64 v65, v1, v2, s[40:41]\n\tv_cmp_lt_f32 s[40:41], v1, v66\n\tv_cndmask_b32_e64 v66, v1, v2, s[40:41]\n\tv_cmp_lt_f32 s[40:41], v1, v67\n\tv_cndmask_b32_e64 v67, v1, v2, s[40:41]\n\tv_cmp_lt_f32 s[40:41], v1, v68\n\tv_cndmask_b32_e64 v68, v1, v2, s[40:41]\n\tv_cmp_lt_f32 s[40:41], v1, v69\n\tv_cndmask_b32_e64 v69, v1, v2, s[40:41]\n\tv_cmp_lt_f32 s[40:41], v1, v70\n\tv_cndmask_b32_e64 v70, v1, v2, s[40:41]\n\tv_cmp_lt_f32 s[40:41], v1, v71\n\tv_cndmask_b32_e64 v71, v1, v2, s[40:41]\n\tv_cmp_lt_f32 s[40:41], v1, v72\n\tv_cndmask_b32_e64 v72, v1, v2, s[40:41]\n\tv_cmp_lt_f32 s[40:41], v1, v73\n\tv_cndmask_b32_e64 v73, v1, v2, s[40:41]\n\tv_cmp_lt_f32 s[40:41], v1, v74\n\tv_cndmask_b32_e64 v74, v1, v2, s[40:41]\n\tv_cmp_lt_f32 s[40:41], v1, v75\n\tv_cndmask_b32_e64 v75, v1, v2, s[40:41]\n\tv_cmp_lt_f32 s[40:41], v1, v76\n\tv_cndmask_b32_e64 v76, v1, v2, s[40:41]\n\tv_cmp_lt_f32 s[40:41], v1, v77\n\tv_cndmask_b32_e64 v77, v1, v2, s[40:41]\n\tv_cmp_lt_f32 s[40:41], v1, v78\n\tv_cndmask_b32_e64 v78, v1, v2, s[40:41]\n\tv_cmp_lt_f32 s[40:41], v1, v79\n\tv_cndmask_b32_e64 v79, v1, v2, s[40:41]" ::: "v64","v65","v66","v67","v68","v69","v70","v71","v72","v73","v74","v75","v76","v77","v78","v79", "v1","v2","v3","s40","s41","s42","s43","s44","s45","s46","s47","vcc");
    if constexpr (OP == 80) asm volatile("v_sub_u32 v64, v1, v2\n\tv_sub_u32 v65, v1, v2\n\tv_sub_u32 v66, v1, v2\n\tv_sub_u32 v67, v1, v2\n\tv_sub_u32 v68, v1, v2\n\tv_sub_u32 v69, v1, v2\n\tv_sub_u32 v70, v1, v2\n\tv_sub_u32 v71, v1, v2\n\tv_sub_u32 v72, v1, v2\n\tv_sub_u32 v73, v1, v2\n\tv_sub_u32 v74, v1, v2\n\tv_sub_u32 v75, v1, v2\n\tv_sub_u32 v76, v1, v2\n\tv_sub_u32 v77, v1, v2\n\tv_sub_u32 v78, v1, v2\n\tv_sub_u32 v79, v1, v2" ::: "v64","v65","v66","v67","v68","v69","v70","v71","v72","v73","v74","v75","v76","v77","v78","v79", "v1","v2","v3","s40","s41","s42","s43","s44","s45","s46","s47","vcc");
    if constexpr (OP == 81) asm volatile("v_bfi_b32 v64, v1, v2, v3\n\tv_bfi_b32 v65, v1, v2, v3\n\tv_bfi_b32 v66, v1, v2, v3\n\tv_bfi_b32 v67, v1, v2, v3\n\tv_bfi_b32 v68, v1, v2, v3\n\tv_bfi_b32 v69, v1, v2, v3\n\tv_bfi_b32 v70, v1, v2, v3\n\tv_bfi_b32 v71, v1, v2, v3\n\tv_bfi_b32 v72, v1, v2, v3\n\tv_bfi_b32 v73, v1, v2, v3\n\tv_bfi_b32 v74, v1, v2, v3\n\tv_bfi_b32 v75, v1, v2, v3\n\tv_bfi_b32 v76, v1, v2, v3\n\tv_bfi_b32 v77, v1, v2, v3\n\tv_bfi_b32 v78, v1, v2, v3\n\tv_bfi_b32 v79, v1, v2, v3" ::: "v64","v65","v66","v67","v68","v69","v70","v71","v72","v73","v74","v75","v76","v77","v78","v79", "v1","v2","v3","s40","s41","s42","s43","s44","s45","s46","s47","vcc");
    if constexpr (OP == 82) asm volatile("v_mul_f32 v64, 0x3b808081, v1\n\tv_mul_f32 v65, 0x3b808081, v1\n\tv_mul_f32 v66, 0x3b808081, v1\n\tv_mul_f32 v67, 0x3b808081, v1\n\tv_mul_f32 v68, 0x3b808081, v1\n\tv_mul_f32 v69, 0x3b808081, v1\n\tv_mul_f32 v70, 0x3b808081, v1\n\tv_mul_f32 v71, 0x3b808081, v1\n\tv_mul_f32 v72, 0x3b808081, v1\n\tv_mul_f32 v73, 0x3b808081, v1\n\tv_mul_f32 v74, 0x3b808081, v1\n\tv_mul_f32 v75, 0x3b808081, v1\n\tv_mul_f32 v76, 0x3b808081, v1\n\tv_mul_f32 v77, 0x3b808081, v1\n\tv_mul_f32 v78, 0x3b808081, v1\n\tv_mul_f32 v79, 0x3b808081, v1" ::: "v64","v65","v66","v67","v68","v69","v70","v71","v72","v73","v74","v75","v76","v77","v78","v79", "v1","v2","v3","s40","s41","s42","s43","s44","s45","s46","s47","vcc");
    if constexpr (OP == 83) asm volatile("v_pk_add_f32 v[64:65], v[2:3], v[4:5]\n\tv_pk_add_f32 v[66:67], v[2:3], v[4:5]\n\tv_pk_add_f32 v[68:69], v[2:3], v[4:5]\n\tv_pk_add_f32 v[70:71], v[2:3], v[4:5]\n\tv_pk_add_f32 v[72:73], v[2:3], v[4:5]\n\tv_pk_add_f32 v[74:75], v[2:3], v[4:5]\n\tv_pk_add_f32 v[76:77], v[2:3], v[4:5]\n\tv_pk_add_f32 v[78:79], v[2:3], v[4:5]" ::: "v64","v65","v66","v67","v68","v69","v70","v71","v72","v73","v74","v75","v76","v77","v78","v79", "v1","v2","v3","s40","s41","s42","s43","s44","s45","s46","s47","vcc");
    if constexpr (OP == 84) asm volatile("v_xad_u32 v64, v1, v2, v3\n\tv_xad_u32 v65, v1, v2, v3\n\tv_xad_u32 v66, v1, v2, v3\n\tv_xad_u32 v67, v1, v2, v3\n\tv_xad_u32 v68, v1, v2, v3\n\tv_xad_u32 v69, v1, v2, v3\n\tv_xad_u32 v70, v1, v2, v3\n\tv_xad_u32 v71, v1, v2, v3\n\tv_xad_u32 v72, v1, v2, v3\n\tv_xad_u32 v73, v1, v2, v3\n\tv_xad_u32 v74, v1, v2, v3\n\tv_xad_u32 v75, v1, v2, v3\n\tv_xad_u32 v76, v1, v2, v3\n\tv_xad_u32 v77, v1, v2, v3\n\tv_xad_u32 v78, v1, v2, v3\n\tv_xad_u32 v79, v1, v2, v3" ::: "v64","v65","v66","v67","v68","v69","v70","v71","v72","v73","v74","v75","v76","v77","v78","v79", "v1","v2","v3","s40","s41","s42","s43","s44","s45","s46","s47","vcc");
    if constexpr (OP == 85) asm volatile("v_fmaak_f32 v64, v1, v2, 0x41200000\n\tv_fmaak_f32 v65, v1, v2, 0x41200000\n\tv_fmaak_f32 v66, v1, v2, 0x41200000\n\tv_fmaak_f32 v67, v1, v2, 0x41200000\n\tv_fmaak_f32 v68, v1, v2, 0x41200000\n\tv_fmaak_f32 v69, v1, v2, 0x41200000\n\tv_fmaak_f32 v70, v1, v2, 0x41200000\n\tv_fmaak_f32 v71, v1, v2, 0x41200000\n\tv_fmaak_f32 v72, v1, v2, 0x41200000\n\tv_fmaak_f32 v73, v1, v2, 0x41200000\n\tv_fmaak_f32 v74, v1, v2, 0x41200000\n\tv_fmaak_f32 v75, v1, v2, 0x41200000\n\tv_fmaak_f32 v76, v1, v2, 0x41200000\n\tv_fmaak_f32 v77, v1, v2, 0x41200000\n\tv_fmaak_f32 v78, v1, v2, 0x41200000\n\tv_fmaak_f32 v79, v1, v2, 0x41200000" ::: "v64","v65","v66","v67","v68","v69","v70","v71","v72","v73","v74","v75","v76","v77","v78","v79", "v1","v2","v3","s40","s41","s42","s43","s44","s45","s46","s47","vcc");
    if constexpr (OP == 86) asm volatile("v_cvt_u32_f32 v64, v1\n\tv_cvt_u32_f32 v65, v1\n\tv_cvt_u32_f32 v66, v1\n\tv_cvt_u32_f32 v67, v1\n\tv_cvt_u32_f32 v68, v1\n\tv_cvt_u32_f32 v69, v1\n\tv_cvt_u32_f32 v70, v1\n\tv_cvt_u32_f32 v71, v1\n\tv_cvt_u32_f32 v72, v1\n\tv_cvt_u32_f32 v73, v1\n\tv_cvt_u32_f32 v74, v1\n\tv_cvt_u32_f32 v75, v1\n\tv_cvt_u32_f32 v76, v1\n\tv_cvt_u32_f32 v77, v1\n\tv_cvt_u32_f32 v78, v1\n\tv_cvt_u32_f32 v79, v1" ::: "v64","v65","v66","v67","v68","v69","v70","v71","v72","v73","v74","v75","v76","v77","v78","v79", "v1","v2","v3","s40","s41","s42","s43","s44","s45","s46","s47","vcc");
    if constexpr (OP == 0) { R16(FMA) }
    if constexpr (OP == 1) { R16(MUL) }
    if constexpr (OP == 2) { R16(MULLO) }
    if constexpr (OP == 3) { R16(XOR) }
    if constexpr (OP == 4) { R16(CVT) }
    if constexpr (OP == 5) { R16(FLOOR) }
    if constexpr (OP == 6) { R16(EXP) }
    if constexpr (OP == 7) { R16(MIN3) }
    if constexpr (OP == 9) { R16(FMAMIX) }
    if constexpr (OP == 8) {
        // v_pk_fma_f32 on 8 register pairs (16 lanes of work per instruction pair)
        for (int i = 0; i < 16; i += 2) {
            float2 v = make_float2(f[i], f[i + 1]);
            asm volatile("v_pk_fma_f32 %0, %0, %1, %1" : "+v"(v) : "v"(make_float2(s, s)));
            f[i] = v.x; f[i + 1] = v.y;
        }
    }
}

template <int OP>
__global__ __launch_bounds__(256) void k_op(float* out, unsigned long long* clk, float s)
{
    float f[16];
    unsigned u[16];
    for (int i = 0; i < 16; ++i) { f[i] = threadIdx.x * 0.001f + i; u[i] = threadIdx.x * 7u + i; }
    const unsigned long long t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
    for (int it = 0; it < ITER; ++it) body<OP>(f, u, s);
    const unsigned long long t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
    float acc = 0.0f;
    for (int i = 0; i < 16; ++i) acc += f[i] + (float)u[i];
    out[blockIdx.x * 256 + threadIdx.x] = acc;
    if (threadIdx.x == 0 && blockIdx.x == 0) { clk[0] = t1 - t0; clk[1] = r1 - r0; }
}

template <int OP>
void run(const char* name, double per_instr, int cus, float* out, unsigned long long* clk)
{
    for (int w : {2, 8}) {
        const int blocks = cus * w;   // 4 waves per block = one per SIMD of a CU
        hipEvent_t a, b;
        hipEventCreate(&a); hipEventCreate(&b);
        k_op<OP><<<blocks, 256>>>(out, clk, 1.0001f);
        hipEventRecord(a);
        k_op<OP><<<blocks, 256>>>(out, clk, 1.0001f);
        hipEventRecord(b);
        hipEventSynchronize(b);
        float ms = 0;
        hipEventElapsedTime(&ms, a, b);
        unsigned long long h[2];
        hipMemcpy(h, clk, sizeof h, hipMemcpyDeviceToHost);
        const double mhz = h[1] ? 100.0 * (double)h[0] / (double)h[1] : 0.0;
        const double instr_per_simd = (double)w * ITER * 16 * per_instr;
        const double cyc = ms * 1e-3 * mhz * 1e6;
        printf("%-10s waves/SIMD %d  %.3f ms  clock %.0f MHz  %.2f cycles per wave64 instr per SIMD\n", name, w, ms,
               mhz, cyc / instr_per_simd);
        hipEventDestroy(a); hipEventDestroy(b);
    }
}

int main()
{
    int cus = 0;
    hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
    float* out;
    unsigned long long* clk;
    hipMalloc(&out, (size_t)cus * 8 * 256 * sizeof(float));
    hipMalloc(&clk, 16);
    run<0>("fma_f32", 1, cus, out, clk);
    run<1>("mul_f32", 1, cus, out, clk);
    run<2>("mul_lo_u32", 1, cus, out, clk);
    run<3>("xor_b32", 1, cus, out, clk);
    run<4>("cvt_i32", 1, cus, out, clk);
    run<5>("floor_f32", 1, cus, out, clk);
    run<6>("exp_f32", 1, cus, out, clk);
    run<7>("min3_f32", 1, cus, out, clk);
    run<8>("pk_fma_f32", 0.5, cus, out, clk);   // per pk instruction (8 per body)
    run<9>("fma+mullo", 2, cus, out, clk);
    run<10>("fma_3reg", 1, cus, out, clk);
    run<11>("fmac_f32", 1, cus, out, clk);
    run<12>("add_f32", 1, cus, out, clk);
    run<13>("cndmask", 1, cus, out, clk);
    run<14>("mul_u24", 1, cus, out, clk);
    run<15>("mad_u24", 1, cus, out, clk);
    run<16>("lshl_add", 1, cus, out, clk);
    run<17>("mov_b32", 1, cus, out, clk);
    run<18>("mul_hi_u32", 1, cus, out, clk);
    run<19>("cvt_f32_i32", 1, cus, out, clk);
    run<20>("fract_f32", 1, cus, out, clk);
    run<21>("pk_mul_f32", 0.5, cus, out, clk);
    run<22>("pk_add_f32", 0.5, cus, out, clk);
    run<23>("pk_fma_3reg", 0.5, cus, out, clk);
    run<24>("fma_banks_diff", 1, cus, out, clk);
    run<25>("fma_banks_same", 1, cus, out, clk);
    run<26>("fma_a_a_c", 1, cus, out, clk);
    run<27>("mul_a_a", 1, cus, out, clk);
    run<28>("mul_banks_same", 1, cus, out, clk);
    run<29>("mul_banks_diff", 1, cus, out, clk);
    run<30>("fma_2same_bank", 1, cus, out, clk);
    run<31>("fma_dst_src", 1, cus, out, clk);
    run<32>("fma_a_c_c", 1, cus, out, clk);
    run<33>("min3_diff", 1, cus, out, clk);
    run<34>("bitop3", 1, cus, out, clk);
    run<35>("and_or", 1, cus, out, clk);
    run<36>("add3_u32", 1, cus, out, clk);
    run<37>("lshl_or", 1, cus, out, clk);
    run<38>("bfe_u32", 1, cus, out, clk);
    run<39>("alignbyte", 1, cus, out, clk);
    run<40>("cvt_flr_i32", 1, cus, out, clk);
    run<41>("cvt_ubyte0", 1, cus, out, clk);
    run<42>("max_f32", 1, cus, out, clk);
    run<43>("rndne", 1, cus, out, clk);
    run<44>("cmp_lt_f32", 1, cus, out, clk);
    run<45>("cndmask_e64", 1, cus, out, clk);
    run<46>("lshrrev", 1, cus, out, clk);
    run<47>("add_u32", 1, cus, out, clk);
    run<48>("fmamk", 1, cus, out, clk);
    run<49>("mul_f32_sgpr", 1, cus, out, clk);
    run<51>("pk_fma_banks", 0.5, cus, out, clk);
    run<52>("mul_sgpr_each", 1, cus, out, clk);
    run<53>("add_sgpr", 1, cus, out, clk);
    run<54>("xor_sgpr", 1, cus, out, clk);
    run<55>("fma_sgpr", 1, cus, out, clk);
    run<56>("mul_inline", 1, cus, out, clk);
    run<57>("min_f32", 1, cus, out, clk);
    run<58>("sub_f32", 1, cus, out, clk);
    run<59>("mul_vv", 1, cus, out, clk);
    run<60>("cnd_vop2", 1, cus, out, clk);
    run<61>("mul_sgpr_e64", 1, cus, out, clk);
    run<68>("fma_mix_f16c", 1, cus, out, clk);
    run<69>("lshlrev_16", 1, cus, out, clk);
    run<70>("cvt_f32_bf16", 1, cus, out, clk);
    run<71>("perm_b32", 1, cus, out, clk);
    run<72>("cvt_ubyte1", 1, cus, out, clk);
    run<73>("and_b32", 1, cus, out, clk);
    run<74>("fma_mix_hi", 1, cus, out, clk);
    run<75>("lshlrev_4", 1, cus, out, clk);
    run<76>("lshlrev_vgpr", 1, cus, out, clk);
    run<77>("ashrrev_4", 1, cus, out, clk);
    run<78>("cmp+cnd_vcc", 2, cus, out, clk);
    run<79>("cmp+cnd_sgpr", 2, cus, out, clk);
    run<80>("sub_u32", 1, cus, out, clk);
    run<81>("bfi_b32", 1, cus, out, clk);
    run<82>("mul_literal", 1, cus, out, clk);
    run<83>("pk_add_vv", 0.5, cus, out, clk);
    run<84>("xad_u32", 1, cus, out, clk);
    run<85>("fmaak_lit", 1, cus, out, clk);
    run<86>("cvt_u32_f32", 1, cus, out, clk);
    run<62>("mullo_sgpr", 1, cus, out, clk);
    run<63>("and_b32", 1, cus, out, clk);
    run<64>("or_b32", 1, cus, out, clk);
    run<65>("cmp_eq_u32", 1, cus, out, clk);
    run<66>("max_i32", 1, cus, out, clk);
    run<67>("med3", 1, cus, out, clk);
    return hipDeviceSynchronize() == hipSuccess ? 0 : 1;
}
