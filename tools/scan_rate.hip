// Issue rate of the RoIPool forward's per-pixel update sequence (tools only):
// 16 channels x (compare, select value, select index) in different orders and
// compare forms, 16 independent channels per wave, 4 waves per SIMD (one
// 1024-thread workgroup per CU).  Cycles per pixel-iteration per SIMD.
// Build: hipcc --offload-arch=gfx950 -O3 -o tools/prev/scan_rate tools/scan_rate.hip
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>

constexpr int kIters = 4096;

#define R16(X) X(0) X(1) X(2) X(3) X(4) X(5) X(6) X(7) X(8) X(9) X(10) X(11) X(12) X(13) X(14) X(15)

template <int MODE>
__global__ __launch_bounds__(1024) void probe(const float* __restrict__ in, float* __restrict__ out) {
    float v[16], m[16];
    int mi[16];
#pragma unroll
    for (int c = 0; c < 16; ++c) {
        v[c] = in[(threadIdx.x * 16 + c) & 1023];
        m[c] = in[(threadIdx.x * 16 + c + 5) & 1023];
        mi[c] = c;
    }
    int ii = threadIdx.x;
    for (int it = 0; it < kIters; ++it) {
        if (MODE == 0) {  // 16 compares into SGPR pairs, then 32 selects (the compiler's schedule)
            uint64_t g[16];
#define C(i) asm volatile("v_cmp_gt_f32_e64 %0, %1, %2" : "=s"(g[i]) : "v"(v[i]), "v"(m[i]));
            R16(C)
#undef C
#define S(i) asm volatile("v_cndmask_b32_e64 %0, %0, %1, %2" : "+v"(mi[i]) : "v"(ii), "s"(g[i]));
            R16(S)
#undef S
#define S(i) asm volatile("v_cndmask_b32_e64 %0, %0, %1, %2" : "+v"(m[i]) : "v"(v[i]), "s"(g[i]));
            R16(S)
#undef S
        } else if (MODE == 1) {  // per channel: compare -> SGPR, select, select
            uint64_t g[16];
#define C(i)                                                                                  \
    asm volatile("v_cmp_gt_f32_e64 %0, %1, %2" : "=s"(g[i]) : "v"(v[i]), "v"(m[i]));        \
    asm volatile("v_cndmask_b32_e64 %0, %0, %1, %2" : "+v"(mi[i]) : "v"(ii), "s"(g[i]));   \
    asm volatile("v_cndmask_b32_e64 %0, %0, %1, %2" : "+v"(m[i]) : "v"(v[i]), "s"(g[i]));
            R16(C)
#undef C
        } else if (MODE == 2) {  // compare -> VCC, s_nop 1, select, select
#define C(i)                                                                                              \
    asm volatile("v_cmp_gt_f32_e32 vcc, %2, %3\n s_nop 1\n v_cndmask_b32_e32 %0, %0, %4, vcc\n"         \
                 " v_cndmask_b32_e32 %1, %1, %2, vcc"                                                    \
                 : "+v"(m[i]), "+v"(mi[i]) : "v"(v[i]), "v"(m[i]), "v"(ii) : "vcc");
            R16(C)
#undef C
        } else if (MODE == 3) {  // compares one channel ahead of their selects (VCC never waited on)
            uint64_t g[16];
            asm volatile("v_cmp_gt_f32_e64 %0, %1, %2" : "=s"(g[0]) : "v"(v[0]), "v"(m[0]));
#define C(i)                                                                                      \
    if (i < 15) asm volatile("v_cmp_gt_f32_e64 %0, %1, %2" : "=s"(g[(i + 1) & 15]) : "v"(v[(i + 1) & 15]), \
                             "v"(m[(i + 1) & 15]));                                               \
    asm volatile("v_cndmask_b32_e64 %0, %0, %1, %2" : "+v"(mi[i]) : "v"(ii), "s"(g[i]));       \
    asm volatile("v_cndmask_b32_e64 %0, %0, %1, %2" : "+v"(m[i]) : "v"(v[i]), "s"(g[i]));
            R16(C)
#undef C
        } else if (MODE == 4) {  // v_max for the value, compare -> SGPR + one select for the index
            uint64_t g[16];
#define C(i) asm volatile("v_cmp_gt_f32_e64 %0, %1, %2" : "=s"(g[i]) : "v"(v[i]), "v"(m[i]));
            R16(C)
#undef C
#define S(i)                                                                                    \
    asm volatile("v_cndmask_b32_e64 %0, %0, %1, %2" : "+v"(mi[i]) : "v"(ii), "s"(g[i]));       \
    asm volatile("v_max_f32_e32 %0, %0, %1" : "+v"(m[i]) : "v"(v[i]));
            R16(S)
#undef S
        } else if (MODE == 5) {  // compares only (-> SGPR)
            uint64_t g[16];
#define C(i) asm volatile("v_cmp_gt_f32_e64 %0, %1, %2" : "=s"(g[i]) : "v"(v[i]), "v"(m[i]));
            R16(C)
#undef C
#define S(i) asm volatile("" ::"s"(g[i]));
            R16(S)
#undef S
        } else if (MODE == 6) {  // selects only (SGPR mask)
            uint64_t g = static_cast<uint64_t>(__builtin_amdgcn_readfirstlane(ii)) * 0x9E3779B97F4A7C15ull;
#define S(i)                                                                                    \
    asm volatile("v_cndmask_b32_e64 %0, %0, %1, %2" : "+v"(mi[i]) : "v"(ii), "s"(g));          \
    asm volatile("v_cndmask_b32_e64 %0, %0, %1, %2" : "+v"(m[i]) : "v"(v[i]), "s"(g));
            R16(S)
#undef S
        } else {  // compares -> VCC only
#define C(i) asm volatile("v_cmp_gt_f32_e32 vcc, %0, %1" ::"v"(v[i]), "v"(m[i]) : "vcc");
            R16(C)
#undef C
        }
        ii += 1;
    }
    float sum = 0;
#pragma unroll
    for (int c = 0; c < 16; ++c) sum += m[c] + static_cast<float>(mi[c]);
    out[blockIdx.x * 1024 + threadIdx.x] = sum;
}

int main() {
    float *in, *out;
    (void)hipMalloc(&in, 1024 * 4);
    float h[1024];
    unsigned s = 12345;
    for (float& x : h) {
        s = s * 1664525u + 1013904223u;
        x = static_cast<float>(s >> 8) / 16777216.0f;
    }
    (void)hipMemcpy(in, h, sizeof(h), hipMemcpyHostToDevice);
    (void)hipMalloc(&out, 1 << 22);
    int cus = 0, khz = 0;
    (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
    (void)hipDeviceGetAttribute(&khz, hipDeviceAttributeClockRate, 0);
    const char* names[8] = {"16 cmp->sgpr, 32 sel", "per ch: cmp->sgpr, sel, sel", "per ch: cmp->vcc, nop, sel, sel",
                            "cmp one ch ahead (sgpr)", "16 cmp, 16 sel + 16 v_max", "16 cmp->sgpr only",
                            "32 sel only", "16 cmp->vcc only"};
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    for (int mode = 0; mode < 8; ++mode) {
        auto launch = [&]() {
            switch (mode) {
                case 0: hipLaunchKernelGGL(probe<0>, dim3(cus), dim3(1024), 0, 0, in, out); break;
                case 1: hipLaunchKernelGGL(probe<1>, dim3(cus), dim3(1024), 0, 0, in, out); break;
                case 2: hipLaunchKernelGGL(probe<2>, dim3(cus), dim3(1024), 0, 0, in, out); break;
                case 3: hipLaunchKernelGGL(probe<3>, dim3(cus), dim3(1024), 0, 0, in, out); break;
                case 4: hipLaunchKernelGGL(probe<4>, dim3(cus), dim3(1024), 0, 0, in, out); break;
                case 5: hipLaunchKernelGGL(probe<5>, dim3(cus), dim3(1024), 0, 0, in, out); break;
                case 6: hipLaunchKernelGGL(probe<6>, dim3(cus), dim3(1024), 0, 0, in, out); break;
                default: hipLaunchKernelGGL(probe<7>, dim3(cus), dim3(1024), 0, 0, in, out); break;
            }
        };
        launch();
        (void)hipDeviceSynchronize();
        (void)hipEventRecord(e0);
        for (int r = 0; r < 5; ++r) launch();
        (void)hipEventRecord(e1);
        (void)hipEventSynchronize(e1);
        float ms = 0;
        (void)hipEventElapsedTime(&ms, e0, e1);
        const double cyc = ms / 5 * 1e-3 * khz * 1e3;  // per SIMD: 4 waves x kIters pixel-iterations
        printf("%-34s %.3f ms  %.1f cycles per pixel-iteration per SIMD (4 waves), %.1f per wave-iteration\n",
               names[mode], ms / 5, cyc / kIters, cyc / kIters / 4);
    }
    return 0;
}
