// VALU issue-rate probe (tools only): cycles per wave64 instruction, 4 waves
// per SIMD (one 1024-thread workgroup per CU), for the forms the RoIPool scan
// uses: v_cmp_gt_f32 into SGPR pairs, v_cndmask_b32 on an SGPR mask,
// v_max3_f32, v_bfi_b32, v_sub_f32, v_ashrrev_i32.  Each mode issues 16
// independent instructions per iteration (inline asm, fixed forms).
// Build: hipcc --offload-arch=gfx950 -O3 -o tools/prev/valu_rate tools/valu_rate.hip
#include <hip/hip_runtime.h>

#include <cstdio>

constexpr int kIters = 8192;

#define R16(X) X(0) X(1) X(2) X(3) X(4) X(5) X(6) X(7) X(8) X(9) X(10) X(11) X(12) X(13) X(14) X(15)

template <int MODE>
__global__ __launch_bounds__(1024) void probe(const float* __restrict__ in, float* __restrict__ out) {
    float v[16];
#pragma unroll
    for (int c = 0; c < 16; ++c) v[c] = in[(threadIdx.x * 16 + c) & 1023];
    float a = in[threadIdx.x & 1023], b = in[(threadIdx.x + 7) & 1023];
    unsigned long long acc = 0;
    for (int it = 0; it < kIters; ++it) {
        if (MODE == 0) {  // 16 x v_cmp_gt_f32 -> distinct SGPR pairs
            unsigned long long s[16];
#define C(i) asm volatile("v_cmp_gt_f32_e64 %0, %1, %2" : "=s"(s[i]) : "v"(v[i]), "v"(a));
            R16(C)
#undef C
#define O(i) acc ^= s[i];
            R16(O)
#undef O
        } else if (MODE == 1) {  // 16 x v_cndmask_b32 on one SGPR mask
            unsigned long long msk = static_cast<unsigned long long>(it) * 0x9E3779B97F4A7C15ull;
            msk = __builtin_amdgcn_readfirstlane(static_cast<unsigned>(msk)) | (1ull << 40);
#define C(i) asm volatile("v_cndmask_b32_e64 %0, %0, %1, %2" : "+v"(v[i]) : "v"(b), "s"(msk));
            R16(C)
#undef C
        } else if (MODE == 2) {  // 16 x v_max3_f32
#define C(i) asm volatile("v_max3_f32 %0, %0, %1, %2" : "+v"(v[i]) : "v"(a), "v"(b));
            R16(C)
#undef C
        } else if (MODE == 3) {  // 16 x v_bfi_b32
#define C(i) asm volatile("v_bfi_b32 %0, %1, %2, %0" : "+v"(v[i]) : "v"(a), "v"(b));
            R16(C)
#undef C
        } else if (MODE == 4) {  // 16 x v_sub_f32
#define C(i) asm volatile("v_sub_f32 %0, %0, %1" : "+v"(v[i]) : "v"(a));
            R16(C)
#undef C
        } else if (MODE == 5) {  // 16 x (v_cmp_gt_f32 -> vcc ; v_cndmask_b32 vcc) pairs, compiler-scheduled
#pragma unroll
            for (int c = 0; c < 16; ++c) v[c] = v[c] > a ? b : v[c];
        } else {  // 16 x v_cmp_gt_f32_e32 -> vcc
#define C(i) asm volatile("v_cmp_gt_f32_e32 vcc, %0, %1" : : "v"(v[i]), "v"(a) : "vcc");
            R16(C)
#undef C
        }
    }
    float sum = static_cast<float>(acc & 1);
#pragma unroll
    for (int c = 0; c < 16; ++c) sum += v[c];
    out[blockIdx.x * 1024 + threadIdx.x] = sum;
}

int main() {
    float *in, *out;
    hipMalloc(&in, 1024 * 4);
    hipMemset(in, 0, 1024 * 4);
    hipMalloc(&out, 1 << 22);
    int cus = 0;
    hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
    int clk = 0;
    hipDeviceGetAttribute(&clk, hipDeviceAttributeClockRate, 0);  // kHz
    const char* names[7] = {"cmp->sgpr", "cndmask", "max3", "bfi", "sub", "cmp+sel(cc)", "cmp->vcc"};
    for (int mode = 0; mode < 7; ++mode) {
        auto launch = [&]() {
            switch (mode) {
                case 0: hipLaunchKernelGGL(probe<0>, dim3(cus), dim3(1024), 0, 0, in, out); break;
                case 1: hipLaunchKernelGGL(probe<1>, dim3(cus), dim3(1024), 0, 0, in, out); break;
                case 2: hipLaunchKernelGGL(probe<2>, dim3(cus), dim3(1024), 0, 0, in, out); break;
                case 3: hipLaunchKernelGGL(probe<3>, dim3(cus), dim3(1024), 0, 0, in, out); break;
                case 4: hipLaunchKernelGGL(probe<4>, dim3(cus), dim3(1024), 0, 0, in, out); break;
                case 5: hipLaunchKernelGGL(probe<5>, dim3(cus), dim3(1024), 0, 0, in, out); break;
                default: hipLaunchKernelGGL(probe<6>, dim3(cus), dim3(1024), 0, 0, in, out); break;
            }
        };
        launch();
        hipEvent_t e0, e1;
        hipEventCreate(&e0);
        hipEventCreate(&e1);
        hipEventRecord(e0, 0);
        launch();
        hipEventRecord(e1, 0);
        hipEventSynchronize(e1);
        float ms = 0;
        hipEventElapsedTime(&ms, e0, e1);
        // per SIMD: 4 waves x kIters x 16 instructions (mode 5: x2)
        const double instr = 4.0 * kIters * 16 * (mode == 5 ? 2 : 1);
        const double cyc = ms * 1e-3 * 2.4e9;
        printf("%-12s %.3f ms -> %.2f cycles (at 2.4 GHz) per wave64 instr per SIMD (device clock %d kHz)\n",
               names[mode], ms, cyc / instr, clk);
    }
    return 0;
}
