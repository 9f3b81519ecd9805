// VALU issue-rate probe (tools only), second set: the forms of the ordered-key
// RoIPool scan.  Cycles per wave64 instruction at 4 waves per SIMD (one
// 1024-thread workgroup per CU), 16 independent chains per wave.
// Build: hipcc --offload-arch=gfx950 -O3 -o tools/prev/valu_rate2 tools/valu_rate2.hip
#include <hip/hip_runtime.h>

#include <cstdio>

constexpr int kIters = 8192;

#define R16(X) X(0) X(1) X(2) X(3) X(4) X(5) X(6) X(7) X(8) X(9) X(10) X(11) X(12) X(13) X(14) X(15)

template <int MODE>
__global__ __launch_bounds__(1024) void probe(const unsigned* __restrict__ in, unsigned* __restrict__ out) {
    unsigned v[16];
#pragma unroll
    for (int c = 0; c < 16; ++c) v[c] = in[(threadIdx.x * 16 + c) & 1023];
    unsigned a = in[threadIdx.x & 1023], b = in[(threadIdx.x + 7) & 1023];
    const unsigned m = __builtin_amdgcn_readfirstlane(in[3]) | 0xFFFFFC00u;
    for (int it = 0; it < kIters; ++it) {
        if (MODE == 0) {  // v_and_or_b32 (SGPR mask)
#define C(i) asm volatile("v_and_or_b32 %0, %0, %1, %2" : "+v"(v[i]) : "s"(m), "v"(a));
            R16(C)
#undef C
        } else if (MODE == 1) {  // v_max3_u32
#define C(i) asm volatile("v_max3_u32 %0, %0, %1, %2" : "+v"(v[i]) : "v"(a), "v"(b));
            R16(C)
#undef C
        } else if (MODE == 2) {  // v_max_u32_e32
#define C(i) asm volatile("v_max_u32_e32 %0, %0, %1" : "+v"(v[i]) : "v"(a));
            R16(C)
#undef C
        } else if (MODE == 3) {  // v_or_b32_e32
#define C(i) asm volatile("v_or_b32_e32 %0, %0, %1" : "+v"(v[i]) : "v"(a));
            R16(C)
#undef C
        } else if (MODE == 4) {  // v_max3_f32
#define C(i) asm volatile("v_max3_f32 %0, %0, %1, %2" : "+v"(v[i]) : "v"(a), "v"(b));
            R16(C)
#undef C
        } else if (MODE == 5) {  // v_bitop3_b32
#define C(i) asm volatile("v_bitop3_b32 %0, %0, %1, %2 bitop3:0xec" : "+v"(v[i]) : "v"(a), "v"(b));
            R16(C)
#undef C
        } else if (MODE == 6) {  // v_pk_add_u16 (VOP3P)
#define C(i) asm volatile("v_pk_max_u16 %0, %0, %1" : "+v"(v[i]) : "v"(a));
            R16(C)
#undef C
        } else {  // v_add_u32_e32
#define C(i) asm volatile("v_add_u32_e32 %0, %0, %1" : "+v"(v[i]) : "v"(a));
            R16(C)
#undef C
        }
    }
    unsigned sum = 0;
#pragma unroll
    for (int c = 0; c < 16; ++c) sum += v[c];
    out[blockIdx.x * 1024 + threadIdx.x] = sum;
}

int main() {
    unsigned *in, *out;
    hipMalloc(&in, 1024 * 4);
    hipMemset(in, 0, 1024 * 4);
    hipMalloc(&out, 1 << 22);
    int cus = 0;
    hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
    const char* names[8] = {"and_or", "max3_u32", "max_u32_e32", "or_e32", "max3_f32", "bitop3", "pk_max_u16", "add_u32_e32"};
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
        hipEvent_t e0, e1;
        hipEventCreate(&e0);
        hipEventCreate(&e1);
        hipEventRecord(e0, 0);
        launch();
        hipEventRecord(e1, 0);
        hipEventSynchronize(e1);
        float ms = 0;
        hipEventElapsedTime(&ms, e0, e1);
        const double instr = 4.0 * kIters * 16;  // per SIMD: 4 waves x kIters x 16
        printf("%-12s %.3f ms -> %.2f cycles (at 2.4 GHz) per wave64 instr per SIMD\n", names[mode], ms,
               ms * 1e-3 * 2.4e9 / instr);
    }
    return 0;
}
