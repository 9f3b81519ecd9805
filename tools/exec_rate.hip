// VALU issue rate vs EXEC pattern (tools only): does a wave64 instruction cost
// less when whole 16-lane quarters (or a 32-lane half) are masked off?  Cycles
// per wave64 v_add_u32 / v_cndmask at 4 waves per SIMD (one 1024-thread
// workgroup per CU), 16 independent chains, executed under `if (mask bit of lane)`.
// Build: hipcc --offload-arch=gfx950 -O3 -o tools/prev/exec_rate tools/exec_rate.hip
#include <hip/hip_runtime.h>

#include <cstdio>

constexpr int kIters = 8192;

#define R16(X) X(0) X(1) X(2) X(3) X(4) X(5) X(6) X(7) X(8) X(9) X(10) X(11) X(12) X(13) X(14) X(15)

template <int MODE>
__global__ __launch_bounds__(1024) void probe(const unsigned* __restrict__ in, unsigned* __restrict__ out,
                                              unsigned long long mask) {
    unsigned v[16];
#pragma unroll
    for (int c = 0; c < 16; ++c) v[c] = in[(threadIdx.x * 16 + c) & 1023];
    unsigned a = in[threadIdx.x & 1023];
    const int lane = threadIdx.x & 63;
    long long t0 = 0, t1 = 0;
    if ((mask >> lane) & 1ull) {
        t0 = clock64();
        for (int it = 0; it < kIters; ++it) {
            if (MODE == 0) {
#define C(i) asm volatile("v_add_u32_e32 %0, %0, %1" : "+v"(v[i]) : "v"(a));
                R16(C)
#undef C
            } else {
#define C(i) asm volatile("v_cndmask_b32_e64 %0, %0, %1, s[0:1]" : "+v"(v[i]) : "v"(a));
                R16(C)
#undef C
            }
        }
        t1 = clock64();
    }
    unsigned sum = 0;
#pragma unroll
    for (int c = 0; c < 16; ++c) sum += v[c];
    out[blockIdx.x * 1024 + threadIdx.x] = sum + static_cast<unsigned>(t1 - t0);
}

int main() {
    unsigned *in, *out;
    hipMalloc(&in, 1024 * 4);
    hipMemset(in, 0, 1024 * 4);
    hipMalloc(&out, 1 << 22);
    int cus = 0;
    hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
    int khz = 0;
    hipDeviceGetAttribute(&khz, hipDeviceAttributeClockRate, 0);
    struct M { const char* name; unsigned long long m; };
    const M masks[] = {
        {"all 64", ~0ull},
        {"lanes 0-48 (49)", (1ull << 49) - 1},
        {"lanes 0-47 (48)", (1ull << 48) - 1},
        {"lanes 0-31 (32)", 0xFFFFFFFFull},
        {"lanes 0-15 (16)", 0xFFFFull},
        {"lane 0 (1)", 1ull},
        {"lanes 0,16,32,48 (4)", 0x0001000100010001ull},
        {"every other lane (32)", 0x5555555555555555ull},
        {"lanes 32-63 (32)", 0xFFFFFFFF00000000ull},
    };
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    for (int mode = 0; mode < 2; ++mode) {
        for (const M& mk : masks) {
            auto launch = [&]() {
                if (mode == 0) hipLaunchKernelGGL(probe<0>, dim3(cus), dim3(1024), 0, 0, in, out, mk.m);
                else hipLaunchKernelGGL(probe<1>, dim3(cus), dim3(1024), 0, 0, in, out, mk.m);
            };
            launch();
            hipDeviceSynchronize();
            hipEventRecord(e0);
            for (int r = 0; r < 5; ++r) launch();
            hipEventRecord(e1);
            hipEventSynchronize(e1);
            float ms = 0;
            hipEventElapsedTime(&ms, e0, e1);
            // per SIMD: 4 waves x kIters x 16 instructions
            const double ins = 4.0 * kIters * 16;
            const double cyc = ms / 5 * 1e-3 * khz * 1e3;
            printf("%-10s %-24s %.3f ms  %.2f cycles/instr (at %d MHz)\n", mode ? "cndmask" : "add_u32", mk.name,
                   ms / 5, cyc / ins, khz / 1000);
        }
    }
    return 0;
}
