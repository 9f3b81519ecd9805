// Store-pattern microbenchmark for the RoIPool forward's output (tools only).
// cfg2 shape: R = 2400 RoIs x C = 256 channels x 49 bins, out fp32 + argmax
// int32 (240.8 MB).  One wave per (RoI, 16-channel block); the block's 784
// elements per array are 3136 contiguous bytes (64-B aligned).  Patterns:
//   bin  : lane = bin (49 lanes), one dword store per channel (the kernel's)
//   row  : 64 lanes x dword, element 64*j + lane (13 instructions per array)
//   x4   : 64 lanes x dwordx4, chunk 64*j + lane (4 instructions per array)
//   x2   : 64 lanes x dwordx2, chunk 64*j + lane (7 instructions per array)
// Build: hipcc --offload-arch=gfx950 -O3 -o tools/prev/store_bench tools/store_bench.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

constexpr int R = 2400, C = 256, PHW = 49, CG = 16;

template <int MODE>
__global__ __launch_bounds__(256) void store_kernel(float* __restrict__ out, int* __restrict__ am, int seed) {
    const int wave = blockIdx.x * 4 + (threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    if (wave >= R * (C / CG)) return;
    const size_t blk = static_cast<size_t>(wave) * CG * PHW;  // 784 elements
    float* o = out + blk;
    int* a = am + blk;
    const float v = static_cast<float>(lane + seed);
    if (MODE == 0) {
        if (lane < PHW) {
#pragma unroll
            for (int c = 0; c < CG; ++c) {
                o[c * PHW + lane] = v + c;
                a[c * PHW + lane] = lane + c;
            }
        }
    } else if (MODE == 1) {
#pragma unroll
        for (int j = 0; j < 13; ++j) {
            const int e = 64 * j + lane;
            if (e < CG * PHW) {
                o[e] = v + j;
                a[e] = lane + j;
            }
        }
    } else if (MODE == 2) {
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int k = 64 * j + lane;
            if (k < CG * PHW / 4) {
                reinterpret_cast<float4*>(o)[k] = make_float4(v, v + 1, v + 2, v + j);
                reinterpret_cast<int4*>(a)[k] = make_int4(lane, j, lane, j);
            }
        }
    } else {
#pragma unroll
        for (int j = 0; j < 7; ++j) {
            const int k = 64 * j + lane;
            if (k < CG * PHW / 2) {
                reinterpret_cast<float2*>(o)[k] = make_float2(v, v + j);
                reinterpret_cast<int2*>(a)[k] = make_int2(lane, j);
            }
        }
    }
}

int main() {
    const size_t n = static_cast<size_t>(R) * C * PHW;
    float* out;
    int* am;
    if (hipMalloc(&out, n * 4) != hipSuccess || hipMalloc(&am, n * 4) != hipSuccess) return 1;
    const int waves = R * (C / CG);
    const dim3 grid((waves + 3) / 4), block(256);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    const char* names[4] = {"bin", "row", "x4", "x2"};
    for (int rnd = 0; rnd < 3; ++rnd) {
        for (int m = 0; m < 4; ++m) {
            auto launch = [&](int s) {
                if (m == 0) hipLaunchKernelGGL(store_kernel<0>, grid, block, 0, 0, out, am, s);
                else if (m == 1) hipLaunchKernelGGL(store_kernel<1>, grid, block, 0, 0, out, am, s);
                else if (m == 2) hipLaunchKernelGGL(store_kernel<2>, grid, block, 0, 0, out, am, s);
                else hipLaunchKernelGGL(store_kernel<3>, grid, block, 0, 0, out, am, s);
            };
            launch(0);
            hipEventRecord(e0, 0);
            for (int it = 0; it < 20; ++it) launch(it);
            hipEventRecord(e1, 0);
            hipEventSynchronize(e1);
            float ms = 0;
            hipEventElapsedTime(&ms, e0, e1);
            const double us = ms * 1e3 / 20;
            printf("round %d %-4s %8.2f us  %7.0f GB/s\n", rnd, names[m], us, 2.0 * n * 4 / (us * 1e-6) / 1e9);
        }
    }
    hipFree(out);
    hipFree(am);
    return 0;
}
