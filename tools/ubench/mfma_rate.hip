// Microbenchmark: v_mfma_f32_16x16x32_f16 issue rate per SIMD (independent vs
// dependent accumulators, 1-3 waves per SIMD).  Prints cycles per MFMA per SIMD.
#include <hip/hip_runtime.h>
#include <cstdio>
typedef _Float16 h8v __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

template <int NACC>
__global__ void k(float* out, long long* cyc, int iters) {
    h8v a, b;
    for (int i = 0; i < 8; ++i) { a[i] = (_Float16)(threadIdx.x * 0.001f + i); b[i] = (_Float16)(i * 0.5f); }
    f32x4 acc[NACC];
    for (int j = 0; j < NACC; ++j) acc[j] = f32x4{0, 0, 0, 0};
    __syncthreads();
    long long t0 = wall_clock64();
    long long c0 = clock64();
    for (int it = 0; it < iters; ++it) {
#pragma unroll
        for (int r = 0; r < 16; ++r)
#pragma unroll
            for (int j = 0; j < NACC; ++j) acc[j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b, acc[j], 0, 0, 0);
    }
    long long c1 = clock64();
    long long t1 = wall_clock64();
    float s = 0;
    for (int j = 0; j < NACC; ++j) s += acc[j][0] + acc[j][1] + acc[j][2] + acc[j][3];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
    if (threadIdx.x == 0 && blockIdx.x == 0) { cyc[0] = c1 - c0; cyc[1] = t1 - t0; }
}

template <int NACC>
void run(int waves, int blocks, int iters) {
    float* out; long long* cyc;
    hipMalloc(&out, sizeof(float) * 64 * waves * blocks);
    hipMalloc(&cyc, 16);
    hipLaunchKernelGGL(k<NACC>, dim3(blocks), dim3(64 * waves), 0, 0, out, cyc, iters);
    hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
    hipEventRecord(e0);
    hipLaunchKernelGGL(k<NACC>, dim3(blocks), dim3(64 * waves), 0, 0, out, cyc, iters);
    hipEventRecord(e1); hipEventSynchronize(e1);
    float ms; hipEventElapsedTime(&ms, e0, e1);
    long long c[2]; hipMemcpy(c, cyc, 16, hipMemcpyDeviceToHost);
    const double mfmaPerWave = 16.0 * NACC * iters;
    const double wavesPerSimd = waves / 4.0;
    printf("nacc=%d waves/WG=%d blocks=%d: clock64 cycles/MFMA/SIMD=%.2f  (kernel %.3f ms, %.1f TFLOP/s f16)\n", NACC, waves, blocks,
           c[0] / (mfmaPerWave * wavesPerSimd), ms,
           2.0 * 16 * 16 * 32 * mfmaPerWave * waves * blocks / (ms * 1e-3) / 1e12);
    hipFree(out); hipFree(cyc);
}

int main() {
    run<1>(4, 256, 256);
    run<2>(4, 256, 256);
    run<4>(4, 256, 256);
    run<4>(8, 256, 256);
    run<4>(12, 256, 256);
    run<4>(10, 256, 256);
    run<1>(12, 256, 256);
    return 0;
}
