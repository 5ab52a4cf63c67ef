// launch_floor.hip -- the per-launch floor of small kernels on this GPU: back-to-back launches of
// (a) an empty kernel, (b) one HBM round trip per thread, (c) four dependent round trips, (d) a
// 1024-thread / 56 KB-LDS workgroup doing one round trip + a barrier (the hxs small-launch shape).
// hipcc --offload-arch=gfx950 -O3 launch_floor.hip -o launch_floor && ./launch_floor
#include <hip/hip_runtime.h>
#include <cstdio>

__global__ void k_empty(float* o) { if (threadIdx.x == 12345) o[0] = 1.f; }
__global__ void k_one(const float* __restrict__ x, float* o, int n) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    const float v = x[(i * 97) % n];
    if (v == 12345.f) o[0] = v;
}
__global__ void k_chain(const int* __restrict__ x, float* o, int n) {
    int j = (blockIdx.x * blockDim.x + threadIdx.x) % n;
    for (int k = 0; k < 4; ++k) j = x[j];
    if (j == 12345) o[0] = 1.f;
}
__global__ __launch_bounds__(1024) void k_lds(const float* __restrict__ x, float* o, int n) {
    extern __shared__ float sm[];
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    sm[threadIdx.x] = x[(i * 97) % n];
    __syncthreads();
    const float v = sm[(threadIdx.x + 1) % blockDim.x];
    o[i] = v;
}

typedef double f64x4 __attribute__((ext_vector_type(4)));
// 40 f64 MFMAs on two alternating accumulators (the bg_rb_kernel program shape), A/B from registers
__global__ void k_mfma64(const double* __restrict__ x, double* o) {
    const int lane = threadIdx.x & 63;
    double a[40], b[40];
#pragma unroll
    for (int s = 0; s < 40; ++s) { a[s] = x[s * 64 + lane]; b[s] = x[4096 + s * 64 + lane]; }
    f64x4 c0 = {0, 0, 0, 0}, c1 = c0;
#pragma unroll
    for (int s = 0; s < 40; ++s) {
        if (s & 1) c1 = __builtin_amdgcn_mfma_f64_16x16x4f64(a[s], b[s], c1, 0, 0, 0);
        else c0 = __builtin_amdgcn_mfma_f64_16x16x4f64(a[s], b[s], c0, 0, 0, 0);
    }
    const f64x4 r = c0 + c1;
    o[(blockIdx.x * blockDim.x + threadIdx.x) * 4] = r[0] + r[1] + r[2] + r[3];
}

#define CK(e) do { if ((e) != hipSuccess) { printf("HIP error %s line %d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)
int main() {
    const int n = 1 << 24;
    float *x, *o;
    int* xi;
    CK(hipMalloc(&x, n * 4)); CK(hipMalloc(&xi, n * 4)); CK(hipMalloc(&o, n * 4));
    int* h = new int[n];
    for (int i = 0; i < n; ++i) h[i] = static_cast<int>((static_cast<long long>(i) * 7919 + 13) % n);
    CK(hipMemcpy(xi, h, n * 4, hipMemcpyHostToDevice));
    CK(hipMemset(x, 0, n * 4));
    CK(hipFuncSetAttribute(reinterpret_cast<const void*>(&k_lds), hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
    hipEvent_t a, b;
    CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
    const int R = 2000;
    for (int blocks : {4, 80, 256}) {
        for (int kind = 0; kind < 5; ++kind) {
            for (int rep = 0; rep < 2; ++rep) {
                CK(hipEventRecord(a, 0));
                for (int r = 0; r < R; ++r) {
                    if (kind == 0) hipLaunchKernelGGL(k_empty, dim3(blocks), dim3(256), 0, 0, o);
                    else if (kind == 1) hipLaunchKernelGGL(k_one, dim3(blocks), dim3(256), 0, 0, x, o, n);
                    else if (kind == 2) hipLaunchKernelGGL(k_chain, dim3(blocks), dim3(256), 0, 0, xi, o, n);
                    else if (kind == 3) hipLaunchKernelGGL(k_lds, dim3(blocks), dim3(1024), 56 * 1024, 0, x, o, n);
                    else hipLaunchKernelGGL(k_mfma64, dim3(blocks), dim3(128), 0, 0, reinterpret_cast<const double*>(x), reinterpret_cast<double*>(o));
                }
                CK(hipEventRecord(b, 0));
                CK(hipEventSynchronize(b));
                float ms = 0;
                CK(hipEventElapsedTime(&ms, a, b));
                if (rep == 1)
                    printf("{\"blocks\": %d, \"kernel\": \"%s\", \"us_per_launch\": %.2f}\n", blocks,
                           kind == 0 ? "empty" : kind == 1 ? "one_round_trip" : kind == 2 ? "four_dependent_round_trips" : kind == 3 ? "1024thr_56KB_lds_barrier" : "f64_mfma_x40_2acc_128thr",
                           ms * 1000.0 / R);
            }
        }
    }
    return 0;
}
