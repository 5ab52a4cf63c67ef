// Microbenchmark: ds_read_b64_tr_b16 throughput per CU with the hx image
// pattern (quad-major, QS = 16*Ws + 64, lane offset (l16&3)*QS + 8*(4*grp + (l16>>2)),
// step +256 B), vs plain ds_read_b64.  Prints bytes per clock per CU.
#include <hip/hip_runtime.h>
#include <cstdio>
typedef short s4v __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) s4v* lds_s4p;

template <int TR, int DEPTH>
__global__ void k(float* out, int iters, int Ws) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    for (int i = threadIdx.x; i < 16 * 1024 * 4 / 4 + 1024; i += blockDim.x) reinterpret_cast<float*>(smem)[i] = 0.f;
    __syncthreads();
    const int lane = threadIdx.x & 63, grp = lane >> 4, l16 = lane & 15;
    const unsigned QS = 16u * Ws + 64u;
    const unsigned base = (unsigned)(size_t)(lds_s4p)smem + (l16 & 3) * QS + 8u * (4 * grp + (l16 >> 2)) + 512u * (threadIdx.x >> 6);
    s4v acc = {0, 0, 0, 0};
    for (int it = 0; it < iters; ++it) {
        s4v v[DEPTH];
#pragma unroll
        for (int d = 0; d < DEPTH; ++d) {
            const unsigned a = base + 256u * ((it * DEPTH + d) & 15);
            if (TR) v[d] = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s4p)a);
            else v[d] = *(lds_s4p)a;
        }
#pragma unroll
        for (int d = 0; d < DEPTH; ++d) acc += v[d];
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = acc[0] + acc[1] + acc[2] + acc[3];
}

template <int TR, int DEPTH>
void run(int waves, int iters) {
    float* out; hipMalloc(&out, sizeof(float) * 64 * waves * 256);
    const size_t lds = 16 * 1024 * 4 + 4096;
    hipFuncSetAttribute(reinterpret_cast<const void*>(&k<TR, DEPTH>), hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    hipLaunchKernelGGL((k<TR, DEPTH>), dim3(256), dim3(64 * waves), lds, 0, out, iters, 1024);
    hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
    hipEventRecord(e0);
    hipLaunchKernelGGL((k<TR, DEPTH>), dim3(256), dim3(64 * waves), lds, 0, out, iters, 1024);
    hipEventRecord(e1); hipEventSynchronize(e1);
    float ms; hipEventElapsedTime(&ms, e0, e1);
    const double bytes = 512.0 * DEPTH * iters * waves;  // per CU
    printf("tr=%d depth=%d waves=%d: %.1f B/clk/CU at 2.1 GHz (%.3f ms)\n", TR, DEPTH, waves, bytes / (ms * 1e-3 * 2.1e9), ms);
    hipFree(out);
}

int main() {
    run<1, 4>(10, 4096);
    run<1, 8>(10, 2048);
    run<1, 16>(10, 1024);
    run<1, 8>(4, 4096);
    run<1, 8>(16, 1024);
    run<0, 8>(10, 2048);
    return 0;
}
