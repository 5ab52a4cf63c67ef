// Microbenchmark: the split-f16 compute loop of hxs/hxt in isolation -- per 32-deep step 4
// ds_read_b64_tr_b16 (B hi, B lo) and 3 v_mfma_f32_16x16x32_f16 -- on W compute waves of a
// 16-wave workgroup (the other waves only join the barriers), one workgroup per CU.  Knobs: B
// lookahead (1 or 2 steps), barrier every G periods (0: none), NS steps per period.  Prints MFMA
// pipe utilisation of the busiest SIMD and the in-kernel clock.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

typedef _Float16 h8v __attribute__((ext_vector_type(8)));
typedef short s4v __attribute__((ext_vector_type(4)));
typedef short s8v __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) s4v* lds_s4p;

__device__ __forceinline__ h8v bFrag(uint32_t a) {
    const s4v lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s4p)(a));
    const s4v hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s4p)(a + 128));
    return __builtin_bit_cast(h8v, __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7));
}
__device__ __forceinline__ f32x4 mfma(h8v a, h8v b, f32x4 c) { return __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b, c, 0, 0, 0); }

template <int NS, int LOOK>
__global__ __launch_bounds__(1024) void k(float* out, unsigned long long* cyc, int W, int G, int nper, int Qc, int half) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    for (int i = threadIdx.x; i < 128 * 1024 / 4; i += blockDim.x)
        reinterpret_cast<float*>(smem)[i] = (float)((i * 2654435761u) >> 20) * 1e-4f;
    __syncthreads();
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, grp = lane >> 4, l16 = lane & 15;
    const uint32_t Rt = 2048, QS = 16 * Rt + 64;
    const uint32_t laneOff = (l16 & 3) * QS + 8u * (4 * grp + (l16 >> 2));
    const uint32_t dL = 8 * Rt;
    const uint32_t ring = static_cast<uint32_t>(reinterpret_cast<uintptr_t>((lds_s4p)smem)) + laneOff + 8u * (15 * (w % 12));
    h8v Ah[NS], Al[NS];
#pragma unroll
    for (int s = 0; s < NS; ++s)
#pragma unroll
        for (int i = 0; i < 8; ++i) { Ah[s][i] = (_Float16)(0.01f * (lane + i + s)); Al[s][i] = (_Float16)(0.001f * (i - s)); }
    f32x4 accA = {0, 0, 0, 0}, accL = accA;
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    const unsigned long long r0 = __builtin_amdgcn_s_memrealtime();
    const int ngroups = G > 0 ? nper / G : 1;
    const int perG = G > 0 ? G : nper;
    for (int g = 0; g < ngroups; ++g) {
        if (w < W) {
            uint32_t aH = ring + 8u * static_cast<uint32_t>((g % 3) * 588);
            for (int p = 0; p < perG; ++p) {
                if (w >= half && (p & 1)) continue;  // waves >= half: every 2nd period
                asm volatile("" : "+v"(aH));
                f32x4 nA = {0, 0, 0, 0}, nL = nA;
                h8v bh[LOOK + 1], bl[LOOK + 1];
#pragma unroll
                for (int d = 0; d < LOOK; ++d) { bh[d] = bFrag(aH + 256 * d); bl[d] = bFrag(aH + dL + 256 * d); }
#pragma unroll
                for (int s = 0; s < NS; ++s) {
                    if (s + LOOK < NS) { bh[(s + LOOK) % (LOOK + 1)] = bFrag(aH + 256 * (s + LOOK)); bl[(s + LOOK) % (LOOK + 1)] = bFrag(aH + dL + 256 * (s + LOOK)); }
                    nA = mfma(Ah[s], bh[s % (LOOK + 1)], nA);
                    nA = mfma(Al[s], bh[s % (LOOK + 1)], nA);
                    nL = mfma(Ah[s], bl[s % (LOOK + 1)], nL);
                    __builtin_amdgcn_sched_group_barrier(0x100, 4, 0);
                    __builtin_amdgcn_sched_group_barrier(0x008, 3, 0);
                    __builtin_amdgcn_sched_barrier(0);
                }
                accA += nA;
                accL += nL;
                aH += 8u * Qc;
            }
        }
        if (G > 0) {
            __atomic_signal_fence(__ATOMIC_SEQ_CST);
            __builtin_amdgcn_s_waitcnt(0xC07F);
            __builtin_amdgcn_s_barrier();
            __atomic_signal_fence(__ATOMIC_SEQ_CST);
        }
    }
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    const unsigned long long r1 = __builtin_amdgcn_s_memrealtime();
    out[blockIdx.x * blockDim.x + threadIdx.x] = accA[0] + accA[1] + accL[2] + accL[3];
    if (threadIdx.x == 0 && blockIdx.x == 0) { cyc[0] = t1 - t0; cyc[1] = r1 - r0; }
}

template <int NS, int LOOK>
void run(int W, int G, int nper, int half = 99) {
    float* out; unsigned long long* cyc;
    hipMalloc(&out, sizeof(float) * 1024 * 256);
    hipMalloc(&cyc, 16);
    hipFuncSetAttribute(reinterpret_cast<const void*>(&k<NS, LOOK>), hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    for (int rep = 0; rep < 3; ++rep) hipLaunchKernelGGL((k<NS, LOOK>), dim3(256), dim3(1024), 128 * 1024, 0, out, cyc, W, G, nper, 147, half);
    hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
    hipEventRecord(e0);
    hipLaunchKernelGGL((k<NS, LOOK>), dim3(256), dim3(1024), 128 * 1024, 0, out, cyc, W, G, nper, 147, half);
    hipEventRecord(e1); hipEventSynchronize(e1);
    float ms; hipEventElapsedTime(&ms, e0, e1);
    unsigned long long c[2]; hipMemcpy(c, cyc, 16, hipMemcpyDeviceToHost);
    // MFMAs on the busiest SIMD: waves w, w+4, w+8 share a SIMD -> ceil(W/4) waves
    const double perSimd = half < W ? (half / 4) + 0.5 * ((W - half) / 4) : (W + 3) / 4;
    const double mfma = 3.0 * NS * nper * perSimd;
    const double ghz = c[1] ? (double)c[0] / (double)c[1] / 10.0 : 0;  // memrealtime = 100 MHz
    printf("NS=%d look=%d W=%2d half>=%2d G=%d: busiest-SIMD MFMA util %.1f%% (loop %llu cyc, clock %.2f GHz, kernel %.3f ms)\n", NS, LOOK, W, half, G,
           100.0 * 16.0 * mfma / (double)c[0], c[0], ghz, ms);
    hipFree(out); hipFree(cyc);
}

int main() {
    const int nper = 88;
    run<9, 1>(12, 0, nper);
    run<9, 1>(12, 0, nper, 8);
    run<9, 1>(10, 0, 90);
    run<9, 1>(8, 0, nper);
    run<9, 1>(12, 4, nper, 8);
    run<9, 1>(12, 2, nper);
    run<9, 1>(12, 8, nper);
    run<9, 1>(12, 22, nper);
    run<9, 1>(16, 0, nper);
    run<9, 1>(16, 4, nper);
    return 0;
}
