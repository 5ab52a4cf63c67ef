// Microbenchmark: the hxs_kernel compute-wave pattern in isolation (no loads, no conversion).
// 256 workgroups x (NC compute + NL idle waves); a compute wave holds A (9 steps x hi/lo
// f16x8) in registers, runs 88 periods of 9 steps x 3 v_mfma_f32_16x16x32_f16 over B
// fragments read from LDS with ds_read_b64_tr_b16 (one step ahead), and per period stores
// 1 KiB of outputs in cfg2's stereo pattern (8 chunks x 128 B); every G periods all waves
// meet at s_barrier.  Variants (template MODE):
//   0 no stores                 1 store after the period's 2nd step (hxs_kernel today)
//   2 store after the period    3 non-temporal store after the 2nd step
//   4 results to LDS, the idle waves store them after the barrier (compute waves: ds_write)
// hipcc --offload-arch=gfx950 -O3 mfma_store.hip -o mfma_store && ./mfma_store
#include <hip/hip_runtime.h>

#include <cstdio>

typedef _Float16 h8v __attribute__((ext_vector_type(8)));
typedef short s4v __attribute__((ext_vector_type(4)));
typedef short s8v __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) s4v* lds_s4p;

constexpr int kNS = 9, kPeriods = 88, kChunks = 8, kPeriodB = 1280;
constexpr long long kChunkB = (long long)kPeriods * kPeriodB;

__device__ __forceinline__ h8v bfrag(uint32_t a) {
    const s4v lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s4p)(a));
    const s4v hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s4p)(a + 128));
    return __builtin_bit_cast(h8v, __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7));
}
__device__ __forceinline__ f32x4 mfma(h8v a, h8v b, f32x4 c) {
    return __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b, c, 0, 0, 0);
}
__device__ __forceinline__ void bar() {
    __builtin_amdgcn_s_waitcnt(0xC07F);
    __builtin_amdgcn_s_barrier();
}

template <int MODE, int NC, int G>
__global__ __launch_bounds__(1024) void k(const h8v* Aimg, char* out) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, nw = blockDim.x >> 6;
    char* blk = out + (long long)blockIdx.x * kChunks * kChunkB;
    const int ngroups = (kPeriods + G - 1) / G;
    float* stage = reinterpret_cast<float*>(smem + 96 * 1024);  // MODE 4: [G][NC][64][4]
    if (w < NC) {
        h8v Ah[kNS], Al[kNS];
#pragma unroll
        for (int s = 0; s < kNS; ++s) {
            Ah[s] = Aimg[(w * kNS + s) * 2 * 64 + lane];
            Al[s] = Aimg[((w * kNS + s) * 2 + 1) * 64 + lane];
        }
        const int grp = lane >> 4, l16 = lane & 15;
        const uint32_t base = (uint32_t)(uintptr_t)(lds_s4p)smem + (l16 & 3) * (16384u + 64u) + 8u * (4 * grp + (l16 >> 2));
        const int ck = l16 >> 1, off = (grp * 2 + (lane & 1)) * 16;
        f32x4 pA = {0, 0, 0, 0}, pL = pA;  // previous period's accumulators (MODE 1/3: stored mid-period)
        h8v breg[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) breg[j] = Ah[j] * (_Float16)0.5f;
        for (int gi = 0; gi < ngroups; ++gi) {
            for (int pp = 0; pp < G; ++pp) {
                const int p = gi * G + pp;
                if (p >= kPeriods) break;
                uint32_t a = base + 1176u * (uint32_t)(p % 8);
                asm volatile("" : "+v"(a));
                f32x4 accA = {0, 0, 0, 0}, accL = accA;
                if (MODE == 5) {  // no LDS: B from registers (opaque per period)
#pragma unroll
                    for (int j = 0; j < 4; ++j) asm volatile("" : "+v"(breg[j]));
#pragma unroll
                    for (int s = 0; s < kNS; ++s) {
                        accA = mfma(Ah[s], breg[s & 3], accA);
                        accA = mfma(Al[s], breg[s & 3], accA);
                        accL = mfma(Ah[s], breg[(s + 1) & 3], accL);
                    }
                } else if (MODE == 7) {  // ds_read_b128 per fragment (column-major image), 1 step ahead
                    typedef __attribute__((address_space(3))) h8v* lds_h8p;
                    const uint32_t cb = (uint32_t)(uintptr_t)(lds_s4p)smem + (uint32_t)lane * 16u + 1024u * (uint32_t)(p % 8);
                    h8v bh = *(lds_h8p)(cb), bl = *(lds_h8p)(cb + 32768);
#pragma unroll
                    for (int s = 0; s < kNS; ++s) {
                        h8v bh1 = bh, bl1 = bl;
                        if (s + 1 < kNS) { bh1 = *(lds_h8p)(cb + 1024 * (s + 1)); bl1 = *(lds_h8p)(cb + 32768 + 1024 * (s + 1)); }
                        accA = mfma(Ah[s], bh, accA);
                        accA = mfma(Al[s], bh, accA);
                        accL = mfma(Ah[s], bl, accL);
                        bh = bh1; bl = bl1;
                    }
                } else if (MODE == 8) {  // tr reads 3 steps ahead
                    h8v bh[4], bl[4];
#pragma unroll
                    for (int j = 0; j < 3; ++j) { bh[j] = bfrag(a + 256 * j); bl[j] = bfrag(a + 8192 + 256 * j); }
#pragma unroll
                    for (int s = 0; s < kNS; ++s) {
                        if (s + 3 < kNS) { bh[(s + 3) & 3] = bfrag(a + 256 * (s + 3)); bl[(s + 3) & 3] = bfrag(a + 8192 + 256 * (s + 3)); }
                        accA = mfma(Ah[s], bh[s & 3], accA);
                        accA = mfma(Al[s], bh[s & 3], accA);
                        accL = mfma(Ah[s], bl[s & 3], accL);
                    }
                } else if (MODE == 6) {  // B two steps ahead
                    h8v bh0 = bfrag(a), bl0 = bfrag(a + 8192), bh1 = bfrag(a + 256), bl1 = bfrag(a + 8192 + 256);
#pragma unroll
                    for (int s = 0; s < kNS; ++s) {
                        h8v bh2 = bh1, bl2 = bl1;
                        if (s + 2 < kNS) { bh2 = bfrag(a + 256 * (s + 2)); bl2 = bfrag(a + 8192 + 256 * (s + 2)); }
                        accA = mfma(Ah[s], bh0, accA);
                        accA = mfma(Al[s], bh0, accA);
                        accL = mfma(Ah[s], bl0, accL);
                        bh0 = bh1; bl0 = bl1; bh1 = bh2; bl1 = bl2;
                    }
                } else {
                    h8v bh = bfrag(a), bl = bfrag(a + 8192);
#pragma unroll
                    for (int s = 0; s < kNS; ++s) {
                        h8v bh1 = bh, bl1 = bl;
                        if (s + 1 < kNS) { bh1 = bfrag(a + 256 * (s + 1)); bl1 = bfrag(a + 8192 + 256 * (s + 1)); }
                        accA = mfma(Ah[s], bh, accA);
                        accA = mfma(Al[s], bh, accA);
                        accL = mfma(Ah[s], bl, accL);
                        bh = bh1; bl = bl1;
                        if (s == 1 && (MODE == 1 || MODE == 3) && p > 0) {  // the previous period's outputs
                            const f32x4 y = pA + pL * 0.00048828125f;
                            f32x4* dst = reinterpret_cast<f32x4*>(blk + ck * kChunkB + (long long)(p - 1) * kPeriodB + w * 128 + off);
                            if (MODE == 3) __builtin_nontemporal_store(y, dst);
                            else *dst = y;
                        }
                    }
                }
                pA = accA;
                pL = accL;
                const f32x4 y = accA + accL * 0.00048828125f;
                if (MODE == 0 || MODE >= 5 || MODE == 1 || MODE == 3) {
                    if (y[0] == 123.f) *reinterpret_cast<f32x4*>(blk + lane * 16) = y;
                } else if (MODE == 2) {
                    *reinterpret_cast<f32x4*>(blk + ck * kChunkB + (long long)p * kPeriodB + w * 128 + off) = y;
                } else if (MODE == 4) {
                    *reinterpret_cast<f32x4*>(stage + ((pp * NC + w) * 64 + lane) * 4) = y;
                }
            }
            bar();
            if (MODE == 4) bar();  // the store waves read the staged group
        }
    } else {
        const int l = w - NC, nl = nw - NC;
        for (int gi = 0; gi < ngroups; ++gi) {
            bar();
            if (MODE == 4) {
                // group gi's results: G periods x NC row blocks x 1 KiB
                for (int it = l; it < G * NC; it += nl) {
                    const int pp = it / NC, rw = it % NC, p = gi * G + pp;
                    if (p >= kPeriods) continue;
                    const int grp = lane >> 4, l16 = lane & 15;
                    const int ck = l16 >> 1, off = (grp * 2 + (lane & 1)) * 16;
                    const f32x4 y = *reinterpret_cast<const f32x4*>(stage + ((pp * NC + rw) * 64 + lane) * 4);
                    *reinterpret_cast<f32x4*>(blk + ck * kChunkB + (long long)p * kPeriodB + rw * 128 + off) = y;
                }
                bar();
            }
        }
    }
}

int main() {
    const long long bytes = 256LL * kChunks * kChunkB;
    char* out;
    h8v* A;
    if (hipMalloc(&out, bytes) != hipSuccess || hipMalloc(&A, 16 * kNS * 2 * 64 * sizeof(h8v)) != hipSuccess) return 1;
    (void)hipMemset(A, 0x11, 16 * kNS * 2 * 64 * sizeof(h8v));
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    auto run = [&](auto kern, int nwaves, const char* name) {
        (void)hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
        for (int i = 0; i < 3; ++i) hipLaunchKernelGGL(kern, dim3(256), dim3(64 * nwaves), 160 * 1024, 0, A, out);
        (void)hipEventRecord(e0);
        for (int i = 0; i < 20; ++i) hipLaunchKernelGGL(kern, dim3(256), dim3(64 * nwaves), 160 * 1024, 0, A, out);
        (void)hipEventRecord(e1);
        (void)hipEventSynchronize(e1);
        float ms;
        (void)hipEventElapsedTime(&ms, e0, e1);
        printf("%-44s %8.1f us\n", name, ms / 20 * 1e3);
    };
    run(k<0, 10, 5>, 16, "10c+6 G5 no stores");
    run(k<1, 10, 5>, 16, "10c+6 G5 store prev period mid-stream");
    run(k<2, 10, 5>, 16, "10c+6 G5 store end of period");
    run(k<3, 10, 5>, 16, "10c+6 G5 NT store prev period mid-stream");
    run(k<4, 10, 5>, 16, "10c+6 G5 LDS-staged, idle waves store");
    run(k<5, 10, 5>, 16, "10c+6 G5 no LDS reads (B in regs)");
    run(k<5, 4, 5>, 16, "4c+12 G5 no LDS reads");
    run(k<5, 8, 5>, 16, "8c+8 G5 no LDS reads");
    run(k<5, 12, 5>, 16, "12c+4 G5 no LDS reads");
    run(k<6, 10, 5>, 16, "10c+6 G5 B 2 steps ahead");
    run(k<8, 10, 5>, 16, "10c+6 G5 B 3 steps ahead");
    run(k<7, 10, 5>, 16, "10c+6 G5 ds_read_b128 1 ahead");
    run(k<7, 4, 5>, 16, "4c+12 G5 ds_read_b128 1 ahead");
    run(k<8, 4, 5>, 16, "4c+12 G5 tr 3 ahead");
    run(k<6, 4, 5>, 16, "4c+12 G5 tr 2 ahead");
    run(k<0, 8, 5>, 16, "8c+8 G5 no stores (8 row blocks)");
    run(k<0, 4, 5>, 16, "4c+12 G5 no stores");
    run(k<0, 12, 5>, 16, "12c+4 G5 no stores (12 row blocks)");
    run(k<0, 10, 88>, 16, "10c+6 no barriers no stores");
    run(k<5, 10, 88>, 16, "10c+6 no barriers no LDS");
    (void)hipFree(out);
    (void)hipFree(A);
    return 0;
}
