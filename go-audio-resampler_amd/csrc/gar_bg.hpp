// gar_bg.hpp -- the banded-GEMM MFMA FIR kernel template (included by the
// per-dtype instantiation units gar_bg_*.hip and by gar_kernels.hip).
#pragma once
#include <hip/hip_runtime.h>

#include <algorithm>

#include "gar_kernels.hpp"

namespace gar {

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef double f64x4 __attribute__((ext_vector_type(4)));

template <class TC>
__device__ __forceinline__ TC srcRead(const SrcDesc& s, int64_t t, int c) {
    if (t < 0 || t >= s.valid_end) return TC(0);
    const int64_t h = t - s.hist_base;
    if (h >= 0 && h < s.hist_len) return s.hist ? static_cast<const TC*>(s.hist)[h * s.hist_ld + c] : TC(0);
    const int64_t i = t - s.in_base;
    if (i >= 0 && i < s.in_len) {
        const int64_t e = i * s.in_fs + static_cast<int64_t>(c) * s.in_cs;
        return s.in_f64 ? static_cast<TC>(static_cast<const double*>(s.in)[e])
                        : static_cast<TC>(static_cast<const float*>(s.in)[e]);
    }
    return TC(0);
}

template <class TC>
__device__ __forceinline__ void outWrite(const OutDesc& o, int64_t idx, int c, TC v) {
    if (idx < o.o_lo || idx >= o.o_hi) return;
    const int64_t e = (idx - o.o0) * o.fs + static_cast<int64_t>(c) * o.cs;
    if (o.f64) static_cast<double*>(o.out)[e] = static_cast<double>(v);
    else static_cast<float*>(o.out)[e] = static_cast<float>(v);
}

// ---------------------------------------------------------------------------
// Banded GEMM.  Geometry (host computed in launchBg):
//   macro period a covers outputs [a*Pc, (a+1)*Pc) and reads inputs starting
//   at a*Qc; a column = (channel c, chunk of G consecutive macro periods);
//   the workgroup owns 16*ncg columns and stages each column's window of
//   W = Kc + (G-1)*Qc inputs in LDS (row stride Ws == 2 mod 32 so the 16x4
//   B-fragment read is bank-conflict free).  Wave (cg, wt) runs tasks
//   wt, wt+nwt, ... ; a task is one 16-row block (optionally one K slice).
// ---------------------------------------------------------------------------
struct BgGrid {
    int Pc, Qc, Kc, W, Ws, G;
    int64_t a_lo;
    int nchunk, ncols, nblocks;
    int C, ntasks, nwt, ncg, ksplit, chan_fast, R;
};

template <class TC> struct Acc;
template <> struct Acc<float> {
    typedef f32x4 V;
    static __device__ __forceinline__ V mfma(float a, float b, V c) {
        return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
    }
    // C/D map of the 16x16 f32 MFMA: col = lane&15, row = 4*(lane>>4) + i
    static __device__ __forceinline__ int row(int lane, int i) { return 4 * (lane >> 4) + i; }
};
template <> struct Acc<double> {
    typedef f64x4 V;
    static __device__ __forceinline__ V mfma(double a, double b, V c) {
        return __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c, 0, 0, 0);
    }
    // f64 MFMA C/D map differs: col = lane&15, row = (lane>>4) + 4*i
    static __device__ __forceinline__ int row(int lane, int i) { return (lane >> 4) + 4 * i; }
};

__device__ __forceinline__ int uni(int v) { return __builtin_amdgcn_readfirstlane(v); }

// Input element kk of column `col`'s window (column = channel c, chunk of G
// macro periods).  Fast path when the whole window lies in one buffer.
typedef __attribute__((address_space(3))) void* lds_ptr_t;
typedef __attribute__((address_space(1))) const void* gbl_ptr_t;

// Column window source: direct pointer to element kk=0 when the whole window
// lies in one buffer of the compute dtype (LDS-DMA eligible), else gathered.
template <class TC>
struct ColSrc {
    const TC* p;
    int64_t stride;
    int64_t t0;
    int c;
    bool ok;
};

template <class TC>
__device__ __forceinline__ ColSrc<TC> colSrc(const SrcDesc& s, const BgGrid& g, int col) {
    ColSrc<TC> r;
    r.ok = col < g.ncols;
    r.c = r.ok ? col % g.C : 0;
    const int chunk = r.ok ? col / g.C : 0;
    r.t0 = (g.a_lo + static_cast<int64_t>(chunk) * g.G) * g.Qc;
    r.p = nullptr;
    r.stride = 0;
    const int64_t t1 = r.t0 + g.W;
    const bool inSame = (s.in_f64 != 0) == (sizeof(TC) == 8);
    if (r.ok && t1 <= s.valid_end) {
        if (inSame && s.in && r.t0 >= s.in_base && t1 <= s.in_base + s.in_len) {
            r.p = static_cast<const TC*>(s.in) + (r.t0 - s.in_base) * s.in_fs + static_cast<int64_t>(r.c) * s.in_cs;
            r.stride = s.in_fs;
        } else if (s.hist && r.t0 >= s.hist_base && t1 <= s.hist_base + s.hist_len) {
            r.p = static_cast<const TC*>(s.hist) + (r.t0 - s.hist_base) * s.hist_ld + r.c;
            r.stride = s.hist_ld;
        }
    }
    return r;
}

// LDS tile of one column group: [WR][16] elements (WR = W rounded up so every
// DMA piece is whole); a workgroup holds ncg such sub-tiles per buffer.
// One LDS-DMA wave instruction (global_load_lds_dword) moves one piece =
// 64 dwords = 4 rows x 16 columns (f32) or 2 rows x 16 columns (f64): lane l
// writes dword l of the piece, so the LDS image is lane-linear as the DMA
// requires; each lane fetches from its own column's global address.
template <class TC>
__device__ __forceinline__ void loadTile(const SrcDesc& src, const BgGrid& g, int b, TC* sub, int cg, int wt,
                                         int lane) {
    constexpr int rowsPerPiece = sizeof(TC) == 8 ? 2 : 4;
    const int n = sizeof(TC) == 8 ? ((lane >> 1) & 15) : (lane & 15);
    const int rsub = sizeof(TC) == 8 ? (lane >> 5) : (lane >> 4);
    const int half = sizeof(TC) == 8 ? (lane & 1) : 0;
    const ColSrc<TC> cs = colSrc<TC>(src, g, b * 16 * g.ncg + cg * 16 + n);
    const bool fast = cs.p != nullptr;
    const bool allFast = __all(fast);
    const int npieces = (g.W + rowsPerPiece - 1) / rowsPerPiece;
    for (int j = wt; j < npieces; j += g.nwt) {
        int kk = j * rowsPerPiece + rsub;
        TC* dst = sub + static_cast<size_t>(j) * rowsPerPiece * 16;
        if (allFast) {
            const int kc = kk < g.W ? kk : g.W - 1;
            const char* gp = reinterpret_cast<const char*>(cs.p + kc * cs.stride) + half * 4;
            __builtin_amdgcn_global_load_lds((gbl_ptr_t)gp, (lds_ptr_t)dst, 4, 0, 0);
        } else {
            // boundary block: gather (history / input / flush zeros, dtype conversion)
            if (half == 0) {
                TC v = TC(0);
                if (kk < g.W && cs.ok) v = fast ? cs.p[kk * cs.stride] : srcRead<TC>(src, cs.t0 + kk, cs.c);
                dst[rsub * 16 + n] = v;
            }
        }
    }
}

// prefetch-free kernel: tiles arrive by LDS-DMA while the previous block computes
template <class TC> struct BgCfg;
template <> struct BgCfg<float> { static constexpr int kMaxThreads = 640; };
template <> struct BgCfg<double> { static constexpr int kMaxThreads = 512; };

template <class TC, int NS, bool GLOBAL_B, bool SINGLE>
__global__ __launch_bounds__(BgCfg<TC>::kMaxThreads) void bg_kernel(BgDev p, SrcDesc src, OutDesc od, BgGrid g) {
    typedef typename Acc<TC>::V V;
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    const int subElems = g.Ws * 16;                           // one column group's sub-tile
    const int tileElems = GLOBAL_B ? 0 : subElems * g.ncg;
    TC* tiles = reinterpret_cast<TC*>(smem);                 // [2][ncg][Ws][16]
    TC* part = tiles + 2 * static_cast<size_t>(tileElems);   // k-split partials [ncg][ntasks][256]

    const int lane = threadIdx.x & 63;
    const int wave = threadIdx.x >> 6;
    const int cg = wave / g.nwt;
    const int wt = wave - cg * g.nwt;
    const int nloc = cg * 16 + (lane & 15);
    const TC* Aimg = static_cast<const TC*>(p.A);

    TC A[NS];
    if (SINGLE && wt < g.ntasks) {
#pragma unroll
        for (int s = 0; s < NS; ++s) A[s] = Aimg[(static_cast<size_t>(wt) * NS + s) * 64 + lane];
    }

    int b = blockIdx.x;
    if (!GLOBAL_B && b < g.nblocks) loadTile<TC>(src, g, b, tiles + cg * subElems, cg, wt, lane);
    for (int it = 0; b < g.nblocks; b += gridDim.x, ++it) {
        TC* tile = tiles + static_cast<size_t>(it & 1) * tileElems + cg * subElems;
        __syncthreads();  // waits for this tile's DMA (vmcnt) + frees the other buffer
        const int bn = b + gridDim.x;
        if (!GLOBAL_B && bn < g.nblocks)
            loadTile<TC>(src, g, bn, tiles + static_cast<size_t>((it + 1) & 1) * tileElems + cg * subElems, cg, wt, lane);

        const int col = b * 16 * g.ncg + nloc;
        const bool colOk = col < g.ncols;
        const int c = colOk ? col % g.C : 0;
        const int chunk = colOk ? col / g.C : 0;

        for (int gi = 0; gi < g.G; ++gi) {
            const int64_t a = g.a_lo + static_cast<int64_t>(chunk) * g.G + gi;
            for (int t = wt; t < g.ntasks; t += g.nwt) {
                const int* ti = p.tasks + 5 * t;
                const int rb = uni(ti[0]), k0 = uni(ti[1]), nks = uni(ti[4]);
                if (!SINGLE) {
#pragma unroll
                    for (int s = 0; s < NS; ++s) A[s] = Aimg[(static_cast<size_t>(t) * NS + s) * 64 + lane];
                }
                V acc0 = {0, 0, 0, 0}, acc1 = {0, 0, 0, 0};
                if (GLOBAL_B) {
                    // window too large for LDS (long decimators): B straight from L1/L2
                    const int64_t tb = a * g.Qc + k0 + (lane >> 4);
#pragma unroll
                    for (int s = 0; s < NS; s += 2) {
                        acc0 = Acc<TC>::mfma(A[s], colOk ? srcRead<TC>(src, tb + 4 * s, c) : TC(0), acc0);
                        if (s + 1 < NS)
                            acc1 = Acc<TC>::mfma(A[s + 1], colOk ? srcRead<TC>(src, tb + 4 * s + 4, c) : TC(0), acc1);
                    }
                } else {
                    // B fragment (k = lane>>4, n = lane&15) at sub-tile [kk][n]; reads
                    // software-pipelined 4 steps ahead, sched_barrier keeps the
                    // compiler from hoisting every ds_read.
                    const TC* bp = tile + (gi * g.Qc + k0 + (lane >> 4)) * 16 + (lane & 15);
                    TC bA[4], bB[4];
#pragma unroll
                    for (int j = 0; j < 4; ++j) bA[j] = bp[64 * j];
#pragma unroll
                    for (int s0 = 0; s0 < NS; s0 += 8) {
                        if (s0 + 4 < NS) {
#pragma unroll
                            for (int j = 0; j < 4; ++j) bB[j] = bp[64 * (s0 + 4 + j)];
                        }
                        __builtin_amdgcn_sched_barrier(0);
                        acc0 = Acc<TC>::mfma(A[s0], bA[0], acc0);
                        acc1 = Acc<TC>::mfma(A[s0 + 1], bA[1], acc1);
                        acc0 = Acc<TC>::mfma(A[s0 + 2], bA[2], acc0);
                        acc1 = Acc<TC>::mfma(A[s0 + 3], bA[3], acc1);
                        __builtin_amdgcn_sched_barrier(0);
                        if (s0 + 4 < NS) {
                            if (s0 + 8 < NS) {
#pragma unroll
                                for (int j = 0; j < 4; ++j) bA[j] = bp[64 * (s0 + 8 + j)];
                            }
                            __builtin_amdgcn_sched_barrier(0);
                            acc0 = Acc<TC>::mfma(A[s0 + 4], bB[0], acc0);
                            acc1 = Acc<TC>::mfma(A[s0 + 5], bB[1], acc1);
                            acc0 = Acc<TC>::mfma(A[s0 + 6], bB[2], acc0);
                            acc1 = Acc<TC>::mfma(A[s0 + 7], bB[3], acc1);
                            __builtin_amdgcn_sched_barrier(0);
                        }
                    }
                }
                const V acc = acc0 + acc1;
                if (nks == 1) {
#pragma unroll
                    for (int i = 0; i < 4; ++i) {
                        const int r = rb * 16 + Acc<TC>::row(lane, i);
                        if (colOk && r < g.Pc) outWrite<TC>(od, a * g.Pc + r, c, acc[i]);
                    }
                } else {
                    TC* slot = part + (static_cast<size_t>(cg) * g.ntasks + t) * 256 + lane * 4;
#pragma unroll
                    for (int i = 0; i < 4; ++i) slot[i] = acc[i];
                }
            }
            if (g.ksplit) {
                __syncthreads();
                for (int t = wt; t < g.ntasks; t += g.nwt) {
                    const int* ti = p.tasks + 5 * t;
                    if (uni(ti[4]) == 1 || uni(ti[3]) != 0) continue;
                    const int rb = uni(ti[0]), nks = uni(ti[4]);
                    const TC* slot = part + (static_cast<size_t>(cg) * g.ntasks + t) * 256 + lane * 4;
#pragma unroll
                    for (int i = 0; i < 4; ++i) {
                        TC sum = slot[i];
                        for (int k = 1; k < nks; ++k) sum += slot[k * 256 + i];
                        const int r = rb * 16 + Acc<TC>::row(lane, i);
                        if (colOk && r < g.Pc) outWrite<TC>(od, a * g.Pc + r, c, sum);
                    }
                }
                __syncthreads();
            }
        }
    }
}

template <class TC, int NS>
static hipError_t bgDispatch(const BgDev& p, const SrcDesc& src, const OutDesc& od, const BgGrid& g, int threads,
                             size_t lds, int64_t blocks, hipStream_t st, bool globalB) {
    static bool attrSet = false;
    if (!attrSet) {
        (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&bg_kernel<TC, NS, false, true>),
                                  hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
        (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&bg_kernel<TC, NS, false, false>),
                                  hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
        attrSet = true;
    }
    const dim3 gd(static_cast<unsigned>(blocks)), bd(threads);
    const bool single = g.ntasks <= g.nwt;
    if (globalB) {
        if (single) hipLaunchKernelGGL((bg_kernel<TC, NS, true, true>), gd, bd, lds, st, p, src, od, g);
        else hipLaunchKernelGGL((bg_kernel<TC, NS, true, false>), gd, bd, lds, st, p, src, od, g);
    } else {
        if (single) hipLaunchKernelGGL((bg_kernel<TC, NS, false, true>), gd, bd, lds, st, p, src, od, g);
        else hipLaunchKernelGGL((bg_kernel<TC, NS, false, false>), gd, bd, lds, st, p, src, od, g);
    }
    return hipGetLastError();
}


// Launch geometry + dispatch into the instantiation units.
hipError_t bgLaunchF64(int NS, const BgDev& p, const SrcDesc& src, const OutDesc& od, const BgGrid& g, int threads,
                       size_t lds, int64_t blocks, hipStream_t st, bool globalB);

}  // namespace gar
