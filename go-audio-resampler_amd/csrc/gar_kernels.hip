// gar_kernels.hip -- HIP kernels for gfx950 (MI355X, CDNA4).
//
//  bg_kernel     periodic banded-GEMM FIR on MFMA (v_mfma_f32_16x16x4_f32 /
//                v_mfma_f64_16x16x4_f64).  Executes every x==0 stage of the
//                reference engine: DFT xf upsampler (dft_stage.go:229-273),
//                integer decimator (dft_stage.go:525-534), and the fused
//                DFT x2 -> polyphase composite (gar_plan.cpp firComposite).
//  poly_kernel   polyphase stage with live cubic coefficient interpolation
//                (polyphase_stage.go:257-293) for ratios whose fixed-point
//                step has fractional bits (x != 0).
//  gather_kernel history compaction (the `copy(history, history[consumed:])`
//                of every stage) and state materialisation.
//  copy_kernel   strided dtype-converting copy (pass-through stages).
#include <hip/hip_runtime.h>

#include "gar_kernels.hpp"

namespace gar {

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef double f64x4 __attribute__((ext_vector_type(4)));

template <class TC>
__device__ __forceinline__ TC srcRead(const SrcDesc& s, int64_t t, int c) {
    if (t < 0 || t >= s.valid_end) return TC(0);
    const int64_t h = t - s.hist_base;
    if (h >= 0 && h < s.hist_len) return static_cast<const TC*>(s.hist)[h * s.hist_ld + c];
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
    int64_t a_lo, nchunk;
    int C, ntasks, nwt, ncg, ksplit, chan_fast;
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

template <class TC, int NS>
__global__ __launch_bounds__(640) void bg_kernel(BgDev p, SrcDesc src, OutDesc od, BgGrid g) {
    typedef typename Acc<TC>::V V;
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    TC* tile = reinterpret_cast<TC*>(smem);
    const int tileN = 16 * g.ncg;
    TC* part = tile + static_cast<size_t>(tileN) * g.Ws;  // k-split partials [ncg][ntasks][256]

    const int lane = threadIdx.x & 63;
    const int wave = threadIdx.x >> 6;
    const int64_t col0 = static_cast<int64_t>(blockIdx.x) * tileN;
    const int64_t ncols = g.nchunk * g.C;

    // ---- stage the 16*ncg input windows into LDS -------------------------
    const int total = tileN * g.W;
    for (int idx = threadIdx.x; idx < total; idx += blockDim.x) {
        int n, kk;
        if (g.chan_fast) { kk = idx / tileN; n = idx - kk * tileN; }
        else { n = idx / g.W; kk = idx - n * g.W; }
        const int64_t col = col0 + n;
        TC v = TC(0);
        if (col < ncols) {
            const int c = static_cast<int>(col % g.C);
            const int64_t chunk = col / g.C;
            const int64_t t = (g.a_lo + chunk * g.G) * g.Qc + kk;
            v = srcRead<TC>(src, t, c);
        }
        tile[n * g.Ws + kk] = v;
    }
    __syncthreads();

    const int cg = wave / g.nwt;
    const int wt = wave - cg * g.nwt;
    const int nloc = cg * 16 + (lane & 15);
    const int64_t col = col0 + nloc;
    const bool colOk = col < ncols;
    const int c = colOk ? static_cast<int>(col % g.C) : 0;
    const int64_t chunk = colOk ? col / g.C : 0;
    const TC* Aimg = static_cast<const TC*>(p.A);
    const bool single = g.ntasks <= g.nwt;

    TC A[NS];
    if (single && wt < g.ntasks) {
#pragma unroll
        for (int s = 0; s < NS; ++s) A[s] = Aimg[(static_cast<size_t>(wt) * NS + s) * 64 + lane];
    }

    for (int gi = 0; gi < g.G; ++gi) {
        const int64_t a = g.a_lo + chunk * g.G + gi;
        for (int t = wt; t < g.ntasks; t += g.nwt) {
            const int* ti = p.tasks + 5 * t;
            const int rb = ti[0], k0 = ti[1], ns = ti[2], nks = ti[4];
            if (!single) {
#pragma unroll
                for (int s = 0; s < NS; ++s) A[s] = Aimg[(static_cast<size_t>(t) * NS + s) * 64 + lane];
            }
            V acc = {0, 0, 0, 0};
            const TC* bp = tile + nloc * g.Ws + gi * g.Qc + k0 + (lane >> 4);
#pragma unroll
            for (int s = 0; s < NS; ++s)
                if (s < ns) acc = Acc<TC>::mfma(A[s], bp[4 * s], acc);
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
                if (ti[4] == 1 || ti[3] != 0) continue;
                const int rb = ti[0], nks = ti[4];
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

template <class TC, int NS>
static hipError_t bgDispatch(const BgDev& p, const SrcDesc& src, const OutDesc& od, const BgGrid& g, int threads,
                             size_t lds, int64_t blocks, hipStream_t st) {
    hipLaunchKernelGGL((bg_kernel<TC, NS>), dim3(static_cast<unsigned>(blocks)), dim3(threads), lds, st, p, src, od, g);
    return hipGetLastError();
}

hipError_t launchBg(const BgDev& p, const SrcDesc& src, const OutDesc& od, int C, hipStream_t stream) {
    if (od.o_hi <= od.o_lo) return hipSuccess;
    const int sz = p.f64 ? 8 : 4;
    BgGrid g;
    g.Pc = p.Pc; g.Qc = p.Qc; g.Kc = p.Kc; g.C = C;
    g.ntasks = p.ntasks;
    g.nwt = p.ntasks < 10 ? p.ntasks : 10;
    g.ncg = 1;
    while (g.ncg * 2 * g.nwt <= 8 && g.ncg < 4) g.ncg *= 2;  // fill >= 4 waves per workgroup
    g.ksplit = p.ksplit;
    g.a_lo = od.o_lo / p.Pc;
    const int64_t a_hi = (od.o_hi + p.Pc - 1) / p.Pc;
    const int64_t nmac = a_hi - g.a_lo;
    // LDS budget ~64 KiB so two workgroups share a CU and overlap load/compute.
    const size_t budget = 64 * 1024;
    const size_t partBytes = g.ksplit ? static_cast<size_t>(g.ncg) * g.ntasks * 256 * sz : 0;
    int G = 1;
    for (int cand = 2; cand <= 8; ++cand) {
        if (cand > nmac) break;
        const int W = p.Kc + (cand - 1) * p.Qc;
        const int Ws = ((W + 29) / 32) * 32 + 2;
        if (static_cast<size_t>(16 * g.ncg) * Ws * sz + partBytes > budget) break;
        G = cand;
    }
    g.G = G;
    g.W = p.Kc + (G - 1) * p.Qc;
    g.Ws = ((g.W + 29) / 32) * 32 + 2;
    g.nchunk = (nmac + G - 1) / G;
    g.chan_fast = C >= 16 ? 1 : 0;
    const int64_t cols = g.nchunk * C;
    const int64_t blocks = (cols + 16 * g.ncg - 1) / (16 * g.ncg);
    const int threads = 64 * g.ncg * g.nwt;
    const size_t lds = static_cast<size_t>(16 * g.ncg) * g.Ws * sz + partBytes;
    if (blocks <= 0) return hipSuccess;
    if (p.f64) {
        switch (p.NS) {
            case 16: return bgDispatch<double, 16>(p, src, od, g, threads, lds, blocks, stream);
            case 32: return bgDispatch<double, 32>(p, src, od, g, threads, lds, blocks, stream);
            case 48: return bgDispatch<double, 48>(p, src, od, g, threads, lds, blocks, stream);
            case 64: return bgDispatch<double, 64>(p, src, od, g, threads, lds, blocks, stream);
            default: return hipErrorInvalidValue;
        }
    }
    switch (p.NS) {
        case 16: return bgDispatch<float, 16>(p, src, od, g, threads, lds, blocks, stream);
        case 32: return bgDispatch<float, 32>(p, src, od, g, threads, lds, blocks, stream);
        case 48: return bgDispatch<float, 48>(p, src, od, g, threads, lds, blocks, stream);
        case 64: return bgDispatch<float, 64>(p, src, od, g, threads, lds, blocks, stream);
        case 80: return bgDispatch<float, 80>(p, src, od, g, threads, lds, blocks, stream);
        case 96: return bgDispatch<float, 96>(p, src, od, g, threads, lds, blocks, stream);
        case 112: return bgDispatch<float, 112>(p, src, od, g, threads, lds, blocks, stream);
        case 128: return bgDispatch<float, 128>(p, src, od, g, threads, lds, blocks, stream);
        default: return hipErrorInvalidValue;
    }
}

// ---------------------------------------------------------------------------
// General polyphase stage (cubic sub-phase interpolation live).
// ---------------------------------------------------------------------------
template <class TC>
__global__ __launch_bounds__(256) void poly_kernel(PolyDev p, SrcDesc src, OutDesc od, int64_t nout, int C) {
    const int64_t total = nout * C;
    const TC* A = static_cast<const TC*>(p.a);
    const TC* B = static_cast<const TC*>(p.b);
    const TC* Cc = static_cast<const TC*>(p.c);
    const TC* D = static_cast<const TC*>(p.d);
    const TC fscale = static_cast<TC>(1.0 / 65536.0);
    for (int64_t idx = blockIdx.x * static_cast<int64_t>(blockDim.x) + threadIdx.x; idx < total;
         idx += static_cast<int64_t>(gridDim.x) * blockDim.x) {
        const int64_t m = idx / C;
        const int c = static_cast<int>(idx - m * C);
        const int64_t at = p.at0 + m * p.step;
        const int64_t full = at >> 16;
        const int64_t div = full / p.L;
        const int ph = static_cast<int>(full % p.L);
        const TC x = static_cast<TC>(at & 0xFFFF) * fscale;
        const int64_t base = p.u_base + div;
        const size_t o = static_cast<size_t>(ph) * p.T;
        TC acc = 0;
        for (int k = 0; k < p.T; ++k) {
            const TC coef = A[o + k] + x * (B[o + k] + x * (Cc[o + k] + x * D[o + k]));
            acc += srcRead<TC>(src, base + k, c) * coef;
        }
        outWrite<TC>(od, od.o_lo + m, c, acc);
    }
}

hipError_t launchPoly(const PolyDev& p, const SrcDesc& src, const OutDesc& od, int64_t nout, int C,
                      hipStream_t stream) {
    if (nout <= 0) return hipSuccess;
    const int64_t total = nout * C;
    int64_t blocks = (total + 255) / 256;
    if (blocks > 65536) blocks = 65536;
    if (p.f64) hipLaunchKernelGGL(poly_kernel<double>, dim3(static_cast<unsigned>(blocks)), dim3(256), 0, stream, p, src, od, nout, C);
    else hipLaunchKernelGGL(poly_kernel<float>, dim3(static_cast<unsigned>(blocks)), dim3(256), 0, stream, p, src, od, nout, C);
    return hipGetLastError();
}

// ---------------------------------------------------------------------------
template <class TC>
__global__ __launch_bounds__(256) void gather_kernel(SrcDesc src, TC* dst, int64_t t0, int64_t n, int C) {
    const int64_t total = n * C;
    for (int64_t idx = blockIdx.x * static_cast<int64_t>(blockDim.x) + threadIdx.x; idx < total;
         idx += static_cast<int64_t>(gridDim.x) * blockDim.x) {
        const int64_t t = idx / C;
        const int c = static_cast<int>(idx - t * C);
        dst[idx] = srcRead<TC>(src, t0 + t, c);
    }
}

hipError_t launchGather(int f64, const SrcDesc& src, void* dst, int64_t t0, int64_t n, int C, hipStream_t stream) {
    if (n <= 0) return hipSuccess;
    int64_t blocks = (n * C + 255) / 256;
    if (blocks > 65536) blocks = 65536;
    if (f64) hipLaunchKernelGGL(gather_kernel<double>, dim3(static_cast<unsigned>(blocks)), dim3(256), 0, stream, src, static_cast<double*>(dst), t0, n, C);
    else hipLaunchKernelGGL(gather_kernel<float>, dim3(static_cast<unsigned>(blocks)), dim3(256), 0, stream, src, static_cast<float*>(dst), t0, n, C);
    return hipGetLastError();
}

__global__ __launch_bounds__(256) void copy_kernel(const void* s, int sf64, int64_t sfs, int64_t scs, void* d, int df64,
                                                   int64_t dfs, int64_t dcs, int64_t n, int C) {
    const int64_t total = n * C;
    for (int64_t idx = blockIdx.x * static_cast<int64_t>(blockDim.x) + threadIdx.x; idx < total;
         idx += static_cast<int64_t>(gridDim.x) * blockDim.x) {
        const int64_t t = idx / C;
        const int c = static_cast<int>(idx - t * C);
        const double v = sf64 ? static_cast<const double*>(s)[t * sfs + c * scs]
                              : static_cast<double>(static_cast<const float*>(s)[t * sfs + c * scs]);
        if (df64) static_cast<double*>(d)[t * dfs + c * dcs] = v;
        else static_cast<float*>(d)[t * dfs + c * dcs] = static_cast<float>(v);
    }
}

hipError_t launchCopy(const void* src, int src_f64, int64_t s_fs, int64_t s_cs, void* dst, int dst_f64, int64_t d_fs,
                      int64_t d_cs, int64_t n, int C, hipStream_t stream) {
    if (n <= 0) return hipSuccess;
    int64_t blocks = (n * C + 255) / 256;
    if (blocks > 65536) blocks = 65536;
    hipLaunchKernelGGL(copy_kernel, dim3(static_cast<unsigned>(blocks)), dim3(256), 0, stream, src, src_f64, s_fs, s_cs,
                       dst, dst_f64, d_fs, d_cs, n, C);
    return hipGetLastError();
}

}  // namespace gar
