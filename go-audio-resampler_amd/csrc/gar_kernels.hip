// gar_kernels.hip -- HIP kernels for gfx950 (MI355X, CDNA4).
//
//  bg_kernel     periodic banded-GEMM FIR on MFMA (v_mfma_f32_16x16x4_f32 /
//                v_mfma_f64_16x16x4_f64).  Executes every x==0 stage of the
//                reference engine: DFT xf upsampler (dft_stage.go:229-273),
//                integer decimator (dft_stage.go:525-534), and the fused
//                DFT x2 -> polyphase composite (gar_plan.cpp firComposite).
//  cubic_kernel  QualityQuick CubicStage (cubic.go:33-90) over host-checkpointed phase walks.
//  poly_kernel   polyphase stage with live cubic coefficient interpolation
//                (polyphase_stage.go:257-293) for ratios whose fixed-point
//                step has fractional bits (x != 0).
//  gather_kernel history compaction (the `copy(history, history[consumed:])`
//                of every stage) and state materialisation.
//  copy_kernel   strided dtype-converting copy (pass-through stages).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdlib>
#include <mutex>
#include <set>
#include <utility>

#include "gar_bg.hpp"
#include "gar_kernels.hpp"

namespace gar {

void setMaxLdsOnce(const void* fn) {
    static std::mutex mu;
    static std::set<std::pair<int, const void*>> done;
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess) return;
    std::lock_guard<std::mutex> lk(mu);
    if (!done.insert({dev, fn}).second) return;
    (void)hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
}

hipError_t bgLaunchF32a(int NS, const BgDev& p, const SrcDesc& src, const OutDesc& od, const BgGrid& g, int threads,
                        size_t lds, int64_t blocks, hipStream_t st, bool globalB);
hipError_t bgLaunchF32b(int NS, const BgDev& p, const SrcDesc& src, const OutDesc& od, const BgGrid& g, int threads,
                        size_t lds, int64_t blocks, hipStream_t st, bool globalB);

hipError_t launchBg(const BgDev& p, const SrcDesc& src, const OutDesc& od, int C, hipStream_t stream, HistCopy* hc) {
    if (od.o_hi <= od.o_lo) return hipSuccess;
    // f32 compute on the split-f16 kernel (every output of the launch, any input dtype)
    if (p.hx && !p.f64) return launchHx(*p.hx, src, od, C, stream, hc);
    const int sz = p.f64 ? 8 : 4;
    BgGrid g;
    g.Pc = p.Pc; g.Qc = p.Qc; g.Kc = p.Kc; g.C = C;
    // Tuning knobs (development sweeps only; defaults are the tuned values).
    static const int knobG = std::getenv("GAR_BG_G") ? std::atoi(std::getenv("GAR_BG_G")) : 0;
    static const int knobWgPerCu = std::getenv("GAR_BG_WGPERCU") ? std::atoi(std::getenv("GAR_BG_WGPERCU")) : 0;
    static const int knobDbg = std::getenv("GAR_BG_DBG") ? std::atoi(std::getenv("GAR_BG_DBG")) : 0;
    static const bool knobNoVst = std::getenv("GAR_BG_NOVST") != nullptr;
    static const bool knobNoParity = std::getenv("GAR_BG_NOPARITY") != nullptr;
    g.nprog = p.nprog;
    g.kch = p.kch;
    g.nwt = p.nw;
    g.ncg = p.ncg;
    g.nred = p.nred;
    g.nslots = p.nslots;
    g.a_lo = od.o_lo / p.Pc;
    const int64_t a_hi = (od.o_hi + p.Pc - 1) / p.Pc;
    const int64_t nmac = a_hi - g.a_lo;
    const int threads = 64 * g.ncg * g.nwt;
    const int tileN = 16 * g.ncg;
    const size_t slotBytes = static_cast<size_t>(g.ncg) * g.nslots * 256 * sz;
    // Two LDS tiles (double buffer) + partial slots (two buffers when they fit
    // beside a tile of >= 4 macro periods, else one + a second barrier).
    const int rowsPerPiece = p.f64 ? 2 : 4;
    auto wsFor = [&](int W) { return (W + rowsPerPiece - 1) / rowsPerPiece * rowsPerPiece; };
    auto tileBytes = [&](int G) { return 2 * static_cast<size_t>(tileN) * wsFor(p.Kread + (G - 1) * p.Qc) * sz; };
    const size_t kLds = 160 * 1024;
    g.parity = (g.nred > 0 && !knobNoParity && tileBytes(std::min<int64_t>(4, std::max<int64_t>(nmac, 1))) + 2 * slotBytes <= kLds) ? 1 : 0;
    const size_t partBytes = (g.parity ? 2 : 1) * slotBytes;
    int G = 1;
    for (int cand = 2; cand <= 8; ++cand) {
        if (cand > nmac) break;
        if (tileBytes(cand) + partBytes > kLds) break;
        G = cand;
    }
    if (knobG > 0 && knobG < G) G = knobG;
    g.G = G;
    g.W = p.Kc + (G - 1) * p.Qc;
    g.Wl = p.Kread + (G - 1) * p.Qc;
    g.Ws = wsFor(g.Wl);
    const int64_t nchunk = (nmac + G - 1) / G;
    g.nchunk = static_cast<int>(nchunk);
    g.ncols = static_cast<int>(nchunk * C);
    g.nblocks = (g.ncols + tileN - 1) / tileN;
    g.dbg = knobDbg;
    g.vst = 0;
    if (!p.f64 && !od.f64 && !od.pcm && !knobNoVst) {
        if (od.fs == 1) g.vst = 1;
        else if (C == 2 && od.fs == 2 && od.cs == 1) g.vst = 2;
    }
    size_t lds = tileBytes(G) + partBytes;
    const bool globalB = lds > kLds;
    if (globalB) lds = partBytes;
    if (lds > kLds) return hipErrorInvalidConfiguration;
    if (g.nblocks <= 0) return hipSuccess;
    int dev = 0, ncu = 256;
    if (hipGetDevice(&dev) == hipSuccess) (void)hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev);
    int64_t blocks = std::min<int64_t>(g.nblocks, static_cast<int64_t>(ncu) * (knobWgPerCu > 0 ? knobWgPerCu : 2));
    g.hdst = nullptr;
    g.ht0 = g.hn = 0;
    if (hc && hc->n > 0 && hc->dst) {  // history keep folded into this launch (no gather_kernel after it)
        g.hdst = hc->dst;
        g.ht0 = hc->t0;
        g.hn = hc->n;
        hc->done = true;
    }
    if (p.f64) return bgLaunchF64(p.NS, p, src, od, g, threads, lds, blocks, stream, globalB);
    if (p.NS < 56) return bgLaunchF32a(p.NS, p, src, od, g, threads, lds, blocks, stream, globalB);
    return bgLaunchF32b(p.NS, p, src, od, g, threads, lds, blocks, stream, globalB);
}

// ---------------------------------------------------------------------------
// General polyphase stage (cubic sub-phase interpolation live).
// ---------------------------------------------------------------------------
// A workgroup owns a tile of consecutive outputs: it first evaluates the
// interpolated coefficients a + x(b + x(c + x d)) of every (output, tap) of the
// tile ONCE into LDS (the reference evaluates them per channel inside
// CubicInterpDot, polyphase_stage.go:283-289), then each thread accumulates
// one (output, channel) dot product over the shared row -- consecutive threads
// are consecutive channels of one output, so the input reads coalesce for
// many channels and the taps of neighbouring outputs hit the same lines.
// Per-tap arithmetic and summation order are those of the reference's loop.
constexpr int kPolyThreads = 256;
constexpr int kPolyLdsBytes = 48 * 1024;

template <class TC>
__global__ __launch_bounds__(kPolyThreads) void poly_kernel(PolyDev p, SrcDesc src, OutDesc od, int64_t nout, int C,
                                                            int MT) {
    extern __shared__ __attribute__((aligned(16))) unsigned char psm[];
    TC* coef = reinterpret_cast<TC*>(psm);  // [MT][T]
    const TC* A = static_cast<const TC*>(p.a);
    const TC* B = static_cast<const TC*>(p.b);
    const TC* Cc = static_cast<const TC*>(p.c);
    const TC* D = static_cast<const TC*>(p.d);
    const TC fscale = static_cast<TC>(1.0 / 65536.0);
    const int T = p.T;
    const int64_t ntiles = (nout + MT - 1) / MT;
    for (int64_t tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
        const int64_t m0 = tile * MT;
        const int mt = static_cast<int>(min<int64_t>(MT, nout - m0));
        __syncthreads();  // previous tile's rows consumed
        for (int e = threadIdx.x; e < mt * T; e += blockDim.x) {
            const int mm = e / T, k = e - mm * T;
            const int64_t at = p.at0 + (m0 + mm) * p.step;
            const int ph = static_cast<int>((at >> 16) % p.L);
            const TC x = static_cast<TC>(at & 0xFFFF) * fscale;
            const size_t o = static_cast<size_t>(ph) * T + k;
            coef[mm * T + k] = A[o] + x * (B[o] + x * (Cc[o] + x * D[o]));
        }
        __syncthreads();
        for (int e = threadIdx.x; e < mt * C; e += blockDim.x) {
            const int mm = e / C, c = e - mm * C;
            const int64_t at = p.at0 + (m0 + mm) * p.step;
            const int64_t base = p.u_base + (at >> 16) / p.L;
            const TC* row = coef + mm * T;
            TC acc = 0;
            for (int k = 0; k < T; ++k) acc += srcRead<TC>(src, base + k, c) * row[k];
            outWrite<TC>(od, od.o_lo + m0 + mm, c, acc);
        }
    }
}

hipError_t launchPoly(const PolyDev& p, const SrcDesc& src, const OutDesc& od, int64_t nout, int C,
                      hipStream_t stream) {
    if (nout <= 0) return hipSuccess;
    const int es = p.f64 ? 8 : 4;
    // outputs per tile: enough (output, channel) pairs for the block, rows within the LDS budget
    int MT = std::max(1, (2 * kPolyThreads + C - 1) / C);
    MT = std::min<int>(MT, std::max(1, kPolyLdsBytes / (p.T * es)));
    const int64_t ntiles = (nout + MT - 1) / MT;
    const int64_t blocks = std::min<int64_t>(ntiles, 8192);
    const size_t lds = static_cast<size_t>(MT) * p.T * es;
    if (p.f64) hipLaunchKernelGGL(poly_kernel<double>, dim3(static_cast<unsigned>(blocks)), dim3(kPolyThreads), lds, stream, p, src, od, nout, C, MT);
    else hipLaunchKernelGGL(poly_kernel<float>, dim3(static_cast<unsigned>(blocks)), dim3(kPolyThreads), lds, stream, p, src, od, nout, C, MT);
    return hipGetLastError();
}

// ---------------------------------------------------------------------------
// CubicStage (QualityQuick, internal/engine/cubic.go:33-90): 4-point cubic
// interpolation at a floating-point phase.  The phase walk is a sequential f64
// recurrence (phase += 1/ratio per output, -= 1 per input); the host runs it
// once for all channels and checkpoints its exact state every kCubicSegInputs
// inputs; one thread per (segment, channel) re-walks its segment with the same
// f64 operations, so every output sits at the reference's phase bit for bit.
// ---------------------------------------------------------------------------
template <class TC>
__global__ __launch_bounds__(256) void cubic_kernel(const CubicSeg* segs, int64_t nseg, int64_t x_end, double step,
                                                    SrcDesc src, OutDesc od, int C) {
#pragma clang fp contract(off)
    const int64_t total = nseg * C;
    for (int64_t idx = blockIdx.x * static_cast<int64_t>(blockDim.x) + threadIdx.x; idx < total;
         idx += static_cast<int64_t>(gridDim.x) * blockDim.x) {
        const int64_t sgi = idx / C;
        const int c = static_cast<int>(idx - sgi * C);
        const CubicSeg sg = segs[sgi];
        const int64_t i1 = min(sg.i + kCubicSegInputs, x_end);
        // history[3..1] = inputs i-3 .. i-1 (zeros before the stream start)
        double h3 = static_cast<double>(srcRead<TC>(src, sg.i - 3, c));
        double h2 = static_cast<double>(srcRead<TC>(src, sg.i - 2, c));
        double h1 = static_cast<double>(srcRead<TC>(src, sg.i - 1, c));
        double ph = sg.phase;
        int64_t o = sg.o;
        for (int64_t i = sg.i; i < i1; ++i) {
            const double h0 = static_cast<double>(srcRead<TC>(src, i, c));
            while (ph < 1.0) {
                // s[-1], s[0], s[1], s[2] = history[3], [2], [1], [0] (cubic.go:78-89)
                const double b = 0.5 * (h1 + h3) - h2;
                const double a = (1.0 / 6.0) * (h0 - h1 + h3 - h2 - 4 * b);
                const double cc = h1 - h2 - a - b;
                outWrite<TC>(od, o, c, static_cast<TC>(((a * ph + b) * ph + cc) * ph + h2));
                ++o;
                ph += step;
            }
            ph -= 1.0;
            h3 = h2; h2 = h1; h1 = h0;
        }
    }
}

hipError_t launchCubic(int f64, const CubicSeg* segs, int64_t nseg, int64_t x_end, double step, const SrcDesc& src,
                       const OutDesc& od, int C, hipStream_t stream) {
    if (nseg <= 0) return hipSuccess;
    const int64_t total = nseg * C;
    int64_t blocks = (total + 255) / 256;
    if (blocks > 65536) blocks = 65536;
    if (f64) hipLaunchKernelGGL(cubic_kernel<double>, dim3(static_cast<unsigned>(blocks)), dim3(256), 0, stream, segs, nseg, x_end, step, src, od, C);
    else hipLaunchKernelGGL(cubic_kernel<float>, dim3(static_cast<unsigned>(blocks)), dim3(256), 0, stream, segs, nseg, x_end, step, src, od, C);
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

__global__ __launch_bounds__(256) void convert_kernel(const void* s, int st, int64_t sfs, int64_t scs, void* d, int dt,
                                                      int64_t dfs, int64_t dcs, int64_t n, int C) {
    const int64_t total = n * C;
    for (int64_t idx = blockIdx.x * static_cast<int64_t>(blockDim.x) + threadIdx.x; idx < total;
         idx += static_cast<int64_t>(gridDim.x) * blockDim.x) {
        const int64_t t = idx / C;
        const int c = static_cast<int>(idx - t * C);
        const int64_t se = t * sfs + c * scs, de = t * dfs + c * dcs;
        const double v = st >= 16 ? pcmRead(s, se, st)
                                  : (st == 1 ? static_cast<const double*>(s)[se] : static_cast<double>(static_cast<const float*>(s)[se]));
        if (dt >= 16) pcmWrite(d, de, dt, v);
        else if (dt == 1) static_cast<double*>(d)[de] = v;
        else static_cast<float*>(d)[de] = static_cast<float>(v);
    }
}

hipError_t launchConvert(const void* src, int s_type, int64_t s_fs, int64_t s_cs, void* dst, int d_type, int64_t d_fs,
                         int64_t d_cs, int64_t n, int C, hipStream_t stream) {
    if (n <= 0) return hipSuccess;
    int64_t blocks = (n * C + 255) / 256;
    if (blocks > 65536) blocks = 65536;
    hipLaunchKernelGGL(convert_kernel, dim3(static_cast<unsigned>(blocks)), dim3(256), 0, stream, src, s_type, s_fs, s_cs,
                       dst, d_type, d_fs, d_cs, n, C);
    return hipGetLastError();
}

}  // namespace gar
