// gar_hx.hip -- launch geometry of the split-f16 FIR kernel (gar_hx.hpp): the
// interior chunks of a launch run on hx_kernel, its edges on fir_kernel.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>

#include "gar_hx.hpp"

namespace gar {

// hxLaunch instantiations live in gar_hx_i*.hip (compiled in parallel)
#define GAR_HX_EXTERN(NS, RB, V) \
    extern template hipError_t hxLaunch<NS, RB, V>(const HxArgs&, int, size_t, int64_t, hipStream_t);
GAR_HX_FOR_ALL(GAR_HX_EXTERN)
#undef GAR_HX_EXTERN

// Direct f32 FIR over outputs [od.o_lo, od.o_hi) x C channels (exact rows,
// any source): the edges of a launch (history seam, flush zeros, partial
// macro periods) and launches too small for hx_kernel.  One wave per output:
// lanes split the taps, then a wave reduction.
__global__ __launch_bounds__(256) void fir_kernel(SrcDesc src, OutDesc od, int C, int P, int Q, const int* rowOff,
                                                  const int* rowLen, const float* rows, int rowMax) {
    const int lane = threadIdx.x & 63;
    const int64_t n = (od.o_hi - od.o_lo) * C;
    const int64_t wstep = static_cast<int64_t>(gridDim.x) * (blockDim.x >> 6);
    for (int64_t idx = blockIdx.x * static_cast<int64_t>(blockDim.x >> 6) + (threadIdx.x >> 6); idx < n; idx += wstep)
        firOne(src, od, od.o_lo + idx / C, static_cast<int>(idx % C), P, Q, rowOff, rowLen, rows, rowMax, lane);
}

namespace {


// row-block mode: the epilogue store layout (HxArgs::vst) is a template parameter
template <int NS, bool RB>
hipError_t hxDispatch(const HxArgs& x, int waves, size_t lds, int64_t blocks, hipStream_t st) {
    if constexpr (!RB) return hxLaunch<NS, false, 0>(x, waves, lds, blocks, st);
    switch (x.vst) {
        case 0: return hxLaunch<NS, RB, 0>(x, waves, lds, blocks, st);
        case 1: return hxLaunch<NS, RB, 1>(x, waves, lds, blocks, st);
        case 2: return hxLaunch<NS, RB, 2>(x, waves, lds, blocks, st);
        default: return hxLaunch<NS, RB, 3>(x, waves, lds, blocks, st);
    }
}

hipError_t launchFir(const HxDev& p, const SrcDesc& src, OutDesc od, int64_t lo, int64_t hi, int C, hipStream_t st) {
    if (hi <= lo) return hipSuccess;
    od.o_lo = lo;
    od.o_hi = hi;
    const int64_t n = (hi - lo) * C;  // one wave per output
    const int64_t blocks = std::min<int64_t>((n + 3) / 4, 65536);
    hipLaunchKernelGGL(fir_kernel, dim3(static_cast<unsigned>(blocks)), dim3(256), 0, st, src, od, C, p.Pc, p.Qc,
                       p.rowOff, p.rowLen, p.rows, p.rowMax);
    return hipGetLastError();
}

int64_t floorDiv(int64_t a, int64_t b) { return a >= 0 ? a / b : -((-a + b - 1) / b); }
int64_t ceilDiv(int64_t a, int64_t b) { return -floorDiv(-a, b); }

}  // namespace

hipError_t launchHx(const HxDev& p, const SrcDesc& src, const OutDesc& od, int C, hipStream_t stream) {
    if (od.o_hi <= od.o_lo) return hipSuccess;
    // development knobs: GAR_HX_G caps macro periods per column; GAR_HX_DBG bits: 1 skip
    // staging after the first block, 2 skip the MFMA programs, 8 skip the fixup, 16 skip the loop,
    // 32 skip the f16 conversion, 64 skip the LDS-DMA
    static const int knobG = std::getenv("GAR_HX_G") ? std::atoi(std::getenv("GAR_HX_G")) : 0;
    static const int knobDbg = std::getenv("GAR_HX_DBG") ? std::atoi(std::getenv("GAR_HX_DBG")) : 0;
    const int64_t Pc = p.Pc, Qc = p.Qc;
    const int64_t a_lo = od.o_lo / Pc;
    const int64_t nmac = (od.o_hi + Pc - 1) / Pc - a_lo;
    const size_t slotBytes = static_cast<size_t>(p.nslots) * 256 * 4;
    const size_t kLds = 160 * 1024;
    // window rows staged per column (the padded program steps read up to Kread + (G-1)*Qc),
    // whole 64-row item slots
    auto wsFor = [&](int G) { return (p.Kread + (G - 1) * p.Qc + 63) / 64 * 64; };
    // two buffers of 4 quads x (16*Ws + 64) B, partial slots, quad exponent sets + fixup flag
    auto ldsFor = [&](int G, int par) {
        return 8 * (16 * static_cast<size_t>(wsFor(G)) + 64) + (par ? 2 : 1) * slotBytes + 160;
    };
    const int parity = (p.nred > 0 && ldsFor(1, 1) <= kLds) ? 1 : 0;
    int dev = 0, ncu = 256;
    if (hipGetDevice(&dev) == hipSuccess) (void)hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev);
    // G macro periods per column: the largest whose window fits LDS without
    // dropping below one block per CU (when the launch is large enough for that)
    auto nbFor = [&](int G) { return ((nmac + G - 1) / G * C + 15) / 16; };
    int G = 1;
    for (int cand = 2; cand <= 8; ++cand) {
        if (cand > nmac || wsFor(cand) > kHxMaxRows || ldsFor(cand, parity) > kLds) break;
        if (nbFor(cand) < ncu && nbFor(1) >= ncu) break;
        G = cand;
    }
    if (knobG > 0 && knobG < G) G = knobG;
    const int64_t W = p.Kc + static_cast<int64_t>(G - 1) * Qc;

    // interior chunks [k0, k1): outputs inside [o_lo, o_hi), window rows [0, W) inside the f32 input
    int64_t k0 = 0, k1 = 0;
    if (src.in && !src.in_f64 && src.in_len > 0 && wsFor(G) <= kHxMaxRows && ldsFor(G, parity) <= kLds) {
        const int64_t GQ = G * Qc, GP = G * Pc;
        const int64_t inEnd = std::min(src.in_base + src.in_len, src.valid_end);
        k0 = std::max<int64_t>({0, ceilDiv(od.o_lo - a_lo * Pc, GP), ceilDiv(src.in_base - a_lo * Qc, GQ)});
        k1 = std::min<int64_t>(floorDiv(od.o_hi - a_lo * Pc, GP), floorDiv(inEnd - W - a_lo * Qc, GQ) + 1);
    }
    const int64_t ncols = (k1 - k0) * C;
    static const bool trace = std::getenv("GAR_HX_TRACE") != nullptr;
    if (trace)
        fprintf(stderr, "hx: o[%lld,%lld) C=%d G=%d W=%lld a_lo=%lld k0=%lld k1=%lld in_base=%lld in_len=%lld valid_end=%lld hist_len=%lld\n",
                (long long)od.o_lo, (long long)od.o_hi, C, G, (long long)W, (long long)a_lo, (long long)k0, (long long)k1,
                (long long)src.in_base, (long long)src.in_len, (long long)src.valid_end, (long long)src.hist_len);
    if (ncols < 64 || ncols > (int64_t(1) << 30)) return launchFir(p, src, od, od.o_lo, od.o_hi, C, stream);

    HxArgs x{};
    x.A = static_cast<const h8v*>(p.A);
    x.progs = p.progs;
    x.reds = p.reds;
    x.fix = p.fix;
    x.fixCap = p.fixCap;
    x.ea = p.ea;
    x.kch = p.kch;
    x.Pc = p.Pc; x.Qc = p.Qc; x.G = G; x.C = C;
    x.W = static_cast<int>(W);
    x.Ws = wsFor(G);
    x.ncols = static_cast<int>(ncols);
    x.nblocks = static_cast<int>((ncols + 15) / 16);
    x.nred = p.nred; x.nslots = p.nslots; x.parity = parity;
    x.dbg = knobDbg;
    x.a0 = a_lo + k0 * G;
    const float* in = static_cast<const float*>(src.in);
    x.in = in + (x.a0 * Qc - src.in_base) * src.in_fs;
    x.in_fs = src.in_fs;
    x.in_cs = src.in_cs;
    x.in_chunk = G * Qc * src.in_fs;
    const int esz = od.f64 ? 8 : 4;
    x.out_f64 = od.f64;
    x.out = static_cast<char*>(od.out) + (x.a0 * Pc - od.o0) * od.fs * esz;
    x.out_fs = od.fs * esz;
    x.out_cs = od.cs * esz;
    x.out_chunk = G * Pc * od.fs * esz;
    // epilogue layout (16-B stores need every row quad 16-B aligned)
    const bool al = (reinterpret_cast<uintptr_t>(x.out) & 15) == 0;
    if (od.f64) x.vst = 3;
    else if (al && C == 2 && od.fs == 2 && od.cs == 1 && Pc % 2 == 0) x.vst = 2;
    else if (al && od.fs == 1 && (od.cs * 4) % 16 == 0 && Pc % 4 == 0) x.vst = 1;
    else x.vst = 0;
    // raw load format: 8-B stereo frames / 16-B four-channel rows where the layout allows it
    const uintptr_t inA = reinterpret_cast<uintptr_t>(in);
    x.fmt = 0;
    if ((inA & 7) == 0 && C == 2 && src.in_fs == 2 && src.in_cs == 1) x.fmt = 1;
    else if ((inA & 15) == 0 && C % 4 == 0 && src.in_cs == 1 && src.in_fs % 4 == 0) x.fmt = 2;
    static const bool noFmt = std::getenv("GAR_HX_DWORD") != nullptr;
    if (noFmt) x.fmt = 0;
    x.src = src;
    x.od = od;
    x.rows = p.rows;
    x.rowOff = p.rowOff;
    x.rowLen = p.rowLen;
    x.rowMax = p.rowMax;
    x.zero = p.zero;

    // the launch edges run inside hx_kernel (spread over its waves before the blocks)
    x.e0lo = od.o_lo;
    x.e0hi = x.a0 * Pc;
    x.e1lo = (a_lo + k1 * G) * Pc;
    x.e1hi = od.o_hi;

    const size_t lds = ldsFor(G, parity);
    const int64_t blocks = std::min<int64_t>(x.nblocks, ncu);
    x.nprog = p.nw;
    if (p.rb) {
        if (p.nw > kHxRbMaxWaves) return hipErrorInvalidConfiguration;
        const int waves = std::max(p.nw, kHxMinWaves);
        switch (p.NS) {
#define GAR_HX_RB(n) case n: return hxDispatch<n, true>(x, waves, lds, blocks, stream);
            GAR_HX_RB(1) GAR_HX_RB(2) GAR_HX_RB(3) GAR_HX_RB(4) GAR_HX_RB(5) GAR_HX_RB(6) GAR_HX_RB(7) GAR_HX_RB(8)
            GAR_HX_RB(9) GAR_HX_RB(10)
#undef GAR_HX_RB
            default: return hipErrorInvalidConfiguration;
        }
    }
    switch (p.NS) {
#define GAR_HX_SEG(n) case n: return hxDispatch<n, false>(x, kHxWaves, lds, blocks, stream);
        GAR_HX_SEG(2) GAR_HX_SEG(4) GAR_HX_SEG(6) GAR_HX_SEG(8)
#undef GAR_HX_SEG
        default: return hipErrorInvalidConfiguration;
    }
}

}  // namespace gar
