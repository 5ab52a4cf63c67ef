// gar_hx.hip -- instantiations and launch geometry of the split-f16 FIR kernel (gar_hx.hpp).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdlib>

#include "gar_hx.hpp"

namespace gar {

template <int NS, bool RB>
static hipError_t hxDispatch(const HxDev& p, const SrcDesc& src, const OutDesc& od, const BgGrid& g, size_t lds,
                             int64_t blocks, hipStream_t st) {
    static bool attrSet = false;
    if (!attrSet) {
        (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&hx_kernel<NS, RB, true>),
                                  hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
        if (!RB)
            (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&hx_kernel<NS, RB, false>),
                                      hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
        attrSet = true;
    }
    const int waves = RB ? std::max(p.nw, 8) : kHxWaves;
    const dim3 gd(static_cast<unsigned>(blocks)), bd(64 * waves);
    if (RB || p.kch == 1) hipLaunchKernelGGL((hx_kernel<NS, RB, true>), gd, bd, lds, st, p, src, od, g, p.ea);
    else hipLaunchKernelGGL((hx_kernel<NS, RB, false>), gd, bd, lds, st, p, src, od, g, p.ea);
    return hipGetLastError();
}

hipError_t launchHx(const HxDev& p, const SrcDesc& src, const OutDesc& od, int C, hipStream_t stream) {
    if (od.o_hi <= od.o_lo) return hipSuccess;
    // development knobs: GAR_HX_G caps macro periods per column; GAR_HX_DBG bit 1 skips staging
    // after the first block, bit 2 skips the MFMA programs (timing decomposition only)
    static const int knobG = std::getenv("GAR_HX_G") ? std::atoi(std::getenv("GAR_HX_G")) : 0;
    static const int knobDbg = std::getenv("GAR_HX_DBG") ? std::atoi(std::getenv("GAR_HX_DBG")) : 0;
    BgGrid g{};
    g.Pc = p.Pc; g.Qc = p.Qc; g.Kc = p.Kc; g.C = C;
    g.nprog = p.nw; g.kch = p.kch; g.nwt = p.nw; g.ncg = 1;
    g.nred = p.nred; g.nslots = p.nslots;
    g.a_lo = od.o_lo / p.Pc;
    const int64_t a_hi = (od.o_hi + p.Pc - 1) / p.Pc;
    const int64_t nmac = a_hi - g.a_lo;
    const size_t slotBytes = static_cast<size_t>(g.nslots) * 256 * 4;
    const size_t kLds = 160 * 1024;
    auto wsFor = [&](int G) { return (p.Kread + (G - 1) * p.Qc + 63) / 64 * 64; };  // whole DMA row chunks
    auto ldsFor = [&](int G, int par) { return 4 * static_cast<size_t>(wsFor(G)) * 32 + (par ? 2 : 1) * slotBytes + 128; };
    g.parity = (g.nred > 0 && ldsFor(1, 1) <= kLds) ? 1 : 0;
    int dev = 0, ncu = 256;
    if (hipGetDevice(&dev) == hipSuccess) (void)hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev);
    // G macro periods per column: the largest whose window fits the producers'
    // register staging and LDS without dropping below one block per CU (when
    // the launch is large enough for that)
    auto nbFor = [&](int G) { return ((nmac + G - 1) / G * C + 15) / 16; };
    int G = 1;
    for (int cand = 2; cand <= 8; ++cand) {
        if (cand > nmac || wsFor(cand) > kHxMaxRows || ldsFor(cand, g.parity) > kLds) break;
        if (nbFor(cand) < ncu && nbFor(1) >= ncu) break;
        G = cand;
    }
    if (knobG > 0 && knobG < G) G = knobG;
    if (wsFor(G) > kHxMaxRows || ldsFor(G, g.parity) > kLds) return hipErrorInvalidConfiguration;
    g.G = G;
    g.W = p.Kc + (G - 1) * p.Qc;
    g.Wl = p.Kread + (G - 1) * p.Qc;
    g.Ws = wsFor(G);
    const int64_t nchunk = (nmac + G - 1) / G;
    g.nchunk = static_cast<int>(nchunk);
    g.ncols = static_cast<int>(nchunk * C);
    g.nblocks = (g.ncols + 15) / 16;
    g.dbg = knobDbg;
    g.vst = 0;
    if (!od.f64) {
        if (od.fs == 1) g.vst = 1;
        else if (C == 2 && od.fs == 2 && od.cs == 1) g.vst = 2;
    }
    if (g.nblocks <= 0) return hipSuccess;
    const size_t lds = ldsFor(G, g.parity);
    const int64_t blocks = std::min<int64_t>(g.nblocks, ncu);
    if (p.rb) {
        if (p.nw > kHxRbMaxWaves) return hipErrorInvalidConfiguration;
        switch (p.NS) {
            case 1: return hxDispatch<1, true>(p, src, od, g, lds, blocks, stream);
            case 2: return hxDispatch<2, true>(p, src, od, g, lds, blocks, stream);
            case 3: return hxDispatch<3, true>(p, src, od, g, lds, blocks, stream);
            case 4: return hxDispatch<4, true>(p, src, od, g, lds, blocks, stream);
            case 5: return hxDispatch<5, true>(p, src, od, g, lds, blocks, stream);
            case 6: return hxDispatch<6, true>(p, src, od, g, lds, blocks, stream);
            case 7: return hxDispatch<7, true>(p, src, od, g, lds, blocks, stream);
            case 8: return hxDispatch<8, true>(p, src, od, g, lds, blocks, stream);
            case 9: return hxDispatch<9, true>(p, src, od, g, lds, blocks, stream);
            case 10: return hxDispatch<10, true>(p, src, od, g, lds, blocks, stream);
            default: return hipErrorInvalidConfiguration;
        }
    }
    switch (p.NS) {
        case 2: return hxDispatch<2, false>(p, src, od, g, lds, blocks, stream);
        case 4: return hxDispatch<4, false>(p, src, od, g, lds, blocks, stream);
        case 6: return hxDispatch<6, false>(p, src, od, g, lds, blocks, stream);
        case 8: return hxDispatch<8, false>(p, src, od, g, lds, blocks, stream);
        case 10: return hxDispatch<10, false>(p, src, od, g, lds, blocks, stream);
        case 12: return hxDispatch<12, false>(p, src, od, g, lds, blocks, stream);
        default: return hipErrorInvalidConfiguration;
    }
}

}  // namespace gar
