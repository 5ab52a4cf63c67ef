// gar_hx.hip -- launch geometry of the split-f16 FIR kernel (gar_hx.hpp).  Every
// output of a launch, edges included, runs on hx_kernel.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>

#include "gar_hx.hpp"

namespace gar {

// hxLaunch instantiations live in gar_hx_i*.hip (compiled in parallel)
#define GAR_HX_EXTERN(NS, RB, V) \
    extern template hipError_t hxLaunch<NS, RB, V>(const HxArgs&, int, size_t, int64_t, int64_t, hipStream_t);
GAR_HX_FOR_ALL(GAR_HX_EXTERN)
#undef GAR_HX_EXTERN

namespace {


// row-block mode: the epilogue store layout (HxArgs::vst) is a template parameter
template <int NS, bool RB>
hipError_t hxDispatch(const HxArgs& x, int waves, size_t lds, int64_t blocks, int64_t eblocks, hipStream_t st) {
    if constexpr (!RB) return hxLaunch<NS, false, 0>(x, waves, lds, blocks, eblocks, st);
    switch (x.vst) {
        case 0: return hxLaunch<NS, RB, 0>(x, waves, lds, blocks, eblocks, st);
        case 1: return hxLaunch<NS, RB, 1>(x, waves, lds, blocks, eblocks, st);
        case 2: return hxLaunch<NS, RB, 2>(x, waves, lds, blocks, eblocks, st);
        default: return hxLaunch<NS, RB, 3>(x, waves, lds, blocks, eblocks, st);
    }
}

int64_t floorDiv(int64_t a, int64_t b) { return a >= 0 ? a / b : -((-a + b - 1) / b); }
int64_t ceilDiv(int64_t a, int64_t b) { return -floorDiv(-a, b); }

}  // namespace

hipError_t launchHx(const HxDev& p, const SrcDesc& src, const OutDesc& od, int C, hipStream_t stream, HistCopy* hc) {
    if (od.o_hi <= od.o_lo) return hipSuccess;
    // row-block plans stream through the wave-specialised kernel (GAR_HXS=0: the block kernel, A/B runs)
    static const bool hxs = !(std::getenv("GAR_HXS") && std::getenv("GAR_HXS")[0] == '0');
    if (p.rb && hxs) {
        const hipError_t e = launchHxs(p, src, od, C, stream, hc);
        if (e != hipErrorNotSupported) return e;
    }
    if (od.pcm) return hipErrorNotSupported;  // PCM output is fused into hxs_kernel only (engine stages it otherwise)
    // development knobs: GAR_HX_G caps macro periods per column; GAR_HX_DBG bits: 1 skip
    // staging after the first block, 2 skip the MFMA programs, 16 skip the loop
    static const int knobG = std::getenv("GAR_HX_G") ? std::atoi(std::getenv("GAR_HX_G")) : 0;
    static const int knobDbg = std::getenv("GAR_HX_DBG") ? std::atoi(std::getenv("GAR_HX_DBG")) : 0;
    const int64_t Pc = p.Pc, Qc = p.Qc;
    const int64_t a_lo = floorDiv(od.o_lo, Pc);
    const int64_t nmac = ceilDiv(od.o_hi, Pc) - a_lo;
    const size_t kLds = 160 * 1024;
    // window rows staged per column (the padded program steps read up to Kread + (G-1)*Qc),
    // whole 64-row item slots
    auto wsFor = [&](int G) { return (p.Kread + (G - 1) * p.Qc + 63) / 64 * 64; };
    const int parity = (p.nred > 0 && hxLdsBytes(wsFor(1), p.nslots, 1) <= kLds) ? 1 : 0;
    auto ldsFor = [&](int G) { return hxLdsBytes(wsFor(G), p.nslots, parity); };
    int dev = 0, ncu = 256;
    if (hipGetDevice(&dev) == hipSuccess) (void)hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev);
    // G macro periods per column: the largest whose window fits LDS without
    // dropping below one block per CU (small launches: G = 1, the most blocks)
    auto nbFor = [&](int G) { return ((nmac + G - 1) / G * C + 15) / 16; };
    int G = 1;
    for (int cand = 2; cand <= 8; ++cand) {
        if (cand > nmac || wsFor(cand) > kHxMaxRows || ldsFor(cand) > kLds) break;
        if (nbFor(cand) < ncu) break;
        G = cand;
    }
    if (knobG > 0 && knobG < G) G = knobG;
    if (wsFor(G) > kHxMaxRows || ldsFor(G) > kLds) return hipErrorInvalidConfiguration;
    const int64_t W = p.Kc + static_cast<int64_t>(G - 1) * Qc;
    const int64_t nchunk = (nmac + G - 1) / G;
    const int64_t ncols = nchunk * C;
    if (ncols > (int64_t(1) << 30)) return hipErrorInvalidConfiguration;

    // interior chunks [k0, k1): outputs inside [o_lo, o_hi), window rows [0, W) inside the f32 input,
    // and 32-bit lane offsets (row * frame stride) inside a buffer resource
    int64_t k0 = 0, k1 = 0;
    const bool fastIn = src.in && !src.in_f64 && !src.in_pcm && src.in_len > 0 &&
                        static_cast<double>(wsFor(G)) * static_cast<double>(std::llabs(src.in_fs)) * 4.0 < 2147483647.0 &&
                        src.in_fs > 0 && src.in_cs >= 0;
    if (fastIn) {
        const int64_t GQ = G * Qc, GP = G * Pc;
        const int64_t inEnd = std::min(src.in_base + src.in_len, src.valid_end);
        k0 = std::max<int64_t>({0, ceilDiv(od.o_lo - a_lo * Pc, GP), ceilDiv(src.in_base - a_lo * Qc, GQ)});
        k1 = std::min<int64_t>({nchunk, floorDiv(od.o_hi - a_lo * Pc, GP), floorDiv(inEnd - W - a_lo * Qc, GQ) + 1});
        // an empty interior range stays inside [0, nchunk]: a short call whose windows all cross the
        // history seam has k0 > nchunk (e.g. 399 frames after 912 history rows), and an interior
        // range placed past the last chunk made ib1 > nblocks below (sweep: 88.2k -> 44.1k High)
        k0 = std::min(k0, nchunk);
        if (k1 < k0) k1 = k0;
    }
    static const bool trace = std::getenv("GAR_HX_TRACE") != nullptr;
    if (trace)
        fprintf(stderr, "hx: o[%lld,%lld) C=%d G=%d W=%lld a_lo=%lld nchunk=%lld k0=%lld k1=%lld in_base=%lld in_len=%lld valid_end=%lld hist_len=%lld\n",
                (long long)od.o_lo, (long long)od.o_hi, C, G, (long long)W, (long long)a_lo, (long long)nchunk,
                (long long)k0, (long long)k1, (long long)src.in_base, (long long)src.in_len, (long long)src.valid_end,
                (long long)src.hist_len);

    HxArgs x{};
    x.A = static_cast<const h8v*>(p.A);
    x.progs = p.progs;
    x.reds = p.reds;
    x.ea = p.ea;
    x.kch = p.kch;
    x.Pc = p.Pc; x.Qc = p.Qc; x.G = G; x.C = C;
    x.W = static_cast<int>(W);
    x.Ws = wsFor(G);
    x.ncols = static_cast<int>(ncols);
    x.nblocks = static_cast<int>((ncols + 15) / 16);
    x.nred = p.nred; x.nslots = p.nslots; x.parity = parity;
    x.dbg = knobDbg;
    x.k0 = static_cast<int>(k0);
    x.k1 = static_cast<int>(k1);
    x.a_lo = a_lo;
    x.o_lo = od.o_lo;
    x.o_hi = od.o_hi;
    // pointer arithmetic in integers: chunk 0 may start before the caller's buffers
    const int isz = 4;
    x.in = reinterpret_cast<const float*>(reinterpret_cast<uintptr_t>(src.in) +
                                          static_cast<intptr_t>((a_lo * Qc - src.in_base) * src.in_fs * isz));
    x.in_fs = src.in_fs;
    x.in_cs = src.in_cs;
    x.in_chunk = G * Qc * src.in_fs;
    const int esz = od.f64 ? 8 : 4;
    x.out_f64 = od.f64;
    x.out = reinterpret_cast<char*>(reinterpret_cast<uintptr_t>(od.out) +
                                    static_cast<intptr_t>((a_lo * Pc - od.o0) * od.fs * esz));
    x.out_fs = od.fs * esz;
    x.out_cs = od.cs * esz;
    x.out_chunk = G * Pc * od.fs * esz;
    // epilogue layout of interior blocks (16-B stores need every row quad 16-B aligned)
    const bool al = (reinterpret_cast<uintptr_t>(x.out) & 15) == 0 && ((G * Pc * od.fs * esz) & 15) == 0;
    if (od.f64) x.vst = 3;
    else if (al && C == 2 && od.fs == 2 && od.cs == 1 && Pc % 2 == 0) x.vst = 2;
    else if (al && od.fs == 1 && (od.cs * 4) % 16 == 0 && Pc % 4 == 0) x.vst = 1;
    else x.vst = 0;
    // raw load format of interior blocks: 8-B stereo frames / 16-B four-channel rows where the layout
    // allows it; per-block buffer resources need every in-block offset below 2^31 (else 64-bit loads)
    const uintptr_t inA = reinterpret_cast<uintptr_t>(src.in);
    x.fmt = 0;
    if ((inA & 7) == 0 && C == 2 && src.in_fs == 2 && src.in_cs == 1) x.fmt = 1;
    else if ((inA & 15) == 0 && C % 4 == 0 && src.in_cs == 1 && src.in_fs % 4 == 0) x.fmt = 2;
    static const bool noFmt = std::getenv("GAR_HX_DWORD") != nullptr;
    if (noFmt) x.fmt = 0;
    {
        const double chunksPerBlock = 16.0 / C + 2.0;
        const double maxOff = chunksPerBlock * static_cast<double>(x.in_chunk) * 4.0 +
                              static_cast<double>(C) * static_cast<double>(src.in_cs) * 4.0 + 16.0;
        if (maxOff >= 2147483647.0) x.fmt = 3;
    }
    x.src = src;
    x.od = od;
    x.rows = p.rows;
    x.rowOff = p.rowOff;
    x.rowLen = p.rowLen;
    x.rowMax = p.rowMax;
    x.twoStage = p.twoStage;
    x.rowPh = p.rowPh;
    x.rowPar = p.rowPar;
    x.polyA = p.polyA;
    x.dftC = p.dftC;
    x.T1 = p.T1;
    x.T2 = p.T2;

    // interior blocks: every column an interior chunk
    x.ib0 = static_cast<int>(std::min<int64_t>((k0 * C + 15) / 16, x.nblocks));
    x.ib1 = static_cast<int>(std::max<int64_t>(x.ib0, std::min<int64_t>((k1 * C) / 16, x.nblocks)));
    x.fix = p.fix;
    x.fixCap = p.fixCap;

    const size_t lds = ldsFor(G);
    const int64_t nInt = x.ib1 - x.ib0;
    const int64_t nEdge = x.nblocks - nInt;
    const int64_t blocks = std::min<int64_t>(nInt, ncu);
    // edge blocks + workgroups draining the interior kernel's (normally empty) fix list
    const int64_t eblocks = std::max<int64_t>(nEdge, 1) + (nInt > 0 ? kHxFixWgs : 0);
    if (nInt > 0) {
        const hipError_t e = hipMemsetAsync(p.fix, 0, sizeof(int), stream);
        if (e != hipSuccess) return e;
    }
    x.nprog = p.nw;
    if (p.rb) {
        if (p.nw > kHxRbMaxWaves) return hipErrorInvalidConfiguration;
        const int waves = std::max(p.nw, kHxMinWaves);
        switch (p.NS) {
#define GAR_HX_RB(n) case n: return hxDispatch<n, true>(x, waves, lds, blocks, eblocks, stream);
            GAR_HX_RB(1) GAR_HX_RB(2) GAR_HX_RB(3) GAR_HX_RB(4) GAR_HX_RB(5) GAR_HX_RB(6) GAR_HX_RB(7) GAR_HX_RB(8)
            GAR_HX_RB(9) GAR_HX_RB(10)
#undef GAR_HX_RB
            default: return hipErrorInvalidConfiguration;
        }
    }
    switch (p.NS) {
#define GAR_HX_SEG(n) case n: return hxDispatch<n, false>(x, kHxWaves, lds, blocks, eblocks, stream);
        GAR_HX_SEG(2) GAR_HX_SEG(4) GAR_HX_SEG(6) GAR_HX_SEG(8)
#undef GAR_HX_SEG
        default: return hipErrorInvalidConfiguration;
    }
}

}  // namespace gar
