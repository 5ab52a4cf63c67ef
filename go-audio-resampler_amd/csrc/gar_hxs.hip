// gar_hxs.hip -- launch geometry of the streaming split-f16 kernel (gar_hxs.hpp)
// for row-block plans.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <utility>
#include <vector>

#include "gar_hxt.hpp"

namespace gar {

// instantiations live in gar_hxs_i1.hip / gar_hxs_i2.hip (compiled in parallel)
#define GAR_HXS_EXT(NS, V) extern template hipError_t hxsLaunch<NS, V>(const HxsArgs&, size_t, int64_t, hipStream_t);
GAR_HXS_FOR_ALL(GAR_HXS_EXT)
#undef GAR_HXS_EXT
// hxt_kernel instantiations: gar_hxt_i1.hip / gar_hxt_i2.hip
#define GAR_HXT_EXT(NS, F, V, L) extern template hipError_t hxtLaunch<NS, F, V, L>(const HxsArgs&, size_t, int64_t, hipStream_t);
GAR_HXT_FOR_A(GAR_HXT_EXT)
GAR_HXT_FOR_B(GAR_HXT_EXT)
#undef GAR_HXT_EXT

namespace {
constexpr int kProfWords = 64 + 2 * 4096;
// development: GAR_HXS_PROF=1 sums per-phase s_memtime cycles of every launch and prints them at exit
unsigned long long* profBuf() {
    static unsigned long long* p = nullptr;
    static bool init = false;
    if (!init) {
        init = true;
        if (std::getenv("GAR_HXS_PROF") && hipMalloc(&p, kProfWords * sizeof(unsigned long long)) == hipSuccess) {
            (void)hipMemset(p, 0, kProfWords * sizeof(unsigned long long));
            (void)hipMemset(p + 10, 0xff, sizeof(unsigned long long));
            (void)hipMemset(p + 13, 0xff, sizeof(unsigned long long));
            std::atexit([] {
                static unsigned long long h[kProfWords] = {};
                if (hipDeviceSynchronize() == hipSuccess && hipMemcpy(h, p, sizeof(h), hipMemcpyDeviceToHost) == hipSuccess) {
                    const double nl = h[3] ? static_cast<double>(h[3]) : 1, nc = h[6] ? static_cast<double>(h[6]) : 1;
                    fprintf(stderr, "hxs prof per wave (cycles): loaders convert %.0f issue+wait %.0f (issue %.0f) barrier %.0f (life %.1f us) | compute convert+mfma %.0f barrier %.0f\n",
                            h[0] / nl, h[1] / nl, h[7] / nl, h[2] / nl, h[9] / nl / 100.0, h[4] / nc, h[5] / nc);
                    fprintf(stderr, "hxs loader pre-loop %.2f us, post-loop %.2f us; compute convert %.0f\n", h[8] / nl / 100.0, h[12] / nl / 100.0, h[15] / nc);
                    if (h[23]) fprintf(stderr, "hxs wave-0 first block (cycles): entry->window %.0f, window->steps done %.0f, ->exit (stores drained) %.0f, n %llu\n",
                                       static_cast<double>(h[20]) / h[23], static_cast<double>(h[21]) / h[23], static_cast<double>(h[22]) / h[23], h[23]);
                    if (h[23]) fprintf(stderr, "hxs wave-0: entry->A landed %.0f, entry->barrier 1 %.0f; wave entry spread in a workgroup %.0f, wave 0 after first wave %.0f\n",
                                       static_cast<double>(h[24]) / h[23], static_cast<double>(h[25]) / h[23], static_cast<double>(h[26]) / h[23], static_cast<double>(h[27]) / h[23]);
                    if (h[34]) fprintf(stderr, "hxt roles per block (cycles): compute wave 0 %.0f (waiting %.0f), loader 0 %.0f (waiting %.0f), n %llu\n",
                                       static_cast<double>(h[30]) / h[34], static_cast<double>(h[32]) / h[34], static_cast<double>(h[31]) / h[34],
                                       static_cast<double>(h[33]) / h[34], h[34]);
                    if (h[34]) fprintf(stderr, "hxt compute wave 0: entry -> first group %.0f cycles, last group -> exit %.0f cycles, periods %.0f, arrivals %.0f\n",
                                       static_cast<double>(h[35]) / h[34], static_cast<double>(h[36]) / h[34],
                                       static_cast<double>(h[37]) / h[34], static_cast<double>(h[38]) / h[34]);
                    if (h[34] && h[57]) fprintf(stderr, "hxt fill (cycles): entry -> A issued %.0f, -> fill barrier %.0f, -> first group %.0f; in-kernel clock %.3f GHz\n",
                                       static_cast<double>(h[53]) / h[34], static_cast<double>(h[54]) / h[34], static_cast<double>(h[55]) / h[34],
                                       0.1 * static_cast<double>(h[56]) / static_cast<double>(h[57]));
                    if (h[34]) fprintf(stderr, "hxt loader 0 phases (cycles): load data wait %.0f, conversion %.0f, arrival %.0f\n",
                                       static_cast<double>(h[50]) / h[34], static_cast<double>(h[51]) / h[34], static_cast<double>(h[52]) / h[34]);
                    if (h[44]) fprintf(stderr, "hxq wave 0 (cycles): entry->barrier 1 %.0f, ->image %.0f, ->MFMA+stores issued %.0f, ->drained %.0f, n %llu\n",
                                       static_cast<double>(h[40]) / h[44], static_cast<double>(h[41]) / h[44], static_cast<double>(h[42]) / h[44],
                                       static_cast<double>(h[43]) / h[44], h[44]);
                    fprintf(stderr, "hxs span: first start -> last end %.1f us; loader wave life min %.1f max %.1f us\n",
                            (h[11] - h[10]) / 100.0, h[13] / 100.0, h[14] / 100.0);
                    // per-workgroup life (last launch): percentiles, by blockIdx % 8, slowest
                    std::vector<std::pair<double, int>> v;
                    unsigned long long t0 = ~0ull;
                    for (int b = 0; b < 4096; ++b)
                        if (h[65 + 2 * b]) { v.push_back({h[65 + 2 * b] / 100.0, b}); t0 = std::min(t0, h[64 + 2 * b]); }
                    if (!v.empty()) {
                        std::vector<std::pair<double, int>> sv = v;
                        std::sort(sv.begin(), sv.end());
                        auto pc = [&](double q) { return sv[std::min(sv.size() - 1, static_cast<size_t>(q * sv.size()))].first; };
                        fprintf(stderr, "hxs WG life us: n %zu min %.1f p10 %.1f p50 %.1f p90 %.1f max %.1f |", sv.size(), sv.front().first, pc(0.1), pc(0.5), pc(0.9), sv.back().first);
                        for (int m = 0; m < 8; ++m) {
                            double s = 0; int n = 0;
                            for (auto& e : v) if (e.second % 8 == m) { s += e.first; ++n; }
                            fprintf(stderr, " x%d %.1f", m, n ? s / n : 0.0);
                        }
                        fprintf(stderr, "\n  slowest:");
                        for (size_t k = sv.size(); k-- > 0 && k + 8 >= sv.size();)
                            fprintf(stderr, " b%d %.1fus@+%.1f", sv[k].second, sv[k].first, (h[64 + 2 * sv[k].second] - t0) / 100.0);
                        fprintf(stderr, "\n");
                    }
                }
            });
        }
    }
    return p;
}

int64_t fdiv(int64_t a, int64_t b) { return a >= 0 ? a / b : -((-a + b - 1) / b); }
int64_t cdiv(int64_t a, int64_t b) { return -fdiv(-a, b); }

template <int NS, int NL>
hipError_t hxtFmtL(const HxsArgs& x, size_t lds, int64_t blocks, hipStream_t st) {
    if (x.fmt == 1 && x.vst == 2) return hxtLaunch<NS, 1, 2, NL>(x, lds, blocks, st);
    if (x.fmt == 2 && x.vst == 0) return hxtLaunch<NS, 2, 0, NL>(x, lds, blocks, st);
    if (x.fmt == 2 && x.vst == 1) return hxtLaunch<NS, 2, 1, NL>(x, lds, blocks, st);
    if (x.fmt == 5 && x.vst == 0) return hxtLaunch<NS, 5, 0, NL>(x, lds, blocks, st);
    return hipErrorNotSupported;
}
template <int NS>
hipError_t hxtFmt(const HxsArgs& x, size_t lds, int64_t blocks, hipStream_t st) {
    return x.ncomp + 6 <= kHxtWaves ? hxtFmtL<NS, 6>(x, lds, blocks, st) : hxtFmtL<NS, 4>(x, lds, blocks, st);
}

// Compute-wave roles of hxt_kernel for nprog row blocks (HxsArgs::role): the first 4*floor(nprog/4)
// row blocks one wave each; one remaining row block shared by 4 waves (every 4th period), two by
// 2 waves each (every 2nd period), so waves w, w+4, w+8 -- one SIMD -- carry equal MFMA work.
// Returns the compute wave count; *maxStride the largest period stride.
static int hxtRoles(int nprog, int NS, int* role, int* maxStride) {
    // knob GAR_HXT_ROLES: 1 balanced, 0 one wave per row block; default balanced for NS >= 10 only
    // (profiles/r04_ab: NS = 9 cfg2 0.125 ms one-per-row-block vs 0.145 balanced -- six loaders
    // beside ten compute waves keep the ring ahead; NS = 10 cfg3 is the other way round)
    static const int knobRoles = std::getenv("GAR_HXT_ROLES") ? std::atoi(std::getenv("GAR_HXT_ROLES")) : -1;
    const bool balanced = knobRoles >= 0 ? knobRoles != 0 : NS >= 10;
    int w = 0;
    *maxStride = 1;
    if (!balanced) {  // one wave per row block (hxs_kernel's mapping), six loaders beside ten compute waves
        for (int i = 0; i < nprog; ++i) role[w++] = i | (1 << 16);
        return w;
    }
    const int q = nprog / 4 * 4, r = nprog - q;
    for (int i = 0; i < q; ++i) role[w++] = i | (1 << 16);
    if (r == 2 && q + 4 <= kHxtMaxComp) {
        for (int i = 0; i < 4; ++i) role[w++] = (q + (i & 1)) | ((i >> 1) << 8) | (2 << 16);
        *maxStride = 2;
    } else if (r == 1 && q + 4 <= kHxtMaxComp) {
        for (int i = 0; i < 4; ++i) role[w++] = q | (i << 8) | (4 << 16);
        *maxStride = 4;
    } else {
        for (int i = q; i < nprog; ++i) role[w++] = i | (1 << 16);
    }
    return w;
}

template <int NS>
hipError_t hxsVst(const HxsArgs& x, size_t lds, int64_t blocks, hipStream_t st) {
    switch (x.vst) {
        case 0: return hxsLaunch<NS, 0>(x, lds, blocks, st);
        case 1: return hxsLaunch<NS, 1>(x, lds, blocks, st);
        case 2: return hxsLaunch<NS, 2>(x, lds, blocks, st);
        case 4: return hxsLaunch<NS, 4>(x, lds, blocks, st);
        default: return hxsLaunch<NS, 3>(x, lds, blocks, st);
    }
}
}  // namespace

// LDS bytes of an hxs launch: ring (four quads of hi + lo rows), loud ranges + flag, hxt_kernel's
// progress counters (kHxtSyncOff + kHxtSyncBytes, rounded up).
static_assert(kHxtSyncOff + kHxtSyncBytes <= 320, "hxt progress counters past the reserved LDS");
static size_t hxsLds(int Rt) { return 4 * (16 * static_cast<size_t>(Rt) + 64) + 320; }
// hxt_kernel FMT 5 (32-channel blocks): eight quads, loudLo/Hi[32] + flag + the progress counters
static_assert(288 + kHxtSyncBytes <= 448, "hxt FMT 5 progress counters past the reserved LDS");
static size_t hxtLdsWide(int Rt) { return 8 * (16 * static_cast<size_t>(Rt) + 64) + 448; }

// Ring geometry of G periods per group: R ring rows, Rt rows incl. the mirror (rounded to 16 so
// the quad stride 16*Rt + 64 is 64 mod 256 B: the four quads of a transposed read land on
// distinct banks), Wg rows one group reads.
static void hxsRingFor(const HxDev& p, int G, int& R, int& Rt, int& Wg) {
    const int GQ = G * p.Qc;
    Wg = (G - 1) * p.Qc + p.Kread;
    const int n = (Wg + GQ + GQ - 1) / GQ;
    R = n * GQ;
    Rt = (R + std::max(0, Wg - GQ) + 15) / 16 * 16;
}
// Static LDS of hxs_kernel next to the dynamic ring: the development build's per-wave stamps.
constexpr size_t kHxsStaticLds = kHxsDev ? sizeof(unsigned long long) * kHxsWaves : 0;
static bool hxsRingFits(const HxDev& p, int G, int Rt) {
    return hxsLds(Rt) + kHxsStaticLds <= 160 * 1024 && (G * p.Qc + 63) / 64 <= kHxsNP;
}

// NS values with an instantiated kernel (GAR_HXS_QUICK development builds: only 9 and 10).
static bool hxsNsBuilt(int ns) { return GAR_HXS_QUICK ? (ns == 9 || ns == 10) : (ns >= 1 && ns <= 10); }

bool hxsPlanFits(const HxDev& p) {
    if (!p.rb || p.nw > kHxRbMaxWaves || !hxsNsBuilt(p.NS)) return false;
    int R, Rt, Wg;
    hxsRingFor(p, 1, R, Rt, Wg);
    return hxsRingFits(p, 1, Rt);
}

// hipErrorNotSupported: the plan does not fit this kernel's geometry (the caller uses hx_kernel).
hipError_t launchHxs(const HxDev& p, const SrcDesc& src, const OutDesc& od, int C, hipStream_t stream, HistCopy* hc) {
    if (od.o_hi <= od.o_lo) return hipSuccess;
    if (!p.rb || p.nw > kHxRbMaxWaves || !hxsNsBuilt(p.NS)) return hipErrorNotSupported;
    static const int knobG = std::getenv("GAR_HXS_G") ? std::atoi(std::getenv("GAR_HXS_G")) : 0;
    static const int knobWg = std::getenv("GAR_HXS_WGPERCU") ? std::atoi(std::getenv("GAR_HXS_WGPERCU")) : 0;
    static const bool trace = std::getenv("GAR_HX_TRACE") != nullptr;
    static const int knobDbg = std::getenv("GAR_HXS_DBG") ? std::atoi(std::getenv("GAR_HXS_DBG")) : 0;
    const int64_t Pc = p.Pc, Qc = p.Qc;
    const int64_t a_lo = fdiv(od.o_lo, Pc), a_hi = cdiv(od.o_hi, Pc);
    const int64_t nmac = a_hi - a_lo;
    int dev = 0, ncu = 256;
    if (hipGetDevice(&dev) == hipSuccess) (void)hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev);

    // small launches (stream chunks, flush tails): one macro period per column, each block's
    // window gathered in one pass -- latency over bandwidth (knob GAR_HXS_SMALL=0/1 forces)
    static const int knobSmall = std::getenv("GAR_HXS_SMALL") ? std::atoi(std::getenv("GAR_HXS_SMALL")) : -1;
    const bool small = knobSmall >= 0 ? knobSmall == 1 : nmac * C <= static_cast<int64_t>(16) * 2 * ncu;
    // 32-channel blocks of f32 rows on hxt_kernel (FMT 5, gar_hxt.hpp): whole 128-B lines per load and
    // store instruction; decided here (the chunk count depends on the block width), confirmed below
    const uintptr_t inA0 = reinterpret_cast<uintptr_t>(src.in);
    bool wide = !small && src.in && !src.in_pcm && !src.in_f64 && !od.pcm && !od.f64 && C % 32 == 0 && od.cs == 1 &&
                (inA0 & 15) == 0 && src.in_cs == 1 && src.in_fs % 4 == 0 && p.rb && p.nw <= kHxRbMaxWaves;
    if (wide) {  // knob GAR_HXT_WIDE=0: 16-channel blocks (read per launch, so one test process compares both)
        const char* e = std::getenv("GAR_HXT_WIDE");
        wide = !e || std::atoi(e) != 0;
    }
    if (wide) {
        // only where the 32-channel ring takes groups of >= 2 periods and the plan runs one compute wave per
        // row block (balanced roles, NS = 10 as cfg3, measured slower on 32 channels) -- decided before the
        // chunk count, which is sized for the block width (r06g: cfg3 fell back to 16-channel blocks after
        // chunks sized for 32, 512 half-length blocks, traffic / algorithmic 1.06 -> 1.12, +7 %)
        int rl[kHxtMaxComp] = {}, ms = 1;
        const int nc = hxtRoles(p.nw, p.NS, rl, &ms);
        int r2, rt2, wg2;
        hxsRingFor(p, 2, r2, rt2, wg2);
        wide = ms == 1 && hxtLdsWide(rt2) <= 160 * 1024 && 2 * Qc <= hxtMaxRowsF(5, nc + 6 <= kHxtWaves ? 6 : 4) &&
               r2 / (2 * static_cast<int>(Qc)) + 3 <= kHxtSlots;
    }
    const int bw = wide ? 32 : 16;
    // chunk length: about one block (bw columns) per CU
    const int64_t targetBlocks = static_cast<int64_t>(ncu) * (knobWg > 0 ? knobWg : 1);
    const int64_t nchunkT = small ? nmac : std::max<int64_t>(1, (targetBlocks * bw + C - 1) / C);
    int64_t Np = std::max<int64_t>(1, cdiv(nmac, nchunkT));
    static const int knobNp = std::getenv("GAR_HXS_NP") ? std::atoi(std::getenv("GAR_HXS_NP")) : 0;
    if (knobNp > 0 && !small) Np = knobNp;  // development: chunk length in macro periods
    // raw loads address a chunk's rows with 32-bit offsets from the chunk's first row:
    // (Np*Qc + rows of one group + a piece) rows must span less than 2^31 bytes
    const int inEsz = src.in_pcm ? pcmBytes(src.in_pcm) : (src.in_f64 ? 8 : 4);
    const int64_t rowBytes = std::max<int64_t>(4, src.in_fs * inEsz);
    const int64_t chunksPerRsrc = (C <= 16 && 16 % C == 0) ? 16 / C : 1;  // STEREO: one resource spans 8 chunks
    const int64_t npMax = ((int64_t(1) << 31) / rowBytes / chunksPerRsrc - (3 * Qc + p.Kread + 256)) / Qc;
    const bool rawSpan = npMax >= 1;
    if (rawSpan) Np = std::min(Np, npMax);
    int64_t nchunk = cdiv(nmac, Np);
    // whole blocks where the channel count divides 16 (empty trailing chunks read zeros, store nothing)
    if (16 % C == 0 && !small) nchunk = cdiv(nchunk * C, 16) * 16 / C;
    const int64_t ncols = nchunk * C;
    if (ncols > (int64_t(1) << 30) || Np > (int64_t(1) << 24)) return hipErrorNotSupported;

    // group size: largest G <= kHxsMaxG that fits the LDS ring and the loaders' registers, not above Np
    // load layout: STEREO frames (two chunks per quad, dwordx2), ROW16 (four channels per quad,
    // dwordx4), or gathered at conversion time for any other layout
    const uintptr_t inA = reinterpret_cast<uintptr_t>(src.in);
    int fmt = 0;
    const bool stereoIl = C == 2 && src.in_fs == 2 && src.in_cs == 1;
    if (!src.in) {
        // no caller input (a flush: history + zeros): every row comes from the history, [t][C] f32 with
        // row stride hist_ld, so take the load layout from it -- STEREO frames or ROW16 rows -- instead
        // of per-column element gathers (cfg2's flush launch: 13.7 us on the gathers, r05d trace)
        const uintptr_t hA = reinterpret_cast<uintptr_t>(src.hist);
        if (C == 2 && src.hist_ld == 2 && (hA & 7) == 0) fmt = 1;
        else if (C % 16 == 0 && src.hist_ld % 4 == 0 && (hA & 15) == 0) fmt = 2;
    } else if (src.in_pcm == 16) {  // PCM16 / PCM24-32 stereo frames; other PCM layouts are gathered
        if ((inA & 3) == 0 && stereoIl) fmt = 3;
    } else if (src.in_pcm) {
        if ((inA & 7) == 0 && stereoIl) fmt = 4;
    } else if (src.in_f64) {
    } else if ((inA & 7) == 0 && stereoIl) {
        fmt = 1;
    } else if ((inA & 15) == 0 && C % 16 == 0 && src.in_cs == 1 && src.in_fs % 4 == 0) {
        fmt = 2;
    }
    // output layout of the epilogue (hxsStoreFast VST), see below
    const int esz = od.pcm ? pcmBytes(od.pcm) : (od.f64 ? 8 : 4);
    char* const outBase = reinterpret_cast<char*>(reinterpret_cast<uintptr_t>(od.out) - static_cast<uintptr_t>(od.o0 * od.fs * esz));
    const bool al = (reinterpret_cast<uintptr_t>(outBase) & 15) == 0;
    int vst;
    if (od.pcm == 16 && al && C == 2 && od.fs == 2 && od.cs == 1 && Pc % 4 == 0) vst = 4;  // int16 stereo frame pairs
    else if (od.pcm) vst = 0;  // other PCM stores: the epilogue's checked per-element path
    else if (od.f64) vst = 3;
    else if (al && C == 2 && od.fs == 2 && od.cs == 1 && Pc % 4 == 0) vst = 2;
    else if (al && od.fs == 1 && (od.cs * 4) % 16 == 0 && Pc % 4 == 0) vst = 1;
    else vst = 0;

    // balanced kernel (hxt_kernel): f32 stereo frames or 16-channel rows in, f32 out (knob GAR_HXT=0: hxs_kernel)
    // Default (knob unset): hxt_kernel wherever its load / store layouts apply -- after its loader spill
    // fixes it beats hxs_kernel on every BASELINE plan (profiles/r04_ab: cfg2 0.125 vs 0.130 ms, ns256
    // 1.81 vs 1.84 ms, cfg3 0.33 vs 0.46 ms); hxs_kernel keeps PCM, f64 and other layouts.
    static const int knobHxt = std::getenv("GAR_HXT") ? std::atoi(std::getenv("GAR_HXT")) : -1;
    int role[kHxtMaxComp] = {}, maxStride = 1, ncomp = 0;
    bool hxt = knobHxt != 0 && !small && !od.pcm && !od.f64 && !src.in_pcm &&
               ((fmt == 1 && vst == 2) || (fmt == 2 && (vst == 0 || vst == 1)));
    if (hxt) ncomp = hxtRoles(p.nw, p.NS, role, &maxStride);
    wide = wide && hxt && fmt == 2 && vst == 0;
    if (wide) fmt = 5;

    int G = 0, R = 0, Rt = 0, Wg = 0;
    auto pickG = [&]() {
        for (int pass = hxt && maxStride > 1 ? 0 : 1; pass < 2 && G == 0; ++pass) {  // hxt: G a multiple of the stride first
            for (int cand = small ? 1 : kHxsMaxG; cand >= 1; --cand) {
                int r, rt, wg;
                hxsRingFor(p, cand, r, rt, wg);
                if (cand > 1 && cand > Np) continue;
                if (knobG > 0 && cand > knobG && cand > 1) continue;
                if (fmt == 5 ? hxtLdsWide(rt) > 160 * 1024 : !hxsRingFits(p, cand, rt)) continue;
                if (hxt && cand * Qc > hxtMaxRowsF(fmt, ncomp + 6 <= kHxtWaves ? 6 : 4)) continue;
                // hxt: a producer runs at most (ring slots + 2) loads / groups ahead of the slowest one,
                // which the arrival slots must cover (gar_hxt.hpp progress counters)
                if (hxt && r / (cand * static_cast<int>(Qc)) + 3 > kHxtSlots) continue;
                if (pass == 0 && cand % maxStride != 0) continue;
                G = cand; R = r; Rt = rt; Wg = wg;
                break;
            }
        }
    };
    pickG();
    // a 32-channel ring holds half the rows: keep it only with groups of >= 2 periods and one compute
    // wave per row block (r06y / r06z: cfg3, NS = 10 on balanced roles at G = 2, lost 4-12 % -- its
    // chunks halve, traffic / algorithmic 1.06 -> 1.12), else 16-channel blocks
    if (fmt == 5 && (G < 2 || maxStride > 1)) {
        fmt = 2;
        G = 0;
        pickG();
    }
    if (G == 0 && hxt) {  // no group size fits hxt_kernel's limits: hxs_kernel's
        hxt = false;
        ncomp = 0;
        maxStride = 1;
        for (int& r : role) r = 0;
        pickG();
    }
    if (G == 0) return hipErrorNotSupported;

    HxsArgs x{};
    x.A = static_cast<const h8v*>(p.A);
    x.progs = p.progs;
    x.ea = p.ea;
    x.Pc = p.Pc; x.Qc = p.Qc; x.Kc = p.Kc; x.Kread = p.Kread; x.G = G; x.C = C;
    x.nprog = p.nw;
    x.ncols = static_cast<int>(ncols);
    x.nblocks = static_cast<int>(fmt == 5 ? (ncols + 31) / 32 : (ncols + 15) / 16);
    x.Np = static_cast<int>(Np);
    x.ngroups = static_cast<int>(cdiv(Np, G));
    x.R = R; x.Rt = Rt; x.mirror = std::max(0, Wg - G * static_cast<int>(Qc)); x.Wg = Wg;
    x.a_lo = a_lo; x.a_hi = a_hi;
    x.dbg = knobDbg;
    x.prof = profBuf();
    x.o_lo = od.o_lo; x.o_hi = od.o_hi;
    // raw input: element (t, c) at in + t*in_fs + c*in_cs for t in [fastLo, fastHi) (integer arithmetic:
    // the base may point outside the caller's buffer, only rows inside it are dereferenced)
    const bool rawOk = src.in && fmt != 0 && src.in_len > 0 && src.in_fs > 0 && src.in_cs >= 0 && rawSpan;
    x.in_esz = inEsz;
    x.in_pcm = src.in_pcm;
    x.in = reinterpret_cast<const char*>(reinterpret_cast<uintptr_t>(src.in) -
                                         static_cast<uintptr_t>(src.in_base * src.in_fs * inEsz));
    x.in_fs = src.in_fs;
    x.in_cs = src.in_cs;
    x.fastLo = rawOk ? src.in_base : 0;
    x.fastHi = rawOk ? std::min(src.in_base + src.in_len, src.valid_end) : 0;
    x.fmt = fmt;
    x.small = small ? 1 : 0;
    static const int knobSmallK = std::getenv("GAR_HXS_SMALLK") ? std::atoi(std::getenv("GAR_HXS_SMALLK")) : 1;
    x.bigSmall = knobSmallK ? 0 : 1;
    static const int knobNt = std::getenv("GAR_HXS_NT") ? std::atoi(std::getenv("GAR_HXS_NT")) : 0;
    static const int knobPair = std::getenv("GAR_HXS_PAIR") ? std::atoi(std::getenv("GAR_HXS_PAIR")) : 1;
    x.nt = knobNt;
    x.xcdPair = knobPair && fmt == 2 && (C / 16) % 2 == 0 && x.nblocks % 16 == 0 ? 1 : 0;
    static const int knobChunkMajor = std::getenv("GAR_HXT_CHUNKMAJOR") ? std::atoi(std::getenv("GAR_HXT_CHUNKMAJOR")) : 1;
    if (knobChunkMajor && fmt == 5 && x.nblocks % 8 == 0) x.xcdPair = 2;
    // output (o, c) at out + o*out_fs + c*out_cs bytes (o absolute)
    x.out_pcm = od.pcm;
    x.out_f64 = od.f64;
    x.out = outBase;
    x.out_fs = od.fs * esz;
    x.out_cs = od.cs * esz;
    x.vst = vst;
    x.ncomp = ncomp;
    for (int w = 0; w < kHxtMaxComp; ++w) x.role[w] = role[w];
    // progress-wait bound and the device status word; development knob GAR_HXT_FAULT=1 (read per
    // launch, so one test process can set it) makes the compute waves' load count unreachable
    // and the bound short: the launch must end with GAR_ERR_DEVICE, not with output
    x.err = od.err;
    x.pollMax = 1 << 24;
    x.faultNeed = 0;
    static const int knobCoop = std::getenv("GAR_HXT_COOP") ? std::atoi(std::getenv("GAR_HXT_COOP")) : 2;
    x.coop = std::max(0, std::min(2, knobCoop));
    if (hxt) {
        const char* f = std::getenv("GAR_HXT_FAULT");
        if (f && f[0] == '1') {
            x.pollMax = 1 << 12;
            x.faultNeed = 1 << 28;
        }
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
    if (trace)
        fprintf(stderr, "%s: small=%d o[%lld,%lld) C=%d G=%d Np=%lld ngroups=%d nblocks=%d R=%d Rt=%d Wg=%d fmt=%d vst=%d fast[%lld,%lld)\n",
                hxt ? "hxt" : "hxs", x.small, (long long)od.o_lo, (long long)od.o_hi, C, G, (long long)Np, x.ngroups, x.nblocks, R, Rt, Wg, x.fmt, x.vst,
                (long long)x.fastLo, (long long)x.fastHi);
    if (hc && hc->n > 0 && hc->dst) {  // history keep folded into this launch (no gather_kernel after it)
        x.hdst = static_cast<float*>(hc->dst);
        x.ht0 = hc->t0;
        x.hn = hc->n;
        hc->done = true;
    }
    // small float launches: hxq_kernel over (block, row-block group) workgroups, the largest group
    // whose launch still has a workgroup per CU (a stereo 4096-frame call: one row block per
    // workgroup, 40 workgroups; 256 channels: all ten, 448 workgroups -- measured 18 us per call
    // against 30 us with five).  Knobs: GAR_HXQ=0 (hxs_small_kernel), GAR_HXQ_NR (group size).
    static const int knobHxq = std::getenv("GAR_HXQ") ? std::atoi(std::getenv("GAR_HXQ")) : 1;
    static const int knobHxqNr = std::getenv("GAR_HXQ_NR") ? std::atoi(std::getenv("GAR_HXQ_NR")) : 0;
    {
        const uintptr_t hA = reinterpret_cast<uintptr_t>(src.hist);
        const int hAl = fmt == 1 ? 8 : (fmt == 2 ? 16 : 4), hLd = fmt == 1 ? 2 : (fmt == 2 ? 4 : 1);
        const bool histOk = !src.hist || src.hist_len <= 0 ||
                            ((hA % hAl) == 0 && src.hist_ld % hLd == 0 && src.hist_len * src.hist_ld * 4 < (int64_t(1) << 31));
        // any other f32 / f64 layout: per-column element loads, every offset from the block's first row < 2^31
        const int64_t spanRows = (16 / C + 2) * Np * Qc + Wg;
        const bool gen = fmt == 0 && !src.in_pcm && src.in_fs >= 0 && src.in_cs >= 0 &&
                         (spanRows * src.in_fs + static_cast<int64_t>(C) * src.in_cs) * inEsz < (int64_t(1) << 31);
        // history keep through buffer loads from row ht0: offsets < 2^31
        const bool hkOk = !hc || hc->n <= 0 || (hc->n * src.in_fs + static_cast<int64_t>(C) * src.in_cs) * inEsz < (int64_t(1) << 31);
        if (small && knobHxq && ((fmt == 1 || fmt == 2) ? rawSpan : gen) && histOk && hkOk && p.nw <= 12 && x.Np == 1) {
            int nr = 1;
            for (int cand = p.nw; cand >= 1; --cand)
                if (x.nblocks * static_cast<int64_t>(cdiv(p.nw, cand)) >= static_cast<int64_t>(ncu)) { nr = cand; break; }
            if (knobHxqNr > 0) nr = std::min(knobHxqNr, p.nw);
            // variant 1 (same-run A/B, profiles/r04j_hxq_variants.txt): the first barrier after the first load
            // batch issues, history keep by gathers -- workgroup life 6.0 us; buffer-load history keep 6.6 us
            static const int knobOpt = std::getenv("GAR_HXQ_OPT") ? std::atoi(std::getenv("GAR_HXQ_OPT")) : 1;
            x.qOpt = knobOpt;
            x.qRbs = nr;
            x.qGroups = static_cast<int>(cdiv(p.nw, nr));
            for (int w = 0; w < p.nw; ++w) { x.qU0[w] = p.hU0[w]; x.qRbw[w] = p.hRbw[w]; }
            if (fmt == 0) {  // raw rows of the input for the general path (per-lane checks)
                x.fastLo = src.in ? src.in_base : 0;
                x.fastHi = src.in ? std::min(src.in_base + src.in_len, src.valid_end) : 0;
            }
        }
    }
    // small launches stage only the window [0, Wg) of one period: no ring wrap, no mirror rows
    if (small && !x.bigSmall) {
        Rt = R = (Wg + 15) / 16 * 16;
        x.R = R; x.Rt = Rt; x.mirror = 0;
    }
    if (trace && x.qGroups > 0) fprintf(stderr, "hxq: qRbs=%d qGroups=%d workgroups=%lld\n", x.qRbs, x.qGroups, (long long)x.nblocks * x.qGroups);
    const size_t lds = fmt == 5 ? hxtLdsWide(Rt) : hxsLds(Rt);
    const int64_t blocks = x.nblocks;
    if (hxt) {
        const int64_t hblocks = blocks;
        switch (p.NS) {
#define GAR_HXT_NS(n) case n: return hxtFmt<n>(x, lds, hblocks, stream);
#if !GAR_HXS_QUICK
            GAR_HXT_NS(1) GAR_HXT_NS(2) GAR_HXT_NS(3) GAR_HXT_NS(4) GAR_HXT_NS(5) GAR_HXT_NS(6) GAR_HXT_NS(7)
            GAR_HXT_NS(8)
#endif
            GAR_HXT_NS(9) GAR_HXT_NS(10)
#undef GAR_HXT_NS
            default: return hipErrorNotSupported;
        }
    }
    switch (p.NS) {
#define GAR_HXS_NS(n) case n: return hxsVst<n>(x, lds, blocks, stream);
#if !GAR_HXS_QUICK
        GAR_HXS_NS(1) GAR_HXS_NS(2) GAR_HXS_NS(3) GAR_HXS_NS(4) GAR_HXS_NS(5) GAR_HXS_NS(6) GAR_HXS_NS(7)
        GAR_HXS_NS(8)
#endif
        GAR_HXS_NS(9) GAR_HXS_NS(10)
#undef GAR_HXS_NS
        default: return hipErrorNotSupported;
    }
}

}  // namespace gar
