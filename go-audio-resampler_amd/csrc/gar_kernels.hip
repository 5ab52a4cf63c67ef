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
#include <cstdio>
#include <cstdlib>
#include <mutex>
#include <set>
#include <type_traits>
#include <utility>

#include <map>

#include "gar_bg.hpp"
#include "gar_kernels.hpp"

namespace gar {

// Raises the kernel's dynamic-LDS limit to what the CU leaves next to its static LDS (160 KiB -
// static; asking for 160 KiB with static LDS present fails, and a launch above the default limit
// then fails with "invalid argument").  Returns the dynamic-LDS limit in force (bytes).
std::string& launchLimitMsg() {
    static thread_local std::string m;
    return m;
}
hipError_t ldsTooBig(const char* kernel, size_t need, size_t limit) {
    launchLimitMsg() = std::string(kernel) + " needs " + std::to_string(need) + " B of dynamic LDS; the device allows " +
                       std::to_string(limit) + " B for it";
    return hipErrorInvalidConfiguration;
}

size_t setMaxLdsOnce(const void* fn) {
    static std::mutex mu;
    static std::map<std::pair<int, const void*>, size_t> done;
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess) return 0;
    std::lock_guard<std::mutex> lk(mu);
    auto it = done.find({dev, fn});
    if (it != done.end()) return it->second;
    hipFuncAttributes fa{};
    size_t lim = 0;
    if (hipFuncGetAttributes(&fa, fn) == hipSuccess && fa.sharedSizeBytes <= 160 * 1024) {
        const size_t want = 160 * 1024 - fa.sharedSizeBytes;
        if (hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, static_cast<int>(want)) == hipSuccess) lim = want;
    }
    (void)hipGetLastError();
    if (lim == 0) lim = 64 * 1024 > fa.sharedSizeBytes ? 64 * 1024 - fa.sharedSizeBytes : 0;  // the default limit
    done[{dev, fn}] = lim;
    return lim;
}

hipError_t bgLaunchF32a(int NS, const BgDev& p, const SrcDesc& src, const OutDesc& od, const BgGrid& g, int threads,
                        size_t lds, int64_t blocks, hipStream_t st, bool globalB);
hipError_t bgLaunchF32b(int NS, const BgDev& p, const SrcDesc& src, const OutDesc& od, const BgGrid& g, int threads,
                        size_t lds, int64_t blocks, hipStream_t st, bool globalB);

// Small-launch geometry of a row-block-aligned f64 plan (stream chunks): returns the launch mode
// (0 not a small launch; 1 bg_rb_kernel, 2 bg_rt_kernel) with g, the dynamic LDS and
// the grid filled in.  The history keep hc is taken (hc->done) when the mode is not 0.
// development: GAR_BG_PROF=1 (with a -DGAR_BG_DEV=1 build of the f64 units) sums the small
// launches' phase stamps and prints them at exit
static unsigned long long* bgProfBuf() {
    static unsigned long long* p = nullptr;
    static bool init = false;
    if (!init) {
        init = true;
        if (std::getenv("GAR_BG_PROF") && hipMalloc(&p, kBgProfWords * sizeof(unsigned long long)) == hipSuccess) {
            (void)hipMemset(p, 0, kBgProfWords * sizeof(unsigned long long));
            (void)hipMemset(p + 18, 0xff, sizeof(unsigned long long));
            (void)hipMemset(p + 32 + 18, 0xff, sizeof(unsigned long long));
            std::atexit([] {
                static unsigned long long h[kBgProfWords] = {};
                if (hipDeviceSynchronize() != hipSuccess || hipMemcpy(h, p, sizeof(h), hipMemcpyDeviceToHost) != hipSuccess) return;
                const char* names[2] = {"bg_rt", "bg_rb"};
                for (int k = 0; k < 2; ++k) {
                    const unsigned long long* q = h + 32 * k;
                    if (!q[16]) continue;
                    for (int w = 0; w < 2; ++w) {
                        const double n = q[8 * w + 6] ? static_cast<double>(q[8 * w + 6]) : 1;
                        fprintf(stderr, "%s wave %d phases (cycles): %.0f %.0f %.0f %.0f %.0f %.0f (n %llu)\n", names[k], w, q[8 * w] / n,
                                q[8 * w + 1] / n, q[8 * w + 2] / n, q[8 * w + 3] / n, q[8 * w + 4] / n, q[8 * w + 5] / n, q[8 * w + 6]);
                    }
                    fprintf(stderr, "%s workgroups %llu: life %.2f us avg\n", names[k], q[16], q[17] / static_cast<double>(q[16]) / 100.0);
                }
            });
        }
    }
    return p;
}

static int bgSmallGrid(const BgDev& p, const OutDesc& od, int C, HistCopy* hc, int ncu, BgGrid& g, size_t& lds,
                       int64_t& blocks) {
    static const int knobDbg = std::getenv("GAR_BG_DBG") ? std::atoi(std::getenv("GAR_BG_DBG")) : 0;
    const int64_t a_lo = od.o_lo / p.Pc;
    const int64_t a_hi = (od.o_hi + p.Pc - 1) / p.Pc;
    const int64_t nmac = a_hi - a_lo;
    // small launch of a row-block-aligned f64 plan (stream chunks): one (column block, row block) per
    // workgroup, one macro period per column (bg_rb_kernel) -- same programs, same sums
    if (!(p.f64 && p.rbAligned && p.rbStart && p.hRbStart && p.nrb <= kBgRbKMaxRb && p.nprog <= kBgRbKMaxProg &&
          (nmac * C + 15) / 16 <= 2 * static_cast<int64_t>(ncu) && !(knobDbg & 8)))
        return 0;
    g.Pc = p.Pc; g.Qc = p.Qc; g.Kc = p.Kc; g.C = C;
    g.nprog = p.nprog;
    g.kch = p.kch;
    g.nwt = p.nw;
    g.ncg = p.ncg;
    g.nred = p.nred;
    g.nslots = p.nslots;
    g.a_lo = a_lo;
    g.rbMode = 1;
    for (int i = 0; i <= p.nrb; ++i) g.rbStart[i] = p.hRbStart[i];
    for (int i = 0; i < p.nprog; ++i) g.rbK0[i] = p.hRbK0[i];
    g.G = 1;
    g.W = p.Kc;
    g.Wl = p.Kread;
    g.Ws = g.Wl;
    g.nchunk = static_cast<int>(nmac);
    g.ncols = static_cast<int>(nmac * C);
    g.nblocks = (g.ncols + 15) / 16;
    g.dbg = knobDbg;
    g.vst = 0;
    g.parity = 0;
    g.hdst = nullptr;
    g.ht0 = g.hn = 0;
    g.prof = kBgDev ? bgProfBuf() : nullptr;
    if (hc && hc->n > 0 && hc->dst) {
        g.hdst = hc->dst;
        g.ht0 = hc->t0;
        g.hn = hc->n;
        hc->done = true;
    }
    // time-major (bg_rt_kernel, knob GAR_BG_RT=0: bg_rb_kernel): workgroups = row blocks x channels
    // x blocks of 16 consecutive macro periods, each window staged once in LDS
    // Default: time-major for plans of one or two row blocks (the integer decimator: each window is
    // staged once; 4800-frame cfg5 calls 26.8 -> 18.9 us), bg_rb_kernel otherwise (a plan of ten row
    // blocks would stage every window ten times: the cfg5 composite 21.8 -> 33.6 us).
    static const int knobRt = std::getenv("GAR_BG_RT") ? std::atoi(std::getenv("GAR_BG_RT")) : -1;
    const size_t rtLds = bgRtLds(p.Qc, p.Kread, p.maxPrb, 8);
    if ((knobRt == 1 || (knobRt < 0 && p.nrb <= 2)) && rtLds <= 64 * 1024) {
        g.rbMode = 2;
        const int64_t nkb = (nmac + 15) / 16;
        blocks = std::min<int64_t>(bgXcdSlots(nkb, static_cast<int64_t>(C) * p.nrb), 65528);  // XCD-grouped slots
        lds = rtLds;
        return 2;
    }
    blocks = std::min<int64_t>(bgXcdSlots(g.nblocks, p.nrb), 65528);  // XCD-grouped slots
    lds = 0;
    return 1;
}

static int numCUs() {
    int dev = 0, ncu = 256;
    if (hipGetDevice(&dev) == hipSuccess) (void)hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev);
    return ncu;
}

hipError_t launchBg(const BgDev& p, const SrcDesc& src, const OutDesc& od, int C, hipStream_t stream, HistCopy* hc) {
    if (od.o_hi <= od.o_lo) return hipSuccess;
    // f32 compute on the split-f16 kernel (every output of the launch, any input dtype)
    if (p.hx && !p.f64) return launchHx(*p.hx, src, od, C, stream, hc);
    const int sz = p.f64 ? 8 : 4;
    BgGrid g;
    const int ncu = numCUs();
    {
        size_t lds = 0;
        int64_t blocks = 0;
        if (bgSmallGrid(p, od, C, hc, ncu, g, lds, blocks))
            return bgLaunchF64(p.NS, p, src, od, g, 64 * p.maxPrb, lds, blocks, stream, false);
    }
    g.Pc = p.Pc; g.Qc = p.Qc; g.Kc = p.Kc; g.C = C;
    // Tuning knobs (development sweeps only; defaults are the tuned values).
    static const int knobG = std::getenv("GAR_BG_G") ? std::atoi(std::getenv("GAR_BG_G")) : 0;
    static const int knobWgPerCu = std::getenv("GAR_BG_WGPERCU") ? std::atoi(std::getenv("GAR_BG_WGPERCU")) : 0;
    static const int knobDbg = std::getenv("GAR_BG_DBG") ? std::atoi(std::getenv("GAR_BG_DBG")) : 0;
    static const bool knobNoVst = std::getenv("GAR_BG_NOVST") != nullptr;
    static const bool knobNoParity = std::getenv("GAR_BG_NOPARITY") != nullptr;
    g.rbMode = 0;
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
    const size_t kLds = 160 * 1024 - kBgStaticLds;  // bg_kernel's static LDS: the non-finite ranges
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
    int64_t blocks = std::min<int64_t>(g.nblocks, static_cast<int64_t>(ncu) * (knobWgPerCu > 0 ? knobWgPerCu : 2));
    g.hdst = nullptr;
    g.prof = nullptr;
    g.ht0 = g.hn = 0;
    if (hc && hc->n > 0 && hc->dst) {  // history keep folded into this launch (no gather_kernel after it)
        g.hdst = hc->dst;
        g.ht0 = hc->t0;
        g.hn = hc->n;
        hc->done = true;
    }
    static const bool trace = std::getenv("GAR_BG_TRACE") != nullptr;
    static int traced = 0;
    if (trace && traced < 64) {
        ++traced;
        fprintf(stderr, "bg: f64=%d Pc=%d Qc=%d Kc=%d Kread=%d NS=%d kch=%d nw=%d ncg=%d nprog=%d nred=%d nslots=%d G=%d nmac=%lld C=%d nblocks=%d blocks=%lld lds=%zu globalB=%d o[%lld,%lld)\n",
                p.f64, p.Pc, p.Qc, p.Kc, p.Kread, p.NS, g.kch, g.nwt, g.ncg, g.nprog, g.nred, g.nslots, g.G,
                (long long)nmac, C, g.nblocks, (long long)blocks, lds, globalB ? 1 : 0, (long long)od.o_lo, (long long)od.o_hi);
    }
    hipError_t e;
    if (p.f64) e = bgLaunchF64(p.NS, p, src, od, g, threads, lds, blocks, stream, globalB);
    else if (p.NS < 56) e = bgLaunchF32a(p.NS, p, src, od, g, threads, lds, blocks, stream, globalB);
    else e = bgLaunchF32b(p.NS, p, src, od, g, threads, lds, blocks, stream, globalB);
    if (e != hipSuccess || !p.nfList) return e;
    // the outputs of blocks that staged a non-finite sample (bg_nf_kernel: returns at once when none did)
    const BgArgs ka{p, src, od, g};
    const dim3 ng(static_cast<unsigned>(std::max(1, std::min(g.nblocks, 256)))), nb(256);
    if (p.f64) hipLaunchKernelGGL(bg_nf_kernel<double>, ng, nb, 0, stream, ka);
    else hipLaunchKernelGGL(bg_nf_kernel<float>, ng, nb, 0, stream, ka);
    return hipGetLastError();
}

// ---------------------------------------------------------------------------
// General polyphase stage (cubic sub-phase interpolation live).
// ---------------------------------------------------------------------------
// One thread per (output, group of CG consecutive channels) -- consecutive threads are consecutive
// channel groups of one output, then consecutive outputs -- accumulating the T taps of its output in
// the reference's order (polyphase_stage.go:257-293: coefficient a + x(b + x(c + x d)) of tap k
// times u[base + k], summed k = 0 .. T-1), the coefficient evaluated once for the CG channels.  The
// four coefficient banks are interleaved ([L][T][4]) so a tap's coefficients are one 16/32-B read;
// when they fit (L*T*16 B <= 144 KiB) every workgroup copies them into LDS once and walks the
// outputs grid-stride.  The window u[base .. base + T) of an output is addressed directly when it
// lies inside the input or the history buffer (the common case: one pointer, one row stride, CG
// channels as one vector load); windows across the history seam or the stream end are gathered
// branch-free (srcReadBF), so the unrolled taps issue their loads together.
constexpr int kPolyThreads = 1024;  // 4 waves per SIMD: the tap loop is load-latency bound
constexpr size_t kPolyLdsMax = 144 * 1024;

template <class TC, int CG>
struct PolyVec { typedef TC __attribute__((ext_vector_type(CG))) V; };
template <class TC>
struct PolyVec<TC, 1> { typedef TC V; };

template <class TC, int CG>
__device__ __forceinline__ TC pvGet(const typename PolyVec<TC, CG>::V& v, int j) {
    if constexpr (CG == 1) return v;
    else return v[j];
}

// WIN (with BANK_LDS): the workgroup's threads form a tile of consecutive (output, channel group)
// items; the tile's whole input window (rows [base(first output), base(last output) + T) x C) is
// staged into LDS once with coalesced branch-free gathers, and the tap loop reads it from there.
// Tap order of output m: k = r, r+1, .., T-1, 0, .., r-1 with r = (m - ph*T) mod 16 (mod T), so
// the bank rows [ph][k] that 16 consecutive outputs read in one step fall on 16 distinct 16-B LDS
// bank groups (slot (ph*T + k) mod 16 = (m + i) mod 16) instead of colliding on ph mod 16.  A
// function of the output's absolute index in the stage's output stream (PolyDev::m0 + the launch-
// relative index; r05: the launch-relative index made the order, and so the bits, depend on the
// chunking -- found by the ragged-call sweep): every launch geometry sums an output in the same order
// (chunk-invariant bits); the reference sums k = 0 .. T-1 (the f32 / f64 tolerances cover it).
__device__ __forceinline__ int polyRot(int64_t m, int ph, int T) {
    return static_cast<int>((static_cast<unsigned>(m) - static_cast<unsigned>(ph) * static_cast<unsigned>(T)) & 15u) % T;
}

template <class TC, bool BANK_LDS, int CG, bool WIN>
__global__ __launch_bounds__(kPolyThreads) void poly_kernel(PolyDev p, SrcDesc src, OutDesc od, int64_t nout, int C,
                                                            int winRows) {
    typedef typename std::conditional<sizeof(TC) == 8, f64x4, f32x4>::type V4;
    typedef typename PolyVec<TC, CG>::V VC;
    extern __shared__ __attribute__((aligned(16))) unsigned char psm[];
    const int T = p.T, L = p.L;
    const V4* bankG = static_cast<const V4*>(p.abcd);
    const V4* bank = bankG;
    if constexpr (BANK_LDS) {
        V4* lb = reinterpret_cast<V4*>(psm);
        for (int i = threadIdx.x; i < L * T; i += blockDim.x) lb[i] = bankG[i];
        __syncthreads();
        bank = lb;
    }
    const TC fscale = static_cast<TC>(1.0 / 65536.0);
    const bool same = srcSameType<TC>(src);
    const int ng = C / CG;  // launcher: CG divides C
    const int64_t total = nout * ng;
    TC* win = reinterpret_cast<TC*>(psm + (BANK_LDS ? static_cast<size_t>(L) * T * sizeof(V4) : 0));
    const int64_t ntile = (total + blockDim.x - 1) / blockDim.x;
    for (int64_t tile = blockIdx.x; tile < (WIN ? ntile : 0); tile += gridDim.x) {  // uniform per workgroup
        const int64_t i0 = tile * blockDim.x, i1 = min<int64_t>(total, i0 + blockDim.x);
        const int64_t mlo = i0 / ng, mhi = (i1 - 1) / ng;
        const int64_t blo = p.u_base + ((p.at0 + mlo * p.step) >> 16) / L;
        const int64_t bhi = p.u_base + ((p.at0 + mhi * p.step) >> 16) / L + T;  // exclusive
        const int nr = static_cast<int>(bhi - blo);                              // <= winRows (launcher bound)
        __syncthreads();  // previous tile's window consumed
        // interior tile (uniform): the window is nr consecutive whole rows of the input or of the
        // history, [t][C] contiguous -> one plain coalesced copy (the general gather's 64-bit source
        // selection per element was a third of the kernel's instructions, r06 ISA census)
        const bool inWin = same && src.in && src.in_cs == 1 && src.in_fs == C && blo >= src.in_base &&
                           bhi <= src.in_base + src.in_len && bhi <= src.valid_end && blo >= 0 && nr <= winRows;
        const bool hWin = !inWin && same && src.hist && src.hist_ld == C && blo >= src.hist_base &&
                          bhi <= src.hist_base + src.hist_len && bhi <= src.valid_end && blo >= 0 && nr <= winRows;
        if (inWin || hWin) {
            const TC* base = inWin ? static_cast<const TC*>(src.in) + (blo - src.in_base) * C
                                   : static_cast<const TC*>(src.hist) + (blo - src.hist_base) * C;
            for (int e = threadIdx.x; e < nr * C; e += blockDim.x) win[e] = base[e];
        } else {
            for (int e = threadIdx.x; e < nr * C; e += blockDim.x) {
                const int r = e / C, c = e - r * C;
                win[e] = same ? srcReadBF<TC>(src, blo + r, c, r < winRows, bankG) : srcRead<TC>(src, blo + r, c);
            }
        }
        __syncthreads();
        if (i0 + threadIdx.x >= i1) continue;
        // 32-bit per-thread index arithmetic relative to the tile's first output (its 64-bit
        // quantities are wave-uniform): output m = mlo + d, position at = atlo + d*step
        const int r0 = static_cast<int>(i0 - mlo * ng);  // item offset of the tile start within output mlo
        const unsigned li = static_cast<unsigned>(r0) + threadIdx.x;
        const unsigned d = li / static_cast<unsigned>(ng);
        const int c0 = static_cast<int>(li - d * static_cast<unsigned>(ng)) * CG;
        const int64_t m = mlo + d;
        const int64_t atlo = p.at0 + mlo * p.step;
        const int64_t ailo = atlo >> 16;
        const int64_t qlo = ailo / L;
        const int phlo = static_cast<int>(ailo - qlo * L);
        const int64_t at = atlo + static_cast<int64_t>(d) * p.step;
        const unsigned t = static_cast<unsigned>(phlo) + static_cast<unsigned>((at >> 16) - ailo);
        const unsigned dq = t / static_cast<unsigned>(L);
        const int ph = static_cast<int>(t - dq * static_cast<unsigned>(L));
        const int64_t q = qlo + dq;
        const TC x = static_cast<TC>(at & 0xFFFF) * fscale;
        const TC* wl = win + (p.u_base + q - blo) * C + c0;
        const V4* row = bank + static_cast<size_t>(ph) * T;
        TC acc[CG];
#pragma unroll
        for (int j = 0; j < CG; ++j) acc[j] = 0;
        // (one loop of T taps with a wrap test: split at the wrap, the two loops' trip counts differ
        // per lane and the wave runs the longest of each -- r06: 1.13 -> 1.58 ms)
        int k = polyRot(p.m0 + m, ph, T);
#pragma unroll 8
        for (int i = 0; i < T; ++i) {
            const V4 cf = row[k];
            const TC co = cf[0] + x * (cf[1] + x * (cf[2] + x * cf[3]));
            const VC v = *reinterpret_cast<const VC*>(wl + k * C);
#pragma unroll
            for (int j = 0; j < CG; ++j) acc[j] += pvGet<TC, CG>(v, j) * co;
            k = k + 1 == T ? 0 : k + 1;
        }
#pragma unroll
        for (int j = 0; j < CG; ++j) outWrite<TC>(od, od.o_lo + m, c0 + j, acc[j]);
    }
    for (int64_t idx = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x; idx < (WIN ? 0 : total);
         idx += static_cast<int64_t>(gridDim.x) * blockDim.x) {
        const int64_t m = idx / ng;
        const int c0 = static_cast<int>(idx - m * ng) * CG;
        const int64_t at = p.at0 + m * p.step;
        const int64_t ai = at >> 16;
        const int64_t q = ai / L;
        const int ph = static_cast<int>(ai - q * L);
        const TC x = static_cast<TC>(at & 0xFFFF) * fscale;
        const int64_t base = p.u_base + q;
        const V4* row = bank + static_cast<size_t>(ph) * T;
        // direct window: inside the input (compute dtype) or inside the history buffer
        const TC* wp = nullptr;
        int64_t ws = 0;
        if (same && src.in && base >= src.in_base && base + T <= src.in_base + src.in_len && base + T <= src.valid_end &&
            base >= 0) {
            wp = static_cast<const TC*>(src.in) + (base - src.in_base) * src.in_fs + static_cast<int64_t>(c0) * src.in_cs;
            ws = src.in_fs;
        } else if (src.hist && base >= src.hist_base && base + T <= src.hist_base + src.hist_len && base + T <= src.valid_end &&
                   base >= 0) {
            wp = static_cast<const TC*>(src.hist) + (base - src.hist_base) * src.hist_ld + c0;
            ws = src.hist_ld;
        }
        TC acc[CG];
#pragma unroll
        for (int j = 0; j < CG; ++j) acc[j] = 0;
        int k = polyRot(p.m0 + m, ph, T);
        if (wp) {
#pragma unroll 8
            for (int i = 0; i < T; ++i) {
                const V4 cf = row[k];
                const TC co = cf[0] + x * (cf[1] + x * (cf[2] + x * cf[3]));
                const VC v = *reinterpret_cast<const VC*>(wp + k * ws);
#pragma unroll
                for (int j = 0; j < CG; ++j) acc[j] += pvGet<TC, CG>(v, j) * co;
                k = k + 1 == T ? 0 : k + 1;
            }
        } else {
#pragma unroll 4
            for (int i = 0; i < T; ++i) {
                const V4 cf = row[k];
                const TC co = cf[0] + x * (cf[1] + x * (cf[2] + x * cf[3]));
#pragma unroll
                for (int j = 0; j < CG; ++j)
                    acc[j] += (same ? srcReadBF<TC>(src, base + k, c0 + j, true, bankG) : srcRead<TC>(src, base + k, c0 + j)) * co;
                k = k + 1 == T ? 0 : k + 1;
            }
        }
#pragma unroll
        for (int j = 0; j < CG; ++j) outWrite<TC>(od, od.o_lo + m, c0 + j, acc[j]);
    }
}

template <class TC, bool BANK_LDS, bool WIN>
static void polyGo(int CG, dim3 gd, dim3 bd, size_t lds, hipStream_t st, const PolyDev& p, const SrcDesc& src,
                   const OutDesc& od, int64_t nout, int C, int winRows) {
    if (BANK_LDS) {
        setMaxLdsOnce(reinterpret_cast<const void*>(&poly_kernel<TC, BANK_LDS, 1, WIN>));
        setMaxLdsOnce(reinterpret_cast<const void*>(&poly_kernel<TC, BANK_LDS, 2, WIN>));
        setMaxLdsOnce(reinterpret_cast<const void*>(&poly_kernel<TC, BANK_LDS, 4, WIN>));
    }
    if (CG == 4) hipLaunchKernelGGL((poly_kernel<TC, BANK_LDS, 4, WIN>), gd, bd, lds, st, p, src, od, nout, C, winRows);
    else if (CG == 2) hipLaunchKernelGGL((poly_kernel<TC, BANK_LDS, 2, WIN>), gd, bd, lds, st, p, src, od, nout, C, winRows);
    else hipLaunchKernelGGL((poly_kernel<TC, BANK_LDS, 1, WIN>), gd, bd, lds, st, p, src, od, nout, C, winRows);
}

hipError_t launchPoly(const PolyDev& p, const SrcDesc& src, const OutDesc& od, int64_t nout, int C,
                      hipStream_t stream) {
    if (nout <= 0) return hipSuccess;
    const size_t es = p.f64 ? 8 : 4;
    const size_t bankB = static_cast<size_t>(p.L) * p.T * 4 * es;
    // channel group: CG consecutive channels share a coefficient evaluation and one vector load per
    // tap, when every direct window has contiguous, CG-aligned channels (stride 1, row strides and
    // bases multiples of CG elements)
    auto alignedFor = [&](int cg) {
        if (C % cg != 0) return false;
        const bool inOk = !src.in || (src.in_cs == 1 && src.in_fs % cg == 0 &&
                                      reinterpret_cast<uintptr_t>(src.in) % (cg * es) == 0);
        const bool hOk = !src.hist || (src.hist_ld % cg == 0 && reinterpret_cast<uintptr_t>(src.hist) % (cg * es) == 0);
        return inOk && hOk;
    };
    const int CG = alignedFor(4) ? 4 : (alignedFor(2) ? 2 : 1);
    const int64_t total = nout * (C / CG);
    int dev = 0, ncu = 256;
    if (hipGetDevice(&dev) == hipSuccess) (void)hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev);
    // LDS bank: one resident workgroup per CU walks the outputs grid-stride (the bank is copied once
    // per workgroup); without it, enough workgroups to cover the launch.
    const bool lbank = bankB <= kPolyLdsMax && total >= static_cast<int64_t>(ncu) * kPolyThreads;
    int64_t blocks = (total + kPolyThreads - 1) / kPolyThreads;
    if (lbank) blocks = std::min<int64_t>(blocks, ncu);
    blocks = std::min<int64_t>(blocks, 65536);
    const dim3 gd(static_cast<unsigned>(blocks)), bd(kPolyThreads);
    // window rows of one tile of kPolyThreads items: (outputs - 1) * step / 2^16 / L + T + 2 (rounding)
    const int64_t mt = (kPolyThreads + (C / CG) - 1) / (C / CG) + 1;
    const int winRows = static_cast<int>(((mt - 1) * p.step >> 16) / p.L + p.T + 2);
    const size_t winB = static_cast<size_t>(winRows) * C * es;
    const bool win = lbank && bankB + winB <= 160 * 1024;
    const size_t lds = lbank ? bankB + (win ? winB : 0) : 0;
    if (p.f64) {
        if (win) polyGo<double, true, true>(CG, gd, bd, lds, stream, p, src, od, nout, C, winRows);
        else if (lbank) polyGo<double, true, false>(CG, gd, bd, lds, stream, p, src, od, nout, C, winRows);
        else polyGo<double, false, false>(CG, gd, bd, 0, stream, p, src, od, nout, C, winRows);
    } else {
        if (win) polyGo<float, true, true>(CG, gd, bd, lds, stream, p, src, od, nout, C, winRows);
        else if (lbank) polyGo<float, true, false>(CG, gd, bd, lds, stream, p, src, od, nout, C, winRows);
        else polyGo<float, false, false>(CG, gd, bd, 0, stream, p, src, od, nout, C, winRows);
    }
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
// The cubic output of phase ph between h2 (s[0]) and h1 (s[1]) (cubic.go:78-89; contraction off).
__device__ __forceinline__ double cubicAt(double h3, double h2, double h1, double h0, double ph) {
#pragma clang fp contract(off)
    const double b = 0.5 * (h1 + h3) - h2;
    const double a = (1.0 / 6.0) * (h0 - h1 + h3 - h2 - 4 * b);
    const double cc = h1 - h2 - a - b;
    return ((a * ph + b) * ph + cc) * ph + h2;
}

// SHORT: segments of kCubicSegInputsShort inputs (short calls) -- the segment's inputs and the three
// before it are loaded up front (one memory round trip) and the walk runs from registers.
template <class TC, bool SHORT>
__global__ __launch_bounds__(256) void cubic_kernel(const CubicSeg* segs, int64_t nseg, int64_t x_end, double step,
                                                    SrcDesc src, OutDesc od, int C, int segLen) {
#pragma clang fp contract(off)
    const int64_t total = nseg * C;
    for (int64_t idx = blockIdx.x * static_cast<int64_t>(blockDim.x) + threadIdx.x; idx < total;
         idx += static_cast<int64_t>(gridDim.x) * blockDim.x) {
        const int64_t sgi = idx / C;
        const int c = static_cast<int>(idx - sgi * C);
        const CubicSeg sg = segs[sgi];
        const int64_t i1 = min(sg.i + segLen, x_end);
        double ph = sg.phase;
        int64_t o = sg.o;
        if constexpr (SHORT) {
            constexpr int L = kCubicSegInputsShort;
            double v[L + 3];
#pragma unroll
            for (int k = 0; k < L + 3; ++k)
                v[k] = (sg.i - 3 + k < i1) ? static_cast<double>(srcRead<TC>(src, sg.i - 3 + k, c)) : 0.0;
#pragma unroll
            for (int k = 0; k < L; ++k) {
                if (sg.i + k >= i1) break;
                // history[3..1] = v[k], v[k+1], v[k+2]; the new input h0 = v[k+3]
                while (ph < 1.0) {
                    outWrite<TC>(od, o, c, static_cast<TC>(cubicAt(v[k], v[k + 1], v[k + 2], v[k + 3], ph)));
                    ++o;
                    ph += step;
                }
                ph -= 1.0;
            }
        } else {
            // history[3..1] = inputs i-3 .. i-1 (zeros before the stream start)
            double h3 = static_cast<double>(srcRead<TC>(src, sg.i - 3, c));
            double h2 = static_cast<double>(srcRead<TC>(src, sg.i - 2, c));
            double h1 = static_cast<double>(srcRead<TC>(src, sg.i - 1, c));
            for (int64_t i = sg.i; i < i1; ++i) {
                const double h0 = static_cast<double>(srcRead<TC>(src, i, c));
                while (ph < 1.0) {
                    // s[-1], s[0], s[1], s[2] = history[3], [2], [1], [0] (cubic.go:78-89)
                    outWrite<TC>(od, o, c, static_cast<TC>(cubicAt(h3, h2, h1, h0, ph)));
                    ++o;
                    ph += step;
                }
                ph -= 1.0;
                h3 = h2; h2 = h1; h1 = h0;
            }
        }
    }
}

hipError_t launchCubic(int f64, const CubicSeg* segs, int64_t nseg, int64_t x_end, double step, const SrcDesc& src,
                       const OutDesc& od, int C, hipStream_t stream, int segLen) {
    if (nseg <= 0) return hipSuccess;
    const int64_t total = nseg * C;
    int64_t blocks = (total + 255) / 256;
    if (blocks > 65536) blocks = 65536;
    const bool sh = segLen <= kCubicSegInputsShort;
    const dim3 gd(static_cast<unsigned>(blocks)), bd(256);
    if (f64) {
        if (sh) hipLaunchKernelGGL((cubic_kernel<double, true>), gd, bd, 0, stream, segs, nseg, x_end, step, src, od, C, segLen);
        else hipLaunchKernelGGL((cubic_kernel<double, false>), gd, bd, 0, stream, segs, nseg, x_end, step, src, od, C, segLen);
    } else {
        if (sh) hipLaunchKernelGGL((cubic_kernel<float, true>), gd, bd, 0, stream, segs, nseg, x_end, step, src, od, C, segLen);
        else hipLaunchKernelGGL((cubic_kernel<float, false>), gd, bd, 0, stream, segs, nseg, x_end, step, src, od, C, segLen);
    }
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
