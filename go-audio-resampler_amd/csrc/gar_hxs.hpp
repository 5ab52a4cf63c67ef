// gar_hxs.hpp -- streaming split-f16 FIR kernel (row-block plans, gfx950).
//
// Same arithmetic as hx_kernel (gar_hx.hpp: constant split scale, three f16
// MFMA products per 32-deep step, lo products in their own accumulator), so
// the two kernels produce identical bits; the difference is the data flow:
//
//  * Wave specialisation.  Waves [0, nprog) are compute waves: each owns one
//    row block (A in registers for the whole kernel), reads B fragments from
//    LDS with ds_read_b64_tr_b16, runs the MFMAs and stores its outputs.  They
//    issue no global loads, so no s_waitcnt on vector memory ever stalls an
//    MFMA stream (on gfx950 stores and loads share vmcnt).  The last
//    kHxsLoaders waves are loader waves: they load the input rows into VGPRs
//    kHxsD groups ahead (a fixed buffer-load pattern the compiler's vmcnt
//    tracking pipelines), convert them to the f16 hi/lo split (or from integer
//    PCM first), detect loud elements and write the LDS ring.
//  * Long columns.  A column is (channel, chunk of Np consecutive macro
//    periods); a workgroup owns 16 columns and walks them group by group (G
//    periods per group, one barrier per group).  Each column's window lives
//    in an LDS ring of R = n*G*Qc rows (+ a mirror of the first Kread - Qc
//    rows, so every group's window is contiguous), so each input row is staged
//    once per column instead of once per G-period window (round-1 kernel:
//    W/(G*Qc) = 1.34x; here (Np*Qc + Kread - Qc)/(Np*Qc) ~ 1.02x).
//  * Loud elements (!(|x| < kHxLoud): |x| >= 16 - 2^-8, Inf, NaN) are staged as zero and their
//    column-relative row range recorded; after the block, every output whose
//    window holds one is recomputed exactly (hxExactT: f64, two stages when
//    non-finite) by the same workgroup.
#pragma once
#include <climits>

#include "gar_hx.hpp"

namespace gar {

#ifndef GAR_HXS_L
#define GAR_HXS_L 6
#endif
constexpr int kHxsLoaders = GAR_HXS_L;                  // loader waves per workgroup
constexpr int kHxsWaves = kHxRbMaxWaves + kHxsLoaders;  // __launch_bounds__ (4 waves per SIMD, 128 VGPRs)
#ifndef GAR_HXS_D
#define GAR_HXS_D 2
#endif
constexpr int kHxsD = GAR_HXS_D;                        // loads in flight per loader wave (register staging)
#ifndef GAR_HXS_NP
#define GAR_HXS_NP 12
#endif
constexpr int kHxsNP = GAR_HXS_NP;                      // 64-row pieces per load (G*Qc <= 768: cfg2 G = 5)
constexpr int kHxsMaxG = 6;                             // periods per group (launcher: largest that fits)
constexpr int kHxsItems = (4 * kHxsNP + kHxsLoaders - 1) / kHxsLoaders;  // (quad, piece) items per loader per load
// Development instrumentation (GAR_HXS_DBG attribution modes, GAR_HXS_PROF phase cycles): compiled
// in only with -DGAR_HXS_DEV=1 (tools/hxs_variant.sh); the production kernel carries none of it.
#ifndef GAR_HXS_DEV
#define GAR_HXS_DEV 0
#endif
constexpr bool kHxsDev = GAR_HXS_DEV != 0;
#ifndef GAR_HXS_QUICK
#define GAR_HXS_QUICK 0
#endif
#ifndef GAR_HXS_PRIO
#define GAR_HXS_PRIO 0
#endif
#ifndef GAR_HXS_PF2
#define GAR_HXS_PF2 0  // B fragments two steps ahead (A/B builds)
#endif

struct HxsArgs {
    const h8v* A;          // [nprog][NS][2][64] f16x8
    const int* progs;      // [nprog][kBgProgInts]
    int ea, Pc, Qc, Kc, Kread, G, C, nprog;
    int ncols, nblocks, Np, ngroups;
    int R, Rt, mirror;     // ring rows (n*G*Qc), rows incl. mirror, mirrored ring rows [0, mirror)
    int Wg;                // rows one group reads: (G-1)*Qc + Kread
    unsigned long long* prof;  // development: per-phase cycle sums (GAR_HXS_PROF), null in production
    int dbg;               // development attribution (GAR_HXS_DBG, wrong output): 1 no steady DMAs, 2 no stores,
                           // 4 no MFMA, 16 no steady conversion
    int small;             // one period per column, window staged in one pass (hxsSmallStage)
    int bigSmall;          // development (GAR_HXS_SMALLK=0): small launches on hxs_kernel instead of hxs_small_kernel
    int vst, fmt;          // epilogue layout (template VST), load layout 0 gathered / 1 STEREO / 2 ROW16
    int xcdPair;           // ROW16 blocks 2m, 2m+1 share every 128-B input/output line: run them on one XCD
    int nt;                // development: non-temporal output stores (GAR_HXS_NT)
    int64_t a_lo, a_hi;    // absolute macro periods of the launch
    int64_t o_lo, o_hi;    // outputs written
    const char* in;        // input element (t, c) at byte in + (t*in_fs + c*in_cs)*in_esz, t absolute, raw loads for t in [fastLo, fastHi)
    int64_t in_fs, in_cs, fastLo, fastHi;
    int in_esz, in_pcm;    // bytes per input element; PCM bits (0: float input)
    int out_pcm;           // PCM output bits (0: float output; stores go through the checked path)
    float* hdst;           // folded history keep (HistCopy): hdst[(t - ht0) * C + c] = src(t, c), t < ht0 + hn
    int64_t ht0, hn;
    char* out;             // output (o, c) at out + o*out_fs + c*out_cs (bytes), o absolute
    int64_t out_fs, out_cs;
    int out_f64;
    // cold fields: edge gathers and the exact fallback (hxExactT)
    SrcDesc src;
    OutDesc od;
    const double* rows;
    const int* rowOff;
    const int* rowLen;
    int rowMax;
    int twoStage;
    const int* rowPh;
    const int* rowPar;
    const double* polyA;
    const double* dftC;
    int T1, T2;
    // hxt_kernel (gar_hxt.hpp): compute wave w runs row block role[w] & 0xff on the periods p with
    // p % stride == phase (phase = (role[w] >> 8) & 0xff, stride = role[w] >> 16)
    int ncomp;
    int role[12];
    int* err;               // the handle's device status word (host-mapped), written when a progress wait expires
    int pollMax;            // progress-wait bound in polls (2^24; development knob GAR_HXT_FAULT: 2^12)
    int faultNeed;          // development (GAR_HXT_FAULT=1): added to the compute waves' load count, unreachable
    int coop;               // hxt_kernel: compute waves stage each block's first window (GAR_HXT_COOP=0: loaders)
    // hxq_kernel (small f32 STEREO / ROW16 launches): workgroup = (block, qRbs row blocks), qGroups per block
    int qRbs, qGroups;
    int qU0[12], qRbw[12];  // first window row / row block of each row-block program (HxDev::hU0)
    int qOpt;               // hxq_kernel variants (GAR_HXQ_OPT): 1 barrier after the first load batch issues, 2 buffer-load history keep
};
typedef const __attribute__((address_space(4))) HxsArgs* HxsArgsP;

// Workgroup barrier for LDS hand-offs only: LDS operations drained
// (lgkmcnt(0)), no vector-memory wait.  __syncthreads() is a release/acquire
// fence and waits vmcnt(0): the loader waves' prefetch loads and the compute
// waves' output stores would both drain at every group.
__device__ __forceinline__ void hxsBarrier() {
    __atomic_signal_fence(__ATOMIC_SEQ_CST);
    __builtin_amdgcn_s_waitcnt(0xC07F);  // vmcnt max, expcnt max, lgkmcnt(0)
    __builtin_amdgcn_s_barrier();
    __atomic_signal_fence(__ATOMIC_SEQ_CST);
}

__device__ __forceinline__ HxsArgsP hxsCold() {
    uint64_t v = reinterpret_cast<uint64_t>(__builtin_amdgcn_kernarg_segment_ptr());
    asm volatile("" : "+s"(v));
    return reinterpret_cast<HxsArgsP>(v);
}

// Logical block of launch slot i.  Workgroups are dispatched round-robin over the 8 XCDs (slot
// i on XCD i % 8); with xcdPair, blocks 2m and 2m+1 -- the two halves of every 128-B line of
// a ROW16 layout (16 channels x 4 B = 64 B per row) -- run as slots i and i + 8 on the same
// XCD, so the second reader / writer of each line meets it in that XCD's L2.
__device__ __forceinline__ int hxsBlock(const HxsArgs& x, int i) {
    if (!x.xcdPair) return i;
    const int s = i >> 3, xc = i & 7;
    return ((s >> 1) * 8 + xc) * 2 + (s & 1);
}

// Exact value of output (a, r) of channel c (see hxExact in gar_hx.hpp).
__device__ __forceinline__ double hxsExact(HxsArgsP x, int64_t a, int r, int c) {
    const SrcDesc src = kload(&x->src);
    const int64_t t = a * x->Qc + x->rowOff[r];
    const int len = x->rowLen[r];
    const double* row = x->rows + static_cast<size_t>(r) * x->rowMax;
    double s = 0.0, z = 0.0;
    for (int k = 0; k < len; ++k) {
        const double v = static_cast<double>(srcRead<float>(src, t + k, c));
        s += row[k] * v;
        z += v * 0.0;
    }
    if (z == z || !x->twoStage) return s;
    const int ph = x->rowPh[r], par = x->rowPar[r], T1 = x->T1, T2 = x->T2;
    const double* pa = x->polyA + static_cast<size_t>(ph) * T2;
    double y = 0.0;
    for (int k2 = 0; k2 < T2; ++k2) {
        const int q = par + k2;
        const double* cq = x->dftC + static_cast<size_t>(q & 1) * T1;
        double u = 0.0;
        for (int k1 = 0; k1 < T1; ++k1) u += cq[k1] * static_cast<double>(srcRead<float>(src, t + (q >> 1) + k1, c));
        y += pa[k2] * u;
    }
    return y;
}

// After a block: recompute every output whose window intersects a column's loud
// row range and really holds a loud element (all threads; out of line).
__device__ __forceinline__ void hxsFixup(HxsArgsP xp, int b, const int* loudLo, const int* loudHi) {
    const SrcDesc src = kload(&xp->src);
    const OutDesc od = kload(&xp->od);
    const int Pc = xp->Pc, Qc = xp->Qc, Np = xp->Np, C = xp->C, ncols = xp->ncols;
    const int64_t a_lo = xp->a_lo, a_hi = xp->a_hi;
    for (int j = 0; j < 16; ++j) {
        const int lo = loudLo[j], hi = loudHi[j];
        const int col = b * 16 + j;
        if (hi < 0 || col >= ncols) continue;
        const int k = col / C, c = col - k * C;
        const int p0 = max(0, (lo - xp->Kread) / Qc), p1 = min(Np - 1, hi / Qc);
        const int n = (p1 - p0 + 1) * Pc;
        for (int idx = threadIdx.x; idx < n; idx += blockDim.x) {
            const int p = p0 + idx / Pc, r = idx - (idx / Pc) * Pc;
            const int64_t a = a_lo + static_cast<int64_t>(k) * Np + p;
            if (a >= a_hi) continue;
            const int64_t o = a * Pc + r;
            if (o < od.o_lo || o >= od.o_hi) continue;
            const int w0 = p * Qc + xp->rowOff[r], w1 = w0 + xp->rowLen[r];
            if (w1 <= lo || w0 > hi) continue;
            const int64_t t0 = a * Qc + xp->rowOff[r];
            bool loud = false;
            for (int kk = 0; kk < w1 - w0 && !loud; ++kk) loud = hxLoud(srcRead<float>(src, t0 + kk, c));
            if (loud) outWrite<float>(od, o, c, static_cast<float>(hxsExact(xp, a, r, c)));
        }
    }
}

// ---- staging --------------------------------------------------------------------
// A load (rows [T0, T0 + nrow) of every column of the block) travels:
//   global --buffer loads (loader waves, kHxsD loads ahead)--> VGPRs --f16 hi/lo split--> ring.
// A load is 4 quads x kHxsNP pieces of 64 rows; loader wave l owns the (quad, piece) items
// l, l + kHxsLoaders, ... (item = 4 * piece + quad), lane = row of the piece.  Layouts:
//  * STEREO (fmt 1, C == 2, frames interleaved): quad q = chunks 2q, 2q+1 (two channels each),
//    one buffer_load_dwordx2 per chunk (64 lanes = 512 B contiguous);
//  * ROW16 (fmt 2, C % 16 == 0, 16-B aligned rows): quad q = channels 4q..4q+3 of the block's
//    chunk, one buffer_load_dwordx4;
//  * every other layout, f64 input and the edges (rows before the input: history seam, stream
//    start; partial blocks): gathered at conversion time.
// Rows past the caller's input read zeros through the buffer records.
struct HxsStage {
    int T0, nrow;   // column-relative first row and row count
    bool fast;      // buffer loads: every column live, no row before the raw f32 input
};

// Buffer resource (raw, stride 0) over the raw input from absolute row `row0`
// of channel offset `cofs` (elements): records end at row fastHi, so loads past
// the caller's input (the tail of the last chunk) read zeros.
typedef unsigned u32x4v __attribute__((ext_vector_type(4)));
template <class XP>
__device__ __forceinline__ u32x4v hxsRsrc(XP x, int64_t row0, int64_t cofs, int elemBytes) {
    const uint64_t base = reinterpret_cast<uint64_t>(x->in + (row0 * x->in_fs + cofs) * x->in_esz);
    const int64_t nb = x->fastHi > row0 ? (x->fastHi - row0 - 1) * x->in_fs * x->in_esz + elemBytes : 0;
    const unsigned nrec = static_cast<unsigned>(nb < 0x7fffffff ? nb : 0x7fffffff);
    u32x4v r;
    r.x = __builtin_amdgcn_readfirstlane(static_cast<unsigned>(base));
    r.y = __builtin_amdgcn_readfirstlane(static_cast<unsigned>(base >> 32) & 0xffffu);
    r.z = __builtin_amdgcn_readfirstlane(nrec);
    r.w = 0x00020000u;
    return r;
}

// The same resource as a buffer-resource value (compiler-tracked raw_buffer_load builtins).
template <class XP>
__device__ __forceinline__ __amdgpu_buffer_rsrc_t hxsRsrcT(XP x, int64_t row0, int64_t cofs, int elemBytes) {
    const u32x4v r = hxsRsrc(x, row0, cofs, elemBytes);
    const uint64_t base = static_cast<uint64_t>(r.x) | (static_cast<uint64_t>(r.y) << 32);
    return __builtin_amdgcn_make_buffer_rsrc(reinterpret_cast<void*>(base), 0, static_cast<int>(r.z), 0x00020000);
}

// Element (t, c) of the stream for edge stages: history | input (f32/f64) |
// zero.  Branch-free address selection (a dummy readable address for zeros)
// so a piece's gathers issue together instead of one dependent load each.
__device__ __forceinline__ float hxsGather(const SrcDesc& s, int64_t t, int c, const void* dummy) {
    const int64_t h = t - s.hist_base, i = t - s.in_base;
    const bool valid = t >= 0 && t < s.valid_end;
    const bool inH = valid && s.hist && h >= 0 && h < s.hist_len;
    const bool inI = valid && !inH && s.in && i >= 0 && i < s.in_len;
    const float* hp = static_cast<const float*>(s.hist) + (inH ? h * s.hist_ld + c : 0);
    if (s.in_pcm) {  // integer PCM input (main.go:444-472 scaling)
        const int64_t e = inI ? i * s.in_fs + static_cast<int64_t>(c) * s.in_cs : 0;
        const float vh = *(inH ? hp : static_cast<const float*>(dummy));
        const float vi = inI ? static_cast<float>(pcmRead(s.in, e, s.in_pcm)) : 0.f;
        return inH ? vh : vi;
    }
    if (s.in_f64) {
        const double* ip = static_cast<const double*>(s.in) + (inI ? i * s.in_fs + static_cast<int64_t>(c) * s.in_cs : 0);
        const float vh = *(inH ? hp : static_cast<const float*>(dummy));
        const double vi = *(inI ? ip : static_cast<const double*>(dummy));
        return inH ? vh : (inI ? static_cast<float>(vi) : 0.f);
    }
    const float* ip = static_cast<const float*>(s.in) + (inI ? i * s.in_fs + static_cast<int64_t>(c) * s.in_cs : 0);
    const float v = *(inH ? hp : (inI ? ip : static_cast<const float*>(dummy)));
    return (inH || inI) ? v : 0.f;
}

template <class XP>
__device__ __forceinline__ int64_t hxsChunkRow(XP x, int k, int T0) {
    return (x->a_lo + static_cast<int64_t>(k) * x->Np) * x->Qc + T0;
}

// Stage k of a block: k = 0 rows [0, Wg) (in parts of at most G*Qc), k >= 1
// rows [Wg + (k-1)*G*Qc, Wg + k*G*Qc).
template <class XP>
__device__ __forceinline__ HxsStage hxsStage(XP x, int b, int T0, int nrow) {
    HxsStage s;
    s.T0 = T0;
    s.nrow = nrow;
    const int c0 = b * 16, c1 = c0 + 15;
    const int64_t tlo = (x->a_lo + static_cast<int64_t>(c0 / x->C) * x->Np) * x->Qc + T0;
    s.fast = x->fmt >= 1 && x->fmt <= 4 && c1 < x->ncols && tlo >= x->fastLo && x->fastHi > x->fastLo;
    return s;
}
// Load j of a block: j < P = ceil(Wg / GQ) the parts of stage 0 (rows [j*GQ, ...) up to Wg),
// then stage j - P + 1 (rows [Wg + (j-P)*GQ, + GQ)).
template <class XP>
__device__ __forceinline__ HxsStage hxsLoad(XP x, int b, int j, int P) {
    const int GQ = x->G * x->Qc;
    if (j < P) return hxsStage(x, b, j * GQ, min(GQ, x->Wg - j * GQ));
    return hxsStage(x, b, x->Wg + (j - P) * GQ, GQ);
}

// One item (row `row` of the stage, quad q) -> ring rows (hi/lo split, mirror, loud marking).
template <class XP>
__device__ __forceinline__ void hxsPutItem(XP x, const HxsStage& st, int p0, int q, int row, f32x4 e,
                                           char* ring, uint32_t QS, int* loudLo, int* loudHi, int* flag) {
    const int t = st.T0 + row;  // column-relative row
    int p = p0 + row;           // ring row (nrow <= R)
    if (p >= x->R) p -= x->R;
    const bool l0 = hxLoud(e[0]), l1 = hxLoud(e[1]), l2 = hxLoud(e[2]), l3 = hxLoud(e[3]);
    if (__builtin_expect(l0 | l1 | l2 | l3, 0)) {
        if (l0) { atomicMin(loudLo + 4 * q, t); atomicMax(loudHi + 4 * q, t); e[0] = 0.f; }
        if (l1) { atomicMin(loudLo + 4 * q + 1, t); atomicMax(loudHi + 4 * q + 1, t); e[1] = 0.f; }
        if (l2) { atomicMin(loudLo + 4 * q + 2, t); atomicMax(loudHi + 4 * q + 2, t); e[2] = 0.f; }
        if (l3) { atomicMin(loudLo + 4 * q + 3, t); atomicMax(loudHi + 4 * q + 3, t); e[3] = 0.f; }
        *flag = 1;
    }
    uint2 hv, lv;
    hxSplit2(e[0], e[1], hv.x, lv.x);
    hxSplit2(e[2], e[3], hv.y, lv.y);
    char* qb = ring + q * QS;
    *reinterpret_cast<uint2*>(qb + 8 * p) = hv;
    *reinterpret_cast<uint2*>(qb + 8 * x->Rt + 8 * p) = lv;
    if (p < x->mirror) {
        p += x->R;
        *reinterpret_cast<uint2*>(qb + 8 * p) = hv;
        *reinterpret_cast<uint2*>(qb + 8 * x->Rt + 8 * p) = lv;
    }
}

// Small launches (x.small: one macro period per column, one group): every wave gathers
// its share of the block's whole window [0, Wg) straight into the ring in one pass --
// one memory round trip instead of the pipeline's chain of DMA stages.
template <class XP>
__device__ __forceinline__ void hxsSmallStage(XP x, int b, int tid, int nth, char* ring, uint32_t QS,
                                              int* loudLo, int* loudHi, int* flag) {
    const HxsArgsP xc = hxsCold();
    const SrcDesc src = kload(&xc->src);
    HxsStage st;
    st.T0 = 0;
    st.nrow = x->Wg;
    st.fast = false;
    // batches of kB items per thread: every gather of a batch issues before the first conversion,
    // so the window costs one memory round trip per batch, not one per item
    constexpr int kB = 4;
    const int nit = 4 * x->Wg;
    for (int i0 = tid; i0 < nit; i0 += kB * nth) {
        f32x4 e[kB];
#pragma unroll
        for (int u = 0; u < kB; ++u) {
            const int i = i0 + u * nth;
            const int q = i & 3, row = i >> 2;
#pragma unroll
            for (int n = 0; n < 4; ++n) {
                const int col = b * 16 + 4 * q + n;
                const int k = col / x->C, c = col - k * x->C;
                e[u][n] = (i < nit && col < x->ncols) ? hxsGather(src, hxsChunkRow(x, k, row), c, x->A) : 0.f;
            }
        }
#pragma unroll
        for (int u = 0; u < kB; ++u) {
            const int i = i0 + u * nth;
            if (i < nit) hxsPutItem(x, st, 0, i & 3, i >> 2, e[u], ring, QS, loudLo, loudHi, flag);
        }
    }
}

// ---- register staging -------------------------------------------------------------
// One load's registers per loader wave: STEREO two f2v per item, ROW16 one f32x4.  One loop per
// format (hxsRegLoadersT<FMT>), so a loaded register is never merged with another format's
// value (a merge is a copy, and a copy waits for the load).
template <int FMT>
struct HxsRegBuf {
    f2v a[kHxsItems], b[kHxsItems];
};
template <>
struct HxsRegBuf<2> {
    f32x4 v[kHxsItems];
};
template <>
struct HxsRegBuf<3> {  // STEREO PCM16: one dword (both channels) per chunk row
    uint32_t a[kHxsItems], b[kHxsItems];
};

// Per-block load source: one resource from the block's first chunk row 0 (records end at the
// caller's input end: zeros past it), the byte stride of a row and of a chunk.
struct HxsRegSrc {
    __amdgpu_buffer_rsrc_t r;
    int rowB, chunkB, lane0;
};

template <int FMT, class XP>
__device__ __forceinline__ HxsRegSrc hxsRegSrc(XP x, int b, int lane) {
    HxsRegSrc r;
    const int col0 = b * (FMT == 5 ? 32 : 16), k = col0 / x->C, c0 = col0 - k * x->C;
    r.rowB = static_cast<int>(x->in_fs) * x->in_esz;
    r.chunkB = x->Np * x->Qc * r.rowB;
    r.r = hxsRsrcT(x, hxsChunkRow(x, k, 0), (FMT == 2 || FMT == 5) ? c0 : 0,
                   FMT == 5 ? 128 : FMT == 2 ? 64 : (FMT == 3 ? 4 : 8));
    // ROW16: lane = 16 q + r reads row r of a 16-row piece, channels 4q..4q+3 -- one instruction
    // covers 16 whole 64-B block rows (16 lines) instead of 16 B of 64 rows (64 lines); ROW32 (FMT 5,
    // hxt_kernel only): lane = 8 r + q, 8 whole 128-B rows per instruction
    r.lane0 = FMT == 5 ? (lane >> 3) * r.rowB + 16 * (lane & 7)
            : FMT == 2 ? (lane & 15) * r.rowB + 16 * (lane >> 4) : lane * r.rowB;
    return r;
}

// Issue load `st` (live: a real load; else nothing to fetch).  Always the same instruction
// pattern, kHxsItems x (2 STEREO | 1 ROW16) loads: items the load does not need (past its
// rows, dead loads, edge loads that are gathered later) get an offset past every record,
// which returns zeros without a memory access -- the compiler's vmcnt tracking then waits
// for exactly the oldest load (a conditional issue would make it wait for all).
template <int FMT>
__device__ __forceinline__ bool hxsRegIssue(const HxsStage& st, bool live, const HxsRegSrc& rs, int l, HxsRegBuf<FMT>& r) {
    const bool fast = FMT != 0 && live && st.fast;
    const int npc = fast ? (st.nrow + 63) >> 6 : 0;
    // loader index and strides opaque per call: otherwise every item's offset and mask is hoisted out
    // of the step loop into SGPRs, which spill (v_readlane per item and step)
    int lq = l;
    HxsRegSrc rq = rs;
    asm volatile("" : "+s"(lq), "+s"(rq.rowB), "+s"(rq.chunkB));
    const int base = st.T0 * rq.rowB + rq.lane0;
#pragma unroll
    for (int k = 0; k < kHxsItems; ++k) {
        const int it = lq + k * kHxsLoaders, q = it & 3, i = it >> 2;
        const bool on = it < 4 * kHxsNP && i < npc;
        if constexpr (FMT == 2) {  // item = 16-row piece (all four quads)
            const bool on16 = it < 4 * kHxsNP && 16 * it < (fast ? st.nrow : 0);
            const int o = on16 ? base + 16 * it * rq.rowB : static_cast<int>(0x80000000u);
            r.v[k] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(rs.r, o, 0, 0));
        } else if constexpr (FMT == 1 || FMT == 4) {  // f32 / int32 stereo frames
            const int o = on ? base + 64 * i * rq.rowB + 2 * q * rq.chunkB : static_cast<int>(0x80000000u);
            const int o2 = on ? o + rq.chunkB : o;
            r.a[k] = __builtin_bit_cast(f2v, __builtin_amdgcn_raw_buffer_load_b64(rs.r, o, 0, 0));
            r.b[k] = __builtin_bit_cast(f2v, __builtin_amdgcn_raw_buffer_load_b64(rs.r, o2, 0, 0));
        } else if constexpr (FMT == 3) {  // int16 stereo frames
            const int o = on ? base + 64 * i * rq.rowB + 2 * q * rq.chunkB : static_cast<int>(0x80000000u);
            const int o2 = on ? o + rq.chunkB : o;
            r.a[k] = __builtin_amdgcn_raw_buffer_load_b32(rs.r, o, 0, 0);
            r.b[k] = __builtin_amdgcn_raw_buffer_load_b32(rs.r, o2, 0, 0);
        }
    }
    return fast;
}

// Small launches, interior blocks of a STEREO (fmt 1) / ROW16 (fmt 2) f32 input: the window [0, Wg)
// of every column comes straight from the raw input through buffer loads -- one 8-B load (both
// channels of a chunk) or one 16-B load (four channels) per lane and row, rows past the input end
// read as zeros through the records -- instead of four branch-free scalar gathers per item, whose
// 64-bit address arithmetic dominated a short call's instruction stream.  Same image, same split.
template <class XP>
__device__ __forceinline__ bool hxsSmallFast(XP x, int b, int tid, int nth, char* ring, uint32_t QS, int* loudLo,
                                             int* loudHi, int* flag) {
    if (x->fmt != 1 && x->fmt != 2) return false;
    const HxsStage st = hxsStage(x, b, 0, x->Wg);  // fast: every column live, row 0 at or after the raw input
    if (!st.fast) return false;
    const int lane = tid & 63, w = tid >> 6, nw = nth >> 6;
    constexpr int kB = 4;  // items per wave in flight
    if (x->fmt == 1) {
        const HxsRegSrc rs = hxsRegSrc<1>(x, b, lane);
        const int nit = 4 * ((st.nrow + 63) >> 6);
        for (int it0 = w; it0 < nit; it0 += kB * nw) {
            f2v a[kB], c[kB];
#pragma unroll
            for (int u = 0; u < kB; ++u) {
                const int it = it0 + u * nw, q = it & 3, pc = it >> 2;
                const int o = it < nit ? rs.lane0 + 64 * pc * rs.rowB + 2 * q * rs.chunkB : static_cast<int>(0x80000000u);
                const int o2 = it < nit ? o + rs.chunkB : o;
                a[u] = __builtin_bit_cast(f2v, __builtin_amdgcn_raw_buffer_load_b64(rs.r, o, 0, 0));
                c[u] = __builtin_bit_cast(f2v, __builtin_amdgcn_raw_buffer_load_b64(rs.r, o2, 0, 0));
            }
#pragma unroll
            for (int u = 0; u < kB; ++u) {
                const int it = it0 + u * nw, row = 64 * (it >> 2) + lane;
                if (it < nit && row < st.nrow)
                    hxsPutItem(x, st, 0, it & 3, row, f32x4{a[u].x, a[u].y, c[u].x, c[u].y}, ring, QS, loudLo, loudHi, flag);
            }
        }
    } else {
        const HxsRegSrc rs = hxsRegSrc<2>(x, b, lane);
        const int nit = (st.nrow + 15) >> 4;
        for (int it0 = w; it0 < nit; it0 += kB * nw) {
            f32x4 v[kB];
#pragma unroll
            for (int u = 0; u < kB; ++u) {
                const int it = it0 + u * nw;
                const int o = it < nit ? rs.lane0 + 16 * it * rs.rowB : static_cast<int>(0x80000000u);
                v[u] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(rs.r, o, 0, 0));
            }
#pragma unroll
            for (int u = 0; u < kB; ++u) {
                const int it = it0 + u * nw, row = 16 * it + (lane & 15);
                if (it < nit && row < st.nrow) hxsPutItem(x, st, 0, lane >> 4, row, v[u], ring, QS, loudLo, loudHi, flag);
            }
        }
    }
    return true;
}

// int(clamp(float64(y), -1, 1) * 32767) with pcmWrite's semantics (f64 product: exact; NaN -> 0).
__device__ __forceinline__ int32_t pcm16Of(float y) {
    const double d = static_cast<double>(y);
    const double v = (d > 1.0 ? 1.0 : (d < -1.0 ? -1.0 : d)) * 32767.0;
    return v == v ? static_cast<int32_t>(v) : 0;
}

// Interior store of a lane's four rows.  VST (the launch's output layout, a template parameter so
// the epilogue carries no layout branches): 0 any f32 layout (4 stores), 1 channel-contiguous f32
// (one 16-B store), 2 stereo-interleaved f32 (lane pairs swap halves by DPP: one 16-B store of two
// frames each), 3 f64 (4 stores), 4 stereo-interleaved PCM16 (two int16 frames, 8 B).
template <int VST>
__device__ __forceinline__ void hxsStoreFast(const HxsArgs& x, char* p, f32x4 y, int lane) {
    const bool nt = kHxsDev && x.nt;
    if (VST == 2 || VST == 4) {
        const bool even = (lane & 1) == 0;
        const float s0 = even ? y[2] : y[0], s1 = even ? y[3] : y[1];
        const float q0 = __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(s0), 0xB1, 0xf, 0xf, false));
        const float q1 = __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(s1), 0xB1, 0xf, 0xf, false));
        f32x4 w;
        if (even) { w[0] = y[0]; w[1] = q0; w[2] = y[1]; w[3] = q1; }
        else      { w[0] = q0; w[1] = y[2]; w[2] = q1; w[3] = y[3]; }
        if constexpr (VST == 4) {  // two int16 stereo frames (8 B): clamp, x32767, truncate (main.go:497-541)
            const int32_t i0 = pcm16Of(w[0]), i1 = pcm16Of(w[1]), i2 = pcm16Of(w[2]), i3 = pcm16Of(w[3]);
            uint2 v;
            v.x = (static_cast<uint32_t>(i0) & 0xffffu) | (static_cast<uint32_t>(i1) << 16);
            v.y = (static_cast<uint32_t>(i2) & 0xffffu) | (static_cast<uint32_t>(i3) << 16);
            *reinterpret_cast<uint2*>(p) = v;
        } else if (nt) {
            __builtin_nontemporal_store(w, reinterpret_cast<f32x4*>(p));
        } else {
            *reinterpret_cast<f32x4*>(p) = w;
        }
    } else if (VST == 1) {
        if (nt) __builtin_nontemporal_store(y, reinterpret_cast<f32x4*>(p));
        else *reinterpret_cast<f32x4*>(p) = y;
    } else if (VST == 0) {
#pragma unroll
        for (int i = 0; i < 4; ++i) *reinterpret_cast<float*>(p + i * x.out_fs) = y[i];
    } else {
#pragma unroll
        for (int i = 0; i < 4; ++i) *reinterpret_cast<double*>(p + i * x.out_fs) = static_cast<double>(y[i]);
    }
}

// The per-block protocol shared by both roles (identical barrier sequences).
// Loads j = 0 .. P + ngroups - 2 (hxsLoad: the P parts of stage 0, then stages 1 ..):
//   reset B | loaders issue loads 0 .. kHxsD-1 | B |
//   step j = 0 .. stepsPad - 1: loaders convert load j (registers -> ring) and issue load
//   j + kHxsD; compute waves run MFMA group j - P (when 0 <= j - P < ngroups: stage 0 and
//   stages 1 .. j - P are in the ring); B | [fixup]
// Steps of a block (P stage-0 parts + ngroups groups), padded to a multiple of kHxsD so the
// loaders' unrolled loop issues the same loads on every path.
__device__ __forceinline__ int hxsStepsPad(const HxsArgs& x) {
    const int GQ = x.G * x.Qc;
    const int n = (x.small ? 0 : (x.Wg + GQ - 1) / GQ) + x.ngroups;
    return (n + kHxsD - 1) / kHxsD * kHxsD;
}

struct HxsShared {
    unsigned long long* stamp;
    char* ring;
    uint32_t QS;
    int* loudLo;
    int* loudHi;
    int* flag;
};

// Register staging: loader l's items of load `st` -> ring rows, from the registers of its issue
// (fast) or gathered now (edge loads).
template <int FMT, class XP>
__device__ __forceinline__ void hxsRegConvert(XP x, const HxsStage& st, bool fast, const HxsRegBuf<FMT>& r,
                                              int b, int l, int lane, const HxsShared& sh) {
    const int p0 = uni(st.T0 % x->R);
    if (FMT != 0 && fast) {  // straight-line: registers -> ring
        int lq = l;  // opaque per call (hxsRegIssue)
        asm volatile("" : "+s"(lq));
#pragma unroll
        for (int k = 0; k < kHxsItems; ++k) {
            const int it = lq + k * kHxsLoaders, q = it & 3, i = it >> 2;
            if constexpr (FMT == 2) {
                const int row = 16 * it + (lane & 15);
                if (it < 4 * kHxsNP && 16 * it < st.nrow && row < st.nrow)
                    hxsPutItem(x, st, p0, lane >> 4, row, r.v[k], sh.ring, sh.QS, sh.loudLo, sh.loudHi, sh.flag);
            } else if (it < 4 * kHxsNP && 64 * i < st.nrow) {  // uniform
                f32x4 e;
                if constexpr (FMT == 1) {
                    e = f32x4{r.a[k].x, r.a[k].y, r.b[k].x, r.b[k].y};
                } else if constexpr (FMT == 3) {  // int16 pairs -> float64(i) * (1 / 32767) -> f32
                    const uint32_t ua = r.a[k], ub = r.b[k];
                    e = f32x4{static_cast<float>(pcmToF64(static_cast<int16_t>(ua & 0xffffu), 16)),
                              static_cast<float>(pcmToF64(static_cast<int16_t>(ua >> 16), 16)),
                              static_cast<float>(pcmToF64(static_cast<int16_t>(ub & 0xffffu), 16)),
                              static_cast<float>(pcmToF64(static_cast<int16_t>(ub >> 16), 16))};
                } else {  // FMT 4: int32 pairs (PCM24 / PCM32)
                    const int bits = x->in_pcm;
                    e = f32x4{static_cast<float>(pcmToF64(__builtin_bit_cast(int32_t, r.a[k].x), bits)),
                              static_cast<float>(pcmToF64(__builtin_bit_cast(int32_t, r.a[k].y), bits)),
                              static_cast<float>(pcmToF64(__builtin_bit_cast(int32_t, r.b[k].x), bits)),
                              static_cast<float>(pcmToF64(__builtin_bit_cast(int32_t, r.b[k].y), bits))};
                }
                const int row = 64 * i + lane;
                if (row < st.nrow) hxsPutItem(x, st, p0, q, row, e, sh.ring, sh.QS, sh.loudLo, sh.loudHi, sh.flag);
            }
        }
        return;
    }
    const HxsArgsP xc = hxsCold();
    const SrcDesc src = kload(&xc->src);
#pragma unroll 1
    for (int k = 0; k < kHxsItems; ++k) {
        const int it = l + k * kHxsLoaders, q = it & 3, i = it >> 2;
        const int row = 64 * i + lane;
        if (it >= 4 * kHxsNP || 64 * i >= st.nrow) break;  // uniform (items ascend in i)
        if (row >= st.nrow) continue;
        f32x4 e;
#pragma unroll
        for (int n = 0; n < 4; ++n) {
            const int col = b * 16 + 4 * q + n;
            const int kk = col / x->C, c = col - kk * x->C;
            e[n] = col < x->ncols ? hxsGather(src, hxsChunkRow(x, kk, st.T0 + row), c, x->A) : 0.f;
        }
        hxsPutItem(x, st, p0, q, row, e, sh.ring, sh.QS, sh.loudLo, sh.loudHi, sh.flag);
    }
}

// Compute waves (one row block each).
// Per block a wave decides once whether every period of its 16 columns is an interior, fully
// stored row block ("fast": the common case -- all but the launch's edge blocks); then the
// epilogue of a period is scale + (stereo) lane swap + one 16-B store at a pointer advanced by a
// constant per period, with no per-period range checks or 64-bit index arithmetic.
template <int NS, int VST, bool FAST>
__device__ __forceinline__ void hxsGroups(const HxsArgs& x, const HxsShared& sh_, int lane, const h8v (&Ah)[NS],
                                          const h8v (&Al)[NS], uint32_t laneOff, int u0, int P, int nslot,
                                          char* obase, int64_t pstride, int64_t aCol, int64_t oRow0, bool colOk,
                                          int ccol, bool fullRb, unsigned long long& tm, unsigned long long& tw) {
    const int sh = -(x.ea + kHxXs);
    const int GQ = x.G * x.Qc;
    const uint32_t dL = 8u * static_cast<uint32_t>(x.Rt);
    const uint32_t pstep = 8u * static_cast<uint32_t>(x.Qc);
    const int dbg = kHxsDev ? x.dbg : 0;
    auto epilogue = [&](const f32x4& oA, const f32x4& oL, int p) {
        const f32x4 y = hxScale(oA, oL, sh);
        if (dbg & 2) return;
        if constexpr (FAST) {
            // periods past the chunk (ngroups * G > Np) belong to the next chunk's column, whose
            // fixup owns their loud outputs: storing them here raced with it (r05 loud sweep, C=3)
            if (p < x.Np) hxsStoreFast<VST>(x, obase + static_cast<int64_t>(p) * pstride, y, lane);
        } else {
            const int64_t a = aCol + p;
            const int64_t o0 = a * x.Pc + oRow0;
            const bool live = colOk && p < x.Np && a < x.a_hi;
            if (fullRb && live && (!x.out_pcm || VST == 4) && a * x.Pc >= x.o_lo && (a + 1) * x.Pc <= x.o_hi) {
                char* pp = x.out + (o0 + (((VST == 2 || VST == 4) && (lane & 1)) ? 2 : 0)) * x.out_fs + ((VST == 2 || VST == 4) ? 0 : ccol * x.out_cs);
                hxsStoreFast<VST>(x, pp, y, lane);
            } else if (live) {
#pragma unroll
                for (int i = 0; i < 4; ++i) {
                    const int64_t o = o0 + i;
                    if (oRow0 + i < x.Pc && o >= x.o_lo && o < x.o_hi) {
                        char* pp = x.out + o * x.out_fs + ccol * x.out_cs;
                        if (x.out_pcm) pcmWrite(pp, 0, x.out_pcm, static_cast<double>(y[i]));
                        else if (x.out_f64) *reinterpret_cast<double*>(pp) = static_cast<double>(y[i]);
                        else *reinterpret_cast<float*>(pp) = y[i];
                    }
                }
            }
        }
    };
    const int nstepsPad = hxsStepsPad(x);
    for (int j = 0; j < nstepsPad; ++j) {
        // load j -> ring (the loaders' share), then the MFMA periods of group j - P
        const unsigned long long t0 = (kHxsDev && x.prof) ? __builtin_amdgcn_s_memtime() : 0;
        const int g = j - P;
        if (g < 0 || g >= x.ngroups) {
            hxsBarrier();
            continue;
        }
        const int slot = g % nslot;
        uint32_t aH = static_cast<uint32_t>(reinterpret_cast<uintptr_t>((lds_s4p)(sh_.ring + laneOff))) +
                      8u * static_cast<uint32_t>(slot * GQ + u0);
        // B fragments read kPF steps ahead of their MFMAs (across period boundaries)
        constexpr int kPF = (NS >= 2 && GAR_HXS_PF2) ? 2 : 1;
        h8v bh0 = bFragA(aH), bl0 = bFragA(aH + dL);
        h8v bh1 = bh0, bl1 = bl0;
        if constexpr (kPF == 2) { bh1 = bFragA(aH + 256); bl1 = bFragA(aH + dL + 256); }
        // one period's MFMA program into nA (hi-x products) and nL (lo-x products); the
        // epilogue of period ep (oA, oL) issues after its second step when epi
        auto period = [&](f32x4& nA, f32x4& nL, const f32x4& oA, const f32x4& oL, bool epi, int ep, bool last) {
            asm volatile("" : "+v"(aH));  // opaque per-period base: reads use base + offset:imm
            uint32_t aL = aH + dL;
            asm volatile("" : "+v"(aL));  // lo reads: aL + offset:imm (hxt_kernel r05: -3 .. -6 %)
            const uint32_t aN = aH + pstep, aNL = aN + dL;
            nA = f32x4{0, 0, 0, 0};
            nL = nA;
#pragma unroll
            for (int s = 0; s < NS; ++s) {
                const int ug = (s + kPF) / NS, us = (s + kPF) % NS;
                h8v bhn = kPF == 2 ? bh1 : bh0, bln = kPF == 2 ? bl1 : bl0;
                if (!(ug == 1 && last)) {
                    bhn = bFragA((ug == 0 ? aH : aN) + 256 * us);
                    bln = bFragA((ug == 0 ? aL : aNL) + 256 * us);
                }
                nA = mfma16(Ah[s], bh0, nA);
                nA = mfma16(Al[s], bh0, nA);
                nL = mfma16(Ah[s], bl0, nL);
                if constexpr (kPF == 2) {
                    bh0 = bh1; bl0 = bl1; bh1 = bhn; bl1 = bln;
                } else {
                    bh0 = bhn; bl0 = bln;
                }
                __builtin_amdgcn_sched_group_barrier(0x100, 4, 0);
                __builtin_amdgcn_sched_group_barrier(0x008, 3, 0);
                __builtin_amdgcn_sched_barrier(0);
                if (s == (NS > 1 ? 1 : 0) && epi) epilogue(oA, oL, ep);
            }
            aH = aN;
        };
        const int p0 = g * x.G;
        f32x4 a0, a1 = {0, 0, 0, 0}, l0, l1 = a1;
        if (dbg & 4) {
            epilogue(a1, l1, p0);
            if (x.G > 1) epilogue(a1, l1, p0 + 1);
            if (x.G > 2) epilogue(a1, l1, p0 + 2);
        } else {
            // periods in pairs (alternating accumulators): period i's stores issue from
            // inside period i+1's MFMA stream
            period(a0, l0, a1, l1, false, 0, x.G == 1);
            int i = 1;
            for (; i + 1 < x.G; i += 2) {
                period(a1, l1, a0, l0, true, p0 + i - 1, false);
                period(a0, l0, a1, l1, true, p0 + i, i + 1 == x.G - 1);
            }
            if (i < x.G) {
                period(a1, l1, a0, l0, true, p0 + i - 1, true);
                epilogue(a1, l1, p0 + i);
            } else {
                epilogue(a0, l0, p0 + i - 1);
            }
        }
        const unsigned long long t1 = (kHxsDev && x.prof) ? __builtin_amdgcn_s_memtime() : 0;
        hxsBarrier();  // step done: load j in the ring, load j + 1 landed
        if (kHxsDev && x.prof) { tm += t1 - t0; tw += __builtin_amdgcn_s_memtime() - t1; }
    }
}

template <int NS, int VST>
__device__ __forceinline__ void hxsCompute(const HxsArgs& x, const HxsShared& sh_, int wt, int lane) {
    const uint32_t QS = sh_.QS;
    const int GQ = x.G * x.Qc;
    const int grp = lane >> 4, l16 = lane & 15;
    const uint32_t laneOff = (l16 & 3) * QS + 8u * (4 * grp + (l16 >> 2));
    const int* pt = x.progs + kBgProgInts * wt;
    const int u0 = uni(pt[4]), rbw = uni(pt[3]);
    const int tid = wt * 64 + lane, nth = 64 * (x.nprog + kHxsLoaders);
    const unsigned long long tEntry = (kHxsDev && x.prof) ? __builtin_amdgcn_s_memtime() : 0;
    unsigned long long tGath = 0, tSteps = 0;
    if constexpr (GAR_HXS_PRIO > 0) __builtin_amdgcn_s_setprio(GAR_HXS_PRIO);  // A/B: MFMA waves win VALU arbitration
    h8v Ah[NS], Al[NS];
#pragma unroll
    for (int s = 0; s < NS; ++s) {
        Ah[s] = x.A[((static_cast<size_t>(wt) * NS + s) * 2 + 0) * 64 + lane];
        Al[s] = x.A[((static_cast<size_t>(wt) * NS + s) * 2 + 1) * 64 + lane];
    }
    unsigned long long tA = 0, tB1 = 0;
    if (kHxsDev && x.prof && wt == 0) {  // development: A landed (an extra wait, stamp only)
        __builtin_amdgcn_s_waitcnt(0);
        tA = __builtin_amdgcn_s_memtime();
    }
    const bool fullRb = (rbw + 1) * 16 <= x.Pc;
    const int nslot = x.R / GQ;
    unsigned long long tm = 0, tw = 0;
    const int P = x.small ? 0 : (x.Wg + GQ - 1) / GQ;
    const int64_t pstride = static_cast<int64_t>(x.Pc) * x.out_fs;

    for (int bi = blockIdx.x; bi < x.nblocks; bi += gridDim.x) {
        const int b = hxsBlock(x, bi);
        hxsBarrier();  // loud state reset; the previous block's ring reads done
        if (kHxsDev && x.prof && bi == static_cast<int>(blockIdx.x)) tB1 = __builtin_amdgcn_s_memtime();
        if (x.small) hxsSmallStage(&x, b, tid, nth, sh_.ring, QS, sh_.loudLo, sh_.loudHi, sh_.flag);
        hxsBarrier();  // load 0 landed (small: the whole window in the ring)
        if (kHxsDev && x.prof && bi == static_cast<int>(blockIdx.x)) tGath = __builtin_amdgcn_s_memtime();
        const int col = b * 16 + l16;
        const bool colOk = col < x.ncols;
        const int kcol = col / x.C, ccol = col - kcol * x.C;
        const int64_t aCol = x.a_lo + static_cast<int64_t>(kcol) * x.Np;
        const int64_t oRow0 = static_cast<int64_t>(rbw) * 16 + 4 * grp;  // first row of this lane's accumulator
        const bool laneFast = fullRb && colOk && (!x.out_pcm || VST == 4) && aCol + x.Np <= x.a_hi &&
                              aCol * x.Pc >= x.o_lo && (aCol + x.Np) * x.Pc <= x.o_hi;
        char* obase = x.out + (aCol * x.Pc + oRow0 + (((VST == 2 || VST == 4) && (lane & 1)) ? 2 : 0)) * x.out_fs +
                      ((VST == 2 || VST == 4) ? 0 : ccol * x.out_cs);
        if (__builtin_amdgcn_ballot_w64(!laneFast) == 0)
            hxsGroups<NS, VST, true>(x, sh_, lane, Ah, Al, laneOff, u0, P, nslot, obase, pstride, aCol, oRow0, colOk,
                                     ccol, fullRb, tm, tw);
        else
            hxsGroups<NS, VST, false>(x, sh_, lane, Ah, Al, laneOff, u0, P, nslot, obase, pstride, aCol, oRow0, colOk,
                                      ccol, fullRb, tm, tw);
        if (kHxsDev && x.prof && bi == static_cast<int>(blockIdx.x)) tSteps = __builtin_amdgcn_s_memtime();
        if (*sh_.flag) {  // uniform (LDS after the barrier; reset only after the barrier below)
            __builtin_amdgcn_s_waitcnt(0);  // this wave's output stores landed
            __syncthreads();
            hxsFixup(hxsCold(), b, sh_.loudLo, sh_.loudHi);
            __syncthreads();  // every wave's fixup read loudLo/loudHi before the next block resets them
        }
    }
    if (kHxsDev && x.prof && wt == 0 && lane == 0) {  // development: first-block phase stamps of wave 0
        __builtin_amdgcn_s_waitcnt(0);
        const unsigned long long tExit = __builtin_amdgcn_s_memtime();
        atomicAdd(x.prof + 20, tGath - tEntry);
        atomicAdd(x.prof + 21, tSteps - tGath);
        atomicAdd(x.prof + 22, tExit - tSteps);
        atomicAdd(x.prof + 23, 1ull);
        atomicAdd(x.prof + 24, tA - tEntry);
        atomicAdd(x.prof + 25, tB1 - tEntry);
        unsigned long long lo = ~0ull, hi = 0;
        for (int w = 0; w < x.nprog + kHxsLoaders; ++w) { lo = min(lo, sh_.stamp[w]); hi = max(hi, sh_.stamp[w]); }
        atomicAdd(x.prof + 26, hi - lo);
        atomicAdd(x.prof + 27, tEntry - lo);
    }
    if (kHxsDev && x.prof && lane == 0) {
        atomicAdd(x.prof + 4, tm);
        atomicAdd(x.prof + 5, tw);
        atomicAdd(x.prof + 6, 1ull);
    }
}

// History keep for the next call (launchGather's job, folded into this launch): hdst is the other
// buffer of the double-buffered history, so it never aliases what the launch reads.  Large launches:
// every thread after its role; small launches: the loader waves during the MFMA step (hxsRegLoadersT).
__device__ __forceinline__ void hxsHistKeep(const HxsArgs& x, int64_t me, int64_t nth) {
    const HxsArgsP xc = hxsCold();
    const SrcDesc src = kload(&xc->src);
    const int64_t total = x.hn * x.C;
    for (int64_t i = me; i < total; i += nth) {
        const int64_t t = i / x.C;
        x.hdst[i] = srcRead<float>(src, x.ht0 + t, static_cast<int>(i - t * x.C));
    }
}

// Loader wave l: same barrier sequence as the compute
// waves; in step j it converts load j (issued kHxsD steps earlier) into the ring
// and issues load j + kHxsD into the registers just freed.
template <int FMT>
__device__ __forceinline__ void hxsRegLoadersT(const HxsArgs& x, const HxsShared& sh_, int l, int lane) {
    // Every argument is read through an opaque kernarg pointer renewed per step (hxsCold), so
    // the scalar loads sit next to their uses instead of pinning ~70 SGPRs for the whole
    // kernel (spilled SGPRs cost a v_readlane per use inside the conversion).
    HxsArgsP xp = hxsCold();
    const int GQ = xp->G * xp->Qc;
    const int P = xp->small ? 0 : (xp->Wg + GQ - 1) / GQ, nL = xp->small ? 0 : P + xp->ngroups - 1;
    const int nstepsPad = hxsStepsPad(x);
    const int tid = (x.nprog + l) * 64 + lane, nth = 64 * (x.nprog + kHxsLoaders);
    for (int bi = blockIdx.x; bi < xp->nblocks; bi += gridDim.x) {
        const int b = hxsBlock(x, bi);
        if (l == 0 && lane < 16) { sh_.loudLo[lane] = INT_MAX; sh_.loudHi[lane] = -1; }
        if (l == 0 && lane == 0) *sh_.flag = 0;
        hxsBarrier();  // loud state reset; the previous block's ring reads done
        HxsRegBuf<FMT> buf[kHxsD];
        bool fastL[kHxsD];
        const HxsRegSrc rs = hxsRegSrc<FMT>(xp, b, lane);
#pragma unroll
        for (int d = 0; d < kHxsD; ++d) fastL[d] = hxsRegIssue<FMT>(hxsLoad(xp, b, d, P), d < nL, rs, l, buf[d]);
        if (xp->small) hxsSmallStage(xp, b, tid, nth, sh_.ring, sh_.QS, sh_.loudLo, sh_.loudHi, sh_.flag);
        hxsBarrier();  // (small: the whole window in the ring)
        for (int j0 = 0; j0 < nstepsPad; j0 += kHxsD) {
#pragma unroll
            for (int d = 0; d < kHxsD; ++d) {
                const int j = j0 + d;
                xp = hxsCold();
                const int dbg = kHxsDev ? xp->dbg : 0;
                if (xp->small && j == 0 && x.hn > 0 && bi == static_cast<int>(blockIdx.x))  // beside the MFMA group
                    hxsHistKeep(x, static_cast<int64_t>(blockIdx.x) * 64 * kHxsLoaders + 64 * l + lane,
                                static_cast<int64_t>(gridDim.x) * 64 * kHxsLoaders);
                if ((dbg & 64) && j >= P) {  // development: consume the registers, no conversion
                    float s = 0.f;
#pragma unroll
                    for (int k = 0; k < kHxsItems; ++k) {
                        if constexpr (FMT == 2) s += buf[d].v[k][0] + buf[d].v[k][3];
                        else if constexpr (FMT == 1 || FMT == 4) s += buf[d].a[k].x + buf[d].b[k].y;
                        else if constexpr (FMT == 3) s += static_cast<float>(buf[d].a[k] ^ buf[d].b[k]);
                    }
                    if (s == 1234.5f) sh_.loudLo[0] = 0;
                } else if (j < nL && !((dbg & 16) && j >= P)) {
                    hxsRegConvert<FMT>(xp, hxsLoad(xp, b, j, P), fastL[d], buf[d], b, l, lane, sh_);
                }
                if (!(dbg & 128))  // development: no issue at all (the skeleton's cost without dummy loads)
                    fastL[d] = hxsRegIssue<FMT>(hxsLoad(xp, b, j + kHxsD, P), j + kHxsD < nL && !((dbg & 1) && j >= P), rs,
                                                l, buf[d]);
                hxsBarrier();  // step done: load j in the ring
            }
        }
        if (*sh_.flag) {  // same sequence as the compute waves
            __builtin_amdgcn_s_waitcnt(0);
            __syncthreads();
            hxsFixup(hxsCold(), b, sh_.loudLo, sh_.loudHi);
            __syncthreads();
        }
    }
}

__device__ __forceinline__ void hxsRegLoaders(const HxsArgs& x, const HxsShared& sh_, int l, int lane) {
#ifdef GAR_HXS_ONLYFMT  // development: one loader format per build (register-allocation studies)
    hxsRegLoadersT<GAR_HXS_ONLYFMT>(x, sh_, l, lane);
    return;
#endif
    if (x.fmt == 1) hxsRegLoadersT<1>(x, sh_, l, lane);
    else if (x.fmt == 2) hxsRegLoadersT<2>(x, sh_, l, lane);
    else if (x.fmt == 3) hxsRegLoadersT<3>(x, sh_, l, lane);
    else if (x.fmt == 4) hxsRegLoadersT<4>(x, sh_, l, lane);
    else hxsRegLoadersT<0>(x, sh_, l, lane);
}

template <int NS, int VST>
__global__ __launch_bounds__(64 * kHxsWaves) void hxs_kernel(HxsArgs x) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    HxsShared s;
#if GAR_HXS_DEV
    __shared__ unsigned long long hxsStamp[kHxsWaves];  // development (GAR_HXS_PROF): wave entry times
    if (x.prof && (threadIdx.x & 63) == 0) hxsStamp[threadIdx.x >> 6] = __builtin_amdgcn_s_memtime();
    s.stamp = hxsStamp;
#else
    s.stamp = nullptr;
#endif
    s.QS = 16u * static_cast<uint32_t>(x.Rt) + 64u;  // quad: hi rows, lo rows, +64 B skew
    s.ring = reinterpret_cast<char*>(smem);
    s.loudLo = reinterpret_cast<int*>(smem + 4 * static_cast<size_t>(s.QS));
    s.loudHi = s.loudLo + 16;
    s.flag = s.loudHi + 16;
    const int lane = threadIdx.x & 63;
    const int wt = uni(threadIdx.x >> 6);
    // History keep for the next call (launchGather's job, folded into this launch; hdst is the other
    // buffer of the double-buffered history, so it never aliases what this launch reads).  Small
    // launches: the loader waves copy it while the compute waves run their MFMAs (the loaders' only
    // other work is the one-pass window gather); otherwise every thread after its role.
    if (wt < x.nprog) hxsCompute<NS, VST>(x, s, wt, lane);
    else hxsRegLoaders(x, s, wt - x.nprog, lane);
    if (x.hn > 0 && !x.small) hxsHistKeep(x, static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x,
                                          static_cast<int64_t>(gridDim.x) * blockDim.x);
}

// One compute wave of a small launch (one macro period per column): NS steps of 3 MFMAs over the
// window image from LDS address aH (hi plane; lo plane at + dL), scale, store row block rbw of
// block b's 16 columns.  Shared by hxs_small_kernel and hxq_kernel: identical bits.
template <int NS, int VST>
__device__ __forceinline__ void hxsSmallOut(const HxsArgs& x, uint32_t aH, uint32_t dL, const h8v* Ah, const h8v* Al, int b,
                                            int rbw, int lane, int sh) {
    const int grp = lane >> 4, l16 = lane & 15;
    f32x4 nA = {0, 0, 0, 0}, nL = nA;
    uint32_t aL = aH + dL;
    asm volatile("" : "+v"(aL));  // lo reads: aL + offset:imm
#pragma unroll
    for (int s = 0; s < NS; ++s) {
        const h8v bh = bFragA(aH + 256 * s), bl = bFragA(aL + 256 * s);
        nA = mfma16(Ah[s], bh, nA);
        nA = mfma16(Al[s], bh, nA);
        nL = mfma16(Ah[s], bl, nL);
    }
    const f32x4 y = hxScale(nA, nL, sh);
    const int col = b * 16 + l16;
    const bool colOk = col < x.ncols;
    const int kcol = col / x.C, ccol = col - kcol * x.C;
    const int64_t a = x.a_lo + static_cast<int64_t>(kcol) * x.Np;  // Np == 1: the column's one period
    const int64_t oRow0 = static_cast<int64_t>(rbw) * 16 + 4 * grp;
    const int64_t o0 = a * x.Pc + oRow0;
    const bool fullRb = (rbw + 1) * 16 <= x.Pc;
    const bool live = colOk && a < x.a_hi;
    // whole-period stores need both lanes of a stereo pair (same chunk: same condition)
    if (fullRb && live && (!x.out_pcm || VST == 4) && a * x.Pc >= x.o_lo && (a + 1) * x.Pc <= x.o_hi) {
        char* pp = x.out + (o0 + (((VST == 2 || VST == 4) && (lane & 1)) ? 2 : 0)) * x.out_fs +
                   ((VST == 2 || VST == 4) ? 0 : ccol * x.out_cs);
        hxsStoreFast<VST>(x, pp, y, lane);
    } else if (live) {
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int64_t o = o0 + i;
            if (oRow0 + i < x.Pc && o >= x.o_lo && o < x.o_hi) {
                char* pp = x.out + o * x.out_fs + ccol * x.out_cs;
                if (x.out_pcm) pcmWrite(pp, 0, x.out_pcm, static_cast<double>(y[i]));
                else if (x.out_f64) *reinterpret_cast<double*>(pp) = static_cast<double>(y[i]);
                else *reinterpret_cast<float*>(pp) = y[i];
            }
        }
    }
}

// Launch (explicitly instantiated in gar_hxs_i*.hip).
// Small launches (x.small: stream chunks, flush tails -- one macro period per column): a compact
// kernel of compute waves only, so the launch runs a short, warm instruction stream instead of the
// streaming kernel's loader / ring / format machinery (whose cold code dominated a 4096-frame call).
// Same window image, same A fragments, same MFMA order and epilogue as hxs_kernel: identical bits.
//   all waves: gather the block's window [0, Wg) into the image (hxsSmallStage) | barrier |
//   wave w < nprog: row block w, NS steps of 3 MFMAs, scale, store | loud fixup | history keep.
template <int NS, int VST>
__global__ __launch_bounds__(64 * kHxRbMaxWaves) void hxs_small_kernel(HxsArgs x) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    const uint32_t QS = 16u * static_cast<uint32_t>(x.Rt) + 64u;
    char* ring = reinterpret_cast<char*>(smem);
    int* loudLo = reinterpret_cast<int*>(smem + 4 * static_cast<size_t>(QS));
    int* loudHi = loudLo + 16;
    int* flag = loudHi + 16;
    const int lane = threadIdx.x & 63;
    const int wt = uni(threadIdx.x >> 6);
    const int grp = lane >> 4, l16 = lane & 15;
    const bool comp = wt < x.nprog;
    h8v Ah[NS], Al[NS];
    int u0 = 0, rbw = 0;
    if (comp) {  // A lands while the window is gathered
        const int* pt = x.progs + kBgProgInts * wt;
        u0 = uni(pt[4]);
        rbw = uni(pt[3]);
#pragma unroll
        for (int s = 0; s < NS; ++s) {
            Ah[s] = x.A[((static_cast<size_t>(wt) * NS + s) * 2 + 0) * 64 + lane];
            Al[s] = x.A[((static_cast<size_t>(wt) * NS + s) * 2 + 1) * 64 + lane];
        }
    }
    const uint32_t laneOff = (l16 & 3) * QS + 8u * (4 * grp + (l16 >> 2));
    const uint32_t dL = 8u * static_cast<uint32_t>(x.Rt);
    const int sh = -(x.ea + kHxXs);
    // history keep for the next call: the first kHk elements of this thread are read up front, so
    // their round trip overlaps the window gather's instead of following the MFMAs
    constexpr int kHk = 2;
    const int64_t hme = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
    const int64_t hnth = static_cast<int64_t>(gridDim.x) * blockDim.x;
    const int64_t htot = x.hn * x.C;
    float hk[kHk];
    if (x.hn > 0) {
        const HxsArgsP xc = hxsCold();
        const SrcDesc src = kload(&xc->src);
#pragma unroll
        for (int u = 0; u < kHk; ++u) {
            const int64_t i = hme + u * hnth;
            const int64_t t = i / x.C;
            hk[u] = i < htot ? hxsGather(src, x.ht0 + t, static_cast<int>(i - t * x.C), x.A) : 0.f;
        }
    }
    for (int b = blockIdx.x; b < x.nblocks; b += gridDim.x) {
        if (threadIdx.x < 16) { loudLo[threadIdx.x] = INT_MAX; loudHi[threadIdx.x] = -1; }
        if (threadIdx.x == 0) *flag = 0;
        __syncthreads();  // loud state reset; the previous block's image reads done
        if (!hxsSmallFast(&x, b, static_cast<int>(threadIdx.x), static_cast<int>(blockDim.x), ring, QS, loudLo, loudHi, flag))
            hxsSmallStage(&x, b, static_cast<int>(threadIdx.x), static_cast<int>(blockDim.x), ring, QS, loudLo, loudHi, flag);
        __syncthreads();  // the whole window in the image
        if (comp)
            hxsSmallOut<NS, VST>(x, static_cast<uint32_t>(reinterpret_cast<uintptr_t>((lds_s4p)(ring + laneOff))) + 8u * static_cast<uint32_t>(u0),
                                 dL, Ah, Al, b, rbw, lane, sh);
        if (*flag) {  // uniform (LDS after the barrier)
            __builtin_amdgcn_s_waitcnt(0);
            __syncthreads();
            hxsFixup(hxsCold(), b, loudLo, loudHi);
        }
        __syncthreads();  // every wave done with the image / loud state before the next block
    }
    if (x.hn > 0) {
#pragma unroll
        for (int u = 0; u < kHk; ++u)
            if (hme + u * hnth < htot) x.hdst[hme + u * hnth] = hk[u];
        if (htot > kHk * hnth) hxsHistKeep(x, hme + kHk * hnth, hnth);  // the rest (long histories)
    }
}

// ---- hxq_kernel: small launches of f32 STEREO / ROW16 input over many workgroups ----------------
// A 4096-frame stereo call is 28 macro periods x 2 channels = 56 columns = 4 blocks: on
// hxs_small_kernel that is 4 workgroups, each gathering its whole window and running all row
// blocks.  Here workgroup (b, g) runs row blocks [g*qRbs, (g+1)*qRbs) of block b (qRbs = 1: 40
// workgroups for the stereo call): its waves load only the union of those row blocks' windows,
// every row -- history seam and flush tail included -- through buffer loads (input and history
// resources, per-lane selection, zeros past both), split it into the same f16 image and run the
// same MFMA order and epilogue (hxsSmallOut): identical bits to hxs_small_kernel / hxs_kernel.
constexpr int kHxqMaxWaves = 12;
constexpr int kHxqB = 6;  // items per wave in flight (4 waves: 24 items, a 5-6 piece window in one round trip)

struct HxqSrc {
    __amdgpu_buffer_rsrc_t in, hist;
    int64_t Tb;           // absolute row of the block's first chunk, row 0
    int64_t fastLo, fastHi, hb, hlen, vend;
    int rowB, hld;        // input row bytes, history row stride (elements)
    bool useH;            // the block's window reaches into the history
};

// Sources of absolute row T: the input (inI: row T - Tb of the input resource) or the history (inH:
// byte offset oh of element cH of its row); neither -> zeros.  Offsets past every record: 0x80000000.
constexpr int kHxqOob = static_cast<int>(0x80000000u);
__device__ __forceinline__ void hxqRow(const HxqSrc& q, int64_t T, int cH, bool& inI, bool& inH, int& oh) {
    const int64_t h = T - q.hb;
    inH = q.useH && T >= 0 && T < q.vend && h >= 0 && h < q.hlen;
    inI = !inH && T >= q.fastLo && T < q.fastHi;
    oh = inH ? (static_cast<int>(h) * q.hld + cH) * 4 : kHxqOob;
}

// Conversion of one item: row `row` of the image (column-relative row lo + row), quad q.
__device__ __forceinline__ void hxqPut(char* ring, uint32_t QS, uint32_t Rt, int q, int row, int t, f32x4 e, int* loudLo,
                                       int* loudHi, int* flag) {
    const bool l0 = hxLoud(e[0]), l1 = hxLoud(e[1]), l2 = hxLoud(e[2]), l3 = hxLoud(e[3]);
    if (__builtin_expect(l0 | l1 | l2 | l3, 0)) {
        if (l0) { atomicMin(loudLo + 4 * q, t); atomicMax(loudHi + 4 * q, t); e[0] = 0.f; }
        if (l1) { atomicMin(loudLo + 4 * q + 1, t); atomicMax(loudHi + 4 * q + 1, t); e[1] = 0.f; }
        if (l2) { atomicMin(loudLo + 4 * q + 2, t); atomicMax(loudHi + 4 * q + 2, t); e[2] = 0.f; }
        if (l3) { atomicMin(loudLo + 4 * q + 3, t); atomicMax(loudHi + 4 * q + 3, t); e[3] = 0.f; }
        *flag = 1;
    }
    uint2 hv, lv;
    hxSplit2(e[0], e[1], hv.x, lv.x);
    hxSplit2(e[2], e[3], hv.y, lv.y);
    char* qb = ring + q * QS + 8 * row;
    *reinterpret_cast<uint2*>(qb) = hv;
    *reinterpret_cast<uint2*>(qb + 8 * Rt) = lv;
}

// hxsFixup restricted to output rows [r0, r1) of each period (the workgroup's row blocks: another
// workgroup owns -- and stores -- the other rows).
__device__ __forceinline__ void hxqFixup(HxsArgsP xp, int b, const int* loudLo, const int* loudHi, int r0, int r1) {
    const SrcDesc src = kload(&xp->src);
    const OutDesc od = kload(&xp->od);
    const int Qc = xp->Qc, Np = xp->Np, C = xp->C, ncols = xp->ncols, Pc = xp->Pc;
    r1 = min(r1, Pc);
    const int nr = r1 - r0;
    const int64_t a_lo = xp->a_lo, a_hi = xp->a_hi;
    for (int j = 0; j < 16; ++j) {
        const int lo = loudLo[j], hi = loudHi[j];
        const int col = b * 16 + j;
        if (hi < 0 || col >= ncols || nr <= 0) continue;
        const int k = col / C, c = col - k * C;
        const int p0 = max(0, (lo - xp->Kread) / Qc), p1 = min(Np - 1, hi / Qc);
        const int n = (p1 - p0 + 1) * nr;
        for (int idx = threadIdx.x; idx < n; idx += blockDim.x) {
            const int p = p0 + idx / nr, r = r0 + (idx - (idx / nr) * nr);
            const int64_t a = a_lo + static_cast<int64_t>(k) * Np + p;
            if (a >= a_hi) continue;
            const int64_t o = a * Pc + r;
            if (o < od.o_lo || o >= od.o_hi) continue;
            const int w0 = p * Qc + xp->rowOff[r], w1 = w0 + xp->rowLen[r];
            if (w1 <= lo || w0 > hi) continue;
            const int64_t t0 = a * Qc + xp->rowOff[r];
            bool loud = false;
            for (int kk = 0; kk < w1 - w0 && !loud; ++kk) loud = hxLoud(srcRead<float>(src, t0 + kk, c));
            if (loud) outWrite<float>(od, o, c, static_cast<float>(hxsExact(xp, a, r, c)));
        }
    }
}

template <int NS, int VST>
__global__ __launch_bounds__(64 * kHxqMaxWaves) void hxq_kernel(HxsArgs x) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    const uint32_t Rt = static_cast<uint32_t>(x.Rt), QS = 16u * Rt + 64u;
    char* ring = reinterpret_cast<char*>(smem);
    int* loudLo = reinterpret_cast<int*>(smem + 4 * static_cast<size_t>(QS));
    int* loudHi = loudLo + 16;
    int* flag = loudHi + 16;
    const int lane = threadIdx.x & 63;
    const int w = uni(threadIdx.x >> 6), nw = uni(blockDim.x >> 6);
    const unsigned long long tEntry = (kHxsDev && x.prof) ? __builtin_amdgcn_s_memtime() : 0;
    const unsigned long long rEntry = (kHxsDev && x.prof) ? __builtin_amdgcn_s_memrealtime() : 0;
    const int b = uni(blockIdx.x / x.qGroups);
    const int r0 = uni((blockIdx.x - b * x.qGroups) * x.qRbs);
    const int nrw = min(x.qRbs, x.nprog - r0);
    // union window [lo, lo + nrow) of the workgroup's row blocks (column-relative rows)
    int lo = INT_MAX, hi = 0;
    for (int i = 0; i < nrw; ++i) {
        const int u = x.qU0[r0 + i];
        lo = min(lo, u);
        hi = max(hi, u);
    }
    const int nrow = hi + 32 * NS - lo;
    const bool comp = w < nrw;
    h8v Ah[NS], Al[NS];
    int u0 = 0, rbw = 0;
    if (comp) {  // A lands while the window loads
        const int wt = r0 + w;
        u0 = x.qU0[wt];
        rbw = x.qRbw[wt];
#pragma unroll
        for (int s = 0; s < NS; ++s) {
            Ah[s] = x.A[((static_cast<size_t>(wt) * NS + s) * 2 + 0) * 64 + lane];
            Al[s] = x.A[((static_cast<size_t>(wt) * NS + s) * 2 + 1) * 64 + lane];
        }
    }
    const HxsArgsP xc = hxsCold();
    const SrcDesc src = kload(&xc->src);
    // load sources
    HxqSrc q;
    const int col0 = b * 16, kb = col0 / x.C, c0 = col0 - kb * x.C;
    const int chunkRows = x.Np * x.Qc;
    q.Tb = hxsChunkRow(&x, kb, 0);
    q.fastLo = x.fastLo;
    q.fastHi = x.fastHi;
    q.hb = src.hist_base;
    q.hlen = src.hist ? src.hist_len : 0;
    q.vend = src.valid_end;
    q.rowB = static_cast<int>(x.in_fs) * 4;
    q.hld = static_cast<int>(src.hist_ld);
    if (x.fmt == 0)  // per-lane checks guard every load (host: every offset < 2^31)
        q.in = __builtin_amdgcn_make_buffer_rsrc(const_cast<char*>(x.in + q.Tb * x.in_fs * x.in_esz), 0, 0x7fffffff, 0x00020000);
    else
        q.in = hxsRsrcT(&x, q.Tb, x.fmt == 2 ? c0 : 0, x.fmt == 2 ? 64 : 8);
    {
        const int64_t hrows = min(q.hlen, q.vend - q.hb);
        const int64_t nb = hrows > 0 ? hrows * q.hld * 4 : 0;
        q.hist = __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(src.hist), 0, static_cast<int>(nb < 0x7fffffff ? nb : 0x7fffffff),
                                                   0x00020000);
    }
    q.useH = q.hlen > 0 && q.Tb + lo < q.hb + q.hlen;  // uniform: some row of the block's window is history
    // history keep for the next call (rows [ht0, ht0 + hn) of the stream): the first kHk elements of
    // this thread up front, through buffer loads (vector-memory counter only: a flat load would also
    // hold every LDS wait and barrier of the window staging until it lands)
    constexpr int kHk = 2;
    const int64_t hme = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
    const int64_t hnth = static_cast<int64_t>(gridDim.x) * blockDim.x;
    const int64_t htot = x.hn * x.C;
    float hk[kHk];
    if (x.hn > 0 && !(x.qOpt & 2)) {  // variant: flat gathers
#pragma unroll
        for (int u = 0; u < kHk; ++u) {
            const int64_t i = hme + u * hnth;
            const int64_t t = i / x.C;
            hk[u] = i < htot ? hxsGather(src, x.ht0 + t, static_cast<int>(i - t * x.C), x.A) : 0.f;
        }
    }
    if (x.hn > 0 && (x.qOpt & 2)) {
        HxqSrc qk = q;
        qk.useH = q.hlen > 0;
        const __amdgpu_buffer_rsrc_t rk =
            __builtin_amdgcn_make_buffer_rsrc(const_cast<char*>(x.in + x.ht0 * x.in_fs * x.in_esz), 0, 0x7fffffff, 0x00020000);
#pragma unroll
        for (int u = 0; u < kHk; ++u) {
            const int64_t i = hme + u * hnth;
            const int64_t t = i / x.C;
            const int c = static_cast<int>(i - t * x.C);
            bool inI, inH;
            int oh;
            hxqRow(qk, i < htot ? x.ht0 + t : -1, c, inI, inH, oh);
            const int oi = inI ? static_cast<int>((t * x.in_fs + static_cast<int64_t>(c) * x.in_cs) * x.in_esz) : kHxqOob;
            const float vi = x.in_esz == 8 ? static_cast<float>(__builtin_bit_cast(double, __builtin_amdgcn_raw_buffer_load_b64(rk, oi, 0, 0)))
                                           : __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rk, oi, 0, 0));
            const float vh = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(qk.hist, oh, 0, 0));
            hk[u] = inH ? vh : vi;
        }
    }
    // loud state reset, then a barrier before any conversion: placed after the first batch's loads
    // issue (every wave runs one batch at least), so the barrier overlaps their round trip
    auto loudReset = [&]() {
        if (threadIdx.x < 16) { loudLo[threadIdx.x] = INT_MAX; loudHi[threadIdx.x] = -1; }
        if (threadIdx.x == 0) *flag = 0;
        hxsBarrier();
    };
    unsigned long long tB1 = 0;
    const bool early = x.qOpt & 1;
    if (!early) { loudReset(); if (kHxsDev && x.prof) tB1 = __builtin_amdgcn_s_memtime(); }
    if (x.fmt == 1) {  // STEREO: item = (quad, 64-row piece), chunks 2q, 2q+1 of the block (both channels)
        const int nit = 4 * ((nrow + 63) >> 6);
        for (int it0 = w, first = 1; first || it0 < nit; it0 += kHxqB * nw) {
            f2v a[kHxqB], c[kHxqB], ah[kHxqB], ch[kHxqB];
            bool hA[kHxqB], hC[kHxqB];
#pragma unroll
            for (int u = 0; u < kHxqB; ++u) {
                const int it = it0 + u * nw, qd = it & 3, pc = it >> 2;
                const int t = lo + 64 * pc + lane;
                const bool on = it < nit && 64 * pc + lane < nrow;
                const int64_t T0 = q.Tb + static_cast<int64_t>(2 * qd) * chunkRows + t;
                int oh0, oh1;
                bool i0, i1;
                hxqRow(q, on ? T0 : -1, 0, i0, hA[u], oh0);
                hxqRow(q, on ? T0 + chunkRows : -1, 0, i1, hC[u], oh1);
                const int oi0 = i0 ? static_cast<int>(T0 - q.Tb) * q.rowB : kHxqOob;
                const int oi1 = i1 ? static_cast<int>(T0 + chunkRows - q.Tb) * q.rowB : kHxqOob;
                a[u] = __builtin_bit_cast(f2v, __builtin_amdgcn_raw_buffer_load_b64(q.in, oi0, 0, 0));
                c[u] = __builtin_bit_cast(f2v, __builtin_amdgcn_raw_buffer_load_b64(q.in, oi1, 0, 0));
                if (q.useH) {
                    ah[u] = __builtin_bit_cast(f2v, __builtin_amdgcn_raw_buffer_load_b64(q.hist, oh0, 0, 0));
                    ch[u] = __builtin_bit_cast(f2v, __builtin_amdgcn_raw_buffer_load_b64(q.hist, oh1, 0, 0));
                }
            }
            if (first && early) { loudReset(); if (kHxsDev && x.prof) tB1 = __builtin_amdgcn_s_memtime(); }
            first = 0;
#pragma unroll
            for (int u = 0; u < kHxqB; ++u) {
                const int it = it0 + u * nw, pc = it >> 2, row = 64 * pc + lane;
                if (it < nit && row < nrow) {
                    const f2v va = (q.useH && hA[u]) ? ah[u] : a[u];
                    const f2v vc = (q.useH && hC[u]) ? ch[u] : c[u];
                    hxqPut(ring, QS, Rt, it & 3, row, lo + row, f32x4{va.x, va.y, vc.x, vc.y}, loudLo, loudHi, flag);
                }
            }
        }
    } else if (x.fmt == 0) {  // any other f32 / f64 layout: item = (quad, 64-row piece), one element load per column
        const int nit = 4 * ((nrow + 63) >> 6);
        const int esz = x.in_esz;
        for (int it0 = w, first = 1; first || it0 < nit; it0 += kHxqB * nw) {
            f32x4 v[kHxqB], vh[kHxqB];
            bool hV[kHxqB][4];
#pragma unroll
            for (int u = 0; u < kHxqB; ++u) {
                const int it = it0 + u * nw, qd = it & 3, pc = it >> 2;
                const int row = 64 * pc + lane;
                const bool on = it < nit && row < nrow;
#pragma unroll
                for (int n = 0; n < 4; ++n) {
                    const int col = col0 + 4 * qd + n, k = col / x.C, c = col - k * x.C;  // wave-uniform
                    const int64_t dT = static_cast<int64_t>(k - kb) * chunkRows + lo + row;  // T - Tb
                    int oh;
                    bool inI;
                    hxqRow(q, on ? q.Tb + dT : -1, c, inI, hV[u][n], oh);
                    const int oi = inI ? static_cast<int>((dT * x.in_fs + static_cast<int64_t>(c) * x.in_cs) * esz) : kHxqOob;
                    if (esz == 8) v[u][n] = static_cast<float>(__builtin_bit_cast(double, __builtin_amdgcn_raw_buffer_load_b64(q.in, oi, 0, 0)));
                    else v[u][n] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(q.in, oi, 0, 0));
                    if (q.useH) vh[u][n] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(q.hist, oh, 0, 0));
                }
            }
            if (first && early) { loudReset(); if (kHxsDev && x.prof) tB1 = __builtin_amdgcn_s_memtime(); }
            first = 0;
#pragma unroll
            for (int u = 0; u < kHxqB; ++u) {
                const int it = it0 + u * nw, row = 64 * (it >> 2) + lane;
                if (it < nit && row < nrow) {
                    f32x4 e = v[u];
                    if (q.useH) {
#pragma unroll
                        for (int n = 0; n < 4; ++n) e[n] = hV[u][n] ? vh[u][n] : e[n];
                    }
                    hxqPut(ring, QS, Rt, it & 3, row, lo + row, e, loudLo, loudHi, flag);
                }
            }
        }
    } else {  // ROW16: item = 16-row piece, lane = 16 quad + row: channels c0 + 4 quad .. + 3 of chunk kb
        const int nit = (nrow + 15) >> 4;
        const int qd = lane >> 4;
        for (int it0 = w, first = 1; first || it0 < nit; it0 += kHxqB * nw) {
            f32x4 v[kHxqB], vh[kHxqB];
            bool hV[kHxqB];
#pragma unroll
            for (int u = 0; u < kHxqB; ++u) {
                const int it = it0 + u * nw;
                const int row = 16 * it + (lane & 15);
                const bool on = it < nit && row < nrow;
                int oh;
                bool inI;
                hxqRow(q, on ? q.Tb + lo + row : -1, c0 + 4 * qd, inI, hV[u], oh);
                const int oi = inI ? (lo + row) * q.rowB + 16 * qd : kHxqOob;
                v[u] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(q.in, oi, 0, 0));
                if (q.useH) vh[u] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(q.hist, oh, 0, 0));
            }
            if (first && early) { loudReset(); if (kHxsDev && x.prof) tB1 = __builtin_amdgcn_s_memtime(); }
            first = 0;
#pragma unroll
            for (int u = 0; u < kHxqB; ++u) {
                const int it = it0 + u * nw, row = 16 * it + (lane & 15);
                if (it < nit && row < nrow) hxqPut(ring, QS, Rt, qd, row, lo + row, (q.useH && hV[u]) ? vh[u] : v[u], loudLo, loudHi, flag);
            }
        }
    }
    hxsBarrier();  // the window image complete
    const unsigned long long tImg = (kHxsDev && x.prof) ? __builtin_amdgcn_s_memtime() : 0;
    if (comp) {
        const int grp = lane >> 4, l16 = lane & 15;
        const uint32_t laneOff = (l16 & 3) * QS + 8u * (4 * grp + (l16 >> 2));
        hxsSmallOut<NS, VST>(x, static_cast<uint32_t>(reinterpret_cast<uintptr_t>((lds_s4p)(ring + laneOff))) + 8u * static_cast<uint32_t>(u0 - lo),
                             8u * Rt, Ah, Al, b, rbw, lane, -(x.ea + kHxXs));
    }
    if (*flag) {  // uniform (LDS after the barrier)
        __builtin_amdgcn_s_waitcnt(0);
        __syncthreads();
        hxqFixup(hxsCold(), b, loudLo, loudHi, 16 * r0, 16 * (r0 + nrw));
    }
    const unsigned long long tOut = (kHxsDev && x.prof) ? __builtin_amdgcn_s_memtime() : 0;
    if (x.hn > 0) {
#pragma unroll
        for (int u = 0; u < kHk; ++u)
            if (hme + u * hnth < htot) x.hdst[hme + u * hnth] = hk[u];
        if (htot > kHk * hnth) hxsHistKeep(x, hme + kHk * hnth, hnth);
    }
    if (kHxsDev && x.prof && threadIdx.x == 0) {  // development: wave 0's phases, workgroup life, launch span
        __builtin_amdgcn_s_waitcnt(0);
        const unsigned long long tEnd = __builtin_amdgcn_s_memtime(), rEnd = __builtin_amdgcn_s_memrealtime();
        atomicAdd(x.prof + 40, tB1 - tEntry);
        atomicAdd(x.prof + 41, tImg - tB1);
        atomicAdd(x.prof + 42, tOut - tImg);
        atomicAdd(x.prof + 43, tEnd - tOut);
        atomicAdd(x.prof + 44, 1ull);
        atomicMin(x.prof + 10, rEntry);
        atomicMax(x.prof + 11, rEnd);
        if (blockIdx.x < 4096) { x.prof[64 + 2 * blockIdx.x] = rEntry; x.prof[65 + 2 * blockIdx.x] = rEnd - rEntry; }
    }
}

template <int NS, int VST>
hipError_t hxsLaunch(const HxsArgs& x, size_t lds, int64_t blocks, hipStream_t st) {
    if (x.small && x.qGroups > 0) {  // hxq_kernel: (block, row-block group) workgroups
        if (const size_t lim_ = setMaxLdsOnce(reinterpret_cast<const void*>(&hxq_kernel<NS, VST>)); lim_ < lds) return ldsTooBig("hxq_kernel", lds, lim_);
        static const int knobW = std::getenv("GAR_HXQ_W") ? std::atoi(std::getenv("GAR_HXQ_W")) : 4;  // waves per workgroup (>= qRbs)
        const int nw = std::min(kHxqMaxWaves, std::max(std::max(knobW, 1), x.qRbs));
        hipLaunchKernelGGL((hxq_kernel<NS, VST>), dim3(static_cast<unsigned>(blocks * x.qGroups)), dim3(64 * nw), lds, st, x);
        return hipGetLastError();
    }
    if (x.small && !x.bigSmall) {
        if (const size_t lim_ = setMaxLdsOnce(reinterpret_cast<const void*>(&hxs_small_kernel<NS, VST>)); lim_ < lds) return ldsTooBig("hxs_small_kernel", lds, lim_);
        hipLaunchKernelGGL((hxs_small_kernel<NS, VST>), dim3(static_cast<unsigned>(blocks)), dim3(64 * x.nprog), lds, st, x);
        return hipGetLastError();
    }
    if (const size_t lim_ = setMaxLdsOnce(reinterpret_cast<const void*>(&hxs_kernel<NS, VST>)); lim_ < lds) return ldsTooBig("hxs_kernel", lds, lim_);
    hipLaunchKernelGGL((hxs_kernel<NS, VST>), dim3(static_cast<unsigned>(blocks)), dim3(64 * (x.nprog + kHxsLoaders)), lds, st, x);
    return hipGetLastError();
}

#define GAR_HXS_FOR4(M, NS) M(NS, 0) M(NS, 1) M(NS, 2) M(NS, 3) M(NS, 4)
#if GAR_HXS_QUICK  // development A/B builds (tools/hxs_variant.sh): only the BASELINE plans' NS = 9, 10
#define GAR_HXS_FOR_LO(M) GAR_HXS_FOR4(M, 9)
#define GAR_HXS_FOR_HI(M) GAR_HXS_FOR4(M, 10)
#else
#define GAR_HXS_FOR_LO(M) GAR_HXS_FOR4(M, 1) GAR_HXS_FOR4(M, 2) GAR_HXS_FOR4(M, 3) GAR_HXS_FOR4(M, 4) GAR_HXS_FOR4(M, 5)
#define GAR_HXS_FOR_HI(M) GAR_HXS_FOR4(M, 6) GAR_HXS_FOR4(M, 7) GAR_HXS_FOR4(M, 8) GAR_HXS_FOR4(M, 9) GAR_HXS_FOR4(M, 10)
#endif
#define GAR_HXS_FOR_ALL(M) GAR_HXS_FOR_LO(M) GAR_HXS_FOR_HI(M)
#define GAR_HXS_INST(NS, V) template hipError_t hxsLaunch<NS, V>(const HxsArgs&, size_t, int64_t, hipStream_t);

}  // namespace gar
