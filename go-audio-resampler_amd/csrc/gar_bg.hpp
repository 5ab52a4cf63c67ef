// gar_bg.hpp -- the banded-GEMM MFMA FIR kernel template (included by the
// per-dtype instantiation units gar_bg_*.hip and by gar_kernels.hip).
#pragma once
#include <hip/hip_runtime.h>

#include <algorithm>

#include "gar_kernels.hpp"
#include "gar_plan.hpp"

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
        if (s.in_pcm) return static_cast<TC>(pcmRead(s.in, e, s.in_pcm));
        return s.in_f64 ? static_cast<TC>(static_cast<const double*>(s.in)[e])
                        : static_cast<TC>(static_cast<const float*>(s.in)[e]);
    }
    return TC(0);
}

// Branch-free srcRead for a source whose input has the compute dtype (no PCM): the element's
// address is selected (history | input | a readable dummy) and loaded unconditionally, so a run
// of these issues its loads together instead of one dependent branch + load each.
template <class TC>
__device__ __forceinline__ bool srcSameType(const SrcDesc& s) {
    return !s.in_pcm && (s.in_f64 != 0) == (sizeof(TC) == 8);
}
template <class TC>
__device__ __forceinline__ TC srcReadBF(const SrcDesc& s, int64_t t, int c, bool ok, const void* dummy) {
    const int64_t h = t - s.hist_base, i = t - s.in_base;
    const bool valid = ok && t >= 0 && t < s.valid_end;
    const bool inH = valid && s.hist != nullptr && h >= 0 && h < s.hist_len;
    const bool inI = valid && !inH && s.in != nullptr && i >= 0 && i < s.in_len;
    const TC* hp = static_cast<const TC*>(s.hist) + (inH ? h * s.hist_ld + c : 0);
    const TC* ip = static_cast<const TC*>(s.in) + (inI ? i * s.in_fs + static_cast<int64_t>(c) * s.in_cs : 0);
    const TC v = *(inH ? hp : (inI ? ip : static_cast<const TC*>(dummy)));
    return (inH || inI) ? v : TC(0);
}

template <class TC>
__device__ __forceinline__ void outWrite(const OutDesc& o, int64_t idx, int c, TC v) {
    if (idx < o.o_lo || idx >= o.o_hi) return;
    const int64_t e = (idx - o.o0) * o.fs + static_cast<int64_t>(c) * o.cs;
    if (o.pcm) pcmWrite(o.out, e, o.pcm, static_cast<double>(v));
    else if (o.f64) static_cast<double*>(o.out)[e] = static_cast<double>(v);
    else static_cast<float*>(o.out)[e] = static_cast<float>(v);
}

// ---- non-finite samples on the plain MFMA programs ---------------------------------------------
// The reference multiplies only the real taps of an output's window (dft_stage.go:259 / :531,
// polyphase_stage.go:288), so an Inf / NaN sample makes exactly the outputs whose real window holds
// it non-finite.  The MFMA programs also multiply the zero-padded taps of a row block's band, and
// 0 * Inf = NaN.  So every kernel here stages a non-finite sample as 0 -- each output then carries the
// value its band gives with that sample zero, whatever the call boundaries, so chunked == one-shot
// bit for bit -- and records where it was; after the item's stores, the outputs whose REAL window
// holds a non-finite sample are recomputed over their real taps in f64 in the reference's order
// (bgNfFixOne: two stages for DFT x2 (*) polyphase composites, as hxsExact does for the split-f16
// kernels), which gives the reference's NaN / +-Inf for each of them and touches nothing else.
__device__ __forceinline__ bool bgFinite(double v) { return __builtin_isfinite(v); }
__device__ __forceinline__ bool bgFinite(float v) { return __builtin_isfinite(v); }

// The bg kernels' arguments as ONE kernel argument, so the rare non-finite path can read them
// through the kernarg segment pointer (bgCold) at the point of use: as plain arguments the
// compiler loads every field that path touches into SGPRs at kernel entry, where they spill
// (v_writelane / v_readlane in the hot loops; measured r06: cfg5 calls +25 %).
// (GAR_BG_NF_ATTR: the rare path as out-of-line calls by default; A/B builds __forceinline__)
#ifndef GAR_BG_NF_ATTR
#define GAR_BG_NF_ATTR __noinline__
#endif
// A struct in the kernarg segment (address space 4) copied out at the point of use.
template <class T>
__device__ __forceinline__ T kload(const __attribute__((address_space(4))) T* p) {
    T v;
    __builtin_memcpy(&v, (const T*)p, sizeof(T));
    return v;
}
struct BgArgs;
typedef const __attribute__((address_space(4))) BgArgs* BgArgsP;
__device__ __forceinline__ BgArgsP bgCold() {
    uint64_t v = reinterpret_cast<uint64_t>(__builtin_amdgcn_kernarg_segment_ptr());
    asm volatile("" : "+s"(v));  // opaque: no field of it is hoisted into the hot path
    return reinterpret_cast<BgArgsP>(v);
}

// Output (a, r) of channel c: recomputed and stored when its real window holds a non-finite sample.
template <class TC>
__device__ GAR_BG_NF_ATTR void bgNfFixOne(BgArgsP ka, int64_t a, int r, int c);

// The outputs (a0 + i, r), i < na, r0 <= r < r1, of channel c whose real window (rows i*Qc + off[r]
// .. + len[r] relative to input a0*Qc) meets the rows [lo, hi] where non-finite samples were staged;
// thread tid of nth.
template <class TC>
__device__ GAR_BG_NF_ATTR void bgNfFixRange(BgArgsP ka, int64_t a0, int na, int r0, int r1, int c, int lo, int hi, int tid,
                                          int nth);

// ---------------------------------------------------------------------------
// Banded GEMM.  Geometry (host computed in launchBg):
//   macro period a covers outputs [a*Pc, (a+1)*Pc) and reads inputs starting
//   at a*Qc; a column = (channel c, chunk of G consecutive macro periods);
//   the workgroup owns 16*ncg columns and stages each column's window of
//   W = Kc + (G-1)*Qc inputs in LDS as [row][16 columns] (the 16x4
//   B-fragment read is 64 consecutive dwords: bank-conflict free).  The
//   zero-padded A steps read up to Wl = Kread + (G-1)*Qc >= W rows; rows
//   [W, Wl) are filled with finite data (A is 0 there, but 0*NaN = NaN).
//   Wave (cg, wt) runs wave programs wt, wt+nwt, ... (gar_plan.hpp BgProg).
// ---------------------------------------------------------------------------
// Development build (-DGAR_BG_DEV=1, GAR_BG_PROF=1): s_memtime phase stamps of the small f64
// launches (bg_rt_kernel / bg_rb_kernel) summed into BgGrid::prof and printed at exit.
#ifndef GAR_BG_DEV
#define GAR_BG_DEV 0
#endif
constexpr bool kBgDev = GAR_BG_DEV;
constexpr size_t kBgStaticLds = 64;  // bg_kernel's static LDS (nfFlag), rounded up
constexpr int kBgProfWords = 64;

struct BgGrid {
    int Pc, Qc, Kc, W, Wl, Ws, G;
    int64_t a_lo;
    int nchunk, ncols, nblocks;
    int C, nprog, kch, nwt, ncg, nred, nslots, parity;
    int dbg;  // development timing knob (GAR_BG_DBG): 1 skip tile DMA after the first, 2 skip stores
    int vst;  // f32 epilogue: 0 scalar, 1 channel-contiguous (fs == 1), 2 stereo interleaved (C == 2, fs == 2, cs == 1)
    int rbMode;  // small launch of a row-block-aligned plan: bg_rb_kernel (G = 1)
    // bg_rb_kernel: program ranges and first input rows passed by value (kernarg), so a wave issues
    // its A and B loads without first loading its program from the tables
    int rbStart[kBgRbKMaxRb + 1];
    int rbK0[kBgRbKMaxProg];
    void* hdst;       // folded history keep (HistCopy): hdst[(t - ht0) * C + c] = src(t, c), t < ht0 + hn
    int64_t ht0, hn;
    unsigned long long* prof;  // development stamps (kBgDev), else null
};

// Development: phase stamps of waves 0 and 1 of a workgroup's first item (words base + 8 wt + k:
// k = 0..5 phase cycles, 6 count) and the workgroup's life (base + 16: count, life sum, first entry,
// last exit, last entry; s_memrealtime ticks of 10 ns).
struct BgStamps {
    unsigned long long t[7];
    unsigned long long r0;
    int k;
    bool on;
    __device__ BgStamps(const BgGrid& g, bool first) : k(0), on(kBgDev && g.prof && first && (threadIdx.x & 63) == 0 && threadIdx.x < 128) {
        if (on) { r0 = __builtin_amdgcn_s_memrealtime(); t[k++] = __builtin_amdgcn_s_memtime(); }
    }
    __device__ void mark() { if (kBgDev && on && k < 7) t[k++] = __builtin_amdgcn_s_memtime(); }
    __device__ void done(const BgGrid& g, int base) {
        if (!(kBgDev && on)) return;
        __builtin_amdgcn_s_waitcnt(0);
        mark();
        const int wt = threadIdx.x >> 6;
        for (int i = 1; i < k; ++i) atomicAdd(g.prof + base + 8 * wt + i - 1, t[i] - t[i - 1]);
        atomicAdd(g.prof + base + 8 * wt + 6, 1ull);
        if (wt == 0) {
            const unsigned long long r1 = __builtin_amdgcn_s_memrealtime();
            atomicAdd(g.prof + base + 16, 1ull);
            atomicAdd(g.prof + base + 17, r1 - r0);
            atomicMin(g.prof + base + 18, r0);
            atomicMax(g.prof + base + 19, r1);
            atomicMax(g.prof + base + 20, r0);
        }
    }
};

struct BgArgs {
    BgDev p;
    SrcDesc src;
    OutDesc od;
    BgGrid g;
};

template <class TC>
__device__ GAR_BG_NF_ATTR void bgNfFixOne(BgArgsP ka, int64_t a, int r, int c) {
    const BgDev p = kload(&ka->p);
    const SrcDesc src = kload(&ka->src);
    const OutDesc od = kload(&ka->od);
    const int64_t o = a * p.Pc + r;
    if (o < od.o_lo || o >= od.o_hi) return;
    const int* xi = p.xInfo;
    const int64_t t = a * p.Qc + xi[r];
    const int len = xi[p.Pc + r];
    const double* row = p.xRows + static_cast<size_t>(r) * p.xRowMax;
    double s = 0.0, z = 0.0;
    for (int k = 0; k < len; ++k) {
        const double v = static_cast<double>(srcRead<TC>(src, t + k, c));
        s += row[k] * v;
        z += v * 0.0;
    }
    if (z == z) return;  // the real window is finite: the MFMA value stands
    if (p.xTwoStage) {   // u = DFT x2 of the window, then the polyphase row (dft_stage.go:259, polyphase_stage.go:288)
        const int ph = xi[2 * p.Pc + r], par = xi[3 * p.Pc + r], T1 = p.xT1, T2 = p.xT2;
        const double* pa = p.xPolyA + static_cast<size_t>(ph) * T2;
        double y = 0.0;
        for (int k2 = 0; k2 < T2; ++k2) {
            const int q = par + k2;
            const double* cq = p.xDftC + static_cast<size_t>(q & 1) * T1;
            double u = 0.0;
            for (int k1 = 0; k1 < T1; ++k1) u += cq[k1] * static_cast<double>(srcRead<TC>(src, t + (q >> 1) + k1, c));
            y += pa[k2] * u;
        }
        s = y;
    }
    outWrite<TC>(od, o, c, static_cast<TC>(s));
}

template <class TC>
__device__ GAR_BG_NF_ATTR void bgNfFixRange(BgArgsP ka, int64_t a0, int na, int r0, int r1, int c, int lo, int hi, int tid,
                                          int nth) {
    const int Qc = ka->p.Qc, Pc = ka->p.Pc;
    const int* xi = ka->p.xInfo;
    const int nr = r1 - r0;
    for (int idx = tid; idx < na * nr; idx += nth) {
        const int i = idx / nr, r = r0 + (idx - i * nr);
        const int w0 = i * Qc + xi[r], w1 = w0 + xi[Pc + r];
        if (w1 <= lo || w0 > hi) continue;
        bgNfFixOne<TC>(ka, a0 + i, r, c);
    }
}

// f32 epilogue of one 16x16 accumulator: lane holds rows r0..r0+3 (r0 =
// rb*16 + 4*(lane>>4)) of column (chunk, c).  vst 1: the four rows are
// contiguous -> one 16-B store.  vst 2: lanes n, n^1 hold channels 0/1 of the
// same chunk; they swap halves so each lane stores two whole stereo frames
// (16 B).  Falls back to checked scalar stores at range edges / misalignment.
__device__ __forceinline__ void storeRows4(const OutDesc& o, const BgGrid& g, int64_t a, int r0, int c, bool colOk,
                                           f32x4 v, int lane) {
    if (g.vst == 2) {
        const bool even = (lane & 1) == 0;
        const float s0 = even ? v[2] : v[0], s1 = even ? v[3] : v[1];
        const float q0 = __shfl_xor(s0, 1), q1 = __shfl_xor(s1, 1);
        const int rr = even ? r0 : r0 + 2;  // first frame this lane stores
        f32x4 w;
        if (even) { w[0] = v[0]; w[1] = q0; w[2] = v[1]; w[3] = q1; }
        else      { w[0] = q0; w[1] = v[2]; w[2] = q1; w[3] = v[3]; }
        if (!colOk) return;
        const int64_t idx = a * g.Pc + rr;
        float* dst = static_cast<float*>(o.out) + (idx - o.o0) * 2;
        if (idx >= o.o_lo && idx + 1 < o.o_hi && rr + 1 < g.Pc && (reinterpret_cast<uintptr_t>(dst) & 15) == 0) {
            *reinterpret_cast<f32x4*>(dst) = w;
        } else {
            if (rr < g.Pc) { outWrite<float>(o, idx, 0, w[0]); outWrite<float>(o, idx, 1, w[1]); }
            if (rr + 1 < g.Pc) { outWrite<float>(o, idx + 1, 0, w[2]); outWrite<float>(o, idx + 1, 1, w[3]); }
        }
        return;
    }
    if (!colOk) return;
    const int64_t idx = a * g.Pc + r0;
    if (g.vst == 1) {
        float* dst = static_cast<float*>(o.out) + (idx - o.o0) + static_cast<int64_t>(c) * o.cs;
        if (idx >= o.o_lo && idx + 3 < o.o_hi && r0 + 3 < g.Pc && (reinterpret_cast<uintptr_t>(dst) & 15) == 0) {
            *reinterpret_cast<f32x4*>(dst) = v;
            return;
        }
    }
#pragma unroll
    for (int i = 0; i < 4; ++i)
        if (r0 + i < g.Pc) outWrite<float>(o, idx + i, c, v[i]);
}

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

// Sets a kernel's 160 KiB dynamic-LDS attribute once per (device, kernel):
// the attribute is per device, and handles on several devices may launch
// from several host threads (gar_kernels.hip).
size_t setMaxLdsOnce(const void* fn);  // raises the kernel's dynamic-LDS limit; returns the limit in force

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
    const bool inSame = !s.in_pcm && (s.in_f64 != 0) == (sizeof(TC) == 8);
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
struct TileSrc {
    ColSrc<TC> cs;
    bool allFast;
};

template <class TC>
__device__ __forceinline__ TileSrc<TC> tileSrc(const SrcDesc& src, const BgGrid& g, int b, int cg, int lane) {
    const int n = sizeof(TC) == 8 ? ((lane >> 1) & 15) : (lane & 15);
    TileSrc<TC> t;
    t.cs = colSrc<TC>(src, g, b * 16 * g.ncg + cg * 16 + n);
    t.allFast = __all(t.cs.p != nullptr);
    return t;
}

template <class TC>
__device__ __forceinline__ int tilePieces(const BgGrid& g) {
    constexpr int rowsPerPiece = sizeof(TC) == 8 ? 2 : 4;
    return (g.Wl + rowsPerPiece - 1) / rowsPerPiece;
}

// Issue this wave's DMA pieces j in [jlo, jhi) (j = wt mod nwt) of one sub-tile.
template <class TC>
__device__ __forceinline__ void loadPieces(const SrcDesc& src, const BgGrid& g, const TileSrc<TC>& ts, TC* sub,
                                           int wt, int lane, int jlo, int jhi, const void* dummy) {
    constexpr int rowsPerPiece = sizeof(TC) == 8 ? 2 : 4;
    const int n = sizeof(TC) == 8 ? ((lane >> 1) & 15) : (lane & 15);
    const int rsub = sizeof(TC) == 8 ? (lane >> 5) : (lane >> 4);
    const int half = sizeof(TC) == 8 ? (lane & 1) : 0;
    const ColSrc<TC>& cs = ts.cs;
    const bool fast = cs.p != nullptr;
    const bool allFast = ts.allFast;
    const int j0 = jlo + ((wt - jlo) % g.nwt + g.nwt) % g.nwt;
    if (!allFast && srcSameType<TC>(src)) {
        // boundary block (history seam, flush zeros): batches of 8 branch-free gathers, loads first
        constexpr int kB = 8;
        for (int jb = j0; jb < jhi; jb += kB * g.nwt) {
            TC v[kB];
#pragma unroll
            for (int u = 0; u < kB; ++u) {
                const int j = jb + u * g.nwt;
                const int kk = j * rowsPerPiece + rsub;
                const bool ok = j < jhi && kk < g.W && cs.ok && half == 0;
                v[u] = fast ? *(ok ? cs.p + kk * cs.stride : static_cast<const TC*>(dummy)) : srcReadBF<TC>(src, cs.t0 + kk, cs.c, ok, dummy);
                if (!ok) v[u] = TC(0);
            }
#pragma unroll
            for (int u = 0; u < kB; ++u) {
                const int j = jb + u * g.nwt;
                if (j < jhi && half == 0) sub[static_cast<size_t>(j) * rowsPerPiece * 16 + rsub * 16 + n] = v[u];
            }
        }
        return;
    }
    for (int j = j0; j < jhi; j += g.nwt) {
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

template <class TC>
__device__ __forceinline__ void loadTile(const SrcDesc& src, const BgGrid& g, int b, TC* sub, int cg, int wt,
                                         int lane, const void* dummy) {
    const TileSrc<TC> ts = tileSrc<TC>(src, g, b, cg, lane);
    loadPieces<TC>(src, g, ts, sub, wt, lane, 0, tilePieces<TC>(g), dummy);
}

// Generic epilogue of one accumulator (row block rb of macro period a).
template <class TC>
__device__ __forceinline__ void storeAcc(const OutDesc& o, const BgGrid& g, int64_t a, int rb, int c, bool colOk,
                                         const typename Acc<TC>::V& v, int lane) {
    if constexpr (sizeof(TC) == 4) {
        storeRows4(o, g, a, rb * 16 + 4 * (lane >> 4), c, colOk, v, lane);
    } else {
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int r = rb * 16 + Acc<TC>::row(lane, i);
            if (colOk && r < g.Pc) outWrite<TC>(o, a * g.Pc + r, c, v[i]);
        }
    }
}

// Uniform fields of one wave program (gar_plan.cpp BgPlan::progTable).
// Scalars only (no runtime-indexed arrays: those would live in scratch).
struct ProgU {
    int nseg, e1, e2;
    int rb0, rb1, rb2, u0, u1, u2, sl0, sl1, sl2, k0, k1, k2;
};

__device__ __forceinline__ ProgU progLoad(const int* t) {
    ProgU q;
    q.nseg = uni(t[0]); q.e1 = uni(t[1]); q.e2 = uni(t[2]);
    q.rb0 = uni(t[3]); q.u0 = uni(t[4]); q.sl0 = uni(t[5]); q.k0 = uni(t[6]);
    q.rb1 = uni(t[7]); q.u1 = uni(t[8]); q.sl1 = uni(t[9]); q.k1 = uni(t[10]);
    q.rb2 = uni(t[11]); q.u2 = uni(t[12]); q.sl2 = uni(t[13]); q.k2 = uni(t[14]);
    return q;
}

// Per-step selections (boundaries e1 <= e2 are wave-uniform).
// Masked arithmetic, not ?: on struct members: clang turns a select of
// member loads into one load through a selected address (struct in scratch).
__device__ __forceinline__ int sel3(int s, int e1, int e2, int v0, int v1, int v2) {
    return v0 + ((v1 - v0) & -static_cast<int>(s >= e1)) + ((v2 - v1) & -static_cast<int>(s >= e2));
}
__device__ __forceinline__ int selU(const ProgU& q, int s) { return sel3(s, q.e1, q.e2, q.u0, q.u1, q.u2); }
__device__ __forceinline__ int selK(const ProgU& q, int s) { return sel3(s, q.e1, q.e2, q.k0, q.k1, q.k2); }
__device__ __forceinline__ int segRb(const ProgU& q, int j) { return sel3(j, 1, 2, q.rb0, q.rb1, q.rb2); }
__device__ __forceinline__ int segSlot(const ProgU& q, int j) { return sel3(j, 1, 2, q.sl0, q.sl1, q.sl2); }

// Segment result: direct store (whole row block) or LDS partial slot.
template <class TC>
__device__ __forceinline__ void segStore(const ProgU& pu, int j, const typename Acc<TC>::V& r, TC* pslots,
                                         const OutDesc& od, const BgGrid& g, int64_t a, int c, bool colOk, int lane) {
    typedef typename Acc<TC>::V V;
    const int slot = segSlot(pu, j);
    if (slot < 0) {
        if (!(g.dbg & 2)) storeAcc<TC>(od, g, a, segRb(pu, j), c, colOk, r, lane);
    } else {
        *reinterpret_cast<V*>(pslots + static_cast<size_t>(slot) * 256 + lane * 4) = r;
    }
}

// B fragment of program step s: LDS tile, or global memory (GLOBAL_B).
// (global-B: a non-finite sample is read as 0 and flagged in nf; LDS tiles were cleaned by bgNfScan)
template <class TC, bool GB>
__device__ __forceinline__ TC fetchB(const TC* bp, const ProgU& pu, int s, const SrcDesc& src, int64_t tb, int c,
                                     bool colOk, bool same, const void* dummy, int& nf) {
    if constexpr (GB) {
        const TC v = colOk ? srcRead<TC>(src, tb + selK(pu, s) + 4 * s, c) : TC(0);
        const bool ok = bgFinite(v);
        nf |= ok ? 0 : 1;
        return ok ? v : TC(0);
    } else {
        return bp[selU(pu, s) + 64 * s];
    }
}

// Non-finite samples of one LDS sub-tile, before the block's barrier: the pieces this wave staged
// (j = wt mod nwt; lane l of a piece wrote dword l) are read back once they have landed, kB reads in
// flight (r06: a read -> compare -> branch chain per piece cost the f64 one-shot launches 13 %, this
// pass 7 %); a non-finite element is set to 0 and the wave flags the block (nf), which bg_kernel then
// records for bg_nf_kernel.
template <class TC>
__device__ __forceinline__ void bgNfScan(TC* sub, const BgGrid& g, int wt, int lane, int& nf) {
    constexpr int rowsPerPiece = sizeof(TC) == 8 ? 2 : 4;
    constexpr int kB = 8;
    const int np = tilePieces<TC>(g), nwt = g.nwt;
    const int e = sizeof(TC) == 8 ? (lane >> 1) : lane;  // element (row e >> 4, column e & 15) of the piece
    __builtin_amdgcn_s_waitcnt(0);  // this wave's pieces landed (LDS-DMA: vmcnt; gathered stores: lgkmcnt)
    bool bad = false;
    for (int j0 = wt; j0 < np; j0 += kB * nwt) {
        TC v[kB];
#pragma unroll
        for (int u = 0; u < kB; ++u) {
            const int j = j0 + u * nwt;
            v[u] = j < np ? sub[static_cast<size_t>(j) * rowsPerPiece * 16 + e] : TC(0);
        }
#pragma unroll
        for (int u = 0; u < kB; ++u) bad |= !bgFinite(v[u]);
    }
    if (__builtin_expect(__any(bad), 0)) {  // rare: clean this wave's pieces
        for (int j = wt; j < np; j += nwt) {
            TC* q = sub + static_cast<size_t>(j) * rowsPerPiece * 16 + e;
            if (!bgFinite(*q)) *q = TC(0);
        }
        nf = 1;
    }
}


// In-loop segment boundary: bank the running sum (stores happen after the loop).
// (e1, e2 are segment starts, always inside the program, or 1<<20 if unused)
#define GAR_SEG_CHECK(s)                                     \
    if ((s) + 1 == pu.e1) {                                  \
        r0 = acc0 + acc1; acc0 = V{0, 0, 0, 0}; acc1 = acc0; \
    } else if ((s) + 1 == pu.e2) {                           \
        r1 = acc0 + acc1; acc0 = V{0, 0, 0, 0}; acc1 = acc0; \
    }

// bg_kernel's non-finite fix list (BgDev::nfList, zeroed between launches by bg_nf_kernel):
// [0] entries, [1] overflow, then kBgNfEntry ints per entry (block, lo[64], hi[64]), then a done
// counter.  bg_kernel only records (a block that staged a non-finite sample adds its column ranges;
// the fixup code would cost the persistent loop registers), bg_nf_kernel -- launched after every
// bg_kernel launch, it returns at once when the list is empty -- recomputes the outputs.
constexpr int kBgNfEntry = 1 + 2 * 64;  // block (+ room for per-column row ranges, unused: whole blocks are checked)
constexpr int kBgNfCap = 256;
constexpr int kBgNfInts = 2 + kBgNfCap * kBgNfEntry + 1;
static_assert(kBgNfListBytes == 4 * kBgNfInts, "the host allocates kBgNfListBytes for the list");

// bg_kernel / bg_nf_kernel: the fixup of block b (every column with a recorded row range; global-B:
// every output of the block).
template <class TC, bool GLOBAL_B>
__device__ GAR_BG_NF_ATTR void bgNfFixBlock(BgArgsP ka, int b, const int* nfLo, const int* nfHi) {
    const int ncg = ka->g.ncg, ncols = ka->g.ncols, C = ka->g.C, G = ka->g.G, Pc = ka->g.Pc;
    const int64_t a_lo = ka->g.a_lo;
    for (int cl = 0; cl < 16 * ncg; ++cl) {
        const int colx = b * 16 * ncg + cl;
        if (colx >= ncols) break;
        const int lo = GLOBAL_B ? 0 : nfLo[cl], hi = GLOBAL_B ? (1 << 30) : nfHi[cl];
        if (hi < 0) continue;
        const int chx = colx / C;
        bgNfFixRange<TC>(ka, a_lo + static_cast<int64_t>(chx) * G, G, 0, Pc, colx - chx * C, lo, hi, threadIdx.x, blockDim.x);
    }
}

// Wave 0 of bg_kernel: block b into the fix list (bg_nf_kernel checks every output of it).
__device__ __forceinline__ void bgNfRecord(int* list, int b, int lane) {
    if (lane == 0) {
        const int e = atomicAdd(list, 1);
        if (e < kBgNfCap) list[2 + e * kBgNfEntry] = b;
        else list[1] = 1;  // overflow: bg_nf_kernel checks every block
    }
}

// After every bg_kernel launch: the outputs of the recorded blocks whose real window holds a
// non-finite sample get the reference's values; the list is emptied for the next launch (by the
// last workgroup out).  An empty list returns at once.
template <class TC>
__global__ __launch_bounds__(256) void bg_nf_kernel(BgArgs ka) {
    int* L = ka.p.nfList;
    const int n = *reinterpret_cast<volatile int*>(L), ovf = *reinterpret_cast<volatile int*>(L + 1);
    if (n == 0 && ovf == 0) return;
    const BgArgsP kp = bgCold();
    if (ovf) {
        for (int b = blockIdx.x; b < ka.g.nblocks; b += gridDim.x) bgNfFixBlock<TC, true>(kp, b, nullptr, nullptr);
    } else {
        for (int e = blockIdx.x; e < min(n, kBgNfCap); e += gridDim.x) bgNfFixBlock<TC, true>(kp, L[2 + e * kBgNfEntry], nullptr, nullptr);
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        __threadfence();
        if (atomicAdd(L + kBgNfInts - 1, 1) == static_cast<int>(gridDim.x) - 1) {
            L[0] = 0;
            L[1] = 0;
            L[kBgNfInts - 1] = 0;
            __threadfence();
        }
    }
}

// Prefetch-free persistent kernel: the next block's tile arrives by LDS-DMA
// (issued 1/G per macro-period iteration) while the current block computes.
template <class TC, int NS, bool GLOBAL_B, bool SINGLE>
__global__ __launch_bounds__(bgMaxThreads(sizeof(TC) == 8, NS)) void bg_kernel(BgArgs ka) {
    const BgDev& p = ka.p;
    const SrcDesc& src = ka.src;
    const OutDesc& od = ka.od;
    const BgGrid& g = ka.g;
    typedef typename Acc<TC>::V V;
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    const int subElems = g.Ws * 16;                           // one column group's sub-tile
    const int tileElems = GLOBAL_B ? 0 : subElems * g.ncg;
    TC* tiles = reinterpret_cast<TC*>(smem);                 // [2][ncg][Ws][16]
    TC* part = tiles + 2 * static_cast<size_t>(tileElems);   // partials [parity][ncg][nslots][256]
    const int partStride = g.ncg * g.nslots * 256;

    const int lane = threadIdx.x & 63;
    const int wave = threadIdx.x >> 6;
    const int cg = wave / g.nwt;
    const int wt = wave - cg * g.nwt;
    const int nloc = cg * 16 + (lane & 15);
    const int laneOff = (lane >> 4) * 16 + (lane & 15);      // B fragment (k = lane>>4, n = lane&15)
    const TC* Aimg = static_cast<const TC*>(p.A);
    const bool same = srcSameType<TC>(src);

    // a wave that staged (or, global-B, read) a non-finite sample of block b (parity it & 1) writes b + 1 here; wave 0
    // records the block for bg_nf_kernel after the next barrier (block indices are unique per
    // workgroup, so the slot needs no reset)
    __shared__ int nfFlag[2];
    if (threadIdx.x < 2) nfFlag[threadIdx.x] = -1;
    __syncthreads();
    int nfl = 0;  // this wave staged / read a non-finite sample of the current block
    int bPrev = -1, parPrev = 0;

    TC A[NS];
    if (SINGLE && wt < g.nprog) {
#pragma unroll
        for (int s = 0; s < NS; ++s) A[s] = Aimg[(static_cast<size_t>(wt) * NS + s) * 64 + lane];
    }

    int b = blockIdx.x;
    if (!GLOBAL_B && b < g.nblocks) loadTile<TC>(src, g, b, tiles + cg * subElems, cg, wt, lane, Aimg);
    int q = 0;  // macro-period iteration counter (partial-slot parity)
    for (int it = 0; b < g.nblocks; b += gridDim.x, ++it) {
        TC* tile = tiles + static_cast<size_t>(it & 1) * tileElems + cg * subElems;
        if (!GLOBAL_B) bgNfScan<TC>(tile, g, wt, lane, nfl);
        __syncthreads();  // this tile's DMA landed (vmcnt) + the other buffer is free
        if (wave == 0 && bPrev >= 0 && nfFlag[(it + 1) & 1] == bPrev + 1) bgNfRecord(p.nfList, bPrev, lane);
        const int bn = b + gridDim.x;
        const bool pre = !GLOBAL_B && bn < g.nblocks && !(g.dbg & 1);
        TC* ntile = tiles + static_cast<size_t>((it + 1) & 1) * tileElems + cg * subElems;
        TileSrc<TC> nts;
        if (pre) nts = tileSrc<TC>(src, g, bn, cg, lane);
        const int np = tilePieces<TC>(g);

        const int col = b * 16 * g.ncg + nloc;
        const bool colOk = col < g.ncols;
        const int c = colOk ? col % g.C : 0;
        const int chunk = colOk ? col / g.C : 0;

        for (int gi = 0; gi < g.G; ++gi, ++q) {
            const int64_t a = g.a_lo + static_cast<int64_t>(chunk) * g.G + gi;
            // next block's tile: 1/G of its DMA pieces per iteration, so the
            // LDS-DMA issue interleaves with the MFMA stream instead of bursting
            if (pre) loadPieces<TC>(src, g, nts, ntile, wt, lane, gi * np / g.G, (gi + 1) * np / g.G, Aimg);
            TC* pslots = part + static_cast<size_t>(g.parity ? (q & 1) : 0) * partStride +
                         static_cast<size_t>(cg) * g.nslots * 256;

            for (int pr = wt; pr < g.nprog; pr += g.nwt) {
                const ProgU pu = progLoad(p.progs + kBgProgInts * pr);
                V acc0 = {0, 0, 0, 0}, acc1 = {0, 0, 0, 0}, r0 = acc0, r1 = acc0;
                for (int ch = 0; ch < (SINGLE ? 1 : g.kch); ++ch) {
                    const int sb = SINGLE ? 0 : ch * NS;  // program step of this chunk's first step
                    if (!SINGLE) {
#pragma unroll
                        for (int s = 0; s < NS; ++s)
                            A[s] = Aimg[(static_cast<size_t>(pr) * g.kch * NS + sb + s) * 64 + lane];
                    }
                    // B reads software-pipelined 4 steps ahead; sched_barrier keeps
                    // the compiler from hoisting every ds_read.
                    // (global-B variant: window too large for LDS, B straight from L1/L2)
                    const TC* bp = tile + gi * g.Qc * 16 + laneOff;
                    const int64_t tb = a * g.Qc + (lane >> 4);
                    constexpr int PF = 4;
                    TC bA[PF], bB[PF];
#pragma unroll
                    for (int j = 0; j < PF; ++j)
                        if (j < NS) bA[j] = fetchB<TC, GLOBAL_B>(bp, pu, sb + j, src, tb, c, colOk, same, Aimg, nfl);
#pragma unroll
                    for (int s0 = 0; s0 < NS; s0 += 2 * PF) {
#pragma unroll
                        for (int j = 0; j < PF; ++j)
                            if (s0 + PF + j < NS) bB[j] = fetchB<TC, GLOBAL_B>(bp, pu, sb + s0 + PF + j, src, tb, c, colOk, same, Aimg, nfl);
                        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
                        for (int j = 0; j < PF; ++j) {
                            const int s = s0 + j;
                            if (s < NS) {
                                if (j & 1) acc1 = Acc<TC>::mfma(A[s], bA[j], acc1);
                                else acc0 = Acc<TC>::mfma(A[s], bA[j], acc0);
                                GAR_SEG_CHECK(sb + s)
                            }
                        }
                        __builtin_amdgcn_sched_barrier(0);
                        if (s0 + PF < NS) {
#pragma unroll
                            for (int j = 0; j < PF; ++j)
                                if (s0 + 2 * PF + j < NS) bA[j] = fetchB<TC, GLOBAL_B>(bp, pu, sb + s0 + 2 * PF + j, src, tb, c, colOk, same, Aimg, nfl);
                            __builtin_amdgcn_sched_barrier(0);
#pragma unroll
                            for (int j = 0; j < PF; ++j) {
                                const int s = s0 + PF + j;
                                if (s < NS) {
                                    if (j & 1) acc1 = Acc<TC>::mfma(A[s], bB[j], acc1);
                                    else acc0 = Acc<TC>::mfma(A[s], bB[j], acc0);
                                    GAR_SEG_CHECK(sb + s)
                                }
                            }
                            __builtin_amdgcn_sched_barrier(0);
                        }
                    }
                }
                const V rl = acc0 + acc1;
                segStore<TC>(pu, 0, pu.nseg > 1 ? r0 : rl, pslots, od, g, a, c, colOk, lane);
                if (pu.nseg > 1) segStore<TC>(pu, 1, pu.nseg > 2 ? r1 : rl, pslots, od, g, a, c, colOk, lane);
                if (pu.nseg > 2) segStore<TC>(pu, 2, rl, pslots, od, g, a, c, colOk, lane);
            }
            if (g.nred > 0) {
                __syncthreads();  // partial slots of this macro period written
                for (int r = wt; r < g.nred; r += g.nwt) {
                    const int* rt = p.reds + kBgRedInts * r;
                    const int rb = uni(rt[0]), n = uni(rt[1]);
                    V sum = *reinterpret_cast<const V*>(pslots + static_cast<size_t>(uni(rt[2])) * 256 + lane * 4);
                    for (int k = 1; k < n; ++k)
                        sum += *reinterpret_cast<const V*>(pslots + static_cast<size_t>(uni(rt[2 + k])) * 256 + lane * 4);
                    if (!(g.dbg & 2)) storeAcc<TC>(od, g, a, rb, c, colOk, sum, lane);
                }
                // with two slot buffers the next iteration writes the other one;
                // its barrier orders this reduction before the buffer's reuse
                if (!g.parity) __syncthreads();
            }
        }
        if (__builtin_expect(__any(nfl), 0) && lane == 0) nfFlag[it & 1] = b + 1;
        nfl = 0;
        bPrev = b;
        parPrev = it & 1;
    }
    if (bPrev >= 0) {  // the workgroup's last block
        __syncthreads();
        if (wave == 0 && nfFlag[parPrev] == bPrev + 1) bgNfRecord(p.nfList, bPrev, lane);
    }
    if (g.hn > 0) {  // history keep for the next call (launchGather's job, folded into this launch)
        const int64_t total = g.hn * g.C;
        for (int64_t i = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x; i < total;
             i += static_cast<int64_t>(gridDim.x) * blockDim.x) {
            const int64_t t = i / g.C;
            static_cast<TC*>(g.hdst)[i] = srcRead<TC>(src, g.ht0 + t, static_cast<int>(i - t * g.C));
        }
    }
}

// Small launches of row-block-aligned plans (BgPlan::rbAligned): workgroup v = (column block
// v / nrb, row block v % nrb), one macro period per column (G = 1); wave w runs program
// rbStart[rb] + w: its A fragments are loaded once, every B fragment of its K piece is fetched up
// front (one memory round trip: a direct pointer when the piece's rows lie in one buffer), the MFMAs
// accumulate exactly as in bg_kernel (acc0/acc1 by step parity), and the row block's pieces are
// summed in program order through LDS -- the persistent kernel's sums, bit for bit, so streams give
// the same output however they are chunked.  The launch is latency-bound (a 4800-frame f64 chunk
// is a few dozen tiles): many small workgroups, each one round trip deep, instead of a few
// workgroups walking every row block.
// History keep of a bg_rb_kernel launch (the `copy(history, history[consumed:])` of the stage):
// element i of the new history is copied by thread i (mod the grid) of the flattened grid, issued right after the program's A / B loads so its memory round trip overlaps theirs.
// Workgroup wg of nwg of the launch's grid.
template <class TC>
__device__ __forceinline__ void bgRbHistKeepW(const SrcDesc& src, const BgGrid& g, int wg, int nwg) {
    if (g.hn <= 0 || (g.dbg & 64)) return;
    const int64_t total = g.hn * g.C;
    for (int64_t i = static_cast<int64_t>(wg) * blockDim.x + threadIdx.x; i < total;
         i += static_cast<int64_t>(nwg) * blockDim.x) {
        const int64_t t = i / g.C;
        static_cast<TC*>(g.hdst)[i] = srcRead<TC>(src, g.ht0 + t, static_cast<int>(i - t * g.C));
    }
}
template <class TC>
__device__ __forceinline__ void bgRbHistKeep(const SrcDesc& src, const BgGrid& g) {
    bgRbHistKeepW<TC>(src, g, blockIdx.x, gridDim.x);
}

// Non-finite samples on the small launches (bg_rb_kernel, bg_rt_kernel): the hot path is the
// finite one -- the item runs as always, and only its final values are checked (a non-finite sample
// under any tap, padded or real, makes the output non-finite).  An item whose outputs hold a
// non-finite value is redone out of line: its samples staged with every non-finite one as 0 (the
// value the band gives with that sample zero, the same bits in every kernel and chunking), then the
// outputs whose REAL window holds a non-finite sample recomputed in the reference's order
// (bgNfFixOne).  Per-wave row ranges: each wave writes only its own entries.
struct BgNfRb {
    int lo[kBgRbMaxWaves][16], hi[kBgRbMaxWaves][16];
};

template <class V>
__device__ __forceinline__ bool bgAccFinite(const V& v) {
    return bgFinite(v[0]) && bgFinite(v[1]) && bgFinite(v[2]) && bgFinite(v[3]);
}

// One program of a bg_rb_kernel item (wave wt < np): A and B loaded, B's non-finite elements set to
// 0 and their rows (k0 + 4 s + lane / 16, relative to the column's a * Qc) recorded, the MFMA chain
// of bgRbItem.  Out of line: the redo of an item whose outputs were non-finite.
template <class TC, int NS>
__device__ GAR_BG_NF_ATTR typename Acc<TC>::V bgRbProgClean(BgArgsP ka, int pr, int64_t a, int c, bool colOk, int wt,
                                                            int lane, BgNfRb* nf) {
    typedef typename Acc<TC>::V V;
    const SrcDesc src = kload(&ka->src);
    const TC* Aimg = static_cast<const TC*>(ka->p.A);
    const int k0 = ka->g.rbK0[pr], Qc = ka->g.Qc;
    if (lane < 16) { nf->lo[wt][lane] = 0x7fffffff; nf->hi[wt][lane] = -1; }
    V acc0 = {0, 0, 0, 0}, acc1 = acc0;
    for (int s = 0; s < NS; ++s) {
        const int rr = k0 + 4 * s + (lane >> 4);
        TC bv = colOk ? srcRead<TC>(src, a * Qc + rr, c) : TC(0);
        if (!bgFinite(bv)) {
            bv = TC(0);
            atomicMin(&nf->lo[wt][lane & 15], rr);
            atomicMax(&nf->hi[wt][lane & 15], rr);
        }
        const TC av = Aimg[(static_cast<size_t>(pr) * NS + s) * 64 + lane];
        if (s & 1) acc1 = Acc<TC>::mfma(av, bv, acc1);
        else acc0 = Acc<TC>::mfma(av, bv, acc0);
    }
    return acc0 + acc1;
}

// Item (column block b, row block rb) of bg_rb_kernel: its outputs whose real window meets a
// recorded row range (waves < np) -- thread tid of nth.
template <class TC>
__device__ GAR_BG_NF_ATTR void bgRbFix(BgArgsP ka, int b, int rb, int np, const BgNfRb* nf, int tid, int nth) {
    const int Pc = ka->g.Pc, ncols = ka->g.ncols, C = ka->g.C;
    const int64_t a_lo = ka->g.a_lo;
    const int* xi = ka->p.xInfo;
    for (int idx = tid; idx < 256; idx += nth) {
        const int n = idx & 15, r = rb * 16 + (idx >> 4);
        const int col = b * 16 + n;
        if (r >= Pc || col >= ncols) continue;
        int lo = 0x7fffffff, hi = -1;
        for (int w = 0; w < np; ++w) { lo = min(lo, nf->lo[w][n]); hi = max(hi, nf->hi[w][n]); }
        if (hi < 0) continue;
        const int w0 = xi[r], w1 = w0 + xi[Pc + r];
        if (w1 <= lo || w0 > hi) continue;
        bgNfFixOne<TC>(ka, a_lo + col / C, r, col % C);
    }
}

// One (column block, row block) item v of a bg_rb_kernel launch.  keep: this workgroup's share
// (workgroup wg of nwg) of the history keep rides on this item.
template <class TC, int NS>
__device__ __forceinline__ void bgRbItem(const BgDev& p, const SrcDesc& src, const OutDesc& od, const BgGrid& g, int v,
                                         typename Acc<TC>::V (*slots)[64], bool keep, int wg, int nwg, BgNfRb& nf,
                                         int* nfItem) {
    typedef typename Acc<TC>::V V;
    const int lane = threadIdx.x & 63;
    const int wt = threadIdx.x >> 6;
    const TC* Aimg = static_cast<const TC*>(p.A);
    BgStamps stm(g, keep);
    const int b = v / p.nrb, rb = v - b * p.nrb;
    const int ps = g.rbStart[rb], np = g.rbStart[rb + 1] - ps;
    const int col = b * 16 + (lane & 15);
    const bool colOk = col < g.ncols;
    const int c = colOk ? col % g.C : 0;
    const int64_t a = g.a_lo + (colOk ? col / g.C : 0);  // G = 1
    V r = {0, 0, 0, 0};
    if (keep && wt >= np) bgRbHistKeepW<TC>(src, g, wg, nwg);  // waves that run no program
    if (wt < np) {
        const int pr = ps + wt;
        const int k0 = g.rbK0[pr];
        TC A[NS], B[NS];
#pragma unroll
        for (int s = 0; s < NS; ++s) A[s] = (g.dbg & 32) ? TC(s) : Aimg[(static_cast<size_t>(pr) * NS + s) * 64 + lane];
        // rows of this lane: t0 + 4 s, s < NS (the zero-A tail steps read finite rows too)
        const int64_t t0 = a * g.Qc + k0 + (lane >> 4);
        const int64_t lo = a * g.Qc + k0, hi = lo + 4 * NS;
        const TC* dp = nullptr;
        int64_t ds = 0;
        if (colOk && hi <= src.valid_end && lo >= 0 && !(g.dbg & (128 | 256))) {
            if (srcSameType<TC>(src) && src.in && lo >= src.in_base && hi <= src.in_base + src.in_len) {
                dp = static_cast<const TC*>(src.in) + (t0 - src.in_base) * src.in_fs + static_cast<int64_t>(c) * src.in_cs;
                ds = 4 * src.in_fs;
            } else if (src.hist && lo >= src.hist_base && hi <= src.hist_base + src.hist_len) {
                dp = static_cast<const TC*>(src.hist) + (t0 - src.hist_base) * src.hist_ld + c;
                ds = 4 * src.hist_ld;
            }
        }
        if (g.dbg & 16) {  // development (GAR_BG_DBG): no B loads
#pragma unroll
            for (int s = 0; s < NS; ++s) B[s] = TC(s);
        } else if (dp) {
#pragma unroll
            for (int s = 0; s < NS; ++s) B[s] = dp[s * ds];
        } else if (srcSameType<TC>(src) && !(g.dbg & 256)) {
            // window across the history seam / past the input: branch-free gathers, so the NS
            // loads issue together (a branchy srcRead per step waits out each round trip)
#pragma unroll
            for (int s = 0; s < NS; ++s) B[s] = srcReadBF<TC>(src, t0 + 4 * s, c, colOk, Aimg);
        } else {
#pragma unroll
            for (int s = 0; s < NS; ++s) B[s] = colOk ? srcRead<TC>(src, t0 + 4 * s, c) : TC(0);
        }
        if (keep) bgRbHistKeepW<TC>(src, g, wg, nwg);  // its round trip beside A / B's
        stm.mark();  // A / B / history loads issued
        if (kBgDev && stm.on) { __builtin_amdgcn_s_waitcnt(0); stm.mark(); }  // ... and landed
        // every A / B load issued before the first MFMA: one memory round trip for the program
        // (left alone, the scheduler interleaves load -> wait -> MFMA, NS round trips deep)
        __builtin_amdgcn_sched_barrier(0);
        V acc0 = {0, 0, 0, 0}, acc1 = acc0;
#pragma unroll
        for (int s = 0; s < NS; ++s) {
            if (s & 1) acc1 = Acc<TC>::mfma(A[s], B[s], acc1);
            else acc0 = Acc<TC>::mfma(A[s], B[s], acc0);
        }
        r = acc0 + acc1;
        if (np > 1) slots[wt][lane] = r;
        if (kBgDev && stm.on) { __builtin_amdgcn_s_waitcnt(0); stm.mark(); }  // MFMA chain done
    }
    if (np > 1) {
        __syncthreads();
        stm.mark();  // reduction barrier
        if (wt == 0) {
            V sum = slots[0][lane];
            for (int k = 1; k < np; ++k) sum += slots[k][lane];
            if (!(g.dbg & 2)) storeAcc<TC>(od, g, a, rb, c, colOk, sum, lane);
            if (__builtin_expect(__any(!bgAccFinite(sum)), 0) && lane == 0) *nfItem = v + 1;
        }
        __syncthreads();  // slots free for the next (column block, row block); wave 0's stores done
        if (__builtin_expect(*nfItem == v + 1, 0)) {  // uniform: redo the item with the non-finite samples as 0
            const BgArgsP ka = bgCold();
            if (wt < np) slots[wt][lane] = bgRbProgClean<TC, NS>(ka, ps + wt, a, c, colOk, wt, lane, &nf);
            __syncthreads();
            if (wt == 0) {
                V sum = slots[0][lane];
                for (int k = 1; k < np; ++k) sum += slots[k][lane];
                storeAcc<TC>(od, g, a, rb, c, colOk, sum, lane);
            }
            __syncthreads();  // the clean outputs stored, every wave's ranges recorded
            bgRbFix<TC>(ka, b, rb, np, &nf, threadIdx.x, blockDim.x);
            __syncthreads();  // slots and ranges free
        }
    } else if (wt == 0) {
        if (!(g.dbg & 2)) storeAcc<TC>(od, g, a, rb, c, colOk, r, lane);
        if (__builtin_expect(__any(!bgAccFinite(r)), 0)) {  // the item's only wave redoes it alone
            const BgArgsP ka = bgCold();
            const V rc = bgRbProgClean<TC, NS>(ka, ps, a, c, colOk, 0, lane, &nf);
            __builtin_amdgcn_s_waitcnt(0);  // the first stores landed before the clean ones
            storeAcc<TC>(od, g, a, rb, c, colOk, rc, lane);
            __builtin_amdgcn_s_waitcnt(0);  // its stores landed before the fixup overwrites some
            bgRbFix<TC>(ka, b, rb, 1, &nf, lane, 64);
        }
    }
    stm.done(g, 32);
}

// XCD-grouped item order of the small launches: workgroup slot bb runs item (group, member) with
// group = 8 (bb / 8 / M) + bb % 8 and member = (bb / 8) % M, so the M items that read the same
// input lines (the row blocks of one column block; the row blocks x channels of one time block) run
// on workgroup slots of one residue mod 8, i.e. on one XCD under the round-robin dispatch, and share
// its L2 (cfg5 decimator: each 64-B line of the 8-channel stream was fetched by 8 XCDs).  The grid
// is 8 M ceil(ngroups / 8) slots (a multiple of 8 also when capped); slots past the last group idle.
__host__ __device__ inline int64_t bgXcdSlots(int64_t ngroups, int64_t M) { return 8 * M * ((ngroups + 7) / 8); }
__device__ __forceinline__ bool bgXcdItem(int64_t bb, int M, int ngroups, int& group, int& member) {
    const int64_t rest = bb >> 3;
    member = static_cast<int>(rest % M);
    group = static_cast<int>((rest / M) * 8 + (bb & 7));
    return group < ngroups;
}

template <class TC, int NS>
__global__ __launch_bounds__(64 * kBgRbMaxWaves) void bg_rb_kernel(BgArgs ka) {
    const BgDev& p = ka.p;
    const SrcDesc& src = ka.src;
    const OutDesc& od = ka.od;
    const BgGrid& g = ka.g;
    typedef typename Acc<TC>::V V;
    __shared__ V slots[kBgRbMaxWaves][64];
    __shared__ BgNfRb nf;
    __shared__ int nfItem;  // item + 1 whose outputs hold a non-finite value (written by wave 0 only)
    if (threadIdx.x == 0) nfItem = -1;
    const int64_t total = bgXcdSlots(g.nblocks, p.nrb);
    bool kept = false;
    for (int64_t bb = blockIdx.x; bb < total; bb += gridDim.x) {  // uniform per workgroup
        int b, rb;
        if (!bgXcdItem(bb, p.nrb, g.nblocks, b, rb)) continue;
        bgRbItem<TC, NS>(p, src, od, g, b * p.nrb + rb, slots, !kept, blockIdx.x, gridDim.x, nf, &nfItem);
        kept = true;
    }
    if (!kept) bgRbHistKeep<TC>(src, g);  // a workgroup without an item
}

// Small launches of row-block-aligned plans, time-major (default; bg_rb_kernel is the GAR_BG_RT=0
// fallback): workgroup v = (row block rb, channel c, chunk block kb) -- the 16 columns are 16
// consecutive macro periods of ONE channel, so their windows overlap: the union window (15*Qc +
// Kread rows of channel c) is staged once in LDS by all waves (one memory round trip of ~4 loads
// per thread instead of every wave gathering NS rows of 16 columns), then wave w runs program
// rbStart[rb] + w with B read from LDS.  LDS rows are padded by kRtPad(Qc) every Qc rows so the 16
// columns of a B read (Qc rows apart) fall on distinct bank pairs.  Same A, same B values, same
// MFMA order and program-order reduction as bg_kernel / bg_rb_kernel: the same bits.
__host__ __device__ constexpr int kRtPad(int Qc) { return ((2 - Qc) % 32 + 32) % 32; }  // (Qc + pad) % 32 == 2
inline size_t bgRtLds(int Qc, int Kread, int nprog, size_t esz) {
    const int nrow = 15 * Qc + Kread;
    const size_t win = (static_cast<size_t>(nrow) + static_cast<size_t>(kRtPad(Qc)) * (nrow / Qc + 1)) * esz;
    return (win + 15) / 16 * 16 + static_cast<size_t>(nprog) * 64 * 4 * esz;
}

// Redo of a bg_rt_kernel item whose outputs hold a non-finite value (all waves; the window is still
// in LDS): its non-finite samples set to 0 and their rows recorded (nf[0] lo, nf[1] hi), the programs
// rerun from the clean window, the sums stored, then the outputs whose real window holds a non-finite
// sample recomputed (bgNfFixRange).
template <class TC, int NS>
__device__ GAR_BG_NF_ATTR void bgRtRedo(BgArgsP ka, int v, unsigned char* smem, int* nf) {
    typedef typename Acc<TC>::V V;
    const int lane = threadIdx.x & 63, wt = threadIdx.x >> 6;
    const int Qc = ka->g.Qc, pad = kRtPad(Qc), nrb = ka->p.nrb, Pc = ka->g.Pc, nchunk = ka->g.nchunk;
    const int nrow = 15 * Qc + ka->g.Wl;
    const int nphys = nrow + pad * (nrow / Qc + 1);
    TC* win = reinterpret_cast<TC*>(smem);
    V* slots = reinterpret_cast<V*>(smem + (static_cast<size_t>(nphys) * sizeof(TC) + 15) / 16 * 16);
    const int nkb = (nchunk + 15) / 16;
    const int rb = v % nrb, cb = v / nrb;
    const int c = cb / nkb, kb = cb - c * nkb;
    const int ps = ka->g.rbStart[rb], np = ka->g.rbStart[rb + 1] - ps;
    if (threadIdx.x == 0) { nf[0] = 0x7fffffff; nf[1] = -1; }
    __syncthreads();
    for (int r = threadIdx.x; r < nrow; r += blockDim.x) {
        TC* e = win + r + pad * (r / Qc);
        if (!bgFinite(*e)) { *e = TC(0); atomicMin(nf, r); atomicMax(nf + 1, r); }
    }
    __syncthreads();  // clean window, ranges final
    const int n = lane & 15, kq = lane >> 4;
    const int64_t a = ka->g.a_lo + 16 * static_cast<int64_t>(kb) + n;
    const bool colOk = 16 * kb + n < nchunk;
    const OutDesc od = kload(&ka->od);
    BgGrid g{};  // the fields storeAcc reads
    g.Pc = Pc;
    g.vst = ka->g.vst;
    V r = {0, 0, 0, 0};
    if (wt < np) {
        const int pr = ps + wt, k0 = ka->g.rbK0[pr];
        const TC* Aimg = static_cast<const TC*>(ka->p.A);
        const int x0 = k0 + kq;
        int q = x0 / Qc, rem = x0 - q * Qc;
        const int nb = n * (Qc + pad);
        V acc0 = {0, 0, 0, 0}, acc1 = acc0;
        for (int s = 0; s < NS; ++s) {
            const TC bv = win[nb + q * (Qc + pad) + rem];
            rem += 4;
            while (rem >= Qc) { rem -= Qc; ++q; }
            const TC av = Aimg[(static_cast<size_t>(pr) * NS + s) * 64 + lane];
            if (s & 1) acc1 = Acc<TC>::mfma(av, bv, acc1);
            else acc0 = Acc<TC>::mfma(av, bv, acc0);
        }
        r = acc0 + acc1;
        if (np > 1) slots[wt * 64 + lane] = r;
    }
    __syncthreads();
    if (wt == 0) {
        V sum = r;
        if (np > 1) {
            sum = slots[lane];
            for (int k = 1; k < np; ++k) sum += slots[k * 64 + lane];
        }
        storeAcc<TC>(od, g, a, rb, c, colOk, sum, lane);
    }
    __syncthreads();  // the clean outputs stored
    bgNfFixRange<TC>(ka, ka->g.a_lo + 16 * static_cast<int64_t>(kb), 16, rb * 16, min(rb * 16 + 16, Pc), c, nf[0], nf[1],
                     threadIdx.x, blockDim.x);
    __syncthreads();  // window, slots and ranges free
}

// One (row block, channel, chunk block) item v of a bg_rt_kernel launch (smem: the window + slots).
template <class TC, int NS>
__device__ __forceinline__ void bgRtItem(const BgDev& p, const SrcDesc& src, const OutDesc& od, const BgGrid& g, int v,
                                         unsigned char* smem, bool keep, int wg, int nwg, int* nfItem, int* nf) {
    typedef typename Acc<TC>::V V;
    const int lane = threadIdx.x & 63;
    const int wt = threadIdx.x >> 6;
    const TC* Aimg = static_cast<const TC*>(p.A);
    const int Qc = g.Qc, pad = kRtPad(Qc);
    const int nrow = 15 * Qc + g.Wl;  // union window of 16 macro periods (Wl = Kread)
    const int nphys = nrow + pad * (nrow / Qc + 1);
    TC* win = reinterpret_cast<TC*>(smem);
    V* slots = reinterpret_cast<V*>(smem + (static_cast<size_t>(nphys) * sizeof(TC) + 15) / 16 * 16);
    const int nkb = (g.nchunk + 15) / 16;
    const bool same = srcSameType<TC>(src);
    BgStamps stm(g, keep);
    const int rb = v % p.nrb, cb = v / p.nrb;
    const int c = cb / nkb, kb = cb - c * nkb;
    const int ps = g.rbStart[rb], np = g.rbStart[rb + 1] - ps;
    TC A[NS];
    int k0 = 0;
    if (wt < np) {  // A lands while the window is staged
        const int pr = ps + wt;
        k0 = g.rbK0[pr];
#pragma unroll
        for (int s = 0; s < NS; ++s) A[s] = (g.dbg & 32) ? TC(s) : Aimg[(static_cast<size_t>(pr) * NS + s) * 64 + lane];
    }
    // stage rows [0, nrow) of channel c from T: batches of kRtB loads per thread in flight
    const int64_t T = (g.a_lo + 16 * static_cast<int64_t>(kb)) * Qc;
    constexpr int kRtB = 8;  // loads per thread in flight: the decimator's ~1.7k-row window in one round trip
    for (int r0 = threadIdx.x; r0 < nrow; r0 += kRtB * blockDim.x) {
        TC vv[kRtB];
#pragma unroll
        for (int u = 0; u < kRtB; ++u) {
            const int r = r0 + u * blockDim.x;
            vv[u] = (g.dbg & 16) ? TC(r) : (same ? srcReadBF<TC>(src, T + r, c, r < nrow, Aimg) : (r < nrow ? srcRead<TC>(src, T + r, c) : TC(0)));
        }
#pragma unroll
        for (int u = 0; u < kRtB; ++u) {
            const int r = r0 + u * blockDim.x;
            if (r < nrow) win[r + pad * (r / Qc)] = vv[u];
        }
    }
    if (keep) bgRbHistKeepW<TC>(src, g, wg, nwg);  // its round trip beside the staging
    stm.mark();  // A issued, window staged by this wave
    __syncthreads();  // window staged
    stm.mark();
    const int n = lane & 15, kq = lane >> 4;
    const int64_t a = g.a_lo + 16 * static_cast<int64_t>(kb) + n;
    const bool colOk = 16 * kb + n < g.nchunk;
    V r = {0, 0, 0, 0};
    if (wt < np) {
        // row n*Qc + k0 + 4s + kq -> LDS index n*(Qc+pad) + x + pad*(x / Qc), x = k0 + 4s + kq
        const int x0 = k0 + kq;
        int q = x0 / Qc, rem = x0 - q * Qc;
        const int nb = n * (Qc + pad);
        TC B[NS];
#pragma unroll
        for (int s = 0; s < NS; ++s) {
            B[s] = win[nb + q * (Qc + pad) + rem];
            rem += 4;
            // a step of 4 rows spans several macro periods when Qc < 4 (integer upsamplers, Qc = 1:
            // r05 sweep, 11025 -> 176400 engine seam in 4096-frame calls)
            while (rem >= Qc) { rem -= Qc; ++q; }
        }
        V acc0 = {0, 0, 0, 0}, acc1 = acc0;
#pragma unroll
        for (int s = 0; s < NS; ++s) {
            if (s & 1) acc1 = Acc<TC>::mfma(A[s], B[s], acc1);
            else acc0 = Acc<TC>::mfma(A[s], B[s], acc0);
        }
        r = acc0 + acc1;
        if (np > 1) slots[wt * 64 + lane] = r;
        if (kBgDev && stm.on) { __builtin_amdgcn_s_waitcnt(0); stm.mark(); }  // B reads + MFMA chain done
    }
    if (np > 1) {
        __syncthreads();
        stm.mark();  // reduction barrier
        if (wt == 0) {
            V sum = slots[lane];
            for (int k = 1; k < np; ++k) sum += slots[k * 64 + lane];
            if (!(g.dbg & 2)) storeAcc<TC>(od, g, a, rb, c, colOk, sum, lane);
            if (__builtin_expect(__any(!bgAccFinite(sum)), 0) && lane == 0) *nfItem = v + 1;
        }
    } else if (wt == 0) {
        if (!(g.dbg & 2)) storeAcc<TC>(od, g, a, rb, c, colOk, r, lane);
        if (__builtin_expect(__any(!bgAccFinite(r)), 0) && lane == 0) *nfItem = v + 1;
    }
    __syncthreads();  // window and slots free for the next (row block, channel, chunk block)
    if (__builtin_expect(*nfItem == v + 1, 0)) bgRtRedo<TC, NS>(bgCold(), v, smem, nf);  // uniform
    stm.done(g, 0);
}

template <class TC, int NS>
__global__ __launch_bounds__(64 * kBgRbMaxWaves) void bg_rt_kernel(BgArgs ka) {
    const BgDev& p = ka.p;
    const SrcDesc& src = ka.src;
    const OutDesc& od = ka.od;
    const BgGrid& g = ka.g;
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    __shared__ int nfItem;  // item + 1 whose outputs hold a non-finite value (written by wave 0 only)
    __shared__ int nf[2];   // its rows of non-finite samples (bgRtRedo)
    if (threadIdx.x == 0) nfItem = -1;
    const int nkb = (g.nchunk + 15) / 16;
    const int M = p.nrb * g.C;  // items of one time block: row blocks x channels
    const int64_t total = bgXcdSlots(nkb, M);
    bool kept = false;
    for (int64_t bb = blockIdx.x; bb < total; bb += gridDim.x) {  // uniform per workgroup
        int kb, m;
        if (!bgXcdItem(bb, M, nkb, kb, m)) continue;
        const int rb = m % p.nrb, c = m / p.nrb;
        bgRtItem<TC, NS>(p, src, od, g, rb + p.nrb * (c * nkb + kb), smem, !kept, blockIdx.x, gridDim.x, &nfItem, nf);
        kept = true;
    }
    // every thread of a workgroup with an item copied its share in its first item (no
    // second pass); a workgroup without one copies it here
    if (!kept) bgRbHistKeep<TC>(src, g);
}

template <class TC, int NS>
static hipError_t bgDispatch(const BgDev& p, const SrcDesc& src, const OutDesc& od, const BgGrid& g, int threads,
                             size_t lds, int64_t blocks, hipStream_t st, bool globalB) {
    setMaxLdsOnce(reinterpret_cast<const void*>(&bg_kernel<TC, NS, false, true>));
    setMaxLdsOnce(reinterpret_cast<const void*>(&bg_kernel<TC, NS, false, false>));
    setMaxLdsOnce(reinterpret_cast<const void*>(&bg_kernel<TC, NS, true, true>));
    setMaxLdsOnce(reinterpret_cast<const void*>(&bg_kernel<TC, NS, true, false>));
    const dim3 gd(static_cast<unsigned>(blocks)), bd(threads);
    const BgArgs ka{p, src, od, g};
    if (g.rbMode) {
        if constexpr (sizeof(TC) == 8 && NS <= kBgRbMaxSteps) {
            if (threads > 64 * kBgRbMaxWaves) return hipErrorInvalidConfiguration;
            if (g.rbMode == 2) {  // time-major, LDS-staged windows
                if (const size_t lim_ = setMaxLdsOnce(reinterpret_cast<const void*>(&bg_rt_kernel<TC, NS>)); lim_ < lds) return ldsTooBig("bg_rt_kernel", lds, lim_);
                hipLaunchKernelGGL((bg_rt_kernel<TC, NS>), gd, bd, lds, st, ka);
            } else {
                hipLaunchKernelGGL((bg_rb_kernel<TC, NS>), gd, bd, 0, st, ka);
            }
            return hipGetLastError();
        }
        return hipErrorNotSupported;
    }
    if (threads > bgMaxThreads(sizeof(TC) == 8, NS)) return hipErrorInvalidConfiguration;
    const bool single = g.kch == 1 && g.nprog <= g.nwt;  // one program per wave: A loaded once
    if (globalB) {
        if (single) hipLaunchKernelGGL((bg_kernel<TC, NS, true, true>), gd, bd, lds, st, ka);
        else hipLaunchKernelGGL((bg_kernel<TC, NS, true, false>), gd, bd, lds, st, ka);
    } else {
        if (single) hipLaunchKernelGGL((bg_kernel<TC, NS, false, true>), gd, bd, lds, st, ka);
        else hipLaunchKernelGGL((bg_kernel<TC, NS, false, false>), gd, bd, lds, st, ka);
    }
    return hipGetLastError();
}


// Launch geometry + dispatch into the instantiation units.
hipError_t bgLaunchF64(int NS, const BgDev& p, const SrcDesc& src, const OutDesc& od, const BgGrid& g, int threads,
                       size_t lds, int64_t blocks, hipStream_t st, bool globalB);

}  // namespace gar
