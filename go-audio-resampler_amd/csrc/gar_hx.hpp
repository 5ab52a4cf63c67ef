// gar_hx.hpp -- split-f16 banded-GEMM FIR kernel for f32 compute (gfx950).
//
// Same periodic banded GEMM as bg_kernel (gar_bg.hpp), but every product
// a*x is formed as ah*xh + ah*xl + al*xh on v_mfma_f32_16x16x32_f16 (f32
// accumulation), where x*2^kHxXs = xh + xl and a*2^ea = ah + al are f16
// pairs (22 significant bits each; ea per plan, kHxXs a constant).  The
// dropped al*xl term and the representation errors are ~2^-22 relative,
// below the f32 accumulation error of the exact-f32 MFMA path, and the f16
// MFMA retires 16x the MACs per cycle of the f32 one.  Because the x scale
// is a constant, an output's bits depend only on its own window and its
// absolute position: chunked and one-shot streams agree bit for bit
// (processinto_test.go:258-308).
//
// One block = 16 columns (channel x chunk of G macro periods) staged in LDS
// as f16 hi/lo images (double-buffered).  Every wave of the workgroup both
// computes and stages: while it runs its MFMA program over block b it
// converts block b+grid's raw rows (loaded into registers during the
// previous block) into the other image buffer and issues block b+2*grid's
// loads; one barrier per block.  Row-block mode (RB): wave w owns row block
// w over its whole band (A in registers, no partial sums).  Segmented mode:
// balanced wave programs of up to 3 row-block segments with LDS partial-sum
// reduction (as bg_kernel).  Launch edges (history seam, partial periods,
// flush zeros, f64 input) are ordinary blocks whose windows are gathered.
// Elements with |x| >= kHxLoud (or Inf/NaN) are staged as zero and the
// outputs whose windows hold one are recomputed exactly in f64 by the same
// workgroup (two-stage for non-finite windows, like the reference).
#pragma once
#include "gar_bg.hpp"

namespace gar {

typedef _Float16 h8v __attribute__((ext_vector_type(8)));
typedef short s4v __attribute__((ext_vector_type(4)));
typedef short s8v __attribute__((ext_vector_type(8)));
typedef float f2v __attribute__((ext_vector_type(2)));
typedef _Float16 h2v __attribute__((ext_vector_type(2)));
typedef __attribute__((address_space(3))) s4v* lds_s4p;

constexpr int kHxNonFinite = 0x40000000;
constexpr int kHxJ = (4 * kHxMaxRows + 64 * kHxMinWaves - 1) / (64 * kHxMinWaves);  // staged row items per lane

__device__ __forceinline__ s4v trRead(const char* p) { return __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s4p)p); }

__device__ __forceinline__ f32x4 mfma16(h8v a, h8v b, f32x4 c) {
    return __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b, c, 0, 0, 0);
}

// ---- launch arguments -------------------------------------------------------
// A launch covers macro periods [a_lo, a_lo + nchunk*G) of C channels; column
// col = chunk * C + c (chunk k = periods a_lo + kG .. + G).  Every output of
// [o_lo, o_hi) goes through the MFMA path, so its value depends only on its own
// window and its absolute position: any chunking of a stream yields the same
// bits (processinto_test.go:258-308).  Interior chunks [k0, k1) (window inside
// the f32 input, outputs inside the range) load raw rows and store whole row
// quads; the other blocks gather their windows through the SrcDesc (history
// seam, flush zeros, f64 input, unfetched tail) and store checked elements.
struct HxArgs {
    const h8v* A;          // [nprog][kch*NS][2][64] f16x8
    const int* progs;      // [nprog][kBgProgInts]
    const int* reds;       // [nred][kBgRedInts]
    int ea, kch;
    int Pc, Qc, W, Ws, G, C, ncols, nblocks, nred, nslots, parity, vst, dbg;
    int fmt;               // interior raw loads: 0 dword gather, 1 stereo frames (x2), 2 four channels (x4)
    int nprog;             // wave programs (waves >= nprog only stage)
    int k0, k1;            // interior chunks
    int ib0, ib1;          // interior blocks (every column an interior chunk)
    int* fix;              // [0] count, [1..fixCap] interior blocks holding loud elements
    int fixCap;
    int64_t a_lo;          // absolute macro period of chunk 0
    int64_t o_lo, o_hi;    // outputs written (absolute)
    const float* in;       // element (row 0 of chunk 0's window, channel 0); dereferenced for interior chunks only
    int64_t in_fs, in_cs, in_chunk;          // elements per row, per channel, per chunk
    char* out;             // byte address of output (row 0 of chunk 0, channel 0); interior chunks only
    int64_t out_fs, out_cs, out_chunk;       // bytes per output row, per channel, per chunk
    int out_f64;
    // cold fields (edge gathers, exact fallback of loud outputs)
    SrcDesc src;
    OutDesc od;
    const double* rows;    // [Pc][rowMax] the FIR rows in f64
    const int* rowOff;     // [Pc] window offset of row r within its macro period
    const int* rowLen;     // [Pc]
    int rowMax;
    int twoStage;          // rows are DFT x2 (*) polyphase composites: loud non-finite windows use the two stages
    const int* rowPh;      // [Pc] polyphase phase / DFT parity of each composite row
    const int* rowPar;
    const double* polyA;   // [L][T2] polyphase bank a (polyphase_stage.go:121-154)
    const double* dftC;    // [2][T1] DFT x2 banks (dft_stage.go:88-101)
    int T1, T2;
};

// ---- staging ----------------------------------------------------------------
// Fixed split scale: x * 2^kHxXs = xh + xl (f16).  Every |x| < kHxLoud (just under 16) keeps
// xh, xl finite, and the split of an element does not depend on its
// neighbours -- the property that makes outputs chunk-invariant.  Elements
// with !(|x| < kHxLoud) (Inf/NaN included) are staged as 0 and marked
// "loud" in a per-column LDS bitmask; every output whose window holds one is
// recomputed exactly (hxFixupBlock).  Small elements keep an absolute
// precision of 2^-(24+kHxXs+kHxLs) (f16 subnormals), far below f32 rounding
// of a full-scale signal.
constexpr int kHxXs = 12;
constexpr int kHxLs = 11;
// 16 - 2^-8 = 65520 / 2^12: the largest bound for which x * 2^12 rounds to a finite f16 (65520 itself
// ties to even, i.e. to +Inf; with 16 here, |x| in [15.99609375, 16) staged hi = Inf and the MFMA
// output was Inf/NaN).  The lo residual of every staged element is then <= 16 * 2^11, finite.
constexpr float kHxLoud = 15.99609375f;

// Image buffer layout: quad q (columns 4q..4q+3) at q*QS, QS = 16*Ws + 64: hi
// rows (4 f16 = 8 B each) then lo rows; the +64 B skew puts the four quads of
// any 8 consecutive rows on distinct banks for ds_read_b64_tr_b16.
// Items: the block's 4*Ws (quad, row) pairs; item t = (wave*kHxJ + j)*64 + lane
// for j < kHxJ, so each wave-instruction's 64 items are 64 consecutive rows of
// one quad (Ws % 64 == 0) and its loads coalesce.
__device__ __forceinline__ uint32_t hxQS(int Ws) { return 16u * static_cast<uint32_t>(Ws) + 64u; }

struct HxItems {
    int n0;          // global index of the wave's slot 0 (slot j covers rows 64*(n0+j) .. of the flattened quads)
    int d, inv;      // Ws/64 and ceil(2^16/d): q = (n*inv) >> 16 exactly for n < 2^10
    int nmax;        // 4*d slots in the block
};

__device__ __forceinline__ HxItems hxItems(int Ws, int wt) {
    HxItems it;
    it.n0 = uni(wt * kHxJ);
    it.d = uni(Ws >> 6);
    it.inv = uni((65536 + it.d - 1) / it.d);
    it.nmax = 4 * it.d;
    return it;
}

// Walks a wave's slots j = 0..kHxJ-1: quad q and first row r (wave-uniform scalars).
#define GAR_HX_SLOTS(it)                                                                                  \
    _Pragma("unroll") for (int j = 0, n = (it).n0, q = (n * (it).inv) >> 16, r = 64 * (n - q * (it).d); \
                           j < kHxJ; ++j, n = (it).n0 + j, q = (n * (it).inv) >> 16, r = 64 * (n - q * (it).d)) if (n < (it).nmax)

__device__ __forceinline__ __amdgpu_buffer_rsrc_t hxRsrc(const float* base) {
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(base), 0, 0x7fffffff, 0x00020000);
}

// Global loads of interior block bl's items into registers (issued, not waited
// on).  Formats 0-2: one buffer resource per block (its first chunk, 64-bit
// base) and per-slot 32-bit scalar offsets (launchHx checks they fit);
// format 3: 64-bit per-lane addresses (strides too large for that).
__device__ __forceinline__ void hxLoad(const HxArgs& x, const HxItems& it, int bl, int lane, f32x4 (&v)[kHxJ]) {
    const uint32_t fsB = static_cast<uint32_t>(x.in_fs) * 4u;
    const uint32_t chB = static_cast<uint32_t>(x.in_chunk) * 4u, csB = static_cast<uint32_t>(x.in_cs) * 4u;
    const int ckB = uni((bl * 16) / x.C);
    const __amdgpu_buffer_rsrc_t rs = hxRsrc(x.in + static_cast<int64_t>(ckB) * x.in_chunk);
    GAR_HX_SLOTS(it) {
        const int rowc = min(r + lane, x.W - 1);
        const int off = static_cast<int>(static_cast<uint32_t>(rowc) * fsB);
        const int col = bl * 16 + 4 * q;
        if (x.fmt == 1) {  // stereo frames: chunks col/2 and col/2 + 1, both channels
            const int k0 = (col >> 1) - ckB;
            const f2v a = __builtin_bit_cast(f2v, __builtin_amdgcn_raw_buffer_load_b64(rs, off, static_cast<int>(k0 * chB), 0));
            const f2v c = __builtin_bit_cast(f2v, __builtin_amdgcn_raw_buffer_load_b64(rs, off, static_cast<int>((k0 + 1) * chB), 0));
            v[j] = f32x4{a.x, a.y, c.x, c.y};
        } else if (x.fmt == 2) {  // four contiguous channels of one chunk
            const int ck = col / x.C, c0 = col - ck * x.C;
            const int so = static_cast<int>((ck - ckB) * chB + c0 * 4u);
            v[j] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(rs, off, so, 0));
        } else if (x.fmt == 0) {
#pragma unroll
            for (int n = 0; n < 4; ++n) {
                const int ck = (col + n) / x.C, c = (col + n) - ck * x.C;
                const int so = static_cast<int>((ck - ckB) * chB + c * csB);
                v[j][n] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rs, off, so, 0));
            }
        } else {
#pragma unroll
            for (int n = 0; n < 4; ++n) {
                const int ck = (col + n) / x.C, c = (col + n) - ck * x.C;
                const float* p = x.in + static_cast<int64_t>(ck) * x.in_chunk + static_cast<int64_t>(c) * x.in_cs +
                                 static_cast<int64_t>(rowc) * x.in_fs;
                v[j][n] = *p;
            }
        }
    }
}

// Edge block: one slot's elements through the SrcDesc (history | input | zeros,
// any dtype); rows >= W and columns past the launch are zero.  Out of line:
// only the first and last blocks of a launch take it.
typedef const __attribute__((address_space(4))) struct HxArgs* HxArgsP;

__device__ __forceinline__ f32x4 hxGatherSlot(HxArgsP xp, int bl, int q, int row) {
    f32x4 v = {0.f, 0.f, 0.f, 0.f};
    const int ncols = xp->ncols, C = xp->C, W = xp->W;
    const int64_t a_lo = xp->a_lo;
    const int G = xp->G, Qc = xp->Qc;
#pragma unroll
    for (int n = 0; n < 4; ++n) {
        const int col = bl * 16 + 4 * q + n;
        if (col < ncols && row < W) {
            const int ck = col / C, c = col - ck * C;
            v[n] = srcRead<float>(kload(&xp->src), (a_lo + static_cast<int64_t>(ck) * G) * Qc + row, c);
        }
    }
    return v;
}

// Two values -> f16 hi halves of s = v * 2^kHxXs and lo halves of
// (s - hi) * 2^kHxLs (the lo products accumulate apart and are scaled back by
// 2^-kHxLs, so a lo half stays normal whenever its hi half is: 22-bit
// precision for every |v| >= 2^-(14+kHxXs)).  Scalar f32 VALU: packed f32
// arithmetic next to MFMAs costs issue cycles.
// GAR_HX_MIXSPLIT: the same halves from mixed-precision FMAs -- hi = f16(v*2^12) and
// lo = f16((v*2^12 - hi)*2^11) each one v_fma_mix{lo,hi}_f16 (rounded once to f16, the product by a
// power of two and the difference exact, as in the plain split), the difference one v_fma_mix_f32:
// 6 VALU per pair instead of 8 (2 v_mul + v_cvt_pk, twice, + 2 v_fma_mix).  A -0 input gives a +0 hi
// half here (-0 * 2^12 + 0), -0 in the plain split: no output changes (an MFMA sum that starts at +0).
#ifndef GAR_HX_MIXSPLIT
#define GAR_HX_MIXSPLIT 0
#endif
__device__ __forceinline__ void hxSplit2Mix(float a, float b, uint32_t& hi, uint32_t& lo) {
    const float kS = static_cast<float>(1 << kHxXs), kL = static_cast<float>(1 << kHxLs);
    uint32_t h, l;
    float ra, rb;
    asm("v_fma_mixlo_f16 %0, %1, %2, 0" : "=v"(h) : "v"(a), "s"(kS));
    asm("v_fma_mixhi_f16 %0, %1, %2, 0" : "+v"(h) : "v"(b), "s"(kS));
    asm("v_fma_mix_f32 %0, %1, %2, -%3 op_sel_hi:[0,0,1]" : "=v"(ra) : "v"(a), "s"(kS), "v"(h));
    asm("v_fma_mix_f32 %0, %1, %2, -%3 op_sel:[0,0,1] op_sel_hi:[0,0,1]" : "=v"(rb) : "v"(b), "s"(kS), "v"(h));
    asm("v_fma_mixlo_f16 %0, %1, %2, 0" : "=v"(l) : "v"(ra), "s"(kL));
    asm("v_fma_mixhi_f16 %0, %1, %2, 0" : "+v"(l) : "v"(rb), "s"(kL));
    hi = h;
    lo = l;
}
__device__ __forceinline__ void hxSplit2Plain(float a, float b, uint32_t& hi, uint32_t& lo) {
    const float sa = a * static_cast<float>(1 << kHxXs), sb = b * static_cast<float>(1 << kHxXs);
    const h2v h = __builtin_convertvector(f2v{sa, sb}, h2v);
    const float ra = (sa - static_cast<float>(h.x)) * static_cast<float>(1 << kHxLs);
    const float rb = (sb - static_cast<float>(h.y)) * static_cast<float>(1 << kHxLs);
    const h2v l = __builtin_convertvector(f2v{ra, rb}, h2v);
    hi = __builtin_bit_cast(uint32_t, h);
    lo = __builtin_bit_cast(uint32_t, l);
}
__device__ __forceinline__ void hxSplit2(float a, float b, uint32_t& hi, uint32_t& lo) {
    if constexpr (GAR_HX_MIXSPLIT) hxSplit2Mix(a, b, hi, lo);
    else hxSplit2Plain(a, b, hi, lo);
}

__device__ __forceinline__ bool hxLoud(float v) { return !(__builtin_fabsf(v) < kHxLoud); }

// Slot j of a wave's items -> f16 hi/lo rows of image buffer buf; loud
// elements -> 0 and a bit in lmask ([16 columns][Ws/32] words) + *lflag = 1.
__device__ __forceinline__ void hxConvertSlot(const HxItems& it, const f32x4 (&v)[kHxJ], int j, int Ws, int lane,
                                              char* buf, uint32_t* lmask, uint32_t* lflag) {
    const int n = it.n0 + j;
    if (n >= it.nmax) return;
    const int q = (n * it.inv) >> 16, r = 64 * (n - q * it.d);
    const int row = r + lane;
    float e0 = v[j][0], e1 = v[j][1], e2 = v[j][2], e3 = v[j][3];
    const bool l0 = hxLoud(e0), l1 = hxLoud(e1), l2 = hxLoud(e2), l3 = hxLoud(e3);
    if (__builtin_expect(l0 | l1 | l2 | l3, 0)) {
        uint32_t* m = lmask + (4 * q) * (Ws >> 5) + (row >> 5);
        const uint32_t bit = 1u << (row & 31);
        if (l0) { atomicOr(m, bit); e0 = 0.f; }
        if (l1) { atomicOr(m + (Ws >> 5), bit); e1 = 0.f; }
        if (l2) { atomicOr(m + 2 * (Ws >> 5), bit); e2 = 0.f; }
        if (l3) { atomicOr(m + 3 * (Ws >> 5), bit); e3 = 0.f; }
        *lflag = 1u;
    }
    uint2 hv, lv;
    hxSplit2(e0, e1, hv.x, lv.x);
    hxSplit2(e2, e3, hv.y, lv.y);
    char* qb = buf + q * hxQS(Ws);
    *reinterpret_cast<uint2*>(qb + 8 * row) = hv;
    *reinterpret_cast<uint2*>(qb + 8 * Ws + 8 * row) = lv;
}

__device__ __forceinline__ h8v bFragA(uint32_t a) {
    const s4v lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s4p)(a));
    const s4v hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s4p)(a + 128));
    const s8v v = __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
    return __builtin_bit_cast(h8v, v);
}

// B fragment (32 K x 16 columns) at the lane's transposed-read address p:
// lane 16g + 4qr + qd supplies row 4g + qr (and +16) of quad qd.
__device__ __forceinline__ h8v bFragQ(const char* p) {
    const s4v lo = trRead(p), hi = trRead(p + 128);  // rows +16 = +128 B
    const s8v v = __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
    return __builtin_bit_cast(h8v, v);
}

// ---- compute --------------------------------------------------------------
// Output of the two accumulators: (main + lo * 2^-kHxLs) * 2^sh, in this order.
__device__ __forceinline__ f32x4 hxScale(f32x4 m, f32x4 l, int sh) {
    f32x4 r;
#pragma unroll
    for (int i = 0; i < 4; ++i) r[i] = ldexpf(__builtin_fmaf(l[i], 1.0f / static_cast<float>(1 << kHxLs), m[i]), sh);
    return r;
}

// Rows r0..r0+3 of the lane's column at byte address p (interior: no checks).
//  vst 2: stereo interleaved f32 (lanes n, n^1 = channels 0/1 swap halves: one 16-B store of two frames each)
//  vst 1: channel-contiguous f32 (one 16-B store)
//  vst 0: any other f32 layout (4 stores);  vst 3: f64 output (4 stores)
template <int VST>
__device__ __forceinline__ void hxPut4(const HxArgs& x, char* p, f32x4 y, int lane) {
    if (VST == 2) {
        const bool even = (lane & 1) == 0;
        const float s0 = even ? y[2] : y[0], s1 = even ? y[3] : y[1];
        // lane ^ 1 (DPP quad_perm [1,0,3,2]: no LDS round trip)
        const float q0 = __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(s0), 0xB1, 0xf, 0xf, false));
        const float q1 = __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(s1), 0xB1, 0xf, 0xf, false));
        f32x4 w;
        if (even) { w[0] = y[0]; w[1] = q0; w[2] = y[1]; w[3] = q1; }
        else      { w[0] = q0; w[1] = y[2]; w[2] = q1; w[3] = y[3]; }
        *reinterpret_cast<f32x4*>(p) = w;
    } else if (VST == 1) {
        *reinterpret_cast<f32x4*>(p) = y;
    } else if (VST == 0) {
#pragma unroll
        for (int i = 0; i < 4; ++i) *reinterpret_cast<float*>(p + i * x.out_fs) = y[i];
    } else {
#pragma unroll
        for (int i = 0; i < 4; ++i) *reinterpret_cast<double*>(p + i * x.out_fs) = static_cast<double>(y[i]);
    }
}

// Byte address of rows r0.. of column (chunk, c) in macro period gi of the chunk.
__device__ __forceinline__ char* hxOutPtr(const HxArgs& x, int chunk, int c, int gi, int r0, int lane) {
    int64_t rr = static_cast<int64_t>(gi) * x.Pc + r0;
    if (x.vst == 2 && (lane & 1)) rr += 2;  // odd lanes store the second frame pair
    return x.out + chunk * x.out_chunk + (x.vst == 2 ? 0 : c * x.out_cs) + rr * x.out_fs;
}

// One output value, checked against the column and the launch's output range
// (edge blocks, segmented-mode results).
__device__ __forceinline__ void hxPut1(const HxArgs& x, int col, int gi, int r, float v) {
    if (col >= x.ncols || r >= x.Pc) return;
    const int chunk = col / x.C, c = col - chunk * x.C;
    const int64_t o = (x.a_lo + static_cast<int64_t>(chunk) * x.G + gi) * x.Pc + r;
    if (o < x.o_lo || o >= x.o_hi) return;
    char* pp = x.out + chunk * x.out_chunk + c * x.out_cs + (static_cast<int64_t>(gi) * x.Pc + r) * x.out_fs;
    if (x.out_f64) *reinterpret_cast<double*>(pp) = v;
    else *reinterpret_cast<float*>(pp) = v;
}

// segment result = hi-x sum + lo-x sum * 2^-kHxLs (unscaled by 2^sh)
__device__ __forceinline__ f32x4 hxComb(f32x4 m, f32x4 l) {
    f32x4 r;
#pragma unroll
    for (int i = 0; i < 4; ++i) r[i] = __builtin_fmaf(l[i], 1.0f / static_cast<float>(1 << kHxLs), m[i]);
    return r;
}

#define GAR_HX_SEG_CHECK(s)                                             \
    if ((s) + 1 == pu.e1) {                                             \
        r0 = hxComb(accB, accS); accB = f32x4{0, 0, 0, 0}; accS = accB; \
    } else if ((s) + 1 == pu.e2) {                                      \
        r1 = hxComb(accB, accS); accB = f32x4{0, 0, 0, 0}; accS = accB; \
    }

// The kernel's argument block behind an opaque pointer: fields the cold paths
// (edges, loud fallback) read through it are loaded where used, instead of
// being hoisted to the kernel entry and held in SGPRs across the block loop.
typedef HxArgsP HxArgsK;
__device__ __forceinline__ HxArgsK hxCold() {
    uint64_t v = reinterpret_cast<uint64_t>(__builtin_amdgcn_kernarg_segment_ptr());
    asm volatile("" : "+s"(v));
    return reinterpret_cast<HxArgsK>(v);
}

// Any bit of [lo, hi) set in a column's loud mask?
__device__ __forceinline__ bool hxBitsAny(const uint32_t* m, int lo, int hi) {
    if (hi <= lo) return false;
    const int w0 = lo >> 5, w1 = (hi - 1) >> 5;
    for (int w = w0; w <= w1; ++w) {
        uint32_t bits = m[w];
        if (w == w0) bits &= ~0u << (lo & 31);
        if (w == w1 && ((hi & 31) != 0)) bits &= (1u << (hi & 31)) - 1u;
        if (bits) return true;
    }
    return false;
}

// Exact value of output (a, r) of channel c in f64 from the stream itself:
// the FIR row, or -- when the window holds Inf/NaN and the row is a DFT x2 (*)
// polyphase composite -- the reference's two stages (a DFT output touched by
// an Inf is +-Inf, their polyphase sum NaN; dft_stage.go:259, polyphase_stage.go:288).
__device__ __forceinline__ double hxExact(HxArgsP x, int64_t a, int r, int c) {
    const SrcDesc src = kload(&x->src);
    const int64_t t = a * x->Qc + x->rowOff[r];
    const int len = x->rowLen[r];
    const double* row = x->rows + static_cast<size_t>(r) * x->rowMax;
    double s = 0.0, z = 0.0;
    for (int k = 0; k < len; ++k) {
        const double v = static_cast<double>(srcRead<float>(src, t + k, c));  // history is f32
        s += row[k] * v;
        z += v * 0.0;
    }
    if (z == z || !x->twoStage) return s;  // finite window (or single-stage FIR: IEEE order-free)
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

// Recompute, exactly, every output of block b whose window holds a loud
// element (all threads of the workgroup; lmask = this buffer's column masks).
__device__ __forceinline__ void hxFixupBlock(HxArgsP xp, int b, const uint32_t* lmask) {
    const HxArgs& x = *(const HxArgs*)(xp);
    const int nout = 16 * x.G * x.Pc;
    const int wpc = x.Ws >> 5;
    for (int idx = threadIdx.x; idx < nout; idx += blockDim.x) {
        const int n = idx & 15, rest = idx >> 4;
        const int r = rest % x.Pc, gi = rest / x.Pc;
        const int col = b * 16 + n;
        if (col >= x.ncols) continue;
        const int chunk = col / x.C, c = col - chunk * x.C;
        const int64_t a = x.a_lo + static_cast<int64_t>(chunk) * x.G + gi;
        const int64_t o = a * x.Pc + r;
        if (o < x.o_lo || o >= x.o_hi) continue;
        const int lo = gi * x.Qc + x.rowOff[r];
        if (!hxBitsAny(lmask + n * wpc, lo, lo + x.rowLen[r])) continue;
        outWrite<float>(x.od, o, c, static_cast<float>(hxExact(xp, a, r, c)));
    }
}

// Loud-element masks of block bl rebuilt from the stream (fix-list blocks of the
// interior kernel, whose LDS masks are gone): all threads, then a barrier.
__device__ __forceinline__ void hxRescan(const HxArgs& x, int bl, uint32_t* lmask) {
    const int wpc = x.Ws >> 5;
    for (int idx = threadIdx.x; idx < 16 * x.W; idx += blockDim.x) {
        const int n = idx / x.W, row = idx - n * x.W;
        const int col = bl * 16 + n;
        if (col >= x.ncols) continue;
        const int ck = col / x.C, c = col - ck * x.C;
        if (hxLoud(srcRead<float>(x.src, (x.a_lo + static_cast<int64_t>(ck) * x.G) * x.Qc + row, c)))
            atomicOr(lmask + n * wpc + (row >> 5), 1u << (row & 31));
    }
}

// EDGE = false: the interior blocks [ib0, ib1) -- raw loads, whole-quad stores;
// a block holding a loud element is appended to x.fix for the edge launch.
// EDGE = true: the edge blocks (gathered windows, checked stores, loud
// outputs fixed in place), then the interior kernel's fix list.
template <int NS, bool RB, bool SINGLE, int VST, bool EDGE>
__global__ __launch_bounds__(64 * kHxMaxWaves) void hx_kernel(HxArgs x) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    const uint32_t QS = hxQS(x.Ws);
    const uint32_t bufB = 4 * QS;
    char* imgs = reinterpret_cast<char*>(smem);  // [2][4 quads][QS]
    float* part = reinterpret_cast<float*>(smem + 2 * static_cast<size_t>(bufB));
    const int partStride = x.nslots * 256;
    // loud masks [2 buffers][16 columns][Ws/32] + flags [2]
    uint32_t* lmaskAll = reinterpret_cast<uint32_t*>(part + (x.parity ? 2 : 1) * partStride);
    const int maskWords = 16 * (x.Ws >> 5);
    uint32_t* lflagAll = lmaskAll + 2 * maskWords;

    const int NW = blockDim.x >> 6;
    const int lane = threadIdx.x & 63;
    const int wt = uni(threadIdx.x >> 6);
    const int nbar = RB ? 0 : (x.nred > 0 ? (x.parity ? 1 : 2) : 0);  // barriers per macro period
    const bool hasProg = wt < x.nprog;
    const int sh = -(x.ea + kHxXs);

    const int grp = lane >> 4, l16 = lane & 15;
    // transposed-read address of this lane: quad (l16 & 3), row 4*grp + (l16 >> 2)
    const uint32_t laneOff = (l16 & 3) * QS + 8u * (4 * grp + (l16 >> 2));
    const ProgU pu = progLoad(x.progs + kBgProgInts * (hasProg ? wt : 0));
    const int nseg = hasProg ? pu.nseg : 0;
    const int plen = uni(x.progs[kBgProgInts * (hasProg ? wt : 0) + 15]);  // program steps (rest: zero A)
    auto uPad = [&](int st) { return st < plen ? selU(pu, st) : -kHxStep * plen; };
    const int u0 = pu.u0, rbw = pu.rb0;
    h8v Ah[NS], Al[NS];
    if (SINGLE) {
#pragma unroll
        for (int s = 0; s < NS; ++s) {
            Ah[s] = x.A[((static_cast<size_t>(hasProg ? wt : 0) * NS + s) * 2 + 0) * 64 + lane];
            Al[s] = x.A[((static_cast<size_t>(hasProg ? wt : 0) * NS + s) * 2 + 1) * 64 + lane];
        }
        // vmcnt(0): A settled on every path into the block loop (else the compiler
        // flushes vmcnt before the MFMA loop -- and with it the staging loads)
        __builtin_amdgcn_s_waitcnt(0x0F70);
    }
    for (int i = threadIdx.x; i < 2 * maskWords + 2; i += blockDim.x) lmaskAll[i] = 0;

    // block sequence of this launch
    const int nB = EDGE ? x.ib0 + (x.nblocks - x.ib1) : x.ib1 - x.ib0;
    auto blockAt = [&](int e) { return EDGE ? (e < x.ib0 ? e : x.ib1 + (e - x.ib0)) : x.ib0 + e; };

    // Staging pipeline (one barrier per block): iteration it computes block b_it
    // from buffer it&1 while converting b_{it+1} (loaded during iteration it-1)
    // into the other buffer, then loads b_{it+2} into registers (landing during
    // the MFMA work).
    const HxItems items = hxItems(x.Ws, wt);
    f32x4 raw[kHxJ];
    int e = blockIdx.x;
    const int G2 = static_cast<int>(gridDim.x);
    const bool staging = !(x.dbg & 1);
    auto fetch = [&](int bl) {
        if (!EDGE) {
            hxLoad(x, items, bl, lane, raw);
        } else {
            const HxArgsK xc = hxCold();
            GAR_HX_SLOTS(items) raw[j] = hxGatherSlot(xc, bl, q, r + lane);
        }
    };
    __syncthreads();  // masks zeroed
    if (e < nB && !(x.dbg & 16)) {  // prologue: block e -> buffer 0, block e+grid -> registers
        fetch(blockAt(e));
#pragma unroll
        for (int j = 0; j < kHxJ; ++j) hxConvertSlot(items, raw, j, x.Ws, lane, imgs, lmaskAll, lflagAll);
        if (e + G2 < nB) fetch(blockAt(e + G2));
    }
    for (int it = 0; e < nB && !(x.dbg & 16); e += G2, ++it) {
        __syncthreads();  // buffer it&1 staged (and its loud flag); buffer (it+1)&1 free
        const int b = blockAt(e);
        const int cur = it & 1;
        const bool conv = e + G2 < nB && staging;
        const bool more = e + 2 * G2 < nB && staging;
        const int b2 = more ? blockAt(e + 2 * G2) : 0;
        char* bufN = imgs + static_cast<size_t>(cur ^ 1) * bufB;
        uint32_t* maskN = lmaskAll + (cur ^ 1) * maskWords;
        uint32_t* flagN = lflagAll + (cur ^ 1);
        const bool loud = lflagAll[cur] != 0u;
        // row-block waves convert block b1's slots inside their first period's MFMA
        // steps and issue block b2's loads after it; everyone else does it here
        const bool convInLoop = RB && nseg > 0 && !(x.dbg & 2);
        if (!convInLoop) {
            if (conv) {
#pragma unroll
                for (int j = 0; j < kHxJ; ++j) hxConvertSlot(items, raw, j, x.Ws, lane, bufN, maskN, flagN);
            }
            if (more) fetch(b2);
        }

        const char* imgH = imgs + static_cast<size_t>(cur) * bufB + laneOff;
        const char* imgL = imgH + 8 * x.Ws;
        const int col = b * 16 + l16;
        const int chunk = col / x.C, c = col - chunk * x.C;

        if (RB) {
            if (nseg > 0 && !(x.dbg & 2)) {
                const bool full = (rbw + 1) * 16 <= x.Pc;
                // interior full row blocks: hxPut4 layout; else rows r0 + i, checked
                char* optr = hxOutPtr(x, chunk, c, 0, rbw * 16 + 4 * grp, lane);
                char* rptr = x.out + chunk * x.out_chunk + c * x.out_cs + (rbw * 16 + 4 * grp) * x.out_fs;
                const int64_t ostep = static_cast<int64_t>(x.Pc) * x.out_fs;
                // the wave's step stream: element u = step u % NS of period u / NS at
                // rows gi*Qc + u0 + 32 s (+8 B per row); B is read one element ahead,
                // across periods (reads past the last period land inside LDS, unused).
                const uint32_t gstep = 8u * static_cast<uint32_t>(x.Qc);
                const uint32_t dL = 8u * static_cast<uint32_t>(x.Ws);
                uint32_t aH = static_cast<uint32_t>(reinterpret_cast<uintptr_t>((lds_s4p)imgH)) + 8u * static_cast<uint32_t>(u0);
                h8v bh0 = bFragA(aH), bl0 = bFragA(aH + dL);
                // epilogue of period gi (issued from inside the next period's MFMA
                // stream so the waves' MFMA pipes never idle through it)
                auto epilogue = [&](const f32x4& oA, const f32x4& oL, int gi) {
                    const f32x4 y = hxScale(oA, oL, sh);
                    if (EDGE) {
#pragma unroll
                        for (int i = 0; i < 4; ++i) hxPut1(x, col, gi, rbw * 16 + 4 * grp + i, y[i]);
                    } else if (full) {
                        hxPut4<VST>(x, optr + gi * ostep, y, lane);
                    } else {  // partial last row block: rows < Pc only
#pragma unroll
                        for (int i = 0; i < 4; ++i)
                            if (rbw * 16 + 4 * grp + i < x.Pc) {
                                char* pp = rptr + gi * ostep + i * x.out_fs;
                                if (VST == 3) *reinterpret_cast<double*>(pp) = y[i];
                                else *reinterpret_cast<float*>(pp) = y[i];
                            }
                    }
                };
                // one period's MFMA program into nA (hi-x products) and nL (lo-x
                // products); the epilogue of period egi (oA, oL) runs after its first step when epi
                auto period = [&](f32x4& nA, f32x4& nL, const f32x4& oA, const f32x4& oL, bool epi, int egi, bool first) {
                    asm volatile("" : "+v"(aH));  // opaque per-period base: reads use base + offset:imm
                    uint32_t aL = aH + dL;
                    asm volatile("" : "+v"(aL));  // lo reads: aL + offset:imm
                    const uint32_t aN = aH + gstep, aNL = aN + dL;
                    nA = f32x4{0, 0, 0, 0};
                    nL = nA;
#pragma unroll
                    for (int s = 0; s < NS; ++s) {
                        const int ug = (s + 1) / NS, us = (s + 1) % NS;
                        const h8v bh1 = bFragA((ug == 0 ? aH : aN) + 256 * us);
                        const h8v bl1 = bFragA((ug == 0 ? aL : aNL) + 256 * us);
                        nA = mfma16(Ah[s], bh0, nA);
                        nA = mfma16(Al[s], bh0, nA);
                        nL = mfma16(Ah[s], bl0, nL);
                        bh0 = bh1; bl0 = bl1;
                        // per step: the 4 LDS reads issue first, then the 3 MFMAs; nothing crosses steps
                        __builtin_amdgcn_sched_group_barrier(0x100, 4, 0);
                        __builtin_amdgcn_sched_group_barrier(0x008, 3, 0);
                        __builtin_amdgcn_sched_barrier(0);
                        if (s == (NS > 1 ? 1 : 0) && epi) epilogue(oA, oL, egi);
                        if (first && conv) {  // block b1's slots j = s, s + NS, ...
#pragma unroll
                            for (int j = s; j < kHxJ; j += NS) hxConvertSlot(items, raw, j, x.Ws, lane, bufN, maskN, flagN);
                        }
                    }
                    aH = aN;
                };
                f32x4 a0, a1 = {0, 0, 0, 0}, l0, l1 = a1;
                // period 0 also converts block b1; block b2's loads follow it and land
                // during the remaining periods
                period(a0, l0, a1, l1, false, 0, true);
                if (more) fetch(b2);
                int gi = 1;
                for (; gi + 1 < x.G; gi += 2) {  // periods in pairs: alternating accumulators
                    period(a1, l1, a0, l0, true, gi - 1, false);
                    period(a0, l0, a1, l1, true, gi, false);
                }
                if (gi < x.G) {
                    period(a1, l1, a0, l0, true, gi - 1, false);
                    epilogue(a1, l1, gi);
                } else {
                    epilogue(a0, l0, gi - 1);
                }
            }
        } else {
            for (int gi = 0; gi < x.G; ++gi) {
                float* pslots = part + static_cast<size_t>(x.parity ? ((it * x.G + gi) & 1) : 0) * partStride;
                if (nseg > 0 && !(x.dbg & 2)) {
                    f32x4 accB = {0, 0, 0, 0}, accS = accB, r0 = accB, r1 = accB;
                    for (int ch = 0; ch < (SINGLE ? 1 : x.kch); ++ch) {
                        const int sb = SINGLE ? 0 : ch * NS;
                        if (!SINGLE) {
#pragma unroll
                            for (int s = 0; s < NS; ++s) {
                                Ah[s] = x.A[((static_cast<size_t>(wt) * x.kch * NS + sb + s) * 2 + 0) * 64 + lane];
                                Al[s] = x.A[((static_cast<size_t>(wt) * x.kch * NS + sb + s) * 2 + 1) * 64 + lane];
                            }
                        }
                        const int rowg = gi * x.Qc;
                        const uint32_t ad = 8u * static_cast<uint32_t>(rowg + uPad(sb) + kHxStep * sb);
                        h8v bh = bFragQ(imgH + ad), bl = bFragQ(imgL + ad);
#pragma unroll
                        for (int s = 0; s < NS; ++s) {
                            h8v nh, nl;
                            if (s + 1 < NS) {
                                const uint32_t an =
                                    8u * static_cast<uint32_t>(rowg + uPad(sb + s + 1) + kHxStep * (sb + s + 1));
                                nh = bFragQ(imgH + an);
                                nl = bFragQ(imgL + an);
                            }
                            accB = mfma16(Ah[s], bh, accB);
                            accB = mfma16(Al[s], bh, accB);
                            accS = mfma16(Ah[s], bl, accS);
                            GAR_HX_SEG_CHECK(sb + s)
                            if (s + 1 < NS) { bh = nh; bl = nl; }
                        }
                    }
                    const f32x4 rlast = hxComb(accB, accS);
#pragma unroll
                    for (int j = 0; j < kBgMaxSeg; ++j) {
                        if (j >= pu.nseg) break;
                        const f32x4 r = j == pu.nseg - 1 ? rlast : (j == 0 ? r0 : r1);
                        const int slot = segSlot(pu, j), rb = segRb(pu, j);
                        if (slot >= 0) {
                            *reinterpret_cast<f32x4*>(pslots + static_cast<size_t>(slot) * 256 + lane * 4) = r;
                        } else {
#pragma unroll
                            for (int i = 0; i < 4; ++i) hxPut1(x, col, gi, rb * 16 + 4 * grp + i, ldexpf(r[i], sh));
                        }
                    }
                }
                if (nbar > 0) {
                    __syncthreads();  // partial slots of this macro period written
                    for (int r = wt; r < x.nred; r += NW) {
                        const int* rt = x.reds + kBgRedInts * r;
                        const int rb = uni(rt[0]), n = uni(rt[1]);
                        f32x4 sum = *reinterpret_cast<const f32x4*>(pslots + static_cast<size_t>(uni(rt[2])) * 256 + lane * 4);
                        for (int k = 1; k < n; ++k)
                            sum += *reinterpret_cast<const f32x4*>(pslots + static_cast<size_t>(uni(rt[2 + k])) * 256 + lane * 4);
#pragma unroll
                        for (int i = 0; i < 4; ++i) hxPut1(x, col, gi, rb * 16 + 4 * grp + i, ldexpf(sum[i], sh));
                    }
                    if (nbar > 1) __syncthreads();
                }
            }
        }
        if (loud) {
            if (EDGE) {
                // outputs whose windows hold a loud element: exact recompute after every
                // wave's MFMA stores of this block landed; then clear the buffer's masks
                __builtin_amdgcn_s_waitcnt(0);
                __syncthreads();
                hxFixupBlock(hxCold(), b, lmaskAll + cur * maskWords);
                __syncthreads();
                for (int i = threadIdx.x; i < maskWords; i += blockDim.x) lmaskAll[cur * maskWords + i] = 0;
            } else {
                if (threadIdx.x == 0) {
                    const int k = atomicAdd(x.fix, 1);
                    if (k < x.fixCap) x.fix[1 + k] = b;
                }
                __syncthreads();  // every wave read the flag / masks before they are cleared
                for (int i = threadIdx.x; i < maskWords; i += blockDim.x) lmaskAll[cur * maskWords + i] = 0;
            }
            if (threadIdx.x == 0) lflagAll[cur] = 0;
        }
        // (the compiler cannot pair the two `more` branches: settle the items on the
        // path it believes skips the fetch, so the conversion above needs no wait)
        __builtin_amdgcn_s_waitcnt(0x0F70);
#pragma unroll
        for (int j = 0; j < kHxJ; ++j) asm volatile("" : "+v"(raw[j]));
    }
    if (EDGE && !(x.dbg & 16)) {
        // the interior kernel's loud blocks (it ran before this launch on the stream);
        // a list that overflowed means: check every interior block
        __syncthreads();
        const int n = *reinterpret_cast<volatile int*>(x.fix);
        const bool all = n > x.fixCap;
        const int cnt = all ? x.ib1 - x.ib0 : n;
        for (int k = blockIdx.x; k < cnt; k += G2) {
            const int bl = all ? x.ib0 + k : x.fix[1 + k];
            hxRescan(x, bl, lmaskAll);
            __syncthreads();
            hxFixupBlock(hxCold(), bl, lmaskAll);
            __syncthreads();
            for (int i = threadIdx.x; i < maskWords; i += blockDim.x) lmaskAll[i] = 0;
            __syncthreads();
        }
    }
}

// Launch of one hx_kernel instantiation pair (explicitly instantiated in
// gar_hx_i*.hip): the interior kernel over `blocks` workgroups (none when
// blocks == 0), then the edge + fix-list kernel over `eblocks`.
template <int NS, bool RB, int VST>
hipError_t hxLaunch(const HxArgs& x, int waves, size_t lds, int64_t blocks, int64_t eblocks, hipStream_t st) {
    const dim3 bd(64 * waves);
    if (blocks > 0) {
        const dim3 gd(static_cast<unsigned>(blocks));
        if (RB || x.kch == 1) {
            setMaxLdsOnce(reinterpret_cast<const void*>(&hx_kernel<NS, RB, true, VST, false>));
            hipLaunchKernelGGL((hx_kernel<NS, RB, true, VST, false>), gd, bd, lds, st, x);
        } else if constexpr (!RB) {
            setMaxLdsOnce(reinterpret_cast<const void*>(&hx_kernel<NS, RB, false, VST, false>));
            hipLaunchKernelGGL((hx_kernel<NS, RB, false, VST, false>), gd, bd, lds, st, x);
        }
    }
    const dim3 ge(static_cast<unsigned>(eblocks));
    if (RB || x.kch == 1) {
        setMaxLdsOnce(reinterpret_cast<const void*>(&hx_kernel<NS, RB, true, 0, true>));
        hipLaunchKernelGGL((hx_kernel<NS, RB, true, 0, true>), ge, bd, lds, st, x);
    } else if constexpr (!RB) {
        setMaxLdsOnce(reinterpret_cast<const void*>(&hx_kernel<NS, RB, false, 0, true>));
        hipLaunchKernelGGL((hx_kernel<NS, RB, false, 0, true>), ge, bd, lds, st, x);
    }
    return hipGetLastError();
}

// every instantiation launchHx can reach: RB NS 1..10 x store layouts 0..3, SEG NS 2..8 (even)
#define GAR_HX_FOR_RB(M, NS) M(NS, true, 0) M(NS, true, 1) M(NS, true, 2) M(NS, true, 3)
#define GAR_HX_FOR_ALL(M)                                                                              \
    GAR_HX_FOR_RB(M, 1) GAR_HX_FOR_RB(M, 2) GAR_HX_FOR_RB(M, 3) GAR_HX_FOR_RB(M, 4) GAR_HX_FOR_RB(M, 5) \
    GAR_HX_FOR_RB(M, 6) GAR_HX_FOR_RB(M, 7) GAR_HX_FOR_RB(M, 8) GAR_HX_FOR_RB(M, 9) GAR_HX_FOR_RB(M, 10) \
    M(2, false, 0) M(4, false, 0) M(6, false, 0) M(8, false, 0)
#define GAR_HX_INST(NS, RB, V) template hipError_t hxLaunch<NS, RB, V>(const HxArgs&, int, size_t, int64_t, int64_t, hipStream_t);

}  // namespace gar
