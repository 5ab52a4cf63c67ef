// gar_hx.hpp -- split-f16 banded-GEMM FIR kernel for f32 compute (gfx950).
//
// Same periodic banded GEMM as bg_kernel (gar_bg.hpp), but every product
// a*x is formed as ah*xh + ah*xl + al*xh on v_mfma_f32_16x16x32_f16 (f32
// accumulation), where x*2^ex = xh + xl and a*2^ea = ah + al are f16 pairs
// (22 significant bits each; power-of-two scales chosen so nothing
// overflows: ex per column pair of a block from its max |x|, ea per plan).
// The dropped al*xl term and the representation errors are ~2^-22
// relative, below the f32 accumulation error of the exact-f32 MFMA path,
// and the f16 MFMA retires 16x the MACs per cycle of the f32 one.
//
// One block = 16 columns (channel x chunk of G macro periods) staged in LDS
// as f16 hi/lo images (double-buffered).  Workgroup = nwc compute waves + 2
// stager waves: while the compute waves run block b from one buffer, the
// stagers LDS-DMA block b+grid's raw f32 windows into the other buffer and
// convert them in place.  Row-block mode (RB): compute wave w owns row block
// w over its whole band (A in registers, no partial sums: one barrier per
// block).  Segmented mode: 8 balanced wave programs of up to 3 row-block
// segments with LDS partial-sum reduction (as bg_kernel).
// Blocks holding Inf/NaN are skipped and recomputed with a plain f32 FIR over
// the exact rows by the last workgroup to finish (IEEE propagation).
#pragma once
#include "gar_bg.hpp"

namespace gar {

typedef _Float16 h8v __attribute__((ext_vector_type(8)));
typedef short s4v __attribute__((ext_vector_type(4)));
typedef short s8v __attribute__((ext_vector_type(8)));
typedef __attribute__((address_space(3))) s4v* lds_s4p;

constexpr int kHxNonFinite = 0x40000000;
constexpr int kHxRpl = kHxMaxRows / 64;  // window rows per stager lane

__device__ __forceinline__ s4v trRead(const char* p) { return __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s4p)p); }

__device__ __forceinline__ f32x4 mfma16(h8v a, h8v b, f32x4 c) {
    return __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b, c, 0, 0, 0);
}

// ---- launch arguments -------------------------------------------------------
// The kernel runs only "interior" chunks: every column window lies inside the
// caller's f32 input and every output inside the launch's range (launchHx
// hands the edges -- history seam, flush zeros, partial macro periods -- to
// fir_kernel).  Column col = chunk * C + c (chunk relative to the first
// interior chunk); element addresses are affine in (chunk, c, row).
struct HxArgs {
    const h8v* A;          // [nprog][kch*NS][2][64] f16x8
    const int* progs;      // [nprog][kBgProgInts]
    const int* reds;       // [nred][kBgRedInts]
    int* fix;              // non-finite block list (HxDev::fix)
    int fixCap, ea, kch;
    int Pc, Qc, W, Ws, G, C, ncols, nblocks, nred, nslots, parity, vst, dbg;
    int fmt;               // raw staging format: 0 dword gather, 1 stereo frame pairs (x4), 2 four channels (x4)
    int par0, gqOdd;       // fmt 1: parity of chunk 0's first frame in the input, parity of G*Qc
    const float* in;       // element (row 0 of chunk 0's window, channel 0)
    int64_t in_fs, in_cs, in_chunk;          // elements per row, per channel, per chunk
    char* out;             // byte address of output (row 0 of chunk 0, channel 0)
    int64_t out_fs, out_cs, out_chunk;       // bytes per output row, per channel, per chunk
    int out_f64;
    // fixup of non-finite blocks (plain f32 FIR over the exact rows, generic source)
    SrcDesc src;
    OutDesc od;
    int64_t a0;            // absolute macro period of chunk 0
    const float* rows;
    const int* rowOff;
    const int* rowLen;
    int rowMax;
    const float* zero;
};

// Staging parameters, by value into the (out-of-line) stager routine.
struct HxStage {
    const float* in;
    const float* zero;
    int64_t in_fs, in_cs, in_chunk;
    int W, Ws, C, ncols, fmt, par0, gqOdd;
};

typedef const __attribute__((address_space(4))) HxArgs* HxKarg;  // the kernel's argument block

template <class X>
__device__ __forceinline__ HxStage hxStageArgs(const X& x) {
    HxStage t;
    t.in = x.in; t.zero = x.zero;
    t.in_fs = x.in_fs; t.in_cs = x.in_cs; t.in_chunk = x.in_chunk;
    t.W = x.W; t.Ws = x.Ws; t.C = x.C; t.ncols = x.ncols; t.fmt = x.fmt; t.par0 = x.par0; t.gqOdd = x.gqOdd;
    return t;
}

// ---- staging ----------------------------------------------------------------
// Two stager waves per workgroup stage the NEXT block while the compute waves
// run the current one; stager s owns column quads 2s and 2s+1.  Image buffer
// layout, quad-major: quad q (columns 4q..4q+3) occupies bytes
// [q*QS, q*QS + 16*Ws), QS = 16*Ws + 64: hi rows (4 f16 = 8 B each) then lo
// rows.  The quad's raw f32 window is LDS-DMA'd (global_load_lds_dword, no
// registers) into the same bytes ([4 columns][Ws] f32), then converted in
// place by the one wave that owns it -- no cross-wave synchronisation.  The
// +64 B skew puts the four quads of any 8 consecutive rows on distinct banks
// for ds_read_b64_tr_b16.  Rows >= W are clamped to row W-1 (finite; A is
// zero there); columns past the launch read zeros.
__device__ __forceinline__ uint32_t hxQS(int Ws) { return 16u * static_cast<uint32_t>(Ws) + 64u; }

// (uniform operands made provably scalar: readfirstlane of the LDS address and base)
__device__ __forceinline__ const char* uniPtr(const char* p) {
    const uint64_t v = reinterpret_cast<uint64_t>(p);
    const uint32_t lo = __builtin_amdgcn_readfirstlane(static_cast<uint32_t>(v));
    const uint32_t hi = __builtin_amdgcn_readfirstlane(static_cast<uint32_t>(v >> 32));
    return reinterpret_cast<const char*>((static_cast<uint64_t>(hi) << 32) | lo);
}

__device__ __forceinline__ void hxDmaOne(uint32_t lds, uint32_t voff, const char* base) {
    lds = __builtin_amdgcn_readfirstlane(lds);
    base = uniPtr(base);
    // inline asm: the compiler would otherwise treat every later LDS read as aliasing
    // this DMA and drain vmcnt before it (the stager waits for it explicitly)
    asm volatile("s_mov_b32 m0, %0\n\ts_nop 0\n\tglobal_load_lds_dword %1, %2" :: "s"(lds), "v"(voff), "s"(base) : "m0");
}
__device__ __forceinline__ void hxDmaOne4(uint32_t lds, uint32_t voff, const char* base) {
    lds = __builtin_amdgcn_readfirstlane(lds);
    base = uniPtr(base);
    asm volatile("s_mov_b32 m0, %0\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, %2" :: "s"(lds), "v"(voff), "s"(base) : "m0");
}

// Stereo (fmt 1): a column quad = 2 chunks x 2 channels; chunk jj's window is
// fetched as 16-B frame pairs starting at an even input frame (off = 1 when
// the window starts at an odd one: one leading row), raw [jj][row + off][2].
__device__ __forceinline__ int hxStereoOff(const HxStage& x, int ck) { return (x.par0 + ck * x.gqOdd) & 1; }

__device__ __forceinline__ void hxDmaQuad(const HxStage& x, int b, int q, int lane, char* buf) {
    const uint32_t qbase = static_cast<uint32_t>(reinterpret_cast<uintptr_t>((lds_ptr_t)(buf + q * hxQS(x.Ws))));
    const int wl = x.W - 1;
    if (x.fmt == 1) {
#pragma unroll
        for (int jj = 0; jj < 2; ++jj) {
            const int col = b * 16 + 4 * q + 2 * jj;
            const bool ok = col < x.ncols;
            const int ck = col >> 1;
            const int off = hxStereoOff(x, ck);
            const char* base = ok ? reinterpret_cast<const char*>(x.in + ck * x.in_chunk - 2 * off)
                                  : reinterpret_cast<const char*>(x.zero);
            const int mmax = (wl + off) >> 1;
            const uint32_t l0 = qbase + 8u * static_cast<uint32_t>(x.Ws) * jj;
#pragma unroll
            for (int k = 0; k < kHxRpl / 2; ++k) {
                if (128 * k >= x.Ws) break;
                const uint32_t voff = ok ? static_cast<uint32_t>(min(64 * k + lane, mmax)) * 16u : 0u;
                hxDmaOne4(l0 + 1024u * k, voff, base);
            }
        }
        return;
    }
    if (x.fmt == 2) {
        const int col = b * 16 + 4 * q;
        const bool ok = col < x.ncols;
        const int ck = col / x.C, c0 = col - ck * x.C;
        const char* base = ok ? reinterpret_cast<const char*>(x.in + ck * x.in_chunk + c0)
                              : reinterpret_cast<const char*>(x.zero);
        const uint32_t sb = ok ? static_cast<uint32_t>(x.in_fs) * 4u : 0u;
#pragma unroll
        for (int k = 0; k < kHxRpl; ++k) {
            if (64 * k >= x.Ws) break;
            hxDmaOne4(qbase + 1024u * k, static_cast<uint32_t>(min(64 * k + lane, wl)) * sb, base);
        }
        return;
    }
    const uint32_t sb = static_cast<uint32_t>(x.in_fs) * 4u;
#pragma unroll
    for (int n = 0; n < 4; ++n) {
        const int col = b * 16 + 4 * q + n;
        const bool ok = col < x.ncols;
        const int ck = col / x.C, c = col - ck * x.C;
        const char* base = ok ? reinterpret_cast<const char*>(x.in + ck * x.in_chunk + c * x.in_cs)
                              : reinterpret_cast<const char*>(x.zero);
        const uint32_t sbn = ok ? sb : 0u;
        const uint32_t l0 = qbase + 4u * static_cast<uint32_t>(x.Ws) * n;
#pragma unroll
        for (int k = 0; k < kHxRpl; ++k) {
            if (k >= (x.Ws >> 6)) break;
            hxDmaOne(l0 + 256u * k, static_cast<uint32_t>(min(64 * k + lane, wl)) * sbn, base);
        }
    }
}

// max |x| bits of a lane's values -> wave max -> scale exponent (max * 2^e in
// [2^14, 2^15)) or the non-finite flag, published in ce[4q..4q+3].
__device__ __forceinline__ int hxQuadExp(uint32_t mu, int q, int lane, int* ce) {
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) mu = max(mu, static_cast<uint32_t>(__shfl_xor(static_cast<int>(mu), o)));
    mu = static_cast<uint32_t>(uni(static_cast<int>(mu)));
    int e = 0;
    if (mu >= 0x7f800000u) {
        e = kHxNonFinite;
    } else if (mu != 0) {
        int ex;
        (void)frexpf(__uint_as_float(mu), &ex);
        e = 15 - ex;
    }
    e = uni(e);
    if (lane < 4) ce[4 * q + lane] = e;
    return e;
}

__device__ __forceinline__ void hxPutRow(char* qb, int Ws, int r, int e, const float (&v)[4]) {
    s4v hv, lv;
#pragma unroll
    for (int n = 0; n < 4; ++n) {
        const float xs = ldexpf(v[n], e);
        const _Float16 hh = static_cast<_Float16>(xs);
        const _Float16 ll = static_cast<_Float16>(xs - static_cast<float>(hh));
        hv[n] = __builtin_bit_cast(short, hh);
        lv[n] = __builtin_bit_cast(short, ll);
    }
    *reinterpret_cast<s4v*>(qb + 8 * r) = hv;
    *reinterpret_cast<s4v*>(qb + 8 * Ws + 8 * r) = lv;
}

// Raw quad (layout FMT, see hxDmaQuad) -> registers; scale exponent; f16 hi/lo
// rows written over the raw (every raw value is in registers before the first
// write).  Rows >= Ws (register slots past the window) are not touched.
template <int FMT>
__device__ __forceinline__ void hxConvertQuadF(const HxStage& x, int b, int q, int lane, char* buf, int* ce) {
    char* qb = buf + q * hxQS(x.Ws);
    const float* rf = reinterpret_cast<const float*>(qb);
    const int nr = x.Ws >> 6;
    int o0 = 0, o1 = 0;
    if (FMT == 1) {
        const int ck0 = (b * 16 + 4 * q) >> 1;
        o0 = hxStereoOff(x, ck0);
        o1 = hxStereoOff(x, ck0 + 1);
    }
    float v[kHxRpl][4];
    uint32_t mu = 0;
#pragma unroll
    for (int i = 0; i < kHxRpl; ++i) {
        const int r = min(64 * i, 64 * (nr - 1)) + lane;  // slots past the window repeat the last chunk
        if (FMT == 1) {
            const float2 a = *reinterpret_cast<const float2*>(rf + 2 * (r + o0));
            const float2 c = *reinterpret_cast<const float2*>(rf + 2 * x.Ws + 2 * (r + o1));
            v[i][0] = a.x; v[i][1] = a.y; v[i][2] = c.x; v[i][3] = c.y;
        } else if (FMT == 2) {
            const f32x4 a = *reinterpret_cast<const f32x4*>(rf + 4 * r);
            v[i][0] = a[0]; v[i][1] = a[1]; v[i][2] = a[2]; v[i][3] = a[3];
        } else {
#pragma unroll
            for (int n = 0; n < 4; ++n) v[i][n] = rf[n * x.Ws + r];
        }
#pragma unroll
        for (int n = 0; n < 4; ++n) mu = max(mu, __float_as_uint(v[i][n]) & 0x7fffffffu);
    }
    const int e = hxQuadExp(mu, q, lane, ce);
    if (e == kHxNonFinite) return;
#pragma unroll
    for (int i = 0; i < kHxRpl; ++i)
        if (i < nr) hxPutRow(qb, x.Ws, 64 * i + lane, e, v[i]);
}

// Stager s: block b's quads 2s, 2s+1 into image buffer buf (DMA, wait, convert).
template <int FMT>
__device__ __noinline__ void hxStageF(HxKarg xp, int b, int s, int lane, char* buf, int* ce) {
    const HxStage x = hxStageArgs(*xp);  // uniform fields: scalar loads from the kernarg segment
    hxDmaQuad(x, b, 2 * s, lane, buf);
    hxDmaQuad(x, b, 2 * s + 1, lane, buf);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's LDS-DMA landed
    hxConvertQuadF<FMT>(x, b, 2 * s, lane, buf, ce);
    hxConvertQuadF<FMT>(x, b, 2 * s + 1, lane, buf, ce);
}

// B fragment (32 K x 16 columns) at the lane's transposed-read address p:
// lane 16g + 4qr + qd supplies row 4g + qr (and +16) of quad qd.
__device__ __forceinline__ h8v bFragQ(const char* p) {
    const s4v lo = trRead(p), hi = trRead(p + 128);  // rows +16 = +128 B
    const s8v v = __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
    return __builtin_bit_cast(h8v, v);
}

// ---- compute --------------------------------------------------------------
__device__ __forceinline__ f32x4 hxScale(f32x4 r, int sh) {
#pragma unroll
    for (int i = 0; i < 4; ++i) r[i] = ldexpf(r[i], sh);
    return r;
}

// Rows r0..r0+3 of the lane's column at byte address p (interior: no checks).
//  vst 2: stereo interleaved f32 (lanes n, n^1 = channels 0/1 swap halves: one 16-B store of two frames each)
//  vst 1: channel-contiguous f32 (one 16-B store)
//  vst 0: any other f32 layout (4 stores);  vst 3: f64 output (4 stores)
__device__ __forceinline__ void hxPut4(const HxArgs& x, char* p, f32x4 y, int lane) {
    if (x.vst == 2) {
        const bool even = (lane & 1) == 0;
        const float s0 = even ? y[2] : y[0], s1 = even ? y[3] : y[1];
        const float q0 = __shfl_xor(s0, 1), q1 = __shfl_xor(s1, 1);
        f32x4 w;
        if (even) { w[0] = y[0]; w[1] = q0; w[2] = y[1]; w[3] = q1; }
        else      { w[0] = q0; w[1] = y[2]; w[2] = q1; w[3] = y[3]; }
        *reinterpret_cast<f32x4*>(p) = w;
    } else if (x.vst == 1) {
        *reinterpret_cast<f32x4*>(p) = y;
    } else if (x.vst == 0) {
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

// One output value (partial row blocks / segmented-mode results).
__device__ __forceinline__ void hxPut1(const HxArgs& x, int chunk, int c, int gi, int r, float v) {
    char* pp = x.out + chunk * x.out_chunk + c * x.out_cs + (static_cast<int64_t>(gi) * x.Pc + r) * x.out_fs;
    if (x.out_f64) *reinterpret_cast<double*>(pp) = v;
    else *reinterpret_cast<float*>(pp) = v;
}

#define GAR_HX_SEG_CHECK(s)                                      \
    if ((s) + 1 == pu.e1) {                                      \
        r0 = accB + accS; accB = f32x4{0, 0, 0, 0}; accS = accB; \
    } else if ((s) + 1 == pu.e2) {                               \
        r1 = accB + accS; accB = f32x4{0, 0, 0, 0}; accS = accB; \
    }

// Plain f32 FIR over one block (Inf/NaN present): exact rows, IEEE propagation.
__device__ __forceinline__ void hxSlowBlock(const HxArgs& x, int b) {
    const int nout = 16 * x.G * x.Pc;
    for (int idx = threadIdx.x; idx < nout; idx += blockDim.x) {
        const int n = idx & 15, rest = idx >> 4;
        const int r = rest % x.Pc, gi = rest / x.Pc;
        const int cl = b * 16 + n;
        if (cl >= x.ncols) continue;
        const int cc = cl % x.C, ck = cl / x.C;
        const int64_t a = x.a0 + static_cast<int64_t>(ck) * x.G + gi;
        const int64_t o = a * x.Pc + r;
        const int64_t t = a * x.Qc + x.rowOff[r];
        const float* row = x.rows + static_cast<size_t>(r) * x.rowMax;
        float s = 0.f;
        for (int k = 0; k < x.rowLen[r]; ++k) s += row[k] * srcRead<float>(x.src, t + k, cc);
        outWrite<float>(x.od, o, cc, s);
    }
}

// Blocks holding Inf/NaN are skipped by the MFMA path and appended to x.fix
// ([0] count, [1] finished workgroups, [2..] block ids); the last workgroup to
// finish recomputes them with hxSlowBlock and resets the counters.
// (s_last is a dynamic-LDS int: a static __shared__ would shift the dynamic
// base off 16 B.)
__device__ __forceinline__ void hxFixup(const HxArgs& x, int* s_last) {
    __syncthreads();
    if (threadIdx.x == 0) {
        __threadfence();
        *s_last = atomicAdd(&x.fix[1], 1) == static_cast<int>(gridDim.x) - 1;
    }
    __syncthreads();
    if (!*s_last) return;
    __threadfence();
    const int n = __hip_atomic_load(&x.fix[0], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (n > x.fixCap) {  // list overflowed: recompute every block
        for (int b = 0; b < x.nblocks; ++b) hxSlowBlock(x, b);
    } else {
        for (int k = 0; k < n; ++k) hxSlowBlock(x, __hip_atomic_load(&x.fix[2 + k], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        __hip_atomic_store(&x.fix[0], 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(&x.fix[1], 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
}

// Compute waves: RB (row-block mode) <= kHxRbMaxWaves, else kHxWaves
// segmented programs; + 2 stager waves.
template <bool RB>
constexpr int hxThreads() { return 64 * ((RB ? kHxRbMaxWaves : kHxWaves) + 2); }

template <int NS, bool RB, bool SINGLE>
__global__ __launch_bounds__(hxThreads<RB>()) void hx_kernel(HxArgs x, int nwc) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    const uint32_t QS = hxQS(x.Ws);
    const uint32_t bufB = 4 * QS;
    char* imgs = reinterpret_cast<char*>(smem);  // [2][4 quads][QS]
    float* part = reinterpret_cast<float*>(smem + 2 * static_cast<size_t>(bufB));
    const int partStride = x.nslots * 256;
    int* colExp = reinterpret_cast<int*>(part + (x.parity ? 2 : 1) * partStride);  // [2][16] + fixup flag

    const int lane = threadIdx.x & 63;
    const int wt = uni(threadIdx.x >> 6);
    const int nbar = RB ? 0 : (x.nred > 0 ? (x.parity ? 1 : 2) : 0);  // barriers per macro period

    if (wt >= nwc) {
        // ---- stager wave: quads 2s, 2s+1 of every next block (it = -1: prologue, buffer 0) ----
        const int s = wt - nwc;
        int b = blockIdx.x;
        for (int it = -1; b < x.nblocks && !(x.dbg & 16); ++it) {
            if (it >= 0) __syncthreads();  // buffer it&1 staged; buffer (it+1)&1 free
            const int bs = it < 0 ? b : b + gridDim.x;
            const int ib = it < 0 ? 0 : ((it & 1) ^ 1);
            if (bs < x.nblocks && !(it >= 0 && (x.dbg & 1))) {
                char* buf = imgs + static_cast<size_t>(ib) * bufB;
                int* ce = colExp + ib * 16;
                const HxKarg st = (HxKarg)__builtin_amdgcn_kernarg_segment_ptr();
                if (x.fmt == 1) hxStageF<1>(st, bs, s, lane, buf, ce);
                else if (x.fmt == 2) hxStageF<2>(st, bs, s, lane, buf, ce);
                else hxStageF<0>(st, bs, s, lane, buf, ce);
            }
            if (it >= 0) {
                for (int gi = 0; gi < x.G; ++gi)
                    for (int k = 0; k < nbar; ++k) __syncthreads();
                b += gridDim.x;
            }
        }
    } else {
        // ---- compute wave ----
        const int grp = lane >> 4, l16 = lane & 15;
        // transposed-read address of this lane: quad (l16 & 3), row 4*grp + (l16 >> 2)
        const uint32_t laneOff = (l16 & 3) * QS + 8u * (4 * grp + (l16 >> 2));
        const ProgU pu = progLoad(x.progs + kBgProgInts * wt);  // one program per wave
        const int u0 = pu.u0, rbw = pu.rb0;
        h8v Ah[NS], Al[NS];
        if (SINGLE) {
#pragma unroll
            for (int s = 0; s < NS; ++s) {
                Ah[s] = x.A[((static_cast<size_t>(wt) * NS + s) * 2 + 0) * 64 + lane];
                Al[s] = x.A[((static_cast<size_t>(wt) * NS + s) * 2 + 1) * 64 + lane];
            }
            __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0): A settled before the loop
        }
        int q = 0;
        for (int b = blockIdx.x, it = 0; b < x.nblocks && !(x.dbg & 16); b += gridDim.x, ++it) {
            __syncthreads();  // buffer it&1 staged; buffer (it+1)&1 free
            const int cur = it & 1;
            const char* imgH = imgs + static_cast<size_t>(cur) * bufB + laneOff;
            const char* imgL = imgH + 8 * x.Ws;
            const int myE = colExp[cur * 16 + l16];
            const bool nonFinite = __any(myE == kHxNonFinite);
            const int sh = -(x.ea + myE);
            const int col = b * 16 + l16;
            const bool colOk = col < x.ncols;
            const int chunk = col / x.C, c = col - chunk * x.C;

            if (nonFinite) {
                if (wt == 0 && lane == 0) {
                    const int k = atomicAdd(&x.fix[0], 1);
                    if (k < x.fixCap) x.fix[2 + k] = b;
                }
                for (int gi = 0; gi < x.G; ++gi, ++q)
                    for (int k = 0; k < nbar; ++k) __syncthreads();
                continue;
            }
            if (RB) {
                if (pu.nseg > 0 && !(x.dbg & 2)) {
                    char* optr = hxOutPtr(x, chunk, c, 0, rbw * 16 + 4 * grp, lane);
                    const int64_t ostep = static_cast<int64_t>(x.Pc) * x.out_fs;
                    const bool full = (rbw + 1) * 16 <= x.Pc;
                    for (int gi = 0; gi < x.G; ++gi) {
                        // step s reads rows 32 s further: +256 B
                        const uint32_t ro = 8u * static_cast<uint32_t>(gi * x.Qc + u0);
                        const char* ph = imgH + ro;
                        const char* pl = imgL + ro;
                        f32x4 accB = {0, 0, 0, 0}, accS = accB;
                        h8v bh0 = bFragQ(ph), bl0 = bFragQ(pl), bh1, bl1;
                        if (NS > 1) { bh1 = bFragQ(ph + 256); bl1 = bFragQ(pl + 256); }
#pragma unroll
                        for (int s = 0; s < NS; ++s) {
                            h8v bh2, bl2;
                            if (s + 2 < NS) {
                                bh2 = bFragQ(ph + 256 * (s + 2));
                                bl2 = bFragQ(pl + 256 * (s + 2));
                            }
                            accB = mfma16(Ah[s], bh0, accB);
                            accS = mfma16(Ah[s], bl0, accS);
                            accS = mfma16(Al[s], bh0, accS);
                            bh0 = bh1; bl0 = bl1;
                            if (s + 2 < NS) { bh1 = bh2; bl1 = bl2; }
                        }
                        const f32x4 y = hxScale(accB + accS, sh);
                        if (full) {
                            if (colOk) hxPut4(x, optr, y, lane);
                        } else {  // partial last row block: rows < Pc only
#pragma unroll
                            for (int i = 0; i < 4; ++i)
                                if (colOk && rbw * 16 + 4 * grp + i < x.Pc) hxPut1(x, chunk, c, gi, rbw * 16 + 4 * grp + i, y[i]);
                        }
                        optr += ostep;
                    }
                }
                continue;
            }
            for (int gi = 0; gi < x.G; ++gi, ++q) {
                float* pslots = part + static_cast<size_t>(x.parity ? (q & 1) : 0) * partStride;
                if (pu.nseg > 0 && !(x.dbg & 2)) {
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
                        const uint32_t ad = 8u * static_cast<uint32_t>(rowg + selU(pu, sb) + kHxStep * sb);
                        h8v bh = bFragQ(imgH + ad), bl = bFragQ(imgL + ad);
#pragma unroll
                        for (int s = 0; s < NS; ++s) {
                            h8v nh, nl;
                            if (s + 1 < NS) {
                                const uint32_t an =
                                    8u * static_cast<uint32_t>(rowg + selU(pu, sb + s + 1) + kHxStep * (sb + s + 1));
                                nh = bFragQ(imgH + an);
                                nl = bFragQ(imgL + an);
                            }
                            accB = mfma16(Ah[s], bh, accB);
                            accS = mfma16(Ah[s], bl, accS);
                            accS = mfma16(Al[s], bh, accS);
                            GAR_HX_SEG_CHECK(sb + s)
                            if (s + 1 < NS) { bh = nh; bl = nl; }
                        }
                    }
                    const f32x4 rlast = accB + accS;
#pragma unroll
                    for (int j = 0; j < kBgMaxSeg; ++j) {
                        if (j >= pu.nseg) break;
                        const f32x4 r = j == pu.nseg - 1 ? rlast : (j == 0 ? r0 : r1);
                        const int slot = segSlot(pu, j), rb = segRb(pu, j);
                        if (slot >= 0) {
                            *reinterpret_cast<f32x4*>(pslots + static_cast<size_t>(slot) * 256 + lane * 4) = r;
                        } else if (colOk) {
#pragma unroll
                            for (int i = 0; i < 4; ++i)
                                if (rb * 16 + 4 * grp + i < x.Pc) hxPut1(x, chunk, c, gi, rb * 16 + 4 * grp + i, ldexpf(r[i], sh));
                        }
                    }
                }
                if (nbar > 0) {
                    __syncthreads();  // partial slots of this macro period written
                    for (int r = wt; r < x.nred; r += nwc) {
                        const int* rt = x.reds + kBgRedInts * r;
                        const int rb = uni(rt[0]), n = uni(rt[1]);
                        f32x4 sum = *reinterpret_cast<const f32x4*>(pslots + static_cast<size_t>(uni(rt[2])) * 256 + lane * 4);
                        for (int k = 1; k < n; ++k)
                            sum += *reinterpret_cast<const f32x4*>(pslots + static_cast<size_t>(uni(rt[2 + k])) * 256 + lane * 4);
                        if (colOk) {
#pragma unroll
                            for (int i = 0; i < 4; ++i)
                                if (rb * 16 + 4 * grp + i < x.Pc) hxPut1(x, chunk, c, gi, rb * 16 + 4 * grp + i, ldexpf(sum[i], sh));
                        }
                    }
                    if (nbar > 1) __syncthreads();
                }
            }
        }
    }
    if (!(x.dbg & 8)) hxFixup(x, colExp + 32);
}

// Direct f32 FIR over outputs [od.o_lo, od.o_hi) x C channels (exact rows,
// any source): the edges of a launch (history seam, flush zeros, partial
// macro periods) and launches too small for hx_kernel.  One wave per output:
// lanes split the taps, then a wave reduction.
__global__ __launch_bounds__(256) void fir_kernel(SrcDesc src, OutDesc od, int C, int P, int Q, const int* rowOff,
                                                  const int* rowLen, const float* rows, int rowMax) {
    const int lane = threadIdx.x & 63;
    const int64_t n = (od.o_hi - od.o_lo) * C;
    const int64_t wstep = static_cast<int64_t>(gridDim.x) * (blockDim.x >> 6);
    for (int64_t idx = blockIdx.x * static_cast<int64_t>(blockDim.x >> 6) + (threadIdx.x >> 6); idx < n; idx += wstep) {
        const int64_t o = od.o_lo + idx / C;
        const int c = static_cast<int>(idx % C);
        const int64_t a = o / P;
        const int r = static_cast<int>(o - a * P);
        const int64_t t = a * Q + rowOff[r];
        const float* row = rows + static_cast<size_t>(r) * rowMax;
        float s = 0.f;
        for (int k = lane; k < rowLen[r]; k += 64) s += row[k] * srcRead<float>(src, t + k, c);
#pragma unroll
        for (int off = 32; off >= 1; off >>= 1) s += __shfl_xor(s, off);
        if (lane == 0) outWrite<float>(od, o, c, s);
    }
}

}  // namespace gar
