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
// as f16 hi/lo images (double-buffered).  Every wave of the workgroup both
// computes and stages: at the top of block b it issues the global loads of
// block b+grid's raw f32 windows into registers (a few items per lane), runs
// its MFMA program over block b (the loads land meanwhile), then publishes
// its per-quad max |x| (LDS atomic max), and after one barrier converts its
// items into the other image buffer.  Row-block mode (RB): wave w owns row
// block w over its whole band (A in registers, no partial sums).  Segmented
// mode: 8 balanced wave programs of up to 3 row-block segments with LDS
// partial-sum reduction (as bg_kernel).
// Blocks holding Inf/NaN are skipped and recomputed with a plain f32 FIR over
// the exact rows by the last workgroup to finish (IEEE propagation).
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
    int fmt;               // raw load format: 0 dword gather, 1 stereo frames (x2 loads), 2 four channels (x4 loads)
    int nprog;             // wave programs (waves >= nprog only stage)
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
    int64_t e0lo, e0hi, e1lo, e1hi;  // launch edges [e0lo, e0hi) + [e1lo, e1hi): plain f32 FIR, spread over all waves
};

// ---- staging ----------------------------------------------------------------
// Image buffer layout: quad q (columns 4q..4q+3) at q*QS, QS = 16*Ws + 64: hi
// rows (4 f16 = 8 B each) then lo rows; the +64 B skew puts the four quads of
// any 8 consecutive rows on distinct banks for ds_read_b64_tr_b16.
// Items: the block's 4*Ws (quad, row) pairs; item t = (wave*kHxJ + j)*64 + lane
// for j < kHxJ, so each wave-instruction's 64 items are 64 consecutive rows of
// one quad (Ws % 64 == 0) and its loads coalesce.  Rows >= W are clamped to
// row W-1 (finite; A is zero there); columns past the launch read zeros.
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

// Raw buffer loads: a wave-uniform resource (SGPRs) per chunk/column base and a
// 32-bit lane offset; the compiler tracks them as loads (vmcnt) and keeps the
// 64-bit address math scalar.
__device__ __forceinline__ __amdgpu_buffer_rsrc_t hxRsrc(const float* base) {
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(base), 0, 0x7fffffff, 0x00020000);
}

// Global loads of block bl's items into registers (issued, not waited on).
// Every slot loads unconditionally (columns past the launch read column 0's
// chunk and are zeroed afterwards), so no branch separates a load from its use.
__device__ __forceinline__ void hxLoad(const HxArgs& x, const HxItems& it, int bl, int lane, f32x4 (&v)[kHxJ]) {
    // one buffer resource per block (its first chunk); per slot a scalar byte
    // offset (chunk, channel) and the lane's row offset
    const uint32_t fsB = static_cast<uint32_t>(x.in_fs) * 4u;
    const uint32_t chB = static_cast<uint32_t>(x.in_chunk) * 4u, csB = static_cast<uint32_t>(x.in_cs) * 4u;
    const int ckB = uni((bl * 16) / x.C);
    const __amdgpu_buffer_rsrc_t rs = hxRsrc(x.in + static_cast<int64_t>(ckB) * x.in_chunk);
    GAR_HX_SLOTS(it) {
        const int off = static_cast<int>(static_cast<uint32_t>(min(r + lane, x.W - 1)) * fsB);
        const int col = bl * 16 + 4 * q;
        if (x.fmt == 1) {  // stereo frames: chunks col/2 and col/2 + 1, both channels
            const int k0 = (col >> 1) - ckB;
            const int s0 = col < x.ncols ? static_cast<int>(k0 * chB) : 0;
            const int s1 = col + 2 < x.ncols ? static_cast<int>((k0 + 1) * chB) : 0;
            const f2v a = __builtin_bit_cast(f2v, __builtin_amdgcn_raw_buffer_load_b64(rs, off, s0, 0));
            const f2v c = __builtin_bit_cast(f2v, __builtin_amdgcn_raw_buffer_load_b64(rs, off, s1, 0));
            v[j] = f32x4{a.x, a.y, c.x, c.y};
        } else if (x.fmt == 2) {  // four contiguous channels of one chunk
            const int cc = col < x.ncols ? col : bl * 16;
            const int ck = cc / x.C, c0 = cc - ck * x.C;
            const int so = static_cast<int>((ck - ckB) * chB + c0 * 4u);
            v[j] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(rs, off, so, 0));
        } else {
#pragma unroll
            for (int n = 0; n < 4; ++n) {
                const int cn = col + n < x.ncols ? col + n : bl * 16;
                const int ck = cn / x.C, c = cn - ck * x.C;
                const int so = static_cast<int>((ck - ckB) * chB + c * csB);
                v[j][n] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rs, off, so, 0));
            }
        }
    }
}

// Zero the lanes of item slots whose columns lie past the launch (after the loads landed).
__device__ __forceinline__ void hxMaskCols(const HxArgs& x, const HxItems& it, int bl, f32x4 (&v)[kHxJ]) {
    GAR_HX_SLOTS(it) {
        const int col = bl * 16 + 4 * q;
        if (col + 4 <= x.ncols) continue;  // uniform: whole quad inside
#pragma unroll
        for (int n = 0; n < 4; ++n)
            if (col + n >= x.ncols) v[j][n] = 0.f;
    }
}

// Wave max of non-negative u32 (DPP row shifts + row broadcasts; lane 63).
__device__ __forceinline__ uint32_t hxWaveMax(uint32_t v) {
    v = max(v, static_cast<uint32_t>(__builtin_amdgcn_update_dpp(0, static_cast<int>(v), 0x111, 0xf, 0xf, true)));
    v = max(v, static_cast<uint32_t>(__builtin_amdgcn_update_dpp(0, static_cast<int>(v), 0x112, 0xf, 0xf, true)));
    v = max(v, static_cast<uint32_t>(__builtin_amdgcn_update_dpp(0, static_cast<int>(v), 0x114, 0xf, 0xf, true)));
    v = max(v, static_cast<uint32_t>(__builtin_amdgcn_update_dpp(0, static_cast<int>(v), 0x118, 0xf, 0xf, true)));
    v = max(v, static_cast<uint32_t>(__builtin_amdgcn_update_dpp(0, static_cast<int>(v), 0x142, 0xa, 0xf, false)));
    v = max(v, static_cast<uint32_t>(__builtin_amdgcn_update_dpp(0, static_cast<int>(v), 0x143, 0xc, 0xf, false)));
    return static_cast<uint32_t>(__builtin_amdgcn_readlane(static_cast<int>(v), 63));
}

// Per-quad max |x| bits (Inf/NaN -> 0x7f800000 via an x*0 accumulator) into
// the LDS slots qe[0..3] (atomic max; one lane per item slot).
__device__ __forceinline__ void hxPublishMax(const HxItems& it, f32x4 (&v)[kHxJ], int lane, uint32_t* qe) {
    const f2v z = {0.f, 0.f};
    // every item slot's load settled here, and the registers re-defined as
    // plain values: else the compiler waits vmcnt(0) again where the items are
    // converted -- by then for the MFMA epilogue's stores
    __builtin_amdgcn_s_waitcnt(0x0F70);
#pragma unroll
    for (int j = 0; j < kHxJ; ++j) asm volatile("" : "+v"(v[j]));
    // running lane max over consecutive slots of one quad; one wave reduction +
    // LDS atomic per quad the wave touches
    uint32_t run = 0;
    GAR_HX_SLOTS(it) {
        const f2v v01 = {v[j][0], v[j][1]}, v23 = {v[j][2], v[j][3]};
        const f2v nacc = __builtin_elementwise_fma(v23, z, __builtin_elementwise_fma(v01, z, z));
        const float m = fmaxf(fmaxf(fabsf(v[j][0]), fabsf(v[j][1])), fmaxf(fabsf(v[j][2]), fabsf(v[j][3])));
        const uint32_t mu = (nacc.x == 0.f && nacc.y == 0.f) ? __float_as_uint(m) : 0x7f800000u;
        run = max(run, mu);
        if (j + 1 == kHxJ || n + 1 >= it.nmax || r + 64 >= 64 * it.d) {  // uniform: last slot of this quad
            const uint32_t w = hxWaveMax(run);
            if (lane == 0) atomicMax(qe + q, w);
            run = 0;
        }
    }
}

// Scale exponent of a quad from its max bits: max * 2^e in [2^14, 2^15);
// kHxNonFinite (block goes to the exact slow path) for Inf/NaN, or when the
// quad is so small (max < 2^-111, denormals included) that 2^e is no f32.
__device__ __forceinline__ int hxExpOf(uint32_t mu) {
    if (mu >= 0x7f800000u) return kHxNonFinite;
    if (mu == 0) return 0;
    const int E = static_cast<int>(mu >> 23);
    return E < 15 ? kHxNonFinite : 141 - E;
}

// One window row (4 columns) -> f16 hi and lo rows: xs = x * 2^e (exact),
// hi = f16(xs), lo = f16(xs - hi); packed f32 / f16 pair conversions.
__device__ __forceinline__ void hxPutRow(char* qb, int Ws, int r, f2v sc, f2v v01, f2v v23) {
    const f2v a = v01 * sc, c = v23 * sc;
    const h2v ah = __builtin_convertvector(a, h2v), ch = __builtin_convertvector(c, h2v);
    const h2v al = __builtin_convertvector(a - __builtin_convertvector(ah, f2v), h2v);
    const h2v cl = __builtin_convertvector(c - __builtin_convertvector(ch, f2v), h2v);
    uint2 hv, lv;
    hv.x = __builtin_bit_cast(uint32_t, ah); hv.y = __builtin_bit_cast(uint32_t, ch);
    lv.x = __builtin_bit_cast(uint32_t, al); lv.y = __builtin_bit_cast(uint32_t, cl);
    *reinterpret_cast<uint2*>(qb + 8 * r) = hv;
    *reinterpret_cast<uint2*>(qb + 8 * Ws + 8 * r) = lv;
}

// Items -> f16 hi/lo rows of image buffer buf (quad exponents from qe).
__device__ __forceinline__ void hxConvert(const HxItems& it, const f32x4 (&v)[kHxJ], int Ws, int lane, char* buf,
                                          const uint32_t* qe) {
    const uint32_t QS = hxQS(Ws);
    // quad exponents once (uniform), then per slot a scalar select
    int e4[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) e4[q] = uni(hxExpOf(qe[q]));
    GAR_HX_SLOTS(it) {
        const int e = q == 0 ? e4[0] : q == 1 ? e4[1] : q == 2 ? e4[2] : e4[3];
        if (e == kHxNonFinite) continue;  // block is recomputed by the slow path
        const float s1 = __uint_as_float(static_cast<uint32_t>(e + 127) << 23);
        hxPutRow(buf + q * QS, Ws, r + lane, f2v{s1, s1}, f2v{v[j][0], v[j][1]}, f2v{v[j][2], v[j][3]});
    }
}

// (same, from a 32-bit LDS byte address: base + constant offsets fold into the
// instruction's offset field)
__device__ __forceinline__ h8v bFragA(uint32_t a) {
    const s4v lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s4p)(a));
    const s4v hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s4p)(a + 128));
    const s8v v = __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
    return __builtin_bit_cast(h8v, v);
}

// Slot j of hxConvert (exponents e4 already decoded); for conversion spread
// over the MFMA steps.
__device__ __forceinline__ void hxConvertSlot(const HxItems& it, const f32x4 (&v)[kHxJ], int j, const int (&e4)[4],
                                              int Ws, int lane, char* buf) {
    const int n = it.n0 + j;
    if (n >= it.nmax) return;
    const int q = (n * it.inv) >> 16, r = 64 * (n - q * it.d);
    const int e = q == 0 ? e4[0] : q == 1 ? e4[1] : q == 2 ? e4[2] : e4[3];
    if (e == kHxNonFinite) return;
    const float s1 = __uint_as_float(static_cast<uint32_t>(e + 127) << 23);
    hxPutRow(buf + q * hxQS(Ws), Ws, r + lane, f2v{s1, s1}, f2v{v[j][0], v[j][1]}, f2v{v[j][2], v[j][3]});
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

// The kernel's argument block behind an opaque pointer: fields the cold paths
// (edges, non-finite fixup) read through it are loaded where used, instead of
// being hoisted to the kernel entry and held in SGPRs across the block loop.
typedef const __attribute__((address_space(4))) HxArgs* HxArgsK;
template <class T>
__device__ __forceinline__ T kload(const __attribute__((address_space(4))) T* p) {
    T v;
    __builtin_memcpy(&v, (const T*)p, sizeof(T));
    return v;
}
__device__ __forceinline__ HxArgsK hxCold() {
    uint64_t v = reinterpret_cast<uint64_t>(__builtin_amdgcn_kernarg_segment_ptr());
    asm volatile("" : "+s"(v));
    return reinterpret_cast<HxArgsK>(v);
}

// One output of the plain f32 FIR (exact rows, any source): lanes split the
// taps, then a wave reduction.  Edges of hx launches and fir_kernel.
__device__ __forceinline__ void firOne(const SrcDesc& src, const OutDesc& od, int64_t o, int c, int P, int Q,
                                       const int* rowOff, const int* rowLen, const float* rows, int rowMax, int lane) {
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

template <int NS, bool RB, bool SINGLE, int VST>
__global__ __launch_bounds__(64 * kHxMaxWaves) void hx_kernel(HxArgs x) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    const uint32_t QS = hxQS(x.Ws);
    const uint32_t bufB = 4 * QS;
    char* imgs = reinterpret_cast<char*>(smem);  // [2][4 quads][QS]
    float* part = reinterpret_cast<float*>(smem + 2 * static_cast<size_t>(bufB));
    const int partStride = x.nslots * 256;
    uint32_t* qeAll = reinterpret_cast<uint32_t*>(part + (x.parity ? 2 : 1) * partStride);  // [4 sets][4 quads] + fixup flag

    const int NW = blockDim.x >> 6;
    const int lane = threadIdx.x & 63;
    const int wt = uni(threadIdx.x >> 6);
    const int nbar = RB ? 0 : (x.nred > 0 ? (x.parity ? 1 : 2) : 0);  // barriers per macro period
    const bool hasProg = wt < x.nprog;

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

    // Staging pipeline (one barrier per block): iteration it computes block
    // b_it from buffer it&1 while, in the same barrier interval, converting
    // b_{it+1} (loaded + max-published during iteration it-1) into the other
    // buffer, then loading b_{it+2} into registers (landing during the MFMA
    // work) and publishing its quad maxima at the end.  Exponent sets rotate
    // over 4 (block k uses set k & 3): iteration it reads sets it, it+1, writes
    // it+2 and zeroes it+3 (last read in iteration it-1).
    {  // launch edges (history seam, partial chunks): one output per wave at a time
        const int64_t n0 = (x.e0hi - x.e0lo) * x.C, n = n0 + (x.e1hi - x.e1lo) * x.C;
        for (int64_t idx = static_cast<int64_t>(blockIdx.x) * NW + wt; idx < n; idx += static_cast<int64_t>(gridDim.x) * NW) {
            const bool first = idx < n0;
            const int64_t k = first ? idx : idx - n0;
            const int64_t o = (first ? x.e0lo : x.e1lo) + k / x.C;
            const HxArgsK xc = hxCold();
            const SrcDesc src = kload(&xc->src);
            const OutDesc od = kload(&xc->od);
            firOne(src, od, o, static_cast<int>(k % x.C), x.Pc, x.Qc, xc->rowOff, xc->rowLen, xc->rows, xc->rowMax, lane);
        }
    }
    const HxItems items = hxItems(x.Ws, wt);
    f32x4 raw[kHxJ];
    if (threadIdx.x < 16) qeAll[threadIdx.x] = 0;
    int b = blockIdx.x;
    const int G2 = static_cast<int>(gridDim.x);
    const bool staging = !(x.dbg & 1);
    if (b < x.nblocks && !(x.dbg & 16)) {  // prologue: block b -> buffer 0 (set 0), block b+grid -> registers (set 1)
        hxLoad(x, items, b, lane, raw);
        __syncthreads();  // sets zeroed
        hxMaskCols(x, items, b, raw);
        hxPublishMax(items, raw, lane, qeAll);
        __syncthreads();
        hxConvert(items, raw, x.Ws, lane, imgs, qeAll);
        if (b + G2 < x.nblocks) {
            hxLoad(x, items, b + G2, lane, raw);
            hxMaskCols(x, items, b + G2, raw);
            hxPublishMax(items, raw, lane, qeAll + 4);
        }
    }
    int q = 0;
    for (int it = 0; b < x.nblocks && !(x.dbg & 16); b += G2, ++it) {
        __syncthreads();  // buffer it&1 staged, set it+1 published; buffer (it+1)&1 free
        const uint32_t* qeCur = qeAll + 4 * (it & 3);
        if (threadIdx.x < 4) qeAll[4 * ((it + 3) & 3) + threadIdx.x] = 0;
        const int b1 = b + G2, b2 = b1 + G2;
        const bool conv = b1 < x.nblocks && staging;
        const bool more = b2 < x.nblocks && staging;
        char* bufN = imgs + static_cast<size_t>((it + 1) & 1) * bufB;
        const int myE = hxExpOf(qeCur[l16 >> 2]);
        const bool nonFinite = __any(myE == kHxNonFinite);
        // row-block waves convert block b1's slots inside their first period's MFMA
        // steps and issue block b2's loads after it; everyone else does it here
        const bool convInLoop = RB && nseg > 0 && !(x.dbg & 2) && !nonFinite;
        int e4[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) e4[k] = uni(hxExpOf(qeAll[4 * ((it + 1) & 3) + k]));
        if (!convInLoop) {
            if (conv) {
#pragma unroll
                for (int j = 0; j < kHxJ; ++j) hxConvertSlot(items, raw, j, e4, x.Ws, lane, bufN);
            }
            if (more) hxLoad(x, items, b2, lane, raw);
        }

        const int cur = it & 1;
        const char* imgH = imgs + static_cast<size_t>(cur) * bufB + laneOff;
        const char* imgL = imgH + 8 * x.Ws;
        const int sh = -(x.ea + myE);
        const int col = b * 16 + l16;
        const bool colOk = col < x.ncols;
        const int chunk = col / x.C, c = col - chunk * x.C;

        if (nonFinite) {
            if (wt == 0 && lane == 0) {
                const HxArgsK xc = hxCold();
                int* fix = xc->fix;
                const int k = atomicAdd(&fix[0], 1);
                if (k < xc->fixCap) fix[2 + k] = b;
            }
            for (int gi = 0; gi < x.G; ++gi, ++q)
                for (int k = 0; k < nbar; ++k) __syncthreads();
        } else if (RB) {
            if (nseg > 0 && !(x.dbg & 2)) {
                const bool full = (rbw + 1) * 16 <= x.Pc;
                // full row blocks: hxPut4 layout; partial: rows r0 + i of the lane's column
                char* optr = full ? hxOutPtr(x, chunk, c, 0, rbw * 16 + 4 * grp, lane)
                                  : x.out + chunk * x.out_chunk + c * x.out_cs + (rbw * 16 + 4 * grp) * x.out_fs;
                const int64_t ostep = static_cast<int64_t>(x.Pc) * x.out_fs;
                // the wave's step stream: element u = step u % NS of period u / NS at
                // rows gi*Qc + u0 + 32 s (+8 B per row); B is read one element ahead,
                // across periods (reads past the last period land inside LDS, unused).
                // Three accumulators (one per product term): no MFMA waits on the one
                // before it.
                const uint32_t gstep = 8u * static_cast<uint32_t>(x.Qc);
                const uint32_t dL = 8u * static_cast<uint32_t>(x.Ws);
                uint32_t aH = static_cast<uint32_t>(reinterpret_cast<uintptr_t>((lds_s4p)imgH)) + 8u * static_cast<uint32_t>(u0);
                h8v bh0 = bFragA(aH), bl0 = bFragA(aH + dL);
                // epilogue of one period: scale, store (the previous period's, issued
                // from inside the next period's MFMA stream so the waves' MFMA pipes
                // never idle through it)
                auto epilogue = [&](const f32x4& oA, char* ep) {
                    const f32x4 y = hxScale(oA, sh);
#ifdef GAR_HX_NOEPI
                    if (!(x.dbg & 4096)) return;  // (experiment: no epilogue stores)
#endif
                    if (full) {
                        if (colOk) hxPut4<VST>(x, ep, y, lane);
                    } else {  // partial last row block: rows < Pc only
#pragma unroll
                        for (int i = 0; i < 4; ++i)
                            if (colOk && rbw * 16 + 4 * grp + i < x.Pc) {
                                char* pp = ep + i * x.out_fs;
                                if (x.out_f64) *reinterpret_cast<double*>(pp) = y[i];
                                else *reinterpret_cast<float*>(pp) = y[i];
                            }
                    }
                };
                // one period's MFMA program into nA (one accumulator for the three
                // product terms); the epilogue of oA at ep runs after its first step when epi
                auto period = [&](f32x4& nA, const f32x4& oA, bool epi, char* ep, bool first) {
                    asm volatile("" : "+v"(aH));  // opaque per-period base: reads use base + offset:imm
                    const uint32_t aL = aH + dL, aN = aH + gstep, aNL = aN + dL;
                    nA = f32x4{0, 0, 0, 0};
#pragma unroll
                    for (int s = 0; s < NS; ++s) {
                        const int ug = (s + 1) / NS, us = (s + 1) % NS;
                        const h8v bh1 = bFragA((ug == 0 ? aH : aN) + 256 * us);
                        const h8v bl1 = bFragA((ug == 0 ? aL : aNL) + 256 * us);
                        nA = mfma16(Ah[s], bh0, nA);
                        nA = mfma16(Al[s], bh0, nA);
                        nA = mfma16(Ah[s], bl0, nA);
                        bh0 = bh1; bl0 = bl1;
                        // per step: the 4 LDS reads issue first, then the 3 MFMAs; nothing crosses steps
                        __builtin_amdgcn_sched_group_barrier(0x100, 4, 0);
                        __builtin_amdgcn_sched_group_barrier(0x008, 3, 0);
                        __builtin_amdgcn_sched_barrier(0);
                        if (s == (NS > 1 ? 1 : 0) && epi) epilogue(oA, ep);
                        if (first && conv) {  // block b1's slots j = s, s + NS, ...
#pragma unroll
                            for (int j = s; j < kHxJ; j += NS) hxConvertSlot(items, raw, j, e4, x.Ws, lane, bufN);
                        }
                    }
                    aH = aN;
                };
                f32x4 a0, a1 = {0, 0, 0, 0};
                // period 0 also converts block b1; block b2's loads follow it and land
                // during the remaining periods
                period(a0, a1, false, optr, true);
                if (more) hxLoad(x, items, b2, lane, raw);
                int gi = 1;
                for (; gi + 1 < x.G; gi += 2) {  // periods in pairs: alternating accumulators
                    period(a1, a0, true, optr, false);
                    optr += ostep;
                    period(a0, a1, true, optr, false);
                    optr += ostep;
                }
                if (gi < x.G) {
                    period(a1, a0, true, optr, false);
                    epilogue(a1, optr + ostep);
                } else {
                    epilogue(a0, optr);
                }
            }
        } else {
            for (int gi = 0; gi < x.G; ++gi, ++q) {
                float* pslots = part + static_cast<size_t>(x.parity ? (q & 1) : 0) * partStride;
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
                    for (int r = wt; r < x.nred; r += NW) {
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
        // block b2's quad maxima (its loads landed during the MFMA work)
        if (more) {
            hxMaskCols(x, items, b2, raw);
            hxPublishMax(items, raw, lane, qeAll + 4 * ((it + 2) & 3));
        }
        // (the compiler cannot pair the two `more` branches: settle the items on the
        // path it believes skips the publish, so the conversion above needs no wait)
        __builtin_amdgcn_s_waitcnt(0x0F70);
#pragma unroll
        for (int j = 0; j < kHxJ; ++j) asm volatile("" : "+v"(raw[j]));
    }
    if (!(x.dbg & 8)) {
        const HxArgs xc = kload(hxCold());
        hxFixup(xc, reinterpret_cast<int*>(qeAll + 16));
    }
}

// Direct f32 FIR (launch edges too small for hx_kernel); defined in gar_hx.hip.
__global__ void fir_kernel(SrcDesc src, OutDesc od, int C, int P, int Q, const int* rowOff, const int* rowLen,
                           const float* rows, int rowMax);

// Launch of one hx_kernel instantiation (explicitly instantiated in gar_hx_i*.hip).
template <int NS, bool RB, int VST>
hipError_t hxLaunch(const HxArgs& x, int waves, size_t lds, int64_t blocks, hipStream_t st) {
    static bool attrSet = false;
    if (!attrSet) {
        (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&hx_kernel<NS, RB, true, VST>),
                                  hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
        if constexpr (!RB)
            (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&hx_kernel<NS, RB, false, VST>),
                                      hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
        attrSet = true;
    }
    const dim3 gd(static_cast<unsigned>(blocks)), bd(64 * waves);
    if constexpr (RB) {
        hipLaunchKernelGGL((hx_kernel<NS, true, true, VST>), gd, bd, lds, st, x);
    } else {
        if (x.kch == 1) hipLaunchKernelGGL((hx_kernel<NS, false, true, VST>), gd, bd, lds, st, x);
        else hipLaunchKernelGGL((hx_kernel<NS, false, false, VST>), gd, bd, lds, st, x);
    }
    return hipGetLastError();
}

// every instantiation launchHx can reach: RB NS 1..10 x store layouts 0..3, SEG NS 2..8 (even)
#define GAR_HX_FOR_RB(M, NS) M(NS, true, 0) M(NS, true, 1) M(NS, true, 2) M(NS, true, 3)
#define GAR_HX_FOR_ALL(M)                                                                              \
    GAR_HX_FOR_RB(M, 1) GAR_HX_FOR_RB(M, 2) GAR_HX_FOR_RB(M, 3) GAR_HX_FOR_RB(M, 4) GAR_HX_FOR_RB(M, 5) \
    GAR_HX_FOR_RB(M, 6) GAR_HX_FOR_RB(M, 7) GAR_HX_FOR_RB(M, 8) GAR_HX_FOR_RB(M, 9) GAR_HX_FOR_RB(M, 10) \
    M(2, false, 0) M(4, false, 0) M(6, false, 0) M(8, false, 0)
#define GAR_HX_INST(NS, RB, V) template hipError_t hxLaunch<NS, RB, V>(const HxArgs&, int, size_t, int64_t, hipStream_t);

}  // namespace gar
