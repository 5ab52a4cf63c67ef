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
// as f16 hi/lo images [buffer][hi, lo][row][16 columns] (32-B rows; the 8-B
// quad of columns 4q..4q+3 of row r sits at quad slot q ^ ((r >> 2) & 3), so
// the transposed B-fragment reads are bank-conflict free).  Every wave both
// computes and stages (one uniform VGPR budget):
//   top barrier -> issue the loads of the NEXT block's column pair (whole
//   window, clamped rows, all in flight) -> run the current block's MFMA
//   program(s) -> max |x| of the pair -> convert -> write image[next].
// Row-block mode (RB): wave w owns row block w over its whole band (A in
// registers, no partial sums: one barrier per block).  Segmented mode: 8
// balanced wave programs of up to 3 row-block segments with LDS partial-sum
// reduction (as bg_kernel).
// Blocks holding Inf/NaN are skipped and recomputed with a plain f32 FIR over
// the exact rows by the last workgroup to finish (IEEE propagation).
#pragma once
#include "gar_bg.hpp"

namespace gar {

typedef _Float16 h8v __attribute__((ext_vector_type(8)));
typedef short s2v __attribute__((ext_vector_type(2)));
typedef short s4v __attribute__((ext_vector_type(4)));
typedef short s8v __attribute__((ext_vector_type(8)));
typedef __attribute__((address_space(3))) s4v* lds_s4p;

constexpr int kHxNonFinite = 0x40000000;
constexpr int kHxRpl = kHxMaxRows / 64;  // staged rows per lane (one column pair)

__device__ __forceinline__ s4v trRead(const char* p) { return __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s4p)p); }

// Byte offset of quad slot `q` (4 columns) of image row `r`.
__device__ __forceinline__ uint32_t hxAddr(int r, int q) {
    return static_cast<uint32_t>(r) * 32u + ((static_cast<uint32_t>(q ^ (r >> 2)) & 3u) << 3);
}

__device__ __forceinline__ h8v bFrag(const char* img, uint32_t addr) {
    const s4v lo = trRead(img + addr), hi = trRead(img + addr + 512);
    const s8v v = __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
    return __builtin_bit_cast(h8v, v);
}

__device__ __forceinline__ f32x4 mfma16(h8v a, h8v b, f32x4 c) {
    return __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b, c, 0, 0, 0);
}

// ---- staging ----------------------------------------------------------------
// Wave wt < 8 stages column pair 2wt, 2wt+1 of the NEXT block.  Its raw f32
// window is LDS-DMA'd (global_load_lds_dword, no registers held across the
// MFMA phase) into the free image buffer itself -- raw pair region
// [2 columns][Ws rows] at byte wt*8*Ws, 64*Ws bytes in all = the buffer's
// size -- while the waves compute the current block.  Afterwards each wave
// reads its pair back, takes max |x|, and after one barrier (every raw read
// done) writes the f16 hi/lo images over it.  Row addresses are clamped to
// the window (rows >= W repeat row W-1: finite, and A is zero there); a
// window crossing history | input | flush zeros picks each element's source
// per lane (zeros from p.zero).
struct HxPair {
    const float* p[2];
    int64_t t0[2];
    int c[2];
    int okMask;
    int64_t stride;
    bool fast;
};

__device__ __forceinline__ HxPair hxPairSrc(const SrcDesc& src, const BgGrid& g, int b, int cp) {
    HxPair h;
    bool f = true;
    h.okMask = 0;
    h.stride = 0;
#pragma unroll
    for (int n = 0; n < 2; ++n) {
        const ColSrc<float> cs = colSrc<float>(src, g, b * 16 + 2 * cp + n);
        h.p[n] = cs.p;
        h.t0[n] = cs.t0;
        h.c[n] = cs.c;
        if (cs.ok) {
            h.okMask |= 1 << n;
            if (cs.p == nullptr || (h.stride != 0 && cs.stride != h.stride)) f = false;
            else h.stride = cs.stride;
        }
    }
    h.fast = f;
    return h;
}

// Address of element t of channel c (srcRead of gar_bg.hpp as a pointer select).
__device__ __forceinline__ const float* hxGenPtr(const SrcDesc& s, int64_t t, int c, const float* zero) {
    const int64_t th = t - s.hist_base, ti = t - s.in_base;
    const bool inH = s.hist != nullptr && th >= 0 && th < s.hist_len;
    const bool inI = s.in != nullptr && ti >= 0 && ti < s.in_len;
    const bool ok = t >= 0 && t < s.valid_end;
    return (ok && inH) ? static_cast<const float*>(s.hist) + th * s.hist_ld + c
                       : ((ok && inI) ? static_cast<const float*>(s.in) + ti * s.in_fs + static_cast<int64_t>(c) * s.in_cs
                                      : zero);
}

__device__ __forceinline__ void hxDma(const SrcDesc& src, const BgGrid& g, const HxPair& h, int lane,
                                      const float* zero, char* raw) {
    const int wl = g.W - 1;
    const int nk = g.Ws >> 6;
#pragma unroll
    for (int n = 0; n < 2; ++n) {
        const bool ok = (h.okMask >> n) & 1;
        for (int k = 0; k < nk; ++k) {
            const int r = min(64 * k + lane, wl);
            const float* gp = !ok ? zero
                                  : (h.fast ? h.p[n] + static_cast<int64_t>(r) * h.stride
                                            : hxGenPtr(src, h.t0[n] + r, h.c[n], zero));
            __builtin_amdgcn_global_load_lds((gbl_ptr_t)gp, (lds_ptr_t)(raw + (n * g.Ws + 64 * k) * 4), 4, 0, 0);
        }
    }
}

// my raw pair -> registers; max |x| -> scale exponent (max * 2^e in
// [2^14, 2^15)) or the non-finite flag, published in ce[2cp .. 2cp+1]
__device__ __forceinline__ int hxGather(const BgGrid& g, int lane, int cp, const char* raw, int* ce,
                                        float (&v)[kHxRpl][2]) {
    const float* rf = reinterpret_cast<const float*>(raw);
    uint32_t mu = 0;
#pragma unroll
    for (int i = 0; i < kHxRpl; ++i) {
        if (64 * i >= g.Ws) break;
        v[i][0] = rf[64 * i + lane];
        v[i][1] = rf[g.Ws + 64 * i + lane];
        mu = max(mu, max(__float_as_uint(v[i][0]) & 0x7fffffffu, __float_as_uint(v[i][1]) & 0x7fffffffu));
    }
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
    if (lane < 2) ce[2 * cp + lane] = e;
    return e;
}

__device__ __forceinline__ void hxConvert(const BgGrid& g, const float (&v)[kHxRpl][2], int lane, int cp, int e,
                                          char* imgH, uint32_t imgB) {
    if (e == kHxNonFinite) return;
    const int q = cp >> 1;
    const uint32_t half = (cp & 1) * 4u;
#pragma unroll
    for (int i = 0; i < kHxRpl; ++i) {
        if (64 * i >= g.Ws) break;
        const int r = lane + 64 * i;
        s2v hv, lv;
#pragma unroll
        for (int n = 0; n < 2; ++n) {
            const float xs = ldexpf(v[i][n], e);
            const _Float16 hh = static_cast<_Float16>(xs);
            const _Float16 ll = static_cast<_Float16>(xs - static_cast<float>(hh));
            hv[n] = __builtin_bit_cast(short, hh);
            lv[n] = __builtin_bit_cast(short, ll);
        }
        const uint32_t a = hxAddr(r, q) + half;
        *reinterpret_cast<s2v*>(imgH + a) = hv;
        *reinterpret_cast<s2v*>(imgH + imgB + a) = lv;
    }
}

// Stage block bn (issued earlier by hxDma into image buffer `img`) in place:
// gather (after this wave's DMA landed), barrier, convert.  Every wave of the
// workgroup calls this (the barrier), stagers with stage = true.
__device__ __forceinline__ void hxStageFinish(const BgGrid& g, int lane, int wt, bool stage, char* img, uint32_t imgB,
                                              int* ce) {
    float v[kHxRpl][2];
    int e = 0;
    if (stage) {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's LDS-DMA landed
        e = hxGather(g, lane, wt, img + static_cast<size_t>(wt) * 8 * g.Ws, ce, v);
    }
    __syncthreads();  // every raw pair read: the images may overwrite them
    if (stage) hxConvert(g, v, lane, wt, e, img, imgB);
}

// ---- compute --------------------------------------------------------------
__device__ __forceinline__ f32x4 hxScale(f32x4 r, int sh) {
#pragma unroll
    for (int i = 0; i < 4; ++i) r[i] = ldexpf(r[i], sh);
    return r;
}

__device__ __forceinline__ void hxStore(const ProgU& pu, int j, f32x4 r, float* pslots, const OutDesc& od,
                                        const BgGrid& g, int64_t a, int c, bool colOk, int lane, int sh) {
    const int slot = segSlot(pu, j);
    if (slot < 0) storeAcc<float>(od, g, a, segRb(pu, j), c, colOk, hxScale(r, sh), lane);
    else *reinterpret_cast<f32x4*>(pslots + static_cast<size_t>(slot) * 256 + lane * 4) = r;
}

#define GAR_HX_SEG_CHECK(s)                                      \
    if ((s) + 1 == pu.e1) {                                      \
        r0 = accB + accS; accB = f32x4{0, 0, 0, 0}; accS = accB; \
    } else if ((s) + 1 == pu.e2) {                               \
        r1 = accB + accS; accB = f32x4{0, 0, 0, 0}; accS = accB; \
    }

// Plain f32 FIR over one block (Inf/NaN present): exact rows, IEEE propagation.
__device__ __forceinline__ void hxSlowBlock(const HxDev& p, const SrcDesc& src, const OutDesc& od, const BgGrid& g, int b,
                                            int tid, int nthreads) {
    const int nout = 16 * g.G * g.Pc;
#pragma unroll 1
    for (int idx = tid; idx < nout; idx += nthreads) {
        const int n = idx & 15, rest = idx >> 4;
        const int r = rest % g.Pc, gi = rest / g.Pc;
        const int cl = b * 16 + n;
        if (cl >= g.ncols) continue;
        const int cc = cl % g.C, ck = cl / g.C;
        const int64_t a = g.a_lo + static_cast<int64_t>(ck) * g.G + gi;
        const int64_t o = a * g.Pc + r;
        if (o < od.o_lo || o >= od.o_hi) continue;
        const int64_t t = a * g.Qc + p.rowOff[r];
        const float* row = p.rows + static_cast<size_t>(r) * p.rowMax;
        float s = 0.f;
#pragma unroll 1
        for (int k = 0; k < p.rowLen[r]; ++k) s += row[k] * srcRead<float>(src, t + k, cc);
        outWrite<float>(od, o, cc, s);
    }
}

// Blocks holding Inf/NaN are skipped by the MFMA path and appended to p.fix
// ([0] count, [1] finished workgroups, [2..] block ids); the last workgroup to
// finish recomputes them with hxSlowBlock and resets the counters.
// (s_last is a dynamic-LDS int: a static __shared__ would shift the dynamic
// base off 16 B.)
__device__ __forceinline__ void hxFixup(const HxDev& p, const SrcDesc& src, const OutDesc& od, const BgGrid& g,
                                        int* s_last) {
    __syncthreads();
    if (threadIdx.x == 0) {
        __threadfence();
        *s_last = atomicAdd(&p.fix[1], 1) == static_cast<int>(gridDim.x) - 1;
    }
    __syncthreads();
    if (!*s_last) return;
    __threadfence();
    const int n = __hip_atomic_load(&p.fix[0], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (n > p.fixCap) {  // list overflowed: recompute every block
        for (int b = 0; b < g.nblocks; ++b) hxSlowBlock(p, src, od, g, b, threadIdx.x, blockDim.x);
    } else {
        for (int k = 0; k < n; ++k) {
            const int b = __hip_atomic_load(&p.fix[2 + k], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            hxSlowBlock(p, src, od, g, b, threadIdx.x, blockDim.x);
        }
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        __hip_atomic_store(&p.fix[0], 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(&p.fix[1], 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
}

// RB: row-block mode (<= kHxRbMaxWaves waves); else kHxWaves segmented programs.
template <bool RB>
constexpr int hxThreads() { return RB ? 64 * kHxRbMaxWaves : 64 * kHxWaves; }

template <int NS, bool RB, bool SINGLE>
__global__ __launch_bounds__(hxThreads<RB>()) void hx_kernel(HxDev p, SrcDesc src, OutDesc od, BgGrid g, int ea) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    const uint32_t imgB = static_cast<uint32_t>(g.Ws) * 32u;
    char* imgs = reinterpret_cast<char*>(smem);                         // [2][hi, lo][Ws][32 B]
    float* part = reinterpret_cast<float*>(smem + 4 * static_cast<size_t>(imgB));
    const int partStride = g.nslots * 256;
    int* colExp = reinterpret_cast<int*>(part + (g.parity ? 2 : 1) * partStride);  // [2][16] + fixup flag

    const int lane = threadIdx.x & 63;
    const int wt = uni(threadIdx.x >> 6);
    const int nbar = RB ? 0 : (g.nred > 0 ? (g.parity ? 1 : 2) : 0);  // barriers per macro period
    const bool stager = wt < 8;  // stages column pair wt of every block

    const int grp = lane >> 4, l16 = lane & 15;
    const int rl = 4 * grp + (l16 >> 2);  // image row offset of this lane's transposed-read address
    const int qp = l16 & 3;
    const h8v* Aimg = static_cast<const h8v*>(p.A);
    const ProgU pu = progLoad(p.progs + kBgProgInts * wt);  // one program per wave

    h8v Ah[NS], Al[NS];
    if (SINGLE) {
#pragma unroll
        for (int s = 0; s < NS; ++s) {
            Ah[s] = Aimg[((static_cast<size_t>(wt) * NS + s) * 2 + 0) * 64 + lane];
            Al[s] = Aimg[((static_cast<size_t>(wt) * NS + s) * 2 + 1) * 64 + lane];
        }
    }
    {  // prologue: stage the first block into image 0
        const bool st = stager && static_cast<int>(blockIdx.x) < g.nblocks;
        if (st) hxDma(src, g, hxPairSrc(src, g, blockIdx.x, wt), lane, p.zero, imgs + static_cast<size_t>(wt) * 8 * g.Ws);
        hxStageFinish(g, lane, wt, st, imgs, imgB, colExp);
    }
    int q = 0;
    for (int b = blockIdx.x, it = 0; b < g.nblocks; b += gridDim.x, ++it) {
        __syncthreads();  // image[it&1] staged; image[(it+1)&1] free
        const int cur = it & 1, nxt = cur ^ 1;
        const int bn = b + gridDim.x;
        const bool pre = stager && bn < g.nblocks && !(g.dbg & 1);
        char* nimg = imgs + static_cast<size_t>(nxt) * 2 * imgB;
        if (pre) hxDma(src, g, hxPairSrc(src, g, bn, wt), lane, p.zero, nimg + static_cast<size_t>(wt) * 8 * g.Ws);

        const char* imgH = imgs + static_cast<size_t>(cur) * 2 * imgB;
        const char* imgL = imgH + imgB;
        const int myE = colExp[cur * 16 + l16];
        const bool nonFinite = __any(myE == kHxNonFinite);
        const int sh = -(ea + myE);
        const int col = b * 16 + l16;
        const bool colOk = col < g.ncols;
        const int c = colOk ? col % g.C : 0;
        const int chunk = colOk ? col / g.C : 0;

        if (nonFinite) {
            if (wt == 0 && lane == 0) {
                const int k = atomicAdd(&p.fix[0], 1);
                if (k < p.fixCap) p.fix[2 + k] = b;
            }
            for (int gi = 0; gi < g.G; ++gi, ++q)
                for (int k = 0; k < nbar; ++k) __syncthreads();
        } else {
            for (int gi = 0; gi < g.G; ++gi, ++q) {
                const int64_t a = g.a_lo + static_cast<int64_t>(chunk) * g.G + gi;
                if (RB) {
                    if (pu.nseg > 0 && !(g.dbg & 2)) {
                        // every step's rows are 32 below the previous one: same swizzle, +1 KiB
                        const uint32_t ad = hxAddr(gi * g.Qc + pu.u0 + rl, qp);
                        f32x4 accB = {0, 0, 0, 0}, accS = accB;
                        h8v bh0 = bFrag(imgH, ad), bl0 = bFrag(imgL, ad);
#pragma unroll
                        for (int s = 0; s < NS; ++s) {
                            h8v bh1, bl1;
                            if (s + 1 < NS) {
                                bh1 = bFrag(imgH, ad + 1024 * (s + 1));
                                bl1 = bFrag(imgL, ad + 1024 * (s + 1));
                            }
                            accB = mfma16(Ah[s], bh0, accB);
                            accS = mfma16(Ah[s], bl0, accS);
                            accS = mfma16(Al[s], bh0, accS);
                            if (s + 1 < NS) { bh0 = bh1; bl0 = bl1; }
                        }
                        storeAcc<float>(od, g, a, wt, c, colOk, hxScale(accB + accS, sh), lane);
                    }
                    continue;
                }
                float* pslots = part + static_cast<size_t>(g.parity ? (q & 1) : 0) * partStride;
                if (pu.nseg > 0 && !(g.dbg & 2)) {
                    f32x4 accB = {0, 0, 0, 0}, accS = accB, r0 = accB, r1 = accB;
                    const int rowBase = gi * g.Qc + rl;
                    for (int ch = 0; ch < (SINGLE ? 1 : p.kch); ++ch) {
                        const int sb = SINGLE ? 0 : ch * NS;
                        if (!SINGLE) {
#pragma unroll
                            for (int s = 0; s < NS; ++s) {
                                Ah[s] = Aimg[((static_cast<size_t>(wt) * p.kch * NS + sb + s) * 2 + 0) * 64 + lane];
                                Al[s] = Aimg[((static_cast<size_t>(wt) * p.kch * NS + sb + s) * 2 + 1) * 64 + lane];
                            }
                        }
                        uint32_t ad = hxAddr(rowBase + selU(pu, sb) + kHxStep * sb, qp);
                        h8v bh = bFrag(imgH, ad), bl = bFrag(imgL, ad);
#pragma unroll
                        for (int s = 0; s < NS; ++s) {
                            h8v nh, nl;
                            if (s + 1 < NS) {
                                const uint32_t an = hxAddr(rowBase + selU(pu, sb + s + 1) + kHxStep * (sb + s + 1), qp);
                                nh = bFrag(imgH, an);
                                nl = bFrag(imgL, an);
                            }
                            accB = mfma16(Ah[s], bh, accB);
                            accS = mfma16(Ah[s], bl, accS);
                            accS = mfma16(Al[s], bh, accS);
                            GAR_HX_SEG_CHECK(sb + s)
                            if (s + 1 < NS) { bh = nh; bl = nl; }
                        }
                    }
                    const f32x4 rlast = accB + accS;
                    hxStore(pu, 0, pu.nseg > 1 ? r0 : rlast, pslots, od, g, a, c, colOk, lane, sh);
                    if (pu.nseg > 1) hxStore(pu, 1, pu.nseg > 2 ? r1 : rlast, pslots, od, g, a, c, colOk, lane, sh);
                    if (pu.nseg > 2) hxStore(pu, 2, rlast, pslots, od, g, a, c, colOk, lane, sh);
                }
                if (nbar > 0) {
                    __syncthreads();  // partial slots of this macro period written
                    for (int r = wt; r < g.nred; r += kHxWaves) {
                        const int* rt = p.reds + kBgRedInts * r;
                        const int rb = uni(rt[0]), n = uni(rt[1]);
                        f32x4 sum = *reinterpret_cast<const f32x4*>(pslots + static_cast<size_t>(uni(rt[2])) * 256 + lane * 4);
                        for (int k = 1; k < n; ++k)
                            sum += *reinterpret_cast<const f32x4*>(pslots + static_cast<size_t>(uni(rt[2 + k])) * 256 + lane * 4);
                        storeAcc<float>(od, g, a, rb, c, colOk, hxScale(sum, sh), lane);
                    }
                    if (nbar > 1) __syncthreads();
                }
            }
        }
        // stage the next block: its DMA was issued before the MFMA work
        if (bn < g.nblocks) hxStageFinish(g, lane, wt, pre, nimg, imgB, colExp + nxt * 16);
    }
    hxFixup(p, src, od, g, colExp + 32);
}

}  // namespace gar
