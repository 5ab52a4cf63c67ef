// gar_hxt.hpp -- balanced streaming split-f16 FIR kernel (row-block plans, gfx950).
//
// Same arithmetic, ring image and per-output MFMA order as hxs_kernel (gar_hxs.hpp), so the two
// kernels (and hxs_small_kernel / hx_kernel) produce identical bits; what changes is how the work
// of a workgroup maps onto the CU's four SIMDs:
//
//  * Balanced compute waves.  hxs_kernel runs one compute wave per row block, so a 10-row-block
//    plan puts 3/3/2/2 MFMA streams on the four SIMDs and the busiest SIMD sets the pace (+20 %).
//    Here the host hands every compute wave a role (row block, period phase, period stride): the
//    first 4*floor(nprog/4) row blocks get one wave each (stride 1), and the remaining one or two
//    row blocks are each shared by 4 / 2 waves that take every 4th / 2nd macro period.  Waves w,
//    w+4, w+8 share a SIMD (a workgroup's waves are dealt round-robin over the SIMDs), so every
//    SIMD carries the same number of MFMA steps per period: 10 row blocks -> 12 compute waves,
//    9 + 9 + 4.5 steps per SIMD.  Each output is still computed by exactly one wave with the same
//    A fragments and MFMA chain, so the bits do not change.
//  * One loader wave per SIMD (4), each specialised at compile time for the launch's input layout
//    (FMT 1 stereo f32 frames, FMT 2 rows of 16 f32 channels): a fixed buffer-load pattern issued
//    kHxtD groups ahead into registers, then a straight-line f16 hi/lo split into the ring with the
//    loud-element test folded into one running integer max per lane (the exact per-element path
//    runs only when that max says a loud element is present).  Edge loads (history seam, stream
//    start, partial blocks) go through an out-of-line gather, so their code does not weigh on the
//    registers of the streaming loop.
//  * Groups never run past the chunk (the last group of a chunk has Np - g*G periods).
#pragma once
#include "gar_hxs.hpp"

namespace gar {

// NL loader waves (template parameter, 4 or 6) + up to 16 - NL compute waves, 16 waves at most.
constexpr int kHxtMaxComp = 12;                         // compute waves (3 per SIMD)
constexpr int kHxtWaves = 16;                           // __launch_bounds__: 16 waves, 128 VGPRs
constexpr int kHxtD = 2;                                // loads in flight per loader (register staging)
// 64-row pieces of one load (G*Qc <= 64 * pieces): 10 with 4 loaders, 12 with 6 (the registers
// of a loader's two loads in flight stay at 80 / 64 VGPRs)
__host__ __device__ constexpr int hxtPieces(int NL) { return NL >= 6 ? 12 : 10; }
__host__ __device__ constexpr int hxtMaxRows(int NL) { return 64 * hxtPieces(NL); }
// Items of loader l (of NL): FMT 1 item it = l + NL*k covers quad it & 3, 64-row piece it >> 2;
// FMT 2 item it = l + NL*k is the 16-row piece it (all four quads, lane = 16 quad + row);
// FMT 5 item it is the 8-row piece it of a 32-channel block (all eight quads, lane = 8 row + quad).
template <int NL>
constexpr int hxtItems() { return (4 * hxtPieces(NL) + NL - 1) / NL; }
// FMT 5 (round 6): 32-channel blocks of f32 rows -- every load and store instruction of a workgroup
// covers whole 128-B lines (tools/ubench/row16_copy: the ns256 memory pattern with 64-B half rows per
// workgroup runs at 3.0 TB/s with no compute at all, 1.86 ms; with 128-B rows 4.0-4.2 TB/s, 1.36-1.40
// ms).  The block is two 16-column tiles (sub-blocks 2b, 2b+1 of the 16-column numbering) over one
// ring of eight quads; each compute wave runs both tiles of its row block per period.
__host__ __device__ constexpr int hxtQuads(int FMT) { return FMT == 5 ? 8 : 4; }
__host__ __device__ constexpr int hxtCols(int FMT) { return 4 * hxtQuads(FMT); }
__host__ __device__ constexpr int hxtMaxRowsF(int FMT, int NL) {
    return FMT == 5 ? 8 * NL * ((4 * hxtPieces(NL) + NL - 1) / NL) : 64 * hxtPieces(NL);
}
// loader waves' issue priority (s_setprio; 0 = the compute waves' level).  The loaders share each
// SIMD with three MFMA-issuing compute waves; at equal priority the arbiter lets the MFMA stream
// starve the loaders' VALU (r05 stamps: ~19 cycles per loader VALU instruction), and the loaders
// are the kernel's critical path.
#ifndef GAR_HXT_CPRIO  // development: s_setprio of the compute waves (r05u: 1, 2, 3 all within noise of 0)
#define GAR_HXT_CPRIO 0
#endif
#ifndef GAR_HXT_LPRIO
#define GAR_HXT_LPRIO 0
#endif
// development: attribution modes compiled into a production build (the GAR_HXS_DBG bits, outputs
// wrong by design) -- the runtime knob needs the GAR_HXS_DEV build, whose stamps and knob loads
// change the kernel being attributed (r06t: 2.28 vs 1.70 ms on ns256)
#ifndef GAR_HXT_CTDBG
#define GAR_HXT_CTDBG 0
#endif
constexpr uint32_t kHxtLoudBits = 0x417FF000u;          // bits(kHxLoud = 15.99609375f): !(|x| < kHxLoud) <=> (bits & 0x7fffffff) >= it
static_assert(__builtin_bit_cast(uint32_t, kHxLoud) == kHxtLoudBits, "hxt's loud test must match hxLoud");

struct HxtRole {
    int rb, ph, st;
};
__device__ __forceinline__ HxtRole hxtRole(const HxsArgs& x, int w) {
    const int r = uni(x.role[w]);
    return HxtRole{r & 0xff, (r >> 8) & 0xff, r >> 16};
}

// ---- loaders ------------------------------------------------------------------------
template <int FMT, int NL>
struct HxtBuf;
template <int NL>
struct HxtBuf<1, NL> {  // stereo f32 frames: two chunks (both channels each) per item
    f2v a[hxtItems<NL>()], b[hxtItems<NL>()];
};
template <int NL>
struct HxtBuf<2, NL> {  // 16-channel f32 rows: four channels of one row per lane
    f32x4 v[hxtItems<NL>()];
};
template <int NL>
struct HxtBuf<5, NL> {  // 32-channel f32 rows: four channels of one row per lane
    f32x4 v[hxtItems<NL>()];
};

// Issue load `st` (a real load when live and fast; otherwise every item's offset lies past the
// records, which returns zeros without a memory access -- the same instruction pattern on every
// path, so the compiler's vmcnt tracking waits for exactly the oldest load).
template <int FMT, int NL>
__device__ __forceinline__ bool hxtIssue(const HxsStage& st, bool live, const HxsRegSrc& rs, int l, HxtBuf<FMT, NL>& r) {
    const bool fast = live && st.fast;
    const int nrow = fast ? st.nrow : 0;
    // loader index and strides opaque per call: otherwise every item's offset and mask is hoisted out
    // of the step loop into SGPRs, which spill (one v_readlane per item and step)
    int lq = l, rowB = rs.rowB, chunkB = rs.chunkB;
    asm volatile("" : "+s"(lq), "+s"(rowB), "+s"(chunkB));
    const int base = st.T0 * rowB + rs.lane0;
#pragma unroll
    for (int k = 0; k < hxtItems<NL>(); ++k) {
        if constexpr (FMT == 1) {  // item it: quad q = chunks 2q, 2q+1; piece it >> 2 = rows 64 (it >> 2) ..
            const int it = lq + NL * k, q = it & 3, pc = it >> 2;
            const bool on = pc < hxtPieces(NL) && 64 * pc < nrow;
            const int o = on ? base + 64 * pc * rowB + 2 * q * chunkB : static_cast<int>(0x80000000u);
            const int o2 = on ? o + chunkB : o;
            r.a[k] = __builtin_bit_cast(f2v, __builtin_amdgcn_raw_buffer_load_b64(rs.r, o, 0, 0));
            r.b[k] = __builtin_bit_cast(f2v, __builtin_amdgcn_raw_buffer_load_b64(rs.r, o2, 0, 0));
        } else {  // FMT 2: 16-row piece l + NL k, lane = 16 quad + row; FMT 5: 8-row piece, lane = 8 row + quad
            constexpr int kRp = FMT == 5 ? 8 : 16;
            const int it = lq + NL * k;
            const bool on = kRp * it < nrow;
            const int o = on ? base + kRp * it * rowB : static_cast<int>(0x80000000u);
            r.v[k] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(rs.r, o, 0, 0));
        }
    }
    return fast;
}

// One ring row (quad q, ring row p) <- hi/lo split of e; the mirror copy when p < mirror.
__device__ __forceinline__ void hxtPut(char* qb, uint32_t dL, int p, int R, int mirror, f32x4 e) {
    uint2 hv, lv;
    hxSplit2(e[0], e[1], hv.x, lv.x);
    hxSplit2(e[2], e[3], hv.y, lv.y);
    *reinterpret_cast<uint2*>(qb + 8 * p) = hv;
    *reinterpret_cast<uint2*>(qb + dL + 8 * p) = lv;
    if (p < mirror) {
        *reinterpret_cast<uint2*>(qb + 8 * (p + R)) = hv;
        *reinterpret_cast<uint2*>(qb + dL + 8 * (p + R)) = lv;
    }
}

__device__ __forceinline__ uint32_t hxtMag(float v) { return __float_as_uint(v) & 0x7fffffffu; }
// GAR_HXT_HILOUD: the loud test read off the f16 hi halves instead of the f32 inputs -- !(|x| < kHxLoud)
// (NaN included) <=> x * 2^12 >= 65520 in magnitude or NaN <=> its f16 rounding is Inf / NaN <=>
// (hi & 0x7fff) >= 0x7c00 (65520 ties to even, i.e. to Inf; hxSplit2).  One v_and + one v_pk_max_u16
// per two elements instead of an and + a max per element.
#ifndef GAR_HXT_HILOUD
#define GAR_HXT_HILOUD 0
#endif
typedef unsigned short u16x2v __attribute__((ext_vector_type(2)));

// (r05: the split with v_pk_mul_f32 for the two power-of-two scalings -- 12 instead of 16 VALU per
// item -- measured slower on every workload, ns256 1.766 vs 1.732 ms, cfg3 0.332 vs 0.317 ms: packed f32
// next to the compute waves' MFMAs costs more issue than it saves; profiles/r05s_ab_pksplit.txt)

template <int FMT, int NL>
__device__ __forceinline__ f32x4 hxtItem(const HxtBuf<FMT, NL>& r, int k) {
    if constexpr (FMT == 1) return f32x4{r.a[k].x, r.a[k].y, r.b[k].x, r.b[k].y};
    else return r.v[k];
}

// Exact per-element path of a load that holds a loud element (rare): loader l's items
// of the load again, re-read from memory through the SrcDesc with the fast path's item mapping and
// staged through hxsPutItem (loud elements as zero, their column rows recorded).
// Inlined (default): as out-of-line calls, the calling convention's register saves made the
// allocator spill a load's destination right after the issue, so every loader step waited for
// its own loads (kHxtD-deep pipeline serialised; 61 us of cfg2's 163 us) -- GAR_HXT_SLOW_ATTR=__noinline__
// restores the calls for A/B.
#ifndef GAR_HXT_SLOW_ATTR
#define GAR_HXT_SLOW_ATTR __forceinline__
#endif
template <int FMT, int NL>
__device__ GAR_HXT_SLOW_ATTR void hxtLoudLoad(HxsArgsP xp, HxsStage st, int b, int l, int lane, HxsShared sh) {
    const SrcDesc src = kload(&xp->src);
    const int p0 = uni(st.T0 % xp->R);
    for (int k = 0; k < hxtItems<NL>(); ++k) {
        int row, q;
        if constexpr (FMT == 1) {
            const int it = l + NL * k, pc = it >> 2;
            if (pc >= hxtPieces(NL) || 64 * pc >= st.nrow) continue;
            row = 64 * pc + lane;
            q = it & 3;
        } else if constexpr (FMT == 5) {
            const int it = l + NL * k;
            if (8 * it >= st.nrow) break;
            row = 8 * it + (lane >> 3);
            q = lane & 7;
        } else {
            const int it = l + NL * k;
            if (16 * it >= st.nrow) break;
            row = 16 * it + (lane & 15);
            q = lane >> 4;
        }
        if (row >= st.nrow) continue;
        f32x4 e;
#pragma unroll
        for (int n = 0; n < 4; ++n) {
            const int col = b * hxtCols(FMT) + 4 * q + n;
            const int kk = col / xp->C, c = col - kk * xp->C;
            e[n] = hxsGather(src, hxsChunkRow(xp, kk, st.T0 + row), c, xp->A);
        }
        hxsPutItem(xp, st, p0, q, row, e, sh.ring, sh.QS, sh.loudLo, sh.loudHi, sh.flag);
    }
}

// Edge load (rows before the raw input, partial blocks, any other layout): every element gathered
// through the SrcDesc (history | input | zeros); out of line.  Loader l takes items l, l+4, ...
// of the 4 quads x ceil(nrow/64) pieces.
template <int NQ>
__device__ GAR_HXT_SLOW_ATTR void hxtGatherLoad(HxsArgsP xp, HxsStage st, int b, int l, int nl, int lane, HxsShared sh) {
    const SrcDesc src = kload(&xp->src);
    const int p0 = uni(st.T0 % xp->R);
    const int nit = NQ * ((st.nrow + 63) >> 6);
    for (int it = l; it < nit; it += nl) {
        const int q = it % NQ, row = 64 * (it / NQ) + lane;
        if (row >= st.nrow) continue;
        f32x4 e;
#pragma unroll
        for (int n = 0; n < 4; ++n) {
            const int col = b * 4 * NQ + 4 * q + n;
            const int kk = col / xp->C, c = col - kk * xp->C;
            e[n] = col < xp->ncols ? hxsGather(src, hxsChunkRow(xp, kk, st.T0 + row), c, xp->A) : 0.f;
        }
        hxsPutItem(xp, st, p0, q, row, e, sh.ring, sh.QS, sh.loudLo, sh.loudHi, sh.flag);
    }
}

// Fast load `st` -> ring (registers of its issue): split, write, one running max for the loud test.
// GAR_HXT_SPLITFIRST (default): every item's f16 split first, as one branch-free block the scheduler
// interleaves across items, then the ring writes (their per-item / per-lane conditions are branches);
// split and write per item inside the branches (0) left each item's dependent VALU chain alone in its
// basic block (r05 stamps: ~730 cycles per item on a loader beside three MFMA waves).
// GAR_HXT_LOBASE (default): the lo rows' base is its own register per period, so the B-lo reads of
// every step are base + immediate offset instead of an add of the (runtime) hi/lo distance per step.
#ifndef GAR_HXT_LOBASE
#define GAR_HXT_LOBASE 1
#endif
#ifndef GAR_HXT_SPLITFIRST
#define GAR_HXT_SPLITFIRST 1
#endif
template <int FMT, int NL>
__device__ __forceinline__ void hxtConvert(const HxsArgs& x, const HxsStage& st, int p0, const HxtBuf<FMT, NL>& r, int b,
                                           int l, int lane, const HxsShared& sh) {
    const int R = x.R, mirror = x.mirror;
    const uint32_t dL = 8u * static_cast<uint32_t>(x.Rt);
    const int nrow = st.nrow;
    // opaque per call: the compiler must not hoist the items' row numbers out of the step loop
    // (ten live row registers spill, and every reload's vmcnt(0) waits for the loads in flight)
    int ln = lane, lq = l;
    asm volatile("" : "+v"(ln), "+s"(lq));
    uint32_t m = 0;
    u16x2v mh = {0, 0};  // GAR_HXT_HILOUD: running max of the hi halves' magnitude bits
    auto itemPos = [&](int k, int& row, int& q) {  // -> whether item k holds rows of this load (uniform)
        if constexpr (FMT == 1) {
            const int it = lq + NL * k, pc = it >> 2;
            row = 64 * pc + ln;
            q = it & 3;
            return pc < hxtPieces(NL) && 64 * pc < nrow;
        } else if constexpr (FMT == 5) {
            const int it = lq + NL * k;
            row = 8 * it + (ln >> 3);
            q = ln & 7;
            return 8 * it < nrow;
        } else {
            const int it = lq + NL * k;
            row = 16 * it + (ln & 15);
            q = ln >> 4;
            return 16 * it < nrow;
        }
    };
#if GAR_HXT_SPLITFIRST
    // in chunks of kSplitChunk items: the split values of a chunk stay within the registers the
    // consumed load buffer frees (a whole load's at once spilled on FMT 2)
    constexpr int K = hxtItems<NL>(), kSplitChunk = 4;
#pragma unroll
    for (int k0 = 0; k0 < K; k0 += kSplitChunk) {
        uint2 hv[kSplitChunk], lv[kSplitChunk];
#pragma unroll
        for (int u = 0; u < kSplitChunk; ++u) {  // items the load does not hold were loaded as zeros
            if (k0 + u >= K) break;
            const f32x4 e = hxtItem<FMT, NL>(r, k0 + u);
            if constexpr (!GAR_HXT_HILOUD)
                m = max(m, max(max(hxtMag(e[0]), hxtMag(e[1])), max(hxtMag(e[2]), hxtMag(e[3]))));
            hxSplit2(e[0], e[1], hv[u].x, lv[u].x);
            hxSplit2(e[2], e[3], hv[u].y, lv[u].y);
            if constexpr (GAR_HXT_HILOUD) {
                mh = __builtin_elementwise_max(mh, __builtin_bit_cast(u16x2v, hv[u].x & 0x7fff7fffu));
                mh = __builtin_elementwise_max(mh, __builtin_bit_cast(u16x2v, hv[u].y & 0x7fff7fffu));
            }
        }
#pragma unroll
        for (int u = 0; u < kSplitChunk; ++u) {
            if (k0 + u >= K) break;
            int row, q;
            if (itemPos(k0 + u, row, q) && row < nrow) {
                int p = p0 + row;
                p = p >= R ? p - R : p;
                uint32_t qs = sh.QS;  // quad base recomputed per item (opaque): hoisted per-quad bases spill
                asm volatile("" : "+s"(qs));
                char* qb = sh.ring + q * qs;
                *reinterpret_cast<uint2*>(qb + 8 * p) = hv[u];
                *reinterpret_cast<uint2*>(qb + dL + 8 * p) = lv[u];
                if (p < mirror) {
                    *reinterpret_cast<uint2*>(qb + 8 * (p + R)) = hv[u];
                    *reinterpret_cast<uint2*>(qb + dL + 8 * (p + R)) = lv[u];
                }
            }
        }
    }
#else
#pragma unroll
    for (int k = 0; k < hxtItems<NL>(); ++k) {
        int row, q;
        if (itemPos(k, row, q)) {  // uniform
            const f32x4 e = hxtItem<FMT, NL>(r, k);
            m = max(m, max(max(hxtMag(e[0]), hxtMag(e[1])), max(hxtMag(e[2]), hxtMag(e[3]))));
            int p = p0 + row;
            p = p >= R ? p - R : p;
            uint32_t qs = sh.QS;
            asm volatile("" : "+s"(qs));
            if (row < nrow) hxtPut(sh.ring + q * qs, dL, p, R, mirror, e);
        }
    }
#endif
    const bool loud = GAR_HXT_HILOUD ? (mh.x >= 0x7c00u || mh.y >= 0x7c00u) : m >= kHxtLoudBits;
    if (__builtin_expect(__builtin_amdgcn_ballot_w64(loud) != 0, 0))
        hxtLoudLoad<FMT, NL>(hxsCold(), st, b, l, lane, sh);
}

// ---- progress counters (LDS) -------------------------------------------------------------
// Inside a block no workgroup barrier is taken.  A producer that is done with item j (a loader with
// load j, a compute wave with group g) adds 1 to the arrival slot arr[j % kHxtSlots] -- lane 0, a
// non-returning ds_add (round 5 first had the last arriver read the sum back and publish a done word:
// the returning atomic's latency behind the LDS queue cost every wave ~1.5k cycles per arrival, 10 %
// of its life in the stamps).  Item j is complete once its slot holds n * (j / kHxtSlots + 1)
// arrivals of its n producers.  Producers finish their items in order, so a complete item also
// means every earlier item is complete, and a waiter checks only the last item it needs: group g
// runs once load P+g-1 is complete (its window: loads 0 .. P+g-1); load j may overwrite ring rows
// once the last group whose window held them is complete (hxtFreeNeed).  A producer runs at most
// (ring slots + 2) items ahead of the slowest one (host check in launchHxs), fewer than kHxtSlots,
// so a slot never holds arrivals of two laps at once and a count never runs past n * (lap + 1).
// A producer arrives after s_waitcnt lgkmcnt(0) (its ring writes / reads done), and LDS executes
// one wave's operations in order, so a waiter that sees the count and then reads the ring sees the
// data.  A waiter polls one dword (broadcast ds_read_b32, s_sleep backoff) -- round 4 polled every
// producer's own counter with two or three ds_read_b128 per poll.
// Waits are bounded (x.pollMax polls): an expired wait means a counting bug, so the wave records
// it in the workgroup's abort word (every later wait of the workgroup returns at once, the grid
// drains) and in the handle's device status word x.err (host-mapped; the C-ABI reports
// GAR_ERR_DEVICE naming hxt_kernel and refuses the handle until Reset) -- never silent output.
typedef __attribute__((address_space(3))) int lds_i32;
constexpr int kHxtSlots = 16;                            // arrival slots per direction
// Explicit LDS pointers: a generic pointer makes the polls flat loads, and a flat load's
// s_waitcnt vmcnt(0) waits for every store the wave has in flight.
struct HxtSync {
    lds_i32* ldArr;   // [kHxtSlots] loader arrivals per load
    lds_i32* cpArr;   // [kHxtSlots] compute-wave arrivals per group
    lds_i32* abort;   // a wait of this workgroup expired (sticky for the launch)
};
// LDS bytes past loudLo (hxsLds reserves them): loudLo[16], loudHi[16], flag, then the counters
// (FMT 5: loudLo[32], loudHi[32], flag)
constexpr int kHxtSyncOff = 160;
__host__ __device__ constexpr int hxtSyncOff(int FMT) { return FMT == 5 ? 288 : kHxtSyncOff; }
constexpr int kHxtSyncBytes = 4 * (2 * kHxtSlots + 1);

// Producer arrival for item j.
__device__ __forceinline__ void hxtArrive(lds_i32* arr, int j, int lane) {
    __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0): this wave's ring writes / reads done
    __atomic_signal_fence(__ATOMIC_SEQ_CST);
    if (lane == 0) (void)__hip_atomic_fetch_add(arr + (j & (kHxtSlots - 1)), 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    __atomic_signal_fence(__ATOMIC_SEQ_CST);
}

__device__ __forceinline__ bool hxtComplete(const lds_i32* arr, int j, int n) {
    return *reinterpret_cast<const volatile lds_i32*>(arr + (j & (kHxtSlots - 1))) >= n * (j / kHxtSlots + 1);
}

// Item j (of n producers) complete, bounded; on expiry the abort word and the handle's status word
// are set.  j < 0: nothing to wait for.
__device__ __forceinline__ void hxtWait(const HxsArgs& x, const HxtSync& sy, const lds_i32* arr, int j, int n, int code,
                                        int lane, unsigned long long* waited = nullptr) {
    if (j < 0) return;
    __atomic_signal_fence(__ATOMIC_SEQ_CST);
    if (hxtComplete(arr, j, n)) return;                                    // the common case: one read
    if (*reinterpret_cast<const volatile lds_i32*>(sy.abort)) return;      // after an expiry: no more waiting
    const unsigned long long t0 = (kHxsDev && waited) ? __builtin_amdgcn_s_memtime() : 0;
    struct Acc {  // development (GAR_HXS_PROF): cycles spent in this wait
        unsigned long long* w;
        unsigned long long t0;
        __device__ ~Acc() { if (kHxsDev && w) *w += __builtin_amdgcn_s_memtime() - t0; }
    } acc{kHxsDev ? waited : nullptr, t0};
    const int pmax = x.pollMax;
    int it = 0;
    for (; it < pmax; ++it) {
        __builtin_amdgcn_s_sleep(1);
        __atomic_signal_fence(__ATOMIC_SEQ_CST);
        if (hxtComplete(arr, j, n)) break;
        if (*reinterpret_cast<const volatile lds_i32*>(sy.abort)) { it = pmax; break; }
    }
    if (it >= pmax) {  // expired (here or in another wave of the workgroup): record, stop waiting
        if (lane == 0) {
            *reinterpret_cast<volatile lds_i32*>(sy.abort) = 1;
            if (x.err) __hip_atomic_store(x.err, code, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        }
    }
    __atomic_signal_fence(__ATOMIC_SEQ_CST);
}

// Groups of a block whose windows a load must not overwrite: load j >= P writes column rows
// [Wg + (j-P)*GQ, + GQ), whose previous occupants (rows - R) belong to groups <= the returned index.
__device__ __forceinline__ int hxtFreeNeed(const HxsArgs& x, int j, int P) {
    const int GQ = x.G * x.Qc;
    const int last = x.Wg + (j - P + 1) * GQ - 1 - x.R;  // highest overwritten row, previous lap
    return last < 0 ? 0 : last / GQ + 1;                 // groups 0 .. last/GQ must be finished
}

// Loader wave l: in step j it waits for the ring rows of load j to be free, converts load j
// (issued kHxtD steps earlier) into the ring, publishes it and issues load j + kHxtD into the
// registers just freed.
// Block b's first window (rows [0, Wg), i.e. loads 0 .. P-1) can come through the buffer records
// (uniform): every column live and the window at or after the raw input's first row.
__device__ __forceinline__ bool hxtStage0Fast(const HxsArgs& x, int b) {
    const int W = x.fmt == 5 ? 32 : 16;
    const bool blockLive = (x.fmt == 1 || x.fmt == 2 || x.fmt == 5) && b * W + W - 1 < x.ncols && x.fastHi > x.fastLo;
    const int64_t row0 = (x.a_lo + static_cast<int64_t>((b * W) / x.C) * x.Np) * x.Qc;
    return blockLive && row0 >= x.fastLo;
}

// Cooperative fill: the compute waves (idle until the first window is in the ring) load and convert
// the block's first window together -- one memory round trip of the whole workgroup -- instead of the
// loaders staging loads 0 .. P-1 one loader step after another (r05 stamps: entry -> first group was
// ~45k cycles, 15 % of a cfg2 workgroup's life).  Items as the loaders' (FMT 1: quad + 64-row piece,
// two chunks of stereo frames; FMT 2: 16-row piece, lane = 16 quad + row), kCoopB in flight per
// wave, each staged through hxsPutItem (split, mirror, loud marking) like the edge gathers.
// Ordered variant (knob GAR_HXT_COOP=2): the compute waves meet the loaders at a first barrier right
// after issuing their first batch; the loaders issue load P only after it and load P + 1 only after the
// window is complete, so the chip's first windows are not queued behind the loaders' loads.
template <int FMT, int kCoopB, bool kOrdered>
__device__ __forceinline__ void hxtCoopStage0(const HxsArgs& x, const HxsShared& sh, int b, int w, int nw, int lane) {
    const HxsArgsP xp = hxsCold();
    const HxsRegSrc rs = hxsRegSrc<FMT>(xp, b, lane);
    HxsStage st;
    st.T0 = 0;
    st.nrow = x.Wg;
    st.fast = true;
    const int Wg = x.Wg;
    const int nit = FMT == 1 ? 4 * ((Wg + 63) >> 6) : FMT == 5 ? (Wg + 7) >> 3 : (Wg + 15) >> 4;
    bool met = !kOrdered;
    for (int it0 = w; it0 < nit; it0 += kCoopB * nw) {
        f32x4 e[kCoopB];
#pragma unroll
        for (int u = 0; u < kCoopB; ++u) {
            const int it = it0 + u * nw;
            const bool on = it < nit;
            if constexpr (FMT == 1) {
                const int q = it & 3, pc = it >> 2;
                const int o = on ? rs.lane0 + 64 * pc * rs.rowB + 2 * q * rs.chunkB : kHxqOob;
                const int o2 = on ? o + rs.chunkB : kHxqOob;
                const f2v a = __builtin_bit_cast(f2v, __builtin_amdgcn_raw_buffer_load_b64(rs.r, o, 0, 0));
                const f2v c = __builtin_bit_cast(f2v, __builtin_amdgcn_raw_buffer_load_b64(rs.r, o2, 0, 0));
                e[u] = f32x4{a.x, a.y, c.x, c.y};
            } else {
                const int o = on ? rs.lane0 + (FMT == 5 ? 8 : 16) * it * rs.rowB : kHxqOob;
                e[u] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(rs.r, o, 0, 0));
            }
        }
        if (!met) {  // first batch issued: let the loaders issue theirs
            hxsBarrier();
            met = true;
        }
#pragma unroll
        for (int u = 0; u < kCoopB; ++u) {
            const int it = it0 + u * nw;
            if (it >= nit) continue;  // uniform
            const int q = FMT == 1 ? (it & 3) : FMT == 5 ? (lane & 7) : (lane >> 4);
            const int row = FMT == 1 ? 64 * (it >> 2) + lane : FMT == 5 ? 8 * it + (lane >> 3) : 16 * it + (lane & 15);
            if (row < Wg) hxsPutItem(xp, st, 0, q, row, e[u], sh.ring, sh.QS, sh.loudLo, sh.loudHi, sh.flag);
        }
    }
    if (!met) hxsBarrier();  // a wave without items still meets the loaders
}

template <int FMT, int NL>
__device__ __forceinline__ void hxtLoaders(const HxsArgs& x, const HxsShared& sh, const HxtSync& sy, int b, int l,
                                           int lane, int coop, unsigned long long* waited) {
    if constexpr (GAR_HXT_LPRIO > 0) __builtin_amdgcn_s_setprio(GAR_HXT_LPRIO);
    const HxsArgsP xp = hxsCold();
    const int GQ = x.G * x.Qc, Wg = x.Wg, R = x.R;
    const int P = (Wg + GQ - 1) / GQ, nL = P + x.ngroups - 1;
    const int nstepsPad = hxsStepsPad(x);
    const int dbg = kHxsDev ? x.dbg : GAR_HXT_CTDBG;
    // per block (uniform): loads go through the buffer records ("fast") when every column of the
    // block is live and the load's first row lies at or after the raw input's first row
    const int c1 = b * hxtCols(FMT) + hxtCols(FMT) - 1;
    const bool blockLive = x.fmt >= 1 && x.fmt <= 5 && c1 < x.ncols && x.fastHi > x.fastLo;
    const int64_t row0 = (x.a_lo + static_cast<int64_t>((b * hxtCols(FMT)) / x.C) * x.Np) * x.Qc;  // column-relative row 0
    const int64_t fastLo = x.fastLo;
    auto stage = [&](int j) {  // load j: the P parts of stage 0, then stages 1 ..
        HxsStage st;
        st.T0 = j < P ? j * GQ : Wg + (j - P) * GQ;
        st.nrow = j < P ? min(GQ, Wg - j * GQ) : GQ;
        st.fast = blockLive && row0 + st.T0 >= fastLo;
        return st;
    };
    HxtBuf<FMT, NL> buf[kHxtD];
    bool fastL[kHxtD];
    const HxsRegSrc rs = hxsRegSrc<FMT>(xp, b, lane);
    // with the cooperative fill the compute waves stage loads 0 .. P-1: the loaders start at P, with
    // its loads in flight across the fill's barrier
    const int jStart = coop ? P : 0;
    if (coop == 2) {
        // ordered fill: load P after the compute waves' first window batch, load P + 1 after the window
        hxsBarrier();
        fastL[0] = hxtIssue<FMT, NL>(stage(jStart), jStart < nL, rs, l, buf[0]);
        hxsBarrier();  // the first window is in the ring
#pragma unroll
        for (int d = 1; d < kHxtD; ++d) fastL[d] = hxtIssue<FMT, NL>(stage(jStart + d), jStart + d < nL, rs, l, buf[d]);
    } else {
#pragma unroll
        for (int d = 0; d < kHxtD; ++d) fastL[d] = hxtIssue<FMT, NL>(stage(jStart + d), jStart + d < nL, rs, l, buf[d]);
        if (coop) hxsBarrier();  // the first window is in the ring (no vector-memory wait: the loads stay in flight)
    }
    // ring row of load j's first row (incremental: T0 % R) and the groups its rows' previous
    // occupants belong to (hxtFreeNeed, incremental)
    int p0 = coop ? Wg : 0, last = Wg + GQ - 1 - R, need = 0;
    for (int j0 = jStart; j0 < nstepsPad; j0 += kHxtD) {
#pragma unroll
        for (int d = 0; d < kHxtD; ++d) {
            const int j = j0 + d;
            if (j < nL) {
                if (j >= P) {
                    if (j == P) p0 = Wg;  // Wg < R
                    need = last < 0 ? 0 : need + 1;
                    if (need > 0 && !(dbg & 64)) hxtWait(x, sy, sy.cpArr, need - 1, x.ncomp, kHxtErrSlotWait, lane, waited);  // development 64: loaders never wait
                    last += GQ;
                }
                // development (GAR_HXS_PROF): loader phases of the first block -- waited[3] load data
                // (an explicit vmcnt wait for this load's instructions), [4] conversion, [5] arrival
                const bool stp = kHxsDev && waited;
                unsigned long long t1 = stp ? __builtin_amdgcn_s_memtime() : 0;
                if (stp && fastL[d]) {
                    constexpr int kNewer = (FMT == 1 ? 2 : 1) * hxtItems<NL>() * (kHxtD - 1);  // younger loads' instructions
                    static_assert(kNewer < 64, "vmcnt field");
                    __builtin_amdgcn_s_waitcnt((kNewer & 15) | (7 << 4) | (15 << 8) | ((kNewer >> 4) << 14));
                    const unsigned long long t2 = __builtin_amdgcn_s_memtime();
                    waited[3] += t2 - t1;
                    t1 = t2;
                }
                if (!((dbg & 16) && j >= P)) {
                    const HxsStage st = stage(j);
                    if (fastL[d]) hxtConvert<FMT, NL>(x, st, uni(p0), buf[d], b, l, lane, sh);
                    else hxtGatherLoad<hxtQuads(FMT)>(xp, st, b, l, NL, lane, sh);
                }
                unsigned long long t3 = stp ? __builtin_amdgcn_s_memtime() : 0;
                if (stp) waited[4] += t3 - t1;
                hxtArrive(sy.ldArr, j, lane);
                if (stp) waited[5] += __builtin_amdgcn_s_memtime() - t3;
                p0 += GQ;
                if (p0 >= R) p0 -= R;
            }
            fastL[d] = hxtIssue<FMT, NL>(stage(j + kHxtD), j + kHxtD < nL && !((dbg & 1) && j >= P), rs, l, buf[d]);
        }
    }
}

// Workgroup slot -> block.  x.xcdPair 2 (FMT 5): chunk-major -- slot i runs block (i % 8) * (nblocks / 8) +
// i / 8, so every channel group of a few consecutive chunks runs on one XCD (the dispatcher deals slots
// round-robin over the 8 XCDs) and the 1-KB rows of those chunks are read and written together.
__device__ __forceinline__ int hxtBlock(const HxsArgs& x, int i) {
    if (x.xcdPair == 2) return (i & 7) * (x.nblocks >> 3) + (i >> 3);
    return hxsBlock(x, i);
}

// ---- compute waves ----------------------------------------------------------------------
// Group g: wait for its window, run this wave's periods p = first, first + st, ... < end
// (chunk-relative), publish.  One accumulator pair per period: with three compute waves per SIMD
// the other waves cover a period's MFMA drain before its epilogue.
// Stereo frame-pair stores (VST 2) of the fast epilogue as non-temporal stores (GAR_HXT_NTST2): the same
// DPP frame-pair swap and 16-B store as hxsStoreFast<2>, with the nt cache policy.  In the headline's
// memory pattern with no compute (tools/ubench/stereo_copy.hip, profiles/r06x4_stereo_copy_nt.txt) the
// read and write streams together run at 4.77 TB/s with plain stores and 6.03 TB/s with nt stores.
#ifndef GAR_HXT_NTST2
#define GAR_HXT_NTST2 1
#endif
__device__ __forceinline__ void hxtStoreStereoNt(char* p, const f32x4& y, int lane) {
    const bool even = (lane & 1) == 0;
    const float s0 = even ? y[2] : y[0], s1 = even ? y[3] : y[1];
    const float q0 = __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(s0), 0xB1, 0xf, 0xf, false));
    const float q1 = __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(s1), 0xB1, 0xf, 0xf, false));
    f32x4 w;
    if (even) { w[0] = y[0]; w[1] = q0; w[2] = y[1]; w[3] = q1; }
    else      { w[0] = q0; w[1] = y[2]; w[2] = q1; w[3] = y[3]; }
    __builtin_nontemporal_store(w, reinterpret_cast<f32x4*>(p));
}

// NT tiles per period (FMT 5: 2, the block's two 16-column halves, quads 4h .. 4h+3 of the ring and
// channels ccol + 16h of the output; one accumulator pair per tile and period, in tile order).
template <int NS, int VST, bool FAST, int NT = 1>
__device__ __forceinline__ void hxtGroups(const HxsArgs& x, const HxsShared& sh_, const HxtSync& sy, int wt, int lane,
                                          const h8v (&Ah)[NS], const h8v (&Al)[NS], uint32_t laneOff, int u0, int P,
                                          int nslot, const HxtRole& ro, char* obase, int64_t pstride, int64_t aCol,
                                          int64_t oRow0, bool colOk, int ccol, bool fullRb, int nl, unsigned long long* st) {
    // st (development, GAR_HXS_PROF): [0] cycles waiting for loads, [1] first group's start, [2] last group's end
    const int sh = -(x.ea + kHxXs);
    const int GQ = x.G * x.Qc;
    const uint32_t dL = 8u * static_cast<uint32_t>(x.Rt);
    const uint32_t pst = 8u * static_cast<uint32_t>(x.Qc) * static_cast<uint32_t>(ro.st);
    const int dbg = kHxsDev ? x.dbg : GAR_HXT_CTDBG;
    const uint32_t tileLds = 4u * sh_.QS;                             // ring bytes between tiles
    const int64_t tileOut = 16 * x.out_cs;                             // output bytes between tiles
    auto epilogue = [&](const f32x4& oA, const f32x4& oL, int p, int h) {
        const f32x4 y = hxScale(oA, oL, sh);
        if (dbg & 2) return;
        if constexpr (FAST && VST == 2 && GAR_HXT_NTST2) {
            hxtStoreStereoNt(obase + static_cast<int64_t>(p) * pstride, y, lane);
        } else if constexpr (FAST) {
            hxsStoreFast<VST>(x, obase + static_cast<int64_t>(p) * pstride + h * tileOut, y, lane);
        } else {
            const int ccol_ = ccol + 16 * h;
            const int64_t a = aCol + p;
            const int64_t o0 = a * x.Pc + oRow0;
            const bool live = colOk && a < x.a_hi;
            if (fullRb && live && a * x.Pc >= x.o_lo && (a + 1) * x.Pc <= x.o_hi) {
                char* pp = x.out + (o0 + ((VST == 2 && (lane & 1)) ? 2 : 0)) * x.out_fs + (VST == 2 ? 0 : ccol_ * x.out_cs);
                hxsStoreFast<VST>(x, pp, y, lane);
            } else if (live) {
#pragma unroll
                for (int i = 0; i < 4; ++i) {
                    const int64_t o = o0 + i;
                    if (oRow0 + i < x.Pc && o >= x.o_lo && o < x.o_hi)
                        *reinterpret_cast<float*>(x.out + o * x.out_fs + ccol_ * x.out_cs) = y[i];
                }
            }
        }
    };
    int first = ro.ph;  // first period of group 0 with p % st == ph
    for (int g = 0; g < x.ngroups; ++g) {
        const int p0 = g * x.G;
        const int pend = min(p0 + x.G, x.Np);
        while (first < p0) first += ro.st;
        const int n = first >= pend ? 0 : (pend - first + ro.st - 1) / ro.st;
        if (n > 0) {
            if (!(dbg & 32)) hxtWait(x, sy, sy.ldArr, P + g - 1 + x.faultNeed, nl, kHxtErrLoadWait, lane, st);  // loads 0 .. P+g-1 in the ring (development 32: no wait)
            if (kHxsDev && st) {
                const unsigned long long tg = __builtin_amdgcn_s_memtime();
                if (st[1] == 0) st[1] = tg;
                st[5] = tg;  // this group's compute starts
            }
            // the lane's ring offset, recomputed per group (a value held across the group loop spills,
            // and its reload's vmcnt(0) would wait for this wave's output stores)
            int ln = lane;
            asm volatile("" : "+v"(ln));
            const uint32_t lo = ((ln & 15) & 3) * sh_.QS + 8u * (4 * (ln >> 4) + ((ln & 15) >> 2));
            uint32_t aH = static_cast<uint32_t>(reinterpret_cast<uintptr_t>((lds_s4p)(sh_.ring))) + lo + 8u * static_cast<uint32_t>(u0) +
                          8u * static_cast<uint32_t>((g % nslot) * GQ) + 8u * static_cast<uint32_t>(x.Qc) * static_cast<uint32_t>(first - p0);
            h8v bh0 = (dbg & 8) ? h8v{} : bFragA(aH), bl0 = (dbg & 8) ? h8v{} : bFragA(aH + dL);  // development 8: no B reads
            for (int i = 0; i < n; ++i) {
#pragma unroll
              for (int h = 0; h < NT; ++h) {
                asm volatile("" : "+v"(aH));  // opaque per-period base: reads use base + offset:imm
                const bool last = i + 1 == n && h + 1 == NT;
                uint32_t aL = aH + dL;
#if GAR_HXT_LOBASE
                asm volatile("" : "+v"(aL));  // lo-row base kept apart: lo reads use aL + offset:imm (no per-step add of dL)
#endif
                // next tile: the other half of this period, or the next period's first tile
                const uint32_t aN = h + 1 < NT ? aH + tileLds : aH - (NT - 1) * tileLds + pst, aNL = aN + dL;
                f32x4 nA = {0, 0, 0, 0}, nL = nA;
#pragma unroll
                for (int s = 0; s < NS; ++s) {
                    const int ug = (s + 1) / NS, us = (s + 1) % NS;
                    h8v bhn = bh0, bln = bl0;
                    if (!(ug == 1 && last) && !(dbg & 8)) {
                        bhn = bFragA((ug == 0 ? aH : aN) + 256 * us);
                        bln = bFragA((ug == 0 ? aL : aNL) + 256 * us);
                    }
                    if (!(dbg & 4)) {
                        nA = mfma16(Ah[s], bh0, nA);
                        nA = mfma16(Al[s], bh0, nA);
                        nL = mfma16(Ah[s], bl0, nL);
                    }
                    bh0 = bhn;
                    bl0 = bln;
                    __builtin_amdgcn_sched_group_barrier(0x100, 4, 0);
                    __builtin_amdgcn_sched_group_barrier(0x008, 3, 0);
                    __builtin_amdgcn_sched_barrier(0);
                }
                epilogue(nA, nL, first + i * ro.st, h);
                aH = aN;
              }
            }
        }
        const unsigned long long ta = (kHxsDev && st) ? __builtin_amdgcn_s_memtime() : 0;
        if (kHxsDev && st && n > 0) st[3] += ta - st[5];  // the group's periods (B reads, MFMA, epilogues)
        hxtArrive(sy.cpArr, g, lane);  // this wave's reads of group g's window are done
        if (kHxsDev && st) st[4] += __builtin_amdgcn_s_memtime() - ta;
    }
    if (kHxsDev && st) st[2] = __builtin_amdgcn_s_memtime();
}

template <int NS, int VST, int FMT>
__device__ __forceinline__ void hxtCompute(const HxsArgs& x, const HxsShared& sh_, const HxtSync& sy, int b, int wt,
                                           int lane, int nl, int coop, unsigned long long* st) {
    // A of the wave's row block (kept in registers only inside this role: the loaders' registers
    // are the load buffers)
    if constexpr (GAR_HXT_CPRIO > 0) __builtin_amdgcn_s_setprio(GAR_HXT_CPRIO);
    const HxtRole ro = hxtRole(x, wt);
    const int* pt = x.progs + kBgProgInts * ro.rb;
    const int u0 = uni(pt[4]), rbw = uni(pt[3]);
    h8v Ah[NS], Al[NS];
#pragma unroll
    for (int i = 0; i < NS; ++i) {
        Ah[i] = x.A[((static_cast<size_t>(ro.rb) * NS + i) * 2 + 0) * 64 + lane];
        Al[i] = x.A[((static_cast<size_t>(ro.rb) * NS + i) * 2 + 1) * 64 + lane];
    }
    if (kHxsDev && st) st[6] = __builtin_amdgcn_s_memtime();
    if (coop) {  // the block's first window, staged by every compute wave (A lands meanwhile)
        if (coop == 2) hxtCoopStage0<FMT, 4, true>(x, sh_, b, wt, x.ncomp, lane);
        else hxtCoopStage0<FMT, 4, false>(x, sh_, b, wt, x.ncomp, lane);
        hxsBarrier();
    }
    if (kHxsDev && st) st[7] = __builtin_amdgcn_s_memtime();
    const uint32_t QS = sh_.QS;
    const int GQ = x.G * x.Qc;
    const int grp = lane >> 4, l16 = lane & 15;
    const uint32_t laneOff = (l16 & 3) * QS + 8u * (4 * grp + (l16 >> 2));
    const bool fullRb = (rbw + 1) * 16 <= x.Pc;
    const int nslot = x.R / GQ;
    const int P = (x.Wg + GQ - 1) / GQ;
    const int64_t pstride = static_cast<int64_t>(x.Pc) * x.out_fs;
    const int col = b * hxtCols(FMT) + l16;  // FMT 5: tile 0's column (tile 1: + 16, the same chunk as C % 32 == 0)
    const bool colOk = col < x.ncols;
    const int kcol = col / x.C, ccol = col - kcol * x.C;
    const int64_t aCol = x.a_lo + static_cast<int64_t>(kcol) * x.Np;
    const int64_t oRow0 = static_cast<int64_t>(rbw) * 16 + 4 * grp;  // first row of this lane's accumulator
    const bool laneFast = fullRb && colOk && aCol + x.Np <= x.a_hi && aCol * x.Pc >= x.o_lo &&
                          (aCol + x.Np) * x.Pc <= x.o_hi;
    char* obase = x.out + (aCol * x.Pc + oRow0 + ((VST == 2 && (lane & 1)) ? 2 : 0)) * x.out_fs +
                  (VST == 2 ? 0 : ccol * x.out_cs);
    constexpr int NT = FMT == 5 ? 2 : 1;
    if (__builtin_amdgcn_ballot_w64(!laneFast) == 0)
        hxtGroups<NS, VST, true, NT>(x, sh_, sy, wt, lane, Ah, Al, laneOff, u0, P, nslot, ro, obase, pstride, aCol, oRow0,
                                     colOk, ccol, fullRb, nl, st);
    else
        hxtGroups<NS, VST, false, NT>(x, sh_, sy, wt, lane, Ah, Al, laneOff, u0, P, nslot, ro, obase, pstride, aCol, oRow0,
                                      colOk, ccol, fullRb, nl, st);
}

// FMT: 1 stereo f32 frames, 2 rows of 16 f32 channels.  VST: 0 any f32 layout, 1 channel-contiguous
// f32, 2 stereo-interleaved f32 (hxsStoreFast).
template <int NS, int FMT, int VST, int NL>
__global__ __launch_bounds__(64 * kHxtWaves) void hxt_kernel(HxsArgs x) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    HxsShared s;
    s.stamp = nullptr;
    s.QS = 16u * static_cast<uint32_t>(x.Rt) + 64u;  // quad: hi rows, lo rows, +64 B skew
    s.ring = reinterpret_cast<char*>(smem);
    constexpr int NQ = hxtQuads(FMT), NC = hxtCols(FMT);
    s.loudLo = reinterpret_cast<int*>(smem + NQ * static_cast<size_t>(s.QS));  // 16-B aligned (QS % 16 == 0)
    s.loudHi = s.loudLo + NC;
    s.flag = s.loudHi + NC;
    HxtSync sy;
    // kHxtSyncOff(FMT) B past loudLo (hxsLds reserves the space past the ring): arrival slots, done counters, abort
    sy.ldArr = (lds_i32*)(smem + NQ * static_cast<size_t>(s.QS) + hxtSyncOff(FMT));
    sy.cpArr = sy.ldArr + kHxtSlots;
    sy.abort = sy.cpArr + kHxtSlots;
    const int lane = threadIdx.x & 63;
    const int wt = uni(threadIdx.x >> 6);
    const bool comp = wt < x.ncomp;
    if (threadIdx.x == 0) *sy.abort = 0;  // sticky for the launch (ordered by the first block's barriers)
    // development (GAR_HXS_PROF): wave 0 (compute) and the first loader stamp their first block
    const bool stampW = kHxsDev && x.prof && lane == 0 && (wt == 0 || wt == x.ncomp);
    const unsigned long long tEntry = stampW ? __builtin_amdgcn_s_memtime() : 0;
    const unsigned long long rEntry = stampW ? __builtin_amdgcn_s_memrealtime() : 0;
    unsigned long long st[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    unsigned long long tBlockEnd = 0;
    for (int bi = blockIdx.x; bi < x.nblocks; bi += gridDim.x) {
        const int b = hxtBlock(x, bi);
        __syncthreads();  // the previous block's ring reads and fixup done
        if (threadIdx.x < NC) {
            s.loudLo[threadIdx.x] = INT_MAX;
            s.loudHi[threadIdx.x] = -1;
        }
        // cooperative fill (knob x.coop, GAR_HXT_COOP: 2 ordered (default), 1 unordered, 0 off): loads
        // 0 .. P-1 complete once the fill's barrier passes
        const int GQb = x.G * x.Qc, Pb = (x.Wg + GQb - 1) / GQb;
        const int coop = hxtStage0Fast(x, b) ? x.coop : 0;  // 0 loaders stage the first window, 1 / 2 the compute waves
        if (threadIdx.x < 2 * kHxtSlots) sy.ldArr[threadIdx.x] = (coop && static_cast<int>(threadIdx.x) < Pb) ? NL : 0;  // arrival slots
        if (threadIdx.x == 64) *s.flag = 0;
        __syncthreads();
        const bool first = bi == static_cast<int>(blockIdx.x);
        unsigned long long* stp = (stampW && first) ? st : nullptr;
        if (comp) hxtCompute<NS, VST, FMT>(x, s, sy, b, wt, lane, NL, coop, stp);
        else hxtLoaders<FMT, NL>(x, s, sy, b, wt - x.ncomp, lane, coop, stp);
        if (stampW && first) tBlockEnd = __builtin_amdgcn_s_memtime();
        __syncthreads();  // every wave's part of the block done; flag final
        if (*s.flag) {  // uniform
            __builtin_amdgcn_s_waitcnt(0);  // this wave's output stores landed
            __syncthreads();
            hxsFixup(hxsCold(), (NC / 16) * b, s.loudLo, s.loudHi);
            if constexpr (NC == 32) hxsFixup(hxsCold(), 2 * b + 1, s.loudLo + 16, s.loudHi + 16);
        }
    }
    if (x.hn > 0) hxsHistKeep(x, static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x,
                              static_cast<int64_t>(gridDim.x) * blockDim.x);
    if (stampW) {  // development: role cycles of the first block, fill / drain, workgroup life, launch span
        __builtin_amdgcn_s_waitcnt(0);
        const unsigned long long tExit = __builtin_amdgcn_s_memtime(), rExit = __builtin_amdgcn_s_memrealtime();
        if (wt == 0) {
            atomicAdd(x.prof + 30, tBlockEnd - tEntry);
            atomicAdd(x.prof + 32, st[0]);
            atomicAdd(x.prof + 37, st[3]);
            atomicAdd(x.prof + 38, st[4]);
            atomicAdd(x.prof + 34, 1ull);
            atomicAdd(x.prof + 35, st[1] ? st[1] - tEntry : 0ull);  // entry -> first group runs (fill)
            atomicAdd(x.prof + 36, tExit - (st[2] ? st[2] : tExit));  // last group done -> exit (drain)
            atomicAdd(x.prof + 53, st[6] - tEntry);  // fill parts: entry -> A issued
            atomicAdd(x.prof + 54, st[7] - st[6]);  // -> cooperative fill's barrier passed
            atomicAdd(x.prof + 55, st[1] ? st[1] - st[7] : 0ull);  // -> first group runs
            atomicAdd(x.prof + 56, tExit - tEntry);  // in-kernel clock: memtime / memrealtime x 100 MHz
            atomicAdd(x.prof + 57, rExit - rEntry);
            atomicMin(x.prof + 10, rEntry);
            atomicMax(x.prof + 11, rExit);
            if (blockIdx.x < 4096) { x.prof[64 + 2 * blockIdx.x] = rEntry; x.prof[65 + 2 * blockIdx.x] = rExit - rEntry; }
        } else {
            atomicAdd(x.prof + 31, tBlockEnd - tEntry);
            atomicAdd(x.prof + 33, st[0]);
            atomicAdd(x.prof + 50, st[3]);
            atomicAdd(x.prof + 51, st[4]);
            atomicAdd(x.prof + 52, st[5]);
        }
    }
}

template <int NS, int FMT, int VST, int NL>
hipError_t hxtLaunch(const HxsArgs& x, size_t lds, int64_t blocks, hipStream_t st) {
    if (x.ncomp + NL > kHxtWaves) return hipErrorInvalidConfiguration;
    if (const size_t lim_ = setMaxLdsOnce(reinterpret_cast<const void*>(&hxt_kernel<NS, FMT, VST, NL>)); lim_ < lds) return ldsTooBig("hxt_kernel", lds, lim_);
    hipLaunchKernelGGL((hxt_kernel<NS, FMT, VST, NL>), dim3(static_cast<unsigned>(blocks)), dim3(64 * (x.ncomp + NL)), lds,
                       st, x);
    return hipGetLastError();
}

#define GAR_HXT_FOR3(M, NS) M(NS, 1, 2, 4) M(NS, 2, 0, 4) M(NS, 2, 1, 4) M(NS, 1, 2, 6) M(NS, 2, 0, 6) M(NS, 2, 1, 6) \
    M(NS, 5, 0, 4) M(NS, 5, 0, 6)
#if GAR_HXS_QUICK
#define GAR_HXT_FOR_A(M) GAR_HXT_FOR3(M, 9)
#define GAR_HXT_FOR_B(M) GAR_HXT_FOR3(M, 10)
#else
#define GAR_HXT_FOR_A(M) GAR_HXT_FOR3(M, 1) GAR_HXT_FOR3(M, 2) GAR_HXT_FOR3(M, 3) GAR_HXT_FOR3(M, 4) GAR_HXT_FOR3(M, 5) \
    GAR_HXT_FOR3(M, 6) GAR_HXT_FOR3(M, 7)
#define GAR_HXT_FOR_B(M) GAR_HXT_FOR3(M, 8) GAR_HXT_FOR3(M, 9) GAR_HXT_FOR3(M, 10)
#endif
#define GAR_HXT_INST(NS, F, V, L) template hipError_t hxtLaunch<NS, F, V, L>(const HxsArgs&, size_t, int64_t, hipStream_t);

}  // namespace gar
