// gar_kernels.hpp -- device-side descriptors and launchers (gar_kernels.hip).
#pragma once
#include <string>
#include <hip/hip_runtime.h>

#include <cstdint>
#include <vector>

namespace gar {

// A channel group's input stream seen by a kernel: the retained history
// (compute dtype, interleaved [t][C] with row stride hist_ld) virtually
// concatenated with the caller's new input (any strides, f32 or f64), and
// zero beyond valid_end -- the zero padding that DFTStage/PolyphaseStage/
// DFTDecimationStage.Flush append (dft_stage.go:347, :582,
// polyphase_stage.go:342) never has to be materialised.
struct SrcDesc {
    const void* hist;
    int64_t hist_base, hist_len, hist_ld;
    const void* in;
    int64_t in_base, in_len, in_fs, in_cs;
    int in_f64;
    int in_pcm;            // 0 float input, else PCM bits (16: int16, 24/32: int32 storage)
    int64_t valid_end;
};

// Output view: element (o, c) -> out[(o - o0) * fs + c * cs]; only o in [o_lo, o_hi) written.
struct OutDesc {
    void* out;
    int64_t o0, fs, cs;
    int f64;
    int pcm;               // 0 float output, else PCM bits (int(clamp(y, -1, 1) * maxVal))
    int64_t o_lo, o_hi;
    int* err;              // the calling handle's device status word (host-mapped), null if none
};

// Integer PCM <-> float, after cmd/resample-wav/main.go:444-543 (maxInt16/24/32, main.go:54-56):
// in = float64(i) * (1 / maxVal); out = int(clamp(float64(y), -1, 1) * maxVal), truncating.
__host__ __device__ inline double pcmMax(int bits) {
    return bits == 16 ? 32767.0 : (bits == 24 ? 8388607.0 : 2147483647.0);
}
__host__ __device__ inline int pcmBytes(int bits) { return bits == 16 ? 2 : 4; }
__host__ __device__ inline double pcmToF64(int32_t i, int bits) { return static_cast<double>(i) * (1.0 / pcmMax(bits)); }
__host__ __device__ inline double pcmRead(const void* p, int64_t e, int bits) {
    return bits == 16 ? pcmToF64(static_cast<const int16_t*>(p)[e], 16) : pcmToF64(static_cast<const int32_t*>(p)[e], bits);
}
__host__ __device__ inline void pcmWrite(void* p, int64_t e, int bits, double y) {
    const double v = y > 1.0 ? 1.0 : (y < -1.0 ? -1.0 : y);  // NaN passes through as in Go, then converts
    const double s = v * pcmMax(bits);
    if (bits == 16) static_cast<int16_t*>(p)[e] = static_cast<int16_t>(s == s ? static_cast<int32_t>(s) : 0);
    else static_cast<int32_t*>(p)[e] = s == s ? static_cast<int32_t>(s) : 0;
}

struct HxDev;

// Device status codes a kernel writes into the handle's status word (OutDesc::err):
// hxt_kernel (gar_hxt.hpp hxtWait) -- 1 a compute wave's load-progress wait expired, 2 a loader's
// ring-slot wait expired.
constexpr int kHxtErrLoadWait = 1, kHxtErrSlotWait = 2;

// A launch whose configuration the device cannot run (dynamic LDS above the kernel's limit): the
// launcher records what was exceeded here and returns hipErrorInvalidConfiguration; the C-ABI turns
// it into GAR_ERR_INVALID_ARGUMENT with this message (gar_engine.cpp wrap).
std::string& launchLimitMsg();
hipError_t ldsTooBig(const char* kernel, size_t need, size_t limit);

// Device copy of a BgPlan (gar_plan.hpp).
struct BgDev {
    int f64;
    int Pc, Qc, Kc, Kread, NS, nrb;
    int nprog, kch, nw, ncg, nred, nslots;
    const void* A;      // [nprog][kch*NS][64]
    const int* progs;   // [nprog][kBgProgInts] (gar_plan.hpp BgPlan::progTable)
    const int* reds;    // [nred][kBgRedInts]
    const HxDev* hx;    // host pointer: split-f16 variant of this plan (f32 compute) or null
    int rbAligned;      // BgPlan::rbAligned: small launches may run bg_rb_kernel
    int maxPrb;         // most programs of one row block
    const int* rbStart; // [nrb + 1]
    const int* hRbStart; // host copies (bg_rb_kernel passes them by value): [nrb + 1]
    const int* hRbK0;    // first input row of each program [nprog]
    // exact recompute of outputs whose real window holds a non-finite sample (gar_bg.hpp bgNfFixOne):
    // the macro period's f64 rows and, for DFT x2 (*) polyphase composites, each row's polyphase
    // phase / DFT parity and the two stages' banks (the reference's two-stage order)
    const double* xRows;   // [Pc][xRowMax]
    const int* xInfo;      // [4][Pc]: window offset, length, polyphase phase, DFT parity
    int xRowMax, xTwoStage, xT1, xT2;
    const double* xPolyA;  // [L][T2]
    const double* xDftC;   // [2][T1]
    int* nfList;           // bg_kernel's non-finite fix list (gar_bg.hpp kBgNfInts ints, zeroed)
};
constexpr size_t kBgNfListBytes = 4 * (2 + 256 * 129 + 1);  // gar_bg.hpp kBgNfInts (static_assert there)

// Device copy of an HxPlan (gar_plan.hpp): split-f16 MFMA FIR, f32 compute.
struct HxDev {
    int Pc, Qc, Kc, Kread, NS, nrb;
    int nw, kch, nred, nslots, ea, rowMax;
    int rb;              // row-block mode (HxPlan::rbMode)
    const void* A;       // [nw][kch*NS][2][64][8] f16
    const int* progs;    // [nw][kBgProgInts] (HxPlan::progTable)
    const int* reds;     // [nred][kBgRedInts]
    // exact fallback of outputs whose windows hold a loud element: !(|x| < kHxLoud = 16 - 2^-8), Inf, NaN
    const double* rows;  // [Pc][rowMax] FIR rows (f64)
    const int* rowOff;   // [Pc]
    const int* rowLen;   // [Pc]
    int twoStage;        // rows are DFT x2 (*) polyphase composites (HxPlan::twoStage)
    int T1, T2;          // DFT taps per phase, polyphase taps per phase
    const int* rowPh;    // [Pc] polyphase phase of each composite row
    const int* rowPar;   // [Pc] DFT output parity of each composite row
    const double* polyA; // [L][T2]
    const double* dftC;  // [2][T1]
    int* fix;            // [1 + fixCap]: interior blocks holding loud elements (count first)
    int fixCap;
    int hxsOk;           // host: the plan fits hxs_kernel (hxsPlanFits), so fused PCM I/O can use it
    int hU0[16], hRbw[16];  // host copies of each row-block program's first row / row block (rb mode, nw <= 16)
};

// General polyphase stage with live cubic coefficient interpolation
// (polyphase_stage.go:257-293): output m uses at = at0 + m*step (local).
struct PolyDev {
    int f64;
    int L, T;
    int64_t step, at0, u_base;  // u_base = global stream index of local history index 0
    int64_t m0;                 // the stage's absolute output index of the launch's first output (tap rotation)
    const void *a, *b, *c, *d;  // [L][T] reversed, compute dtype
    const void* abcd;           // [L][T][4] the same four banks interleaved (poly_kernel's one-load tap)
};

// CubicStage checkpoint (cubic.go:42-61): before input i (absolute stage-input
// index) the phase is `phase` and the next output index is o.  Checkpoints are
// kCubicSegInputs inputs apart.
struct CubicSeg {
    double phase;
    int64_t o, i;
};
constexpr int64_t kCubicSegInputs = 256;
constexpr int kCubicSegInputsShort = 16;  // segment of short calls (closed-form walks only)

// Launchers (all asynchronous on `stream`).  Return hipSuccess or the launch error.
// Optional history keep folded into a streaming FIR launch: dst[(t - t0) * C + c] = src(t, c) for
// t in [t0, t0 + n) (what launchGather does), written by the launch's workgroups after their
// blocks; `done` set when the launch took it (hxs_kernel only), else the caller gathers.
struct HistCopy {
    void* dst = nullptr;
    int64_t t0 = 0, n = 0;
    bool done = false;
};

hipError_t launchBg(const BgDev& p, const SrcDesc& src, const OutDesc& out, int C, hipStream_t stream,
                    HistCopy* hc = nullptr);
hipError_t launchHx(const HxDev& p, const SrcDesc& src, const OutDesc& out, int C, hipStream_t stream,
                    HistCopy* hc = nullptr);
// True when a row-block plan fits launchHxs's geometry at one period per group (its smallest
// ring), i.e. launchHxs never returns hipErrorNotSupported for it (gar_hxs.hip).
bool hxsPlanFits(const HxDev& p);
// Streaming wave-specialised variant of launchHx for row-block plans (gar_hxs.hip).
hipError_t launchHxs(const HxDev& p, const SrcDesc& src, const OutDesc& out, int C, hipStream_t stream,
                     HistCopy* hc = nullptr);
hipError_t launchPoly(const PolyDev& p, const SrcDesc& src, const OutDesc& out, int64_t nout, int C,
                      hipStream_t stream);
// CubicStage outputs of nseg checkpointed segments (segs readable by the device:
// pinned host or device memory); x_end = one past the last input; step = 1/ratio.
hipError_t launchCubic(int f64, const CubicSeg* segs, int64_t nseg, int64_t x_end, double step, const SrcDesc& src,
                       const OutDesc& od, int C, hipStream_t stream, int segLen = static_cast<int>(kCubicSegInputs));
// dst[(t - t0) * C + c] = src(t, c) for t in [t0, t0 + n): history compaction / materialisation.
hipError_t launchGather(int f64, const SrcDesc& src, void* dst, int64_t t0, int64_t n, int C, hipStream_t stream);
// Strided copy with dtype conversion (pass-through stages, group split).
hipError_t launchCopy(const void* src, int src_f64, int64_t s_fs, int64_t s_cs, void* dst, int dst_f64,
                      int64_t d_fs, int64_t d_cs, int64_t n, int C, hipStream_t stream);
// PCM staging of the non-fused paths: type codes 0 f32, 1 f64, 16/24/32 PCM (pcmRead / pcmWrite).
hipError_t launchConvert(const void* src, int s_type, int64_t s_fs, int64_t s_cs, void* dst, int d_type, int64_t d_fs,
                         int64_t d_cs, int64_t n, int C, hipStream_t stream);

}  // namespace gar
