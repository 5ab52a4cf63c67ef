// gar_plan.hpp -- turns a resampling stage into a periodic FIR description and
// then into a banded-GEMM plan for the MFMA kernel (gar_kernels.hip).
//
// Every x==0 stage of the reference engine is a periodic FIR:
//     y[o] = sum_k v[s(o) + k] * G_{o mod P}[k],   s(a*P + r) = a*Q + off[r]
//   * DFT x factor f      (dft_stage.go:229-273):        P=f, Q=1,  off=0,  G_p = polyCoeffs[p]
//   * integer decimator   (dft_stage.go:525-534):        P=1, Q=f,  off=0,  G = reversed coeffs
//   * polyphase, frac==0  (polyphase_stage.go:257-293):  P=L/g, Q=S/g, off=floor(r*S/L), G=a[r*S mod L]
//   * fused DFTx2 -> polyphase (frac==0): the two linear stages composed into
//     one FIR over the *input* stream: P=2L/g2, Q=S/g2 (g2=gcd(S,2L)).
// The MFMA kernel computes blocks of 16 consecutive outputs ("row blocks") for
// 16 columns at a time as D(16x16) = A(16xK) * B(Kx16), A = the banded
// coefficient rows (constant), B = 16 input windows staged in LDS.
#pragma once
#include <cstdint>
#include <vector>

#include "gar_design.hpp"

namespace gar {

struct FirPeriodic {
    int P = 0, Q = 0;                 // outputs / inputs per period
    std::vector<int64_t> off;         // [P] input offset of output r within the period
    std::vector<std::vector<double>> rows;  // [P] coefficient row (multiplies v[s+k])
    // composite rows only (firComposite): row r = polyphase phase ph[r] of the DFT
    // output stream starting at parity par[r]
    bool composite = false;
    std::vector<int> ph, par;
};

FirPeriodic firFromDft(const DftBank& d);
FirPeriodic firFromDecim(const DecimBank& d);
bool firFromPoly(const PolyBank& p, FirPeriodic& out);                          // needs fracFree()
bool firComposite(const DftBank& d, const PolyBank& p, FirPeriodic& out);       // needs factor 2 + fracFree()

// Wave program = the MFMA steps one wavefront runs per macro period: up to 3
// segments, each a contiguous K range of one row block.  The total step count
// of all row blocks is split evenly over the programs so every SIMD carries
// the same MFMA load; a row block cut across programs is finished by an LDS
// reduction of its partial accumulators (slot >= 0).  A program longer than
// the register budget runs as kch chunks of NS steps (A re-read per chunk).
constexpr int kBgMaxSeg = 3;
constexpr int kBgMaxRedSlots = 16;
constexpr int kBgProgInts = 16;                    // device table stride
constexpr int kBgRedInts = 2 + kBgMaxRedSlots;

struct BgSeg { int rb = 0, k0 = 0, ns = 0, start = 0, slot = -1; };
struct BgProg { int nseg = 0, len = 0; BgSeg seg[kBgMaxSeg]; };
struct BgRed { int rb = 0, n = 0; int slot[kBgMaxRedSlots] = {}; };

// Register budget of the kernel instantiation for NS steps -> the largest
// workgroup it may be launched with (__launch_bounds__).  Overheads measured
// with -Rpass-analysis=kernel-resource-usage (no spills at these bounds).
constexpr int bgMaxThreads(bool f64, int NS) {
    return f64 ? (2 * NS + 140 <= 128 ? 1024 : (2 * NS + 140 <= 168 ? 768 : 512))
               : (NS + 92 <= 128 ? 1024 : (NS + 92 <= 168 ? 768 : 512));
}

struct BgPlan {
    bool f64 = false;
    int P = 0, Q = 0, mp = 1;         // macro period = mp periods
    int Pc = 0, Qc = 0;               // outputs / inputs per macro period
    int nrb = 0;                      // row blocks of 16 outputs
    int Kc = 0;                       // input window (elements) one macro period needs
    int Kread = 0;                    // rows the zero-padded MFMA loop reads (>= Kc)
    int NS = 0;                       // steps per chunk (template bucket); a program is kch chunks
    int kch = 1;                      // chunks per program (> 1: A re-read per chunk, long filters)
    int nw = 1;                       // waves (= programs) per column group
    int ncg = 1;                      // column groups (16 columns each) per workgroup
    int nslots = 0;                   // LDS partial slots per column group
    std::vector<BgProg> progs;        // [nw]
    std::vector<BgRed> reds;          // row blocks finished by reduction
    // Row-block-aligned plans (f64): every program is one K piece of one row block, so a workgroup
    // can own one (column block, row block) pair -- the small-launch grid (bg_rb_kernel) -- and
    // produce the same sums as the persistent kernel.  rbStart[rb] .. rbStart[rb + 1] = its programs.
    bool rbAligned = false;
    std::vector<int> rbStart;
    std::vector<int> rbK0;            // first input row of each program (one segment each)
    std::vector<float> A32;           // [nw][kch*NS][64] MFMA A fragments
    std::vector<double> A64;
    // exact rows of the macro period (non-finite fixup, BgDev::xRows): f64 rows [Pc][rowMax] and
    // [offset | length | polyphase phase | DFT parity] per row (phase / parity of composite rows)
    int rowMax = 0;
    bool twoStage = false;
    std::vector<double> rows;
    std::vector<int> rowInfo;
    double usefulMacsPerOutput = 0;   // sum of row lengths / P
    double mfmaMacsPerOutput = 0;     // MFMA MACs / output over the band (excl. bucket padding)
    std::vector<int> progTable() const;  // [nprog][kBgProgInts]
    std::vector<int> redTable() const;   // [nred][kBgRedInts]
};

constexpr int kBgRbMaxSteps = 40;   // row-block-aligned plans: K steps per program (f64 MFMA: 40 x 64 cycles)
constexpr int kBgRbMaxWaves = 8;    // ... and programs per row block (bg_rb_kernel workgroup <= 512 threads)
constexpr int kBgRbKMaxRb = 24;     // bg_rb_kernel launches: row blocks / programs whose tables fit the kernel
constexpr int kBgRbKMaxProg = 96;   // arguments (BgGrid::rbStart, rbK0)

// Builds the MFMA plan (macro period, balanced wave programs, A image).
bool buildBgPlan(const FirPeriodic& f, bool f64, BgPlan& plan);

// ---------------------------------------------------------------------------
// Split-f16 plan (gar_hx.hpp): the same banded GEMM on
// v_mfma_f32_16x16x32_f16 with every operand split into two f16 halves
// (x = xh + xl, a = ah + al, both power-of-two scaled) and the three
// products ah*xh + ah*xl + al*xh accumulated in f32.  One program step =
// one 32-deep K slice of one row block = 3 MFMAs.  Within a slice, lane
// group g (lanes 16g..16g+15) holds the inputs k0 + 4g + j (j < 4) and
// k0 + 16 + 4g + (j - 4) (j >= 4), which is what two ds_read_b64_tr_b16 of
// a [row][16 columns] f16 image deliver conflict-free; A is laid out in the
// same permuted K order.
// ---------------------------------------------------------------------------
constexpr int kHxStep = 32;        // K per program step
constexpr int kHxWaves = 10;       // segmented mode: wave programs per workgroup
constexpr int kHxMaxNS = 8;        // segmented mode register budget: 8 VGPRs of A per step (10 waves: 168 VGPRs)
constexpr int kHxRbMaxWaves = 10;  // row-block mode: one wave per row block
constexpr int kHxRbMaxNS = 10;     // row-block mode register budget (168 VGPRs)
constexpr int kHxMaxRows = 1024;   // window rows per block (4*1024 staged items: 7 per lane at 10 waves)
constexpr int kHxMinWaves = 10;    // waves per workgroup (waves past the programs only stage)
constexpr int kHxMaxWaves = 10;    // __launch_bounds__ (3 waves per SIMD: 168 VGPRs)
constexpr int kHxFixWgs = 32;      // extra workgroups of the edge launch that drain the fix list
inline int hxPermK(int g, int j) { return j < 4 ? 4 * g + j : 16 + 4 * g + (j - 4); }

struct HxPlan {
    int P = 0, Q = 0, mp = 1;
    int Pc = 0, Qc = 0, nrb = 0;
    int Kc = 0;                       // rows of a macro period's window holding input the band reads
    int Kread = 0;                    // rows the padded program steps read (>= Kc)
    int NS = 0, kch = 1, nw = kHxWaves, nslots = 0;
    bool rbMode = false;              // one row block per compute wave: no segments, no partial sums
    int ea = 0;                       // coefficient scale: A * 2^ea has max |.| in [2^14, 2^15)
    std::vector<BgProg> progs;        // [nw]; BgSeg::k0 = first input row of the segment
    std::vector<BgRed> reds;
    std::vector<uint16_t> A;          // [nw][kch*NS][2 (hi, lo)][64 lanes][8] f16 bits
    int rowMax = 0;                   // exact fallback (loud windows): f64 rows [Pc][rowMax], offsets, lengths
    std::vector<double> rows;
    std::vector<int> rowOff, rowLen;
    bool twoStage = false;            // composite rows: per-row polyphase phase / DFT parity
    std::vector<int> rowPh, rowPar;
    double usefulMacsPerOutput = 0;
    double mfmaMacsPerOutput = 0;     // executed MACs (one of the three products) per output
    std::vector<int> progTable() const;  // [nw][kBgProgInts]
    std::vector<int> redTable() const;
};

bool buildHxPlan(const FirPeriodic& f, HxPlan& plan);

// LDS bytes of one hx launch with Ws window rows per column: two hi/lo image
// buffers, partial slots, the loud-element masks [2][16][Ws/32] + flags.
inline size_t hxLdsBytes(int Ws, int nslots, int parity) {
    return 8 * (16 * static_cast<size_t>(Ws) + 64) + static_cast<size_t>(parity ? 2 : 1) * nslots * 256 * 4 +
           (2 * 16 * static_cast<size_t>(Ws / 32) + 2) * 4 + 16;
}

}  // namespace gar
