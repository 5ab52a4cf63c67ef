// gar_engine.cpp -- host state machine + C ABI (include/gar.h).
//
// The reference keeps, per channel, a chain of engine.Resampler stages
// (constant.go:16-85) whose streaming state is history slices plus integer
// counters (dft_stage.go:156-207, polyphase_stage.go:186-312,
// dft_stage.go:488-554).  Here the *counters* are tracked on the host with the
// reference's exact integer arithmetic -- so every call returns exactly the
// reference's number of samples -- while the sample histories live in HBM as
// interleaved [t][channel] rows and all sample arithmetic runs in HIP kernels
// (gar_kernels.hip).  Channels in lockstep share one group and one launch.
#include <hip/hip_runtime.h>
#include <immintrin.h>

#include <algorithm>
#include <chrono>
#include <atomic>
#include <cmath>
#include <condition_variable>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <type_traits>
#include <vector>

#include "gar.h"
#include "gar_design.hpp"
#include "gar_kernels.hpp"
#include "gar_plan.hpp"
#include "gar_pool.hpp"

namespace gar {
namespace {

thread_local std::string g_err;

struct DevError {
    hipError_t e;
    std::string what;
};
#define HIPCHK(x)                                                   \
    do {                                                            \
        hipError_t e_ = (x);                                        \
        if (e_ != hipSuccess) throw DevError{e_, #x};               \
    } while (0)

struct DevBuf {
    void* p = nullptr;
    size_t cap = 0;
    DevBuf() = default;
    DevBuf(const DevBuf&) = delete;
    DevBuf& operator=(const DevBuf&) = delete;
    DevBuf(DevBuf&& o) noexcept : p(o.p), cap(o.cap) { o.p = nullptr; o.cap = 0; }
    DevBuf& operator=(DevBuf&& o) noexcept {
        if (this != &o) { release(); p = o.p; cap = o.cap; o.p = nullptr; o.cap = 0; }
        return *this;
    }
    ~DevBuf() { release(); }
    void release() {
        if (p) (void)hipFree(p);
        p = nullptr;
        cap = 0;
    }
    void ensure(size_t bytes) {
        if (bytes <= cap) return;
        release();
        const size_t nb = bytes + bytes / 4 + 256;
        HIPCHK(hipMalloc(&p, nb));
        cap = nb;
    }
    template <class T>
    void upload(const std::vector<T>& v) {
        ensure(sizeof(T) * std::max<size_t>(v.size(), 1));
        if (!v.empty()) HIPCHK(hipMemcpy(p, v.data(), sizeof(T) * v.size(), hipMemcpyHostToDevice));
    }
};

// ---------------------------------------------------------------------------
// Stage runtime: one engine design + its device plans, shared by all channels
// (the reference designs the same filters once per channel, constant.go:57-70).
// ---------------------------------------------------------------------------
struct StageRT {
    EngineDesign d;
    bool f64 = false;
    bool fused = false;
    FirPeriodic compositeFir;
    BgPlan fusedP, dftP, decimP;
    DevBuf fusedA, fusedT, dftA, dftT, decimA, decimT;
    DevBuf fusedX, dftX, decimX, xBankA, xBankC;  // exact rows of the non-finite fixup (attachExact)
    BgDev fusedD{}, dftD{}, decimD{};
    DevBuf pa, pb, pc, pd, pabcd;
    PolyDev polyD{};
    // split-f16 variants (f32 compute), referenced from the BgDev's .hx
    struct HxRT {
        HxPlan plan;
        DevBuf A, T, rows, rowInfo, banks, banks2, fix;
        HxDev d{};
    } fusedH, dftH, decimH;

    int tc() const { return f64 ? 8 : 4; }
};

// Builds + uploads the split-f16 plan of `f` and points bg.hx at it; `ed` (the
// engine design) supplies the two stages of a composite FIR for the exact
// fallback of non-finite windows.
bool attachHx(const FirPeriodic& f, StageRT::HxRT& h, BgDev& bg, bool dry, const EngineDesign& ed) {
    if (!buildHxPlan(f, h.plan)) return false;
    HxDev& d = h.d;
    const HxPlan& p = h.plan;
    // two double-buffered hi/lo images of one macro period + one partial-slot buffer must fit LDS;
    // longer filters (e.g. the 1223-tap decimator) stay on the exact-f32 kernel
    const size_t ws1 = (static_cast<size_t>(p.Kread) + 63) / 64 * 64;
    if (ws1 > static_cast<size_t>(kHxMaxRows)) return false;
    if (hxLdsBytes(static_cast<int>(ws1), p.nslots, 0) > 160 * 1024) return false;
    d = HxDev{};
    d.Pc = p.Pc; d.Qc = p.Qc; d.Kc = p.Kc; d.Kread = p.Kread; d.NS = p.NS; d.nrb = p.nrb;
    d.nw = p.nw; d.kch = p.kch; d.nred = static_cast<int>(p.reds.size()); d.nslots = p.nslots;
    d.ea = p.ea; d.rowMax = p.rowMax; d.rb = p.rbMode ? 1 : 0;
    d.twoStage = p.twoStage ? 1 : 0;
    d.T1 = ed.dft.taps;
    d.T2 = ed.poly.taps;
    if (p.rbMode && p.nw <= 16) {  // hxq_kernel takes them by value
        const std::vector<int> pt = p.progTable();
        for (int w = 0; w < p.nw; ++w) { d.hU0[w] = pt[kBgProgInts * w + 4]; d.hRbw[w] = pt[kBgProgInts * w + 3]; }
    }
    if (!dry) {
        h.A.upload(p.A);
        std::vector<int> t = p.progTable();
        const std::vector<int> rt = p.redTable();
        const size_t redOff = t.size();
        t.insert(t.end(), rt.begin(), rt.end());
        h.T.upload(t);
        h.rows.upload(p.rows);
        std::vector<int> ri = p.rowOff;  // [rowOff | rowLen | rowPh | rowPar]
        ri.insert(ri.end(), p.rowLen.begin(), p.rowLen.end());
        ri.insert(ri.end(), p.rowPh.begin(), p.rowPh.end());
        ri.insert(ri.end(), p.rowPar.begin(), p.rowPar.end());
        h.rowInfo.upload(ri);
        d.A = h.A.p;
        d.progs = static_cast<const int*>(h.T.p);
        d.reds = static_cast<const int*>(h.T.p) + redOff;
        d.rows = static_cast<const double*>(h.rows.p);
        d.rowOff = static_cast<const int*>(h.rowInfo.p);
        d.rowLen = d.rowOff + p.Pc;
        d.rowPh = d.rowOff + 2 * p.Pc;
        d.rowPar = d.rowOff + 3 * p.Pc;
        d.fixCap = 1 << 16;
        h.fix.upload(std::vector<int>(1 + d.fixCap, 0));
        d.fix = static_cast<int*>(h.fix.p);
        if (p.twoStage) {
            h.banks.upload(ed.poly.a);
            h.banks2.upload(ed.dft.c);
            d.polyA = static_cast<const double*>(h.banks.p);
            d.dftC = static_cast<const double*>(h.banks2.p);
        }
    }
    d.hxsOk = hxsPlanFits(d) ? 1 : 0;  // PCM stores/loads fuse only into hxs_kernel (pcmFusable)
    bg.hx = &h.d;
    return true;
}

BgDev uploadPlan(const BgPlan& p, DevBuf& A, DevBuf& T, bool dry) {
    BgDev d{};
    d.f64 = p.f64 ? 1 : 0;
    d.Pc = p.Pc; d.Qc = p.Qc; d.Kc = p.Kc; d.Kread = p.Kread; d.NS = p.NS; d.nrb = p.nrb;
    d.nprog = static_cast<int>(p.progs.size());
    d.kch = p.kch;
    d.nw = p.nw;
    d.ncg = p.ncg;
    d.nred = static_cast<int>(p.reds.size());
    d.nslots = p.nslots;
    d.rbAligned = p.rbAligned ? 1 : 0;
    d.hRbStart = p.rbAligned ? p.rbStart.data() : nullptr;  // the plan lives as long as the stage
    d.hRbK0 = p.rbAligned ? p.rbK0.data() : nullptr;
    for (size_t rb = 0; p.rbAligned && rb + 1 < p.rbStart.size(); ++rb)
        d.maxPrb = std::max(d.maxPrb, p.rbStart[rb + 1] - p.rbStart[rb]);
    if (dry) return d;
    if (p.f64) A.upload(p.A64); else A.upload(p.A32);
    std::vector<int> t = p.progTable();
    const std::vector<int> rt = p.redTable();
    const size_t redOff = t.size();
    t.insert(t.end(), rt.begin(), rt.end());
    const size_t rbOff = t.size();
    t.insert(t.end(), p.rbStart.begin(), p.rbStart.end());
    T.upload(t);
    d.A = A.p;
    d.progs = static_cast<const int*>(T.p);
    d.reds = static_cast<const int*>(T.p) + redOff;
    d.rbStart = p.rbAligned ? static_cast<const int*>(T.p) + rbOff : nullptr;
    return d;
}

// Exact rows of a plan (non-finite fixup, BgDev::xRows): [rows | rowInfo] in one buffer; the
// composite's two stages' banks are shared by the stage (xBankA / xBankC).
void attachExact(const BgPlan& p, DevBuf& X, StageRT& s, BgDev& d, bool dry) {
    d.xRowMax = p.rowMax;
    d.xTwoStage = p.twoStage ? 1 : 0;
    d.xT1 = s.d.dft.taps;
    d.xT2 = s.d.poly.taps;
    if (dry) return;
    // [rows (f64) | rowInfo (int) | bg_kernel's fix list (kBgNfInts ints, zeroed)]
    const size_t nr = p.rows.size(), ni = p.rowInfo.size();
    const size_t listOff = (nr * 8 + ni * 4 + 15) / 16 * 16;
    X.ensure(listOff + kBgNfListBytes);
    HIPCHK(hipMemcpy(X.p, p.rows.data(), nr * 8, hipMemcpyHostToDevice));
    HIPCHK(hipMemcpy(static_cast<char*>(X.p) + nr * 8, p.rowInfo.data(), ni * 4, hipMemcpyHostToDevice));
    HIPCHK(hipMemset(static_cast<char*>(X.p) + listOff, 0, kBgNfListBytes));
    d.xRows = static_cast<const double*>(X.p);
    d.xInfo = reinterpret_cast<const int*>(static_cast<const char*>(X.p) + nr * 8);
    d.nfList = reinterpret_cast<int*>(static_cast<char*>(X.p) + listOff);
    if (p.twoStage) {
        if (!s.xBankA.p) s.xBankA.upload(s.d.poly.a);
        if (!s.xBankC.p) s.xBankC.upload(s.d.dft.c);
        d.xPolyA = static_cast<const double*>(s.xBankA.p);
        d.xDftC = static_cast<const double*>(s.xBankC.p);
    }
}

template <class T>
void uploadBank(const std::vector<double>& v, DevBuf& b) {
    std::vector<T> c(v.begin(), v.end());
    b.upload(c);
}

bool buildStage(StageRT& s, bool f64, bool hx, bool dry, std::string& err) {
    s.f64 = f64;
    hx = hx && !f64;
    const EngineDesign& d = s.d;
    if (d.kind == EngineKind::Cubic) return true;  // no filter banks (cubic.go:75-90)
    if (d.kind == EngineKind::DftOnly || d.kind == EngineKind::DftPoly) {
        if (!buildBgPlan(firFromDft(d.dft), f64, s.dftP)) { err = "DFT plan"; return false; }
        s.dftD = uploadPlan(s.dftP, s.dftA, s.dftT, dry);
        attachExact(s.dftP, s.dftX, s, s.dftD, dry);
        if (hx) attachHx(firFromDft(d.dft), s.dftH, s.dftD, dry, d);
    }
    if (d.kind == EngineKind::Decim) {
        if (!buildBgPlan(firFromDecim(d.decim), f64, s.decimP)) { err = "decimator plan"; return false; }
        s.decimD = uploadPlan(s.decimP, s.decimA, s.decimT, dry);
        attachExact(s.decimP, s.decimX, s, s.decimD, dry);
        if (hx) attachHx(firFromDecim(d.decim), s.decimH, s.decimD, dry, d);
    }
    if (d.kind == EngineKind::DftPoly) {
        if (firComposite(d.dft, d.poly, s.compositeFir) && buildBgPlan(s.compositeFir, f64, s.fusedP)) {
            s.fused = true;
            s.fusedD = uploadPlan(s.fusedP, s.fusedA, s.fusedT, dry);
            attachExact(s.fusedP, s.fusedX, s, s.fusedD, dry);
            if (hx) attachHx(s.compositeFir, s.fusedH, s.fusedD, dry, d);
        }
        PolyDev& p = s.polyD;
        p.f64 = f64 ? 1 : 0;
        p.L = d.poly.L;
        p.T = d.poly.taps;
        p.step = d.poly.step;
        if (!dry) {
            if (f64) {
                uploadBank<double>(d.poly.a, s.pa); uploadBank<double>(d.poly.b, s.pb);
                uploadBank<double>(d.poly.cc, s.pc); uploadBank<double>(d.poly.d, s.pd);
            } else {
                uploadBank<float>(d.poly.a, s.pa); uploadBank<float>(d.poly.b, s.pb);
                uploadBank<float>(d.poly.cc, s.pc); uploadBank<float>(d.poly.d, s.pd);
            }
            p.a = s.pa.p; p.b = s.pb.p; p.c = s.pc.p; p.d = s.pd.p;
            std::vector<double> il(4 * d.poly.a.size());
            for (size_t i = 0; i < d.poly.a.size(); ++i) {
                il[4 * i] = d.poly.a[i]; il[4 * i + 1] = d.poly.b[i]; il[4 * i + 2] = d.poly.cc[i]; il[4 * i + 3] = d.poly.d[i];
            }
            if (f64) uploadBank<double>(il, s.pabcd); else uploadBank<float>(il, s.pabcd);
            p.abcd = s.pabcd.p;
        }
    }
    return true;
}

// StageAdapter.GetLatency (internal/engine/stage_adapter.go:43-57)
int stageLatency(const EngineDesign& d) {
    if (d.kind == EngineKind::Cubic) return 2;  // cubicLatencySamples (internal/engine/constants.go:12)
    int lat = 0;
    if ((d.kind == EngineKind::DftOnly || d.kind == EngineKind::DftPoly) && d.dft.factor > 1)
        lat += (d.dft.taps * d.dft.factor) / 2;
    if (d.kind == EngineKind::DftPoly) lat += d.poly.taps / 2;
    return lat;
}

// ---------------------------------------------------------------------------
// Per-stage streaming counters (exact reference integer semantics).
// ---------------------------------------------------------------------------
struct Counters {
    bool staged = false;       // DFT+poly engine running stage-by-stage (else fused)
    int64_t x_count = 0;       // samples appended to the stage input stream
    int64_t dft_hist = 0;      // len(DFTStage.history)
    int64_t poly_hist = 0;     // len(PolyphaseStage.history)
    int64_t at = 0;            // PolyphaseStage.at
    int64_t u_base = 0;        // poly-stream index of PolyphaseStage.history[0]
    int64_t u_count = 0;       // samples appended to the poly stream
    int64_t dec_hist = 0;      // len(DFTDecimationStage.history)
    int dec_phase = 0;         // DFTDecimationStage.decimPhase
    int64_t y_count = 0;       // samples emitted
    double cub_phase = 0.0;    // CubicStage.phase (cubic.go:17)
};

// DFTStage.processZeroCopy counts (dft_stage.go:156-207)
int64_t cntDft(Counters& s, const DftBank& b, int64_t n) {
    if (b.factor == 1) return n;
    if (n == 0) return 0;
    s.x_count += n;
    s.dft_hist += n;
    if (s.dft_hist < b.taps) return 0;
    const int64_t p = s.dft_hist - b.taps + 1;
    s.dft_hist -= p;
    return p * b.factor;
}

// PolyphaseStage.processZeroCopy counts (polyphase_stage.go:186-312)
int64_t cntPoly(Counters& s, const PolyBank& b, int64_t m, bool& quirk) {
    if (m == 0) return 0;
    s.poly_hist += m;
    s.u_count += m;
    const int64_t numIn = s.poly_hist - b.taps + 1;
    if (numIn <= 0) return 0;
    const int64_t L = b.L;
    const int64_t limit = (numIn * L) << 16;
    const int64_t nout = (limit - s.at + b.step - 1) / b.step;
    if (nout <= 0) return 0;
    const int64_t at = s.at + nout * b.step;
    const int64_t consumed = (at >> 16) / L;
    if (consumed > 0 && consumed <= s.poly_hist) {
        s.poly_hist -= consumed;
        s.u_base += consumed;
    } else if (consumed > s.poly_hist) {
        quirk = true;  // history left untrimmed, `at` still rebased (polyphase_stage.go:300-307)
    }
    s.at = at - ((consumed * L) << 16);
    return nout;
}

// DFTDecimationStage.processZeroCopy counts (dft_stage.go:488-554)
int64_t cntDecim(Counters& s, const DecimBank& b, int64_t n) {
    if (b.factor == 1) return n;
    if (n == 0) return 0;
    s.x_count += n;
    s.dec_hist += n;
    if (s.dec_hist < b.taps) return 0;
    const int64_t nf = s.dec_hist - b.taps + 1;
    const int64_t nout = s.dec_phase < nf ? (nf - s.dec_phase + b.factor - 1) / b.factor : 0;
    if (nout == 0) return 0;  // early return leaves history and phase untouched (dft_stage.go:516-518)
    s.dec_phase = static_cast<int>(((s.dec_phase - nf) % b.factor + b.factor) % b.factor);
    s.dec_hist -= nf;
    return nout;
}

// Exact closed form of the CubicStage phase walk.  In units of 2^-F (F = 53 - exponent of step,
// so step = S units exactly) every value the walk forms -- ph, ph + k*step < 1, the first sum >= 1,
// that sum minus 1 -- is an integer.  When S, the start phase P0 and 2^F are all multiples of the
// rounding grid of the largest binade a sum reaches (sums < 1 + step), no float64 addition of the
// walk rounds (the "- 1" never does: Sterbenz), so the walk is the exact rotation
//     P_{i+1} = P_i + n_i*S - 2^F in [0, S)   =>   P_i = (P0 - i*2^F) mod S,
//     outputs before input i: N_i = (i*2^F + P_i - P0) / S,
// the same phases and counts as the sequential loop, in O(1) per checkpoint (e.g. 44.1k->48k:
// S even, grid 2 units).  Ratios whose step has a low set bit on a coarser grid (48k->44.1k) walk.
namespace {
struct CubicRot {
    int F = 0;
    int64_t S = 0, P0 = 0;
};
bool cubicRotation(double step, double ph, CubicRot& r) {
    int e = 0;
    (void)std::frexp(step, &e);  // step = m * 2^e, m in [0.5, 1)
    r.F = 53 - e;
    if (r.F < 1 || r.F > 60) return false;
    const double Sd = std::ldexp(step, r.F), Pd = std::ldexp(ph, r.F);  // exact (powers of two)
    if (Sd != std::floor(Sd) || Pd != std::floor(Pd) || Pd < 0.0 || Pd >= Sd) return false;
    r.S = static_cast<int64_t>(Sd);
    r.P0 = static_cast<int64_t>(Pd);
    const int64_t one = int64_t(1) << r.F;
    // bits of the largest sum (< one + S): its binade's grid is 2^(bits - 53) units
    int bits = 0;
    for (uint64_t v = static_cast<uint64_t>(one + r.S - 1); v; v >>= 1) ++bits;
    const int64_t grid = bits > 53 ? (int64_t(1) << (bits - 53)) : 1;
    return r.S % grid == 0 && r.P0 % grid == 0 && one % grid == 0;
}
}  // namespace

// CubicStage.Process walk (cubic.go:42-61): the f64 phase recurrence, run once for
// all channels; `segs` (when given) receives the state every segLen inputs (the closed form takes the
// caller's spacing -- short segments for short calls; the sequential walk uses kCubicSegInputs).
int64_t cntCubic(Counters& s, double ratio, int64_t n, std::vector<CubicSeg>* segs, int* segLen = nullptr) {
    const double step = 1.0 / ratio;
    CubicRot rot;
    if (n > 0 && cubicRotation(step, s.cub_phase, rot)) {
        const __int128 one = static_cast<__int128>(1) << rot.F, S = rot.S, P0 = rot.P0;
        auto phaseAt = [&](int64_t i) {  // P_i in [0, S)
            __int128 v = (P0 - static_cast<__int128>(i) * one) % S;
            return v < 0 ? v + S : v;
        };
        auto outsBefore = [&](int64_t i, __int128 Pi) {
            return static_cast<int64_t>((static_cast<__int128>(i) * one + Pi - P0) / S);
        };
        if (segs)
            for (int64_t i = 0; i < n; i += (segLen ? *segLen : kCubicSegInputs)) {
                const __int128 Pi = phaseAt(i);
                segs->push_back({std::ldexp(static_cast<double>(static_cast<int64_t>(Pi)), -rot.F), s.y_count + outsBefore(i, Pi),
                                 s.x_count + i});
            }
        const __int128 Pn = phaseAt(n);
        const int64_t nout = outsBefore(n, Pn);
        s.cub_phase = std::ldexp(static_cast<double>(static_cast<int64_t>(Pn)), -rot.F);
        s.x_count += n;
        return nout;
    }
    if (segLen) *segLen = static_cast<int>(kCubicSegInputs);
    double ph = s.cub_phase;
    int64_t nout = 0;
    for (int64_t i = 0; i < n; ++i) {
        if (segs && i % kCubicSegInputs == 0) segs->push_back({ph, s.y_count + nout, s.x_count + i});
        while (ph < 1.0) {
            ++nout;
            ph += step;
        }
        ph -= 1.0;
    }
    s.cub_phase = ph;
    s.x_count += n;
    return nout;
}

// ---------------------------------------------------------------------------
struct Hist {
    DevBuf buf[2];
    int cur = 0;
    int64_t base = 0, len = 0;
    bool zero = false;  // rows known to be all zero (post-flush state); nothing stored
    void* ptr() const { return zero ? nullptr : buf[cur].p; }
    void clear() { base = 0; len = 0; zero = false; }
};

struct StageDev {
    Hist xh;  // stage input stream history
    Hist uh;  // poly-stream history (staged DFT+poly)
};

struct InView {
    const void* p = nullptr;
    int64_t fs = 0, cs = 0;
    int f64 = 0;
    int pcm = 0;  // integer PCM input bits (fused into hxs_kernel's loads; gar_process_device only)
    int64_t n = 0;
    bool zeros = false;
};

struct OutView {
    void* p = nullptr;
    int64_t fs = 0, cs = 0;
    int f64 = 0;
    int pcm = 0;  // integer PCM output bits (fused into hxs_kernel's stores)
};

// Pinned host buffer the device reads in place (CubicStage checkpoints); reused only
// after the launch that read it has completed (event).
struct PinBuf {
    void* p = nullptr;
    size_t cap = 0;
    hipEvent_t ev = nullptr;
    bool pending = false;
    PinBuf() = default;
    PinBuf(const PinBuf&) = delete;
    PinBuf& operator=(const PinBuf&) = delete;
    PinBuf(PinBuf&& o) noexcept : p(o.p), cap(o.cap), ev(o.ev), pending(o.pending) { o.p = nullptr; o.ev = nullptr; o.cap = 0; o.pending = false; }
    PinBuf& operator=(PinBuf&& o) noexcept {
        if (this != &o) {
            release();
            p = o.p; cap = o.cap; ev = o.ev; pending = o.pending;
            o.p = nullptr; o.ev = nullptr; o.cap = 0; o.pending = false;
        }
        return *this;
    }
    ~PinBuf() { release(); }
    void release() {
        if (ev) { (void)hipEventSynchronize(ev); (void)hipEventDestroy(ev); }
        if (p) (void)hipHostFree(p);
        p = nullptr; ev = nullptr; cap = 0; pending = false;
    }
    // Wait for the previous reader, grow if needed; returns the host pointer.
    void* acquire(size_t bytes) {
        if (pending) HIPCHK(hipEventSynchronize(ev));
        pending = false;
        if (!ev) HIPCHK(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
        if (bytes > cap) {
            if (p) HIPCHK(hipHostFree(p));
            p = nullptr;
            cap = 0;
            const size_t nb = bytes + bytes / 2 + 4096;
            HIPCHK(hipHostMalloc(&p, nb, hipHostMallocDefault));
            cap = nb;
        }
        return p;
    }
    void issued(hipStream_t s) {
        HIPCHK(hipEventRecord(ev, s));
        pending = true;
    }
};

// Pinned host buffer the kernels read / write in place (the host C-ABI's staging: the caller's
// pageable arrays are packed into it on the host, the first stage's kernel reads it over PCIe and
// the last stage's kernel writes its outputs into the output one -- no DMA round trip per call).
// Used only between a launch and the stream synchronise of the same call.
struct HostBuf {
    void* p = nullptr;
    size_t cap = 0;
    unsigned flags = 0;
    HostBuf() = default;
    explicit HostBuf(unsigned f) : flags(f) {}
    HostBuf(const HostBuf&) = delete;
    HostBuf& operator=(const HostBuf&) = delete;
    ~HostBuf() { release(); }
    void release() {
        if (p) (void)hipHostFree(p);
        p = nullptr;
        cap = 0;
    }
    void* ensure(size_t bytes) {
        if (bytes <= cap) return p;
        release();
        const size_t nb = bytes + bytes / 4 + 4096;
        HIPCHK(hipHostMalloc(&p, nb, hipHostMallocMapped | flags));
        cap = nb;
        return p;
    }
};

// Runs f(c, lo, hi) over channels x [0, n) samples: inline below ~1 MiB of data, else split over
// the pool -- whole channels per job when there are many channels (2 jobs per worker), else
// slices of channels.
inline void forSlices(int C, int64_t n, size_t bytesPerSample, const std::function<void(int, int64_t, int64_t)>& f) {
    const size_t total = static_cast<size_t>(C) * static_cast<size_t>(std::max<int64_t>(n, 0)) * bytesPerSample;
    if (total < (size_t(1) << 20)) {
        for (int c = 0; c < C; ++c) f(c, 0, n);
        return;
    }
    Pool& pool = Pool::get();
    const int J = pool.workers() * 2;
    if (C >= J) {
        pool.run(J, [&](int j) {
            for (int c = static_cast<int>(static_cast<int64_t>(C) * j / J); c < static_cast<int64_t>(C) * (j + 1) / J; ++c) f(c, 0, n);
        });
        return;
    }
    const int per = std::max<int>(1, (J + C - 1) / C);  // slices per channel
    const int64_t step = (n + per - 1) / per;
    pool.run(C * per, [&](int i) {
        const int c = i / per, k = i - c * per;
        const int64_t lo = k * step, hi = std::min<int64_t>(n, lo + step);
        if (lo < hi) f(c, lo, hi);
    });
}

struct Group {
    int c0 = 0, C = 1;
    std::vector<Counters> cnt;
    // engine.Resampler.GetStatistics counters per channel (resampler.go:187-195,270,320,338-339):
    // samples in per non-empty Process, samples out per Process and Flush, zeroed by Reset
    int64_t statIn = 0, statOut = 0;
    std::vector<StageDev> dev;
    std::vector<DevBuf> tmp;   // per stage-boundary output buffers
    DevBuf utmp;               // staged DFT output (u) scratch
    PinBuf cubPin[2];          // CubicStage checkpoints, double-buffered
    int cubCur = 0;
    std::vector<CubicSeg> cubSegs;
};

}  // namespace
}  // namespace gar

struct gar_resampler {
    bool newPath = true;
    int channels = 1;      // total (streams * channels for a batch)
    double ratio = 1.0;
    bool f64 = true;       // compute dtype
    bool hx = false;       // f32 compute on the split-f16 MFMA kernel (GAR_F32) instead of exact-f32 MFMA
    bool dry = false;
    int device = 0;
    bool engineF32Io = false;
    hipStream_t stream = nullptr;
    // cross-stream ordering: every call's work is recorded on orderEv; a call on another
    // stream waits for it first, so one handle's launches never overlap (they share
    // histories, scratch and the fix lists)
    hipEvent_t orderEv = nullptr;
    hipStream_t lastStream = nullptr;
    bool orderValid = false;
    // Recording orderEv costs ~3.5 us of stream time per call (r05f trace: dispatch gaps 7.9 / 8.2 ->
    // 4.3 / 5.8 us without it), so a handle used on one stream only records none: `unordered` marks
    // device work not covered by an event.  The first call on a second stream waits for the device
    // once and turns `multiStream` on; from then on every call records the event.
    bool unordered = false;
    bool multiStream = false;
    // a HIP failure mid-call may leave counters advanced past the histories: refuse
    // further work until Reset (ADVICE: no silent wrong output)
    bool poisoned = false;
    hipEvent_t failEv = nullptr;  // recorded on the failing call's stream (the caller may destroy that stream)
    bool failEvValid = false;
    // device status word (pinned, host-mapped): a kernel that detects a broken invariant of its own
    // (hxt_kernel: an expired progress wait) writes a nonzero code; every ABI call checks it first
    int* errHost = nullptr;
    int* errDev = nullptr;
    gar_config cfg{};
    std::vector<std::unique_ptr<gar::StageRT>> stages;
    std::vector<gar::Group> groups;
    gar::DevBuf inStage, outStage;
    // host C-ABI staging: pinned, mapped; input write-combined (the host only writes it)
    gar::HostBuf hostIn{hipHostMallocWriteCombined | hipHostMallocCoherent}, hostOut{hipHostMallocCoherent};
    std::vector<int64_t> scratchSizes;
    // optional HIP-event timing of the MFMA FIR launches (bench.py roofline)
    bool profile = false;
    uint32_t profileKinds = 0x3f;  // kinds whose launches get events (gar_profile_kinds)
    struct Ev { int tag; hipEvent_t a, b; };
    std::vector<Ev> events;
    std::vector<std::pair<hipEvent_t, hipEvent_t>> evPool;
    double profiledMs[6] = {0, 0, 0, 0, 0, 0};
    int64_t profiledLaunches[6] = {0, 0, 0, 0, 0, 0};
    std::vector<float> launchMs[6], readMs[6];  // per-launch ms since the last read / of the last read
};

namespace gar {
namespace {

using Handle = gar_resampler;

// Pinned host staging above kPinKeep bytes is released when the call that grew it returns, so a
// one-shot call on a long stream does not keep hundreds of MB of page-locked memory per handle.
constexpr size_t kPinKeep = size_t(64) << 20;
// Called only after the call's stream has been synchronised (no kernel still reads the buffers).
void trimHost(Handle* h) {
    if (h->hostIn.cap > kPinKeep) h->hostIn.release();
    if (h->hostOut.cap > kPinKeep) h->hostOut.release();
}

struct Ctx {
    Handle* h;
    Group* g;
    hipStream_t s;
    bool launch;
};

// A launch bracketed by HIP events on its stream when profiling is on (tag = gar_profile_read kind).
template <class L>
hipError_t timed(Ctx& x, int tag, L&& launch) {
    if (!x.h->profile || !((x.h->profileKinds >> tag) & 1u)) return launch();
    hipEvent_t a, b;
    if (!x.h->evPool.empty()) {  // reuse event pairs (creation is not free)
        a = x.h->evPool.back().first;
        b = x.h->evPool.back().second;
        x.h->evPool.pop_back();
    } else {
        // timing events without the system-scope release: a default event's record writes back the
        // L2 for host visibility, which costs stream time the measured kernel does not own
        HIPCHK(hipEventCreateWithFlags(&a, hipEventDisableSystemFence));
        HIPCHK(hipEventCreateWithFlags(&b, hipEventDisableSystemFence));
    }
    HIPCHK(hipEventRecord(a, x.s));
    const hipError_t e = launch();
    HIPCHK(hipEventRecord(b, x.s));
    x.h->events.push_back({tag, a, b});
    return e;
}

hipError_t timedBg(Ctx& x, int tag, const BgDev& p, const SrcDesc& src, const OutDesc& od, int C,
                   HistCopy* hc = nullptr) {
    return timed(x, tag, [&] { return launchBg(p, src, od, C, x.s, hc); });
}

SrcDesc mkSrc(const Hist& hs, int C, int64_t x0, const InView& in) {
    SrcDesc s{};
    s.hist = hs.ptr();
    s.hist_base = hs.base;
    s.hist_len = hs.len;
    s.hist_ld = C;
    s.in = in.zeros ? nullptr : in.p;
    s.in_base = x0;
    s.in_len = in.zeros ? 0 : in.n;
    s.in_fs = in.fs;
    s.in_cs = in.cs;
    s.in_f64 = in.f64;
    s.in_pcm = in.zeros ? 0 : in.pcm;
    s.valid_end = in.zeros ? x0 : x0 + in.n;
    return s;
}

thread_local int* g_curErr = nullptr;  // device status word of the handle whose call is running (callOn)

OutDesc mkOut(const OutView& o, int64_t o0, int64_t n) {
    OutDesc d{};
    d.err = g_curErr;
    d.out = o.p;
    d.o0 = o0;
    d.fs = o.fs;
    d.cs = o.cs;
    d.f64 = o.f64;
    d.pcm = o.pcm;
    d.o_lo = o0;
    d.o_hi = o0 + n;
    return d;
}

void hist_update(Ctx& x, Hist& hs, const SrcDesc& src, int64_t k0, int64_t k1) {
    const int C = x.g->C;
    const int tc = x.h->f64 ? 8 : 4;
    if (k1 < k0) k1 = k0;
    if (!x.launch) { hs.base = k0; hs.len = k1 - k0; hs.zero = false; return; }
    const int other = 1 - hs.cur;
    hs.buf[other].ensure(static_cast<size_t>(std::max<int64_t>(k1 - k0, 1)) * C * tc);
    HIPCHK(launchGather(x.h->f64, src, hs.buf[other].p, k0, k1 - k0, C, x.s));
    hs.cur = other;
    hs.base = k0;
    hs.len = k1 - k0;
    hs.zero = false;
}

// A FIR launch `l(HistCopy*)` (when `launch`) with the history keep hs <- src[k0, k1) folded into it
// when the kernel takes it (hxs_kernel, bg_kernel); otherwise the keep is a gather launch after it.
template <class L>
void withHist(Ctx& x, Hist& hs, const SrcDesc& src, int64_t k0, int64_t k1, bool launch, L&& l) {
    HistCopy hc;
    const int other = 1 - hs.cur;
    if (x.launch && launch && k1 > k0) {
        hs.buf[other].ensure(static_cast<size_t>(k1 - k0) * x.g->C * (x.h->f64 ? 8 : 4));
        hc.dst = hs.buf[other].p;
        hc.t0 = k0;
        hc.n = k1 - k0;
    }
    if (x.launch && launch) HIPCHK(l(&hc));
    if (hc.done) {
        hs.cur = other;
        hs.base = k0;
        hs.len = k1 - k0;
        hs.zero = false;
    } else {
        hist_update(x, hs, src, k0, k1);
    }
}

// FUSED -> STAGED: rebuild the poly-stream history u[u_base, u_count) from x by
// the DFT plan and keep the DFT's own history x[x_count - dft_hist, x_count).
void materialize(Ctx& x, StageRT& rt, Counters& c, StageDev& dv, const SrcDesc& xsrc) {
    const int C = x.g->C;
    const int tc = rt.tc();
    if (x.launch) {
        Hist& uh = dv.uh;
        const int other = 1 - uh.cur;
        const int64_t n = c.u_count - c.u_base;
        uh.buf[other].ensure(static_cast<size_t>(std::max<int64_t>(n, 1)) * C * tc);
        OutView ov{uh.buf[other].p, C, 1, rt.f64 ? 1 : 0};
        HIPCHK(timedBg(x, 1, rt.dftD, xsrc, mkOut(ov, c.u_base, n), C));
        uh.cur = other;
        uh.base = c.u_base;
        uh.len = n;
    } else {
        dv.uh.base = c.u_base;
        dv.uh.len = c.u_count - c.u_base;
    }
    hist_update(x, dv.xh, xsrc, c.x_count - c.dft_hist, c.x_count);
    c.staged = true;
}

// engine.Resampler.ProcessZeroCopy for one stage (resampler.go:232-272).
int64_t stageProcess(Ctx& x, int si, const InView& in, const OutView& out) {
    StageRT& rt = *x.h->stages[si];
    Counters& c = x.g->cnt[si];
    StageDev& dv = x.g->dev[si];
    const int C = x.g->C;
    const EngineDesign& d = rt.d;
    const int64_t n = in.n;
    if (n == 0) return 0;
    switch (d.kind) {
        case EngineKind::Cubic: {
            // CubicStage.Process (cubic.go:33-64); Flush emits nothing (cubic.go:93-96)
            const int64_t x0 = c.x_count;
            std::vector<CubicSeg>* segs = x.launch ? &x.g->cubSegs : nullptr;
            if (segs) segs->clear();
            const SrcDesc src = mkSrc(dv.xh, C, x0, in);
            const int64_t y0 = c.y_count;
            // short calls (streaming chunks): short segments, so each GPU thread re-walks only a few
            // inputs from registers (a 4096-frame call would otherwise be 16 serial 256-input walks)
            int segLen = n * C <= (int64_t(1) << 20) ? kCubicSegInputsShort : static_cast<int>(kCubicSegInputs);
            const int64_t nout = cntCubic(c, d.ratio, n, segs, &segLen);
            if (x.launch && nout > 0) {
                PinBuf& pb = x.g->cubPin[x.g->cubCur];
                x.g->cubCur ^= 1;
                void* hp = pb.acquire(segs->size() * sizeof(CubicSeg));
                std::memcpy(hp, segs->data(), segs->size() * sizeof(CubicSeg));
                HIPCHK(timed(x, 5, [&] {
                    return launchCubic(rt.f64 ? 1 : 0, static_cast<const CubicSeg*>(hp), static_cast<int64_t>(segs->size()),
                                       c.x_count, 1.0 / d.ratio, src, mkOut(out, y0, nout), C, x.s, segLen);
                }));
                pb.issued(x.s);
            }
            hist_update(x, dv.xh, src, std::max<int64_t>(0, c.x_count - 3), c.x_count);
            c.y_count += nout;
            return nout;
        }
        case EngineKind::Passthrough: {
            if (x.launch && !in.zeros) {
                HIPCHK(launchCopy(in.p, in.f64, in.fs, in.cs, out.p, out.f64, out.fs, out.cs, n, C, x.s));
            }
            c.y_count += n;
            return n;
        }
        case EngineKind::DftOnly: {
            const int64_t x0 = c.x_count;
            const int64_t y0 = c.y_count;
            const int64_t nout = cntDft(c, d.dft, n);
            const SrcDesc src = mkSrc(dv.xh, C, x0, in);
            withHist(x, dv.xh, src, c.x_count - c.dft_hist, c.x_count, nout > 0,
                     [&](HistCopy* hc) { return timedBg(x, 1, rt.dftD, src, mkOut(out, y0, nout), C, hc); });
            c.y_count += nout;
            return nout;
        }
        case EngineKind::Decim: {
            const int64_t x0 = c.x_count;
            const int64_t y0 = c.y_count;
            const int64_t nout = cntDecim(c, d.decim, n);
            const SrcDesc src = mkSrc(dv.xh, C, x0, in);
            withHist(x, dv.xh, src, c.x_count - c.dec_hist, c.x_count, nout > 0,
                     [&](HistCopy* hc) { return timedBg(x, 2, rt.decimD, src, mkOut(out, y0, nout), C, hc); });
            c.y_count += nout;
            return nout;
        }
        case EngineKind::DftPoly: {
            const int64_t x0 = c.x_count;
            const int64_t y0 = c.y_count;
            const Counters before = c;
            const SrcDesc xsrc = mkSrc(dv.xh, C, x0, in);
            const int64_t nu = cntDft(c, d.dft, n);
            bool quirk = false;
            const int64_t nout = cntPoly(c, d.poly, nu, quirk);
            if (!c.staged) {
                // Fused: DFT x2 and polyphase composed into one MFMA FIR over x; the history keep
                // x[u_base/2, x_count) rides along in the same launch when the kernel takes it.
                if (quirk) {
                    if (x.launch && nout > 0) HIPCHK(timedBg(x, 0, rt.fusedD, xsrc, mkOut(out, y0, nout), C));
                    materialize(x, rt, c, dv, xsrc);
                } else {
                    withHist(x, dv.xh, xsrc, c.u_base / 2, c.x_count, nout > 0, [&](HistCopy* hc) {
                        return timedBg(x, 0, rt.fusedD, xsrc, mkOut(out, y0, nout), C, hc);
                    });
                }
            } else {
                // Staged: DFT (MFMA FIR) into u scratch, polyphase with live cubic interpolation.
                const int64_t p0 = before.x_count - before.dft_hist;   // DFT positions done before
                const int64_t dy0 = p0 * d.dft.factor;
                InView uin;
                if (x.launch) x.g->utmp.ensure(static_cast<size_t>(std::max<int64_t>(nu, 1)) * C * rt.tc());
                // the x history keep depends on x only: it rides in the DFT launch
                withHist(x, dv.xh, xsrc, c.x_count - c.dft_hist, c.x_count, nu > 0, [&](HistCopy* hc) {
                    OutView uv{x.g->utmp.p, C, 1, rt.f64 ? 1 : 0};
                    return timedBg(x, 1, rt.dftD, xsrc, mkOut(uv, dy0, nu), C, hc);
                });
                uin.p = x.g->utmp.p; uin.fs = C; uin.cs = 1; uin.f64 = rt.f64 ? 1 : 0; uin.n = nu;
                const SrcDesc usrc = mkSrc(dv.uh, C, before.u_count, uin);
                if (x.launch && nout > 0) {
                    PolyDev p = rt.polyD;
                    p.at0 = before.at;
                    p.u_base = before.u_base;
                    p.m0 = before.y_count;
                    HIPCHK(timed(x, 4, [&] { return launchPoly(p, usrc, mkOut(out, y0, nout), nout, C, x.s); }));
                }
                if (nu > 0) hist_update(x, dv.uh, usrc, c.u_base, c.u_count);
            }
            c.y_count += nout;
            return nout;
        }
        default:
            throw DevError{hipErrorNotSupported, "unsupported stage"};
    }
}

// engine.Resampler.Flush for one stage (resampler.go:275-322).
int64_t stageFlush(Ctx& x, int si, const OutView& out) {
    StageRT& rt = *x.h->stages[si];
    Counters& c = x.g->cnt[si];
    StageDev& dv = x.g->dev[si];
    const int C = x.g->C;
    const EngineDesign& d = rt.d;
    InView z;
    z.zeros = true;
    switch (d.kind) {
        case EngineKind::Passthrough:
            return 0;
        case EngineKind::DftOnly:
            if (c.dft_hist == 0) return 0;
            z.n = d.dft.taps;
            return stageProcess(x, si, z, out);
        case EngineKind::Decim:
            if (c.dec_hist == 0) return 0;
            z.n = d.decim.taps;
            return stageProcess(x, si, z, out);
        case EngineKind::DftPoly: {
            if (!c.staged) {
                InView none;
                none.zeros = true;
                const SrcDesc xsrc = mkSrc(dv.xh, C, c.x_count, none);
                // Fused flush: DFTStage.Flush + PolyphaseStage.Process + PolyphaseStage.Flush
                // counted exactly, all samples by one composite launch over x zero-extended
                // (the zero pads of both flushes are zero samples of the same composite FIR).
                Counters t = c;
                bool quirk = false;
                int64_t nA = 0, nB = 0;
                if (t.dft_hist > 0) nA = cntPoly(t, d.poly, cntDft(t, d.dft, d.dft.taps), quirk);
                if (t.poly_hist > 0) nB = cntPoly(t, d.poly, d.poly.taps, quirk);
                if (!quirk) {
                    const int64_t y0 = c.y_count, n = nA + nB;
                    if (x.launch && n > 0) HIPCHK(timedBg(x, 3, rt.fusedD, xsrc, mkOut(out, y0, n), C));
                    c = t;
                    c.y_count = y0 + n;
                    c.staged = true;
                    // both delay lines now hold only flush zeros (their last T-1 pad samples)
                    dv.xh.base = c.x_count - c.dft_hist;
                    dv.xh.len = c.dft_hist;
                    dv.xh.zero = true;
                    dv.uh.base = c.u_base;
                    dv.uh.len = c.u_count - c.u_base;
                    dv.uh.zero = true;
                    return n;
                }
                materialize(x, rt, c, dv, xsrc);
            }
            int64_t total = 0;
            // DFTStage.Flush -> PolyphaseStage.Process(intermediate)
            if (c.dft_hist > 0) {
                z.n = d.dft.taps;
                total += stageProcess(x, si, z, out);
            }
            // PolyphaseStage.Flush: tapsPerPhase zeros into the poly stream
            if (c.poly_hist > 0) {
                const int64_t y0 = c.y_count;
                const Counters before = c;
                bool quirk = false;
                const int64_t nout = cntPoly(c, d.poly, d.poly.taps, quirk);
                InView uz;
                uz.zeros = true;
                uz.n = d.poly.taps;
                const SrcDesc usrc = mkSrc(dv.uh, C, before.u_count, uz);
                OutView o2 = out;
                if (x.launch && nout > 0) {
                    const int es = out.f64 ? 8 : 4;
                    o2.p = static_cast<char*>(out.p) + total * out.fs * es;
                    PolyDev p = rt.polyD;
                    p.at0 = before.at;
                    p.u_base = before.u_base;
                    p.m0 = before.y_count;
                    HIPCHK(timed(x, 4, [&] { return launchPoly(p, usrc, mkOut(o2, y0, nout), nout, C, x.s); }));
                }
                hist_update(x, dv.uh, usrc, c.u_base, c.u_count);
                c.y_count += nout;
                total += nout;
            }
            return total;
        }
        default:
            return 0;
    }
}

OutView offsetView(const OutView& o, int64_t rows) {
    OutView r = o;
    if (o.p) r.p = static_cast<char*>(o.p) + rows * o.fs * (o.pcm ? pcmBytes(o.pcm) : (o.f64 ? 8 : 4));
    return r;
}

// constantRateResampler.processChannel[Into] (constant.go:255-345): the whole
// chain; sizes[i] = samples produced by stage i (buffer i+1).
int64_t chainProcess(Ctx& x, const InView& in, const OutView& out, std::vector<int64_t>& sizes) {
    const int ns = static_cast<int>(x.h->stages.size());
    sizes.assign(ns, 0);
    if (ns == 0) {  // ratio within 0.1% of 1: no stages, the ring buffer passes input through
        if (x.launch && in.n > 0)
            HIPCHK(launchCopy(in.p, in.f64, in.fs, in.cs, out.p, out.f64, out.fs, out.cs, in.n, x.g->C, x.s));
        return in.n;
    }
    InView cur = in;
    for (int i = 0; i < ns; ++i) {
        const bool last = i == ns - 1;
        OutView o = out;
        if (!last) {
            const int tc = x.h->f64 ? 8 : 4;
            if (x.launch) {
                x.g->tmp[i].ensure(static_cast<size_t>(std::max<int64_t>(x.h->scratchSizes[i], 1)) * x.g->C * tc);
                o = OutView{x.g->tmp[i].p, x.g->C, 1, x.h->f64 ? 1 : 0};
            }
        }
        int64_t m = 0;
        if (cur.n >= 1) m = stageProcess(x, i, cur, o);  // Available() >= GetMinInput() (constant.go:277,314)
        sizes[i] = m;
        InView nx;
        nx.p = o.p; nx.fs = o.fs; nx.cs = o.cs; nx.f64 = o.f64; nx.n = m;
        cur = nx;
    }
    return cur.n;
}

// flushChannel (constant.go:360-386)
int64_t chainFlush(Ctx& x, const OutView& out, std::vector<int64_t>& sizes) {
    const int ns = static_cast<int>(x.h->stages.size());
    sizes.assign(ns, 0);
    if (ns == 0) return 0;
    InView pending;  // previous stage's flushed tail
    for (int i = 0; i < ns; ++i) {
        const bool last = i == ns - 1;
        OutView o = out;
        if (!last && x.launch) {
            const int tc = x.h->f64 ? 8 : 4;
            x.g->tmp[i].ensure(static_cast<size_t>(std::max<int64_t>(x.h->scratchSizes[i], 1)) * x.g->C * tc);
            o = OutView{x.g->tmp[i].p, x.g->C, 1, x.h->f64 ? 1 : 0};
        }
        int64_t m = 0;
        if (pending.n > 0) m += stageProcess(x, i, pending, o);
        m += stageFlush(x, i, offsetView(o, m));
        sizes[i] = m;
        InView nx;
        nx.p = o.p; nx.fs = o.fs; nx.cs = o.cs; nx.f64 = o.f64; nx.n = m;
        pending = nx;
    }
    return pending.n;
}

Group* groupOf(Handle* h, int ch) {
    for (auto& g : h->groups)
        if (ch >= g.c0 && ch < g.c0 + g.C) return &g;
    return nullptr;
}

Group freshGroup(Handle* h, int c0, int C) {
    Group g;
    g.c0 = c0;
    g.C = C;
    const size_t ns = h->stages.size();
    g.cnt.assign(ns, Counters());
    g.dev.resize(ns);
    g.tmp.resize(ns);
    for (size_t i = 0; i < ns; ++i)
        if (!h->stages[i]->fused) g.cnt[i].staged = true;
    return g;
}

// Copy channels [k0, k0+kc) of group g into a new group (Process on channel 0
// of a multi-channel handle advances only that channel, constant.go:88-95).
Group splitCopy(Handle* h, Group& g, int k0, int kc) {
    Group ng = freshGroup(h, g.c0 + k0, kc);
    const int tc = h->f64 ? 8 : 4;
    for (size_t i = 0; i < h->stages.size(); ++i) {
        ng.cnt[i] = g.cnt[i];
        ng.statIn = g.statIn;
        ng.statOut = g.statOut;
        Hist* src[2] = {&g.dev[i].xh, &g.dev[i].uh};
        Hist* dst[2] = {&ng.dev[i].xh, &ng.dev[i].uh};
        for (int k = 0; k < 2; ++k) {
            dst[k]->base = src[k]->base;
            dst[k]->len = src[k]->len;
            dst[k]->zero = src[k]->zero;
            if (!h->dry && src[k]->len > 0 && !src[k]->zero) {
                dst[k]->buf[0].ensure(static_cast<size_t>(src[k]->len) * kc * tc);
                const char* sp = static_cast<const char*>(src[k]->ptr()) + static_cast<size_t>(k0) * tc;
                HIPCHK(launchCopy(sp, h->f64, g.C, 1, dst[k]->buf[0].p, h->f64, kc, 1, src[k]->len, kc, h->stream));
            }
        }
    }
    return ng;
}

void isolate(Handle* h, int ch) {
    Group* g = groupOf(h, ch);
    if (!g || g->C == 1) return;
    std::vector<Group> out;
    for (auto& gg : h->groups) {
        if (&gg != g) { out.push_back(std::move(gg)); continue; }
        const int k = ch - gg.c0;
        if (k > 0) out.push_back(splitCopy(h, gg, 0, k));
        out.push_back(splitCopy(h, gg, k, 1));
        if (k + 1 < gg.C) out.push_back(splitCopy(h, gg, k + 1, gg.C - k - 1));
    }
    if (!h->dry) HIPCHK(hipStreamSynchronize(h->stream));
    h->groups = std::move(out);
}

// Dry-run a process (or flush) on copies of the group counters.
int64_t simulate(Handle* h, Group& g, int64_t n, bool flush, std::vector<int64_t>& sizes) {
    Group sim;
    sim.c0 = g.c0;
    sim.C = g.C;
    sim.cnt = g.cnt;
    sim.dev.resize(g.dev.size());
    for (size_t i = 0; i < g.dev.size(); ++i) {
        sim.dev[i].xh.base = g.dev[i].xh.base; sim.dev[i].xh.len = g.dev[i].xh.len;
        sim.dev[i].uh.base = g.dev[i].uh.base; sim.dev[i].uh.len = g.dev[i].uh.len;
    }
    Ctx x{h, &sim, nullptr, false};
    InView in;
    in.n = n;
    OutView o;
    return flush ? chainFlush(x, o, sizes) : chainProcess(x, in, o, sizes);
}

// Run one group for real: sizes first (so scratch can be sized), then launches.
// GetStatistics bookkeeping of one successful call (resampler.go:182-322): Process counts its
// input only when non-empty (the early return of an empty call counts nothing); the cubic
// engine's Flush returns CubicStage.Flush directly, uncounted (resampler.go:276-279).
void countStats(const Handle* h, Group& g, int64_t nIn, int64_t nOut, bool flush) {
    if (!flush) {
        if (nIn <= 0) return;
        g.statIn += nIn;
        g.statOut += nOut;
        return;
    }
    const bool cubicEngine = !h->newPath && h->stages.size() == 1 && h->stages[0]->d.kind == EngineKind::Cubic;
    if (!cubicEngine) g.statOut += nOut;
}

int64_t runGroup(Handle* h, Group& g, const InView& in, const OutView& out, bool flush, hipStream_t s,
                 int64_t cap, gar_status& st) {
    std::vector<int64_t> sizes;
    const int64_t n = simulate(h, g, in.n, flush, sizes);
    if (n > cap) { st = GAR_ERR_BUFFER_TOO_SMALL; return n; }
    st = GAR_OK;
    if (h->dry) {
        Ctx x{h, &g, nullptr, false};
        std::vector<int64_t> s2;
        OutView o;
        if (flush) chainFlush(x, o, s2); else chainProcess(x, in, o, s2);
        countStats(h, g, in.n, n, flush);
        return n;
    }
    h->scratchSizes = sizes;
    Ctx x{h, &g, s, true};
    std::vector<int64_t> s2;
    const int64_t got = flush ? chainFlush(x, out, s2) : chainProcess(x, in, out, s2);
    if (got != n) { st = GAR_ERR_INTERNAL; g_err = "size mismatch between count and launch"; }
    else countStats(h, g, in.n, got, flush);
    return got;
}

gar_status guard(gar_status s, const char* msg) {
    if (s != GAR_OK) g_err = msg;
    return s;
}

// Makes the handle's device current for one call and restores the caller's.
struct DeviceGuard {
    int prev = -1;
    bool set = false;
    explicit DeviceGuard(int dev) {
        if (dev < 0) return;
        if (hipGetDevice(&prev) == hipSuccess && prev != dev && hipSetDevice(dev) == hipSuccess) set = true;
    }
    ~DeviceGuard() {
        if (set) (void)hipSetDevice(prev);
    }
    DeviceGuard(const DeviceGuard&) = delete;
    DeviceGuard& operator=(const DeviceGuard&) = delete;
};

thread_local bool g_launchLimit = false;  // the last wrap() failed on a launch limit (callOn poisons the handle)

template <class F>
gar_status wrap(F&& f) {
    g_launchLimit = false;
    try {
        return f();
    } catch (const DevError& e) {
        if (e.e == hipErrorInvalidConfiguration && !launchLimitMsg().empty()) {  // a launch the device cannot run
            g_err = launchLimitMsg() + " (at " + e.what + ")";
            launchLimitMsg().clear();
            g_launchLimit = true;
            return GAR_ERR_INVALID_ARGUMENT;
        }
        g_err = std::string("HIP error ") + hipGetErrorString(e.e) + " at " + e.what;
        return GAR_ERR_DEVICE;
    } catch (const std::bad_alloc&) {
        g_err = "out of host memory";
        return GAR_ERR_INTERNAL;
    }
}

// One ABI call that touches the device: handle's device current, ordered after
// the handle's previous call (any stream), recorded for the next; a device
// error poisons the handle until Reset.
// A kernel of an earlier (asynchronous) call raised the handle's device status word: the outputs of
// that call are not the reference's, so the handle is poisoned until Reset (no silent wrong output).
bool devFault(Handle* h) {
    if (!h->errHost) return false;
    const int v = __atomic_load_n(h->errHost, __ATOMIC_ACQUIRE);
    if (!v) return false;
    h->poisoned = true;
    const char* what = v == kHxtErrLoadWait   ? "hxt_kernel: a compute wave's LDS load-progress wait expired"
                       : v == kHxtErrSlotWait ? "hxt_kernel: a loader's LDS ring-slot wait expired"
                                              : "unknown code";
    g_err = std::string("device error reported by ") + what + " (code " + std::to_string(v) +
            "); outputs of the launch are invalid; call Reset";
    return true;
}

// Waits until no device work of the handle's calls is pending (free / reset / synchronize): the
// order event when one covers the last call, else -- work of single-stream calls left no event --
// the device (the caller's stream may already be destroyed).
void drainOrder(Handle* h) {
    if (h->orderValid) (void)hipEventSynchronize(h->orderEv);
    else if (h->unordered) (void)hipDeviceSynchronize();
    h->unordered = false;
}

template <class F>
gar_status callOn(Handle* h, hipStream_t s, F&& f, bool hostSynced = false) {
    if (h->poisoned) return guard(GAR_ERR_DEVICE, "handle unusable after an earlier device error; call Reset");
    if (h->dry) return wrap(f);
    if (devFault(h)) return GAR_ERR_DEVICE;
    DeviceGuard dg(h->device);
    struct ErrScope {  // the kernels launched by this call report into this handle's status word
        int* prev;
        explicit ErrScope(int* e) : prev(g_curErr) { g_curErr = e; }
        ~ErrScope() { g_curErr = prev; }
    } es(h->errDev);
    gar_status st = wrap([&]() -> gar_status {
        if (h->orderValid && h->lastStream != s) {
            HIPCHK(hipStreamWaitEvent(s, h->orderEv, 0));
        } else if (h->unordered && h->lastStream != s) {  // first switch of stream: earlier calls left no event
            HIPCHK(hipDeviceSynchronize());
            h->unordered = false;
            h->multiStream = true;
        }
        const gar_status r = f();
        if (hostSynced) {  // the call synchronised its stream: nothing of it is left to order after
            h->orderValid = false;
            h->unordered = false;
        } else if (h->multiStream) {
            HIPCHK(hipEventRecord(h->orderEv, s));
            h->lastStream = s;
            h->orderValid = true;
        } else {
            h->lastStream = s;
            h->orderValid = false;
            h->unordered = true;
        }
        return r;
    });
    if (st == GAR_ERR_DEVICE || (st == GAR_ERR_INVALID_ARGUMENT && g_launchLimit)) {  // state may be half-updated
        h->poisoned = true;
        // drained by Reset through an event: the caller may destroy `s` after the failed call
        h->failEvValid = h->failEv && hipEventRecord(h->failEv, s) == hipSuccess;
    } else if (st == GAR_OK && hostSynced && devFault(h)) {  // this call's own kernels reported
        st = GAR_ERR_DEVICE;
    }
    return st;
}

// Precision carried by a preset (resample.go:217-267).
gar_quality_spec presetSpec(int32_t preset) {
    gar_quality_spec q{};
    switch (preset) {
        case GAR_QUALITY_QUICK: q = {GAR_QUALITY_QUICK, 8, 50.0, 0.7, 1.0, 0}; break;
        case GAR_QUALITY_LOW: q = {GAR_QUALITY_LOW, 16, 50.0, 0.80, 0.95, 0}; break;
        case GAR_QUALITY_MEDIUM: q = {GAR_QUALITY_MEDIUM, 16, 50.0, 0.90, 0.98, 0}; break;
        case GAR_QUALITY_HIGH: q = {GAR_QUALITY_HIGH, 24, 50.0, 0.95, 0.99, 0}; break;
        case GAR_QUALITY_VERYHIGH: q = {GAR_QUALITY_VERYHIGH, 32, 50.0, 0.99, 0.995, 0}; break;
        default: q = {GAR_QUALITY_MEDIUM, 0, 0, 0, 0, 0}; break;
    }
    return q;
}

gar_status validate(const gar_config* c) {
    if (!c) return guard(GAR_ERR_INVALID_CONFIG, "invalid resampler configuration: config is nil");
    if (!(c->input_rate > 0) || !(c->output_rate > 0))
        return guard(GAR_ERR_INVALID_CONFIG, "invalid resampler configuration: sample rates must be positive");
    if (c->channels < 1) return guard(GAR_ERR_INVALID_CONFIG, "invalid resampler configuration: channels must be at least 1");
    if (c->channels > 256) return guard(GAR_ERR_INVALID_CONFIG, "invalid resampler configuration: too many channels (max 256)");
    const double r = c->output_rate / c->input_rate;
    if (r < 1.0 / 256.0 || r > 256.0)
        return guard(GAR_ERR_INVALID_CONFIG, "invalid resampler configuration: resampling ratio out of range");
    const gar_quality_spec& q = c->quality;
    if (q.preset == GAR_QUALITY_CUSTOM) {
        if (q.precision < 8 || q.precision > 33) return guard(GAR_ERR_INVALID_CONFIG, "precision must be 8-33 bits");
        if (q.phase_response < 0 || q.phase_response > 100) return guard(GAR_ERR_INVALID_CONFIG, "phase response must be 0-100");
        if (q.passband_end <= 0 || q.passband_end >= 1) return guard(GAR_ERR_INVALID_CONFIG, "passband end must be in (0, 1)");
        if (q.stopband_begin <= q.passband_end || q.stopband_begin > 1)
            return guard(GAR_ERR_INVALID_CONFIG, "stopband begin must be in (passband_end, 1]");
    }
    return GAR_OK;
}

// GAR_HX=0 in the environment routes GAR_F32 compute to the exact-f32 MFMA kernel (A/B comparisons).
bool hxEnabled() {
    static const bool on = [] {
        const char* e = std::getenv("GAR_HX");
        return !(e && e[0] == '0');
    }();
    return on;
}

gar_status initDevice(Handle* h) {
    if (h->dry) return GAR_OK;
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || n <= h->device) {
        g_err = "no HIP device visible (the GPU path requires an MI355X / gfx950)";
        return GAR_ERR_DEVICE;
    }
    HIPCHK(hipSetDevice(h->device));
    HIPCHK(hipStreamCreateWithFlags(&h->stream, hipStreamNonBlocking));
    // device-scope release: the event only orders this handle's calls across streams of its
    // device (host visibility of results goes through the stream syncs of the host paths); a
    // system-scope release would write back every dirty L2 line after each call
    HIPCHK(hipEventCreateWithFlags(&h->orderEv, hipEventDisableTiming | hipEventDisableSystemFence));
    HIPCHK(hipEventCreateWithFlags(&h->failEv, hipEventDisableTiming));
    // the device status word: coherent pinned host memory, so a kernel's system-scope store is seen by
    // the next ABI call without a synchronisation
    void* w = nullptr;
    HIPCHK(hipHostMalloc(&w, 64, hipHostMallocMapped | hipHostMallocCoherent));
    h->errHost = static_cast<int*>(w);
    *h->errHost = 0;
    void* d = nullptr;
    HIPCHK(hipHostGetDevicePointer(&d, w, 0));
    h->errDev = static_cast<int*>(d);
    return GAR_OK;
}

gar_status addStage(Handle* h, double inRate, double outRate, Quality q) {
    auto rt = std::make_unique<StageRT>();
    std::string err;
    if (!designEngine(inRate, outRate, q, rt->d, err)) return guard(GAR_ERR_INVALID_CONFIG, err.c_str());
    if (!buildStage(*rt, h->f64, h->hx, h->dry, err)) {
        g_err = err;
        return GAR_ERR_INTERNAL;
    }
    h->stages.push_back(std::move(rt));
    return GAR_OK;
}

gar_status newCommon(gar_config* cfg, int32_t nstreams, gar_resampler** out) {
    if (!out) return guard(GAR_ERR_INVALID_ARGUMENT, "out is NULL");
    *out = nullptr;
    gar_status s = validate(cfg);
    if (s != GAR_OK) return s;
    if (nstreams < 1) return guard(GAR_ERR_INVALID_CONFIG, "n_streams must be >= 1");
    if (cfg->quality.preset != GAR_QUALITY_CUSTOM) cfg->quality = presetSpec(cfg->quality.preset);
    auto h = std::make_unique<Handle>();
    h->newPath = true;
    h->cfg = *cfg;
    h->channels = cfg->channels * nstreams;
    h->ratio = cfg->output_rate / cfg->input_rate;
    h->f64 = cfg->compute_dtype != GAR_F32 && cfg->compute_dtype != GAR_F32_EXACT;
    h->hx = cfg->compute_dtype == GAR_F32 && hxEnabled();
    h->dry = cfg->dry_run != 0;
    h->device = cfg->device;
    DeviceGuard dg(h->dry ? -1 : cfg->device);
    return wrap([&]() -> gar_status {
        gar_status st = initDevice(h.get());
        if (st != GAR_OK) return st;
        const int prec = cfg->quality.precision;
        const std::vector<StageSpec> specs = buildPipeline(h->ratio, prec);
        for (const StageSpec& sp : specs) {
            // createStage -> engine.NewResampler[float64](48000, 48000*ratio, q) (stages.go:54-70)
            if (sp.type == StageType::Cubic) {
                // newCubicStage(ratio) -> engine.NewCubicStage[float64] at the total ratio (stages.go:21-23)
                st = addStage(h.get(), 1.0, sp.ratio, Quality::Quick);
                if (st != GAR_OK) return st;
                continue;
            }
            const double ir = 48000.0;
            st = addStage(h.get(), ir, ir * sp.ratio, precisionToEngineQuality(prec));
            if (st != GAR_OK) return st;
        }
        h->groups.push_back(freshGroup(h.get(), 0, h->channels));
        *out = h.release();
        return GAR_OK;
    });
}

// engine.NewResampler[F] behind NewEngine / NewEngineFloat32 / the engine seam
// (convenience.go:125-135, :329-336; internal/engine/resampler.go:51-179).
gar_status newEngineCommon(double in_rate, double out_rate, Quality q, int32_t dtype, bool dry, gar_resampler** out) {
    if (!out) return guard(GAR_ERR_INVALID_ARGUMENT, "out is NULL");
    *out = nullptr;
    if (dtype != GAR_F64 && dtype != GAR_F32 && dtype != GAR_F32_EXACT) return guard(GAR_ERR_INVALID_ARGUMENT, "unknown dtype");
    if (!(in_rate > 0) || !(out_rate > 0)) return guard(GAR_ERR_INVALID_CONFIG, "sample rates must be positive");
    auto h = std::make_unique<gar_resampler>();
    h->newPath = false;
    h->channels = 1;
    h->dry = dry;
    h->f64 = dtype == GAR_F64;
    h->hx = dtype == GAR_F32 && hxEnabled();
    h->engineF32Io = dtype != GAR_F64;
    h->ratio = out_rate / in_rate;
    DeviceGuard dg(dry ? -1 : 0);
    return wrap([&]() -> gar_status {
        gar_status st = initDevice(h.get());
        if (st != GAR_OK) return st;
        st = addStage(h.get(), in_rate, out_rate, q);
        if (st != GAR_OK) return st;
        h->ratio = h->stages[0]->d.ratio;
        h->groups.push_back(freshGroup(h.get(), 0, 1));
        *out = h.release();
        return GAR_OK;
    });
}

int64_t estimate(const Handle* h, int64_t n) {
    return static_cast<int64_t>(static_cast<double>(n) * h->ratio) + 64;
}

// Host input -> pinned staging in the compute dtype (f64 -> f32 rounds exactly as the kernels'
// loads would: the result is bit-identical to handing them the f64 input).
// Host conversions of the staging copies, AVX2 where the CPU has it.  The output copy into the
// caller's arrays uses streaming stores (no read-for-ownership of 8.9 MB per 256-channel 4096-frame
// call); each job ends with an sfence so the stores are globally visible before the pool's hand-off.
__attribute__((target("avx2"))) void cvtD2F(float* d, const double* s, int64_t n) {
    int64_t i = 0;
    for (; i + 8 <= n; i += 8)
        _mm256_storeu_ps(d + i, _mm256_set_m128(_mm256_cvtpd_ps(_mm256_loadu_pd(s + i + 4)),
                                                _mm256_cvtpd_ps(_mm256_loadu_pd(s + i))));
    for (; i < n; ++i) d[i] = static_cast<float>(s[i]);
}
__attribute__((target("avx2"))) void cvtF2DStream(double* d, const float* s, int64_t n) {
    int64_t i = 0;
    for (; i < n && (reinterpret_cast<uintptr_t>(d + i) & 31); ++i) d[i] = static_cast<double>(s[i]);
    for (; i + 8 <= n; i += 8) {
        _mm256_stream_pd(d + i, _mm256_cvtps_pd(_mm_loadu_ps(s + i)));
        _mm256_stream_pd(d + i + 4, _mm256_cvtps_pd(_mm_loadu_ps(s + i + 4)));
    }
    for (; i < n; ++i) d[i] = static_cast<double>(s[i]);
    _mm_sfence();
}
__attribute__((target("avx2"))) void copyD2DStream(double* d, const double* s, int64_t n) {
    int64_t i = 0;
    for (; i < n && (reinterpret_cast<uintptr_t>(d + i) & 31); ++i) d[i] = s[i];
    for (; i + 8 <= n; i += 8) {
        _mm256_stream_pd(d + i, _mm256_loadu_pd(s + i));
        _mm256_stream_pd(d + i + 4, _mm256_loadu_pd(s + i + 4));
    }
    for (; i < n; ++i) d[i] = s[i];
    _mm_sfence();
}
bool hostAvx2() {
    static const bool a = __builtin_cpu_supports("avx2");
    return a;
}

template <class T>
void packChannel(void* dst, bool f64, const T* src, int64_t lo, int64_t hi) {
    if constexpr (std::is_same<T, double>::value) {
        if (!f64 && hostAvx2()) {
            cvtD2F(static_cast<float*>(dst) + lo, src + lo, hi - lo);
            return;
        }
    }
    if (f64) {
        double* d = static_cast<double*>(dst);
        for (int64_t i = lo; i < hi; ++i) d[i] = static_cast<double>(src[i]);
    } else {
        float* d = static_cast<float*>(dst);
        for (int64_t i = lo; i < hi; ++i) d[i] = static_cast<float>(src[i]);
    }
}
template <class T>
void unpackChannel(T* dst, bool f64, const void* src, int64_t lo, int64_t hi) {
    if constexpr (std::is_same<T, double>::value) {
        if (hostAvx2() && hi - lo >= 64) {
            if (f64) copyD2DStream(dst + lo, static_cast<const double*>(src) + lo, hi - lo);
            else cvtF2DStream(dst + lo, static_cast<const float*>(src) + lo, hi - lo);
            return;
        }
    }
    if (f64) {
        const double* s = static_cast<const double*>(src);
        for (int64_t i = lo; i < hi; ++i) dst[i] = static_cast<T>(s[i]);
    } else {
        const float* s = static_cast<const float*>(src);
        for (int64_t i = lo; i < hi; ++i) dst[i] = static_cast<T>(s[i]);
    }
}

template <class T>
gar_status monoCall(Handle* h, int ch, const T* in, int64_t n, T* out, int64_t cap, int64_t* nOut, bool flush,
                    bool intoSemantics) {
    if (!h) return guard(GAR_ERR_INVALID_ARGUMENT, "nil resampler");
    if (ch < 0 || ch >= h->channels) return guard(GAR_ERR_INVALID_ARGUMENT, "channel out of range");
    if (nOut) *nOut = 0;
    if (!flush && n < 0) return guard(GAR_ERR_INVALID_ARGUMENT, "negative length");
    if (!flush && intoSemantics && cap < estimate(h, n)) return guard(GAR_ERR_BUFFER_TOO_SMALL, "output buffer too small");
    const size_t es = h->f64 ? 8 : 4;  // compute dtype: the staging holds exactly what the kernels compute in
    return callOn(h, h->stream, [&]() -> gar_status {
        isolate(h, ch);
        Group* g = groupOf(h, ch);
        std::vector<int64_t> sizes;
        const int64_t need = simulate(h, *g, flush ? 0 : n, flush, sizes);
        if (need > cap) {
            if (intoSemantics && !flush) { g_err = "EstimateOutput underestimated actual output length"; return GAR_ERR_INTERNAL; }
            return guard(GAR_ERR_BUFFER_TOO_SMALL, "output buffer too small");
        }
        InView iv;
        iv.n = flush ? 0 : n;
        iv.f64 = h->f64 ? 1 : 0;
        iv.fs = 1;
        iv.cs = 0;
        OutView ov;
        ov.fs = 1;
        ov.cs = 0;
        ov.f64 = h->f64 ? 1 : 0;
        if (!h->dry) {
            if (!flush && n > 0) {
                void* hp = h->hostIn.ensure(static_cast<size_t>(n) * es);
                forSlices(1, n, es + sizeof(T), [&](int, int64_t lo, int64_t hi) { packChannel<T>(hp, h->f64, in, lo, hi); });
                iv.p = hp;
            }
            ov.p = h->hostOut.ensure(static_cast<size_t>(std::max<int64_t>(need, 1)) * es);
        }
        gar_status st;
        const int64_t got = runGroup(h, *g, iv, ov, flush, h->stream, cap, st);
        if (st != GAR_OK) return st;
        if (!h->dry) {
            HIPCHK(hipStreamSynchronize(h->stream));
            forSlices(1, got, es + sizeof(T), [&](int, int64_t lo, int64_t hi) { unpackChannel<T>(out, h->f64, ov.p, lo, hi); });
            trimHost(h);
        }
        if (nOut) *nOut = got;
        return GAR_OK;
    }, true);
}

}  // namespace
}  // namespace gar

namespace gar {
namespace {
bool isPcm(int32_t t) { return t == GAR_PCM16 || t == GAR_PCM24 || t == GAR_PCM32; }
bool ioTypeOk(int32_t t) { return t == GAR_F64 || t == GAR_F32 || t == GAR_F32_EXACT || isPcm(t); }
// PCM conversion fused into hxs_kernel's loads and stores: one fused split-f16 stage streaming
// through the row-block kernel (launchHxs's geometry); anything else stages the conversion.
bool pcmFusable(const Handle* h) {
    if (h->dry || h->f64 || !h->hx || h->stages.size() != 1 || h->groups.size() != 1) return false;
    const StageRT& st = *h->stages[0];
    if (!st.fused || h->groups[0].cnt.empty() || h->groups[0].cnt[0].staged) return false;
    const HxDev* hx = st.fusedD.hx;
    return hx && hx->hxsOk;
}
}  // namespace
}  // namespace gar

namespace gar {
namespace {
void fillGeometry(const EngineDesign& d, gar_engine_geometry* geom) {
    std::memset(geom, 0, sizeof(*geom));
    geom->kind = static_cast<int32_t>(d.kind);
    geom->dft_factor = d.dft.factor;
    geom->dft_taps = d.dft.taps;
    geom->poly_phases = d.poly.L;
    geom->poly_taps = d.poly.taps;
    geom->poly_step = d.poly.step;
    geom->decim_factor = d.decim.factor;
    geom->decim_taps = d.decim.taps;
    FirPeriodic f;
    bool have = false;
    if (d.kind == EngineKind::DftPoly && firComposite(d.dft, d.poly, f)) { geom->fused = 1; have = true; }
    else if (d.kind == EngineKind::DftOnly) { f = firFromDft(d.dft); have = true; }
    else if (d.kind == EngineKind::Decim) { f = firFromDecim(d.decim); have = true; }
    if (have) {
        geom->fir_period_out = f.P;
        geom->fir_period_in = f.Q;
        for (const auto& row : f.rows) geom->fir_taps_max = std::max<int32_t>(geom->fir_taps_max, static_cast<int32_t>(row.size()));
        BgPlan p;
        if (buildBgPlan(f, false, p)) {
            geom->useful_macs_per_output = p.usefulMacsPerOutput;
            geom->mfma_macs_per_output = p.mfmaMacsPerOutput;
        }
    }
}
}  // namespace
}  // namespace gar

// ===========================================================================
// C ABI
// ===========================================================================
using namespace gar;

extern "C" {

gar_status gar_config_validate(const gar_config* cfg) { return validate(cfg); }

gar_quality_spec gar_preset_spec(int32_t preset) { return presetSpec(preset); }

gar_status gar_new(gar_config* cfg, gar_resampler** out) { return newCommon(cfg, 1, out); }

gar_status gar_new_batch(gar_config* cfg, int32_t n_streams, gar_resampler** out) {
    return newCommon(cfg, n_streams, out);
}

gar_status gar_new_engine(double in_rate, double out_rate, int32_t preset, int32_t dtype, gar_resampler** out) {
    return newEngineCommon(in_rate, out_rate, presetToEngineQuality(preset), dtype, false, out);
}

gar_status gar_new_engine_quality(double in_rate, double out_rate, int32_t engine_quality, int32_t dtype,
                                  gar_resampler** out) {
    if (engine_quality < GAR_ENGINE_QUICK || engine_quality > GAR_ENGINE_32BIT) {
        if (out) *out = nullptr;
        return guard(GAR_ERR_INVALID_CONFIG, "unknown engine quality");
    }
    return newEngineCommon(in_rate, out_rate, static_cast<Quality>(engine_quality), dtype, false, out);
}

gar_status gar_new_engine_dry(double in_rate, double out_rate, int32_t preset, int32_t dtype, gar_resampler** out) {
    // Host-only engine (used by CPU tests of the stream-length state machine).
    return newEngineCommon(in_rate, out_rate, presetToEngineQuality(preset), dtype, true, out);
}

void gar_free(gar_resampler* r) {
    if (!r) return;
    DeviceGuard dg(r->dry ? -1 : r->device);
    try {
        if (r->stream) (void)hipStreamSynchronize(r->stream);
        drainOrder(r);
        if (r->orderEv) (void)hipEventDestroy(r->orderEv);
        for (auto& ev : r->events) {
            (void)hipEventDestroy(ev.a);
            (void)hipEventDestroy(ev.b);
        }
        for (auto& ev : r->evPool) {
            (void)hipEventDestroy(ev.first);
            (void)hipEventDestroy(ev.second);
        }
        r->groups.clear();
        r->stages.clear();
        if (r->failEv) (void)hipEventDestroy(r->failEv);
        if (r->errHost) (void)hipHostFree(r->errHost);
        if (r->stream) (void)hipStreamDestroy(r->stream);
    } catch (...) {
    }
    delete r;
}

gar_status gar_synchronize(gar_resampler* r) {
    if (!r) return GAR_ERR_INVALID_ARGUMENT;
    if (r->dry) return GAR_OK;
    DeviceGuard dg(r->device);
    const gar_status st = wrap([&]() -> gar_status {
        if (r->orderValid) HIPCHK(hipEventSynchronize(r->orderEv));
        else if (r->unordered) HIPCHK(hipDeviceSynchronize());
        r->unordered = false;
        if (r->stream) HIPCHK(hipStreamSynchronize(r->stream));
        return GAR_OK;
    });
    if (st != GAR_OK) {
        r->poisoned = true;
        return st;
    }
    if (devFault(r)) return GAR_ERR_DEVICE;
    if (r->poisoned) return guard(GAR_ERR_DEVICE, "handle unusable after an earlier device error; call Reset");
    return GAR_OK;
}

int64_t gar_estimate_output(const gar_resampler* r, int64_t n) { return r ? estimate(r, n) : -1; }

int64_t gar_output_size(const gar_resampler* r, int32_t ch, int64_t n) {
    if (!r || ch < 0 || ch >= r->channels) return -1;
    gar_resampler* h = const_cast<gar_resampler*>(r);
    Group* g = groupOf(h, ch);
    std::vector<int64_t> s;
    return simulate(h, *g, n, false, s);
}

int64_t gar_flush_size(const gar_resampler* r, int32_t ch) {
    if (!r || ch < 0 || ch >= r->channels) return -1;
    gar_resampler* h = const_cast<gar_resampler*>(r);
    Group* g = groupOf(h, ch);
    std::vector<int64_t> s;
    return simulate(h, *g, 0, true, s);
}

gar_status gar_process_f64(gar_resampler* r, const double* in, int64_t n, double* out, int64_t cap, int64_t* n_out) {
    return monoCall<double>(r, 0, in, n, out, cap, n_out, false, false);
}
gar_status gar_process_f32(gar_resampler* r, const float* in, int64_t n, float* out, int64_t cap, int64_t* n_out) {
    return monoCall<float>(r, 0, in, n, out, cap, n_out, false, false);
}
gar_status gar_process_into_f64(gar_resampler* r, const double* in, int64_t n, double* out, int64_t cap,
                                int64_t* n_out) {
    return monoCall<double>(r, 0, in, n, out, cap, n_out, false, true);
}
gar_status gar_process_into_f32(gar_resampler* r, const float* in, int64_t n, float* out, int64_t cap,
                                int64_t* n_out) {
    return monoCall<float>(r, 0, in, n, out, cap, n_out, false, true);
}
gar_status gar_flush_f64(gar_resampler* r, double* out, int64_t cap, int64_t* n_out) {
    return monoCall<double>(r, 0, nullptr, 0, out, cap, n_out, true, false);
}
gar_status gar_flush_f32(gar_resampler* r, float* out, int64_t cap, int64_t* n_out) {
    return monoCall<float>(r, 0, nullptr, 0, out, cap, n_out, true, false);
}

// Development (GAR_HOST_TRACE=1, read once): per-call phase times of the host multi-channel path on
// stderr (pack into the pinned staging, launches, wait for the device, unpack), microseconds.
struct HostTrace {
    bool on;
    std::chrono::steady_clock::time_point t0;
    double ph[4] = {0, 0, 0, 0};
    HostTrace() : on(enabled()), t0(std::chrono::steady_clock::now()) {}
    static bool enabled() {
        static const bool e = [] { const char* v = std::getenv("GAR_HOST_TRACE"); return v && v[0] == '1'; }();
        return e;
    }
    void add(int k) {  // the time since the previous mark belongs to phase k
        if (!on) return;
        const auto t = std::chrono::steady_clock::now();
        ph[k] += std::chrono::duration<double, std::micro>(t - t0).count();
        t0 = t;
    }
    ~HostTrace() {
        if (on) fprintf(stderr, "host-trace pack %.1f launch %.1f device-wait %.1f unpack %.1f us\n", ph[0], ph[1], ph[2], ph[3]);
    }
};

gar_status gar_process_multi_f64(gar_resampler* r, const double* const* in, int32_t nch, int64_t n,
                                 double* const* out, int64_t cap, int64_t* n_out) {
    if (!r) return guard(GAR_ERR_INVALID_ARGUMENT, "nil resampler");
    if (nch != r->channels) {
        g_err = "expected " + std::to_string(r->channels) + " channels, got " + std::to_string(nch);
        return GAR_ERR_CHANNEL_MISMATCH;
    }
    if (n < 0) return guard(GAR_ERR_INVALID_ARGUMENT, "negative length");
    return callOn(r, r->stream, [&]() -> gar_status {
        gar_resampler* h = r;
        // exact sizes first: no state changes on BUFFER_TOO_SMALL
        int64_t need = 0;
        for (auto& g : h->groups) {
            std::vector<int64_t> s;
            const int64_t m = simulate(h, g, n, false, s);
            if (m > cap) return guard(GAR_ERR_BUFFER_TOO_SMALL, "output buffer too small");
            need = std::max(need, m);
        }
        const int C = h->channels;
        const size_t es = h->f64 ? 8 : 4;
        // planar [channel][frame] in the compute dtype, staged for the exact output length (not the
        // caller's capacity); output rows 16-B aligned (vector stores)
        const int64_t ocap = (std::max<int64_t>(need, 1) + 3) / 4 * 4;
        char* hin = nullptr;
        char* hout = nullptr;
        HostTrace tr;
        if (!h->dry) {
            if (n > 0) {
                hin = static_cast<char*>(h->hostIn.ensure(static_cast<size_t>(n) * C * es));
                forSlices(C, n, es + 8, [&](int c, int64_t lo, int64_t hi) {
                    packChannel<double>(hin + static_cast<size_t>(c) * n * es, h->f64, in[c], lo, hi);
                });
            }
            hout = static_cast<char*>(h->hostOut.ensure(static_cast<size_t>(ocap) * C * es));
        }
        tr.add(0);
        std::vector<int64_t> got(h->groups.size());
        for (size_t gi = 0; gi < h->groups.size(); ++gi) {
            Group& g = h->groups[gi];
            InView iv;
            iv.n = n;
            iv.f64 = h->f64 ? 1 : 0;
            iv.fs = 1;
            iv.cs = n;
            if (hin) iv.p = hin + static_cast<size_t>(g.c0) * n * es;
            OutView ov;
            ov.f64 = h->f64 ? 1 : 0;
            ov.fs = 1;
            ov.cs = ocap;
            if (hout) ov.p = hout + static_cast<size_t>(g.c0) * ocap * es;
            gar_status st;
            got[gi] = runGroup(h, g, iv, ov, false, h->stream, cap, st);
            if (st != GAR_OK) return st;
            for (int c = g.c0; c < g.c0 + g.C; ++c)
                if (n_out) n_out[c] = got[gi];
        }
        tr.add(1);
        if (!h->dry) {
            HIPCHK(hipStreamSynchronize(h->stream));
            tr.add(2);
            const int64_t gmax = got.empty() ? 0 : *std::max_element(got.begin(), got.end());
            forSlices(C, gmax, es + 8, [&](int c, int64_t lo, int64_t hi) {
                const int64_t m = got[groupOf(h, c) - h->groups.data()];
                if (lo < m) unpackChannel<double>(out[c], h->f64, hout + static_cast<size_t>(c) * ocap * es, lo, std::min(hi, m));
            });
            tr.add(3);
            trimHost(h);
        }
        return GAR_OK;
    }, true);
}

gar_status gar_flush_multi_f64(gar_resampler* r, double* const* out, int32_t nch, int64_t cap, int64_t* n_out) {
    if (!r) return guard(GAR_ERR_INVALID_ARGUMENT, "nil resampler");
    if (nch != r->channels) return guard(GAR_ERR_CHANNEL_MISMATCH, "channel count mismatch");
    return callOn(r, r->stream, [&]() -> gar_status {
        gar_resampler* h = r;
        int64_t need = 0;
        for (auto& g : h->groups) {
            std::vector<int64_t> s;
            const int64_t m = simulate(h, g, 0, true, s);
            if (m > cap) return guard(GAR_ERR_BUFFER_TOO_SMALL, "output buffer too small");
            need = std::max(need, m);
        }
        const int C = h->channels;
        const size_t es = h->f64 ? 8 : 4;
        const int64_t ocap = (std::max<int64_t>(need, 1) + 3) / 4 * 4;
        char* hout = h->dry ? nullptr : static_cast<char*>(h->hostOut.ensure(static_cast<size_t>(ocap) * C * es));
        std::vector<int64_t> got(h->groups.size());
        for (size_t gi = 0; gi < h->groups.size(); ++gi) {
            Group& g = h->groups[gi];
            OutView ov;
            ov.f64 = h->f64 ? 1 : 0;
            ov.fs = 1;
            ov.cs = ocap;
            if (hout) ov.p = hout + static_cast<size_t>(g.c0) * ocap * es;
            gar_status st;
            got[gi] = runGroup(h, g, InView(), ov, true, h->stream, cap, st);
            if (st != GAR_OK) return st;
            for (int c = g.c0; c < g.c0 + g.C; ++c)
                if (n_out) n_out[c] = got[gi];
        }
        if (!h->dry) {
            HIPCHK(hipStreamSynchronize(h->stream));
            const int64_t gmax = got.empty() ? 0 : *std::max_element(got.begin(), got.end());
            forSlices(C, gmax, es + 8, [&](int c, int64_t lo, int64_t hi) {
                const int64_t m = got[groupOf(h, c) - h->groups.data()];
                if (lo < m) unpackChannel<double>(out[c], h->f64, hout + static_cast<size_t>(c) * ocap * es, lo, std::min(hi, m));
            });
            trimHost(h);
        }
        return GAR_OK;
    }, true);
}

int64_t gar_device_output_size(const gar_resampler* r, int64_t frames) {
    if (!r || r->groups.size() != 1) return -1;
    gar_resampler* h = const_cast<gar_resampler*>(r);
    std::vector<int64_t> s;
    return simulate(h, h->groups[0], frames, false, s);
}

int64_t gar_device_flush_size(const gar_resampler* r) {
    if (!r || r->groups.size() != 1) return -1;
    gar_resampler* h = const_cast<gar_resampler*>(r);
    std::vector<int64_t> s;
    return simulate(h, h->groups[0], 0, true, s);
}

gar_status gar_process_device(gar_resampler* r, const void* in, int32_t in_dtype, int64_t in_fs, int64_t in_cs,
                              int64_t frames, int32_t channels, void* out, int32_t out_dtype, int64_t out_fs,
                              int64_t out_cs, int64_t out_cap, int64_t* out_frames, void* stream) {
    if (!r) return guard(GAR_ERR_INVALID_ARGUMENT, "nil resampler");
    if (out_frames) *out_frames = 0;
    if (channels != r->channels) {
        g_err = "expected " + std::to_string(r->channels) + " channels, got " + std::to_string(channels);
        return GAR_ERR_CHANNEL_MISMATCH;
    }
    if (frames < 0) return guard(GAR_ERR_INVALID_ARGUMENT, "negative length");
    if (frames > 0 && !in) return guard(GAR_ERR_INVALID_ARGUMENT, "input is NULL");
    if (!ioTypeOk(in_dtype) || !ioTypeOk(out_dtype)) return guard(GAR_ERR_INVALID_ARGUMENT, "unknown sample type");
    if (r->groups.size() != 1) return guard(GAR_ERR_NOT_SUPPORTED, "channels are not in lockstep (per-channel calls were made)");
    return callOn(r, static_cast<hipStream_t>(stream), [&]() -> gar_status {
        hipStream_t s = static_cast<hipStream_t>(stream);  // NULL = legacy default stream
        const bool fuse = pcmFusable(r);
        InView iv;
        iv.p = in;
        iv.f64 = in_dtype == GAR_F64 ? 1 : 0;
        iv.fs = in_fs;
        iv.cs = in_cs;
        iv.n = frames;
        if (isPcm(in_dtype)) {
            iv.f64 = 0;
            if (fuse) {
                iv.pcm = in_dtype;
            } else if (!r->dry) {  // staged: PCM -> compute dtype, then the ordinary path
                const int cf = r->f64 ? 1 : 0;
                r->inStage.ensure(static_cast<size_t>(std::max<int64_t>(frames, 1)) * r->channels * (cf ? 8 : 4));
                HIPCHK(launchConvert(in, in_dtype, in_fs, in_cs, r->inStage.p, cf, r->channels, 1, frames, r->channels, s));
                iv.p = r->inStage.p;
                iv.f64 = cf;
                iv.fs = r->channels;
                iv.cs = 1;
            }
        }
        OutView ov;
        ov.p = out;
        ov.f64 = out_dtype == GAR_F64 ? 1 : 0;
        ov.fs = out_fs;
        ov.cs = out_cs;
        const bool stageOut = isPcm(out_dtype) && !fuse && !r->dry;
        if (isPcm(out_dtype)) {
            ov.f64 = 0;
            if (fuse) ov.pcm = out_dtype;
        }
        if (stageOut) {
            std::vector<int64_t> sz;
            const int64_t need = simulate(r, r->groups[0], frames, false, sz);
            const int cf = r->f64 ? 1 : 0;
            r->outStage.ensure(static_cast<size_t>(std::max<int64_t>(need, 1)) * r->channels * (cf ? 8 : 4));
            ov.p = r->outStage.p;
            ov.f64 = cf;
            ov.fs = r->channels;
            ov.cs = 1;
        }
        gar_status st;
        const int64_t got = runGroup(r, r->groups[0], iv, ov, false, s, out_cap, st);
        if (st == GAR_OK && stageOut && got > 0)
            HIPCHK(launchConvert(r->outStage.p, r->f64 ? 1 : 0, r->channels, 1, out, out_dtype, out_fs, out_cs, got,
                                 r->channels, s));
        if (st == GAR_OK && out_frames) *out_frames = got;
        return st;
    });
}

gar_status gar_flush_device(gar_resampler* r, int32_t channels, void* out, int32_t out_dtype, int64_t out_fs,
                            int64_t out_cs, int64_t out_cap, int64_t* out_frames, void* stream) {
    if (!r) return guard(GAR_ERR_INVALID_ARGUMENT, "nil resampler");
    if (out_frames) *out_frames = 0;
    if (channels != r->channels) {
        g_err = "expected " + std::to_string(r->channels) + " channels, got " + std::to_string(channels);
        return GAR_ERR_CHANNEL_MISMATCH;
    }
    if (!ioTypeOk(out_dtype)) return guard(GAR_ERR_INVALID_ARGUMENT, "unknown sample type");
    if (r->groups.size() != 1) return guard(GAR_ERR_NOT_SUPPORTED, "channels are not in lockstep");
    return callOn(r, static_cast<hipStream_t>(stream), [&]() -> gar_status {
        hipStream_t s = static_cast<hipStream_t>(stream);  // NULL = legacy default stream
        const bool fuse = pcmFusable(r);
        OutView ov;
        ov.p = out;
        ov.f64 = out_dtype == GAR_F64 ? 1 : 0;
        ov.fs = out_fs;
        ov.cs = out_cs;
        const bool stageOut = isPcm(out_dtype) && !fuse && !r->dry;
        if (isPcm(out_dtype)) {
            ov.f64 = 0;
            if (fuse) ov.pcm = out_dtype;
        }
        if (stageOut) {
            std::vector<int64_t> sz;
            const int64_t need = simulate(r, r->groups[0], 0, true, sz);
            const int cf = r->f64 ? 1 : 0;
            r->outStage.ensure(static_cast<size_t>(std::max<int64_t>(need, 1)) * r->channels * (cf ? 8 : 4));
            ov.p = r->outStage.p;
            ov.f64 = cf;
            ov.fs = r->channels;
            ov.cs = 1;
        }
        gar_status st;
        const int64_t got = runGroup(r, r->groups[0], InView(), ov, true, s, out_cap, st);
        if (st == GAR_OK && stageOut && got > 0)
            HIPCHK(launchConvert(r->outStage.p, r->f64 ? 1 : 0, r->channels, 1, out, out_dtype, out_fs, out_cs, got,
                                 r->channels, s));
        if (st == GAR_OK && out_frames) *out_frames = got;
        return st;
    });
}

void gar_reset(gar_resampler* r) {
    if (!r) return;
    DeviceGuard dg(r->dry ? -1 : r->device);
    try {
        if (!r->dry) (void)devFault(r);  // a raised status word takes the recovery path (and is cleared there)
        if (r->poisoned) {  // recover: drain the handle's streams, fresh state
            // the failing call recorded no order event, and launches it already queued on its
            // caller stream may still read the histories and scratch freed below: drain the failing
            // call's stream through the event recorded on it (the caller may have destroyed it), then
            // the earlier calls (drainOrder: their order event, or -- a handle used on one stream
            // records none -- the whole device, gar.h gar_process_device)
            if (r->failEvValid) (void)hipEventSynchronize(r->failEv);
            if (r->stream) (void)hipStreamSynchronize(r->stream);
            drainOrder(r);
            (void)hipGetLastError();
            if (r->errHost) __atomic_store_n(r->errHost, 0, __ATOMIC_RELEASE);  // every launch that could write it has drained
            r->groups.clear();
            r->groups.push_back(freshGroup(r, 0, r->channels));
            r->poisoned = false;
            r->failEvValid = false;
            r->orderValid = false;
            return;
        }
        // one group over every channel: reset in place, keeping its device buffers
        // (stream order covers kernels still reading them; no allocation, no sync)
        if (r->groups.size() == 1 && r->groups[0].c0 == 0 && r->groups[0].C == r->channels) {
            gar::Group& g = r->groups[0];
            for (size_t i = 0; i < g.cnt.size(); ++i) {
                g.cnt[i] = gar::Counters();
                g.cnt[i].staged = !r->stages[i]->fused;
            }
            for (auto& d : g.dev) {
                d.xh.clear();
                d.uh.clear();
            }
            g.statIn = g.statOut = 0;
            return;
        }
        if (r->stream) (void)hipStreamSynchronize(r->stream);
        drainOrder(r);
        r->groups.clear();
        r->groups.push_back(freshGroup(r, 0, r->channels));
    } catch (...) {
    }
}

double gar_get_ratio(const gar_resampler* r) { return r ? r->ratio : 0.0; }

int32_t gar_get_latency(const gar_resampler* r) {
    if (!r || r->stages.empty()) return 0;
    int tot = 0;
    for (const auto& s : r->stages) tot += static_cast<int>(static_cast<double>(stageLatency(s->d)) * s->d.ratio);
    return tot;
}

int32_t gar_channels(const gar_resampler* r) { return r ? r->channels : 0; }

gar_status gar_get_statistics(const gar_resampler* r, int32_t ch, int64_t* samples_in, int64_t* samples_out) {
    if (samples_in) *samples_in = 0;
    if (samples_out) *samples_out = 0;
    if (!r || ch < 0 || ch >= r->channels) return guard(GAR_ERR_INVALID_ARGUMENT, "channel out of range");
    const Group* g = groupOf(const_cast<gar_resampler*>(r), ch);
    if (!g) return guard(GAR_ERR_INTERNAL, "channel without a group");
    if (samples_in) *samples_in = g->statIn;
    if (samples_out) *samples_out = g->statOut;
    return GAR_OK;
}

gar_status gar_get_info(const gar_resampler* r, gar_info* info) {
    if (!r || !info) return GAR_ERR_INVALID_ARGUMENT;
    std::memset(info, 0, sizeof(*info));
    std::snprintf(info->algorithm, sizeof(info->algorithm), "%s", "multi-stage");
    info->latency = gar_get_latency(r);
    // MemoryUsage as the reference counts it for a fresh handle (constant.go:457-468), per channel:
    //  * every ring buffer's capacity in float64 -- defaultBufferSize 8192, buffer 0 sized
    //    MaxInputSize * bufferSizeMultiplier when set (constant.go:72-78, constants.go:55-57);
    //  * StageAdapter.GetMemoryUsage (stage_adapter.go:66-96) of each stage, whose elements are
    //    float64 on the New path (Resampler[float64], stages.go:63): the DFT pre-stage's
    //    factor x taps coefficients + history capacity taps * historyBufferMultiplier (2,
    //    dft_stage.go:142), the polyphase stage's `a` bank L x taps + history capacity 2 * taps
    //    (polyphase_stage.go:167); decimation stages are not counted.
    // The reference's history capacities then grow with use (appendStable, polyphase.go:36-44);
    // the device histories here are shared per group, so the figure stays the fresh one.
    const int64_t es = 8;
    int64_t perCh = 0;
    for (size_t j = 0; j <= r->stages.size(); ++j)
        perCh += (j == 0 && r->cfg.max_input_size > 0 ? r->cfg.max_input_size * 2 : 8192) * 8;
    for (const auto& s : r->stages) {
        const EngineDesign& d = s->d;
        if ((d.kind == EngineKind::DftOnly || d.kind == EngineKind::DftPoly) && d.dft.factor > 1)
            perCh += static_cast<int64_t>(d.dft.factor) * d.dft.taps * es + 2 * static_cast<int64_t>(d.dft.taps) * es;
        if (d.kind == EngineKind::DftPoly)
            perCh += static_cast<int64_t>(d.poly.L) * d.poly.taps * es + 2 * static_cast<int64_t>(d.poly.taps) * es;
    }
    info->memory_usage = perCh * r->channels;
    if (!r->stages.empty()) {
        const EngineDesign& d = r->stages[0]->d;
        int len = 0;
        if ((d.kind == EngineKind::DftOnly || d.kind == EngineKind::DftPoly) && d.dft.factor > 1) len += d.dft.taps * d.dft.factor;
        if (d.kind == EngineKind::DftPoly) len += d.poly.taps * d.poly.L;
        if (d.kind == EngineKind::Cubic) {
            // CubicStage: 4 points, no phases, no SIMD info (cubic.go:119-137)
            info->filter_length = 4;
            info->phases = 0;
            info->memory_usage += 64 * r->channels;  // cubicMemoryUsage (internal/engine/constants.go:15)
        } else {
            info->filter_length = len;
            info->phases = d.kind == EngineKind::DftPoly ? d.poly.L : 0;
            info->simd_enabled = 1;
            std::snprintf(info->simd_type, sizeof(info->simd_type), "%s", "gfx950 MFMA (HIP)");
        }
    }
    return GAR_OK;
}

const char* gar_status_string(gar_status s) {
    switch (s) {
        case GAR_OK: return "ok";
        case GAR_ERR_INVALID_CONFIG: return "invalid resampler configuration";
        case GAR_ERR_BUFFER_TOO_SMALL: return "output buffer too small";
        case GAR_ERR_NOT_SUPPORTED: return "operation not supported";
        case GAR_ERR_CHANNEL_MISMATCH: return "channel count mismatch";
        case GAR_ERR_DEVICE: return "device error";
        case GAR_ERR_INTERNAL: return "internal error";
        case GAR_ERR_INVALID_ARGUMENT: return "invalid argument";
    }
    return "unknown";
}

const char* gar_last_error(void) { return g_err.c_str(); }

void gar_profile_enable(gar_resampler* r, int32_t on) {
    if (!r) return;
    r->profile = on != 0;
}

int64_t gar_dev_pool_selftest(int32_t threads, int32_t iters, int32_t channels, int64_t frames) {
    if (threads < 1 || iters < 0 || channels < 1 || frames < 0) return -1;
    std::atomic<int64_t> bad{0};
    // thread t uses channels + t channels, so consecutive jobs on the pool have different job
    // counts (whole-channel jobs for C >= 2 * workers, channel slices below) -- the case where a
    // stale ticket could claim an index of the next job
    auto body = [&](int t) {
        const int channels_t = channels + t;
        std::vector<double> src(static_cast<size_t>(channels_t) * frames), dst(src.size());
        std::vector<float> mid(src.size());
        for (size_t i = 0; i < src.size(); ++i) src[i] = static_cast<double>((i * 2654435761u + t) % 65536) / 65536.0 - 0.5;
        for (int k = 0; k < iters; ++k) {
            std::fill(dst.begin(), dst.end(), -9.0);
            gar::forSlices(channels_t, frames, 12, [&](int c, int64_t lo, int64_t hi) {
                gar::packChannel<double>(mid.data() + static_cast<size_t>(c) * frames, false,
                                         src.data() + static_cast<size_t>(c) * frames, lo, hi);
            });
            gar::forSlices(channels_t, frames, 12, [&](int c, int64_t lo, int64_t hi) {
                gar::unpackChannel<double>(dst.data() + static_cast<size_t>(c) * frames, false,
                                           mid.data() + static_cast<size_t>(c) * frames, lo, hi);
            });
            int64_t b = 0;
            for (size_t i = 0; i < src.size(); ++i) b += dst[i] != static_cast<double>(static_cast<float>(src[i]));
            bad += b;
        }
    };
    std::vector<std::thread> th;
    for (int t = 1; t < threads; ++t) th.emplace_back(body, t);
    body(0);
    for (auto& x : th) x.join();
    return bad.load();
}

void gar_profile_kinds(gar_resampler* r, uint32_t kinds) {
    if (!r) return;
    r->profileKinds = kinds & 0x3fu;
}

gar_status gar_stage_state(const gar_resampler* r, int32_t stage, int32_t* fused_plan, int32_t* fused_now) {
    if (!r || !fused_plan || !fused_now || stage < 0 || stage >= static_cast<int32_t>(r->stages.size()))
        return GAR_ERR_INVALID_ARGUMENT;
    const gar::StageRT& st = *r->stages[stage];
    *fused_plan = st.fused ? 1 : 0;
    const gar::Group* g = r->groups.empty() ? nullptr : &r->groups[0];
    *fused_now = (st.fused && g && !g->cnt[stage].staged) ? 1 : 0;
    return GAR_OK;
}

gar_status gar_stage_geometry(const gar_resampler* r, int32_t stage, double* stage_ratio, gar_engine_geometry* geom) {
    if (!r || !geom || stage < 0 || stage >= static_cast<int32_t>(r->stages.size())) return GAR_ERR_INVALID_ARGUMENT;
    const gar::EngineDesign& d = r->stages[stage]->d;
    fillGeometry(d, geom);
    if (stage_ratio) *stage_ratio = d.ratio;
    return GAR_OK;
}

int32_t gar_num_stages(const gar_resampler* r) { return r ? static_cast<int32_t>(r->stages.size()) : 0; }

gar_status gar_profile_read(gar_resampler* r, int32_t kind, double* ms, int64_t* launches) {
    if (!r || kind < 0 || kind > 5) return GAR_ERR_INVALID_ARGUMENT;
    DeviceGuard dg(r->dry ? -1 : r->device);
    return wrap([&]() -> gar_status {
        for (auto& ev : r->events) {
            HIPCHK(hipEventSynchronize(ev.b));
            float t = 0;
            HIPCHK(hipEventElapsedTime(&t, ev.a, ev.b));
            r->profiledMs[ev.tag] += t;
            r->profiledLaunches[ev.tag] += 1;
            r->launchMs[ev.tag].push_back(t);
            r->evPool.emplace_back(ev.a, ev.b);
        }
        r->events.clear();
        if (ms) *ms = r->profiledMs[kind];
        if (launches) *launches = r->profiledLaunches[kind];
        r->profiledMs[kind] = 0;
        r->profiledLaunches[kind] = 0;
        r->readMs[kind].swap(r->launchMs[kind]);
        r->launchMs[kind].clear();
        return GAR_OK;
    });
}

gar_status gar_profile_launch_stats(gar_resampler* r, int32_t kind, double* min_ms, double* median_ms, double* max_ms) {
    if (!r || kind < 0 || kind > 5) return GAR_ERR_INVALID_ARGUMENT;
    std::vector<float> v = r->readMs[kind];
    if (v.empty()) {
        if (min_ms) *min_ms = 0;
        if (median_ms) *median_ms = 0;
        if (max_ms) *max_ms = 0;
        return GAR_OK;
    }
    std::sort(v.begin(), v.end());
    const size_t n = v.size();
    if (min_ms) *min_ms = v.front();
    if (max_ms) *max_ms = v.back();
    if (median_ms) *median_ms = n % 2 ? v[n / 2] : 0.5 * (static_cast<double>(v[n / 2 - 1]) + v[n / 2]);
    return GAR_OK;
}

gar_status gar_design_engine(double in_rate, double out_rate, int32_t q, gar_engine_geometry* geom, double* dft,
                             double* pa, double* pb, double* pc, double* pd, double* decim) {
    EngineDesign d;
    std::string err;
    if (!designEngine(in_rate, out_rate, static_cast<Quality>(q), d, err)) return guard(GAR_ERR_INVALID_CONFIG, err.c_str());
    if (geom) fillGeometry(d, geom);
    if (dft && !d.dft.c.empty()) std::memcpy(dft, d.dft.c.data(), d.dft.c.size() * 8);
    if (pa && !d.poly.a.empty()) std::memcpy(pa, d.poly.a.data(), d.poly.a.size() * 8);
    if (pb && !d.poly.b.empty()) std::memcpy(pb, d.poly.b.data(), d.poly.b.size() * 8);
    if (pc && !d.poly.cc.empty()) std::memcpy(pc, d.poly.cc.data(), d.poly.cc.size() * 8);
    if (pd && !d.poly.d.empty()) std::memcpy(pd, d.poly.d.data(), d.poly.d.size() * 8);
    if (decim && !d.decim.c.empty()) std::memcpy(decim, d.decim.c.data(), d.decim.c.size() * 8);
    return GAR_OK;
}

gar_status gar_design_composite(double in_rate, double out_rate, int32_t q, double* rows, int64_t* offsets) {
    EngineDesign d;
    std::string err;
    if (!designEngine(in_rate, out_rate, static_cast<Quality>(q), d, err)) return guard(GAR_ERR_INVALID_CONFIG, err.c_str());
    FirPeriodic f;
    if (d.kind != EngineKind::DftPoly || !firComposite(d.dft, d.poly, f)) return guard(GAR_ERR_NOT_SUPPORTED, "no composite FIR");
    size_t w = 0;
    for (const auto& r : f.rows) w = std::max(w, r.size());
    for (int r = 0; r < f.P; ++r) {
        if (offsets) offsets[r] = f.off[r];
        if (rows)
            for (size_t k = 0; k < w; ++k) rows[r * w + k] = k < f.rows[r].size() ? f.rows[r][k] : 0.0;
    }
    return GAR_OK;
}

}  // extern "C"
