// gar_design.cpp -- host filter design (see gar_design.hpp).
// Built with -ffp-contract=off: the Go amd64 build does not fuse multiply-add,
// so the design arithmetic is evaluated with separate roundings.
#include "gar_design.hpp"

#include <cmath>
#include <numeric>

namespace gar {
namespace design {

namespace {
// A&S 9.8.1 / 9.8.2 coefficients (internal/mathutil/constants.go:21-41)
constexpr double kSmall[6] = {3.5156229, 3.0899424, 1.2067492, 0.2659732, 0.360768e-1, 0.45813e-2};
constexpr double kLarge[9] = {0.39894228, 0.1328592e-1, 0.225319e-2, -0.157565e-2, 0.916281e-2,
                              -0.2057706e-1, 0.2635537e-1, -0.1647633e-1, 0.392377e-2};
constexpr double kPi = 3.14159265358979323846;

double hornerTail(const double* c, int n, double t) {
    // c[0] + t*(c[1] + t*(... + t*c[n-1]))  -- same nesting as bessel.go:33-45
    double r = c[n - 1];
    for (int i = n - 2; i >= 0; --i) r = c[i] + t * r;
    return r;
}

double sequentialSum(const std::vector<double>& v) {
    double s = 0.0;
    for (double x : v) s += x;
    return s;
}
}  // namespace

double besselI0(double x) {
    const double ax = std::fabs(x);
    if (ax < 3.75) {
        double t = x / 3.75;
        t *= t;
        return 1.0 + t * hornerTail(kSmall, 6, t);
    }
    const double t = 3.75 / ax;
    return std::exp(ax) * hornerTail(kLarge, 9, t) / std::sqrt(ax);
}

double kaiserBeta(double att) {
    if (att > 50.0) return 0.1102 * (att - 8.7);
    if (att >= 21.0) {
        const double d = att - 21.0;
        return 0.5842 * std::pow(d, 0.4) + 0.07886 * d;
    }
    return 0.0;
}

int estimateFilterLength(double att, double tbw) {
    if (tbw <= 0) tbw = 0.01;
    const double n = (att - 8.0) / (2.285 * 2.0 * kPi * tbw);
    int taps = static_cast<int>(std::ceil(n));
    taps |= 1;  // force odd
    if (taps < 3) taps = 3;
    if (taps > 8191) taps = 8191;
    return taps;
}

std::vector<double> kaiserWindow(int length, double beta) {
    std::vector<double> w(length > 0 ? length : 0);
    if (length < 1) return w;
    if (length == 1) { w[0] = 1.0; return w; }
    beta = std::fabs(beta);
    const double alpha = static_cast<double>(length - 1) / 2.0;
    const double i0b = besselI0(beta);
    for (int n = 0; n < length; ++n) {
        const double x = (static_cast<double>(n) - alpha) / alpha;
        const double arg = beta * std::sqrt(1.0 - x * x);
        const double i0a = besselI0(arg);
        w[n] = (std::isinf(i0a) && i0a > 0 && std::isinf(i0b) && i0b > 0) ? std::exp(arg - beta) : i0a / i0b;
    }
    return w;
}

bool designLowPass(int numTaps, double cutoff, double att, double gain, std::vector<double>& out) {
    if (numTaps < 3 || numTaps > 8191 || !(cutoff > 0 && cutoff < 0.5) || att < 0 || att > 500 || !(gain > 0))
        return false;
    const std::vector<double> win = kaiserWindow(numTaps, kaiserBeta(att));
    out.assign(numTaps, 0.0);
    const double center = static_cast<double>(numTaps - 1) / 2.0;
    for (int n = 0; n < numTaps; ++n) {
        const double x = static_cast<double>(n) - center;
        double s;
        if (std::fabs(x) < 1e-10) {
            s = 2.0 * cutoff;
        } else {
            const double arg = 2.0 * kPi * cutoff * x;
            s = std::sin(arg) / (kPi * x);
        }
        out[n] = s * win[n];
    }
    const double sum = sequentialSum(out);
    if (std::fabs(sum) > 1e-10) {
        const double scale = gain / sum;
        for (double& v : out) v = v * scale;
    }
    return true;
}

bool designLowPassAuto(double cutoff, double tbw, double att, double gain, std::vector<double>& out) {
    return designLowPass(estimateFilterLength(att, tbw), cutoff, att, gain, out);
}

double attenuationFor(Quality q) {
    int bits;
    switch (q) {
        case Quality::Quick: bits = 8; break;
        case Quality::Low: case Quality::Medium: case Quality::Bits16: bits = 16; break;
        case Quality::High: case Quality::Bits20: bits = 20; break;
        case Quality::Bits24: bits = 24; break;
        case Quality::VeryHigh: case Quality::Bits28: bits = 28; break;
        case Quality::Bits32: bits = 32; break;
        default: bits = 20; break;
    }
    return (bits + 1) * 6.0206;
}

double passbandEndFor(Quality q) {
    switch (q) {
        case Quality::Quick: case Quality::Low: case Quality::Bits16: return 0.67625;
        case Quality::Medium: return 0.91;
        case Quality::High: case Quality::Bits20: return 0.912;
        case Quality::VeryHigh: case Quality::Bits24: case Quality::Bits28: case Quality::Bits32: return 0.913;
        default: return 0.912;
    }
}

void findRationalApprox(double ratio, int& numPhases, int& step) {
    const double inv = 1.0 / ratio;
    int bestL = 80;
    int bestStep = static_cast<int>(std::round(inv * 80.0));
    double bestErr = std::fabs(static_cast<double>(bestStep) / bestL - inv);
    for (int L = 64; L <= 256; ++L) {
        const int cand = static_cast<int>(std::round(inv * static_cast<double>(L)));
        if (cand <= 0) continue;
        const double e = std::fabs(static_cast<double>(cand) / static_cast<double>(L) - inv);
        if (e < bestErr) { bestL = L; bestStep = cand; bestErr = e; }
        if (bestErr < 1e-10) break;
    }
    numPhases = bestL;
    step = bestStep;
}

double lsxInvFResp(double drop, double a) {
    a = a < 1.0 ? 1.0 : (a > 300.0 ? 300.0 : a);
    double x = ((2.0517e-07 * a + -1.1303e-04) * a + 0.023154) * a + 0.55924;
    const double dropLin = std::exp(drop * 2.30258509299404568402 * 0.05);
    const double s = dropLin > 0.5 ? 1 - dropLin : dropLin;
    double sv = std::sin(x * 0.5);
    if (sv <= 1e-10) sv = 1e-10;
    const double sinePow = std::log(0.5) / std::log(sv);
    x = std::asin(std::pow(s, 1.0 / sinePow)) / x;
    return dropLin > 0.5 ? x : 1 - x;
}

bool isIntegerRatio(double r) {
    const double rr = std::round(r);
    return std::fabs(r - rr) < 1e-9 && rr >= 1.0;
}

PolyParams polyphaseParams(int L, double ratio, double tio, bool hasPre, double att, double pbe) {
    PolyParams p;
    const double phases = static_cast<double>(L);
    p.upsampling = tio < 1.0;
    p.mult = p.upsampling ? 1.0 : tio;
    if (p.upsampling) { p.fp1 = tio * pbe; p.fs1 = tio * 1.0; }
    else { p.fp1 = pbe * ratio; p.fs1 = ratio; }
    if (!p.upsampling && hasPre) {
        p.fn = 2.0 * p.mult;
        p.fsRaw = 3.0 + std::fabs(p.fs1 - 1.0);
    } else {
        p.fn = 1.0;
        p.fsRaw = 2.0 - (p.fp1 + (p.fs1 - p.fp1) * 0.7);
    }
    p.fpRaw = p.fp1;
    const double inv = lsxInvFResp(-0.01, att);
    if (inv < 0.999) {
        const double adj = p.fsRaw - (p.fsRaw - p.fpRaw) / (1.0 - inv);
        if (adj > 0 && adj < p.fsRaw) p.fpRaw = adj;
    }
    p.fp = p.fpRaw / std::fabs(p.fn);
    p.fs = p.fsRaw / std::fabs(p.fn);
    p.trBw = 0.5 * (p.fs - p.fp);
    p.trBw /= phases;
    const double lim = 0.5 * p.fs / phases;
    if (p.trBw > lim) p.trBw = lim;
    if (p.trBw < 0.001) p.trBw = 0.001;
    p.fc = p.fs / phases - p.trBw;
    if (p.fc < 0.001) p.fc = 0.001;
    const int maxTaps = att < 110.0 ? 32 : att < 130.0 ? 64 : att < 160.0 ? 100 : 8191 / L;
    p.totalTaps = static_cast<int>(std::ceil(att / p.trBw + 1));
    p.tapsPerPhase = (p.totalTaps + L - 1) / L;
    if (p.tapsPerPhase < 8) p.tapsPerPhase = 8;
    else if (p.tapsPerPhase > maxTaps) p.tapsPerPhase = maxTaps;
    p.totalTaps = L * p.tapsPerPhase - 1;
    if (p.totalTaps > 8190) {
        p.tapsPerPhase = std::max(8191 / L, 8);
        p.totalTaps = L * p.tapsPerPhase - 1;
    }
    return p;
}

}  // namespace design

// ---------------------------------------------------------------------------
namespace {

// dft_stage.go:50-146
bool makeDft(int factor, Quality q, DftBank& b) {
    b = DftBank();
    b.factor = factor;
    if (factor == 1) return true;
    std::vector<double> proto;
    if (!design::designLowPassAuto(0.4778321 / factor, 0.05 / factor, design::attenuationFor(q), 1.0, proto))
        return false;
    const int n = static_cast<int>(proto.size());
    b.taps = (n + factor - 1) / factor;
    b.c.assign(static_cast<size_t>(factor) * b.taps, 0.0);
    for (int p = 0; p < factor; ++p)
        for (int t = 0; t < b.taps; ++t) {
            const int idx = t * factor + p;
            if (idx < n) b.c[static_cast<size_t>(p) * b.taps + (b.taps - 1 - t)] = proto[idx] * factor;
        }
    if (factor == 2) {  // half-band passthrough detection (dft_stage.go:112-133)
        int nsig = 0, where = 0;
        double val = 0;
        for (int i = 0; i < b.taps; ++i)
            if (std::fabs(b.c[i]) > 1e-8) { ++nsig; where = i; val = b.c[i]; }
        if (nsig == 1 && std::fabs(val - 1.0) < 0.01) { b.halfBand = true; b.p0Offset = where; b.p0Scale = val; }
    }
    return true;
}

// dft_stage.go:401-475
bool makeDecim(int factor, Quality q, DecimBank& b) {
    b = DecimBank();
    b.factor = factor;
    if (factor == 1) return true;
    const double fpN = design::passbandEndFor(q) / factor, fsN = 1.0 / factor;
    const double trBw = 0.5 * (fsN - fpN);
    const double fc = fsN - trBw;
    std::vector<double> proto;
    if (!design::designLowPassAuto(fc * 0.5, trBw * 0.5, design::attenuationFor(q), 1.0, proto)) return false;
    b.taps = static_cast<int>(proto.size());
    b.c.assign(proto.rbegin(), proto.rend());
    return true;
}

// polyphase_stage.go:69-170 + designPolyphaseFilter filter_params.go:229-286
bool makePoly(double ratio, double tio, bool hasPre, Quality q, PolyBank& b, std::string& err) {
    if (!(ratio > 0)) { err = "ratio must be positive"; return false; }
    int L = 0, unused = 0;
    design::findRationalApprox(ratio, L, unused);
    const double att = design::attenuationFor(q);
    const design::PolyParams pp = design::polyphaseParams(L, ratio, tio, hasPre, att, design::passbandEndFor(q));
    double cutoff = pp.fc / 2.0;
    if (cutoff <= 0) cutoff = 0.001;
    if (cutoff >= 0.5) cutoff = 0.499;
    std::vector<double> proto;
    if (!design::designLowPass(pp.totalTaps, cutoff, att, 1.0, proto)) {
        err = "failed to design prototype filter";
        return false;
    }
    double sum = 0.0;
    for (double v : proto) sum += v;
    if (sum != 0) {
        const double scale = static_cast<double>(L) / sum;
        for (double& v : proto) v = v * scale;
    }
    const int T = pp.tapsPerPhase;
    // coeffs[tap*L + phase]; the bank has T*L entries, the prototype T*L-1.
    auto coef = [&](int phase, int tap) -> double {
        int w = phase % L;
        if (w < 0) w += L;
        const long idx = static_cast<long>(tap) * L + w;
        return (idx >= 0 && idx < static_cast<long>(proto.size())) ? proto[idx] : 0.0;
    };
    b = PolyBank();
    b.L = L;
    b.taps = T;
    b.step = static_cast<int64_t>(std::round((1.0 / ratio) * static_cast<double>(L) * 65536.0));
    const size_t n = static_cast<size_t>(L) * T;
    b.a.assign(n, 0); b.b.assign(n, 0); b.cc.assign(n, 0); b.d.assign(n, 0);
    for (int ph = 0; ph < L; ++ph)
        for (int t = 0; t < T; ++t) {
            const double f0 = coef(ph, t), f1 = coef(ph + 1, t), fm1 = coef(ph - 1, t), f2 = coef(ph + 2, t);
            const double c = 0.5 * (f1 + fm1) - f0;
            const double d = (1.0 / 6.0) * (f2 - f1 + fm1 - f0 - 4.0 * c);
            const double bb = f1 - f0 - d - c;
            const size_t o = static_cast<size_t>(ph) * T + (T - 1 - t);
            b.a[o] = f0; b.b[o] = bb; b.cc[o] = c; b.d[o] = d;
        }
    return true;
}
}  // namespace

bool designEngine(double inRate, double outRate, Quality q, EngineDesign& e, std::string& err) {
    if (!(inRate > 0) || !(outRate > 0)) { err = "sample rates must be positive"; return false; }
    const double ratio = outRate / inRate;
    if (ratio < 1.0 / 256.0 || ratio > 256.0) { err = "resampling ratio out of valid range"; return false; }
    e = EngineDesign();
    e.inRate = inRate; e.outRate = outRate; e.ratio = ratio; e.quality = q;
    if (q == Quality::Quick) { e.kind = EngineKind::Cubic; return true; }
    if (ratio >= 1.0) {
        if (design::isIntegerRatio(ratio)) {
            const int f = static_cast<int>(std::round(ratio));
            if (!makeDft(f, q, e.dft)) { err = "failed to create DFT stage"; return false; }
            e.kind = f == 1 ? EngineKind::Passthrough : EngineKind::DftOnly;
            return true;
        }
        if (!makeDft(2, q, e.dft)) { err = "failed to create DFT pre-stage"; return false; }
        if (!makePoly(outRate / (inRate * 2.0), inRate / outRate, true, q, e.poly, err)) return false;
        e.kind = EngineKind::DftPoly;
        return true;
    }
    const double io = inRate / outRate;
    if (design::isIntegerRatio(io) && io >= 2.0) {
        if (!makeDecim(static_cast<int>(std::round(io)), q, e.decim)) { err = "failed to create DFT decimation stage"; return false; }
        e.kind = EngineKind::Decim;
        return true;
    }
    if (!makeDft(2, q, e.dft)) { err = "failed to create DFT pre-stage"; return false; }
    if (!makePoly(outRate / (inRate * 2.0), io, false, q, e.poly, err)) return false;
    e.kind = EngineKind::DftPoly;
    return true;
}

// ---------------------------------------------------------------------------
std::vector<StageSpec> buildPipeline(double ratio, int precision) {
    std::vector<StageSpec> st;
    if (precision <= 8) { st.push_back({StageType::Cubic, ratio}); return st; }
    double rem = ratio;
    if (ratio < 1.0)
        while (rem < 0.5) { st.push_back({StageType::HalfBand, 0.5}); rem *= 2.0; }
    if (ratio > 1.0)
        while (rem > 2.0) { st.push_back({StageType::HalfBand, 2.0}); rem /= 2.0; }
    if (std::fabs(rem - 1.0) > 0.001) {
        static const double common[6] = {44100.0 / 48000.0, 48000.0 / 44100.0, 44100.0 / 88200.0,
                                         88200.0 / 44100.0, 48000.0 / 96000.0, 96000.0 / 48000.0};
        bool fft = precision >= 28;
        for (double c : common) fft = fft || std::fabs(rem - c) < 0.0001;
        st.push_back({fft ? StageType::FFT : StageType::Polyphase, rem});
    }
    return st;
}

Quality precisionToEngineQuality(int p) {
    if (p <= 8) return Quality::Quick;
    if (p <= 16) return Quality::Low;
    if (p <= 20) return Quality::High;
    if (p <= 24) return Quality::Bits24;
    if (p <= 28) return Quality::VeryHigh;
    return Quality::Bits32;
}

Quality presetToEngineQuality(int preset) {
    switch (preset) {
        case 0: case 1: return Quality::Low;
        case 2: return Quality::Medium;
        case 3: case 4: return Quality::High;
        default: return Quality::Medium;
    }
}

}  // namespace gar
