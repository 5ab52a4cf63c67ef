// gar_design.hpp -- host-side filter design for the MI355X resampling engine.
//
// Designs the exact coefficient banks the Go reference designs (it is the
// product's own implementation; the CPU oracle under oracle/ is only used by
// tests to check it).  Citations are path:line in tphakala/go-audio-resampler.
#pragma once
#include <cstdint>
#include <string>
#include <vector>

namespace gar {

// engine.Quality (internal/engine/filter_params.go:16-41)
enum class Quality : int {
    Quick = 0, Low, Medium, High, VeryHigh, Bits16, Bits20, Bits24, Bits28, Bits32
};

namespace design {

double besselI0(double x);                                  // internal/mathutil/bessel.go:22
double kaiserBeta(double attenuationDb);                    // bessel.go:126
int estimateFilterLength(double attenuationDb, double tbw); // bessel.go:245
std::vector<double> kaiserWindow(int length, double beta);  // internal/filter/kaiser.go:47
// kaiser.go:159 (returns false on invalid parameters, kaiser.go:112-138)
bool designLowPass(int numTaps, double cutoff, double attenuationDb, double gain, std::vector<double>& out);
bool designLowPassAuto(double cutoff, double tbw, double attenuationDb, double gain, std::vector<double>& out);

double attenuationFor(Quality q);   // filter_params.go:150
double passbandEndFor(Quality q);   // filter_params.go:180
void findRationalApprox(double ratio, int& numPhases, int& step); // filter_params.go:294
double lsxInvFResp(double drop, double a);                        // filter_params.go:355
bool isIntegerRatio(double r);                                    // internal/engine/resampler.go:356

struct PolyParams {  // filter_params.go:402-428
    bool upsampling = false;
    double mult = 0, fn = 0, fp1 = 0, fs1 = 0, fpRaw = 0, fsRaw = 0, fp = 0, fs = 0, trBw = 0, fc = 0;
    int totalTaps = 0, tapsPerPhase = 0;
};
PolyParams polyphaseParams(int numPhases, double ratio, double totalIORatio, bool hasPreStage,
                           double attenuationDb, double passbandEnd);  // filter_params.go:446

}  // namespace design

// ---------------------------------------------------------------------------
// Coefficient banks, stored exactly as the Go stages store them.
// ---------------------------------------------------------------------------
struct DftBank {          // internal/engine/dft_stage.go:22-146
    int factor = 1;
    int taps = 0;                 // tapsPerPhase
    std::vector<double> c;        // [factor][taps], reversed, scaled by factor
    bool halfBand = false;
    int p0Offset = 0;
    double p0Scale = 1.0;
};

struct DecimBank {        // dft_stage.go:370-475
    int factor = 1;
    int taps = 0;
    std::vector<double> c;        // reversed
};

struct PolyBank {         // internal/engine/polyphase_stage.go:25-170
    int L = 0, taps = 0;
    int64_t step = 0;             // fixed point, 16 fractional bits
    std::vector<double> a, b, cc, d;  // [L][taps], reversed
    bool fracFree() const { return (step & 0xFFFF) == 0; }
};

// engine.NewResampler[F] stage architecture (internal/engine/resampler.go:51-179)
enum class EngineKind : int { Cubic = 0, DftOnly = 1, DftPoly = 2, Decim = 3, Passthrough = 4 };

struct EngineDesign {
    EngineKind kind = EngineKind::Passthrough;
    double inRate = 0, outRate = 0, ratio = 0;
    Quality quality = Quality::High;
    DftBank dft;
    PolyBank poly;
    DecimBank decim;
};

// Returns false + message on the reference's constructor errors.
bool designEngine(double inRate, double outRate, Quality q, EngineDesign& out, std::string& err);

// ---------------------------------------------------------------------------
// Top-level pipeline (internal/pipeline/pipeline.go:104-183, stages.go)
// ---------------------------------------------------------------------------
enum class StageType : int { Cubic = 0, HalfBand = 1, Polyphase = 2, FFT = 3 };
struct StageSpec { StageType type; double ratio; };
std::vector<StageSpec> buildPipeline(double ratio, int precision);   // pipeline.go:104
Quality precisionToEngineQuality(int precision);                     // stages.go:92
Quality presetToEngineQuality(int preset);                           // convenience.go:189

}  // namespace gar
