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
};

FirPeriodic firFromDft(const DftBank& d);
FirPeriodic firFromDecim(const DecimBank& d);
bool firFromPoly(const PolyBank& p, FirPeriodic& out);                          // needs fracFree()
bool firComposite(const DftBank& d, const PolyBank& p, FirPeriodic& out);       // needs factor 2 + fracFree()

// Task = (row block, K slice) executed by one wavefront.
struct BgTask { int rb, k0, ns, ks, nks; };

struct BgPlan {
    bool f64 = false;
    int P = 0, Q = 0, mp = 1;         // macro period = mp periods
    int Pc = 0, Qc = 0;               // outputs / inputs per macro period
    int nrb = 0;                      // row blocks of 16 outputs
    int Kc = 0;                       // input window (elements) one macro period needs
    int NS = 0;                       // steps per task (template bucket)
    bool ksplit = false;
    std::vector<BgTask> tasks;
    std::vector<float> A32;           // [ntasks][NS][64] MFMA A fragments
    std::vector<double> A64;
    double usefulMacsPerOutput = 0;   // sum of row lengths / P
    double mfmaMacsPerOutput = 0;     // executed MFMA MACs / output (incl. band padding)
};

// Builds the MFMA plan; maxNS bounds steps per task (register budget).
bool buildBgPlan(const FirPeriodic& f, bool f64, BgPlan& plan);

}  // namespace gar
