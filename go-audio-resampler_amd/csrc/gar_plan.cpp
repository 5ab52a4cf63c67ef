// gar_plan.cpp -- periodic-FIR descriptions and MFMA banded-GEMM plans.
#include "gar_plan.hpp"

#include <algorithm>
#include <numeric>

namespace gar {

FirPeriodic firFromDft(const DftBank& d) {
    FirPeriodic f;
    f.P = d.factor;
    f.Q = 1;
    f.off.assign(d.factor, 0);
    for (int p = 0; p < d.factor; ++p)
        f.rows.emplace_back(d.c.begin() + static_cast<long>(p) * d.taps, d.c.begin() + static_cast<long>(p + 1) * d.taps);
    return f;
}

FirPeriodic firFromDecim(const DecimBank& d) {
    FirPeriodic f;
    f.P = 1;
    f.Q = d.factor;
    f.off.assign(1, 0);
    f.rows.push_back(d.c);
    return f;
}

bool firFromPoly(const PolyBank& p, FirPeriodic& f) {
    if (!p.fracFree()) return false;
    const int64_t S = p.step >> 16;
    const int64_t g = std::gcd<int64_t>(S, p.L);
    f = FirPeriodic();
    f.P = static_cast<int>(p.L / g);
    f.Q = static_cast<int>(S / g);
    for (int r = 0; r < f.P; ++r) {
        const int64_t full = r * S;
        f.off.push_back(full / p.L);
        const int ph = static_cast<int>(full % p.L);
        f.rows.emplace_back(p.a.begin() + static_cast<long>(ph) * p.taps, p.a.begin() + static_cast<long>(ph + 1) * p.taps);
    }
    return true;
}

// y_j = sum_k2 a[ph_j][k2] * u[d_j + k2],  u[q] = sum_k1 c[q&1][k1] * x[(q>>1) + k1]
//     = sum_n G_{ph_j, d_j&1}[n] * x[(d_j>>1) + n]
// (polyphase_stage.go:257-293 composed with dft_stage.go:229-273).  The
// composition is exact in real arithmetic; G is accumulated in f64.
bool firComposite(const DftBank& d, const PolyBank& p, FirPeriodic& f) {
    if (d.factor != 2 || !p.fracFree()) return false;
    const int64_t S = p.step >> 16;
    const int64_t L = p.L;
    const int64_t g2 = std::gcd<int64_t>(S, 2 * L);
    f = FirPeriodic();
    f.P = static_cast<int>(2 * L / g2);
    f.Q = static_cast<int>(S / g2);
    const int T1 = d.taps, T2 = p.taps;
    for (int r = 0; r < f.P; ++r) {
        const int64_t full = r * S;
        const int64_t dd = full / L;
        const int ph = static_cast<int>(full % L);
        const int par = static_cast<int>(dd & 1);
        f.off.push_back(dd >> 1);
        const int ng = ((par + T2 - 1) >> 1) + T1;
        std::vector<double> row(ng, 0.0);
        const double* a = p.a.data() + static_cast<long>(ph) * T2;
        for (int k2 = 0; k2 < T2; ++k2) {
            const int q = par + k2;
            const double* c = d.c.data() + static_cast<long>(q & 1) * T1;
            const int sh = q >> 1;
            const double ak = a[k2];
            for (int k1 = 0; k1 < T1; ++k1) row[sh + k1] += ak * c[k1];
        }
        f.rows.push_back(std::move(row));
    }
    return true;
}

namespace {
struct RbGeom { int klo, nsteps; };

// Row r of a macro period of mp periods.
inline void macroRow(const FirPeriodic& f, int r, int64_t& off, const std::vector<double>*& row) {
    const int a = r / f.P, rr = r % f.P;
    off = static_cast<int64_t>(a) * f.Q + f.off[rr];
    row = &f.rows[rr];
}

std::vector<RbGeom> geomFor(const FirPeriodic& f, int mp, double& eff) {
    const int Pc = f.P * mp;
    const int nrb = (Pc + 15) / 16;
    std::vector<RbGeom> g(nrb);
    double useful = 0, executed = 0;
    for (int rb = 0; rb < nrb; ++rb) {
        int64_t lo = INT64_MAX, hi = 0;
        for (int m = 0; m < 16; ++m) {
            const int r = rb * 16 + m;
            if (r >= Pc) break;
            int64_t off;
            const std::vector<double>* row;
            macroRow(f, r, off, row);
            lo = std::min(lo, off);
            hi = std::max<int64_t>(hi, off + static_cast<int64_t>(row->size()));
            useful += static_cast<double>(row->size());
        }
        const int64_t klo = (lo / 4) * 4;
        g[rb].klo = static_cast<int>(klo);
        g[rb].nsteps = static_cast<int>((hi - klo + 3) / 4);
        executed += 64.0 * g[rb].nsteps;
    }
    eff = useful / executed;
    return g;
}
}  // namespace

bool buildBgPlan(const FirPeriodic& f, bool f64, BgPlan& plan) {
    if (f.P <= 0 || f.Q <= 0) return false;
    // Pick the macro period (multiple of the FIR period) with the best
    // useful/executed MAC ratio; prefer >= 16 rows so row blocks are full.
    int bestMp = 1;
    double bestEff = -1;
    for (int mp = 1; mp <= 64; ++mp) {
        const int Pc = f.P * mp;
        if (Pc > 320) break;
        double eff;
        geomFor(f, mp, eff);
        if (Pc < 16) eff *= static_cast<double>(Pc) / 16.0;  // partially filled row block
        if (eff > bestEff + 1e-9) { bestEff = eff; bestMp = mp; }
    }
    double eff;
    const std::vector<RbGeom> rbs = geomFor(f, bestMp, eff);
    plan = BgPlan();
    plan.f64 = f64;
    plan.P = f.P; plan.Q = f.Q; plan.mp = bestMp;
    plan.Pc = f.P * bestMp;
    plan.Qc = f.Q * bestMp;
    plan.nrb = static_cast<int>(rbs.size());
    const int maxNS = f64 ? 48 : 112;
    int needNS = 0;
    for (int rb = 0; rb < plan.nrb; ++rb) {
        const int nst = rbs[rb].nsteps;
        const int nks = (nst + maxNS - 1) / maxNS;
        const int per = (nst + nks - 1) / nks;
        for (int ks = 0; ks < nks; ++ks) {
            BgTask t;
            t.rb = rb;
            t.ks = ks;
            t.nks = nks;
            t.k0 = rbs[rb].klo + 4 * ks * per;
            t.ns = std::min(per, nst - ks * per);
            plan.tasks.push_back(t);
            needNS = std::max(needNS, t.ns);
        }
        if (nks > 1) plan.ksplit = true;
        plan.Kc = std::max(plan.Kc, rbs[rb].klo + 4 * nst);
    }
    // Kernel instantiations exist for NS = 8, 12, ..., maxNS; the A image is
    // zero padded to NS steps so the MFMA loop has no per-step guard.
    plan.NS = std::max(8, (needNS + 3) / 4 * 4);
    if (plan.NS > maxNS) return false;

    const size_t nt = plan.tasks.size();
    const size_t img = nt * plan.NS * 64;
    std::vector<double> A(img, 0.0);
    for (size_t ti = 0; ti < nt; ++ti) {
        const BgTask& t = plan.tasks[ti];
        for (int s = 0; s < t.ns; ++s)
            for (int lane = 0; lane < 64; ++lane) {
                const int m = lane & 15, kq = lane >> 4;
                const int r = t.rb * 16 + m;
                if (r >= plan.Pc) continue;
                int64_t off;
                const std::vector<double>* row;
                macroRow(f, r, off, row);
                const int64_t kk = t.k0 + 4 * s + kq;
                const int64_t idx = kk - off;
                if (idx >= 0 && idx < static_cast<int64_t>(row->size()))
                    A[(ti * plan.NS + s) * 64 + lane] = (*row)[idx];
            }
    }
    if (f64) plan.A64 = std::move(A);
    else plan.A32.assign(A.begin(), A.end());

    double useful = 0;
    for (const auto& r : f.rows) useful += static_cast<double>(r.size());
    plan.usefulMacsPerOutput = useful / f.P;
    double exec = 0;
    for (const auto& t : plan.tasks) exec += 16.0 * 4.0 * t.ns;  // per column per macro period
    plan.mfmaMacsPerOutput = exec / plan.Pc;
    return true;
}

}  // namespace gar
