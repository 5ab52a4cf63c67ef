// gar_plan.cpp -- periodic-FIR descriptions and MFMA banded-GEMM plans.
#include "gar_plan.hpp"

#include <algorithm>
#include <cmath>
#include <cstring>
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
    f.composite = true;
    f.P = static_cast<int>(2 * L / g2);
    f.Q = static_cast<int>(S / g2);
    const int T1 = d.taps, T2 = p.taps;
    for (int r = 0; r < f.P; ++r) {
        const int64_t full = r * S;
        const int64_t dd = full / L;
        const int ph = static_cast<int>(full % L);
        const int par = static_cast<int>(dd & 1);
        f.off.push_back(dd >> 1);
        f.ph.push_back(ph);
        f.par.push_back(par);
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

std::vector<RbGeom> geomFor(const FirPeriodic& f, int mp, double& eff, int kstep = 4, int kalign = 4) {
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
        const int64_t klo = (lo / kalign) * kalign;
        g[rb].klo = static_cast<int>(klo);
        g[rb].nsteps = static_cast<int>((hi - klo + kstep - 1) / kstep);
        executed += 16.0 * kstep * g[rb].nsteps;
    }
    eff = useful / executed;
    return g;
}
}  // namespace

namespace {
// Even split of the row blocks' steps over nprog programs (<= kBgMaxSeg
// segments each); row blocks cut across programs get LDS slots + a reduction.
bool splitPrograms(const std::vector<RbGeom>& rbs, int nprog, std::vector<BgProg>& progs, std::vector<BgRed>& reds,
                   int& nslots, int& maxLen, int kstep = 4) {
    int64_t S = 0;
    for (const auto& r : rbs) S += r.nsteps;
    const int T = static_cast<int>((S + nprog - 1) / nprog);
    progs.assign(nprog, BgProg());
    reds.clear();
    int w = 0;
    std::vector<std::vector<std::pair<int, int>>> owners(rbs.size());  // rb -> (prog, seg)
    for (size_t rb = 0; rb < rbs.size(); ++rb) {
        int pos = 0, rem = rbs[rb].nsteps;
        while (rem > 0) {
            if (w >= nprog) return false;
            BgProg& pg = progs[w];
            if (pg.nseg == kBgMaxSeg) return false;
            const int take = std::min(rem, T - pg.len);
            BgSeg& sg = pg.seg[pg.nseg];
            sg.rb = static_cast<int>(rb);
            sg.k0 = rbs[rb].klo + kstep * pos;
            sg.ns = take;
            sg.start = pg.len;
            owners[rb].push_back({w, pg.nseg});
            pg.nseg++;
            pg.len += take;
            pos += take;
            rem -= take;
            if (pg.len == T) ++w;
        }
    }
    nslots = 0;
    for (size_t rb = 0; rb < rbs.size(); ++rb) {
        if (owners[rb].size() <= 1) continue;
        if (owners[rb].size() > static_cast<size_t>(kBgMaxRedSlots)) return false;
        BgRed r;
        r.rb = static_cast<int>(rb);
        for (const auto& o : owners[rb]) {
            progs[o.first].seg[o.second].slot = nslots;
            r.slot[r.n++] = nslots++;
        }
        reds.push_back(r);
    }
    maxLen = 0;
    for (const auto& pg : progs) maxLen = std::max(maxLen, pg.len);
    return true;
}
}  // namespace

std::vector<int> BgPlan::progTable() const {
    std::vector<int> t(progs.size() * kBgProgInts, 0);
    for (size_t i = 0; i < progs.size(); ++i) {
        int* e = &t[i * kBgProgInts];
        const BgProg& pg = progs[i];
        e[0] = pg.nseg;
        // in-loop flush boundaries (the last segment runs to NS and flushes after the loop)
        e[1] = pg.nseg >= 2 ? pg.seg[1].start : 1 << 20;
        e[2] = pg.nseg >= 3 ? pg.seg[2].start : 1 << 20;
        for (int j = 0; j < kBgMaxSeg; ++j) {
            const BgSeg& sg = pg.seg[j];
            e[3 + 4 * j] = sg.rb;
            e[4 + 4 * j] = (sg.k0 - 4 * sg.start) * 16;   // LDS element offset so step s reads +64*s
            e[5 + 4 * j] = sg.slot;
            e[6 + 4 * j] = sg.k0 - 4 * sg.start;          // input offset (global-B path)
        }
    }
    return t;
}

std::vector<int> BgPlan::redTable() const {
    std::vector<int> t(reds.size() * kBgRedInts, 0);
    for (size_t i = 0; i < reds.size(); ++i) {
        int* e = &t[i * kBgRedInts];
        e[0] = reds[i].rb;
        e[1] = reds[i].n;
        for (int k = 0; k < reds[i].n; ++k) e[2 + k] = reds[i].slot[k];
    }
    return t;
}

namespace {
// Wave programs for macro period mp (waves per column group nw, column groups ncg) minimising
// the critical SIMD's MFMA steps per column:
//   ceil(waves/4) * kch*NS / (16 * ncg), x latency factor for < 3 waves/SIMD
// (a program longer than maxNS runs as kch chunks of NS steps).  False when no split fits
// the segment / reduction-slot / register limits.
bool planPrograms(const FirPeriodic& f, bool f64, int mp, BgPlan& plan) {
    double eff;
    const std::vector<RbGeom> rbs = geomFor(f, mp, eff);
    plan = BgPlan();
    plan.f64 = f64;
    plan.P = f.P; plan.Q = f.Q; plan.mp = mp;
    plan.Pc = f.P * mp;
    plan.Qc = f.Q * mp;
    plan.nrb = static_cast<int>(rbs.size());
    for (const auto& r : rbs) plan.Kc = std::max(plan.Kc, r.klo + 4 * r.nsteps);
    const int maxNS = f64 ? 48 : 96;
    double bestCost = 1e300;
    for (int nw = 1; nw <= 16; ++nw) {
        std::vector<BgProg> progs;
        std::vector<BgRed> reds;
        int nslots = 0, maxLen = 0;
        if (!splitPrograms(rbs, nw, progs, reds, nslots, maxLen)) continue;
        const int kch = (maxLen + maxNS - 1) / maxNS;
        const int NS = std::max(8, ((maxLen + kch - 1) / kch + 3) / 4 * 4);
        for (int ncg = 1; ncg <= 4; ncg *= 2) {
            const int waves = nw * ncg;
            if (waves > 16 || 64 * waves > bgMaxThreads(f64, NS)) continue;
            const int wps = (waves + 3) / 4;
            const double lat = wps == 1 ? 1.4 : (wps == 2 ? 1.1 : 1.0);
            const double cost = static_cast<double>(wps) * NS * kch / (16.0 * ncg) * lat * (kch > 1 ? 1.2 : 1.0) *
                                (1.0 + 0.01 * static_cast<double>(reds.size()));
            if (cost < bestCost - 1e-9) {
                bestCost = cost;
                plan.nw = nw;
                plan.ncg = ncg;
                plan.NS = NS;
                plan.kch = kch;
                plan.progs = progs;
                plan.reds = reds;
                plan.nslots = nslots;
            }
        }
    }
    return !plan.progs.empty();
}
}  // namespace

// Row-block-aligned programs (f64 plans): row block rb is cut into p = ceil(steps / kBgRbMaxSteps)
// balanced K pieces, one program (one segment) each, finished by an LDS reduction in program order
// when p > 1.  The persistent kernel runs them like any plan; bg_rb_kernel runs one (column block,
// row block) per workgroup for small launches -- same programs, same sums.
bool planProgramsRb(const FirPeriodic& f, bool f64, int mp, BgPlan& plan) {
    double eff;
    const std::vector<RbGeom> rbs = geomFor(f, mp, eff);
    plan = BgPlan();
    plan.f64 = f64;
    plan.P = f.P; plan.Q = f.Q; plan.mp = mp;
    plan.Pc = f.P * mp;
    plan.Qc = f.Q * mp;
    plan.nrb = static_cast<int>(rbs.size());
    plan.rbAligned = true;
    int maxLen = 0;
    for (size_t rb = 0; rb < rbs.size(); ++rb) {
        plan.Kc = std::max(plan.Kc, rbs[rb].klo + 4 * rbs[rb].nsteps);
        const int n = rbs[rb].nsteps;
        const int np = std::max(1, (n + kBgRbMaxSteps - 1) / kBgRbMaxSteps);
        if (np > kBgRbMaxWaves || np > kBgMaxRedSlots) return false;
        plan.rbStart.push_back(static_cast<int>(plan.progs.size()));
        BgRed red;
        red.rb = static_cast<int>(rb);
        for (int i = 0, pos = 0; i < np; ++i) {
            const int len = (n - pos + (np - i) - 1) / (np - i);  // balanced pieces, in K order
            BgProg pg;
            pg.nseg = 1;
            pg.len = len;
            pg.seg[0].rb = static_cast<int>(rb);
            pg.seg[0].k0 = rbs[rb].klo + 4 * pos;
            pg.seg[0].ns = len;
            pg.seg[0].start = 0;
            pg.seg[0].slot = np > 1 ? plan.nslots++ : -1;
            if (np > 1) red.slot[red.n++] = pg.seg[0].slot;
            plan.progs.push_back(pg);
            plan.rbK0.push_back(pg.seg[0].k0);
            maxLen = std::max(maxLen, len);
            pos += len;
        }
        if (np > 1) plan.reds.push_back(red);
    }
    plan.rbStart.push_back(static_cast<int>(plan.progs.size()));
    plan.kch = 1;
    plan.NS = std::max(8, (maxLen + 3) / 4 * 4);
    plan.ncg = 1;
    plan.nw = std::min<int>(static_cast<int>(plan.progs.size()), std::min(16, bgMaxThreads(f64, plan.NS) / 64));
    return true;
}

bool buildBgPlan(const FirPeriodic& f, bool f64, BgPlan& plan) {
    if (f.P <= 0 || f.Q <= 0) return false;
    // Macro period (multiple of the FIR period) with the best useful/executed MAC ratio among
    // those whose programs fit (prefer >= 16 rows so row blocks are full).  A long period of a
    // long f64 filter (48k->44.1k Q32: Pc = 294, 19 row blocks x 78 steps) can need more
    // segments per program than kBgMaxSeg at the f64 register budget; a shorter one fits.
    std::vector<std::pair<double, int>> cand;
    for (int mp = 1; mp <= 64; ++mp) {
        const int Pc = f.P * mp;
        if (Pc > 320) break;
        double eff;
        geomFor(f, mp, eff);
        if (Pc < 16) eff *= static_cast<double>(Pc) / 16.0;  // partially filled row block
        cand.push_back({-eff, mp});
    }
    std::stable_sort(cand.begin(), cand.end(),
                     [](const std::pair<double, int>& a, const std::pair<double, int>& b) { return a.first < b.first - 1e-9; });
    bool ok = false;
    // f64: row-block-aligned programs where every row block fits kBgRbMaxWaves pieces (small
    // launches then run bg_rb_kernel); longer filters (e.g. an 8191-tap decimator) the general split
    for (const auto& c : cand)
        if (f64 && (ok = planProgramsRb(f, f64, c.second, plan))) break;
    for (size_t i = 0; !ok && i < cand.size(); ++i) ok = planPrograms(f, f64, cand[i].second, plan);
    if (!ok) return false;

    const size_t np = plan.progs.size();
    const int plen = plan.kch * plan.NS;  // steps per program incl. padding
    std::vector<double> A(np * plen * 64, 0.0);
    plan.Kread = plan.Kc;
    for (size_t pi = 0; pi < np; ++pi) {
        const BgProg& pg = plan.progs[pi];
        for (int j = 0; j < pg.nseg; ++j) {
            const BgSeg& sg = pg.seg[j];
            const int runLen = j == pg.nseg - 1 ? plen - sg.start : sg.ns;  // last segment runs to the end
            plan.Kread = std::max(plan.Kread, sg.k0 + 4 * runLen);
            for (int s = 0; s < sg.ns; ++s)
                for (int lane = 0; lane < 64; ++lane) {
                    const int m = lane & 15, kq = lane >> 4;
                    const int r = sg.rb * 16 + m;
                    if (r >= plan.Pc) continue;
                    int64_t off;
                    const std::vector<double>* row;
                    macroRow(f, r, off, row);
                    const int64_t idx = sg.k0 + 4 * s + kq - off;
                    if (idx >= 0 && idx < static_cast<int64_t>(row->size()))
                        A[(pi * plen + sg.start + s) * 64 + lane] = (*row)[idx];
                }
        }
    }
    if (f64) plan.A64 = std::move(A);
    else plan.A32.assign(A.begin(), A.end());

    plan.rowMax = 0;
    for (const auto& r : f.rows) plan.rowMax = std::max(plan.rowMax, static_cast<int>(r.size()));
    plan.twoStage = f.composite;
    plan.rows.assign(static_cast<size_t>(plan.Pc) * plan.rowMax, 0.0);
    plan.rowInfo.assign(4 * static_cast<size_t>(plan.Pc), 0);
    for (int r = 0; r < plan.Pc; ++r) {
        int64_t off;
        const std::vector<double>* row;
        macroRow(f, r, off, row);
        plan.rowInfo[r] = static_cast<int>(off);
        plan.rowInfo[plan.Pc + r] = static_cast<int>(row->size());
        if (f.composite) {
            plan.rowInfo[2 * plan.Pc + r] = f.ph[r % f.P];
            plan.rowInfo[3 * plan.Pc + r] = f.par[r % f.P];
        }
        std::copy(row->begin(), row->end(), plan.rows.begin() + static_cast<size_t>(r) * plan.rowMax);
    }

    double useful = 0;
    for (const auto& r : f.rows) useful += static_cast<double>(r.size());
    plan.usefulMacsPerOutput = useful / f.P;
    double eff, exec = 0;
    for (const auto& r : geomFor(f, plan.mp, eff)) exec += 16.0 * 4.0 * r.nsteps;  // per column per macro period
    plan.mfmaMacsPerOutput = exec / plan.Pc;
    return true;
}

// ---------------------------------------------------------------------------
// Split-f16 plan
// ---------------------------------------------------------------------------
std::vector<int> HxPlan::progTable() const {
    std::vector<int> t(progs.size() * kBgProgInts, 0);
    for (size_t i = 0; i < progs.size(); ++i) {
        int* e = &t[i * kBgProgInts];
        const BgProg& pg = progs[i];
        e[0] = pg.nseg;
        e[1] = pg.nseg >= 2 ? pg.seg[1].start : 1 << 20;
        e[2] = pg.nseg >= 3 ? pg.seg[2].start : 1 << 20;
        for (int j = 0; j < kBgMaxSeg; ++j) {
            const BgSeg& sg = pg.seg[j];
            e[3 + 4 * j] = sg.rb;
            e[4 + 4 * j] = sg.k0 - kHxStep * sg.start;  // input row of step s = this + 32*s
            e[5 + 4 * j] = sg.slot;
            e[6 + 4 * j] = 0;
        }
        e[15] = rbMode ? kch * NS : pg.len;  // steps >= len (zero A) re-read rows [0, 32*(kch*NS - len))
    }
    return t;
}

std::vector<int> HxPlan::redTable() const {
    std::vector<int> t(reds.size() * kBgRedInts, 0);
    for (size_t i = 0; i < reds.size(); ++i) {
        int* e = &t[i * kBgRedInts];
        e[0] = reds[i].rb;
        e[1] = reds[i].n;
        for (int k = 0; k < reds[i].n; ++k) e[2 + k] = reds[i].slot[k];
    }
    return t;
}

static uint16_t f16bits(double v) {
    const _Float16 h = static_cast<_Float16>(v);
    uint16_t b;
    std::memcpy(&b, &h, 2);
    return b;
}

bool buildHxPlan(const FirPeriodic& f, HxPlan& plan) {
    if (f.P <= 0 || f.Q <= 0) return false;
    // macro period: the best MFMA efficiency among the ones whose row blocks fit the streaming
    // kernel (one compute wave per row block, <= kHxRbMaxNS steps: hxs_kernel, gar_hxs.hpp), else
    // the best overall (segmented programs on hx_kernel)
    int bestMp = 1, bestRbMp = 0;
    double bestEff = -1, bestRbEff = -1;
    for (int mp = 1; mp <= 64; ++mp) {
        const int Pc = f.P * mp;
        if (Pc > 320) break;
        double eff;
        const std::vector<RbGeom> g = geomFor(f, mp, eff, kHxStep, 1);
        if (Pc < 16) eff *= static_cast<double>(Pc) / 16.0;
        if (eff > bestEff + 1e-9) { bestEff = eff; bestMp = mp; }
        int ml = 0;
        for (const auto& r : g) ml = std::max(ml, r.nsteps);
        if (static_cast<int>(g.size()) <= kHxRbMaxWaves && ml <= kHxRbMaxNS && eff > bestRbEff + 1e-9) {
            bestRbEff = eff;
            bestRbMp = mp;
        }
    }
    if (bestRbMp > 0) bestMp = bestRbMp;
    double eff;
    const std::vector<RbGeom> rbs = geomFor(f, bestMp, eff, kHxStep, 1);
    plan = HxPlan();
    plan.P = f.P; plan.Q = f.Q; plan.mp = bestMp;
    plan.Pc = f.P * bestMp;
    plan.Qc = f.Q * bestMp;
    plan.nrb = static_cast<int>(rbs.size());
    for (const auto& r : rbs) plan.Kc = std::max(plan.Kc, r.klo + kHxStep * r.nsteps);

    int maxLen = 0;
    for (const auto& r : rbs) maxLen = std::max(maxLen, r.nsteps);
    if (plan.nrb <= kHxRbMaxWaves && maxLen <= kHxRbMaxNS) {
        // row-block mode: wave w runs row block w over its whole band
        plan.rbMode = true;
        plan.nw = plan.nrb;
        plan.progs.assign(plan.nw, BgProg());
        for (int w = 0; w < plan.nw; ++w) {
            BgProg& pg = plan.progs[w];
            pg.nseg = 1;
            pg.len = rbs[w].nsteps;
            pg.seg[0].rb = w;
            pg.seg[0].k0 = rbs[w].klo;
            pg.seg[0].ns = rbs[w].nsteps;
        }
        plan.kch = 1;
        plan.NS = maxLen;
    } else {
        plan.nw = kHxWaves;
        if (!splitPrograms(rbs, plan.nw, plan.progs, plan.reds, plan.nslots, maxLen, kHxStep)) return false;
        plan.kch = (maxLen + kHxMaxNS - 1) / kHxMaxNS;
        plan.NS = std::max(2, ((maxLen + plan.kch - 1) / plan.kch + 1) / 2 * 2);
        if (plan.NS > kHxMaxNS) return false;
    }

    double amax = 0;
    for (const auto& r : f.rows)
        for (double v : r) amax = std::max(amax, std::fabs(v));
    int ex = 0;
    if (amax > 0) std::frexp(amax, &ex);
    plan.ea = amax > 0 ? 15 - ex : 0;
    const double sc = std::ldexp(1.0, plan.ea);

    const int plen = plan.kch * plan.NS;
    const int nprog = static_cast<int>(plan.progs.size());
    plan.A.assign(static_cast<size_t>(nprog) * plen * 2 * 64 * 8, 0);
    plan.Kread = plan.Kc;
    for (int pi = 0; pi < nprog; ++pi) {
        const BgProg& pg = plan.progs[pi];
        for (int j = 0; j < pg.nseg; ++j) {
            const BgSeg& sg = pg.seg[j];
            // row-block mode runs the last segment on to plen; segmented mode
            // points the padding steps at rows [0, 32*(plen - len))
            const int runLen = j == pg.nseg - 1 && plan.rbMode ? plen - sg.start : sg.ns;
            plan.Kread = std::max(plan.Kread, sg.k0 + kHxStep * runLen);
            if (!plan.rbMode) plan.Kread = std::max(plan.Kread, kHxStep * (plen - pg.len));
            for (int s = 0; s < sg.ns; ++s)
                for (int lane = 0; lane < 64; ++lane) {
                    const int m = lane & 15, g = lane >> 4;
                    const int r = sg.rb * 16 + m;
                    if (r >= plan.Pc) continue;
                    int64_t off;
                    const std::vector<double>* row;
                    macroRow(f, r, off, row);
                    const size_t base = ((static_cast<size_t>(pi) * plen + sg.start + s) * 2 * 64 + lane) * 8;
                    for (int jj = 0; jj < 8; ++jj) {
                        const int64_t idx = sg.k0 + kHxStep * s + hxPermK(g, jj) - off;
                        if (idx < 0 || idx >= static_cast<int64_t>(row->size())) continue;
                        const double v = (*row)[idx] * sc;
                        const uint16_t hb = f16bits(v);
                        _Float16 hh;
                        std::memcpy(&hh, &hb, 2);
                        plan.A[base + jj] = hb;
                        plan.A[base + 64 * 8 + jj] = f16bits(v - static_cast<double>(hh));
                    }
                }
        }
    }

    plan.rowMax = 0;
    for (const auto& r : f.rows) plan.rowMax = std::max(plan.rowMax, static_cast<int>(r.size()));
    plan.rows.assign(static_cast<size_t>(plan.Pc) * plan.rowMax, 0.0);
    plan.rowOff.assign(plan.Pc, 0);
    plan.rowLen.assign(plan.Pc, 0);
    plan.twoStage = f.composite;
    plan.rowPh.assign(plan.Pc, 0);
    plan.rowPar.assign(plan.Pc, 0);
    for (int r = 0; r < plan.Pc; ++r) {
        int64_t off;
        const std::vector<double>* row;
        macroRow(f, r, off, row);
        plan.rowOff[r] = static_cast<int>(off);
        plan.rowLen[r] = static_cast<int>(row->size());
        for (size_t k = 0; k < row->size(); ++k) plan.rows[static_cast<size_t>(r) * plan.rowMax + k] = (*row)[k];
        if (f.composite) {
            plan.rowPh[r] = f.ph[r % f.P];
            plan.rowPar[r] = f.par[r % f.P];
        }
    }

    double useful = 0;
    for (const auto& r : f.rows) useful += static_cast<double>(r.size());
    plan.usefulMacsPerOutput = useful / f.P;
    double exec = 0;
    for (const auto& r : rbs) exec += 16.0 * kHxStep * r.nsteps;
    plan.mfmaMacsPerOutput = exec / plan.Pc;
    return true;
}

}  // namespace gar
