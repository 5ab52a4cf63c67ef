/*
 * gar_oracle.c -- CPU restatement of tphakala/go-audio-resampler's resampling
 * path, used ONLY as test infrastructure (parity checker + CPU baseline).
 *
 *   *** TEST INFRASTRUCTURE ***  Only tests/, __graft_entry__.smoke() and
 *   bench.py's cpu_baseline leg may load this library.  The product
 *   (go-audio-resampler_amd/) never links or calls it.
 *
 * Every function below restates one Go function of the reference and cites it
 * as path:line relative to /root/reference.  The restatement keeps the Go
 * state variables (history slices, fixed-point `at`, decimPhase, ring buffers)
 * so stream lengths, flush padding and chunking behave exactly as the Go code.
 *
 * Pinning (see DESIGN.md "Oracle"): the Go toolchain and the SIMD dependency
 * github.com/tphakala/simd v1.1.0 are absent, so the reference cannot be run
 * here.  This oracle is pinned against every known-answer test the reference
 * holds for this path (Bessel table, simdops KATs, tap-count table in
 * README.md:466-471, rational-approx / Fn tables, flush length bounds, DC
 * gain, bit-identity invariants) -- tests/test_oracle_kat.py.  Bit-level
 * parity is NOT claimed: the summation order inside tphakala/simd's AVX2
 * kernels (f64.Sum, DotProductUnsafe, ConvolveValid, CubicInterpDot) and Go's
 * pure-Go math.Sin/Pow/Asin vs glibc differ by <= a few ulp.
 *
 * Semantics notes (Go -> C): math.Round == C round (half away from zero);
 * Go int conversion truncates == C cast; Go / and % on ints truncate toward
 * zero == C99.  Compile with -ffp-contract=off so no FMA contraction changes
 * the design arithmetic (the Go amd64 default build does not fuse).
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#define API __attribute__((visibility("default")))

/* ------------------------------------------------------------------------- */
/* internal/mathutil/constants.go:10-99                                      */
/* ------------------------------------------------------------------------- */
#define BESSEL_SMALL 3.75
static const double I0C[7] = {1.0, 3.5156229, 3.0899424, 1.2067492, 0.2659732, 0.360768e-1, 0.45813e-2};
static const double I0A[9] = {0.39894228, 0.1328592e-1, 0.225319e-2, -0.157565e-2, 0.916281e-2,
                              -0.2057706e-1, 0.2635537e-1, -0.1647633e-1, 0.392377e-2};

/* internal/mathutil/bessel.go:22-49 (A&S 9.8.1 / 9.8.2 polynomial I0) */
API double o_bessel_i0(double x) {
    double ax = fabs(x);
    if (ax < BESSEL_SMALL) {
        double t = x / BESSEL_SMALL;
        t *= t;
        return 1.0 + t * (I0C[1] + t * (I0C[2] + t * (I0C[3] + t * (I0C[4] + t * (I0C[5] + t * I0C[6])))));
    }
    double t = BESSEL_SMALL / ax;
    double r = I0A[0] + t * (I0A[1] + t * (I0A[2] + t * (I0A[3] + t * (I0A[4] + t * (I0A[5] +
               t * (I0A[6] + t * (I0A[7] + t * I0A[8])))))));
    return exp(ax) * r / sqrt(ax);
}

/* internal/mathutil/bessel.go:126-134 */
API double o_kaiser_beta(double att) {
    if (att > 50.0) return 0.1102 * (att - 8.7);
    if (att >= 21.0) {
        double d = att - 21.0;
        return 0.5842 * pow(d, 0.4) + 0.07886 * d;
    }
    return 0.0;
}

/* internal/mathutil/bessel.go:245-268 */
API int o_estimate_filter_length(double att, double tbw) {
    if (tbw <= 0) tbw = 0.01;
    double n = (att - 8.0) / (2.285 * 2.0 * M_PI * tbw);
    int taps = (int)ceil(n);
    if (taps % 2 == 0) taps++;
    if (taps < 3) taps = 3;
    if (taps > 8191) taps = 8191;
    return taps;
}

/* ------------------------------------------------------------------------- */
/* internal/filter/kaiser.go                                                 */
/* ------------------------------------------------------------------------- */
/* kaiser.go:47-91 */
API void o_kaiser_window(int length, double beta, double *w) {
    if (length < 1) return;
    if (length == 1) { w[0] = 1.0; return; }
    beta = fabs(beta);
    double alpha = (double)(length - 1) / 2.0;
    double i0b = o_bessel_i0(beta);
    for (int n = 0; n < length; n++) {
        double x = ((double)n - alpha) / alpha;
        double arg = beta * sqrt(1.0 - x * x);
        double i0a = o_bessel_i0(arg);
        if (isinf(i0a) && i0a > 0 && isinf(i0b) && i0b > 0)
            w[n] = exp(arg - beta);
        else
            w[n] = i0a / i0b;
    }
}

/* sequential f64.Sum stand-in (tphakala/simd order unknown; kaiser.go:195) */
static double sum_seq(const double *a, int n) {
    double s = 0;
    for (int i = 0; i < n; i++) s += a[i];
    return s;
}

/* kaiser.go:112-138 + 159-203.  Returns 0 on success, -1 on invalid params. */
API int o_design_lowpass(int ntaps, double fc, double att, double gain, double *out) {
    if (ntaps < 3 || ntaps > 8191) return -1;
    if (fc <= 0 || fc >= 0.5) return -1;
    if (att < 0 || att > 500) return -1;
    if (gain <= 0) return -1;
    double beta = o_kaiser_beta(att);
    double *win = (double *)malloc(sizeof(double) * ntaps);
    o_kaiser_window(ntaps, beta, win);
    double center = (double)(ntaps - 1) / 2.0;
    for (int n = 0; n < ntaps; n++) {
        double x = (double)n - center;
        double s;
        if (fabs(x) < 1e-10) s = 2.0 * fc;
        else {
            double arg = 2.0 * M_PI * fc * x;
            s = sin(arg) / (M_PI * x);
        }
        out[n] = s * win[n];
    }
    free(win);
    double sum = sum_seq(out, ntaps);
    if (fabs(sum) > 1e-10) {
        double scale = gain / sum;
        for (int n = 0; n < ntaps; n++) out[n] = out[n] * scale;
    }
    return 0;
}

/* kaiser.go:221-233.  *ntaps receives the length; out must hold 8191. */
API int o_design_lowpass_auto(double fc, double tbw, double att, double gain, double *out, int *ntaps) {
    int n = o_estimate_filter_length(att, tbw);
    *ntaps = n;
    return o_design_lowpass(n, fc, att, gain, out);
}

/* ------------------------------------------------------------------------- */
/* internal/engine/filter_params.go                                          */
/* ------------------------------------------------------------------------- */
enum { Q_QUICK = 0, Q_LOW, Q_MEDIUM, Q_HIGH, Q_VERYHIGH, Q_16, Q_20, Q_24, Q_28, Q_32 };
#define DB_PER_BIT 6.0206

/* filter_params.go:150-175 */
API double o_quality_to_attenuation(int q) {
    switch (q) {
    case Q_QUICK: return (8 + 1) * DB_PER_BIT;
    case Q_LOW: return (16 + 1) * DB_PER_BIT;
    case Q_MEDIUM: return (16 + 1) * DB_PER_BIT;
    case Q_HIGH: return (20 + 1) * DB_PER_BIT;
    case Q_VERYHIGH: return (28 + 1) * DB_PER_BIT;
    case Q_16: return (16 + 1) * DB_PER_BIT;
    case Q_20: return (20 + 1) * DB_PER_BIT;
    case Q_24: return (24 + 1) * DB_PER_BIT;
    case Q_28: return (28 + 1) * DB_PER_BIT;
    case Q_32: return (32 + 1) * DB_PER_BIT;
    default: return (20 + 1) * DB_PER_BIT;
    }
}

/* filter_params.go:180-195 */
API double o_quality_to_passband_end(int q) {
    switch (q) {
    case Q_QUICK: case Q_LOW: return 0.67625;
    case Q_MEDIUM: return 0.91;
    case Q_HIGH: case Q_20: return 0.912;
    case Q_VERYHIGH: case Q_24: case Q_28: case Q_32: return 0.913;
    case Q_16: return 0.67625;
    default: return 0.912;
    }
}

/* filter_params.go:294-329 */
API void o_find_rational_approx(double ratio, int *L_out, int *step_out) {
    double inv = 1.0 / ratio;
    int bestL = 80;
    int bestStep = (int)round(inv * 80.0);
    double bestErr = fabs((double)bestStep / (double)bestL - inv);
    for (int L = 64; L <= 256; L++) {
        int cs = (int)round(inv * (double)L);
        if (cs <= 0) continue;
        double e = fabs((double)cs / (double)L - inv);
        if (e < bestErr) { bestL = L; bestStep = cs; bestErr = e; }
        if (bestErr < 1e-10) break;
    }
    *L_out = bestL;
    *step_out = bestStep;
}

/* filter_params.go:355-394 */
API double o_lsx_inv_f_resp(double drop, double a) {
    if (a < 1.0) a = 1.0;
    else if (a > 300.0) a = 300.0;
    double x = ((2.0517e-07 * a + -1.1303e-04) * a + 0.023154) * a + 0.55924;
    double dl = exp(drop * M_LN10 * 0.05);
    double s = dl > 0.5 ? 1 - dl : dl;
    double sv = sin(x * 0.5);
    if (sv <= 1e-10) sv = 1e-10;
    double sp = log(0.5) / log(sv);
    x = asin(pow(s, 1.0 / sp)) / x;
    return dl > 0.5 ? x : 1 - x;
}

typedef struct {
    int num_phases; double ratio, total_io_ratio; int has_pre; double attenuation;
    int is_upsampling; double mult, fn, fp1, fs1, fp_raw, fs_raw, fp, fs, tr_bw, fc;
    int total_taps, taps_per_phase;
} o_poly_params;

/* filter_params.go:446-630 */
API void o_compute_poly_params(int L, double ratio, double tio, int has_pre, double att, double pbe,
                               o_poly_params *p) {
    memset(p, 0, sizeof(*p));
    p->num_phases = L; p->ratio = ratio; p->total_io_ratio = tio; p->has_pre = has_pre; p->attenuation = att;
    double phases = (double)L;
    p->is_upsampling = tio < 1.0;
    p->mult = p->is_upsampling ? 1.0 : tio;
    if (p->is_upsampling) { p->fp1 = tio * pbe; p->fs1 = tio * 1.0; }
    else { p->fp1 = pbe * ratio; p->fs1 = ratio; }
    if (!p->is_upsampling && has_pre) {
        p->fn = 2.0 * p->mult;
        p->fs_raw = 3.0 + fabs(p->fs1 - 1.0);
        p->fp_raw = p->fp1;
    } else {
        p->fn = 1.0;
        p->fs_raw = 2.0 - (p->fp1 + (p->fs1 - p->fp1) * 0.7);
        p->fp_raw = p->fp1;
    }
    double inv = o_lsx_inv_f_resp(-0.01, att);
    if (inv < 0.999) {
        double adj = p->fs_raw - (p->fs_raw - p->fp_raw) / (1.0 - inv);
        if (adj > 0 && adj < p->fs_raw) p->fp_raw = adj;
    }
    p->fp = p->fp_raw / fabs(p->fn);
    p->fs = p->fs_raw / fabs(p->fn);
    p->tr_bw = 0.5 * (p->fs - p->fp);
    p->tr_bw /= phases;
    double lim = 0.5 * p->fs / phases;
    if (p->tr_bw > lim) p->tr_bw = lim;
    if (p->tr_bw < 0.001) p->tr_bw = 0.001;
    double fsph = p->fs / phases;
    p->fc = fsph - p->tr_bw;
    if (p->fc < 0.001) p->fc = 0.001;
    int maxT;
    if (att < 110.0) maxT = 32;
    else if (att < 130.0) maxT = 64;
    else if (att < 160.0) maxT = 100;
    else maxT = (8190 + 1) / L;
    int ideal = (int)ceil(att / p->tr_bw + 1);
    p->total_taps = ideal;
    p->taps_per_phase = (p->total_taps + L - 1) / L;
    if (p->taps_per_phase < 8) p->taps_per_phase = 8;
    else if (p->taps_per_phase > maxT) p->taps_per_phase = maxT;
    p->total_taps = L * p->taps_per_phase - 1;
    if (p->total_taps > 8190) {
        int t = (8190 + 1) / L;
        p->taps_per_phase = t > 8 ? t : 8;
        p->total_taps = L * p->taps_per_phase - 1;
    }
}

/* filter_params.go:229-286.  coeffs: [taps_per_phase * L], layout tap*L+phase.
 * Returns taps_per_phase, or -1 on design error. */
API int o_design_polyphase_filter(int L, double ratio, double tio, int has_pre, int q, double *coeffs) {
    double att = o_quality_to_attenuation(q);
    double pbe = o_quality_to_passband_end(q);
    o_poly_params p;
    o_compute_poly_params(L, ratio, tio, has_pre, att, pbe, &p);
    double cutoff = p.fc / 2.0;
    if (cutoff <= 0) cutoff = 0.001;
    if (cutoff >= 0.5) cutoff = 0.499;
    double *proto = (double *)malloc(sizeof(double) * p.total_taps);
    if (o_design_lowpass(p.total_taps, cutoff, att, 1.0, proto) != 0) { free(proto); return -1; }
    double sum = sum_seq(proto, p.total_taps);
    if (sum != 0) {
        double scale = (double)L / sum;
        for (int i = 0; i < p.total_taps; i++) proto[i] = proto[i] * scale;
    }
    for (int tap = 0; tap < p.taps_per_phase; tap++)
        for (int ph = 0; ph < L; ph++) {
            int idx = tap * L + ph;
            coeffs[idx] = idx < p.total_taps ? proto[idx] : 0.0;
        }
    free(proto);
    return p.taps_per_phase;
}

/* internal/engine/resampler.go:356-360 */
API int o_is_integer_ratio(double r) {
    double rr = round(r);
    return fabs(r - rr) < 1e-9 && rr >= 1.0;
}

/* ------------------------------------------------------------------------- */
/* Go-slice helpers (internal/engine/polyphase.go:23-44 semantics: only the  */
/* capacity policy differs from append, values/lengths are identical)        */
/* ------------------------------------------------------------------------- */
/* Geometry/introspection of an engine (white-box, like export_test.go). */
typedef struct {
    int kind;           /* 0 quick-cubic, 1 dft-only, 2 dft+poly, 3 decim, 4 passthrough(dft factor 1) */
    int dft_factor, dft_taps_per_phase, dft_is_halfband;
    int poly_phases, poly_taps_per_phase; int64_t poly_step;
    int decim_factor, decim_taps;
} o_engine_info;

#define F double
#define SFX(n) n##_d
#include "gar_oracle_stages.inc"
#undef F
#undef SFX
#define F float
#define SFX(n) n##_f
#include "gar_oracle_stages.inc"
#undef F
#undef SFX

/* ------------------------------------------------------------------------- */
/* Engine handle (internal/engine/resampler.go) for F=float64 or float32     */
/* ------------------------------------------------------------------------- */
typedef struct {
    int is_f32;
    void *r;
} o_engine;

API o_engine *o_engine_new(double in_rate, double out_rate, int q, int is_f32) {
    void *r = is_f32 ? (void *)resampler_new_f(in_rate, out_rate, q) : (void *)resampler_new_d(in_rate, out_rate, q);
    if (!r) return NULL;
    o_engine *e = (o_engine *)calloc(1, sizeof(o_engine));
    e->is_f32 = is_f32;
    e->r = r;
    return e;
}

API void o_engine_free(o_engine *e) {
    if (!e) return;
    if (e->is_f32) resampler_free_f((resampler_f *)e->r); else resampler_free_d((resampler_d *)e->r);
    free(e);
}

/* Process: in/out are double for the f64 engine, float for the f32 engine.
 * Returns n_out (>=0) or -(needed) if cap is too small (state untouched only
 * for the f64/f32 copy-out; callers size cap generously). */
API int64_t o_engine_process(o_engine *e, const void *in, int64_t n, void *out, int64_t cap) {
    if (e->is_f32) {
        vec_f o = resampler_process_f((resampler_f *)e->r, (const float *)in, n);
        int64_t m = o.len;
        if (m > cap) { free(o.a); return -m; }
        if (m) memcpy(out, o.a, sizeof(float) * m);
        free(o.a);
        return m;
    }
    vec_d o = resampler_process_d((resampler_d *)e->r, (const double *)in, n);
    int64_t m = o.len;
    if (m > cap) { free(o.a); return -m; }
    if (m) memcpy(out, o.a, sizeof(double) * m);
    free(o.a);
    return m;
}

API int64_t o_engine_flush(o_engine *e, void *out, int64_t cap) {
    if (e->is_f32) {
        vec_f o = resampler_flush_f((resampler_f *)e->r);
        int64_t m = o.len;
        if (m > cap) { free(o.a); return -m; }
        if (m) memcpy(out, o.a, sizeof(float) * m);
        free(o.a);
        return m;
    }
    vec_d o = resampler_flush_d((resampler_d *)e->r);
    int64_t m = o.len;
    if (m > cap) { free(o.a); return -m; }
    if (m) memcpy(out, o.a, sizeof(double) * m);
    free(o.a);
    return m;
}

API void o_engine_reset(o_engine *e) {
    if (e->is_f32) resampler_reset_f((resampler_f *)e->r); else resampler_reset_d((resampler_d *)e->r);
}

/* GetStatistics (resampler.go:348-353): out[0] = samplesIn, out[1] = samplesOut */
API void o_engine_stats(o_engine *e, int64_t *out) {
    if (e->is_f32) { out[0] = ((resampler_f *)e->r)->samples_in; out[1] = ((resampler_f *)e->r)->samples_out; }
    else { out[0] = ((resampler_d *)e->r)->samples_in; out[1] = ((resampler_d *)e->r)->samples_out; }
}

API double o_engine_ratio(o_engine *e) {
    return e->is_f32 ? ((resampler_f *)e->r)->ratio : ((resampler_d *)e->r)->ratio;
}


API void o_engine_get_info(o_engine *e, o_engine_info *inf) {
    memset(inf, 0, sizeof(*inf));
    if (e->is_f32) resampler_info_f((resampler_f *)e->r, inf); else resampler_info_d((resampler_d *)e->r, inf);
}

/* Coefficient banks (f64 engine only): which 0=dft phase p (p in sel), 1..4 = poly a,b,c,d
 * flattened [phase][tap]; 5 = decim (reversed). Returns element count. */
API int64_t o_engine_get_coeffs(o_engine *e, int which, int sel, double *out) {
    if (e->is_f32) return -1;
    resampler_d *r = (resampler_d *)e->r;
    return resampler_coeffs_d(r, which, sel, out);
}

/* ------------------------------------------------------------------------- */
/* Top-level package (resample.go, constant.go, pipeline_builder.go,         */
/* stages.go, internal/pipeline/pipeline.go, buffer.go)                      */
/* ------------------------------------------------------------------------- */

/* stages.go:92-107 */
API int o_precision_to_engine_quality(int prec) {
    if (prec <= 8) return Q_QUICK;
    if (prec <= 16) return Q_LOW;
    if (prec <= 20) return Q_HIGH;
    if (prec <= 24) return Q_24;
    if (prec <= 28) return Q_VERYHIGH;
    return Q_32;
}

/* convenience.go:189-200 */
API int o_preset_to_engine_quality(int preset) {
    switch (preset) {
    case 0: case 1: return Q_LOW;
    case 2: return Q_MEDIUM;
    case 3: case 4: return Q_HIGH;
    default: return Q_MEDIUM;
    }
}

/* resample.go:217-267: preset -> precision (only Precision reaches the engine) */
static int preset_precision(int preset) {
    switch (preset) {
    case 0: return 8;
    case 1: return 16;
    case 2: return 16;
    case 3: return 24;
    case 4: return 32;
    default: return 0; /* QualitySpec{Preset: QualityMedium} with Precision 0 */
    }
}

/* internal/pipeline/buffer.go:12-172 -- ring buffer, values-only semantics */
typedef struct { double *data; int cap, size, rpos, wpos; } ring;
static void ring_init(ring *b, int cap) { if (cap < 1) cap = 1; b->data = (double *)calloc(cap, sizeof(double)); b->cap = cap; b->size = b->rpos = b->wpos = 0; }
static void ring_grow(ring *b, int minc) {
    int nc = b->cap;
    while (nc < minc) nc *= 2;
    double *nd = (double *)calloc(nc, sizeof(double));
    for (int i = 0; i < b->size; i++) nd[i] = b->data[(b->rpos + i) % b->cap];
    free(b->data);
    b->data = nd; b->cap = nc; b->rpos = 0; b->wpos = b->size;
}
static void ring_write(ring *b, const double *s, int64_t n) {
    if (n == 0) return;
    if (b->size + n > b->cap) ring_grow(b, (int)(b->size + n));
    for (int64_t i = 0; i < n; i++) { b->data[b->wpos] = s[i]; b->wpos = (b->wpos + 1) % b->cap; b->size++; }
}
static vec_d ring_read(ring *b, int n) {
    vec_d r = {0};
    if (n > b->size) n = b->size;
    if (n <= 0) return r;
    r.a = (double *)malloc(sizeof(double) * n); r.len = r.cap = n;
    for (int i = 0; i < n; i++) { r.a[i] = b->data[b->rpos]; b->rpos = (b->rpos + 1) % b->cap; b->size--; }
    return r;
}

/* StageSpec (internal/pipeline/pipeline.go:75-84), types :58-73 */
enum { ST_CUBIC = 0, ST_HALFBAND, ST_POLYPHASE, ST_FFT, ST_DELAY };
typedef struct { int type; double ratio; } stage_spec;

static const double common_ratios[6] = {44100.0 / 48000.0, 48000.0 / 44100.0, 44100.0 / 88200.0,
                                        88200.0 / 44100.0, 48000.0 / 96000.0, 96000.0 / 48000.0};

/* internal/pipeline/pipeline.go:320-334 */
static int should_use_fft(double ratio, int prec) {
    if (prec >= 28) return 1;
    for (int i = 0; i < 6; i++) if (fabs(ratio - common_ratios[i]) < 0.0001) return 1;
    return 0;
}

/* internal/pipeline/pipeline.go:104-183 (stage types/ratios only: the
 * FilterLength/Phases/CutoffFactor fields are discarded by stages.go:54) */
API int o_build_pipeline(double ratio, int prec, int *types, double *ratios, int max_stages) {
    if (ratio <= 0) return -1;
    int n = 0;
    if (prec <= 8) { types[0] = ST_CUBIC; ratios[0] = ratio; return 1; }
    double rem = ratio;
    if (ratio < 1.0) while (rem < 0.5) { if (n < max_stages) { types[n] = ST_HALFBAND; ratios[n] = 0.5; } n++; rem *= 2.0; }
    if (ratio > 1.0) while (rem > 2.0) { if (n < max_stages) { types[n] = ST_HALFBAND; ratios[n] = 2.0; } n++; rem /= 2.0; }
    if (fabs(rem - 1.0) > 0.001) {
        if (n < max_stages) { types[n] = should_use_fft(rem, prec) ? ST_FFT : ST_POLYPHASE; ratios[n] = rem; }
        n++;
    }
    return n;
}

/* One pipeline stage instance = CubicStage (ST_CUBIC) or StageAdapter over
 * engine.Resampler[float64](48000, 48000*ratio, q) (stages.go:54-70). */
typedef struct { int is_cubic; cubic_d *cubic; resampler_d *eng; } stage_inst;
typedef struct { int nstages; stage_inst *st; ring *bufs; } chan_state;

typedef struct {
    double in_rate, out_rate, ratio;
    int channels, precision;
    int nstages; int types[16]; double ratios[16];
    chan_state *ch;
} o_new_rs;

static int stage_create(stage_inst *s, int type, double ratio, int prec) {
    memset(s, 0, sizeof(*s));
    if (type == ST_CUBIC) { s->is_cubic = 1; s->cubic = cubic_new_d(ratio); return 0; }
    int q = o_precision_to_engine_quality(prec);
    double ir = 48000.0, orate = ir * ratio;
    s->eng = resampler_new_d(ir, orate, q);
    return s->eng ? 0 : -1;
}
static vec_d stage_process(stage_inst *s, const double *in, int64_t n) {
    if (s->is_cubic) return cubic_process_d(s->cubic, in, n);
    return resampler_process_d(s->eng, in, n);
}
static vec_d stage_flush(stage_inst *s) {
    if (s->is_cubic) { vec_d r = {0}; return r; }
    return resampler_flush_d(s->eng);
}
static void stage_reset(stage_inst *s) {
    if (s->is_cubic) cubic_reset_d(s->cubic); else resampler_reset_d(s->eng);
}
/* StageAdapter.GetLatency stage_adapter.go:43-57; CubicStage cubic.go:110 */
static int stage_latency(stage_inst *s) {
    if (s->is_cubic) return 2;
    resampler_d *r = s->eng;
    int lat = 0;
    if (r->pre && r->pre->factor > 1) lat += (r->pre->taps_per_phase * r->pre->factor) / 2;
    if (r->poly) lat += r->poly->T / 2;
    return lat;
}
static double stage_ratio(stage_inst *s) { return s->is_cubic ? s->cubic->ratio : s->eng->ratio; }

/* resample.go:168-191 + 272-292 + constant.go:42-85.
 * preset: 0..4 presets, 5 = custom (uses precision).  Returns NULL on invalid config. */
API o_new_rs *o_new(double in_rate, double out_rate, int channels, int preset, int precision) {
    if (in_rate <= 0 || out_rate <= 0) return NULL;
    if (channels < 1 || channels > 256) return NULL;
    double ratio = out_rate / in_rate;
    if (ratio < 1.0 / 256.0 || ratio > 256.0) return NULL;
    if (preset == 5) { if (precision < 8 || precision > 33) return NULL; }
    else precision = preset_precision(preset);
    o_new_rs *r = (o_new_rs *)calloc(1, sizeof(o_new_rs));
    r->in_rate = in_rate; r->out_rate = out_rate; r->ratio = ratio; r->channels = channels; r->precision = precision;
    r->nstages = o_build_pipeline(ratio, precision, r->types, r->ratios, 16);
    if (r->nstages < 0 || r->nstages > 16) { free(r); return NULL; }
    r->ch = (chan_state *)calloc(channels, sizeof(chan_state));
    for (int c = 0; c < channels; c++) {
        chan_state *cs = &r->ch[c];
        cs->nstages = r->nstages;
        cs->st = (stage_inst *)calloc(r->nstages ? r->nstages : 1, sizeof(stage_inst));
        cs->bufs = (ring *)calloc(r->nstages + 1, sizeof(ring));
        for (int j = 0; j < r->nstages; j++)
            if (stage_create(&cs->st[j], r->types[j], r->ratios[j], precision) != 0) return NULL;
        for (int j = 0; j <= r->nstages; j++) ring_init(&cs->bufs[j], 8192);
    }
    return r;
}

API void o_new_free(o_new_rs *r) {
    if (!r) return;
    for (int c = 0; c < r->channels; c++) {
        chan_state *cs = &r->ch[c];
        for (int j = 0; j < cs->nstages; j++) {
            if (cs->st[j].is_cubic) free(cs->st[j].cubic); else resampler_free_d(cs->st[j].eng);
        }
        for (int j = 0; j <= cs->nstages; j++) free(cs->bufs[j].data);
        free(cs->st); free(cs->bufs);
    }
    free(r->ch);
    free(r);
}

static int64_t copy_out(vec_d o, double *out, int64_t cap) {
    int64_t m = o.len;
    if (m > cap) { free(o.a); return -m; }
    if (m) memcpy(out, o.a, sizeof(double) * m);
    free(o.a);
    return m;
}

/* constant.go:255-294 (processChannel; ProcessInto yields identical values) */
API int64_t o_new_process(o_new_rs *r, int ch, const double *in, int64_t n, double *out, int64_t cap) {
    if (ch < 0 || ch >= r->channels) return -1;
    chan_state *cs = &r->ch[ch];
    ring_write(&cs->bufs[0], in, n);
    for (int i = 0; i < cs->nstages; i++) {
        int avail = cs->bufs[i].size;
        if (avail >= 1) {
            vec_d chunk = ring_read(&cs->bufs[i], avail);
            vec_d o = stage_process(&cs->st[i], chunk.a, chunk.len);
            free(chunk.a);
            ring_write(&cs->bufs[i + 1], o.a, o.len);
            free(o.a);
        }
    }
    ring *fb = &cs->bufs[cs->nstages];
    return copy_out(ring_read(fb, fb->size), out, cap);
}

/* constant.go:360-386 */
API int64_t o_new_flush(o_new_rs *r, int ch, double *out, int64_t cap) {
    if (ch < 0 || ch >= r->channels) return -1;
    chan_state *cs = &r->ch[ch];
    for (int i = 0; i < cs->nstages; i++) {
        int avail = cs->bufs[i].size;
        if (avail > 0) {
            vec_d chunk = ring_read(&cs->bufs[i], avail);
            vec_d o = stage_process(&cs->st[i], chunk.a, chunk.len);
            free(chunk.a);
            if (o.len > 0) ring_write(&cs->bufs[i + 1], o.a, o.len);
            free(o.a);
        }
        vec_d o = stage_flush(&cs->st[i]);
        if (o.len > 0) ring_write(&cs->bufs[i + 1], o.a, o.len);
        free(o.a);
    }
    ring *fb = &cs->bufs[cs->nstages];
    return copy_out(ring_read(fb, fb->size), out, cap);
}

/* constant.go:429-444 */
API void o_new_reset(o_new_rs *r) {
    for (int c = 0; c < r->channels; c++) {
        chan_state *cs = &r->ch[c];
        for (int j = 0; j < cs->nstages; j++) stage_reset(&cs->st[j]);
        for (int j = 0; j <= cs->nstages; j++) { cs->bufs[j].size = cs->bufs[j].rpos = cs->bufs[j].wpos = 0; }
    }
}

/* constant.go:407-426 */
API int o_new_latency(o_new_rs *r) {
    if (r->channels == 0 || r->nstages == 0) return 0;
    int tot = 0;
    for (int j = 0; j < r->nstages; j++) {
        stage_inst *s = &r->ch[0].st[j];
        tot += (int)((double)stage_latency(s) * stage_ratio(s));
    }
    return tot;
}

/* constant.go:117-119 */
API int64_t o_new_estimate_output(o_new_rs *r, int64_t n) { return (int64_t)((double)n * r->ratio) + 64; }
API double o_new_ratio(o_new_rs *r) { return r->ratio; }
API int o_new_nstages(o_new_rs *r, int *types, double *ratios) {
    for (int j = 0; j < r->nstages; j++) { types[j] = r->types[j]; ratios[j] = r->ratios[j]; }
    return r->nstages;
}
API void o_new_stage_info(o_new_rs *r, int j, o_engine_info *inf) {
    memset(inf, 0, sizeof(*inf));
    stage_inst *s = &r->ch[0].st[j];
    if (s->is_cubic) { inf->kind = 0; return; }
    resampler_info_d(s->eng, inf);
}

/* ------------------------------------------------------------------------- */
/* simdops primitive stand-ins exported for the KAT tests                     */
/* (internal/simdops/ops_test.go:25-70)                                      */
/* ------------------------------------------------------------------------- */
API double o_dot(const double *a, const double *b, int64_t n) { return dot_d(a, b, n); }
API void o_convolve_valid(double *dst, const double *sig, int64_t nsig, const double *ker, int64_t nker) {
    convolve_valid_d(dst, sig, nsig, ker, nker);
}
API double o_cubic_interp_dot(const double *h, const double *a, const double *b, const double *c, const double *d,
                              double x, int64_t n) {
    return cubic_interp_dot_d(h, a, b, c, d, x, n);
}
