/*
 * gar.h -- C ABI of the MI355X-native polyphase-FIR resampling engine.
 *
 * Drop-in boundary for tphakala/go-audio-resampler's resampling path: every
 * entry point below replaces one Go entry point (cited path:line relative to
 * the reference repo) and keeps its argument meaning, output lengths, state
 * semantics and error behaviour.  A cgo shim implementing the Go
 * `resampler.Resampler` interface over this ABI is given in INTEGRATION.md.
 *
 * Plain C types only: pointers, sizes, doubles.  Host-memory entry points
 * (the cgo path) copy through the GPU; the *_device entry points take
 * device-resident buffers and a HIP stream (hipStream_t passed as void*).
 *
 * Streams: interleaved multi-channel data uses element (t, c) at
 * base[t * frame_stride + c * channel_stride]  (interleaved: (C, 1);
 * planar with pitch P: (1, P)).
 */
#ifndef GAR_H
#define GAR_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct gar_resampler gar_resampler;

/* Status codes map 1:1 to the Go sentinels (resample.go:156-165). */
typedef enum gar_status {
    GAR_OK = 0,
    GAR_ERR_INVALID_CONFIG = 1,   /* ErrInvalidConfig   resample.go:158 */
    GAR_ERR_BUFFER_TOO_SMALL = 2, /* ErrBufferTooSmall  resample.go:161 -- returned before any state change */
    GAR_ERR_NOT_SUPPORTED = 3,    /* ErrNotSupported    resample.go:164 */
    GAR_ERR_CHANNEL_MISMATCH = 4, /* "expected %d channels, got %d" constant.go:205-207 */
    GAR_ERR_DEVICE = 5,           /* HIP runtime failure / no MI355X visible */
    GAR_ERR_INTERNAL = 6,         /* EstimateOutput underestimate (the Go code panics, constant.go:340-342) */
    GAR_ERR_INVALID_ARGUMENT = 7  /* NULL handle / bad channel index ("channel %d out of range" constant.go:256) */
} gar_status;

/* resampler.QualityPreset (resample.go:104-131) */
enum { GAR_QUALITY_QUICK = 0, GAR_QUALITY_LOW = 1, GAR_QUALITY_MEDIUM = 2, GAR_QUALITY_HIGH = 3,
       GAR_QUALITY_VERYHIGH = 4, GAR_QUALITY_CUSTOM = 5 };
/* resampler.QualityFlags (resample.go:133-153) */
enum { GAR_FLAG_NO_INTERPOLATION = 1, GAR_FLAG_MINIMUM_PHASE = 2, GAR_FLAG_LINEAR_PHASE = 4,
       GAR_FLAG_ALLOW_ALIASING = 8, GAR_FLAG_NO_SIMD = 16 };
/* sample / compute types.  Compute: GAR_F64 (the reference's float64), GAR_F32 (float32-class:
 * f16-split products on the f16 matrix cores, f32 accumulation, error <= exact-f32 arithmetic's
 * for full-scale material; the fixed input split scale 2^12 gives inputs an ABSOLUTE precision
 * floor of about 2^-47 (f16 subnormals), so material quieter than ~2^-26 (-156 dBFS) loses the
 * relative precision the reference's float64 New path keeps -- choose GAR_F64 or GAR_F32_EXACT
 * for such signals; |x| >= 16, Inf and NaN are recomputed exactly in f64),
 * GAR_F32_EXACT (exact f32 products on the f32 matrix cores). */
enum { GAR_F64 = 0, GAR_F32 = 1, GAR_F32_EXACT = 2 };
/* integer PCM sample types of the device entry points (in_dtype / out_dtype of gar_process_device
 * and gar_flush_device), after cmd/resample-wav/main.go:444-543: input sample i -> float64(i) *
 * (1 / maxVal) in the compute type; output y -> int(clamp(float64(y), -1, 1) * maxVal) (truncation),
 * maxVal = 32767 (PCM16, int16 storage), 8388607 (PCM24, int32 storage), 2147483647 (PCM32, int32).
 * Fused into the split-f16 kernel's loads and stores for single-stage float32 plans; staged
 * through a conversion kernel otherwise. */
enum { GAR_PCM16 = 16, GAR_PCM24 = 24, GAR_PCM32 = 32 };
/* engine.Quality (internal/engine/filter_params.go:16-41), for gar_design_engine */
enum { GAR_ENGINE_QUICK = 0, GAR_ENGINE_LOW, GAR_ENGINE_MEDIUM, GAR_ENGINE_HIGH, GAR_ENGINE_VERYHIGH,
       GAR_ENGINE_16BIT, GAR_ENGINE_20BIT, GAR_ENGINE_24BIT, GAR_ENGINE_28BIT, GAR_ENGINE_32BIT };

/* resampler.QualitySpec (resample.go:77-102) */
typedef struct gar_quality_spec {
    int32_t preset;
    int32_t precision;
    double phase_response;
    double passband_end;
    double stopband_begin;
    uint32_t flags;
} gar_quality_spec;

/* resampler.Config (resample.go:46-73) + three engine extensions. */
typedef struct gar_config {
    double input_rate;
    double output_rate;
    int32_t channels;
    gar_quality_spec quality;
    int64_t max_input_size;
    int32_t enable_simd;
    int32_t enable_parallel;
    /* extensions (zero = reference behaviour) */
    int32_t compute_dtype; /* GAR_F64 (the New path computes in float64, constant.go:121-146), GAR_F32, GAR_F32_EXACT */
    int32_t device;        /* HIP device ordinal */
    int32_t dry_run;       /* 1: host state machine only, no GPU work; process calls report lengths only */
} gar_config;

/* resampler.Info (resample.go:294-316) */
typedef struct gar_info {
    char algorithm[32];
    int32_t filter_length;
    int32_t phases;
    int32_t latency;
    int64_t memory_usage;
    int32_t simd_enabled;
    char simd_type[48];
} gar_info;

/* ---- construction -------------------------------------------------------- */
/* Config.Validate (resample.go:168-214). */
gar_status gar_config_validate(const gar_config *cfg);
/* GetPresetSpec (resample.go:217-267). */
gar_quality_spec gar_preset_spec(int32_t preset);
/* resampler.New (resample.go:272-292).  Like the Go code, a non-custom preset
 * is expanded into cfg->quality (resample.go:282-284). */
gar_status gar_new(gar_config *cfg, gar_resampler **out);
/* n_streams independent New(cfg) resamplers processed in lockstep as one GPU
 * batch (channel index = stream * cfg->channels + ch).  Each stream obeys the
 * reference's 256-channel limit (constants.go:9). */
gar_status gar_new_batch(gar_config *cfg, int32_t n_streams, gar_resampler **out);
/* resampler.NewEngine (convenience.go:125) when dtype == GAR_F64,
 * resampler.NewEngineFloat32 (convenience.go:329) when dtype == GAR_F32. */
gar_status gar_new_engine(double input_rate, double output_rate, int32_t preset, int32_t dtype,
                          gar_resampler **out);
void gar_free(gar_resampler *r);
/* engine.NewResampler[F](in, out, quality) (internal/engine/resampler.go:51-179)
 * with an engine.Quality (GAR_ENGINE_*) -- the engine seam cmd/resample-wav
 * drives directly (cmd/resample-wav/helpers.go:77-97) and the reference's
 * engine tests use.  dtype GAR_F64 = Resampler[float64]; GAR_F32 /
 * GAR_F32_EXACT = Resampler[float32] (float32 I/O). */
gar_status gar_new_engine_quality(double input_rate, double output_rate, int32_t engine_quality, int32_t dtype,
                                  gar_resampler **out);
/* Host-only NewEngine (no GPU work; process calls report exact lengths only).
 * Used to test the stream-length state machine on machines without a GPU. */
gar_status gar_new_engine_dry(double input_rate, double output_rate, int32_t preset, int32_t dtype,
                              gar_resampler **out);

/* ---- host-memory streaming (cgo path; channel 0 unless noted) ------------- */
/* EstimateOutput (constant.go:117-119, convenience.go:168-170). */
int64_t gar_estimate_output(const gar_resampler *r, int64_t input_len);
/* Exact number of samples the next process call on `channel` would return. */
int64_t gar_output_size(const gar_resampler *r, int32_t channel, int64_t input_len);
/* Exact number of samples Flush on `channel` would return now. */
int64_t gar_flush_size(const gar_resampler *r, int32_t channel);

/* Process / ProcessFloat32 (constant.go:88-146, convenience.go:138,341): fills
 * out[0:*n_out]; GAR_ERR_BUFFER_TOO_SMALL (no state change) if cap < the exact
 * output size. */
gar_status gar_process_f64(gar_resampler *r, const double *in, int64_t n, double *out, int64_t cap, int64_t *n_out);
gar_status gar_process_f32(gar_resampler *r, const float *in, int64_t n, float *out, int64_t cap, int64_t *n_out);
/* ProcessInto / ProcessFloat32Into (constant.go:103-112, :161-199,
 * convenience.go:145-160, :351-366): GAR_ERR_BUFFER_TOO_SMALL before any state
 * change when cap < EstimateOutput(n). */
gar_status gar_process_into_f64(gar_resampler *r, const double *in, int64_t n, double *out, int64_t cap,
                                int64_t *n_out);
gar_status gar_process_into_f32(gar_resampler *r, const float *in, int64_t n, float *out, int64_t cap,
                                int64_t *n_out);
/* ProcessMulti (constant.go:204-252): in[c][0:n] planar; out[c] with capacity
 * cap each; n_out[c] per channel. */
gar_status gar_process_multi_f64(gar_resampler *r, const double *const *in, int32_t n_channels, int64_t n,
                                 double *const *out, int64_t cap, int64_t *n_out);
/* Flush (constant.go:349-354, resampler.go:275-322): channel 0. */
gar_status gar_flush_f64(gar_resampler *r, double *out, int64_t cap, int64_t *n_out);
gar_status gar_flush_f32(gar_resampler *r, float *out, int64_t cap, int64_t *n_out);
/* FlushMulti (constant.go:390-404). */
gar_status gar_flush_multi_f64(gar_resampler *r, double *const *out, int32_t n_channels, int64_t cap,
                               int64_t *n_out);

/* ---- device-resident batched streaming (all channels in lockstep) -------- */
/* Process `frames` frames of all `channels` channels (must equal the handle's
 * channel count: GAR_ERR_CHANNEL_MISMATCH otherwise, like ProcessMulti,
 * constant.go:205-207) from device memory `in` (dtype in_dtype) into device
 * memory `out`; *out_frames = frames produced per channel.
 * GAR_ERR_BUFFER_TOO_SMALL (no state change) if out_cap_frames is smaller than
 * the exact output size.  Asynchronous on `stream` (NULL = the default
 * stream); returns once the work is enqueued.  Calls on one handle are
 * ordered even across streams (each waits for the handle's previous call);
 * the caller keeps `in` alive and `out` untouched until `stream` has run the
 * call.  Cost of that ordering: while a handle is used on ONE stream its calls
 * record no event (an event costs ~3.5 us of stream time per call), so the
 * first call on a different stream, gar_synchronize, gar_reset and gar_free
 * wait with hipDeviceSynchronize -- every stream of the device, including
 * other handles' work; do not call them while another thread captures a
 * stream.  After the first switch every call records an event and these wait
 * for that event only.  A device error leaves the handle refusing work (GAR_ERR_DEVICE)
 * until gar_reset.  The handle's device is made current for the call and the
 * caller's current device restored. */
gar_status gar_process_device(gar_resampler *r, const void *in, int32_t in_dtype, int64_t in_frame_stride,
                              int64_t in_channel_stride, int64_t frames, int32_t channels, void *out,
                              int32_t out_dtype, int64_t out_frame_stride, int64_t out_channel_stride,
                              int64_t out_cap_frames, int64_t *out_frames, void *stream);
/* Flush all channels into device memory (FlushMulti semantics); `channels` as above. */
gar_status gar_flush_device(gar_resampler *r, int32_t channels, void *out, int32_t out_dtype,
                            int64_t out_frame_stride, int64_t out_channel_stride, int64_t out_cap_frames,
                            int64_t *out_frames, void *stream);
/* Exact lockstep output sizes (-1 if channels are not in lockstep). */
int64_t gar_device_output_size(const gar_resampler *r, int64_t frames);
int64_t gar_device_flush_size(const gar_resampler *r);
/* Waits until every call enqueued on the handle has run and reports how it ended: GAR_OK, or
 * GAR_ERR_DEVICE when a kernel of one of them reported a broken invariant into the handle's
 * device status word (e.g. an expired progress wait of the streaming kernel: its outputs are
 * invalid) or a HIP error occurred; the handle then refuses work until gar_reset.  Every ABI call
 * also checks the status word on entry, and the host-memory calls (which synchronise) after their
 * own kernels.  No Go counterpart: the reference's calls are synchronous (constant.go:88-146); this
 * is the synchronisation point of the asynchronous *_device entry points. */
gar_status gar_synchronize(gar_resampler *r);

/* ---- state / introspection ----------------------------------------------- */
void gar_reset(gar_resampler *r);                       /* Reset (constant.go:429-444, resampler.go:325-340) */
double gar_get_ratio(const gar_resampler *r);           /* GetRatio (constant.go:447) */
int32_t gar_get_latency(const gar_resampler *r);        /* GetLatency (constant.go:407-426) */
gar_status gar_get_info(const gar_resampler *r, gar_info *info); /* GetInfo (constant.go:452-485) */
int32_t gar_channels(const gar_resampler *r);
/* GetStatistics (internal/engine/resampler.go:348-353; SimpleResampler{,Float32}.GetStatistics
 * convenience.go:184-187,393-396): samplesIn / samplesOut of channel `ch`'s engine -- input frames of
 * every non-empty Process, output frames of every Process and Flush (the QualityQuick engine's Flush
 * is uncounted, resampler.go:276-279), both zeroed by Reset.  GAR_ERR_INVALID_ARGUMENT for a bad ch. */
gar_status gar_get_statistics(const gar_resampler *r, int32_t ch, int64_t *samples_in, int64_t *samples_out);
const char *gar_status_string(gar_status s);
const char *gar_last_error(void);                       /* thread-local detail for the last failure */
/* HIP-event timing of every MFMA FIR launch (bracketed on its own stream). */
void gar_profile_enable(gar_resampler *r, int32_t on);
/* Restricts the event timing to the launch kinds whose bit is set (kind k = bit k, see
 * gar_profile_read; default all): an event pair costs a few microseconds of stream time, so a
 * timed region brackets only the kernel it measures. */
void gar_profile_kinds(gar_resampler *r, uint32_t kinds);
/* Sum of launch durations (ms) and launch count of one kernel kind (0 fused
 * DFT+polyphase FIR, 1 DFT FIR, 2 decimator FIR, 3 fused FIR launched by a
 * flush, 4 polyphase stage with live cubic coefficients, 5 QualityQuick cubic
 * stage) since its last read. */
gar_status gar_profile_read(gar_resampler *r, int32_t kind, double *ms, int64_t *launches);
/* Spread of the launches the last gar_profile_read of `kind` summed: min, median, max ms per launch
 * (zeros when there were none). */
gar_status gar_profile_launch_stats(gar_resampler *r, int32_t kind, double *min_ms, double *median_ms,
                                    double *max_ms);
/* Execution mode of pipeline stage `stage` of channel 0's group: *fused_plan = 1 when the
 * stage's DFT x2 + polyphase pair has a composite MFMA plan, *fused_now = 1 while the stream
 * still runs on it (0 after a stage-by-stage fallback: Process after Flush, the
 * polyphase_stage.go:300-307 history quirk).  Works on dry-run handles. */
gar_status gar_stage_state(const gar_resampler *r, int32_t stage, int32_t *fused_plan, int32_t *fused_now);

/* Host self-test of the staging pool the host calls convert through (no GPU): `threads` caller
 * threads each run `iters` conversion jobs of channels x frames through the pool at once (one job
 * at a time uses the workers, the others run inline) and check every element.  0 = every element
 * right; else the number of wrong elements.  For tests (CPU suite; tools/asan_tests.sh with TSan). */
int64_t gar_dev_pool_selftest(int32_t threads, int32_t iters, int32_t channels, int64_t frames);

/* ---- host-only design introspection (no GPU needed) ----------------------- */
typedef struct gar_engine_geometry {
    int32_t kind; /* 0 cubic, 1 DFT-only, 2 DFT x2 + polyphase, 3 decimator, 4 pass-through */
    int32_t dft_factor, dft_taps;
    int32_t poly_phases, poly_taps;
    int64_t poly_step;
    int32_t decim_factor, decim_taps;
    int32_t fused;                 /* DFT+polyphase composed into one MFMA FIR (step has no fraction) */
    int32_t fir_period_out, fir_period_in, fir_taps_max;
    double useful_macs_per_output; /* of the MFMA FIR executed for this engine */
    double mfma_macs_per_output;
} gar_engine_geometry;
/* engine.NewResampler[float64](in, out, quality) design (resampler.go:51-179).
 * Any output buffer may be NULL: dft [factor*taps], poly_* [phases*taps] (the
 * Go layout), decim [taps]. */
gar_status gar_design_engine(double input_rate, double output_rate, int32_t engine_quality,
                             gar_engine_geometry *geom, double *dft, double *poly_a, double *poly_b,
                             double *poly_c, double *poly_d, double *decim);
/* Composite FIR of a fused DFT+polyphase engine: rows [P][taps_max] (zero padded), offsets [P]. */
gar_status gar_design_composite(double input_rate, double output_rate, int32_t engine_quality, double *rows,
                                int64_t *offsets);

/* Pipeline stages of a handle (pipeline.BuildPipeline, internal/pipeline/pipeline.go:104-183; 0 when the
 * ratio is within 0.1 % of 1) and the design geometry + engine ratio of stage `stage`
 * (engine.NewResampler[float64](48000, 48000*ratio, q), stages.go:54-70). */
int32_t gar_num_stages(const gar_resampler *r);
gar_status gar_stage_geometry(const gar_resampler *r, int32_t stage, double *stage_ratio, gar_engine_geometry *geom);

#ifdef __cplusplus
}
#endif
#endif /* GAR_H */
