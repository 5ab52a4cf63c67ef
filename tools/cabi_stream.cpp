// cabi_stream.cpp -- the drop-in streaming pattern driven straight through the C-ABI
// (what a cgo caller pays per call, without Python in the loop).
//
//   device mode: input already in HBM, gar_process_device per chunk (asynchronous),
//                one synchronise at the end (processinto_bench_test.go:12-205 shape)
//   host mode:   planar float64 host buffers, gar_process_multi_f64 per chunk
//                (H2D + launches + D2H + synchronise inside every call)
//
// build: hipcc -O2 -I include tools/cabi_stream.cpp -L go-audio-resampler_amd -lgar \
//          -Wl,-rpath,'$ORIGIN/../go-audio-resampler_amd' -o tools/cabi_stream
// usage: tools/cabi_stream [chunk=4096] [seconds=60] [channels=2]
#include <hip/hip_runtime.h>

#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "gar.h"

static double now() {
    return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

#define CK(x)                                                                         \
    do {                                                                              \
        int _s = (x);                                                                 \
        if (_s != 0) {                                                                \
            fprintf(stderr, "%s failed: %d (%s)\n", #x, _s, gar_last_error());        \
            exit(1);                                                                  \
        }                                                                             \
    } while (0)

int main(int argc, char** argv) {
    const int chunk = argc > 1 ? atoi(argv[1]) : 4096;
    const double seconds = argc > 2 ? atof(argv[2]) : 60.0;
    const int C = argc > 3 ? atoi(argv[3]) : 2;
    const int64_t frames = static_cast<int64_t>(seconds * 44100);
    std::vector<float> xh(static_cast<size_t>(frames) * C);
    for (int64_t t = 0; t < frames; ++t)
        for (int c = 0; c < C; ++c)
            xh[t * C + c] = static_cast<float>(0.7 * std::sin(2 * M_PI * 440 * t / 44100.0 + c) +
                                               0.2 * std::sin(2 * M_PI * 1750 * t / 44100.0));
    float *xd = nullptr, *yd = nullptr;
    const int64_t ycap = frames * 48000 / 44100 + 64 * (frames / chunk + 2);
    if (hipMalloc(&xd, xh.size() * 4) != hipSuccess || hipMalloc(&yd, static_cast<size_t>(ycap) * C * 4) != hipSuccess)
        return 1;
    (void)hipMemcpy(xd, xh.data(), xh.size() * 4, hipMemcpyHostToDevice);
    hipStream_t st;
    (void)hipStreamCreate(&st);

    gar_config cfg{};
    cfg.input_rate = 44100;
    cfg.output_rate = 48000;
    cfg.channels = C;
    cfg.quality.preset = GAR_QUALITY_HIGH;
    cfg.compute_dtype = GAR_F32;
    gar_resampler* r = nullptr;
    CK(gar_new(&cfg, &r));

    auto devPass = [&]() {
        gar_reset(r);
        int64_t o = 0;
        for (int64_t s = 0; s < frames; s += chunk) {
            const int64_t n = std::min<int64_t>(chunk, frames - s);
            int64_t got = 0;
            CK(gar_process_device(r, xd + s * C, GAR_F32, C, 1, n, C, yd + o * C, GAR_F32, C, 1, ycap - o, &got, st));
            o += got;
        }
        int64_t got = 0;
        CK(gar_flush_device(r, C, yd + o * C, GAR_F32, C, 1, ycap - o, &got, st));
        (void)hipStreamSynchronize(st);
        return o + got;
    };
    devPass();
    const double t0 = now();
    const int64_t nout = devPass();
    const double t1 = now();
    const int64_t calls = (frames + chunk - 1) / chunk;
    printf("{\"mode\": \"device\", \"chunk\": %d, \"channels\": %d, \"seconds\": %.1f, \"calls\": %lld, \"us_per_call\": %.2f, "
           "\"msamples_per_s\": %.2f, \"outputs\": %lld}\n",
           chunk, C, seconds, (long long)calls, (t1 - t0) / calls * 1e6, frames * C / (t1 - t0) / 1e6, (long long)nout);

    // enqueue cost alone (no synchronise inside the timed loop of calls)
    gar_reset(r);
    double tq = 0;
    {
        int64_t o = 0;
        const double a = now();
        for (int64_t s = 0; s < frames; s += chunk) {
            const int64_t n = std::min<int64_t>(chunk, frames - s);
            int64_t got = 0;
            CK(gar_process_device(r, xd + s * C, GAR_F32, C, 1, n, C, yd + o * C, GAR_F32, C, 1, ycap - o, &got, st));
            o += got;
        }
        tq = now() - a;
        (void)hipStreamSynchronize(st);
    }
    printf("{\"mode\": \"device_enqueue_only\", \"us_per_call\": %.2f}\n", tq / calls * 1e6);

    // host C-ABI (ProcessMulti over planar float64), bounded to 15 s (3 s at >= 64 channels)
    const int64_t hf = std::min<int64_t>(frames, (C >= 64 ? 3 : 15) * 44100);
    std::vector<std::vector<double>> in(C, std::vector<double>(hf)), out(C, std::vector<double>(chunk * 2 + 64));
    for (int c = 0; c < C; ++c)
        for (int64_t t = 0; t < hf; ++t) in[c][t] = xh[t * C + c];
    std::vector<const double*> ip(C);
    std::vector<double*> op(C);
    for (int c = 0; c < C; ++c) op[c] = out[c].data();
    std::vector<int64_t> cnt(C);
    auto hostPass = [&]() {
        gar_reset(r);
        for (int64_t s = 0; s < hf; s += chunk) {
            const int64_t n = std::min<int64_t>(chunk, hf - s);
            for (int c = 0; c < C; ++c) ip[c] = in[c].data() + s;
            CK(gar_process_multi_f64(r, ip.data(), C, n, op.data(), chunk * 2 + 64, cnt.data()));
        }
    };
    hostPass();
    const double h0 = now();
    hostPass();
    const double h1 = now();
    const int64_t hcalls = (hf + chunk - 1) / chunk;
    printf("{\"mode\": \"host_multi_f64\", \"chunk\": %d, \"calls\": %lld, \"us_per_call\": %.2f, \"msamples_per_s\": %.2f}\n",
           chunk, (long long)hcalls, (h1 - h0) / hcalls * 1e6, hf * C / (h1 - h0) / 1e6);
    gar_free(r);

    // the reference's own ProcessInto benchmark shape (processinto_bench_test.go:30-47): NewEngine
    // 48k->16k QualityMedium, Reset + ProcessInto of 3 s of mono float64 per iteration
    gar_resampler* e = nullptr;
    CK(gar_new_engine(48000, 16000, GAR_QUALITY_MEDIUM, GAR_F64, &e));
    std::vector<double> min(48000 * 3), mout(gar_estimate_output(e, 48000 * 3));
    for (size_t i = 0; i < min.size(); ++i) min[i] = static_cast<double>(i) * 1e-5;
    auto monoPass = [&]() {
        gar_reset(e);
        int64_t got = 0;
        CK(gar_process_into_f64(e, min.data(), static_cast<int64_t>(min.size()), mout.data(),
                                static_cast<int64_t>(mout.size()), &got));
        return got;
    };
    for (int i = 0; i < 3; ++i) monoPass();
    const int iters = 200;
    const double m0 = now();
    for (int i = 0; i < iters; ++i) monoPass();
    const double m1 = now();
    printf("{\"mode\": \"engine_processinto_48k_16k_medium_3s\", \"us_per_call\": %.2f, \"msamples_per_s\": %.2f}\n",
           (m1 - m0) / iters * 1e6, 48000.0 * 3 * iters / (m1 - m0) / 1e6);
    gar_free(e);
    return 0;
}
