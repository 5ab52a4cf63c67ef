// Microbenchmark: HBM write rate of the streaming kernel's output pattern (cfg2 stereo: 256
// workgroups x 8 chunks of 88 periods x 1280 B, chunk stride 112,640 B) against contiguous
// variants.  hipcc --offload-arch=gfx950 -O3 store_pattern.hip -o /tmp/sp && /tmp/sp
//   A: per instruction 8 x 128-B segments (one per chunk), 10 waves = 10 row blocks of a period
//   B: per instruction 1 KiB contiguous inside one chunk (chunks written one after the other)
//   C: per instruction 1 KiB contiguous, the workgroup's region swept linearly
//   D: as A, but 4 chunks x 256 B per instruction
#include <hip/hip_runtime.h>
#include <cstdio>
typedef float f32x4 __attribute__((ext_vector_type(4)));

constexpr int kChunks = 8, kPeriods = 88, kPeriodB = 1280, kWaves = 10;
constexpr long long kChunkB = (long long)kPeriods * kPeriodB;

template <int MODE>
__global__ __launch_bounds__(640) void k(char* out) {
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    char* blk = out + (long long)blockIdx.x * kChunks * kChunkB;
    const f32x4 v = {1.f, 2.f, 3.f, (float)lane};
    if (MODE == 0) {
        // lane -> chunk (lane & 15) >> 1, 32 B of the row block's 128 B: ((lane >> 4) * 2 + (lane & 1)) * 16
        const int ck = (lane & 15) >> 1, off = ((lane >> 4) * 2 + (lane & 1)) * 16;
        for (int p = 0; p < kPeriods; ++p)
            *reinterpret_cast<f32x4*>(blk + ck * kChunkB + (long long)p * kPeriodB + w * 128 + off) = v;
    } else if (MODE == 1) {
        // each wave: its 1/10 of every period of every chunk as whole KiB pieces (same bytes)
        const long long total = kChunks * kChunkB;  // bytes per workgroup
        for (long long o = (long long)w * 1024; o < total; o += kWaves * 1024) {
            // walk chunks in period order: piece index -> (period group, chunk)
            const long long piece = o / 1024;
            const long long perChunk = kChunkB / 1024;  // 110 pieces
            const long long ck = piece / perChunk, in = piece % perChunk;
            *reinterpret_cast<f32x4*>(blk + ck * kChunkB + in * 1024 + lane * 16) = v;
        }
    } else if (MODE == 2) {
        const long long total = kChunks * kChunkB;
        for (long long o = (long long)w * 1024; o < total; o += kWaves * 1024)
            *reinterpret_cast<f32x4*>(blk + o + lane * 16) = v;
    } else {
        // 4 chunks per instruction, 256 B each; two instructions per (period, row-block pair)
        const int ck = lane >> 4, off = (lane & 15) * 16;
        for (int p = 0; p < kPeriods; ++p)
            if (w < 5)
                for (int h = 0; h < 2; ++h)
                    *reinterpret_cast<f32x4*>(blk + (ck + 4 * h) * kChunkB + (long long)p * kPeriodB + w * 256 + off) = v;
    }
}

int main() {
    const long long bytes = 256LL * kChunks * kChunkB;
    char* out;
    hipMalloc(&out, bytes);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    auto run = [&](auto kern, const char* name) {
        for (int i = 0; i < 3; ++i) kern<<<256, 640>>>(out);
        hipEventRecord(e0);
        for (int i = 0; i < 20; ++i) kern<<<256, 640>>>(out);
        hipEventRecord(e1);
        hipEventSynchronize(e1);
        float ms;
        hipEventElapsedTime(&ms, e0, e1);
        printf("%s: %.1f us  %.2f TB/s\n", name, ms / 20 * 1e3, bytes / (ms / 20 * 1e-3) / 1e12);
    };
    run(k<0>, "A 8x128B segments");
    run(k<1>, "B 1KiB in-chunk");
    run(k<2>, "C 1KiB linear");
    run(k<3>, "D 4x256B segments");
    hipFree(out);
    return 0;
}
