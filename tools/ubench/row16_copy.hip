// Microbenchmark: the memory pattern of the north-star launch (ns256: 256-channel f32 rows, 60 s at
// 44.1 kHz in, 48 kHz out) with no compute, to price the attainable HBM rate of that pattern.
// Workgroup = block of W channels x one chunk of 1125 macro periods (147 rows in, 160 out each);
// 256 workgroups, blocks 2m / 2m+1 (the two 64-B halves of every 128-B row) on one XCD like
// hxt_kernel's xcdPair.  Loader waves: 6, each with D = 2 loads of 8 buffer_load_dwordx4 in flight
// (lane = 16 quad + row: 16 rows x 64 B per instruction), as hxt_kernel's FMT 2 loaders.  Store waves:
// 10, one 16x16 output tile per period each (VST 0: four 4-B stores per lane to four rows, as the
// kernel's epilogue) or (S16) one 16-B store per lane.  The two roles run free (no hand-off), so the
// time is what the memory pipes and HBM allow for this mix.  W = 32 (full 128-B rows, 256 workgroups
// and two 16-channel output tiles per period and row block) prices a 32-channel block.
//   hipcc --offload-arch=gfx950 -O3 row16_copy.hip -o row16_copy && ./row16_copy
#include <hip/hip_runtime.h>
#include <cstdio>
typedef float f32x4 __attribute__((ext_vector_type(4)));

constexpr int kC = 256, kQc = 147, kPc = 160, kPeriods = 16 * 1125;  // 60 s of 44.1 kHz: 18000 macro periods
constexpr long long kRowsIn = (long long)kPeriods * kQc, kRowsOut = (long long)kPeriods * kPc;
constexpr int kL = 6, kItems = 8;

// MODE bit 1 loads, bit 2 stores; S16: 16-B stores; W: channels per workgroup (16 or 32).  256
// workgroups: (kC / W) channel groups x (256 W / kC) chunks of the stream.
template <int MODE, int S16, int W, int MAP = 0>
__global__ __launch_bounds__(1024) void k(const float* in, float* out) {
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int bi = blockIdx.x;
    // workgroup slot -> block (W = 16, xcdPair: slots i and i + 8 are blocks 2m and 2m + 1)
    constexpr int ngrp = kC / W, nchunk = 256 / ngrp, np = kPeriods / nchunk;
    // MAP 1 (chunk-major): XCD x = bi % 8 runs every channel group of chunks (nchunk / 8) x .. -- each
    // row's 1 KB read and written by the workgroups of one XCD, in step
    const int b = MAP == 1 ? (bi / 8) % ngrp + ngrp * ((bi % 8) * (nchunk / 8) + (bi / 8) / ngrp)
                : W == 16 ? 2 * ((bi >> 4) * 8 + (bi & 7)) + ((bi >> 3) & 1) : bi;
    const int g = b % ngrp, chunk = b / ngrp;
    const long long r0 = (long long)chunk * np * kQc, o0 = (long long)chunk * np * kPc;
    float acc = 0.f;
    if (w < kL) {
        if (!(MODE & 1)) return;
        const char* base = reinterpret_cast<const char*>(in + r0 * kC + W * g);
        __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(const_cast<char*>(base), 0, 0x7fffffff, 0x00020000);
        constexpr int kLanesRow = W / 4;          // 16-B lanes per row
        constexpr int kRowsPer = 64 / kLanesRow;   // rows per instruction (a piece)
        constexpr int kPieces = (np * kQc + kRowsPer - 1) / kRowsPer;
        constexpr int kLoads = (kPieces + kL * kItems - 1) / (kL * kItems);
        const int lr = lane / kLanesRow, lc = lane % kLanesRow;
        f32x4 buf[2][kItems];
        auto issue = [&](int j, f32x4 (&r)[kItems]) {
#pragma unroll
            for (int i = 0; i < kItems; ++i) {
                const int pc = j * kL * kItems + w + kL * i;
                const int row = pc * kRowsPer + lr;
                const bool on = j < kLoads && row < np * kQc;
                const int o = on ? row * kC * 4 + lc * 16 : (int)0x80000000u;
                r[i] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(rs, o, 0, 0));
            }
        };
        issue(0, buf[0]);
        issue(1, buf[1]);
        for (int j0 = 0; j0 < kLoads; j0 += 2) {
#pragma unroll
            for (int d = 0; d < 2; ++d) {
#pragma unroll
                for (int i = 0; i < kItems; ++i) acc += buf[d][i].x + buf[d][i].w;
                issue(j0 + d + 2, buf[d]);
            }
        }
        if (acc == 1234.5f) out[threadIdx.x] = acc;
    } else {
        if (!(MODE & 2)) return;
        const int sw = w - kL, nsw = (blockDim.x >> 6) - kL;
        const int grp = lane >> 4, l16 = lane & 15;
        for (int p = 0; p < np; ++p) {
            if (S16 == 2) {  // W = 32: a row block's 16 rows x 32 channels as 8 dword stores of 2 whole 128-B rows
                for (int t = sw; t < kPc / 16; t += nsw) {
                    const long long row = (long long)p * kPc + 16 * t;
                    float* ob = out + o0 * kC + W * g;
#pragma unroll
                    for (int i = 0; i < 8; ++i) ob[(row + 2 * i + (lane >> 5)) * kC + (lane & 31)] = acc + p + i;
                }
                continue;
            }
            for (int t = sw; t < (kPc / 16) * (W / 16); t += nsw) {  // row block t % 10 of period p, column half t / 10
                const int h = t / (kPc / 16), rb = t % (kPc / 16);
                float* ob = out + o0 * kC + W * g + 16 * h;
                const long long row = (long long)p * kPc + 16 * rb;
                const f32x4 y = {acc + p, acc + t, acc, acc};
                if (S16) {
                    *reinterpret_cast<f32x4*>(ob + (row + l16) * kC + 4 * grp) = y;
                } else {
#pragma unroll
                    for (int i = 0; i < 4; ++i) ob[(row + 4 * grp + i) * kC + l16] = y[i];
                }
            }
        }
    }
}

int main() {
    const long long inB = kRowsIn * kC * 4, outB = kRowsOut * kC * 4;
    float *in, *out;
    if (hipMalloc(&in, inB) != hipSuccess || hipMalloc(&out, outB) != hipSuccess) { printf("alloc failed\n"); return 1; }
    (void)hipMemset(in, 0, inB);
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    auto run = [&](auto kern, int wgs, int threads, double bytes, const char* name) {
        for (int i = 0; i < 2; ++i) kern<<<wgs, threads>>>(in, out);
        (void)hipEventRecord(e0);
        for (int i = 0; i < 5; ++i) kern<<<wgs, threads>>>(in, out);
        (void)hipEventRecord(e1);
        (void)hipEventSynchronize(e1);
        float ms;
        (void)hipEventElapsedTime(&ms, e0, e1);
        printf("%-48s %8.3f ms  %.2f TB/s\n", name, ms / 5, bytes / (ms / 5 * 1e-3) / 1e12);
    };
    const int T = 64 * 16;
    run(k<1, 0, 16>, 256, T, (double)inB, "W16 loads only (6 loader waves)");
    run(k<2, 0, 16>, 256, T, (double)outB, "W16 stores only, 4x4-B per lane (VST 0)");
    run(k<2, 1, 16>, 256, T, (double)outB, "W16 stores only, 16-B per lane");
    run(k<3, 0, 16>, 256, T, (double)(inB + outB), "W16 loads + 4x4-B stores (ns256 pattern)");
    run(k<3, 1, 16>, 256, T, (double)(inB + outB), "W16 loads + 16-B stores");
    run(k<1, 0, 16, 1>, 256, T, (double)inB, "W16 chunk-major XCD map: loads only");
    run(k<2, 0, 16, 1>, 256, T, (double)outB, "W16 chunk-major XCD map: 4x4-B stores only");
    run(k<3, 0, 16, 1>, 256, T, (double)(inB + outB), "W16 chunk-major XCD map: loads + 4x4-B stores");
    run(k<3, 1, 16, 1>, 256, T, (double)(inB + outB), "W16 chunk-major XCD map: loads + 16-B stores");
    run(k<1, 0, 32>, 256, T, (double)inB, "W32 loads only (128-B rows)");
    run(k<3, 0, 32>, 256, T, (double)(inB + outB), "W32 loads + 4x4-B stores");
    run(k<3, 1, 32>, 256, T, (double)(inB + outB), "W32 loads + 16-B stores");
    run(k<3, 0, 32, 1>, 256, T, (double)(inB + outB), "W32 chunk-major XCD map: loads + 4x4-B stores");
    run(k<2, 0, 32>, 256, T, (double)outB, "W32 stores only, 4x4-B per lane (64-B row halves)");
    run(k<2, 2, 32>, 256, T, (double)outB, "W32 stores only, 2 whole rows per dword store");
    run(k<3, 2, 32>, 256, T, (double)(inB + outB), "W32 loads + 2-whole-row dword stores");
    run(k<3, 2, 32, 1>, 256, T, (double)(inB + outB), "W32 chunk-major: loads + 2-whole-row stores");
    return 0;
}
