// Microbenchmark: the memory pattern of the headline launch (cfg2: one stereo f32 stream, 600 s at
// 44.1 kHz in, 48 kHz out) with no compute -- the attainable rate of that pattern.  256 workgroups, each
// 8 chunks of 88 macro periods (147 frames in, 160 out each) of the interleaved stream.  Loader waves:
// 6, each with 2 loads of its items in flight, an item = one 64-frame piece of one chunk pair (two
// buffer_load_dwordx2: 512 B contiguous per instruction), as hxt_kernel's FMT 1 loaders.  Store
// waves: 10, one 16-output row block per period each, one 16-B store per lane covering 8 chunks x
// 128 B (16 frames x 2 channels), as the VST 2 epilogue.  The roles run free (no hand-off).
//   hipcc --offload-arch=gfx950 -O3 stereo_copy.hip -o stereo_copy && ./stereo_copy
#include <hip/hip_runtime.h>
#include <cstdio>
typedef float f2v __attribute__((ext_vector_type(2)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

constexpr int kQc = 147, kPc = 160, kNp = 88, kChunks = 8, kWg = 256, kL = 6, kG = 5;
constexpr long long kChunkIn = (long long)kNp * kQc, kChunkOut = (long long)kNp * kPc;  // frames per chunk
constexpr int kPieces = (kG * kQc + 63) / 64;          // 64-frame pieces per chunk and step
constexpr int kItems = (4 * kPieces + kL - 1) / kL;   // (quad = chunk pair, piece) items per loader
constexpr int kSteps = kNp / kG + 1;

template <int MODE>
__global__ __launch_bounds__(1024) void k(const float* in, float* out) {
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const long long f0 = (long long)blockIdx.x * kChunks * kChunkIn, o0 = (long long)blockIdx.x * kChunks * kChunkOut;
    float acc = 0.f;
    if (w < kL) {
        if (!(MODE & 1)) return;
        const char* base = reinterpret_cast<const char*>(in + 2 * f0);
        __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(const_cast<char*>(base), 0, 0x7fffffff, 0x00020000);
        f2v a[2][kItems], b[2][kItems];
        auto issue = [&](int s, f2v (&ra)[kItems], f2v (&rb)[kItems]) {
#pragma unroll
            for (int i = 0; i < kItems; ++i) {
                const int it = w + kL * i, q = it & 3, pc = it >> 2;
                const int row = s * kG * kQc + 64 * pc + lane;
                const bool on = s < kSteps && pc < kPieces && row < kChunkIn;
                const int o = on ? (row + 2 * q * (int)kChunkIn) * 8 : (int)0x80000000u;
                if (MODE & 8) {  // non-temporal global loads (zeros for items past the chunk)
                    const f2v* pa = reinterpret_cast<const f2v*>(base + (on ? o : 0));
                    const f2v* pb = reinterpret_cast<const f2v*>(base + (on ? o + (int)kChunkIn * 8 : 0));
                    ra[i] = on ? __builtin_nontemporal_load(pa) : f2v{0, 0};
                    rb[i] = on ? __builtin_nontemporal_load(pb) : f2v{0, 0};
                } else {
                    ra[i] = __builtin_bit_cast(f2v, __builtin_amdgcn_raw_buffer_load_b64(rs, o, 0, 0));
                    rb[i] = __builtin_bit_cast(f2v, __builtin_amdgcn_raw_buffer_load_b64(rs, on ? o + (int)kChunkIn * 8 : o, 0, 0));
                }
            }
        };
        issue(0, a[0], b[0]);
        issue(1, a[1], b[1]);
        for (int s0 = 0; s0 < kSteps; s0 += 2) {
#pragma unroll
            for (int d = 0; d < 2; ++d) {
#pragma unroll
                for (int i = 0; i < kItems; ++i) acc += a[d][i].x + b[d][i].y;
                issue(s0 + d + 2, a[d], b[d]);
            }
        }
        if (acc == 1234.5f) out[threadIdx.x] = acc;
    } else {
        if (!(MODE & 2)) return;
        const int sw = w - kL, nsw = (blockDim.x >> 6) - kL;
        const int ck = lane >> 3, fr = 2 * (lane & 7);  // lane: chunk lane / 8, frames 2 (lane % 8) .. +1
        for (int p = 0; p < kNp; ++p)
            for (int t = sw; t < kPc / 16; t += nsw) {
                const long long frame = o0 + ck * kChunkOut + (long long)p * kPc + 16 * t + fr;
                const f32x4 y = {acc + p, acc + t, acc, acc};
                if (MODE & 4) __builtin_nontemporal_store(y, reinterpret_cast<f32x4*>(out + 2 * frame));
                else *reinterpret_cast<f32x4*>(out + 2 * frame) = y;
            }
    }
}

int main() {
    const long long inB = (long long)kWg * kChunks * kChunkIn * 8, outB = (long long)kWg * kChunks * kChunkOut * 8;
    float *in, *out;
    if (hipMalloc(&in, inB) != hipSuccess || hipMalloc(&out, outB) != hipSuccess) { printf("alloc failed\n"); return 1; }
    (void)hipMemset(in, 0, inB);
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    auto run = [&](auto kern, double bytes, const char* name) {
        for (int i = 0; i < 3; ++i) kern<<<kWg, 1024>>>(in, out);
        (void)hipEventRecord(e0);
        for (int i = 0; i < 20; ++i) kern<<<kWg, 1024>>>(in, out);
        (void)hipEventRecord(e1);
        (void)hipEventSynchronize(e1);
        float ms;
        (void)hipEventElapsedTime(&ms, e0, e1);
        printf("%-40s %8.4f ms  %.2f TB/s\n", name, ms / 20, bytes / (ms / 20 * 1e-3) / 1e12);
    };
    printf("cfg2 pattern: %lld MB in, %lld MB out\n", inB >> 20, outB >> 20);
    run(k<1>, (double)inB, "loads only (6 loader waves)");
    run(k<2>, (double)outB, "stores only (10 waves, 16 B per lane)");
    run(k<3>, (double)(inB + outB), "loads + stores (cfg2 pattern)");
    run(k<7>, (double)(inB + outB), "loads + non-temporal stores");
    run(k<11>, (double)(inB + outB), "non-temporal loads + stores");
    run(k<15>, (double)(inB + outB), "non-temporal loads + nt stores");
    run(k<3>, (double)(inB + outB), "loads + stores (again)");
    return 0;
}
