// Microbenchmark: HBM read rate of the streaming kernel's input pattern (cfg2 stereo: 256
// workgroups x 8 chunks, chunk stride 88*147*8 B; per step each chunk's next 441 rows x 8 B),
// 6 loader waves per workgroup with D loads in flight (registers), optional s_barrier per step
// with 10 idle waves.  hipcc --offload-arch=gfx950 -O3 load_pattern.hip -o /tmp/lp && /tmp/lp
#include <hip/hip_runtime.h>
#include <cstdio>
typedef float f2v __attribute__((ext_vector_type(2)));

constexpr int kChunks = 8, kSteps = 30, kRows = 441, kNP = 7, kL = 6;
constexpr int kItems = (4 * kNP + kL - 1) / kL;
constexpr long long kChunkB = 88LL * 147 * 8;

template <int D, int BAR>
__global__ __launch_bounds__(1024) void k(const char* in, float* sink) {
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int nw = blockDim.x >> 6;
    const char* blk = in + (long long)blockIdx.x * kChunks * kChunkB;
    __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(const_cast<char*>(blk), 0, 0x7fffffff, 0x00020000);
    float acc = 0.f;
    if (w < nw - kL) {  // idle "compute" waves: only the barriers
        if (BAR)
            for (int s = 0; s < (kSteps + 2 * D - 1) / D * D; ++s) __builtin_amdgcn_s_barrier();
    } else {
        const int l = w - (nw - kL);
        f2v a[D][kItems], b[D][kItems];
        auto issue = [&](int s, f2v (&ra)[kItems], f2v (&rb)[kItems]) {
#pragma unroll
            for (int kk = 0; kk < kItems; ++kk) {
                const int it = l + kk * kL, q = it & 3, i = it >> 2;
                const bool on = it < 4 * kNP && 64 * i + lane < kRows && s < kSteps;
                const int o = on ? (s * kRows + 64 * i + lane) * 8 + 2 * q * (int)kChunkB : (int)0x80000000u;
                ra[kk] = __builtin_bit_cast(f2v, __builtin_amdgcn_raw_buffer_load_b64(rs, o, 0, 0));
                rb[kk] = __builtin_bit_cast(f2v, __builtin_amdgcn_raw_buffer_load_b64(rs, on ? o + (int)kChunkB : o, 0, 0));
            }
        };
#pragma unroll
        for (int d = 0; d < D; ++d) issue(d, a[d], b[d]);
        for (int s0 = 0; s0 < kSteps + D; s0 += D) {
#pragma unroll
            for (int d = 0; d < D; ++d) {
#pragma unroll
                for (int kk = 0; kk < kItems; ++kk) acc += a[d][kk].x + a[d][kk].y + b[d][kk].x + b[d][kk].y;
                issue(s0 + d + D, a[d], b[d]);
                if (BAR) __builtin_amdgcn_s_barrier();
            }
        }
    }
    if (acc == 12345.f) sink[threadIdx.x] = acc;
}

int main() {
    const long long bytes = 256LL * kChunks * kChunkB;
    char* in;
    float* sink;
    (void)hipMalloc(&in, bytes);
    (void)hipMalloc(&sink, 4096);
    (void)hipMemset(in, 0, bytes);
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    const double useful = 256.0 * kChunks * kSteps * kRows * 8;
    auto run = [&](auto kern, int threads, const char* name) {
        for (int i = 0; i < 3; ++i) kern<<<256, threads>>>(in, sink);
        (void)hipEventRecord(e0);
        for (int i = 0; i < 20; ++i) kern<<<256, threads>>>(in, sink);
        (void)hipEventRecord(e1);
        (void)hipEventSynchronize(e1);
        float ms;
        (void)hipEventElapsedTime(&ms, e0, e1);
        printf("%s: %.1f us  %.2f TB/s\n", name, ms / 20 * 1e3, useful / (ms / 20 * 1e-3) / 1e12);
    };
    run(k<2, 0>, 64 * kL, "D2 no barrier, 6 waves");
    run(k<3, 0>, 64 * kL, "D3 no barrier, 6 waves");
    run(k<2, 1>, 64 * (kL + 10), "D2 barrier, 16 waves");
    run(k<3, 1>, 64 * (kL + 10), "D3 barrier, 16 waves");
    run(k<4, 1>, 64 * (kL + 10), "D4 barrier, 16 waves");
    return 0;
}
