// Calibration of rocprofv3 FETCH_SIZE / WRITE_SIZE on gfx950 for the load and store widths the
// product kernels use (MI355X_MICROARCH.md, HBM section: "other access widths are uncalibrated:
// calibrate on a known byte count in your own access pattern").  Each kernel streams exactly
// kBytes (1 GiB, 4x the Infinity Cache) once:
//   rd16  buffer_load_dwordx4, 16 B/lane (ROW16 loads, LDS-DMA tiles)
//   rd8   buffer_load_dwordx2, 8 B/lane, 512 B contiguous per instruction (STEREO loads)
//   rd4   buffer_load_dword, 4 B/lane (PCM16 stereo frames)
//   wr16  16-B/lane stores (hxs epilogue), wr8 8-B/lane stores (PCM16 frame pairs)
// FETCH_SIZE/WRITE_SIZE per dispatch (KiB) x 1024 / kBytes = the counter's fraction of the bytes.
// hipcc --offload-arch=gfx950 -O3 fetch_calib.hip -o fetch_calib
//   rocprofv3 --pmc FETCH_SIZE -d out -o run --output-format csv -- ./fetch_calib
#include <hip/hip_runtime.h>

#include <cstdio>

constexpr long long kBytes = 1LL << 30;
constexpr int kBlocks = 2048, kThreads = 256;

typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
typedef unsigned u32x2 __attribute__((ext_vector_type(2)));

template <int W>
__global__ __launch_bounds__(kThreads) void rd(const char* in, unsigned* sink) {
    // each 2^28-B segment gets its own resource (31-bit offsets)
    unsigned acc = 0;
    const long long per = static_cast<long long>(kThreads) * W;  // bytes per block-iteration
    for (long long base = static_cast<long long>(blockIdx.x) * per; base < kBytes; base += per * gridDim.x) {
        const long long seg = base >> 28;
        __amdgpu_buffer_rsrc_t rs =
            __builtin_amdgcn_make_buffer_rsrc(const_cast<char*>(in + (seg << 28)), 0, 1 << 28, 0x00020000);
        const int o = static_cast<int>(base - (seg << 28)) + threadIdx.x * W;
        if constexpr (W == 16) {
            const u32x4 v = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(rs, o, 0, 0));
            acc += v.x ^ v.y ^ v.z ^ v.w;
        } else if constexpr (W == 8) {
            const u32x2 v = __builtin_bit_cast(u32x2, __builtin_amdgcn_raw_buffer_load_b64(rs, o, 0, 0));
            acc += v.x ^ v.y;
        } else {
            acc += __builtin_amdgcn_raw_buffer_load_b32(rs, o, 0, 0);
        }
    }
    if (acc == 0x12345678u) sink[threadIdx.x] = acc;
}

template <int W>
__global__ __launch_bounds__(kThreads) void wr(char* out) {
    const long long per = static_cast<long long>(kThreads) * W;
    for (long long base = static_cast<long long>(blockIdx.x) * per; base < kBytes; base += per * gridDim.x) {
        char* p = out + base + threadIdx.x * W;
        if constexpr (W == 16) *reinterpret_cast<u32x4*>(p) = u32x4{1u, 2u, 3u, static_cast<unsigned>(base)};
        else *reinterpret_cast<u32x2*>(p) = u32x2{1u, static_cast<unsigned>(base)};
    }
}

int main() {
    char* buf = nullptr;
    unsigned* sink = nullptr;
    if (hipMalloc(&buf, kBytes) != hipSuccess || hipMalloc(&sink, 4096) != hipSuccess) return 1;
    (void)hipMemset(buf, 1, kBytes);
    for (int rep = 0; rep < 2; ++rep) {
        hipLaunchKernelGGL(rd<16>, dim3(kBlocks), dim3(kThreads), 0, 0, buf, sink);
        hipLaunchKernelGGL(rd<8>, dim3(kBlocks), dim3(kThreads), 0, 0, buf, sink);
        hipLaunchKernelGGL(rd<4>, dim3(kBlocks), dim3(kThreads), 0, 0, buf, sink);
        hipLaunchKernelGGL(wr<16>, dim3(kBlocks), dim3(kThreads), 0, 0, buf);
        hipLaunchKernelGGL(wr<8>, dim3(kBlocks), dim3(kThreads), 0, 0, buf);
    }
    if (hipDeviceSynchronize() != hipSuccess) return 2;
    std::printf("fetch_calib: %lld bytes per kernel\n", kBytes);
    (void)hipFree(buf);
    (void)hipFree(sink);
    return 0;
}
