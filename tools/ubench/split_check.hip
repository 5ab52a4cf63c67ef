// Bit check of the two f16 hi/lo splits (gar_hx.hpp hxSplit2Plain vs hxSplit2Mix) and of the hi-half
// loud test (gar_hxt.hpp GAR_HXT_HILOUD) against !(|x| < kHxLoud), over every f32 bit pattern with a
// stride and a set of edge values.  usage: split_check [stride]   (prints mismatches; exit 1 on any)
#include "gar_hx.hpp"
#include <cstdio>
#include <cstdlib>
using namespace gar;
__global__ void check(uint32_t stride, unsigned long long* bad, unsigned long long* n) {
    const uint64_t t = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
    const uint64_t i0 = t * stride * 2;
    if (i0 >= (1ull << 32)) return;
    const float a = __uint_as_float(static_cast<uint32_t>(i0)), b = __uint_as_float(static_cast<uint32_t>(i0 + stride));
    uint32_t h0, l0, h1, l1;
    hxSplit2Plain(a, b, h0, l0);
    hxSplit2Mix(a, b, h1, l1);
    const bool la = hxLoud(a), lb = hxLoud(b);
    const bool ha = (h1 & 0x7fffu) >= 0x7c00u, hb = ((h1 >> 16) & 0x7fffu) >= 0x7c00u;
    const bool hpa = (h0 & 0x7fffu) >= 0x7c00u, hpb = ((h0 >> 16) & 0x7fffu) >= 0x7c00u;
    // loud elements are staged as zero (their halves never reach the MFMAs): compare halves only for
    // quiet ones; -0 may differ in the hi sign bit only (documented in gar_hx.hpp)
    bool ok = la == ha && lb == hb && la == hpa && lb == hpb;
    if (!la) ok &= ((h0 ^ h1) & 0xffffu) == 0 || (((h0 ^ h1) & 0xffffu) == 0x8000u && (h0 & 0x7fffu) == 0);
    if (!lb) ok &= ((h0 ^ h1) >> 16) == 0 || (((h0 ^ h1) >> 16) == 0x8000u && ((h0 >> 16) & 0x7fffu) == 0);
    if (!la) ok &= (l0 & 0xffffu) == (l1 & 0xffffu);
    if (!lb) ok &= (l0 >> 16) == (l1 >> 16);
    atomicAdd(n, 1ull);
    if (!ok && atomicAdd(bad, 1ull) < 8)
        printf("mismatch a=%08x b=%08x plain %08x/%08x mix %08x/%08x loud %d%d hi %d%d\n", __float_as_uint(a), __float_as_uint(b),
               h0, l0, h1, l1, la, lb, ha, hb);
}
int main(int argc, char** argv) {
    const uint32_t stride = argc > 1 ? atoi(argv[1]) : 1;
    unsigned long long *bad, *n;
    hipMallocManaged(&bad, 8); hipMallocManaged(&n, 8);
    *bad = 0; *n = 0;
    const uint64_t pairs = (1ull << 32) / (2ull * stride);
    const uint64_t blocks = (pairs + 255) / 256;
    hipLaunchKernelGGL(check, dim3(static_cast<unsigned>(blocks)), dim3(256), 0, 0, stride, bad, n);
    if (hipDeviceSynchronize() != hipSuccess) { printf("launch failed\n"); return 2; }
    printf("split_check stride %u: %llu pairs, %llu mismatches\n", stride, *n, *bad);
    return *bad ? 1 : 0;
}
