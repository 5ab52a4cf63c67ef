// Lane semantics of the gfx950 swaps hxtStoreRows relies on (gar_hxt.hpp): v_permlane16_swap_b32 swaps
// the odd 16-lane rows of its first operand with the even rows of its second, v_permlane32_swap_b32 the
// upper 32 lanes of the first with the lower 32 of the second.  Prints OK or the first mismatch.
#include <hip/hip_runtime.h>
#include <cstdio>
__global__ void k(unsigned* o) {
    const unsigned l = threadIdx.x;
    unsigned a = l, b = 100 + l;
    auto r = __builtin_amdgcn_permlane16_swap(a, b, false, false);
    o[l] = r[0]; o[64 + l] = r[1];
    a = l; b = 100 + l;
    auto q = __builtin_amdgcn_permlane32_swap(a, b, false, false);
    o[128 + l] = q[0]; o[192 + l] = q[1];
}
int main() {
    unsigned* d; unsigned h[256];
    if (hipMalloc(&d, sizeof(h)) != hipSuccess) return 2;
    hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, d);
    if (hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost) != hipSuccess) return 2;
    int bad = 0;
    for (unsigned l = 0; l < 64; ++l) {
        const unsigned row = l >> 4;
        // permlane16: a's odd rows <- b's even rows (row - 1), b's even rows <- a's odd rows (row + 1)
        const unsigned a16 = (row & 1) ? 100 + l - 16 : l, b16 = (row & 1) ? 100 + l : l + 16;
        const unsigned a32 = l >= 32 ? 100 + l - 32 : l, b32 = l < 32 ? l + 32 : 100 + l;
        if (h[l] != a16 || h[64 + l] != b16 || h[128 + l] != a32 || h[192 + l] != b32) {
            if (bad++ < 4) printf("lane %u: p16 %u %u (want %u %u) p32 %u %u (want %u %u)\n", l, h[l], h[64 + l], a16, b16,
                                  h[128 + l], h[192 + l], a32, b32);
        }
    }
    printf(bad ? "permlane semantics MISMATCH (%d lanes)\n" : "permlane semantics OK\n", bad);
    return bad ? 1 : 0;
}
