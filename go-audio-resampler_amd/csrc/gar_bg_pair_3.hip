// gar_bg_pair_3.hip -- bg_pair_kernel instantiations (decimator NS 32/36/40 x composite NS 8..40).
#include "gar_bg.hpp"

namespace gar {
template <int NS0, int NS1>
static hipError_t pairLaunch(const BgPair& a, size_t lds, int64_t blocks, int threads, hipStream_t st) {
    if (threads > 64 * kBgRbMaxWaves) return hipErrorInvalidConfiguration;
    if (const size_t lim = setMaxLdsOnce(reinterpret_cast<const void*>(&bg_pair_kernel<NS0, NS1>)); lim < lds)
        return ldsTooBig("bg_pair_kernel", lds, lim);
    hipLaunchKernelGGL((bg_pair_kernel<NS0, NS1>), dim3(static_cast<unsigned>(blocks)), dim3(threads), lds, st, a);
    return hipGetLastError();
}

hipError_t bgPairDispatch3(int NS0, int NS1, const BgPair& a, size_t lds, int64_t blocks, int threads, hipStream_t st) {
#define GAR_PAIR_NS1(N0)                                                      \
    switch (NS1) {                                                            \
        case 8: return pairLaunch<N0, 8>(a, lds, blocks, threads, st);         \
        case 12: return pairLaunch<N0, 12>(a, lds, blocks, threads, st);       \
        case 16: return pairLaunch<N0, 16>(a, lds, blocks, threads, st);       \
        case 20: return pairLaunch<N0, 20>(a, lds, blocks, threads, st);       \
        case 24: return pairLaunch<N0, 24>(a, lds, blocks, threads, st);       \
        case 28: return pairLaunch<N0, 28>(a, lds, blocks, threads, st);       \
        case 32: return pairLaunch<N0, 32>(a, lds, blocks, threads, st);       \
        case 36: return pairLaunch<N0, 36>(a, lds, blocks, threads, st);       \
        case 40: return pairLaunch<N0, 40>(a, lds, blocks, threads, st);       \
        default: return hipErrorNotSupported;                                  \
    }
    switch (NS0) {
        case 32: GAR_PAIR_NS1(32)
        case 36: GAR_PAIR_NS1(36)
        case 40: GAR_PAIR_NS1(40)
        default: return hipErrorNotSupported;
    }
#undef GAR_PAIR_NS1
}
}  // namespace gar
