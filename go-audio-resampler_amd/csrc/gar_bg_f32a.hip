// gar_bg_f32a.hip -- bg_kernel instantiations (float, NS in 8..52).
#include "gar_bg.hpp"

namespace gar {
hipError_t bgLaunchF32a(int NS, const BgDev& p, const SrcDesc& src, const OutDesc& od, const BgGrid& g, int threads,
                 size_t lds, int64_t blocks, hipStream_t st, bool globalB) {
    switch (NS) {
        case 8: return bgDispatch<float, 8>(p, src, od, g, threads, lds, blocks, st, globalB); case 12: return bgDispatch<float, 12>(p, src, od, g, threads, lds, blocks, st, globalB); case 16: return bgDispatch<float, 16>(p, src, od, g, threads, lds, blocks, st, globalB); case 20: return bgDispatch<float, 20>(p, src, od, g, threads, lds, blocks, st, globalB); case 24: return bgDispatch<float, 24>(p, src, od, g, threads, lds, blocks, st, globalB); case 28: return bgDispatch<float, 28>(p, src, od, g, threads, lds, blocks, st, globalB); case 32: return bgDispatch<float, 32>(p, src, od, g, threads, lds, blocks, st, globalB); case 36: return bgDispatch<float, 36>(p, src, od, g, threads, lds, blocks, st, globalB); case 40: return bgDispatch<float, 40>(p, src, od, g, threads, lds, blocks, st, globalB); case 44: return bgDispatch<float, 44>(p, src, od, g, threads, lds, blocks, st, globalB); case 48: return bgDispatch<float, 48>(p, src, od, g, threads, lds, blocks, st, globalB); case 52: return bgDispatch<float, 52>(p, src, od, g, threads, lds, blocks, st, globalB);
        default: return hipErrorInvalidValue;
    }
}
}  // namespace gar
