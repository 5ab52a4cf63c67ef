// gar_bg_f32b.hip -- bg_kernel instantiations (float, NS in 56..96).
#include "gar_bg.hpp"

namespace gar {
hipError_t bgLaunchF32b(int NS, const BgDev& p, const SrcDesc& src, const OutDesc& od, const BgGrid& g, int threads,
                 size_t lds, int64_t blocks, hipStream_t st, bool globalB) {
    switch (NS) {
        case 56: return bgDispatch<float, 56>(p, src, od, g, threads, lds, blocks, st, globalB); case 60: return bgDispatch<float, 60>(p, src, od, g, threads, lds, blocks, st, globalB); case 64: return bgDispatch<float, 64>(p, src, od, g, threads, lds, blocks, st, globalB); case 68: return bgDispatch<float, 68>(p, src, od, g, threads, lds, blocks, st, globalB); case 72: return bgDispatch<float, 72>(p, src, od, g, threads, lds, blocks, st, globalB); case 76: return bgDispatch<float, 76>(p, src, od, g, threads, lds, blocks, st, globalB); case 80: return bgDispatch<float, 80>(p, src, od, g, threads, lds, blocks, st, globalB); case 84: return bgDispatch<float, 84>(p, src, od, g, threads, lds, blocks, st, globalB); case 88: return bgDispatch<float, 88>(p, src, od, g, threads, lds, blocks, st, globalB); case 92: return bgDispatch<float, 92>(p, src, od, g, threads, lds, blocks, st, globalB); case 96: return bgDispatch<float, 96>(p, src, od, g, threads, lds, blocks, st, globalB);
        default: return hipErrorInvalidValue;
    }
}
}  // namespace gar
