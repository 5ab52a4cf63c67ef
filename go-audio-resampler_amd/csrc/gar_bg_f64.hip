// gar_bg_f64.hip -- bg_kernel instantiations (double, NS in 8..48).
#include "gar_bg.hpp"

namespace gar {
hipError_t bgLaunchF64(int NS, const BgDev& p, const SrcDesc& src, const OutDesc& od, const BgGrid& g, int threads,
                 size_t lds, int64_t blocks, hipStream_t st, bool globalB) {
    switch (NS) {
        case 8: return bgDispatch<double, 8>(p, src, od, g, threads, lds, blocks, st, globalB); case 12: return bgDispatch<double, 12>(p, src, od, g, threads, lds, blocks, st, globalB); case 16: return bgDispatch<double, 16>(p, src, od, g, threads, lds, blocks, st, globalB); case 20: return bgDispatch<double, 20>(p, src, od, g, threads, lds, blocks, st, globalB); case 24: return bgDispatch<double, 24>(p, src, od, g, threads, lds, blocks, st, globalB); case 28: return bgDispatch<double, 28>(p, src, od, g, threads, lds, blocks, st, globalB); case 32: return bgDispatch<double, 32>(p, src, od, g, threads, lds, blocks, st, globalB); case 36: return bgDispatch<double, 36>(p, src, od, g, threads, lds, blocks, st, globalB); case 40: return bgDispatch<double, 40>(p, src, od, g, threads, lds, blocks, st, globalB); case 44: return bgDispatch<double, 44>(p, src, od, g, threads, lds, blocks, st, globalB); case 48: return bgDispatch<double, 48>(p, src, od, g, threads, lds, blocks, st, globalB);
        default: return hipErrorInvalidValue;
    }
}
}  // namespace gar
