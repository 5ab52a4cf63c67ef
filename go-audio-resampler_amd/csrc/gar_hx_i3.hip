// gar_hx_i3.hip -- explicit hx_kernel instantiations (parallel build unit 3)
#include "gar_hx.hpp"

namespace gar {
GAR_HX_INST(8, true, 0)
GAR_HX_INST(8, true, 1)
GAR_HX_INST(8, true, 2)
GAR_HX_INST(8, true, 3)
GAR_HX_INST(2, false, 0)
GAR_HX_INST(4, false, 0)
GAR_HX_INST(6, false, 0)
GAR_HX_INST(8, false, 0)
}  // namespace gar
