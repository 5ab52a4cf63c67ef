// gar_hx_i2.hip -- explicit hx_kernel instantiations (parallel build unit 2)
#include "gar_hx.hpp"

namespace gar {
GAR_HX_INST(6, true, 0)
GAR_HX_INST(6, true, 1)
GAR_HX_INST(6, true, 2)
GAR_HX_INST(6, true, 3)
GAR_HX_INST(7, true, 0)
GAR_HX_INST(7, true, 1)
GAR_HX_INST(7, true, 2)
GAR_HX_INST(7, true, 3)
}  // namespace gar
