// gar_hx_i5.hip -- explicit hx_kernel instantiations (parallel build unit 5)
#include "gar_hx.hpp"

namespace gar {
GAR_HX_INST(10, true, 0)
GAR_HX_INST(10, true, 1)
GAR_HX_INST(10, true, 2)
GAR_HX_INST(10, true, 3)
}  // namespace gar
