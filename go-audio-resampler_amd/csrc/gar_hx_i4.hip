// gar_hx_i4.hip -- explicit hx_kernel instantiations (parallel build unit 4)
#include "gar_hx.hpp"

namespace gar {
GAR_HX_INST(9, true, 0)
GAR_HX_INST(9, true, 1)
GAR_HX_INST(9, true, 2)
GAR_HX_INST(9, true, 3)
}  // namespace gar
