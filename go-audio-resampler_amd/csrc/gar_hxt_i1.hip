// gar_hxt_i1.hip -- explicit hxt_kernel instantiations (parallel build unit 1)
#include "gar_hxt.hpp"

namespace gar {
GAR_HXT_FOR_A(GAR_HXT_INST)
}  // namespace gar
