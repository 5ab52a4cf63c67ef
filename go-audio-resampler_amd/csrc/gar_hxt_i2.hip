// gar_hxt_i2.hip -- explicit hxt_kernel instantiations (parallel build unit 2)
#include "gar_hxt.hpp"

namespace gar {
GAR_HXT_FOR_B(GAR_HXT_INST)
}  // namespace gar
