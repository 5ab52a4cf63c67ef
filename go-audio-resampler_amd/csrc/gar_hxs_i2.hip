// gar_hxs_i2.hip -- explicit hxs_kernel instantiations (parallel build unit 2)
#include "gar_hxs.hpp"

namespace gar {
GAR_HXS_FOR_HI(GAR_HXS_INST)
}  // namespace gar
