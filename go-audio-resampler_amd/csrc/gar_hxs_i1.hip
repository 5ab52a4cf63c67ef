// gar_hxs_i1.hip -- explicit hxs_kernel instantiations (parallel build unit 1)
#include "gar_hxs.hpp"

namespace gar {
GAR_HXS_FOR_LO(GAR_HXS_INST)
}  // namespace gar
