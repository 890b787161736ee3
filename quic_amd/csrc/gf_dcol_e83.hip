// gf_dcol_e83.hip — gf_dcol_kernel<kDcolS, 8, false, 3> (gf_dcol.h), one instantiation per
// translation unit so the D kernels compile in parallel.
#include "gf_dcol.h"

namespace qfec {
QD_DEFINE_GO(dcol_go_e83, 8, false, 3)
}  // namespace qfec
