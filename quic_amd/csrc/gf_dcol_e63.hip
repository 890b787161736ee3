// gf_dcol_e63.hip — gf_dcol_kernel<kDcolS, 6, false, 3> (gf_dcol.h), one instantiation per
// translation unit so the D kernels compile in parallel.
#include "gf_dcol.h"

namespace qfec {
QD_DEFINE_GO(dcol_go_e63, 6, false, 3)
}  // namespace qfec
