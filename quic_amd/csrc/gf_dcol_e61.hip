// gf_dcol_e61.hip — gf_dcol_kernel<kDcolS, 6, false, 1> (gf_dcol.h), one instantiation per
// translation unit so the D kernels compile in parallel.
#include "gf_dcol.h"

namespace qfec {
QD_DEFINE_GO(dcol_go_e61, 6, false, 1)
}  // namespace qfec
