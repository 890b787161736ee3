// gf_dcol_d62.hip — gf_dcol_kernel<kDcolS, 6, true, 2> (gf_dcol.h), one instantiation per
// translation unit so the D kernels compile in parallel.
#include "gf_dcol.h"

namespace qfec {
QD_DEFINE_GO(dcol_go_d62, 6, true, 2)
}  // namespace qfec
