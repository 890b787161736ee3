// gf_dcol_h43.hip — gf_dcol_kernel<kDcolS, 4, false, 3, 8> (gf_dcol.h): the encode with 8 rows
// per wave (four waves per SIMD), one instantiation per translation unit.
#include "gf_dcol.h"

namespace qfec {
QD_DEFINE_GO(dcol_go_h43, 4, false, 3, 8)
}  // namespace qfec
