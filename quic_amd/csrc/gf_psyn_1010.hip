// gf_psyn_1010.hip — the gf_psyn_kernel variants of FEC_10_10 (gf_psyn.h).
#include "gf_psyn.h"

namespace qfec {
QP_DEFINE_GO(psyn_go_1010, 10, 10)
}  // namespace qfec
