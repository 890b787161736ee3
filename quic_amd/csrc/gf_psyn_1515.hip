// gf_psyn_1515.hip — the gf_psyn_kernel variants of FEC_15_15 (gf_psyn.h).
#include "gf_psyn.h"

namespace qfec {
QP_DEFINE_GO(psyn_go_1515, 15, 15)
}  // namespace qfec
