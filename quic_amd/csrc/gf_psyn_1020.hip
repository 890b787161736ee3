// gf_psyn_1020.hip — the gf_psyn_kernel variants of FEC_10_20 (gf_psyn.h).
#include "gf_psyn.h"

namespace qfec {
QP_DEFINE_GO(psyn_go_1020, 10, 20)
}  // namespace qfec
