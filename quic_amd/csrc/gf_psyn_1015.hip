// gf_psyn_1015.hip — the gf_psyn_kernel variants of FEC_10_15 (gf_psyn.h).
#include "gf_psyn.h"

namespace qfec {
QP_DEFINE_GO(psyn_go_1015, 10, 15)
}  // namespace qfec
