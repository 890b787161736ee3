// gf_psyn_55.hip — the gf_psyn_kernel variants of FEC_5_5 (gf_psyn.h).
#include "gf_psyn.h"

namespace qfec {
QP_DEFINE_GO(psyn_go_55, 5, 5)
}  // namespace qfec
