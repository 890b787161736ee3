// gf_dcol.hip — launchers of the config D kernels (gf_dcol.h); the kernel instantiations are
// in gf_dcol_<e|d><depth><cache>.hip, one per translation unit.
#include "gf_dcol.h"

namespace qfec {


bool gf_dcol_supported(int k, int m, int bb, const Tune& t) {
    return t.dcol && t.const_enc && k == 128 && m == 16 && bb == 8 * kDcolS;
}

// wg_cu: workgroups of 4 waves a CU holds by registers (2 at <= 256 VGPRs), LDS permitting
static unsigned dcol_grid(long long groups, const Tune& t, size_t lds, int wg_cu) {
    using SH = DcShape<kDcolS>;
    const long long units = groups * SH::NT;
    const long long want = (units + kDcWaves - 1) / kDcWaves;
    const int per_cu = std::max(1, std::min(wg_cu, (int)((160 * 1024) / lds)));
    long long cap = (long long)t.cus * per_cu;
    if (t.dcol_wg > 0)   // oversubscribed: about dcol_wg units per wave
        cap = (units + (long long)kDcWaves * t.dcol_wg - 1) / ((long long)kDcWaves * t.dcol_wg);
    if (t.dcol_grid > 0) cap = t.dcol_grid;          // tests: many units per wave
    return (unsigned)std::min<long long>(want, cap);
}

hipError_t launch_gf_dcol_encode(const uint8_t* in, uint8_t* out, int k, int m, int bb,
                                 long long groups, long long out_gstride, hipStream_t st,
                                 const Tune& t) {
    if (groups <= 0) return hipSuccess;
    if (!gf_dcol_supported(k, m, bb, t)) return hipErrorInvalidValue;
    if (((uintptr_t)in & 15) != 0) return hipErrorInvalidValue;
    using SH = DcShape<kDcolS>;
    const int D = t.dcol_depth;
    if (D != 6 && D != 8) return hipErrorInvalidValue;
    const size_t lds = (size_t)kDcWaves * (D + 1) * SH::BUFB;
    const unsigned grid = dcol_grid(groups, t, lds, 2);
    const long long waves = (long long)grid * kDcWaves;
    if ((groups * SH::NT + waves - 1) / waves >= (1LL << 31)) return hipErrorInvalidValue;
    note_kernel("gf_dcol_kernel<encode,k128m16>");
    note_grid("gf_dcol_kernel<encode>", grid);
    const long long in_bytes = groups * (long long)k * bb;
#define QD_ENC(NAME) return NAME(dim3(grid), lds, st, in, out, nullptr, nullptr, nullptr, nullptr, \
                             groups, 0, in_bytes, 0LL, out_gstride)
    // cached loads and stores: the parity's partial cache lines at tile edges merge in L2
    // instead of going to HBM twice (D encode 20.3 -> 16.5 ms; non-temporal loads too: 21.7
    // ms)
    if (D == 8) QD_ENC(dcol_go_e83);
    QD_ENC(dcol_go_e63);
#undef QD_ENC
    return hipGetLastError();
}

hipError_t launch_gf_dcol_syndrome(const uint8_t* in, uint8_t* out, const uint8_t* tab,
                                   const uint8_t* slots, const int32_t* nout,
                                   const uint8_t* cenc, int k, int m, int bb, long long groups,
                                   int rmax, long long tab_gstride, long long out_gstride,
                                   hipStream_t st, const Tune& t) {
    if (groups <= 0) return hipSuccess;
    if (!gf_dcol_supported(k, m, bb, t) || rmax > 16 || tab_gstride < syn::kBytes)
        return hipErrorInvalidValue;
    if ((((uintptr_t)in) & 15) || ((((uintptr_t)tab) | (uintptr_t)tab_gstride |
                                     (uintptr_t)cenc | (uintptr_t)slots) & 3))
        return hipErrorInvalidValue;
    using SH = DcShape<kDcolS>;
    const int D = t.dcol_depth;
    if (D != 6 && D != 8) return hipErrorInvalidValue;
    const size_t lds = (size_t)kDcWaves * (D + 1) * SH::BUFB;
    const unsigned grid = dcol_grid(groups, t, lds, 2);
    const long long waves = (long long)grid * kDcWaves;
    if ((groups * SH::NT + waves - 1) / waves >= (1LL << 31)) return hipErrorInvalidValue;
    note_kernel("gf_dcol_kernel<decode,k128m16>");
    note_grid("gf_dcol_kernel<decode>", grid);
    // decode: non-temporal loads, plain stores (cached loads: 1.011x instead of 1.167x the
    // algorithmic reads, but 18.3 vs 16.9 ms and the next encode over-reads)
    const long long in_bytes = groups * (long long)k * bb;
#define QD_DEC(NAME) return NAME(dim3(grid), lds, st, in, out, tab, slots, nout, cenc, groups, \
                             rmax, in_bytes, tab_gstride, out_gstride)
    if (D == 8) QD_DEC(dcol_go_d82);
    QD_DEC(dcol_go_d62);
#undef QD_DEC
    return hipGetLastError();
}

}  // namespace qfec

