// gf_psyn.hip — syndrome decode of the QuicR preset codes at 1350-byte payloads:
// FEC_10_10, FEC_10_15, FEC_10_20, FEC_15_15 (quic_fec_group.cc:22-82), bb = 1352, any
// erasure count up to min(k, m).
//
// The reference decodes in two stages (cauchy_256_decode, cauchy_256.cpp:1269-1420; for
// more than 4 erasures its windowed forms win_original :578-653 and
// win_gaussian_elimination :809-1018): eliminate the received originals from the recovery
// rows, then solve the r x r system over the erased rows.  Here, with y_s the received
// parity rows sorted ascending and e_j the erased data rows ascending:
//   T_y = R_y ^ sum_{present x} C[y][x] D_x          syndromes of ALL m parity rows, with
//                                                    the compile-time coefficients of the
//                                                    preset code (windowed form, one
//                                                    v_bitop3 per (row, sub-row), no
//                                                    scalar dispatch)
//   T_s <- T_{y_s}                                   in place: y_s >= s, ascending
//   Gauss-Jordan on S[s][j] = C[y_s][e_j], replayed on the data in place: for pivot p,
//   T_i ^= g[p][i] * T_p for every slot i (g[p][p] = 1 ^ 1/S'[p][p] normalises the pivot
//   row by linearity), one W/Z expansion of T_p per pivot, r^2 run-time applies per group
//   T_j = E_{e_j}
// For m >= 7 the reference's matrix is C[y][x] = b_x / (b_x + g_y) (cauchy_256.cpp:
// 459-477; row 0, all ones, is g_0 = 0 and b_0 = 1): a column-scaled Cauchy matrix with
// distinct nodes (checked for these codes by tests/test_psyn_prep.py), so every square
// submatrix of it is nonsingular and the elimination needs no pivoting in any row order.
// The recovered bytes are the unique solution, so the result is bit-exact with the
// reference's bit-matrix elimination.  A zero pivot can only come from a malformed receive
// set (a repeated parity row): status -3, group unchanged, as in every other decode here.
//
// Against the run-time decode it replaces (gf_stream_kernel<decode>, k x r run-time applies
// with two scalar nibble dispatches each): (10, 10) at 5 losses goes from 50 run-time
// applies per group to 25, and the other 5 x 10 row contributions are compile-time.
//
// Stream: as gf_bsyn (every wave owns groups g0, g0 + W, ...; a group's k received blocks in
// the prep table's order: present data rows ascending, then the extras in slot order; each
// block's 16-byte aligned envelope DMA'd into a ring of D + 1 block buffers, read at its
// 8-byte skew).  Groups of odd k start 8 bytes off a 16-byte boundary; the block address
// decides the skew.  Loads go through a buffer resource bounded by the end of the input, so
// the envelope of the last block of the buffer reads zeros past it.
//
// vmcnt bookkeeping as in gf_bsyn: a block is NPC DMA instructions; a group's stores
// (8 * SPR per recovered block) sit in the count before the waits for the next group's
// blocks 1 .. D - 1.  tests/test_isa.py checks the compiler adds no VMEM instruction or
// vmcnt wait of its own.
#include "gf_psyn.h"

namespace qfec {

__constant__ GfTables c_gf_psyn = make_gf_tables();   // this code object's copy

// ------------------------------------------------------------------ prep
// 16 lanes per group: the bookkeeping of cauchy_256_decode (sort_blocks :543-575, the erased
// rows ascending, the recovery blocks in array order receive them, the row rewrite :791, the
// status codes :1287-1294), then Gauss-Jordan without pivoting on S[s][j] = C[y_s][e_j]
// (received parity rows ascending), recording per pivot p the coefficient g[p][i] the kernel
// applies to T_p for slot i, and the psyn:: table.  k <= 64, m <= 32, rmax <= 16.
// Lane s holds row s of S in registers (16 bytes); a pivot row reaches the group's lanes by
// four shuffles, and a row update is n GF(256) products through the LDS log / exp tables.
constexpr int kPsynLanes = 16;

__device__ __forceinline__ void psyn_wave_sync() {
    __builtin_amdgcn_wave_barrier();
    asm volatile("" ::: "memory");
}

__device__ __forceinline__ int psyn_byte(const uint32_t (&w)[4], int c) {
    const uint32_t v = c < 4 ? w[0] : c < 8 ? w[1] : c < 12 ? w[2] : w[3];
    return (int)((v >> (8 * (c & 3))) & 0xFFu);
}

__global__ __launch_bounds__(256) void decode_prep_psyn_kernel(
    const uint8_t* __restrict__ rows_in, uint8_t* rows_out, int32_t* __restrict__ status,
    const uint8_t* __restrict__ cenc, uint8_t* __restrict__ tab, uint8_t* __restrict__ slots,
    int32_t* __restrict__ nout, uint8_t* __restrict__ rec_rows, long long groups, int k, int m,
    int bb, int rmax) {
    __shared__ uint8_t gexp[512];
    __shared__ uint8_t glog[256];
    constexpr int GPB = 256 / kPsynLanes;                       // groups per block
    __shared__ uint8_t lrows[GPB][64];
    __shared__ uint8_t llist[GPB][3][16];                       // recpos, y (array order), era
    __shared__ __attribute__((aligned(16))) uint8_t ltab[GPB][psyn::kBytes];
    extern __shared__ __attribute__((aligned(16))) uint8_t lcenc[];   // m x k
    for (int i = threadIdx.x; i < 512; i += blockDim.x) gexp[i] = c_gf_psyn.exp[i];
    for (int i = threadIdx.x; i < 256; i += blockDim.x) glog[i] = c_gf_psyn.log[i];
    for (int i = threadIdx.x; i < m * k; i += blockDim.x) lcenc[i] = cenc[i];
    const long long gfirst = (long long)blockIdx.x * GPB;
    const int ng = (int)min((long long)GPB, groups - gfirst);
    for (int i = threadIdx.x; i < ng * k; i += blockDim.x)
        lrows[i / k][i % k] = rows_in[gfirst * k + i];
    for (int i = threadIdx.x; i < GPB * psyn::kBytes / 4; i += blockDim.x)
        ((uint32_t*)ltab)[i] = 0;
    __syncthreads();
    const int gl = threadIdx.x / kPsynLanes, l = threadIdx.x % kPsynLanes;
    const int seg = (threadIdx.x & 63) / kPsynLanes;            // the group's 16 lanes in the wave
    const int sbase = (threadIdx.x & 63) - l;                   // lane 0 of the group in the wave
    const bool live = gl < ng;
    const long long g = gfirst + gl;
    const uint8_t* rg = lrows[gl];
    uint8_t* lrec = llist[gl][0];
    uint8_t* ly = llist[gl][1];
    uint8_t* lera = llist[gl][2];
    uint8_t* T = ltab[gl];

    // ---- bookkeeping: slot i = 16 q + l.  isrec: slot i holds a recovery block; first: slot
    // i holds the first copy of its data row; present: data row r was received
    uint64_t isrec = 0, isdat = 0, present = 0;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        const int i = kPsynLanes * q + l;
        const int r = (live && i < k) ? rg[i] : 0;
        const bool rec = live && i < k && r >= k;
        const bool dat = live && i < k && r < k;
        if (dat) present |= 1ull << r;
        const uint64_t b1 = __ballot(rec), b2 = __ballot(dat);
        isrec |= ((b1 >> (kPsynLanes * seg)) & 0xFFFFull) << (kPsynLanes * q);
        isdat |= ((b2 >> (kPsynLanes * seg)) & 0xFFFFull) << (kPsynLanes * q);
    }
#pragma unroll
    for (int o = 1; o < kPsynLanes; o <<= 1) present |= __shfl_xor(present, o, kPsynLanes);
    uint64_t first = isdat;
    if (__popcll(isdat) != __popcll(present)) {   // a repeated data row (rare): find firsts
        first = 0;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const int i = kPsynLanes * q + l;
            bool fst = (isdat >> i) & 1;
            if (fst)
                for (int j = 0; j < i; ++j)
                    if (rg[j] == rg[i]) { fst = false; break; }
            first |= ((__ballot(fst) >> (kPsynLanes * seg)) & 0xFFFFull) << (kPsynLanes * q);
        }
    }
    const int nrec = __popcll(isrec);
    const uint64_t kmask = k == 64 ? ~0ull : ((1ull << k) - 1);
    const uint64_t missing = ~present & kmask;
    const int nera = __popcll(missing);
    // entry l of the lists: the l-th recovery slot, its parity row, the l-th erased row
    int myrec = -1, myera = -1;
    {
        uint64_t a = isrec, e = missing;
        for (int j = 0; j < l && a; ++j) a &= a - 1;
        for (int j = 0; j < l && e; ++j) e &= e - 1;
        if (a) myrec = __ffsll((long long)a) - 1;
        if (e) myera = __ffsll((long long)e) - 1;
    }
    const int myy = myrec >= 0 ? rg[myrec] - k : 0;
    const bool badrow = l < nrec && myy >= m;
    const bool anybad = (__ballot(badrow) >> (kPsynLanes * seg)) & 0xFFFFull;
    int early = 1;
    if (nrec == 0) early = 0;                                               // :1287-1289
    else if (k + m > 256 || (bb & 7)) early = -1;                           // :1292-1294
    else if (nrec > rmax || nera < nrec || anybad) early = -3;              // malformed rows
    int n = early == 1 ? nrec : 0;
    if (l < n) {
        lrec[l] = (uint8_t)myrec;
        ly[l] = (uint8_t)myy;
        lera[l] = (uint8_t)myera;
    }
    psyn_wave_sync();
    // ---- row s of S = C[ys_s][e_j] in lane s (s = the rank of y_l: sorted ascending, ties by
    // array order), packed 4 bytes per dword
    int mys = 0;
    for (int j = 0; j < n; ++j) mys += (ly[j] < myy) || (ly[j] == myy && j < l);
    uint32_t row[4] = {0u, 0u, 0u, 0u};
    if (l < n) {
#pragma unroll
        for (int j = 0; j < 16; ++j)   // compile-time indices: row[] stays in registers
            if (j < n) row[j >> 2] |= (uint32_t)lcenc[myy * k + lera[j]] << (8 * (j & 3));
    }
    // lane l ends up holding row s = mys; the shuffles below address rows by s, so the lane
    // holding row s is found through lsrc (lane of row s)
    __shared__ uint8_t lsrc[GPB][16];
    if (l < n) lsrc[gl][mys] = (uint8_t)l;
    psyn_wave_sync();
    const int ok_n = n;
    // ---- Gauss-Jordan without pivoting (every leading minor of a Cauchy submatrix is
    // nonzero); a zero pivot means a repeated parity row: malformed, status -3
    for (int p = 0; p < ok_n; ++p) {
        const int src = sbase + lsrc[gl][p];
        uint32_t prow[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) prow[q] = (uint32_t)__shfl((int)row[q], src, 64);
        const int piv = psyn_byte(prow, p);
        if (piv == 0) {
            early = -3;
            n = 0;
            break;
        }
        const int linv = 255 - glog[piv];                       // log of the inverse pivot
        const int inv = gexp[linv];
        const bool me = mys == p;
        const int f = psyn_byte(row, p);
        // the coefficient the kernel applies to T_p (before this step) for slot mys
        int lg = 0, gco = 0;
        if (me) {
            gco = 1 ^ inv;
            lg = linv;                                          // new row p = inv * row p
        } else if (f) {
            lg = glog[f] + linv;                                // row ^= (f / piv) * row p
            gco = gexp[lg];
        }
        if (lg >= 255) lg -= 255;                               // lg + log(x) < 512: gexp's range
        if (l < ok_n) T[psyn::kCoef + 16 * p + mys] = (uint8_t)gco;
        if (l < ok_n && (me || f)) {
            uint32_t nrow[4] = {0u, 0u, 0u, 0u};
#pragma unroll
            for (int c = 0; c < 16; ++c) {
                if (c < ok_n) {
                    const int pc = psyn_byte(prow, c);
                    const int prod = pc ? gexp[lg + glog[pc]] : 0;
                    nrow[c >> 2] |= (uint32_t)prod << (8 * (c & 3));
                }
            }
#pragma unroll
            for (int q = 0; q < 4; ++q) row[q] = me ? nrow[q] : (row[q] ^ nrow[q]);
        }
    }
    // ---- the table: a changed group streams its present rows ascending, then the extras in
    // slot order; an unchanged one streams its slots in order as no-op extras (row tag 255)
    if (n > 0) {
        const int np = __popcll(present);
        const uint64_t extra = ~first & kmask;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const int i = kPsynLanes * q + l;
            if (i < k) {
                const int r = rg[i];
                if ((first >> i) & 1) {
                    T[psyn::kPerm + __popcll(present & ((1ull << r) - 1))] = (uint8_t)i;
                } else {
                    const int e = __popcll(extra & ((1ull << i) - 1));
                    T[psyn::kPerm + np + e] = (uint8_t)i;
                    T[psyn::kERow + e] = (uint8_t)r;
                }
            }
        }
        if (l == 0) {
            *(uint32_t*)(T + psyn::kMask) = (uint32_t)present;
            *(uint32_t*)(T + psyn::kMask + 4) = (uint32_t)(present >> 32);
        }
        if (l < n) T[psyn::kYs + mys] = (uint8_t)myy;
        // the syndrome rows the solve uses: the kernel accumulates only these
        uint32_t need = l < n ? 1u << myy : 0u;
#pragma unroll
        for (int o = 1; o < kPsynLanes; o <<= 1) need |= (uint32_t)__shfl_xor((int)need, o, kPsynLanes);
        if (l == 0) *(uint32_t*)(T + psyn::kNeed) = need;
    } else {
        for (int i = l; i < k; i += kPsynLanes) {
            T[psyn::kPerm + i] = (uint8_t)i;
            T[psyn::kERow + i] = 255;
        }
        if (l == 0) {                                            // mask: nothing present
            *(uint32_t*)(T + psyn::kMask) = 0u;
            *(uint32_t*)(T + psyn::kMask + 4) = 0u;
        }
    }
    if (live) {
        const uint8_t* rgg = rows_in + g * k;
        uint8_t* ro = rows_out ? rows_out + g * k : nullptr;
        uint8_t* rec = rec_rows ? rec_rows + g * rmax : nullptr;
        if (ro && ro != rgg)
            for (int i = l; i < k; i += kPsynLanes) ro[i] = rg[i];
        psyn_wave_sync();
        if (l < n) {
            slots[g * rmax + l] = lrec[l];
            if (ro) ro[lrec[l]] = lera[l];                                     // :791
        }
        if (rec)
            for (int j = l; j < rmax; j += kPsynLanes) rec[j] = j < n ? lera[j] : 255;
        if (l == 0) {
            nout[g] = n;
            if (status) status[g] = early == 1 ? 0 : early;
        }
    }
    __syncthreads();
    // coalesced copy of the block's tables
    uint32_t* dst = (uint32_t*)(tab + gfirst * (long long)psyn::kBytes);
    const int nd = ng * psyn::kBytes / 4;
    for (int d = threadIdx.x; d < nd; d += blockDim.x) dst[d] = ((const uint32_t*)ltab)[d];
}

// ------------------------------------------------------------------ launchers
// The codes compiled here, at 1352-byte blocks: the QuicR presets with m >= 7 (their matrices
// are column-scaled Cauchy matrices: no pivoting needed) and FEC_5_5, whose 5 x 5 matrix (the
// ones row and CAUCHY_MATRIX_5's rows, cauchy_256.cpp:428-442) has every square submatrix
// nonsingular (checked exhaustively by tests/test_psyn_prep.py), so it needs no pivoting
// either.
bool gf_psyn_supported(int k, int m, int bb, int rmax, const Tune& t) {
    if (!t.psyn || !t.const_enc || bb != 8 * kPsynS || rmax > 16) return false;
    return (k == 10 && (m == 10 || m == 15 || m == 20)) || (k == 15 && m == 15) ||
           (k == 5 && m == 5);
}

hipError_t launch_decode_prep_psyn(const uint8_t* rows_in, uint8_t* rows_out, int32_t* status,
                                   const uint8_t* cenc, uint8_t* tab, uint8_t* slots,
                                   int32_t* nout, uint8_t* rec_rows, int k, int m, int bb,
                                   int rmax, long long groups, hipStream_t st) {
    if (groups <= 0) return hipSuccess;
    if (k > 64 || m > 32 || rmax > 16 || (((uintptr_t)tab) & 3))
        return hipErrorInvalidValue;
    const unsigned nb = (unsigned)((groups + 15) / 16);
    note_kernel("decode_prep_psyn_kernel");
    qlaunch((decode_prep_psyn_kernel), dim3(nb), dim3(256), (uint32_t)(((size_t)m * k + 15) & ~(size_t)15),
            st, rows_in, rows_out, status, cenc, tab, slots, nout, rec_rows, groups, k, m, bb, rmax);
    return hipGetLastError();
}

hipError_t launch_gf_psyn(const uint8_t* in, uint8_t* out, const uint8_t* tab,
                          const uint8_t* cenc, const uint8_t* slots, const int32_t* nout, int k,
                          int m, int bb, long long groups, int rmax, long long out_gstride,
                          hipStream_t st, const Tune& t) {
    if (groups <= 0) return hipSuccess;
    if (!gf_psyn_supported(k, m, bb, rmax, t)) return hipErrorInvalidValue;
    if ((((uintptr_t)in) & 15) || ((((uintptr_t)tab) | (uintptr_t)cenc | (uintptr_t)slots) & 3))
        return hipErrorInvalidValue;
    using SH = PsynShape<kPsynS>;
    PsynLaunch a;
    a.in = in, a.out = out, a.tab = tab, a.cenc = cenc, a.slots = slots, a.nout = nout;
    a.groups = groups, a.rmax = rmax, a.out_gstride = out_gstride, a.st = st, a.t = &t, a.k = k;
    // wide recovered-block stores: measured faster for (10, 10) (0.370-0.382 -> 0.348-0.356
    // ms) and (5, 5) (0.185 -> 0.156 ms); (15, 15) and (10, 20) unchanged, (10, 15) 0.392 ->
    // 0.410; so psyn_wide = 1 (default) takes them for those two and psyn_wide = 2 for every
    // code; out 8-byte aligned
    a.wide = (t.psyn_wide == 2 || (t.psyn_wide == 1 && ((k == 10 && m == 10) || (k == 5 && m == 5)))) &&
             ((((uintptr_t)out) | (uintptr_t)out_gstride) & 7) == 0;
    a.lds = (size_t)kPsynWaves * ((5 + 1) * SH::BUFB + (a.wide ? kPsynStage : 0));   // ring depth 5
    note_kernel("gf_psyn_kernel<decode,preset>");
    switch (k * 256 + m) {
        case 10 * 256 + 10: return psyn_go_1010(a);
        case 10 * 256 + 15: return psyn_go_1015(a);
        case 10 * 256 + 20: return psyn_go_1020(a);
        case 5 * 256 + 5: return psyn_go_55(a);
        default: return psyn_go_1515(a);
    }
}

}  // namespace qfec
