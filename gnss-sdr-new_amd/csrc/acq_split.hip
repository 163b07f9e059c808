// Split register four-step correlate (acq_correlate_split_kernel, acq_impl.h) for
// the FFT sizes of configs C4 / C5 beyond the LDS engine: plan choice, launch and
// one-time setup, selected by gsdr_acq::split.
#include <cstdlib>
#include "acq_impl.h"

namespace gsdr_acq_impl
{

// Inner M-point register four-step plans (RegFourStep<R, NT, H, WPE, pads, row radices>):
//   25000 = 25 x (10 x 10 x 10): 512 lanes, two columns per lane (50 complex in
//           VGPRs), 5 rows of 1000 per LDS round (40 KB)
//   32000 = 32 x (10 x 10 x 10): 1024 lanes, one column per lane (32 complex),
//           8 rows per LDS round (64 KB)
using Reg25k = RegFourStep<25, 512, 5, 1, NoPads<1000>, 10, 10, 10>;
using Reg25kP = RegFourStep<25, 512, 5, 1, Pads25k, 10, 10, 10>;  // the same with the bank-model pads
using Reg32k = RegFourStep<32, 1024, 8, 1, NoPads<1000>, 10, 10, 10>;
//   16000 = 16 x (10 x 10 x 10): the C3 plan (variant 93's register four-step), 512
//           lanes, two columns per lane, 8 rows per LDS round (64 KB)
using Reg16k = RegFourStep<16, 512, 8, 1, NoPads<1000>, 10, 10, 10>;
// Wave-local rows (H = 0): each LDS round holds one row per wave and every wave
// transforms its row without workgroup barriers.
using Wl25k = RegFourStep<25, 512, 0, 1, NoPads<1000>, 10, 10, 10>;      // rounds 8 + 8 + 8 + 1
using Wl25kW = RegFourStep<25, 1024, 0, 1, NoPads<1000>, 10, 10, 10>;    // one column per lane, rounds 16 + 9
using Wl32k = RegFourStep<32, 1024, 0, 1, NoPads<1000>, 10, 10, 10>;     // rounds 16 + 16 (128 KB)
using Wl32kP = RegFourStep<32, 1024, 0, 1, Pads1000, 10, 10, 10>;        // the same, bank-model pads
using Wl16k = RegFourStep<16, 512, 0, 1, NoPads<1000>, 10, 10, 10>;      // rounds 8 + 8 (64 KB)

// split ids: (N, outer radix ROUT, inner plan)
//   1: 25000 = 1 x 25000 (C5 GPS L1 / BeiDou B1I at 25 Msps, 1 ms)
//   2: 32000 = 1 x 32000 (Galileo E1 at 8 Msps, 4 ms)
//   3: 64000 = 2 x 32000 (C4: Galileo E1 at 8 Msps with bit transition)
//   4: 100000 = 4 x 25000 (C5 Galileo E1 at 25 Msps, 4 ms)
//   7: 25000 (Reg25kP)   8: 100000 = 4 x Reg25kP (padded row layouts)
//   5: 32000 = 2 x 16000
//   6: 64000 = 4 x 16000
// wave-local rows:
//   11: 25000 (Wl25k)   12: 32000 (Wl32k)   13: 64000 = 2 x Wl32k   14: 100000 = 4 x Wl25k
//   15: 32000 = 2 x Wl16k   16: 64000 = 4 x Wl16k   17: 25000 (Wl25kW)   18: 100000 = 4 x Wl25kW
//   19: 32000 (Wl32kP)   20: 64000 = 2 x Wl32kP
// (round 4 measured and removed: 100000 = 2 x 50000 (25 x 2000 register four-step,
// 164 B/lane of spills, -3.5 %), the outer DIF step as its own pass (-11 % / -29 %),
// mirror-pair loads of the Hermitian code spectra (within +-3 %))
namespace
{
struct SplitId
{
    int id;
    uint32_t n;
};
// the first entry of a size is its default (r04a: wave-local rows 12 / 13 for 32000 /
// 64000, +4 % / +10 % over 2 / 3; the 512-lane 25000 plan keeps its LDS rounds)
constexpr SplitId kSplits[] = {{1, 25000}, {12, 32000}, {13, 64000}, {4, 100000}, {2, 32000}, {3, 64000}, {5, 32000},
    {6, 64000}, {11, 25000}, {14, 100000}, {15, 32000}, {16, 64000}, {17, 25000}, {18, 100000}, {19, 32000},
    {20, 64000}, {7, 25000}, {8, 100000}};

// PRN group of an XCD pass: the largest divisor of P whose code rows fit in ~2 MB
// (half an XCD's L2), so the rows of the group's codes stay resident while the X
// rows stream past
uint32_t prn_group(uint32_t P, uint32_t N)
{
    const size_t row = (size_t)N * sizeof(float2);
    // code bytes per group walked by every XCD at once: 2 MB (r04x: 1 MB within
    // noise, 4 MB -7 % at Galileo, 8 MB -10-12 %: the per-XCD L2 sets it)
    constexpr size_t cap = (size_t)2 << 20;
    uint32_t best = 1;
    for (uint32_t g = 1; g <= P; ++g)
        if (P % g == 0 && (size_t)g * row <= cap) best = g;
    return best;
}

// ARG = false: the grid pass (row maxima into d_stats); ARG = true: the selected
// rows' pass (keys into d_keys, |R|^2 rows into rowbuf for the peak ratio; the
// caller zeroes d_keys and runs acq_argmax_split_finish_kernel)
template <int ROUT, class RP, bool HALF, bool ARG = false>
int launch_one(gsdr_acq* a, uint32_t nblocks, hipStream_t s, const gsdr_acq_result* sel = nullptr,
    float* rowbuf = nullptr, float* psum = nullptr, uint32_t* rout = nullptr)
{
    if (rout) *rout = ROUT;
    static_assert(RP::N * ROUT > 0, "plan");
    if (RP::N * ROUT != (int)a->N)
        {
            gsdr::set_error("internal: split plan for N = %d, handle N = %u", RP::N * ROUT, a->N);
            return GSDR_E_STATE;
        }
    if (ROUT > 1 && !ARG)
        GSDR_HIP(hipMemsetAsync(a->d_stats, 0, (size_t)nblocks * a->nprn * a->D * sizeof(RowStat), s));
    const uint32_t grid = ARG ? nblocks * a->nprn * ROUT : nblocks * a->D * a->nprn * ROUT;
    hipLaunchKernelGGL((acq_correlate_split_kernel<ROUT, RP, HALF, ARG>), dim3(grid), dim3(RP::NT), RP::lds_bytes(), s,
        a->d_X, a->d_code_fft, a->d_stats, a->d_tw, a->D, a->nprn, nblocks, prn_group(a->nprn, a->N), a->xm, sel,
        a->d_keys, rowbuf, psum);
    GSDR_HIP(hipGetLastError());
    return GSDR_OK;
}

template <int ROUT, class RP, bool HALF>
int attrs_one()
{
    GSDR_HIP(hipFuncSetAttribute((const void*)acq_correlate_split_kernel<ROUT, RP, HALF>,
        hipFuncAttributeMaxDynamicSharedMemorySize, (int)RP::lds_bytes()));
    GSDR_HIP(hipFuncSetAttribute((const void*)acq_correlate_split_kernel<ROUT, RP, HALF, true>,
        hipFuncAttributeMaxDynamicSharedMemorySize, (int)RP::lds_bytes()));
    return GSDR_OK;
}

// The selected rows' pass on the handle's split plan (ablation ids on their base plan).
int launch_split_arg(gsdr_acq* a, uint32_t nblocks, hipStream_t s, const gsdr_acq_result* sel, float* rowbuf,
    float* psum, uint32_t* rout)
{
    const bool half = a->eff != a->N;
#define GSDR_ARG(RO, RP)                                                                                    \
    return half ? launch_one<RO, RP, true, true>(a, nblocks, s, sel, rowbuf, psum, rout)                    \
                : launch_one<RO, RP, false, true>(a, nblocks, s, sel, rowbuf, psum, rout)
    switch (a->split)
        {
        case 1: GSDR_ARG(1, Reg25k);
        case 2: GSDR_ARG(1, Reg32k);
        case 3: GSDR_ARG(2, Reg32k);
        case 4: GSDR_ARG(4, Reg25k);
        case 7: GSDR_ARG(1, Reg25kP);
        case 8: GSDR_ARG(4, Reg25kP);
        case 5: GSDR_ARG(2, Reg16k);
        case 6: GSDR_ARG(4, Reg16k);
        case 11: GSDR_ARG(1, Wl25k);
        case 12: GSDR_ARG(1, Wl32k);
        case 13: GSDR_ARG(2, Wl32k);
        case 14: GSDR_ARG(4, Wl25k);
        case 15: GSDR_ARG(2, Wl16k);
        case 16: GSDR_ARG(4, Wl16k);
        case 17: GSDR_ARG(1, Wl25kW);
        case 18: GSDR_ARG(4, Wl25kW);
        case 19: GSDR_ARG(1, Wl32kP);
        case 20: GSDR_ARG(2, Wl32kP);
        default: gsdr::set_error("internal: bad split variant %d", a->split); return GSDR_E_STATE;
        }
#undef GSDR_ARG
}
}  // namespace

int launch_split_argmax(gsdr_acq* a, uint32_t nblocks, gsdr_acq_result* res, hipStream_t s)
{
    const bool half = a->eff != a->N;
    const AcqParams ap = params_of(a);
    GSDR_HIP(hipMemsetAsync(a->d_keys, 0, (size_t)nblocks * a->nprn * sizeof(unsigned long long), s));
    float* rowbuf = ap.cfar ? nullptr : a->d_rowbuf;
    // CFAR (not in step two, whose input power is the first step's): the Parseval
    // shares of the opposite row come from the split pass itself
    float* psum = (ap.cfar && !ap.step_two && !half) ? a->d_psum : nullptr;
    uint32_t rout = 1;
    int rc = launch_split_arg(a, nblocks, s, res, rowbuf, psum, &rout);
    if (rc != GSDR_OK) return rc;
    hipLaunchKernelGGL((acq_argmax_split_finish_kernel<1024>), dim3(nblocks * a->nprn), dim3(1024), 0, s, a->d_X,
        a->d_code_fft, res, a->d_keys, rowbuf, psum, rout, ap);
    GSDR_HIP(hipGetLastError());
    return GSDR_OK;
}

int launch_split(gsdr_acq* a, uint32_t nblocks, hipStream_t s)
{
    const bool half = a->eff != a->N;
    switch (a->split)
        {
        case 1: return half ? launch_one<1, Reg25k, true>(a, nblocks, s) : launch_one<1, Reg25k, false>(a, nblocks, s);
        case 2: return half ? launch_one<1, Reg32k, true>(a, nblocks, s) : launch_one<1, Reg32k, false>(a, nblocks, s);
        case 3: return half ? launch_one<2, Reg32k, true>(a, nblocks, s) : launch_one<2, Reg32k, false>(a, nblocks, s);
        case 4: return half ? launch_one<4, Reg25k, true>(a, nblocks, s) : launch_one<4, Reg25k, false>(a, nblocks, s);
        case 7: return half ? launch_one<1, Reg25kP, true>(a, nblocks, s) : launch_one<1, Reg25kP, false>(a, nblocks, s);
        case 8: return half ? launch_one<4, Reg25kP, true>(a, nblocks, s) : launch_one<4, Reg25kP, false>(a, nblocks, s);
        case 5: return half ? launch_one<2, Reg16k, true>(a, nblocks, s) : launch_one<2, Reg16k, false>(a, nblocks, s);
        case 6: return half ? launch_one<4, Reg16k, true>(a, nblocks, s) : launch_one<4, Reg16k, false>(a, nblocks, s);
        case 11: return half ? launch_one<1, Wl25k, true>(a, nblocks, s) : launch_one<1, Wl25k, false>(a, nblocks, s);
        case 12: return half ? launch_one<1, Wl32k, true>(a, nblocks, s) : launch_one<1, Wl32k, false>(a, nblocks, s);
        case 13: return half ? launch_one<2, Wl32k, true>(a, nblocks, s) : launch_one<2, Wl32k, false>(a, nblocks, s);
        case 14: return half ? launch_one<4, Wl25k, true>(a, nblocks, s) : launch_one<4, Wl25k, false>(a, nblocks, s);
        case 15: return half ? launch_one<2, Wl16k, true>(a, nblocks, s) : launch_one<2, Wl16k, false>(a, nblocks, s);
        case 16: return half ? launch_one<4, Wl16k, true>(a, nblocks, s) : launch_one<4, Wl16k, false>(a, nblocks, s);
        case 17: return half ? launch_one<1, Wl25kW, true>(a, nblocks, s) : launch_one<1, Wl25kW, false>(a, nblocks, s);
        case 18: return half ? launch_one<4, Wl25kW, true>(a, nblocks, s) : launch_one<4, Wl25kW, false>(a, nblocks, s);
        case 19: return half ? launch_one<1, Wl32kP, true>(a, nblocks, s) : launch_one<1, Wl32kP, false>(a, nblocks, s);
        case 20: return half ? launch_one<2, Wl32kP, true>(a, nblocks, s) : launch_one<2, Wl32kP, false>(a, nblocks, s);
        default: gsdr::set_error("internal: bad split variant %d", a->split); return GSDR_E_STATE;
        }
}

// Select the split correlate for a single-dwell four-step handle (K = 1, with or
// without bit transition).  Default: 25000 / 32000 (ROUT = 1), 64000 = 2 x 32000
// (C4 bit transition: 52 -> 61 Msps, profiles/r03q) and 100000 = 4 x 25000.  The last
// was slower than the packed four-step (87 vs 100 Msps: every sub-transform re-reads
// the whole X and code rows) until the forward-spectrum reuse (XMap) left one X row
// per block in L2: 116 vs 107 Msps (profiles/r04h).  The wave-local 100000 plans
// (14 / 18) and the 16000-based splits 5 / 6 / 15 / 16 run with GSDR_ACQ_SPLIT=2 /
// GSDR_ACQ_SPLIT_ID; GSDR_ACQ_SPLIT=0 keeps the packed four-step everywhere.
int setup_split(gsdr_acq* a)
{
    a->split = 0;
    if (a->K != 1) return GSDR_OK;  // non-coherent dwells: the accumulating general path
    int mode = 1;
    if (const char* e = std::getenv("GSDR_ACQ_SPLIT")) mode = std::atoi(e);
    if (mode == 0) return GSDR_OK;
    for (const SplitId& sp : kSplits)
        if (sp.n == a->N && !a->split) a->split = sp.id;
    if ((a->split == 14 || a->split == 18) && mode < 2) a->split = 0;
    // experiments: GSDR_ACQ_SPLIT_ID forces a split of the handle's N
    if (const char* e = std::getenv("GSDR_ACQ_SPLIT_ID"))
        {
            const int want = std::atoi(e);
            for (const SplitId& sp : kSplits)
                if (sp.id == want && sp.n == a->N) a->split = want;
        }
    if (!a->split) return GSDR_OK;
    int rc = GSDR_OK;
    switch (a->split)
        {
        case 1: rc = attrs_one<1, Reg25k, true>() | attrs_one<1, Reg25k, false>(); break;
        case 2: rc = attrs_one<1, Reg32k, true>() | attrs_one<1, Reg32k, false>(); break;
        case 3: rc = attrs_one<2, Reg32k, true>() | attrs_one<2, Reg32k, false>(); break;
        case 4: rc = attrs_one<4, Reg25k, true>() | attrs_one<4, Reg25k, false>(); break;
        case 7: rc = attrs_one<1, Reg25kP, true>() | attrs_one<1, Reg25kP, false>(); break;
        case 8: rc = attrs_one<4, Reg25kP, true>() | attrs_one<4, Reg25kP, false>(); break;
        case 5: rc = attrs_one<2, Reg16k, true>() | attrs_one<2, Reg16k, false>(); break;
        case 6: rc = attrs_one<4, Reg16k, true>() | attrs_one<4, Reg16k, false>(); break;
        case 11: rc = attrs_one<1, Wl25k, true>() | attrs_one<1, Wl25k, false>(); break;
        case 12: rc = attrs_one<1, Wl32k, true>() | attrs_one<1, Wl32k, false>(); break;
        case 13: rc = attrs_one<2, Wl32k, true>() | attrs_one<2, Wl32k, false>(); break;
        case 14: rc = attrs_one<4, Wl25k, true>() | attrs_one<4, Wl25k, false>(); break;
        case 15: rc = attrs_one<2, Wl16k, true>() | attrs_one<2, Wl16k, false>(); break;
        case 16: rc = attrs_one<4, Wl16k, true>() | attrs_one<4, Wl16k, false>(); break;
        case 17: rc = attrs_one<1, Wl25kW, true>() | attrs_one<1, Wl25kW, false>(); break;
        case 18: rc = attrs_one<4, Wl25kW, true>() | attrs_one<4, Wl25kW, false>(); break;
        case 19: rc = attrs_one<1, Wl32kP, true>() | attrs_one<1, Wl32kP, false>(); break;
        case 20: rc = attrs_one<2, Wl32kP, true>() | attrs_one<2, Wl32kP, false>(); break;
        default: break;
        }
    if (rc != GSDR_OK) a->split = 0;
    return rc;
}

}  // namespace gsdr_acq_impl
