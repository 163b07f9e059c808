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
//   32000 = 32 x (10 x 10 x 10) with wave-local rows (H = 0): 1024 lanes, one column
//           per lane (32 complex), each LDS round holds one row per wave and every
//           wave transforms its row without workgroup barriers; rounds 16 + 16 (128 KB)
using Reg25k = RegFourStep<25, 512, 5, 1, NoPads<1000>, 10, 10, 10>;
using Wl32k = RegFourStep<32, 1024, 0, 1, NoPads<1000>, 10, 10, 10>;
// 25000 = 25 x (10 x 10 x 10) on 1024 lanes, one column per lane, 10 rows per LDS
// round: the plan of the two-sub-transform workgroups (QPW 2) of 100000 = 4 x 25000
using Reg25kW = RegFourStep<25, 1024, 10, 1, NoPads<1000>, 10, 10, 10>;

// split ids: (N, outer radix ROUT, inner plan)
//   1: 25000 = 1 x 25000 (C5 GPS L1 / BeiDou B1I at 25 Msps, 1 ms)
//   4: 100000 = 4 x 25000 (C5 Galileo E1 at 25 Msps, 4 ms), one sub-transform per workgroup
//   24: the same, two sub-transforms (q, q + 2) per 1024-lane workgroup (the default)
//   12: 32000 = 1 x Wl32k (Galileo E1 at 8 Msps, 4 ms)
//   13: 64000 = 2 x Wl32k (C4: Galileo E1 at 8 Msps with bit transition)
// Measured and removed: round 4's 100000 = 2 x 50000 (25 x 2000 register
// four-step, 164 B/lane of spills, -3.5 %), the outer DIF step as its own pass (-11 % /
// -29 %), mirror-pair loads of the Hermitian code spectra (within +-3 %); round 5's
// round 6's 25000 alternatives (profiles/r06j): 10-row LDS rounds on 512 lanes (capped at
// 128 VGPRs, -3-5 %) and one column per lane on 1024 lanes (-22 %); round 5's
// pruning of the alternatives that lost their A/Bs: 32000 / 64000 on 8-row LDS rounds
// (ids 2 / 3, -4 % / -10 %), the 16000-based splits (5 / 6), the wave-local 25000 /
// 100000 plans (11 / 14 / 17 / 18, -25 % / -20 % at 25000), 2 x / 4 x 16000 wave-local
// (15 / 16), the bank-model padded rows (19 / 20 and 7 / 8: conflicts halved, time
// unchanged, profiles/r05p).
namespace
{
struct SplitId
{
    int id;
    uint32_t n;
};
// one plan per size (r04a: wave-local rows 12 / 13 for 32000 / 64000, +4 % / +10 %
// over 8-row LDS rounds; the 512-lane 25000 plan keeps its LDS rounds)
constexpr SplitId kSplits[] = {{1, 25000}, {12, 32000}, {13, 64000}, {4, 100000}};

// PRN group of an XCD pass: the largest divisor of P whose code rows fit in ~2 MB
// (half an XCD's L2), so the rows of the group's codes stay resident while the X
// rows stream past
#ifndef GSDR_ACQ_PPW_DEFAULT
#define GSDR_ACQ_PPW_DEFAULT 1
#endif
#ifndef GSDR_ACQ_QPW_DEFAULT
#define GSDR_ACQ_QPW_DEFAULT 2
#endif

uint32_t prn_group(uint32_t P, uint32_t N)
{
    const size_t row = (size_t)N * sizeof(float2);
    // code bytes per group walked by every XCD at once: 2 MB (r04x: 1 MB within
    // noise, 4 MB -7 % at Galileo, 8 MB -10-12 %: the per-XCD L2 sets it; r06g2 with
    // warm clocks: 0.5 / 1 / 4 MB within noise, 8 MB -15 % at 25000)
    constexpr size_t cap = (size_t)2 << 20;
    uint32_t best = 1;
    for (uint32_t g = 1; g <= P; ++g)
        if (P % g == 0 && (size_t)g * row <= cap) best = g;
    return best;
}

// ARG = false: the grid pass (row maxima into d_stats); ARG = true: the selected
// rows' pass (keys into d_keys, |R|^2 rows into rowbuf for the peak ratio; the
// caller zeroes d_keys and runs acq_argmax_split_finish_kernel)
template <int ROUT, class RP, bool HALF, bool ARG = false, int QPW = 1, int PPW = 1>
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
    constexpr uint32_t RQ = ROUT / QPW;  // workgroups per transform
    if (a->nprn % PPW != 0)
        {
            gsdr::set_error("internal: %d PRNs per workgroup with %u PRNs", PPW, a->nprn);
            return GSDR_E_STATE;
        }
    const uint32_t grid = ARG ? nblocks * a->nprn * RQ : nblocks * a->D * (a->nprn / PPW) * RQ;
    hipLaunchKernelGGL((acq_correlate_split_kernel<ROUT, RP, HALF, ARG, QPW, PPW>), dim3(grid), dim3(RP::NT),
        (split_lds_bytes<ROUT, RP, PPW>()), s,
        a->d_X, a->d_code_fft, a->d_stats, a->d_tw, a->D, a->nprn, nblocks, prn_group(a->nprn / PPW, a->N * PPW), a->xm, sel,
        a->d_keys, rowbuf, psum);
    GSDR_HIP(hipGetLastError());
    return GSDR_OK;
}

template <int ROUT, class RP, bool HALF, int QPW = 1, int PPW = 1>
int attrs_one()
{
    GSDR_HIP(hipFuncSetAttribute((const void*)acq_correlate_split_kernel<ROUT, RP, HALF, false, QPW, PPW>,
        hipFuncAttributeMaxDynamicSharedMemorySize, (int)(split_lds_bytes<ROUT, RP, PPW>())));
    GSDR_HIP(hipFuncSetAttribute((const void*)acq_correlate_split_kernel<ROUT, RP, HALF, true, QPW>,
        hipFuncAttributeMaxDynamicSharedMemorySize, (int)(split_lds_bytes<ROUT, RP>())));
    return GSDR_OK;
}

// The selected rows' pass on the handle's split plan.
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
        case 4: GSDR_ARG(4, Reg25k);
        case 24:
            return half ? launch_one<4, Reg25kW, true, true, 2>(a, nblocks, s, sel, rowbuf, psum, rout)
                        : launch_one<4, Reg25kW, false, true, 2>(a, nblocks, s, sel, rowbuf, psum, rout);
        case 25: GSDR_ARG(1, Reg25kW);
        case 12: GSDR_ARG(1, Wl32k);
        case 13: GSDR_ARG(2, Wl32k);
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
        case 4: return half ? launch_one<4, Reg25k, true>(a, nblocks, s) : launch_one<4, Reg25k, false>(a, nblocks, s);
        case 24:
            return half ? launch_one<4, Reg25kW, true, false, 2>(a, nblocks, s)
                        : launch_one<4, Reg25kW, false, false, 2>(a, nblocks, s);
        case 25:
            // an odd active PRN count: one PRN per workgroup on the same plan
            if (a->nprn % 2)
                return half ? launch_one<1, Reg25kW, true>(a, nblocks, s) : launch_one<1, Reg25kW, false>(a, nblocks, s);
            return half ? launch_one<1, Reg25kW, true, false, 1, 2>(a, nblocks, s)
                        : launch_one<1, Reg25kW, false, false, 1, 2>(a, nblocks, s);
        case 12: return half ? launch_one<1, Wl32k, true>(a, nblocks, s) : launch_one<1, Wl32k, false>(a, nblocks, s);
        case 13: return half ? launch_one<2, Wl32k, true>(a, nblocks, s) : launch_one<2, Wl32k, false>(a, nblocks, s);
        default: gsdr::set_error("internal: bad split variant %d", a->split); return GSDR_E_STATE;
        }
}

// Select the split correlate for a single-dwell four-step handle (K = 1, with or
// without bit transition): 25000 / 32000 (ROUT = 1), 64000 = 2 x 32000 (C4 bit
// transition: 52 -> 61 Msps, profiles/r03q) and 100000 = 4 x 25000.  The last was
// slower than the packed four-step (87 vs 100 Msps: every sub-transform re-reads the
// whole X and code rows) until the forward-spectrum reuse (XMap) left one X row per
// block in L2: 116 vs 107 Msps (profiles/r04h).  GSDR_ACQ_SPLIT=0 keeps the packed
// four-step everywhere (the A/B reference and a second parity path).
int setup_split(gsdr_acq* a)
{
    a->split = 0;
    if (a->K != 1) return GSDR_OK;  // non-coherent dwells: the accumulating general path
    int mode = 1;
    if (const char* e = std::getenv("GSDR_ACQ_SPLIT")) mode = std::atoi(e);
    if (mode == 0) return GSDR_OK;
    for (const SplitId& sp : kSplits)
        if (sp.n == a->N && !a->split) a->split = sp.id;
    // 100000: two sub-transforms per 1024-lane workgroup sharing their products
    // (GSDR_ACQ_QPW=2, the default: half the workgroups, each product formed once for
    // two sub-transforms -- C5 Galileo 133.6 -> 168.0 Msps, profiles/r06f) or one per
    // 512-lane workgroup (1)
    if (a->split == 4)
        {
            int qpw = GSDR_ACQ_QPW_DEFAULT;
            if (const char* e = std::getenv("GSDR_ACQ_QPW")) qpw = std::atoi(e);
            if (qpw == 2) a->split = 24;
        }
    // 25000: two PRNs per 1024-lane workgroup sharing the X row's copies
    // (GSDR_ACQ_PPW=2; a launch with an odd active PRN count runs one per workgroup on
    // the same plan) or one PRN per 512-lane workgroup (1)
    if (a->split == 1)
        {
            int ppw = GSDR_ACQ_PPW_DEFAULT;
            if (const char* e = std::getenv("GSDR_ACQ_PPW")) ppw = std::atoi(e);
            if (ppw == 2) a->split = 25;
        }
    if (!a->split) return GSDR_OK;
    int rc = GSDR_OK;
    switch (a->split)
        {
        case 1: rc = attrs_one<1, Reg25k, true>() | attrs_one<1, Reg25k, false>(); break;
        case 4: rc = attrs_one<4, Reg25k, true>() | attrs_one<4, Reg25k, false>(); break;
        case 24: rc = attrs_one<4, Reg25kW, true, 2>() | attrs_one<4, Reg25kW, false, 2>(); break;
        case 25:
            rc = attrs_one<1, Reg25kW, true, 1, 2>() | attrs_one<1, Reg25kW, false, 1, 2>() | attrs_one<1, Reg25kW, true>() |
                 attrs_one<1, Reg25kW, false>();
            break;
        case 12: rc = attrs_one<1, Wl32k, true>() | attrs_one<1, Wl32k, false>(); break;
        case 13: rc = attrs_one<2, Wl32k, true>() | attrs_one<2, Wl32k, false>(); break;
        default: break;
        }
    if (rc != GSDR_OK) a->split = 0;
    return rc;
}

}  // namespace gsdr_acq_impl
