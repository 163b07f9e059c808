// Packed-f32 correlate-kernel variants for N = 4000 (the C2 bench configuration):
// launch and one-time setup, selected by gsdr_acq::corr_variant.
#include <cstdlib>
#include "acq_impl.h"

namespace gsdr_acq_impl
{

// The variant whose correlate kernel is not acq_correlate_pk_kernel (its forward
// and argmax passes use the variant's PkPlan): 93 = N 16000 on the register
// four-step 16 x (10 x 10 x 10), 512 lanes, 8 rows per LDS round, each XCD's
// rows walked in groups of 16 PRNs.
using RegPlan93 = RegFourStep<16, 512, 8, 1 | (16 << 4), NoPads<1000>, 10, 10, 10>;
// 94: 93 with wave-local rows (two rounds of 8 rows, one per wave, no barriers
// inside a row transform)
using RegPlan94 = RegFourStep<16, 512, 0, 1 | (16 << 4), NoPads<1000>, 10, 10, 10>;

template <class RP>
int launch_reg(gsdr_acq* a, uint32_t nblocks, hipStream_t s)
{
    hipLaunchKernelGGL((acq_correlate_reg_kernel<RP>), dim3(nblocks * a->D * a->nprn), dim3(RP::NT), RP::lds_bytes(),
        s, a->d_X, a->d_code_fft, a->d_stats, a->d_tw, a->D, a->nprn, nblocks, a->xm);
    return GSDR_OK;
}

template <class RP>
int setup_reg()
{
    GSDR_HIP(hipFuncSetAttribute((const void*)acq_correlate_reg_kernel<RP>, hipFuncAttributeMaxDynamicSharedMemorySize,
        (int)RP::lds_bytes()));
    return GSDR_OK;
}

int launch_corr_variant(gsdr_acq* a, uint32_t nblocks, hipStream_t s)
{
    switch (a->corr_variant)
        {
        case 93: return launch_reg<RegPlan93>(a, nblocks, s);
        case 94: return launch_reg<RegPlan94>(a, nblocks, s);
        default: break;
        }
#define GSDR_PK_CASE(ID, MP, PG, WPE, ST)                                                                       \
    case ID:                                                                                                    \
        {                                                                                                       \
            using M = GSDR_UNPAREN MP;                                                                          \
            const uint32_t groups = (a->nprn + pg_count(PG) - 1) / pg_count(PG);                                                  \
            if (ST == 3)                                                                                        \
                GSDR_HIP(hipMemsetAsync(a->d_stats, 0, (size_t)nblocks * a->nprn * a->D * sizeof(RowStat), s)); \
            hipLaunchKernelGGL((acq_correlate_pk_kernel<M, PG, WPE, ST>), dim3(nblocks * a->D * groups),         \
                dim3(M::NT), a->corr_lds_bytes, s, a->d_X, a->d_code_fft, a->d_stats, a->d_tw, a->D, a->nprn,   \
                nblocks, a->xm);                                                                                \
            return GSDR_OK;                                                                                     \
        }
#define GSDR_UNPAREN(...) __VA_ARGS__
    switch (a->corr_variant)
        {
            GSDR_PK_VARIANTS(GSDR_PK_CASE)
        default: gsdr::set_error("internal: bad correlate variant %d", a->corr_variant); return GSDR_E_STATE;
        }
#undef GSDR_PK_CASE
#undef GSDR_UNPAREN
}

// The STAT-1 variants' first-maximum pass over the selected rows.
int launch_argmax_variant(gsdr_acq* a, uint32_t nblocks, gsdr_acq_result* res, hipStream_t s)
{
#define GSDR_PKA_CASE(ID, MP, PG, WPE, ST)                                                                      \
    case ID:                                                                                                    \
        {                                                                                                       \
            using M = GSDR_UNPAREN MP;                                                                          \
            hipLaunchKernelGGL((acq_argmax_pk_kernel<M, ST>), dim3(nblocks * a->nprn), dim3(M::NT),             \
                a->corr_lds_bytes, s, a->d_X, a->d_code_fft, res, a->d_tw, a->D, a->nprn,                       \
                a->conf.samples_per_code, params_of(a));                                                        \
            GSDR_HIP(hipGetLastError());                                                                        \
            return GSDR_OK;                                                                                     \
        }
#define GSDR_UNPAREN(...) __VA_ARGS__
    switch (a->corr_variant)
        {
            GSDR_PK_VARIANTS(GSDR_PKA_CASE)
        default: gsdr::set_error("internal: bad argmax variant %d", a->corr_variant); return GSDR_E_STATE;
        }
#undef GSDR_PKA_CASE
#undef GSDR_UNPAREN
}

// Forward spectra on the packed plan of the selected variant.
int launch_forward_pk(gsdr_acq* a, const void* iq, int item_type, uint32_t nblocks, uint64_t stride, hipStream_t s)
{
#define GSDR_PKF_CASE(ID, MP, PG, WPE, ST)                                                                          \
    case ID:                                                                                                    \
        {                                                                                                       \
            using M = GSDR_UNPAREN MP;                                                                          \
            if (item_type == GSDR_ITEM_GR_COMPLEX)                                                              \
                hipLaunchKernelGGL((acq_forward_pk_kernel<M, GSDR_ITEM_GR_COMPLEX>), dim3(nblocks, a->xm.q),       \
                    dim3(M::NT), M::lds_bytes(), s, iq, stride, a->d_wipe, a->d_X, a->d_tw, a->consumed, a->xm); \
            else if (item_type == GSDR_ITEM_CSHORT)                                                             \
                hipLaunchKernelGGL((acq_forward_pk_kernel<M, GSDR_ITEM_CSHORT>), dim3(nblocks, a->xm.q),           \
                    dim3(M::NT), M::lds_bytes(), s, iq, stride, a->d_wipe, a->d_X, a->d_tw, a->consumed, a->xm); \
            else                                                                                                \
                hipLaunchKernelGGL((acq_forward_pk_kernel<M, GSDR_ITEM_IBYTE>), dim3(nblocks, a->xm.q),            \
                    dim3(M::NT), M::lds_bytes(), s, iq, stride, a->d_wipe, a->d_X, a->d_tw, a->consumed, a->xm); \
            GSDR_HIP(hipGetLastError());                                                                        \
            return GSDR_OK;                                                                                     \
        }
#define GSDR_UNPAREN(...) __VA_ARGS__
    switch (a->corr_variant)
        {
            GSDR_PK_VARIANTS(GSDR_PKF_CASE)
        default: gsdr::set_error("internal: bad forward variant %d", a->corr_variant); return GSDR_E_STATE;
        }
#undef GSDR_PKF_CASE
#undef GSDR_UNPAREN
}

// Select and configure a correlate variant (N must be 4000).
int setup_corr_variant(gsdr_acq* a, int v)
{

#define GSDR_PK_SETUP(ID, MP, PG, WPE, ST)                                                                      \
    case ID:                                                                                                    \
        {                                                                                                       \
            using M = GSDR_UNPAREN MP;                                                                          \
            a->corr_lds_bytes = M::lds_bytes() + (size_t)2 * (M::NT / 64) * sizeof(RowStat);                   \
            GSDR_HIP(hipFuncSetAttribute((const void*)acq_correlate_pk_kernel<M, PG, WPE, ST>,                  \
                hipFuncAttributeMaxDynamicSharedMemorySize, (int)a->corr_lds_bytes));                           \
            GSDR_HIP(hipFuncSetAttribute((const void*)acq_argmax_pk_kernel<M, ST>,                              \
                hipFuncAttributeMaxDynamicSharedMemorySize, (int)a->corr_lds_bytes));                           \
            if (M::N != (int)a->N)                                                                              \
                {                                                                                               \
                    gsdr::set_error("correlate variant %d is for N = %d, not %u", ID, M::N, a->N);            \
                    return GSDR_E_UNSUPPORTED;                                                                  \
                }                                                                                               \
            GSDR_HIP(hipFuncSetAttribute((const void*)acq_forward_pk_kernel<M, GSDR_ITEM_GR_COMPLEX>,          \
                hipFuncAttributeMaxDynamicSharedMemorySize, (int)M::lds_bytes()));                              \
            GSDR_HIP(hipFuncSetAttribute((const void*)acq_forward_pk_kernel<M, GSDR_ITEM_CSHORT>,              \
                hipFuncAttributeMaxDynamicSharedMemorySize, (int)M::lds_bytes()));                              \
            GSDR_HIP(hipFuncSetAttribute((const void*)acq_forward_pk_kernel<M, GSDR_ITEM_IBYTE>,               \
                hipFuncAttributeMaxDynamicSharedMemorySize, (int)M::lds_bytes()));                              \
            if (ID == 93 && setup_reg<RegPlan93>() != GSDR_OK) return GSDR_E_DEVICE;                           \
            if (ID == 94 && setup_reg<RegPlan94>() != GSDR_OK) return GSDR_E_DEVICE;                           \
            a->corr_variant = ID;                                                                               \
            a->corr_stat = ST;                                                                                  \
            return GSDR_OK;                                                                                     \
        }
#define GSDR_UNPAREN(...) __VA_ARGS__
    switch (v)
        {
            GSDR_PK_VARIANTS(GSDR_PK_SETUP)
        default: a->corr_variant = 0; return GSDR_OK;
        }
#undef GSDR_PK_SETUP
#undef GSDR_UNPAREN
}

// The plan object a plan type's kernels take (LDS plan or four-step plan).

}  // namespace gsdr_acq_impl
