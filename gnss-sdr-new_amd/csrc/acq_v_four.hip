// Acquisition launch templates instantiated for the four-step FFT (sizes beyond one workgroup's LDS).
#include "acq_impl.h"

namespace gsdr_acq_impl
{

int dispatch_four(gsdr_acq* a, int op, const void* iq, uint32_t nblocks, uint64_t stride, uint64_t stamp0,
    gsdr_acq_result* res, hipStream_t s, uint32_t aux)
{
#define GSDR_CASE(ID, PT)                                                                               \
    case ID:                                                                                            \
        switch (op)                                                                                     \
            {                                                                                           \
            case 0: return launch_all<GSDR_UNPAREN PT>(a, iq, a->conf.item_type, nblocks, stride, stamp0, res, s); \
            case 1: return launch_code_fft<GSDR_UNPAREN PT>(a, aux);                                     \
            case 2: return launch_dump<GSDR_UNPAREN PT>(a, false, 0);                                    \
            case 3: return launch_dump<GSDR_UNPAREN PT>(a, true, aux);                                   \
            case 5: return launch_dwell<GSDR_UNPAREN PT>(a, aux, stamp0, res, s);                         \
            default: return set_lds_attrs<GSDR_UNPAREN PT>(a->lds_bytes);                                \
            }
#define GSDR_UNPAREN(...) __VA_ARGS__
    switch (a->variant)
        {
            GSDR_CASE(20, (FourStepPlan<256>))
            GSDR_CASE(22, (FourStepPlan<1024>))
            GSDR_CASE(24, (gsdr::fft::FourStepPkPlan<8, gsdr::pk::PkPlan<256, 1, 25, 16, 10>>))
            GSDR_CASE(25, (gsdr::fft::FourStepPkPlan<16, gsdr::pk::PkPlan<256, 1, 25, 16, 10>>))
            GSDR_CASE(26, (gsdr::fft::FourStepPkPlan<25, gsdr::pk::PkPlan<256, 1, 25, 16, 10>>))
            GSDR_CASE(27, (gsdr::fft::FourStepPkPlan<5, gsdr::pk::PkPlan<256, 1, 25, 20, 10>>))
        default: gsdr::set_error("internal: bad FFT variant %d", a->variant); return GSDR_E_STATE;
        }
#undef GSDR_CASE
#undef GSDR_UNPAREN
}

}  // namespace gsdr_acq_impl
