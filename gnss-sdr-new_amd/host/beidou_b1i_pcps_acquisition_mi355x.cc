#include "beidou_b1i_pcps_acquisition_mi355x.h"

#include "gnss_replicas.h"

namespace
{
constexpr double BEIDOU_B1I_CODE_RATE_CPS = 2.046e6;  // Beidou_B1I.h:33-34
constexpr double BEIDOU_B1I_CODE_LENGTH_CHIPS = 2046.0;
constexpr double BEIDOU_B1I_OPT_ACQ_FS_SPS = 10e6;  // beidou_b1i_pcps_acquisition.cc:50
}  // namespace

// beidou_b1i_pcps_acquisition.cc:38-90 (ms_per_code 1).  The reference takes the
// code length from fs_in, not the resampled rate (:63); the two agree unless the
// acquisition resampler is enabled.
BeidouB1iPcpsAcquisitionMI355X::BeidouB1iPcpsAcquisitionMI355X(const ConfigurationInterface* configuration,
    const std::string& role, unsigned int in_streams, unsigned int out_streams, int device)
    : PcpsAcquisitionAdapterMI355X(configuration, role, 1, BEIDOU_B1I_CODE_RATE_CPS, BEIDOU_B1I_CODE_LENGTH_CHIPS,
          BEIDOU_B1I_OPT_ACQ_FS_SPS, device)
{
    (void)in_streams;
    (void)out_streams;
}

// init also loads the replica (:135-139)
void BeidouB1iPcpsAcquisitionMI355X::init()
{
    acquisition_->init();
    set_local_code();
}

// set_local_code (:141-153): sampled at fs_in, repeated sampled_ms times
void BeidouB1iPcpsAcquisitionMI355X::set_local_code()
{
    const uint32_t prn = gnss_synchro_ ? gnss_synchro_->PRN : 1;
    load_code(beidou_b1i_code_gen_complex_sampled(prn, static_cast<int32_t>(acq_parameters_.fs_in), 0), sampled_ms_);
}
