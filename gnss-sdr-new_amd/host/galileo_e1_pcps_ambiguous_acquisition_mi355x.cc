#include "galileo_e1_pcps_ambiguous_acquisition_mi355x.h"

#include "gnss_replicas.h"

namespace
{
constexpr double GALILEO_E1_CODE_CHIP_RATE_CPS = 1.023e6;  // Galileo_E1.h
constexpr double GALILEO_E1_B_CODE_LENGTH_CHIPS = 4092.0;
constexpr double GALILEO_E1_OPT_ACQ_FS_SPS = 2000000.0;
}  // namespace

// galileo_e1_pcps_ambiguous_acquisition.cc:37-90
GalileoE1PcpsAmbiguousAcquisitionMI355X::GalileoE1PcpsAmbiguousAcquisitionMI355X(
    const ConfigurationInterface* configuration, const std::string& role, unsigned int in_streams,
    unsigned int out_streams, int device)
    : PcpsAcquisitionAdapterMI355X(configuration, role, 4, GALILEO_E1_CODE_CHIP_RATE_CPS, GALILEO_E1_B_CODE_LENGTH_CHIPS,
          GALILEO_E1_OPT_ACQ_FS_SPS, device)
{
    (void)in_streams;
    (void)out_streams;
    acquire_pilot_ = configuration->property(role + ".acquire_pilot", false);
}

// set_local_code (:150-196): E1-C (acquire_pilot) or the channel's signal; cboc is
// read from "Acquisition<channel>.cboc" as in the reference (:152-153), not from
// the role; one 4 ms period repeated sampled_ms / 4 times.
void GalileoE1PcpsAmbiguousAcquisitionMI355X::set_local_code()
{
    const bool cboc = configuration_->property("Acquisition" + std::to_string(channel_) + ".cboc", false);
    char signal[3] = {'1', 'C', '\0'};
    if (!acquire_pilot_ && gnss_synchro_)
        {
            signal[0] = gnss_synchro_->Signal[0];
            signal[1] = gnss_synchro_->Signal[1];
        }
    else if (!acquire_pilot_)
        signal[1] = 'B';
    const uint32_t prn = gnss_synchro_ ? gnss_synchro_->PRN : 1;
    load_code(galileo_e1_code_gen_complex_sampled(signal, cboc, prn, replica_fs(), 0, false), sampled_ms_ / 4);
}
