#include "gps_l1_ca_pcps_acquisition_mi355x.h"

#include "gnss_replicas.h"

namespace
{
constexpr double GPS_L1_CA_CODE_RATE_CPS = 1.023e6;  // GPS_L1_CA.h
constexpr double GPS_L1_CA_CODE_LENGTH_CHIPS = 1023.0;
constexpr double GPS_L1_CA_OPT_ACQ_FS_SPS = 2000000.0;
}  // namespace

// gps_l1_ca_pcps_acquisition.cc:39-90 (ms_per_code 1)
GpsL1CaPcpsAcquisitionMI355X::GpsL1CaPcpsAcquisitionMI355X(const ConfigurationInterface* configuration,
    const std::string& role, unsigned int in_streams, unsigned int out_streams, int device)
    : PcpsAcquisitionAdapterMI355X(configuration, role, 1, GPS_L1_CA_CODE_RATE_CPS, GPS_L1_CA_CODE_LENGTH_CHIPS,
          GPS_L1_CA_OPT_ACQ_FS_SPS, device)
{
    (void)in_streams;
    (void)out_streams;
}

// gps_l1_ca_pcps_acquisition.cc:151-170: one code period sampled at fs, repeated
// sampled_ms times.
void GpsL1CaPcpsAcquisitionMI355X::set_local_code()
{
    load_code(gps_l1_ca_code_gen_complex_sampled(gnss_synchro_ ? gnss_synchro_->PRN : 1, replica_fs(), 0), sampled_ms_);
}
