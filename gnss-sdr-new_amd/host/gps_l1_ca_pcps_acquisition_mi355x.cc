#include "gps_l1_ca_pcps_acquisition_mi355x.h"

#include <algorithm>
#include <cmath>

#include "gnss_replicas.h"

namespace
{
constexpr double GPS_L1_CA_CODE_RATE_CPS = 1.023e6;    // GPS_L1_CA.h
constexpr double GPS_L1_CA_CODE_LENGTH_CHIPS = 1023.0;
constexpr double GPS_L1_CA_OPT_ACQ_FS_SPS = 2000000.0;
}  // namespace

// gps_l1_ca_pcps_acquisition.cc:39-90
GpsL1CaPcpsAcquisitionMI355X::GpsL1CaPcpsAcquisitionMI355X(const ConfigurationInterface* configuration,
    const std::string& role, unsigned int in_streams, unsigned int out_streams, int device)
    : role_(role)
{
    (void)in_streams;
    (void)out_streams;
    acq_parameters_.ms_per_code = 1;
    acq_parameters_.SetFromConfiguration(configuration, role, GPS_L1_CA_CODE_RATE_CPS, GPS_L1_CA_OPT_ACQ_FS_SPS);
    doppler_max_ = static_cast<unsigned int>(acq_parameters_.doppler_max);
    doppler_step_ = static_cast<unsigned int>(acq_parameters_.doppler_step);
    code_length_ = static_cast<unsigned int>(std::floor(static_cast<double>(acq_parameters_.resampled_fs) /
                                                        (GPS_L1_CA_CODE_RATE_CPS / GPS_L1_CA_CODE_LENGTH_CHIPS)));
    vector_length_ = static_cast<unsigned int>(std::floor(acq_parameters_.sampled_ms * acq_parameters_.samples_per_ms) *
                                               (acq_parameters_.bit_transition_flag ? 2.0 : 1.0));
    code_.resize(vector_length_);
    sampled_ms_ = acq_parameters_.sampled_ms;
    acquisition_ = std::make_unique<pcps_acquisition_mi355x>(acq_parameters_, device);
}

void GpsL1CaPcpsAcquisitionMI355X::stop_acquisition() { acquisition_->set_active(false); }

void GpsL1CaPcpsAcquisitionMI355X::set_threshold(float threshold)
{
    threshold_ = threshold;
    acquisition_->set_threshold(threshold_);
}

void GpsL1CaPcpsAcquisitionMI355X::set_doppler_max(unsigned int doppler_max)
{
    doppler_max_ = doppler_max;
    acquisition_->set_doppler_max(doppler_max_);
}

void GpsL1CaPcpsAcquisitionMI355X::set_doppler_step(unsigned int doppler_step)
{
    doppler_step_ = doppler_step;
    acquisition_->set_doppler_step(doppler_step_);
}

void GpsL1CaPcpsAcquisitionMI355X::set_doppler_center(int doppler_center)
{
    doppler_center_ = doppler_center;
    acquisition_->set_doppler_center(doppler_center_);
}

void GpsL1CaPcpsAcquisitionMI355X::set_gnss_synchro(Gnss_Synchro* gnss_synchro)
{
    gnss_synchro_ = gnss_synchro;
    acquisition_->set_gnss_synchro(gnss_synchro_);
}

void GpsL1CaPcpsAcquisitionMI355X::set_channel(unsigned int channel)
{
    channel_ = channel;
    acquisition_->set_channel(channel_);
}

signed int GpsL1CaPcpsAcquisitionMI355X::mag() { return static_cast<signed int>(acquisition_->mag()); }

void GpsL1CaPcpsAcquisitionMI355X::init() { acquisition_->init(); }

// gps_l1_ca_pcps_acquisition.cc:151-170: one code period sampled at fs, repeated
// sampled_ms times.
void GpsL1CaPcpsAcquisitionMI355X::set_local_code()
{
    const int32_t fs = static_cast<int32_t>(acq_parameters_.use_automatic_resampler ? acq_parameters_.resampled_fs
                                                                                    : acq_parameters_.fs_in);
    const auto one = gps_l1_ca_code_gen_complex_sampled(gnss_synchro_ ? gnss_synchro_->PRN : 1, fs, 0);
    for (unsigned int i = 0; i < sampled_ms_; i++)
        std::copy_n(one.data(), std::min<size_t>(code_length_, one.size()), code_.data() + i * code_length_);
    acquisition_->set_local_code(code_.data());
}

void GpsL1CaPcpsAcquisitionMI355X::reset() { acquisition_->set_active(true); }

void GpsL1CaPcpsAcquisitionMI355X::set_state(int state) { acquisition_->set_state(state); }

void GpsL1CaPcpsAcquisitionMI355X::set_resampler_latency(uint32_t latency_samples)
{
    acquisition_->set_resampler_latency(latency_samples);
}
