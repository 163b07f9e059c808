#include "pcps_acquisition_adapter.h"

#include <algorithm>
#include <cmath>

#include "gnss_sdr_flags.h"

PcpsAcquisitionAdapterMI355X::PcpsAcquisitionAdapterMI355X(const ConfigurationInterface* configuration,
    const std::string& role, uint32_t ms_per_code, double chip_rate, double code_length_chips, double opt_freq, int device)
    : configuration_(configuration), role_(role)
{
    acq_parameters_.ms_per_code = ms_per_code;
    acq_parameters_.SetFromConfiguration(configuration, role, chip_rate, opt_freq);
    // --doppler_max overrides the .conf (gps_l1_ca_pcps_acquisition.cc:57-60 and the
    // Galileo / BeiDou adapters alike)
    if (FLAGS_doppler_max != 0) acq_parameters_.doppler_max = FLAGS_doppler_max;
    doppler_max_ = static_cast<unsigned int>(acq_parameters_.doppler_max);
    doppler_step_ = static_cast<unsigned int>(acq_parameters_.doppler_step);
    code_length_ = static_cast<unsigned int>(
        std::floor(static_cast<double>(acq_parameters_.resampled_fs) / (chip_rate / code_length_chips)));
    vector_length_ = static_cast<unsigned int>(std::floor(acq_parameters_.sampled_ms * acq_parameters_.samples_per_ms) *
                                               (acq_parameters_.bit_transition_flag ? 2.0 : 1.0));
    code_.assign(vector_length_, std::complex<float>(0.0F, 0.0F));
    sampled_ms_ = acq_parameters_.sampled_ms;
    acquisition_ = std::make_unique<pcps_acquisition_mi355x>(acq_parameters_, device);
}

void PcpsAcquisitionAdapterMI355X::stop_acquisition() { acquisition_->set_active(false); }

void PcpsAcquisitionAdapterMI355X::set_threshold(float threshold)
{
    threshold_ = threshold;
    acquisition_->set_threshold(threshold_);
}

void PcpsAcquisitionAdapterMI355X::set_doppler_max(unsigned int doppler_max)
{
    doppler_max_ = doppler_max;
    acquisition_->set_doppler_max(doppler_max_);
}

void PcpsAcquisitionAdapterMI355X::set_doppler_step(unsigned int doppler_step)
{
    doppler_step_ = doppler_step;
    acquisition_->set_doppler_step(doppler_step_);
}

void PcpsAcquisitionAdapterMI355X::set_doppler_center(int doppler_center)
{
    doppler_center_ = doppler_center;
    acquisition_->set_doppler_center(doppler_center_);
}

void PcpsAcquisitionAdapterMI355X::set_gnss_synchro(Gnss_Synchro* gnss_synchro)
{
    gnss_synchro_ = gnss_synchro;
    acquisition_->set_gnss_synchro(gnss_synchro_);
}

void PcpsAcquisitionAdapterMI355X::set_channel(unsigned int channel)
{
    channel_ = channel;
    acquisition_->set_channel(channel_);
}

// set_channel_fsm (gps_l1_ca_pcps_acquisition.h:102-106 and the Galileo / BeiDou
// adapters alike): stored, and forwarded to the block
void PcpsAcquisitionAdapterMI355X::set_channel_fsm(std::weak_ptr<ChannelFsm> channel_fsm)
{
    channel_fsm_ = channel_fsm;
    acquisition_->set_channel_fsm(std::move(channel_fsm));
}

signed int PcpsAcquisitionAdapterMI355X::mag() { return static_cast<signed int>(acquisition_->mag()); }

void PcpsAcquisitionAdapterMI355X::init() { acquisition_->init(); }

void PcpsAcquisitionAdapterMI355X::reset() { acquisition_->set_active(true); }

void PcpsAcquisitionAdapterMI355X::set_state(int state) { acquisition_->set_state(state); }

void PcpsAcquisitionAdapterMI355X::set_resampler_latency(uint32_t latency_samples)
{
    acquisition_->set_resampler_latency(latency_samples);
}

int32_t PcpsAcquisitionAdapterMI355X::replica_fs() const
{
    return static_cast<int32_t>(acq_parameters_.use_automatic_resampler ? acq_parameters_.resampled_fs
                                                                        : acq_parameters_.fs_in);
}

void PcpsAcquisitionAdapterMI355X::load_code(const std::vector<std::complex<float>>& one_period, unsigned int repeats)
{
    std::fill(code_.begin(), code_.end(), std::complex<float>(0.0F, 0.0F));
    const size_t n = std::min<size_t>(code_length_, one_period.size());
    for (unsigned int i = 0; i < repeats && static_cast<size_t>(i + 1) * code_length_ <= code_.size(); i++)
        std::copy_n(one_period.data(), n, code_.data() + static_cast<size_t>(i) * code_length_);
    acquisition_->set_local_code(code_.data());
}
