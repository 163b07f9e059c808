// Shared body of the PCPS acquisition adapters on the MI355X engine.  The
// reference repeats the same AcquisitionInterface plumbing in every adapter
// (gps_l1_ca_pcps_acquisition.cc:93-250, galileo_e1_pcps_ambiguous_acquisition.cc:
// 111-260, beidou_b1i_pcps_acquisition.cc:95-220): setters forwarded to the
// pcps_acquisition block, reset = set_active(true), stop = set_active(false).
// Each signal's adapter supplies its Acq_Conf chip rate / code period and its
// sampled replica (set_local_code).
#ifndef GSDR_HOST_PCPS_ACQUISITION_ADAPTER_H
#define GSDR_HOST_PCPS_ACQUISITION_ADAPTER_H

#include <complex>
#include <memory>
#include <string>
#include <vector>

#include "acq_conf.h"
#include "acquisition_interface.h"
#include "configuration.h"
#include "pcps_acquisition_mi355x.h"

class PcpsAcquisitionAdapterMI355X : public AcquisitionInterface
{
public:
    ~PcpsAcquisitionAdapterMI355X() override = default;

    std::string role() override { return role_; }
    size_t item_size() override { return acq_parameters_.it_size; }

    void set_gnss_synchro(Gnss_Synchro* gnss_synchro) override;
    void set_channel(unsigned int channel) override;
    void set_channel_fsm(std::weak_ptr<ChannelFsm> channel_fsm) override;
    void set_threshold(float threshold) override;
    void set_doppler_max(unsigned int doppler_max) override;
    void set_doppler_step(unsigned int doppler_step) override;
    void set_doppler_center(int doppler_center) override;
    void init() override;
    void set_state(int state) override;
    signed int mag() override;
    void reset() override;
    void stop_acquisition() override;
    void set_resampler_latency(uint32_t latency_samples) override;

    // the gr::block the reference connects into the flowgraph (get_left_block)
    pcps_acquisition_mi355x* get_block() { return acquisition_.get(); }
    const Acq_Conf& conf() const { return acq_parameters_; }

protected:
    // Acq_Conf::SetFromConfiguration with the signal's constants, the block, and
    // the code / vector lengths of the reference adapters:
    //   code_length_   = floor(resampled_fs / (chip_rate / code_length_chips))
    //   vector_length_ = floor(sampled_ms * samples_per_ms) * (bit_transition ? 2 : 1)
    PcpsAcquisitionAdapterMI355X(const ConfigurationInterface* configuration, const std::string& role,
        uint32_t ms_per_code, double chip_rate, double code_length_chips, double opt_freq, int device);
    // one code period (code_length_ samples) repeated over the block, then the
    // block's set_local_code (FFT + conjugate on the device)
    void load_code(const std::vector<std::complex<float>>& one_period, unsigned int repeats);
    // the sampling rate the replica is generated at (use_acquisition_resampler)
    int32_t replica_fs() const;

    const ConfigurationInterface* configuration_;
    Acq_Conf acq_parameters_;
    std::unique_ptr<pcps_acquisition_mi355x> acquisition_;
    std::vector<std::complex<float>> code_;
    Gnss_Synchro* gnss_synchro_{nullptr};
    std::weak_ptr<ChannelFsm> channel_fsm_;
    std::string role_;
    float threshold_{0.0};
    unsigned int doppler_max_{0};
    unsigned int doppler_step_{0};
    int doppler_center_{0};
    unsigned int channel_{0};
    unsigned int code_length_{0};
    unsigned int vector_length_{0};
    unsigned int sampled_ms_{1};
};

#endif
