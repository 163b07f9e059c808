// Acq_Conf mirror (src/algorithms/acquisition/libs/acq_conf.h:33-82): the
// Acquisition_XX.* keys that drive pcps_acquisition, with the reference's
// defaults and derived parameters.
#ifndef GSDR_HOST_ACQ_CONF_H
#define GSDR_HOST_ACQ_CONF_H

#include <cstddef>
#include <cstdint>
#include <string>

#include "configuration.h"

class Acq_Conf
{
public:
    Acq_Conf() = default;

    // acq_conf.cc:24-90.  Throws std::invalid_argument on an unknown item type,
    // like the reference.
    void SetFromConfiguration(const ConfigurationInterface* configuration, const std::string& role, double chip_rate,
        double opt_freq);

    std::string item_type{"gr_complex"};
    std::string dump_filename;

    int64_t fs_in{4000000LL};
    int64_t resampled_fs{0LL};

    size_t it_size{8};

    float doppler_step{250.0};
    float samples_per_ms{0.0};
    float doppler_step2{125.0};
    float pfa{0.0};
    float pfa2{0.0};
    float samples_per_code{0.0};
    float resampler_ratio{1.0};

    uint32_t sampled_ms{1U};
    uint32_t ms_per_code{1U};
    uint32_t samples_per_chip{2U};
    uint32_t chips_per_second{1023000U};
    uint32_t max_dwells{1U};
    uint32_t num_doppler_bins_step2{4U};
    uint32_t resampler_latency_samples{0U};
    uint32_t dump_channel{0U};
    int32_t doppler_max{5000};
    int32_t doppler_min{-5000};

    bool bit_transition_flag{false};
    bool use_CFAR_algorithm_flag{true};
    bool dump{false};
    bool blocking{true};
    bool blocking_on_standby{false};
    // MI355X extension: the Doppler grid's carrier model (gsdr_acq_set_wipeoff): "exact"
    // (default), "generic" or "avx2" -- the VOLK sincos protokernel replayed bit for bit
    std::string mi355x_carrier{"exact"};
    int wipeoff_mode() const { return mi355x_carrier == "generic" ? 1 : (mi355x_carrier == "avx2" ? 2 : 0); }
    bool make_2_steps{false};
    bool make_repeat_steps{false};
    bool use_automatic_resampler{false};
    bool enable_monitor_output{false};

private:
    void SetDerivedParams();
    void ConfigureAutomaticResampler(double opt_freq);
};

#endif
