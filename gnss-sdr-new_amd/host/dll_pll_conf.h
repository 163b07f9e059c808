// Dll_Pll_Conf mirror (src/algorithms/tracking/libs/dll_pll_conf.h:30-84,
// dll_pll_conf.cc:20-126): the Tracking_XX.* keys that drive dll_pll_veml_tracking,
// with the reference defaults: cn0_samples, cn0_min, max_lock_fail,
// max_carrier_lock_fail and carrier_lock_th taken from the gflags at construction
// (dll_pll_conf.cc:24-28, gnss_sdr_flags.h), --pll_bw_hz / --dll_bw_hz overriding
// the .conf (:53-63); and the mapping onto the engine's gsdr_trk_conf.
#ifndef GSDR_HOST_DLL_PLL_CONF_H
#define GSDR_HOST_DLL_PLL_CONF_H

#include <cstdint>
#include <string>

#include "configuration.h"
#include "gsdr.h"

class Dll_Pll_Conf
{
public:
    Dll_Pll_Conf();
    // dll_pll_conf.cc:38-126 (an unknown item type falls back to gr_complex with a warning)
    void SetFromConfiguration(const ConfigurationInterface* configuration, const std::string& role);
    // the engine configuration for one pool of max_channels channels of `signal`
    // (GSDR_SIGNAL_*); returns GSDR_E_UNSUPPORTED text in *why for an item type the
    // engine does not read
    gsdr_trk_conf to_engine(int32_t signal, uint32_t max_channels) const;

    std::string item_type{"gr_complex"};
    std::string dump_filename{"./dll_pll_dump.dat"};
    double fs_in{2000000.0};
    double carrier_lock_th{0.7};
    float fll_bw_hz{35.0};
    float pll_bw_hz{35.0};
    float dll_bw_hz{2.0};
    float pll_bw_narrow_hz{5.0};
    float dll_bw_narrow_hz{0.75};
    float early_late_space_chips{0.25};
    float very_early_late_space_chips{0.5};
    float early_late_space_narrow_chips{0.15};
    float very_early_late_space_narrow_chips{0.5};
    float cn0_smoother_alpha{0.002};
    float carrier_lock_test_smoother_alpha{0.002};
    uint32_t pull_in_time_s{10U};
    uint32_t bit_synchronization_time_limit_s{20U};
    uint32_t vector_length{0U};
    uint32_t smoother_length{10U};
    int32_t fll_filter_order{1};
    int32_t pll_filter_order{3};
    int32_t dll_filter_order{2};
    int32_t extend_correlation_symbols{1};
    int32_t cn0_samples{20};
    int32_t cn0_smoother_samples{200};
    int32_t carrier_lock_test_smoother_samples{25};
    int32_t cn0_min{25};
    int32_t max_code_lock_fail{50};
    int32_t max_carrier_lock_fail{5000};
    char signal[3]{};
    char system{'G'};
    bool enable_fll_pull_in{false};
    bool enable_fll_steady_state{false};
    bool track_pilot{true};
    bool carrier_aiding{true};
    bool high_dyn{false};
    bool dump{false};
    bool dump_mat{true};  // read for parity; the .mat conversion is not reproduced (tracking_dump.h)
};

#endif
