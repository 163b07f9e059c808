#include "gnss_tracking_mi355x.h"

#include <cmath>
#include <iostream>

namespace
{
constexpr double GPS_L1_CA_CODE_RATE_CPS = 1.023e6;  // GPS_L1_CA.h
constexpr double GPS_L1_CA_CODE_LENGTH_CHIPS = 1023.0;
constexpr double GALILEO_E1_CODE_CHIP_RATE_CPS = 1.023e6;  // Galileo_E1.h
constexpr double GALILEO_E1_B_CODE_LENGTH_CHIPS = 4092.0;
constexpr double BEIDOU_B1I_CODE_RATE_CPS = 2.046e6;  // Beidou_B1I.h
constexpr double BEIDOU_B1I_CODE_LENGTH_CHIPS = 2046.0;
}  // namespace

void DllPllTrackingAdapterMI355X::make_block(const ConfigurationInterface* configuration, int32_t signal, int device)
{
    item_size_ = trk_params_.item_type == "cshort" ? 4 : (trk_params_.item_type == "cbyte" ? 2 : 8);
    // pooled by default: every channel of the signal on this GPU in one engine
    // handle over the device ring, one launch per <role>.mi355x_pool_batch
    // correlation lengths for all its channels, instead of a per-channel block's
    // synchronous H2D + launch + D2H per general_work call
    pooled_ = configuration->property(role_ + ".mi355x_pool", true);
    if (!pooled_)
        {
            std::cerr << role_ << ": " << implementation_
                      << " built per channel (" << role_ << ".mi355x_pool=false): one synchronous device round trip "
                      << "per general_work call, about 10x the pooled block's cost\n";
            tracking_ = std::make_unique<dll_pll_veml_tracking_mi355x>(trk_params_, signal, device);
            return;
        }
    // the role's suffix names the signal's channel count key (Tracking_1C -> Channels_1C.count)
    const std::string sig = role_.size() >= 2 ? role_.substr(role_.size() - 2) : std::string("1C");
    const int count = configuration->property("Channels_" + sig + ".count", 32);
    const int slots = configuration->property(role_ + ".mi355x_pool_channels", count > 0 ? count : 32);
    const int window = configuration->property(role_ + ".mi355x_pool_window",
        static_cast<int>(SharedTrackingPool::kDefaultWindowCalls));
    const int batch = configuration->property(role_ + ".mi355x_pool_batch",
        static_cast<int>(SharedTrackingPool::kDefaultBatchCalls));
    // the input stream's shared device ring: roles naming the same ring read the same
    // conditioner output (a multi-constellation receiver on one front end names one
    // ring for all its signals, so the stream crosses PCIe once); default: the role's own
    const std::string ring = configuration->property(role_ + ".mi355x_ring", role_);
    tracking_ = std::make_unique<dll_pll_veml_tracking_pool_mi355x>(trk_params_, signal,
        static_cast<uint32_t>(slots > 0 ? slots : 32), device, role_, static_cast<uint32_t>(window),
        static_cast<uint32_t>(batch), ring);
}

// gps_l1_ca_dll_pll_tracking.cc:34-91
GpsL1CaDllPllTrackingMI355X::GpsL1CaDllPllTrackingMI355X(const ConfigurationInterface* configuration,
    const std::string& role, unsigned int in_streams, unsigned int out_streams, int device)
    : DllPllTrackingAdapterMI355X(role, "GPS_L1_CA_DLL_PLL_Tracking_MI355X")
{
    (void)in_streams;
    (void)out_streams;
    trk_params_.SetFromConfiguration(configuration, role);
    trk_params_.vector_length = static_cast<uint32_t>(
        std::round(trk_params_.fs_in / (GPS_L1_CA_CODE_RATE_CPS / GPS_L1_CA_CODE_LENGTH_CHIPS)));
    if (trk_params_.extend_correlation_symbols < 1) trk_params_.extend_correlation_symbols = 1;
    if (trk_params_.extend_correlation_symbols > 20) trk_params_.extend_correlation_symbols = 20;
    // GPS L1 C/A has no pilot: data tracking (:52-57)
    trk_params_.track_pilot = false;
    trk_params_.system = 'G';
    trk_params_.signal[0] = '1';
    trk_params_.signal[1] = 'C';
    make_block(configuration, GSDR_SIGNAL_GPS_1C, device);
}

// galileo_e1_dll_pll_veml_tracking.cc:34-75: extended integration only when
// tracking the pilot
GalileoE1DllPllVemlTrackingMI355X::GalileoE1DllPllVemlTrackingMI355X(const ConfigurationInterface* configuration,
    const std::string& role, unsigned int in_streams, unsigned int out_streams, int device)
    : DllPllTrackingAdapterMI355X(role, "Galileo_E1_DLL_PLL_VEML_Tracking_MI355X")
{
    (void)in_streams;
    (void)out_streams;
    trk_params_.SetFromConfiguration(configuration, role);
    if (trk_params_.extend_correlation_symbols < 1)
        trk_params_.extend_correlation_symbols = 1;
    else if (!trk_params_.track_pilot && trk_params_.extend_correlation_symbols > 1)
        trk_params_.extend_correlation_symbols = 1;
    trk_params_.vector_length = static_cast<uint32_t>(
        std::round(trk_params_.fs_in / (GALILEO_E1_CODE_CHIP_RATE_CPS / GALILEO_E1_B_CODE_LENGTH_CHIPS)));
    trk_params_.system = 'E';
    trk_params_.signal[0] = '1';
    trk_params_.signal[1] = 'B';
    make_block(configuration, GSDR_SIGNAL_GAL_1B, device);
}

// beidou_b1i_dll_pll_tracking.cc:34-90
BeidouB1iDllPllTrackingMI355X::BeidouB1iDllPllTrackingMI355X(const ConfigurationInterface* configuration,
    const std::string& role, unsigned int in_streams, unsigned int out_streams, int device)
    : DllPllTrackingAdapterMI355X(role, "BEIDOU_B1I_DLL_PLL_Tracking_MI355X")
{
    (void)in_streams;
    (void)out_streams;
    trk_params_.SetFromConfiguration(configuration, role);
    trk_params_.vector_length = static_cast<uint32_t>(
        std::round(trk_params_.fs_in / (BEIDOU_B1I_CODE_RATE_CPS / BEIDOU_B1I_CODE_LENGTH_CHIPS)));
    if (trk_params_.extend_correlation_symbols < 1) trk_params_.extend_correlation_symbols = 1;
    if (trk_params_.extend_correlation_symbols > 20) trk_params_.extend_correlation_symbols = 20;
    trk_params_.track_pilot = false;
    trk_params_.system = 'C';
    trk_params_.signal[0] = 'B';
    trk_params_.signal[1] = '1';
    make_block(configuration, GSDR_SIGNAL_BDS_B1, device);
}
