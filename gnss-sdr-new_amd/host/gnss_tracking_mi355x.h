// Tracking adapters on the MI355X engine, the counterparts of
//   GpsL1CaDllPllTracking      (src/algorithms/tracking/adapters/gps_l1_ca_dll_pll_tracking.cc:34-148)
//   GalileoE1DllPllVemlTracking (galileo_e1_dll_pll_veml_tracking.cc:34-130)
//   BeidouB1iDllPllTracking    (beidou_b1i_dll_pll_tracking.cc:34-130)
// selected with Tracking_1C / _1B / _B1 .implementation = GPS_L1_CA_DLL_PLL_Tracking_MI355X,
// Galileo_E1_DLL_PLL_VEML_Tracking_MI355X, BEIDOU_B1I_DLL_PLL_Tracking_MI355X.
// Each builds Dll_Pll_Conf from the role, sets vector_length =
// round(fs_in / (chip rate / code length)) and the signal's extend / pilot rules,
// and owns a tracking block: dll_pll_veml_tracking_mi355x (one engine handle per
// channel), or with <role>.mi355x_pool=true a dll_pll_veml_tracking_pool_mi355x
// slot in the GPU's shared pool of that role (every channel of the signal on the
// GPU in one engine handle over the device IQ ring; <role>.mi355x_pool_channels
// slots, default Channels_<signal>.count; <role>.mi355x_pool_window /
// .mi355x_pool_batch the ring window and the launch batch in vector lengths).
#ifndef GSDR_HOST_GNSS_TRACKING_MI355X_H
#define GSDR_HOST_GNSS_TRACKING_MI355X_H

#include <memory>
#include <string>

#include "configuration.h"
#include "dll_pll_conf.h"
#include "dll_pll_veml_tracking_mi355x.h"
#include "dll_pll_veml_tracking_pool_mi355x.h"
#include "tracking_block_mi355x.h"
#include "tracking_interface.h"

class DllPllTrackingAdapterMI355X : public TrackingInterface
{
public:
    std::string role() override { return role_; }
    std::string implementation() override { return implementation_; }
    size_t item_size() override { return item_size_; }
    void start_tracking() override { tracking_->start_tracking(); }
    void stop_tracking() override { tracking_->stop_tracking(); }
    void set_gnss_synchro(Gnss_Synchro* p_gnss_synchro) override { tracking_->set_gnss_synchro(p_gnss_synchro); }
    void set_channel(unsigned int channel) override
    {
        channel_ = channel;
        tracking_->set_channel(channel);
    }
    // the gr::block the reference connects (get_left_block / get_right_block)
    TrackingBlockMI355X* get_block() { return tracking_.get(); }
    bool pooled() const { return pooled_; }
    const Dll_Pll_Conf& conf() const { return trk_params_; }

protected:
    DllPllTrackingAdapterMI355X(const std::string& role, std::string implementation)
        : role_(role), implementation_(std::move(implementation))
    {
    }
    void make_block(const ConfigurationInterface* configuration, int32_t signal, int device);

    Dll_Pll_Conf trk_params_;
    std::unique_ptr<TrackingBlockMI355X> tracking_;
    bool pooled_{false};
    std::string role_;
    std::string implementation_;
    size_t item_size_{8};
    unsigned int channel_{0};
};

class GpsL1CaDllPllTrackingMI355X : public DllPllTrackingAdapterMI355X
{
public:
    GpsL1CaDllPllTrackingMI355X(const ConfigurationInterface* configuration, const std::string& role,
        unsigned int in_streams, unsigned int out_streams, int device = 0);
};

class GalileoE1DllPllVemlTrackingMI355X : public DllPllTrackingAdapterMI355X
{
public:
    GalileoE1DllPllVemlTrackingMI355X(const ConfigurationInterface* configuration, const std::string& role,
        unsigned int in_streams, unsigned int out_streams, int device = 0);
};

class BeidouB1iDllPllTrackingMI355X : public DllPllTrackingAdapterMI355X
{
public:
    BeidouB1iDllPllTrackingMI355X(const ConfigurationInterface* configuration, const std::string& role,
        unsigned int in_streams, unsigned int out_streams, int device = 0);
};

#endif
