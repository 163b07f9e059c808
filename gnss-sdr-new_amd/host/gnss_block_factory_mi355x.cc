#include "gnss_block_factory_mi355x.h"

#include "beidou_b1i_pcps_acquisition_mi355x.h"
#include "galileo_e1_pcps_ambiguous_acquisition_mi355x.h"
#include "gnss_tracking_mi355x.h"
#include "gps_l1_ca_pcps_acquisition_mi355x.h"
#include "gsdr.h"

namespace gsdr_factory
{
int device_for_channel(const ConfigurationInterface* configuration, const std::string& role, int channel)
{
    const int pinned = configuration->property(role + ".device", -1);
    if (pinned >= 0) return pinned;
    int visible = 0;
    if (gsdr_device_count(&visible) != GSDR_OK || visible < 1) visible = 1;
    int g = configuration->property("GNSS-SDR.mi355x_devices", visible);
    if (g < 1 || g > visible) g = visible;
    return (channel < 0 ? 0 : channel) % g;
}

std::unique_ptr<AcquisitionInterface> GetAcqBlock(const ConfigurationInterface* configuration, const std::string& role,
    unsigned int in_streams, unsigned int out_streams, int channel)
{
    const std::string implementation = configuration->property(role + ".implementation", std::string("Wrong"));
    const int device = device_for_channel(configuration, role, channel);
    if (implementation == "GPS_L1_CA_PCPS_Acquisition_MI355X")
        return std::make_unique<GpsL1CaPcpsAcquisitionMI355X>(configuration, role, in_streams, out_streams, device);
    if (implementation == "Galileo_E1_PCPS_Ambiguous_Acquisition_MI355X")
        return std::make_unique<GalileoE1PcpsAmbiguousAcquisitionMI355X>(configuration, role, in_streams, out_streams,
            device);
    if (implementation == "BEIDOU_B1I_PCPS_Acquisition_MI355X")
        return std::make_unique<BeidouB1iPcpsAcquisitionMI355X>(configuration, role, in_streams, out_streams, device);
    return nullptr;
}

std::unique_ptr<TrackingInterface> GetTrkBlock(const ConfigurationInterface* configuration, const std::string& role,
    unsigned int in_streams, unsigned int out_streams, int channel)
{
    const std::string implementation = configuration->property(role + ".implementation", std::string("Wrong"));
    const int device = device_for_channel(configuration, role, channel);
    if (implementation == "GPS_L1_CA_DLL_PLL_Tracking_MI355X")
        return std::make_unique<GpsL1CaDllPllTrackingMI355X>(configuration, role, in_streams, out_streams, device);
    if (implementation == "Galileo_E1_DLL_PLL_VEML_Tracking_MI355X")
        return std::make_unique<GalileoE1DllPllVemlTrackingMI355X>(configuration, role, in_streams, out_streams, device);
    if (implementation == "BEIDOU_B1I_DLL_PLL_Tracking_MI355X")
        return std::make_unique<BeidouB1iDllPllTrackingMI355X>(configuration, role, in_streams, out_streams, device);
    return nullptr;
}
}  // namespace gsdr_factory
