// GPS L1 C/A PCPS acquisition adapter on the MI355X engine: the counterpart of
// GpsL1CaPcpsAcquisition (src/algorithms/acquisition/adapters/
// gps_l1_ca_pcps_acquisition.cc:39-250), selected in a .conf with
//   Acquisition_1C.implementation=GPS_L1_CA_PCPS_Acquisition_MI355X
#ifndef GSDR_HOST_GPS_L1_CA_PCPS_ACQUISITION_MI355X_H
#define GSDR_HOST_GPS_L1_CA_PCPS_ACQUISITION_MI355X_H

#include "pcps_acquisition_adapter.h"

class GpsL1CaPcpsAcquisitionMI355X : public PcpsAcquisitionAdapterMI355X
{
public:
    GpsL1CaPcpsAcquisitionMI355X(const ConfigurationInterface* configuration, const std::string& role,
        unsigned int in_streams, unsigned int out_streams, int device = 0);
    std::string implementation() override { return "GPS_L1_CA_PCPS_Acquisition_MI355X"; }
    void set_local_code() override;
};

#endif
