// BeiDou B1I PCPS acquisition adapter on the MI355X engine: the counterpart of
// BeidouB1iPcpsAcquisition (src/algorithms/acquisition/adapters/
// beidou_b1i_pcps_acquisition.cc:38-220), selected with
// Acquisition_B1.implementation=BEIDOU_B1I_PCPS_Acquisition_MI355X.
#ifndef GSDR_HOST_BEIDOU_B1I_PCPS_ACQUISITION_MI355X_H
#define GSDR_HOST_BEIDOU_B1I_PCPS_ACQUISITION_MI355X_H

#include "pcps_acquisition_adapter.h"

class BeidouB1iPcpsAcquisitionMI355X : public PcpsAcquisitionAdapterMI355X
{
public:
    BeidouB1iPcpsAcquisitionMI355X(const ConfigurationInterface* configuration, const std::string& role,
        unsigned int in_streams, unsigned int out_streams, int device = 0);
    std::string implementation() override { return "BEIDOU_B1I_PCPS_Acquisition_MI355X"; }
    void init() override;
    void set_local_code() override;
};

#endif
