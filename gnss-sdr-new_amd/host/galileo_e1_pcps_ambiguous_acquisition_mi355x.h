// Galileo E1 PCPS (ambiguous) acquisition adapter on the MI355X engine: the
// counterpart of GalileoE1PcpsAmbiguousAcquisition
// (src/algorithms/acquisition/adapters/galileo_e1_pcps_ambiguous_acquisition.cc:37-260),
// selected with Acquisition_1B.implementation=Galileo_E1_PCPS_Ambiguous_Acquisition_MI355X.
// 4 ms primary code period (ms_per_code 4), sinBOC(1,1) or CBOC replica.
#ifndef GSDR_HOST_GALILEO_E1_PCPS_AMBIGUOUS_ACQUISITION_MI355X_H
#define GSDR_HOST_GALILEO_E1_PCPS_AMBIGUOUS_ACQUISITION_MI355X_H

#include "pcps_acquisition_adapter.h"

class GalileoE1PcpsAmbiguousAcquisitionMI355X : public PcpsAcquisitionAdapterMI355X
{
public:
    GalileoE1PcpsAmbiguousAcquisitionMI355X(const ConfigurationInterface* configuration, const std::string& role,
        unsigned int in_streams, unsigned int out_streams, int device = 0);
    std::string implementation() override { return "Galileo_E1_PCPS_Ambiguous_Acquisition_MI355X"; }
    void set_local_code() override;

private:
    bool acquire_pilot_{false};
};

#endif
