// GPS L1 C/A PCPS acquisition adapter on the MI355X engine: the counterpart of
// GpsL1CaPcpsAcquisition (src/algorithms/acquisition/adapters/
// gps_l1_ca_pcps_acquisition.cc:39-250), selected in a .conf with
//   Acquisition_1C.implementation=GPS_L1_CA_PCPS_Acquisition_MI355X
#ifndef GSDR_HOST_GPS_L1_CA_PCPS_ACQUISITION_MI355X_H
#define GSDR_HOST_GPS_L1_CA_PCPS_ACQUISITION_MI355X_H

#include <complex>
#include <memory>
#include <string>
#include <vector>

#include "acq_conf.h"
#include "acquisition_interface.h"
#include "configuration.h"
#include "pcps_acquisition_mi355x.h"

class GpsL1CaPcpsAcquisitionMI355X : public AcquisitionInterface
{
public:
    GpsL1CaPcpsAcquisitionMI355X(const ConfigurationInterface* configuration, const std::string& role,
        unsigned int in_streams, unsigned int out_streams, int device = 0);
    ~GpsL1CaPcpsAcquisitionMI355X() override = default;

    std::string role() override { return role_; }
    std::string implementation() override { return "GPS_L1_CA_PCPS_Acquisition_MI355X"; }
    size_t item_size() override { return acq_parameters_.it_size; }

    void set_gnss_synchro(Gnss_Synchro* gnss_synchro) override;
    void set_channel(unsigned int channel) override;
    void set_threshold(float threshold) override;
    void set_doppler_max(unsigned int doppler_max) override;
    void set_doppler_step(unsigned int doppler_step) override;
    void set_doppler_center(int doppler_center) override;
    void init() override;
    void set_local_code() override;
    void set_state(int state) override;
    signed int mag() override;
    void reset() override;
    void stop_acquisition() override;
    void set_resampler_latency(uint32_t latency_samples) override;

    // the gr::block the reference would connect into the flowgraph
    pcps_acquisition_mi355x* get_block() { return acquisition_.get(); }

private:
    Acq_Conf acq_parameters_;
    std::unique_ptr<pcps_acquisition_mi355x> acquisition_;
    std::vector<std::complex<float>> code_;
    Gnss_Synchro* gnss_synchro_{nullptr};
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
