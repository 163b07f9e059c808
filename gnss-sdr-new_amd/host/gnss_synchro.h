// Gnss_Synchro mirror: the acquisition/tracking exchange record of GNSS-SDR
// (src/core/system_parameters/gnss_synchro.h:36-90), restricted to the fields the
// acquisition and tracking hot path reads or writes.  Same names and types so
// adapter code reads like the reference's.
#ifndef GSDR_HOST_GNSS_SYNCHRO_H
#define GSDR_HOST_GNSS_SYNCHRO_H

#include <cstdint>

class Gnss_Synchro
{
public:
    char System{};
    char Signal[3]{};
    uint32_t PRN{};
    int32_t Channel_ID{};

    double Acq_delay_samples{};
    double Acq_doppler_hz{};
    uint64_t Acq_samplestamp_samples{};
    uint32_t Acq_doppler_step{};

    int64_t fs{};
    double Prompt_I{};
    double Prompt_Q{};
    double CN0_dB_hz{};
    double Carrier_Doppler_hz{};
    double Carrier_phase_rads{};
    double Code_phase_samples{};
    uint64_t Tracking_sample_counter{};
    int32_t correlation_length_ms{};
    double EVM{};  // the fork's error-vector-magnitude lock indicator (gnss_synchro.h:84)

    bool Flag_valid_acquisition{};
    bool Flag_valid_symbol_output{};
    bool Flag_valid_word{};
    bool Flag_valid_pseudorange{};
    bool Flag_PLL_180_deg_phase_locked{};
};

#endif
