// Code replica generators used on the acquisition / tracking hot path:
// GPS L1 C/A (src/algorithms/libs/gps_sdr_signal_replica.cc:25-176).
#ifndef GSDR_HOST_GNSS_REPLICAS_H
#define GSDR_HOST_GNSS_REPLICAS_H

#include <complex>
#include <cstdint>
#include <vector>

// +1 / -1 chips of GPS L1 C/A for PRN 1-32 and SBAS 120-138 (empty on a bad PRN).
std::vector<int32_t> gps_l1_ca_code_gen_int(int32_t prn, uint32_t chip_shift = 0);
// float chips, one sample per chip (tracking replica, :104-115)
std::vector<float> gps_l1_ca_code_gen_float(int32_t prn, uint32_t chip_shift = 0);
// (0, +-1) chips (:118-131)
std::vector<std::complex<float>> gps_l1_ca_code_gen_complex(int32_t prn, uint32_t chip_shift = 0);
// sampled at fs with the reference's float index arithmetic (:136-176)
std::vector<std::complex<float>> gps_l1_ca_code_gen_complex_sampled(uint32_t prn, int32_t sampling_freq,
    uint32_t chip_shift = 0);

#endif
