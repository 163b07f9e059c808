// Code replica generators used on the acquisition / tracking hot path:
// GPS L1 C/A (src/algorithms/libs/gps_sdr_signal_replica.cc:25-176),
// Galileo E1 OS (src/algorithms/libs/galileo_e1_signal_replica.cc:29-233) and
// BeiDou B1I (src/algorithms/libs/beidou_b1i_signal_replica.cc:26-176).
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

// ---- Galileo E1 (E1-B data "1B", E1-C pilot "1C") ----
// The ICD primary memory codes (Galileo OS SIS ICD Annex C, 50 PRNs x 4092 chips)
// are data: the bit-packed table gsdr/data/galileo_e1_codes.bin is assembled into
// the library (galileo_e1_codes.cc).  signal: "1B" or "1C".
// galileo_e1_code_gen_int (:29-58): +1 / -1 chips (hex_to_binary_converter: bit 0 -> +1)
std::vector<int32_t> galileo_e1_code_gen_int(const char* signal, int32_t prn);
// galileo_e1_code_gen_sinboc11_float (:100-111): tracking replica, 2 samples/chip (8184 floats)
std::vector<float> galileo_e1_code_gen_sinboc11_float(const char* signal, uint32_t prn);
// galileo_e1_code_gen_float_sampled (:146-210): sinBOC(1,1) (cboc false) or CBOC(6,1,1/11)
// sampled at fs (resampler of gnss_signal_replica.cc:257-272), optionally with the
// E1-C secondary code (25 primary periods)
std::vector<float> galileo_e1_code_gen_float_sampled(const char* signal, bool cboc, uint32_t prn, int32_t sampling_freq,
    uint32_t chip_shift = 0, bool secondary_flag = false);
// galileo_e1_code_gen_complex_sampled (:213-233): the same as real part, imaginary 0
std::vector<std::complex<float>> galileo_e1_code_gen_complex_sampled(const char* signal, bool cboc, uint32_t prn,
    int32_t sampling_freq, uint32_t chip_shift = 0, bool secondary_flag = false);

// ---- BeiDou B1I ----
// beidou_b1i_code_gen_int (:26-106): +1 / -1 chips of PRN 1-63 (2046 chips; empty on a bad PRN)
std::vector<int32_t> beidou_b1i_code_gen_int(int32_t prn, uint32_t chip_shift = 0);
// beidou_b1i_code_gen_float (:109-120): tracking replica, one sample per chip
std::vector<float> beidou_b1i_code_gen_float(int32_t prn, uint32_t chip_shift = 0);
// beidou_b1i_code_gen_complex_sampled (:137-176): (+-1, 0) sampled at fs
std::vector<std::complex<float>> beidou_b1i_code_gen_complex_sampled(uint32_t prn, int32_t sampling_freq,
    uint32_t chip_shift = 0);

#endif
