// Drop-in for Cpu_Multicorrelator_Real_Codes
// (src/algorithms/tracking/libs/cpu_multicorrelator_real_codes.h:37-61): same
// method set and argument meaning, running the fused MI355X correlator kernel
// through the C ABI (gsdr_corr_*).  One instance = one correlator channel slot.
#ifndef GSDR_HOST_HIP_MULTICORRELATOR_REAL_CODES_H
#define GSDR_HOST_HIP_MULTICORRELATOR_REAL_CODES_H

#include <complex>
#include <vector>

#include "gsdr.h"

class Hip_Multicorrelator_Real_Codes
{
public:
    explicit Hip_Multicorrelator_Real_Codes(int device = 0) : d_device(device) {}
    ~Hip_Multicorrelator_Real_Codes();
    Hip_Multicorrelator_Real_Codes(const Hip_Multicorrelator_Real_Codes&) = delete;
    Hip_Multicorrelator_Real_Codes& operator=(const Hip_Multicorrelator_Real_Codes&) = delete;

    void set_high_dynamics_resampler(bool use_high_dynamics_resampler);
    bool init(int max_signal_length_samples, int n_correlators);
    bool set_local_code_and_taps(int code_length_chips, const float* local_code_in, float* shifts_chips);
    bool set_input_output_vectors(std::complex<float>* corr_out, const std::complex<float>* sig_in);
    // The fused kernel never materialises the K resampled replicas; this keeps the
    // NCO parameters for the next correlation (reference: writes K x N floats).
    void update_local_code(int correlator_length_samples, float rem_code_phase_chips, float code_phase_step_chips,
        float code_phase_rate_step_chips = 0.0);
    bool Carrier_wipeoff_multicorrelator_resampler(float rem_carrier_phase_in_rad, float phase_step_rad,
        float phase_rate_step_rad, float rem_code_phase_chips, float code_phase_step_chips,
        float code_phase_rate_step_chips, int signal_length_samples);
    bool Carrier_wipeoff_multicorrelator_resampler(float rem_carrier_phase_in_rad, float phase_step_rad,
        float rem_code_phase_chips, float code_phase_step_chips, float code_phase_rate_step_chips,
        int signal_length_samples);
    bool free();

private:
    bool push_code();
    int d_device;
    gsdr_corr* d_engine{nullptr};
    const std::complex<float>* d_sig_in{nullptr};
    const float* d_local_code_in{nullptr};
    std::complex<float>* d_corr_out{nullptr};
    float* d_shifts_chips{nullptr};
    int d_code_length_chips{0};
    int d_n_correlators{0};
    int d_max_len{0};
    bool d_use_high_dynamics_resampler{true};  // reference default (cpu_multicorrelator_real_codes.h:60)
    bool d_pushed_hd{false};
    std::vector<float> d_pushed_shifts;  // last uploaded taps
    const float* d_pushed_code{nullptr};
};

// Drop-in for Cpu_Multicorrelator (complex replicas, cpu_multicorrelator.h:37-58).
class Hip_Multicorrelator
{
public:
    explicit Hip_Multicorrelator(int device = 0) : d_device(device) {}
    ~Hip_Multicorrelator();
    Hip_Multicorrelator(const Hip_Multicorrelator&) = delete;
    Hip_Multicorrelator& operator=(const Hip_Multicorrelator&) = delete;

    bool init(int max_signal_length_samples, int n_correlators);
    bool set_local_code_and_taps(int code_length_chips, const std::complex<float>* local_code_in, float* shifts_chips);
    bool set_input_output_vectors(std::complex<float>* corr_out, const std::complex<float>* sig_in);
    bool Carrier_wipeoff_multicorrelator_resampler(float rem_carrier_phase_in_rad, float phase_step_rad,
        float rem_code_phase_chips, float code_phase_step_chips, int signal_length_samples);
    bool free();

private:
    int d_device;
    gsdr_corr* d_engine{nullptr};
    const std::complex<float>* d_sig_in{nullptr};
    std::complex<float>* d_corr_out{nullptr};
    int d_n_correlators{0};
};

#endif
