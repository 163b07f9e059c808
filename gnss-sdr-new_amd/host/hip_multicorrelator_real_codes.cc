#include "hip_multicorrelator_real_codes.h"

#include <algorithm>
#include <iostream>

namespace
{
bool report(int rc, const char* what)
{
    if (rc == GSDR_OK) return true;
    // the reference logs and keeps running (SURVEY §8b error conventions)
    std::cerr << what << ": " << gsdr_last_error() << '\n';
    return false;
}
}  // namespace

Hip_Multicorrelator_Real_Codes::~Hip_Multicorrelator_Real_Codes() { free(); }

bool Hip_Multicorrelator_Real_Codes::init(int max_signal_length_samples, int n_correlators)
{
    free();
    d_n_correlators = n_correlators;
    d_max_len = max_signal_length_samples;
    return report(gsdr_corr_create(d_device, 1, max_signal_length_samples, n_correlators, &d_engine),
        "Hip_Multicorrelator_Real_Codes::init");
}

bool Hip_Multicorrelator_Real_Codes::push_code()
{
    if (!d_engine || !d_local_code_in || !d_shifts_chips) return false;
    if (d_pushed_code == d_local_code_in && d_pushed_hd == d_use_high_dynamics_resampler &&
        d_pushed_shifts.size() == static_cast<size_t>(d_n_correlators) &&
        std::equal(d_pushed_shifts.begin(), d_pushed_shifts.end(), d_shifts_chips))
        return true;
    d_pushed_code = d_local_code_in;
    d_pushed_hd = d_use_high_dynamics_resampler;
    d_pushed_shifts.assign(d_shifts_chips, d_shifts_chips + d_n_correlators);
    if (!report(gsdr_corr_set_local_code_and_taps(d_engine, 0, d_code_length_chips, d_local_code_in, d_shifts_chips,
                    d_n_correlators),
            "Hip_Multicorrelator_Real_Codes::set_local_code_and_taps"))
        return false;
    return report(gsdr_corr_set_high_dynamics_resampler(d_engine, 0, d_use_high_dynamics_resampler ? 1 : 0),
        "Hip_Multicorrelator_Real_Codes::set_high_dynamics_resampler");
}

// The reference stores the caller's pointers (cpu_multicorrelator_real_codes.cc:53-63);
// here the replica and shifts are uploaded, and re-uploaded before every correlation
// so a caller that edits them in place (narrow correlator after bit sync,
// dll_pll_veml_tracking.cc:1963-1977) sees the same behaviour.
bool Hip_Multicorrelator_Real_Codes::set_local_code_and_taps(int code_length_chips, const float* local_code_in,
    float* shifts_chips)
{
    d_local_code_in = local_code_in;
    d_shifts_chips = shifts_chips;
    d_code_length_chips = code_length_chips;
    d_pushed_code = nullptr;  // new replica: force the upload
    return push_code();
}

bool Hip_Multicorrelator_Real_Codes::set_input_output_vectors(std::complex<float>* corr_out,
    const std::complex<float>* sig_in)
{
    d_sig_in = sig_in;
    d_corr_out = corr_out;
    return true;
}

void Hip_Multicorrelator_Real_Codes::update_local_code(int, float, float, float) {}

bool Hip_Multicorrelator_Real_Codes::Carrier_wipeoff_multicorrelator_resampler(float rem_carrier_phase_in_rad,
    float phase_step_rad, float phase_rate_step_rad, float rem_code_phase_chips, float code_phase_step_chips,
    float code_phase_rate_step_chips, int signal_length_samples)
{
    if (!d_engine || !d_sig_in || !d_corr_out || !push_code()) return false;
    return report(gsdr_corr_run(d_engine, 0, d_sig_in, GSDR_ITEM_GR_COMPLEX, rem_carrier_phase_in_rad,
                      phase_step_rad, phase_rate_step_rad, rem_code_phase_chips, code_phase_step_chips,
                      code_phase_rate_step_chips, signal_length_samples, reinterpret_cast<float*>(d_corr_out)),
        "Hip_Multicorrelator_Real_Codes::Carrier_wipeoff_multicorrelator_resampler");
}

// 6-argument form (cpu_multicorrelator_real_codes.cc:129-144): the resampler honours
// the high-dynamics flag, the rotator has no phase rate.
bool Hip_Multicorrelator_Real_Codes::Carrier_wipeoff_multicorrelator_resampler(float rem_carrier_phase_in_rad,
    float phase_step_rad, float rem_code_phase_chips, float code_phase_step_chips, float code_phase_rate_step_chips,
    int signal_length_samples)
{
    return Carrier_wipeoff_multicorrelator_resampler(rem_carrier_phase_in_rad, phase_step_rad, 0.0F,
        rem_code_phase_chips, code_phase_step_chips, code_phase_rate_step_chips, signal_length_samples);
}

bool Hip_Multicorrelator_Real_Codes::free()
{
    gsdr_corr_destroy(d_engine);
    d_engine = nullptr;
    return true;
}

void Hip_Multicorrelator_Real_Codes::set_high_dynamics_resampler(bool use_high_dynamics_resampler)
{
    d_use_high_dynamics_resampler = use_high_dynamics_resampler;
    if (d_engine && d_local_code_in) push_code();
}

Hip_Multicorrelator::~Hip_Multicorrelator() { free(); }

bool Hip_Multicorrelator::init(int max_signal_length_samples, int n_correlators)
{
    free();
    d_n_correlators = n_correlators;
    return report(gsdr_corr_create(d_device, 1, max_signal_length_samples, n_correlators, &d_engine),
        "Hip_Multicorrelator::init");
}

bool Hip_Multicorrelator::set_local_code_and_taps(int code_length_chips, const std::complex<float>* local_code_in,
    float* shifts_chips)
{
    if (!d_engine) return false;
    return report(gsdr_corr_set_local_code_and_taps_complex(d_engine, 0, code_length_chips,
                      reinterpret_cast<const float*>(local_code_in), shifts_chips, d_n_correlators),
        "Hip_Multicorrelator::set_local_code_and_taps");
}

bool Hip_Multicorrelator::set_input_output_vectors(std::complex<float>* corr_out, const std::complex<float>* sig_in)
{
    d_sig_in = sig_in;
    d_corr_out = corr_out;
    return true;
}

bool Hip_Multicorrelator::Carrier_wipeoff_multicorrelator_resampler(float rem_carrier_phase_in_rad,
    float phase_step_rad, float rem_code_phase_chips, float code_phase_step_chips, int signal_length_samples)
{
    if (!d_engine || !d_sig_in || !d_corr_out) return false;
    return report(gsdr_corr_run(d_engine, 0, d_sig_in, GSDR_ITEM_GR_COMPLEX, rem_carrier_phase_in_rad, phase_step_rad,
                      0.0F, rem_code_phase_chips, code_phase_step_chips, 0.0F, signal_length_samples,
                      reinterpret_cast<float*>(d_corr_out)),
        "Hip_Multicorrelator::Carrier_wipeoff_multicorrelator_resampler");
}

bool Hip_Multicorrelator::free()
{
    gsdr_corr_destroy(d_engine);
    d_engine = nullptr;
    return true;
}
