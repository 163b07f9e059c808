#include "pcps_acquisition_mi355x.h"

#include <cmath>
#include <cstring>
#include <iostream>
#include <stdexcept>

pcps_acquisition_mi355x::pcps_acquisition_mi355x(const Acq_Conf& conf, int device)
    : d_acq_parameters(conf),
      d_device(device),
      d_doppler_step(static_cast<uint32_t>(conf.doppler_step)),
      d_consumed_samples(static_cast<uint32_t>(conf.sampled_ms * conf.samples_per_ms * (conf.bit_transition_flag ? 2.0 : 1.0)))
{
    // item types the block accepts (Acq_Conf item_type_valid: gr_complex, cshort,
    // cbyte); anything else is the reference's std::invalid_argument (acq_conf.cc:28-31)
    d_item_type = engine_item_type(conf.item_type);
    // make_two_steps with non-coherent dwells would need a step-two dwell grid;
    // the engine's narrow grid runs one block per call
    if (conf.make_2_steps && conf.max_dwells > 1 && !conf.bit_transition_flag)
        throw std::invalid_argument("pcps_acquisition_mi355x: make_two_steps with max_dwells > 1 is not supported");
    d_data_buffer.resize(static_cast<size_t>(d_consumed_samples) * conf.it_size);
}

// Acq_Conf::item_type -> engine item type.  cbyte (lv_8sc_t, it_size 2) is what
// the reference adapter turns into gr_complex with complex_byte_to_float_x2 +
// float_to_complex (gps_l1_ca_pcps_acquisition.cc:76-80, :191-196): interleaved
// int8 I/Q at scale 1, GSDR_ITEM_IBYTE converts it exactly in the kernels' loads.
int pcps_acquisition_mi355x::engine_item_type(const std::string& item_type)
{
    if (item_type == "gr_complex") return GSDR_ITEM_GR_COMPLEX;
    if (item_type == "cshort") return GSDR_ITEM_CSHORT;
    if (item_type == "cbyte") return GSDR_ITEM_IBYTE;
    throw std::invalid_argument("Unknown item type: " + item_type);
}

pcps_acquisition_mi355x::~pcps_acquisition_mi355x() { gsdr_acq_destroy(d_engine); }

void pcps_acquisition_mi355x::ensure_engine()
{
    const int32_t dmax = d_acq_parameters.doppler_max;
    if (d_engine && dmax == d_engine_dmax && d_doppler_step == d_engine_step) return;
    gsdr_acq_destroy(d_engine);
    d_engine = nullptr;
    gsdr_acq_conf c{};
    c.fs_in = d_acq_parameters.resampled_fs ? d_acq_parameters.resampled_fs : d_acq_parameters.fs_in;
    c.consumed_samples = d_consumed_samples;
    c.fft_size = 0;
    c.samples_per_code = d_acq_parameters.samples_per_code;
    c.samples_per_chip = d_acq_parameters.samples_per_chip;
    c.doppler_max = dmax;
    c.doppler_step = d_doppler_step;
    c.doppler_center = d_doppler_center;
    c.pfa = d_acq_parameters.use_CFAR_algorithm_flag ? d_acq_parameters.pfa : 0.0F;
    c.max_dwells = d_acq_parameters.max_dwells;
    c.bit_transition_flag = d_acq_parameters.bit_transition_flag ? 1 : 0;
    c.item_type = d_item_type;
    c.max_prns = 1;
    c.max_blocks = 1;
    c.sampled_ms = d_acq_parameters.sampled_ms;
    c.ms_per_code = d_acq_parameters.ms_per_code;
    if (gsdr_acq_create(d_device, &c, &d_engine) != GSDR_OK)
        {
            d_engine = nullptr;
            throw std::runtime_error(std::string("pcps_acquisition_mi355x: ") + gsdr_last_error());
        }
    d_engine_dmax = dmax;
    d_engine_step = d_doppler_step;
    // make_two_steps narrow grid (Acq_Conf second_nbins / second_doppler_step / pfa2)
    if (d_acq_parameters.make_2_steps &&
        gsdr_acq_set_step_two(d_engine, d_acq_parameters.num_doppler_bins_step2, d_acq_parameters.doppler_step2,
            d_acq_parameters.pfa2) != GSDR_OK)
        throw std::runtime_error(std::string("pcps_acquisition_mi355x: ") + gsdr_last_error());
    uint32_t D = 0, N = 0;
    gsdr_acq_get_dims(d_engine, &D, &N);
    d_num_doppler_bins = D;
    if (d_code_set)
        {
            const uint32_t prn = d_gnss_synchro ? d_gnss_synchro->PRN : 0;
            gsdr_acq_set_local_codes(d_engine, reinterpret_cast<const float*>(d_code.data()), &prn, 1);
        }
}

// pcps_acquisition::init (:249-296): reset Gnss_Synchro acquisition fields and
// (re)build the Doppler grid for the current doppler_max / step / center.
void pcps_acquisition_mi355x::init()
{
    std::lock_guard<std::mutex> lk(d_setlock);
    if (d_gnss_synchro)
        {
            d_gnss_synchro->Flag_valid_acquisition = false;
            d_gnss_synchro->Flag_valid_symbol_output = false;
            d_gnss_synchro->Flag_valid_pseudorange = false;
            d_gnss_synchro->Flag_valid_word = false;
            d_gnss_synchro->Acq_doppler_step = 0U;
            d_gnss_synchro->Acq_delay_samples = 0.0;
            d_gnss_synchro->Acq_doppler_hz = 0.0;
            d_gnss_synchro->Acq_samplestamp_samples = 0ULL;
        }
    d_mag = 0.0F;
    d_input_power = 0.0F;
    d_step_repeat = false;  // :262
    ensure_engine();
    gsdr_acq_set_doppler(d_engine, d_acq_parameters.doppler_max, d_doppler_step, d_doppler_center);
}

void pcps_acquisition_mi355x::set_doppler_center(int32_t doppler_center)
{
    std::lock_guard<std::mutex> lk(d_setlock);
    if (doppler_center != d_doppler_center)
        {
            d_doppler_center = doppler_center;
            if (d_engine) gsdr_acq_set_doppler(d_engine, d_acq_parameters.doppler_max, d_doppler_step, d_doppler_center);
        }
}

// set_local_code (:176-209): the GPU places, transforms and conjugates the replica.
void pcps_acquisition_mi355x::set_local_code(std::complex<float>* code)
{
    std::lock_guard<std::mutex> lk(d_setlock);
    d_code.assign(code, code + d_consumed_samples);
    d_code_set = true;
    ensure_engine();
    const uint32_t prn = d_gnss_synchro ? d_gnss_synchro->PRN : 0;
    if (gsdr_acq_set_local_codes(d_engine, reinterpret_cast<const float*>(d_code.data()), &prn, 1) != GSDR_OK)
        std::cerr << "pcps_acquisition_mi355x: set_local_code: " << gsdr_last_error() << '\n';
}

void pcps_acquisition_mi355x::set_active(bool active)
{
    std::lock_guard<std::mutex> lk(d_setlock);
    d_active = active;
}

// set_state (:318-342)
void pcps_acquisition_mi355x::set_state(int32_t state)
{
    std::lock_guard<std::mutex> lk(d_setlock);
    d_state = state;
    if (d_state == 1)
        {
            if (d_gnss_synchro && !d_step_repeat)  // :324
                {
                    d_gnss_synchro->Acq_delay_samples = 0.0;
                    d_gnss_synchro->Acq_doppler_hz = 0.0;
                    d_gnss_synchro->Acq_samplestamp_samples = 0ULL;
                    d_gnss_synchro->Acq_doppler_step = 0U;
                }
            d_mag = 0.0F;
            d_test_statistics = 0.0F;
            d_active = true;
        }
    else if (d_state != 0)
        {
            std::cerr << "State can only be set to 0 or 1\n";
        }
}

bool pcps_acquisition_mi355x::start()
{
    d_sample_counter = 0ULL;
    calculate_threshold();
    return true;
}

// calculate_threshold (:894-909): computed by the engine from pfa, or from pfa2
// and the narrow bin count while d_step_two.
void pcps_acquisition_mi355x::calculate_threshold()
{
    const float pfa = d_step_two ? d_acq_parameters.pfa2 : d_acq_parameters.pfa;
    if (pfa <= 0.0F) return;
    ensure_engine();
    if (d_step_two)
        gsdr_acq_get_step_two_threshold(d_engine, &d_threshold);
    else
        gsdr_acq_get_threshold(d_engine, &d_threshold);
}

// send_positive_acquisition (:344-386) with the fork's repeat steps (:360-368):
// the channel FSM directly when one is set (:370-373), else event 1 (:374-377)
void pcps_acquisition_mi355x::send_positive_acquisition()
{
    if (!d_step_repeat) d_positive_acq = 1;
    if (d_acq_parameters.make_repeat_steps) d_step_repeat = true;
    if (auto fsm = d_channel_fsm.lock())
        fsm->Event_valid_acquisition();
    else if (d_events)
        d_events(1);
}

void pcps_acquisition_mi355x::send_negative_acquisition()
{
    d_positive_acq = 0;
    if (d_events) d_events(2);
}

// acquisition_core (:615-882).  One call integrates the block in d_data_buffer:
// a single-dwell configuration runs the whole grid per call (gsdr_acq_run); with
// max_dwells > 1 the engine keeps the |R|^2 grid of the attempt on the device
// and this call adds its dwell (gsdr_acq_run_dwell, the counter as in :638);
// with bit_transition_flag the engine's N/2-output grid decides every call
// (:831-869); make_two_steps searches the narrow grid (:717-773).
void pcps_acquisition_mi355x::acquisition_core(uint64_t samp_count)
{
    d_mag = 0.0F;
    d_num_noncoherent_integrations_counter++;
    // the engine keeps the first-step threshold (calculate_threshold reads it back
    // after step two); the step-two decision below uses d_threshold
    if (!d_step_two) gsdr_acq_set_threshold(d_engine, d_threshold);
    gsdr_acq_result r{};
    int rc;
    if (d_step_two)
        {
            const uint32_t slot = 0;
            rc = gsdr_acq_run_step_two(d_engine, d_data_buffer.data(), 1, &slot, &d_doppler_center_step_two,
                &d_input_power, samp_count, &r);
        }
    else if (d_acq_parameters.max_dwells > 1 && !d_acq_parameters.bit_transition_flag)
        {
            rc = gsdr_acq_run_dwell(d_engine, d_data_buffer.data(), d_num_noncoherent_integrations_counter - 1U, samp_count,
                &r);
        }
    else
        {
            rc = gsdr_acq_run(d_engine, d_data_buffer.data(), 1, samp_count, &r);
        }
    if (rc != GSDR_OK)
        {
            // device error -> negative acquisition, the reference's failure convention
            std::cerr << "pcps_acquisition_mi355x: " << gsdr_last_error() << '\n';
            d_state = 0;
            d_active = false;
            d_num_noncoherent_integrations_counter = 0;
            send_negative_acquisition();
            return;
        }
    d_mag = r.peak;
    // CFAR input power (:534) -- kept from the coarse step during step two (:531)
    if (!d_step_two) d_input_power = r.input_power;
    d_test_statistics = r.test_statistic;
    // with make_2_steps and repeat steps only the narrow grid updates Gnss_Synchro (:697)
    if (d_gnss_synchro && (d_step_two || !(d_acq_parameters.make_2_steps && d_step_repeat)))
        {
            if (d_acq_parameters.use_automatic_resampler)
                {
                    d_gnss_synchro->Acq_delay_samples = r.acq_delay_samples * d_acq_parameters.resampler_ratio -
                                                        static_cast<double>(d_acq_parameters.resampler_latency_samples);
                    d_gnss_synchro->Acq_samplestamp_samples =
                        static_cast<uint64_t>(std::rint(static_cast<double>(samp_count) * d_acq_parameters.resampler_ratio));
                }
            else
                {
                    d_gnss_synchro->Acq_delay_samples = r.acq_delay_samples;
                    d_gnss_synchro->Acq_samplestamp_samples = samp_count;
                }
            d_gnss_synchro->Acq_doppler_hz = static_cast<double>(r.doppler_hz);
            if (d_step_two) d_gnss_synchro->Acq_doppler_step = static_cast<uint32_t>(d_acq_parameters.doppler_step2);
        }
    if (!d_acq_parameters.bit_transition_flag)
        {
            // decision and dwell FSM (:781-829)
            if (d_test_statistics > d_threshold)
                {
                    d_active = false;
                    if (d_acq_parameters.make_2_steps)
                        {
                            if (d_step_two)
                                {
                                    send_positive_acquisition();
                                    d_step_two = false;
                                    d_state = 0;
                                }
                            else
                                {
                                    // clear the buffer and search the narrow grid on the next block
                                    d_step_two = true;
                                    d_num_noncoherent_integrations_counter = 0;
                                    d_positive_acq = 0;
                                    d_state = 0;
                                }
                            calculate_threshold();
                        }
                    else
                        {
                            send_positive_acquisition();
                            d_state = 0;
                        }
                }
            else
                {
                    d_buffer_count = 0;
                    d_state = 1;
                }
            if (d_num_noncoherent_integrations_counter == d_acq_parameters.max_dwells)
                {
                    if (d_state != 0) send_negative_acquisition();
                    d_state = 0;
                    d_active = false;
                    const bool was_step_two = d_step_two;
                    d_step_two = false;
                    if (was_step_two) calculate_threshold();
                }
        }
    else
        {
            // bit transition: every call decides on its own (:831-869)
            d_active = false;
            if (d_test_statistics > d_threshold)
                {
                    if (d_acq_parameters.make_2_steps)
                        {
                            if (d_step_two)
                                {
                                    send_positive_acquisition();
                                    d_step_two = false;
                                    d_state = 0;
                                }
                            else
                                {
                                    d_step_two = true;
                                    d_num_noncoherent_integrations_counter = 0U;
                                    d_state = 0;
                                }
                            calculate_threshold();
                        }
                    else
                        {
                            send_positive_acquisition();
                            d_state = 0;
                        }
                }
            else
                {
                    d_state = 0;
                    const bool was_step_two = d_step_two;
                    d_step_two = false;
                    if (was_step_two) calculate_threshold();
                    send_negative_acquisition();
                }
        }
    if (d_num_noncoherent_integrations_counter == d_acq_parameters.max_dwells || d_positive_acq == 1 ||
        d_acq_parameters.bit_transition_flag)
        {
            d_num_noncoherent_integrations_counter = 0U;
            d_positive_acq = 0;
        }
}

// general_work (:912-1050) with blocking acquisition.
int pcps_acquisition_mi355x::work(const void* in, int ninput_items)
{
    std::unique_lock<std::mutex> lk(d_setlock);
    if (!d_active)
        {
            int consumed = 0;
            if (!d_acq_parameters.blocking_on_standby)
                {
                    d_sample_counter += static_cast<uint64_t>(ninput_items);
                    consumed = ninput_items;
                }
            // make_two_steps: centre the narrow grid on the coarse Doppler (:937-943)
            if (d_step_two)
                {
                    d_doppler_center_step_two = d_gnss_synchro ? static_cast<float>(d_gnss_synchro->Acq_doppler_hz) : 0.0F;
                    d_state = 0;
                    d_active = true;
                }
            if (d_step_repeat) d_active = true;  // :944-947
            return consumed;
        }
    switch (d_state)
        {
        case 0:
            {
                if (d_gnss_synchro && !d_step_repeat)  // :956-963
                    {
                        d_gnss_synchro->Acq_delay_samples = 0.0;
                        d_gnss_synchro->Acq_doppler_hz = 0.0;
                        d_gnss_synchro->Acq_samplestamp_samples = 0ULL;
                        d_gnss_synchro->Acq_doppler_step = 0U;
                    }
                d_mag = 0.0F;
                d_state = 1;
                d_buffer_count = 0U;
                if (!d_acq_parameters.blocking_on_standby)
                    {
                        d_sample_counter += static_cast<uint64_t>(ninput_items);
                        return ninput_items;
                    }
                return 0;
            }
        case 1:
            {
                uint32_t inc = (static_cast<uint32_t>(ninput_items) + d_buffer_count <= d_consumed_samples)
                                   ? static_cast<uint32_t>(ninput_items)
                                   : d_consumed_samples - d_buffer_count;
                const size_t isz = d_acq_parameters.it_size;
                std::memcpy(d_data_buffer.data() + static_cast<size_t>(d_buffer_count) * isz, in, static_cast<size_t>(inc) * isz);
                if (d_buffer_count >= d_consumed_samples) d_state = 2;
                d_buffer_count += inc;
                d_sample_counter += static_cast<uint64_t>(inc);
                return static_cast<int>(inc);
            }
        case 2:
            {
                lk.unlock();
                acquisition_core(d_sample_counter);
                d_buffer_count = 0U;
                return 0;
            }
        default:
            return 0;
        }
}
