#include "pcps_acquisition_mi355x.h"

#include <cmath>
#include <cstring>
#include <filesystem>
#include <iostream>
#include <stdexcept>

#include "mat5_writer.h"

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
    // dump file stem and directory (:135-165): basename without extension, default
    // "acquisition", in the dump_filename's directory (created), else "."
    d_dump = conf.dump;
    if (d_dump)
        {
            std::string name = conf.dump_filename, dir = ".";
            const auto slash = name.find_last_of('/');
            if (slash != std::string::npos)
                {
                    dir = name.substr(0, slash);
                    name = name.substr(slash + 1);
                }
            if (name.empty()) name = "acquisition";
            if (name.size() > 1 && name.substr(1).find_last_of('.') != std::string::npos)
                name = name.substr(0, name.find_last_of('.'));
            std::error_code ec;
            std::filesystem::create_directories(dir, ec);
            if (ec)
                {
                    std::cerr << "GNSS-SDR cannot create dump file for the Acquisition block. Wrong permissions?\n";
                    d_dump = false;
                }
            d_dump_filename = dir + "/" + name;
        }
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

pcps_acquisition_mi355x::~pcps_acquisition_mi355x()
{
    if (d_worker.joinable()) d_worker.join();
    gsdr_acq_destroy(d_engine);
}

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
    // the configuration's carrier model, whatever GSDR_ACQ_WIPE says
    if (gsdr_acq_set_wipeoff(d_engine, d_acq_parameters.wipeoff_mode()) != GSDR_OK)
        throw std::runtime_error(std::string("pcps_acquisition_mi355x: ") + gsdr_last_error());
    // make_two_steps narrow grid (Acq_Conf second_nbins / second_doppler_step / pfa2)
    if (d_acq_parameters.make_2_steps &&
        gsdr_acq_set_step_two(d_engine, d_acq_parameters.num_doppler_bins_step2, d_acq_parameters.doppler_step2,
            d_acq_parameters.pfa2) != GSDR_OK)
        throw std::runtime_error(std::string("pcps_acquisition_mi355x: ") + gsdr_last_error());
    uint32_t D = 0, N = 0;
    gsdr_acq_get_dims(d_engine, &D, &N);
    d_num_doppler_bins = D;
    d_eff = d_acq_parameters.bit_transition_flag ? N / 2 : N;
    if (d_dump)
        {
            // init (:287-292): zeroed grids of the effective FFT size
            d_grid.assign(static_cast<size_t>(d_eff) * D, 0.0F);
            d_narrow_grid.assign(static_cast<size_t>(d_eff) * d_acq_parameters.num_doppler_bins_step2, 0.0F);
        }
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
    // (:617) the core holds d_setlock; a blocking block releases it for the grid
    // (:655-658), the worker of a non-blocking one keeps it to the end
    std::unique_lock<std::mutex> lk(d_setlock);
    if (d_acq_parameters.blocking) lk.unlock();
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
            d_worker_active = false;
            send_negative_acquisition();
            return;
        }
    if (d_dump && d_channel == d_acq_parameters.dump_channel) dump_grid_dwell();
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
    d_worker_active = false;
    if (d_num_noncoherent_integrations_counter == d_acq_parameters.max_dwells || d_positive_acq == 1 ||
        d_acq_parameters.bit_transition_flag)
        {
            // record results to file if required (:873-877)
            if (d_dump && d_channel == d_acq_parameters.dump_channel) dump_results();
            d_num_noncoherent_integrations_counter = 0U;
            d_positive_acq = 0;
        }
}

// The magnitude grid of this dwell for the dump channel (:680-685, :741-746): the
// engine recomputes the block's |R|^2 grid (gsdr_acq_dump_grid, the narrow one in
// step two), whose effective window (outputs [N - eff, N), :671) is stored -- on the
// first dwell of the attempt -- or added in float (volk_32f_x2_add_32f, :673-675).
void pcps_acquisition_mi355x::dump_grid_dwell()
{
    uint32_t D = 0, N = 0;
    gsdr_acq_get_dims(d_engine, &D, &N);
    const bool two = d_step_two;
    const uint32_t rows = two ? d_acq_parameters.num_doppler_bins_step2 : D;
    d_grid_tmp.resize(static_cast<size_t>(rows) * N);
    const int rc = two ? gsdr_acq_dump_grid_step_two(d_engine, d_data_buffer.data(), 0, d_doppler_center_step_two,
                             d_grid_tmp.data())
                       : gsdr_acq_dump_grid(d_engine, d_data_buffer.data(), 0, d_grid_tmp.data());
    if (rc != GSDR_OK)
        {
            std::cerr << "pcps_acquisition_mi355x: dump grid: " << gsdr_last_error() << '\n';
            return;
        }
    std::vector<float>& g = two ? d_narrow_grid : d_grid;
    g.resize(static_cast<size_t>(d_eff) * rows);
    const uint32_t off = N - d_eff;
    const bool first = d_num_noncoherent_integrations_counter == 1;
    for (uint32_t d = 0; d < rows; ++d)
        for (uint32_t i = 0; i < d_eff; ++i)
            {
                const float v = d_grid_tmp[static_cast<size_t>(d) * N + off + i];
                float& o = g[static_cast<size_t>(d) * d_eff + i];
                o = first ? v : o + v;
            }
}

// dump_results (:408-508): <dump_filename>_<System>_<Signal>_ch_<channel>_<n>_sat_<PRN>.mat
// with the reference's variables (names, classes, dimensions); Level-5 MAT-file
// (mat5_writer.h) instead of matio's MAT 7.3.
void pcps_acquisition_mi355x::dump_results()
{
    if (!d_gnss_synchro) return;
    d_dump_number++;
    std::string fn = d_dump_filename + "_";
    fn.append(1, d_gnss_synchro->System);
    fn += "_";
    fn.append(1, d_gnss_synchro->Signal[0]);
    fn.append(1, d_gnss_synchro->Signal[1]);
    fn += "_ch_" + std::to_string(d_channel) + "_" + std::to_string(d_dump_number) + "_sat_" +
          std::to_string(d_gnss_synchro->PRN) + ".mat";
    Mat5Writer m;
    if (!m.open(fn))
        {
            std::cout << "Unable to create or open Acquisition dump file\n";
            return;
        }
    m.write("acq_grid", Mat5Writer::kSingle, d_eff, d_num_doppler_bins, d_grid.data());
    m.write_int32("doppler_max", d_acq_parameters.doppler_max);
    m.write_int32("doppler_step", static_cast<int32_t>(d_doppler_step));
    m.write_int32("d_positive_acq", d_positive_acq);
    m.write_single("acq_doppler_hz", static_cast<float>(d_gnss_synchro->Acq_doppler_hz));
    m.write_single("acq_delay_samples", static_cast<float>(d_gnss_synchro->Acq_delay_samples));
    m.write_single("test_statistic", d_test_statistics);
    m.write_single("threshold", d_threshold);
    m.write_single("input_power", d_input_power);
    m.write_uint64("sample_counter", d_sample_counter);
    m.write_uint32("PRN", d_gnss_synchro->PRN);
    m.write_int32("num_dwells", static_cast<int32_t>(d_num_noncoherent_integrations_counter));
    if (d_acq_parameters.make_2_steps)
        {
            m.write("acq_grid_narrow", Mat5Writer::kSingle, d_eff, d_acq_parameters.num_doppler_bins_step2,
                d_narrow_grid.data());
            m.write_single("doppler_step_narrow", d_acq_parameters.doppler_step2);
            m.write_single("doppler_grid_narrow_min",
                d_doppler_center_step_two -
                    static_cast<float>(std::floor(d_acq_parameters.num_doppler_bins_step2 / 2.0)) *
                        d_acq_parameters.doppler_step2);
        }
    if (!m.close())
        std::cout << "Unable to create or open Acquisition dump file\n";
    else
        d_last_dump = fn;
}

// general_work (:912-1050) with blocking acquisition.
int pcps_acquisition_mi355x::work(const void* in, int ninput_items)
{
    std::unique_lock<std::mutex> lk(d_setlock);
    if (!d_active || d_worker_active)
        {
            // do not consume samples while performing a non-coherent integration (:928-936)
            const bool consume_samples =
                !d_active || d_num_noncoherent_integrations_counter == d_acq_parameters.max_dwells;
            int consumed = 0;
            if (!d_acq_parameters.blocking_on_standby && consume_samples)
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
                // :1013-1029: the core inline (blocking) or on a worker thread
                if (d_acq_parameters.blocking)
                    {
                        lk.unlock();
                        acquisition_core(d_sample_counter);
                    }
                else
                    {
                        if (d_worker.joinable()) d_worker.join();  // the previous core ended (d_worker_active false)
                        d_worker_active = true;
                        ++d_async_cores;
                        d_worker = std::thread(&pcps_acquisition_mi355x::acquisition_core, this, d_sample_counter);
                    }
                d_buffer_count = 0U;
                return 0;
            }
        default:
            return 0;
        }
}
