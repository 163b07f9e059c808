// pcps_acquisition on the MI355X engine: the public method set of
// src/algorithms/acquisition/gnuradio_blocks/pcps_acquisition.h:84-286 with the
// GNU Radio plumbing replaced by work() (general_work's state machine,
// pcps_acquisition.cc:912-1050) and an event callback (the "events" message
// port: 1 positive, 2 negative).  acquisition_core runs on the GPU through
// gsdr_acq_run (include/gsdr.h).
#ifndef GSDR_HOST_PCPS_ACQUISITION_MI355X_H
#define GSDR_HOST_PCPS_ACQUISITION_MI355X_H

#include <complex>
#include <cstdint>
#include <functional>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "acq_conf.h"
#include "channel_fsm.h"
#include "gnss_synchro.h"
#include "gsdr.h"

class pcps_acquisition_mi355x
{
public:
    explicit pcps_acquisition_mi355x(const Acq_Conf& conf, int device = 0);
    ~pcps_acquisition_mi355x();
    pcps_acquisition_mi355x(const pcps_acquisition_mi355x&) = delete;
    pcps_acquisition_mi355x& operator=(const pcps_acquisition_mi355x&) = delete;

    void set_gnss_synchro(Gnss_Synchro* p_gnss_synchro) { d_gnss_synchro = p_gnss_synchro; }
    uint32_t mag() const { return static_cast<uint32_t>(d_mag); }
    void init();
    void set_local_code(std::complex<float>* code);
    void set_active(bool active);
    void set_state(int32_t state);
    void set_channel(uint32_t channel) { d_channel = channel; }
    void set_threshold(float threshold) { d_threshold = threshold; }
    void set_doppler_max(uint32_t doppler_max) { d_acq_parameters.doppler_max = static_cast<int32_t>(doppler_max); }
    void set_doppler_step(uint32_t doppler_step) { d_doppler_step = doppler_step; }
    void set_doppler_center(int32_t doppler_center);
    void set_resampler_latency(uint32_t latency_samples) { d_acq_parameters.resampler_latency_samples = latency_samples; }
    void set_event_handler(std::function<void(int)> h) { d_events = std::move(h); }
    // the channel FSM notified directly of a positive acquisition (pcps_acquisition.h:159-161)
    void set_channel_fsm(std::weak_ptr<ChannelFsm> channel_fsm) { d_channel_fsm = std::move(channel_fsm); }
    // start(): sample counter reset and threshold from pfa (pcps_acquisition.cc:885-891)
    bool start();
    void calculate_threshold();

    // general_work: consumes up to ninput_items items of it_size bytes; returns the
    // number consumed (consume_each).  Runs acquisition_core when the buffer is full.
    int work(const void* in, int ninput_items);

    float threshold() const { return d_threshold; }
    float test_statistics() const { return d_test_statistics; }
    float input_power() const { return d_input_power; }
    uint32_t num_doppler_bins() const { return d_num_doppler_bins; }
    bool step_two() const { return d_step_two; }
    bool step_repeat() const { return d_step_repeat; }

    uint32_t num_noncoherent_integrations() const { return d_num_noncoherent_integrations_counter; }
    static int engine_item_type(const std::string& item_type);
    // blocking = false: acquisition_core calls run on a worker thread (and how many did)
    uint64_t async_cores() const { return d_async_cores; }
    bool worker_active() const { return d_worker_active; }
    // dump = true: the dump files written so far (dump_results), and the last one's path
    int64_t dump_number() const { return d_dump_number; }
    const std::string& last_dump_path() const { return d_last_dump; }

private:
    void acquisition_core(uint64_t samp_count);
    void dump_grid_dwell();
    void dump_results();
    void ensure_engine();
    void send_positive_acquisition();
    void send_negative_acquisition();

    Acq_Conf d_acq_parameters;
    int d_device;
    int d_item_type{GSDR_ITEM_GR_COMPLEX};
    gsdr_acq* d_engine{nullptr};
    int32_t d_engine_dmax{0};
    uint32_t d_engine_step{0};
    Gnss_Synchro* d_gnss_synchro{nullptr};
    std::function<void(int)> d_events;
    std::weak_ptr<ChannelFsm> d_channel_fsm;
    std::vector<uint8_t> d_data_buffer;
    std::vector<std::complex<float>> d_code;
    bool d_code_set{false};
    uint64_t d_sample_counter{0};
    float d_threshold{0.0F};
    float d_mag{0.0F};
    float d_input_power{0.0F};
    float d_test_statistics{0.0F};
    int32_t d_state{0};
    int32_t d_positive_acq{0};
    int32_t d_doppler_center{0};
    uint32_t d_channel{0};
    uint32_t d_doppler_step;
    uint32_t d_num_noncoherent_integrations_counter{0};
    uint32_t d_consumed_samples;
    uint32_t d_num_doppler_bins{0};
    uint32_t d_buffer_count{0};
    bool d_active{false};
    bool d_step_two{false};                // make_2_steps: the next core call is the narrow grid
    float d_doppler_center_step_two{0.0F};
    bool d_step_repeat{false};  // fork's make_repeat_steps: keep re-acquiring after a positive
    // blocking = false (:1013-1029): the core on a worker thread that holds d_setlock
    std::thread d_worker;
    bool d_worker_active{false};
    uint64_t d_async_cores{0};
    // dump (:135-165, :408-508): the magnitude grids of the attempt for the dump channel
    bool d_dump{false};
    std::string d_dump_filename;
    std::string d_last_dump;
    int64_t d_dump_number{0};
    uint32_t d_eff{0};                 // effective_fft_size
    std::vector<float> d_grid;         // eff x D, column-major (arma::fmat d_grid)
    std::vector<float> d_narrow_grid;  // eff x num_doppler_bins_step2
    std::vector<float> d_grid_tmp;
    std::mutex d_setlock;
};

#endif
