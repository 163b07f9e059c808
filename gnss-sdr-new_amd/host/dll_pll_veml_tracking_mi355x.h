// dll_pll_veml_tracking on the MI355X engine: the public method set of
// src/algorithms/tracking/gnuradio_blocks/dll_pll_veml_tracking.h:58-213 with the
// GNU Radio plumbing replaced by work() (general_work, dll_pll_veml_tracking.cc:
// 1784-2152) and an event callback (the "events" message port: 3 = loss of lock).
// Every correlation and loop update of a call runs on the GPU through the
// gsdr_trk_* C ABI (include/gsdr.h); this block owns a one-channel pool.
#ifndef GSDR_HOST_DLL_PLL_VEML_TRACKING_MI355X_H
#define GSDR_HOST_DLL_PLL_VEML_TRACKING_MI355X_H

#include <cstdint>
#include <functional>
#include <mutex>
#include <vector>

#include "dll_pll_conf.h"
#include "gnss_synchro.h"
#include "gsdr.h"
#include "tracking_block_mi355x.h"
#include "tracking_dump.h"
#include "tracking_output.h"

class dll_pll_veml_tracking_mi355x : public TrackingBlockMI355X
{
public:
    // signal: GSDR_SIGNAL_GPS_1C / GSDR_SIGNAL_GAL_1B / GSDR_SIGNAL_BDS_B1
    dll_pll_veml_tracking_mi355x(const Dll_Pll_Conf& conf, int32_t signal, int device = 0);
    ~dll_pll_veml_tracking_mi355x() override;
    dll_pll_veml_tracking_mi355x(const dll_pll_veml_tracking_mi355x&) = delete;
    dll_pll_veml_tracking_mi355x& operator=(const dll_pll_veml_tracking_mi355x&) = delete;

    void set_gnss_synchro(Gnss_Synchro* p_gnss_synchro) override;
    void set_channel(uint32_t channel) override;
    // start_tracking (:640-882): takes Acq_delay_samples / Acq_doppler_hz /
    // Acq_samplestamp_samples from the channel's Gnss_Synchro and the PRN's
    // replica; the pull-in (state 1) runs on the next work() call
    void start_tracking() override;
    void stop_tracking() override;
    void set_event_handler(std::function<void(int)> h) override { d_events = std::move(h); }
    void msg_handler_telemetry_to_trk(int tlm_event) override;

    // forecast (:604-611): items general_work needs
    int forecast() const override { return 2 * static_cast<int>(d_vector_length); }
    // general_work: `in` holds ninput_items items of the configured item type, the
    // first one being input sample nitems_read.  Returns the items consumed
    // (consume_each); *noutput = 1 with *out filled when a Gnss_Synchro is
    // emitted (valid symbol output or loss of lock), else 0.
    int work(const void* in, int ninput_items, uint64_t nitems_read, Gnss_Synchro* out, int* noutput,
        TrackingTags* tags) override;
    using TrackingBlockMI355X::work;

    int32_t state() const override { return d_state; }
    const gsdr_trk_epoch& last_record() const override { return d_last; }

private:
    void load_codes(uint32_t prn, std::vector<float>& code);

    Dll_Pll_Conf d_conf;
    int32_t d_signal;
    int d_device;
    gsdr_trk* d_engine{nullptr};
    uint32_t d_vector_length{0};
    size_t d_item_bytes{8};
    Gnss_Synchro* d_acquisition_gnss_synchro{nullptr};
    uint32_t d_channel{0};
    int32_t d_state{0};  // 0 standby, 1 pull-in pending, 2 tracking (engine states 2..4)
    gsdr_trk_epoch d_last{};
    std::function<void(int)> d_events;
    std::mutex d_setlock;
    TrackingDump d_dump;  // <role>.dump: the reference's per-channel .dat (log_data), .mat on destruction
    TrackingOutput d_output;
    bool d_fault_pending{false};  // telemetry fault between start_tracking and the pull-in
};

#endif
