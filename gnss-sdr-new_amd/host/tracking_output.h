// The Gnss_Synchro record and the time tag dll_pll_veml_tracking::general_work hands
// downstream (src/algorithms/tracking/gnuradio_blocks/dll_pll_veml_tracking.cc:
// 1784-2152), built on the host from the engine's per-call gsdr_trk_epoch records.
// Shared by the per-channel block, the pooled block and the ring TrackingPool so the
// three emit the same record:
//   * a valid output (states 3 / 4, :2000-2017, :2053-2070): the channel's
//     Gnss_Synchro with Prompt_I/Q, Code_phase_samples, Carrier_phase_rads,
//     Carrier_Doppler_hz, CN0_dB_hz, correlation_length_ms, EVM of the call;
//   * a loss of lock (:1873-1878, :2037-2042): the acquisition record itself
//     (*d_acquisition_gnss_synchro) -- none of the call's tracking values;
//   * both: fs, Tracking_sample_counter = nitems_read, Flag_valid_symbol_output =
//     !loss_of_lock, Flag_PLL_180_deg_phase_locked (:2121-2127).
// Time tags: every call in states 2..4 keeps the last GnssTime "timetag" tag of its
// input window [nitems_read, nitems_read + consumed) (:2088-2116); the next output
// re-emits it, advanced to the output's sample counter, at output item
// nitems_written + 1 (:2129-2147).
#ifndef GSDR_HOST_TRACKING_OUTPUT_H
#define GSDR_HOST_TRACKING_OUTPUT_H

#include <cstdint>

#include "gnss_synchro.h"
#include "gsdr.h"

// GnssTime (src/algorithms/libs/gnss_time.h:23-30): the payload of the
// "timetag" stream tags gnss_sdr_timestamp attaches to the sample stream
class GnssTime
{
public:
    double rx_time{};
    int week{};               // GPS week number (since January 1980)
    int tow_ms{};             // time of week [ms]
    double tow_ms_fraction{}; // tow ms fractional part [ms]
};

// one stream tag: absolute item offset and its GnssTime
struct GnssTimeTag
{
    uint64_t offset{};
    GnssTime time{};
};

// A tracking block's stream-tag I/O for one general_work call: the tags on its input
// items (get_tags_in_range over what the scheduler handed it, in offset order) and
// the tag the call attaches to its output (add_item_tag, :2143).
struct TrackingTags
{
    const GnssTimeTag* in{nullptr};
    int n_in{0};
    bool has_out{false};
    GnssTimeTag out{};  // offset: the output item index (nitems_written(0) + 1)
};

// d_correlation_length_ms of the signal (:178 GPS L1 C/A 1, :269 Galileo E1 4,
// :766 / :783 BeiDou B1I 1)
int32_t tracking_correlation_length_ms(int32_t signal);

class TrackingOutput
{
public:
    TrackingOutput() = default;
    TrackingOutput(double fs_in, int32_t signal) : fs_(fs_in), corr_ms_(tracking_correlation_length_ms(signal)) {}

    // true when the call emits a Gnss_Synchro (valid output or loss of lock); *out
    // is then filled from the record r of the call at nitems_read and the channel's
    // acquisition record acq
    bool emit(const gsdr_trk_epoch& r, const Gnss_Synchro& acq, uint64_t nitems_read, Gnss_Synchro* out) const;

    // the time-tag part of a call that ran (states 2..4): the last tag of
    // [nitems_read, nitems_read + consumed) is kept; with an emitted output `out`
    // the kept tag is re-emitted at output item nitems_written + 1 (tags->out)
    void call_tags(TrackingTags* tags, uint64_t nitems_read, int32_t consumed, const Gnss_Synchro* out,
        uint64_t nitems_written);

private:
    double fs_{0.0};
    int32_t corr_ms_{1};
    GnssTime last_{};
    uint64_t last_offset_{0};
    bool waiting_{false};
};

#endif
