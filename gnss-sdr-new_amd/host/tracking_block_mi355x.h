// The block-level method set every MI355X tracking block provides (the public
// part of dll_pll_veml_tracking.h:58-213 plus work() for general_work): the
// per-channel block (dll_pll_veml_tracking_mi355x, one gsdr_trk handle per
// channel, synchronous calls) and the pooled block (dll_pll_veml_tracking_pool_
// mi355x, every channel of one signal on one GPU in one gsdr_trk handle over the
// GPU's device IQ ring).  The tracking adapters hold either behind this interface.
#ifndef GSDR_HOST_TRACKING_BLOCK_MI355X_H
#define GSDR_HOST_TRACKING_BLOCK_MI355X_H

#include <cstdint>
#include <functional>

#include "gnss_synchro.h"
#include "gsdr.h"
#include "tracking_output.h"

class TrackingBlockMI355X
{
public:
    virtual ~TrackingBlockMI355X() = default;
    virtual void set_gnss_synchro(Gnss_Synchro* p_gnss_synchro) = 0;
    virtual void set_channel(uint32_t channel) = 0;
    virtual void start_tracking() = 0;
    virtual void stop_tracking() = 0;
    // the "events" message port: 3 = loss of lock
    virtual void set_event_handler(std::function<void(int)> h) = 0;
    // the "telemetry_to_trk" message port (msg_handler_telemetry_to_trk,
    // dll_pll_veml_tracking.cc:614-637): tlm_event 1 = telemetry fault, which forces
    // the loss-of-lock condition at the channel's next lock check
    virtual void msg_handler_telemetry_to_trk(int tlm_event) = 0;
    // forecast (:604-611): items general_work needs
    virtual int forecast() const = 0;
    // general_work (:1784-2152): `in` holds ninput_items items, the first being input
    // sample nitems_read; returns the items consumed, *noutput = 1 with *out filled
    // when a Gnss_Synchro is emitted (valid symbol output or loss of lock).  tags
    // (optional): the GnssTime stream tags of the input and the output's tag
    // (:2088-2147, TrackingOutput)
    virtual int work(const void* in, int ninput_items, uint64_t nitems_read, Gnss_Synchro* out, int* noutput,
        TrackingTags* tags) = 0;
    int work(const void* in, int ninput_items, uint64_t nitems_read, Gnss_Synchro* out, int* noutput)
    {
        return work(in, ninput_items, nitems_read, out, noutput, nullptr);
    }
    // end of input: compute what the block has been handed but not run yet (the
    // pooled block batches its launches; the per-channel block has nothing pending)
    virtual void flush() {}
    virtual int32_t state() const = 0;
    virtual const gsdr_trk_epoch& last_record() const = 0;
    // nitems_written(0): the Gnss_Synchro items emitted so far
    uint64_t nitems_written() const { return d_nitems_written; }
    // every per-call engine record the block hands out, in call order (tests, dumps)
    void set_record_sink(std::function<void(const gsdr_trk_epoch&)> sink) { d_record_sink = std::move(sink); }

protected:
    uint64_t d_nitems_written{0};
    std::function<void(const gsdr_trk_epoch&)> d_record_sink;
};

#endif
