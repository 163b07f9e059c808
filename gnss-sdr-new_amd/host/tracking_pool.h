// Batched tracking service: one gsdr_trk handle
// holding every channel of one signal on this GPU, advanced in place over the
// GPU's device IQ ring after each push -- the reference runs one
// dll_pll_veml_tracking block per channel on its own scheduler thread, each
// consuming its own copy of the stream (dll_pll_veml_tracking.cc:1784-2152).  A
// channel is started from its Gnss_Synchro acquisition fields, like
// TrackingInterface::start_tracking (tracking_interface.h:50), and its
// Gnss_Synchro outputs (valid symbol outputs and loss-of-lock records,
// :2120-2147) come back through a callback per general_work call that emits one.
#ifndef GSDR_HOST_TRACKING_POOL_H
#define GSDR_HOST_TRACKING_POOL_H

#include <cstdint>
#include <functional>
#include <vector>

#include "dll_pll_conf.h"
#include "gnss_synchro.h"
#include "gsdr.h"
#include "tracking_output.h"

class TrackingPool
{
public:
    using Output = std::function<void(uint32_t slot, const Gnss_Synchro& out)>;

    // signal: GSDR_SIGNAL_*; conf.vector_length as the signal's adapter sets it
    TrackingPool(const Dll_Pll_Conf& conf, int32_t signal, uint32_t max_channels, gsdr_stream* ring, int device = 0);
    ~TrackingPool();
    TrackingPool(const TrackingPool&) = delete;
    TrackingPool& operator=(const TrackingPool&) = delete;

    // start_tracking of slot from gs (kept; its Acq_* fields and PRN are read now),
    // the pull-in aligned after input position nitems_read (usually the ring head)
    void start(uint32_t slot, Gnss_Synchro* gs, uint64_t nitems_read);
    void stop(uint32_t slot);
    // every started channel over the ring up to its head; out() for each emitted
    // record; returns the number of general_work calls run
    uint64_t advance(const Output& out, uint32_t max_epochs = 256);

private:
    Dll_Pll_Conf d_conf;
    int32_t d_signal;
    uint32_t d_max;
    gsdr_stream* d_ring;
    gsdr_trk* d_engine{nullptr};
    std::vector<Gnss_Synchro*> d_synchro;
    std::vector<gsdr_trk_epoch> d_recs;
    std::vector<uint32_t> d_n;
    TrackingOutput d_output;
};

#endif
