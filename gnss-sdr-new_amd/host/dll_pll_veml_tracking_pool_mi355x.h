// Pooled dll_pll_veml_tracking on the MI355X engine: the same block method set as
// dll_pll_veml_tracking_mi355x (tracking_block_mi355x.h), but every channel of one
// signal on one GPU lives in ONE gsdr_trk handle (a SharedTrackingPool) that reads
// the GPU's device IQ ring in place.
//
// The reference runs one dll_pll_veml_tracking block per channel, each on its own
// scheduler thread over the shared conditioner output (gnss_flowgraph.cc:1007-1135,
// dll_pll_veml_tracking.cc:1784-2152), consuming exactly one correlation's items per
// general_work call.  The per-channel MI355X block keeps that shape and pays one
// synchronous H2D + launch + D2H + sync per call.  The pooled block
// decouples consumption from computation: work() pushes the items it is handed into
// the pool's ring (whichever block sees a stretch first) and consumes them; the
// pool advances every started channel over the ring in one launch per batch of
// batch_calls correlation lengths (and whenever window/2 items arrived since the
// last advance, so no channel falls out of the ring whatever the scheduler's buffer
// sizes); each block then hands out its channel's per-call records in order, one
// Gnss_Synchro per work() call that emits (Tracking_sample_counter = the call's
// nitems_read, as the reference).  The per-call records equal the per-channel
// block's bit for bit (host self-test); outputs come up to one batch later.
#ifndef GSDR_HOST_DLL_PLL_VEML_TRACKING_POOL_MI355X_H
#define GSDR_HOST_DLL_PLL_VEML_TRACKING_POOL_MI355X_H

#include <cstdint>
#include <deque>
#include <functional>
#include <memory>
#include <mutex>
#include <string>
#include <vector>

#include "device_iq_ring.h"
#include "dll_pll_conf.h"
#include "gnss_synchro.h"
#include "gsdr.h"
#include "tracking_block_mi355x.h"
#include "tracking_dump.h"
#include "tracking_output.h"

class SharedTrackingPool
{
public:
    // window_calls: the ring window in vector lengths (the ring holds twice that);
    // batch_calls: vector lengths of new items per advance launch
    // ring_key: the input stream's DeviceIqRing key (pools of one key read one stream)
    SharedTrackingPool(const Dll_Pll_Conf& conf, int32_t signal, uint32_t max_channels, int device,
        uint32_t window_calls = kDefaultWindowCalls, uint32_t batch_calls = kDefaultBatchCalls,
        const std::string& ring_key = "rf0");
    static constexpr uint32_t kDefaultWindowCalls = 64;
    static constexpr uint32_t kDefaultBatchCalls = 8;
    ~SharedTrackingPool();
    SharedTrackingPool(const SharedTrackingPool&) = delete;
    SharedTrackingPool& operator=(const SharedTrackingPool&) = delete;

    // the pool of (key, device, signal): created by the first block, shared by the
    // rest while any holds it (GNSSBlockFactory builds one block per channel)
    static std::shared_ptr<SharedTrackingPool> get(const std::string& key, const Dll_Pll_Conf& conf, int32_t signal,
        uint32_t max_channels, int device, uint32_t window_calls = kDefaultWindowCalls,
        uint32_t batch_calls = kDefaultBatchCalls, const std::string& ring_key = "rf0");

    int acquire_slot();  // -1 when every slot is taken
    void release_slot(int slot);
    // start_tracking + the state-1 pull-in of `slot` at input position nitems_read
    // (gsdr_trk_start); returns the first sample of its first correlation
    uint64_t start(int slot, uint32_t prn, const char signal[2], double acq_delay_samples, double acq_doppler_hz,
        uint64_t acq_samplestamp, uint64_t nitems_read);
    void stop(int slot);
    // a telemetry fault on `slot` (gsdr_trk_force_loss_of_lock)
    void force_loss_of_lock(int slot);
    // input items [nitems_read, nitems_read + n): the part the GPU's shared ring
    // (DeviceIqRing) has not seen is pushed; every pool on the ring advances its
    // started channels whenever half its window arrived since its last advance
    void feed(const void* in, uint64_t nitems_read, int n);
    // an advance launch when batch_calls vector lengths arrived since the last one,
    // asynchronous: its records land in the queues when a later call finds it done
    // (force: when anything arrived, and wait for the records)
    void advance_if_due(bool force);
    // the next per-call record of `slot` (in call order), taken out of the queue when
    // its call ends at or before handed_end (the items its block has been handed:
    // the time tags of a later call have not reached the block yet)
    bool pop(int slot, uint64_t handed_end, gsdr_trk_epoch* rec);
    // the next record is there and pop() would take it
    bool ready(int slot, uint64_t handed_end);
    size_t queued(int slot);  // records computed and not yet handed out

    uint64_t launches() const { return d_launches; }
    uint64_t window_items() const { return d_window; }
    DeviceIqRing* ring() const { return d_ring.get(); }
    uint64_t batch_items() const { return d_batch; }

private:
    void advance_locked(uint64_t head, bool wait);
    bool take_locked(bool wait);  // the oldest submission in flight -> the queues (false: not landed)
    void on_pushed(uint64_t from, uint64_t head);  // the ring's hook

    Dll_Pll_Conf d_conf;
    int32_t d_signal;
    uint32_t d_max;
    int d_device;
    uint64_t d_window{0};
    uint64_t d_batch{0};
    gsdr_trk* d_engine{nullptr};
    std::shared_ptr<DeviceIqRing> d_ring;
    int d_hook{-1};
    bool d_seen{false};      // d_advanced holds a ring head
    uint64_t d_advanced{0};  // the ring head at the last advance
    uint64_t d_launches{0};
    std::vector<bool> d_used;
    std::vector<bool> d_active;
    std::vector<std::deque<gsdr_trk_epoch>> d_queue;
    std::vector<gsdr_trk_epoch> d_recs;
    std::vector<uint32_t> d_n;
    std::vector<uint32_t> d_gen;                  // per slot: bumped by start / stop / release
    std::deque<std::vector<uint32_t>> d_sub_gens;  // d_gen at each submission in flight, oldest first
    static constexpr size_t kInFlight = 2;         // gsdr_trk_submit_stream's queue depth
    uint32_t d_epochs{0};                         // calls per channel per submission
    bool d_more{false};                           // the last collected one filled a channel's batch
    std::mutex d_mu;
};

class dll_pll_veml_tracking_pool_mi355x : public TrackingBlockMI355X
{
public:
    // pool_key: the pool's registry key (the adapters use role + device);
    // window_calls / batch_calls: <role>.mi355x_pool_window / .mi355x_pool_batch;
    // ring_key: <role>.mi355x_ring, the input stream's shared device ring
    dll_pll_veml_tracking_pool_mi355x(const Dll_Pll_Conf& conf, int32_t signal, uint32_t pool_channels, int device,
        const std::string& pool_key, uint32_t window_calls = SharedTrackingPool::kDefaultWindowCalls,
        uint32_t batch_calls = SharedTrackingPool::kDefaultBatchCalls, const std::string& ring_key = "rf0");
    ~dll_pll_veml_tracking_pool_mi355x() override;

    void set_gnss_synchro(Gnss_Synchro* p_gnss_synchro) override;
    void set_channel(uint32_t channel) override;
    void start_tracking() override;
    void stop_tracking() override;
    void set_event_handler(std::function<void(int)> h) override { d_events = std::move(h); }
    void msg_handler_telemetry_to_trk(int tlm_event) override;
    // any items are useful: work() feeds what it is handed to the ring
    int forecast() const override { return 1; }
    int work(const void* in, int ninput_items, uint64_t nitems_read, Gnss_Synchro* out, int* noutput,
        TrackingTags* tags) override;
    using TrackingBlockMI355X::work;
    void flush() override;
    int32_t state() const override { return d_state; }
    const gsdr_trk_epoch& last_record() const override { return d_last; }
    SharedTrackingPool* pool() { return d_pool.get(); }
    int slot() const { return d_slot; }
    // loss-of-lock records the engine marked GSDR_TRK_F_OVERRUN (a channel started
    // before the oldest item the ring still held)
    uint64_t overruns() const { return d_overruns; }

private:
    // work() without the landed-items clamp: the items it would consume
    int work_locked(const void* in, int ninput_items, uint64_t nitems_read, Gnss_Synchro* out, int* noutput,
        TrackingTags* tags);

    Dll_Pll_Conf d_conf;
    int32_t d_signal;
    std::shared_ptr<SharedTrackingPool> d_pool;
    int d_slot{-1};
    Gnss_Synchro* d_acquisition_gnss_synchro{nullptr};
    uint32_t d_channel{0};
    int32_t d_state{0};  // 0 standby, 1 pull-in pending, 2 tracking
    gsdr_trk_epoch d_last{};
    std::function<void(int)> d_events;
    std::mutex d_setlock;
    uint64_t d_overruns{0};
    TrackingDump d_dump;  // <role>.dump: the reference's per-channel .dat (log_data), .mat on destruction
    TrackingOutput d_output;
    std::deque<GnssTimeTag> d_tags;  // input time tags not yet matched to a call
    uint64_t d_handed_end{0};        // end of the items the scheduler has handed this block
    std::vector<GnssTimeTag> d_in_call;  // the tags of the call being emitted
    bool d_fault_pending{false};     // telemetry fault between start_tracking and the pull-in
};

#endif
