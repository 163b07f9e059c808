// Pooled dll_pll_veml_tracking on the MI355X engine: the same block method set as
// dll_pll_veml_tracking_mi355x (tracking_block_mi355x.h), but every channel of one
// signal on one GPU lives in ONE gsdr_trk handle (a SharedTrackingPool) that reads
// the GPU's device IQ ring in place.
//
// The reference runs one dll_pll_veml_tracking block per channel, each on its own
// scheduler thread over the shared conditioner output (gnss_flowgraph.cc:1007-1135,
// dll_pll_veml_tracking.cc:1784-2152).  The per-channel MI355X block keeps that
// shape and pays one synchronous H2D + launch + D2H + sync per general_work call
// (SURVEY §7 H6).  Here the blocks keep their GNU Radio contract -- work() gets the
// stream at nitems_read and returns the items its channel consumed, one Gnss_Synchro
// per valid call -- while the pool pushes each stretch of the stream once (whichever
// block sees it first), advances every started channel over the ring in one launch
// per chunk, and queues each channel's per-call records for its block to hand out
// in order.
#ifndef GSDR_HOST_DLL_PLL_VEML_TRACKING_POOL_MI355X_H
#define GSDR_HOST_DLL_PLL_VEML_TRACKING_POOL_MI355X_H

#include <cstdint>
#include <deque>
#include <functional>
#include <memory>
#include <mutex>
#include <string>
#include <vector>

#include "dll_pll_conf.h"
#include "gnss_synchro.h"
#include "gsdr.h"
#include "tracking_block_mi355x.h"
#include "tracking_dump.h"

class SharedTrackingPool
{
public:
    // window_calls: the ring window in vector lengths -- how far (in items) a
    // channel's next call may start behind the newest pushed item before the
    // engine reports it as an overrun (loss of lock with GSDR_TRK_F_OVERRUN)
    SharedTrackingPool(const Dll_Pll_Conf& conf, int32_t signal, uint32_t max_channels, int device,
        uint32_t window_calls = kDefaultWindowCalls);
    static constexpr uint32_t kDefaultWindowCalls = 8;
    ~SharedTrackingPool();
    SharedTrackingPool(const SharedTrackingPool&) = delete;
    SharedTrackingPool& operator=(const SharedTrackingPool&) = delete;

    // the pool of (key, device, signal): created by the first block, shared by the
    // rest while any holds it (GNSSBlockFactory builds one block per channel)
    static std::shared_ptr<SharedTrackingPool> get(const std::string& key, const Dll_Pll_Conf& conf, int32_t signal,
        uint32_t max_channels, int device, uint32_t window_calls = kDefaultWindowCalls);

    int acquire_slot();  // -1 when every slot is taken
    void release_slot(int slot);
    // start_tracking + the state-1 pull-in of `slot` at input position nitems_read
    // (gsdr_trk_start); returns the first sample of its first correlation
    uint64_t start(int slot, uint32_t prn, const char signal[2], double acq_delay_samples, double acq_doppler_hz,
        uint64_t acq_samplestamp, uint64_t nitems_read);
    void stop(int slot);
    // input items [nitems_read, nitems_read + n): the part the ring has not seen is
    // pushed (chunked), and every started channel advances over the ring after each
    // chunk (advance = false: push only, for blocks in standby)
    void feed(const void* in, uint64_t nitems_read, int n, bool advance = true);
    // the next per-call record of `slot` (in call order), left in the queue by peek
    bool peek(int slot, gsdr_trk_epoch* rec);
    void drop(int slot);

    size_t item_bytes() const { return d_item_bytes; }
    uint64_t launches() const { return d_launches; }
    uint64_t pushed() const { return d_head - d_origin; }
    uint64_t window_items() const { return d_window; }

private:
    void advance_locked();

    Dll_Pll_Conf d_conf;
    int32_t d_signal;
    uint32_t d_max;
    int d_device;
    size_t d_item_bytes{8};
    uint64_t d_window{0};
    gsdr_trk* d_engine{nullptr};
    gsdr_stream* d_ring{nullptr};
    bool d_started{false};
    uint64_t d_origin{0}, d_head{0};
    uint64_t d_launches{0};
    std::vector<bool> d_used;
    std::vector<bool> d_active;
    std::vector<std::deque<gsdr_trk_epoch>> d_queue;
    std::vector<gsdr_trk_epoch> d_recs;
    std::vector<uint32_t> d_n;
    std::mutex d_mu;
};

class dll_pll_veml_tracking_pool_mi355x : public TrackingBlockMI355X
{
public:
    // pool_key: the pool's registry key (the adapters use role + device);
    // window_calls: <role>.mi355x_pool_window (SharedTrackingPool)
    dll_pll_veml_tracking_pool_mi355x(const Dll_Pll_Conf& conf, int32_t signal, uint32_t pool_channels, int device,
        const std::string& pool_key, uint32_t window_calls = SharedTrackingPool::kDefaultWindowCalls);
    ~dll_pll_veml_tracking_pool_mi355x() override;

    void set_gnss_synchro(Gnss_Synchro* p_gnss_synchro) override;
    void set_channel(uint32_t channel) override;
    void start_tracking() override;
    void stop_tracking() override;
    void set_event_handler(std::function<void(int)> h) override { d_events = std::move(h); }
    int forecast() const override { return 2 * static_cast<int>(d_conf.vector_length); }
    int work(const void* in, int ninput_items, uint64_t nitems_read, Gnss_Synchro* out, int* noutput) override;
    int32_t state() const override { return d_state; }
    const gsdr_trk_epoch& last_record() const override { return d_last; }
    SharedTrackingPool* pool() { return d_pool.get(); }
    // loss-of-lock records the engine marked GSDR_TRK_F_OVERRUN (the channel's next
    // call started before the oldest item the ring window still held)
    uint64_t overruns() const { return d_overruns; }

private:
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
    TrackingDump d_dump;  // <role>.dump: the reference's per-channel .dat (log_data)
};

#endif
