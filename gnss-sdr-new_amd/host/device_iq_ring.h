// One device IQ ring per (GPU, item type, input stream) shared by every pooled
// tracking block and acquisition service that reads that stream: the
// conditioner output that GNU Radio hands to every channel's blocks
// (gnss_flowgraph.cc:1007-1135, the channel's RF_channel_ID picking the conditioner)
// crosses PCIe once -- whichever block sees a stretch of it first pushes it -- and
// every consumer reads its windows in place by absolute sample index (nitems_read,
// dll_pll_veml_tracking.cc:1797,1818,2122).
//
// The key names the input stream: consumers that pass the same key must be handed the
// same items at the same nitems_read (one conditioner's output).  feed() checks the
// last item it pushed against every later feeder whose items cover it and throws
// std::logic_error on a mismatch (two streams under one key).
//
// Consumers that must keep up with the ring (the tracking pools, whose channels read
// their next call from the newest window) register a hook; feed() pushes in pieces of
// at most window/2 items and runs the hooks after each piece, outside the ring's
// lock, so a pool advances its channels before the ring can overwrite what they
// still need, whoever pushes.
#ifndef GSDR_HOST_DEVICE_IQ_RING_H
#define GSDR_HOST_DEVICE_IQ_RING_H

#include <atomic>
#include <cstdint>
#include <functional>
#include <map>
#include <memory>
#include <mutex>
#include <string>

#include "gsdr.h"

class DeviceIqRing
{
public:
    // after a piece [from, head) was pushed
    using Hook = std::function<void(uint64_t from, uint64_t head)>;
    // the smallest window a shared ring is created with (items): every consumer of
    // this path up to Galileo E1 pools at 25 Msps (64 x 100000 items) fits
    static constexpr uint64_t kMinWindow = uint64_t(1) << 23;

    // the process's ring of (device, item_type, key) whose window holds window_items;
    // a consumer needing a larger window than the existing ring's gets one of its own
    static std::shared_ptr<DeviceIqRing> get(int device, int item_type, uint64_t window_items,
        const std::string& key = "rf0");

    DeviceIqRing(int device, int item_type, uint64_t window_items);  // 2 x window positions
    ~DeviceIqRing();
    DeviceIqRing(const DeviceIqRing&) = delete;
    DeviceIqRing& operator=(const DeviceIqRing&) = delete;

    gsdr_stream* stream() const { return d_ring; }
    uint64_t window() const { return d_window; }
    size_t item_bytes() const { return d_item_bytes; }
    int device() const { return d_device; }

    int add_hook(Hook h);
    // returns once no feed() is running hooks: the hook's owner may then be destroyed
    // (not to be called from inside a hook)
    void remove_hook(int id);

    // input items [nitems_read, nitems_read + n): the part the ring has not seen is
    // pushed (pieces <= window/2, the hooks after each); items before the first push
    // start the ring; throws std::logic_error when nitems_read is past the head (a
    // stretch no consumer pushed)
    void feed(const void* in, uint64_t nitems_read, int n);
    // the next item to push (absolute index); false before the first push
    bool head(uint64_t* h) const;
    // every item before the returned index is in device memory: a push copies from
    // the feeder's buffer after feed() returns, so a block consumes (and its upstream
    // may recycle) only items before it (gsdr_stream_landed)
    // (want: the caller's question "has everything before want landed?" -- answered
    // from the last value seen without a query when it has)
    uint64_t landed(uint64_t want = UINT64_MAX);
    void wait_landed(uint64_t upto);  // gsdr_stream_wait_landed

private:
    int d_device;
    size_t d_item_bytes;
    uint64_t d_window;
    gsdr_stream* d_ring{nullptr};
    bool d_started{false};
    uint64_t d_head{0};
    std::map<int, Hook> d_hooks;
    unsigned char d_last[8]{};  // the last item pushed (at d_head - 1): the stream check
    int d_next_hook{0};
    mutable std::mutex d_mu;       // head / started / hooks
    std::mutex d_push_mu;          // one pusher at a time (pieces in order)
    std::atomic<uint64_t> d_landed{0};  // the last landed index seen (monotone)
};

#endif
