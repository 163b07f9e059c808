#include "device_iq_ring.h"

#include <algorithm>
#include <cstring>
#include <stdexcept>
#include <string>
#include <tuple>
#include <vector>

std::shared_ptr<DeviceIqRing> DeviceIqRing::get(int device, int item_type, uint64_t window_items,
    const std::string& key)
{
    static std::mutex mu;
    static std::map<std::tuple<int, int, std::string>, std::weak_ptr<DeviceIqRing>> registry;
    std::lock_guard<std::mutex> lk(mu);
    auto& w = registry[std::make_tuple(device, item_type, key)];
    if (auto p = w.lock())
        {
            if (p->window() >= window_items) return p;
            return std::make_shared<DeviceIqRing>(device, item_type, window_items);  // its own ring
        }
    auto p = std::make_shared<DeviceIqRing>(device, item_type, std::max(window_items, kMinWindow));
    w = p;
    return p;
}

DeviceIqRing::DeviceIqRing(int device, int item_type, uint64_t window_items)
    : d_device(device),
      d_item_bytes(item_type == GSDR_ITEM_CSHORT ? 4 : (item_type == GSDR_ITEM_IBYTE ? 2 : 8)),
      d_window(window_items)
{
    if (gsdr_stream_create(device, item_type, 2 * d_window, d_window, &d_ring) != GSDR_OK)
        throw std::runtime_error(std::string("DeviceIqRing: ") + gsdr_last_error());
}

DeviceIqRing::~DeviceIqRing() { gsdr_stream_destroy(d_ring); }

int DeviceIqRing::add_hook(Hook h)
{
    std::lock_guard<std::mutex> lk(d_mu);
    const int id = d_next_hook++;
    d_hooks[id] = std::move(h);
    return id;
}

void DeviceIqRing::remove_hook(int id)
{
    // feed() runs the hooks outside d_mu but under d_push_mu: taking it first waits
    // for a dispatch in progress, so no hook runs after its owner removed it (and
    // destroys itself); the same order as feed (push lock, then d_mu)
    std::lock_guard<std::mutex> push_lk(d_push_mu);
    std::lock_guard<std::mutex> lk(d_mu);
    d_hooks.erase(id);
}

bool DeviceIqRing::head(uint64_t* h) const
{
    std::lock_guard<std::mutex> lk(d_mu);
    *h = d_head;
    return d_started;
}

uint64_t DeviceIqRing::landed(uint64_t want)
{
    const uint64_t seen = d_landed.load(std::memory_order_acquire);
    if (seen >= want) return seen;  // most calls: their items landed long ago
    uint64_t v = 0;
    if (gsdr_stream_landed(d_ring, &v) != GSDR_OK)
        throw std::runtime_error(std::string("DeviceIqRing::landed: ") + gsdr_last_error());
    uint64_t cur = seen;
    while (v > cur && !d_landed.compare_exchange_weak(cur, v, std::memory_order_acq_rel)) {}
    return v;
}

void DeviceIqRing::wait_landed(uint64_t upto)
{
    if (gsdr_stream_wait_landed(d_ring, upto) != GSDR_OK)
        throw std::runtime_error(std::string("DeviceIqRing::wait_landed: ") + gsdr_last_error());
    (void)landed(upto);
}

void DeviceIqRing::feed(const void* in, uint64_t nitems_read, int n)
{
    const uint64_t end0 = nitems_read + static_cast<uint64_t>(std::max(n, 0));
    {
        // the common case of a ring shared by many blocks: another feeder pushed these
        // items already (the same stream check as below, without the push lock)
        std::lock_guard<std::mutex> lk(d_mu);
        if (d_started && d_head >= end0 && nitems_read <= d_head)
            {
                if (d_head > 0 && d_head - 1 >= nitems_read && d_head - 1 < end0 &&
                    std::memcmp(static_cast<const uint8_t*>(in) + (d_head - 1 - nitems_read) * d_item_bytes, d_last,
                        d_item_bytes) != 0)
                    throw std::logic_error(
                        "DeviceIqRing::feed: two input streams under one ring key (<role>.mi355x_ring)");
                return;
            }
    }
    std::lock_guard<std::mutex> push_lk(d_push_mu);
    const uint64_t end = nitems_read + static_cast<uint64_t>(std::max(n, 0));
    const auto* bytes = static_cast<const uint8_t*>(in);
    const uint64_t half = std::max<uint64_t>(1, d_window / 2);
    for (;;)
        {
            uint64_t from, head;
            std::vector<Hook> hooks;
            {
                std::lock_guard<std::mutex> lk(d_mu);
                if (!d_started)
                    {
                        if (n <= 0) return;
                        d_started = true;
                        d_head = nitems_read;
                    }
                if (nitems_read > d_head)
                    throw std::logic_error("DeviceIqRing::feed: the stream skipped items no consumer has pushed");
                // items this feeder shares with the last push must be the same items
                if (d_head > 0 && d_head - 1 >= nitems_read && d_head - 1 < end &&
                    std::memcmp(bytes + (d_head - 1 - nitems_read) * d_item_bytes, d_last, d_item_bytes) != 0)
                    throw std::logic_error(
                        "DeviceIqRing::feed: two input streams under one ring key (<role>.mi355x_ring)");
                if (d_head >= end) return;
                const uint64_t len = std::min(half, end - d_head);
                if (gsdr_stream_push(d_ring, bytes + (d_head - nitems_read) * d_item_bytes, d_head, len) != GSDR_OK)
                    throw std::runtime_error(std::string("DeviceIqRing::feed: ") + gsdr_last_error());
                from = d_head;
                d_head += len;
                std::memcpy(d_last, bytes + (d_head - 1 - nitems_read) * d_item_bytes, d_item_bytes);
                head = d_head;
                for (const auto& kv : d_hooks) hooks.push_back(kv.second);
            }
            // the consumers keep up with the new head (outside the ring's lock: a hook
            // launches on the ring, and a pool's own feed may have called this)
            for (const auto& h : hooks) h(from, head);
        }
}
