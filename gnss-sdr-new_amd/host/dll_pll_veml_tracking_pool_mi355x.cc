#include "dll_pll_veml_tracking_pool_mi355x.h"

#include <algorithm>
#include <cstdlib>
#include <iostream>
#include <map>
#include <stdexcept>
#include <tuple>

#include "gnss_replicas.h"

namespace
{
std::runtime_error gsdr_error(const char* what) { return std::runtime_error(std::string(what) + ": " + gsdr_last_error()); }
}  // namespace

SharedTrackingPool::SharedTrackingPool(const Dll_Pll_Conf& conf, int32_t signal, uint32_t max_channels, int device,
    uint32_t window_calls, uint32_t batch_calls, const std::string& ring_key)
    : d_conf(conf), d_signal(signal), d_max(max_channels), d_device(device)
{
    const gsdr_trk_conf c = d_conf.to_engine(signal, max_channels);
    if (gsdr_trk_create(device, &c, &d_engine) != GSDR_OK) throw gsdr_error("SharedTrackingPool");
    // the newest window the channels' calls are read from (window_calls vector
    // lengths, twice that of ring positions); the pool advances every channel
    // whenever half a window arrived, so a channel is never more than that behind
    // the head, and a channel started by a block whose nitems_read lags the head by
    // up to the ring's extent still finds its items
    if (window_calls < 4)
        throw std::invalid_argument("SharedTrackingPool: mi355x_pool_window must be >= 4 vector lengths");
    if (batch_calls < 1 || batch_calls > window_calls / 2)
        throw std::invalid_argument("SharedTrackingPool: mi355x_pool_batch must be in [1, mi355x_pool_window / 2]");
    d_window = static_cast<uint64_t>(window_calls) * d_conf.vector_length;
    d_batch = static_cast<uint64_t>(batch_calls) * d_conf.vector_length;
    try
        {
            d_ring = DeviceIqRing::get(device, c.item_type, d_window, ring_key);
        }
    catch (...)
        {
            gsdr_trk_destroy(d_engine);
            throw;
        }
    d_used.assign(max_channels, false);
    d_active.assign(max_channels, false);
    d_gen.assign(max_channels, 0);
    // one submission covers every call a channel can have in the ring: a channel is
    // advanced whenever half a window arrived, so it never lags the head by more
    d_epochs = window_calls + 2;
    d_queue.resize(max_channels);
    d_n.assign(max_channels, 0);
    d_hook = d_ring->add_hook([this](uint64_t from, uint64_t head) { on_pushed(from, head); });
}

SharedTrackingPool::~SharedTrackingPool()
{
    d_ring->remove_hook(d_hook);
    d_recs.resize(static_cast<size_t>(d_max) * d_epochs);
    for (; !d_sub_gens.empty(); d_sub_gens.pop_front())
        {
            uint32_t me = 0;
            (void)gsdr_trk_collect(d_engine, 1, d_recs.data(), d_n.data(), &me);
        }
    gsdr_trk_destroy(d_engine);
}

std::shared_ptr<SharedTrackingPool> SharedTrackingPool::get(const std::string& key, const Dll_Pll_Conf& conf,
    int32_t signal, uint32_t max_channels, int device, uint32_t window_calls, uint32_t batch_calls,
    const std::string& ring_key)
{
    static std::mutex mu;
    static std::map<std::tuple<std::string, int, int32_t>, std::weak_ptr<SharedTrackingPool>> registry;
    std::lock_guard<std::mutex> lk(mu);
    auto& w = registry[std::make_tuple(key, device, signal)];
    if (auto p = w.lock()) return p;
    auto p = std::make_shared<SharedTrackingPool>(conf, signal, max_channels, device, window_calls, batch_calls, ring_key);
    w = p;
    return p;
}

int SharedTrackingPool::acquire_slot()
{
    std::lock_guard<std::mutex> lk(d_mu);
    for (uint32_t s = 0; s < d_max; ++s)
        if (!d_used[s])
            {
                d_used[s] = true;
                return static_cast<int>(s);
            }
    return -1;
}

void SharedTrackingPool::release_slot(int slot)
{
    std::lock_guard<std::mutex> lk(d_mu);
    if (slot < 0 || static_cast<uint32_t>(slot) >= d_max) return;
    gsdr_trk_stop(d_engine, slot);
    d_used[slot] = false;
    d_active[slot] = false;
    ++d_gen[slot];
    d_queue[slot].clear();
}

uint64_t SharedTrackingPool::start(int slot, uint32_t prn, const char signal[2], double acq_delay_samples,
    double acq_doppler_hz, uint64_t acq_samplestamp, uint64_t nitems_read)
{
    std::lock_guard<std::mutex> lk(d_mu);
    // the tracking replica of start_tracking (:661-700), as dll_pll_veml_tracking_mi355x
    std::vector<float> code;
    if (d_signal == GSDR_SIGNAL_GAL_1B)
        {
            const char sig[3] = {signal[0], signal[1], '\0'};
            code = galileo_e1_code_gen_sinboc11_float(d_conf.track_pilot ? "1C" : sig, prn);
            if (d_conf.track_pilot)
                {
                    const auto data = galileo_e1_code_gen_sinboc11_float(sig, prn);
                    if (gsdr_trk_set_data_code(d_engine, slot, data.data(), static_cast<int>(data.size())) != GSDR_OK)
                        throw gsdr_error("SharedTrackingPool::start");
                }
        }
    else if (d_signal == GSDR_SIGNAL_BDS_B1)
        code = beidou_b1i_code_gen_float(static_cast<int32_t>(prn), 0);
    else
        code = gps_l1_ca_code_gen_float(static_cast<int32_t>(prn), 0);
    uint64_t first = 0;
    if (gsdr_trk_start(d_engine, slot, prn, code.data(), static_cast<int>(code.size()), acq_delay_samples,
            acq_doppler_hz, acq_samplestamp, nitems_read, &first) != GSDR_OK)
        throw gsdr_error("SharedTrackingPool::start");
    d_queue[slot].clear();
    d_active[slot] = true;
    ++d_gen[slot];  // records of a submission in flight belong to the previous track
    return first;
}

void SharedTrackingPool::force_loss_of_lock(int slot)
{
    std::lock_guard<std::mutex> lk(d_mu);
    if (slot < 0 || static_cast<uint32_t>(slot) >= d_max) return;
    if (gsdr_trk_force_loss_of_lock(d_engine, slot) != GSDR_OK) throw gsdr_error("SharedTrackingPool::force_loss_of_lock");
}

void SharedTrackingPool::stop(int slot)
{
    std::lock_guard<std::mutex> lk(d_mu);
    if (slot < 0 || static_cast<uint32_t>(slot) >= d_max) return;
    gsdr_trk_stop(d_engine, slot);
    d_active[slot] = false;
    ++d_gen[slot];
    d_queue[slot].clear();
}

bool SharedTrackingPool::take_locked(bool wait)
{
    if (d_sub_gens.empty()) return true;
    d_recs.resize(static_cast<size_t>(d_max) * d_epochs);
    uint32_t me = 0;
    const int rc = gsdr_trk_collect(d_engine, wait ? 1 : 0, d_recs.data(), d_n.data(), &me);
    if (rc == 1) return false;  // still in flight
    const std::vector<uint32_t> gens = std::move(d_sub_gens.front());
    d_sub_gens.pop_front();
    if (rc != GSDR_OK) throw gsdr_error("SharedTrackingPool::advance");
    uint32_t most = 0;
    for (uint32_t c = 0; c < d_max; ++c)
        {
            most = std::max(most, d_n[c]);
            // a slot started or stopped since the submission: its records are stale
            if (!d_active[c] || d_gen[c] != gens[c]) continue;
            for (uint32_t e = 0; e < d_n[c]; ++e) d_queue[c].push_back(d_recs[static_cast<size_t>(c) * me + e]);
        }
    d_more = most >= me;  // a full batch: more calls may be ready in the ring
    return true;
}

void SharedTrackingPool::advance_locked(uint64_t head, bool wait)
{
    // two submissions in flight: the next launch queues behind the one running, so the
    // GPU does not idle while the host collects; collect the oldest before a third
    if (d_sub_gens.size() >= kInFlight) take_locked(true);
    for (;;)
        {
            // on the engine's stream, ordered after the ring's pushes and the launch in
            // flight; the records come back behind it while the host pushes and runs
            // the blocks
            if (gsdr_trk_submit_stream(d_engine, d_ring->stream(), d_epochs) != GSDR_OK)
                throw gsdr_error("SharedTrackingPool::advance");
            d_sub_gens.push_back(d_gen);
            ++d_launches;
            d_advanced = head;
            if (!wait) return;
            while (!d_sub_gens.empty()) take_locked(true);
            if (!d_more) return;
        }
}

void SharedTrackingPool::on_pushed(uint64_t from, uint64_t head)
{
    std::lock_guard<std::mutex> lk(d_mu);
    if (!d_seen)
        {
            d_seen = true;
            d_advanced = from;
        }
    // no started channel's next call may leave the ring: advance after half a window
    if (head - d_advanced >= d_window / 2) advance_locked(head, false);
}

void SharedTrackingPool::feed(const void* in, uint64_t nitems_read, int n)
{
    // without the pool's lock: the ring runs every pool's hook (this one's included)
    d_ring->feed(in, nitems_read, n);
}

void SharedTrackingPool::advance_if_due(bool force)
{
    std::lock_guard<std::mutex> lk(d_mu);
    uint64_t head = 0;
    if (!d_ring->head(&head)) return;
    if (!d_seen)
        {
            d_seen = true;
            d_advanced = head;
        }
    if (force)
        {
            if (head != d_advanced || d_more)
                advance_locked(head, true);
            else
                while (!d_sub_gens.empty()) take_locked(true);
            return;
        }
    if (head == d_advanced && !d_more) return;
    if (d_more || head - d_advanced >= d_batch) advance_locked(head, false);
}

namespace
{
uint64_t call_end(const gsdr_trk_epoch& r) { return r.sample_counter + static_cast<uint64_t>(std::max(r.consumed, 0)); }
}  // namespace

bool SharedTrackingPool::pop(int slot, uint64_t handed_end, gsdr_trk_epoch* rec)
{
    std::lock_guard<std::mutex> lk(d_mu);
    if (slot < 0 || d_queue[slot].empty() || call_end(d_queue[slot].front()) > handed_end) return false;
    *rec = d_queue[slot].front();
    d_queue[slot].pop_front();
    return true;
}

bool SharedTrackingPool::ready(int slot, uint64_t handed_end)
{
    std::lock_guard<std::mutex> lk(d_mu);
    return slot >= 0 && !d_queue[slot].empty() && call_end(d_queue[slot].front()) <= handed_end;
}

size_t SharedTrackingPool::queued(int slot)
{
    std::lock_guard<std::mutex> lk(d_mu);
    return slot < 0 ? 0 : d_queue[slot].size();
}

dll_pll_veml_tracking_pool_mi355x::dll_pll_veml_tracking_pool_mi355x(const Dll_Pll_Conf& conf, int32_t signal,
    uint32_t pool_channels, int device, const std::string& pool_key, uint32_t window_calls, uint32_t batch_calls,
    const std::string& ring_key)
    : d_conf(conf), d_signal(signal)
{
    if (d_conf.dump) d_dump.configure(d_conf.dump_filename);
    d_output = TrackingOutput(d_conf.fs_in, signal);
    d_pool = SharedTrackingPool::get(pool_key, conf, signal, pool_channels, device, window_calls, batch_calls, ring_key);
    d_slot = d_pool->acquire_slot();
    if (d_slot < 0)
        throw std::runtime_error("dll_pll_veml_tracking_pool_mi355x: every slot of pool '" + pool_key + "' is taken");
}

dll_pll_veml_tracking_pool_mi355x::~dll_pll_veml_tracking_pool_mi355x()
{
    d_pool->release_slot(d_slot);
    // the destructor's .dat close and save_matfile (:884-906)
    if (d_conf.dump && d_conf.dump_mat) d_dump.save_matfile();
}

void dll_pll_veml_tracking_pool_mi355x::set_gnss_synchro(Gnss_Synchro* p_gnss_synchro)
{
    std::lock_guard<std::mutex> l(d_setlock);
    d_acquisition_gnss_synchro = p_gnss_synchro;
}

void dll_pll_veml_tracking_pool_mi355x::set_channel(uint32_t channel)
{
    std::lock_guard<std::mutex> l(d_setlock);
    d_channel = channel;
    if (d_conf.dump) d_dump.open(channel);
}

void dll_pll_veml_tracking_pool_mi355x::start_tracking()
{
    std::lock_guard<std::mutex> l(d_setlock);
    if (!d_acquisition_gnss_synchro)
        throw std::logic_error("dll_pll_veml_tracking_pool_mi355x: set_gnss_synchro first");
    d_state = 1;
}

void dll_pll_veml_tracking_pool_mi355x::stop_tracking()
{
    std::lock_guard<std::mutex> l(d_setlock);
    d_state = 0;
    d_fault_pending = false;
    d_pool->stop(d_slot);
}

void dll_pll_veml_tracking_pool_mi355x::msg_handler_telemetry_to_trk(int tlm_event)
{
    if (tlm_event != 1) return;
    std::lock_guard<std::mutex> l(d_setlock);
    // as dll_pll_veml_tracking_mi355x: on the pool's channel while it tracks (the
    // records the pool already computed for this block precede the fault and are
    // handed out first), after the pull-in when one is pending
    try
        {
            if (d_state == 2)
                d_pool->force_loss_of_lock(d_slot);
            else if (d_state == 1)
                d_fault_pending = true;
        }
    catch (const std::exception& e)
        {
            std::cerr << "dll_pll_veml_tracking_pool_mi355x: " << e.what() << '\n';
        }
}

void dll_pll_veml_tracking_pool_mi355x::flush()
{
    std::lock_guard<std::mutex> l(d_setlock);
    try
        {
            d_pool->advance_if_due(true);
        }
    catch (const std::exception& e)
        {
            std::cerr << "dll_pll_veml_tracking_pool_mi355x: " << e.what() << '\n';
        }
}

int dll_pll_veml_tracking_pool_mi355x::work(const void* in, int ninput_items, uint64_t nitems_read, Gnss_Synchro* out,
    int* noutput, TrackingTags* tags)
{
    std::lock_guard<std::mutex> l(d_setlock);
    const int c = work_locked(in, ninput_items, nitems_read, out, noutput, tags);
    // the ring's pushes copy from the scheduler's buffer after feed() returned, and
    // the scheduler recycles consumed items (consume_each, :2119): consume only items
    // that landed in device memory.  An output is progress on its own (the scheduler
    // calls again); without one, wait for the copy rather than stall the scheduler
    if (c <= 0) return c;
    try
        {
            DeviceIqRing* ring = d_pool->ring();
            const uint64_t want = nitems_read + static_cast<uint64_t>(c);
            const uint64_t landed = ring->landed(want);
            if (landed >= want) return c;
            // the landed part is progress (the scheduler calls again for the rest)
            if (*noutput || landed > nitems_read) return static_cast<int>(landed > nitems_read ? landed - nitems_read : 0);
            ring->wait_landed(want);
        }
    catch (const std::exception& e)
        {
            std::cerr << "dll_pll_veml_tracking_pool_mi355x: " << e.what() << '\n';
        }
    return c;
}

int dll_pll_veml_tracking_pool_mi355x::work_locked(const void* in, int ninput_items, uint64_t nitems_read,
    Gnss_Synchro* out, int* noutput, TrackingTags* tags)
{
    *noutput = 0;
    if (tags) tags->has_out = false;
    const int n = std::max(ninput_items, 0);
    try
        {
            // the items handed over go into the pool's ring and are consumed; their
            // time tags wait for the calls that cover them
            d_pool->feed(in, nitems_read, n);
            // items not consumed are handed again with the next call: take each tag once
            const uint64_t from = std::max(nitems_read, d_handed_end);
            if (tags)
                for (int i = 0; i < tags->n_in; ++i)
                    if (tags->in[i].offset >= from && tags->in[i].offset < nitems_read + static_cast<uint64_t>(n))
                        d_tags.push_back(tags->in[i]);
            d_handed_end = std::max(d_handed_end, nitems_read + static_cast<uint64_t>(n));
            switch (d_state)
                {
                case 0:  // standby: consume at full throttle (:1806-1811)
                    d_tags.clear();
                    return n;
                case 1:
                    {
                        // pull-in (:1813-1844): the channel aligns to the next code start
                        // after nitems_read on the device
                        const Gnss_Synchro* g = d_acquisition_gnss_synchro;
                        d_pool->start(d_slot, g->PRN, g->Signal, g->Acq_delay_samples, g->Acq_doppler_hz,
                            g->Acq_samplestamp_samples, nitems_read);
                        if (d_conf.dump)
                            d_dump.set_acquisition(g->PRN,
                                TrackingDump::pull_in_code_phase(d_signal, d_conf.fs_in, nitems_read,
                                    g->Acq_samplestamp_samples, g->Acq_delay_samples),
                                g->Acq_doppler_hz);
                        d_state = 2;
                        if (d_fault_pending)
                            {
                                d_fault_pending = false;
                                d_pool->force_loss_of_lock(d_slot);
                            }
                        return n;
                    }
                default:
                    break;
                }
            d_pool->advance_if_due(false);
        }
    catch (const std::exception& e)
        {
            // device error -> loss of lock, the reference's failure convention; the
            // slot leaves the engine so later advances stop queueing its records
            std::cerr << "dll_pll_veml_tracking_pool_mi355x: " << e.what() << '\n';
            try
                {
                    d_pool->stop(d_slot);
                }
            catch (const std::exception& e2)
                {
                    std::cerr << "dll_pll_veml_tracking_pool_mi355x: stop after error: " << e2.what() << '\n';
                }
            d_state = 0;
            if (d_events) d_events(3);
            return n;
        }
    // hand out this channel's computed calls in order, up to the first that emits;
    // only calls inside the items handed over so far (their time tags are here)
    gsdr_trk_epoch rec;
    uint64_t last_end = 0;
    while (d_state == 2 && d_pool->pop(d_slot, d_handed_end, &rec))
        {
            d_last = rec;
            if (d_record_sink) d_record_sink(rec);
            if (d_conf.dump) d_dump.write(rec, d_conf.fs_in, d_signal == GSDR_SIGNAL_GAL_1B, d_conf.track_pilot);
            const bool loss_of_lock = (rec.flags & GSDR_TRK_F_LOSS_OF_LOCK) != 0;
            if (d_output.emit(rec, *d_acquisition_gnss_synchro, rec.sample_counter, out)) *noutput = 1;
            // the call's time tags: those on [sample_counter, sample_counter + consumed)
            const uint64_t end = rec.sample_counter + static_cast<uint64_t>(std::max(rec.consumed, 0));
            d_in_call.clear();  // a member: no allocation per call
            while (!d_tags.empty() && d_tags.front().offset < end)
                {
                    if (d_tags.front().offset >= rec.sample_counter) d_in_call.push_back(d_tags.front());
                    d_tags.pop_front();
                }
            TrackingTags call_tags;
            call_tags.in = d_in_call.data();
            call_tags.n_in = static_cast<int>(d_in_call.size());
            d_output.call_tags(&call_tags, rec.sample_counter, rec.consumed, *noutput ? out : nullptr, d_nitems_written);
            if (tags && call_tags.has_out)
                {
                    tags->has_out = true;
                    tags->out = call_tags.out;
                }
            d_nitems_written += static_cast<uint64_t>(*noutput);
            last_end = end;
            if (loss_of_lock)
                {
                    if (rec.flags & GSDR_TRK_F_OVERRUN)
                        {
                            // not a signal loss: the channel started before the ring's oldest item
                            ++d_overruns;
                            std::cerr << "dll_pll_veml_tracking_pool_mi355x: channel " << d_channel << " call at "
                                      << rec.sample_counter << " fell out of the ring window ("
                                      << d_pool->window_items() << " items; raise <role>.mi355x_pool_window)\n";
                        }
                    d_state = 0;
                    d_tags.clear();
                    if (d_events) d_events(3);
                }
            if (*noutput) break;
        }
    // one output per call, as the reference (set_max_noutput_items(1), :131): while
    // computed calls wait behind the one emitted, consume only up to its end, so the
    // scheduler calls again (its items are still in the input) and the backlog is
    // handed out call by call instead of growing; otherwise every item handed over
    // is in the ring and is consumed
    if (*noutput && d_state == 2 && d_pool->ready(d_slot, d_handed_end))
        return static_cast<int>(std::min<uint64_t>(static_cast<uint64_t>(n), last_end > nitems_read ? last_end - nitems_read : 0));
    return n;
}
