#include "dll_pll_veml_tracking_pool_mi355x.h"

#include <algorithm>
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
    uint32_t window_calls)
    : d_conf(conf), d_signal(signal), d_max(max_channels), d_device(device)
{
    const gsdr_trk_conf c = d_conf.to_engine(signal, max_channels);
    if (gsdr_trk_create(device, &c, &d_engine) != GSDR_OK) throw gsdr_error("SharedTrackingPool");
    d_item_bytes = c.item_type == GSDR_ITEM_CSHORT ? 4 : (c.item_type == GSDR_ITEM_IBYTE ? 2 : 8);
    // the newest window every channel's next call must fall in: window_calls calls'
    // worth (default 8: four forecasts of slack behind the head), and twice that of
    // ring positions.  A block whose nitems_read lags the pool head by more (a
    // flowgraph buffer deeper than that) needs a larger <role>.mi355x_pool_window.
    if (window_calls < 4)
        throw std::invalid_argument("SharedTrackingPool: mi355x_pool_window must be >= 4 vector lengths");
    d_window = static_cast<uint64_t>(window_calls) * d_conf.vector_length;
    if (gsdr_stream_create(device, c.item_type, 2 * d_window, d_window, &d_ring) != GSDR_OK)
        {
            gsdr_trk_destroy(d_engine);
            throw gsdr_error("SharedTrackingPool ring");
        }
    d_used.assign(max_channels, false);
    d_active.assign(max_channels, false);
    d_queue.resize(max_channels);
    d_n.assign(max_channels, 0);
}

SharedTrackingPool::~SharedTrackingPool()
{
    gsdr_stream_destroy(d_ring);
    gsdr_trk_destroy(d_engine);
}

std::shared_ptr<SharedTrackingPool> SharedTrackingPool::get(const std::string& key, const Dll_Pll_Conf& conf,
    int32_t signal, uint32_t max_channels, int device, uint32_t window_calls)
{
    static std::mutex mu;
    static std::map<std::tuple<std::string, int, int32_t>, std::weak_ptr<SharedTrackingPool>> registry;
    std::lock_guard<std::mutex> lk(mu);
    auto& w = registry[std::make_tuple(key, device, signal)];
    if (auto p = w.lock()) return p;
    auto p = std::make_shared<SharedTrackingPool>(conf, signal, max_channels, device, window_calls);
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
    return first;
}

void SharedTrackingPool::stop(int slot)
{
    std::lock_guard<std::mutex> lk(d_mu);
    if (slot < 0 || static_cast<uint32_t>(slot) >= d_max) return;
    gsdr_trk_stop(d_engine, slot);
    d_active[slot] = false;
    d_queue[slot].clear();
}

void SharedTrackingPool::advance_locked()
{
    const uint32_t me = 16;  // calls per channel per launch
    d_recs.resize(static_cast<size_t>(d_max) * me);
    for (;;)
        {
            if (gsdr_trk_run_stream_host(d_engine, d_ring, me, d_recs.data(), d_n.data()) != GSDR_OK)
                throw gsdr_error("SharedTrackingPool::advance");
            ++d_launches;
            uint32_t most = 0;
            for (uint32_t c = 0; c < d_max; ++c)
                {
                    most = std::max(most, d_n[c]);
                    if (!d_active[c]) continue;
                    for (uint32_t e = 0; e < d_n[c]; ++e) d_queue[c].push_back(d_recs[static_cast<size_t>(c) * me + e]);
                }
            if (most < me) break;  // a full batch: more calls may be ready in the ring
        }
}

void SharedTrackingPool::feed(const void* in, uint64_t nitems_read, int n, bool advance)
{
    std::lock_guard<std::mutex> lk(d_mu);
    const uint64_t end = nitems_read + static_cast<uint64_t>(std::max(n, 0));
    if (!d_started)
        {
            d_started = true;
            d_origin = d_head = nitems_read;
        }
    if (nitems_read > d_head)
        throw std::logic_error("SharedTrackingPool::feed: the stream skipped items no pooled block has seen");
    const auto* bytes = static_cast<const uint8_t*>(in);
    // chunks of half the window, the channels advanced after each, so no active
    // channel falls out of the ring's newest window
    const uint64_t chunk = std::max<uint64_t>(1, d_window / 2);
    bool pushed = false;
    while (d_head < end)
        {
            const uint64_t len = std::min(chunk, end - d_head);
            if (gsdr_stream_push(d_ring, bytes + (d_head - nitems_read) * d_item_bytes, d_head, len) != GSDR_OK)
                throw gsdr_error("SharedTrackingPool::feed");
            d_head += len;
            pushed = true;
            if (advance) advance_locked();
        }
    if (advance && !pushed) advance_locked();
}

bool SharedTrackingPool::peek(int slot, gsdr_trk_epoch* rec)
{
    std::lock_guard<std::mutex> lk(d_mu);
    if (slot < 0 || d_queue[slot].empty()) return false;
    *rec = d_queue[slot].front();
    return true;
}

void SharedTrackingPool::drop(int slot)
{
    std::lock_guard<std::mutex> lk(d_mu);
    if (slot >= 0 && !d_queue[slot].empty()) d_queue[slot].pop_front();
}

dll_pll_veml_tracking_pool_mi355x::dll_pll_veml_tracking_pool_mi355x(const Dll_Pll_Conf& conf, int32_t signal,
    uint32_t pool_channels, int device, const std::string& pool_key, uint32_t window_calls)
    : d_conf(conf), d_signal(signal)
{
    if (d_conf.dump) d_dump.configure(d_conf.dump_filename);
    d_pool = SharedTrackingPool::get(pool_key, conf, signal, pool_channels, device, window_calls);
    d_slot = d_pool->acquire_slot();
    if (d_slot < 0)
        throw std::runtime_error("dll_pll_veml_tracking_pool_mi355x: every slot of pool '" + pool_key + "' is taken");
}

dll_pll_veml_tracking_pool_mi355x::~dll_pll_veml_tracking_pool_mi355x() { d_pool->release_slot(d_slot); }

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
    d_pool->stop(d_slot);
}

int dll_pll_veml_tracking_pool_mi355x::work(const void* in, int ninput_items, uint64_t nitems_read, Gnss_Synchro* out,
    int* noutput)
{
    std::lock_guard<std::mutex> l(d_setlock);
    *noutput = 0;
    try
        {
            switch (d_state)
                {
                case 0:  // standby: consume at full throttle (:1806-1811), keeping the ring gap-free
                    d_pool->feed(in, nitems_read, ninput_items, false);
                    return ninput_items;
                case 1:
                    {
                        // pull-in (:1813-1844): align to the next code start after nitems_read
                        const Gnss_Synchro* g = d_acquisition_gnss_synchro;
                        d_pool->feed(in, nitems_read, ninput_items, false);
                        const uint64_t first = d_pool->start(d_slot, g->PRN, g->Signal, g->Acq_delay_samples,
                            g->Acq_doppler_hz, g->Acq_samplestamp_samples, nitems_read);
                        if (d_conf.dump)
                            d_dump.set_acquisition(g->PRN,
                                TrackingDump::pull_in_code_phase(d_signal, d_conf.fs_in, nitems_read,
                                    g->Acq_samplestamp_samples, g->Acq_delay_samples),
                                g->Acq_doppler_hz);
                        d_state = 2;
                        return static_cast<int>(first - nitems_read);
                    }
                default:
                    break;
                }
            gsdr_trk_epoch rec;
            if (!d_pool->peek(d_slot, &rec))
                {
                    d_pool->feed(in, nitems_read, ninput_items, true);
                    if (!d_pool->peek(d_slot, &rec)) return 0;  // the call needs more items
                }
            // a block consumes at most what the scheduler handed it: a call computed
            // from items other blocks pushed waits until this block is given them
            if (rec.sample_counter == nitems_read && rec.consumed > ninput_items) return 0;
            d_pool->drop(d_slot);
            d_last = rec;
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
            return 0;
        }
    if (d_last.sample_counter != nitems_read)
        {
            // the record belongs to another position than the scheduler's: a desync
            // (items dropped upstream); report it as a loss of lock
            std::cerr << "dll_pll_veml_tracking_pool_mi355x: record at " << d_last.sample_counter << ", input at "
                      << nitems_read << '\n';
            d_pool->stop(d_slot);
            d_state = 0;
            if (d_events) d_events(3);
            return 0;
        }
    if (d_conf.dump) d_dump.write(d_last, d_conf.fs_in, d_signal == GSDR_SIGNAL_GAL_1B, d_conf.track_pilot);
    const bool loss_of_lock = (d_last.flags & GSDR_TRK_F_LOSS_OF_LOCK) != 0;
    if ((d_last.flags & GSDR_TRK_F_VALID_OUTPUT) || loss_of_lock)
        {
            // output record (:2000-2017, :2120-2127)
            Gnss_Synchro s = *d_acquisition_gnss_synchro;
            s.Prompt_I = d_last.prompt_i;
            s.Prompt_Q = d_last.prompt_q;
            s.Code_phase_samples = d_last.rem_code_phase_samples;
            s.Carrier_phase_rads = d_last.acc_carrier_phase_rad;
            s.Carrier_Doppler_hz = d_last.carrier_doppler_hz;
            s.CN0_dB_hz = d_last.cn0_db_hz;
            s.EVM = d_last.evm;
            s.fs = static_cast<int64_t>(d_conf.fs_in);
            s.Tracking_sample_counter = nitems_read;
            s.Flag_valid_symbol_output = !loss_of_lock;
            s.Flag_PLL_180_deg_phase_locked = (d_last.flags & GSDR_TRK_F_PLL_180) != 0;
            *out = s;
            *noutput = 1;
        }
    if (loss_of_lock)
        {
            if (d_last.flags & GSDR_TRK_F_OVERRUN)
                {
                    // not a signal loss: the call fell out of the pool's ring window
                    ++d_overruns;
                    std::cerr << "dll_pll_veml_tracking_pool_mi355x: channel " << d_channel << " call at "
                              << d_last.sample_counter << " fell out of the ring window (" << d_pool->window_items()
                              << " items behind the newest pushed; raise <role>.mi355x_pool_window)\n";
                }
            d_state = 0;
            if (d_events) d_events(3);
        }
    return d_last.consumed;
}
