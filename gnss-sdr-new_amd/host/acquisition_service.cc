#include "acquisition_service.h"

#include "pcps_acquisition_mi355x.h"

#include <algorithm>
#include <cstring>
#include <stdexcept>
#include <string>

AcquisitionService::AcquisitionService(const Acq_Conf& conf, uint32_t max_requests, int device, uint32_t batch_blocks)
    : d_conf(conf),
      d_max(max_requests),
      d_consumed(static_cast<uint32_t>(conf.sampled_ms * conf.samples_per_ms)),
      d_isz(conf.it_size),
      d_batch(batch_blocks ? batch_blocks : 1)
{
    if (max_requests == 0) throw std::invalid_argument("AcquisitionService: max_requests must be > 0");
    gsdr_acq_conf c{};
    c.fs_in = conf.resampled_fs ? conf.resampled_fs : conf.fs_in;
    c.consumed_samples = d_consumed;
    c.samples_per_code = conf.samples_per_code;
    c.samples_per_chip = conf.samples_per_chip;
    c.doppler_max = conf.doppler_max;
    c.doppler_step = static_cast<uint32_t>(conf.doppler_step);
    c.pfa = conf.use_CFAR_algorithm_flag ? conf.pfa : 0.0F;
    c.max_dwells = 1;
    c.item_type = pcps_acquisition_mi355x::engine_item_type(conf.item_type);
    c.max_prns = max_requests;
    c.max_blocks = d_batch;
    c.sampled_ms = conf.sampled_ms;
    c.ms_per_code = conf.ms_per_code;
    if (gsdr_acq_create(device, &c, &d_engine) != GSDR_OK)
        throw std::runtime_error(std::string("AcquisitionService: ") + gsdr_last_error());
    // the configuration's carrier model, whatever GSDR_ACQ_WIPE says
    if (gsdr_acq_set_wipeoff(d_engine, conf.wipeoff_mode()) != GSDR_OK)
        throw std::runtime_error(std::string("AcquisitionService: ") + gsdr_last_error());
    gsdr_acq_get_threshold(d_engine, &d_threshold);
    d_buffer.resize(static_cast<size_t>(d_consumed) * d_isz);
    d_slots.resize(max_requests);
    d_res.resize(static_cast<size_t>(d_batch) * max_requests);
}

AcquisitionService::~AcquisitionService()
{
    for (; !d_flights.empty(); d_flights.pop_front())
        {
            uint32_t nb = 0, np = 0;
            gsdr_acq_collect(d_engine, d_res.data(), &nb, &np);
        }
    gsdr_acq_destroy(d_engine);
}

void AcquisitionService::request(uint32_t channel, uint32_t prn, const std::complex<float>* code, Callback done)
{
    std::lock_guard<std::mutex> lk(d_mu);
    Slot* s = nullptr;
    for (auto& x : d_slots)
        if (x.used && x.channel == channel) s = &x;
    if (!s)
        {
            // a free slot, preferably one still holding this PRN's spectrum
            for (auto& x : d_slots)
                if (!x.used && (!s || (x.loaded && x.prn == prn && !(s->loaded && s->prn == prn)))) s = &x;
            if (!s) throw std::length_error("AcquisitionService: more requests than max_requests");
            s->used = true;
            s->channel = channel;
        }
    if (!s->loaded || s->prn != prn)
        {
            s->prn = prn;
            s->loaded = false;
            s->code.assign(code, code + d_consumed);
        }
    s->armed = true;
    s->done = std::move(done);
}

void AcquisitionService::cancel(uint32_t channel)
{
    std::lock_guard<std::mutex> lk(d_mu);
    for (auto& x : d_slots)
        if (x.used && x.channel == channel)
            {
                x.used = false;
                x.armed = false;
                x.done = nullptr;
            }
}

size_t AcquisitionService::pending() const
{
    std::lock_guard<std::mutex> lk(d_mu);
    size_t n = 0;
    for (const auto& x : d_slots) n += x.armed ? 1 : 0;
    return n;
}

bool AcquisitionService::prepare_locked(std::vector<uint64_t>& gen)
{
    uint32_t top = 0;
    for (uint32_t i = 0; i < d_max; ++i)
        {
            Slot& s = d_slots[i];
            if (!s.armed) continue;
            top = i + 1;
            if (!s.loaded)
                {
                    // set_local_code (pcps_acquisition.cc:176-209) for this slot only
                    if (gsdr_acq_set_local_code(d_engine, i, reinterpret_cast<const float*>(s.code.data()), s.prn) != GSDR_OK)
                        throw std::runtime_error(std::string("AcquisitionService: ") + gsdr_last_error());
                    s.loaded = true;
                    ++s.gen;
                    ++d_code_uploads;
                    std::vector<std::complex<float>>().swap(s.code);
                }
        }
    if (top == 0) return false;
    // slots below the highest armed one without a spectrum yet (never requested)
    // are searched with whatever they hold and not answered
    if (gsdr_acq_set_active_prns(d_engine, top) != GSDR_OK)
        throw std::runtime_error(std::string("AcquisitionService: ") + gsdr_last_error());
    gen.resize(top);
    for (uint32_t i = 0; i < top; ++i) gen[i] = d_slots[i].loaded ? d_slots[i].gen : ~0ULL;
    return true;
}

void AcquisitionService::answer(const std::vector<gsdr_acq_result>& res, uint32_t nblocks, uint32_t nprn,
    const std::vector<uint64_t>& gen, bool device_error)
{
    struct Ans
    {
        uint32_t channel;
        Callback done;
        gsdr_acq_result r;
        bool positive;
    };
    std::vector<Ans> ans;
    for (uint32_t b = 0; b < nblocks; ++b)
        {
            ans.clear();
            {
                std::lock_guard<std::mutex> lk(d_mu);
                for (uint32_t i = 0; i < nprn && i < d_max; ++i)
                    {
                        Slot& s = d_slots[i];
                        // answered by this block when armed with the spectrum the launch used
                        if (!s.armed || !s.loaded || s.gen != gen[i]) continue;
                        s.armed = false;
                        if (device_error)
                            {
                                // device failure: a negative acquisition, the reference's failure convention
                                gsdr_acq_result r{};
                                r.prn = s.prn;
                                ans.push_back({s.channel, s.done, r, false});
                            }
                        else
                            {
                                const gsdr_acq_result& r = res[static_cast<size_t>(b) * nprn + i];
                                ans.push_back({s.channel, s.done, r, r.test_statistic > d_threshold});
                            }
                    }
            }
            // callbacks outside the lock: they may re-arm (same PRN: answered by the
            // next block of this launch)
            for (auto& a : ans)
                if (a.done) a.done(a.channel, a.r, a.positive);
            if (device_error) break;
        }
}

int AcquisitionService::work(const void* in, int ninput_items)
{
    const auto* src = static_cast<const uint8_t*>(in);
    int used = 0;
    while (used < ninput_items)
        {
            const uint32_t take = std::min<uint32_t>(static_cast<uint32_t>(ninput_items - used), d_consumed - d_fill);
            std::memcpy(d_buffer.data() + static_cast<size_t>(d_fill) * d_isz, src + static_cast<size_t>(used) * d_isz,
                static_cast<size_t>(take) * d_isz);
            d_fill += take;
            used += static_cast<int>(take);
            d_sample_counter += take;
            if (d_fill == d_consumed)
                {
                    d_fill = 0;
                    std::vector<uint64_t> gen;
                    bool any;
                    {
                        std::lock_guard<std::mutex> lk(d_mu);
                        any = prepare_locked(gen);
                    }
                    if (!any) continue;
                    const auto nprn = static_cast<uint32_t>(gen.size());
                    // sample stamp: the counter after the block (pcps_acquisition.cc:1009, :1019)
                    const int rc = gsdr_acq_run(d_engine, d_buffer.data(), 1, d_sample_counter, d_res.data());
                    ++d_grids;
                    ++d_launches;
                    answer(d_res, 1, nprn, gen, rc != GSDR_OK);
                }
        }
    return used;
}

void AcquisitionService::collect_oldest()
{
    const Flight f = std::move(d_flights.front());
    d_flights.pop_front();
    uint32_t nb = 0, np = 0;
    const int rc = gsdr_acq_collect(d_engine, d_res.data(), &nb, &np);
    answer(d_res, rc == GSDR_OK ? nb : 1, rc == GSDR_OK ? np : static_cast<uint32_t>(f.gen.size()), f.gen, rc != GSDR_OK);
}

void AcquisitionService::flush()
{
    while (!d_flights.empty()) collect_oldest();
}

int AcquisitionService::work_ring(gsdr_stream* ring, uint64_t head)
{
    if (!d_ring_started)
        {
            d_ring_started = true;
            d_ring_cursor = head;
            d_sample_counter = head;
            return 0;
        }
    const uint64_t ready = head > d_ring_cursor ? (head - d_ring_cursor) / d_consumed : 0;
    if (ready < d_batch) return 0;  // a full batch of blocks per launch
    int blocks = 0;
    // blocks the ring no longer holds (the caller pushed past them) are skipped
    uint64_t span_first = 0, span_n = 0;
    if (gsdr_stream_span(ring, &span_first, &span_n) == GSDR_OK && span_first > d_ring_cursor)
        {
            const uint64_t skip = (span_first - d_ring_cursor + d_consumed - 1) / d_consumed;
            d_ring_cursor += skip * d_consumed;
            d_sample_counter = d_ring_cursor;
        }
    uint64_t left = head > d_ring_cursor ? (head - d_ring_cursor) / d_consumed : 0;
    while (left >= d_batch)
        {
            const uint32_t nb = d_batch;
            // two launches in flight: answer the oldest before a third (its answers
            // re-arm requests)
            if (d_flights.size() >= kMaxFlights) collect_oldest();
            Flight f;
            f.nblocks = nb;
            bool any;
            {
                std::lock_guard<std::mutex> lk(d_mu);
                any = prepare_locked(f.gen);
            }
            if (any)
                {
                    // sample stamps: the counter after each block (pcps_acquisition.cc:1009, :1019)
                    const int rc = gsdr_acq_submit_stream(d_engine, ring, d_ring_cursor, nb, d_ring_cursor + d_consumed);
                    ++d_launches;
                    d_grids += nb;
                    if (rc != GSDR_OK)
                        answer(d_res, 1, static_cast<uint32_t>(f.gen.size()), f.gen, true);
                    else
                        d_flights.push_back(std::move(f));
                }
            d_ring_cursor += static_cast<uint64_t>(nb) * d_consumed;
            d_sample_counter = d_ring_cursor;
            blocks += static_cast<int>(nb);
            left -= nb;
        }
    return blocks;
}
