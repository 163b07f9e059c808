#include "acquisition_service.h"

#include "pcps_acquisition_mi355x.h"

#include <algorithm>
#include <cstring>
#include <stdexcept>
#include <string>

AcquisitionService::AcquisitionService(const Acq_Conf& conf, uint32_t max_requests, int device)
    : d_conf(conf),
      d_max(max_requests),
      d_consumed(static_cast<uint32_t>(conf.sampled_ms * conf.samples_per_ms)),
      d_isz(conf.it_size)
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
    c.max_blocks = 1;
    c.sampled_ms = conf.sampled_ms;
    c.ms_per_code = conf.ms_per_code;
    if (gsdr_acq_create(device, &c, &d_engine) != GSDR_OK)
        throw std::runtime_error(std::string("AcquisitionService: ") + gsdr_last_error());
    if (conf.wipeoff_mode() != GSDR_WIPE_EXACT && gsdr_acq_set_wipeoff(d_engine, conf.wipeoff_mode()) != GSDR_OK)
        throw std::runtime_error(std::string("AcquisitionService: ") + gsdr_last_error());
    gsdr_acq_get_threshold(d_engine, &d_threshold);
    d_buffer.resize(static_cast<size_t>(d_consumed) * d_isz);
}

AcquisitionService::~AcquisitionService() { gsdr_acq_destroy(d_engine); }

void AcquisitionService::request(uint32_t channel, uint32_t prn, const std::complex<float>* code, Callback done)
{
    std::lock_guard<std::mutex> lk(d_mu);
    auto it = std::find_if(d_requests.begin(), d_requests.end(), [&](const Request& r) { return r.channel == channel; });
    Request r{channel, prn, std::vector<std::complex<float>>(code, code + d_consumed), std::move(done)};
    if (it != d_requests.end())
        *it = std::move(r);
    else
        {
            if (d_requests.size() >= d_max) throw std::length_error("AcquisitionService: more requests than max_requests");
            d_requests.push_back(std::move(r));
        }
    d_codes_dirty = true;
}

void AcquisitionService::cancel(uint32_t channel)
{
    std::lock_guard<std::mutex> lk(d_mu);
    const auto n = d_requests.size();
    d_requests.erase(std::remove_if(d_requests.begin(), d_requests.end(),
                         [&](const Request& r) { return r.channel == channel; }),
        d_requests.end());
    if (d_requests.size() != n) d_codes_dirty = true;
}

size_t AcquisitionService::pending() const
{
    std::lock_guard<std::mutex> lk(d_mu);
    return d_requests.size();
}

// One batched acquisition_core over all pending requests; each request is
// answered once (the channel re-arms it for another attempt, as the channel FSM
// re-arms its acquisition block after a negative result).
void AcquisitionService::run_grid(gsdr_stream* ring, uint64_t first_sample)
{
    std::vector<Request> reqs;
    {
        std::lock_guard<std::mutex> lk(d_mu);
        if (d_requests.empty()) return;
        const uint32_t P = static_cast<uint32_t>(d_requests.size());
        if (d_codes_dirty)
            {
                std::vector<std::complex<float>> codes(static_cast<size_t>(P) * d_consumed);
                std::vector<uint32_t> prns(P);
                for (uint32_t i = 0; i < P; ++i)
                    {
                        std::copy(d_requests[i].code.begin(), d_requests[i].code.end(), codes.begin() + static_cast<size_t>(i) * d_consumed);
                        prns[i] = d_requests[i].prn;
                    }
                if (gsdr_acq_set_local_codes(d_engine, reinterpret_cast<const float*>(codes.data()), prns.data(), P) != GSDR_OK)
                    throw std::runtime_error(std::string("AcquisitionService: ") + gsdr_last_error());
                d_codes_dirty = false;
            }
        reqs.swap(d_requests);
        d_codes_dirty = true;
    }
    std::vector<gsdr_acq_result> res(reqs.size());
    // sample stamp: the counter after the block (pcps_acquisition.cc:1009, :1019)
    const int rc = ring ? gsdr_acq_run_stream(d_engine, ring, first_sample, 1, first_sample + d_consumed, res.data())
                        : gsdr_acq_run(d_engine, d_buffer.data(), 1, d_sample_counter, res.data());
    ++d_grids;
    for (size_t i = 0; i < reqs.size(); ++i)
        {
            if (rc != GSDR_OK)
                {
                    // device failure: a negative acquisition, the reference's failure convention
                    gsdr_acq_result r{};
                    r.prn = reqs[i].prn;
                    reqs[i].done(reqs[i].channel, r, false);
                }
            else
                reqs[i].done(reqs[i].channel, res[i], res[i].test_statistic > d_threshold);
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
                    run_grid();
                    d_fill = 0;
                }
        }
    return used;
}

int AcquisitionService::work_ring(gsdr_stream* ring, uint64_t head)
{
    if (!d_ring_started)
        {
            d_ring_started = true;
            d_ring_cursor = head;
            return 0;
        }
    int blocks = 0;
    while (d_ring_cursor + d_consumed <= head)
        {
            run_grid(ring, d_ring_cursor);
            d_ring_cursor += d_consumed;
            d_sample_counter = d_ring_cursor;
            ++blocks;
        }
    return blocks;
}
