#include "tracking_pool.h"

#include <stdexcept>
#include <string>

#include "gnss_replicas.h"

TrackingPool::TrackingPool(const Dll_Pll_Conf& conf, int32_t signal, uint32_t max_channels, gsdr_stream* ring, int device)
    : d_conf(conf), d_signal(signal), d_max(max_channels), d_ring(ring)
{
    const gsdr_trk_conf c = d_conf.to_engine(signal, max_channels);
    if (gsdr_trk_create(device, &c, &d_engine) != GSDR_OK)
        throw std::runtime_error(std::string("TrackingPool: ") + gsdr_last_error());
    d_output = TrackingOutput(d_conf.fs_in, signal);
    d_synchro.assign(max_channels, nullptr);
    d_n.assign(max_channels, 0);
}

TrackingPool::~TrackingPool() { gsdr_trk_destroy(d_engine); }

void TrackingPool::start(uint32_t slot, Gnss_Synchro* gs, uint64_t nitems_read)
{
    if (slot >= d_max || !gs) throw std::invalid_argument("TrackingPool::start: bad slot or Gnss_Synchro");
    std::vector<float> code;
    if (d_signal == GSDR_SIGNAL_GAL_1B)
        {
            const char sig[3] = {gs->Signal[0], gs->Signal[1], '\0'};
            code = galileo_e1_code_gen_sinboc11_float(d_conf.track_pilot ? "1C" : sig, gs->PRN);
            if (d_conf.track_pilot)
                {
                    const auto data = galileo_e1_code_gen_sinboc11_float(sig, gs->PRN);
                    if (gsdr_trk_set_data_code(d_engine, static_cast<int>(slot), data.data(), static_cast<int>(data.size())) !=
                        GSDR_OK)
                        throw std::runtime_error(std::string("TrackingPool: ") + gsdr_last_error());
                }
        }
    else if (d_signal == GSDR_SIGNAL_BDS_B1)
        code = beidou_b1i_code_gen_float(static_cast<int32_t>(gs->PRN));
    else
        code = gps_l1_ca_code_gen_float(static_cast<int32_t>(gs->PRN));
    uint64_t first = 0;
    if (gsdr_trk_start(d_engine, static_cast<int>(slot), gs->PRN, code.data(), static_cast<int>(code.size()),
            gs->Acq_delay_samples, gs->Acq_doppler_hz, gs->Acq_samplestamp_samples, nitems_read, &first) != GSDR_OK)
        throw std::runtime_error(std::string("TrackingPool: ") + gsdr_last_error());
    d_synchro[slot] = gs;
}

void TrackingPool::stop(uint32_t slot)
{
    if (slot < d_max) gsdr_trk_stop(d_engine, static_cast<int>(slot));
    if (slot < d_max) d_synchro[slot] = nullptr;
}

uint64_t TrackingPool::advance(const Output& out, uint32_t max_epochs)
{
    d_recs.resize(static_cast<size_t>(d_max) * max_epochs);
    uint64_t calls = 0;
    for (;;)
        {
            if (gsdr_trk_run_stream_host(d_engine, d_ring, max_epochs, d_recs.data(), d_n.data()) != GSDR_OK)
                throw std::runtime_error(std::string("TrackingPool: ") + gsdr_last_error());
            uint32_t most = 0;
            for (uint32_t c = 0; c < d_max; ++c)
                {
                    most = std::max(most, d_n[c]);
                    calls += d_n[c];
                    for (uint32_t e = 0; e < d_n[c]; ++e)
                        {
                            const gsdr_trk_epoch& r = d_recs[static_cast<size_t>(c) * max_epochs + e];
                            Gnss_Synchro s;
                            if (!d_synchro[c] || !d_output.emit(r, *d_synchro[c], r.sample_counter, &s)) continue;
                            out(c, s);
                        }
                }
            // a full batch of records: more calls may be ready in the ring
            if (most < max_epochs) break;
        }
    return calls;
}
