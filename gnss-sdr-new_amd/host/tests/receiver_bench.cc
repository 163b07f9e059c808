// Throughput of the drop-in receiver path at configuration scale:
// the factory-built pooled TrackingInterface blocks (dll_pll_veml_tracking_pool_mi355x,
// the MI355X adapters' default) fed GNU-Radio style -- every block's work() with the
// items its upstream buffer holds at its own nitems_read -- beside AcquisitionService
// grids on the GPU's device IQ ring (host pushes), searching the PRNs that no channel
// tracks (each answer re-arms the request, as a receiver's idle channels keep
// searching).  The reference's shape: gnss_flowgraph.cc:1007-1135 (one tracking and
// one acquisition block per channel over the conditioner output).
//   receiver_bench c3|c5 [seconds] [search] [pinned] [pool batch] [lookahead] [threads]
// search 1 (default): the acquisition services search every untracked PRN of GPS
// and Galileo and BeiDou PRNs up to 32 on every block; 0: the tracking blocks only.
// pinned 1 (default): the host sample buffer is page-locked (gsdr_host_register), as
// a flowgraph's buffers would be for DMA; 0: pageable (a staging copy per push).
// lookahead L (default 0): the source runs L chunks ahead of what the blocks are offered,
// as a flowgraph's source thread fills its output buffer ahead of the consumers; with 0
// the blocks see every chunk the moment it is pushed, so the first block to reach it
// waits for its DMA (the push lifetime contract: consume only landed items).
// threads T (default 0): the tracking blocks' work() calls run on T threads (block i on
// thread i % T) beside the source thread that pushes and runs the acquisition services,
// as GNU Radio's thread-per-block scheduler runs them concurrently; the source keeps
// within 4 chunks of the slowest block (a bounded upstream buffer).  0: one thread,
// every block's work() after each push.
// Every consumer reads the GPU's one shared ring (DeviceIqRing, key "rf0"): each stretch of the
// stream crosses PCIe once.
// C3: GPS L1 C/A at 16 Msps, 12 tracked channels; C5: one GPU's share of the 25 Msps
// hybrid job, 12 GPS L1 C/A + 12 Galileo E1 (pilot) + 8 BeiDou B1I channels.
// Prints one JSON line: stream Msps through the whole receiver path (host loop,
// pushes, launches, records) and per-signal outputs / Doppler errors.
#include <algorithm>
#include <atomic>
#include <chrono>
#include <cmath>
#include <complex>
#include <cstdio>
#include <cstring>
#include <memory>
#include <string>
#include <thread>
#include <vector>

#include "acquisition_service.h"
#include "device_iq_ring.h"
#include "gnss_block_factory_mi355x.h"
#include "gnss_replicas.h"
#include "gnss_tracking_mi355x.h"
#include "synth_stream.h"

namespace
{
struct Sig
{
    const char* role;       // Tracking_<xx> / Acquisition_<xx>
    const char* impl_trk;
    const char* impl_acq;
    char sys;
    char s0, s1;
    int nch;                // tracked channels
    int nprn;               // PRNs of the constellation (the rest are searched)
    double chip_rate;       // chips/s
    double carrier;
    int code_ms;            // code period [ms]
};

std::vector<float> code_of(char sys, uint32_t prn)
{
    if (sys == 'E') return galileo_e1_code_gen_sinboc11_float("1B", prn);
    if (sys == 'C') return beidou_b1i_code_gen_float(static_cast<int32_t>(prn), 0);
    return gps_l1_ca_code_gen_float(static_cast<int32_t>(prn), 0);
}
}  // namespace

int main(int argc, char** argv)
{
    const std::string cfg = argc > 1 ? argv[1] : "c3";
    const bool c5 = cfg == "c5";
    const double fs = c5 ? 25.0e6 : 16.0e6;
    // >= 1.5 s: the pull-in transitory ends after 1 s (integer seconds,
    // dll_pll_veml_tracking.cc:1797), then bit / secondary-code sync and outputs
    const double seconds = argc > 2 ? std::atof(argv[2]) : 1.6;
    const bool search = argc > 3 ? std::atoi(argv[3]) != 0 : true;
    const bool pinned = argc > 4 ? std::atoi(argv[4]) != 0 : true;
    const int pool_batch = argc > 5 ? std::atoi(argv[5]) : 0;  // 0: the blocks' default
    const int lookahead = argc > 6 ? std::max(0, std::atoi(argv[6])) : 0;
    const int threads = argc > 7 ? std::max(0, std::atoi(argv[7])) : 0;
    std::vector<Sig> sigs = {{"1C", "GPS_L1_CA_DLL_PLL_Tracking_MI355X", "GPS_L1_CA_PCPS_Acquisition_MI355X", 'G', '1',
        'C', 12, 32, 1.023e6, 1575.42e6, 1}};
    if (c5)
        {
            sigs.push_back({"1B", "Galileo_E1_DLL_PLL_VEML_Tracking_MI355X", "Galileo_E1_PCPS_Ambiguous_Acquisition_MI355X",
                'E', '1', 'B', 12, 36, 1.023e6, 1575.42e6, 4});
            sigs.push_back({"B1", "BEIDOU_B1I_DLL_PLL_Tracking_MI355X", "BEIDOU_B1I_PCPS_Acquisition_MI355X", 'C', 'B',
                '1', 8, 63, 2.046e6, 1561.098e6, 1});
        }
    // the stream: every tracked satellite at 45 dB-Hz, seeded delays and Dopplers
    const size_t n = static_cast<size_t>(fs * seconds);
    const double sigma = 1.0;
    const double amp = std::sqrt(2.0 * std::pow(10.0, 4.5) / fs) * sigma;
    std::mt19937 gen(42);
    std::uniform_real_distribution<double> ud(0.0, 1.0);
    std::vector<SynthSat> sats;
    struct Truth
    {
        uint32_t prn;
        double delay, doppler;
    };
    std::vector<std::vector<Truth>> truth(sigs.size());
    const std::vector<float> bits = {1, -1, -1, -1, 1, -1, 1, 1};
    std::vector<float> e1c_sec(25);
    const char* sec_str = "0011100000001010110110010";
    for (int i = 0; i < 25; ++i) e1c_sec[i] = sec_str[i] == '0' ? 1.0F : -1.0F;
    // BeiDou B1I D1 (MEO / IGSO, PRN 6..58): the NH secondary code on every 1 ms code
    // period under the 50 bps data (Beidou_B1I.h:40-48), which the tracking loop's
    // secondary-code synchronisation needs before it emits
    std::vector<float> bds_nh(20);
    const char* nh_str = "00000100110101001110";
    for (int i = 0; i < 20; ++i) bds_nh[i] = nh_str[i] == '0' ? 1.0F : -1.0F;
    for (size_t g = 0; g < sigs.size(); ++g)
        for (int c = 0; c < sigs[g].nch; ++c)
            {
                const auto& s = sigs[g];
                const uint32_t prn = static_cast<uint32_t>(c + (s.sys == 'C' ? 6 : 1));
                const double per = fs * s.code_ms / 1000.0;
                const double delay = std::floor(ud(gen) * per);
                const double dop = 250.0 * std::round((ud(gen) * 8000.0 - 4000.0) / 250.0) + 37.0;
                truth[g].push_back({prn, delay, dop});
                if (s.sys == 'E')
                    {
                        // E1-B data + E1-C pilot (secondary code), 2 replica samples per chip
                        const double a = amp / std::sqrt(2.0);
                        auto e1c = galileo_e1_code_gen_sinboc11_float("1C", prn);
                        for (auto& v : e1c) v = -v;
                        sats.push_back({galileo_e1_code_gen_sinboc11_float("1B", prn), 2.046e6, s.carrier, delay, dop, a,
                            {}, {}, 0.004});
                        sats.push_back({e1c, 2.046e6, s.carrier, delay, dop, a, e1c_sec, {}, 0.004});
                    }
                else
                    sats.push_back({code_of(s.sys, prn), s.chip_rate, s.carrier, delay, dop, amp,
                        s.sys == 'C' ? bds_nh : std::vector<float>{}, bits, 0.02});
            }
    const auto x = synth_stream(sats, fs, n, 7, sigma);

    InMemoryConfiguration config;
    config.set_property("GNSS-SDR.internal_fs_sps", std::to_string(static_cast<long long>(fs)));
    for (const auto& s : sigs)
        {
            const std::string t = std::string("Tracking_") + s.role, a = std::string("Acquisition_") + s.role;
            config.set_property(t + ".implementation", s.impl_trk);
            config.set_property(t + ".item_type", "gr_complex");
            config.set_property(t + ".mi355x_ring", "rf0");  // every signal reads the one front end
            if (pool_batch > 0) config.set_property(t + ".mi355x_pool_batch", std::to_string(pool_batch));
            config.set_property(t + ".pll_bw_hz", s.sys == 'G' ? "40.0" : "15.0");
            config.set_property(t + ".dll_bw_hz", s.sys == 'G' ? "4.0" : "1.0");
            config.set_property(t + ".pull_in_time_s", "0");
            if (s.sys == 'E') config.set_property(t + ".track_pilot", "true");
            config.set_property(std::string("Channels_") + s.role + ".count", std::to_string(s.nch));
            config.set_property(a + ".implementation", s.impl_acq);
            config.set_property(a + ".item_type", "gr_complex");
            config.set_property(a + ".coherent_integration_time_ms", std::to_string(s.code_ms));
            config.set_property(a + ".pfa", "0.01");
            config.set_property(a + ".doppler_max", "5000");
            config.set_property(a + ".doppler_step", "250");
        }
    // tracking blocks (pooled, the adapters' default) started from the true acquisition
    struct Ch
    {
        std::unique_ptr<TrackingInterface> trk;
        TrackingBlockMI355X* blk;
        Gnss_Synchro gs;
        uint64_t nread;
        size_t sig;
        double truth_dop;
        int outputs;
        double dop;
        uint64_t calls;  // correlation calls run (records handed out)
    };
    std::vector<Ch> chans;
    chans.reserve(64);
    for (size_t g = 0; g < sigs.size(); ++g)
        for (int c = 0; c < sigs[g].nch; ++c)
            {
                chans.push_back({});
                Ch& ch = chans.back();
                ch.trk = gsdr_factory::GetTrkBlock(&config, std::string("Tracking_") + sigs[g].role, 1, 1, 0);
                ch.blk = dynamic_cast<DllPllTrackingAdapterMI355X*>(ch.trk.get())->get_block();
                const double per = fs * sigs[g].code_ms / 1000.0;
                ch.gs = Gnss_Synchro{};
                ch.gs.System = sigs[g].sys;
                ch.gs.Signal[0] = sigs[g].s0;
                ch.gs.Signal[1] = sigs[g].s1;
                ch.gs.PRN = truth[g][c].prn;
                ch.gs.Acq_delay_samples = std::fmod(truth[g][c].delay, per);
                // GPS from the 250 Hz grid (40 Hz PLL pulls in from <= 125 Hz); Galileo /
                // BeiDou (15 Hz PLL) from a 25 Hz grid, as a make_two_steps fine search
                // hands over -- from 125 Hz their narrow loops take longer than the run
                const double grid = sigs[g].sys == 'G' ? 250.0 : 25.0;
                ch.gs.Acq_doppler_hz = grid * std::round(truth[g][c].doppler / grid);
                ch.gs.Acq_samplestamp_samples = 0;
                ch.trk->set_channel(static_cast<unsigned int>(chans.size() - 1));
                ch.trk->set_gnss_synchro(&ch.gs);
                ch.trk->start_tracking();
                ch.nread = 0;
                ch.sig = g;
                ch.truth_dop = truth[g][c].doppler;
                ch.outputs = 0;
                ch.dop = 0.0;
                ch.calls = 0;
            }
    for (auto& ch : chans)
        {
            Ch* p = &ch;
            ch.blk->set_record_sink([p](const gsdr_trk_epoch& r) {
                p->dop = r.carrier_doppler_hz;
                ++p->calls;
            });
        }
    // acquisition services on the device ring: every untracked PRN of each signal,
    // re-armed after each answer
    // the GPU's shared ring (the pooled tracking blocks' too): the bench pushes the
    // stream into it, the pools' hooks keep their channels inside its window
    const uint64_t per_max = static_cast<uint64_t>(fs * 4 / 1000);
    const auto hub = DeviceIqRing::get(0, GSDR_ITEM_GR_COMPLEX, 8 * per_max, "rf0");
    gsdr_stream* ring = hub->stream();
    if (pinned && gsdr_host_register(const_cast<std::complex<float>*>(x.data()), x.size() * sizeof(x[0])) != GSDR_OK)
        {
            std::fprintf(stderr, "pin: %s\n", gsdr_last_error());
            return 1;
        }
    std::vector<std::unique_ptr<AcquisitionService>> svcs;
    std::vector<std::vector<std::vector<std::complex<float>>>> reps(sigs.size());
    std::vector<uint64_t> answers(sigs.size(), 0), positives(sigs.size(), 0);
    std::vector<std::unique_ptr<AcquisitionService::Callback>> cbs;
    for (size_t g = 0; g < sigs.size(); ++g)
        {
            Acq_Conf ac;
            ac.ms_per_code = static_cast<uint32_t>(sigs[g].code_ms);
            ac.SetFromConfiguration(&config, std::string("Acquisition_") + sigs[g].role, sigs[g].chip_rate,
                sigs[g].sys == 'C' ? 4000000.0 : 2000000.0);
            // the searched PRNs: every untracked one (BeiDou: up to PRN 32)
            const int nsearch = search ? std::min(sigs[g].nprn, 32) - sigs[g].nch - (sigs[g].sys == 'C' ? 5 : 0) : 0;
            if (nsearch <= 0)
                {
                    svcs.push_back(nullptr);
                    continue;
                }
            svcs.push_back(std::make_unique<AcquisitionService>(ac, static_cast<uint32_t>(nsearch), 0));
            for (int k = 0; k < nsearch; ++k)
                {
                    const uint32_t prn = static_cast<uint32_t>(sigs[g].nch + k + (sigs[g].sys == 'C' ? 6 : 1));
                    std::vector<std::complex<float>> r;
                    if (sigs[g].sys == 'E')
                        r = galileo_e1_code_gen_complex_sampled("1B", false, prn, static_cast<int32_t>(fs), 0, false);
                    else if (sigs[g].sys == 'C')
                        r = beidou_b1i_code_gen_complex_sampled(static_cast<int32_t>(prn), static_cast<int32_t>(fs), 0);
                    else
                        r = gps_l1_ca_code_gen_complex_sampled(prn, static_cast<int32_t>(fs), 0);
                    reps[g].push_back(std::move(r));
                }
            AcquisitionService* svc = svcs.back().get();
            for (int k = 0; k < nsearch; ++k)
                {
                    const uint32_t prn = static_cast<uint32_t>(sigs[g].nch + k + (sigs[g].sys == 'C' ? 6 : 1));
                    auto* code = reps[g][k].data();
                    // the callback lives in cbs (stable storage): an answer re-arms the
                    // request with a copy of it -- the idle channel keeps searching
                    cbs.push_back(std::make_unique<AcquisitionService::Callback>());
                    AcquisitionService::Callback* cb = cbs.back().get();
                    *cb = [&answers, &positives, g, prn, code, svc, cb](uint32_t c, const gsdr_acq_result&, bool pos) {
                        ++answers[g];
                        if (pos) ++positives[g];
                        svc->request(c, prn, code, *cb);
                    };
                    svc->request(static_cast<uint32_t>(k), prn, code, *cb);
                }
        }
    for (auto& s : svcs)
        if (s) s->work_ring(ring, 0);

    const auto t0 = std::chrono::steady_clock::now();
    size_t pushed = 0;
    const size_t chunk = 16384;
    bool progress = true;
    uint64_t trk_calls = 0;
    // where the host's time goes: pushes (with the pools' advance launches their hooks
    // make), the acquisition services, the tracking blocks' work() calls
    using clk = std::chrono::steady_clock;
    double t_feed = 0, t_svc = 0, t_work = 0;
    if (threads > 0)
        {
            // the blocks on T threads; the source (this thread) pushes, runs the services
            // and keeps within `lag` items of the slowest block
            const size_t look = static_cast<size_t>(lookahead) * chunk;
            const size_t lag = 4 * chunk + look;
            std::atomic<size_t> vis_a{0};
            std::atomic<bool> fed_all{false};
            std::unique_ptr<std::atomic<uint64_t>[]> nread_a(new std::atomic<uint64_t>[chans.size()]);
            for (size_t i = 0; i < chans.size(); ++i) nread_a[i].store(0);
            std::atomic<uint64_t> calls_a{0};
            auto worker = [&](int t) {
                uint64_t my_calls = 0;
                for (;;)
                    {
                        const bool fin = fed_all.load(std::memory_order_acquire);
                        const size_t vis = vis_a.load(std::memory_order_acquire);
                        bool prog = false;
                        for (size_t i = static_cast<size_t>(t); i < chans.size(); i += static_cast<size_t>(threads))
                            {
                                Ch& ch = chans[i];
                                for (;;)
                                    {
                                        if (ch.nread >= vis) break;
                                        const int fc = ch.blk->forecast();
                                        const uint64_t avail = vis - ch.nread;
                                        if (avail < static_cast<uint64_t>(fc)) break;
                                        const int give =
                                            static_cast<int>(std::min<uint64_t>(std::max<uint64_t>(chunk, fc), avail));
                                        Gnss_Synchro out{};
                                        int nout = 0;
                                        const int used = ch.blk->work(x.data() + ch.nread, give, ch.nread, &out, &nout);
                                        if (nout == 1 && out.Flag_valid_symbol_output) ++ch.outputs;
                                        if (used <= 0 && nout == 0) break;
                                        prog = true;
                                        ch.nread += static_cast<uint64_t>(std::max(used, 0));
                                        ++my_calls;
                                    }
                                nread_a[i].store(ch.nread, std::memory_order_release);
                            }
                        if (!prog)
                            {
                                if (fin && vis == n) break;
                                std::this_thread::yield();
                            }
                    }
                calls_a += my_calls;
            };
            const auto w0 = clk::now();
            std::vector<std::thread> pool;
            for (int t = 0; t < threads; ++t) pool.emplace_back(worker, t);
            uint64_t stalls = 0;
            while (pushed < n)
                {
                    // a bounded upstream buffer: wait (at most ~50 ms, for a block that
                    // stopped consuming) until the slowest block is within `lag` of the head
                    const auto s0 = clk::now();
                    for (;;)
                        {
                            uint64_t slowest = UINT64_MAX;
                            for (size_t i = 0; i < chans.size(); ++i)
                                slowest = std::min<uint64_t>(slowest, nread_a[i].load(std::memory_order_acquire));
                            if (slowest + lag >= pushed) break;
                            if (std::chrono::duration<double>(clk::now() - s0).count() > 0.05)
                                {
                                    ++stalls;
                                    break;
                                }
                            std::this_thread::yield();
                        }
                    const size_t m = std::min(chunk, n - pushed);
                    const auto a = clk::now();
                    hub->feed(x.data() + pushed, pushed, static_cast<int>(m));
                    const auto b = clk::now();
                    pushed += m;
                    const size_t visible = pushed == n ? n : (pushed > look ? pushed - look : 0);
                    vis_a.store(visible, std::memory_order_release);
                    for (auto& s : svcs)
                        if (s) s->work_ring(ring, visible);
                    t_feed += std::chrono::duration<double>(b - a).count();
                    t_svc += std::chrono::duration<double>(clk::now() - b).count();
                }
            fed_all.store(true, std::memory_order_release);
            for (auto& th : pool) th.join();
            trk_calls = calls_a.load();
            t_work = std::chrono::duration<double>(clk::now() - w0).count();  // the threads' wall
            if (stalls) std::fprintf(stderr, "receiver_bench: %llu source stalls past 50 ms\n", (unsigned long long)stalls);
            progress = false;
        }
    while (progress)
        {
            progress = false;
            size_t visible = pushed;
            if (pushed < n)
                {
                    const size_t m = std::min(chunk, n - pushed);
                    const auto a = clk::now();
                    hub->feed(x.data() + pushed, pushed, static_cast<int>(m));
                    const auto b = clk::now();
                    pushed += m;
                    progress = true;
                    // the items the blocks are offered: all but the source's lookahead
                    const size_t look = static_cast<size_t>(lookahead) * chunk;
                    visible = pushed == n ? n : (pushed > look ? pushed - look : 0);
                    for (auto& s : svcs)
                        if (s) s->work_ring(ring, visible);
                    t_feed += std::chrono::duration<double>(b - a).count();
                    t_svc += std::chrono::duration<double>(clk::now() - b).count();
                }
            // every tracking block gets what the upstream buffer holds at its position
            const auto w0 = clk::now();
            for (auto& ch : chans)
                for (;;)
                    {
                        if (ch.nread >= visible) break;
                        const int fc = ch.blk->forecast();
                        const uint64_t avail = visible - ch.nread;
                        if (avail < static_cast<uint64_t>(fc)) break;  // GNU Radio's forecast: wait for more items
                        const int give = static_cast<int>(std::min<uint64_t>(std::max<uint64_t>(chunk, fc), avail));
                        Gnss_Synchro out{};
                        int nout = 0;
                        const int used = ch.blk->work(x.data() + ch.nread, give, ch.nread, &out, &nout);
                        if (nout == 1 && out.Flag_valid_symbol_output) ++ch.outputs;
                        if (used <= 0 && nout == 0) break;
                        progress = true;
                        ch.nread += static_cast<uint64_t>(std::max(used, 0));
                        ++trk_calls;
                    }
            t_work += std::chrono::duration<double>(clk::now() - w0).count();
        }
    const auto f0 = clk::now();
    // end of the stream: the blocks compute what they were handed and hand out the rest
    for (auto& ch : chans)
        {
            ch.blk->flush();
            for (int guard = 0; guard < 1000000; ++guard)
                {
                    Gnss_Synchro out{};
                    int nout = 0;
                    ch.blk->work(nullptr, 0, ch.nread, &out, &nout);
                    if (nout == 0) break;
                    if (out.Flag_valid_symbol_output) ++ch.outputs;
                }
        }
    for (auto& s : svcs)
        if (s) s->flush();
    const double t_flush = std::chrono::duration<double>(clk::now() - f0).count();
    const double sec = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    std::string per_sig;
    for (size_t g = 0; g < sigs.size(); ++g)
        {
            int outs = 0, within = 0, with_outputs = 0, min_out = -1;
            uint64_t calls = 0;
            for (const auto& ch : chans)
                if (ch.sig == g)
                    {
                        outs += ch.outputs;
                        with_outputs += ch.outputs > 0 ? 1 : 0;
                        min_out = min_out < 0 ? ch.outputs : std::min(min_out, ch.outputs);
                        within += std::abs(ch.dop - ch.truth_dop) < 25.0 ? 1 : 0;
                        calls += ch.calls;
                    }
            char buf[512];
            std::snprintf(buf, sizeof buf,
                "%s\"%c%c%c\": {\"channels\": %d, \"outputs\": %d, \"channels_with_outputs\": %d, "
                "\"min_outputs_per_channel\": %d, \"channels_within_25hz\": %d, \"trk_calls\": %llu, "
                "\"acq_answers\": %llu, \"acq_positive\": %llu, \"acq_grids\": %llu, \"acq_launches\": %llu, "
                "\"acq_code_uploads\": %llu}",
                g ? ", " : "", sigs[g].sys, sigs[g].s0, sigs[g].s1, sigs[g].nch, outs, with_outputs, min_out, within,
                static_cast<unsigned long long>(calls), static_cast<unsigned long long>(answers[g]),
                static_cast<unsigned long long>(positives[g]),
                static_cast<unsigned long long>(svcs[g] ? svcs[g]->grids_run() : 0),
                static_cast<unsigned long long>(svcs[g] ? svcs[g]->launches() : 0),
                static_cast<unsigned long long>(svcs[g] ? svcs[g]->code_uploads() : 0));
            per_sig += buf;
        }
    std::printf("{\"config\": \"%s\", \"search\": %d, \"path\": \"factory-built pooled TrackingInterface blocks (work() per block at its "
                "nitems_read, batched advances) + AcquisitionService grids on the device IQ ring (batched, asynchronous), host "
                "pushes of %zu-item chunks\", "
                "\"host_buffer\": \"%s\", \"pool_batch\": %d, \"source_lookahead_chunks\": %d, \"block_threads\": %d, \"fs_sps\": %.0f, \"samples\": %zu, \"seconds\": %.4f, \"msps\": %.2f, \"real_time_factor\": %.2f, "
                "\"tracking_channels\": %zu, \"trk_work_calls\": %llu, \"host_seconds\": {\"feed_and_pool_advances\": %.4f, "
                "\"acquisition_services\": %.4f, \"tracking_work_calls\": %.4f, \"flush\": %.4f}, \"signals\": {%s}}\n",
        cfg.c_str(), search ? 1 : 0, chunk, pinned ? "pinned" : "pageable", pool_batch, lookahead, threads, fs, n, sec, n / sec / 1e6, n / sec / fs, chans.size(),
        static_cast<unsigned long long>(trk_calls), t_feed, t_svc, t_work, t_flush, per_sig.c_str());
    chans.clear();
    svcs.clear();
    if (pinned) gsdr_host_unregister(const_cast<std::complex<float>*>(x.data()));
    return 0;
}
