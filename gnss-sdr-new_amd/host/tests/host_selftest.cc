// Host-side drop-in self-test, written like the reference's unit tests:
//  1. GpsL1CaPcpsAcquisitionTest.ValidationOfResults
//     (src/tests/unit-tests/signal-processing-blocks/acquisition/gps_l1_ca_pcps_acquisition_test.cc:283-366)
//     on the reference capture, through the adapter + block mirror + GPU engine.
//  2. Hip_Multicorrelator_Real_Codes / Hip_Multicorrelator on the acquired signal,
//     checked against an fp64 evaluation of the reference's phasor model.
//  3. The dwell FSM across calls (max_dwells = 2) against the one-shot dwell
//     engine, the bit-transition branch, cbyte input.
//  4. GalileoE1PcpsAmbiguousAcquisitionTest.ValidationOfResults
//     (galileo_e1_pcps_ambiguous_acquisition_test.cc:289-371) through the Galileo
//     adapter on Galileo_E1_ID_1_Fs_4Msps_8ms.dat, and the BeiDou adapter on a
//     synthetic B1I signal (the reference's B1I capture is not in the tree).
//  5. Acquisition -> tracking hand-off through the factory-built adapters
//     (TrackingInterface::start_tracking from the acquisition's Gnss_Synchro,
//     Gnss_Synchro records out) on synthetic GPS L1 C/A and Galileo E1 streams.
//  6. AcquisitionInterface::set_channel_fsm: a positive acquisition reaches the
//     channel FSM's Event_valid_acquisition directly (pcps_acquisition.cc:370-373).
//  7. The pooled tracking block (<role>.mi355x_pool=true): factory-built channels
//     sharing one engine handle over the device ring, fed GNU-Radio style, give the
//     per-channel blocks' records bit for bit; the rates of both are printed.
//  8. The gflags overrides (--pll_bw_hz, --dll_bw_hz, --doppler_max) and defaults.
// Usage: host_selftest <GPS_L1_CA_ID_1_Fs_4Msps_2ms.dat> [Galileo_E1_ID_1_Fs_4Msps_8ms.dat]
#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdlib>
#include <cmath>
#include <complex>
#include <cstring>
#include <cstdio>
#include <filesystem>
#include <fstream>
#include <iostream>
#include <string>
#include <vector>

#include <random>
#include <stdexcept>

#include "acquisition_service.h"
#include "beidou_b1i_pcps_acquisition_mi355x.h"
#include "galileo_e1_pcps_ambiguous_acquisition_mi355x.h"
#include "channel_fsm.h"
#include "gnss_block_factory_mi355x.h"
#include "gnss_replicas.h"
#include "gnss_sdr_flags.h"
#include "gnss_tracking_mi355x.h"
#include "gps_l1_ca_pcps_acquisition_mi355x.h"
#include "hip_multicorrelator_real_codes.h"
#include "tracking_dump.h"
#include "tracking_pool.h"
#include "synth_stream.h"
#include <unistd.h>

namespace
{
int failures = 0;
#define EXPECT(cond, msg)                                              \
    do                                                                 \
        {                                                              \
            if (!(cond))                                               \
                {                                                      \
                    std::cerr << "FAIL: " << msg << " (" #cond ")\n"; \
                    ++failures;                                        \
                }                                                      \
        }                                                              \
    while (0)

std::vector<std::complex<float>> read_capture(const std::string& path)
{
    std::ifstream f(path, std::ios::binary);
    std::vector<std::complex<float>> v;
    if (!f) return v;
    f.seekg(0, std::ios::end);
    const auto bytes = static_cast<size_t>(f.tellg());
    f.seekg(0);
    v.resize(bytes / sizeof(std::complex<float>));
    f.read(reinterpret_cast<char*>(v.data()), static_cast<std::streamsize>(v.size() * sizeof(std::complex<float>)));
    return v;
}

// fp64 value of the reference rotator/resampler for real codes (generic association).
std::vector<std::complex<double>> exact_correlation(const std::complex<float>* x, const std::vector<float>& code,
    const std::vector<float>& shifts, float rem_carr, float carr_step, float rem_code, float code_step, int n)
{
    const std::complex<float> off(std::cos(rem_carr), -std::sin(rem_carr));
    const std::complex<float> inc = std::exp(std::complex<float>(0.0F, -carr_step));
    const double psi = std::atan2(static_cast<double>(off.imag()), static_cast<double>(off.real()));
    const double th = std::atan2(static_cast<double>(inc.imag()), static_cast<double>(inc.real()));
    const int L = static_cast<int>(code.size());
    std::vector<std::complex<double>> out(shifts.size());
    for (int i = 0; i < n; ++i)
        {
            const std::complex<double> t = std::complex<double>(x[i]) * std::polar(1.0, psi + th * i);
            for (size_t k = 0; k < shifts.size(); ++k)
                {
                    volatile float a = code_step * static_cast<float>(i);
                    volatile float b = shifts[k] - rem_code;
                    int idx = static_cast<int>(std::floor(a + b));
                    idx = ((idx % L) + L) % L;
                    out[k] += t * static_cast<double>(code[idx]);
                }
        }
    return out;
}

// carrier: Acquisition_1C.mi355x_carrier (exact, or the generic / AVX2 sincos
// protokernel replayed); returns the test statistic
double test_acquisition_validation(const std::vector<std::complex<float>>& capture, const char* carrier = "exact")
{
    InMemoryConfiguration config;
    config.set_property("Acquisition_1C.mi355x_carrier", carrier);
    config.set_property("GNSS-SDR.internal_fs_sps", "4000000");
    config.set_property("Acquisition_1C.implementation", "GPS_L1_CA_PCPS_Acquisition_MI355X");
    config.set_property("Acquisition_1C.item_type", "gr_complex");
    config.set_property("Acquisition_1C.coherent_integration_time_ms", "1");
    config.set_property("Acquisition_1C.dump", "false");
    config.set_property("Acquisition_1C.threshold", "0.00001");
    config.set_property("Acquisition_1C.doppler_max", "5000");
    config.set_property("Acquisition_1C.doppler_step", "100");
    config.set_property("Acquisition_1C.repeat_satellite", "false");

    Gnss_Synchro gnss_synchro{};
    gnss_synchro.Channel_ID = 0;
    gnss_synchro.System = 'G';
    gnss_synchro.Signal[0] = '1';
    gnss_synchro.Signal[1] = 'C';
    gnss_synchro.PRN = 1;

    GpsL1CaPcpsAcquisitionMI355X acquisition(&config, "Acquisition_1C", 1, 0);
    int rx_message = 0;
    acquisition.get_block()->set_event_handler([&](int ev) { rx_message = ev; });
    acquisition.set_channel(1);
    acquisition.set_gnss_synchro(&gnss_synchro);
    acquisition.set_threshold(0.001);
    acquisition.set_doppler_max(5000);
    acquisition.set_doppler_step(100);
    acquisition.set_local_code();
    acquisition.set_state(1);
    acquisition.init();
    acquisition.get_block()->start();

    // feed the file like a GNU Radio file_source, 1024 items per general_work call
    size_t pos = 0;
    int guard = 0;
    while (rx_message == 0 && guard++ < 10000)
        {
            const int n = static_cast<int>(std::min<size_t>(1024, capture.size() - pos));
            const int used = acquisition.get_block()->work(capture.data() + pos, n);
            pos += static_cast<size_t>(used);
            if (n == 0 && used == 0 && pos >= capture.size()) break;
        }
    EXPECT(rx_message == 1, "Acquisition failure. Expected message: 1=ACQ SUCCESS.");
    const double delay_error_samples = std::abs(524.0 - gnss_synchro.Acq_delay_samples);
    const auto delay_error_chips = static_cast<float>(delay_error_samples * 1023 / 4000);
    const double doppler_error_hz = std::abs(1680.0 - gnss_synchro.Acq_doppler_hz);
    EXPECT(doppler_error_hz <= 666, "Doppler error exceeds 666 Hz");
    EXPECT(delay_error_chips < 0.5, "Delay error exceeds 0.5 chips");
    EXPECT(acquisition.get_block()->num_doppler_bins() == 100, "D = ceil(2*5000/100)");
    std::printf("acquisition (%s carrier): message %d delay %.1f samples doppler %.0f Hz stat %.6f stamp %llu\n",
        carrier, rx_message, gnss_synchro.Acq_delay_samples, gnss_synchro.Acq_doppler_hz,
        acquisition.get_block()->test_statistics(), static_cast<unsigned long long>(gnss_synchro.Acq_samplestamp_samples));
    return acquisition.get_block()->test_statistics();
}

// the three carrier models agree on the reference capture within the protokernels'
// own drift (C1: 4 Msps, +-5 kHz, 1 ms: well under 1e-3 of the statistic); an unknown
// model is a configuration error
void test_acquisition_carriers(const std::vector<std::complex<float>>& capture)
{
    const double e = test_acquisition_validation(capture, "exact");
    const double g = test_acquisition_validation(capture, "generic");
    const double a = test_acquisition_validation(capture, "avx2");
    EXPECT(std::abs(g - e) <= 1e-3 * e && std::abs(a - e) <= 1e-3 * e, "carrier models: statistics agree");
    InMemoryConfiguration config;
    config.set_property("Acquisition_1C.mi355x_carrier", "fast");
    bool threw = false;
    try
        {
            Acq_Conf c;
            c.SetFromConfiguration(&config, "Acquisition_1C", 1.023e6, 0.001);
        }
    catch (const std::invalid_argument&)
        {
            threw = true;
        }
    EXPECT(threw, "carrier models: unknown .mi355x_carrier rejected");
}

// Acquisition_1C.blocking = false (pcps_acquisition.cc:1013-1029): the core runs on
// a worker thread; general_work calls during it consume nothing (single dwell,
// :928-936) and the answer equals the blocking block's.
void test_acquisition_nonblocking(const std::vector<std::complex<float>>& capture)
{
    Gnss_Synchro res[2]{};
    uint64_t cores = 0;
    for (int blocking = 1; blocking >= 0; --blocking)
        {
            InMemoryConfiguration config;
            config.set_property("GNSS-SDR.internal_fs_sps", "4000000");
            config.set_property("Acquisition_1C.implementation", "GPS_L1_CA_PCPS_Acquisition_MI355X");
            config.set_property("Acquisition_1C.item_type", "gr_complex");
            config.set_property("Acquisition_1C.coherent_integration_time_ms", "1");
            config.set_property("Acquisition_1C.doppler_max", "5000");
            config.set_property("Acquisition_1C.doppler_step", "100");
            config.set_property("Acquisition_1C.blocking", blocking ? "true" : "false");
            Gnss_Synchro& gs = res[blocking];
            gs.System = 'G';
            gs.Signal[0] = '1';
            gs.Signal[1] = 'C';
            gs.PRN = 1;
            GpsL1CaPcpsAcquisitionMI355X acquisition(&config, "Acquisition_1C", 1, 0);
            std::atomic<int> rx_message{0};
            acquisition.get_block()->set_event_handler([&](int ev) { rx_message = ev; });
            acquisition.set_gnss_synchro(&gs);
            acquisition.set_threshold(0.001);
            acquisition.set_local_code();
            acquisition.set_state(1);
            acquisition.init();
            acquisition.get_block()->start();
            size_t pos = 0;
            int guard = 0;
            while (rx_message == 0 && guard++ < 10000)
                {
                    const int n = static_cast<int>(std::min<size_t>(1024, capture.size() - pos));
                    pos += static_cast<size_t>(acquisition.get_block()->work(capture.data() + pos, n));
                }
            EXPECT(rx_message == 1, "blocking=" << blocking << ": positive acquisition");
            if (!blocking) cores = acquisition.get_block()->async_cores();
        }
    EXPECT(cores >= 1, "blocking=false: the core ran on the worker thread");
    EXPECT(res[0].Acq_delay_samples == res[1].Acq_delay_samples && res[0].Acq_doppler_hz == res[1].Acq_doppler_hz &&
               res[0].Acq_samplestamp_samples == res[1].Acq_samplestamp_samples,
        "blocking=false: same Gnss_Synchro as blocking");
    std::printf("non-blocking acquisition: %llu worker cores, delay %.1f doppler %.0f stamp %llu\n",
        static_cast<unsigned long long>(cores), res[0].Acq_delay_samples, res[0].Acq_doppler_hz,
        static_cast<unsigned long long>(res[0].Acq_samplestamp_samples));
}

// Acquisition_1C.dump (pcps_acquisition.cc:135-165, :408-508): the dump channel's
// grid and fields per decided attempt as a .mat file -- a single-step attempt on
// channel 1 (dump_channel 1) and a make_two_steps attempt (with the narrow grid).
// tests/test_host_mirror.py checks the files' grids against the oracle.
void test_acquisition_dump(const std::vector<std::complex<float>>& capture, const std::string& dir)
{
    for (int two = 0; two <= 1; ++two)
        {
            InMemoryConfiguration config;
            config.set_property("GNSS-SDR.internal_fs_sps", "4000000");
            config.set_property("Acquisition_1C.implementation", "GPS_L1_CA_PCPS_Acquisition_MI355X");
            config.set_property("Acquisition_1C.item_type", "gr_complex");
            config.set_property("Acquisition_1C.coherent_integration_time_ms", "1");
            config.set_property("Acquisition_1C.pfa", "0.01");
            config.set_property("Acquisition_1C.doppler_max", "5000");
            config.set_property("Acquisition_1C.doppler_step", two ? "500" : "100");
            config.set_property("Acquisition_1C.dump", "true");
            config.set_property("Acquisition_1C.dump_filename", dir + (two ? "/acq_two.dat" : "/acq_one.dat"));
            config.set_property("Acquisition_1C.dump_channel", "1");
            if (two)
                {
                    config.set_property("Acquisition_1C.make_two_steps", "true");
                    config.set_property("Acquisition_1C.second_nbins", "5");
                    config.set_property("Acquisition_1C.second_doppler_step", "100");
                    config.set_property("Acquisition_1C.blocking_on_standby", "true");
                }
            Gnss_Synchro gs{};
            gs.System = 'G';
            gs.Signal[0] = '1';
            gs.Signal[1] = 'C';
            gs.PRN = 1;
            GpsL1CaPcpsAcquisitionMI355X acquisition(&config, "Acquisition_1C", 1, 0);
            int rx_message = 0;
            acquisition.get_block()->set_event_handler([&](int ev) { rx_message = ev; });
            acquisition.set_channel(1);
            acquisition.set_gnss_synchro(&gs);
            acquisition.set_local_code();
            acquisition.set_state(1);
            acquisition.init();
            acquisition.get_block()->start();
            size_t pos = 0;
            int guard = 0;
            while (rx_message == 0 && guard++ < 200)
                {
                    const int n = static_cast<int>(std::min<size_t>(1000, capture.size() - pos));
                    pos += static_cast<size_t>(acquisition.get_block()->work(capture.data() + pos, n));
                }
            EXPECT(rx_message == 1, "dump " << (two ? "two-step" : "single-step") << ": positive acquisition");
            const std::string want = dir + (two ? "/acq_two" : "/acq_one") + "_G_1C_ch_1_1_sat_1.mat";
            EXPECT(acquisition.get_block()->dump_number() == 1 && acquisition.get_block()->last_dump_path() == want,
                "dump file " << want << " (got " << acquisition.get_block()->last_dump_path() << ")");
            EXPECT(std::filesystem::exists(want), "dump file exists: " << want);
            std::printf("acquisition dump: %s (delay %.1f doppler %.0f)\n", want.c_str(), gs.Acq_delay_samples,
                gs.Acq_doppler_hz);
        }
    // a channel other than dump_channel writes nothing
    InMemoryConfiguration config;
    config.set_property("GNSS-SDR.internal_fs_sps", "4000000");
    config.set_property("Acquisition_1C.implementation", "GPS_L1_CA_PCPS_Acquisition_MI355X");
    config.set_property("Acquisition_1C.pfa", "0.01");
    config.set_property("Acquisition_1C.dump", "true");
    config.set_property("Acquisition_1C.dump_filename", dir + "/acq_other.dat");
    config.set_property("Acquisition_1C.dump_channel", "1");
    Gnss_Synchro gs{};
    gs.System = 'G';
    gs.Signal[0] = '1';
    gs.Signal[1] = 'C';
    gs.PRN = 1;
    GpsL1CaPcpsAcquisitionMI355X acquisition(&config, "Acquisition_1C", 1, 0);
    int rx_message = 0;
    acquisition.get_block()->set_event_handler([&](int ev) { rx_message = ev; });
    acquisition.set_channel(2);
    acquisition.set_gnss_synchro(&gs);
    acquisition.set_local_code();
    acquisition.set_state(1);
    acquisition.init();
    acquisition.get_block()->start();
    size_t pos = 0;
    int guard = 0;
    while (rx_message == 0 && guard++ < 200)
        pos += static_cast<size_t>(acquisition.get_block()->work(capture.data() + pos,
            static_cast<int>(std::min<size_t>(1000, capture.size() - pos))));
    EXPECT(acquisition.get_block()->dump_number() == 0, "no dump for a channel other than dump_channel");
}

// make_two_steps on the same capture: coarse 500 Hz grid on the first millisecond,
// then a 5-bin 100 Hz narrow grid around it on the second (blocking_on_standby so
// the 2 ms capture holds both blocks).
void test_acquisition_two_steps(const std::vector<std::complex<float>>& capture)
{
    InMemoryConfiguration config;
    config.set_property("GNSS-SDR.internal_fs_sps", "4000000");
    config.set_property("Acquisition_1C.implementation", "GPS_L1_CA_PCPS_Acquisition_MI355X");
    config.set_property("Acquisition_1C.item_type", "gr_complex");
    config.set_property("Acquisition_1C.coherent_integration_time_ms", "1");
    config.set_property("Acquisition_1C.pfa", "0.01");
    config.set_property("Acquisition_1C.doppler_max", "5000");
    config.set_property("Acquisition_1C.doppler_step", "500");
    config.set_property("Acquisition_1C.make_two_steps", "true");
    config.set_property("Acquisition_1C.second_nbins", "5");
    config.set_property("Acquisition_1C.second_doppler_step", "100");
    config.set_property("Acquisition_1C.blocking_on_standby", "true");

    Gnss_Synchro gnss_synchro{};
    gnss_synchro.System = 'G';
    gnss_synchro.Signal[0] = '1';
    gnss_synchro.Signal[1] = 'C';
    gnss_synchro.PRN = 1;
    GpsL1CaPcpsAcquisitionMI355X acquisition(&config, "Acquisition_1C", 1, 0);
    int rx_message = 0;
    acquisition.get_block()->set_event_handler([&](int ev) { rx_message = ev; });
    acquisition.set_gnss_synchro(&gnss_synchro);
    acquisition.set_doppler_max(5000);
    acquisition.set_doppler_step(500);
    acquisition.set_local_code();
    acquisition.set_state(1);
    acquisition.init();
    acquisition.get_block()->start();
    const float thr1 = acquisition.get_block()->threshold();
    size_t pos = 0;
    int guard = 0;
    bool saw_step_two = false;
    double coarse = 0.0;
    float thr2 = thr1;
    // at the end of the capture keep calling with no new items: the state machine
    // still has to run the core on its full buffer
    while (rx_message == 0 && guard++ < 100)
        {
            const int n = static_cast<int>(std::min<size_t>(1000, capture.size() - pos));
            const bool before = acquisition.get_block()->step_two();
            pos += static_cast<size_t>(acquisition.get_block()->work(capture.data() + pos, n));
            if (!before && acquisition.get_block()->step_two())
                {
                    saw_step_two = true;
                    coarse = gnss_synchro.Acq_doppler_hz;
                    thr2 = acquisition.get_block()->threshold();
                }
        }
    EXPECT(saw_step_two, "first step positive -> step two");
    EXPECT(rx_message == 1, "two-step acquisition positive");
    EXPECT(gnss_synchro.Acq_doppler_step == 100U, "Acq_doppler_step = second_doppler_step");
    EXPECT(std::abs(gnss_synchro.Acq_doppler_hz - coarse) <= 200.0, "narrow grid within +-2 bins of the coarse Doppler");
    EXPECT(std::abs(gnss_synchro.Acq_doppler_hz - 1680.0) < std::abs(coarse - 1680.0) + 1e-9,
        "refinement does not move away from the capture's Doppler");
    EXPECT(gnss_synchro.Acq_samplestamp_samples == 8000ULL, "step two on the second block");
    EXPECT(thr2 < thr1, "step-two threshold from the narrow bin count");
    EXPECT(acquisition.get_block()->threshold() == thr1, "first-step threshold restored after step two");
    std::printf("two steps: coarse %.0f Hz -> fine %.0f Hz, delay %.1f samples, stat %.3f\n", coarse,
        gnss_synchro.Acq_doppler_hz, gnss_synchro.Acq_delay_samples, acquisition.get_block()->test_statistics());
}

// The fork's make_repeat_steps: after a positive the block re-arms itself and
// acquires again on the next block without a new set_state(1).
void test_acquisition_repeat_steps(const std::vector<std::complex<float>>& capture)
{
    InMemoryConfiguration config;
    config.set_property("GNSS-SDR.internal_fs_sps", "4000000");
    config.set_property("Acquisition_1C.implementation", "GPS_L1_CA_PCPS_Acquisition_MI355X");
    config.set_property("Acquisition_1C.item_type", "gr_complex");
    config.set_property("Acquisition_1C.coherent_integration_time_ms", "1");
    config.set_property("Acquisition_1C.pfa", "0.01");
    config.set_property("Acquisition_1C.doppler_max", "5000");
    config.set_property("Acquisition_1C.doppler_step", "250");
    config.set_property("Acquisition_1C.make_repeat_steps", "true");
    config.set_property("Acquisition_1C.blocking_on_standby", "true");
    Gnss_Synchro gnss_synchro{};
    gnss_synchro.System = 'G';
    gnss_synchro.Signal[0] = '1';
    gnss_synchro.Signal[1] = 'C';
    gnss_synchro.PRN = 1;
    GpsL1CaPcpsAcquisitionMI355X acquisition(&config, "Acquisition_1C", 1, 0);
    int positives = 0;
    std::vector<uint64_t> stamps;
    acquisition.get_block()->set_event_handler([&](int ev) {
        if (ev == 1)
            {
                ++positives;
                stamps.push_back(gnss_synchro.Acq_samplestamp_samples);
            }
    });
    acquisition.set_gnss_synchro(&gnss_synchro);
    acquisition.set_local_code();
    acquisition.set_state(1);
    acquisition.init();
    acquisition.get_block()->start();
    size_t pos = 0;
    for (int guard = 0; guard < 100 && positives < 2; ++guard)
        {
            const int n = static_cast<int>(std::min<size_t>(1000, capture.size() - pos));
            pos += static_cast<size_t>(acquisition.get_block()->work(capture.data() + pos, n));
        }
    EXPECT(positives == 2, "repeat steps: a second positive without set_state(1)");
    EXPECT(acquisition.get_block()->step_repeat(), "d_step_repeat latched");
    EXPECT(stamps.size() == 2 && stamps[0] == 4000ULL && stamps[1] == 8000ULL, "one positive per block");
    EXPECT(std::abs(gnss_synchro.Acq_delay_samples - 524.0) < 1.0, "repeated acquisition keeps the code phase");
    std::printf("repeat steps: %d positives, stamps %llu %llu\n", positives,
        stamps.size() > 0 ? static_cast<unsigned long long>(stamps[0]) : 0ULL,
        stamps.size() > 1 ? static_cast<unsigned long long>(stamps[1]) : 0ULL);
}

// Batched acquisition service: 4 channels' requests answered by one grid per
// block, each answer bit-identical to a one-PRN engine on the same block.
void test_acquisition_service(const std::vector<std::complex<float>>& capture)
{
    InMemoryConfiguration config;
    config.set_property("GNSS-SDR.internal_fs_sps", "4000000");
    config.set_property("Acquisition_1C.item_type", "gr_complex");
    config.set_property("Acquisition_1C.coherent_integration_time_ms", "1");
    config.set_property("Acquisition_1C.pfa", "0.01");
    config.set_property("Acquisition_1C.doppler_max", "5000");
    config.set_property("Acquisition_1C.doppler_step", "250");
    Acq_Conf conf;
    conf.ms_per_code = 1;
    conf.SetFromConfiguration(&config, "Acquisition_1C", 1023000.0, 4000000.0);
    AcquisitionService svc(conf, 8, 0);
    const uint32_t prns[4] = {1, 2, 11, 20};
    std::vector<std::vector<std::complex<float>>> codes;
    struct Answer
    {
        uint32_t channel;
        gsdr_acq_result r;
        bool positive;
    };
    std::vector<Answer> answers;
    for (uint32_t ch = 0; ch < 4; ++ch)
        {
            codes.push_back(gps_l1_ca_code_gen_complex_sampled(prns[ch], 4000000));
            svc.request(ch, prns[ch], codes.back().data(),
                [&](uint32_t c, const gsdr_acq_result& r, bool pos) { answers.push_back({c, r, pos}); });
        }
    EXPECT(svc.pending() == 4, "four pending requests");
    svc.work(capture.data(), 4000);
    EXPECT(svc.grids_run() == 1 && answers.size() == 4 && svc.pending() == 0, "one grid answers every request");
    // channel 0 re-arms, the others stay idle: the second block runs a 1-PRN grid
    svc.request(0, 1, codes[0].data(), [&](uint32_t c, const gsdr_acq_result& r, bool pos) { answers.push_back({c, r, pos}); });
    svc.work(capture.data() + 4000, 4000);
    EXPECT(svc.grids_run() == 2 && answers.size() == 5, "second grid for the re-armed channel");
    // reference: one engine per channel (the reference's one-PRN-per-block layout)
    for (size_t i = 0; i < answers.size(); ++i)
        {
            const uint32_t ch = answers[i].channel;
            const size_t blk = i < 4 ? 0 : 1;
            gsdr_acq_conf c{};
            c.fs_in = 4000000;
            c.consumed_samples = 4000;
            c.samples_per_code = conf.samples_per_code;
            c.samples_per_chip = conf.samples_per_chip;
            c.doppler_max = 5000;
            c.doppler_step = 250;
            c.pfa = 0.01F;
            c.max_dwells = 1;
            c.item_type = GSDR_ITEM_GR_COMPLEX;
            c.max_prns = 1;
            c.max_blocks = 1;
            c.sampled_ms = 1;
            c.ms_per_code = 1;
            gsdr_acq* one = nullptr;
            EXPECT(gsdr_acq_create(0, &c, &one) == GSDR_OK, "single engine");
            gsdr_acq_set_local_codes(one, reinterpret_cast<const float*>(codes[ch].data()), &prns[ch], 1);
            gsdr_acq_result r{};
            gsdr_acq_run(one, capture.data() + 4000 * blk, 1, 4000 * (blk + 1), &r);
            gsdr_acq_destroy(one);
            EXPECT(std::memcmp(&r, &answers[i].r, sizeof(r)) == 0, "batched answer == one-PRN engine");
        }
    EXPECT(answers[0].channel == 0 && answers[0].positive && std::abs(answers[0].r.acq_delay_samples - 524.0) < 1.0,
        "PRN 1 acquired at 524 samples");
    std::printf("acquisition service: %zu answers from %llu grids; PRN 1 stat %.2f (thr %.2f), positives:", answers.size(),
        static_cast<unsigned long long>(svc.grids_run()), answers[0].r.test_statistic, svc.threshold());
    for (const auto& a : answers) std::printf(" %u:%d", a.r.prn, a.positive ? 1 : 0);
    std::printf("\n");
}


// Feed an acquisition block like a GNU Radio source until it sends an event;
// returns the event (0: none before the data ran out).
template <class T>
int run_acquisition(pcps_acquisition_mi355x* blk, const T* data, size_t n, int chunk, int* last_event)
{
    size_t pos = 0;
    *last_event = 0;
    for (int guard = 0; guard < 100000 && *last_event == 0; ++guard)
        {
            const int m = static_cast<int>(std::min<size_t>(static_cast<size_t>(chunk), n - pos));
            const int used = blk->work(data + pos, m);
            pos += static_cast<size_t>(used);
            if (m == 0 && used == 0 && guard > 16) break;
        }
    return *last_event;
}

InMemoryConfiguration gps_acq_config(const std::string& extra_key = "", const std::string& extra_value = "")
{
    InMemoryConfiguration config;
    config.set_property("GNSS-SDR.internal_fs_sps", "4000000");
    config.set_property("Acquisition_1C.implementation", "GPS_L1_CA_PCPS_Acquisition_MI355X");
    config.set_property("Acquisition_1C.item_type", "gr_complex");
    config.set_property("Acquisition_1C.coherent_integration_time_ms", "1");
    config.set_property("Acquisition_1C.doppler_max", "5000");
    config.set_property("Acquisition_1C.doppler_step", "250");
    config.set_property("Acquisition_1C.blocking_on_standby", "true");
    if (!extra_key.empty()) config.set_property(extra_key, extra_value);
    return config;
}

// max_dwells = 2 across two general_work calls (pcps_acquisition.cc:672-680,
// :815-829): with an unreachable threshold the block integrates both blocks and
// reports negative after the second; its statistic equals the one-shot dwell
// engine's (gsdr_acq_run over the two-block attempt); with threshold 0 the first
// dwell is positive and the counter resets.
void test_acquisition_dwells(const std::vector<std::complex<float>>& capture)
{
    for (const char* pfa : {"0", "0.01"})
        {
            InMemoryConfiguration config = gps_acq_config("Acquisition_1C.max_dwells", "2");
            config.set_property("Acquisition_1C.pfa", pfa);
            Gnss_Synchro gs{};
            gs.System = 'G';
            gs.Signal[0] = '1';
            gs.Signal[1] = 'C';
            gs.PRN = 1;
            GpsL1CaPcpsAcquisitionMI355X acq(&config, "Acquisition_1C", 1, 0);
            int ev = 0;
            int events = 0;
            acq.get_block()->set_event_handler([&](int e) {
                ev = e;
                ++events;
            });
            acq.set_gnss_synchro(&gs);
            acq.set_local_code();
            acq.set_state(1);
            acq.init();
            acq.get_block()->start();
            const bool cfar = std::string(pfa) != "0";
            if (!cfar) acq.get_block()->set_threshold(1e30F);
            // the CFAR threshold comes from pfa with 2 dwells; make it unreachable too
            if (cfar) acq.get_block()->set_threshold(1e30F);
            run_acquisition(acq.get_block(), capture.data(), capture.size(), 1000, &ev);
            EXPECT(ev == 2 && events == 1, "max_dwells=2, unreachable threshold: one negative after the second dwell");
            EXPECT(gs.Acq_samplestamp_samples == 8000ULL, "decision on the second block");
            const float stat_block = acq.get_block()->test_statistics();
            // one-shot: both dwells of the attempt in one engine call
            gsdr_acq_conf c{};
            c.fs_in = 4000000;
            c.consumed_samples = 4000;
            c.samples_per_code = 4000.0F;
            c.samples_per_chip = 4;
            c.doppler_max = 5000;
            c.doppler_step = 250;
            c.pfa = cfar ? 0.01F : 0.0F;
            c.max_dwells = 2;
            c.item_type = GSDR_ITEM_GR_COMPLEX;
            c.max_prns = 1;
            c.max_blocks = 1;
            c.sampled_ms = 1;
            c.ms_per_code = 1;
            gsdr_acq* one = nullptr;
            EXPECT(gsdr_acq_create(0, &c, &one) == GSDR_OK, "dwell engine");
            const auto code = gps_l1_ca_code_gen_complex_sampled(1, 4000000);
            const uint32_t prn = 1;
            gsdr_acq_set_local_codes(one, reinterpret_cast<const float*>(code.data()), &prn, 1);
            gsdr_acq_set_threshold(one, 1e30F);
            gsdr_acq_result r{};
            EXPECT(gsdr_acq_run(one, capture.data(), 1, 4000, &r) == GSDR_OK, "dwell engine run");
            gsdr_acq_destroy(one);
            EXPECT(r.num_dwells == 2, "one-shot attempt reports its last dwell");
            EXPECT(std::abs(r.test_statistic - stat_block) <= 1e-5F * std::abs(r.test_statistic),
                "per-call dwell statistic == one-shot dwell statistic");
            EXPECT(std::abs(gs.Acq_delay_samples - r.acq_delay_samples) < 0.5 &&
                       std::abs(gs.Acq_doppler_hz - r.doppler_hz) < 0.5,
                "per-call dwell cell == one-shot dwell cell");
            std::printf("dwells (pfa %s): per-call stat %.5f, one-shot %.5f, delay %.0f doppler %.0f\n", pfa, stat_block,
                r.test_statistic, gs.Acq_delay_samples, gs.Acq_doppler_hz);
            // threshold 0: positive on the first dwell, counter reset
            acq.get_block()->set_threshold(0.0F);
            acq.set_state(1);
            ev = 0;
            events = 0;
            run_acquisition(acq.get_block(), capture.data(), capture.size(), 1000, &ev);
            EXPECT(ev == 1 && acq.get_block()->num_noncoherent_integrations() == 0, "positive first dwell resets the counter");
            EXPECT(std::abs(gs.Acq_delay_samples - 524.0) < 1.0, "PRN 1 at 524 samples");
        }
}

// bit_transition_flag (pcps_acquisition.cc:71, :85-92, :831-869): a 2 ms buffer,
// the code in the second half of the 8000-point FFT, every call decides.
void test_acquisition_bit_transition(const std::vector<std::complex<float>>& capture)
{
    InMemoryConfiguration config = gps_acq_config("Acquisition_1C.bit_transition_flag", "true");
    config.set_property("Acquisition_1C.pfa", "0.01");
    Gnss_Synchro gs{};
    gs.System = 'G';
    gs.Signal[0] = '1';
    gs.Signal[1] = 'C';
    gs.PRN = 1;
    GpsL1CaPcpsAcquisitionMI355X acq(&config, "Acquisition_1C", 1, 0);
    int ev = 0;
    acq.get_block()->set_event_handler([&](int e) { ev = e; });
    acq.set_gnss_synchro(&gs);
    acq.set_local_code();
    acq.set_state(1);
    acq.init();
    acq.get_block()->start();
    run_acquisition(acq.get_block(), capture.data(), capture.size(), 1000, &ev);
    EXPECT(ev == 1, "bit transition: positive");
    EXPECT(std::abs(gs.Acq_delay_samples - 524.0) < 1.0 && std::abs(gs.Acq_doppler_hz - 1680.0) <= 666.0,
        "bit transition: 524 samples / 1680 Hz");
    EXPECT(gs.Acq_samplestamp_samples == 8000ULL, "bit transition: one 8000-sample buffer");
    // a negative bit-transition call: unreachable threshold, no re-arm (:858-868)
    acq.get_block()->set_threshold(1e30F);
    acq.set_state(1);
    ev = 0;
    run_acquisition(acq.get_block(), capture.data(), capture.size(), 1000, &ev);
    EXPECT(ev == 2, "bit transition: immediate negative");
    std::printf("bit transition: delay %.0f doppler %.0f stat %.2f\n", gs.Acq_delay_samples, gs.Acq_doppler_hz,
        acq.get_block()->test_statistics());
}

// item_type=cbyte: interleaved int8 I/Q (complex_byte_to_float_x2 + float_to_complex)
void test_acquisition_cbyte(const std::vector<std::complex<float>>& capture)
{
    std::vector<int8_t> bytes(2 * capture.size());
    for (size_t i = 0; i < capture.size(); ++i)
        {
            bytes[2 * i] = static_cast<int8_t>(std::lrint(std::max(-127.0F, std::min(127.0F, 1000.0F * capture[i].real()))));
            bytes[2 * i + 1] = static_cast<int8_t>(std::lrint(std::max(-127.0F, std::min(127.0F, 1000.0F * capture[i].imag()))));
        }
    InMemoryConfiguration config = gps_acq_config("Acquisition_1C.item_type", "cbyte");
    config.set_property("Acquisition_1C.pfa", "0.01");
    Gnss_Synchro gs{};
    gs.System = 'G';
    gs.Signal[0] = '1';
    gs.Signal[1] = 'C';
    gs.PRN = 1;
    GpsL1CaPcpsAcquisitionMI355X acq(&config, "Acquisition_1C", 1, 0);
    EXPECT(acq.item_size() == 2, "cbyte item size");
    int ev = 0;
    acq.get_block()->set_event_handler([&](int e) { ev = e; });
    acq.set_gnss_synchro(&gs);
    acq.set_local_code();
    acq.set_state(1);
    acq.init();
    acq.get_block()->start();
    size_t pos = 0;
    for (int guard = 0; guard < 100 && ev == 0; ++guard)
        {
            const int m = static_cast<int>(std::min<size_t>(1000, capture.size() - pos));
            pos += static_cast<size_t>(acq.get_block()->work(bytes.data() + 2 * pos, m));
        }
    EXPECT(ev == 1 && std::abs(gs.Acq_delay_samples - 524.0) < 1.0, "cbyte: PRN 1 acquired at 524 samples");
    bool threw = false;
    try
        {
            InMemoryConfiguration bad = gps_acq_config("Acquisition_1C.item_type", "ishort");
            GpsL1CaPcpsAcquisitionMI355X b(&bad, "Acquisition_1C", 1, 0);
        }
    catch (const std::invalid_argument&)
        {
            threw = true;
        }
    EXPECT(threw, "unknown item type -> std::invalid_argument");
    std::printf("cbyte: delay %.0f doppler %.0f\n", gs.Acq_delay_samples, gs.Acq_doppler_hz);
}

void test_galileo_acquisition(const std::vector<std::complex<float>>& capture)
{
    InMemoryConfiguration config;
    config.set_property("Acquisition_1B.implementation", "Galileo_E1_PCPS_Ambiguous_Acquisition_MI355X");
    config.set_property("GNSS-SDR.internal_fs_sps", "4000000");
    config.set_property("Acquisition_1B.item_type", "gr_complex");
    config.set_property("Acquisition_1B.coherent_integration_time_ms", "4");
    config.set_property("Acquisition_1B.dump", "false");
    config.set_property("Acquisition_1B.pfa", "0.001");
    config.set_property("Acquisition_1B.doppler_max", "10000");
    config.set_property("Acquisition_1B.doppler_step", "250");
    config.set_property("Acquisition_1B.repeat_satellite", "false");
    config.set_property("Acquisition_1B.cboc", "true");
    Gnss_Synchro gs{};
    gs.Channel_ID = 0;
    gs.System = 'E';
    gs.Signal[0] = '1';
    gs.Signal[1] = 'B';
    gs.PRN = 1;
    auto acq_ = gsdr_factory::GetAcqBlock(&config, "Acquisition_1B", 1, 0, 0);
    auto* acquisition = dynamic_cast<GalileoE1PcpsAmbiguousAcquisitionMI355X*>(acq_.get());
    EXPECT(acquisition != nullptr, "factory builds the Galileo adapter");
    if (!acquisition) return;
    int ev = 0;
    acquisition->get_block()->set_event_handler([&](int e) { ev = e; });
    acquisition->set_channel(gs.Channel_ID);
    acquisition->set_gnss_synchro(&gs);
    acquisition->set_threshold(config.property("Acquisition_1B.threshold", 1e-9F));
    acquisition->set_doppler_max(10000);
    acquisition->set_doppler_step(250);
    acquisition->set_local_code();
    acquisition->init();
    acquisition->reset();
    acquisition->set_state(1);
    acquisition->get_block()->start();
    run_acquisition(acquisition->get_block(), capture.data(), capture.size(), 4096, &ev);
    EXPECT(ev == 1, "Galileo: Acquisition failure. Expected message: 1=ACQ SUCCESS.");
    const double delay_error_samples = std::abs(2920.0 - gs.Acq_delay_samples);
    const auto delay_error_chips = static_cast<float>(delay_error_samples * 1023 / 4000000);
    const double doppler_error_hz = std::abs(-632.0 - gs.Acq_doppler_hz);
    EXPECT(doppler_error_hz <= 166, "Galileo: Doppler error exceeds 166 Hz");
    EXPECT(delay_error_chips < 0.175, "Galileo: Delay error exceeds 0.175 chips");
    std::printf("galileo acquisition: message %d delay %.1f samples doppler %.0f Hz stat %.2f (thr %.2f)\n", ev,
        gs.Acq_delay_samples, gs.Acq_doppler_hz, acquisition->get_block()->test_statistics(),
        acquisition->get_block()->threshold());
}

void test_beidou_acquisition()
{
    const double fs = 4000000.0;
    SynthSat s{beidou_b1i_code_gen_float(6), 2.046e6, 1561.098e6, 1234.0, 2000.0, 0.2, {}, {}, 0.02};
    const auto x = synth_stream({s}, fs, 8000, 7, 1.0);
    InMemoryConfiguration config;
    config.set_property("GNSS-SDR.internal_fs_sps", "4000000");
    config.set_property("Acquisition_B1.implementation", "BEIDOU_B1I_PCPS_Acquisition_MI355X");
    config.set_property("Acquisition_B1.item_type", "gr_complex");
    config.set_property("Acquisition_B1.coherent_integration_time_ms", "1");
    config.set_property("Acquisition_B1.pfa", "0.01");
    config.set_property("Acquisition_B1.doppler_max", "5000");
    config.set_property("Acquisition_B1.doppler_step", "250");
    config.set_property("Acquisition_B1.blocking_on_standby", "true");
    Gnss_Synchro gs{};
    gs.System = 'C';
    gs.Signal[0] = 'B';
    gs.Signal[1] = '1';
    gs.PRN = 6;
    auto acq_ = gsdr_factory::GetAcqBlock(&config, "Acquisition_B1", 1, 0, 0);
    auto* acq = dynamic_cast<BeidouB1iPcpsAcquisitionMI355X*>(acq_.get());
    EXPECT(acq != nullptr, "factory builds the BeiDou adapter");
    if (!acq) return;
    int ev = 0;
    acq->get_block()->set_event_handler([&](int e) { ev = e; });
    acq->set_gnss_synchro(&gs);
    acq->init();  // loads the replica (beidou_b1i_pcps_acquisition.cc:135-139)
    acq->set_state(1);
    acq->get_block()->start();
    run_acquisition(acq->get_block(), x.data(), x.size(), 1000, &ev);
    // code start 1234 samples after the block start; the grid is 250 Hz
    EXPECT(ev == 1 && std::abs(gs.Acq_delay_samples - 1234.0) <= 1.0 && std::abs(gs.Acq_doppler_hz - 2000.0) <= 125.0,
        "BeiDou B1I synthetic: PRN 6 at 1234 samples / 2000 Hz");
    std::printf("beidou acquisition: message %d delay %.1f doppler %.0f stat %.2f\n", ev, gs.Acq_delay_samples,
        gs.Acq_doppler_hz, acq->get_block()->test_statistics());
}

// End of input: the block computes what it was handed (flush) and hands out the
// remaining outputs, one per work() call without new items.
template <class F>
void drain_block(TrackingBlockMI355X* blk, uint64_t nread, F&& take)
{
    blk->flush();
    for (int guard = 0; guard < 100000; ++guard)
        {
            Gnss_Synchro out{};
            int nout = 0;
            blk->work(nullptr, 0, nread, &out, &nout);
            if (nout == 0) break;
            take(out, nout);
        }
}

// Channel-level hand-off: acquisition adapter -> Gnss_Synchro -> tracking adapter
// start_tracking (ChannelFsm::start_tracking, channel_fsm.cc:204-208), then the
// tracking block's general_work over the rest of the stream in GNU-Radio-sized
// chunks; Gnss_Synchro records out.
struct HandOff
{
    int outputs{0};
    int loss{0};
    double doppler{0.0};
    double cn0{0.0};
    double prompt_i{0.0}, prompt_q{0.0};
    bool pll_locked{false};
};

HandOff run_handoff(AcquisitionInterface* acq, pcps_acquisition_mi355x* ablk, TrackingInterface* trk,
    TrackingBlockMI355X* tblk, Gnss_Synchro* gs, const std::vector<std::complex<float>>& x)
{
    HandOff h;
    int ev = 0;
    ablk->set_event_handler([&](int e) { ev = e; });
    acq->set_gnss_synchro(gs);
    acq->set_local_code();
    acq->init();
    acq->set_state(1);
    ablk->start();
    size_t pos = 0;
    for (int guard = 0; guard < 1000 && ev == 0 && pos < x.size(); ++guard)
        pos += static_cast<size_t>(ablk->work(x.data() + pos, static_cast<int>(std::min<size_t>(4096, x.size() - pos))));
    EXPECT(ev == 1, "hand-off: acquisition positive");
    if (ev != 1) return h;
    trk->set_gnss_synchro(gs);
    trk->start_tracking();
    tblk->set_event_handler([&](int e) {
        if (e == 3) ++h.loss;
    });
    // the tracking block sees the stream from the acquisition stamp on
    uint64_t nread = gs->Acq_samplestamp_samples;
    std::vector<double> dop;
    const uint64_t settle = gs->Acq_samplestamp_samples + 4 * static_cast<uint64_t>(std::max(tblk->forecast(), 4000));
    tblk->set_record_sink([&](const gsdr_trk_epoch& r) {
        // every call's record (the loop state after the call), incl. state 2
        if (r.sample_counter > settle)
            {
                dop.push_back(r.carrier_doppler_hz);
                h.cn0 = r.cn0_db_hz;
            }
    });
    auto take = [&](const Gnss_Synchro& out, int nout) {
        if (nout == 1 && out.Flag_valid_symbol_output)
            {
                ++h.outputs;
                h.prompt_i = out.Prompt_I;
                h.prompt_q = out.Prompt_Q;
                h.pll_locked = true;
            }
    };
    while (nread + static_cast<uint64_t>(tblk->forecast()) <= x.size())
        {
            Gnss_Synchro out{};
            int nout = 0;
            // GNU Radio honours the block's forecast (2 x vector_length items for the
            // per-channel block)
            const int avail = static_cast<int>(
                std::min<uint64_t>(std::max<uint64_t>(8192, static_cast<uint64_t>(tblk->forecast())), x.size() - nread));
            const int used = tblk->work(x.data() + nread, avail, nread, &out, &nout);
            take(out, nout);
            if (used <= 0 && nout == 0) break;
            nread += static_cast<uint64_t>(std::max(used, 0));
        }
    drain_block(tblk, nread, take);
    tblk->set_record_sink(nullptr);
    const size_t k = std::min<size_t>(dop.size(), 20);
    for (size_t i = dop.size() - k; i < dop.size(); ++i) h.doppler += dop[i] / static_cast<double>(k);
    return h;
}

void test_tracking_handoff()
{
    const double fs = 4000000.0;
    // GPS L1 C/A, PRN 1: code start 524.3 samples, 1680 Hz, 50 dB-Hz (A^2/(2 sigma^2) fs)
    const double sigma = 1.0;
    const double amp_gps = std::sqrt(2.0 * std::pow(10.0, 5.0) / fs) * sigma;
    // navigation symbols: the TLM preamble 10001011 repeated, 20 ms per bit, so the
    // 160-symbol bit-synchronisation pattern (GPS_CA_PREAMBLE_SYMBOLS_STR) is found
    const std::vector<float> bits = {1, -1, -1, -1, 1, -1, 1, 1};
    SynthSat g{gps_l1_ca_code_gen_float(1), 1.023e6, 1575.42e6, 524.3, 1680.0, amp_gps, {}, bits, 0.02};
    // pull_in_time_s = 0 ends the pull-in transitory after 1 s (integer seconds,
    // dll_pll_veml_tracking.cc:1797), then bit synchronisation and state 4 outputs
    const auto x = synth_stream({g}, fs, static_cast<size_t>(fs * 1.7), 11, sigma);
    InMemoryConfiguration config = gps_acq_config();
    config.set_property("Acquisition_1C.pfa", "0.01");
    config.set_property("Tracking_1C.implementation", "GPS_L1_CA_DLL_PLL_Tracking_MI355X");
    config.set_property("Tracking_1C.item_type", "gr_complex");
    config.set_property("Tracking_1C.pll_bw_hz", "40.0");  // conf/gnss-sdr_GPS_L1_gr_complex.conf:66-67
    config.set_property("Tracking_1C.dll_bw_hz", "4.0");
    config.set_property("Tracking_1C.pull_in_time_s", "0");
    Gnss_Synchro gs{};
    gs.System = 'G';
    gs.Signal[0] = '1';
    gs.Signal[1] = 'C';
    gs.PRN = 1;
    auto acq = gsdr_factory::GetAcqBlock(&config, "Acquisition_1C", 1, 0, 0);
    auto trk = gsdr_factory::GetTrkBlock(&config, "Tracking_1C", 1, 1, 0);
    auto* gacq = dynamic_cast<GpsL1CaPcpsAcquisitionMI355X*>(acq.get());
    auto* gtrk = dynamic_cast<GpsL1CaDllPllTrackingMI355X*>(trk.get());
    EXPECT(gacq && gtrk, "factory builds the GPS acquisition and tracking adapters");
    if (!gacq || !gtrk) return;
    EXPECT(gtrk->conf().vector_length == 4000U && gtrk->item_size() == 8, "GPS tracking: vector_length 4000");
    const HandOff h = run_handoff(gacq, gacq->get_block(), gtrk, gtrk->get_block(), &gs, x);
    EXPECT(h.outputs > 8 && h.loss == 0, "GPS hand-off: bit-synchronised Gnss_Synchro outputs (one per 20 ms bit), no loss of lock");
    EXPECT(std::abs(h.doppler - 1680.0) < 3.0, "GPS hand-off: carrier Doppler converged to 1680 Hz");
    EXPECT(h.cn0 > 44.0 && h.cn0 < 56.0, "GPS hand-off: CN0 estimate near 50 dB-Hz");
    EXPECT(std::abs(h.prompt_i) > 4.0 * std::abs(h.prompt_q), "GPS hand-off: carrier phase locked (|I| >> |Q|)");
    std::printf("gps hand-off: %d outputs, doppler %.2f Hz, CN0 %.1f dB-Hz, prompt (%.1f, %.1f), losses %d\n",
        h.outputs, h.doppler, h.cn0, h.prompt_i, h.prompt_q, h.loss);

    // Galileo E1: E1-B data + E1-C pilot with its secondary code, sinBOC(1,1)
    // replicas at 2 samples per chip, 4 ms code, pilot tracking (track_pilot)
    const double amp_gal = std::sqrt(2.0 * std::pow(10.0, 5.0) / fs) * sigma / std::sqrt(2.0);
    std::vector<float> sec(25);
    const char* sec_str = "0011100000001010110110010";
    for (int i = 0; i < 25; ++i) sec[i] = sec_str[i] == '0' ? 1.0F : -1.0F;
    auto e1c = galileo_e1_code_gen_sinboc11_float("1C", 11);
    for (auto& v : e1c) v = -v;  // E1-C enters the composite signal with a minus sign
    SynthSat gb{galileo_e1_code_gen_sinboc11_float("1B", 11), 2.046e6, 1575.42e6, 2920.0, -632.0, amp_gal, {}, {}, 0.02};
    SynthSat gc{e1c, 2.046e6, 1575.42e6, 2920.0, -632.0, amp_gal, sec, {}, 0.02};
    const auto y = synth_stream({gb, gc}, fs, static_cast<size_t>(fs * 1.5), 13, sigma);
    InMemoryConfiguration gcfg;
    gcfg.set_property("GNSS-SDR.internal_fs_sps", "4000000");
    gcfg.set_property("Acquisition_1B.implementation", "Galileo_E1_PCPS_Ambiguous_Acquisition_MI355X");
    gcfg.set_property("Acquisition_1B.item_type", "gr_complex");
    gcfg.set_property("Acquisition_1B.coherent_integration_time_ms", "4");
    gcfg.set_property("Acquisition_1B.pfa", "0.01");
    gcfg.set_property("Acquisition_1B.doppler_max", "5000");
    gcfg.set_property("Acquisition_1B.doppler_step", "125");
    gcfg.set_property("Acquisition_1B.blocking_on_standby", "true");
    gcfg.set_property("Tracking_1B.implementation", "Galileo_E1_DLL_PLL_VEML_Tracking_MI355X");
    gcfg.set_property("Tracking_1B.item_type", "gr_complex");
    gcfg.set_property("Tracking_1B.pll_bw_hz", "15.0");
    gcfg.set_property("Tracking_1B.dll_bw_hz", "2.0");
    gcfg.set_property("Tracking_1B.pull_in_time_s", "0");
    Gnss_Synchro es{};
    es.System = 'E';
    es.Signal[0] = '1';
    es.Signal[1] = 'B';
    es.PRN = 11;
    auto eacq_ = gsdr_factory::GetAcqBlock(&gcfg, "Acquisition_1B", 1, 0, 0);
    auto etrk_ = gsdr_factory::GetTrkBlock(&gcfg, "Tracking_1B", 1, 1, 0);
    auto* eacq = dynamic_cast<GalileoE1PcpsAmbiguousAcquisitionMI355X*>(eacq_.get());
    auto* etrk = dynamic_cast<GalileoE1DllPllVemlTrackingMI355X*>(etrk_.get());
    EXPECT(eacq && etrk, "factory builds the Galileo acquisition and tracking adapters");
    if (!eacq || !etrk) return;
    EXPECT(etrk->conf().vector_length == 16000U && etrk->conf().track_pilot, "Galileo tracking: 16000 samples, pilot");
    const HandOff e = run_handoff(eacq, eacq->get_block(), etrk, etrk->get_block(), &es, y);
    EXPECT(e.outputs > 40 && e.loss == 0, "Galileo hand-off: secondary-code-locked Gnss_Synchro outputs (one per 4 ms), no loss of lock");
    EXPECT(std::abs(e.doppler + 632.0) < 3.0, "Galileo hand-off: carrier Doppler converged to -632 Hz");
    // the pilot carries half the 50 dB-Hz composite (47 dB-Hz); the M2M4 estimate
    // on the E1-C prompt reads a few dB under it
    EXPECT(e.cn0 > 40.0 && e.cn0 < 50.0, "Galileo hand-off: CN0 estimate of the 47 dB-Hz pilot");
    std::printf("galileo hand-off: %d outputs, doppler %.2f Hz, CN0 %.1f dB-Hz, prompt (%.1f, %.1f), losses %d\n",
        e.outputs, e.doppler, e.cn0, e.prompt_i, e.prompt_q, e.loss);
}

// The receiver on the device IQ ring: the stream pushed once into
// the GPU's ring in 4096-item chunks; the batched acquisition service runs its
// grids in place on the ring (answers identical to the host-buffer service) and
// the tracking pool, started from the positive answers' Gnss_Synchro, advances
// over the ring after every push.
void test_receiver_on_ring()
{
    const double fs = 4000000.0;
    const double sigma = 1.0;
    const double amp = std::sqrt(2.0 * std::pow(10.0, 5.0) / fs) * sigma;
    const std::vector<float> bits = {1, -1, -1, -1, 1, -1, 1, 1};
    SynthSat a{gps_l1_ca_code_gen_float(1), 1.023e6, 1575.42e6, 524.3, 1680.0, amp, {}, bits, 0.02};
    SynthSat b{gps_l1_ca_code_gen_float(7), 1.023e6, 1575.42e6, 2100.8, -3250.0, amp, {}, bits, 0.02};
    const auto x = synth_stream({a, b}, fs, static_cast<size_t>(fs * 1.6), 17, sigma);
    InMemoryConfiguration config = gps_acq_config();
    config.set_property("Acquisition_1C.pfa", "0.01");
    config.set_property("Acquisition_1C.doppler_max", "5000");
    config.set_property("Acquisition_1C.doppler_step", "250");
    config.set_property("Tracking_1C.pll_bw_hz", "40.0");
    config.set_property("Tracking_1C.dll_bw_hz", "4.0");
    config.set_property("Tracking_1C.pull_in_time_s", "0");
    Acq_Conf aconf;
    aconf.ms_per_code = 1;
    aconf.SetFromConfiguration(&config, "Acquisition_1C", 1023000.0, 2000000.0);
    Dll_Pll_Conf tconf;
    tconf.SetFromConfiguration(&config, "Tracking_1C");
    tconf.vector_length = 4000;
    tconf.track_pilot = false;
    gsdr_stream* ring = nullptr;
    EXPECT(gsdr_stream_create(0, GSDR_ITEM_GR_COMPLEX, 64 * 4000, 32 * 4000, &ring) == GSDR_OK, "ring");
    if (!ring) return;
    AcquisitionService svc_ring(aconf, 4, 0), svc_host(aconf, 4, 0);
    TrackingPool pool(tconf, GSDR_SIGNAL_GPS_1C, 4, ring, 0);
    const uint32_t prns[3] = {1, 7, 20};
    std::vector<std::vector<std::complex<float>>> codes;
    std::vector<Gnss_Synchro> gs(3);
    struct Ans
    {
        gsdr_acq_result r;
        bool pos;
    };
    std::vector<Ans> ans_ring(3), ans_host(3);
    std::vector<int> answered(3, 0);
    uint64_t head = 0;
    for (uint32_t ch = 0; ch < 3; ++ch)
        {
            codes.push_back(gps_l1_ca_code_gen_complex_sampled(prns[ch], 4000000));
            gs[ch].System = 'G';
            gs[ch].Signal[0] = '1';
            gs[ch].Signal[1] = 'C';
            gs[ch].PRN = prns[ch];
            gs[ch].Channel_ID = static_cast<int32_t>(ch);
            svc_ring.request(ch, prns[ch], codes[ch].data(), [&](uint32_t c, const gsdr_acq_result& r, bool pos) {
                ans_ring[c] = {r, pos};
                answered[c] = 1;
                if (pos)
                    {
                        gs[c].Acq_delay_samples = r.acq_delay_samples;
                        gs[c].Acq_doppler_hz = r.doppler_hz;
                        gs[c].Acq_samplestamp_samples = r.samplestamp;
                        pool.start(c, &gs[c], head);
                    }
            });
            svc_host.request(ch, prns[ch], codes[ch].data(),
                [&](uint32_t c, const gsdr_acq_result& r, bool pos) { ans_host[c] = {r, pos}; });
        }
    std::vector<int> outputs(3, 0);
    std::vector<double> last_dop(3, 0.0);
    svc_ring.work_ring(ring, 0);  // origin of the ring's block grid
    size_t pos = 0;
    while (pos < x.size())
        {
            const size_t n = std::min<size_t>(4096, x.size() - pos);
            if (gsdr_stream_push(ring, x.data() + pos, pos, n) != GSDR_OK) break;
            pos += n;
            head = pos;
            svc_ring.work_ring(ring, head);
            svc_host.work(x.data() + pos - n, static_cast<int>(n));
            pool.advance([&](uint32_t slot, const Gnss_Synchro& o) {
                if (o.Flag_valid_symbol_output) ++outputs[slot];
                last_dop[slot] = o.Carrier_Doppler_hz;
            });
        }
    for (int c = 0; c < 3; ++c)
        EXPECT(answered[c] && std::memcmp(&ans_ring[c].r, &ans_host[c].r, sizeof(gsdr_acq_result)) == 0,
            "ring acquisition answer == host-buffer answer");
    EXPECT(ans_ring[0].pos && ans_ring[1].pos && !ans_ring[2].pos, "PRN 1 and 7 acquired, PRN 20 not");
    EXPECT(outputs[0] > 8 && outputs[1] > 8, "tracking pool: bit-synchronised outputs on both channels");
    EXPECT(std::abs(last_dop[0] - 1680.0) < 3.0 && std::abs(last_dop[1] + 3250.0) < 3.0,
        "tracking pool: Doppler converged on both channels");
    std::printf("receiver on ring: acq PRN1 %d PRN7 %d PRN20 %d; pool outputs %d / %d, doppler %.2f / %.2f Hz\n",
        ans_ring[0].pos ? 1 : 0, ans_ring[1].pos ? 1 : 0, ans_ring[2].pos ? 1 : 0, outputs[0], outputs[1], last_dop[0],
        last_dop[1]);
    gsdr_stream_destroy(ring);
}


// A channel FSM that counts the events the acquisition block fires at it.
class CountingFsm : public ChannelFsm
{
public:
    int valid{0};
    bool Event_valid_acquisition() override
    {
        ++valid;
        return true;
    }
};

// Channel's constructor hands the acquisition adapter its FSM (channel.cc:50);
// the block then reports a positive acquisition through it instead of event 1
// (pcps_acquisition.cc:370-377), and a negative one still as event 2.
void test_channel_fsm_handoff(const std::vector<std::complex<float>>& capture)
{
    InMemoryConfiguration config = gps_acq_config();
    config.set_property("Acquisition_1C.pfa", "0.01");
    auto acq_ = gsdr_factory::GetAcqBlock(&config, "Acquisition_1C", 1, 0, 0);
    auto* acq = dynamic_cast<GpsL1CaPcpsAcquisitionMI355X*>(acq_.get());
    EXPECT(acq != nullptr, "factory builds the GPS acquisition adapter");
    if (!acq) return;
    auto fsm = std::make_shared<CountingFsm>();
    acq->set_channel_fsm(fsm);
    Gnss_Synchro gs{};
    gs.System = 'G';
    gs.Signal[0] = '1';
    gs.Signal[1] = 'C';
    gs.PRN = 1;
    int ev = 0, last = 0;
    acq->get_block()->set_event_handler([&](int e) {
        ++ev;
        last = e;
    });
    acq->set_gnss_synchro(&gs);
    acq->set_local_code();
    acq->init();
    acq->set_state(1);
    acq->get_block()->start();
    for (size_t pos = 0; pos < 8000 && fsm->valid == 0;)
        pos += static_cast<size_t>(acq->get_block()->work(capture.data() + pos, static_cast<int>(std::min<size_t>(1000, 8000 - pos))));
    EXPECT(fsm->valid == 1 && ev == 0, "set_channel_fsm: positive -> ChannelFsm::Event_valid_acquisition, no event 1");
    EXPECT(std::abs(gs.Acq_delay_samples - 524.0) < 1.0, "set_channel_fsm: PRN 1 at 524 samples");
    // PRN 20 is absent: the negative result still goes out as event 2
    gs.PRN = 20;
    acq->set_local_code();
    acq->init();
    acq->set_state(1);
    acq->get_block()->start();
    for (size_t pos = 0; pos < 8000 && ev == 0;)
        pos += static_cast<size_t>(acq->get_block()->work(capture.data() + pos, static_cast<int>(std::min<size_t>(1000, 8000 - pos))));
    EXPECT(fsm->valid == 1 && ev == 1 && last == 2, "set_channel_fsm: negative -> event 2");
    // an expired FSM falls back to the message port (event 1)
    fsm.reset();
    gs.PRN = 1;
    ev = 0;
    acq->set_local_code();
    acq->init();
    acq->set_state(1);
    acq->get_block()->start();
    for (size_t pos = 0; pos < 8000 && ev == 0;)
        pos += static_cast<size_t>(acq->get_block()->work(capture.data() + pos, static_cast<int>(std::min<size_t>(1000, 8000 - pos))));
    EXPECT(ev == 1 && last == 1, "expired channel FSM: positive -> event 1");
    std::printf("channel fsm hand-off: Event_valid_acquisition, negative event 2, expired FSM event 1\n");
}

// gnss_sdr_flags.cc:41-58 defaults into Dll_Pll_Conf, and the command-line
// overrides of the .conf (dll_pll_conf.cc:24-28, :53-63; the acquisition
// adapters' --doppler_max, gps_l1_ca_pcps_acquisition.cc:57-60).
void test_flag_overrides()
{
    InMemoryConfiguration config = gps_acq_config();
    config.set_property("Tracking_1C.pll_bw_hz", "40.0");
    config.set_property("Tracking_1C.dll_bw_hz", "4.0");
    Dll_Pll_Conf a;
    a.SetFromConfiguration(&config, "Tracking_1C");
    EXPECT(a.pll_bw_hz == 40.0F && a.dll_bw_hz == 4.0F, ".conf bandwidths without flags");
    EXPECT(a.cn0_samples == 20 && a.cn0_min == 25 && a.max_code_lock_fail == 50 && a.max_carrier_lock_fail == 5000 &&
               a.carrier_lock_th == 0.7,
        "lock-detector defaults from the gflags");
    FLAGS_pll_bw_hz = 25.0;
    FLAGS_dll_bw_hz = 1.5;
    FLAGS_cn0_min = 30;
    FLAGS_doppler_max = 7000;
    Dll_Pll_Conf b;
    b.SetFromConfiguration(&config, "Tracking_1C");
    EXPECT(b.pll_bw_hz == 25.0F && b.dll_bw_hz == 1.5F, "--pll_bw_hz / --dll_bw_hz override the .conf");
    EXPECT(b.cn0_min == 30, "--cn0_min sets the default");
    auto acq_ = gsdr_factory::GetAcqBlock(&config, "Acquisition_1C", 1, 0, 0);
    auto* acq = dynamic_cast<GpsL1CaPcpsAcquisitionMI355X*>(acq_.get());
    EXPECT(acq && acq->conf().doppler_max == 7000, "--doppler_max overrides Acquisition_1C.doppler_max");
    FLAGS_pll_bw_hz = 0.0;
    FLAGS_dll_bw_hz = 0.0;
    FLAGS_cn0_min = 25;
    FLAGS_doppler_max = 0;
}

// Several GPS channels tracked by factory-built blocks in GNU Radio fashion: every
// block's work() is called in turn on the shared input from its own nitems_read.
// pooled = false: one engine handle per channel (a synchronous H2D + launch + D2H
// per general_work call); true: one shared pool per GPU over the device ring.
struct PoolRun
{
    std::vector<std::vector<gsdr_trk_epoch>> recs;
    std::vector<int> outputs;
    double seconds{0.0};
    uint64_t calls{0};
};

PoolRun run_tracking_blocks(bool pooled, const std::vector<std::complex<float>>& x, const std::vector<Gnss_Synchro>& acq,
    const std::string& dump_filename)
{
    InMemoryConfiguration config;
    config.set_property("GNSS-SDR.internal_fs_sps", "4000000");
    config.set_property("Tracking_1C.implementation", "GPS_L1_CA_DLL_PLL_Tracking_MI355X");
    config.set_property("Tracking_1C.item_type", "gr_complex");
    config.set_property("Tracking_1C.pll_bw_hz", "40.0");
    config.set_property("Tracking_1C.dll_bw_hz", "4.0");
    config.set_property("Tracking_1C.pull_in_time_s", "0");
    config.set_property("Channels_1C.count", std::to_string(acq.size()));
    config.set_property("Tracking_1C.mi355x_pool", pooled ? "true" : "false");
    if (!dump_filename.empty())
        {
            config.set_property("Tracking_1C.dump", "true");
            config.set_property("Tracking_1C.dump_filename", dump_filename);
        }
    const size_t n = acq.size();
    std::vector<std::unique_ptr<TrackingInterface>> trk;
    std::vector<Gnss_Synchro> gs(acq);
    PoolRun r;
    r.recs.resize(n);
    r.outputs.assign(n, 0);
    std::vector<uint64_t> nread(n);
    for (size_t c = 0; c < n; ++c)
        {
            trk.push_back(gsdr_factory::GetTrkBlock(&config, "Tracking_1C", 1, 1, 0));
            trk[c]->set_channel(static_cast<unsigned int>(c));
            trk[c]->set_gnss_synchro(&gs[c]);
            trk[c]->start_tracking();
            nread[c] = gs[c].Acq_samplestamp_samples;
        }
    auto* a0 = dynamic_cast<DllPllTrackingAdapterMI355X*>(trk[0].get());
    EXPECT(a0 && a0->pooled() == pooled, "factory: pooled block iff Tracking_1C.mi355x_pool");
    std::vector<TrackingBlockMI355X*> blks(n);
    for (size_t c = 0; c < n; ++c)
        {
            blks[c] = dynamic_cast<DllPllTrackingAdapterMI355X*>(trk[c].get())->get_block();
            blks[c]->set_record_sink([&r, c](const gsdr_trk_epoch& e) {
                r.recs[c].push_back(e);
                ++r.calls;
            });
        }
    const auto t0 = std::chrono::steady_clock::now();
    bool progress = true;
    while (progress)
        {
            progress = false;
            for (size_t c = 0; c < n; ++c)
                {
                    auto* blk = blks[c];
                    if (nread[c] + static_cast<uint64_t>(blk->forecast()) > x.size()) continue;
                    // the scheduler hands each block what the upstream buffer holds (>= forecast)
                    const int avail = static_cast<int>(std::min<uint64_t>(16384, x.size() - nread[c]));
                    Gnss_Synchro out{};
                    int nout = 0;
                    const int used = blk->work(x.data() + nread[c], avail, nread[c], &out, &nout);
                    if (nout == 1 && out.Flag_valid_symbol_output) ++r.outputs[c];
                    if (used <= 0 && nout == 0) continue;
                    progress = true;
                    nread[c] += static_cast<uint64_t>(std::max(used, 0));
                }
        }
    for (size_t c = 0; c < n; ++c)
        drain_block(blks[c], nread[c], [&r, c](const Gnss_Synchro& out, int nout) {
            if (nout == 1 && out.Flag_valid_symbol_output) ++r.outputs[c];
        });
    r.seconds = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    trk.clear();  // closes the dump files
    return r;
}

std::vector<char> read_file(const std::string& path)
{
    std::ifstream f(path, std::ios::binary);
    return std::vector<char>((std::istreambuf_iterator<char>(f)), std::istreambuf_iterator<char>());
}

// The reference's tracking dump (log_data, dll_pll_veml_tracking.cc:1403-1500) as the
// adapters write it: one 108-byte record per logged call, decoded against the
// engine's records, and the pooled blocks' files byte-identical to the per-channel ones.
void check_tracking_dump(const PoolRun& one, const std::string& stem_one, const std::string& stem_pool,
    const std::vector<Gnss_Synchro>& acq)
{
    bool sizes = true, fields = true, same = true, mats = true;
    size_t logged_total = 0;
    for (size_t c = 0; c < acq.size(); ++c)
        {
            const auto a = read_file(stem_one + std::to_string(c) + ".dat");
            const auto b = read_file(stem_pool + std::to_string(c) + ".dat");
            std::vector<const gsdr_trk_epoch*> logged;
            for (const auto& r : one.recs[c])
                if (r.flags & GSDR_TRK_F_LOGGED) logged.push_back(&r);
            logged_total += logged.size();
            sizes = sizes && a.size() == logged.size() * TrackingDump::kRecordBytes && !logged.empty();
            // the pooled blocks run up to two more calls at the stream's end
            same = same && b.size() >= a.size() && b.size() <= a.size() + 2 * TrackingDump::kRecordBytes &&
                   std::equal(a.begin(), a.end(), b.begin());
            // dump_mat (default true): the destructor converted each .dat (save_matfile)
            mats = mats && std::filesystem::exists(stem_one + std::to_string(c) + ".mat") &&
                   std::filesystem::exists(stem_pool + std::to_string(c) + ".mat");
            for (size_t i = 0; fields && i < logged.size() && (i + 1) * TrackingDump::kRecordBytes <= a.size(); ++i)
                {
                    const char* p = a.data() + i * TrackingDump::kRecordBytes;
                    float f[7];
                    uint64_t stamp;
                    uint32_t prn;
                    float pll_err, cn0, evm;
                    std::memcpy(f, p, sizeof(f));
                    std::memcpy(&stamp, p + 28, 8);
                    std::memcpy(&pll_err, p + 36 + 5 * 4, 4);
                    std::memcpy(&cn0, p + 36 + 9 * 4, 4);
                    std::memcpy(&prn, p + 36 + 12 * 4 + 8, 4);
                    std::memcpy(&evm, p + 104, 4);
                    const gsdr_trk_epoch& r = *logged[i];
                    fields = fields && f[0] == 0.0F && f[4] == 0.0F && f[2] == r.log_accu[2] && f[1] == r.log_accu[1] &&
                             f[5] == r.taps[2] && f[6] == r.taps[3] &&
                             stamp == r.sample_counter + static_cast<uint64_t>(r.consumed) &&
                             pll_err == r.carr_phase_error_hz && cn0 == static_cast<float>(r.cn0_db_hz) &&
                             prn == acq[c].PRN && evm == static_cast<float>(r.evm) && r.log_accu[2] > 0.0F;
                }
        }
    EXPECT(sizes, "tracking dump: one 108-byte record per logged call in <dump_filename stem><channel>.dat");
    EXPECT(fields, "tracking dump: records decode to the engine's log_data fields");
    EXPECT(same, "tracking dump: pooled blocks write the per-channel blocks' bytes");
    EXPECT(mats, "tracking dump: <stem><channel>.mat written on destruction (dump_mat)");
    std::printf("tracking dump: %zu logged calls over %zu channels (%s<ch>.dat)\n", logged_total, acq.size(),
        stem_one.c_str());
}

void test_pooled_tracking()
{
    const double fs = 4000000.0;
    const double sigma = 1.0;
    const double amp = std::sqrt(2.0 * std::pow(10.0, 4.8) / fs) * sigma;
    const std::vector<float> bits = {1, -1, -1, -1, 1, -1, 1, 1};
    const uint32_t prns[6] = {1, 7, 13, 19, 22, 30};
    const double dly[6] = {524.3, 2100.8, 77.1, 3333.3, 1500.5, 999.9};
    const double dop[6] = {1680.0, -3250.0, 500.0, 2750.0, -1250.0, 4000.0};
    std::vector<SynthSat> sats;
    std::vector<Gnss_Synchro> acq(6);
    for (int i = 0; i < 6; ++i)
        {
            sats.push_back({gps_l1_ca_code_gen_float(prns[i]), 1.023e6, 1575.42e6, dly[i], dop[i], amp, {}, bits, 0.02});
            acq[i].System = 'G';
            acq[i].Signal[0] = '1';
            acq[i].Signal[1] = 'C';
            acq[i].PRN = prns[i];
            acq[i].Channel_ID = i;
            acq[i].Acq_delay_samples = std::fmod(std::round(dly[i]), 4000.0);
            acq[i].Acq_doppler_hz = 250.0 * std::round(dop[i] / 250.0);
            acq[i].Acq_samplestamp_samples = 0;
        }
    // pull_in_time_s = 0 ends the pull-in transitory after 1 s, then bit sync and outputs
    const auto x = synth_stream(sats, fs, static_cast<size_t>(fs * 1.7), 23, sigma);
    // GSDR_SELFTEST_DUMP_DIR: the dumps stay there for tests/test_host_mirror.py (.mat read-back)
    const char* keep = std::getenv("GSDR_SELFTEST_DUMP_DIR");
    const std::string dir = keep ? std::string(keep) + "/trk"
                                 : (std::filesystem::temp_directory_path() / ("gsdr_selftest_" + std::to_string(getpid()))).string();
    const PoolRun one = run_tracking_blocks(false, x, acq, dir + "/one/trk_dump.dat");
    const PoolRun pool = run_tracking_blocks(true, x, acq, dir + "/pool/trk_dump.dat");
    check_tracking_dump(one, dir + "/one/trk_dump", dir + "/pool/trk_dump", acq);
    std::error_code ec;
    if (!keep) std::filesystem::remove_all(dir, ec);
    // the per-channel block stops when fewer than its forecast (2 vector lengths)
    // items remain, the pooled block runs every call the stream holds: the records
    // agree over the per-channel block's calls, and each block's outputs are its
    // records' valid-output calls
    bool same = true, outs = true;
    for (int c = 0; c < 6; ++c)
        {
            same = same && one.recs[c].size() > 1000 && pool.recs[c].size() >= one.recs[c].size() &&
                   pool.recs[c].size() <= one.recs[c].size() + 2;
            for (size_t e = 0; same && e < one.recs[c].size(); ++e)
                same = std::memcmp(&one.recs[c][e], &pool.recs[c][e], sizeof(gsdr_trk_epoch)) == 0;
            for (const PoolRun* run : {&one, &pool})
                {
                    int v = 0;
                    for (const auto& e : run->recs[c]) v += (e.flags & GSDR_TRK_F_VALID_OUTPUT) ? 1 : 0;
                    outs = outs && v == run->outputs[c];
                }
        }
    EXPECT(same, "pooled tracking blocks: every call's record identical to the per-channel blocks'");
    EXPECT(pool.outputs[0] > 8 && outs, "pooled tracking: one Gnss_Synchro per valid-output call");
    if (!outs || pool.outputs[0] <= 8)
        std::fprintf(stderr, "outputs per channel: per-channel %d %d %d, pooled %d %d %d\n", one.outputs[0], one.outputs[1],
            one.outputs[2], pool.outputs[0], pool.outputs[1], pool.outputs[2]);
    const double msps_one = static_cast<double>(one.calls) * 4000.0 / one.seconds / 1e6;
    const double msps_pool = static_cast<double>(pool.calls) * 4000.0 / pool.seconds / 1e6;
    std::printf("tracking blocks, 6 GPS channels x %zu calls: per-channel adapters %.1f M ch-samples/s (%.1f us per "
                "general_work call), pooled %.1f M ch-samples/s (%.1f us per call)\n",
        one.recs[0].size(), msps_one, one.seconds / static_cast<double>(one.calls) * 1e6, msps_pool,
        pool.seconds / static_cast<double>(pool.calls) * 1e6);
}

// A lagging pooled block: block B tracks while block A (same pool, standby) is
// handed items 2.5 ring windows past B's position -- a flowgraph buffer deeper than
// the pool's window.  The pool advances every started channel whenever half a
// window arrives, so B's channel keeps up on the device and B's calls continue
// without a gap, an overrun or a loss of lock when B is called again.
void test_pool_overrun()
{
    const double fs = 4000000.0;
    const double amp = std::sqrt(2.0 * std::pow(10.0, 4.8) / fs);
    SynthSat s{gps_l1_ca_code_gen_float(7), 1.023e6, 1575.42e6, 1200.4, 1250.0, amp, {}, {1, -1}, 0.02};
    const auto x = synth_stream({s}, fs, static_cast<size_t>(fs * 0.2), 31, 1.0);
    InMemoryConfiguration config;
    config.set_property("GNSS-SDR.internal_fs_sps", "4000000");
    config.set_property("Tracking_1C.implementation", "GPS_L1_CA_DLL_PLL_Tracking_MI355X");
    config.set_property("Tracking_1C.item_type", "gr_complex");
    config.set_property("Tracking_1C.pll_bw_hz", "40.0");
    config.set_property("Tracking_1C.dll_bw_hz", "4.0");
    config.set_property("Channels_1C.count", "2");
    config.set_property("Tracking_1C.mi355x_pool_window", "4");  // 4 calls = 16000 items
    config.set_property("Tracking_1C.mi355x_pool_batch", "1");
    Gnss_Synchro g{};
    g.System = 'G';
    g.Signal[0] = '1';
    g.Signal[1] = 'C';
    g.PRN = 7;
    g.Acq_delay_samples = 1200.0;
    g.Acq_doppler_hz = 1250.0;
    g.Acq_samplestamp_samples = 0;
    auto ta = gsdr_factory::GetTrkBlock(&config, "Tracking_1C", 1, 1, 0);
    auto tb = gsdr_factory::GetTrkBlock(&config, "Tracking_1C", 1, 1, 0);
    Gnss_Synchro ga = g;
    ta->set_channel(0);
    ta->set_gnss_synchro(&ga);
    tb->set_channel(1);
    tb->set_gnss_synchro(&g);
    tb->start_tracking();
    auto* a = dynamic_cast<DllPllTrackingAdapterMI355X*>(ta.get())->get_block();
    auto* b = dynamic_cast<dll_pll_veml_tracking_pool_mi355x*>(
        dynamic_cast<DllPllTrackingAdapterMI355X*>(tb.get())->get_block());
    EXPECT(b != nullptr, "lagging block: pooled block");
    if (!b) return;
    EXPECT(b->pool()->window_items() == 16000 && b->pool()->batch_items() == 4000,
        "lagging block: <role>.mi355x_pool_window / _batch set the window and the batch in calls");
    std::vector<gsdr_trk_epoch> recs;
    b->set_record_sink([&recs](const gsdr_trk_epoch& r) { recs.push_back(r); });
    uint64_t na = 0, nb = 0;
    Gnss_Synchro out{};
    int nout = 0;
    // both blocks side by side for 80000 items
    while (nb < 80000)
        {
            nb += static_cast<uint64_t>(b->work(x.data() + nb, 8000, nb, &out, &nout));
            while (na < nb) na += static_cast<uint64_t>(a->work(x.data() + na, 4000, na, &out, &nout));
        }
    const size_t before = recs.size();
    // A runs 40000 items (2.5 windows) past B, which the scheduler does not call
    while (na < nb + 40000) na += static_cast<uint64_t>(a->work(x.data() + na, 8000, na, &out, &nout));
    // B is handed its items again
    while (nb < na) nb += static_cast<uint64_t>(b->work(x.data() + nb, 8000, nb, &out, &nout));
    drain_block(b, nb, [](const Gnss_Synchro&, int) {});
    bool contiguous = recs.size() > 25;
    for (size_t i = 0; contiguous && i + 1 < recs.size(); ++i)
        contiguous = recs[i + 1].sample_counter == recs[i].sample_counter + static_cast<uint64_t>(recs[i].consumed) &&
                     (recs[i].flags & (GSDR_TRK_F_OVERRUN | GSDR_TRK_F_LOSS_OF_LOCK)) == 0;
    EXPECT(contiguous && b->overruns() == 0 && b->state() == 2,
        "lagging block: its calls continue over the lag without a gap, an overrun or a loss of lock");
    std::printf("lagging block: %zu calls before the lag, %zu after A ran %d items ahead; overruns %llu\n", before,
        recs.size() - before, 40000, static_cast<unsigned long long>(b->overruns()));
    b->set_record_sink(nullptr);

    // a failing feed (items the pool never saw: the scheduler skipped ahead of every
    // pooled block) -> the block reports a loss of lock and takes its slot out of the
    // engine, so later advances queue nothing for it
    int events = 0;
    b->set_event_handler([&events](int e) { events += e == 3 ? 1 : 0; });
    tb->start_tracking();
    b->work(x.data() + na, 8000, na, &out, &nout);  // pull-in at the head
    EXPECT(b->state() == 2, "pool failing feed: block restarted at the head");
    const uint64_t skip = na + 100000;
    nout = 0;
    b->work(x.data() + na, 8000, skip, &out, &nout);
    EXPECT(b->state() == 0 && events == 1, "pool failing feed: loss of lock (event 3), block in standby");
    // another block's advance must not resurrect the stopped slot
    ta->start_tracking();
    a->work(x.data() + na, 8000, na, &out, &nout);
    a->work(x.data() + na, 8000, na, &out, &nout);
    EXPECT(b->state() == 0, "pool failing feed: the slot stays stopped");
}

// The shared device ring of an input stream (DeviceIqRing): one ring per key, shared
// by the pools of every role that names it, and two input streams under one key
// refused on the first overlapping feed.
void test_ring_keys()
{
    const auto r1 = DeviceIqRing::get(0, GSDR_ITEM_GR_COMPLEX, 1 << 16, "selftest_a");
    const auto r2 = DeviceIqRing::get(0, GSDR_ITEM_GR_COMPLEX, 1 << 16, "selftest_a");
    const auto r3 = DeviceIqRing::get(0, GSDR_ITEM_GR_COMPLEX, 1 << 16, "selftest_b");
    EXPECT(r1 == r2 && r1 != r3, "ring keys: one ring per key, shared by its consumers");
    std::vector<std::complex<float>> a(8000), b(8000);
    for (size_t i = 0; i < a.size(); ++i)
        {
            a[i] = {static_cast<float>(i), 1.0F};
            b[i] = {static_cast<float>(i), 2.0F};
        }
    uint64_t head = 0;
    r1->feed(a.data(), 0, 4000);
    r2->feed(a.data(), 0, 6000);  // the same stream, further: pushes [4000, 6000)
    EXPECT(r1->head(&head) && head == 6000, "ring keys: a second feeder of the same stream pushes only what is new");
    bool refused = false;
    try
        {
            r2->feed(b.data(), 0, 8000);  // another stream under the same key
        }
    catch (const std::logic_error&)
        {
            refused = true;
        }
    EXPECT(refused && r1->head(&head) && head == 6000, "ring keys: a different stream under the same key is refused");
    r3->feed(b.data(), 0, 8000);
    EXPECT(r3->head(&head) && head == 8000, "ring keys: another key is another stream");
    std::printf("ring keys: shared ring per key, mismatching feeder refused\n");
}

// Gnss_Synchro emission of both tracking blocks (dll_pll_veml_tracking.cc:1784-2152)
// on a GPS channel driven past bit synchronisation, with GnssTime "timetag" input
// tags every 100 ms and a telemetry fault (msg_handler_telemetry_to_trk, :614-637)
// at 1.9 s.  Each block's per-call records, emitted Gnss_Synchro items, output tags
// and the channel's acquisition record go to <dir>/synchro_<kind>.txt, which
// tests/test_host_mirror.py replays through the oracle channel (with the fault
// before the same call) and checks field by field.
void test_synchro_emission(const std::string& dir)
{
    const double fs = 4000000.0;
    const double amp = std::sqrt(2.0 * std::pow(10.0, 5.0) / fs);
    const std::vector<float> bits = {1, -1, -1, -1, 1, -1, 1, 1};
    SynthSat g{gps_l1_ca_code_gen_float(1), 1.023e6, 1575.42e6, 524.3, 1680.0, amp, {}, bits, 0.02};
    const auto x = synth_stream({g}, fs, static_cast<size_t>(fs * 2.2), 11, 1.0);
    std::vector<GnssTimeTag> tags;
    for (int k = 0; k < 22; ++k)
        {
            GnssTimeTag t;
            t.offset = static_cast<uint64_t>(k) * 400000 + 1234;
            t.time.week = 2200;
            t.time.tow_ms = 345600000 + 100 * k;
            t.time.tow_ms_fraction = 0.25;
            t.time.rx_time = 0.0;
            tags.push_back(t);
        }
    std::error_code ec;
    std::filesystem::create_directories(dir, ec);
    for (const bool pooled : {false, true})
        {
            InMemoryConfiguration config;
            config.set_property("GNSS-SDR.internal_fs_sps", "4000000");
            config.set_property("Tracking_1C.implementation", "GPS_L1_CA_DLL_PLL_Tracking_MI355X");
            config.set_property("Tracking_1C.item_type", "gr_complex");
            config.set_property("Tracking_1C.pll_bw_hz", "40.0");
            config.set_property("Tracking_1C.dll_bw_hz", "4.0");
            config.set_property("Tracking_1C.pull_in_time_s", "0");
            config.set_property("Channels_1C.count", "1");
            config.set_property("Tracking_1C.mi355x_pool", pooled ? "true" : "false");
            Gnss_Synchro acq{};
            acq.System = 'G';
            acq.Signal[0] = '1';
            acq.Signal[1] = 'C';
            acq.PRN = 1;
            acq.Channel_ID = 3;
            acq.Acq_delay_samples = 524.0;
            acq.Acq_doppler_hz = 1750.0;
            acq.Acq_samplestamp_samples = 0;
            acq.Acq_doppler_step = 250;
            acq.Flag_valid_acquisition = true;
            // values only the acquisition record carries: a loss-of-lock output repeats them
            acq.Prompt_I = 111.5;
            acq.Prompt_Q = -222.25;
            acq.CN0_dB_hz = 33.0;
            acq.Carrier_Doppler_hz = 1750.0;
            acq.correlation_length_ms = 0;
            auto trk = gsdr_factory::GetTrkBlock(&config, "Tracking_1C", 1, 1, 0);
            trk->set_channel(3);
            trk->set_gnss_synchro(&acq);
            trk->start_tracking();
            auto* blk = dynamic_cast<DllPllTrackingAdapterMI355X*>(trk.get())->get_block();
            std::vector<gsdr_trk_epoch> recs;
            blk->set_record_sink([&recs](const gsdr_trk_epoch& r) { recs.push_back(r); });
            struct Emitted
            {
                Gnss_Synchro s;
                bool tag;
                GnssTimeTag t;
            };
            std::vector<Emitted> outs;
            int events = 0;
            blk->set_event_handler([&events](int e) { events += e == 3 ? 1 : 0; });
            uint64_t nread = 0;
            bool faulted = false;
            auto take = [&outs](const Gnss_Synchro& o, int nout, const TrackingTags& tt) {
                if (nout == 1) outs.push_back({o, tt.has_out, tt.out});
            };
            while (nread + static_cast<uint64_t>(blk->forecast()) <= x.size() && blk->state() != 0)
                {
                    if (!faulted && nread >= 7600000)
                        {
                            blk->msg_handler_telemetry_to_trk(1);
                            faulted = true;
                        }
                    const int avail = static_cast<int>(std::min<uint64_t>(
                        std::max<uint64_t>(16384, static_cast<uint64_t>(blk->forecast())), x.size() - nread));
                    std::vector<GnssTimeTag> in_tags;
                    for (const auto& t : tags)
                        if (t.offset >= nread && t.offset < nread + static_cast<uint64_t>(avail)) in_tags.push_back(t);
                    TrackingTags tt;
                    tt.in = in_tags.data();
                    tt.n_in = static_cast<int>(in_tags.size());
                    Gnss_Synchro o{};
                    int nout = 0;
                    const int used = blk->work(x.data() + nread, avail, nread, &o, &nout, &tt);
                    take(o, nout, tt);
                    if (used <= 0 && nout == 0) break;
                    nread += static_cast<uint64_t>(std::max(used, 0));
                }
            blk->flush();
            for (int guard = 0; guard < 100000 && blk->state() != 0; ++guard)
                {
                    TrackingTags tt;
                    Gnss_Synchro o{};
                    int nout = 0;
                    blk->work(nullptr, 0, nread, &o, &nout, &tt);
                    take(o, nout, tt);
                    if (nout == 0) break;
                }
            blk->set_record_sink(nullptr);
            const std::string path = dir + (pooled ? "/synchro_pooled.txt" : "/synchro_channel.txt");
            FILE* f = std::fopen(path.c_str(), "w");
            EXPECT(f != nullptr, "synchro emission: output file");
            if (!f) return;
            std::fprintf(f, "acq %u %d %.17g %.17g %llu %.17g %.17g %.17g %.17g %d\n", acq.PRN, acq.Channel_ID,
                acq.Acq_delay_samples, acq.Acq_doppler_hz, static_cast<unsigned long long>(acq.Acq_samplestamp_samples),
                acq.Prompt_I, acq.Prompt_Q, acq.CN0_dB_hz, acq.Carrier_Doppler_hz, acq.correlation_length_ms);
            for (const auto& t : tags)
                std::fprintf(f, "tag %llu %d %d %.17g\n", static_cast<unsigned long long>(t.offset), t.time.week,
                    t.time.tow_ms, t.time.tow_ms_fraction);
            for (const auto& r : recs)
                std::fprintf(f, "rec %llu %d %d %d %.17g %.17g\n", static_cast<unsigned long long>(r.sample_counter),
                    r.state, r.consumed, r.flags, r.prompt_i, r.prompt_q);
            for (const auto& e : outs)
                {
                    const Gnss_Synchro& o = e.s;
                    std::fprintf(f,
                        "out %u %d %c%c %.17g %.17g %llu %lld %.17g %.17g %.17g %.17g %.17g %.17g %llu %d %.17g %d %d %d",
                        o.PRN, o.Channel_ID, o.Signal[0], o.Signal[1], o.Acq_delay_samples, o.Acq_doppler_hz,
                        static_cast<unsigned long long>(o.Acq_samplestamp_samples), static_cast<long long>(o.fs), o.Prompt_I,
                        o.Prompt_Q, o.CN0_dB_hz, o.Carrier_Doppler_hz, o.Carrier_phase_rads, o.Code_phase_samples,
                        static_cast<unsigned long long>(o.Tracking_sample_counter), o.correlation_length_ms, o.EVM,
                        o.Flag_valid_symbol_output ? 1 : 0, o.Flag_PLL_180_deg_phase_locked ? 1 : 0,
                        o.Flag_valid_acquisition ? 1 : 0);
                    if (e.tag)
                        std::fprintf(f, " tag %llu %d %d %.17g %.17g\n", static_cast<unsigned long long>(e.t.offset),
                            e.t.time.week, e.t.time.tow_ms, e.t.time.tow_ms_fraction, e.t.time.rx_time);
                    else
                        std::fprintf(f, "\n");
                }
            std::fclose(f);
            // the records themselves (gsdr_trk_epoch, 192 bytes each) for the oracle replay
            const std::string rpath = dir + (pooled ? "/synchro_pooled.recs" : "/synchro_channel.recs");
            if (FILE* fr = std::fopen(rpath.c_str(), "wb"))
                {
                    std::fwrite(recs.data(), sizeof(gsdr_trk_epoch), recs.size(), fr);
                    std::fclose(fr);
                }
            int valid = 0, lol = 0;
            for (const auto& e : outs) (e.s.Flag_valid_symbol_output ? valid : lol) += 1;
            EXPECT(valid > 20 && lol == 1 && events == 1 && faulted,
                "synchro emission: valid outputs, then the telemetry fault's loss of lock (one invalid output, event 3)");
            if (!(valid > 20 && lol == 1 && events == 1 && faulted))
                std::fprintf(stderr, "synchro emission (%s): %zu calls, valid %d, lol %d, events %d, faulted %d, nread %llu\n",
                    pooled ? "pooled" : "per-channel", recs.size(), valid, lol, events, faulted ? 1 : 0,
                    static_cast<unsigned long long>(nread));
            std::printf("synchro emission (%s block): %zu calls, %d valid outputs, %d loss-of-lock output, %s\n",
                pooled ? "pooled" : "per-channel", recs.size(), valid, lol, path.c_str());
        }
}

// GNU Radio's buffer protocol around pooled blocks: one upstream buffer of kBuf items
// (double-mapped: every item also at +kBuf, so each reader sees one contiguous span),
// page-locked so ring pushes DMA straight from it, with the writer overwriting every
// item as soon as all readers consumed it.  Two pooled blocks of one pool read it:
// A on every round, B only on every third (it lags by up to the buffer, while A's
// pushes run the ring and the pool ahead of B's items).  Each block is called while
// it makes progress (an output or consumed items) -- never with zero input items --
// and its GnssTime tags come with its items.  A block must (1) consume only items
// whose copy landed (otherwise the writer's overwrite tears the input and the records
// change), (2) keep its record queue bounded (one output per call, consumption
// matching production), (3) emit the per-channel blocks' outputs and output tags.
void test_pool_recycled_buffer()
{
    const double fs = 4000000.0;
    const double amp = std::sqrt(2.0 * std::pow(10.0, 5.0) / fs);
    const std::vector<float> bits = {1, -1, -1, -1, 1, -1, 1, 1};
    const uint32_t prns[2] = {1, 7};
    const double dly[2] = {524.3, 2100.8};
    const double dop[2] = {1680.0, -3250.0};
    std::vector<SynthSat> sats;
    std::vector<Gnss_Synchro> acq(2);
    for (int i = 0; i < 2; ++i)
        {
            sats.push_back({gps_l1_ca_code_gen_float(prns[i]), 1.023e6, 1575.42e6, dly[i], dop[i], amp, {}, bits, 0.02});
            acq[i].System = 'G';
            acq[i].Signal[0] = '1';
            acq[i].Signal[1] = 'C';
            acq[i].PRN = prns[i];
            acq[i].Channel_ID = i;
            acq[i].Acq_delay_samples = std::fmod(std::round(dly[i]), 4000.0);
            acq[i].Acq_doppler_hz = 250.0 * std::round(dop[i] / 250.0);
            acq[i].Acq_samplestamp_samples = 0;
        }
    const auto x = synth_stream(sats, fs, static_cast<size_t>(fs * 1.6), 41, 1.0);
    std::vector<GnssTimeTag> tags;
    for (uint64_t off = 777; off < x.size(); off += 100000)
        {
            GnssTimeTag t;
            t.offset = off;
            t.time.week = 2300;
            t.time.tow_ms = static_cast<int32_t>(100000 + off / 4000);
            t.time.tow_ms_fraction = 0.5;
            t.time.rx_time = 0.0;
            tags.push_back(t);
        }
    struct Out
    {
        uint64_t counter;
        bool valid;
        double pi;
        bool tag;
        uint64_t tag_offset;
        int32_t tow;
        bool drained;  // handed out by the end-of-stream drain (no tags passed)
    };
    auto make_config = [](bool pooled) {
        InMemoryConfiguration config;
        config.set_property("GNSS-SDR.internal_fs_sps", "4000000");
        config.set_property("Tracking_1C.implementation", "GPS_L1_CA_DLL_PLL_Tracking_MI355X");
        config.set_property("Tracking_1C.item_type", "gr_complex");
        config.set_property("Tracking_1C.pll_bw_hz", "40.0");
        config.set_property("Tracking_1C.dll_bw_hz", "4.0");
        config.set_property("Tracking_1C.pull_in_time_s", "0");
        config.set_property("Channels_1C.count", "2");
        config.set_property("Tracking_1C.mi355x_pool", pooled ? "true" : "false");
        config.set_property("Tracking_1C.mi355x_ring", pooled ? "recycled" : "rf0");
        return config;
    };
    auto tags_in = [&tags](uint64_t lo, uint64_t hi) {
        std::vector<GnssTimeTag> v;
        for (const auto& t : tags)
            if (t.offset >= lo && t.offset < hi) v.push_back(t);
        return v;
    };
    // the per-channel blocks (synchronous copies) on the never-rewritten stream
    std::vector<std::vector<gsdr_trk_epoch>> ref_recs(2);
    std::vector<std::vector<Out>> ref_outs(2);
    {
        InMemoryConfiguration config = make_config(false);
        for (int c = 0; c < 2; ++c)
            {
                auto trk = gsdr_factory::GetTrkBlock(&config, "Tracking_1C", 1, 1, 0);
                Gnss_Synchro g = acq[c];
                trk->set_channel(static_cast<unsigned int>(c));
                trk->set_gnss_synchro(&g);
                trk->start_tracking();
                auto* blk = dynamic_cast<DllPllTrackingAdapterMI355X*>(trk.get())->get_block();
                blk->set_record_sink([&ref_recs, c](const gsdr_trk_epoch& r) { ref_recs[c].push_back(r); });
                uint64_t nread = 0;
                while (nread + static_cast<uint64_t>(blk->forecast()) <= x.size())
                    {
                        const int avail = static_cast<int>(std::min<uint64_t>(16384, x.size() - nread));
                        auto in = tags_in(nread, nread + static_cast<uint64_t>(avail));
                        TrackingTags tt;
                        tt.in = in.data();
                        tt.n_in = static_cast<int>(in.size());
                        Gnss_Synchro o{};
                        int nout = 0;
                        const int used = blk->work(x.data() + nread, avail, nread, &o, &nout, &tt);
                        if (nout == 1)
                            ref_outs[c].push_back({o.Tracking_sample_counter, o.Flag_valid_symbol_output, o.Prompt_I,
                                tt.has_out, tt.out.offset, tt.out.time.tow_ms, false});
                        if (used <= 0 && nout == 0) break;
                        nread += static_cast<uint64_t>(std::max(used, 0));
                    }
                blk->set_record_sink(nullptr);
            }
    }
    // the pooled blocks behind the upstream buffer: kBuf items, recycled at once
    // (recycle), or the whole stream (no item overwritten: the same control flow
    // without the writer's overwrites, which separates a torn input from the rest)
    struct PooledRun
    {
        std::vector<std::vector<gsdr_trk_epoch>> recs{2};
        std::vector<std::vector<Out>> outs{2};
        size_t max_queue[2] = {0, 0};
        uint64_t calls = 0, zero_consumed = 0;
    };
    auto run_pooled = [&](bool recycle) {
        PooledRun pr;
        // the scheduler's buffer: its writer runs at most kLead items ahead of the
        // slowest reader; slots are reused (recycle) or every item has its own
        constexpr uint64_t kLead = 32768;
        const uint64_t kBuf = recycle ? kLead : static_cast<uint64_t>(x.size());
        std::vector<std::complex<float>> buf(2 * kBuf);
        EXPECT(gsdr_host_register(buf.data(), buf.size() * sizeof(buf[0])) == GSDR_OK, "recycled buffer: page-locked");
        {
            InMemoryConfiguration config = make_config(true);
            config.set_property("Tracking_1C.mi355x_ring", recycle ? "recycled" : "static");
            std::vector<std::unique_ptr<TrackingInterface>> trk;
            std::vector<Gnss_Synchro> gs(acq);
            std::vector<dll_pll_veml_tracking_pool_mi355x*> blk(2);
            for (int c = 0; c < 2; ++c)
                {
                    trk.push_back(gsdr_factory::GetTrkBlock(&config, "Tracking_1C", 1, 1, 0));
                    trk[c]->set_channel(static_cast<unsigned int>(c));
                    trk[c]->set_gnss_synchro(&gs[c]);
                    trk[c]->start_tracking();
                    blk[c] = dynamic_cast<dll_pll_veml_tracking_pool_mi355x*>(
                        dynamic_cast<DllPllTrackingAdapterMI355X*>(trk[c].get())->get_block());
                    EXPECT(blk[c] != nullptr, "recycled buffer: pooled blocks");
                    if (!blk[c]) return pr;
                    blk[c]->set_record_sink([&pr, c](const gsdr_trk_epoch& r) { pr.recs[c].push_back(r); });
                }
            uint64_t nread[2] = {0, 0}, written = 0;
            const uint64_t end = x.size();
            for (int round = 0; nread[0] < end || nread[1] < end; ++round)
                {
                    // the writer fills every slot all readers released (overwriting at once)
                    const uint64_t limit = std::min(std::min(nread[0], nread[1]) + kLead, end);
                    for (; written < limit; ++written)
                        {
                            buf[written % kBuf] = x[written];
                            buf[written % kBuf + kBuf] = x[written];
                        }
                    bool progress = false;
                    for (int c = 0; c < 2; ++c)
                        {
                            if (c == 1 && round % 3 != 0) continue;  // B's scheduler thread lags
                            for (int guard = 0; guard < 64 && nread[c] < written; ++guard)
                                {
                                    // GNU Radio hands at most the buffer's worth ahead of the reader
                                    const int avail = static_cast<int>(std::min<uint64_t>(written - nread[c], kLead));
                                    auto in = tags_in(nread[c], nread[c] + static_cast<uint64_t>(avail));
                                    TrackingTags tt;
                                    tt.in = in.data();
                                    tt.n_in = static_cast<int>(in.size());
                                    Gnss_Synchro o{};
                                    int nout = 0;
                                    const int used =
                                        blk[c]->work(buf.data() + nread[c] % kBuf, avail, nread[c], &o, &nout, &tt);
                                    ++pr.calls;
                                    pr.zero_consumed += used == 0 ? 1 : 0;
                                    if (nout == 1)
                                        pr.outs[c].push_back({o.Tracking_sample_counter, o.Flag_valid_symbol_output,
                                            o.Prompt_I, tt.has_out, tt.out.offset, tt.out.time.tow_ms, false});
                                    pr.max_queue[c] = std::max(pr.max_queue[c], blk[c]->pool()->queued(blk[c]->slot()));
                                    if (used <= 0 && nout == 0) break;
                                    progress = true;
                                    nread[c] += static_cast<uint64_t>(std::max(used, 0));
                                }
                        }
                    if (!progress && written >= end) break;
                }
            // end of the stream (only here): the blocks compute what they were handed
            // and hand out the rest
            for (int c = 0; c < 2; ++c)
                drain_block(blk[c], nread[c], [&pr, c](const Gnss_Synchro& o, int nout) {
                    if (nout == 1)
                        pr.outs[c].push_back({o.Tracking_sample_counter, o.Flag_valid_symbol_output, o.Prompt_I, false, 0, 0, true});
                });
            for (int c = 0; c < 2; ++c) blk[c]->set_record_sink(nullptr);
        }
        gsdr_host_unregister(buf.data());
        return pr;
    };
    auto compare = [&](const PooledRun& pr, const char* what, bool& same_recs, bool& same_outs) {
        same_recs = true;
        same_outs = true;
        for (int c = 0; c < 2; ++c)
            {
                const size_t k = std::min(pr.recs[c].size(), ref_recs[c].size());
                bool ok = k > 300 && pr.recs[c].size() + 2 >= ref_recs[c].size();
                size_t e = 0;
                for (; ok && e < k; ++e) ok = std::memcmp(&pr.recs[c][e], &ref_recs[c][e], sizeof(gsdr_trk_epoch)) == 0;
                if (!ok && e > 0 && e <= k)
                    {
                        const gsdr_trk_epoch& a = pr.recs[c][e - 1];
                        const gsdr_trk_epoch& b = ref_recs[c][e - 1];
                        size_t off = 0;
                        while (off < sizeof(gsdr_trk_epoch) &&
                               reinterpret_cast<const char*>(&a)[off] == reinterpret_cast<const char*>(&b)[off])
                            ++off;
                        std::fprintf(stderr,
                            "%s: channel %d record %zu of %zu / %zu differs at byte %zu: counter %llu / %llu, state %d / %d, "
                            "prompt %.9g / %.9g\n",
                            what, c, e - 1, pr.recs[c].size(), ref_recs[c].size(), off,
                            static_cast<unsigned long long>(a.sample_counter), static_cast<unsigned long long>(b.sample_counter),
                            a.state, b.state, a.prompt_i, b.prompt_i);
                    }
                same_recs = same_recs && ok;
                const size_t m = std::min(pr.outs[c].size(), ref_outs[c].size());
                same_outs = same_outs && m > 10 && pr.outs[c].size() >= ref_outs[c].size();
                for (size_t i = 0; same_outs && i < m; ++i)
                    {
                        const Out& a = pr.outs[c][i];
                        const Out& b = ref_outs[c][i];
                        same_outs = a.counter == b.counter && a.valid == b.valid && a.pi == b.pi &&
                                    (a.drained || (a.tag == b.tag && (!a.tag || (a.tag_offset == b.tag_offset && a.tow == b.tow))));
                    }
            }
        std::printf("%s: %zu / %zu records (per-channel %zu / %zu), %zu / %zu outputs, max queue %zu / %zu, %llu work "
                    "calls (%llu consumed nothing)\n",
            what, pr.recs[0].size(), pr.recs[1].size(), ref_recs[0].size(), ref_recs[1].size(), pr.outs[0].size(),
            pr.outs[1].size(), pr.max_queue[0], pr.max_queue[1], static_cast<unsigned long long>(pr.calls),
            static_cast<unsigned long long>(pr.zero_consumed));
    };
    int tagged = 0;
    for (const auto& o : ref_outs[0]) tagged += o.tag ? 1 : 0;
    const PooledRun still = run_pooled(false);
    bool rs = false, os = false;
    compare(still, "pooled blocks, stream never overwritten", rs, os);
    EXPECT(rs, "pooled blocks (no overwrite): records identical to the per-channel blocks'");
    EXPECT(os && tagged > 5, "pooled blocks (no overwrite): outputs and output time tags identical to the per-channel blocks'");
    const PooledRun rec = run_pooled(true);
    compare(rec, "pooled blocks, recycled upstream buffer", rs, os);
    EXPECT(rs, "recycled buffer: pooled records identical to the per-channel blocks' (no torn input)");
    EXPECT(os, "recycled buffer: outputs and output time tags identical to the per-channel blocks'");
    EXPECT(rec.max_queue[0] <= 24 && rec.max_queue[1] <= 24, "recycled buffer: record queues bounded without drain calls");
}

void test_multicorrelator(const std::vector<std::complex<float>>& capture)
{
    const int n = 4000;
    const auto code = gps_l1_ca_code_gen_float(1, 0);
    std::vector<float> shifts = {-0.5F, 0.0F, 0.5F};
    Hip_Multicorrelator_Real_Codes corr;
    corr.set_high_dynamics_resampler(false);  // dll_pll_veml_tracking sets it from high_dyn=false
    EXPECT(corr.init(2 * n, 3), "init");
    EXPECT(corr.set_local_code_and_taps(1023, code.data(), shifts.data()), "set_local_code_and_taps");
    std::vector<std::complex<float>> out(3);
    // align to the acquired code phase: start at sample 524, Doppler 1700 Hz
    const std::complex<float>* sig = capture.data() + 524;
    corr.set_input_output_vectors(out.data(), sig);
    const float carr_step = static_cast<float>(2.0 * M_PI * 1700.0 / 4e6);
    const float code_step = static_cast<float>(1.023e6 / 4e6);
    EXPECT(corr.Carrier_wipeoff_multicorrelator_resampler(0.0F, carr_step, 0.0F, 0.0F, code_step, 0.0F, n), "run");
    const auto ref = exact_correlation(sig, code, shifts, 0.0F, carr_step, 0.0F, code_step, n);
    double num = 0.0, den = 0.0;
    for (int k = 0; k < 3; ++k)
        {
            num += std::norm(std::complex<double>(out[k]) - ref[k]);
            den += std::norm(ref[k]);
        }
    const double rel = std::sqrt(num / den);
    EXPECT(rel < 1e-5, "real-code taps vs fp64 evaluation");
    // the acquired code phase is the nearest sample (0.25 chip): the peak lies between P and L
    EXPECT(std::max(std::abs(out[1]), std::abs(out[2])) > 2.0F * std::abs(out[0]), "on-peak taps dominate the early tap");
    std::printf("multicorrelator: |E| %.1f |P| %.1f |L| %.1f rel err %.2e\n", std::abs(out[0]), std::abs(out[1]),
        std::abs(out[2]), rel);

    // complex-replica drop-in on the same data: code (0, +-1) gives taps rotated by +j
    const auto ccode = gps_l1_ca_code_gen_complex(1, 0);
    Hip_Multicorrelator cc;
    EXPECT(cc.init(2 * n, 3), "complex init");
    EXPECT(cc.set_local_code_and_taps(1023, ccode.data(), shifts.data()), "complex set_local_code_and_taps");
    std::vector<std::complex<float>> cout3(3);
    cc.set_input_output_vectors(cout3.data(), sig);
    EXPECT(cc.Carrier_wipeoff_multicorrelator_resampler(0.0F, carr_step, 0.0F, code_step, n), "complex run");
    double cnum = 0.0;
    for (int k = 0; k < 3; ++k) cnum += std::norm(std::complex<double>(cout3[k]) - std::complex<double>(0, 1) * ref[k]);
    EXPECT(std::sqrt(cnum / den) < 1e-5, "complex-code taps");
}
}  // namespace

int main(int argc, char** argv)
{
    if (argc < 2)
        {
            std::cerr << "usage: host_selftest <GPS_L1_CA_ID_1_Fs_4Msps_2ms.dat>\n";
            return 2;
        }
    const auto capture = read_capture(argv[1]);
    if (capture.size() < 8000)
        {
            std::cerr << "cannot read capture " << argv[1] << '\n';
            return 2;
        }
    const char* only = std::getenv("GSDR_SELFTEST_ONLY");
    if (only && std::string(only) == "recycled")
        {
            test_pool_recycled_buffer();
            if (failures == 0) std::printf("host_selftest: PASS\n");
            return failures == 0 ? 0 : 1;
        }
    if (only && std::string(only) == "synchro")
        {
            const char* d = std::getenv("GSDR_SELFTEST_DUMP_DIR");
            test_synchro_emission(d ? std::string(d) : std::string("/tmp/gsdr_selftest_dump"));
            if (failures == 0) std::printf("host_selftest: PASS\n");
            return failures == 0 ? 0 : 1;
        }
    test_acquisition_carriers(capture);  // the validation case with each carrier model
    test_acquisition_nonblocking(capture);
    {
        const char* d = std::getenv("GSDR_SELFTEST_DUMP_DIR");
        test_acquisition_dump(capture, d ? std::string(d) : std::string("/tmp/gsdr_selftest_dump"));
    }
    test_acquisition_two_steps(capture);
    test_acquisition_repeat_steps(capture);
    test_acquisition_service(capture);
    test_acquisition_dwells(capture);
    test_acquisition_bit_transition(capture);
    test_acquisition_cbyte(capture);
    test_multicorrelator(capture);
    if (argc > 2)
        {
            const auto gal = read_capture(argv[2]);
            if (gal.size() < 32000)
                {
                    std::cerr << "cannot read capture " << argv[2] << '\n';
                    return 2;
                }
            test_galileo_acquisition(gal);
        }
    test_beidou_acquisition();
    test_tracking_handoff();
    test_receiver_on_ring();
    test_channel_fsm_handoff(capture);
    test_flag_overrides();
    test_pooled_tracking();
    test_pool_overrun();
    test_ring_keys();
    test_pool_recycled_buffer();
    {
        const char* d = std::getenv("GSDR_SELFTEST_DUMP_DIR");
        test_synchro_emission(d ? std::string(d) : std::string("/tmp/gsdr_selftest_dump"));
    }
    if (failures == 0) std::printf("host_selftest: PASS\n");
    return failures == 0 ? 0 : 1;
}
