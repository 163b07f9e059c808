// Host-side drop-in self-test, written like the reference's unit tests:
//  1. GpsL1CaPcpsAcquisitionTest.ValidationOfResults
//     (src/tests/unit-tests/signal-processing-blocks/acquisition/gps_l1_ca_pcps_acquisition_test.cc:283-366)
//     on the reference capture, through the adapter + block mirror + GPU engine.
//  2. Hip_Multicorrelator_Real_Codes / Hip_Multicorrelator on the acquired signal,
//     checked against an fp64 evaluation of the reference's phasor model.
// Usage: host_selftest <GPS_L1_CA_ID_1_Fs_4Msps_2ms.dat>
#include <algorithm>
#include <cmath>
#include <complex>
#include <cstring>
#include <cstdio>
#include <fstream>
#include <iostream>
#include <string>
#include <vector>

#include "acquisition_service.h"
#include "gnss_replicas.h"
#include "gps_l1_ca_pcps_acquisition_mi355x.h"
#include "hip_multicorrelator_real_codes.h"

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

void test_acquisition_validation(const std::vector<std::complex<float>>& capture)
{
    InMemoryConfiguration config;
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
    std::printf("acquisition: message %d delay %.1f samples doppler %.0f Hz stat %.3f stamp %llu\n", rx_message,
        gnss_synchro.Acq_delay_samples, gnss_synchro.Acq_doppler_hz, acquisition.get_block()->test_statistics(),
        static_cast<unsigned long long>(gnss_synchro.Acq_samplestamp_samples));
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
    test_acquisition_validation(capture);
    test_acquisition_two_steps(capture);
    test_acquisition_repeat_steps(capture);
    test_acquisition_service(capture);
    test_multicorrelator(capture);
    if (failures == 0) std::printf("host_selftest: PASS\n");
    return failures == 0 ? 0 : 1;
}
