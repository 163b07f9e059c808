// Synthetic GNSS streams for the host self-test and the receiver benchmark:
// code x carrier (+ secondary code, navigation symbols) + AWGN, code Doppler
// included.  Test tooling only.
#ifndef GSDR_HOST_TESTS_SYNTH_STREAM_H
#define GSDR_HOST_TESTS_SYNTH_STREAM_H

#include <algorithm>
#include <cmath>
#include <complex>
#include <cstdint>
#include <random>
#include <vector>

struct SynthSat
{
    std::vector<float> chips;  // one sample per chip (or sub-chip replica)
    double chip_rate;          // replica samples per second (chips/s x samples per chip)
    double carrier_hz;         // L1 / E1 / B1I carrier [Hz]
    double delay_samples;      // code start sample
    double doppler_hz;
    double amplitude;
    std::vector<float> secondary;  // per code period (empty: none)
    std::vector<float> data;       // navigation symbols, data_period_s each (empty: none)
    double data_period_s{0.02};
};

inline std::vector<std::complex<float>> synth_stream(const std::vector<SynthSat>& sats, double fs, size_t n,
    uint32_t seed, double noise_sigma)
{
    std::vector<std::complex<float>> x(n);
    std::mt19937 gen(seed);
    std::normal_distribution<double> nd(0.0, noise_sigma);
    for (size_t i = 0; i < n; ++i) x[i] = std::complex<float>(static_cast<float>(nd(gen)), static_cast<float>(nd(gen)));
    for (const auto& s : sats)
        {
            const double L = static_cast<double>(s.chips.size());
            const double rate = s.chip_rate * (1.0 + s.doppler_hz / s.carrier_hz);
            // carrier by a unit phasor recursion, re-anchored every 4096 samples
            const double w = 2.0 * M_PI * s.doppler_hz / fs;
            const std::complex<double> step(std::cos(w), std::sin(w));
            std::complex<double> ph;
            for (size_t i = 0; i < n; ++i)
                {
                    if ((i & 4095) == 0) ph = std::polar(1.0, w * static_cast<double>(i) + 0.3);
                    const double t = (static_cast<double>(i) - s.delay_samples) / fs;
                    const double c = t * rate;  // replica samples since the code start
                    const double period = std::floor(c / L);
                    const double k = c - period * L;
                    const auto idx = static_cast<size_t>(std::min(L - 1.0, std::max(0.0, std::floor(k))));
                    double v = s.chips[idx];
                    if (!s.secondary.empty())
                        {
                            const auto p = static_cast<long long>(period);
                            const long long ns = static_cast<long long>(s.secondary.size());
                            v *= s.secondary[static_cast<size_t>(((p % ns) + ns) % ns)];
                        }
                    if (!s.data.empty() && t >= 0.0)
                        v *= s.data[static_cast<size_t>(std::floor(t / s.data_period_s)) % s.data.size()];
                    const std::complex<double> a = s.amplitude * v * ph;
                    x[i] += std::complex<float>(static_cast<float>(a.real()), static_cast<float>(a.imag()));
                    ph *= step;
                }
        }
    return x;
}

#endif
