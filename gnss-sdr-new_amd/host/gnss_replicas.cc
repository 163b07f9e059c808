#include "gnss_replicas.h"

#include <array>

namespace
{
// G2 output delays per PRN, IS-GPS-200 (PRN 1-32) and SBAS PRN 120-138.
constexpr std::array<int32_t, 51> kG2Delay = {5, 6, 7, 8, 17, 18, 139, 140, 141, 251, 252, 254, 255, 256, 257, 258, 469,
    470, 471, 472, 473, 474, 509, 512, 513, 514, 515, 516, 859, 860, 861, 862, 145, 175, 52, 21, 237, 235, 886, 657,
    634, 762, 355, 1012, 176, 603, 130, 359, 595, 68, 386};

// One period of a 10-stage maximal LFSR, all-ones start, output = stage 1.
template <size_t NT>
std::array<uint8_t, 1023> lfsr(const std::array<int, NT>& taps)
{
    std::array<uint8_t, 1023> out{};
    uint16_t reg = 0x3FF;  // bit i = stage i+1
    for (int i = 0; i < 1023; ++i)
        {
            out[i] = reg & 1u;
            uint16_t fb = 0;
            for (int t : taps) fb ^= (reg >> t) & 1u;
            reg = static_cast<uint16_t>((reg >> 1) | (fb << 9));
        }
    return out;
}
}  // namespace

std::vector<int32_t> gps_l1_ca_code_gen_int(int32_t prn, uint32_t chip_shift)
{
    static const auto g1 = lfsr<2>({7, 0});
    static const auto g2 = lfsr<6>({8, 7, 4, 2, 1, 0});
    const int32_t idx = (prn >= 120 && prn <= 138) ? prn - 88 : prn - 1;
    if (idx < 0 || idx > 50) return {};
    std::vector<int32_t> dest(1023);
    uint32_t delay = (1023u - kG2Delay[idx] + chip_shift) % 1023u;
    for (uint32_t n = 0; n < 1023; ++n)
        {
            dest[n] = (g1[(n + chip_shift) % 1023u] ^ g2[delay]) ? 1 : -1;
            delay = (delay + 1) % 1023u;
        }
    return dest;
}

std::vector<float> gps_l1_ca_code_gen_float(int32_t prn, uint32_t chip_shift)
{
    auto c = gps_l1_ca_code_gen_int(prn, chip_shift);
    return std::vector<float>(c.begin(), c.end());
}

std::vector<std::complex<float>> gps_l1_ca_code_gen_complex(int32_t prn, uint32_t chip_shift)
{
    auto c = gps_l1_ca_code_gen_int(prn, chip_shift);
    std::vector<std::complex<float>> out(c.size());
    for (size_t i = 0; i < c.size(); ++i) out[i] = std::complex<float>(0.0F, static_cast<float>(c[i]));
    return out;
}

std::vector<std::complex<float>> gps_l1_ca_code_gen_complex_sampled(uint32_t prn, int32_t sampling_freq,
    uint32_t chip_shift)
{
    constexpr int32_t code_freq = 1023000;
    constexpr int32_t code_len = 1023;
    const auto spc = static_cast<int32_t>(static_cast<double>(sampling_freq) /
                                          (static_cast<double>(code_freq) / static_cast<double>(code_len)));
    const float tc = 1.0F / static_cast<float>(code_freq);
    const float ts = 1.0F / static_cast<float>(sampling_freq);
    const auto chips = gps_l1_ca_code_gen_complex(static_cast<int32_t>(prn), chip_shift);
    std::vector<std::complex<float>> dest(spc);
    if (chips.empty()) return dest;
    for (int32_t i = 0; i < spc; ++i)
        {
            const float aux = (ts * (static_cast<float>(i) + 1)) / tc;
            const int32_t k = static_cast<int32_t>(static_cast<int64_t>(aux + 1)) - 1;
            dest[i] = (i == spc - 1) ? chips[code_len - 1] : chips[k];
        }
    return dest;
}
