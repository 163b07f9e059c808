#include "gnss_replicas.h"

#include <algorithm>
#include <array>
#include <bitset>
#include <cmath>
#include <cstring>
#include <string>

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

// ======================================================================= Galileo E1
extern "C" const unsigned char gsdr_galileo_e1_codes[];  // galileo_e1_codes.cc: 100 rows x 512 bytes

namespace
{
constexpr int32_t kGalE1CodeLength = 4092;                      // GALILEO_E1_B_CODE_LENGTH_CHIPS
constexpr int32_t kGalE1ChipRate = 1023000;                     // GALILEO_E1_CODE_CHIP_RATE_CPS
constexpr char kGalE1CSecondary[] = "0011100000001010110110010";  // GALILEO_E1_C_SECONDARY_CODE (Galileo_E1.h:52)

bool is_signal(const char* signal, const char* id)
{
    const std::string s(signal ? signal : "");
    return s.length() >= 2 && s.rfind(id) != std::string::npos;
}

// galileo_e1_sinboc_11_gen_int (:61-77) / _61_ (:80-97) for dest of `length` samples
std::vector<int32_t> sinboc_11(const std::vector<int32_t>& prn, uint32_t length)
{
    std::vector<int32_t> dest(length);
    const uint32_t period = length / static_cast<uint32_t>(kGalE1CodeLength);
    for (uint32_t i = 0; i < static_cast<uint32_t>(kGalE1CodeLength); i++)
        {
            for (uint32_t j = 0; j < period / 2; j++) dest[i * period + j] = prn[i];
            for (uint32_t j = period / 2; j < period; j++) dest[i * period + j] = -prn[i];
        }
    return dest;
}

std::vector<int32_t> sinboc_61(const std::vector<int32_t>& prn, uint32_t length)
{
    std::vector<int32_t> dest(length);
    const uint32_t period = length / static_cast<uint32_t>(kGalE1CodeLength);
    for (uint32_t i = 0; i < static_cast<uint32_t>(kGalE1CodeLength); i++)
        {
            for (uint32_t j = 0; j < period; j += 2) dest[i * period + j] = prn[i];
            for (uint32_t j = 1; j < period; j += 2) dest[i * period + j] = -prn[i];
        }
    return dest;
}

// resampler (gnss_signal_replica.cc:257-272): float index arithmetic, last sample
// forced to the last input sample
std::vector<float> resample(const std::vector<float>& src, uint32_t dest_size, float fs_in, float fs_out)
{
    std::vector<float> dest(dest_size);
    const float t_out = 1.0F / fs_out;
    for (uint32_t i = 0; i + 1 < dest_size; i++)
        {
            const float aux = (t_out * (static_cast<float>(i) + 1.0F)) * fs_in;
            const auto idx = static_cast<int32_t>(static_cast<int64_t>(aux + 1.0F)) - 1;
            dest[i] = src[static_cast<size_t>(idx)];
        }
    if (dest_size > 0) dest[dest_size - 1] = src.back();
    return dest;
}
}  // namespace

std::vector<int32_t> galileo_e1_code_gen_int(const char* signal, int32_t prn)
{
    if (prn < 1 || prn > 50) return {};
    int row;
    if (is_signal(signal, "1B"))
        row = prn - 1;
    else if (is_signal(signal, "1C"))
        row = 50 + prn - 1;
    else
        return {};
    const unsigned char* bits = gsdr_galileo_e1_codes + static_cast<size_t>(row) * 512;
    std::vector<int32_t> dest(kGalE1CodeLength);
    for (int32_t i = 0; i < kGalE1CodeLength; i++)
        dest[i] = ((bits[i >> 3] >> (7 - (i & 7))) & 1) ? -1 : 1;
    return dest;
}

std::vector<float> galileo_e1_code_gen_sinboc11_float(const char* signal, uint32_t prn)
{
    const auto chips = galileo_e1_code_gen_int(signal, static_cast<int32_t>(prn));
    std::vector<float> dest(2 * kGalE1CodeLength);
    if (chips.empty()) return dest;
    for (int32_t i = 0; i < kGalE1CodeLength; i++)
        {
            dest[2 * i] = static_cast<float>(chips[i]);
            dest[2 * i + 1] = -dest[2 * i];
        }
    return dest;
}

std::vector<float> galileo_e1_code_gen_float_sampled(const char* signal, bool cboc, uint32_t prn, int32_t sampling_freq,
    uint32_t chip_shift, bool secondary_flag)
{
    const int32_t samples_per_chip = cboc ? 12 : 2;
    const uint32_t code_length = static_cast<uint32_t>(samples_per_chip * kGalE1CodeLength);
    auto samples_per_code = static_cast<uint32_t>(static_cast<double>(sampling_freq) /
                                                  (static_cast<double>(kGalE1ChipRate) / static_cast<double>(kGalE1CodeLength)));
    const uint32_t delay = static_cast<uint32_t>((kGalE1CodeLength - static_cast<int32_t>(chip_shift)) % kGalE1CodeLength) *
                           samples_per_code / static_cast<uint32_t>(kGalE1CodeLength);
    auto chips = galileo_e1_code_gen_int(signal, static_cast<int32_t>(prn));
    if (chips.empty()) chips.assign(kGalE1CodeLength, 0);
    std::vector<float> sig(code_length);
    if (cboc)
        {
            // galileo_e1_gen_float (:114-143), CBOC(6,1,1/11) at 12 samples per chip
            const float alpha = std::sqrt(10.0F / 11.0F);
            const float beta = std::sqrt(1.0F / 11.0F);
            const auto s11 = sinboc_11(chips, code_length);
            const auto s61 = sinboc_61(chips, code_length);
            const bool e1b = is_signal(signal, "1B");
            for (uint32_t i = 0; i < code_length; i++)
                {
                    const float a = alpha * static_cast<float>(s11[i]);
                    const float b = beta * static_cast<float>(s61[i]);
                    sig[i] = e1b ? a + b : a - b;
                }
        }
    else
        {
            const auto s11 = sinboc_11(chips, code_length);
            for (uint32_t i = 0; i < code_length; i++) sig[i] = static_cast<float>(s11[i]);
        }
    if (sampling_freq != samples_per_chip * kGalE1ChipRate)
        sig = resample(sig, samples_per_code, static_cast<float>(samples_per_chip * kGalE1ChipRate),
            static_cast<float>(sampling_freq));
    if (is_signal(signal, "1C") && secondary_flag)
        {
            const uint32_t ns = static_cast<uint32_t>(std::strlen(kGalE1CSecondary));
            std::vector<float> sec(static_cast<size_t>(ns) * samples_per_code);
            for (uint32_t i = 0; i < ns; i++)
                for (uint32_t k = 0; k < samples_per_code; k++)
                    sec[i * samples_per_code + k] = sig[k] * (kGalE1CSecondary[i] == '0' ? 1.0F : -1.0F);
            samples_per_code *= ns;
            sig = std::move(sec);
        }
    std::vector<float> dest(samples_per_code);
    for (uint32_t i = 0; i < samples_per_code; i++) dest[(i + delay) % samples_per_code] = sig[i];
    return dest;
}

std::vector<std::complex<float>> galileo_e1_code_gen_complex_sampled(const char* signal, bool cboc, uint32_t prn,
    int32_t sampling_freq, uint32_t chip_shift, bool secondary_flag)
{
    const auto re = galileo_e1_code_gen_float_sampled(signal, cboc, prn, sampling_freq, chip_shift, secondary_flag);
    std::vector<std::complex<float>> dest(re.size());
    for (size_t i = 0; i < re.size(); i++) dest[i] = std::complex<float>(re[i], 0.0F);
    return dest;
}

// ======================================================================= BeiDou B1I
std::vector<int32_t> beidou_b1i_code_gen_int(int32_t prn, uint32_t chip_shift)
{
    constexpr uint32_t code_length = 2046;
    static constexpr std::array<int32_t, 63> phase1 = {1, 1, 1, 1, 1, 1, 1, 1, 2, 3, 3, 3, 3, 3, 3, 3, 4, 4, 4, 4, 4,
        4, 5, 5, 5, 5, 5, 6, 6, 6, 6, 8, 8, 8, 9, 9, 10, 2, 3, 3, 3, 3, 3, 4, 4, 5, 5, 5, 5, 6, 8, 9, 9, 3, 5, 7, 4, 4,
        5, 5, 5, 5, 6};
    static constexpr std::array<int32_t, 63> phase2 = {3, 4, 5, 6, 8, 9, 10, 11, 7, 4, 5, 6, 8, 9, 10, 11, 5, 6, 8, 9,
        10, 11, 6, 8, 9, 10, 11, 8, 9, 10, 11, 9, 10, 11, 10, 11, 11, 7, 4, 6, 8, 10, 11, 5, 9, 6, 8, 10, 11, 9, 9, 10,
        11, 7, 7, 9, 5, 9, 6, 8, 10, 11, 9};
    // phase3: PRN 38-53 one extra tap, 54-56 two, 57-63 three (ICD G2 phase table)
    static constexpr std::array<int32_t, 63> phase3 = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0,
        0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 2, 2, 2, 3, 3, 3, 3,
        3, 3, 3};
    const int32_t idx = prn - 1;
    if (idx < 0 || idx > 62) return {};
    // 11-stage registers loaded with 01010101010 (bit i = character 10 - i)
    std::bitset<11> g1r(std::string("01010101010"));
    std::bitset<11> g2r(std::string("01010101010"));
    std::vector<uint8_t> g1(code_length), g2(code_length);
    for (uint32_t n = 0; n < code_length; n++)
        {
            g1[n] = g1r[0];
            g2[n] = static_cast<uint8_t>(g2r[static_cast<size_t>(11 - phase1[idx])] ^ g2r[static_cast<size_t>(11 - phase2[idx])] ^
                                         (phase3[idx] ? g2r[static_cast<size_t>(11 - phase3[idx])] : false));
            const bool f1 = g1r[0] ^ g1r[1] ^ g1r[2] ^ g1r[3] ^ g1r[4] ^ g1r[10];
            const bool f2 = g2r[0] ^ g2r[2] ^ g2r[3] ^ g2r[6] ^ g2r[7] ^ g2r[8] ^ g2r[9] ^ g2r[10];
            g1r >>= 1;
            g2r >>= 1;
            g1r[10] = f1;
            g2r[10] = f2;
        }
    std::vector<int32_t> dest(code_length);
    uint32_t delay = (code_length + chip_shift) % code_length;
    for (uint32_t n = 0; n < code_length; n++)
        {
            dest[n] = (g1[(n + chip_shift) % code_length] ^ g2[delay]) ? 1 : -1;
            delay = (delay + 1) % code_length;
        }
    return dest;
}

std::vector<float> beidou_b1i_code_gen_float(int32_t prn, uint32_t chip_shift)
{
    const auto c = beidou_b1i_code_gen_int(prn, chip_shift);
    return std::vector<float>(c.begin(), c.end());
}

std::vector<std::complex<float>> beidou_b1i_code_gen_complex_sampled(uint32_t prn, int32_t sampling_freq, uint32_t chip_shift)
{
    constexpr int32_t code_freq = 2046000;
    constexpr int32_t code_len = 2046;
    const auto spc = static_cast<int32_t>(static_cast<double>(sampling_freq) /
                                          (static_cast<double>(code_freq) / static_cast<double>(code_len)));
    const float tc = 1.0F / static_cast<float>(code_freq);
    const float ts = 1.0F / static_cast<float>(sampling_freq);
    const auto chips = beidou_b1i_code_gen_int(static_cast<int32_t>(prn), chip_shift);
    std::vector<std::complex<float>> dest(static_cast<size_t>(std::max(spc, 0)));
    if (chips.empty()) return dest;
    for (int32_t i = 0; i < spc; ++i)
        {
            const float aux = (ts * (static_cast<float>(i) + 1)) / tc;
            const int32_t k = static_cast<int32_t>(static_cast<int64_t>(aux + 1)) - 1;
            dest[i] = std::complex<float>(static_cast<float>(i == spc - 1 ? chips[code_len - 1] : chips[k]), 0.0F);
        }
    return dest;
}
