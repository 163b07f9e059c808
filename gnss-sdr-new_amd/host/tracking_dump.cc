#include "tracking_dump.h"

#include "mat5_writer.h"

#include <cmath>
#include <cstring>
#include <filesystem>
#include <iostream>
#include <system_error>
#include <vector>

namespace
{
constexpr double kTwoPi = 2.0 * 3.1415926535897932384626433832795;  // MATH_CONSTANTS.h:49

template <class T>
char* put(char* p, T v)
{
    std::memcpy(p, &v, sizeof(T));
    return p + sizeof(T);
}
}  // namespace

bool TrackingDump::configure(const std::string& dump_filename)
{
    // :565-597
    std::string name = dump_filename;
    std::string dir;
    const size_t slash = name.find_last_of('/');
    if (slash != std::string::npos)
        {
            dir = name.substr(0, slash);
            name = name.substr(slash + 1);
        }
    else
        dir = ".";
    if (name.empty()) name = "trk_channel_";
    if (name.substr(1).find_last_of('.') != std::string::npos) name = name.substr(0, name.find_last_of('.'));
    stem_ = dir + std::string(1, std::filesystem::path::preferred_separator) + name;
    std::error_code ec;
    std::filesystem::create_directories(dir, ec);
    if (ec && !std::filesystem::is_directory(dir))
        {
            std::cerr << "GNSS-SDR cannot create dump files for the tracking block. Wrong permissions?\n";
            stem_.clear();
            return false;
        }
    return true;
}

bool TrackingDump::open(uint32_t channel)
{
    // set_channel (:1733-1760): the file of the first channel the block is given
    channel_ = channel;
    if (stem_.empty() || file_.is_open()) return file_.is_open();
    path_ = stem_ + std::to_string(channel) + ".dat";
    file_.open(path_, std::ios::out | std::ios::binary);
    if (!file_.is_open()) std::cerr << "channel " << channel << " Exception opening trk dump file " << path_ << '\n';
    return file_.is_open();
}

void TrackingDump::set_acquisition(uint32_t prn, double acq_code_phase_samples, double acq_carrier_doppler_hz)
{
    prn_ = prn;
    acq_code_phase_ = acq_code_phase_samples;
    acq_doppler_ = acq_carrier_doppler_hz;
}

double TrackingDump::pull_in_code_phase(int32_t signal, double fs_in, uint64_t nitems_read, uint64_t acq_sample_stamp,
    double acq_delay_samples)
{
    // code rate and length of the signal (dll_pll_veml_tracking.cc:170-430)
    double rate = 1.023e6, length = 1023.0;
    if (signal == GSDR_SIGNAL_GAL_1B) length = 4092.0;
    if (signal == GSDR_SIGNAL_BDS_B1)
        {
            rate = 2.046e6;
            length = 2046.0;
        }
    const int64_t diff = static_cast<int64_t>(nitems_read) - static_cast<int64_t>(acq_sample_stamp);
    const double delta = static_cast<double>(diff) - acq_delay_samples;
    const double t_prn_samples = 1.0 / rate * length * fs_in;
    return t_prn_samples - std::fmod(delta, t_prn_samples);
}

void TrackingDump::encode(const gsdr_trk_epoch& r, double fs_in, bool veml, bool track_pilot, uint32_t prn,
    double acq_code_phase_samples, double acq_carrier_doppler_hz, char* out)
{
    // log_data (:1403-1500), field by field
    const int iP = veml ? 2 : 1;
    const float prompt_i = track_pilot ? r.data_prompt[0] : r.taps[2 * iP];
    const float prompt_q = track_pilot ? r.data_prompt[1] : r.taps[2 * iP + 1];
    char* p = out;
    p = put<float>(p, veml ? r.log_accu[0] : 0.0F);
    p = put<float>(p, r.log_accu[1]);
    p = put<float>(p, r.log_accu[2]);
    p = put<float>(p, r.log_accu[3]);
    p = put<float>(p, veml ? r.log_accu[4] : 0.0F);
    p = put<float>(p, prompt_i);
    p = put<float>(p, prompt_q);
    // nitems_read(0) + d_current_prn_length_samples (the updated length = consume_each count)
    const uint64_t stamp = r.sample_counter + static_cast<uint64_t>(r.consumed);
    p = put<uint64_t>(p, stamp);
    p = put<float>(p, static_cast<float>(r.acc_carrier_phase_rad));
    p = put<float>(p, static_cast<float>(r.carrier_doppler_hz));
    // the engine keeps the rate steps as float (gsdr_trk_epoch::carrier_rate)
    p = put<float>(p, static_cast<float>(static_cast<double>(r.carrier_rate) * fs_in * fs_in / kTwoPi));
    p = put<float>(p, static_cast<float>(r.code_freq_chips));
    p = put<float>(p, static_cast<float>(static_cast<double>(r.code_rate) * fs_in * fs_in));
    p = put<float>(p, r.carr_phase_error_hz);
    p = put<float>(p, r.carr_error_filt_hz);
    p = put<float>(p, r.code_error_chips);
    p = put<float>(p, r.code_error_filt_chips);
    p = put<float>(p, static_cast<float>(r.cn0_db_hz));
    p = put<float>(p, static_cast<float>(r.carrier_lock_test));
    p = put<float>(p, static_cast<float>(r.rem_code_phase_samples));
    p = put<double>(p, static_cast<double>(stamp));
    p = put<uint32_t>(p, prn);
    p = put<float>(p, static_cast<float>(acq_code_phase_samples));
    p = put<float>(p, static_cast<float>(acq_carrier_doppler_hz));
    p = put<float>(p, static_cast<float>(r.evm));
    (void)p;
}

void TrackingDump::write(const gsdr_trk_epoch& r, double fs_in, bool veml, bool track_pilot)
{
    if (!file_.is_open() || !(r.flags & GSDR_TRK_F_LOGGED)) return;
    char buf[kRecordBytes];
    encode(r, fs_in, veml, track_pilot, prn_, acq_code_phase_, acq_doppler_, buf);
    file_.write(buf, kRecordBytes);
    if (!file_) std::cerr << "Exception writing trk dump file " << path_ << '\n';
}

bool TrackingDump::save_matfile()
{
    if (stem_.empty()) return false;
    if (file_.is_open()) file_.close();
    // :1511-1600: read every 108-byte epoch of <stem><channel>.dat
    const std::string dat = stem_ + std::to_string(channel_) + ".dat";
    std::ifstream in(dat, std::ios::binary | std::ios::ate);
    if (!in.is_open())
        {
            std::cerr << "Problem opening dump file:" << dat << '\n';
            return false;
        }
    const auto size = static_cast<int64_t>(in.tellg());
    const size_t n = static_cast<size_t>(size / static_cast<int64_t>(kRecordBytes));
    in.seekg(0, std::ios::beg);
    std::vector<char> raw(n * kRecordBytes);
    if (n && !in.read(raw.data(), static_cast<std::streamsize>(raw.size())))
        {
            std::cerr << "Problem reading dump file:" << dat << '\n';
            return false;
        }
    // the record's fields in file order: 7 floats, the uint64 sample count, 12 floats,
    // the double aux2, the uint32 PRN, 3 floats (log_data, :1403-1500)
    static const char* const kF1[7] = {"abs_VE", "abs_E", "abs_P", "abs_L", "abs_VL", "Prompt_I", "Prompt_Q"};
    static const char* const kF2[12] = {"acc_carrier_phase_rad", "carrier_doppler_hz", "carrier_doppler_rate_hz",
        "code_freq_chips", "code_freq_rate_chips", "carr_error_hz", "carr_error_filt_hz", "code_error_chips",
        "code_error_filt_chips", "CN0_SNV_dB_Hz", "carrier_lock_test", "aux1"};
    static const char* const kF3[3] = {"acq_code_phase_samples", "acq_carrier_doppler_hz", "EVM"};
    std::vector<std::vector<float>> f1(7, std::vector<float>(n)), f2(12, std::vector<float>(n)),
        f3(3, std::vector<float>(n));
    std::vector<uint64_t> start(n);
    std::vector<double> aux2(n);
    std::vector<uint32_t> prn(n);
    for (size_t i = 0; i < n; ++i)
        {
            const char* p = raw.data() + i * kRecordBytes;
            for (int k = 0; k < 7; ++k, p += 4) std::memcpy(&f1[k][i], p, 4);
            std::memcpy(&start[i], p, 8);
            p += 8;
            for (int k = 0; k < 12; ++k, p += 4) std::memcpy(&f2[k][i], p, 4);
            std::memcpy(&aux2[i], p, 8);
            p += 8;
            std::memcpy(&prn[i], p, 4);
            p += 4;
            for (int k = 0; k < 3; ++k, p += 4) std::memcpy(&f3[k][i], p, 4);
        }
    // :1602-1726: <stem><channel>.mat, every variable 1 x num_epoch, in this order
    const std::string mat = stem_ + std::to_string(channel_) + ".mat";
    Mat5Writer w;
    if (!w.open(mat)) return false;
    const auto cols = static_cast<uint32_t>(n);
    for (int k = 0; k < 7; ++k) w.write(kF1[k], Mat5Writer::kSingle, 1, cols, f1[k].data());
    w.write("PRN_start_sample_count", Mat5Writer::kUint64, 1, cols, start.data());
    for (int k = 0; k < 12; ++k) w.write(kF2[k], Mat5Writer::kSingle, 1, cols, f2[k].data());
    w.write("aux2", Mat5Writer::kDouble, 1, cols, aux2.data());
    w.write("PRN", Mat5Writer::kUint32, 1, cols, prn.data());
    for (int k = 0; k < 3; ++k) w.write(kF3[k], Mat5Writer::kSingle, 1, cols, f3[k].data());
    return w.close();
}
