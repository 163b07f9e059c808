// CPU-only probe (no HIP): TrackingDump writes N synthetic log_data records into
// <dir>/trk_dump<channel>.dat and converts them with save_matfile
// (tests/test_host_mirror.py reads both back).
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>

#include "tracking_dump.h"

int main(int argc, char** argv)
{
    if (argc < 2) return 2;
    const std::string dir = argv[1];
    TrackingDump d;
    if (!d.configure(dir + "/trk_dump.dat")) return 3;
    d.open(5);
    d.set_acquisition(17, 1234.5, -2750.0);
    for (int i = 0; i < 37; ++i)
        {
            gsdr_trk_epoch r;
            std::memset(&r, 0, sizeof r);
            r.sample_counter = 4000ULL * static_cast<uint64_t>(i) + 17;
            r.consumed = 4000 + (i % 3) - 1;
            r.flags = GSDR_TRK_F_LOGGED;
            for (int k = 0; k < 5; ++k) r.log_accu[k] = 100.0F * static_cast<float>(i) + static_cast<float>(k);
            for (int k = 0; k < 10; ++k) r.taps[k] = static_cast<float>(i) - 0.5F * static_cast<float>(k);
            r.acc_carrier_phase_rad = 0.125 * i;
            r.carrier_doppler_hz = 1000.0 + i;
            r.code_freq_chips = 1.023e6 + 0.5 * i;
            r.carrier_rate = 1e-9F * static_cast<float>(i);
            r.code_rate = 2e-12F * static_cast<float>(i);
            r.carr_phase_error_hz = 0.01F * static_cast<float>(i);
            r.carr_error_filt_hz = 0.02F * static_cast<float>(i);
            r.code_error_chips = 0.001F * static_cast<float>(i);
            r.code_error_filt_chips = 0.002F * static_cast<float>(i);
            r.cn0_db_hz = 40.0 + 0.1 * i;
            r.carrier_lock_test = 0.9;
            r.rem_code_phase_samples = 0.25 * i;
            r.evm = 0.03 * i;
            d.write(r, 4000000.0, true, false);
        }
    return d.save_matfile() ? 0 : 1;
}
