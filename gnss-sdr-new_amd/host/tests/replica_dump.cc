// Test tool: writes one code replica of the C++ generators (gnss_replicas.h) to
// stdout as raw float32 (complex replicas as interleaved re, im), for the CPU
// parity test tests/test_host_replicas.py against oracle/replica.py.  No GPU.
// Usage: replica_dump <kind> <prn> [fs] [cboc] [secondary]
//   kind: gps_float | gps_sampled | gal_b_sinboc11 | gal_c_sinboc11 | gal_b_sampled |
//         gal_c_sampled | bds_float | bds_sampled
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>

#include "gnss_replicas.h"

int main(int argc, char** argv)
{
    if (argc < 3) return 2;
    const std::string kind = argv[1];
    const int prn = std::atoi(argv[2]);
    const int fs = argc > 3 ? std::atoi(argv[3]) : 0;
    const bool cboc = argc > 4 && std::atoi(argv[4]) != 0;
    const bool sec = argc > 5 && std::atoi(argv[5]) != 0;
    auto put = [](const void* p, size_t bytes) { return std::fwrite(p, 1, bytes, stdout) == bytes ? 0 : 1; };
    if (kind == "gps_float")
        {
            const auto v = gps_l1_ca_code_gen_float(prn);
            return put(v.data(), v.size() * 4);
        }
    if (kind == "gps_sampled")
        {
            const auto v = gps_l1_ca_code_gen_complex_sampled(static_cast<uint32_t>(prn), fs);
            return put(v.data(), v.size() * 8);
        }
    if (kind == "gal_b_sinboc11" || kind == "gal_c_sinboc11")
        {
            const auto v = galileo_e1_code_gen_sinboc11_float(kind[4] == 'b' ? "1B" : "1C", static_cast<uint32_t>(prn));
            return put(v.data(), v.size() * 4);
        }
    if (kind == "gal_b_sampled" || kind == "gal_c_sampled")
        {
            const auto v = galileo_e1_code_gen_complex_sampled(kind[4] == 'b' ? "1B" : "1C", cboc,
                static_cast<uint32_t>(prn), fs, 0, sec);
            return put(v.data(), v.size() * 8);
        }
    if (kind == "bds_float")
        {
            const auto v = beidou_b1i_code_gen_float(prn);
            return put(v.data(), v.size() * 4);
        }
    if (kind == "bds_sampled")
        {
            const auto v = beidou_b1i_code_gen_complex_sampled(static_cast<uint32_t>(prn), fs);
            return put(v.data(), v.size() * 8);
        }
    return 2;
}
