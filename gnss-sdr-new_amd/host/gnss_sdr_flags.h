// The gflags of src/algorithms/libs/gnss_sdr_flags.cc:41-58 that the blocks on
// this path read: command-line overrides of the .conf (pll_bw_hz, dll_bw_hz,
// doppler_max; 0 = not given) and the lock-detector defaults of Dll_Pll_Conf
// (dll_pll_conf.cc:24-28).  Same names, types and defaults; a maintainer building
// the adapters in the reference tree uses the reference's gnss_sdr_flags.h (gflags
// DEFINE_*) instead, and `gnss-sdr --pll_bw_hz=...` sets them.  Here they are plain
// globals (set them before building the blocks, as gflags parsing would).
#ifndef GSDR_HOST_GNSS_SDR_FLAGS_H
#define GSDR_HOST_GNSS_SDR_FLAGS_H

#include <cstdint>

extern int32_t FLAGS_doppler_max;          // "If defined, sets the maximum Doppler value in the search grid"
extern int32_t FLAGS_doppler_step;         // "If defined, sets the frequency step in the search grid"
extern int32_t FLAGS_cn0_samples;          // 20
extern int32_t FLAGS_cn0_min;              // 25
extern int32_t FLAGS_max_carrier_lock_fail;  // 5000
extern int32_t FLAGS_max_lock_fail;        // 50
extern double FLAGS_carrier_lock_th;       // 0.7
extern double FLAGS_dll_bw_hz;             // 0.0: "If defined, bandwidth of the DLL low pass filter"
extern double FLAGS_pll_bw_hz;             // 0.0: "If defined, bandwidth of the PLL low pass filter"

#endif
