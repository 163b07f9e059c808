// Defaults of src/algorithms/libs/gnss_sdr_flags.cc:41-58.
#include "gnss_sdr_flags.h"

int32_t FLAGS_doppler_max = 0;
int32_t FLAGS_doppler_step = 0;
int32_t FLAGS_cn0_samples = 20;
int32_t FLAGS_cn0_min = 25;
int32_t FLAGS_max_carrier_lock_fail = 5000;
int32_t FLAGS_max_lock_fail = 50;
double FLAGS_carrier_lock_th = 0.7;
double FLAGS_dll_bw_hz = 0.0;
double FLAGS_pll_bw_hz = 0.0;
