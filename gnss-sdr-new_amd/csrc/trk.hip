// Device-resident DLL/PLL tracking loop for MI355X (gfx950).
//
// Restates dll_pll_veml_tracking (src/algorithms/tracking/gnuradio_blocks/
// dll_pll_veml_tracking.cc) for GPS L1 C/A as one kernel that keeps every
// channel's loop state on the device: one workgroup per channel iterates over
// its general_work calls ("epochs") without returning to the host --
//
//   correlation  (do_correlation_step, :1064-1089) -- 256 lanes, fused carrier
//                wipe-off + code resampler + E/P/L dot products, replica in LDS;
//   loop update  (lane 0)  save results / cn0_and_tracking_lock_status (:970-1056)
//                / run_dll_pll (:1092-1179) / update_tracking_vars (:1216-1287)
//                / bit synchronisation (acquire_secondary, :923-967) and the
//                state machine of general_work (:1784-2152, states 2 and 4).
//
// The tracking loop is sequential in time per channel (each epoch's NCO comes
// from the previous epoch's discriminators), so the parallel axes are the
// samples of one correlation and the channels; the per-epoch host round trip of
// the reference (one general_work call per code period) becomes a loop inside
// one launch.
//
// Types follow the reference members (dll_pll_veml_tracking.h:117-209): float
// where it uses float, double where it uses double, so the device loop tracks
// the CPU restatement (oracle/trk_oracle.c) to fp rounding.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstddef>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <new>
#include <vector>

#include "gsdr_internal.h"

// The reference loop is compiled for x86-64 without FMA contraction; keep every
// a*b+c of the restatement as two roundings.
#pragma clang fp contract(off)

namespace
{

constexpr int kTrkThreads = 512;
constexpr int kMaxCn0 = 64;         // cn0_samples capacity
constexpr int kMaxTrkTaps = 5;
constexpr int kMaxCodeFloats = 16384;
constexpr int kPreambleLen = 160;   // GPS_CA_PREAMBLE_LENGTH_SYMBOLS (GPS_L1_CA.h:61)
constexpr int kSpl = 8;                       // samples per lane per correlation chunk
constexpr int kWinCore = kSpl * kTrkThreads;  // 4096: the next call's window staged in LDS
constexpr int kHalo = 16;                     // slack around the predicted next start

// MATH_CONSTANTS.h:47-50
constexpr double kGnssPi = 3.1415926535898;
constexpr double kTwoPi = 2.0 * kGnssPi;
constexpr double kHalfPi = kGnssPi / 2.0;

// GPS_L1_CA.h:34-73
constexpr double kGpsL1Hz = 1.57542e9;
constexpr double kGpsCaRate = 1.023e6;
constexpr double kGpsCaPeriod = 0.001;
constexpr int kGpsCaLength = 1023;
constexpr int kGpsCaSymbolsPerBit = 20;
// GPS_CA_PREAMBLE_SYMBOLS_STR as a 160-bit register, string index i at bit
// (159 - i) of the 5-word big register (word 4 = most significant)
// '1' -> 1; built on the host by preamble_register().

// ------------------------------------------------------------------ loop library
struct LoopFilter  // Tracking_loop_filter (tracking_loop_filter.cc)
{
    float inputs[4], outputs[4], icoef[4], ocoef[3];
    int nin, nout, idx, order;
    float bw, T;
};

struct CarrierFilter  // Tracking_FLL_PLL_filter (tracking_FLL_PLL_filter.cc)
{
    float w, w0p3, w0f2, x, a2, w0f, a3, w0p2, b3, w0p;
    int order;
};

struct Smoother  // Exponential_Smoother; the init buffer's in-order float sum is kept running
{
    float alpha, one_minus_alpha, old, min_value, offset, init_sum;
    int samples_init, counter, initializing, nbuf;
};

__host__ __device__ inline void lf_update(LoopFilter& f)  // :98-197
{
    float g1, g2, g3, wn;
    const float T = f.T;
    const float zeta = 1.0F / sqrtf(2.0F);
    switch (f.order)
        {
        case 1:
            wn = f.bw * 4.0F;
            g1 = wn;
            f.nin = 1;
            f.icoef[0] = g1;
            f.nout = 0;
            break;
        case 2:
            wn = f.bw * (8.0F * zeta) / (4.0F * zeta * zeta + 1.0F);
            g1 = wn * wn;
            g2 = wn * 2.0F * zeta;
            f.nin = 2;
            f.icoef[0] = (float)(g1 * T / 2.0 + g2);
            f.icoef[1] = (float)(g1 * T / 2.0 - g2);
            f.nout = 1;
            f.ocoef[0] = 1.0F;
            break;
        default:
            {
                wn = f.bw / 0.7845F;
                const float a3 = 1.1F, b3 = 2.4F;
                g1 = wn * wn * wn;
                g2 = a3 * wn * wn;
                g3 = b3 * wn;
                f.nin = 3;
                f.icoef[0] = (float)(g3 + T / 2.0 * (g2 + T / 2.0 * g1));
                f.icoef[1] = (float)(g1 * T * T / 2.0 - 2.0 * g3);
                f.icoef[2] = (float)(g3 + T / 2.0 * (-g2 + T / 2.0 * g1));
                f.nout = 2;
                f.ocoef[0] = 2.0F;
                f.ocoef[1] = -1.0F;
            }
            break;
        }
}

__host__ __device__ inline void lf_initialize(LoopFilter& f, float y0)  // :258-263
{
    for (int i = 0; i < 4; ++i)
        {
            f.inputs[i] = 0.0F;
            f.outputs[i] = y0;
        }
    f.idx = 3;
}

__device__ inline float lf_apply(LoopFilter& f, float in)  // :58-93
{
    float r = 0.0F;
    for (int ii = 0; ii < f.nout; ++ii) r += f.ocoef[ii] * f.outputs[(f.idx + ii) % 4];
    f.idx--;
    if (f.idx < 0) f.idx += 4;
    f.inputs[f.idx] = in;
    for (int ii = 0; ii < f.nin; ++ii) r += f.icoef[ii] * f.inputs[(f.idx + ii) % 4];
    f.outputs[f.idx] = r;
    return r;
}

__host__ __device__ inline void cf_set_params(CarrierFilter& p, float fll_bw, float pll_bw, int order)  // :23-58
{
    p.order = order;
    if (order == 3)
        {
            p.b3 = 2.400F;
            p.a3 = 1.100F;
            p.a2 = 1.414F;
            p.w0p = pll_bw / 0.7845F;
            p.w0p2 = p.w0p * p.w0p;
            p.w0p3 = p.w0p2 * p.w0p;
            p.w0f = fll_bw / 0.53F;
            p.w0f2 = p.w0f * p.w0f;
        }
    else
        {
            p.a2 = 1.414F;
            p.w0p = pll_bw / 0.53F;
            p.w0p2 = p.w0p * p.w0p;
            p.w0f = fll_bw / 0.25F;
        }
}

__host__ __device__ inline void cf_initialize(CarrierFilter& p, float dop)  // :61-74
{
    if (p.order == 3)
        {
            p.x = 2.0F * dop;
            p.w = 0;
        }
    else
        {
            p.w = dop;
            p.x = 0;
        }
}

__device__ inline float cf_error(CarrierFilter& p, float fll, float pll, float t)  // :77-101
{
    float e;
    if (p.order == 3)
        {
            p.w = p.w + t * (p.w0p3 * pll + p.w0f2 * fll);
            p.x = p.x + t * (0.5F * p.w + p.a2 * p.w0f * fll + p.a3 * p.w0p2 * pll);
            e = 0.5F * p.x + p.b3 * p.w0p * pll;
        }
    else
        {
            const float wn = p.w + pll * p.w0p2 * t + fll * p.w0f * t;
            e = 0.5F * (wn + p.w) + p.a2 * p.w0p * pll;
            p.w = wn;
        }
    return e;
}

__host__ __device__ inline void sm_reset(Smoother& s)
{
    s.initializing = 1;
    s.counter = 0;
    s.nbuf = 0;
    s.init_sum = 0.0F;
}

__device__ inline float sm_smooth(Smoother& s, float raw)  // exponential_smoother.cc:84-110
{
    float v;
    if (s.initializing)
        {
            s.counter++;
            v = raw;
            s.init_sum = s.init_sum + v;
            s.nbuf++;
            if (s.counter == s.samples_init)
                {
                    s.old = s.init_sum / (float)s.nbuf;
                    if (s.old < (s.min_value + s.offset))
                        {
                            s.counter = 0;
                            s.nbuf = 0;
                            s.init_sum = 0.0F;
                        }
                    else
                        s.initializing = 0;
                }
        }
    else
        {
            v = s.alpha * raw + s.one_minus_alpha * s.old;
            s.old = v;
        }
    return v;
}

// ------------------------------------------------------------------ channel state
// Scalar loop state: lives in lane 0's registers for a whole launch.
struct TrkHot
{
    // configuration (Dll_Pll_Conf + signal constants)
    double fs_in, code_period, code_chip_rate, signal_carrier_freq, carrier_lock_threshold;
    float early_late_space_chips;
    int32_t vector_length, code_length_chips, code_samples_per_chip, symbols_per_bit;
    int32_t cn0_samples, cn0_min, max_code_lock_fail, max_carrier_lock_fail;
    uint32_t pull_in_time_s, bit_sync_limit_s;
    int32_t extend_correlation_symbols, enable_fll_pull_in, enable_fll_steady_state, carrier_aiding;
    int32_t n_taps, code_samples;
    float shifts[kMaxTrkTaps];
    uint32_t preamble[5];
    // loop objects without history arrays
    Smoother cn0_sm, lock_sm;
    CarrierFilter carrier_filter;
    // state (dll_pll_veml_tracking.h:117-209)
    double acq_code_phase_samples, acq_carrier_doppler_hz, current_correlation_time_s;
    double carr_phase_error_hz, carr_freq_error_hz, carr_error_filt_hz, code_error_chips, code_error_filt_chips;
    double code_freq_chips, carrier_doppler_hz, acc_carrier_phase_rad, rem_code_phase_chips;
    double carrier_lock_test, cn0_db_hz, evm;
    double carrier_phase_step_rad, carrier_phase_rate_step_rad, code_phase_step_chips, code_phase_rate_step_chips;
    double rem_code_phase_samples;
    float2 taps[kMaxTrkTaps];
    float2 E_accu, P_accu, P_accu_old, L_accu, P_data_accu;
    uint32_t circ[5];  // signs of the last kPreambleLen prompts (1 = real < 0), newest at bit 0
    int32_t circ_size;
    uint64_t acq_sample_stamp, next_sample;
    float rem_carr_phase_rad, spc;
    int32_t state, current_prn_length_samples, current_symbol, current_data_symbol, cn0_estimation_counter;
    int32_t carrier_lock_fail_counter, code_lock_fail_counter;
    int32_t pull_in_transitory, cloop, acc_carrier_phase_initialized, flag_pll_180;
    uint32_t prn;
    int32_t assoc;
};

// Device-memory image of one channel: the scalars plus the dynamically indexed
// histories (kept in LDS during a launch).
struct TrkChan
{
    TrkHot h;
    LoopFilter code_filter;
    float2 prompt_buffer[kMaxCn0];
};

struct Prep  // lane-0 -> workgroup broadcast of one epoch's NCO
{
    double psi0, theta;
    float2 wstep;
    float rem_code, code_step;
    int64_t off;
    int32_t go;
    int32_t woff;  // >= 0: this call's samples are in the LDS window at that offset
    int32_t fast;  // every code index of the call lies in [-L, 2L): branch-free wrap
};

// ------------------------------------------------------------------ lane-0 loop body
__device__ inline double pll_cloop_two_quadrant_atan(float2 p)  // tracking_discriminators.cc:92-99
{
    if (p.x != 0.0F) return (double)atanf(p.y / p.x);
    return 0.0;
}

__device__ inline double phase_unwrap(double p)
{
    if (p >= kHalfPi) return p - kGnssPi;
    if (p <= -kHalfPi) return p + kGnssPi;
    return p;
}

__device__ inline double fll_diff_atan(float2 s1, float2 s2, double t1, double t2)  // :62-70
{
    double d = (double)(atanf(s2.y / s2.x) - atanf(s1.y / s1.x));
    if (isnan(d)) d = 0;
    return phase_unwrap(d) / (t2 - t1);
}

__device__ inline double dll_nc_e_minus_l(float2 e, float2 l, float spc, float slope, float y)  // :110-120
{
    const double pe = (double)hypotf(e.x, e.y);
    const double pl = (double)hypotf(l.x, l.y);
    const double s = pe + pl;
    if (s == 0.0) return 0.0;
    return (double)((y - slope * spc) / slope) * (pe - pl) / s;
}

__device__ inline float cn0_m2m4(const float2* b, int length, float coh)  // lock_detectors.cc:90-120
{
    float snr, psig = 0.0F, m2 = 0.0F, m4 = 0.0F, aux;
    const float n = (float)length;
    for (int i = 0; i < length; i++)
        {
            psig += fabsf(b[i].x);
            aux = b[i].y * b[i].y + b[i].x * b[i].x;
            m2 += aux;
            m4 += (aux * aux);
        }
    psig /= n;
    psig = psig * psig;
    m2 /= n;
    m4 /= n;
    aux = sqrtf(2.0F * m2 * m2 - m4);
    if (isnan(aux))
        snr = psig / (m2 - psig);
    else
        snr = aux / (m2 - aux);
    return 10.0F * log10f(snr) - 10.0F * log10f(coh);
}

__device__ inline float carrier_lock_detector(const float2* b, int length)  // :133-148
{
    float si = 0.0F, sq = 0.0F;
    for (int i = 0; i < length; i++)
        {
            si += b[i].x;
            sq += b[i].y;
        }
    const float nbp = si * si + sq * sq;
    const float nbd = si * si - sq * sq;
    return nbd / nbp;
}

__device__ inline void clear_tracking_vars(TrkHot& t)  // :1192-1213
{
    for (int k = 0; k < kMaxTrkTaps; ++k) t.taps[k] = make_float2(0.f, 0.f);
    t.P_accu_old = make_float2(0.f, 0.f);
    t.carr_phase_error_hz = 0.0;
    t.carr_freq_error_hz = 0.0;
    t.carr_error_filt_hz = 0.0;
    t.code_error_chips = 0.0;
    t.code_error_filt_chips = 0.0;
    t.current_symbol = 0;
    t.current_data_symbol = 0;
    t.circ_size = 0;
    for (int w = 0; w < 5; ++w) t.circ[w] = 0u;
    t.carrier_phase_rate_step_rad = 0.0;
    t.code_phase_rate_step_chips = 0.0;
}

__device__ inline int cn0_and_lock(TrkHot& t, float2* pbuf, double coh)  // :970-1056
{
    const int n = t.cn0_samples;
    if (t.cn0_estimation_counter < n)
        {
            pbuf[t.cn0_estimation_counter] = t.P_accu;
            t.cn0_estimation_counter++;
            return 1;
        }
    pbuf[t.cn0_estimation_counter % n] = t.P_accu;
    t.cn0_estimation_counter++;
    const float raw = cn0_m2m4(pbuf, n, (float)coh);
    t.cn0_db_hz = (double)sm_smooth(t.cn0_sm, raw);
    t.carrier_lock_test = (double)sm_smooth(t.lock_sm, carrier_lock_detector(pbuf, 1));
    if (!t.pull_in_transitory)
        {
            if (t.carrier_lock_test < t.carrier_lock_threshold)
                t.carrier_lock_fail_counter++;
            else if (t.carrier_lock_fail_counter > 0)
                t.carrier_lock_fail_counter--;
            if (t.cn0_db_hz < t.cn0_min)
                t.code_lock_fail_counter++;
            else if (t.code_lock_fail_counter > 0)
                t.code_lock_fail_counter--;
        }
    if (t.carrier_lock_fail_counter > t.max_carrier_lock_fail || t.code_lock_fail_counter > t.max_code_lock_fail)
        {
            t.carrier_lock_fail_counter = 0;
            t.code_lock_fail_counter = 0;
            return 0;
        }
    // EVM (fork indicator, :1027-1053)
    float d, s = 0;
    for (int i = 0; i < n; i++) s = s + pbuf[i].x * pbuf[i].x;
    d = s / (float)n;
    d = sqrtf(d);
    s = 0;
    for (int i = 0; i < n; i++)
        {
            const float a = fabsf(pbuf[i].x / d) - 1.0F;
            const float b = fabsf(pbuf[i].y / d) - 0.0F;
            s = s + a * a + b * b;
        }
    t.evm = sqrt((double)(s / (float)n / 1.0F));
    return 1;
}

__device__ inline void run_dll_pll(TrkHot& t, LoopFilter& lf)  // :1092-1179 (no Doppler correction)
{
    t.carr_phase_error_hz = pll_cloop_two_quadrant_atan(t.P_accu) / kTwoPi;
    if ((t.pull_in_transitory && t.enable_fll_pull_in) || t.enable_fll_steady_state)
        {
            t.carr_freq_error_hz = fll_diff_atan(t.P_accu_old, t.P_accu, 0, t.current_correlation_time_s) / kTwoPi;
            t.P_accu_old = t.P_accu;
            if (t.pull_in_transitory && t.enable_fll_pull_in)
                t.carr_error_filt_hz = (double)cf_error(t.carrier_filter, (float)t.carr_freq_error_hz, 0.0F,
                    (float)t.current_correlation_time_s);
            else
                t.carr_error_filt_hz = (double)cf_error(t.carrier_filter, (float)t.carr_freq_error_hz,
                    (float)t.carr_phase_error_hz, (float)t.current_correlation_time_s);
        }
    else
        {
            t.carr_error_filt_hz = (double)cf_error(t.carrier_filter, 0, (float)t.carr_phase_error_hz,
                (float)t.current_correlation_time_s);
        }
    t.carrier_doppler_hz = t.carr_error_filt_hz;
    t.code_error_chips = dll_nc_e_minus_l(t.E_accu, t.L_accu, t.spc, 1.0F, 1.0F);
    t.code_error_filt_chips = (double)lf_apply(lf, (float)t.code_error_chips);
    t.code_freq_chips = t.code_chip_rate - t.code_error_filt_chips;
    if (t.carrier_aiding) t.code_freq_chips += t.carrier_doppler_hz * t.code_chip_rate / t.signal_carrier_freq;
}

__device__ inline void update_tracking_vars(TrkHot& t)  // :1216-1287 (high_dyn = false)
{
    const double T_chip = 1.0 / t.code_freq_chips;
    const double T_prn = T_chip * (double)t.code_length_chips;
    const double T_prn_samples = T_prn * t.fs_in;
    const double K_blk = T_prn_samples + t.rem_code_phase_samples;
    t.current_prn_length_samples = (int32_t)floor(K_blk);
    t.carrier_phase_step_rad = kTwoPi * t.carrier_doppler_hz / t.fs_in;
    const double len = (double)t.current_prn_length_samples;
    t.rem_carr_phase_rad += (float)(t.carrier_phase_step_rad * len + 0.5 * t.carrier_phase_rate_step_rad * len * len);
    t.rem_carr_phase_rad = (float)fmod((double)t.rem_carr_phase_rad, kTwoPi);
    t.acc_carrier_phase_rad -= (t.carrier_phase_step_rad * len + 0.5 * t.carrier_phase_rate_step_rad * len * len);
    t.code_phase_step_chips = t.code_freq_chips / t.fs_in;
    t.rem_code_phase_samples = K_blk - len;
    t.rem_code_phase_chips = t.code_freq_chips * t.rem_code_phase_samples / t.fs_in;
}

__device__ inline void circ_push(TrkHot& t, float2 prompt)
{
    // shift the 160-bit register left by one, new sign in at bit 0
    const uint32_t in = prompt.x < 0.0F ? 1u : 0u;
    uint32_t carry = in;
    for (int w = 0; w < 5; ++w)
        {
            const uint32_t out = t.circ[w] >> 31;
            t.circ[w] = (t.circ[w] << 1) | carry;
            carry = out;
        }
    if (t.circ_size < kPreambleLen) t.circ_size++;
}

// acquire_secondary (:923-967): corr = sum over the buffer of +-1 by sign match
// = 160 - 2 * mismatches; |corr| == 160 only on a full match or full inversion.
__device__ inline int acquire_secondary(TrkHot& t)
{
    int mism = 0;
    for (int w = 0; w < 5; ++w) mism += __popc(t.circ[w] ^ t.preamble[w]);
    if (mism == 0)
        {
            t.flag_pll_180 = 0;  // corr = +160 (string '1' <-> real >= 0 mismatch accounted in the register)
            return 1;
        }
    if (mism == kPreambleLen)
        {
            t.flag_pll_180 = 1;
            return 1;
        }
    return 0;
}

struct EpochOut
{
    int32_t flags;
    double prompt_i, prompt_q;
};

// One general_work call after the correlation (taps in t.taps): states 2 and 4.
__device__ inline void after_correlation(TrkHot& t, LoopFilter& lf, float2* pbuf, uint64_t nitems_read, EpochOut& o,
    uint64_t* ts = nullptr)
{
    o.flags = 0;
    o.prompt_i = 0.0;
    o.prompt_q = 0.0;
    if (t.state == 2)
        {
            t.E_accu = t.taps[0];
            t.P_accu = t.taps[1];
            t.L_accu = t.taps[2];
            t.spc = t.early_late_space_chips;
            if ((uint64_t)t.bit_sync_limit_s < (nitems_read - t.acq_sample_stamp) / (uint64_t)(int)t.fs_in)
                t.carrier_lock_fail_counter = 300000;
            const int lock_ok = cn0_and_lock(t, pbuf, t.code_period);
            if (ts) ts[0] = clock64();
            if (!lock_ok)
                {
                    clear_tracking_vars(t);
                    t.state = 0;
                    o.flags |= GSDR_TRK_F_LOSS_OF_LOCK;
                }
            else
                {
                    int next_state = 0;
                    run_dll_pll(t, lf);
                    if (ts) ts[1] = clock64();
                    update_tracking_vars(t);
                    if (ts) ts[2] = clock64();
                    if (!t.pull_in_transitory)
                        {
                            circ_push(t, t.taps[1]);
                            if (t.circ_size == kPreambleLen) next_state = acquire_secondary(t);
                        }
                    if (next_state)
                        {
                            t.E_accu = t.P_accu = t.L_accu = t.P_data_accu = make_float2(0.f, 0.f);
                            t.circ_size = 0;
                            for (int w = 0; w < 5; ++w) t.circ[w] = 0u;
                            t.current_symbol = 0;
                            t.current_data_symbol = 0;
                            t.state = 4;
                            o.flags |= GSDR_TRK_F_BIT_SYNC;
                        }
                }
        }
    else  // state 4
        {
            t.E_accu.x += t.taps[0].x;
            t.E_accu.y += t.taps[0].y;
            t.P_accu.x += t.taps[1].x;
            t.P_accu.y += t.taps[1].y;
            t.L_accu.x += t.taps[2].x;
            t.L_accu.y += t.taps[2].y;
            t.P_data_accu.x += t.taps[1].x;
            t.P_data_accu.y += t.taps[1].y;
            t.current_data_symbol++;
            t.current_data_symbol %= t.symbols_per_bit;
            t.cloop = 1;
            if (!cn0_and_lock(t, pbuf, t.code_period * (double)t.extend_correlation_symbols))
                {
                    clear_tracking_vars(t);
                    t.state = 0;
                    o.flags |= GSDR_TRK_F_LOSS_OF_LOCK;
                }
            else
                {
                    run_dll_pll(t, lf);
                    update_tracking_vars(t);
                    if (!t.acc_carrier_phase_initialized)
                        {
                            t.acc_carrier_phase_rad = -(double)t.rem_carr_phase_rad;
                            t.acc_carrier_phase_initialized = 1;
                        }
                    if (t.current_data_symbol == 0)
                        {
                            o.prompt_i = (double)t.P_data_accu.x;
                            o.prompt_q = (double)t.P_data_accu.y;
                            o.flags |= GSDR_TRK_F_VALID_OUTPUT;
                            t.P_data_accu = make_float2(0.f, 0.f);
                        }
                    t.E_accu = t.P_accu = t.L_accu = make_float2(0.f, 0.f);
                }
        }
    if (t.flag_pll_180) o.flags |= GSDR_TRK_F_PLL_180;
}

template <int IT>
__device__ __forceinline__ float2 load_iq(const void* __restrict__ p, int64_t i)
{
    if constexpr (IT == GSDR_ITEM_GR_COMPLEX)
        return reinterpret_cast<const float2*>(p)[i];
    else
        {
            const short2 s = reinterpret_cast<const short2*>(p)[i];
            return make_float2((float)s.x, (float)s.y);
        }
}

__device__ __forceinline__ int wrap_code(int raw, int L)
{
    if (raw < 0) raw += L;
    if (raw >= L) raw -= L;
    if ((unsigned)raw >= (unsigned)L)
        {
            raw %= L;
            if (raw < 0) raw += L;
        }
    return raw;
}

// One correlation chunk of kSpl samples per lane (n = n0 + tid + j*256), KT taps,
// no branches inside: samples past the end are zero and their index clamped.
template <int IT, bool FROM_WIN, bool FAST, int KT>
__device__ __forceinline__ void correlate_chunk(const void* __restrict__ iq, const float2* s_win, const float* s_code,
    const Prep& p, int n0, int vl, int L, const float (&sh_rem)[kMaxTrkTaps], float2& ph, float2 (&acc)[kMaxTrkTaps])
{
    float2 xs[kSpl];
#pragma unroll
    for (int j = 0; j < kSpl; ++j)
        {
            const int n = n0 + (int)threadIdx.x + j * kTrkThreads;
            const int nc = min(n, vl - 1);
            const float2 v = FROM_WIN ? s_win[p.woff + nc] : load_iq<IT>(iq, p.off + nc);
            xs[j] = n < vl ? v : make_float2(0.f, 0.f);
        }
#pragma unroll
    for (int j = 0; j < kSpl; ++j)
        {
            const int n = min(n0 + (int)threadIdx.x + j * kTrkThreads, vl - 1);
            const float2 x = xs[j];
            const float2 tt = make_float2(x.x * ph.x - x.y * ph.y, x.x * ph.y + x.y * ph.x);
            const float a = gsdr::mul_rn(p.code_step, (float)n);
#pragma unroll
            for (int k = 0; k < KT; ++k)
                {
                    // a_avx association: floor(step*n + (shift - rem))
                    int raw = (int)floorf(gsdr::add_rn(a, sh_rem[k]));
                    if (FAST)
                        {
                            raw += raw < 0 ? L : 0;
                            raw -= raw >= L ? L : 0;
                        }
                    else
                        raw = wrap_code(raw, L);
                    const float cv = s_code[raw];
                    acc[k].x += tt.x * cv;
                    acc[k].y += tt.y * cv;
                }
            ph = make_float2(ph.x * p.wstep.x - ph.y * p.wstep.y, ph.x * p.wstep.y + ph.y * p.wstep.x);
        }
}

template <int IT, int KT>
__device__ __forceinline__ void correlate_call(const void* __restrict__ iq, const float2* s_win, const float* s_code,
    const Prep& p, int vl, int L, const float (&sh_rem)[kMaxTrkTaps], float2& ph, float2 (&acc)[kMaxTrkTaps])
{
    for (int n0 = 0; n0 < vl; n0 += kWinCore)
        {
            if (p.woff >= 0)
                {
                    if (p.fast)
                        correlate_chunk<IT, true, true, KT>(iq, s_win, s_code, p, n0, vl, L, sh_rem, ph, acc);
                    else
                        correlate_chunk<IT, true, false, KT>(iq, s_win, s_code, p, n0, vl, L, sh_rem, ph, acc);
                }
            else
                {
                    if (p.fast)
                        correlate_chunk<IT, false, true, KT>(iq, s_win, s_code, p, n0, vl, L, sh_rem, ph, acc);
                    else
                        correlate_chunk<IT, false, false, KT>(iq, s_win, s_code, p, n0, vl, L, sh_rem, ph, acc);
                }
        }
}

// grid = channels; one 256-lane workgroup per channel.  Lane 0 holds the scalar
// loop state in registers for the whole launch; the histories indexed at run
// time (prompt buffer, DLL filter), the replica and the next call's input window
// sit in LDS.  While lane 0 runs the loop update of call e, every lane fetches the
// samples call e+1 will most likely read (the consumed count is one code period
// +-1 sample) into the LDS window, so the update hides the HBM latency.
template <int IT>
__global__ void __launch_bounds__(kTrkThreads) trk_kernel(TrkChan* __restrict__ chans, const float* const* __restrict__ codes,
    const void* __restrict__ iq, uint64_t iq_first, uint64_t iq_items, uint32_t max_epochs,
    gsdr_trk_epoch* __restrict__ out, uint32_t* __restrict__ nout, int code_pad, uint64_t* __restrict__ timing)
{
    extern __shared__ float s_dyn[];
    float* s_code = s_dyn;
    float2* s_win = reinterpret_cast<float2*>(s_dyn + code_pad);
    __shared__ LoopFilter s_lf;
    __shared__ float2 s_pbuf[kMaxCn0];
    __shared__ float s_shifts[kMaxTrkTaps];
    __shared__ int s_meta[4];  // state, n_taps, code_samples, vector_length
    __shared__ Prep prep;
    __shared__ float2 s_red[kTrkThreads / 64][kMaxTrkTaps];
    __shared__ TrkHot s_hot;  // lane 0 copies it into registers only around its loop update
    const int ch = blockIdx.x;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    TrkChan* gc = chans + ch;
    if (tid == 0)
        {
            const TrkHot t = gc->h;
            s_hot = t;
            s_lf = gc->code_filter;
            s_meta[0] = t.state;
            s_meta[1] = t.n_taps;
            s_meta[2] = t.code_samples;
            s_meta[3] = t.vector_length;
            for (int k = 0; k < kMaxTrkTaps; ++k) s_shifts[k] = t.shifts[k];
        }
    if (tid < kMaxCn0) s_pbuf[tid] = gc->prompt_buffer[tid];
    __syncthreads();
    if (s_meta[0] != 2 && s_meta[0] != 4)
        {
            if (tid == 0) nout[ch] = 0;
            return;
        }
    const int K = s_meta[1];
    const int L = s_meta[2];
    const int vl = s_meta[3];
    const bool use_window = vl <= kWinCore;
    {
        const float* c = codes[ch];
        for (int i = tid; i < L; i += kTrkThreads) s_code[i] = c[i];
    }
    int64_t win_base = INT64_MIN;  // absolute-index base of the staged window (uniform)
    uint32_t e = 0;
    for (;; ++e)
        {
            uint64_t tm0 = 0, tm1 = 0, tm2 = 0, tmA = 0, tmB = 0, tmC = 0;
            if (timing && tid == 0) tm0 = clock64();
            if (tid == 0)
                {
                    const TrkHot& t = s_hot;
                    Prep p{};
                    const int64_t off = (int64_t)(t.next_sample - iq_first);
                    p.go = (e < max_epochs) && (t.state == 2 || t.state == 4) && t.next_sample >= iq_first &&
                           (uint64_t)off + (uint64_t)vl <= iq_items;
                    p.off = off;
                    p.woff = -1;
                    if (use_window && win_base != INT64_MIN && off >= win_base && off - win_base + vl <= kWinCore + kHalo)
                        p.woff = (int32_t)(off - win_base);
                    if (p.go)
                        {
                            // do_correlation_step's float arguments (:1069-1075); the
                            // reference's phasors (cos r, -sin r) and exp(-j step)
                            // (cpu_multicorrelator_real_codes.cc:114-123) as angles
                            const float rem_carr = t.rem_carr_phase_rad;
                            const float carr_step = (float)t.carrier_phase_step_rad;
                            p.rem_code = (float)t.rem_code_phase_chips * (float)t.code_samples_per_chip;
                            p.code_step = (float)t.code_phase_step_chips * (float)t.code_samples_per_chip;
                            p.psi0 = -(double)rem_carr;
                            p.theta = -(double)carr_step;
                            // index range of the call (monotone in n for step > 0)
                            float smin = 1e30f, smax = -1e30f;
                            for (int k = 0; k < t.n_taps; ++k)
                                {
                                    const float sr = gsdr::sub_rn(t.shifts[k], p.rem_code);
                                    smin = fminf(smin, sr);
                                    smax = fmaxf(smax, sr);
                                }
                            const float lo = floorf(smin);
                            const float hi = floorf(gsdr::add_rn(gsdr::mul_rn(p.code_step, (float)(vl - 1)), smax));
                            const float Lf = (float)t.code_samples;
                            p.fast = p.code_step >= 0.0f && lo >= -Lf && hi < 2.0f * Lf;
                            const double w = p.theta * (double)kTrkThreads;
                            float sn, cs;
                            sincosf((float)fma(-rint(w * 0.15915494309189533576888376337251), 6.283185307179586476925286766559, w),
                                &sn, &cs);
                            p.wstep = make_float2(cs, sn);
                        }
                    prep = p;
                }
            __syncthreads();
            if (!prep.go) break;
            if (timing && tid == 0) tm1 = clock64();
            // ---- correlation: lane-interleaved samples, fp64 phasor anchor + fp32 steps
            const Prep p = prep;
            if (timing && tid == 0) tmA = clock64();
            float2 acc[kMaxTrkTaps];
#pragma unroll
            for (int k = 0; k < kMaxTrkTaps; ++k) acc[k] = make_float2(0.f, 0.f);
            float2 ph;
            {
                const double phi = p.psi0 + (double)tid * p.theta;
                const float a = (float)fma(-rint(phi * 0.15915494309189533576888376337251), 6.283185307179586476925286766559, phi);
                float sn, cs;
                sincosf(a, &sn, &cs);
                ph = make_float2(cs, sn);
            }
            float sh_rem[kMaxTrkTaps];
#pragma unroll
            for (int k = 0; k < kMaxTrkTaps; ++k) sh_rem[k] = gsdr::sub_rn(s_shifts[k], p.rem_code);
            if (timing && tid == 0) tmB = clock64();
            if (K <= 3)
                correlate_call<IT, 3>(iq, s_win, s_code, p, vl, L, sh_rem, ph, acc);
            else
                correlate_call<IT, kMaxTrkTaps>(iq, s_win, s_code, p, vl, L, sh_rem, ph, acc);
            if (timing && tid == 0) tmC = clock64();
#pragma unroll
            for (int k = 0; k < kMaxTrkTaps; ++k)
                {
                    if (k < K)
                        {
#pragma unroll
                            for (int off = 32; off > 0; off >>= 1)
                                {
                                    acc[k].x += __shfl_xor(acc[k].x, off);
                                    acc[k].y += __shfl_xor(acc[k].y, off);
                                }
                        }
                }
            if (lane == 0)
                {
#pragma unroll
                    for (int k = 0; k < kMaxTrkTaps; ++k) s_red[wave][k] = acc[k];
                }
            __syncthreads();  // partials visible; every read of the LDS window done
            if (timing && tid == 0) tm2 = clock64();
            // ---- fetch the window the next call most likely reads: [off + vl - kHalo/2, +kWinCore+kHalo)
            float2 wv[kSpl];
            float2 wh = make_float2(0.f, 0.f);
            const int64_t nb = p.off + vl - kHalo / 2;
            if (use_window)
                {
#pragma unroll
                    for (int j = 0; j < kSpl; ++j)
                        {
                            const int64_t i = nb + tid + j * kTrkThreads;
                            wv[j] = (i >= 0 && (uint64_t)i < iq_items) ? load_iq<IT>(iq, i) : make_float2(0.f, 0.f);
                        }
                    if (tid < kHalo)
                        {
                            const int64_t i = nb + kWinCore + tid;
                            wh = (i >= 0 && (uint64_t)i < iq_items) ? load_iq<IT>(iq, i) : make_float2(0.f, 0.f);
                        }
                }
            if (tid == 0)
                {
                    TrkHot t = s_hot;
#pragma unroll
                    for (int k = 0; k < kMaxTrkTaps; ++k)
                        {
                            float2 r = make_float2(0.f, 0.f);
                            if (k < K)
                                {
                                    for (int w = 0; w < kTrkThreads / 64; ++w)
                                        {
                                            r.x += s_red[w][k].x;
                                            r.y += s_red[w][k].y;
                                        }
                                }
                            t.taps[k] = r;
                        }
                    const uint64_t n_read = t.next_sample;
                    const int32_t state0 = t.state;
                    // pull-in transitory check at the top of general_work (:1794-1803)
                    if (t.pull_in_transitory &&
                        (uint64_t)t.pull_in_time_s < (n_read - t.acq_sample_stamp) / (uint64_t)(int)t.fs_in)
                        {
                            t.pull_in_transitory = 0;
                            t.carrier_lock_fail_counter = 0;
                            t.code_lock_fail_counter = 0;
                        }
                    EpochOut o;
                    const uint64_t tmD = timing ? clock64() : 0;
                    after_correlation(t, s_lf, s_pbuf, n_read, o, timing ? timing + ((size_t)ch * max_epochs + e) * 12 + 8 : nullptr);
                    const uint64_t tmE = timing ? clock64() : 0;
                    gsdr_trk_epoch r;
                    r.sample_counter = n_read;
                    r.state = state0;
                    r.consumed = t.current_prn_length_samples;
#pragma unroll
                    for (int k = 0; k < 5; ++k)
                        {
                            r.taps[2 * k] = t.taps[k].x;
                            r.taps[2 * k + 1] = t.taps[k].y;
                        }
                    r.rem_carr_phase_rad = t.rem_carr_phase_rad;
                    r.flags = o.flags;
                    r.carrier_doppler_hz = t.carrier_doppler_hz;
                    r.code_freq_chips = t.code_freq_chips;
                    r.rem_code_phase_samples = t.rem_code_phase_samples;
                    r.acc_carrier_phase_rad = t.acc_carrier_phase_rad;
                    r.cn0_db_hz = t.cn0_db_hz;
                    r.carrier_lock_test = t.carrier_lock_test;
                    r.prompt_i = o.prompt_i;
                    r.prompt_q = o.prompt_q;
                    r.evm = t.evm;
                    out[(size_t)ch * max_epochs + e] = r;
                    t.next_sample = n_read + (uint64_t)(int64_t)t.current_prn_length_samples;
                    s_hot = t;
                    if (timing)
                        {
                            uint64_t* tr = timing + ((size_t)ch * max_epochs + e) * 12;
                            tr[0] = tm0;
                            tr[1] = tm1;
                            tr[2] = tmA;
                            tr[3] = tmB;
                            tr[4] = tmC;
                            tr[5] = tm2;
                            tr[6] = tmD;
                            tr[7] = tmE;
                            tr[11] = clock64();
                        }
                }
            if (use_window)
                {
#pragma unroll
                    for (int j = 0; j < kSpl; ++j) s_win[tid + j * kTrkThreads] = wv[j];
                    if (tid < kHalo) s_win[kWinCore + tid] = wh;
                    win_base = nb;
                }
            // the next iteration's prep barrier orders the window writes and s_red reuse
        }
    __syncthreads();
    if (tid == 0)
        {
            gc->h = s_hot;
            gc->code_filter = s_lf;
            nout[ch] = e;
        }
    if (tid < kMaxCn0) gc->prompt_buffer[tid] = s_pbuf[tid];
}

void preamble_register(uint32_t reg[5])
{
    // GPS_CA_PREAMBLE_SYMBOLS_STR (GPS_L1_CA.h:73); oldest entry (string index 0)
    // at register bit 159.  A register bit is 1 where the prompt's real part is
    // negative; acquire_secondary counts a match for real < 0 against '0', so the
    // register form of the string is 1 where the character is '0'.
    static const char kStr[161] =
        "1111111111111111111100000000000000000000000000000000000000000000000000000000000011111111111111111111000000000000"
        "000000001111111111111111111111111111111111111111";
    for (int w = 0; w < 5; ++w) reg[w] = 0u;
    for (int i = 0; i < kPreambleLen; ++i)
        {
            const int bit = kPreambleLen - 1 - i;
            if (kStr[i] == '0') reg[bit >> 5] |= 1u << (bit & 31);
        }
}

}  // namespace

struct gsdr_trk
{
    int device{0};
    gsdr_trk_conf conf{};
    hipStream_t stream{nullptr};
    std::vector<TrkChan> h_chans;
    TrkChan* d_chans{nullptr};
    TrkChan* d_snap[2]{nullptr, nullptr};
    std::vector<float*> code_bufs;
    float** d_codes{nullptr};
    gsdr_trk_epoch* d_out{nullptr};
    uint32_t* d_nout{nullptr};
    uint32_t out_cap{0};
    void* d_iq{nullptr};
    uint64_t iq_cap{0};
    size_t lds_bytes{0};
    int code_pad{1024};  // floats reserved for the replica ahead of the LDS window
    // GSDR_TRK_TIMING=1: per-phase clock64 stamps of every call, summarised on destroy
    bool timing_on{false};
    uint64_t* d_timing{nullptr};
    size_t timing_cap{0};
    double tsum[11]{};
    uint64_t tcount{0};
    bool profiling{false};
    std::vector<std::pair<hipEvent_t, hipEvent_t>> prof_recs;
    std::vector<hipEvent_t> prof_pool;
    std::mutex mu;
};

namespace
{

size_t trk_item_bytes(int it) { return it == GSDR_ITEM_CSHORT ? 4 : 8; }

// constructor (dll_pll_veml_tracking.cc:85-560) for one channel slot, GPS L1 C/A
void init_channel(const gsdr_trk_conf& c, TrkChan& ch)
{
    std::memset(&ch, 0, sizeof(ch));
    TrkHot& t = ch.h;
    t.fs_in = c.fs_in;
    t.code_period = kGpsCaPeriod;
    t.code_chip_rate = kGpsCaRate;
    t.signal_carrier_freq = kGpsL1Hz;
    t.carrier_lock_threshold = c.carrier_lock_th;
    t.early_late_space_chips = c.early_late_space_chips;
    t.vector_length = (int32_t)c.vector_length;
    t.code_length_chips = kGpsCaLength;
    t.code_samples_per_chip = 1;
    t.symbols_per_bit = kGpsCaSymbolsPerBit;
    t.cn0_samples = c.cn0_samples;
    t.cn0_min = c.cn0_min;
    t.max_code_lock_fail = c.max_code_lock_fail;
    t.max_carrier_lock_fail = c.max_carrier_lock_fail;
    t.pull_in_time_s = c.pull_in_time_s;
    t.bit_sync_limit_s = c.bit_synchronization_time_limit_s;
    t.extend_correlation_symbols = c.extend_correlation_symbols;
    t.enable_fll_pull_in = c.enable_fll_pull_in;
    t.enable_fll_steady_state = c.enable_fll_steady_state;
    t.carrier_aiding = c.carrier_aiding;
    t.n_taps = 3;
    t.shifts[0] = -c.early_late_space_chips * (float)t.code_samples_per_chip;
    t.shifts[1] = 0.0F;
    t.shifts[2] = c.early_late_space_chips * (float)t.code_samples_per_chip;
    preamble_register(t.preamble);
    t.spc = c.early_late_space_chips;
    t.code_freq_chips = t.code_chip_rate;
    ch.code_filter.T = (float)t.code_period;
    ch.code_filter.bw = c.dll_bw_hz;
    ch.code_filter.order = c.dll_filter_order;
    lf_update(ch.code_filter);
    cf_set_params(t.carrier_filter, c.fll_bw_hz, c.pll_bw_hz, c.pll_filter_order);
    // Exponential_Smoother defaults + dll_pll_veml_tracking.cc:540-552
    t.cn0_sm.alpha = c.cn0_smoother_alpha;
    if (t.cn0_sm.alpha < 0) t.cn0_sm.alpha = 0;
    if (t.cn0_sm.alpha > 1) t.cn0_sm.alpha = 1;
    t.cn0_sm.one_minus_alpha = 1.0F - t.cn0_sm.alpha;
    t.cn0_sm.min_value = 25.0F;
    t.cn0_sm.offset = 12.0F;
    t.cn0_sm.samples_init = std::max(1, c.cn0_smoother_samples / (int)(t.code_period * 1000.0));
    sm_reset(t.cn0_sm);
    t.lock_sm.alpha = c.carrier_lock_test_smoother_alpha;
    if (t.lock_sm.alpha < 0) t.lock_sm.alpha = 0;
    if (t.lock_sm.alpha > 1) t.lock_sm.alpha = 1;
    t.lock_sm.one_minus_alpha = 1.0F - t.lock_sm.alpha;
    t.lock_sm.min_value = -1.0F;
    t.lock_sm.offset = 0.0F;
    t.lock_sm.samples_init = std::max(1, c.carrier_lock_test_smoother_samples);
    sm_reset(t.lock_sm);
    t.state = 0;
    t.assoc = GSDR_ASSOC_AVX;
}

int ensure_out(gsdr_trk* k, uint32_t max_epochs)
{
    const uint64_t need = (uint64_t)k->conf.max_channels * max_epochs;
    if (need <= k->out_cap) return GSDR_OK;
    if (k->d_out) GSDR_HIP(hipFree(k->d_out));
    k->d_out = nullptr;
    k->out_cap = 0;
    GSDR_HIP(hipMalloc(&k->d_out, need * sizeof(gsdr_trk_epoch)));
    k->out_cap = (uint32_t)need;
    return GSDR_OK;
}

size_t lds_for(int code_pad) { return (size_t)code_pad * sizeof(float) + (size_t)(kWinCore + kHalo) * sizeof(float2); }

int launch(gsdr_trk* k, const void* iq, uint64_t iq_first, uint64_t iq_items, uint32_t max_epochs, gsdr_trk_epoch* out,
    uint32_t* nout, hipStream_t s)
{
    uint64_t* timing = nullptr;
    if (k->timing_on)
        {
            const size_t need = (size_t)k->conf.max_channels * max_epochs * 12;
            if (need > k->timing_cap)
                {
                    if (k->d_timing) GSDR_HIP(hipFree(k->d_timing));
                    k->d_timing = nullptr;
                    k->timing_cap = 0;
                    GSDR_HIP(hipMalloc(&k->d_timing, need * sizeof(uint64_t)));
                    k->timing_cap = need;
                }
            timing = k->d_timing;
        }
    hipEvent_t e0 = nullptr, e1 = nullptr;
    if (k->profiling)
        {
            for (hipEvent_t* e : {&e0, &e1})
                {
                    if (!k->prof_pool.empty())
                        {
                            *e = k->prof_pool.back();
                            k->prof_pool.pop_back();
                        }
                    else
                        GSDR_HIP(hipEventCreate(e));
                }
            GSDR_HIP(hipEventRecord(e0, s));
        }
    const dim3 grid(k->conf.max_channels);
    if (k->conf.item_type == GSDR_ITEM_GR_COMPLEX)
        hipLaunchKernelGGL((trk_kernel<GSDR_ITEM_GR_COMPLEX>), grid, dim3(kTrkThreads), k->lds_bytes, s, k->d_chans,
            (const float* const*)k->d_codes, iq, iq_first, iq_items, max_epochs, out, nout, k->code_pad, timing);
    else
        hipLaunchKernelGGL((trk_kernel<GSDR_ITEM_CSHORT>), grid, dim3(kTrkThreads), k->lds_bytes, s, k->d_chans,
            (const float* const*)k->d_codes, iq, iq_first, iq_items, max_epochs, out, nout, k->code_pad, timing);
    GSDR_HIP(hipGetLastError());
    if (k->profiling)
        {
            GSDR_HIP(hipEventRecord(e1, s));
            k->prof_recs.push_back({e0, e1});
        }
    if (timing)
        {
            const uint32_t nch = k->conf.max_channels;
            std::vector<uint64_t> tm((size_t)nch * max_epochs * 12);
            std::vector<uint32_t> cnt(nch);
            GSDR_HIP(hipMemcpyAsync(tm.data(), timing, tm.size() * sizeof(uint64_t), hipMemcpyDeviceToHost, s));
            GSDR_HIP(hipMemcpyAsync(cnt.data(), nout, nch * sizeof(uint32_t), hipMemcpyDeviceToHost, s));
            GSDR_HIP(hipStreamSynchronize(s));
            for (uint32_t c = 0; c < nch; ++c)
                for (uint32_t e = 0; e < cnt[c]; ++e)
                    {
                        const uint64_t* r = &tm[((size_t)c * max_epochs + e) * 12];
                        const int seq[] = {0, 1, 2, 3, 4, 5, 6, 8, 9, 10, 7, 11};
                        for (int q = 0; q + 1 < 12; ++q)
                            if (r[seq[q + 1]] >= r[seq[q]]) k->tsum[q] += (double)(r[seq[q + 1]] - r[seq[q]]);
                        k->tcount++;
                    }
        }
    return GSDR_OK;
}

}  // namespace

extern "C" {

void gsdr_trk_conf_default(gsdr_trk_conf* c)
{
    if (!c) return;
    std::memset(c, 0, sizeof(*c));
    c->fs_in = 2000000.0;
    c->carrier_lock_th = 0.7;
    c->signal = GSDR_SIGNAL_GPS_1C;
    c->item_type = GSDR_ITEM_GR_COMPLEX;
    c->max_channels = 1;
    c->fll_bw_hz = 35.0F;
    c->pll_bw_hz = 35.0F;
    c->dll_bw_hz = 2.0F;
    c->pll_bw_narrow_hz = 5.0F;
    c->dll_bw_narrow_hz = 0.75F;
    c->early_late_space_chips = 0.25F;
    c->very_early_late_space_chips = 0.5F;
    c->early_late_space_narrow_chips = 0.15F;
    c->very_early_late_space_narrow_chips = 0.5F;
    c->cn0_smoother_alpha = 0.002F;
    c->carrier_lock_test_smoother_alpha = 0.002F;
    c->pull_in_time_s = 10U;
    c->bit_synchronization_time_limit_s = 20U;
    c->pll_filter_order = 3;
    c->dll_filter_order = 2;
    c->extend_correlation_symbols = 1;
    c->cn0_samples = 20;
    c->cn0_smoother_samples = 200;
    c->carrier_lock_test_smoother_samples = 25;
    c->cn0_min = 25;
    c->max_code_lock_fail = 50;
    c->max_carrier_lock_fail = 5000;
    c->carrier_aiding = 1;
}

int gsdr_trk_create(int device, const gsdr_trk_conf* conf, gsdr_trk** out)
{
    GSDR_REQUIRE(conf && out, GSDR_E_ARG, "gsdr_trk_create: null argument");
    *out = nullptr;
    GSDR_REQUIRE(conf->fs_in > 0.0, GSDR_E_ARG, "gsdr_trk_create: fs_in must be > 0");
    GSDR_REQUIRE(conf->max_channels > 0, GSDR_E_ARG, "gsdr_trk_create: max_channels must be > 0");
    GSDR_REQUIRE(conf->signal == GSDR_SIGNAL_GPS_1C, GSDR_E_UNSUPPORTED, "gsdr_trk_create: signal %d not implemented",
        conf->signal);
    GSDR_REQUIRE(conf->item_type == GSDR_ITEM_GR_COMPLEX || conf->item_type == GSDR_ITEM_CSHORT, GSDR_E_ARG,
        "gsdr_trk_create: unknown item type %d", conf->item_type);
    GSDR_REQUIRE(conf->extend_correlation_symbols == 1, GSDR_E_UNSUPPORTED,
        "gsdr_trk_create: extend_correlation_symbols > 1 not implemented yet");
    GSDR_REQUIRE(conf->high_dyn == 0, GSDR_E_UNSUPPORTED, "gsdr_trk_create: high_dyn not implemented in the loop");
    GSDR_REQUIRE(conf->cn0_samples >= 1 && conf->cn0_samples <= kMaxCn0, GSDR_E_UNSUPPORTED,
        "gsdr_trk_create: cn0_samples %d outside [1,%d]", conf->cn0_samples, kMaxCn0);
    GSDR_REQUIRE(conf->pll_filter_order == 2 || conf->pll_filter_order == 3, GSDR_E_ARG,
        "gsdr_trk_create: pll_filter_order must be 2 or 3");
    GSDR_REQUIRE(conf->dll_filter_order >= 1 && conf->dll_filter_order <= 3, GSDR_E_ARG,
        "gsdr_trk_create: dll_filter_order must be 1..3");
    int ndev = 0;
    GSDR_HIP(hipGetDeviceCount(&ndev));
    GSDR_REQUIRE(device >= 0 && device < ndev, GSDR_E_ARG, "gsdr_trk_create: device %d of %d", device, ndev);
    gsdr::DeviceGuard g(device);
    gsdr_trk* k = new (std::nothrow) gsdr_trk();
    GSDR_REQUIRE(k, GSDR_E_ALLOC, "gsdr_trk_create: out of host memory");
    k->device = device;
    k->conf = *conf;
    if (k->conf.vector_length == 0)
        k->conf.vector_length = (uint32_t)std::lround(conf->fs_in / (kGpsCaRate / kGpsCaLength));
    const uint32_t nch = k->conf.max_channels;
    k->h_chans.resize(nch);
    for (auto& t : k->h_chans) init_channel(k->conf, t);
    k->code_bufs.assign(nch, nullptr);
    k->code_pad = 1024;  // grows with the longest replica started (gsdr_trk_start)
    k->lds_bytes = lds_for(k->code_pad);
    if (const char* tv = std::getenv("GSDR_TRK_TIMING")) k->timing_on = std::atoi(tv) != 0;
    hipError_t e = hipStreamCreateWithFlags(&k->stream, hipStreamNonBlocking);
    if (e == hipSuccess) e = hipMalloc(&k->d_chans, nch * sizeof(TrkChan));
    if (e == hipSuccess) e = hipMalloc(&k->d_snap[0], nch * sizeof(TrkChan));
    if (e == hipSuccess) e = hipMalloc(&k->d_snap[1], nch * sizeof(TrkChan));
    if (e == hipSuccess) e = hipMalloc(&k->d_codes, nch * sizeof(float*));
    if (e == hipSuccess) e = hipMalloc(&k->d_nout, nch * sizeof(uint32_t));
    for (uint32_t c = 0; c < nch && e == hipSuccess; ++c) e = hipMalloc(&k->code_bufs[c], kMaxCodeFloats * sizeof(float));
    if (e == hipSuccess) e = hipMemcpy(k->d_codes, k->code_bufs.data(), nch * sizeof(float*), hipMemcpyHostToDevice);
    if (e == hipSuccess) e = hipMemcpy(k->d_chans, k->h_chans.data(), nch * sizeof(TrkChan), hipMemcpyHostToDevice);
    if (e == hipSuccess)
        e = hipFuncSetAttribute((const void*)trk_kernel<GSDR_ITEM_GR_COMPLEX>, hipFuncAttributeMaxDynamicSharedMemorySize,
            (int)lds_for(kMaxCodeFloats));
    if (e == hipSuccess)
        e = hipFuncSetAttribute((const void*)trk_kernel<GSDR_ITEM_CSHORT>, hipFuncAttributeMaxDynamicSharedMemorySize,
            (int)lds_for(kMaxCodeFloats));
    if (e != hipSuccess)
        {
            gsdr::set_error("gsdr_trk_create: %s", hipGetErrorString(e));
            gsdr_trk_destroy(k);
            return GSDR_E_ALLOC;
        }
    *out = k;
    return GSDR_OK;
}

void gsdr_trk_destroy(gsdr_trk* k)
{
    if (!k) return;
    gsdr::DeviceGuard g(k->device);
    if (k->stream) (void)hipStreamSynchronize(k->stream);
    if (k->timing_on && k->tcount)
        {
            static const char* names[] = {"prep", "barrier", "anchor", "samples", "reduce+barrier", "to-update",
                "cn0+lock", "dll/pll", "nco", "rest", "record"};
            std::fprintf(stderr, "gsdr_trk timing: %llu calls, clock64 ticks per call:", (unsigned long long)k->tcount);
            for (int q = 0; q < 11; ++q) std::fprintf(stderr, " %s %.0f", names[q], k->tsum[q] / k->tcount);
            std::fprintf(stderr, "\n");
        }
    if (k->d_timing) (void)hipFree(k->d_timing);
    for (auto& r : k->prof_recs)
        {
            (void)hipEventDestroy(r.first);
            (void)hipEventDestroy(r.second);
        }
    for (hipEvent_t e : k->prof_pool) (void)hipEventDestroy(e);
    for (float* p : k->code_bufs)
        if (p) (void)hipFree(p);
    void* bufs[] = {k->d_chans, k->d_snap[0], k->d_snap[1], k->d_codes, k->d_nout, k->d_out, k->d_iq};
    for (void* p : bufs)
        if (p) (void)hipFree(p);
    if (k->stream) (void)hipStreamDestroy(k->stream);
    delete k;
}

int gsdr_trk_start(gsdr_trk* k, int ch, uint32_t prn, const float* code, int code_samples, double acq_delay_samples,
    double acq_doppler_hz, uint64_t acq_samplestamp, uint64_t nitems_read, uint64_t* first_sample)
{
    GSDR_REQUIRE(k && code && first_sample, GSDR_E_ARG, "gsdr_trk_start: null argument");
    GSDR_REQUIRE(ch >= 0 && ch < (int)k->conf.max_channels, GSDR_E_ARG, "gsdr_trk_start: channel %d outside [0,%u)", ch,
        k->conf.max_channels);
    GSDR_REQUIRE(code_samples >= 1 && code_samples <= kMaxCodeFloats, GSDR_E_UNSUPPORTED,
        "gsdr_trk_start: code replica of %d samples outside [1,%d]", code_samples, kMaxCodeFloats);
    std::lock_guard<std::mutex> lk(k->mu);
    gsdr::DeviceGuard g(k->device);
    // the device copy is authoritative between launches (the loop runs there)
    GSDR_HIP(hipMemcpyAsync(&k->h_chans[ch], k->d_chans + ch, sizeof(TrkChan), hipMemcpyDeviceToHost, k->stream));
    GSDR_HIP(hipStreamSynchronize(k->stream));
    TrkChan& tc = k->h_chans[ch];
    TrkHot& t = tc.h;
    // start_tracking (:640-882)
    t.prn = prn;
    t.code_samples = code_samples;
    t.acq_code_phase_samples = acq_delay_samples;
    t.acq_carrier_doppler_hz = acq_doppler_hz;
    t.acq_sample_stamp = acq_samplestamp;
    t.carrier_doppler_hz = t.acq_carrier_doppler_hz;
    t.carrier_phase_step_rad = kTwoPi * t.carrier_doppler_hz / t.fs_in;
    t.carrier_phase_rate_step_rad = 0.0;
    for (int i = 0; i < kMaxTrkTaps; ++i) t.taps[i] = make_float2(0.f, 0.f);
    t.carrier_lock_fail_counter = 0;
    t.code_lock_fail_counter = 0;
    t.rem_code_phase_samples = 0.0;
    t.rem_carr_phase_rad = 0.0F;
    t.rem_code_phase_chips = 0.0;
    t.acc_carrier_phase_rad = 0.0;
    t.cn0_estimation_counter = 0;
    t.carrier_lock_test = 1.0;
    t.cn0_db_hz = 0.0;
    t.evm = 0.0;
    t.shifts[0] = -k->conf.early_late_space_chips * (float)t.code_samples_per_chip;
    t.shifts[2] = k->conf.early_late_space_chips * (float)t.code_samples_per_chip;
    t.current_correlation_time_s = t.code_period;
    cf_set_params(t.carrier_filter, k->conf.fll_bw_hz, k->conf.pll_bw_hz, k->conf.pll_filter_order);
    tc.code_filter.bw = k->conf.dll_bw_hz;
    lf_update(tc.code_filter);
    tc.code_filter.T = (float)t.code_period;
    lf_update(tc.code_filter);
    cf_initialize(t.carrier_filter, (float)t.acq_carrier_doppler_hz);
    lf_initialize(tc.code_filter, 0.0F);
    t.cloop = 1;
    t.pull_in_transitory = 1;
    t.circ_size = 0;
    for (int w = 0; w < 5; ++w) t.circ[w] = 0u;
    t.acc_carrier_phase_initialized = 0;
    // state 1: pull-in alignment (:1813-1844)
    const int64_t diff = (int64_t)nitems_read - (int64_t)t.acq_sample_stamp;
    const double delta = (double)diff - t.acq_code_phase_samples;
    t.code_freq_chips = t.code_chip_rate;
    t.code_phase_step_chips = t.code_freq_chips / t.fs_in;
    t.code_phase_rate_step_chips = 0.0;
    const double T_chip_mod = 1.0 / t.code_freq_chips;
    const double T_prn_mod = T_chip_mod * (double)t.code_length_chips;
    const double T_prn_mod_samples = T_prn_mod * t.fs_in;
    t.acq_code_phase_samples = T_prn_mod_samples - std::fmod(delta, T_prn_mod_samples);
    t.current_prn_length_samples = (int32_t)std::round(T_prn_mod_samples);
    const int32_t offset = (int32_t)std::round(t.acq_code_phase_samples);
    t.acc_carrier_phase_rad -= t.carrier_phase_step_rad * (double)offset;
    t.state = 2;
    sm_reset(t.cn0_sm);
    sm_reset(t.lock_sm);
    t.next_sample = nitems_read + (uint64_t)(int64_t)offset;
    *first_sample = t.next_sample;
    k->code_pad = std::max(k->code_pad, (code_samples + 1) & ~1);
    k->lds_bytes = lds_for(k->code_pad);
    GSDR_HIP(hipMemcpyAsync(k->code_bufs[ch], code, (size_t)code_samples * sizeof(float), hipMemcpyHostToDevice,
        k->stream));
    GSDR_HIP(hipMemcpyAsync(k->d_chans + ch, &tc, sizeof(TrkChan), hipMemcpyHostToDevice, k->stream));
    GSDR_HIP(hipStreamSynchronize(k->stream));
    return GSDR_OK;
}

int gsdr_trk_stop(gsdr_trk* k, int ch)
{
    GSDR_REQUIRE(k, GSDR_E_ARG, "gsdr_trk_stop: null handle");
    GSDR_REQUIRE(ch >= 0 && ch < (int)k->conf.max_channels, GSDR_E_ARG, "gsdr_trk_stop: channel %d", ch);
    std::lock_guard<std::mutex> lk(k->mu);
    gsdr::DeviceGuard g(k->device);
    const int32_t zero = 0;
    GSDR_HIP(hipMemcpyAsync(reinterpret_cast<char*>(k->d_chans + ch) + offsetof(TrkChan, h) + offsetof(TrkHot, state),
        &zero, sizeof(zero),
        hipMemcpyHostToDevice, k->stream));
    GSDR_HIP(hipStreamSynchronize(k->stream));
    return GSDR_OK;
}

int gsdr_trk_run_device(gsdr_trk* k, const void* iq_dev, uint64_t iq_first_sample, uint64_t iq_items, uint32_t max_epochs,
    gsdr_trk_epoch* out_dev, uint32_t* n_out_dev, void* stream)
{
    GSDR_REQUIRE(k && iq_dev && out_dev && n_out_dev, GSDR_E_ARG, "gsdr_trk_run_device: null argument");
    std::lock_guard<std::mutex> lk(k->mu);
    gsdr::DeviceGuard g(k->device);
    hipStream_t s = stream ? (hipStream_t)stream : k->stream;
    return launch(k, iq_dev, iq_first_sample, iq_items, max_epochs, out_dev, n_out_dev, s);
}

int gsdr_trk_run(gsdr_trk* k, const void* iq_host, uint64_t iq_first_sample, uint64_t iq_items, uint32_t max_epochs,
    gsdr_trk_epoch* out_host, uint32_t* n_out_host)
{
    GSDR_REQUIRE(k && iq_host && out_host && n_out_host, GSDR_E_ARG, "gsdr_trk_run: null argument");
    std::lock_guard<std::mutex> lk(k->mu);
    gsdr::DeviceGuard g(k->device);
    const size_t bytes = (size_t)iq_items * trk_item_bytes(k->conf.item_type);
    if (iq_items > k->iq_cap)
        {
            if (k->d_iq) GSDR_HIP(hipFree(k->d_iq));
            k->d_iq = nullptr;
            k->iq_cap = 0;
            GSDR_HIP(hipMalloc(&k->d_iq, bytes));
            k->iq_cap = iq_items;
        }
    int rc = ensure_out(k, max_epochs);
    if (rc != GSDR_OK) return rc;
    GSDR_HIP(hipMemcpyAsync(k->d_iq, iq_host, bytes, hipMemcpyHostToDevice, k->stream));
    rc = launch(k, k->d_iq, iq_first_sample, iq_items, max_epochs, k->d_out, k->d_nout, k->stream);
    if (rc != GSDR_OK) return rc;
    GSDR_HIP(hipMemcpyAsync(n_out_host, k->d_nout, k->conf.max_channels * sizeof(uint32_t), hipMemcpyDeviceToHost,
        k->stream));
    GSDR_HIP(hipMemcpyAsync(out_host, k->d_out, (size_t)k->conf.max_channels * max_epochs * sizeof(gsdr_trk_epoch),
        hipMemcpyDeviceToHost, k->stream));
    GSDR_HIP(hipStreamSynchronize(k->stream));
    return GSDR_OK;
}

int gsdr_trk_get_channel(gsdr_trk* k, int ch, int32_t* state, uint64_t* next_sample, double* doppler, double* cn0)
{
    GSDR_REQUIRE(k, GSDR_E_ARG, "gsdr_trk_get_channel: null handle");
    GSDR_REQUIRE(ch >= 0 && ch < (int)k->conf.max_channels, GSDR_E_ARG, "gsdr_trk_get_channel: channel %d", ch);
    std::lock_guard<std::mutex> lk(k->mu);
    gsdr::DeviceGuard g(k->device);
    GSDR_HIP(hipMemcpyAsync(&k->h_chans[ch], k->d_chans + ch, sizeof(TrkChan), hipMemcpyDeviceToHost, k->stream));
    GSDR_HIP(hipStreamSynchronize(k->stream));
    const TrkHot& t = k->h_chans[ch].h;
    if (state) *state = t.state;
    if (next_sample) *next_sample = t.next_sample;
    if (doppler) *doppler = t.carrier_doppler_hz;
    if (cn0) *cn0 = t.cn0_db_hz;
    return GSDR_OK;
}

int gsdr_trk_save_state(gsdr_trk* k, int slot, void* stream)
{
    GSDR_REQUIRE(k && (slot == 0 || slot == 1), GSDR_E_ARG, "gsdr_trk_save_state: bad argument");
    gsdr::DeviceGuard g(k->device);
    hipStream_t s = stream ? (hipStream_t)stream : k->stream;
    GSDR_HIP(hipMemcpyAsync(k->d_snap[slot], k->d_chans, k->conf.max_channels * sizeof(TrkChan), hipMemcpyDeviceToDevice, s));
    return GSDR_OK;
}

int gsdr_trk_restore_state(gsdr_trk* k, int slot, void* stream)
{
    GSDR_REQUIRE(k && (slot == 0 || slot == 1), GSDR_E_ARG, "gsdr_trk_restore_state: bad argument");
    gsdr::DeviceGuard g(k->device);
    hipStream_t s = stream ? (hipStream_t)stream : k->stream;
    GSDR_HIP(hipMemcpyAsync(k->d_chans, k->d_snap[slot], k->conf.max_channels * sizeof(TrkChan), hipMemcpyDeviceToDevice, s));
    return GSDR_OK;
}

int gsdr_trk_set_profiling(gsdr_trk* k, int enable)
{
    GSDR_REQUIRE(k, GSDR_E_ARG, "gsdr_trk_set_profiling: null handle");
    std::lock_guard<std::mutex> lk(k->mu);
    k->profiling = enable != 0;
    return GSDR_OK;
}

int gsdr_trk_read_profile(gsdr_trk* k, double* kernel_ms, uint32_t* launches)
{
    GSDR_REQUIRE(k && kernel_ms && launches, GSDR_E_ARG, "gsdr_trk_read_profile: null argument");
    std::lock_guard<std::mutex> lk(k->mu);
    gsdr::DeviceGuard g(k->device);
    *kernel_ms = 0.0;
    *launches = 0;
    for (auto& r : k->prof_recs)
        {
            GSDR_HIP(hipEventSynchronize(r.second));
            float ms = 0.0f;
            GSDR_HIP(hipEventElapsedTime(&ms, r.first, r.second));
            *kernel_ms += ms;
            *launches += 1;
            k->prof_pool.push_back(r.first);
            k->prof_pool.push_back(r.second);
        }
    k->prof_recs.clear();
    return GSDR_OK;
}

}  // extern "C"
